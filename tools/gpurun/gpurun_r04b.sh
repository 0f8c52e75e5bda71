# round 4, call b: is the small-call penalty the partial EXEC of lone waves?  
#   1. tools/bin/clock_idle, CLOCK_LANES: shader clock and chain time of 1 / 8 waves with 64 / 16 / 2 / 1 live lanes
#   2. tools/small_call_probe.py with DWPA_LONE_PAD = 0 / 64 / 256 (lone-wave derives padded to whole waves / WGs)
#   3. the rule-family crack test (fixed word choice) and the rule-language GPU tests
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04b}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
CLOCK_LANES=1 timeout -k 10 120 tools/bin/clock_idle 4 > $O/clock_lanes.jsonl 2> $O/clock_lanes.err
guard $?
python3 -c "
import json
for l in open('$O/clock_lanes.jsonl'):
    d=json.loads(l)
    if d['rep']==2: print(d['waves'], d['lanes'], d['clock_mhz_mean'], d['kernel_ms'])
"
for pad in 0 64 256; do
  DWPA_LONE_PAD=$pad timeout -k 10 200 python3 tools/small_call_probe.py > $O/probe_pad$pad.json 2> $O/probe_pad$pad.err
  guard $?
  python3 -c "
import json; d=json.load(open('$O/probe_pad$pad.json'))
print('pad $pad', {k: v for k, v in d['summary_median_ms'].items() if k.startswith('interleaved') or k.startswith('gap1')})"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "rules or rule_family" > $O/pytest_rules.log 2>&1
rc=$?; tail -3 $O/pytest_rules.log; guard $rc
