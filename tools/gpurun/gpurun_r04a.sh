# round 4, call a: the small-call penalty and the host's CPU share (item 4).
#   1. host facts: cgroup CPU quota, affinity, physical cores (is a 128-process CPU baseline meaningful here?)
#   2. tools/bin/clock_idle: shader clock of 1 / 8 / 1024 lone waves after 0-2 s of GPU idle
#   3. tools/small_call_probe.py under rocprofv3 --kernel-trace: 1/2/16/202-key calls, sequential, interleaved and
#      after idle gaps, cut per call
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04a}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
{
  echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
  echo "cpuset.cpus.effective: $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null)"
  echo "nproc: $(nproc)"
  python3 -c "import os; from oracle.php_pool import physical_cores; a=os.sched_getaffinity(0); print('affinity', len(a), 'physical', physical_cores(a))"
  grep -m1 'model name' /proc/cpuinfo
  cat /proc/loadavg
} > $O/host.txt 2>&1
cat $O/host.txt
timeout -k 10 120 tools/bin/clock_idle 4 > $O/clock_idle.jsonl 2> $O/clock_idle.err
guard $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/probe_trace -o run -- python3 tools/small_call_probe.py \
    > $O/small_call_probe.json 2> $O/small_call_probe.err
guard $?
python3 -c "
import json; d=json.load(open('$O/small_call_probe.json'))
for k,v in d['summary_median_ms'].items(): print(k, v)
"
python3 -c "
import json
for l in open('$O/clock_idle.jsonl'):
    d=json.loads(l)
    if d['rep']==0 or d['rep']==3: print(d)
"
# the rule language on the GPU
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "rules or rule_family" > $O/pytest_rules.log 2>&1
rc=$?; tail -3 $O/pytest_rules.log; guard $rc
# the bench line's new roofline object and the whole-host CPU baseline
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 > $O/bench_short.json 2> $O/bench_short.err
guard $?
python3 -c "
import json; d=json.load(open('$O/bench_short.json')); r=d['roofline']; c=d['cpu_baseline']
print(d['value'], r['frac'], r['frac_issue_cost_model'], r['frac_attainable_on_gfx950'], c['value'], c['one_thread']['value'], c['all_host'])"
