# round 4, call q: does the head slow beside the tail because the tail runs other code?  The tail through the head's
# own kernel (DWPA_TAIL_ISSUE=1) against the plain tail kernel: kernel-traced C5 runs (head / tail durations) and
# C5 one / two callers, alternating.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04q}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 200 env DWPA_TAIL_ISSUE=1 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -k "head_tail_split or c5_mixed" -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
guard $?
tail -2 $O/pytest.log
for t in 0 1; do
  DWPA_TAIL_ISSUE=$t timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$t -o run -- python3 bench.py --workload c5 --steps 8 --warmup 2 --no-cpu-baseline > $O/c5_t$t.json 2> $O/c5_t$t.err
  guard $?
  python3 - $O/t$t/run_kernel_stats.csv $O/c5_t$t.json "$t" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.load(open(sys.argv[2]))
print("tail_issue", sys.argv[3], "C5", d["value"], d["ms_per_step"], {r["Name"][:30]: (int(r["Calls"]), round(float(r["AverageNs"]) / 1e6, 3)) for r in rows if "pbkdf2" in r["Name"]})
PY
done
for rep in 1 2; do
  for t in 0 1; do
    DWPA_TAIL_ISSUE=$t timeout -k 10 120 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/k1_t${t}_r$rep.json 2>/dev/null
    guard $?
    DWPA_TAIL_ISSUE=$t timeout -k 10 120 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 --no-cpu-baseline > $O/k2_t${t}_r$rep.json 2>/dev/null
    guard $?
    python3 -c "import json;a=json.load(open('$O/k1_t${t}_r$rep.json'));b=json.load(open('$O/k2_t${t}_r$rep.json'));print('tail_issue $t rep $rep k1', a['value'], a['mismatches'], 'k2', b['value'], b['mismatches'])"
  done
done
