# round 4, call s: the check path's derive as one work queue of iteration chunks (DWPA_CHECK_CHUNKS, chains move
# between waves at chunk boundaries) against the head/tail split: parity first (the split test at 0 / 16 / 7 chunks,
# C5 at 16), then a kernel-traced C5 run per setting and C5 one / two callers alternating.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04s}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -k "head_tail_split" -x -v --timeout 60 --timeout-method thread > $O/pytest_split.log 2>&1
guard $?
tail -5 $O/pytest_split.log
DWPA_CHECK_CHUNKS=16 timeout -k 10 200 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -k "c5_mixed or concurrent" -x -v --timeout 150 --timeout-method thread > $O/pytest_c5.log 2>&1
guard $?
tail -4 $O/pytest_c5.log
for c in 0 16; do
  DWPA_CHECK_CHUNKS=$c timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$c -o run -- python3 bench.py --workload c5 --steps 8 --warmup 2 --no-cpu-baseline > $O/c5_c$c.json 2> $O/c5_c$c.err
  guard $?
  python3 - $O/c$c/run_kernel_stats.csv $O/c5_c$c.json "$c" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.load(open(sys.argv[2]))
print("chunks", sys.argv[3], "C5", d["value"], d["ms_per_step"], d["mismatches"], {r["Name"][:30]: (int(r["Calls"]), round(float(r["AverageNs"]) / 1e6, 3)) for r in rows if "pbkdf2" in r["Name"] or "verify_att" in r["Name"]})
PY
done
for rep in 1 2; do
  for c in 0 16 8 32; do
    DWPA_CHECK_CHUNKS=$c timeout -k 10 120 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/k1_c${c}_r$rep.json 2>/dev/null
    guard $?
    python3 -c "import json;a=json.load(open('$O/k1_c${c}_r$rep.json'));print('chunks $c rep $rep k1', a['value'], a['ms_per_step'], a['mismatches'])"
  done
  for c in 0 16; do
    DWPA_CHECK_CHUNKS=$c timeout -k 10 120 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 --no-cpu-baseline > $O/k2_c${c}_r$rep.json 2>/dev/null
    guard $?
    python3 -c "import json;b=json.load(open('$O/k2_c${c}_r$rep.json'));print('chunks $c rep $rep k2', b['value'], b['ms_per_step'], b['mismatches'])"
  done
done
