# round 4, call u: the chunked derive with the issue pass applied to it (r04s ran it with the plain schedule):
# parity, then traced C5 per chunk count and C5 one caller alternating with the head/tail split.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04u}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -k "head_tail_split" -x -q --timeout 60 --timeout-method thread > $O/pytest_split.log 2>&1
guard $?
tail -2 $O/pytest_split.log
for c in 0 16 64; do
  DWPA_CHECK_CHUNKS=$c timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$c -o run -- python3 bench.py --workload c5 --steps 8 --warmup 2 --no-cpu-baseline > $O/c5_c$c.json 2> $O/c5_c$c.err
  guard $?
  python3 - $O/c$c/run_kernel_stats.csv $O/c5_c$c.json "$c" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.load(open(sys.argv[2]))
print("chunks", sys.argv[3], "C5", d["value"], d["ms_per_step"], d["mismatches"], {r["Name"][:30]: (int(r["Calls"]), round(float(r["AverageNs"]) / 1e6, 3)) for r in rows if "pbkdf2" in r["Name"] or "verify_att" in r["Name"]})
PY
done
