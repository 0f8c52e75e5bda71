# round 4, call x: the chunked derive with one ready queue per XCD (no L2 write-back / invalidate per piece)
# instead of chunk-major items: parity, then traced C5 per (chunks, resident-wave sixteenths), then C5 one / two
# callers against the head/tail split.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04x}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -k "head_tail_split" -x -q --timeout 60 --timeout-method thread > $O/pytest_split.log 2>&1
guard $?
tail -2 $O/pytest_split.log
for v in "0 14" "16 14" "32 14" "64 14" "16 15" "32 12"; do
  set -- $v
  DWPA_CHECK_CHUNKS=$1 DWPA_CHUNK_WAVES=$2 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$1_w$2 -o run -- python3 bench.py --workload c5 --steps 6 --warmup 2 --no-cpu-baseline > $O/c5_c$1_w$2.json 2> $O/c5_c$1_w$2.err
  guard $?
  python3 - $O/c$1_w$2/run_kernel_stats.csv $O/c5_c$1_w$2.json "$1 $2" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.load(open(sys.argv[2]))
print("chunks/waves16", sys.argv[3], "C5", d["value"], d["ms_per_step"], d["mismatches"], {r["Name"][:22]: round(float(r["AverageNs"]) / 1e6, 3) for r in rows if "pbkdf2" in r["Name"] or "verify_att" in r["Name"]})
PY
done
