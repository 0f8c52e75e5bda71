# round 4, call v: chunked derive -- resident waves as a fraction of the chains (DWPA_CHUNK_WAVES sixteenths):
# fewer waves space a chain's consecutive chunks further apart (fewer dependency waits), at lower occupancy.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04v}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for v in "64 14" "64 12" "64 10" "64 8" "32 10" "128 12"; do
  set -- $v
  DWPA_CHECK_CHUNKS=$1 DWPA_CHUNK_WAVES=$2 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$1_w$2 -o run -- python3 bench.py --workload c5 --steps 6 --warmup 2 --no-cpu-baseline > $O/c5_c$1_w$2.json 2> $O/c5_c$1_w$2.err
  guard $?
  python3 - $O/c$1_w$2/run_kernel_stats.csv $O/c5_c$1_w$2.json "$1 $2" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.load(open(sys.argv[2]))
print("chunks/waves16", sys.argv[3], "C5", d["value"], d["ms_per_step"], d["mismatches"], {r["Name"][:22]: round(float(r["AverageNs"]) / 1e6, 3) for r in rows if "pbkdf2" in r["Name"]})
PY
done
