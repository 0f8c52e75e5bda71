# round 5, call m: rocprofv3 kernel statistics of the expansion leg (k_rules_expand + the k_text_* packing kernels)
# and of one caller's C5 calls, at the last code.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05m}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/expand -o run -- python3 bench.py \
    --workload expand --rule-words 5000000 --steps 1 --warmup 0 > $O/expand.json 2> $O/expand.err
guard $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python3 bench.py \
    --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
guard $?
for d in expand c5; do
  python3 - $O/$d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print(r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), round(float(r["AverageNs"]) / 1e6, 3))
PY
done
