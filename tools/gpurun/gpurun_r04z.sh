# round 4, call z: where C3's 4 % over the PBKDF2 kernel goes -- kernel statistics of the C3 bench command.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04z}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err
guard $?
python3 - $O/c3/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print(r["Name"][:60], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), round(float(r["AverageNs"]) / 1e6, 3))
PY
