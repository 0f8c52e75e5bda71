# round 3, call l: C5 two callers re-measured (the r03k legs run gave 110 ms per 2 calls against 98 ms in r03i)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03l
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for rep in 1 2 3; do
  for k in 2 1; do
    timeout -k 10 200 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 --no-cpu-baseline \
        > $O/c5_k${k}_$rep.json 2> $O/c5_k${k}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c5_k${k}_$rep.json'));print('k$k rep$rep', d['value'], d['ms_per_step'], d['mismatches'])"
  done
done
nproc; cat /proc/loadavg
