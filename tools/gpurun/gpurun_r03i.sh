# round 3, call i (re-entry): validate HEAD after the container was re-created: the whole GPU suite, smoke, the C2
# bench line under rocprofv3 --kernel-trace --stats, C5 one and two callers.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03i
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; guard $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; guard $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2_rocprof -o run -- python3 bench.py --steps 5 --warmup 1 \
    > $O/c2_rocprof.json 2> $O/c2_rocprof.err
guard $?
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 > $O/c2.json 2> $O/c2.err
guard $?
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 --no-cpu-baseline \
      > $O/c5_k$k.json 2> $O/c5_k$k.err
  guard $?
done
cat $O/c2.json $O/c5_k1.json $O/c5_k2.json
