# round 3, call b: GPU suite, then the bench legs whose code changed (process-pool CPU baseline, C1 latency)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 240 python bench.py --workload c1lat --steps 9 > $O/c1lat.json 2> $O/c1lat.err
timeout -k 10 240 python bench.py --workload c1 --steps 20 --warmup 3 > $O/c1.json 2> $O/c1.err
timeout -k 10 240 python bench.py --workload c5 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err
timeout -k 10 300 python bench.py --steps 8 --warmup 2 > $O/c2.json 2> $O/c2.err
cat $O/*.json
