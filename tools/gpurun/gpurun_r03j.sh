# round 3, call j: weak scaling with one shard per rank (own dictionary / ESSIDs): the N=2 GPU tests, then N=8
# rehearsals of the spawn path on the one GPU (DWPA_BENCH_ONE_DEVICE=1; control path, not a scaling measurement).
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03j
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; guard $rc
export DWPA_BENCH_ONE_DEVICE=1
timeout -k 10 300 python3 bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline --dict-words 2000000 \
    --batch 1048576 > $O/c2_n8.json 2> $O/c2_n8.err
guard $?
timeout -k 10 300 python3 bench.py --gpus 8 --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --batch 1048576 \
    > $O/c4_n8.json 2> $O/c4_n8.err
guard $?
timeout -k 10 300 python3 bench.py --gpus 4 --workload c3 --steps 1 --warmup 1 --no-cpu-baseline --batch 1048576 \
    > $O/c3_n4.json 2> $O/c3_n4.err
guard $?
for f in c2_n8 c4_n8 c3_n4; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['n_gpus'], d['hits_verified'], d['value'], d['config'].get('shards'))"; done
