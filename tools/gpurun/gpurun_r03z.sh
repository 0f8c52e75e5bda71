# round 3, call z: multi-device rehearsals on one GPU -- every crack-path GPU test with 8 shard workers per device
# (DWPA_CRACK_SHARDS_PER_DEVICE=8, as on an 8-GPU node), and C4 strong scaling with 8 ranks (DWPA_BENCH_ONE_DEVICE=1).
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03z
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
DWPA_CRACK_SHARDS_PER_DEVICE=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py \
    -k "crack or help_crack" -x -v --timeout 300 --timeout-method thread > $O/pytest_w8.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_w8.log | tail -20; guard $rc
DWPA_BENCH_ONE_DEVICE=1 timeout -k 10 400 python3 bench.py --gpus 8 --workload c4 --scaling strong --steps 1 --warmup 0 \
    --no-cpu-baseline --t1-s 20.04 > $O/c4_strong_n8.json 2> $O/c4_strong_n8.err
guard $?
python3 -c "import json;d=json.load(open('$O/c4_strong_n8.json'));print(d['n_gpus'], d['hits_verified'], d['t_exhaust_s'], d['speedup'], [s[:2] for s in d['shards']])"
