set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r03a/pytest.log 2>&1 || { tail -30 gpurun_out/r03a/pytest.log; exit 1; }
tail -3 gpurun_out/r03a/pytest.log
timeout -k 10 200 python bench.py --workload c4 --scaling strong --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03a/c4_strong_g1.json 2> gpurun_out/r03a/c4_strong_g1.err
T1=$(python -c "import json;print(json.load(open('gpurun_out/r03a/c4_strong_g1.json'))['t_exhaust_s'])")
echo T1=$T1
DWPA_BENCH_ONE_DEVICE=1 timeout -k 10 200 python bench.py --gpus 2 --workload c4 --scaling strong --steps 1 --warmup 1 --no-cpu-baseline --t1-s $T1 > gpurun_out/r03a/c4_strong_g2_one_device.json 2> gpurun_out/r03a/c4_strong_g2.err
timeout -k 10 240 python bench.py --workload c5 --steps 10 --warmup 2 > gpurun_out/r03a/c5.json 2> gpurun_out/r03a/c5.err
cat gpurun_out/r03a/*.json
