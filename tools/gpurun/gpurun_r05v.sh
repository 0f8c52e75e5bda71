# round 5, call v: after the Python nc guard and bench's device selection -- the GPU suite, smoke, the default bench
# line, and the driver's torch.distributed.run form at N=2 on the one GPU (DWPA_BENCH_ONE_DEVICE=1, control path).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05v}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
guard $?
tail -1 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
guard $?
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
guard $?
DWPA_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
    --dict-words 2000000 --batch 1048576 > $O/c2_torchrun_n2.json 2> $O/c2_torchrun_n2.err
guard $?
for f in bench_default c2_torchrun_n2; do
  python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['n_gpus'], d['value'], (d.get('roofline') or {}).get('frac'), d.get('hits_verified'))"
done
