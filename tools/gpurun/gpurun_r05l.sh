# round 5, call l: the driver's multi-GPU launch form rehearsed on the one GPU at the last code
# (torch.distributed.run, one rank per "GPU", DWPA_BENCH_ONE_DEVICE=1 maps every rank to device 0; control path,
# not a scaling measurement), plus bench.py's own spawn path at N=4.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05l}
mkdir -p $O
export DWPA_BENCH_ONE_DEVICE=1
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --dict-words 2000000 \
    --batch 1048576 > $O/c2_torchrun_n2.json 2> $O/c2_torchrun_n2.err
guard $?
timeout -k 10 300 python3 bench.py --gpus 4 --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --batch 1048576 \
    > $O/c4_spawn_n4.json 2> $O/c4_spawn_n4.err
guard $?
for f in c2_torchrun_n2 c4_spawn_n4; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['n_gpus'], d.get('hits_verified'), d['value'], d['scaling'], d['config'].get('parallelism'))"; done
