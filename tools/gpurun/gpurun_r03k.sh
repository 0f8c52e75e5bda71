# round 3, call k: every bench leg at HEAD (tools/bench_legs.sh) after the GPU suite, plus the N=8 one-GPU rehearsal
# of the weak-scaling spawn path (stdout must be the JSON line alone).
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03k
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; guard $rc
OUT=$O/legs timeout -k 10 2400 bash tools/bench_legs.sh > $O/legs.log 2>&1
rc=$?; tail -3 $O/legs.log; guard $rc
DWPA_BENCH_ONE_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline \
    --dict-words 2000000 --batch 1048576 > $O/c2_n8_rehearsal.json 2> $O/c2_n8_rehearsal.err
guard $?
wc -l $O/c2_n8_rehearsal.json
for f in $O/legs/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f', d.get('value'), d.get('ms_per_step'), d.get('hits_verified'), d.get('mismatches'))"; done
