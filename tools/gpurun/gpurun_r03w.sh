# round 3, call w: crack_files work balance across shard workers after the guided-self-scheduling change: the
# 8-worker one-GPU rehearsal of call v again (c2files 20M words, c3files 300k words), then 2 workers on the 100M c2files
# dictionary, then the one-worker c2files/c3files legs (unchanged path) and the crack-path GPU tests.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03w
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
export DWPA_TRACE=1
DWPA_CRACK_SHARDS_PER_DEVICE=8 timeout -k 10 400 python3 bench.py --workload c2files --dict-words 20000000 --steps 1 --warmup 1 > $O/c2files_w8.json 2> $O/c2files_w8.err
guard $?; grep "crack worker" $O/c2files_w8.err | tail -8
DWPA_CRACK_SHARDS_PER_DEVICE=8 timeout -k 10 400 python3 bench.py --workload c3files --rule-words 300000 --steps 1 --warmup 0 > $O/c3files_w8.json 2> $O/c3files_w8.err
guard $?; grep "crack worker" $O/c3files_w8.err | tail -8
DWPA_CRACK_SHARDS_PER_DEVICE=2 timeout -k 10 400 python3 bench.py --workload c2files --steps 1 --warmup 0 > $O/c2files_w2.json 2> $O/c2files_w2.err
guard $?; grep "crack worker" $O/c2files_w2.err | tail -2
timeout -k 10 400 python3 bench.py --workload c2files --steps 1 --warmup 0 > $O/c2files_w1.json 2> $O/c2files_w1.err
guard $?
timeout -k 10 400 python3 bench.py --workload c3files --steps 1 --warmup 0 > $O/c3files_w1.json 2> $O/c3files_w1.err
guard $?
for f in c2files_w8 c3files_w8 c2files_w2 c2files_w1 c3files_w1; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['pass_s'], d['hits_verified'])"; done
unset DWPA_TRACE
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "crack or help_crack" -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; exit $rc
