# round 3, call v: the 8-device crack_files control path rehearsed on one GPU (DWPA_CRACK_SHARDS_PER_DEVICE=8: 8
# shard workers, each a stager + scanner thread, one shared item queue), C2 shape via a 20M-word gz dictionary, and
# the client rule pass with 8 workers.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03v
mkdir -p $O
export DWPA_TRACE=1 DWPA_CRACK_SHARDS_PER_DEVICE=8
timeout -k 10 400 python3 bench.py --workload c2files --dict-words 20000000 --steps 1 --warmup 1 > $O/c2files_w8.json 2> $O/c2files_w8.err
rc=$?; grep "crack worker\|cache" $O/c2files_w8.err | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --workload c3files --rule-words 300000 --steps 1 --warmup 0 > $O/c3files_w8.json 2> $O/c3files_w8.err
rc=$?; grep "crack worker" $O/c3files_w8.err | tail -10
for f in c2files_w8 c3files_w8; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['pass_s'], d['hits_verified'])"; done
exit $rc
