# round 5, call ak (ah again after the verifiers took the folded pad and outer compressions: MsgKey, sha1_84 for HMAC outer hashes): validation at the round's code -- the GPU suite, smoke, the driver's default bench command, its
# rocprofv3 kernel statistics, then every BASELINE leg (tools/bench_legs.sh, including the server rule set under
# both rule loaders).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ak}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
guard $?
tail -2 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
guard $?
cat $O/smoke.log
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
guard $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_rocprof -o run -- python3 bench.py \
    --steps 5 --warmup 1 --no-cpu-baseline > $O/c2_rocprof.json 2> $O/c2_rocprof.err
guard $?
cut -c1-150 $O/c2_rocprof/run_kernel_stats.csv | head -6
for f in bench_default c2_rocprof; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['unit'], (d.get('roofline') or {}).get('frac'), d.get('hits_verified'))"; done
OUT=$O/legs LEGS="c4 c3 c5 c5k2 c1 c1lat c2files c2files_warm c3files c3files_server c3files_server_full expand" \
    bash tools/bench_legs.sh
guard $?
for f in $O/legs/*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f'.split('/')[-1], d['value'], d['unit'], d.get('hits_verified'), d.get('mismatches'))"; done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_rocprof -o run -- python3 bench.py \
    --workload c5 --steps 12 --warmup 2 --no-cpu-baseline > $O/c5_rocprof.json 2> $O/c5_rocprof.err
guard $?
cut -c1-120 $O/c5_rocprof/run_kernel_stats.csv | head -12
