# round 4, call y: end-of-round validation at the last code -- GPU suite, smoke, the default bench line (what the
# driver runs), the same command under rocprofv3 --kernel-trace --stats, C5 one and two callers, server latency.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04y}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 480 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
guard $?
tail -2 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
guard $?
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
guard $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_rocprof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/c2_rocprof.json 2> $O/c2_rocprof.err
guard $?
timeout -k 10 240 python3 bench.py --workload c5 --steps 20 --warmup 3 > $O/c5_k1.json 2> $O/c5_k1.err
guard $?
timeout -k 10 240 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_k2.json 2> $O/c5_k2.err
guard $?
timeout -k 10 240 python3 bench.py --workload c1lat --steps 9 > $O/c1lat.json 2> $O/c1lat.err
guard $?
for f in bench_default c2_rocprof c5_k1 c5_k2 c1lat; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['unit'], (d.get('roofline') or {}).get('frac'), d.get('mismatches'))"; done
