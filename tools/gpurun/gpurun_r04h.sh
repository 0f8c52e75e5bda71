# round 4, call h: validation at HEAD -- GPU suite, smoke, the default bench line (what the driver runs), the bench
# command under rocprofv3 --kernel-trace --stats, C5 one and two callers, server call latency.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04h}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; guard $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; guard $rc
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
guard $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_rocprof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline \
    > $O/c2_rocprof.json 2> $O/c2_rocprof.err
guard $?
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_k$k.json 2> $O/c5_k$k.err
  guard $?
done
timeout -k 10 300 python3 bench.py --workload c1lat --steps 9 > $O/c1lat.json 2> $O/c1lat.err
guard $?
for f in bench_default c2_rocprof c5_k1 c5_k2; do python3 -c "import json;d=json.load(open('$O/$f.json'));r=d.get('roofline') or {};print('$f', d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('frac'), r.get('frac_issue_cost_model'), d['hits_verified'], d.get('mismatches'))"; done
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print(json.dumps(d['cpu_baseline'])[:600])"
cut -c1-150 $O/c2_rocprof/run_kernel_stats.csv
