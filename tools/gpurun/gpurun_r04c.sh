# round 4, call c: GPU suite at HEAD (rule language, lone-wave padding), c1lat with the caller-PMK rows, a short
# default bench line with the new roofline and CPU baseline objects.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04c}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; guard $rc
timeout -k 10 300 python3 bench.py --workload c1lat --steps 9 > $O/c1lat.json 2> $O/c1lat.err
guard $?
python3 -c "
import json; d=json.load(open('$O/c1lat.json'))
for r in d['rows']: print('%-100s %8.3f %8.3f %s' % (r['call'][:100], r['gpu_ms_per_call'], r['cpu_1core_ms_per_call'], r['same_result']))"
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 > $O/bench_short.json 2> $O/bench_short.err
guard $?
python3 -c "
import json; d=json.load(open('$O/bench_short.json')); r=d['roofline']; c=d['cpu_baseline']
print(d['value'], r['frac'], r['frac_issue_cost_model'], r['frac_attainable_on_gfx950'], c['value'], c['one_thread']['value'], c['all_host'])"
