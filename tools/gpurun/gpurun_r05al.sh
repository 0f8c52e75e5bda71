# round 5, call al: HEAD's default bench line and smoke once more (bench.py's issued-ops constant changed).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05al}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
guard $?
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
guard $?
python3 -c "import json;d=json.load(open('$O/bench_default.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['frac'], r['frac_issue_cost_model'], r['frac_nominal_ops'], d['cpu_baseline']['value'], d.get('hits_verified'))"
