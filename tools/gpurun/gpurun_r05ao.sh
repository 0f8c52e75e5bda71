# round 5, call ao: the round-end sequence the driver runs, at the final tree: the GPU suite, smoke, the default
# bench line (library byte-identical to final_head/final_verify's).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ao}
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
python3 -c "import json;d=json.load(open('$O/bench_default.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['frac'], r['frac_issue_cost_model'], d['cpu_baseline']['value'], d.get('hits_verified'))"
