# round 4, call f: GPU suite at HEAD (rule fuzz, early exit), the client rule pass with the WPA set and with the
# server set (the rest of hashcat's rule language), C5 one / two callers.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04f}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; guard $rc
for set in wpa server; do
  DWPA_TRACE=1 timeout -k 10 400 python3 bench.py --workload c3files --rules-set $set --steps 2 --warmup 0 \
      > $O/c3files_$set.json 2> $O/c3files_$set.err
  guard $?
  python3 -c "import json;d=json.load(open('$O/c3files_$set.json'));c=d['config'];print('c3files $set', d['value'], d['pass_s'], c['rules'], c['rules_loaded_skipped'], c['candidates_per_pass'], c['candidates_reported_by_library'], d['hits_verified'])"
done
for k in 1 2; do
  timeout -k 10 150 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_k$k.json 2> $O/c5_k$k.err
  guard $?
  python3 -c "import json;d=json.load(open('$O/c5_k$k.json'));print('c5 callers=$k', d['value'], d['ms_per_step'], d['hits_verified'], d['mismatches'])"
done
