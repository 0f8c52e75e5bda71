# round 4, call i: wordlist expansion through the library (dwpa_rules_expand_file, help_crack's `hashcat --stdout`):
# its tests, then the expand leg at 1M and 5M source words.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04i}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "expand or rules" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; guard $rc
for n in 1000000 5000000; do
  timeout -k 10 300 python3 bench.py --workload expand --rule-words $n --steps 2 --warmup 1 > $O/expand_$n.json 2> $O/expand_$n.err
  guard $?
  python3 -c "import json;d=json.load(open('$O/expand_$n.json'));print($n, d['value'], d['ms_per_step'], d['config']['candidates'], d['config']['output_bytes'], d['hits_verified'])"
done
