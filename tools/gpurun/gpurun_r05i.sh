# round 5, call i: the wordlist expansion packed on the GPU (k_text_*) -- its GPU tests, then the A/B against the
# round-4 library (ab/r04) and the bench leg.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05i}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_help_crack.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -k "expand or help_crack or rules" > $O/pytest.log 2>&1
guard $?
tail -3 $O/pytest.log
timeout -k 10 600 python3 tools/expand_ab.py ab/r04/libdwpa22000.so dwpa_amd/lib/libdwpa22000.so 3 > $O/ab_tmp.jsonl 2> $O/ab_tmp.err
guard $?
tail -1 $O/ab_tmp.jsonl
timeout -k 10 300 python3 bench.py --workload expand --rule-words 5000000 --steps 2 --warmup 1 > $O/expand.json 2> $O/expand.err
guard $?
python3 -c "import json;d=json.load(open('$O/expand.json'));print('expand', d['value'], d['ms_per_step'], d['hits_verified'])"
