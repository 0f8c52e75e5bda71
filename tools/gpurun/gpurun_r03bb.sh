# round 3, call bb: check-path contexts drain their streams before the lock is released (DrainOnExit): check-path GPU
# tests, then C5 one and two callers.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03bb
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "golden or c5 or random or concurrent or mutated or nc_windows or c1 or head_tail or long_eapol" \
    -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; guard $rc
for k in 1 1 2; do
  timeout -k 10 200 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_k$k.json 2> $O/c5_k$k.err
  guard $?
  python3 -c "import json;d=json.load(open('$O/c5_k$k.json'));print('callers $k', d['value'], d['ms_per_step'], d['mismatches'])"
done
