# round 3, call p: PBKDF2 issue-pass A/B -- every v_add3_u32 of the main loop split into two v_add_u32 (fewer
# 4-cycle ops, same additive cost), with nops before each alignbit / none / only before a 2->4-cycle transition.
# Parity of the split build first, then C2 bench lines interleaved.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03p
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for lib in split split_nonop split_trans; do
  DWPA_LIB=$PWD/ab/$lib.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "pbkdf2 or issue_pass or challenge" \
      -x -q --timeout 150 --timeout-method thread > $O/pytest_$lib.log 2>&1
  rc=$?; echo "$lib parity: $(tail -1 $O/pytest_$lib.log)"; guard $rc
done
for rep in 1 2; do
  for lib in base split split_nonop split_trans; do
    DWPA_LIB=$PWD/ab/$lib.so timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline \
        > $O/c2_${lib}_$rep.json 2> $O/c2_${lib}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c2_${lib}_$rep.json'));r=d['roofline'];print('$lib rep$rep', d['value'], r['kernel_ms'], r['frac'], d['hits_verified'])"
  done
done
