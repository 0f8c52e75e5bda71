# round 3, call m: mutation fuzz of the parse semantics and the longest EAPOL frames, GPU path vs the oracle
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "mutated or long_eapol" -x -v --timeout 240 \
    --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; exit $rc
