# round 3, call t: degenerate client-path inputs (empty / ragged dictionaries and hash files, filter edges)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "degenerate" -x -v --timeout 240 \
    --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -30 $O/pytest.log; exit $rc
