# round 3, call u: dwpa_crack_last_stats and the drop-in's end-of-run block, then the whole GPU suite
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "last_stats" -x -v --timeout 240 \
    --timeout-method thread > $O/stats.log 2>&1
rc=$?; tail -15 $O/stats.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; exit $rc
