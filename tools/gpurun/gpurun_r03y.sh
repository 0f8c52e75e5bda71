# round 3, call y: host phase trace of C5 calls (DWPA_TRACE=1), one caller, to see where the ~1.5 ms of GPU idle per
# call goes at HEAD.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03y
mkdir -p $O
DWPA_TRACE=1 timeout -k 10 200 python3 bench.py --workload c5 --steps 6 --warmup 2 --no-cpu-baseline > $O/c5_trace.json 2> $O/c5_trace.err
rc=$?; grep "\[dwpa\]" $O/c5_trace.err | tail -40; exit $rc
