# round 3, call r: HBM traffic of the bench line's kernels at HEAD (tools/profile_traffic.sh: kernel-trace/stats
# pass + FETCH_SIZE and WRITE_SIZE passes, each on its own), C2 shape with 3 timed steps.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03r/traffic_c2 BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline" timeout -k 10 1000 bash tools/profile_traffic.sh \
    > gpurun_out/r03r.log 2>&1
rc=$?; tail -40 gpurun_out/r03r.log; exit $rc
