# round 4, call o: HBM traffic of the bench line's kernel at the round's last code (tools/profile_traffic.sh:
# FETCH_SIZE and WRITE_SIZE in passes of their own, plus a kernel-trace/stats pass of the same command).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04o/traffic_c2 BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline" timeout -k 10 1000 bash tools/profile_traffic.sh
