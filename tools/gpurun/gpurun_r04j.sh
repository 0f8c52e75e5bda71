# round 4, call j: where a C5 call's time goes now (first-key early exit on): host phases (DWPA_TRACE) and a kernel
# trace of the same command.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04j}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
DWPA_TRACE=1 timeout -k 10 150 python3 bench.py --workload c5 --steps 8 --warmup 2 --no-cpu-baseline > $O/c5_trace.json 2> $O/c5_trace.txt
guard $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --workload c5 --steps 8 --warmup 2 --no-cpu-baseline > $O/c5_prof.json 2> $O/c5_prof.err
guard $?
python3 tools/trace_window.py $O/prof/run_kernel_trace.csv 6 > $O/window6.txt
cat $O/window6.txt | cut -c1-100
tail -24 $O/c5_trace.txt
