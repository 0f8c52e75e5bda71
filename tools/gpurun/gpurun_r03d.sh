# round 3, call d: LDS counters of the keyver-3 verify (new lane-sliced Te0 vs the round-2 tables), and a kernel
# trace of the small-call latency leg.  Each counter pass in its own run (kernels serialized: times alone).
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
B="bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline"
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $C -d $O/pmc_aes1 -o run --output-format csv -- python3 $B > $O/pmc_aes1.log 2>&1 || exit $?
DWPA_LIB=$PWD/ab/aes0.so timeout -s KILL 150 rocprofv3 --pmc $C -d $O/pmc_aes0 -o run --output-format csv -- python3 $B > $O/pmc_aes0.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c1lat_trace -o run -- python3 bench.py --workload c1lat --steps 5 > $O/c1lat.json 2> $O/c1lat.err || exit $?
echo ok
