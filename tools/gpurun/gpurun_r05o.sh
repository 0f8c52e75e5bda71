# round 5, call o: the GPU suite and smoke at the current code (warning cleanups: no code change expected), then
# the PBKDF2 kernel's counters at the round's last code -- VALU issue (two SQ passes) and HBM traffic (FETCH_SIZE /
# WRITE_SIZE passes, MI355X_MICROARCH.md's recipe, tools/profile_traffic.sh) on the bench line's workload.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05o}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
guard $?
tail -1 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
guard $?
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --dict-words 40000000"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv \
    -d $O/pmc1 -o run -- python3 $B > $O/pmc1.json 2> $O/pmc1.err
guard $?
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $O/pmc2 -o run -- python3 $B > $O/pmc2.json 2> $O/pmc2.err
guard $?
OUT=$O/traffic BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --dict-words 40000000" timeout -k 10 700 \
    bash tools/profile_traffic.sh > $O/traffic.log 2>&1
guard $?
python3 tools/pmc_summary.py $(find $O/pmc1 $O/pmc2 -name '*counter_collection.csv') > $O/pmc_summary.txt
cat $O/pmc_summary.txt | cut -c1-400
cat $O/traffic/traffic.json
