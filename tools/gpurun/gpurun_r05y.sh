# round 5, call y: at the schedule-identity code -- VALU counters of the PBKDF2 kernel on the bench line's workload
# (two SQ passes), and the issue-pass rule raced again on the new instruction mix (ab/r6_*.so, C2 kernel at 4M PMKs
# per launch, two alternating passes).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05y}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --dict-words 40000000"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv \
    -d $O/pmc1 -o run -- python3 $B > $O/pmc1.json 2> $O/pmc1.err
guard $?
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $O/pmc2 -o run -- python3 $B > $O/pmc2.json 2> $O/pmc2.err
guard $?
python3 tools/pmc_summary.py $(find $O/pmc1 $O/pmc2 -name '*counter_collection.csv') > $O/pmc_summary.txt
cut -c1-300 $O/pmc_summary.txt | head -3
for rep in 1 2; do
  for v in base salt4 s2alt trans; do
    DWPA_LIB=$PWD/ab/r6_$v.so timeout -k 10 150 python3 bench.py --batch 4194304 --steps 6 --warmup 1 \
        --no-cpu-baseline --dict-words 30000000 > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c2_${v}_$rep.json'));r=d['roofline'];print('c2 $v $rep', r['kernel_ms'], d['value'])"
  done
done
