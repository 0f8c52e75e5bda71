# round 5, call am (ac again at HEAD, after the verifiers took the folded compressions) -- the check-path
# differential test at scale (3 x 10,000 jobs), the crack-path differential (2 x 1,200 lines), and the PBKDF2 kernel's
# VALU counters on the bench line's workload.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05am}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for seed in 21 22 23; do
  DWPA_DIFF_JOBS=10000 DWPA_DIFF_SEED=$seed timeout -k 10 400 python3 -u -m pytest tests/test_gpu_differential.py \
      -x -s -q --timeout 380 --timeout-method thread > $O/diff_$seed.log 2>&1
  guard $?
  grep "differential:" $O/diff_$seed.log
done
for seed in 21 22; do
  DWPA_CRACK_DIFF_LINES=1200 DWPA_CRACK_DIFF_SEED=$seed timeout -k 10 400 python3 -u -m pytest \
      tests/test_gpu_crack_differential.py -x -s -v --timeout 380 --timeout-method thread > $O/crack_$seed.log 2>&1
  guard $?
  grep "crack differential" $O/crack_$seed.log
done
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --dict-words 40000000"
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv \
    -d $O/pmc1 -o run -- python3 $B > $O/pmc1.json 2> $O/pmc1.err
guard $?
python3 tools/pmc_summary.py $(find $O/pmc1 -name '*counter_collection.csv') > $O/pmc_summary.txt
cut -c1-250 $O/pmc_summary.txt | head -2
