# round 5, call r: the differential test at scale -- 6 x 10,000 mixed check jobs (seeds 1-6) through the HIP path,
# every result tuple against the oracle (tests/test_gpu_differential.py), one pytest process per seed so that each
# prints its line when it ends.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05r}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for seed in 1 2 3 4 5 6; do
  DWPA_DIFF_JOBS=10000 DWPA_DIFF_SEED=$seed timeout -k 10 400 python3 -u -m pytest tests/test_gpu_differential.py \
      -x -s -q --timeout 380 --timeout-method thread > $O/diff_$seed.log 2>&1
  guard $?
  grep "differential:" $O/diff_$seed.log
done
