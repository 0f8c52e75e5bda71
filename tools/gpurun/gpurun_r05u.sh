# round 5, call u: the crack-path differential test at scale -- seeds 1-3, 1,200 lines over 300 ESSIDs each, both
# nonce windows (tests/test_gpu_crack_differential.py), one pytest process per seed.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05u}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for seed in 1 2 3; do
  DWPA_CRACK_DIFF_LINES=1200 DWPA_CRACK_DIFF_SEED=$seed timeout -k 10 400 python3 -u -m pytest \
      tests/test_gpu_crack_differential.py -x -s -v --timeout 380 --timeout-method thread > $O/crack_$seed.log 2>&1
  guard $?
  grep "crack differential" $O/crack_$seed.log
done
