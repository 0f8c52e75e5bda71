# round 5, call k: flakiness check -- the whole GPU suite twice more in fresh processes at the round's last code.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05k}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for rep in 1 2; do
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_$rep.log 2>&1
  guard $?
  tail -1 $O/pytest_$rep.log
done
