# round 4, call t: why the chunked derive stalls (r04s: the split test at 16 chunks ran past its 60 s limit).
# One process per setting, each under its own limit: 0 (head/tail split), 1 (no waits at all), 2, 16.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04t}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for c in 0 1 2 16; do
  DWPA_CHECK_CHUNKS=$c timeout -k 10 60 python3 tools/chunked_probe.py >> $O/probe.txt 2>&1
  guard $?
done
cat $O/probe.txt
