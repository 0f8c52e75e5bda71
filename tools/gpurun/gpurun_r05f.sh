# round 5, calls f, g (alternating order, a sync between calls, 4 reps) and h (after the SWAR line-break check): the expand leg measured 15.8 s per 740M-candidate expansion in r05e against 10.15 s in round 4.
# Same box, same source, the round-4 library (ab/r04, built from a186d45) against this round's, alternating -- a
# regression or the box?  Output on /tmp and on the repo's own filesystem.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05h}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
df -h /tmp . > $O/df.txt 2>&1
timeout -k 10 600 python3 tools/expand_ab.py ab/r04/libdwpa22000.so dwpa_amd/lib/libdwpa22000.so 4 > $O/ab_tmp.jsonl 2> $O/ab_tmp.err
guard $?
OUT_DIR=$GRAFT_REPO_ROOT/gpurun_scratch timeout -k 10 400 bash -c 'mkdir -p $OUT_DIR && python3 tools/expand_ab.py ab/r04/libdwpa22000.so dwpa_amd/lib/libdwpa22000.so 2' > $O/ab_repo.jsonl 2> $O/ab_repo.err
guard $?
rm -rf $GRAFT_REPO_ROOT/gpurun_scratch
cat $O/df.txt
tail -1 $O/ab_tmp.jsonl
tail -1 $O/ab_repo.jsonl
