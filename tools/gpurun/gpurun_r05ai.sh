# round 5, call ai: C5 with one and two callers, the j = 2 issue-pass kernels (ab/r10_head.so = HEAD) against j <= 1
# (ab/r9_cur.so), two alternating passes -- call ah read 4.148 M with one caller but 4.049 M with two.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ai}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for rep in 1 2; do
  for v in r10_head r9_cur; do
    DWPA_LIB=$PWD/ab/$v.so timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
        > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err
    guard $?
    DWPA_LIB=$PWD/ab/$v.so timeout -k 10 200 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 \
        --no-cpu-baseline > $O/c5k2_${v}_$rep.json 2> $O/c5k2_${v}_$rep.err
    guard $?
    python3 -c "import json;a=json.load(open('$O/c5_${v}_$rep.json'));b=json.load(open('$O/c5k2_${v}_$rep.json'));print('$v $rep', a['value'], a['mismatches'], b['value'], b['mismatches'])"
  done
done
