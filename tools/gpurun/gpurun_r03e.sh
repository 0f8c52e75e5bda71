# round 3, call e: the dictionary reader with parallel inflate on the box's host, and the C2 client path
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e
mkdir -p $O
OUT=$O/reader_ab timeout -k 10 600 bash tools/reader_ab.sh > $O/reader_ab.log 2>&1 || { tail -5 $O/reader_ab.log; exit 1; }
DWPA_TRACE=1 timeout -k 10 400 python3 bench.py --workload c2files --steps 1 --warmup 0 > $O/c2files.json 2> $O/c2files.err || exit $?
cat $O/reader_ab/*.json; cat $O/reader_ab/*pcheck*; cat $O/c2files.json
