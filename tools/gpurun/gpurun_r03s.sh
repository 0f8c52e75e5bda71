# round 3, call s: the client's rule pass through dwpa_crack_files (bench.py --workload c3files): 1M-word gz
# dictionary x 148 WPA rules, first pass and a replay from the decoded-dictionary cache.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03s
mkdir -p $O
DWPA_TRACE=1 timeout -k 10 400 python3 bench.py --workload c3files --steps 2 --warmup 0 > $O/c3files.json 2> $O/c3files.err
rc=$?; grep -v "hostname\|amdgpu.ids" $O/c3files.err | tail -12; cat $O/c3files.json; exit $rc
