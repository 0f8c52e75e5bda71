# round 5, call ap: the lone-wave kernel (k_pbkdf2_ms: one-key calls, C1) without its 8-wave occupancy bound, so the
# j = 2 schedule forms fit in registers (74 VGPRs, 1,095 VALU per loop iteration against 1,125):
# ab/r10_L2 (j <= 2, kernels.hip built with it) and ab/r10_L1u (j <= 1, bound lifted only) against HEAD (r10_cur).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ap}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for v in L2 L1u; do
  DWPA_LIB=$PWD/ab/r10_$v.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
      --timeout-method thread > $O/parity_$v.log 2>&1
  guard $?
  echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
for rep in 1 2; do
  for v in cur L2 L1u; do
    DWPA_LIB=$PWD/ab/r10_$v.so timeout -k 10 200 python3 bench.py --workload c1lat --steps 9 > $O/c1lat_${v}_$rep.json \
        2> $O/c1lat_${v}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c1lat_${v}_$rep.json'));print('c1lat $v $rep', d['value'])"
    DWPA_LIB=$PWD/ab/r10_$v.so timeout -k 10 200 python3 bench.py --workload c1 > $O/c1_${v}_$rep.json \
        2> $O/c1_${v}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c1_${v}_$rep.json'));print('c1 $v $rep', d['value'], d.get('ms_per_step'))"
  done
done
