# round 5, call an: the PBKDF2 loop unrolled to two iterations per trip (DWPA_PBKDF2_UNROLL2, non-priority kernels:
# one issue-pass block of 4 compressions, 2,226 VALU against 2 x 1,116) -- ab/r10_u2 against HEAD (ab/r10_cur):
# PBKDF2 parity, C2's kernel at 4M PMKs (3 passes) and 196,608 PMKs (2 passes), C3.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05an}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
DWPA_LIB=$PWD/ab/r10_u2.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread -k "pbkdf2 or challenge or mixed_golden or random_batch" > $O/parity_u2.log 2>&1
guard $?
echo "parity u2: $(tail -1 $O/parity_u2.log)"
for rep in 1 2 3; do
  for v in cur u2; do
    for b in 4194304 196608; do
      [ $rep = 3 ] && [ $b = 196608 ] && continue
      DWPA_LIB=$PWD/ab/r10_$v.so timeout -k 10 150 python3 bench.py --batch $b --steps 6 --warmup 1 \
          --no-cpu-baseline --dict-words 30000000 > $O/c2_${v}_${b}_$rep.json 2> $O/c2_${v}_${b}_$rep.err
      guard $?
      python3 -c "import json;d=json.load(open('$O/c2_${v}_${b}_$rep.json'));r=d['roofline'];print('c2 $v $b $rep', r['kernel_ms'], d.get('hits_verified'))"
    done
  done
done
for v in cur u2; do
  DWPA_LIB=$PWD/ab/r10_$v.so timeout -k 10 200 python3 bench.py --workload c3 > $O/c3_$v.json 2> $O/c3_$v.err
  guard $?
  python3 -c "import json;d=json.load(open('$O/c3_$v.json'));print('c3 $v', d['value'])"
done
