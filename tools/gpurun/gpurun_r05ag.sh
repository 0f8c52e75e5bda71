# round 5, call ag: the j = 2 schedule forms again, now with the list scheduler (rule
# sched=1:alt:orig:asmnop,before_half: LLVM's s_nop after inline asm dropped first) -- ab/r9_j73 / r9_j75 against
# the product (r9_cur): PBKDF2 parity, C2's kernel at 4M PMKs (3 passes) and 196,608 PMKs (2 passes), the one-key call.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ag}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for v in j73 j75; do
  DWPA_LIB=$PWD/ab/r9_$v.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
      --timeout-method thread -k "pbkdf2 or challenge or mixed_golden or random_batch" > $O/parity_$v.log 2>&1
  guard $?
  echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
for rep in 1 2 3; do
  for v in cur j73 j75; do
    for b in 4194304 196608; do
      [ $rep = 3 ] && [ $b = 196608 ] && continue
      DWPA_LIB=$PWD/ab/r9_$v.so timeout -k 10 150 python3 bench.py --batch $b --steps 6 --warmup 1 \
          --no-cpu-baseline --dict-words 30000000 > $O/c2_${v}_${b}_$rep.json 2> $O/c2_${v}_${b}_$rep.err
      guard $?
      python3 -c "import json;d=json.load(open('$O/c2_${v}_${b}_$rep.json'));r=d['roofline'];print('c2 $v $b $rep', r['kernel_ms'], d.get('hits_verified'))"
    done
  done
done
for v in cur j73; do
  DWPA_LIB=$PWD/ab/r9_$v.so timeout -k 10 200 python3 bench.py --workload c1lat --steps 9 > $O/c1lat_$v.json \
      2> $O/c1lat_$v.err
  guard $?
  python3 -c "import json;d=json.load(open('$O/c1lat_$v.json'));print('c1lat $v', d['value'])"
done
