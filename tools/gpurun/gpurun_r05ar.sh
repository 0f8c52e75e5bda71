# round 5, call ar: VGPR banks. tools/vgpr_bank.hip (which source-bank patterns cost issue slots), then the issue
# pass's bank renaming (rule sched=1:alt:orig:asmnop:bank,before_half: loop-local values moved so that fewer
# v_bitop3_b32 read two sources from one bank, 99 -> 36 pairs per loop) -- ab/r10_bank against HEAD (ab/r10_cur):
# parity, C2's kernel at 4M PMKs (3 passes) and 196,608 PMKs (2 passes), C5 (one caller, 2 passes).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ar}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 60 ./tools/bin/vgpr_bank 4000 > $O/bank.json 2> $O/bank.err
guard $?
grep '"waves_per_simd": 8' $O/bank.json
DWPA_LIB=$PWD/ab/r10_bank.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread > $O/parity_bank.log 2>&1
guard $?
echo "parity bank: $(tail -1 $O/parity_bank.log)"
for rep in 1 2 3; do
  for v in cur bank; do
    for b in 4194304 196608; do
      [ $rep = 3 ] && [ $b = 196608 ] && continue
      DWPA_LIB=$PWD/ab/r10_$v.so timeout -k 10 150 python3 bench.py --batch $b --steps 6 --warmup 1 \
          --no-cpu-baseline --dict-words 30000000 > $O/c2_${v}_${b}_$rep.json 2> $O/c2_${v}_${b}_$rep.err
      guard $?
      python3 -c "import json;d=json.load(open('$O/c2_${v}_${b}_$rep.json'));r=d['roofline'];print('c2 $v $b $rep', r['kernel_ms'], d.get('hits_verified'))"
    done
  done
done
for rep in 1 2; do
  for v in cur bank; do
    DWPA_LIB=$PWD/ab/r10_$v.so timeout -k 10 200 python3 bench.py --workload c5 > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c5_${v}_$rep.json'));print('c5 $v $rep', d['value'], d.get('mismatches'))"
  done
done
