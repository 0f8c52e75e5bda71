# round 5, call w: the SHA-1 schedule identities (crypto_dev.hpp sched84: W[t] from the recurrence applied 2^j times
# reaches the 84-byte message's zero words, fewer XORs).  Libraries ab/sched_{w0,w1,j73,j75}.so: w0 = the plain
# recurrence (the round's code before), w1 = j <= 1 (-13 VALU per compression, 61 VGPRs), j73 / j75 = also j = 2
# from T = 73 / 75 (-17.5 / -17, 64 / 63 VGPRs).  First bit-exactness with every library (PBKDF2 vectors, random and
# long keys, the C2/C1 checks), then C2's kernel at 4M PMKs per launch, three alternating passes, then the
# one-key latency (c1lat) for w0 and the best candidates.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05w}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for v in w0 w1 j73 j75; do
  DWPA_LIB=$PWD/ab/sched_$v.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
      --timeout-method thread -k "pbkdf2 or challenge or mixed_golden or random_batch" > $O/parity_$v.log 2>&1
  guard $?
  echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
for rep in 1 2 3; do
  for v in w0 w1 j73 j75; do
    DWPA_LIB=$PWD/ab/sched_$v.so timeout -k 10 150 python3 bench.py --batch 4194304 --steps 6 --warmup 1 \
        --no-cpu-baseline --dict-words 30000000 > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c2_${v}_$rep.json'));r=d['roofline'];print('c2 $v $rep', r['kernel_ms'], d['value'], r['frac'], d.get('hits_verified'))"
  done
done
for v in w0 w1 j73; do
  DWPA_LIB=$PWD/ab/sched_$v.so timeout -k 10 200 python3 bench.py --workload c1lat --steps 9 > $O/c1lat_$v.json \
      2> $O/c1lat_$v.err
  guard $?
  python3 -c "import json;d=json.load(open('$O/c1lat_$v.json'));print('c1lat $v', d['value'], [r['gpu_ms_per_call'] for r in d['rows'][:3]])"
done
