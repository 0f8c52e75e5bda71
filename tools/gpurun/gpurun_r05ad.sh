# round 5, call ad: the list scheduler's tie-break -- critical path (the product, sched=1:alt) against the compiler's
# order (sched=1:alt:orig, sched=2:alt:orig), C2's kernel at 4M PMKs per launch, two alternating passes.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ad}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for rep in 1 2; do
  for v in cur orig s2orig; do
    DWPA_LIB=$PWD/ab/r8_$v.so timeout -k 10 150 python3 bench.py --batch 4194304 --steps 6 --warmup 1 \
        --no-cpu-baseline --dict-words 30000000 > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c2_${v}_$rep.json'));r=d['roofline'];print('c2 $v $rep', r['kernel_ms'], d['value'])"
  done
done
