# round 5, call ae: confirmation of call ad -- sched=1:alt (the product) against sched=1:alt:orig, three alternating
# passes at 8 waves (4M PMKs per launch) and at 6 waves (196,608).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05ae}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for rep in 1 2 3; do
  for v in cur orig; do
    for b in 4194304 196608; do
      DWPA_LIB=$PWD/ab/r8_$v.so timeout -k 10 150 python3 bench.py --batch $b --steps 6 --warmup 1 \
          --no-cpu-baseline --dict-words 30000000 > $O/c2_${v}_${b}_$rep.json 2> $O/c2_${v}_${b}_$rep.err
      guard $?
      python3 -c "import json;d=json.load(open('$O/c2_${v}_${b}_$rep.json'));r=d['roofline'];print('c2 $v $b $rep', r['kernel_ms'])"
    done
  done
done
