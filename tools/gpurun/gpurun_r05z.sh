# round 5, call z: the issue pass's list scheduler (rule sched=D:alt before before_half) on the schedule-identity
# code, where call y found sched=2:alt 0.9 % faster than before_half alone.  D = 1..4 with alternation, D = 2 without,
# against the product rule: C2's kernel at 4M PMKs per launch (8 waves) and at 196,608 (6 waves, the C5 head's
# occupancy), two alternating passes.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05z}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for rep in 1 2; do
  for v in base s1alt s2alt s3alt s4alt s2; do
    for b in 4194304 196608; do
      DWPA_LIB=$PWD/ab/r6_$v.so timeout -k 10 150 python3 bench.py --batch $b --steps 6 --warmup 1 \
          --no-cpu-baseline --dict-words 30000000 > $O/c2_${v}_${b}_$rep.json 2> $O/c2_${v}_${b}_$rep.err
      guard $?
      python3 -c "import json;d=json.load(open('$O/c2_${v}_${b}_$rep.json'));r=d['roofline'];print('c2 $v $b $rep', r['kernel_ms'], d['value'])"
    done
  done
done
