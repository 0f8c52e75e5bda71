# round 5, call aj: the scheduler's variants on HEAD's j = 2 code -- sched=1:alt:orig (HEAD), sched=2:alt:orig and
# sched=1:alt (critical-path ties), all with asmnop and before_half; C2's kernel at 4M PMKs (3 passes) and 196,608.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05aj}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for rep in 1 2 3; do
  for v in cur s2o cp; do
    for b in 4194304 196608; do
      [ $rep = 3 ] && [ $b = 196608 ] && continue
      DWPA_LIB=$PWD/ab/r11_$v.so timeout -k 10 150 python3 bench.py --batch $b --steps 6 --warmup 1 \
          --no-cpu-baseline --dict-words 30000000 > $O/c2_${v}_${b}_$rep.json 2> $O/c2_${v}_${b}_$rep.err
      guard $?
      python3 -c "import json;d=json.load(open('$O/c2_${v}_${b}_$rep.json'));r=d['roofline'];print('c2 $v $b $rep', r['kernel_ms'])"
    done
  done
done
