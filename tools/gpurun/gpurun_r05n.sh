# round 5, call n: issue-pass rules at low occupancy.  The C5 head runs 6 waves per SIMD and takes 7% longer per
# wave-time than an 8-wave launch (profiles/r05/head_deficit/).  The rule (before_half) was raced at 8 waves in
# round 1; here every rule variant (ab/w6_*.so, tools/pbkdf2_rule_ab.sh) runs C2's kernel at 6, 7 and 8 waves per
# SIMD (196,608 / 229,376 / 262,144 PMKs per launch), two alternating passes.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05n}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for rep in 1 2; do
  for v in base nop1 trans salt4 s8 split s6g; do
    for b in 196608 229376 262144; do
      DWPA_LIB=$PWD/ab/w6_$v.so timeout -k 10 120 python3 bench.py --batch $b --steps 30 --warmup 2 --no-cpu-baseline \
          --dict-words 2000000 > $O/${v}_${b}_$rep.json 2> $O/${v}_${b}_$rep.err
      guard $?
      python3 -c "import json;d=json.load(open('$O/${v}_${b}_$rep.json'));r=d['roofline'];print('$v $b $rep', r['kernel_ms'], d['ms_per_step'])"
    done
  done
done
