# round 4, call g: PBKDF2 loop schedules for LONE waves (one-key calls, C1, the C5 tail run one wave per SIMD):
# tools/bin/asm_lab races issue-pass variants (tools/asm/build_variants.sh) at 2 lone waves, 1 wave per SIMD and
# full occupancy, outputs compared word for word with the first variant.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04g}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
V="none before_half before_half_trans sched_2:group sched_2:group_before_half_trans sched_1:group sched_1:group_before_half_trans sched_3:group_before_half_trans sched_2:alt"
H=""; for v in $V; do H="$H tools/bin/asm/$v.hsaco"; done
for n in 64 32768 4194304; do
  r=5; [ $n -gt 100000 ] && r=2
  timeout -k 10 200 tools/bin/asm_lab $n $r $H > $O/lab_$n.json 2> $O/lab_$n.err
  guard $?
  python3 -c "
import json; d=json.load(open('$O/lab_$n.json'))
for v in d['variants']: print($n, '%-45s %9.3f ms %s' % (v['hsaco'].split('/')[-1], v['best_ms'], v['matches_first']))"
done
