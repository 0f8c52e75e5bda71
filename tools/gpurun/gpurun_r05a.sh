# round 5, call a: the round's first GPU pass -- the whole GPU suite (new: help_crack install() end to end, the
# hashcat -r loader mode, raw --stdout, first-key exit across chunks), smoke, then the tail head-done flag:
# C5 with the tail raising itself (DWPA_TAIL_PRIO=2, the polled flag now read with an atomic RMW) against never
# (0), alternating, each line carrying dwpa_check_last_stats (tail waves, tail waves raised).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05a}
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
guard $?
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
guard $?
cat $O/smoke.log
for rep in 1 2; do
  for p in 2 0; do
    DWPA_TAIL_PRIO=$p timeout -k 10 180 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
        > $O/c5_prio${p}_$rep.json 2> $O/c5_prio${p}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c5_prio${p}_$rep.json'));print('prio $p rep $rep', d['value'], d['ms_per_step'], d['mismatches'], d['last_call'])"
  done
done
