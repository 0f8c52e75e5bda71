# round 4, call m: C5's PBKDF2 tail cut into sequential pieces at priority 3 ahead of a head at 2..0
# (DWPA_TAIL_PIECES) against the single tail launch beside the head: parity (the split test with 0/8/7 pieces),
# then C5 one and two callers alternating, and a kernel trace of one 8-piece call.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04m}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -k "head_tail_split or c5_mixed" -x -v \
  --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
guard $?
tail -6 $O/pytest.log
for rep in 1 2; do
  for p in 0 8 16 4; do
    DWPA_TAIL_PIECES=$p timeout -k 10 120 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
      > $O/c5_p${p}_k1_r$rep.json 2> $O/c5_p${p}_k1_r$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c5_p${p}_k1_r$rep.json'));print('k1 pieces $p rep $rep', d['value'], d['ms_per_step'], d['mismatches'])"
  done
done
for p in 0 8; do
  DWPA_TAIL_PIECES=$p timeout -k 10 120 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 --no-cpu-baseline \
    > $O/c5_p${p}_k2.json 2> $O/c5_p${p}_k2.err
  guard $?
  python3 -c "import json;d=json.load(open('$O/c5_p${p}_k2.json'));print('k2 pieces $p', d['value'], d['ms_per_step'], d['mismatches'])"
done
DWPA_TAIL_PIECES=8 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --workload c5 --steps 8 --warmup 2 --no-cpu-baseline > $O/c5_prof.json 2> $O/c5_prof.err
guard $?
python3 tools/trace_window.py $O/prof/run_kernel_trace.csv 6 > $O/window6.txt
cut -c1-100 $O/window6.txt
