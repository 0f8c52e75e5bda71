# round 3, call cc: C5 host phases with the pool's workers polling 300 us before they sleep (default) against
# sleeping at once (DWPA_POOL_SPIN_US=0, the previous behaviour), one caller, interleaved; then the phase traces.
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03cc
mkdir -p $O
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for rep in 1 2 3; do
  for spin in 0 300; do
    DWPA_POOL_SPIN_US=$spin timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_s${spin}_$rep.json 2> $O/c5_s${spin}_$rep.err
    guard $?
    python3 -c "import json;d=json.load(open('$O/c5_s${spin}_$rep.json'));print('spin $spin rep $rep', d['value'], d['ms_per_step'], d['mismatches'])"
  done
done
for spin in 0 300; do
  DWPA_TRACE=1 DWPA_POOL_SPIN_US=$spin timeout -k 10 200 python3 bench.py --workload c5 --steps 4 --warmup 2 --no-cpu-baseline > $O/trace_s$spin.json 2> $O/trace_s$spin.err
  guard $?
  echo "spin $spin"; grep "\[dwpa\]" $O/trace_s$spin.err | tail -11
done
timeout -k 10 200 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_k2.json 2> $O/c5_k2.err
guard $?
python3 -c "import json;d=json.load(open('$O/c5_k2.json'));print('callers 2', d['value'], d['ms_per_step'], d['mismatches'])"
