# round 5, call q: after the ABI hardening (guarded entry points, exception-safe host pool, DWPA_NC_MAX) and the new
# long-key / ESSID-length parity tests -- the GPU suite, smoke, the default bench line and C5 (host phases changed).
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05q}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
guard $?
tail -1 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
guard $?
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
guard $?
timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
guard $?
for f in bench_default c5; do
  python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), d.get('mismatches'))"
done
