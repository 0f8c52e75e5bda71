# round 4, call k: the round's full measurement on one box, in two parts (one call each, PART=1|2):
#   1: GPU suite, smoke, then the in-memory bench legs (tools/bench_legs.sh)
#   2: the file legs (gz dictionaries, rules, expansion), a rocprofv3 kernel-trace summary of the default bench, and
#      the C5 test with every one of its 1,010 jobs prefix-checked against the oracle (DWPA_FULL_ORACLE=1)
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04k}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  guard $?
  tail -3 $O/pytest.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  guard $?
  LEGS="peak c2 c4 c4strong c3 c5 c5k2 c1 c1lat" OUT=$O/legs timeout -k 10 900 bash tools/bench_legs.sh
  guard $?
else
  LEGS="c2files c2files_warm c3files c3files_server expand" OUT=$O/legs timeout -k 10 700 bash tools/bench_legs.sh
  guard $?
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err
  guard $?
  DWPA_FULL_ORACLE=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -k c5_mixed -x -v -s --timeout 380 \
    --timeout-method thread > $O/c5_full_oracle_pytest.txt 2>&1
  guard $?
  grep -h "DWPA_FULL_ORACLE\|passed\|failed" $O/c5_full_oracle_pytest.txt
fi
for f in $O/legs/*.json; do echo "$f $(python3 -c "import json;d=json.load(open('$f'));print(d.get('value'),d.get('unit'))" 2>/dev/null)"; done
