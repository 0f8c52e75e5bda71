# round 4, call d: C5's post-head phase.
#   * first-key early exit of the attempt-parallel verify (DWPA_FIRST_KEY_EXIT, default on) against off;
#   * keyver-3 AES layout: 1 = lane-sliced Te0 x32 (default), 3 = Te0 + Te1 x16 (one rotate per column instead of
#     three, 2-way bank conflicts).
# Per library: check-path parity tests, C5 with one and two callers, one PMC pass (SQ_INSTS_VALU, LDS bank
# conflicts) over C5.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04d}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
for lib in aes1 aes1_noexit aes3; do
  L=$PWD/ab/${lib%_noexit}.so
  if [ "$lib" = aes1_noexit ]; then export DWPA_FIRST_KEY_EXIT=0; else export DWPA_FIRST_KEY_EXIT=1; fi
  DWPA_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py \
      -k "golden or c5 or random_batch or nc_windows or batch" -x -q --timeout 200 --timeout-method thread > $O/pytest_$lib.txt 2>&1
  rc=$?; echo "$lib pytest rc=$rc $(tail -1 $O/pytest_$lib.txt)"; guard $rc
  for k in 1 2; do
    DWPA_LIB=$L timeout -k 10 150 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 --no-cpu-baseline \
        > $O/c5_${lib}_k$k.json 2> $O/c5_${lib}_k$k.err
    guard $?
    echo "$lib callers=$k $(python3 -c "import json;d=json.load(open('$O/c5_${lib}_k$k.json'));print(d['value'], d['ms_per_step'], d['hits_verified'], d['mismatches'])")"
  done
  DWPA_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_$lib -o run --output-format csv \
      -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_$lib.log 2>&1
  guard $?
  python3 - <<PY
import csv
from collections import defaultdict
agg = defaultdict(float); t = defaultdict(list)
for r in csv.DictReader(open('$O/pmc_$lib/run_counter_collection.csv')):
    if 'verify_att' in r['Kernel_Name'] and '<8u>' in r['Kernel_Name']:
        agg[r['Counter_Name']] += float(r['Counter_Value'])
        t[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
print('$lib kv3 verify:', {k: int(v) for k, v in agg.items()}, 'ms per dispatch', sorted(t.values()))
PY
done
