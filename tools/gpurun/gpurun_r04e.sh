# round 4, call e: segment size of the first-key early exit (DWPA_ATT_SEG_KEYS: keys per attempt-parallel segment,
# default 16) on C5, with the check-path parity tests at the default.
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r04e}
mkdir -p $O
export TMPDIR=/tmp
guard() { case $1 in 0) ;; 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; *) echo "fail: rc $1" >&2; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py \
    -k "golden or c5 or random_batch or nc_windows or batch" -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.txt)"; guard $rc
for seg in 16 64 32 8 16; do
  DWPA_ATT_SEG_KEYS=$seg timeout -k 10 150 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
      > $O/c5_seg${seg}.json 2> $O/c5_seg${seg}.err
  guard $?
  echo "seg=$seg callers=1 $(python3 -c "import json;d=json.load(open('$O/c5_seg${seg}.json'));print(d['value'], d['ms_per_step'], d['hits_verified'], d['mismatches'])")"
done
timeout -k 10 150 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5_k2.json 2> $O/c5_k2.err
guard $?
echo "seg=16 callers=2 $(python3 -c "import json;d=json.load(open('$O/c5_k2.json'));print(d['value'], d['ms_per_step'], d['hits_verified'], d['mismatches'])")"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv \
    -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc.log 2>&1
guard $?
python3 - <<PY
import csv
from collections import defaultdict
for kern in ('<8u>', '<6u>'):
    agg = defaultdict(float); t = {}
    for r in csv.DictReader(open('$O/pmc/run_counter_collection.csv')):
        if 'verify_att' in r['Kernel_Name'] and kern in r['Kernel_Name']:
            agg[r['Counter_Name']] += float(r['Counter_Value'])
            t[r['Dispatch_Id']] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    print('verify_att' + kern, {k: int(v) for k, v in agg.items()}, 'ms per dispatch', sorted(t.values()))
PY
