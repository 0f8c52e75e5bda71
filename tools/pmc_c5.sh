#!/bin/bash
# SQ counter passes over the C5 check path (kernels run serialized under --pmc, so each dispatch's timestamps are
# its time alone).  Two passes, each within the per-block counter limits.  OUT defaults to gpurun_out/pmc_c5.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pmc_c5}
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/p1 -o run --output-format csv -- python3 $B \
    > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU \
    SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY -d $OUT/p2 -o run --output-format csv -- python3 $B > $OUT/p2.log 2>&1
python3 tools/pmc_summary.py $OUT/p1/run_counter_collection.csv $OUT/p2/run_counter_collection.csv > $OUT/summary.txt
