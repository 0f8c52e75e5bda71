#!/bin/bash
# Keyver-3 verify A/B: AES T-tables with S interleaved copies per table (ab/s8.so, ab/s16.so: -DDWPA_KV3_SLICES=S,
# 512-thread workgroups) vs the plain tables (ab/base.so).  Parity tests on each variant, bench lines + traces
# (tools/lib_ab.sh, each library twice), and one SQ/LDS counter pass per library (kernels serialized).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/kv3_slices}
mkdir -p $OUT
export TMPDIR=/tmp
for lib in s8 s16; do
  DWPA_LIB=$PWD/ab/$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py \
      -k "golden or random or c5 or dedup or challenge" -x -v --timeout 200 --timeout-method thread \
      > $OUT/pytest_$lib.txt 2>&1
done
LIBS="ab/base.so ab/s8.so ab/s16.so ab/baseb.so ab/s8b.so ab/s16b.so" WORKLOAD=c5 OUT=$OUT STEPS=20 \
    timeout -k 10 700 tools/lib_ab.sh > $OUT/ab.log 2>&1
for lib in base s8 s16; do
  DWPA_LIB=$PWD/ab/$lib.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_$lib -o run \
      --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_$lib.log 2>&1
done
echo done
