#!/bin/bash
# Keyver-3 verify A/B: AES round keys recomputed per CMAC block (ab/base.so, the default build) vs expanded once per
# key into LDS (ab/rk.so, -DDWPA_KV3_RK_LDS=1 -DDWPA_KV3_WAVES=3).  Parity tests on the variant, bench lines and
# traces (tools/lib_ab.sh), and one SQ counter pass per library (kernels serialized: each dispatch's time alone).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/kv3_rk}
mkdir -p $OUT
export TMPDIR=/tmp
DWPA_LIB=$PWD/ab/rk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py \
    -k "golden or random or c5 or dedup or challenge" -x -v --timeout 200 --timeout-method thread > $OUT/pytest_rk.txt 2>&1
LIBS="ab/base.so ab/rk.so ab/base2.so ab/rk2.so" WORKLOAD=c5 OUT=$OUT timeout -k 10 500 tools/lib_ab.sh > $OUT/ab.log 2>&1
for lib in base rk; do
  DWPA_LIB=$PWD/ab/$lib.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_$lib -o run \
      --output-format csv -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_$lib.log 2>&1
done
echo done
