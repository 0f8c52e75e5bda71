#!/bin/bash
# A/B of the check path's PBKDF2 remainder: on the GPU (DWPA_HOST_TAIL=0, lone tail waves beside the head) or on the
# host backend beside the head (default).  C5 with one and two callers, alternating, twice; then the tail tests.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/host_tail_ab}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread \
  -k "tail or c5" > $OUT/tests.log 2>&1
for r in 1 2; do
  for ht in 0 1; do
    DWPA_HOST_TAIL=$ht timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
      > $OUT/c5_ht${ht}_$r.json 2>> $OUT/err.log
    DWPA_HOST_TAIL=$ht timeout -k 10 200 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 \
      --no-cpu-baseline > $OUT/c5k2_ht${ht}_$r.json 2>> $OUT/err.log
  done
done
