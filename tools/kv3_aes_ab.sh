#!/bin/bash
# Keyver-3 AES layouts A/B (crypto_dev.hpp DWPA_KV3_AES): 0 = four plain T-tables (round 2), 1 = lane-sliced Te0 x32
# (32 KiB, conflict-free, the default build), 2 = Te0 + Te2 x32 with v_perm addressing (64 KiB; 256- and 512-thread
# workgroups).  Per library: kv3 parity tests, C5 with one and two callers, a kernel trace.  GPU box, repo root.
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/kv3_aes}
mkdir -p $OUT
export TMPDIR=/tmp
guard() { local rc=$1; case $rc in 124|134|137|139) echo "stop: rc $rc" >&2; exit $rc;; esac; }
for lib in ${LIBS:-aes1 aes0 aes2 aes2b}; do
  L=$PWD/ab/$lib.so
  DWPA_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py \
      -k "golden or c5 or random_batch or nc_windows" -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$lib.txt 2>&1
  rc=$?; guard $rc; echo "$lib pytest rc=$rc $(tail -1 $OUT/pytest_$lib.txt)"
  [ $rc -eq 0 ] || continue
  for k in 1 2; do
    DWPA_LIB=$L timeout -k 10 150 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 --no-cpu-baseline \
        > $OUT/c5_${lib}_k$k.json 2> $OUT/c5_${lib}_k$k.err
    guard $?
    echo "$lib callers=$k $(python3 -c "import json;d=json.load(open('$OUT/c5_${lib}_k$k.json'));print(d['value'], d['ms_per_step'], d['hits_verified'], d['mismatches'])")"
  done
  DWPA_LIB=$L timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$lib -o run \
      -- python3 bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_$lib.json 2> $OUT/prof_$lib.err
  guard $?
done
echo done
