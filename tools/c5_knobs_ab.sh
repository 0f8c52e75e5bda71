#!/bin/bash
# C5 check-path scheduling knobs with the round-3 AES layout, interleaved twice on one box (GPU box, repo root).
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/c5_knobs}
mkdir -p $OUT
guard() { case $1 in 124|134|137|139) echo "stop: rc $1" >&2; exit $1;; esac; }
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline \
      > $OUT/$name.json 2> $OUT/$name.err
  guard $?
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(d['value'], d['ms_per_step'], d['mismatches'])")"
}
DWPA_LIB=$PWD/ab/aes1f.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py \
    -k "golden or c5 or random_batch or nc_windows" -x -q --timeout 200 --timeout-method thread > $OUT/pytest_aes1f.txt 2>&1
rc=$?; guard $rc; echo "aes1f pytest rc=$rc $(tail -1 $OUT/pytest_aes1f.txt)"; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  run base_$rep DWPA_LIB=$PWD/ab/aes1.so
  run fill_$rep DWPA_LIB=$PWD/ab/aes1f.so
  run kv3p1_$rep DWPA_LIB=$PWD/ab/aes1f.so DWPA_KV3_PRIO=1
  run kv3p2_$rep DWPA_LIB=$PWD/ab/aes1f.so DWPA_KV3_PRIO=2
  run kv3first_$rep DWPA_LIB=$PWD/ab/aes1f.so DWPA_VERIFY_KV3_FIRST=1
  run tailp1_$rep DWPA_LIB=$PWD/ab/aes1f.so DWPA_TAIL_PRIO=1
  run kv3p2tail1_$rep DWPA_LIB=$PWD/ab/aes1f.so DWPA_KV3_PRIO=2 DWPA_TAIL_PRIO=1
done
echo done
