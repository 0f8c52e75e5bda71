#!/bin/bash
# C5 verify-order A/B: the head slots' keyver-1/2 and keyver-3 verifies side by side on two streams (default), one
# after the other (DWPA_VERIFY_FANOUT=0), and keyver 3 first (DWPA_VERIFY_KV3_FIRST=1), one and two callers,
# interleaved; plus a kernel trace of each single-caller variant.  OUT defaults to gpurun_out/c5_order.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/c5_order}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, callers, env...
  local name=$1 callers=$2; shift 2
  env "$@" timeout -k 10 120 python3 bench.py --workload c5 --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      --callers $callers > $OUT/$name.json 2> $OUT/$name.err
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(d['value'], d['ms_per_step'], d['hits_verified'])")"
}
for rep in 1 2; do
  run k1_fan_r$rep 1
  run k1_serial_r$rep 1 DWPA_VERIFY_FANOUT=0
  run k1_serial_kv3first_r$rep 1 DWPA_VERIFY_FANOUT=0 DWPA_VERIFY_KV3_FIRST=1
  run k1_fan_kv3first_r$rep 1 DWPA_VERIFY_KV3_FIRST=1
done
run k2_fan 2
run k2_serial_kv3first 2 DWPA_VERIFY_FANOUT=0 DWPA_VERIFY_KV3_FIRST=1
for v in "fan" "serial_kv3first DWPA_VERIFY_FANOUT=0 DWPA_VERIFY_KV3_FIRST=1"; do
  set -- $v
  name=$1; shift
  env "$@" timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$name -o run -- \
      python3 bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_$name.json 2> $OUT/prof_$name.err
done
echo done
