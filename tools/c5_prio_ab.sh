#!/bin/bash
# C5 priority re-sweep at the round's last HEAD: tail priority after the head (DWPA_TAIL_PRIO 2 default / 3 / 0) and
# post-derive kernel priority (DWPA_CHECK_PRIO 0 default / 1), one caller, interleaved twice.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/c5_prio}
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --workload c5 --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      > $OUT/$name.json 2> $OUT/$name.err
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(d['value'], d['ms_per_step'], d['hits_verified'])")"
}
for rep in 1 2; do
  run default_r$rep
  run tail3_r$rep DWPA_TAIL_PRIO=3
  run tail0_r$rep DWPA_TAIL_PRIO=0
  run check1_r$rep DWPA_CHECK_PRIO=1
  run tail3_check1_r$rep DWPA_TAIL_PRIO=3 DWPA_CHECK_PRIO=1
done
