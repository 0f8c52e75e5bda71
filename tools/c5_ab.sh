#!/bin/bash
# C5 scheduling A/B: the check-path knobs of engine.cpp (DWPA_TAIL_PRIO, DWPA_VERIFY_FANOUT, DWPA_CHECK_PRIO,
# DWPA_HEAD_FENCE) with one and two concurrent callers, one bench line each, plus a kernel trace of the default.
# Run on the GPU box from the repo root; OUT defaults to gpurun_out/c5_ab.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/c5_ab}
mkdir -p $OUT
run() {  # name, callers, env...
  local name=$1 callers=$2; shift 2
  env "$@" timeout -k 10 120 python3 bench.py --workload c5 --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      --callers $callers > $OUT/$name.json 2> $OUT/$name.err
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(d['value'], d['ms_per_step'], d['hits_verified'])")"
}
run k1_default 1
run k1_f0 1 DWPA_VERIFY_FANOUT=0
run k1_h16 1 DWPA_HOST_THREADS=16
run k1_t0 1 DWPA_TAIL_PRIO=0
run k2_default 2
run k2_nofence 2 DWPA_HEAD_FENCE=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DWPA_TRACE=1 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_k1 -o c5k1 -- \
    python3 bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_k1.json 2> $OUT/prof_k1.err
echo "prof done"
