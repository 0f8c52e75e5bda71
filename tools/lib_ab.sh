#!/bin/bash
# A/B of alternative builds of libdwpa22000.so (DWPA_LIB) on one bench workload: a bench line and a rocprofv3 kernel
# trace per library.  LIBS="ab/a.so ab/b.so" WORKLOAD=c5 OUT=gpurun_out/lib_ab tools/lib_ab.sh (GPU box, repo root).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/lib_ab}
WORKLOAD=${WORKLOAD:-c5}
mkdir -p $OUT
export TMPDIR=/tmp
for lib in $LIBS; do
  name=$(basename $lib .so)
  DWPA_LIB=$PWD/$lib timeout -k 10 150 python3 bench.py --workload $WORKLOAD --steps ${STEPS:-20} --warmup 3 \
      --no-cpu-baseline > $OUT/$name.json 2> $OUT/$name.err
  DWPA_LIB=$PWD/$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$name \
      -o run -- python3 bench.py --workload $WORKLOAD --steps 10 --warmup 2 --no-cpu-baseline \
      > $OUT/prof_$name.json 2> $OUT/prof_$name.err
  echo "$name $(python3 -c "import json;d=json.load(open('$OUT/$name.json'));print(d['value'], d['ms_per_step'], d['hits_verified'])")"
done
