#!/bin/bash
# C5 with one and two concurrent callers for each library in $LIBS (DWPA_LIB), interleaved: the keyver-3 table layout
# decides whether one call's verify fits beside the next call's PBKDF2 head.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/kv3_callers}
mkdir -p $OUT
for lib in $LIBS; do
  name=$(basename $lib .so)
  for k in 1 2; do
    DWPA_LIB=$PWD/$lib timeout -k 10 150 python3 bench.py --workload c5 --callers $k --steps 20 --warmup 3 \
        --no-cpu-baseline > $OUT/${name}_k$k.json 2> $OUT/${name}_k$k.err
    echo "$name k$k $(python3 -c "import json;d=json.load(open('$OUT/${name}_k$k.json'));print(d['value'], d['ms_per_step'], d['hits_verified'])")"
  done
done
