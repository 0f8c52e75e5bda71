#!/bin/bash
# Engine clock and socket power sampled while the C2 bench runs (box-to-box variation check).  Run on the GPU box
# from the repo root; samples land in gpurun_out/clkprobe/.
set -uo pipefail
OUT=${OUT:-gpurun_out/clkprobe}
mkdir -p $OUT
timeout -k 10 150 python bench.py --no-cpu-baseline --steps 30 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err &
B=$!
sleep 8
for i in 1 2 3 4 5 6 7 8; do
  timeout 20 amd-smi metric -c -p --json > $OUT/amd_smi_$i.json 2>> $OUT/amd_smi.err
  sleep 2
done
wait $B
