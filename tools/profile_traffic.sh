#!/bin/bash
# HBM traffic of the hot kernels (MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE each in a pass of
# their own, FETCH_SIZE doubled for wide coalesced reads on gfx950) plus a kernel-trace/stats pass of the same
# bench command.  Run on the GPU box from the repo root; results land in gpurun_out/traffic/.
set -euo pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/traffic}
mkdir -p $OUT
BENCH="bench.py ${BENCH_ARGS:-}"  # default: the bench line itself (C2, 100M words)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $BENCH > $OUT/stats.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $BENCH > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $BENCH > $OUT/write.log 2>&1
python3 tools/pmc_traffic.py $OUT > $OUT/traffic.json
cat $OUT/traffic.json
