#!/bin/bash
# Round 6 validation on the GPU box: the GPU suite, smoke(), the default bench line under rocprofv3 --kernel-trace
# --stats, and the BASELINE legs (tools/bench_legs.sh).  Results in gpurun_out/$TAG/.  Every step has its own limit;
# the chain stops at the first failure.
set -euo pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/suite.log 2>&1
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 8 --warmup 2 \
    > $OUT/bench_prof.json 2> $OUT/bench_prof.err
fi
OUT=$OUT/legs LEGS=${LEGS:-"c1lat host c5 c5k2 c1 c4 c2files_node8"} tools/bench_legs.sh
