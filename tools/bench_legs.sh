#!/bin/bash
# Every BASELINE.json config as a bench.py leg, one JSON line each, plus the VALU issue-cost re-measurement the
# roofline is priced on.  Run on the GPU box from the repo root; results land in gpurun_out/legs/.
# LEGS="c2 c4" restricts the set (c1cold, the PHP-FPM worker-process leg, runs only when named).  Each step has its own time limit and the chain stops at the first failure.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/legs}
mkdir -p $OUT
LEGS=${LEGS:-"peak c2 c4 c4strong c3 c5 c5k2 c1 c1lat host c2files c2files_node8 c3files c3files_server c3files_server_full expand"}
for leg in $LEGS; do
  case $leg in
    peak)    OUT=$OUT/peak tools/regen_peak.sh > /dev/null ;;
    c2)      timeout -k 10 240 python3 bench.py --steps 8 --warmup 2 > $OUT/c2.json 2> $OUT/c2.err ;;
    c4)      timeout -k 10 240 python3 bench.py --workload c4 --steps 8 --warmup 2 > $OUT/c4.json 2> $OUT/c4.err ;;
    c4strong) timeout -k 10 240 python3 bench.py --workload c4 --scaling strong --steps 2 --warmup 1 --no-cpu-baseline \
               > $OUT/c4strong.json 2> $OUT/c4strong.err ;;
    c1lat)   timeout -k 10 240 python3 bench.py --workload c1lat --steps 9 > $OUT/c1lat.json 2> $OUT/c1lat.err ;;
    c3)      timeout -k 10 300 python3 bench.py --workload c3 --steps 4 --warmup 1 > $OUT/c3.json 2> $OUT/c3.err ;;
    c5)      timeout -k 10 240 python3 bench.py --workload c5 --steps 20 --warmup 3 > $OUT/c5.json 2> $OUT/c5.err ;;
    c5k2)    timeout -k 10 240 python3 bench.py --workload c5 --callers 2 --steps 20 --warmup 3 --no-cpu-baseline \
               > $OUT/c5k2.json 2> $OUT/c5k2.err ;;
    c1)      timeout -k 10 240 python3 bench.py --workload c1 --steps 20 --warmup 3 > $OUT/c1.json 2> $OUT/c1.err ;;
    host)    timeout -k 10 240 python3 tools/host_backend_bench.py > $OUT/host.json 2> $OUT/host.err ;;
    # the client's node mode: one process over every visible device (--gpus = their count), dictionary + rule pass
    c2files) timeout -k 10 600 python3 bench.py --workload c2files --gpus ${NODE_GPUS:-1} --steps 1 --warmup 1 \
               > $OUT/c2files.json 2> $OUT/c2files.err ;;
    # its 8-worker rehearsal on one GPU (an 8-GPU node's worker count and shared feed, not its throughput)
    c2files_node8) DWPA_CRACK_SHARDS_PER_DEVICE=8 timeout -k 10 600 python3 bench.py --workload c2files --steps 1 \
               --warmup 1 > $OUT/c2files_node8.json 2> $OUT/c2files_node8.err ;;
    c3files) DWPA_TRACE=1 timeout -k 10 400 python3 bench.py --workload c3files --steps 2 --warmup 0 \
               > $OUT/c3files.json 2> $OUT/c3files.err ;;
    c3files_server) DWPA_TRACE=1 timeout -k 10 400 python3 bench.py --workload c3files --rules-set server --steps 2 \
               --warmup 0 > $OUT/c3files_server.json 2> $OUT/c3files_server.err ;;
    c3files_server_full) DWPA_TRACE=1 timeout -k 10 400 python3 bench.py --workload c3files --rules-set server \
               --rule-mode full --steps 2 --warmup 0 > $OUT/c3files_server_full.json 2> $OUT/c3files_server_full.err ;;
    c1cold)  timeout -k 10 900 python3 bench.py --workload c1cold --steps 20 > $OUT/c1cold.json 2> $OUT/c1cold.err ;;
    expand)  timeout -k 10 300 python3 bench.py --workload expand --rule-words 5000000 --steps 2 --warmup 1 \
               > $OUT/expand.json 2> $OUT/expand.err ;;
    *) echo "unknown leg $leg" >&2; exit 2 ;;
  esac
  echo "leg $leg done" >&2
done
