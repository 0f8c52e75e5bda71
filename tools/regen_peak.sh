#!/bin/bash
# Re-measure the gfx950 VALU issue costs the PBKDF2 roofline is priced on (tools/valu_peak.hip, in-kernel clock)
# and recompute C_min / the peak from them (tools/cmin.py).  Run on the GPU box from the repo root, next to any
# bench run whose roofline is quoted; results land in gpurun_out/peak/.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/peak}
mkdir -p $OUT
timeout -k 10 120 ./tools/bin/valu_peak > $OUT/valu_issue_costs.json
python3 tools/cmin.py $OUT/valu_issue_costs.json | tee $OUT/peak.json
