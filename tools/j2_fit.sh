#!/bin/bash
# Does the j = 2 schedule form fit the issue-pass kernels' 64 VGPRs (8 waves per SIMD) from an earlier round t?
# Compiles pbkdf2_gfx950.hip (device-only asm, as the Makefile does) at DWPA_SCHED_J2_MIN = 64..73 and prints each
# kernel's VGPR count and spill count.  CPU only (hipcc cross-compiles for gfx950).
set -euo pipefail
cd "$(dirname "$0")/.."
T=$(mktemp -d)
for J in ${J2S:-64 66 68 69 70 71 72 73}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S dwpa_amd/csrc/pbkdf2_gfx950.hip \
    -DDWPA_SCHED_J2_MIN=$J -o $T/j$J.s
  python3 - "$T/j$J.s" "$J" <<'PY'
import re, sys
s = open(sys.argv[1]).read()
ks = re.findall(r"\.name:\s+(k_pbkdf2_gfx950\w*)", s)
vg = re.findall(r"\.vgpr_count:\s+(\d+)", s)
sp = re.findall(r"\.vgpr_spill_count:\s+(\d+)", s)
print(f"J2_MIN={sys.argv[2]}: " + ", ".join(f"{k[len('k_pbkdf2_gfx950'):] or '(base)'} {v} VGPR/{p} spilled"
                                         for k, v, p in zip(ks, vg, sp)))
PY
done
rm -rf $T
