#!/bin/bash
# Builds tools/bin/asm_lab and one hsaco per nop rule from the PBKDF2 kernel's device assembly.
set -e
cd "$(dirname "$0")/../.."
LLVM=/opt/rocm/lib/llvm/bin
OUT=tools/bin/asm
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S dwpa_amd/csrc/pbkdf2_gfx950.hip -o $OUT/base.s 2>/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/asm_lab tools/asm/asm_lab.hip
for rule in "$@"; do
  name=$(echo "$rule" | tr ',=' '__')
  python3 dwpa_amd/csrc/gen/issue_pass.py $OUT/base.s $OUT/$name.s k_pbkdf2_gfx950 "$rule"
  $LLVM/clang -target amdgcn-amd-amdhsa -mcpu=gfx950 -c $OUT/$name.s -o $OUT/$name.o
  $LLVM/ld.lld -shared $OUT/$name.o -o $OUT/$name.hsaco
  echo "$OUT/$name.hsaco"
done
