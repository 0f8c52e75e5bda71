#!/bin/bash
# A/B build of the product PBKDF2 code object with another issue-pass rule set: ab/<name>.so is the default library
# with only the embedded hsaco rebuilt.  tools/pbkdf2_rule_ab.sh split split_add3,before_half   (CPU, repo root)
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1
rules=$2
B=build/pbkdf2_$name
LLVM=/opt/rocm/lib/llvm/bin
make -s build/pbkdf2/pbkdf2_gfx950.s dwpa_amd/lib/libdwpa22000.so
mkdir -p $B ab
python3 dwpa_amd/csrc/gen/issue_pass.py build/pbkdf2/pbkdf2_gfx950.s $B/pbkdf2_issue.s \
    k_pbkdf2_gfx950+k_pbkdf2_gfx950_ms+k_pbkdf2_gfx950_mg+k_pbkdf2_gfx950_p+k_pbkdf2_gfx950_ms_p+k_pbkdf2_gfx950_mg_p+k_pbkdf2_gfx950_q+k_pbkdf2_gfx950_mg_q \
    $rules
$LLVM/clang -target amdgcn-amd-amdhsa -mcpu=gfx950 -c $B/pbkdf2_issue.s -o $B/pbkdf2_issue.o
$LLVM/ld.lld -shared $B/pbkdf2_issue.o -o $B/pbkdf2_gfx950.hsaco
python3 dwpa_amd/csrc/gen/embed.py $B/pbkdf2_gfx950.hsaco $B/pbkdf2_hsaco.cpp pbkdf2_gfx950_hsaco
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -c $B/pbkdf2_hsaco.cpp -o $B/pbkdf2_hsaco.o
objs=$(ls build/obj/*.o | grep -v pbkdf2_hsaco.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/$name.so $objs $B/pbkdf2_hsaco.o -lz -lpthread
echo ab/$name.so
