#!/bin/bash
# Builds an A/B variant of libdwpa22000.so into ab/<name>.so with extra compile flags (the PBKDF2 code object is
# shared with the default build).  tools/build_ab.sh aes0 -DDWPA_KV3_AES=0
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p ab
make -s -j8 LIB=ab/$name.so OBJ=build/obj_$name CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function $*" \
    ab/$name.so 2>&1 | grep -v "hip-link" || true
test -f ab/$name.so && echo "ab/$name.so"
