// prep_dev.hpp -- device helpers shared by the candidate-materialisation kernels (kernels.hip, rules.hip):
// key bytes -> HMAC-SHA1 key block -> ipad/opad midstates, and wave-aggregated slot compaction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crypto_dev.hpp"

namespace dwpa {

// ------------------------------------------------------------------------------------------------
// key loading
// ------------------------------------------------------------------------------------------------

// Up to 64 bytes at p (any alignment) as 16 big-endian words, zero beyond len.  Reads only dwords that hold at
// least one byte of [p, p+len), so it never touches more than the word-aligned span of the key.
__device__ __forceinline__ void load_key_block(const uint8_t* p, uint32_t len, uint32_t w[16]) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t nw = (len + sh + 3) >> 2;  // dwords spanned
    uint32_t lo = nw > 0 ? q[0] : 0u;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint32_t hi = (uint32_t)(j + 1) < nw ? q[j + 1] : 0u;
        uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sh);  // bytes p[4j..4j+3], little-endian
        lo = hi;
        v = bswap32(v);
        const int rem = (int)len - 4 * j;
        if (rem <= 0) v = 0;
        else if (rem < 4) v &= 0xffffffffu << (8 * (4 - rem));
        w[j] = v;
    }
}

// SHA1 of an arbitrary-length key (HMAC keys longer than the 64-byte block are hashed first, RFC 2104).
__device__ __noinline__ static void sha1_long_key(const uint8_t* p, uint32_t len, uint32_t out[5]) {
    sha1_iv(out);
    const uint32_t nblk = (len + 9 + 63) >> 6;
    const uint64_t bits = (uint64_t)len * 8;
    for (uint32_t b = 0; b < nblk; b++) {
        uint32_t m[16];
        for (int j = 0; j < 16; j++) {
            uint32_t v = 0;
            for (int i = 0; i < 4; i++) {
                const uint32_t k = b * 64 + 4 * j + i;
                uint32_t byte = k < len ? p[k] : (k == len ? 0x80u : 0u);
                v = (v << 8) | byte;
            }
            m[j] = v;
        }
        if (b == nblk - 1) {
            m[14] = (uint32_t)(bits >> 32);
            m[15] = (uint32_t)bits;
        }
        sha1_compress(out, m);
    }
}

__device__ __forceinline__ void key_block_from_bytes(const uint8_t* p, uint32_t len, uint32_t kb[16]) {
    if (len <= 64) {
        load_key_block(p, len, kb);
    } else {
        uint32_t h[5];
        sha1_long_key(p, len, h);
#pragma unroll
        for (int j = 0; j < 16; j++) kb[j] = j < 5 ? h[j] : 0u;
    }
}

__device__ __forceinline__ void store_mid(uint32_t* mid, uint32_t cap, uint32_t slot, const uint32_t kb[16]) {
    uint32_t ip[5], op[5];
    sha1_hmac_mid(kb, ip, op);
#pragma unroll
    for (int k = 0; k < 5; k++) {
        mid[(size_t)k * cap + slot] = ip[k];
        mid[(size_t)(5 + k) * cap + slot] = op[k];
    }
}

// Wave-aggregated compaction: one atomic per wave, slots stay in lane order inside the wave.
__device__ __forceinline__ uint32_t compact_slot(bool keep, uint32_t* counter) {
    const uint64_t m = __ballot(keep);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t leader = m ? (uint32_t)__builtin_ctzll(m) : 0u;
    uint32_t base = 0;
    if (m && lane == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

}  // namespace dwpa
