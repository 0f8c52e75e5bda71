// pbkdf2_dev.hpp -- body of the PBKDF2-HMAC-SHA1 x4096 kernel (shared by the product kernel k_pbkdf2_gfx950 in
// pbkdf2_gfx950.hip, which goes through the gfx950 issue pass, and the plain hipcc build k_pbkdf2 in kernels.hip).
//
// One lane = one (candidate, output block): blockIdx.y selects T_1 (PMK bytes 0..19) or T_2 (bytes 20..31).
// SHA-1 state and both HMAC midstates live in VGPRs (56 VGPRs -> 8 waves/SIMD); the ESSID salt blocks
// (ESSID || INT(i) || padding, pre-padded on the host) are wave-uniform and arrive through scalar loads.
// PMK = PBKDF2(PSK, ESSID, 4096, 32) as in web/common.php:178-180,246-248.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crypto_dev.hpp"

namespace dwpa {

__device__ __forceinline__ void pbkdf2_body(const uint32_t* __restrict__ mid, uint32_t cap, uint32_t base,
                                            uint32_t count, const uint32_t* __restrict__ counter,
                                            const uint32_t* __restrict__ salt, uint32_t nsalt,
                                            uint32_t* __restrict__ pmk) {
    const uint32_t blk = blockIdx.y;
    const uint32_t s = base + blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = counter ? min(*counter, cap) : min(base + count, cap);
    if (s >= n) return;
    uint32_t hi[5], ho[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        hi[k] = mid[(size_t)k * cap + s];
        ho[k] = mid[(size_t)(5 + k) * cap + s];
    }
    // U_1 = HMAC(P, S || INT(blk+1))
    uint32_t st[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]};
    const uint32_t* sb = salt + (size_t)blk * nsalt * 16;
    for (uint32_t b = 0; b < nsalt; b++) {
        uint32_t m[16];
#pragma unroll
        for (int j = 0; j < 16; j++) m[j] = sb[b * 16 + j];
        sha1_compress(st, m);
    }
    const Sha1Mid MI = sha1_mid(hi);
    const Sha1Mid MO = sha1_mid(ho);
    uint32_t u[5], x[5], t[5];
    sha1_84(MO, st, u);
#pragma unroll
    for (int k = 0; k < 5; k++) t[k] = u[k];
#pragma unroll 1
    for (int it = 1; it < 4096; it++) {
        sha1_84(MI, u, x);
        sha1_84(MO, x, u);
#pragma unroll
        for (int k = 0; k < 5; k++) t[k] ^= u[k];
    }
    if (blk == 0) {
#pragma unroll
        for (int k = 0; k < 5; k++) pmk[(size_t)k * cap + s] = t[k];
    } else {
#pragma unroll
        for (int k = 0; k < 3; k++) pmk[(size_t)(5 + k) * cap + s] = t[k];
    }
}

}  // namespace dwpa
