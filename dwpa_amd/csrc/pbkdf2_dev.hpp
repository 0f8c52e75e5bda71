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

// One lane's PBKDF2 output block: T = U_1 ^ ... ^ U_4096 with U_1 = HMAC(P, S || INT(blk+1)).  `sb` points at
// the nsalt pre-padded 16-word salt blocks of this output block.
//
// PRIO: progress-ordered wave priority.  A SIMD issues by priority, then age, so the oldest of its waves runs
// almost alone-fast and the youngest gets leftovers: in a launch of one wave round (server checks, C1/C5) the waves
// finish one after another and the last one runs its remaining iterations alone, latency-bound.  With PRIO a wave
// starts at priority 3 and drops to 2 at iteration 3584 and to 1 at 3968, so waves that are behind get the issue
// slots and the waves of a SIMD reach the end together (spread <= ~128 iterations instead of up to a whole wave).
// Priority 0 stays free for work that should only take the slots these waves leave (the check path's tail).
template <bool PRIO = false>
__device__ __forceinline__ void pbkdf2_lane(const uint32_t hi[5], const uint32_t ho[5], const uint32_t* sb,
                                            uint32_t nsalt, uint32_t t[5]) {
    uint32_t st[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]};
    for (uint32_t b = 0; b < nsalt; b++) {
        uint32_t m[16];
#pragma unroll
        for (int j = 0; j < 16; j++) m[j] = sb[b * 16 + j];
        sha1_compress(st, m);
    }
    const Sha1Mid MI = sha1_mid(hi);
    const Sha1Mid MO = sha1_mid(ho);
    uint32_t u[5], x[5];
    sha1_84(MO, st, u);
#pragma unroll
    for (int k = 0; k < 5; k++) t[k] = u[k];
    if constexpr (!PRIO) {
#pragma unroll 1
        for (int it = 1; it < 4096; it++) {
            sha1_84(MI, u, x);
            sha1_84(MO, x, u);
#pragma unroll
            for (int k = 0; k < 5; k++) t[k] ^= u[k];
        }
    } else {
        __builtin_amdgcn_s_setprio(3);
        int it = 1;
#pragma unroll 1
        for (int phase = 0; phase < 3; phase++) {
            const int end = phase == 0 ? 3584 : phase == 1 ? 3968 : 4096;
            if (phase == 1) __builtin_amdgcn_s_setprio(2);
            else if (phase == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll 1
            for (; it < end; it++) {
                sha1_84(MI, u, x);
                sha1_84(MO, x, u);
#pragma unroll
                for (int k = 0; k < 5; k++) t[k] ^= u[k];
            }
        }
    }
}

__device__ __forceinline__ void set_wave_prio(uint32_t p) {
    switch (p) {  // s_setprio takes an immediate
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
    }
}

// The check path's tail lane (the PBKDF2 remainder of under one wave per SIMD, launched beside the head): wave
// priority 0 while *flag == 0, so it takes only the issue slots the head leaves; once the head has ended (the
// engine sets the flag from the head's stream) it raises itself to `prio`, ahead of the verify waves that share its
// SIMDs.  The flag is polled every 64 iterations with an agent-scope read-modify-write (fetch_add 0): the writer
// may sit on another XCD, and a plain agent-scope load of a word this XCD's L2 already holds can keep returning
// that stale copy, while an atomic is performed where every XCD sees the same word.  Each wave that
// raises itself bumps *raised once (dwpa_check_last_stats.tail_waves_raised).
__device__ __forceinline__ void pbkdf2_lane_tail(const uint32_t hi[5], const uint32_t ho[5], const uint32_t* sb,
                                                 uint32_t nsalt, uint32_t t[5], uint32_t* flag, uint32_t prio,
                                                 uint32_t* raised) {
    uint32_t st[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]};
    for (uint32_t b = 0; b < nsalt; b++) {
        uint32_t m[16];
#pragma unroll
        for (int j = 0; j < 16; j++) m[j] = sb[b * 16 + j];
        sha1_compress(st, m);
    }
    const Sha1Mid MI = sha1_mid(hi);
    const Sha1Mid MO = sha1_mid(ho);
    uint32_t u[5], x[5];
    sha1_84(MO, st, u);
#pragma unroll
    for (int k = 0; k < 5; k++) t[k] = u[k];
    int it = 1;
    if (prio) {
        bool up = false;  // wave-uniform (readfirstlane)
        // an operand the compiler cannot see is zero: an RMW of a known 0 is folded into a plain atomic load
        uint32_t zero;
        __asm__ volatile("s_mov_b32 %0, 0" : "=s"(zero));
#pragma unroll 1
        for (; it < 4096; it++) {
            if ((it & 63) == 0 &&
                __builtin_amdgcn_readfirstlane(
                    __hip_atomic_fetch_add(flag, zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                set_wave_prio(prio);
                up = true;
                break;
            }
            sha1_84(MI, u, x);
            sha1_84(MO, x, u);
#pragma unroll
            for (int k = 0; k < 5; k++) t[k] ^= u[k];
        }
        // outside the loop: a lane-0-only atomic inside a loop can make the compiler split the loop by lanes
        const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        if (up && lane == (uint32_t)__builtin_amdgcn_readfirstlane(lane))
            __hip_atomic_fetch_add(raised, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll 1
    for (; it < 4096; it++) {
        sha1_84(MI, u, x);
        sha1_84(MO, x, u);
#pragma unroll
        for (int k = 0; k < 5; k++) t[k] ^= u[k];
    }
}

__device__ __forceinline__ void load_mid(const uint32_t* __restrict__ mid, uint32_t cap, uint32_t s, uint32_t hi[5],
                                         uint32_t ho[5]) {
#pragma unroll
    for (int k = 0; k < 5; k++) {
        hi[k] = mid[(size_t)k * cap + s];
        ho[k] = mid[(size_t)(5 + k) * cap + s];
    }
}

__device__ __forceinline__ void store_block(uint32_t* __restrict__ pmk, uint32_t cap, uint32_t s, uint32_t blk,
                                            const uint32_t t[5]) {
    if (blk == 0) {
#pragma unroll
        for (int k = 0; k < 5; k++) pmk[(size_t)k * cap + s] = t[k];
    } else {
#pragma unroll
        for (int k = 0; k < 3; k++) pmk[(size_t)(5 + k) * cap + s] = t[k];
    }
}

// One ESSID for the whole launch: salt = [2 blocks][nsalt][16] words, read with scalar loads.
template <bool PRIO = false>
__device__ __forceinline__ void pbkdf2_body(const uint32_t* __restrict__ mid, uint32_t cap, uint32_t base,
                                            uint32_t count, const uint32_t* __restrict__ counter,
                                            const uint32_t* __restrict__ salt, uint32_t nsalt,
                                            uint32_t* __restrict__ pmk) {
    const uint32_t blk = blockIdx.y;
    const uint32_t s = base + blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = counter ? min(*counter, cap) : min(base + count, cap);
    if (s >= n) return;
    uint32_t hi[5], ho[5], t[5];
    load_mid(mid, cap, s, hi, ho);
    pbkdf2_lane<PRIO>(hi, ho, salt + (size_t)blk * nsalt * 16, nsalt, t);
    store_block(pmk, cap, s, blk, t);
}

// Work-queue form of pbkdf2_body: a fixed grid of 8 waves per SIMD, each wave taking (output block, 64-slot) items
// from the counter at `work` (zeroed before the launch) until they run out.  Workgroups go to the 8 XCDs round-robin
// whatever their progress, so a regular launch ends with its slowest XCD; here every wave keeps taking items, so a
// faster XCD takes more of them.  Every wave exits once the counter passes the item count.
__device__ __forceinline__ void pbkdf2_body_queue(const uint32_t* __restrict__ mid, uint32_t cap, uint32_t base,
                                                  uint32_t count, const uint32_t* __restrict__ counter,
                                                  const uint32_t* __restrict__ salt, uint32_t nsalt,
                                                  uint32_t* __restrict__ pmk, uint32_t* __restrict__ work) {
    const uint32_t n = counter ? min(*counter, cap) : min(base + count, cap);
    const uint32_t nitems = base < n ? 2u * ((n - base + 63u) / 64u) : 0u;
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll 1
    for (;;) {
        uint32_t item = 0;
        if (lane == 0) item = atomicAdd(work, 1u);
        item = __builtin_amdgcn_readfirstlane(__shfl(item, 0));
        if (item >= nitems) break;
        const uint32_t blk = item & 1u;  // both output blocks of a slot range are taken back to back
        const uint32_t s = base + (item >> 1) * 64u + lane;
        if (s < n) {
            uint32_t hi[5], ho[5], t[5];
            load_mid(mid, cap, s, hi, ho);
            pbkdf2_lane(hi, ho, salt + (size_t)blk * nsalt * 16, nsalt, t);
            store_block(pmk, cap, s, blk, t);
        }
    }
}

// Many ESSIDs in one launch (server batches, common.php:902): slot s derives with the salt entry at
// pool + sref[s] = {nsalt, [2 blocks][nsalt][16] words}.  Only the U_1 blocks differ per lane; the 4096 loop is
// the same code as pbkdf2_body's.
template <bool PRIO = false>
__device__ __forceinline__ void pbkdf2_body_ms(const uint32_t* __restrict__ mid, uint32_t cap, uint32_t count,
                                               const uint32_t* __restrict__ pool,
                                               const uint32_t* __restrict__ sref, uint32_t* __restrict__ pmk) {
    const uint32_t blk = blockIdx.y;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= min(count, cap)) return;
    uint32_t hi[5], ho[5], t[5];
    load_mid(mid, cap, s, hi, ho);
    const uint32_t* e = pool + sref[s];
    const uint32_t nsalt = e[0];
    pbkdf2_lane<PRIO>(hi, ho, e + 1 + (size_t)blk * nsalt * 16, nsalt, t);
    store_block(pmk, cap, s, blk, t);
}

// Many ESSID groups x one candidate batch in one launch (scan work units with many ESSIDs):
// lane i -> chunk group c = i / cap, slot s = i % cap.  cap is a multiple of 64, so c is wave-uniform and the
// salt entry is read with scalar loads.  gsalt[c] = {word offset of the group's [2][nsalt][16] salt blocks, nsalt};
// PMK word k of (c, s) lands at pmk[k * pstride + c * cap + s].
template <bool PRIO = false>
__device__ __forceinline__ void pbkdf2_body_mg(const uint32_t* __restrict__ mid, uint32_t cap,
                                               const uint32_t* __restrict__ counter, uint32_t ngroups,
                                               const uint32_t* __restrict__ salt, const uint32_t* __restrict__ gsalt,
                                               uint32_t* __restrict__ pmk, uint32_t pstride) {
    const uint32_t blk = blockIdx.y;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t c = __builtin_amdgcn_readfirstlane(i / cap);
    const uint32_t s = i - c * cap;
    if (c >= ngroups || s >= min(*counter, cap)) return;
    uint32_t hi[5], ho[5], t[5];
    load_mid(mid, cap, s, hi, ho);
    const uint32_t off = gsalt[2 * c], nsalt = gsalt[2 * c + 1];
    pbkdf2_lane<PRIO>(hi, ho, salt + off + (size_t)blk * nsalt * 16, nsalt, t);
    store_block(pmk + (size_t)c * cap, pstride, s, blk, t);
}

// Work-queue form of pbkdf2_body_mg: items are (output block, 64-lane wave of the ngroups x cap lane space); waves
// past a group's loaded slots take the next item at once.
__device__ __forceinline__ void pbkdf2_body_mg_queue(const uint32_t* __restrict__ mid, uint32_t cap,
                                                     const uint32_t* __restrict__ counter, uint32_t ngroups,
                                                     const uint32_t* __restrict__ salt,
                                                     const uint32_t* __restrict__ gsalt, uint32_t* __restrict__ pmk,
                                                     uint32_t pstride, uint32_t* __restrict__ work) {
    const uint32_t n = min(*counter, cap);
    const uint32_t nitems = 2u * ngroups * (cap / 64u);
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll 1
    for (;;) {
        uint32_t item = 0;
        if (lane == 0) item = atomicAdd(work, 1u);
        item = __builtin_amdgcn_readfirstlane(__shfl(item, 0));
        if (item >= nitems) break;
        const uint32_t blk = item & 1u;
        const uint32_t i = (item >> 1) * 64u + lane;
        const uint32_t c = __builtin_amdgcn_readfirstlane(i / cap);
        const uint32_t s = i - c * cap;
        if (s < n) {
            uint32_t hi[5], ho[5], t[5];
            load_mid(mid, cap, s, hi, ho);
            const uint32_t off = gsalt[2 * c], nsalt = gsalt[2 * c + 1];
            pbkdf2_lane(hi, ho, salt + off + (size_t)blk * nsalt * 16, nsalt, t);
            store_block(pmk + (size_t)c * cap, pstride, s, blk, t);
        }
    }
}

}  // namespace dwpa
