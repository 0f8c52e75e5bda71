// kernels.hip -- the m22000 hot path on gfx950: candidate materialisation -> PBKDF2-HMAC-SHA1 x4096 -> verify.
//
//   k_prep_dict     dictionary words in HBM (offsets+bytes)  -> HMAC-SHA1 key midstates (ipad/opad), compacted
//   k_prep_numeric  in-kernel decimal keyspace (C4)          -> midstates
//   k_prep_keys     check path: unique keys (slot indices into the call's key bytes) -> midstates
//   k_pbkdf2        midstates x ESSID salt                    -> PMK (32 B)      [~99 % of all work]
//   k_verify        PMK x hashline(s) of that ESSID           -> hit records     [PMKID / EAPOL keyver 1,2,3 + NC]
//
// The PMK is defined by web/common.php:178-180,246-248 (openssl_pbkdf2($key,$essid,32,4096,'sha1')), the checks by
// common.php:167-189 (PMKID) and :192-300 (EAPOL with nonce-error-correction).
//
// Layouts in HBM (cap = candidate slots per batch):
//   mid[10][cap]  u32  SoA   ipad h0..h4, opad h0..h4     (40 B / candidate, written once, reused for every ESSID)
//   ids[cap]      u64        candidate id of each slot (dictionary order survives compaction)
//   pmk[8][cap]   u32  SoA   PMK big-endian words         (32 B / candidate / ESSID)
// All loads/stores of these arrays are lane-contiguous (coalesced dwords).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crypto_dev.hpp"
#include "pbkdf2_dev.hpp"
#include "prep_dev.hpp"
#include "tables.hpp"
#include "kernels.hpp"

namespace dwpa {

// ------------------------------------------------------------------------------------------------
// stage 1: candidates -> HMAC key midstates
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prep_dict(const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                                                   uint64_t first, uint32_t count, uint32_t minlen, uint32_t maxlen,
                                                   uint32_t* __restrict__ mid, uint64_t* __restrict__ ids,
                                                   uint32_t* __restrict__ counter, uint32_t cap, uint32_t compact) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool keep = false;
    uint64_t b0 = 0;
    uint32_t len = 0;
    if (i < count) {
        b0 = off[first + i];
        const uint64_t b1 = off[first + i + 1];
        len = (uint32_t)(b1 - b0);
        keep = !compact || (len >= minlen && len <= maxlen);
    }
    uint32_t slot = i;
    if (compact) slot = compact_slot(keep, counter);
    if (!keep || slot >= cap) return;
    uint32_t kb[16];
    key_block_from_bytes(bytes + b0, len, kb);
    store_mid(mid, cap, slot, kb);
    if (ids) ids[slot] = first + i;
}

// Check path: unique key u -> its midstates at row u.  The key is slot uslot[u]'s bytes; koff/klen index the
// call's key bytes in slot order, so the host never copies the unique keys into a contiguous list.
__global__ __launch_bounds__(256) void k_prep_keys(const uint64_t* __restrict__ koff, const uint32_t* __restrict__ klen,
                                                   const uint8_t* __restrict__ kbytes, const uint32_t* __restrict__ uslot,
                                                   uint32_t count, uint32_t* __restrict__ mid, uint32_t cap) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= count || u >= cap) return;
    const uint32_t s = uslot[u];
    uint32_t kb[16];
    key_block_from_bytes(kbytes + koff[s], klen[s], kb);
    store_mid(mid, cap, u, kb);
}

// Decimal keyspace: candidate v -> its `digits`-wide zero-padded decimal string (C4: 00000000..99999999).
__global__ __launch_bounds__(256) void k_prep_numeric(uint64_t first, uint32_t count, uint32_t digits,
                                                      uint32_t* __restrict__ mid, uint64_t* __restrict__ ids, uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count || i >= cap) return;
    uint64_t v = first + i;
    uint32_t kb[16];
#pragma unroll
    for (int j = 0; j < 16; j++) kb[j] = 0;
    // digits <= 20; fill from the least significant character
    for (int k = (int)digits - 1; k >= 0; k--) {
        const uint32_t d = (uint32_t)(v % 10u);
        v /= 10u;
        const uint32_t c = 0x30u + d;
        const int wi = k >> 2, sh = 24 - 8 * (k & 3);
#pragma unroll
        for (int j = 0; j < 5; j++)
            if (j == wi) kb[j] |= c << sh;
    }
    store_mid(mid, cap, i, kb);
    ids[i] = first + i;
}

// ------------------------------------------------------------------------------------------------
// stage 2: PBKDF2-HMAC-SHA1 x4096 (body in pbkdf2_dev.hpp).  This is the plain hipcc-scheduled build, kept as the
// A/B reference; the product launch uses k_pbkdf2_gfx950 after the gfx950 issue pass (pbkdf2_module.cpp).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pbkdf2(const uint32_t* __restrict__ mid, uint32_t cap, uint32_t base,
                                                uint32_t count, const uint32_t* __restrict__ counter,
                                                const uint32_t* __restrict__ salt, uint32_t nsalt,
                                                uint32_t* __restrict__ pmk) {
    pbkdf2_body(mid, cap, base, count, counter, salt, nsalt, pmk);
}

// Lanes [live, count) of a padded launch (lone_pad below) repeat slot live-1's derivation and store nothing.
// Occupancy bound 8 waves per SIMD (lifting it measured slower, CHANGELOG.md round 5).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_ms(
    const uint32_t* __restrict__ mid, uint32_t cap, uint32_t count, const uint32_t* __restrict__ pool,
    const uint32_t* __restrict__ sref, uint32_t* __restrict__ pmk, uint32_t live) {
    const uint32_t blk = blockIdx.y;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= count) return;
    const uint32_t ss = min(s, live - 1);
    uint32_t hi[5], ho[5], t[5];
    load_mid(mid, cap, ss, hi, ho);
    const uint32_t* e = pool + sref[ss];
    const uint32_t nsalt = e[0];
    pbkdf2_lane<false>(hi, ho, e + 1 + (size_t)blk * nsalt * 16, nsalt, t);
    if (s < live) store_block(pmk, cap, s, blk, t);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_mg(const uint32_t* __restrict__ mid, uint32_t cap,
                                                   const uint32_t* __restrict__ counter, uint32_t ngroups,
                                                   const uint32_t* __restrict__ salt,
                                                   const uint32_t* __restrict__ gsalt, uint32_t* __restrict__ pmk,
                                                   uint32_t pstride) {
    pbkdf2_body_mg(mid, cap, counter, ngroups, salt, gsalt, pmk, pstride);
}

// The check path's PBKDF2 tail (pbkdf2_lane_tail): same slots and salt entries as k_pbkdf2_ms.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_ms_tail(
    const uint32_t* __restrict__ mid, uint32_t cap, uint32_t count, const uint32_t* __restrict__ pool,
    const uint32_t* __restrict__ sref, uint32_t* __restrict__ pmk, uint32_t* flag, uint32_t prio, uint32_t* raised) {
    const uint32_t blk = blockIdx.y;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= min(count, cap)) return;
    uint32_t hi[5], ho[5], t[5];
    load_mid(mid, cap, s, hi, ho);
    const uint32_t* e = pool + sref[s];
    const uint32_t nsalt = e[0];
    pbkdf2_lane_tail(hi, ho, e + 1 + (size_t)blk * nsalt * 16, nsalt, t, flag, prio, raised);
    store_block(pmk, cap, s, blk, t);
}

// Sets the tail's head-done flag with an agent-scope atomic (the tail's waves poll it with atomics from every XCD).
__global__ void k_set_flag(uint32_t* flag) {
    if (threadIdx.x == 0) __hip_atomic_exchange(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Slot PMKs from the derived unique (ESSID, key) PMKs or from caller-supplied PMKs:
// src[i] = u -> upmk[.][u];  src[i] = GATHER_CALLER | c -> cpmk[c][0..7] (check_key_m22000's $pmk, common.php:178).
__global__ __launch_bounds__(256) void k_gather_pmk(const uint32_t* __restrict__ upmk, uint32_t ucap,
                                                    const uint32_t* __restrict__ cpmk,
                                                    const uint32_t* __restrict__ src, uint32_t n,
                                                    uint32_t* __restrict__ pmk, uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = src[i];
    if (r & GATHER_CALLER) {
        const uint32_t* c = cpmk + 8 * (size_t)(r & ~GATHER_CALLER);
#pragma unroll
        for (int k = 0; k < 8; k++) pmk[(size_t)k * cap + i] = c[k];
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++) pmk[(size_t)k * cap + i] = upmk[(size_t)k * ucap + r];
    }
}

// Hit count and hits -> host-mapped pinned memory (word 0 = count, the min(count, hitcap) HitDev records from byte
// 16): the check path reads its results without a device-to-host copy, whose runtime blit kernel would run at wave
// priority 0 and starve beside another call's PBKDF2 head.
// Word 1 = *raised (the tail waves that raised their priority, pbkdf2_lane_tail; 0 without a counter).
__global__ __launch_bounds__(256) void k_hits_out(const uint32_t* __restrict__ hitcnt,
                                                  const HitDev* __restrict__ hits, uint32_t hitcap,
                                                  uint32_t* __restrict__ out, const uint32_t* __restrict__ raised) {
    __builtin_amdgcn_s_setprio(3);
    const uint32_t n = min(*hitcnt, hitcap);
    constexpr uint32_t W = sizeof(HitDev) / 4;
    const uint32_t* src = (const uint32_t*)hits;
    const uint32_t total = n * W;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x)
        out[4 + i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[0] = *hitcnt;
        out[1] = raised ? *raised : 0u;
    }
}

// Caller-supplied PMK for one slot (check_key_m22000's $pmk argument, common.php:157,178).
__global__ void k_set_pmk(uint32_t* __restrict__ pmk, uint32_t cap, uint32_t slot, uint4 lo, uint4 hi) {
    if (threadIdx.x == 0) {
        pmk[0 * (size_t)cap + slot] = lo.x; pmk[1 * (size_t)cap + slot] = lo.y;
        pmk[2 * (size_t)cap + slot] = lo.z; pmk[3 * (size_t)cap + slot] = lo.w;
        pmk[4 * (size_t)cap + slot] = hi.x; pmk[5 * (size_t)cap + slot] = hi.y;
        pmk[6 * (size_t)cap + slot] = hi.z; pmk[7 * (size_t)cap + slot] = hi.w;
    }
}

// ------------------------------------------------------------------------------------------------
// stage 3: verification.  One wave = one segment = up to 64 slots x one line (line data wave-uniform).
// ------------------------------------------------------------------------------------------------
// KW blocks (tables.hpp): wave-uniform blocks with host-expanded schedules, read with scalar loads.
__device__ __forceinline__ void sha1_blocks_kw(uint32_t st[5], const uint32_t* __restrict__ kw, uint32_t nblk) {
    for (uint32_t b = 0; b < nblk; b++) sha1_compress_kw(st, kw + b * SHA1_KW_WORDS);
}
__device__ __forceinline__ void sha256_blocks_kw(uint32_t st[8], const uint32_t* __restrict__ kw, uint32_t nblk) {
    for (uint32_t b = 0; b < nblk; b++) sha256_compress_kw(st, kw + b * SHA256_KW_WORDS);
}
__device__ __forceinline__ void md5_blocks_km(uint32_t st[4], const uint32_t* __restrict__ km, uint32_t nblk) {
    for (uint32_t b = 0; b < nblk; b++) md5_compress_km(st, km + b * MD5_KM_WORDS);
}

// Block b of an attempt's PRF stream: shared words with the attempt's two patched words substituted
// (LineDev.patch_w0/_w1; NO_PATCH never matches, so explicit per-attempt blocks pass through unchanged).
__device__ __forceinline__ void att_block(const uint32_t* __restrict__ w, uint32_t b, uint32_t pw0, uint32_t pw1,
                                          uint32_t v0, uint32_t v1, uint32_t m[16]) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint32_t idx = b * 16 + j;
        uint32_t x = w[idx];
        x = idx == pw0 ? v0 : x;
        x = idx == pw1 ? v1 : x;
        m[j] = x;
    }
}

// The attempt's PRF blocks after the shared prefix, fed to `compress`.  Patched lines take the stream from the line
// (LineDev.att_off/att_nblk, wave-uniform): in k_verify_att the lanes hold different attempts, and the per-attempt
// copy of the same offset would turn every message word into a per-lane vector load.  Explicit per-attempt
// streams (short ANONCE) are per lane.
template <typename F>
__device__ __forceinline__ void prf_blocks(const LineDev& L, const uint32_t* __restrict__ pool, const AttDev& at,
                                           F&& compress) {
    uint32_t m[16];
    if (L.patch_w0 != NO_PATCH) {
        const uint32_t* aw = pool + L.att_off;
        for (uint32_t b = 0; b < L.att_nblk; b++) {
            att_block(aw, b, L.patch_w0, L.patch_w1, at.v0, at.v1, m);
            compress(m);
        }
    } else {
        const uint32_t* aw = pool + at.blk_off;
        for (uint32_t b = 0; b < at.nblk; b++) {
#pragma unroll
            for (int j = 0; j < 16; j++) m[j] = aw[b * 16 + j];
            compress(m);
        }
    }
}

// Everything of an EAPOL check that depends on the PMK but not on the nonce-correction attempt.
struct EapolKey {
    uint32_t op1[5], pre1[5];  // keyver 1/2: HMAC-SHA1(PMK) opad midstate, inner state after the shared PRF prefix
    uint32_t op2[8], pre2[8];  // keyver 3: same for HMAC-SHA256
};

// VC: the verify classes (VC_* in tables.hpp) a kernel instantiation handles; code for the others is not emitted,
// so a launch over keyver-2 lines only carries neither the SHA-256/AES-CMAC nor the MD5 path's registers.
template <uint32_t VC>
__device__ __forceinline__ void eapol_key(const LineDev& L, const uint32_t* __restrict__ pool, const uint32_t p[8],
                                          EapolKey& K) {
    constexpr bool has12 = (VC & (VC_KV1 | VC_KV2)) != 0, has3 = (VC & VC_KV3) != 0;
    if (has12 && (!has3 || L.keyver != 3)) {
        uint32_t ip1[5];
        sha1_hmac_mid_pmk(p, ip1, K.op1);
#pragma unroll
        for (int k = 0; k < 5; k++) K.pre1[k] = ip1[k];
        sha1_blocks_kw(K.pre1, pool + L.pre_off, L.pre_nblk);
    } else if constexpr (has3) {
        uint32_t kb[16];
#pragma unroll
        for (int k = 0; k < 16; k++) kb[k] = k < 8 ? p[k] : 0u;
        uint32_t ip2[8];
        sha256_hmac_mid(kb, ip2, K.op2);
#pragma unroll
        for (int k = 0; k < 8; k++) K.pre2[k] = ip2[k];
        sha256_blocks_kw(K.pre2, pool + L.pre_off, L.pre_nblk);
    }
}

// The attempt's PRF blocks after the shared prefix when the attempt is wave-uniform (key-parallel verifier): its
// KW blocks (AttDev.kw_off), patched words included.
__device__ __forceinline__ uint32_t att_nblk(const LineDev& L, const AttDev& at) {
    return L.patch_w0 != NO_PATCH ? L.att_nblk : at.nblk;
}

// MIC of one nonce-correction attempt (common.php:250-300): PRF-512 (keyver 1/2: HMAC-SHA1, first 20 bytes;
// keyver 3: KDF-SHA256) -> KCK -> HMAC-MD5 (1), HMAC-SHA1 (2) or AES-128-CMAC (3) over the EAPOL frame.
// KP (key-parallel): `at` is the same for every lane, so its PRF blocks come as KW blocks; otherwise (attempt-
// parallel, lanes hold different attempts) they are patched per lane.  The EAPOL frame's blocks are KW blocks.
// (AES round keys in LDS, once per key, measured level: the compiler already hoists the loop-invariant key schedule
// out of the CMAC loop, CHANGELOG.md round 2.)
template <uint32_t VC, bool KP>
__device__ __forceinline__ void eapol_mic(const LineDev& L, const uint32_t* __restrict__ pool, const EapolKey& K,
                                          const AttDev& at, const uint32_t* te, uint32_t mic[4]) {
    constexpr bool has1 = (VC & VC_KV1) != 0, has2 = (VC & VC_KV2) != 0, has3 = (VC & VC_KV3) != 0;
    if ((has1 || has2) && (!has3 || L.keyver != 3)) {
        uint32_t st[5], ptk[5];
#pragma unroll
        for (int k = 0; k < 5; k++) st[k] = K.pre1[k];
        if constexpr (KP) sha1_blocks_kw(st, pool + at.kw_off, att_nblk(L, at));
        else prf_blocks(L, pool, at, [&](const uint32_t m[16]) { sha1_compress(st, m); });
        sha1_outer20(K.op1, st, ptk);  // PTK[0..19]; KCK = PTK[0..15]
        if (has2 && (!has1 || L.keyver == 2)) {
            // HMAC-SHA1(KCK, EAPOL): the opad midstate is computed after the inner hash so that the two key-pad
            // compressions are not live at the same time (keeps this class inside 64 VGPRs)
            uint32_t mi[5], mo[5];
            sha1_keypad<4, 0x36363636u>(ptk, mi);
            sha1_blocks_kw(mi, pool + L.mic_off, L.mic_nblk);
            sha1_keypad<4, 0x5c5c5c5cu>(ptk, mo);
            uint32_t o[5];
            sha1_outer20(mo, mi, o);
            mic[0] = o[0]; mic[1] = o[1]; mic[2] = o[2]; mic[3] = o[3];
        } else if constexpr (has1) {
            uint32_t k1[16], mi[4], mo[4];
#pragma unroll
            for (int k = 0; k < 16; k++) k1[k] = k < 4 ? bswap32(ptk[k]) : 0u;
            md5_hmac_mid(k1, mi, mo);
            md5_blocks_km(mi, pool + L.mic_off, L.mic_nblk);
            uint32_t m[16] = {mi[0], mi[1], mi[2], mi[3], 0x80u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 640u, 0};
            md5_compress(mo, m);
            mic[0] = mo[0]; mic[1] = mo[1]; mic[2] = mo[2]; mic[3] = mo[3];
        }
    } else if constexpr (has3) {
        uint32_t st[8];
#pragma unroll
        for (int k = 0; k < 8; k++) st[k] = K.pre2[k];
        if constexpr (KP) sha256_blocks_kw(st, pool + at.kw_off, att_nblk(L, at));
        else prf_blocks(L, pool, at, [&](const uint32_t m[16]) { sha256_compress(st, m); });
        uint32_t m[16] = {st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7],
                          0x80000000u, 0, 0, 0, 0, 0, 0, 768u};
        uint32_t ptk[8];
#pragma unroll
        for (int k = 0; k < 8; k++) ptk[k] = K.op2[k];
        sha256_compress(ptk, m);
        // AES-128-CMAC(KCK = PTK[0..15], EAPOL)  (common.php:72-112)
        uint32_t Lb[4] = {0, 0, 0, 0}, K1[4], K2[4];
        aes128_encrypt_te4(te, ptk, Lb);
        cmac_dbl(Lb, K1);
        cmac_dbl(K1, K2);
        uint32_t c[4] = {0, 0, 0, 0};
        const uint32_t* eb = pool + L.mic_off;
        for (uint32_t b = 0; b < L.mic_nblk; b++) {
            const bool last = b + 1 == L.mic_nblk;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t v = eb[4 * b + k];
                if (last) v ^= L.cmac_complete ? K1[k] : K2[k];
                c[k] ^= v;
            }
            aes128_encrypt_te4(te, ptk, c);
        }
        mic[0] = c[0]; mic[1] = c[1]; mic[2] = c[2]; mic[3] = c[3];
    }
}

__device__ __forceinline__ bool mic_match(const LineDev& L, const uint32_t mic[4]) {
    return mic[0] == L.target[0] && mic[1] == L.target[1] && mic[2] == L.target[2] && mic[3] == L.target[3];
}

// hit reporting: one ballot, one atomic per wave, append to the small hit buffer
// The PMK is re-read from `pw` (word k at pw[k * stride]) only for hit lanes, so it is not held in registers across
// the attempt loop.
__device__ __forceinline__ void report_hits(bool found, uint32_t lane, uint64_t cand, uint32_t line, uint32_t att,
                                            const uint32_t* __restrict__ pw, size_t stride, HitDev* __restrict__ hits,
                                            uint32_t* __restrict__ hitcnt, uint32_t hitcap) {
    const uint64_t m = __ballot(found);
    if (!m) return;
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(hitcnt, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    if (found) {
        const uint32_t idx = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (idx < hitcap) {
            HitDev h;
            h.cand = cand;
            h.line = line;
            h.attempt = att;
#pragma unroll
            for (int k = 0; k < 8; k++) h.pmk[k] = pw[(size_t)k * stride];
            hits[idx] = h;
        }
    }
}

// The AES table image (crypto_dev.hpp: lane-sliced Te0) into the workgroup's LDS, for kernels that verify keyver 3;
// returns the table base (every lane picks its copy inside the lookups).
template <uint32_t VC>
__device__ __forceinline__ const uint32_t* aes_table_lds(uint32_t* te) {
    if constexpr ((VC & VC_KV3) != 0) {
        // four copies of one entry per 16-byte store (words 4j..4j+3 all hold entry 4j >> 5)
        for (uint32_t j = threadIdx.x; j < AES_LDS_WORDS / 4; j += blockDim.x) {
            const uint32_t v = aes_lds_word(4 * j);
            reinterpret_cast<uint4*>(te)[j] = make_uint4(v, v, v, v);
        }
        __syncthreads();
    }
    return te;
}
// Every verify class runs 256-thread workgroups; the keyver-3 ones (32 KiB of LDS) also fit beside a concurrent
// call's PBKDF2 head.
constexpr uint32_t vc_block(uint32_t) { return 256; }

// Key-parallel verification (client scans: many candidates, few attempts): one lane = one candidate slot, one
// wave = up to 64 slots x one line; the line and every attempt are wave-uniform (scalar loads).
// Occupancy target per class: PMKID and keyver 1 fit 64 VGPRs (8 waves/SIMD); keyver 2 is held at 64 too and spills
// 9 VGPRs, which measured level with a 6-wave, spill-free build (profiles/r01/verify_waves_ab); keyver 3 runs at 4
// waves (106 VGPRs, AES round keys computed on the fly; 2 and 6 waves level, 8 waves with 18 spilled VGPRs slower:
// profiles/r02/c5_sched/kv3_waves).
constexpr uint32_t vc_waves(uint32_t vc) { return (vc & VC_KV3) ? 4 : 8; }

template <uint32_t VC>
__global__ __launch_bounds__(vc_block(VC)) __attribute__((amdgpu_waves_per_eu(vc_waves(VC)))) void k_verify(
                                                const uint32_t* __restrict__ pmk, uint32_t cap,
                                                const uint64_t* __restrict__ ids, const uint32_t* __restrict__ counter,
                                                const SegDev* __restrict__ segs, uint32_t nsegs, uint32_t line_base,
                                                const uint32_t* __restrict__ line_list,
                                                const uint32_t* __restrict__ line_poff, uint32_t pstride,
                                                const LineDev* __restrict__ lines, const uint32_t* __restrict__ pool,
                                                const AttDev* __restrict__ atts, HitDev* __restrict__ hits,
                                                uint32_t* __restrict__ hitcnt, uint32_t hitcap) {
    __shared__ __attribute__((aligned(16))) uint32_t te_lds[(VC & VC_KV3) ? AES_LDS_WORDS : 4];
    const uint32_t* te = aes_table_lds<VC>(te_lds);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t segi = blockIdx.x * (blockDim.x >> 6) + wave;
    if (segi >= nsegs) return;
    SegDev sg;
    if (segs) sg = segs[segi];
    else {  // implicit: every 64-slot chunk of the batch against line line_base + blockIdx.y (or line_list[y])
        sg.line = line_list ? line_list[line_base + blockIdx.y] : line_base + blockIdx.y;
        sg.slot = segi * 64;
        sg.count = 64;
    }
    const uint32_t n = counter ? min(*counter, cap) : cap;
    const uint32_t slot = sg.slot + lane;
    const bool active = lane < sg.count && slot < n;
    if (!__any(active)) return;
    const LineDev L = lines[sg.line];
    // PMKs of multi-group launches: the line's ESSID group owns slots [poff, poff + cap) of a pstride-wide array
    const uint32_t poff = line_poff ? line_poff[sg.line] : 0u;

    uint32_t p[8];
#pragma unroll
    for (int k = 0; k < 8; k++) p[k] = active ? pmk[(size_t)k * pstride + poff + slot] : 0u;
    const uint64_t cand = active ? (ids ? ids[slot] : (uint64_t)slot) : 0ull;

    bool found = false;
    uint32_t found_att = 0;

    constexpr bool has_pmkid = (VC & VC_PMKID) != 0, has_eapol = (VC & ~VC_PMKID) != 0;
    if (has_pmkid && (!has_eapol || L.kind == LINE_PMKID)) {
        uint32_t ip[5], op[5], st[5], out[5];
        sha1_hmac_mid_pmk(p, ip, op);
#pragma unroll
        for (int k = 0; k < 5; k++) st[k] = ip[k];
        sha1_blocks_kw(st, pool + L.msg_off, L.msg_nblk);
        sha1_outer20(op, st, out);
        found = active && out[0] == L.target[0] && out[1] == L.target[1] && out[2] == L.target[2] &&
                out[3] == L.target[3];
    } else if constexpr (has_eapol) {
        EapolKey K;
        eapol_key<VC>(L, pool, p, K);
        // PHP mutates $n across keys (common.php:255-259): list k serves the k-th non-null key, the last list the rest
        const uint32_t sel = active ? (uint32_t)min<uint64_t>(cand, (uint64_t)(L.nlists - 1)) : 0xffffffffu;
        uint32_t lo = sel, hi = active ? sel : 0u;
        for (int o = 32; o >= 1; o >>= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
        }
        lo = __builtin_amdgcn_readfirstlane(lo);
        hi = __builtin_amdgcn_readfirstlane(hi);
        for (uint32_t list = lo; list <= hi; list++) {
            const bool mine = active && sel == list;
            if (!__any(mine)) continue;
            const AttDev* al = atts + L.list_off + list * L.natt;
            for (uint32_t a = 0; a < L.natt; a++) {
                uint32_t mic[4];
                eapol_mic<VC, true>(L, pool, K, al[a], te, mic);
                if (mine && !found && mic_match(L, mic)) {
                    found = true;
                    found_att = a;
                }
            }
        }
    }
    report_hits(found, lane, cand, sg.line, found_att, pmk + poff + slot, pstride, hits, hitcnt, hitcap);
}

// Attempt-parallel verification (server checks with wide nonce windows, e.g. nc=128 -> 261 attempts,
// common.php:250-300) in two launches.
//
// k_eapol_keys: lane = (segment, key) pair, computes everything of the check that depends on the PMK but not on
// the attempt (HMAC key midstates, PRF prefix: EapolKey) once per pair into a SoA scratch array, word w of pair
// (segment i, key k) at keys[w * kstride + segk * i + k] (segk = the most keys a segment holds, 1..64: the host cuts
// attempt-parallel segments to ATT_SEG_KEYS (16) keys, so the scratch is sized for that, not for 64).
//
// k_verify_att: the (key, attempt) items of a segment are laid out key-major and cut into waves of 64 lanes, so
// every lane runs one attempt and a wave ends only where the segment does (segs[i].pad = the segment's first wave
// within the launch).  A wave spans at most two keys (natt >= ATT_PARALLEL_MIN = 64); each lane loads its key's
// EapolKey.  One wave per key with 64 attempts per pass left 59 of 64 lanes idle in the fifth pass of a 261-attempt
// list and recomputed the key state in every wave; here no lane idles before the segment's last wave.  Every
// matching attempt is reported (at most two per key: one BE, one LE value can equal the true nonce); the host
// keeps the first key in input order, then the first attempt in PHP order.
template <uint32_t VC>
constexpr uint32_t eapol_key_words() { return (VC & VC_KV3) ? 16u : 10u; }

template <uint32_t VC>
__global__ __launch_bounds__(256) void k_eapol_keys(const uint32_t* __restrict__ pmk, uint32_t cap,
                                                    const SegDev* __restrict__ segs, uint32_t nsegs,
                                                    const LineDev* __restrict__ lines,
                                                    const uint32_t* __restrict__ pool, uint32_t* __restrict__ keys,
                                                    uint32_t kstride, uint32_t segk) {
    const uint32_t segi = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint32_t k = threadIdx.x & 63;
    if (segi >= nsegs) return;
    const SegDev sg = segs[segi];
    if (k >= sg.count || k >= segk) return;
    const LineDev L = lines[sg.line];
    uint32_t p[8];
#pragma unroll
    for (int w = 0; w < 8; w++) p[w] = pmk[(size_t)w * cap + sg.slot + k];
    EapolKey K;
    eapol_key<VC>(L, pool, p, K);
    uint32_t* o = keys + (size_t)segi * segk + k;
    if ((VC & VC_KV3) && L.keyver == 3) {
#pragma unroll
        for (int w = 0; w < 8; w++) {
            o[(size_t)w * kstride] = K.op2[w];
            o[(size_t)(8 + w) * kstride] = K.pre2[w];
        }
    } else {
#pragma unroll
        for (int w = 0; w < 5; w++) {
            o[(size_t)w * kstride] = K.op1[w];
            o[(size_t)(5 + w) * kstride] = K.pre1[w];
        }
    }
}

template <uint32_t VC>
__global__ __launch_bounds__(vc_block(VC)) __attribute__((amdgpu_waves_per_eu(vc_waves(VC)))) void k_verify_att(
                                                    const uint32_t* __restrict__ pmk, uint32_t cap,
                                                    const uint64_t* __restrict__ ids,
                                                    const SegDev* __restrict__ segs, uint32_t nsegs, uint32_t nwaves,
                                                    const uint32_t* __restrict__ keys, uint32_t kstride,
                                                    uint32_t segk, const LineDev* __restrict__ lines,
                                                    const uint32_t* __restrict__ pool,
                                                    const AttDev* __restrict__ atts, HitDev* __restrict__ hits,
                                                    uint32_t* __restrict__ hitcnt, uint32_t hitcap,
                                                    uint32_t* __restrict__ first_hit) {
    __shared__ __attribute__((aligned(16))) uint32_t te_lds[(VC & VC_KV3) ? AES_LDS_WORDS : 4];
    const uint32_t* te = aes_table_lds<VC>(te_lds);  // (every wave of the block helps fill the table first)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (gw >= nwaves) return;
    // the segment holding wave gw: last i with segs[i].pad <= gw (wave-uniform binary search, scalar loads)
    uint32_t lo = 0, hi = nsegs;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (segs[mid].pad <= gw) lo = mid;
        else hi = mid;
    }
    const uint32_t segi = lo;
    const SegDev sg = segs[segi];
    const LineDev L = lines[sg.line];
    // first-key early exit: every key of this wave comes after a key of the same job that already matched.
    // first_hit holds key ordinals (ids: a job's keys in input order, numbered across the call's chunks), so the
    // rule holds across chunks too.
    if (first_hit) {
        const uint32_t f = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(first_hit + sg.line, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const uint32_t s0 = sg.slot + (gw - sg.pad) * 64 / L.natt;  // the wave's first key (wave-uniform)
        const uint32_t o0 = ids ? (uint32_t)ids[s0] : s0;
        if (o0 > f) return;
    }
    const uint32_t item = (gw - sg.pad) * 64 + lane;
    const uint32_t k = item / L.natt, a = item - k * L.natt;
    const bool active = k < sg.count;
    const uint32_t kk = active ? k : sg.count - 1;  // idle lanes of the segment's last wave repeat a real key
    const uint32_t slot = sg.slot + kk;
    const uint64_t cand = ids ? ids[slot] : (uint64_t)slot;
    EapolKey K;
    const uint32_t* kp = keys + (size_t)segi * segk + kk;
    if ((VC & VC_KV3) && L.keyver == 3) {
#pragma unroll
        for (int w = 0; w < 8; w++) {
            K.op2[w] = kp[(size_t)w * kstride];
            K.pre2[w] = kp[(size_t)(8 + w) * kstride];
        }
    } else {
#pragma unroll
        for (int w = 0; w < 5; w++) {
            K.op1[w] = kp[(size_t)w * kstride];
            K.pre1[w] = kp[(size_t)(5 + w) * kstride];
        }
    }
    const uint32_t sel = (uint32_t)min<uint64_t>(cand, (uint64_t)(L.nlists - 1));
    uint32_t mic[4];
    eapol_mic<VC, false>(L, pool, K, atts[L.list_off + sel * L.natt + a], te, mic);
    const bool found = active && mic_match(L, mic);
    if (found && first_hit)
        __hip_atomic_fetch_min(first_hit + sg.line, (uint32_t)cand, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    report_hits(found, lane, cand, sg.line, a, pmk + slot, cap, hits, hitcnt, hitcap);
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_prep_dict(const uint64_t* off, const uint8_t* bytes, uint64_t first, uint32_t count, uint32_t minlen,
                            uint32_t maxlen, uint32_t* mid, uint64_t* ids, uint32_t* counter, uint32_t cap,
                            bool compact, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prep_dict, dim3(cdiv(count, 256)), dim3(256), 0, s, off, bytes, first, count, minlen, maxlen,
                       mid, ids, counter, cap, compact ? 1u : 0u);
    return hipGetLastError();
}

hipError_t launch_prep_keys(const uint64_t* koff, const uint32_t* klen, const uint8_t* kbytes, const uint32_t* uslot,
                            uint32_t count, uint32_t* mid, uint32_t cap, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prep_keys, dim3(cdiv(count, 256)), dim3(256), 0, s, koff, klen, kbytes, uslot, count, mid, cap);
    return hipGetLastError();
}

hipError_t launch_prep_numeric(uint64_t first, uint32_t count, uint32_t digits, uint32_t* mid, uint64_t* ids,
                               uint32_t cap, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(k_prep_numeric, dim3(cdiv(count, 256)), dim3(256), 0, s, first, count, digits, mid, ids, cap);
    return hipGetLastError();
}

hipError_t launch_pbkdf2_plain(const uint32_t* mid, uint32_t cap, uint32_t base, uint32_t count,
                               const uint32_t* counter, const uint32_t* salt, uint32_t nsalt, uint32_t* pmk,
                               hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pbkdf2, dim3(cdiv(count, 256), 2), dim3(256), 0, s, mid, cap, base, count, counter, salt, nsalt,
                       pmk);
    return hipGetLastError();
}

// Lone-wave derives are rounded up to whole waves of live lanes (the extra lanes repeat the last key and store
// nothing).  On gfx950 a wave whose EXEC mask is partial runs a dependent VALU chain 18 % slower alone on its SIMD
// and 39 % slower with 8 such waves on the chip, at the same shader clock (tools/clock_idle.hip,
// profiles/r04/small_call/clock_lanes.jsonl); a one-key server call took 9.6-11.8 ms against 8.3 ms for 202 keys.
// Padded, it takes 8.4 ms.
constexpr uint32_t LONE_PAD = 64;

hipError_t launch_pbkdf2_ms_plain(const uint32_t* mid, uint32_t cap, uint32_t count, const uint32_t* pool,
                                  const uint32_t* sref, uint32_t* pmk, hipStream_t s) {
    count = min(count, cap);
    if (count == 0) return hipSuccess;
    const uint32_t launch = (count + LONE_PAD - 1) / LONE_PAD * LONE_PAD;
    hipLaunchKernelGGL(k_pbkdf2_ms, dim3(cdiv(launch, 256), 2), dim3(256), 0, s, mid, cap, launch, pool, sref, pmk,
                       count);
    return hipGetLastError();
}

hipError_t launch_gather_pmk(const uint32_t* upmk, uint32_t ucap, const uint32_t* cpmk, const uint32_t* src,
                             uint32_t n, uint32_t* pmk, uint32_t cap, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_pmk, dim3(cdiv(n, 256)), dim3(256), 0, s, upmk, ucap, cpmk, src, n, pmk, cap);
    return hipGetLastError();
}

hipError_t launch_hits_out(const uint32_t* hitcnt, const HitDev* hits, uint32_t hitcap, uint32_t* out,
                           const uint32_t* raised, hipStream_t s) {
    const uint32_t blocks = cdiv((uint64_t)hitcap * (sizeof(HitDev) / 4), 256);
    hipLaunchKernelGGL(k_hits_out, dim3(blocks < 1 ? 1 : blocks > 64 ? 64 : blocks), dim3(256), 0, s, hitcnt, hits,
                       hitcap, out, raised);
    return hipGetLastError();
}

hipError_t launch_pbkdf2_ms_tail(const uint32_t* mid, uint32_t cap, uint32_t count, const uint32_t* pool,
                                 const uint32_t* sref, uint32_t* pmk, uint32_t* flag, uint32_t prio,
                                 uint32_t* raised, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pbkdf2_ms_tail, dim3(cdiv(count, 256), 2), dim3(256), 0, s, mid, cap, count, pool, sref, pmk,
                       flag, prio, raised);
    return hipGetLastError();
}

hipError_t launch_set_flag(uint32_t* flag, hipStream_t s) {
    hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(64), 0, s, flag);
    return hipGetLastError();
}


hipError_t launch_set_pmk(uint32_t* pmk, uint32_t cap, uint32_t slot, const uint32_t w[8], hipStream_t s) {
    uint4 lo = make_uint4(w[0], w[1], w[2], w[3]), hi = make_uint4(w[4], w[5], w[6], w[7]);
    hipLaunchKernelGGL(k_set_pmk, dim3(1), dim3(64), 0, s, pmk, cap, slot, lo, hi);
    return hipGetLastError();
}

#define DWPA_VC_DISPATCH(VCV, CALL) \
    switch (VCV) {                  \
    case VC_PMKID: CALL(VC_PMKID); break; \
    case VC_KV1: CALL(VC_KV1); break;     \
    case VC_KV2: CALL(VC_KV2); break;     \
    case VC_KV3: CALL(VC_KV3); break;     \
    case VC_KV1 | VC_KV2: CALL(VC_KV1 | VC_KV2); break; \
    default: CALL(VC_ALL); break;         \
    }

hipError_t launch_verify(const uint32_t* pmk, uint32_t cap, const uint64_t* ids, const uint32_t* counter,
                         const SegDev* segs, uint32_t nsegs, uint32_t line_base, uint32_t nlines, const LineDev* lines,
                         const uint32_t* pool, const AttDev* atts, HitDev* hits, uint32_t* hitcnt, uint32_t hitcap,
                         uint32_t vc, hipStream_t s, const uint32_t* line_list, const uint32_t* line_poff,
                         uint32_t pstride) {
    if (nsegs == 0 || nlines == 0) return hipSuccess;
    if (!pstride) pstride = cap;
#define DWPA_LAUNCH_VERIFY(V)                                                                                  \
    hipLaunchKernelGGL(k_verify<V>, dim3(cdiv(nsegs, vc_block(V) / 64), segs ? 1 : nlines), dim3(vc_block(V)),  \
                       0, s, pmk, cap, ids, counter, segs, nsegs, line_base, line_list, line_poff, pstride, lines,  \
                       pool, atts, hits, hitcnt, hitcap)
    DWPA_VC_DISPATCH(vc, DWPA_LAUNCH_VERIFY)
#undef DWPA_LAUNCH_VERIFY
    return hipGetLastError();
}

uint32_t eapol_key_words(uint32_t vc) { return (vc & VC_KV3) ? 16u : 10u; }

hipError_t launch_verify_att(const uint32_t* pmk, uint32_t cap, const uint64_t* ids, const SegDev* segs,
                             uint32_t nsegs, uint32_t nwaves, uint32_t* keys, uint32_t kstride, uint32_t segk,
                             const LineDev* lines, const uint32_t* pool, const AttDev* atts, HitDev* hits,
                             uint32_t* hitcnt, uint32_t hitcap, uint32_t* first_hit, uint32_t vc, hipStream_t s) {
    if (nsegs == 0 || nwaves == 0) return hipSuccess;
    if (segk < 1 || segk > 64 || kstride < (uint64_t)nsegs * segk) return hipErrorInvalidValue;
#define DWPA_LAUNCH_VERIFY_ATT(V)                                                                                 \
    hipLaunchKernelGGL(k_eapol_keys<V>, dim3(cdiv((uint64_t)nsegs * 64, 256)), dim3(256), 0, s, pmk, cap, segs,   \
                       nsegs, lines, pool, keys, kstride, segk);                                                   \
    hipLaunchKernelGGL(k_verify_att<V>, dim3(cdiv(nwaves, vc_block(V) / 64)), dim3(vc_block(V)), 0, s, pmk, cap, \
                       ids, segs, nsegs, nwaves, keys, kstride, segk, lines, pool, atts, hits, hitcnt, hitcap,    \
                       first_hit)
    DWPA_VC_DISPATCH(vc & ~VC_PMKID, DWPA_LAUNCH_VERIFY_ATT)
#undef DWPA_LAUNCH_VERIFY_ATT
    return hipGetLastError();
}

hipError_t launch_pbkdf2_mg_plain(const uint32_t* mid, uint32_t cap, const uint32_t* counter, uint32_t ngroups,
                                  const uint32_t* salt, const uint32_t* gsalt, uint32_t* pmk, uint32_t pstride,
                                  hipStream_t s) {
    if (ngroups == 0 || cap == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pbkdf2_mg, dim3(cdiv((uint64_t)ngroups * cap, 256), 2), dim3(256), 0, s, mid, cap, counter,
                       ngroups, salt, gsalt, pmk, pstride);
    return hipGetLastError();
}

}  // namespace dwpa
