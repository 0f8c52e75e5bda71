// crypto_dev.hpp -- gfx950 device primitives for the m22000 path (integer VALU only, no MFMA).
//
// SHA-1 is the hot primitive: PBKDF2-HMAC-SHA1 x4096 (web/common.php:178-180,246-248) is ~99 % of all work.
// Rotates lower to v_alignbit_b32, Ch/Maj/Parity to v_bfi_b32 / v_bitop3_b32 / v_xor3_b32, and sums of three
// to v_add3_u32.  MD5 (keyver 1 MIC, common.php:262-265), SHA-256 (keyver 3 KDF, :270-273) and AES-128
// (CMAC, :56-112) are the verifier-side primitives; they run once per nonce-correction attempt, not 4096x.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

namespace dwpa {

__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, 32u - n); }
__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 3-input XOR in one VALU op: v_bitop3_b32 with truth table 0x96 (gfx950).  LLVM selects bitop3 for Ch/Maj but
// splits XOR3 into two v_xor_b32, which costs ~100 extra ops per compression in the schedule and parity rounds.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// Majority in one op (bitop3 truth table 0xE8); left to itself LLVM emits v_xor + v_bfi for it.
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// Ch(b, c, d) = (b & c) | (~b & d) in one full-rate op (bitop3 truth table 0xCA: src0 = 0xF0, src1 = 0xCC,
// src2 = 0xAA).  Left to itself LLVM emits a bitop3 for (c ^ d) & b and folds the final xor into the next add as
// v_xad_u32, one instruction fewer but a half-rate (4-cycle) op on gfx950: 2 extra SIMD-cycles per Ch round.
__device__ __forceinline__ uint32_t ch3(uint32_t b, uint32_t c, uint32_t d) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(b), "v"(c), "v"(d));
    return r;
}
// a ^ b ^ K with a wave-uniform constant K in an SGPR (VOP3 on gfx9 takes no literal operand).
__device__ __forceinline__ uint32_t xor3s(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}


// ------------------------------------------------------------------------------------------------
// SHA-1
// ------------------------------------------------------------------------------------------------
#define DWPA_SHA1_CH(b, c, d) ((((c) ^ (d)) & (b)) ^ (d))
#define DWPA_SHA1_PAR(b, c, d) ((b) ^ (c) ^ (d))
#define DWPA_SHA1_MAJ(b, c, d) (((b) & (c)) | (((b) | (c)) & (d)))

constexpr uint32_t SHA1_K0 = 0x5a827999u, SHA1_K1 = 0x6ed9eba1u, SHA1_K2 = 0x8f1bbcdcu, SHA1_K3 = 0xca62c1d6u;
constexpr uint32_t SHA1_IV0 = 0x67452301u, SHA1_IV1 = 0xefcdab89u, SHA1_IV2 = 0x98badcfeu, SHA1_IV3 = 0x10325476u,
                   SHA1_IV4 = 0xc3d2e1f0u;

// Generic round functions and schedule (verify kernels).  DWPA_SHA1_GENERIC_BITOP selects how many of them are
// forced into one v_bitop3_b32: 0 none (LLVM splits XOR3 into two v_xor and emits Ch/Maj as bitop3 + v_xad),
// 1 the schedule's XOR3, 2 also the parity rounds, 3 also Ch and Maj.  3 keeps every verify class inside its VGPR
// budget and took k_verify<kv2> from 13.2 to 11.2 ms per C2 step, k_verify_att<kv2> from 3.66 to 3.11 ms per C5
// call (profiles/r01/generic_sha1_ab.json).
#ifndef DWPA_SHA1_GENERIC_BITOP
#define DWPA_SHA1_GENERIC_BITOP 3
#endif
template <int T>
__device__ __forceinline__ uint32_t sha1_f(uint32_t b, uint32_t c, uint32_t d) {
    if constexpr (T < 20) {
        if constexpr (DWPA_SHA1_GENERIC_BITOP >= 3) return ch3(b, c, d);
        else return DWPA_SHA1_CH(b, c, d);
    } else if constexpr (T < 40 || T >= 60) {
        if constexpr (DWPA_SHA1_GENERIC_BITOP >= 2) return xor3(b, c, d);
        else return DWPA_SHA1_PAR(b, c, d);
    } else {
        if constexpr (DWPA_SHA1_GENERIC_BITOP >= 3) return maj3(b, c, d);
        else return DWPA_SHA1_MAJ(b, c, d);
    }
}
// W[t] of the generic schedule: xor of four words (one bitop3 + one xor when DWPA_SHA1_GENERIC_BITOP >= 1)
__device__ __forceinline__ uint32_t sha1_w4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    if constexpr (DWPA_SHA1_GENERIC_BITOP >= 1) return xor3(a, b, c) ^ d;
    else return a ^ b ^ c ^ d;
}
template <int T>
__device__ __forceinline__ constexpr uint32_t sha1_k() {
    return T < 20 ? SHA1_K0 : T < 40 ? SHA1_K1 : T < 60 ? SHA1_K2 : SHA1_K3;
}

// Generic compression: st <- SHA1_compress(st, m[0..15]) (big-endian message words).
__device__ __forceinline__ void sha1_compress(uint32_t st[5], const uint32_t m[16]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = m[i];
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
#define DWPA_SHA1_STEP(T)                                                                                   \
    {                                                                                                       \
        uint32_t wt;                                                                                        \
        if constexpr ((T) < 16) wt = w[(T)];                                                                \
        else {                                                                                              \
            wt = rotl(sha1_w4(w[((T) - 3) & 15], w[((T) - 8) & 15], w[((T) - 14) & 15], w[(T) & 15]), 1);   \
            w[(T) & 15] = wt;                                                                               \
        }                                                                                                   \
        uint32_t t = rotl(a, 5) + sha1_f<(T)>(b, c, d) + e + sha1_k<(T)>() + wt;                            \
        e = d; d = c; c = rotl(b, 30); b = a; a = t;                                                        \
    }
#define DWPA_SHA1_STEP4(T) DWPA_SHA1_STEP(T) DWPA_SHA1_STEP(T + 1) DWPA_SHA1_STEP(T + 2) DWPA_SHA1_STEP(T + 3)
#define DWPA_SHA1_STEP20(T) DWPA_SHA1_STEP4(T) DWPA_SHA1_STEP4(T + 4) DWPA_SHA1_STEP4(T + 8) DWPA_SHA1_STEP4(T + 12) DWPA_SHA1_STEP4(T + 16)
    DWPA_SHA1_STEP20(0)
    DWPA_SHA1_STEP20(20)
    DWPA_SHA1_STEP20(40)
    DWPA_SHA1_STEP20(60)
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}

// HMAC-SHA1 key midstate with the per-midstate invariants of rounds 0-1 folded out of the 4096-iteration loop.
// For a fixed state H the first two rounds only depend on H and the first two message words:
//   round 0: a1 = rotl(H0,5) + Ch(H1,H2,H3) + H4 + K + W0            = c0 + W0
//   round 1: a2 = rotl(a1,5) + Ch(H0,rotl(H1,30),H2) + H3 + K + W1     = rotl(a1,5) + c1 + W1
// leaving (a2, a1, rotl(H0,30), rotl(H1,30), H2) as the state entering round 2.
struct Sha1Mid {
    uint32_t h0, h1, h2, h3, h4;
    uint32_t c0, c1, r0, r1;
};

__device__ __forceinline__ Sha1Mid sha1_mid(const uint32_t h[5]) {
    Sha1Mid m;
    m.h0 = h[0]; m.h1 = h[1]; m.h2 = h[2]; m.h3 = h[3]; m.h4 = h[4];
    m.r0 = rotl(h[0], 30);
    m.r1 = rotl(h[1], 30);
    m.c0 = rotl(h[0], 5) + DWPA_SHA1_CH(h[1], h[2], h[3]) + h[4] + SHA1_K0;
    m.c1 = DWPA_SHA1_CH(h[0], m.r1, h[2]) + h[3] + SHA1_K0;
    return m;
}

// Message layouts with compile-time words: var(s) says whether W[s] (s < 16) is a run-time value, cst(s) is its value
// otherwise.  Words past 15 are schedule words (run-time).
// Msg84: the 84-byte HMAC inner/outer message (a 20-byte digest after a 64-byte pad block): W0..W4 variable,
// W5 = 0x80000000, W6..W14 = 0, W15 = 672.
struct Msg84 {
    static constexpr bool var(int s) { return s >= 16 || s <= 4; }
    static constexpr uint32_t cst(int s) { return s == 5 ? 0x80000000u : s == 15 ? 672u : 0u; }
};
// MsgKey<NV, P>: an HMAC key pad block of a key of NV words (PMK: 8, KCK: 4): W[s] = key[s] ^ P for s < NV, P after.
template <int NV, uint32_t P>
struct MsgKey {
    static constexpr bool var(int s) { return s >= 16 || s < NV; }
    static constexpr uint32_t cst(int s) { return s >= NV && s < 16 ? P : 0u; }
};
constexpr bool w84_var(int s) { return Msg84::var(s); }
constexpr uint32_t w84_const(int s) { return Msg84::cst(s); }

// W[T]: the recurrence applied 2^j times -- for T >= 16 * 2^j,
//   W[T] = rotl(W[T - 3s] ^ W[T - 8s] ^ W[T - 14s] ^ W[T - 16s], s),  s = 2^j
// (j = 0 is the schedule's definition; j = 1 and j = 2 follow by substituting it into itself).  Each form costs one
// rotate; the XORs depend on how many of its four sources are variable (compile-time words fold into one constant).
// The 84-byte message's zero words W6..W14 make the j = 1 form cheaper for T = 34..46 and the j = 2 form for
// T = 64..78: 84 instead of 112 XOR-type ops per compression, at the price of keeping W0..W4 and W16..W22 live
// longer.  DWPA_SCHED_WIDE is the largest j used (0 = the plain recurrence) and DWPA_SCHED_J2_MIN the first t that may
// use j = 2: j <= 1 by default (the lone-wave kernels of kernels.hip), j = 2 from t = 73 in the issue-pass kernels,
// which define both at the top of pbkdf2_gfx950.hip (profiles/r05/sched_identities/).
#ifndef DWPA_SCHED_WIDE
#define DWPA_SCHED_WIDE 1
#endif
template <class M>
constexpr uint32_t sched_const(int T, int j) {
    const int sh = 1 << j;
    return (M::var(T - 3 * sh) ? 0u : M::cst(T - 3 * sh)) ^ (M::var(T - 8 * sh) ? 0u : M::cst(T - 8 * sh)) ^
           (M::var(T - 14 * sh) ? 0u : M::cst(T - 14 * sh)) ^ (M::var(T - 16 * sh) ? 0u : M::cst(T - 16 * sh));
}
template <class M>
constexpr int sched_nv(int T, int j) {
    const int sh = 1 << j;
    return (int)M::var(T - 3 * sh) + (int)M::var(T - 8 * sh) + (int)M::var(T - 14 * sh) + (int)M::var(T - 16 * sh);
}
// XOR-type ops of form j: a 3-input op takes two more terms, the folded constant counts as one term
template <class M>
constexpr int sched_cost(int T, int j) { return (sched_nv<M>(T, j) + (sched_const<M>(T, j) != 0u ? 1 : 0)) / 2; }
#ifndef DWPA_SCHED_J2_MIN
#define DWPA_SCHED_J2_MIN 64
#endif
template <class M>
constexpr int sched_form(int T) {
    int best = 0;
    for (int j = 1; j <= DWPA_SCHED_WIDE; j++)
        if (T >= (16 << j) && (j < 2 || T >= DWPA_SCHED_J2_MIN) && sched_cost<M>(T, j) < sched_cost<M>(T, best))
            best = j;
    return best;
}

// W[T] (T >= 16) of layout M from the full message array w[0..T-1] (compile-time indices: registers, not memory).
template <class M, int T>
__device__ __forceinline__ uint32_t sched_w(const uint32_t w[80]) {
    constexpr int j = sched_form<M>(T), sh = 1 << j;
    constexpr int s0 = T - 3 * sh, s1 = T - 8 * sh, s2 = T - 14 * sh, s3 = T - 16 * sh;
    constexpr uint32_t K = sched_const<M>(T, j);
    constexpr int nv = sched_nv<M>(T, j);
    uint32_t v[4] = {0, 0, 0, 0};
    int n = 0;
    if constexpr (M::var(s0)) v[n++] = w[s0];
    if constexpr (M::var(s1)) v[n++] = w[s1];
    if constexpr (M::var(s2)) v[n++] = w[s2];
    if constexpr (M::var(s3)) v[n++] = w[s3];
    uint32_t x;
    if constexpr (nv == 4) x = xor3(v[0], v[1], v[2]) ^ v[3];
    else if constexpr (nv == 3) {
        if constexpr (K == 0) x = xor3(v[0], v[1], v[2]);
        else x = xor3(v[0], v[1], v[2]) ^ K;
    } else if constexpr (nv == 2) {
        if constexpr (K == 0) x = v[0] ^ v[1];
        else x = xor3s(v[0], v[1], K);
    } else if constexpr (nv == 1) {
        if constexpr (K == 0) x = v[0];
        else x = v[0] ^ K;
    } else {
        x = K;
    }
    return rotl(x, (uint32_t)sh);
}

// Issue-slot spacer.  On gfx950 a wave whose VALU stream mixes 4-cycle ops (alignbit, add3) with 2-cycle ops
// (xor, bitop3, add) issues every VALU at the 4-cycle rate; a scalar s_nop between them restores near-additive
// issue (tools/valu_mix*, profiles/).  NOP selects where spacers go in the SHA-1 rounds (0 = none).
template <int NOP, int WHERE>
__device__ __forceinline__ void spacer() {
    if constexpr ((NOP & WHERE) != 0) asm volatile("s_nop 0");
}

template <class M, int T, int NOP = 0>
__device__ __forceinline__ void step_m(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e, uint32_t w[80]) {
    uint32_t f;
    if constexpr (T < 20) f = ch3(b, c, d);
    else if constexpr (T < 40) f = xor3(b, c, d);
    else if constexpr (T < 60) f = maj3(b, c, d);
    else f = xor3(b, c, d);
    uint32_t t;
    if constexpr (T < 16 && !M::var(T)) {
        t = rotl(a, 5) + f + e + (sha1_k<T>() + M::cst(T));
    } else {
        uint32_t wt;
        if constexpr (T < 16) wt = w[T];
        else {
            wt = sched_w<M, T>(w);
            spacer<NOP, 1>();
            w[T] = wt;
        }
        t = rotl(a, 5) + f + e + sha1_k<T>() + wt;
    }
    spacer<NOP, 2>();
    e = d; d = c; c = rotl(b, 30); b = a; a = t;
    spacer<NOP, 4>();
}

template <class M, int NOP, int T0, int... Ts>
__device__ __forceinline__ void steps_m(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e, uint32_t w[80],
                                        std::integer_sequence<int, T0, Ts...>) {
    step_m<M, T0, NOP>(a, b, c, d, e, w);
    if constexpr (sizeof...(Ts) > 0) steps_m<M, NOP>(a, b, c, d, e, w, std::integer_sequence<int, Ts...>{});
}
template <class M, int Lo, int NOP, int... Is>
__device__ __forceinline__ void run_steps_m(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                                            uint32_t w[80], std::integer_sequence<int, Is...>) {
    steps_m<M, NOP>(a, b, c, d, e, w, std::integer_sequence<int, (Lo + Is)...>{});
}

// out <- SHA1_compress(M, in[0..4] || 0x80 || 0.. || bitlen(64+20)): the PBKDF2/HMAC inner-loop compression
// (a 20-byte digest hashed after a 64-byte key pad block).  Rounds 0-1 come from the folded midstate invariants,
// rounds 2-79 use the constant-folded message schedule above.
template <int NOP = 0>
__device__ __forceinline__ void sha1_84(const Sha1Mid& M, const uint32_t in[5], uint32_t out[5]) {
    uint32_t w[80];
    w[0] = in[0]; w[1] = in[1]; w[2] = in[2]; w[3] = in[3]; w[4] = in[4];
#pragma unroll
    for (int i = 5; i < 16; i++) w[i] = w84_const(i);
    uint32_t a1 = M.c0 + w[0];
    uint32_t a2 = rotl(a1, 5) + M.c1 + w[1];
    uint32_t a = a2, b = a1, c = M.r0, d = M.r1, e = M.h2;
    run_steps_m<Msg84, 2, NOP>(a, b, c, d, e, w, std::make_integer_sequence<int, 78>{});
    out[0] = M.h0 + a; out[1] = M.h1 + b; out[2] = M.h2 + c; out[3] = M.h3 + d; out[4] = M.h4 + e;
}

// Compression of a wave-uniform message block whose schedule the host has expanded: kw[t] = K_t + W_t for t < 80
// (tables.hpp "KW blocks").  kw is read with scalar loads, so a round costs rotl5 + f + 3 adds + rotl30 and the
// 64-word schedule (64 rotl1 + 128 xor per compression) is gone -- about a third of the generic compression.
__device__ __forceinline__ void sha1_compress_kw(uint32_t st[5], const uint32_t* __restrict__ kw) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
#define DWPA_SHA1_KW(T)                                                                                     \
    {                                                                                                       \
        const uint32_t t = rotl(a, 5) + sha1_f<(T)>(b, c, d) + e + kw[(T)];                                 \
        e = d; d = c; c = rotl(b, 30); b = a; a = t;                                                        \
    }
#define DWPA_SHA1_KW4(T) DWPA_SHA1_KW(T) DWPA_SHA1_KW(T + 1) DWPA_SHA1_KW(T + 2) DWPA_SHA1_KW(T + 3)
#define DWPA_SHA1_KW20(T) DWPA_SHA1_KW4(T) DWPA_SHA1_KW4(T + 4) DWPA_SHA1_KW4(T + 8) DWPA_SHA1_KW4(T + 12) DWPA_SHA1_KW4(T + 16)
    DWPA_SHA1_KW20(0)
    DWPA_SHA1_KW20(20)
    DWPA_SHA1_KW20(40)
    DWPA_SHA1_KW20(60)
#undef DWPA_SHA1_KW20
#undef DWPA_SHA1_KW4
#undef DWPA_SHA1_KW
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}

__device__ __forceinline__ void sha1_iv(uint32_t st[5]) {
    st[0] = SHA1_IV0; st[1] = SHA1_IV1; st[2] = SHA1_IV2; st[3] = SHA1_IV3; st[4] = SHA1_IV4;
}

// SHA1_compress(IV, key ^ P || P..P) for a key of NV words: an HMAC ipad (P = 0x36363636) or opad (0x5c5c5c5c)
// midstate, with the pad words folded into the schedule (MsgKey).  The verifiers' PMK (8 words) and KCK (4 words).
template <int NV, uint32_t P>
__device__ __forceinline__ void sha1_keypad(const uint32_t* key, uint32_t out[5]) {
    uint32_t w[80];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = i < NV ? key[i] ^ P : P;
    uint32_t a = SHA1_IV0, b = SHA1_IV1, c = SHA1_IV2, d = SHA1_IV3, e = SHA1_IV4;
    run_steps_m<MsgKey<NV, P>, 0, 0>(a, b, c, d, e, w, std::make_integer_sequence<int, 80>{});
    out[0] = SHA1_IV0 + a; out[1] = SHA1_IV1 + b; out[2] = SHA1_IV2 + c; out[3] = SHA1_IV3 + d; out[4] = SHA1_IV4 + e;
}
// HMAC-SHA1 midstates of a 32-byte key (the PMK).
__device__ __forceinline__ void sha1_hmac_mid_pmk(const uint32_t p[8], uint32_t ipad[5], uint32_t opad[5]) {
    sha1_keypad<8, 0x36363636u>(p, ipad);
    sha1_keypad<8, 0x5c5c5c5cu>(p, opad);
}
// HMAC outer hash over a 20-byte inner digest: the 84-byte message's folded schedule (sha1_84) from the opad state.
__device__ __forceinline__ void sha1_outer20(const uint32_t opad[5], const uint32_t in[5], uint32_t out[5]) {
    sha1_84(sha1_mid(opad), in, out);
}

// HMAC-SHA1 key block (<= 64 bytes, big-endian words, zero padded) -> ipad / opad midstates.
__device__ __forceinline__ void sha1_hmac_mid(const uint32_t kb[16], uint32_t ipad[5], uint32_t opad[5]) {
    uint32_t blk[16];
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = kb[i] ^ 0x36363636u;
    sha1_iv(ipad);
    sha1_compress(ipad, blk);
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = kb[i] ^ 0x5c5c5c5cu;
    sha1_iv(opad);
    sha1_compress(opad, blk);
}

// ------------------------------------------------------------------------------------------------
// SHA-256 (keyver 3 KDF: HMAC-SHA256(PMK, "\1\0Pairwise key expansion" || m || n || "\x80\1"))
// ------------------------------------------------------------------------------------------------
__constant__ static const uint32_t SHA256_K[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

__device__ __forceinline__ void sha256_iv(uint32_t st[8]) {
    st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
    st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

__device__ __forceinline__ void sha256_compress(uint32_t st[8], const uint32_t m[16]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = m[i];
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t++) {
        uint32_t wt;
        if (t < 16) wt = w[t];
        else {
            uint32_t x = w[(t - 15) & 15], y = w[(t - 2) & 15];
            uint32_t s0 = xor3(rotr(x, 7), rotr(x, 18), x >> 3);
            uint32_t s1 = xor3(rotr(y, 17), rotr(y, 19), y >> 10);
            wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
            w[t & 15] = wt;
        }
        uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        uint32_t ch = ch3(e, f, g);
        uint32_t t1 = h + S1 + ch + SHA256_K[t] + wt;
        uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        uint32_t mj = maj3(a, b, c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// SHA-256 compression of a wave-uniform block with host-expanded kw[t] = K_t + W_t (t < 64, scalar loads).
__device__ __forceinline__ void sha256_compress_kw(uint32_t st[8], const uint32_t* __restrict__ kw) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t++) {
        uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        uint32_t ch = ch3(e, f, g);
        uint32_t t1 = h + S1 + ch + kw[t];
        uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        uint32_t mj = maj3(a, b, c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__device__ __forceinline__ void sha256_hmac_mid(const uint32_t kb[16], uint32_t ipad[8], uint32_t opad[8]) {
    uint32_t blk[16];
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = kb[i] ^ 0x36363636u;
    sha256_iv(ipad);
    sha256_compress(ipad, blk);
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = kb[i] ^ 0x5c5c5c5cu;
    sha256_iv(opad);
    sha256_compress(opad, blk);
}

// ------------------------------------------------------------------------------------------------
// MD5 (keyver 1 MIC: HMAC-MD5(KCK, EAPOL)); little-endian message words
// ------------------------------------------------------------------------------------------------
__constant__ static const uint32_t MD5_K[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
    0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
    0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
    0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
    0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
    0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
    0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
    0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};

__device__ __forceinline__ void md5_iv(uint32_t st[4]) {
    st[0] = 0x67452301u; st[1] = 0xefcdab89u; st[2] = 0x98badcfeu; st[3] = 0x10325476u;
}

__device__ __forceinline__ void md5_compress(uint32_t st[4], const uint32_t m[16]) {
    constexpr int S[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) { f = ((c ^ d) & b) ^ d; g = i; }
        else if (i < 32) { f = ((b ^ c) & d) ^ c; g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        uint32_t t = d;
        d = c;
        c = b;
        b = b + rotl(a + f + MD5_K[i] + m[g], S[i >> 4][i & 3]);
        a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

// MD5 compression of a wave-uniform block with host-folded km[i] = K_i + M[g(i)] (scalar loads).
__device__ __forceinline__ void md5_compress_km(uint32_t st[4], const uint32_t* __restrict__ km) {
    constexpr int S[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        if (i < 16) f = ((c ^ d) & b) ^ d;
        else if (i < 32) f = ((b ^ c) & d) ^ c;
        else if (i < 48) f = b ^ c ^ d;
        else f = c ^ (b | ~d);
        uint32_t t = d;
        d = c;
        c = b;
        b = b + rotl(a + f + km[i], S[i >> 4][i & 3]);
        a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

__device__ __forceinline__ void md5_hmac_mid(const uint32_t kb[16], uint32_t ipad[4], uint32_t opad[4]) {
    uint32_t blk[16];
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = kb[i] ^ 0x36363636u;
    md5_iv(ipad);
    md5_compress(ipad, blk);
#pragma unroll
    for (int i = 0; i < 16; i++) blk[i] = kb[i] ^ 0x5c5c5c5cu;
    md5_iv(opad);
    md5_compress(opad, blk);
}

// ------------------------------------------------------------------------------------------------
// AES-128 encryption (keyver 3 MIC = AES-128-CMAC(KCK, EAPOL)), T-tables in LDS.
// Te0[x] = (2s, s, s, 3s) big-endian bytes of s = S(x); Te1..3 are its byte rotations.
// The table is built at compile time from GF(2^8) arithmetic (no table copied from anywhere).
// ------------------------------------------------------------------------------------------------
struct AesTables {
    uint32_t te0[256];
};
constexpr uint8_t gf_xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
constexpr AesTables make_aes_tables() {
    // multiplicative inverses via exp/log tables over the generator 0x03, then the FIPS-197 affine map
    uint8_t ex[256] = {}, lg[256] = {};
    uint8_t x = 1;
    for (int i = 0; i < 255; i++) {
        ex[i] = x;
        lg[x] = (uint8_t)i;
        x = (uint8_t)(x ^ gf_xt(x));
    }
    AesTables t{};
    for (int a = 0; a < 256; a++) {
        uint8_t inv = a ? ex[(255 - lg[a]) % 255] : 0;
        uint8_t s = inv;
        for (int k = 1; k < 5; k++) s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
        s ^= 0x63;
        t.te0[a] = ((uint32_t)gf_xt(s) << 24) | ((uint32_t)s << 16) | ((uint32_t)s << 8) | (uint32_t)(gf_xt(s) ^ s);
    }
    return t;
}
__constant__ static const AesTables AES_TABLES = make_aes_tables();

// AES-128 encryption for the keyver-3 CMAC, one lane-sliced T-table in LDS, with the key schedule computed round by
// round (FIPS-197 5.2) instead of held as rk[44] (40 fewer live registers; 40 more lookups per block).
//
// ONE table, Te0, in 32 interleaved copies -- entry x of copy c at word 32 x + c, lane l reads copy l % 32 -- so every
// ds_read_b32 of a 32-lane group hits 32 distinct banks whatever the indices are: no bank conflicts at all, in 32 KiB
// per workgroup.  Te1..Te3 are Te0 rotated right by 8/16/24 (one v_alignbit each, 12 per round) and the S-box byte is
// byte 2 of Te0.  A 256-thread workgroup (one wave per SIMD) fits beside another call's PBKDF2 head: it needs one
// 106-VGPR wave slot per SIMD.  (The four-table layouts, sliced or not, a two-table layout and round keys in LDS were
// measured and dropped: CHANGELOG.md, rounds 2-4.)
constexpr uint32_t AES_SLICES = 32;                     // copies of Te0
constexpr uint32_t AES_LDS_WORDS = 256 * AES_SLICES;    // 32 KiB
// Byte offset of Te0[byte K of s] in the lane's copy: (x << 7) | cw, cw = 4 (lane % 32).  Two full-rate ops for
// K = 1..3 (a right shift that lands the byte on bits 7..14, then one v_bitop3_b32 (t & 0x7f80) | cw, truth table
// 0xEA); LLVM's own choice was v_bfe + v_lshl_or, two half-rate ops.  The key schedule's lookups stay hoisted out of
// the CMAC loop (the builtin, unlike inline asm, is a pure value to LLVM).
template <int K>
__device__ __forceinline__ uint32_t aes_v1_off(uint32_t s, uint32_t cw) {
    const uint32_t t = K == 3 ? s >> 17 : K == 2 ? s >> 9 : K == 1 ? s >> 1 : s << 7;
    return __builtin_amdgcn_bitop3_b32(t, 0x7f80u, cw, 0xea);  // the builtin (not asm) so LLVM can still hoist
}
template <int K>
__device__ __forceinline__ uint32_t aes_v1_ld(const uint32_t* te, uint32_t s, uint32_t cw) {
    return *(const uint32_t*)((const char*)te + aes_v1_off<K>(s, cw));
}
// (S[a], S[b], S[c], S[d]) with a = byte KA of wa, ...; S[x] = byte 2 (and byte 1) of Te0[x]
template <int KA, int KB, int KC, int KD>
__device__ __forceinline__ uint32_t aes4_subword_v1(const uint32_t* te, uint32_t cw, uint32_t wa, uint32_t wb,
                                                    uint32_t wc, uint32_t wd) {
    const uint32_t hi = __builtin_amdgcn_perm(aes_v1_ld<KA>(te, wa, cw), aes_v1_ld<KB>(te, wb, cw), 0x06020000u);
    const uint32_t lo = __builtin_amdgcn_perm(aes_v1_ld<KC>(te, wc, cw), aes_v1_ld<KD>(te, wd, cw), 0x00000501u);
    return __builtin_amdgcn_perm(hi, lo, 0x07060100u);
}
// The table image for the workgroup's LDS: word k of AES_LDS_WORDS.
__device__ __forceinline__ uint32_t aes_lds_word(uint32_t k) { return AES_TABLES.te0[k >> 5]; }
// te = the table base (every lane's copy is picked by cw inside the lookups)
__device__ __forceinline__ void aes128_encrypt_te4(const uint32_t* te, const uint32_t key[4], uint32_t s[4]) {
    constexpr uint32_t RCON[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
    const uint32_t cw = (threadIdx.x & 31u) << 2;
    uint32_t k0 = key[0], k1 = key[1], k2 = key[2], k3 = key[3];
    uint32_t s0 = s[0] ^ k0, s1 = s[1] ^ k1, s2 = s[2] ^ k2, s3 = s[3] ^ k3;
#define T(w, k) aes_v1_ld<k>(te, w, cw)
#pragma unroll
    for (int r = 1; r < 10; r++) {
        k0 ^= aes4_subword_v1<2, 1, 0, 3>(te, cw, k3, k3, k3, k3) ^ (RCON[r - 1] << 24);
        k1 ^= k0;
        k2 ^= k1;
        k3 ^= k2;
        const uint32_t t0 = xor3(xor3(T(s0, 3), rotr(T(s1, 2), 8), rotr(T(s2, 1), 16)), rotr(T(s3, 0), 24), k0);
        const uint32_t t1 = xor3(xor3(T(s1, 3), rotr(T(s2, 2), 8), rotr(T(s3, 1), 16)), rotr(T(s0, 0), 24), k1);
        const uint32_t t2 = xor3(xor3(T(s2, 3), rotr(T(s3, 2), 8), rotr(T(s0, 1), 16)), rotr(T(s1, 0), 24), k2);
        const uint32_t t3 = xor3(xor3(T(s3, 3), rotr(T(s0, 2), 8), rotr(T(s1, 1), 16)), rotr(T(s2, 0), 24), k3);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
#undef T
    k0 ^= aes4_subword_v1<2, 1, 0, 3>(te, cw, k3, k3, k3, k3) ^ (RCON[9] << 24);
    k1 ^= k0;
    k2 ^= k1;
    k3 ^= k2;
    s[0] = aes4_subword_v1<3, 2, 1, 0>(te, cw, s0, s1, s2, s3) ^ k0;
    s[1] = aes4_subword_v1<3, 2, 1, 0>(te, cw, s1, s2, s3, s0) ^ k1;
    s[2] = aes4_subword_v1<3, 2, 1, 0>(te, cw, s2, s3, s0, s1) ^ k2;
    s[3] = aes4_subword_v1<3, 2, 1, 0>(te, cw, s3, s0, s1, s2) ^ k3;
}

// CMAC subkey doubling on a 128-bit big-endian value held in 4 words
__device__ __forceinline__ void cmac_dbl(const uint32_t in[4], uint32_t out[4]) {
    uint32_t msb = in[0] >> 31;
    out[0] = (in[0] << 1) | (in[1] >> 31);
    out[1] = (in[1] << 1) | (in[2] >> 31);
    out[2] = (in[2] << 1) | (in[3] >> 31);
    out[3] = (in[3] << 1) ^ (msb ? 0x87u : 0u);
}

}  // namespace dwpa
