// host_crypto.cpp -- the host backend's SHA-1 / SHA-256 / MD5 / AES-128 and PBKDF2 (see host_crypto.hpp).
//
// Instruction-set paths: SHA-NI (sha1rnds4 / sha1nexte / sha1msg1/2, sha256rnds2 / sha256msg1/2) and AES-NI, in SSE
// registers, and AVX-512F for PBKDF2 over many keys.  A SHA-1 compression under SHA-NI is a chain of 20 dependent
// sha1rnds4, so one PBKDF2 chain is bound by their latency; pbkdf2_sha1 steps PBKDF2_CHAINS independent chains (two
// output blocks of each key) in lock step, and the out-of-order core overlaps them -- the path for a call of a few
// keys.  With many keys, 16 chains share each 512-bit register (vprold rotates, vpternlogd round functions) and two
// such groups run in lock step: the throughput path.  The scalar paths are the FIPS 180-4 / RFC 1321 / FIPS 197
// definitions and serve CPUs without the extensions (and DWPA_HOST_SIMD=0).
#include "host_crypto.hpp"

#include <cpuid.h>
#include <immintrin.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>

namespace dwpa {
namespace hostc {

const uint32_t SHA1_IV[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
const uint32_t SHA256_IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                               0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
const uint32_t MD5_IV[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};

static const uint32_t K256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

static inline uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static inline uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static inline uint32_t be32(const uint8_t* p) {
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
static inline void put_be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

// =========================================================================================================
// scalar paths
// =========================================================================================================
static void sha1_scalar(uint32_t st[5], const uint32_t m[16]) {
    uint32_t w[16];
    memcpy(w, m, 64);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
    for (int t = 0; t < 80; t++) {
        uint32_t wt = w[t & 15];
        if (t >= 16) {
            wt = rol(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20) { f = (b & c) | (~b & d); k = 0x5a827999u; }
        else if (t < 40) { f = b ^ c ^ d; k = 0x6ed9eba1u; }
        else if (t < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8f1bbcdcu; }
        else { f = b ^ c ^ d; k = 0xca62c1d6u; }
        const uint32_t x = rol(a, 5) + f + e + k + wt;
        e = d;
        d = c;
        c = rol(b, 30);
        b = a;
        a = x;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
    st[4] += e;
}

static void sha256_scalar(uint32_t st[8], const uint32_t m[16]) {
    uint32_t w[64];
    memcpy(w, m, 64);
    for (int t = 16; t < 64; t++) {
        const uint32_t s0 = ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3);
        const uint32_t s1 = ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int t = 0; t < 64; t++) {
        const uint32_t t1 = h + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K256[t] + w[t];
        const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// MD5 (RFC 1321): K_i = floor(2^32 |sin(i + 1)|), per-round shifts, message index g(i)
static const uint32_t MD5_K[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
    0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
    0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
    0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
    0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
    0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
    0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
    0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};
static const uint8_t MD5_S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};

void md5_compress(uint32_t st[4], const uint32_t m[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        const uint32_t x = d;
        d = c;
        c = b;
        b = b + rol(a + f + MD5_K[i] + m[g], MD5_S[(i >> 4) * 4 + (i & 3)]);
        a = x;
    }
    st[0] += a;
    st[1] += b;
    st[2] += c;
    st[3] += d;
}

// AES-128 (FIPS 197), byte-oriented: S-box built once from the GF(2^8) inverse and the affine map
struct AesTables {
    uint8_t sbox[256];
    AesTables() {
        uint8_t p = 1, q = 1;
        do {  // p runs over the powers of 3, q over those of 3^-1 = 0xf6: q = p^-1
            p = (uint8_t)(p ^ (p << 1) ^ (p & 0x80 ? 0x1b : 0));
            q ^= (uint8_t)(q << 1);
            q ^= (uint8_t)(q << 2);
            q ^= (uint8_t)(q << 4);
            if (q & 0x80) q ^= 0x09;
            const uint8_t x = (uint8_t)(q ^ (q << 1 | q >> 7) ^ (q << 2 | q >> 6) ^ (q << 3 | q >> 5) ^ (q << 4 | q >> 4));
            sbox[p] = (uint8_t)(x ^ 0x63);
        } while (p != 1);
        sbox[0] = 0x63;
    }
};
static const AesTables& aes_tables() {
    static const AesTables t;
    return t;
}
static inline uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ (x & 0x80 ? 0x1b : 0)); }

static void aes128_expand_scalar(const uint8_t key[16], Aes128Key& ks) {
    const uint8_t* S = aes_tables().sbox;
    memcpy(ks.rk, key, 16);
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t t[4];
        memcpy(t, ks.rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            const uint8_t t0 = t[0];
            t[0] = (uint8_t)(S[t[1]] ^ rcon);
            t[1] = S[t[2]];
            t[2] = S[t[3]];
            t[3] = S[t0];
            rcon = xtime(rcon);
        }
        for (int k = 0; k < 4; k++) ks.rk[4 * i + k] = (uint8_t)(ks.rk[4 * (i - 4) + k] ^ t[k]);
    }
}

static void aes128_encrypt_scalar(const Aes128Key& ks, const uint8_t in[16], uint8_t out[16]) {
    const uint8_t* S = aes_tables().sbox;
    uint8_t s[16];
    for (int k = 0; k < 16; k++) s[k] = (uint8_t)(in[k] ^ ks.rk[k]);
    for (int r = 1; r <= 10; r++) {
        uint8_t t[16];
        for (int c = 0; c < 4; c++)      // SubBytes + ShiftRows: row i of column c comes from column c + i
            for (int i = 0; i < 4; i++) t[4 * c + i] = S[s[4 * ((c + i) & 3) + i]];
        if (r < 10)
            for (int c = 0; c < 4; c++) {  // MixColumns
                uint8_t* a = t + 4 * c;
                const uint8_t all = (uint8_t)(a[0] ^ a[1] ^ a[2] ^ a[3]), a0 = a[0];
                a[0] ^= (uint8_t)(all ^ xtime((uint8_t)(a[0] ^ a[1])));
                a[1] ^= (uint8_t)(all ^ xtime((uint8_t)(a[1] ^ a[2])));
                a[2] ^= (uint8_t)(all ^ xtime((uint8_t)(a[2] ^ a[3])));
                a[3] ^= (uint8_t)(all ^ xtime((uint8_t)(a[3] ^ a0)));
            }
        for (int k = 0; k < 16; k++) s[k] = (uint8_t)(t[k] ^ ks.rk[16 * r + k]);
    }
    memcpy(out, s, 16);
}

// =========================================================================================================
// SHA-NI / AES-NI paths
// =========================================================================================================
#define DWPA_SHA_TARGET __attribute__((target("sha,sse4.1,ssse3")))
#define DWPA_AES_TARGET __attribute__((target("aes,sse4.1")))
#define DWPA_AVX512_TARGET __attribute__((target("avx512f")))

// N SHA-1 compressions in lock step.  State in SHA-NI form: abcd = {A, B, C, D} from the high lane down, e = {E, 0,
// 0, 0}; message m[n][q] = words 4q..4q+3, the first in the high lane.  Round group g (4 rounds) takes e_g = E + W for
// g = 0 and sha1nexte(state before group g-1, W) after; from g = 4 the schedule is
// W_g = msg2(msg1(W_{g-4}, W_{g-3}) ^ W_{g-2}, W_{g-1}).  m is consumed.
template <int N>
DWPA_SHA_TARGET __attribute__((always_inline)) static inline void sha1ni_x(__m128i* abcd, __m128i* e,
                                                                           __m128i (*m)[4]) {
    __m128i s[N], sp[N], ee[N];
    for (int n = 0; n < N; n++) {
        s[n] = abcd[n];
        ee[n] = _mm_add_epi32(e[n], m[n][0]);
        sp[n] = s[n];
        s[n] = _mm_sha1rnds4_epu32(s[n], ee[n], 0);
    }
#define DWPA_SHA1NI_G(g, f)                                                                                         \
    for (int n = 0; n < N; n++) {                                                                                   \
        if ((g) >= 4)                                                                                               \
            m[n][(g) & 3] = _mm_sha1msg2_epu32(                                                                     \
                _mm_xor_si128(_mm_sha1msg1_epu32(m[n][(g) & 3], m[n][((g) + 1) & 3]), m[n][((g) + 2) & 3]),         \
                m[n][((g) + 3) & 3]);                                                                               \
        ee[n] = _mm_sha1nexte_epu32(sp[n], m[n][(g) & 3]);                                                          \
        sp[n] = s[n];                                                                                               \
        s[n] = _mm_sha1rnds4_epu32(s[n], ee[n], f);                                                                 \
    }
    DWPA_SHA1NI_G(1, 0) DWPA_SHA1NI_G(2, 0) DWPA_SHA1NI_G(3, 0) DWPA_SHA1NI_G(4, 0)
    DWPA_SHA1NI_G(5, 1) DWPA_SHA1NI_G(6, 1) DWPA_SHA1NI_G(7, 1) DWPA_SHA1NI_G(8, 1) DWPA_SHA1NI_G(9, 1)
    DWPA_SHA1NI_G(10, 2) DWPA_SHA1NI_G(11, 2) DWPA_SHA1NI_G(12, 2) DWPA_SHA1NI_G(13, 2) DWPA_SHA1NI_G(14, 2)
    DWPA_SHA1NI_G(15, 3) DWPA_SHA1NI_G(16, 3) DWPA_SHA1NI_G(17, 3) DWPA_SHA1NI_G(18, 3) DWPA_SHA1NI_G(19, 3)
#undef DWPA_SHA1NI_G
    for (int n = 0; n < N; n++) {
        e[n] = _mm_sha1nexte_epu32(sp[n], e[n]);
        abcd[n] = _mm_add_epi32(s[n], abcd[n]);
    }
}

DWPA_SHA_TARGET static void sha1_ni(uint32_t st[5], const uint32_t w[16]) {
    __m128i abcd[1] = {_mm_set_epi32((int)st[0], (int)st[1], (int)st[2], (int)st[3])};
    __m128i e[1] = {_mm_set_epi32((int)st[4], 0, 0, 0)};
    __m128i m[1][4];
    for (int q = 0; q < 4; q++)
        m[0][q] = _mm_set_epi32((int)w[4 * q], (int)w[4 * q + 1], (int)w[4 * q + 2], (int)w[4 * q + 3]);
    sha1ni_x<1>(abcd, e, m);
    st[0] = (uint32_t)_mm_extract_epi32(abcd[0], 3);
    st[1] = (uint32_t)_mm_extract_epi32(abcd[0], 2);
    st[2] = (uint32_t)_mm_extract_epi32(abcd[0], 1);
    st[3] = (uint32_t)_mm_extract_epi32(abcd[0], 0);
    st[4] = (uint32_t)_mm_extract_epi32(e[0], 3);
}

// Four independent compressions in lock step (the verify's nonce-correction attempts, host_check.cpp).
DWPA_SHA_TARGET static void sha1_ni_x4(uint32_t (*st)[5], const uint32_t* const* w) {
    __m128i abcd[4], e[4], m[4][4];
    for (int n = 0; n < 4; n++) {
        abcd[n] = _mm_set_epi32((int)st[n][0], (int)st[n][1], (int)st[n][2], (int)st[n][3]);
        e[n] = _mm_set_epi32((int)st[n][4], 0, 0, 0);
        for (int q = 0; q < 4; q++)
            m[n][q] = _mm_set_epi32((int)w[n][4 * q], (int)w[n][4 * q + 1], (int)w[n][4 * q + 2], (int)w[n][4 * q + 3]);
    }
    sha1ni_x<4>(abcd, e, m);
    for (int n = 0; n < 4; n++) {
        st[n][0] = (uint32_t)_mm_extract_epi32(abcd[n], 3);
        st[n][1] = (uint32_t)_mm_extract_epi32(abcd[n], 2);
        st[n][2] = (uint32_t)_mm_extract_epi32(abcd[n], 1);
        st[n][3] = (uint32_t)_mm_extract_epi32(abcd[n], 0);
        st[n][4] = (uint32_t)_mm_extract_epi32(e[n], 3);
    }
}

// SHA-256: state as {A, B, E, F} and {C, D, G, H} from the high lane down; message words W_4q.. with W_4q in the low
// lane.  sha256rnds2 runs two rounds on the low two lanes of W + K; block q >= 4 of the schedule is
// msg2(msg1(W_{q-4}, W_{q-3}) + alignr(W_{q-1}, W_{q-2}, 4), W_{q-1}).
DWPA_SHA_TARGET static void sha256_ni(uint32_t st[8], const uint32_t w[16]) {
    __m128i s0 = _mm_set_epi32((int)st[0], (int)st[1], (int)st[4], (int)st[5]);  // ABEF
    __m128i s1 = _mm_set_epi32((int)st[2], (int)st[3], (int)st[6], (int)st[7]);  // CDGH
    const __m128i a0 = s0, c0 = s1;
    __m128i m[4];
    for (int q = 0; q < 4; q++)
        m[q] = _mm_set_epi32((int)w[4 * q + 3], (int)w[4 * q + 2], (int)w[4 * q + 1], (int)w[4 * q]);
    for (int q = 0; q < 16; q++) {
        if (q >= 4)
            m[q & 3] = _mm_sha256msg2_epu32(
                _mm_add_epi32(_mm_sha256msg1_epu32(m[q & 3], m[(q + 1) & 3]),
                              _mm_alignr_epi8(m[(q + 3) & 3], m[(q + 2) & 3], 4)),
                m[(q + 3) & 3]);
        __m128i wk = _mm_add_epi32(m[q & 3], _mm_loadu_si128((const __m128i*)(K256 + 4 * q)));
        s1 = _mm_sha256rnds2_epu32(s1, s0, wk);
        wk = _mm_shuffle_epi32(wk, 0x0e);
        s0 = _mm_sha256rnds2_epu32(s0, s1, wk);
    }
    s0 = _mm_add_epi32(s0, a0);
    s1 = _mm_add_epi32(s1, c0);
    st[0] = (uint32_t)_mm_extract_epi32(s0, 3);
    st[1] = (uint32_t)_mm_extract_epi32(s0, 2);
    st[4] = (uint32_t)_mm_extract_epi32(s0, 1);
    st[5] = (uint32_t)_mm_extract_epi32(s0, 0);
    st[2] = (uint32_t)_mm_extract_epi32(s1, 3);
    st[3] = (uint32_t)_mm_extract_epi32(s1, 2);
    st[6] = (uint32_t)_mm_extract_epi32(s1, 1);
    st[7] = (uint32_t)_mm_extract_epi32(s1, 0);
}

DWPA_AES_TARGET static inline __m128i aes_expand_step(__m128i k, __m128i t) {
    t = _mm_shuffle_epi32(t, 0xff);
    k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
    k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
    k = _mm_xor_si128(k, _mm_slli_si128(k, 4));
    return _mm_xor_si128(k, t);
}

DWPA_AES_TARGET static void aes128_expand_ni(const uint8_t key[16], Aes128Key& ks) {
    __m128i* rk = (__m128i*)ks.rk;
    __m128i k = _mm_loadu_si128((const __m128i*)key);
    rk[0] = k;
#define DWPA_AES_EXP(i, rc)                                         \
    k = aes_expand_step(k, _mm_aeskeygenassist_si128(k, rc));       \
    rk[i] = k;
    DWPA_AES_EXP(1, 0x01) DWPA_AES_EXP(2, 0x02) DWPA_AES_EXP(3, 0x04) DWPA_AES_EXP(4, 0x08) DWPA_AES_EXP(5, 0x10)
    DWPA_AES_EXP(6, 0x20) DWPA_AES_EXP(7, 0x40) DWPA_AES_EXP(8, 0x80) DWPA_AES_EXP(9, 0x1b) DWPA_AES_EXP(10, 0x36)
#undef DWPA_AES_EXP
}

DWPA_AES_TARGET static inline __m128i aes128_enc_ni(const __m128i* rk, __m128i x) {
    x = _mm_xor_si128(x, rk[0]);
    for (int r = 1; r < 10; r++) x = _mm_aesenc_si128(x, rk[r]);
    return _mm_aesenclast_si128(x, rk[10]);
}

DWPA_AES_TARGET static void aes128_encrypt_ni(const Aes128Key& ks, const uint8_t in[16], uint8_t out[16]) {
    _mm_storeu_si128((__m128i*)out, aes128_enc_ni((const __m128i*)ks.rk, _mm_loadu_si128((const __m128i*)in)));
}

// SHA-1 over 16 lanes per register (AVX-512F), G independent groups in lock step: st[g][k] += compress(st[g], w[g])
// with w[g] the 16 message words of every lane (consumed by the in-place schedule).  vprold rotates, vpternlogd
// computes Ch (0xCA), parity (0x96) and Maj (0xE8) in one op each; the loop over t unrolls, so the round function and
// the schedule's start are resolved at compile time and constant message words fold.
template <int G>
DWPA_AVX512_TARGET __attribute__((always_inline)) static inline void sha1x16(__m512i (*st)[5], __m512i (*w)[16]) {
    __m512i a[G], b[G], c[G], d[G], e[G];
    for (int g = 0; g < G; g++) {
        a[g] = st[g][0];
        b[g] = st[g][1];
        c[g] = st[g][2];
        d[g] = st[g][3];
        e[g] = st[g][4];
    }
#pragma unroll
    for (int t = 0; t < 80; t++) {
        const __m512i K = _mm512_set1_epi32((int)(t < 20 ? 0x5a827999u : t < 40 ? 0x6ed9eba1u : t < 60 ? 0x8f1bbcdcu
                                                                                                   : 0xca62c1d6u));
        for (int g = 0; g < G; g++) {
            __m512i wt = w[g][t & 15];
            if (t >= 16) {
                wt = _mm512_rol_epi32(_mm512_xor_si512(_mm512_ternarylogic_epi32(w[g][(t - 3) & 15], w[g][(t - 8) & 15],
                                                                                 w[g][(t - 14) & 15], 0x96),
                                                       wt),
                                      1);
                w[g][t & 15] = wt;
            }
            const __m512i f = t < 20 ? _mm512_ternarylogic_epi32(b[g], c[g], d[g], 0xca)
                            : (t < 40 || t >= 60) ? _mm512_ternarylogic_epi32(b[g], c[g], d[g], 0x96)
                                                  : _mm512_ternarylogic_epi32(b[g], c[g], d[g], 0xe8);
            const __m512i x = _mm512_add_epi32(_mm512_add_epi32(_mm512_rol_epi32(a[g], 5), f),
                                               _mm512_add_epi32(e[g], _mm512_add_epi32(K, wt)));
            e[g] = d[g];
            d[g] = c[g];
            c[g] = _mm512_rol_epi32(b[g], 30);
            b[g] = a[g];
            a[g] = x;
        }
    }
    for (int g = 0; g < G; g++) {
        st[g][0] = _mm512_add_epi32(st[g][0], a[g]);
        st[g][1] = _mm512_add_epi32(st[g][1], b[g]);
        st[g][2] = _mm512_add_epi32(st[g][2], c[g]);
        st[g][3] = _mm512_add_epi32(st[g][3], d[g]);
        st[g][4] = _mm512_add_epi32(st[g][4], e[g]);
    }
}

// U_2..U_4096 of 16 G chains, lane l of group g = chain 16 g + l (the same message shape as pbkdf2_loop_ni).
template <int G>
DWPA_AVX512_TARGET static void pbkdf2_loop_avx512(const uint32_t* const* mid, uint32_t* const* t, int iters = 4096) {
    __m512i ih[G][5], oh[G][5], u[G][5], T[G][5];
    alignas(64) uint32_t lanes[16];
    for (int g = 0; g < G; g++)
        for (int k = 0; k < 5; k++) {
            for (int l = 0; l < 16; l++) lanes[l] = mid[16 * g + l][k];
            ih[g][k] = _mm512_load_si512(lanes);
            for (int l = 0; l < 16; l++) lanes[l] = mid[16 * g + l][5 + k];
            oh[g][k] = _mm512_load_si512(lanes);
            for (int l = 0; l < 16; l++) lanes[l] = t[16 * g + l][k];
            u[g][k] = T[g][k] = _mm512_load_si512(lanes);
        }
    const __m512i pad = _mm512_set1_epi32((int)0x80000000u), zero = _mm512_setzero_si512(),
                  len = _mm512_set1_epi32((64 + 20) * 8);
    for (int it = 1; it < iters; it++) {
        __m512i st[G][5], w[G][16];
        for (int g = 0; g < G; g++) {
            for (int k = 0; k < 5; k++) {
                st[g][k] = ih[g][k];
                w[g][k] = u[g][k];
            }
            w[g][5] = pad;
            for (int k = 6; k < 15; k++) w[g][k] = zero;
            w[g][15] = len;
        }
        sha1x16<G>(st, w);
        for (int g = 0; g < G; g++) {
            for (int k = 0; k < 5; k++) {
                w[g][k] = st[g][k];
                st[g][k] = oh[g][k];
            }
            w[g][5] = pad;
            for (int k = 6; k < 15; k++) w[g][k] = zero;
            w[g][15] = len;
        }
        sha1x16<G>(st, w);
        for (int g = 0; g < G; g++)
            for (int k = 0; k < 5; k++) {
                u[g][k] = st[g][k];
                T[g][k] = _mm512_xor_si512(T[g][k], st[g][k]);
            }
    }
    for (int g = 0; g < G; g++)
        for (int k = 0; k < 5; k++) {
            _mm512_store_si512(lanes, T[g][k]);
            for (int l = 0; l < 16; l++) t[16 * g + l][k] = lanes[l];
        }
}

// One 16-lane compression of word-form states and blocks (the self-test's view of sha1x16).
DWPA_AVX512_TARGET static void sha1x16_words(uint32_t st[16][5], const uint32_t w[16][16]) {
    __m512i s[1][5], m[1][16];
    alignas(64) uint32_t lanes[16];
    for (int k = 0; k < 5; k++) {
        for (int l = 0; l < 16; l++) lanes[l] = st[l][k];
        s[0][k] = _mm512_load_si512(lanes);
    }
    for (int k = 0; k < 16; k++) {
        for (int l = 0; l < 16; l++) lanes[l] = w[l][k];
        m[0][k] = _mm512_load_si512(lanes);
    }
    sha1x16<1>(s, m);
    for (int k = 0; k < 5; k++) {
        _mm512_store_si512(lanes, s[0][k]);
        for (int l = 0; l < 16; l++) st[l][k] = lanes[l];
    }
}

// =========================================================================================================
// dispatch + self-test
// =========================================================================================================
static bool selftest(const Caps& k) {
    // instruction-set paths against the scalar ones on a few pseudo-random blocks and keys
    uint32_t x = 0x12345678u;
    auto rnd = [&x] {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        return x;
    };
    for (int rep = 0; rep < 8; rep++) {
        uint32_t w[16], a[8], b[8];
        for (int i = 0; i < 16; i++) w[i] = rnd();
        for (int i = 0; i < 8; i++) a[i] = b[i] = rnd();
        if (k.sha_ni) {
            sha1_scalar(a, w);
            sha1_ni(b, w);
            if (memcmp(a, b, 20)) return false;
            sha256_scalar(a, w);
            sha256_ni(b, w);
            if (memcmp(a, b, 32)) return false;
        }
        if (k.avx512) {
            uint32_t s16[16][5], w16[16][16], ref[5];
            for (int l = 0; l < 16; l++) {
                for (int i = 0; i < 5; i++) s16[l][i] = rnd();
                for (int i = 0; i < 16; i++) w16[l][i] = rnd();
            }
            uint32_t keep[16][5];
            memcpy(keep, s16, sizeof keep);
            sha1x16_words(s16, w16);
            for (int l = 0; l < 16; l++) {
                memcpy(ref, keep[l], 20);
                sha1_scalar(ref, w16[l]);
                if (memcmp(ref, s16[l], 20)) return false;
            }
        }
        if (k.aes_ni) {
            uint8_t key[16], in[16], o1[16], o2[16];
            memcpy(key, w, 16);
            memcpy(in, w + 4, 16);
            Aes128Key k1, k2;
            aes128_expand_scalar(key, k1);
            aes128_expand_ni(key, k2);
            if (memcmp(k1.rk, k2.rk, 176)) return false;
            aes128_encrypt_scalar(k1, in, o1);
            aes128_encrypt_ni(k2, in, o2);
            if (memcmp(o1, o2, 16)) return false;
        }
    }
    return true;
}

static Caps detect() {
    Caps k;
    const char* env = getenv("DWPA_HOST_SIMD");
    if (env && *env == '0') return k;
    unsigned a = 0, b = 0, c = 0, d = 0;
    bool sse41 = false, ssse3 = false;
    if (__get_cpuid(1, &a, &b, &c, &d)) {
        ssse3 = (c >> 9) & 1;
        sse41 = (c >> 19) & 1;
        k.aes_ni = ((c >> 25) & 1) && sse41;
    }
    bool osxsave = false;
    if (__get_cpuid(1, &a, &b, &c, &d)) osxsave = (c >> 27) & 1;
    if (__get_cpuid_count(7, 0, &a, &b, &c, &d)) {
        k.sha_ni = ((b >> 29) & 1) && sse41 && ssse3;
        // AVX-512F, with the OS saving the opmask and all of the ZMM state (XCR0 bits 1, 2, 5, 6, 7)
        if (((b >> 16) & 1) && osxsave) {
            uint32_t lo, hi;
            __asm__("xgetbv" : "=a"(lo), "=d"(hi) : "c"(0));
            k.avx512 = (lo & 0xe6u) == 0xe6u;
        }
    }
    // test each extension on its own, so one failing leaves the others usable
    const Caps found = k;
    for (int x = 0; x < 3; x++) {
        Caps one;
        bool* have = x == 0 ? &k.sha_ni : x == 1 ? &k.aes_ni : &k.avx512;
        if (!*have) continue;
        (x == 0 ? one.sha_ni : x == 1 ? one.aes_ni : one.avx512) = true;
        if (!selftest(one)) *have = false;
    }
    (void)found;
    return k;
}

const Caps& caps() {
    static const Caps k = detect();
    return k;
}

void sha1_compress(uint32_t st[5], const uint32_t w[16]) {
    if (caps().sha_ni) sha1_ni(st, w);
    else sha1_scalar(st, w);
}
void sha1_compress_x4(uint32_t (*st)[5], const uint32_t* const* w) {
    if (caps().sha_ni) {
        sha1_ni_x4(st, w);
    } else {
        for (int n = 0; n < 4; n++) sha1_scalar(st[n], w[n]);
    }
}
void sha256_compress(uint32_t st[8], const uint32_t w[16]) {
    if (caps().sha_ni) sha256_ni(st, w);
    else sha256_scalar(st, w);
}
void aes128_expand(const uint8_t key[16], Aes128Key& ks) {
    if (caps().aes_ni) aes128_expand_ni(key, ks);
    else aes128_expand_scalar(key, ks);
}
void aes128_encrypt(const Aes128Key& ks, const uint8_t in[16], uint8_t out[16]) {
    if (caps().aes_ni) aes128_encrypt_ni(ks, in, out);
    else aes128_encrypt_scalar(ks, in, out);
}

void sha1_bytes(const uint8_t* p, size_t n, uint32_t out[5]) {
    memcpy(out, SHA1_IV, 20);
    uint32_t w[16];
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        for (int t = 0; t < 16; t++) w[t] = be32(p + i + 4 * t);
        sha1_compress(out, w);
    }
    uint8_t tail[128] = {0};
    const size_t r = n - i;
    memcpy(tail, p + i, r);
    tail[r] = 0x80;
    const size_t tl = r + 9 <= 64 ? 64 : 128;
    const uint64_t bits = (uint64_t)n * 8;
    for (int k = 0; k < 8; k++) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
    for (size_t b = 0; b < tl; b += 64) {
        for (int t = 0; t < 16; t++) w[t] = be32(tail + b + 4 * t);
        sha1_compress(out, w);
    }
}

void hmac_sha1_mid(const uint8_t* key, size_t len, uint32_t ipad[5], uint32_t opad[5]) {
    uint8_t kb[64] = {0};
    if (len > 64) {
        uint32_t h[5];
        sha1_bytes(key, len, h);
        for (int k = 0; k < 5; k++) put_be32(kb + 4 * k, h[k]);
    } else if (len) {
        memcpy(kb, key, len);
    }
    uint32_t wi[16], wo[16];
    for (int t = 0; t < 16; t++) {
        const uint32_t v = be32(kb + 4 * t);
        wi[t] = v ^ 0x36363636u;
        wo[t] = v ^ 0x5c5c5c5cu;
    }
    memcpy(ipad, SHA1_IV, 20);
    memcpy(opad, SHA1_IV, 20);
    sha1_compress(ipad, wi);
    sha1_compress(opad, wo);
}

void aes128_cmac(const uint8_t key[16], const uint8_t* blocks, size_t nb, bool complete, uint8_t mac[16]) {
    Aes128Key ks;
    aes128_expand(key, ks);
    uint8_t L[16] = {0}, K[16];
    aes128_encrypt(ks, L, L);
    // K1 = L << 1 (^ 0x87 if the msb was set); K2 = K1 << 1 likewise (common.php:56-75)
    for (int round = 0; round < (complete ? 1 : 2); round++) {
        const uint8_t msb = L[0] >> 7;
        for (int i = 0; i < 15; i++) K[i] = (uint8_t)(L[i] << 1 | L[i + 1] >> 7);
        K[15] = (uint8_t)(L[15] << 1);
        if (msb) K[15] ^= 0x87;
        memcpy(L, K, 16);
    }
    uint8_t x[16] = {0};
    for (size_t b = 0; b < nb; b++) {
        for (int i = 0; i < 16; i++) x[i] ^= blocks[16 * b + i];
        if (b + 1 == nb)
            for (int i = 0; i < 16; i++) x[i] ^= K[i];
        aes128_encrypt(ks, x, x);
    }
    memcpy(mac, x, 16);
}

// =========================================================================================================
// PBKDF2-HMAC-SHA1 x4096
// =========================================================================================================
// U_1 of output block b: HMAC over the salt blocks (inner, after the ipad block), then the outer compression.
static void pbkdf2_u1(const uint32_t mid[10], const uint32_t* salt, uint32_t nblk, int b, uint32_t u[5]) {
    uint32_t st[5], w[16];
    memcpy(st, mid, 20);
    for (uint32_t k = 0; k < nblk; k++) sha1_compress(st, salt + (size_t)(b * nblk + k) * 16);
    memcpy(w, st, 20);
    w[5] = 0x80000000u;
    for (int t = 6; t < 15; t++) w[t] = 0;
    w[15] = (64 + 20) * 8;
    memcpy(u, mid + 5, 20);
    sha1_compress(u, w);
}

// U_2..U_4096 of one chain, scalar: inner and outer compressions of the 20-byte U with fixed padding.
static void pbkdf2_loop_scalar(const uint32_t mid[10], uint32_t t[5], int iters = 4096) {
    uint32_t u[5], w[16], st[5];
    memcpy(u, t, 20);
    for (int it = 1; it < iters; it++) {
        memcpy(w, u, 20);
        w[5] = 0x80000000u;
        for (int k = 6; k < 15; k++) w[k] = 0;
        w[15] = (64 + 20) * 8;
        memcpy(st, mid, 20);
        sha1_scalar(st, w);
        memcpy(w, st, 20);
        memcpy(u, mid + 5, 20);
        sha1_scalar(u, w);
        for (int k = 0; k < 5; k++) t[k] ^= u[k];
    }
}

// The same for N chains in SHA-NI form.  Message block of both compressions: U (5 words), 0x80000000, zeros, the
// bit length 672 -- so W0..W3 = the previous digest's abcd as is, W4 = its e lane, W5 = the padding bit.
template <int N>
DWPA_SHA_TARGET static void pbkdf2_loop_ni(const uint32_t* const* mid, uint32_t* const* t, int iters = 4096) {
    __m128i ia[N], ie[N], oa[N], oe[N], ua[N], ue[N], ta[N], te[N];
    const __m128i pad = _mm_set_epi32(0, (int)0x80000000u, 0, 0), zero = _mm_setzero_si128(),
                  len = _mm_set_epi32(0, 0, 0, (64 + 20) * 8);
    for (int n = 0; n < N; n++) {
        const uint32_t* m = mid[n];
        ia[n] = _mm_set_epi32((int)m[0], (int)m[1], (int)m[2], (int)m[3]);
        ie[n] = _mm_set_epi32((int)m[4], 0, 0, 0);
        oa[n] = _mm_set_epi32((int)m[5], (int)m[6], (int)m[7], (int)m[8]);
        oe[n] = _mm_set_epi32((int)m[9], 0, 0, 0);
        ta[n] = ua[n] = _mm_set_epi32((int)t[n][0], (int)t[n][1], (int)t[n][2], (int)t[n][3]);
        te[n] = ue[n] = _mm_set_epi32((int)t[n][4], 0, 0, 0);
    }
    for (int it = 1; it < iters; it++) {
        __m128i a[N], e[N], m[N][4];
        for (int n = 0; n < N; n++) {
            a[n] = ia[n];
            e[n] = ie[n];
            m[n][0] = ua[n];
            m[n][1] = _mm_or_si128(ue[n], pad);
            m[n][2] = zero;
            m[n][3] = len;
        }
        sha1ni_x<N>(a, e, m);
        for (int n = 0; n < N; n++) {
            m[n][0] = a[n];
            m[n][1] = _mm_or_si128(e[n], pad);
            m[n][2] = zero;
            m[n][3] = len;
            a[n] = oa[n];
            e[n] = oe[n];
        }
        sha1ni_x<N>(a, e, m);
        for (int n = 0; n < N; n++) {
            ua[n] = a[n];
            ue[n] = e[n];
            ta[n] = _mm_xor_si128(ta[n], a[n]);
            te[n] = _mm_xor_si128(te[n], e[n]);
        }
    }
    for (int n = 0; n < N; n++) {
        t[n][0] = (uint32_t)_mm_extract_epi32(ta[n], 3);
        t[n][1] = (uint32_t)_mm_extract_epi32(ta[n], 2);
        t[n][2] = (uint32_t)_mm_extract_epi32(ta[n], 1);
        t[n][3] = (uint32_t)_mm_extract_epi32(ta[n], 0);
        t[n][4] = (uint32_t)_mm_extract_epi32(te[n], 3);
    }
}

// Each path timed over 64 iterations on this CPU (best of 3), scaled to 4,095.  Zen 5 (the MI355X box's EPYC 9575F)
// runs 16 keys on AVX-512 in ~2.9x the time of 2 keys on SHA-NI; other CPUs differ, so derive_all's chunk size is
// chosen from these figures rather than from a fixed rule.
static Pbkdf2Costs measure_costs() {
    Pbkdf2Costs c;
    uint32_t mids[PBKDF2_WIDE][10], T[PBKDF2_WIDE][5];
    const uint32_t* cm[PBKDF2_WIDE];
    uint32_t* ct[PBKDF2_WIDE];
    for (int i = 0; i < PBKDF2_WIDE; i++) {
        for (int k = 0; k < 10; k++) mids[i][k] = 0x9e3779b9u * (uint32_t)(10 * i + k + 1);
        cm[i] = mids[i];
        ct[i] = T[i];
    }
    constexpr int IT = 65;
    auto best = [&](auto&& run) {
        double b = 1e30;
        for (int rep = 0; rep < 3; rep++) {
            for (int i = 0; i < PBKDF2_WIDE; i++) memset(T[i], 0, 20);
            const auto t0 = std::chrono::steady_clock::now();
            run();
            b = std::min(b, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        return b * 4095.0 / (IT - 1);
    };
    const Caps& k = caps();
    if (k.sha_ni) {
        c.ni1 = best([&] { pbkdf2_loop_ni<2>(cm, ct, IT); });
        c.ni = best([&] { pbkdf2_loop_ni<PBKDF2_CHAINS>(cm, ct, IT); });
    } else {
        c.ni1 = best([&] {
            for (int i = 0; i < 2; i++) pbkdf2_loop_scalar(cm[i], ct[i], IT);
        });
        c.ni = 2 * c.ni1;
    }
    if (k.avx512) {
        c.avx1 = best([&] { pbkdf2_loop_avx512<1>(cm, ct, IT); });
        c.avx2 = best([&] { pbkdf2_loop_avx512<2>(cm, ct, IT); });
    }
    return c;
}

const Pbkdf2Costs& pbkdf2_costs() {
    static const Pbkdf2Costs c = measure_costs();
    return c;
}


void pbkdf2_sha1(size_t n, const uint32_t (*mid)[10], const uint32_t* const* salt, const uint32_t* nblk,
                 uint32_t (*pmk)[8]) {
    const Caps& k = caps();
    // chain 2i + b = output block b + 1 of key i
    uint32_t T[PBKDF2_WIDE][5];
    const uint32_t* cm[PBKDF2_WIDE];
    uint32_t* ct[PBKDF2_WIDE];
    const size_t chains = 2 * n;
    auto prep = [&](size_t c0, int nc) {
        for (int c = 0; c < nc; c++) {
            const size_t i = (c0 + c) >> 1;
            pbkdf2_u1(mid[i], salt[i], nblk[i], (int)((c0 + c) & 1), T[c]);
            cm[c] = mid[i];
            ct[c] = T[c];
        }
    };
    auto store = [&](size_t c0, int nc) {
        for (int c = 0; c < nc; c++) {
            const size_t i = (c0 + c) >> 1;
            if ((c0 + c) & 1) memcpy(pmk[i] + 5, T[c], 12);  // T_2: the PMK's last 12 bytes
            else memcpy(pmk[i], T[c], 20);
        }
    };
    size_t c0 = 0;
    if (k.avx512) {
        for (; chains - c0 >= PBKDF2_WIDE; c0 += PBKDF2_WIDE) {
            prep(c0, PBKDF2_WIDE);
            pbkdf2_loop_avx512<PBKDF2_WIDE / 16>(cm, ct);
            store(c0, PBKDF2_WIDE);
        }
        if (chains - c0 >= 16) {
            prep(c0, 16);
            pbkdf2_loop_avx512<1>(cm, ct);
            store(c0, 16);
            c0 += 16;
        }
    }
    constexpr int C = PBKDF2_CHAINS;
    for (; c0 < chains; c0 += C) {
        const int nc = (int)std::min<size_t>(chains - c0, C);
        prep(c0, nc);
        if (!k.sha_ni) {
            for (int c = 0; c < nc; c++) pbkdf2_loop_scalar(cm[c], T[c]);
        } else {
            for (int c = nc; c < C; c++) {  // a partial last group: pad with copies of chain 0 (results dropped)
                memcpy(T[c], T[0], 20);
                cm[c] = cm[0];
                ct[c] = T[c];
            }
            if (nc <= 2) pbkdf2_loop_ni<2>(cm, ct);
            else pbkdf2_loop_ni<C>(cm, ct);
        }
        store(c0, nc);
    }
}

}  // namespace hostc
}  // namespace dwpa
