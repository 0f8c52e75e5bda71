// host_crypto.hpp -- hash and cipher primitives of the host (CPU) backend (internal).
//
// The library's own implementations -- not OpenSSL's, not the oracle's -- of what check_key_m22000 computes
// (web/common.php:56-112,157-307): SHA-1 (PBKDF2, HMAC-SHA1 for the PMKID, the keyver 1/2 PRF and the keyver 2 MIC),
// SHA-256 (the keyver 3 KDF), MD5 (the keyver 1 MIC) and AES-128 (the keyver 3 CMAC).  Each primitive has an x86
// instruction-set path (SHA-NI, AES-NI: SSE registers, no AVX state) chosen at run time by CPUID, and a portable
// scalar path.  The choice is made once per process, after a known-answer self-test of the instruction-set path
// against the scalar one; DWPA_HOST_SIMD=0 forces the scalar path.
//
// PBKDF2 has a third path, AVX-512F (16 lanes per register) for many keys at once.
//
// Conventions: SHA-1 / SHA-256 message words and states are big-endian words (the host integers of the bytes read
// big-endian), MD5's little-endian words, as in the device tables (tables.hpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace dwpa {
namespace hostc {

struct Caps {
    bool sha_ni = false;  // SHA-1 and SHA-256 compressions, PBKDF2 of a few keys
    bool aes_ni = false;  // AES-128
    bool avx512 = false;  // PBKDF2 of many keys: 16 chains per 512-bit register (AVX-512F, ZMM state enabled by the OS)
};
const Caps& caps();       // detected once (CPUID + self-test of each path); DWPA_HOST_SIMD=0 clears all

extern const uint32_t SHA1_IV[5];
extern const uint32_t SHA256_IV[8];
extern const uint32_t MD5_IV[4];

void sha1_compress(uint32_t st[5], const uint32_t w[16]);
// Four independent SHA-1 compressions in lock step (SHA-NI hides one compression's round latency behind the others).
void sha1_compress_x4(uint32_t (*st)[5], const uint32_t* const* w);
void sha256_compress(uint32_t st[8], const uint32_t w[16]);
void md5_compress(uint32_t st[4], const uint32_t w[16]);
// Whole-message SHA-1 (HMAC keys longer than one block are hashed first, RFC 2104).
void sha1_bytes(const uint8_t* p, size_t n, uint32_t out[5]);

struct Aes128Key {
    alignas(16) uint8_t rk[176];  // FIPS-197 expanded key, 11 round keys of 16 bytes
};
void aes128_expand(const uint8_t key[16], Aes128Key& ks);
void aes128_encrypt(const Aes128Key& ks, const uint8_t in[16], uint8_t out[16]);
// AES-128-CMAC (RFC 4493, common.php:56-112) over nb >= 1 pre-padded 16-byte blocks: `complete` says whether the last
// block is a whole message block (XOR K1) or was padded with 0x80 0.. (XOR K2).
void aes128_cmac(const uint8_t key[16], const uint8_t* blocks, size_t nb, bool complete, uint8_t mac[16]);

// HMAC midstates (the states after the key block XOR ipad / opad) of a key of any length.
void hmac_sha1_mid(const uint8_t* key, size_t len, uint32_t ipad[5], uint32_t opad[5]);

// PBKDF2-HMAC-SHA1(key, salt, 4096, 32) for n keys.  mid[i] = the key's HMAC-SHA1 midstates (ipad h0..h4, opad
// h0..h4); salt[i] = its salt blocks as build_salt_blocks (m22000_host.hpp) lays them out, [2][nblk[i]][16] words of
// ESSID || INT(b) || padding; pmk[i] = the 8 big-endian words of the PMK.  A chain is one output block of one key
// (4,095 dependent iterations).  With AVX-512, groups of PBKDF2_WIDE chains (16 keys) run as 2 x 16 lanes; the rest
// (and everything without AVX-512) as PBKDF2_CHAINS SHA-NI chains in lock step, which hides the round latency of one.
constexpr int PBKDF2_CHAINS = 4;
constexpr int PBKDF2_WIDE = 32;
// Seconds one thread takes for one pbkdf2_sha1 call of 1 key (ni1: two SHA-NI chains, or scalar without SHA-NI),
// 2 keys (ni: four chains in lock step), 8 keys (avx1: one AVX-512 group of 16 chains) and 16 keys (avx2: two groups
// in lock step); 0 = path absent.  Measured once per process on this CPU.
struct Pbkdf2Costs {
    double ni1 = 0, ni = 0, avx1 = 0, avx2 = 0;
};
const Pbkdf2Costs& pbkdf2_costs();
void pbkdf2_sha1(size_t n, const uint32_t (*mid)[10], const uint32_t* const* salt, const uint32_t* nblk,
                 uint32_t (*pmk)[8]);

}  // namespace hostc
}  // namespace dwpa
