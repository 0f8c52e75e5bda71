// tables.hpp -- device-resident job tables shared by host builder (m22000_host.cpp) and kernels (kernels.hip).
//
// A work unit is a set of m22000 hashlines grouped by ESSID ("salt group"): one PMK per (ESSID, candidate) is
// computed once and tested against every line of that ESSID (north_star "salt reuse"; get_work hands out one
// ESSID per work unit, web/content/get_work.php:96-109).  Everything that is uniform across candidates -- the
// PRF messages of every nonce-correction attempt, EAPOL frames, PMKID messages -- is pre-padded on the host into
// hash blocks so that the verifier kernel reads it with wave-uniform (scalar) loads.
//
// KW blocks.  A block that every lane of a wave hashes alike has the same message schedule in every lane, so the
// host expands it once: SHA-1 kw[t] = K_t + W_t (80 words per block), SHA-256 kw[t] = K_t + W_t (64 words), MD5
// km[i] = K_i + M[g(i)] (64 words).  The kernels read them with scalar loads and skip the schedule (~1/3 of a
// SHA-1 compression).  Blocks that differ per lane (the attempt-parallel verifier's patched PRF blocks) stay raw.
#pragma once
#include <stdint.h>

namespace dwpa {

enum : uint32_t { LINE_PMKID = 1, LINE_EAPOL = 2 };

struct LineDev {
    uint32_t kind;        // LINE_PMKID / LINE_EAPOL
    uint32_t keyver;      // EAPOL key version 1/2/3 (key_information & 3, common.php:215-217)
    uint32_t target[4];   // PMKID or MIC (first 16 bytes): BE words (SHA1/CMAC) or LE words (MD5, keyver 1)
    uint32_t msg_off;     // PMKID: HMAC-SHA1 inner blocks of "PMK Name"||AP||STA as SHA-1 KW blocks (pool words)
    uint32_t msg_nblk;
    uint32_t pre_off;     // EAPOL: PRF message blocks shared by every attempt, KW blocks (SHA-1, keyver 3 SHA-256)
    uint32_t pre_nblk;
    uint32_t list_off;    // EAPOL: attempt lists; list k = attempts [list_off + k*natt, +natt) in the attempt table
    uint32_t nlists;      // list k applies to the k-th non-null key (PHP mutates $n across keys); last list to the rest
    uint32_t natt;        // attempts per list (1 + 4*halfnc in PHP order, common.php:250-300)
    uint32_t mic_off;     // EAPOL: HMAC inner blocks of the EAPOL frame as KW blocks (keyver 1 MD5 km, keyver 2 SHA-1
    uint32_t mic_nblk;    // kw), or raw 4-word CMAC blocks (keyver 3)
    uint32_t cmac_complete;  // keyver 3: 1 if the last EAPOL block is complete (XOR K1), else padded (XOR K2)
    // Attempt patching: in the usual case every attempt's PRF message differs from the others only in the 4
    // nonce-correction bytes, so all attempts share one block stream (AttDev.blk_off) and each attempt carries
    // just the two big-endian words that hold those bytes (words patch_w0/patch_w1 of the stream; equal when the
    // bytes are word-aligned).  NO_PATCH: every attempt has its own pre-padded blocks (short ANONCE, where PHP's
    // substr_replace grows $n).
    uint32_t patch_w0;
    uint32_t patch_w1;
    uint32_t att_off;     // patched lines: the shared stream (word offset, blocks) every AttDev.blk_off/nblk repeats,
    uint32_t att_nblk;    // read from the line so that the attempt-parallel kernel keeps it wave-uniform
};
static_assert(sizeof(LineDev) % 16 == 0, "LineDev must stay 16-byte aligned");
constexpr uint32_t NO_PATCH = 0xffffffffu;

struct AttDev {
    uint32_t blk_off;     // word offset of this attempt's PRF blocks after the shared prefix
    uint32_t nblk;
    int32_t nc;           // signed correction reported on a hit (0 for the first attempt)
    uint32_t endian;      // 0 none (exact), 1 BE ('N'), 2 LE ('V')
    uint32_t v0, v1;      // values of stream words patch_w0 / patch_w1 for this attempt (LineDev.patch_w0 != NO_PATCH)
    uint32_t kw_off;      // this attempt's PRF blocks after the prefix as KW blocks (key-parallel verifier), or NO_KW
    uint32_t pad1;
};
constexpr uint32_t NO_KW = 0xffffffffu;
constexpr uint32_t SHA1_KW_WORDS = 80, SHA256_KW_WORDS = 64, MD5_KM_WORDS = 64;
// Verify classes: kernels are instantiated per class so that each launch carries only one MAC's code and registers.
enum : uint32_t { VC_PMKID = 1, VC_KV1 = 2, VC_KV2 = 4, VC_KV3 = 8, VC_ALL = 15 };
inline uint32_t verify_class(const LineDev& L) {
    return L.kind == LINE_PMKID ? VC_PMKID : L.keyver == 1 ? VC_KV1 : L.keyver == 2 ? VC_KV2 : VC_KV3;
}
// attempt-parallel verification (one wave = one key x 64 attempts) pays off once a list has this many attempts
constexpr uint32_t ATT_PARALLEL_MIN = 64;

// One wave (64 lanes) verifies up to 64 consecutive candidate slots against one line.
struct SegDev {
    uint32_t line;        // index into the line table
    uint32_t slot;        // first candidate slot (PMK buffer index)
    uint32_t count;       // <= 64
    uint32_t pad;
};

struct HitDev {
    uint64_t cand;        // candidate id (dictionary word index / key ordinal / numeric value / word*nrules+rule)
    uint32_t line;
    uint32_t attempt;     // attempt index within the applicable list (PMKID: 0)
    uint32_t pmk[8];      // PMK as big-endian words
};

constexpr int MID_WORDS = 10;   // ipad h0..h4, opad h0..h4 (SoA: word k of slot s at mid[k*cap + s])
constexpr int PMK_WORDS = 8;

}  // namespace dwpa
