// rules_dev.hip -- on-GPU hashcat rule amplification of HBM-resident dictionaries (north_star "rule expansion").
//
// Grid = (word chunks) x (rules): every wave applies ONE rule (blockIdx.y) to 64 consecutive words, so the rule
// byte code is wave-uniform (scalar loads, uniform branches) and only the word bytes differ per lane.  Each lane
// works on a private 256-byte buffer (hashcat's RP_PASSWORD_SIZE); results outside 8..63 bytes are dropped
// (hashcat -m 22000 limits), the survivors are compacted into the batch as HMAC-SHA1 key midstates exactly like
// k_prep_dict.  Candidate id = word * nrules + rule.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crypto_dev.hpp"
#include "prep_dev.hpp"
#include "rules.hpp"

namespace dwpa {

__device__ __forceinline__ bool r_lower(uint32_t c) { return c - 'a' < 26u; }
__device__ __forceinline__ bool r_upper(uint32_t c) { return c - 'A' < 26u; }

// Returns the new length, or -1 when the input is rejected (empty or longer than RP_PASSWORD_SIZE).
__device__ int apply_rule(uint8_t* w, int len, const uint8_t* __restrict__ code, uint32_t nops) {
    constexpr int RP = RP_PASSWORD_SIZE;
    if (len < 1 || len > RP) return -1;
    for (uint32_t k = 0; k < nops; k++) {
        const uint32_t op = code[3 * k], p1 = code[3 * k + 1], p2 = code[3 * k + 2];
        switch (op) {
        case 'l':
            for (int i = 0; i < len; i++) if (r_upper(w[i])) w[i] ^= 0x20;
            break;
        case 'u':
            for (int i = 0; i < len; i++) if (r_lower(w[i])) w[i] ^= 0x20;
            break;
        case 'c':
            for (int i = 0; i < len; i++) if (r_upper(w[i])) w[i] ^= 0x20;
            if (len && r_lower(w[0])) w[0] ^= 0x20;
            break;
        case 'C':
            for (int i = 0; i < len; i++) if (r_lower(w[i])) w[i] ^= 0x20;
            if (len && r_upper(w[0])) w[0] ^= 0x20;
            break;
        case 't':
            for (int i = 0; i < len; i++) if (r_lower(w[i]) || r_upper(w[i])) w[i] ^= 0x20;
            break;
        case 'T':
            if ((int)p1 < len && (r_lower(w[p1]) || r_upper(w[p1]))) w[p1] ^= 0x20;
            break;
        case 'r':
            for (int i = 0, j = len - 1; i < j; i++, j--) { uint8_t t = w[i]; w[i] = w[j]; w[j] = t; }
            break;
        case 'd':
            if (2 * len < RP) { for (int i = 0; i < len; i++) w[len + i] = w[i]; len *= 2; }
            break;
        case 'p':
            if (len * (int)p1 + len < RP) {
                for (int t = 1; t <= (int)p1; t++)
                    for (int i = 0; i < len; i++) w[t * len + i] = w[i];
                len += len * (int)p1;
            }
            break;
        case 'f':
            if (2 * len < RP) { for (int i = 0; i < len; i++) w[len + i] = w[len - 1 - i]; len *= 2; }
            break;
        case '{':
            if (len) { uint8_t c = w[0]; for (int i = 0; i + 1 < len; i++) w[i] = w[i + 1]; w[len - 1] = c; }
            break;
        case '}':
            if (len) { uint8_t c = w[len - 1]; for (int i = len - 1; i > 0; i--) w[i] = w[i - 1]; w[0] = c; }
            break;
        case '[':
            if (len) { for (int i = 0; i + 1 < len; i++) w[i] = w[i + 1]; len--; }
            break;
        case ']':
            if (len) len--;
            break;
        case 'q':
            if (2 * len < RP) { for (int i = len - 1; i >= 0; i--) { w[2 * i] = w[i]; w[2 * i + 1] = w[i]; } len *= 2; }
            break;
        case 'D':
            if ((int)p1 < len) { for (int i = (int)p1; i + 1 < len; i++) w[i] = w[i + 1]; len--; }
            break;
        case '\'':
            if ((int)p1 < len) len = (int)p1;
            break;
        case 'z':
            if (len && len + (int)p1 < RP) {
                for (int i = len - 1; i >= 0; i--) w[i + p1] = w[i];
                for (int i = 1; i <= (int)p1; i++) w[i] = w[0];
                len += (int)p1;
            }
            break;
        case 'Z':
            if (len && len + (int)p1 < RP) { for (int i = 0; i < (int)p1; i++) w[len + i] = w[len - 1]; len += (int)p1; }
            break;
        case '$':
            if (len + 1 < RP) w[len++] = (uint8_t)p1;
            break;
        case '^':
            if (len + 1 < RP) { for (int i = len; i > 0; i--) w[i] = w[i - 1]; w[0] = (uint8_t)p1; len++; }
            break;
        case 's':
            for (int i = 0; i < len; i++) if (w[i] == p1) w[i] = (uint8_t)p2;
            break;
        case '@': {
            int o = 0;
            for (int i = 0; i < len; i++) if (w[i] != p1) w[o++] = w[i];
            len = o;
            break;
        }
        default:
            break;  // ':' and anything the parser let through as a no-op
        }
    }
    return len;
}

__device__ __forceinline__ int load_word(const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes, uint64_t wi,
                                         uint8_t* w) {
    const uint64_t b0 = off[wi], b1 = off[wi + 1];
    const uint64_t n = b1 - b0;
    if (n < 1 || n > (uint64_t)RP_PASSWORD_SIZE) return -1;
    for (uint32_t i = 0; i < (uint32_t)n; i++) w[i] = bytes[b0 + i];
    return (int)n;
}

__global__ __launch_bounds__(256) void k_rules_prep(const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                                                    uint64_t first, uint32_t nwords, const uint32_t* __restrict__ roffs,
                                                    const uint8_t* __restrict__ rcode, uint32_t nrules, uint32_t minlen,
                                                    uint32_t maxlen, uint32_t* __restrict__ mid,
                                                    uint64_t* __restrict__ ids, uint32_t* __restrict__ counter,
                                                    uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = blockIdx.y;
    uint8_t w[RP_PASSWORD_SIZE + 4];
    int len = -1;
    if (i < nwords) {
        len = load_word(off, bytes, first + i, w);
        if (len > 0) {
            const uint32_t c0 = roffs[r], c1 = roffs[r + 1];
            len = apply_rule(w, len, rcode + c0, (c1 - c0) / 3);
        }
    }
    const bool keep = len >= (int)minlen && len <= (int)maxlen && len <= 64;
    const uint32_t slot = compact_slot(keep, counter);
    if (!keep || slot >= cap) return;
    uint32_t kb[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int k = 4 * j + b;
            v = (v << 8) | (k < len ? (uint32_t)w[k] : 0u);
        }
        kb[j] = v;
    }
    store_mid(mid, cap, slot, kb);
    ids[slot] = (first + i) * (uint64_t)nrules + r;
}

__global__ __launch_bounds__(256) void k_rules_expand(const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                                                      uint32_t nwords, const uint32_t* __restrict__ roffs,
                                                      const uint8_t* __restrict__ rcode, uint32_t nrules,
                                                      uint8_t* __restrict__ out, uint32_t* __restrict__ out_len) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = blockIdx.y;
    if (i >= nwords) return;
    uint8_t w[RP_PASSWORD_SIZE + 4];
    int len = load_word(off, bytes, i, w);
    if (len > 0) {
        const uint32_t c0 = roffs[r], c1 = roffs[r + 1];
        len = apply_rule(w, len, rcode + c0, (c1 - c0) / 3);
    }
    const size_t c = (size_t)i * nrules + r;
    out_len[c] = len < 0 ? 0xffffffffu : (uint32_t)len;
    for (int k = 0; k < len; k++) out[c * RP_PASSWORD_SIZE + k] = w[k];
}

hipError_t launch_rules_prep(const uint64_t* off, const uint8_t* bytes, uint64_t first, uint32_t nwords,
                             const uint32_t* roffs, const uint8_t* rcode, uint32_t nrules, uint32_t minlen,
                             uint32_t maxlen, uint32_t* mid, uint64_t* ids, uint32_t* counter, uint32_t cap,
                             hipStream_t s) {
    if (nwords == 0 || nrules == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rules_prep, dim3((nwords + 255) / 256, nrules), dim3(256), 0, s, off, bytes, first, nwords,
                       roffs, rcode, nrules, minlen, maxlen, mid, ids, counter, cap);
    return hipGetLastError();
}

hipError_t launch_rules_expand(const uint64_t* off, const uint8_t* bytes, uint32_t nwords, const uint32_t* roffs,
                               const uint8_t* rcode, uint32_t nrules, uint8_t* out, uint32_t* out_len,
                               hipStream_t s) {
    if (nwords == 0 || nrules == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rules_expand, dim3((nwords + 255) / 256, nrules), dim3(256), 0, s, off, bytes, nwords, roffs,
                       rcode, nrules, out, out_len);
    return hipGetLastError();
}

}  // namespace dwpa
