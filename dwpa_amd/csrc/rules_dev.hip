// rules_dev.hip -- on-GPU hashcat rule amplification of HBM-resident dictionaries (north_star "rule expansion").
//
// Grid = (word chunks) x (rules): every wave applies ONE rule (blockIdx.y) to 64 consecutive words, so the rule
// code is wave-uniform (scalar loads, uniform branches) and only the word bytes differ per lane.  Each lane works on
// a private 256-byte buffer (hashcat's RP_PASSWORD_SIZE), plus a second one for the memory functions, touched only
// by a rule that saves the word (M); until then the memory is the input word, read where it lies in HBM.  The
// interpreter is rules_apply.hpp (shared with the host).  Results outside 8..63 bytes or rejected by a rule are
// dropped (hashcat -m 22000 limits), the survivors are compacted into the batch as HMAC-SHA1 key midstates exactly
// like k_prep_dict.  Candidate id = word * nrules + rule.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crypto_dev.hpp"
#include "prep_dev.hpp"
#include "rules.hpp"
#include "rules_apply.hpp"

namespace dwpa {

// Copies word wi into w; returns its length, or -1 if hashcat's rule engine rejects it (empty or > 256 bytes).
// *src = where the word lies in HBM (the memory functions' initial memory).
__device__ __forceinline__ int load_word(const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes, uint64_t wi,
                                         uint8_t* w, const uint8_t** src) {
    const uint64_t b0 = off[wi], b1 = off[wi + 1];
    const uint64_t n = b1 - b0;
    *src = bytes + b0;
    if (n < 1 || n > (uint64_t)RP_PASSWORD_SIZE) return -1;
    for (uint32_t i = 0; i < (uint32_t)n; i++) w[i] = bytes[b0 + i];
    return (int)n;
}

__global__ __launch_bounds__(256) void k_rules_prep(const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                                                    uint64_t first, uint32_t nwords, const uint32_t* __restrict__ roffs,
                                                    const uint32_t* __restrict__ rcode, uint32_t nrules, uint32_t minlen,
                                                    uint32_t maxlen, uint32_t* __restrict__ mid,
                                                    uint64_t* __restrict__ ids, uint32_t* __restrict__ counter,
                                                    uint32_t cap) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = blockIdx.y;
    uint8_t w[RP_PASSWORD_SIZE + 4], mem[RP_PASSWORD_SIZE + 4];
    int len = -1;
    if (i < nwords) {
        const uint8_t* src;
        len = load_word(off, bytes, first + i, w, &src);
        if (len > 0) {
            const uint32_t c0 = roffs[r], c1 = roffs[r + 1];
            len = rule_apply(w, len, mem, src, len, rcode + c0, c1 - c0);
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
                                                      const uint32_t* __restrict__ rcode, uint32_t nrules,
                                                      uint8_t* __restrict__ out, uint32_t* __restrict__ out_len) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = blockIdx.y;
    if (i >= nwords) return;
    uint8_t w[RP_PASSWORD_SIZE + 4], mem[RP_PASSWORD_SIZE + 4];
    const uint8_t* src;
    int len = load_word(off, bytes, i, w, &src);
    if (len > 0) {
        const uint32_t c0 = roffs[r], c1 = roffs[r + 1];
        len = rule_apply(w, len, mem, src, len, rcode + c0, c1 - c0);
    }
    const size_t c = (size_t)i * nrules + r;
    out_len[c] = len < 0 ? 0xffffffffu : (uint32_t)len;
    for (int k = 0; k < len; k++) out[c * RP_PASSWORD_SIZE + k] = w[k];
}

hipError_t launch_rules_prep(const uint64_t* off, const uint8_t* bytes, uint64_t first, uint32_t nwords,
                             const uint32_t* roffs, const uint32_t* rcode, uint32_t nrules, uint32_t minlen,
                             uint32_t maxlen, uint32_t* mid, uint64_t* ids, uint32_t* counter, uint32_t cap,
                             hipStream_t s) {
    if (nwords == 0 || nrules == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rules_prep, dim3((nwords + 255) / 256, nrules), dim3(256), 0, s, off, bytes, first, nwords,
                       roffs, rcode, nrules, minlen, maxlen, mid, ids, counter, cap);
    return hipGetLastError();
}

hipError_t launch_rules_expand(const uint64_t* off, const uint8_t* bytes, uint32_t nwords, const uint32_t* roffs,
                               const uint32_t* rcode, uint32_t nrules, uint8_t* out, uint32_t* out_len,
                               hipStream_t s) {
    if (nwords == 0 || nrules == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rules_expand, dim3((nwords + 255) / 256, nrules), dim3(256), 0, s, off, bytes, nwords, roffs,
                       rcode, nrules, out, out_len);
    return hipGetLastError();
}

}  // namespace dwpa
