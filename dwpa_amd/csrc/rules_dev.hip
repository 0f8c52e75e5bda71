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

// text_len (nullable): the candidate's bytes in the wordlist text as hashcat's --stdout writes it -- its raw bytes
// and '\n', or "$HEX[<2n hex digits>]\n" when it holds a '\n' or '\r' (which would not stay one line); 0 when
// rejected.  k_text_block_sums / k_text_scan_sums / k_text_pack then pack the text on the GPU (TEXT_BLOCK
// candidates per block), so only the text crosses PCIe, not the 256-byte slots.
__global__ __launch_bounds__(256) void k_rules_expand(const uint64_t* __restrict__ off, const uint8_t* __restrict__ bytes,
                                                      uint32_t nwords, const uint32_t* __restrict__ roffs,
                                                      const uint32_t* __restrict__ rcode, uint32_t nrules,
                                                      uint8_t* __restrict__ out, uint32_t* __restrict__ out_len,
                                                      uint32_t* __restrict__ text_len) {
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
    bool brk = false;
    for (int k = 0; k < len; k++) {
        out[c * RP_PASSWORD_SIZE + k] = w[k];
        brk |= w[k] == '\n' || w[k] == '\r';
    }
    if (text_len) text_len[c] = len < 0 ? 0u : brk ? 7u + 2u * (uint32_t)len : (uint32_t)len + 1u;
}

constexpr uint32_t TEXT_BLOCK = 1024;  // candidates per block of the text scan (256 threads x 4)

// Block b: the sum of text_len over candidates [b * TEXT_BLOCK, (b+1) * TEXT_BLOCK) and how many are kept.
__global__ __launch_bounds__(256) void k_text_block_sums(const uint32_t* __restrict__ text_len, uint32_t n,
                                                         uint32_t* __restrict__ bsum, uint32_t* __restrict__ bcnt) {
    __shared__ uint32_t ssum[4], scnt[4];
    const uint32_t base = blockIdx.x * TEXT_BLOCK;
    uint32_t s = 0, k = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t c = base + j * 256 + threadIdx.x;
        const uint32_t v = c < n ? text_len[c] : 0u;
        s += v;
        k += v != 0;
    }
    for (int d = 32; d; d >>= 1) {
        s += __shfl_xor(s, d);
        k += __shfl_xor(k, d);
    }
    if ((threadIdx.x & 63) == 0) {
        ssum[threadIdx.x >> 6] = s;
        scnt[threadIdx.x >> 6] = k;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        bsum[blockIdx.x] = ssum[0] + ssum[1] + ssum[2] + ssum[3];
        bcnt[blockIdx.x] = scnt[0] + scnt[1] + scnt[2] + scnt[3];
    }
}

// One block: bsum[] -> exclusive prefix sums in place (any nblocks, 256 at a time); tot[0] = text bytes,
// tot[1] = kept candidates.
__global__ __launch_bounds__(256) void k_text_scan_sums(uint32_t* __restrict__ bsum, const uint32_t* __restrict__ bcnt,
                                                        uint32_t nblocks, uint32_t* __restrict__ tot) {
    __shared__ uint32_t part[256];
    uint32_t carry = 0, kept = 0;
    for (uint32_t b0 = 0; b0 < nblocks; b0 += 256) {
        const uint32_t b = b0 + threadIdx.x;
        const uint32_t v = b < nblocks ? bsum[b] : 0u;
        kept += b < nblocks ? bcnt[b] : 0u;
        part[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t d = 1; d < 256; d <<= 1) {  // Hillis-Steele inclusive scan of 256 values
            const uint32_t add = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
            __syncthreads();
            part[threadIdx.x] += add;
            __syncthreads();
        }
        if (b < nblocks) bsum[b] = carry + part[threadIdx.x] - v;
        carry += part[255];
        __syncthreads();
    }
    for (int d = 32; d; d >>= 1) kept += __shfl_xor(kept, d);
    __shared__ uint32_t skept[4];
    if ((threadIdx.x & 63) == 0) skept[threadIdx.x >> 6] = kept;
    __syncthreads();
    if (threadIdx.x == 0) {
        tot[0] = carry;
        tot[1] = skept[0] + skept[1] + skept[2] + skept[3];
    }
}

// Candidate c's text at text + boff[c / TEXT_BLOCK] + (its exclusive prefix within the block, scanned in LDS).  A
// candidate whose text would end past `cap` is not written (the host sees tot[0] > cap, grows the buffer and packs
// the sub-batch again).
__global__ __launch_bounds__(256) void k_text_pack(const uint8_t* __restrict__ out, const uint32_t* __restrict__ out_len,
                                                   const uint32_t* __restrict__ text_len, uint32_t n,
                                                   const uint32_t* __restrict__ boff, uint8_t* __restrict__ text,
                                                   uint64_t cap) {
    __shared__ uint32_t sc[TEXT_BLOCK];
    const uint32_t base = blockIdx.x * TEXT_BLOCK;
    // thread t owns candidates base + 4t .. 4t+3 (contiguous, so its prefix is a running sum)
    uint32_t v[4], run = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t c = base + 4 * threadIdx.x + j;
        v[j] = c < n ? text_len[c] : 0u;
        run += v[j];
    }
    sc[threadIdx.x] = run;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {
        const uint32_t add = threadIdx.x >= d ? sc[threadIdx.x - d] : 0u;
        __syncthreads();
        sc[threadIdx.x] += add;
        __syncthreads();
    }
    uint32_t pos = boff[blockIdx.x] + sc[threadIdx.x] - run;
    static constexpr char HEXD[] = "0123456789abcdef";
#pragma unroll 1
    for (int j = 0; j < 4; j++) {
        const uint32_t c = base + 4 * threadIdx.x + j;
        const uint32_t at = pos;
        pos += v[j];  // advanced whether or not this candidate is written: the next one's offset depends on it
        if (!v[j] || (uint64_t)at + v[j] > cap) continue;
        const uint32_t len = out_len[c];
        const uint8_t* p = out + (size_t)c * RP_PASSWORD_SIZE;
        uint8_t* d = text + at;
        if (v[j] == len + 1) {
            for (uint32_t k = 0; k < len; k++) d[k] = p[k];
            d[len] = '\n';
        } else {
            d[0] = '$'; d[1] = 'H'; d[2] = 'E'; d[3] = 'X'; d[4] = '[';
            for (uint32_t k = 0; k < len; k++) {
                d[5 + 2 * k] = (uint8_t)HEXD[p[k] >> 4];
                d[6 + 2 * k] = (uint8_t)HEXD[p[k] & 15];
            }
            d[5 + 2 * len] = ']';
            d[6 + 2 * len] = '\n';
        }
    }
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
                               hipStream_t s, uint32_t* text_len) {
    if (nwords == 0 || nrules == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rules_expand, dim3((nwords + 255) / 256, nrules), dim3(256), 0, s, off, bytes, nwords, roffs,
                       rcode, nrules, out, out_len, text_len);
    return hipGetLastError();
}

uint32_t text_pack_blocks(uint32_t n) { return (n + TEXT_BLOCK - 1) / TEXT_BLOCK; }

hipError_t launch_text_pack(const uint8_t* out, const uint32_t* out_len, const uint32_t* text_len, uint32_t n,
                            uint32_t* bsum, uint32_t* bcnt, uint32_t* tot, uint8_t* text, uint64_t cap,
                            hipStream_t s) {
    const uint32_t nb = text_pack_blocks(n);
    if (nb == 0) return hipMemsetAsync(tot, 0, 8, s);
    hipLaunchKernelGGL(k_text_block_sums, dim3(nb), dim3(256), 0, s, text_len, n, bsum, bcnt);
    hipLaunchKernelGGL(k_text_scan_sums, dim3(1), dim3(256), 0, s, bsum, bcnt, nb, tot);
    hipLaunchKernelGGL(k_text_pack, dim3(nb), dim3(256), 0, s, out, out_len, text_len, n, bsum, text, cap);
    return hipGetLastError();
}

}  // namespace dwpa
