// tail_placement.hip -- where do the waves of small launches land beside a running one-round launch?
//
// Question (C5's PBKDF2 tail): the check path's tail (176 waves) runs beside a head of 6 waves
// per SIMD, so the SIMDs that host a tail wave carry 7 waves of work.  Cutting the tail into P sequential launches
// of 4096/P iterations each would spread that work only if consecutive launches land on different SIMDs.  This
// probe runs a head-like launch (6 waves per SIMD of issue-bound VALU work) and, on a second stream beside it, P
// small launches one after another; lane 0 of every probe wave records its hardware ids (HW_ID: SIMD/CU/SH/SE,
// XCC_ID).  Prints, per probe launch, its distinct SIMDs and how many of them earlier launches already used.
//   tools/bin/tail_placement [pieces] [probe_wgs] [probe_threads]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <set>
#include <tuple>
#include <vector>

#define CHK(x)                                                                         \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// Four independent chains of full-rate ops: enough independent work that 6 waves keep a SIMD issue-bound.
__device__ __forceinline__ void spin(unsigned iters, unsigned& a, unsigned& b, unsigned& c, unsigned& d) {
    for (unsigned i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            a = (a ^ b) + 0x9e3779b9u;
            c = (c ^ d) + 0x7f4a7c15u;
            b = b + (a >> 3);
            d = d + (c >> 5);
        }
    }
}

__global__ __launch_bounds__(256) void k_head(unsigned iters, unsigned* sink) {
    unsigned a = threadIdx.x, b = blockIdx.x, c = a * 3u + 1u, d = b * 5u + 7u;
    spin(iters, a, b, c, d);
    if ((a ^ b ^ c ^ d) == 0x12345678u) sink[0] = a;  // keeps the loop; practically never stores
}

__global__ void k_probe(unsigned* out, unsigned piece, unsigned waves, unsigned iters, unsigned* sink) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID, 32 bits
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID, bits 3:0
    const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    unsigned a = threadIdx.x, b = piece, c = 3u, d = 7u;
    spin(iters, a, b, c, d);
    if ((threadIdx.x & 63) == 0 && wave < waves) {
        out[2 * (piece * waves + wave)] = hw;
        out[2 * (piece * waves + wave) + 1] = xcc;
    }
    if ((a ^ b ^ c ^ d) == 0x12345678u) sink[1] = a;
}

int main(int argc, char** argv) {
    const unsigned pieces = argc > 1 ? atoi(argv[1]) : 8;
    const unsigned wgs = argc > 2 ? atoi(argv[2]) : 44;
    const unsigned threads = argc > 3 ? atoi(argv[3]) : 256;
    if (pieces < 1 || pieces > 64 || wgs < 1 || wgs > 4096 || threads < 64 || threads > 1024 || threads % 64) return 2;
    const unsigned waves = wgs * threads / 64;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const unsigned cus = prop.multiProcessorCount;
    unsigned *out, *sink;
    CHK(hipMalloc(&out, (size_t)pieces * waves * 8));
    CHK(hipMemset(out, 0xff, (size_t)pieces * waves * 8));
    CHK(hipMalloc(&sink, 64));
    hipStream_t sh, st;
    CHK(hipStreamCreateWithFlags(&sh, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    // head: 6 waves per SIMD, ~40 ms; probes: each ~1/pieces of that for one wave alone
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, sh));
    hipLaunchKernelGGL(k_head, dim3(cus * 6), dim3(256), 0, sh, 60000u, sink);
    CHK(hipEventRecord(e1, sh));
    for (unsigned p = 0; p < pieces; p++)
        hipLaunchKernelGGL(k_probe, dim3(wgs), dim3(threads), 0, st, out, p, waves, 60000u / pieces, sink);
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned> h((size_t)pieces * waves * 2);
    CHK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
    using Key = std::tuple<unsigned, unsigned, unsigned, unsigned, unsigned>;  // xcc, se, sh, cu, simd
    std::set<Key> seen;
    printf("{\"cus\": %u, \"pieces\": %u, \"probe_wgs\": %u, \"probe_threads\": %u, \"head_ms\": %.2f, \"launches\": [\n",
           cus, pieces, wgs, threads, ms);
    for (unsigned p = 0; p < pieces; p++) {
        std::set<Key> mine;
        std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> cu_set;
        for (unsigned w = 0; w < waves; w++) {
            const unsigned hw = h[2 * (p * waves + w)], xcc = h[2 * (p * waves + w) + 1] & 0xf;
            const Key k{xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15, (hw >> 4) & 3};
            mine.insert(k);
            cu_set.insert({xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15});
        }
        unsigned again = 0;
        for (const Key& k : mine) again += seen.count(k);
        printf("  {\"piece\": %u, \"simds\": %zu, \"cus\": %zu, \"simds_used_before\": %u}%s\n", p, mine.size(),
               cu_set.size(), again, p + 1 < pieces ? "," : "");
        seen.insert(mine.begin(), mine.end());
    }
    printf("], \"distinct_simds_all_pieces\": %zu}\n", seen.size());
    return 0;
}
