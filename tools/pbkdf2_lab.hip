// pbkdf2_lab.hip -- A/B harness for PBKDF2-HMAC-SHA1 kernel variants on gfx950 (design exploration, not product).
//
// Variants are run interleaved in one process (MI355X methodology rule: perf deltas from interleaved rounds),
// each reports wall ms per launch, in-kernel clock (s_memtime / s_memrealtime) and PMK/s; outputs are checked
// against variant 0 word for word.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../dwpa_amd/csrc/crypto_dev.hpp"

using namespace dwpa;

#define CHK(x)                                                                           \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

struct Clk {
    unsigned long long cyc, rt;
};

__device__ __forceinline__ void stamp_end(Clk* clk, unsigned long long t0, unsigned long long r0) {
    if ((threadIdx.x & 63) == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t w = (blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
        clk[w].cyc = t1 - t0;
        clk[w].rt = r1 - r0;
    }
}

// V0: the product kernel's structure (one output block per lane, blockIdx.y = block)
template <int ITERS>
__global__ __launch_bounds__(256) void v0(const uint32_t* __restrict__ mid, uint32_t n, const uint32_t* __restrict__ salt,
                                          uint32_t* __restrict__ out, Clk* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t blk = blockIdx.y;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) {
        uint32_t hi[5], ho[5];
        for (int k = 0; k < 5; k++) { hi[k] = mid[k * n + s]; ho[k] = mid[(5 + k) * n + s]; }
        uint32_t st[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]};
        uint32_t m[16];
        for (int j = 0; j < 16; j++) m[j] = salt[blk * 16 + j];
        sha1_compress(st, m);
        const Sha1Mid MI = sha1_mid(hi), MO = sha1_mid(ho);
        uint32_t u[5], x[5], t[5];
        sha1_84(MO, st, u);
        for (int k = 0; k < 5; k++) t[k] = u[k];
#pragma unroll 1
        for (int it = 1; it < ITERS; it++) {
            sha1_84(MI, u, x);
            sha1_84(MO, x, u);
            for (int k = 0; k < 5; k++) t[k] ^= u[k];
        }
        for (int k = 0; k < 5; k++) out[(blk * 5 + k) * n + s] = t[k];
    }
    stamp_end(clk, t0, r0);
}

// VN: V0 with s_nop spacer policy NOP inside the SHA-1 rounds
template <int ITERS, int NOP>
__global__ __launch_bounds__(256) void vn(const uint32_t* __restrict__ mid, uint32_t n, const uint32_t* __restrict__ salt,
                                          uint32_t* __restrict__ out, Clk* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t blk = blockIdx.y;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) {
        uint32_t hi[5], ho[5];
        for (int k = 0; k < 5; k++) { hi[k] = mid[k * n + s]; ho[k] = mid[(5 + k) * n + s]; }
        uint32_t st[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]};
        uint32_t m[16];
        for (int j = 0; j < 16; j++) m[j] = salt[blk * 16 + j];
        sha1_compress(st, m);
        const Sha1Mid MI = sha1_mid(hi), MO = sha1_mid(ho);
        uint32_t u[5], x[5], t[5];
        sha1_84(MO, st, u);
        for (int k = 0; k < 5; k++) t[k] = u[k];
#pragma unroll 1
        for (int it = 1; it < ITERS; it++) {
            sha1_84<NOP>(MI, u, x);
            sha1_84<NOP>(MO, x, u);
            for (int k = 0; k < 5; k++) t[k] ^= u[k];
        }
        for (int k = 0; k < 5; k++) out[(blk * 5 + k) * n + s] = t[k];
    }
    stamp_end(clk, t0, r0);
}

// V1: both output blocks in one lane, interleaved (two independent chains -> ILP 2, ~2x VGPRs)
template <int ITERS>
__global__ __launch_bounds__(256) void v1(const uint32_t* __restrict__ mid, uint32_t n, const uint32_t* __restrict__ salt,
                                          uint32_t* __restrict__ out, Clk* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) {
        uint32_t hi[5], ho[5];
        for (int k = 0; k < 5; k++) { hi[k] = mid[k * n + s]; ho[k] = mid[(5 + k) * n + s]; }
        uint32_t sa[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]}, sb[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]};
        uint32_t m[16];
        for (int j = 0; j < 16; j++) m[j] = salt[j];
        sha1_compress(sa, m);
        for (int j = 0; j < 16; j++) m[j] = salt[16 + j];
        sha1_compress(sb, m);
        const Sha1Mid MI = sha1_mid(hi), MO = sha1_mid(ho);
        uint32_t ua[5], xa[5], ta[5], ub[5], xb[5], tb[5];
        sha1_84(MO, sa, ua);
        sha1_84(MO, sb, ub);
        for (int k = 0; k < 5; k++) { ta[k] = ua[k]; tb[k] = ub[k]; }
#pragma unroll 1
        for (int it = 1; it < ITERS; it++) {
            sha1_84(MI, ua, xa);
            sha1_84(MI, ub, xb);
            sha1_84(MO, xa, ua);
            sha1_84(MO, xb, ub);
            for (int k = 0; k < 5; k++) { ta[k] ^= ua[k]; tb[k] ^= ub[k]; }
        }
        for (int k = 0; k < 5; k++) { out[k * n + s] = ta[k]; out[(5 + k) * n + s] = tb[k]; }
    }
    stamp_end(clk, t0, r0);
}

// V2: V0 with the 4096-loop unrolled by 2 (scheduler sees two iterations)
template <int ITERS>
__global__ __launch_bounds__(256) void v2(const uint32_t* __restrict__ mid, uint32_t n, const uint32_t* __restrict__ salt,
                                          uint32_t* __restrict__ out, Clk* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t blk = blockIdx.y;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) {
        uint32_t hi[5], ho[5];
        for (int k = 0; k < 5; k++) { hi[k] = mid[k * n + s]; ho[k] = mid[(5 + k) * n + s]; }
        uint32_t st[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]};
        uint32_t m[16];
        for (int j = 0; j < 16; j++) m[j] = salt[blk * 16 + j];
        sha1_compress(st, m);
        const Sha1Mid MI = sha1_mid(hi), MO = sha1_mid(ho);
        uint32_t u[5], x[5], t[5];
        sha1_84(MO, st, u);
        for (int k = 0; k < 5; k++) t[k] = u[k];
        int it = 1;
        sha1_84(MI, u, x);
        sha1_84(MO, x, u);
        for (int k = 0; k < 5; k++) t[k] ^= u[k];
        it++;
#pragma unroll 1
        for (; it < ITERS; it += 2) {
            sha1_84(MI, u, x);
            sha1_84(MO, x, u);
            for (int k = 0; k < 5; k++) t[k] ^= u[k];
            sha1_84(MI, u, x);
            sha1_84(MO, x, u);
            for (int k = 0; k < 5; k++) t[k] ^= u[k];
        }
        for (int k = 0; k < 5; k++) out[(blk * 5 + k) * n + s] = t[k];
    }
    stamp_end(clk, t0, r0);
}

// V3: V0 launched as 64-thread workgroups
template <int ITERS>
__global__ __launch_bounds__(64) void v3(const uint32_t* __restrict__ mid, uint32_t n, const uint32_t* __restrict__ salt,
                                         uint32_t* __restrict__ out, Clk* clk) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t blk = blockIdx.y;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) {
        uint32_t hi[5], ho[5];
        for (int k = 0; k < 5; k++) { hi[k] = mid[k * n + s]; ho[k] = mid[(5 + k) * n + s]; }
        uint32_t st[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]};
        uint32_t m[16];
        for (int j = 0; j < 16; j++) m[j] = salt[blk * 16 + j];
        sha1_compress(st, m);
        const Sha1Mid MI = sha1_mid(hi), MO = sha1_mid(ho);
        uint32_t u[5], x[5], t[5];
        sha1_84(MO, st, u);
        for (int k = 0; k < 5; k++) t[k] = u[k];
#pragma unroll 1
        for (int it = 1; it < ITERS; it++) {
            sha1_84(MI, u, x);
            sha1_84(MO, x, u);
            for (int k = 0; k < 5; k++) t[k] ^= u[k];
        }
        for (int k = 0; k < 5; k++) out[(blk * 5 + k) * n + s] = t[k];
    }
    stamp_end(clk, t0, r0);
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    constexpr int IT = 4096;
    std::vector<uint32_t> h_mid(10 * (size_t)n), h_salt(32);
    uint32_t x = 12345;
    for (auto& v : h_mid) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = x; }
    for (auto& v : h_salt) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = x; }
    uint32_t *mid, *salt, *out[8];
    Clk* clk;
    const size_t nw = (size_t)n * 2 / 64 + 64;
    CHK(hipMalloc(&mid, h_mid.size() * 4));
    CHK(hipMalloc(&salt, 128));
    for (int v = 0; v < 8; v++) CHK(hipMalloc(&out[v], (size_t)n * 10 * 4));
    CHK(hipMalloc(&clk, nw * sizeof(Clk)));
    CHK(hipMemcpy(mid, h_mid.data(), h_mid.size() * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(salt, h_salt.data(), 128, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    constexpr int NV = 8;
    const char* names[NV] = {"v0_baseline", "v2_unroll2", "nop1_after_sched", "nop2_after_sum", "nop4_after_rot30",
                             "nop3_sched+sum", "nop6_sum+rot30", "nop7_all"};
    std::vector<double> best(NV, 1e30), clkmhz(NV, 0);
    for (int r = 0; r < rounds; r++) {
        for (int v = 0; v < NV; v++) {
            CHK(hipEventRecord(e0, 0));
            dim3 g((n + 255) / 256, 2);
            if (v == 0) hipLaunchKernelGGL(v0<IT>, g, dim3(256), 0, 0, mid, n, salt, out[v], clk);
            if (v == 1) hipLaunchKernelGGL(v2<IT>, g, dim3(256), 0, 0, mid, n, salt, out[v], clk);
            if (v == 2) hipLaunchKernelGGL((vn<IT, 1>), g, dim3(256), 0, 0, mid, n, salt, out[v], clk);
            if (v == 3) hipLaunchKernelGGL((vn<IT, 2>), g, dim3(256), 0, 0, mid, n, salt, out[v], clk);
            if (v == 4) hipLaunchKernelGGL((vn<IT, 4>), g, dim3(256), 0, 0, mid, n, salt, out[v], clk);
            if (v == 5) hipLaunchKernelGGL((vn<IT, 3>), g, dim3(256), 0, 0, mid, n, salt, out[v], clk);
            if (v == 6) hipLaunchKernelGGL((vn<IT, 6>), g, dim3(256), 0, 0, mid, n, salt, out[v], clk);
            if (v == 7) hipLaunchKernelGGL((vn<IT, 7>), g, dim3(256), 0, 0, mid, n, salt, out[v], clk);
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            const size_t waves = (size_t)(n + 63) / 64 * 2;
            std::vector<Clk> hc(waves);
            CHK(hipMemcpy(hc.data(), clk, waves * sizeof(Clk), hipMemcpyDeviceToHost));
            std::vector<double> f;
            for (auto& c : hc)
                if (c.rt) f.push_back((double)c.cyc / ((double)c.rt / 100e6));
            std::sort(f.begin(), f.end());
            if (ms < best[v]) { best[v] = ms; clkmhz[v] = f.empty() ? 0 : f[f.size() / 2] / 1e6; }
        }
    }
    std::vector<uint32_t> ref((size_t)n * 10), o((size_t)n * 10);
    CHK(hipMemcpy(ref.data(), out[0], ref.size() * 4, hipMemcpyDeviceToHost));
    printf("{\"n\": %u, \"iterations\": %d, \"variants\": [", n, IT);
    for (int v = 0; v < NV; v++) {
        CHK(hipMemcpy(o.data(), out[v], o.size() * 4, hipMemcpyDeviceToHost));
        const bool same = memcmp(o.data(), ref.data(), o.size() * 4) == 0;
        printf("%s\n  {\"name\": \"%s\", \"best_ms\": %.3f, \"pmk_per_s\": %.0f, \"median_wave_clock_mhz\": %.0f, "
               "\"matches_v0\": %s}", v ? "," : "", names[v], best[v], n / (best[v] * 1e-3), clkmhz[v],
               same ? "true" : "false");
    }
    printf("]}\n");
    return 0;
}
