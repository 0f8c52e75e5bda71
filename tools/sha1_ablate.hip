// sha1_ablate.hip -- where does the PBKDF2 inner loop lose issue slots on gfx950?  (design exploration)
//
// Runs variants of the HMAC inner-loop compression (sha1_84) and reports SIMD cycles per compression per wave,
// next to the static VALU cost the compiler emitted (counted offline from the .s).  Occupancy is swept with
// dynamic LDS.  Values are kept live with asm so nothing is dead-code eliminated.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

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

// rounds only: W_t = in[t % 5] (no schedule work), same round functions
__device__ __forceinline__ void rounds_only(const Sha1Mid& M, const uint32_t in[5], uint32_t out[5]) {
    uint32_t a1 = M.c0 + in[0];
    uint32_t a2 = rotl(a1, 5) + M.c1 + in[1];
    uint32_t a = a2, b = a1, c = M.r0, d = M.r1, e = M.h2;
#pragma unroll
    for (int t = 2; t < 80; t++) {
        uint32_t f;
        if (t < 20) f = DWPA_SHA1_CH(b, c, d);
        else if (t < 40 || t >= 60) f = xor3(b, c, d);
        else f = maj3(b, c, d);
        const uint32_t k = t < 20 ? SHA1_K0 : t < 40 ? SHA1_K1 : t < 60 ? SHA1_K2 : SHA1_K3;
        uint32_t tt = rotl(a, 5) + f + e + k + in[t % 5];
        e = d; d = c; c = rotl(b, 30); b = a; a = tt;
    }
    out[0] = M.h0 + a; out[1] = M.h1 + b; out[2] = M.h2 + c; out[3] = M.h3 + d; out[4] = M.h4 + e;
}

// schedule only: W16..W79 of the 84-byte message, folded into 5 outputs
__device__ __forceinline__ void sched_only(const uint32_t in[5], uint32_t out[5]) {
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = i < 5 ? in[i] : w84_const(i);
    uint32_t acc[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int t = 16; t < 80; t++) {
        uint32_t x = rotl(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15], 1);
        w[t & 15] = x;
        acc[t % 5] += x;
    }
    for (int i = 0; i < 5; i++) out[i] = acc[i];
}

template <int V>
__global__ __launch_bounds__(256) void k_abl(const uint32_t* __restrict__ mid, uint32_t* __restrict__ out, uint32_t iters,
                                            unsigned long long* clk) {
    extern __shared__ uint32_t pad[];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t hi[5], ho[5], u[5], x[5];
    for (int k = 0; k < 5; k++) { hi[k] = mid[k * 64 + (s & 63)]; ho[k] = mid[(5 + k) * 64 + (s & 63)]; u[k] = hi[k] ^ s; }
    const Sha1Mid MI = sha1_mid(hi), MO = sha1_mid(ho);
    uint32_t t[5] = {0, 0, 0, 0, 0};
#pragma unroll 1
    for (uint32_t it = 0; it < iters; it++) {
        if constexpr (V == 0) { sha1_84(MI, u, x); sha1_84(MO, x, u); }
        if constexpr (V == 1) { rounds_only(MI, u, x); rounds_only(MO, x, u); }
        if constexpr (V == 2) { sched_only(u, x); sched_only(x, u); }
        for (int k = 0; k < 5; k++) t[k] ^= u[k];
    }
    if (pad == nullptr) out[0] = 0;
    for (int k = 0; k < 5; k++) out[k * gridDim.x * blockDim.x + s] = t[k];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
        clk[2 * w] = t1 - t0;
        clk[2 * w + 1] = r1 - r0;
    }
}

static const char* NAMES[] = {"sha1_84 (full)", "rounds only", "schedule only"};

template <int V>
static void run(int cus, int blocks_per_cu, uint32_t iters, uint32_t* mid, uint32_t* out, unsigned long long* clk,
                bool first) {
    const int rounds = 4;  // grid = 4 full residency rounds
    const int blocks = cus * blocks_per_cu * rounds;
    const size_t lds = blocks_per_cu >= 8 ? 0 : (160 * 1024) / blocks_per_cu - 512;
    hipLaunchKernelGGL(k_abl<V>, dim3(cus * 8), dim3(256), lds, 0, mid, out, 4u, clk);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_abl<V>, dim3(blocks), dim3(256), lds, 0, mid, out, iters, clk);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const int waves = blocks * 4;
    std::vector<unsigned long long> h(2 * (size_t)waves);
    CHK(hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (int i = 0; i < waves; i++) { cyc += (double)h[2 * i]; rt += (double)h[2 * i + 1]; }
    const double clock_hz = cyc / (rt / 100e6);
    const double comps = (double)waves * iters * 2.0;  // wave-compressions
    printf("%s{\"variant\": \"%s\", \"waves_per_simd\": %d, \"clock_mhz\": %.0f, \"simd_cycles_per_compression\": %.1f}",
           first ? "" : ",\n  ", NAMES[V], blocks_per_cu, clock_hz / 1e6, (ms * 1e-3) * clock_hz * cus * 4 / comps);
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t *mid, *out;
    unsigned long long* clk;
    CHK(hipMalloc(&mid, 640 * 4));
    std::vector<uint32_t> hm(640);
    uint32_t x = 777;
    for (auto& v : hm) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = x; }
    CHK(hipMemcpy(mid, hm.data(), 640 * 4, hipMemcpyHostToDevice));
    CHK(hipMalloc(&out, (size_t)cus * 8 * 4 * 256 * 5 * 4));
    CHK(hipMalloc(&clk, (size_t)cus * 8 * 4 * 4 * 16));
    const uint32_t iters = 400;
    printf("{\"results\": [\n  ");
    bool f = true;
    for (int bpc : {8, 7, 6, 4, 2}) {
        run<0>(cus, bpc, iters, mid, out, clk, f); f = false;
        run<1>(cus, bpc, iters, mid, out, clk, f);
        run<2>(cus, bpc, iters, mid, out, clk, f);
    }
    printf("]}\n");
    return 0;
}
