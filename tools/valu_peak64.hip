// valu_peak64.hip -- gfx950 issue costs of the 64-bit / packed VALU ops that could carry SHA-1 rotates: a value
// held twice in a VGPR pair (x:x) is rotated by one 64-bit shift (low word of (x:x) >> n = rotr(x, n)).  Same
// method as valu_peak.hip: 8 independent chains per lane, 8 waves per SIMD, in-kernel shader clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                           \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

#define OPS(X)                                                                \
    X(0, "v_lshrrev_b64", "v_lshrrev_b64 %0, 27, %0")                         \
    X(1, "v_lshlrev_b64", "v_lshlrev_b64 %0, 5, %0")                          \
    X(2, "v_lshl_add_u64", "v_lshl_add_u64 %0, %0, 5, %1")                    \
    X(3, "v_pk_mov_b32", "v_pk_mov_b32 %0, %0, %1 op_sel:[0,1]")              \
    X(4, "v_mov_b64", "v_mov_b64 %0, %1")

constexpr int NOPS = 5;

template <int OP>
__global__ __launch_bounds__(256) void k_valu(uint64_t* out, unsigned long long* clk, uint32_t iters, uint32_t seed) {
    uint64_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = (uint64_t)(seed * (threadIdx.x + 1)) * 0x9e3779b97f4a7c15ull + i;
    const uint64_t b = seed ^ 0x5bd1e9955bd1e995ull;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
#define X(N, NAME, ASM) \
    if constexpr (OP == N) asm volatile(ASM : "+v"(a[i]) : "v"(b));
                OPS(X)
#undef X
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int OP>
static void run(int blocks, uint32_t iters, uint64_t* d_out, unsigned long long* d_clk, int cus, const char* name,
                bool first) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, 64u, 1u);  // warm
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, d_out, d_clk, iters, 1u);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 16);
    CHK(hipMemcpy(h, d_clk, (size_t)blocks * 16, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (int i = 0; i < blocks; i++) { cyc += (double)h[2 * i]; rt += (double)h[2 * i + 1]; }
    free(h);
    const double clock_hz = cyc / (rt / 100e6);
    const double wave_insts = (double)blocks * 4.0 * iters * 16.0 * 8.0;
    const double simd_cycles = (ms * 1e-3) * clock_hz * cus * 4.0;
    printf("%s{\"op\": \"%s\", \"ms\": %.3f, \"clock_mhz\": %.0f, \"simd_cycles_per_wave_inst\": %.3f}",
           first ? "" : ",\n  ", name, ms, clock_hz / 1e6, simd_cycles / wave_insts);
}

int main(int argc, char** argv) {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8 * (argc > 1 ? atoi(argv[1]) : 2);
    const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 2000;
    uint64_t* d_out;
    unsigned long long* d_clk;
    CHK(hipMalloc(&d_out, (size_t)blocks * 256 * 8));
    CHK(hipMalloc(&d_clk, (size_t)blocks * 16));
    printf("{\"gcnArch\": \"%s\", \"cus\": %d, \"results\": [\n  ", p.gcnArchName, cus);
#define X(N, NAME, ASM) run<N>(blocks, iters, d_out, d_clk, cus, NAME, N == 0);
    OPS(X)
#undef X
    printf("]}\n");
    CHK(hipFree(d_out));
    CHK(hipFree(d_clk));
    return 0;
}
