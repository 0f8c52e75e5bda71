// valu_peak.hip -- gfx950 integer VALU issue costs for the instruction classes a SHA-1 loop can use.
//
// Each lane runs 8 independent dependency chains of one instruction (or a fixed pair), with 8 waves per SIMD
// (full occupancy), so latency is hidden and the SIMD's issue rate is what is measured.  The in-kernel clock is
// taken from s_memtime / s_memrealtime (100 MHz), so the result is reported as SIMD cycles per wave64
// instruction independent of DVFS, plus lane-ops/s at the observed clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHK(x)                                                                           \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

// one instruction applied to chain register a (b, c are loop-invariant VGPRs)
#define OPS(X)                                                                                   \
    X(0, "v_alignbit_b32", "v_alignbit_b32 %0, %0, %0, 27")                                      \
    X(1, "v_add3_u32", "v_add3_u32 %0, %0, %1, %2")                                              \
    X(2, "v_bitop3_b32", "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")                              \
    X(3, "v_xor_b32", "v_xor_b32 %0, %0, %1")                                                    \
    X(4, "v_add_u32", "v_add_u32 %0, %0, %1")                                                    \
    X(5, "v_lshlrev_b32", "v_lshlrev_b32 %0, 5, %0")                                             \
    X(6, "v_lshl_add_u32", "v_lshl_add_u32 %0, %0, 5, %1")                                       \
    X(7, "v_lshl_or_b32", "v_lshl_or_b32 %0, %0, 5, %1")                                         \
    X(8, "v_xad_u32", "v_xad_u32 %0, %0, %1, %2")                                                \
    X(9, "v_or3_b32", "v_or3_b32 %0, %0, %1, %2")                                                \
    X(10, "v_bfi_b32", "v_bfi_b32 %0, %0, %1, %2")                                               \
    X(11, "v_perm_b32", "v_perm_b32 %0, %0, %1, %2")                                             \
    X(12, "v_alignbyte_b32", "v_alignbyte_b32 %0, %0, %1, 1")                                    \
    X(13, "v_add_lshl_u32", "v_add_lshl_u32 %0, %0, %1, 1")                                      \
    X(14, "v_and_or_b32", "v_and_or_b32 %0, %0, %1, %2")                                         \
    X(15, "v_mad_u32_u24", "v_mad_u32_u24 %0, %0, %1, %2")                                       \
    X(16, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1")                                             \
    X(17, "v_lshrrev_b32", "v_lshrrev_b32 %0, 27, %0")                                           \
    X(18, "v_add_co_u32", "v_add_co_u32 %0, vcc, %0, %1")                                        \
    X(19, "v_sub_u32", "v_sub_u32 %0, %0, %1")                                                   \
    X(20, "alignbit+xor", "v_alignbit_b32 %0, %0, %0, 27\n\tv_xor_b32 %0, %0, %1")               \
    X(21, "add3+bitop3", "v_add3_u32 %0, %0, %1, %2\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0x96") \
    X(22, "alignbit+add_u32", "v_alignbit_b32 %0, %0, %0, 27\n\tv_add_u32 %0, %0, %1")           \
    X(23, "v_add3_u32 (b=c)", "v_add3_u32 %0, %0, %1, %1")                                       \
    X(24, "v_add3_u32 (sgpr)", "v_add3_u32 %0, %0, %1, s0")

constexpr int NOPS = 25;
static const int kInstPerStep[NOPS] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1};

template <int OP>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, unsigned long long* clk, uint32_t iters, uint32_t seed) {
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = seed * (threadIdx.x + 1) + i * 0x9e3779b9u;
    const uint32_t b = seed ^ 0x5bd1e995u, c = seed + 0x12345678u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
#define X(N, NAME, ASM) \
    if constexpr (OP == N) asm volatile(ASM : "+v"(a[i]) : "v"(b), "v"(c) : "vcc");
                OPS(X)
#undef X
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int OP>
static void run(int blocks, uint32_t iters, uint32_t* d_out, unsigned long long* d_clk, int cus, const char* name,
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
    const double clock_hz = cyc / (rt / 100e6);  // shader clock seen inside the kernel
    const double wave_insts = (double)blocks * 4.0 * iters * 16.0 * 8.0 * kInstPerStep[OP];  // 4 waves/block
    const double simd_cycles = (ms * 1e-3) * clock_hz * cus * 4.0;
    printf("%s{\"op\": \"%s\", \"ms\": %.3f, \"clock_mhz\": %.0f, \"simd_cycles_per_wave_inst\": %.3f, "
           "\"lane_ops_per_s\": %.4e}",
           first ? "" : ",\n  ", name, ms, clock_hz / 1e6, simd_cycles / wave_insts,
           wave_insts * 64.0 / (ms * 1e-3));
}

int main(int argc, char** argv) {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8 * (argc > 1 ? atoi(argv[1]) : 2);
    const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 2000;
    uint32_t* d_out;
    unsigned long long* d_clk;
    CHK(hipMalloc(&d_out, (size_t)blocks * 256 * 4));
    CHK(hipMalloc(&d_clk, (size_t)blocks * 16));
    printf("{\"gcnArch\": \"%s\", \"cus\": %d, \"max_clock_mhz\": %.0f, \"results\": [\n  ", p.gcnArchName, cus,
           p.clockRate / 1e3);
#define X(N, NAME, ASM) run<N>(blocks, iters, d_out, d_clk, cus, NAME, N == 0);
    OPS(X)
#undef X
    printf("]}\n");
    CHK(hipFree(d_out));
    CHK(hipFree(d_clk));
    return 0;
}
