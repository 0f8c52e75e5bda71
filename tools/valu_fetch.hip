// valu_fetch.hip -- does straight-line code length change gfx950 VALU issue cost?  (design exploration)
// Same instruction mix in a short loop body (64 instructions) vs a long unrolled body (1024 instructions,
// 4-8 KB of code), for VOP2 xor (4 B), VOP3 bitop3 (8 B) and VOP3 alignbit (8 B).  8 chains per wave,
// 8 waves per SIMD.  Reports SIMD cycles per wave64 instruction (in-kernel clock).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                       \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

#define X2(S) S S
#define X4(S) X2(X2(S))
#define X16(S) X4(X4(S))
#define X128(S) X16(X4(X2(S)))

#define XOR8 "v_xor_b32 v40, v40, v49\n v_xor_b32 v41, v41, v50\n v_xor_b32 v42, v42, v49\n v_xor_b32 v43, v43, v50\n v_xor_b32 v44, v44, v49\n v_xor_b32 v45, v45, v50\n v_xor_b32 v46, v46, v49\n v_xor_b32 v47, v47, v50\n"
#define BOP8 "v_bitop3_b32 v40, v40, v49, v50 bitop3:0x96\n v_bitop3_b32 v41, v41, v50, v51 bitop3:0x96\n v_bitop3_b32 v42, v42, v49, v51 bitop3:0x96\n v_bitop3_b32 v43, v43, v52, v49 bitop3:0x96\n v_bitop3_b32 v44, v44, v49, v50 bitop3:0x96\n v_bitop3_b32 v45, v45, v50, v51 bitop3:0x96\n v_bitop3_b32 v46, v46, v49, v51 bitop3:0x96\n v_bitop3_b32 v47, v47, v52, v49 bitop3:0x96\n"
#define ALB8 "v_alignbit_b32 v40, v40, v40, 27\n v_alignbit_b32 v41, v41, v41, 27\n v_alignbit_b32 v42, v42, v42, 27\n v_alignbit_b32 v43, v43, v43, 27\n v_alignbit_b32 v44, v44, v44, 27\n v_alignbit_b32 v45, v45, v45, 27\n v_alignbit_b32 v46, v46, v46, 27\n v_alignbit_b32 v47, v47, v47, 27\n"
#define ADD8 "v_add_u32 v40, v40, v49\n v_add_u32 v41, v41, v50\n v_add_u32 v42, v42, v49\n v_add_u32 v43, v43, v50\n v_add_u32 v44, v44, v49\n v_add_u32 v45, v45, v50\n v_add_u32 v46, v46, v49\n v_add_u32 v47, v47, v50\n"
#define MIX8 "v_alignbit_b32 v40, v40, v40, 27\n v_xor_b32 v41, v41, v50\n v_bitop3_b32 v42, v42, v49, v51 bitop3:0x96\n v_add_u32 v43, v43, v50\n v_add3_u32 v44, v44, v49, v50\n v_xor_b32 v45, v45, v50\n v_alignbit_b32 v46, v46, v46, 2\n v_bitop3_b32 v47, v47, v52, v49 bitop3:0x96\n"
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47"

template <int T>
__global__ __launch_bounds__(256) void k(unsigned long long* clk, uint32_t iters) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("v_mov_b32 v49, 3\n v_mov_b32 v50, 5\n v_mov_b32 v51, 7\n v_mov_b32 v52, 9" ::: "v49", "v50", "v51", "v52");
    for (uint32_t it = 0; it < iters; it++) {
        if constexpr (T == 0) asm volatile(X4(X2(XOR8)) ::: CLOB);   // short: 64 insts
        if constexpr (T == 1) asm volatile(X128(XOR8) ::: CLOB);     // long: 1024 insts
        if constexpr (T == 2) asm volatile(X4(X2(BOP8)) ::: CLOB);
        if constexpr (T == 3) asm volatile(X128(BOP8) ::: CLOB);
        if constexpr (T == 4) asm volatile(X4(X2(ALB8)) ::: CLOB);
        if constexpr (T == 5) asm volatile(X128(ALB8) ::: CLOB);
        if constexpr (T == 6) asm volatile(X4(X2(ADD8)) ::: CLOB);
        if constexpr (T == 7) asm volatile(X128(ADD8) ::: CLOB);
        if constexpr (T == 8) asm volatile(X4(X2(MIX8)) ::: CLOB);
        if constexpr (T == 9) asm volatile(X128(MIX8) ::: CLOB);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

static const char* NAMES[] = {"xor short", "xor long", "bitop3 short", "bitop3 long", "alignbit short",
                              "alignbit long", "add_u32 short", "add_u32 long", "mix short", "mix long"};
static const int INSTS[] = {64, 1024, 64, 1024, 64, 1024, 64, 1024, 64, 1024};

template <int T>
static void run(int cus, int wps, unsigned long long* d_clk, bool first) {
    const int blocks = cus * wps;
    const uint32_t iters = INSTS[T] == 64 ? 16000 : 1000;
    hipLaunchKernelGGL(k<T>, dim3(blocks), dim3(256), 0, 0, d_clk, 4u);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k<T>, dim3(blocks), dim3(256), 0, 0, d_clk, iters);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 16);
    CHK(hipMemcpy(h, d_clk, (size_t)blocks * 16, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0;
    for (int i = 0; i < blocks; i++) { cyc += (double)h[2 * i]; rt += (double)h[2 * i + 1]; }
    free(h);
    const double clock_hz = cyc / (rt / 100e6);
    const double wave_insts = (double)blocks * 4 * iters * INSTS[T];
    printf("%s{\"test\": \"%s\", \"waves_per_simd\": %d, \"clock_mhz\": %.0f, \"simd_cycles_per_wave_inst\": %.3f}",
           first ? "" : ",\n  ", NAMES[T], wps, clock_hz / 1e6, (ms * 1e-3) * clock_hz * cus * 4 / wave_insts);
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    unsigned long long* d_clk;
    CHK(hipMalloc(&d_clk, (size_t)p.multiProcessorCount * 8 * 16));
    printf("{\"results\": [\n  ");
    bool f = true;
    for (int w : {8, 2}) {
        run<0>(p.multiProcessorCount, w, d_clk, f); f = false;
        run<1>(p.multiProcessorCount, w, d_clk, f);
        run<2>(p.multiProcessorCount, w, d_clk, f);
        run<3>(p.multiProcessorCount, w, d_clk, f);
        run<4>(p.multiProcessorCount, w, d_clk, f);
        run<5>(p.multiProcessorCount, w, d_clk, f);
        run<6>(p.multiProcessorCount, w, d_clk, f);
        run<7>(p.multiProcessorCount, w, d_clk, f);
        run<8>(p.multiProcessorCount, w, d_clk, f);
        run<9>(p.multiProcessorCount, w, d_clk, f);
    }
    printf("]}\n");
    return 0;
}
