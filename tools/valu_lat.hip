// valu_lat.hip -- gfx950 VALU issue details that bound a SHA-1 loop beyond per-instruction cost:
//   (1) VGPR bank conflicts of 3-source VOP3 instructions (explicit physical registers, bank = reg % 4),
//   (2) dependent-issue latency: throughput with 1/2/4/8 independent chains per wave at 8 and 4 waves/SIMD.
// Reports SIMD cycles per wave64 instruction from the in-kernel clock (s_memtime / s_memrealtime).
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

#define R8(S) S S S S S S S S
#define R64(S) R8(R8(S))

// bank-conflict tests on fixed registers v40..v63 (all 8 instructions independent per group)
template <int T>
__global__ __launch_bounds__(256) void k_bank(unsigned long long* clk, uint32_t iters) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("v_mov_b32 v40, 1\n v_mov_b32 v41, 2\n v_mov_b32 v42, 3\n v_mov_b32 v43, 4\n v_mov_b32 v44, 5\n"
                 "v_mov_b32 v45, 6\n v_mov_b32 v46, 7\n v_mov_b32 v47, 8\n v_mov_b32 v48, 9\n v_mov_b32 v49, 10\n"
                 "v_mov_b32 v50, 11\n v_mov_b32 v51, 12\n v_mov_b32 v52, 13\n v_mov_b32 v53, 14\n v_mov_b32 v54, 15\n"
                 "v_mov_b32 v55, 16\n v_mov_b32 v56, 17\n v_mov_b32 v57, 18\n v_mov_b32 v58, 19\n v_mov_b32 v59, 20\n"
                 "v_mov_b32 v60, 21\n v_mov_b32 v61, 22\n v_mov_b32 v62, 23\n v_mov_b32 v63, 24" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63");
    for (uint32_t it = 0; it < iters; it++) {
        if constexpr (T == 0)  // add3, sources in 3 different banks (48:0, 49:1, 50:2), dst chains v40..47
            asm volatile(R8("v_add3_u32 v40, v40, v49, v50\n v_add3_u32 v41, v41, v50, v51\n v_add3_u32 v42, v42, v49, v51\n v_add3_u32 v43, v43, v52, v49\n"
                            "v_add3_u32 v44, v44, v49, v50\n v_add3_u32 v45, v45, v50, v51\n v_add3_u32 v46, v46, v49, v51\n v_add3_u32 v47, v47, v52, v49\n")
                         ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
        if constexpr (T == 1)  // add3, all three sources in the same bank (v40:0, v48:0, v52:0 ...)
            asm volatile(R8("v_add3_u32 v40, v40, v48, v52\n v_add3_u32 v41, v41, v49, v53\n v_add3_u32 v42, v42, v50, v54\n v_add3_u32 v43, v43, v51, v55\n"
                            "v_add3_u32 v44, v44, v48, v52\n v_add3_u32 v45, v45, v49, v53\n v_add3_u32 v46, v46, v50, v54\n v_add3_u32 v47, v47, v51, v55\n")
                         ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
        if constexpr (T == 2)  // bitop3 different banks
            asm volatile(R8("v_bitop3_b32 v40, v40, v49, v50 bitop3:0x96\n v_bitop3_b32 v41, v41, v50, v51 bitop3:0x96\n v_bitop3_b32 v42, v42, v49, v51 bitop3:0x96\n v_bitop3_b32 v43, v43, v52, v49 bitop3:0x96\n"
                            "v_bitop3_b32 v44, v44, v49, v50 bitop3:0x96\n v_bitop3_b32 v45, v45, v50, v51 bitop3:0x96\n v_bitop3_b32 v46, v46, v49, v51 bitop3:0x96\n v_bitop3_b32 v47, v47, v52, v49 bitop3:0x96\n")
                         ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
        if constexpr (T == 3)  // bitop3 same bank
            asm volatile(R8("v_bitop3_b32 v40, v40, v48, v52 bitop3:0x96\n v_bitop3_b32 v41, v41, v49, v53 bitop3:0x96\n v_bitop3_b32 v42, v42, v50, v54 bitop3:0x96\n v_bitop3_b32 v43, v43, v51, v55 bitop3:0x96\n"
                            "v_bitop3_b32 v44, v44, v48, v52 bitop3:0x96\n v_bitop3_b32 v45, v45, v49, v53 bitop3:0x96\n v_bitop3_b32 v46, v46, v50, v54 bitop3:0x96\n v_bitop3_b32 v47, v47, v51, v55 bitop3:0x96\n")
                         ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
        if constexpr (T == 4)  // xor VOP2, same bank pairs
            asm volatile(R8("v_xor_b32 v40, v40, v48\n v_xor_b32 v41, v41, v49\n v_xor_b32 v42, v42, v50\n v_xor_b32 v43, v43, v51\n"
                            "v_xor_b32 v44, v44, v48\n v_xor_b32 v45, v45, v49\n v_xor_b32 v46, v46, v50\n v_xor_b32 v47, v47, v51\n")
                         ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
        if constexpr (T == 5)  // single dependent chain of v_add_u32 (latency)
            asm volatile(R64("v_add_u32 v40, v40, v49\n") ::: "v40");
        if constexpr (T == 6)  // two interleaved chains of v_add_u32
            asm volatile(R8(R8("v_add_u32 v40, v40, v49\n v_add_u32 v41, v41, v49\n")) ::: "v40", "v41");
        if constexpr (T == 7)  // four chains
            asm volatile(R8(R8("v_add_u32 v40, v40, v49\n v_add_u32 v41, v41, v49\n v_add_u32 v42, v42, v49\n v_add_u32 v43, v43, v49\n")) ::: "v40", "v41", "v42", "v43");
        if constexpr (T == 8)  // single dependent chain of v_alignbit_b32
            asm volatile(R64("v_alignbit_b32 v40, v40, v40, 27\n") ::: "v40");
        if constexpr (T == 9)  // two chains alignbit
            asm volatile(R8(R8("v_alignbit_b32 v40, v40, v40, 27\n v_alignbit_b32 v41, v41, v41, 27\n")) ::: "v40", "v41");
        if constexpr (T == 10)  // four chains alignbit
            asm volatile(R8(R8("v_alignbit_b32 v40, v40, v40, 27\n v_alignbit_b32 v41, v41, v41, 27\n v_alignbit_b32 v42, v42, v42, 27\n v_alignbit_b32 v43, v43, v43, 27\n")) ::: "v40", "v41", "v42", "v43");
        if constexpr (T == 11)  // single chain add3
            asm volatile(R64("v_add3_u32 v40, v40, v49, v50\n") ::: "v40");
        if constexpr (T == 12)  // alignbit feeding add feeding alignbit (mixed dependent chain, SHA-1 critical path shape)
            asm volatile(R8(R8("v_alignbit_b32 v41, v40, v40, 27\n v_add_u32 v40, v41, v49\n")) ::: "v40", "v41");
        if constexpr (T == 13)  // alignbit different src regs (a, b both used)
            asm volatile(R8("v_alignbit_b32 v40, v40, v49, 27\n v_alignbit_b32 v41, v41, v50, 27\n v_alignbit_b32 v42, v42, v49, 27\n v_alignbit_b32 v43, v43, v52, 27\n"
                            "v_alignbit_b32 v44, v44, v49, 27\n v_alignbit_b32 v45, v45, v50, 27\n v_alignbit_b32 v46, v46, v49, 27\n v_alignbit_b32 v47, v47, v52, 27\n")
                         ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

static const char* NAMES[] = {"add3 3 banks", "add3 same bank", "bitop3 3 banks", "bitop3 same bank", "xor same bank",
                              "add_u32 1 chain", "add_u32 2 chains", "add_u32 4 chains", "alignbit 1 chain",
                              "alignbit 2 chains", "alignbit 4 chains", "add3 1 chain", "alignbit->add chain",
                              "alignbit a!=b"};
static const int INSTS[] = {64, 64, 64, 64, 64, 64, 128, 256, 64, 128, 256, 64, 128, 64};

template <int T>
static void run(int cus, int waves_per_simd, uint32_t iters, unsigned long long* d_clk, bool first) {
    const int blocks = cus * waves_per_simd;  // 256-thread blocks = 4 waves, one per SIMD
    hipLaunchKernelGGL(k_bank<T>, dim3(blocks), dim3(256), 0, 0, d_clk, 8u);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_bank<T>, dim3(blocks), dim3(256), 0, 0, d_clk, iters);
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
           first ? "" : ",\n  ", NAMES[T], waves_per_simd, clock_hz / 1e6,
           (ms * 1e-3) * clock_hz * cus * 4 / wave_insts);
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    unsigned long long* d_clk;
    CHK(hipMalloc(&d_clk, (size_t)p.multiProcessorCount * 8 * 16));
    const int cus = p.multiProcessorCount;
    const uint32_t it = 20000;
    printf("{\"results\": [\n  ");
    bool f = true;
    for (int w : {8, 4, 2, 1}) {
        run<0>(cus, w, it, d_clk, f); f = false;
        run<1>(cus, w, it, d_clk, f);
        run<2>(cus, w, it, d_clk, f);
        run<3>(cus, w, it, d_clk, f);
        run<4>(cus, w, it, d_clk, f);
        run<5>(cus, w, it, d_clk, f);
        run<6>(cus, w, it, d_clk, f);
        run<7>(cus, w, it, d_clk, f);
        run<8>(cus, w, it, d_clk, f);
        run<9>(cus, w, it, d_clk, f);
        run<10>(cus, w, it, d_clk, f);
        run<11>(cus, w, it, d_clk, f);
        run<12>(cus, w, it, d_clk, f);
        run<13>(cus, w, it, d_clk, f);
    }
    printf("]}\n");
    return 0;
}
