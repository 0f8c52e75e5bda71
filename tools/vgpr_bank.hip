// vgpr_bank.hip -- does the VGPR bank of a VALU's source operands change its issue cost on gfx950?
//
// Each pattern is one instruction with fixed source VGPRs and eight rotating destinations (no RAW dependences
// between instructions), 64 per loop trip, all in one inline-asm block with explicit registers.  The sources are
// either in one bank (v16, v20, v24: equal mod 4) or in distinct banks (v16, v17, v18).  Run with one wave per SIMD
// (a lone wave's issue) and with 8 waves per SIMD (the SIMD's issue rate).  The clock is s_memtime, so results are
// s_memtime ticks per wave64 instruction: per-wave ticks / instructions for a lone wave, / 8 for eight waves (the
// tick is not the shader clock here: compare patterns within one run; round 5 measured xor 0.86, add3 1.82).
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

#define R8(I)                                                                                           \
    I("v8") I("v9") I("v10") I("v11") I("v12") I("v13") I("v14") I("v15")
#define R64(I) R8(I) R8(I) R8(I) R8(I) R8(I) R8(I) R8(I) R8(I)

#define ADD3_SAME(d) "v_add3_u32 " d ", v16, v20, v24\n\t"
#define ADD3_DIFF(d) "v_add3_u32 " d ", v16, v17, v18\n\t"
#define ADD3_TWO(d) "v_add3_u32 " d ", v16, v20, v17\n\t"
#define BOP3_SAME(d) "v_bitop3_b32 " d ", v16, v20, v24 bitop3:0x96\n\t"
#define BOP3_DIFF(d) "v_bitop3_b32 " d ", v16, v17, v18 bitop3:0x96\n\t"
#define XOR_SAME(d) "v_xor_b32 " d ", v16, v20\n\t"
#define XOR_DIFF(d) "v_xor_b32 " d ", v16, v17\n\t"
#define ALB_ROT(d) "v_alignbit_b32 " d ", v16, v16, 27\n\t"
#define ALB_SAME(d) "v_alignbit_b32 " d ", v16, v20, 27\n\t"
#define ALB_DIFF(d) "v_alignbit_b32 " d ", v16, v17, 27\n\t"
#define ADD_SAME(d) "v_add_u32 " d ", v16, v20\n\t"
#define ADD_DIFF(d) "v_add_u32 " d ", v16, v17\n\t"
#define BOP3_TWO(d) "v_bitop3_b32 " d ", v16, v20, v17 bitop3:0x96\n\t"
#define BOP3_123(d) "v_bitop3_b32 " d ", v17, v18, v19 bitop3:0x96\n\t"
#define BOP3_REP(d) "v_bitop3_b32 " d ", v16, v16, v17 bitop3:0x96\n\t"
#define MIX_DIFF(d) "v_add3_u32 " d ", v16, v17, v18\n\tv_bitop3_b32 " d ", v17, v18, v19 bitop3:0x96\n\t"
#define MIX_TWO(d) "v_add3_u32 " d ", v16, v17, v18\n\tv_bitop3_b32 " d ", v16, v20, v17 bitop3:0x96\n\t"
#define MIX_SAME(d) "v_add3_u32 " d ", v16, v17, v18\n\tv_bitop3_b32 " d ", v16, v20, v24 bitop3:0x96\n\t"

#define PATTERNS(X)                                      \
    X(0, "v_add3_u32 one bank", ADD3_SAME)               \
    X(1, "v_add3_u32 three banks", ADD3_DIFF)            \
    X(2, "v_add3_u32 two in one bank", ADD3_TWO)         \
    X(3, "v_bitop3_b32 one bank", BOP3_SAME)             \
    X(4, "v_bitop3_b32 three banks", BOP3_DIFF)          \
    X(5, "v_xor_b32 one bank", XOR_SAME)                 \
    X(6, "v_xor_b32 two banks", XOR_DIFF)                \
    X(7, "v_alignbit_b32 rotate (x, x)", ALB_ROT)        \
    X(8, "v_alignbit_b32 one bank", ALB_SAME)            \
    X(9, "v_alignbit_b32 two banks", ALB_DIFF)           \
    X(10, "v_add_u32 one bank", ADD_SAME)                \
    X(11, "v_add_u32 two banks", ADD_DIFF)                \
    X(12, "v_bitop3_b32 two in one bank", BOP3_TWO)      \
    X(13, "v_bitop3_b32 banks 1, 2, 3", BOP3_123)        \
    X(14, "v_bitop3_b32 (x, x, y)", BOP3_REP)            \
    X(15, "add3 + bitop3 three banks", MIX_DIFF)         \
    X(16, "add3 + bitop3 two in one bank", MIX_TWO)      \
    X(17, "add3 + bitop3 one bank", MIX_SAME)

constexpr int NPAT = 18;
static const int kInstPerDest[NPAT] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2};

template <int P>
__device__ __forceinline__ void body(uint32_t& x, uint32_t iters);

#define DEF(ID, NAME, M)                                                                                     \
    template <>                                                                                              \
    __device__ __forceinline__ void body<ID>(uint32_t & x, uint32_t iters) {                                 \
        __asm__ volatile(                                                                                    \
            "v_mov_b32 v16, %0\n\tv_add_u32 v17, 1, %0\n\tv_add_u32 v18, 2, %0\n\tv_add_u32 v20, 3, %0\n\t"  \
            "v_add_u32 v24, 4, %0\n\tv_add_u32 v19, 5, %0\n\ts_mov_b32 s20, %1\n"                                                   \
            "L_bank_loop_%=:\n\t" R64(M) "s_sub_u32 s20, s20, 1\n\ts_cmp_lg_u32 s20, 0\n\t"                  \
            "s_cbranch_scc1 L_bank_loop_%=\n\t"                                                              \
            "v_xor_b32 %0, v8, v9\n\tv_xor_b32 %0, %0, v10\n\tv_xor_b32 %0, %0, v11\n\tv_xor_b32 %0, %0, v12\n\t" \
            "v_xor_b32 %0, %0, v13\n\tv_xor_b32 %0, %0, v14\n\tv_xor_b32 %0, %0, v15"                       \
            : "+v"(x)                                                                                        \
            : "s"(iters)                                                                                     \
            : "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v24", "s20", \
              "scc");                                                                                        \
    }
PATTERNS(DEF)

template <int P>
__global__ __launch_bounds__(256) void k_bank(uint32_t* out, unsigned long long* clk, uint32_t iters) {
    uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    body<P>(x, iters);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) clk[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

typedef void (*KFn)(uint32_t*, unsigned long long*, uint32_t);
#define PTR(ID, NAME, M) k_bank<ID>,
#define NAMES(ID, NAME, M) NAME,
static const KFn kFns[NPAT] = {PATTERNS(PTR)};
static const char* kNames[NPAT] = {PATTERNS(NAMES)};

int main(int argc, char** argv) {
    const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 4000;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int maxblocks = cus * 8;
    uint32_t* out;
    unsigned long long* clk;
    CHK(hipMalloc(&out, (size_t)maxblocks * 256 * 4));
    CHK(hipMalloc(&clk, (size_t)maxblocks * 4 * 8));
    unsigned long long* h = (unsigned long long*)malloc((size_t)maxblocks * 4 * 8);
    printf("{\"cus\": %d, \"iters\": %u, \"insts_per_wave\": %llu, \"results\": [\n", cus, iters,
           (unsigned long long)iters * 64);
    for (int p = 0; p < NPAT; p++) {
        for (int wps = 1; wps <= 8; wps *= 8) {
            const int blocks = cus * wps;  // 4 waves per block, one per SIMD
            hipLaunchKernelGGL(kFns[p], dim3(blocks), dim3(256), 0, 0, out, clk, 16u);
            CHK(hipDeviceSynchronize());
            hipLaunchKernelGGL(kFns[p], dim3(blocks), dim3(256), 0, 0, out, clk, iters);
            CHK(hipDeviceSynchronize());
            CHK(hipMemcpy(h, clk, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost));
            double sum = 0;
            for (int i = 0; i < blocks * 4; i++) sum += (double)h[i];
            const double per_wave = sum / (blocks * 4) / ((double)iters * 64 * kInstPerDest[p]);
            printf("  {\"pattern\": \"%s\", \"waves_per_simd\": %d, \"ticks_per_inst_per_wave\": %.3f, "
                   "\"simd_ticks_per_inst\": %.3f}%s\n",
                   kNames[p], wps, per_wave, per_wave / wps, (p == NPAT - 1 && wps == 8) ? "" : ",");
        }
    }
    printf("]}\n");
    return 0;
}
