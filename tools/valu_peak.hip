// valu_peak.hip -- measures the gfx950 integer VALU issue rate for the instruction classes the SHA-1 loop uses
// (v_alignbit_b32, v_add3_u32, v_bitop3_b32, v_xor_b32), to pin the roofline denominator of bench.py on hardware.
// Each lane runs 8 independent dependency chains (ILP) x enough waves for full occupancy; the reported figure is
// lane-ops / s and lane-ops / clock / CU at the measured wall time.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHK(x)                                                                  \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

template <int OP>
__global__ __launch_bounds__(256) void k_valu(uint32_t* out, uint32_t iters, uint32_t seed) {
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = seed * (threadIdx.x + 1) + i * 0x9e3779b9u;
    const uint32_t b = seed ^ 0x5bd1e995u, c = seed + 0x12345678u;
    for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if constexpr (OP == 0) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(a[i]));
                else if constexpr (OP == 1) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                else if constexpr (OP == 2) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
                else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            }
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int OP>
static double run(int blocks, uint32_t iters, uint32_t* d_out, double* ms_out) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, d_out, 16u, 1u);  // warm
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_valu<OP>, dim3(blocks), dim3(256), 0, 0, d_out, iters, 1u);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    *ms_out = ms;
    const double lane_ops = (double)blocks * 256.0 * iters * 16.0 * 8.0;
    return lane_ops / (ms * 1e-3);
}

int main(int argc, char** argv) {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate * 1e3;  // Hz (max engine clock)
    const int blocks = cus * 8 * (argc > 1 ? atoi(argv[1]) : 4);  // 8 waves/SIMD x rounds
    const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 4000;
    uint32_t* d_out;
    CHK(hipMalloc(&d_out, (size_t)blocks * 256 * 4));
    const char* names[4] = {"v_alignbit_b32", "v_add3_u32", "v_bitop3_b32", "v_xor_b32"};
    printf("{\"device\": \"%s\", \"gcnArch\": \"%s\", \"cus\": %d, \"max_clock_mhz\": %.0f, \"results\": [", p.name,
           p.gcnArchName, cus, clk / 1e6);
    for (int op = 0; op < 4; op++) {
        double ms = 0, r = 0;
        if (op == 0) r = run<0>(blocks, iters, d_out, &ms);
        if (op == 1) r = run<1>(blocks, iters, d_out, &ms);
        if (op == 2) r = run<2>(blocks, iters, d_out, &ms);
        if (op == 3) r = run<3>(blocks, iters, d_out, &ms);
        printf("%s{\"op\": \"%s\", \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"lane_ops_per_clk_per_cu_at_max_clock\": %.2f}",
               op ? ", " : "", names[op], ms, r, r / clk / cus);
    }
    printf("]}\n");
    CHK(hipFree(d_out));
    return 0;
}
