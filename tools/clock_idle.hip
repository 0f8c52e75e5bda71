// clock_idle.hip -- the shader clock a lone wave sees, after the GPU has idled for a given time (VERDICT r3 item 2:
// is a one-key server call slow because the chip runs its single PBKDF2 wave at a low clock?).
//
// One kernel = W waves (one per SIMD at most) each running a dependent chain of full-rate VALU ops for ~6 ms, the
// length of one PBKDF2 chain.  Lane 0 of every wave stamps s_memtime (shader clock) and s_memrealtime (100 MHz
// reference) at start and end; clock = d(memtime) / d(memrealtime) x 100 MHz.  The host sleeps `gap` seconds before
// each launch (the idle time between two server requests) and prints one JSON line per (gap, waves, rep).
//   tools/bin/clock_idle [reps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>

#define CHK(x)                                                                         \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ __launch_bounds__(64) void k_chain(unsigned long long* stamps, unsigned iters, unsigned seed,
                                              unsigned* sink, unsigned lanes) {
    if (threadIdx.x >= lanes) return;  // partial EXEC: only `lanes` lanes of the wave run the chain
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned a = seed + threadIdx.x, b = a * 7u + 1u;
    for (unsigned i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 32; k++) {  // 64 dependent full-rate ops per unrolled step
            a = a ^ b;
            b = b + a;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        stamps[4 * blockIdx.x + 0] = t1 - t0;
        stamps[4 * blockIdx.x + 1] = r1 - r0;
    }
    if (a == 0x12345678u && b == 0x9abcdef0u) sink[0] = a;  // keep the chain alive
}

static double now_s() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const int waves[] = {1, 8, 1024};
    const double gaps[] = {0.0, 0.01, 0.05, 0.2, 0.5, 1.0, 2.0};
    unsigned long long* d_st;
    unsigned* d_sink;
    CHK(hipMalloc(&d_st, 4 * 1024 * sizeof(unsigned long long)));
    CHK(hipMalloc(&d_sink, 4));
    unsigned long long h[4 * 1024];
    // calibrate: iterations for ~6 ms at a warm clock (dependent full-rate op: ~4-8 cycles each at 1 wave per SIMD)
    unsigned iters = 1000;
    for (int c = 0; c < 6; c++) {
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, d_st, iters, 1u, d_sink, 64u);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(h, d_st, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        const double ms = h[1] / 1e5;
        iters = (unsigned)(iters * 6.0 / (ms > 0.01 ? ms : 0.01));
    }
    fprintf(stderr, "iters %u\n", iters);
    const unsigned lane_modes[] = {64, 16, 2, 1};
    const bool lanes_only = getenv("CLOCK_LANES") != nullptr;  // only the partial-EXEC sweep (1 and 8 waves, no gap)
    for (double gap : gaps)
        for (int w : waves)
            for (unsigned lanes : lane_modes)
            for (int r = 0; r < reps; r++) {
                if (lanes_only ? (gap > 0 || w > 8) : lanes != 64) continue;
                if (gap > 0) usleep((useconds_t)(gap * 1e6));
                const double t0 = now_s();
                hipLaunchKernelGGL(k_chain, dim3(w), dim3(64), 0, 0, d_st, iters, (unsigned)r, d_sink, lanes);
                CHK(hipDeviceSynchronize());
                const double wall = now_s() - t0;
                CHK(hipMemcpy(h, d_st, 4 * w * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                double mhz_min = 1e9, mhz_max = 0, mhz_sum = 0, ms_max = 0;
                for (int i = 0; i < w; i++) {
                    const double mhz = (double)h[4 * i] / (double)h[4 * i + 1] * 100.0;
                    mhz_min = mhz < mhz_min ? mhz : mhz_min;
                    mhz_max = mhz > mhz_max ? mhz : mhz_max;
                    mhz_sum += mhz;
                    const double ms = h[4 * i + 1] / 1e5;
                    ms_max = ms > ms_max ? ms : ms_max;
                }
                printf("{\"gap_s\": %.3f, \"waves\": %d, \"lanes\": %u, \"rep\": %d, \"clock_mhz_mean\": %.1f, \"clock_mhz_min\": %.1f, "
                       "\"clock_mhz_max\": %.1f, \"kernel_ms\": %.3f, \"wall_ms\": %.3f}\n",
                       gap, w, lanes, r, mhz_sum / w, mhz_min, mhz_max, ms_max, wall * 1e3);
                fflush(stdout);
            }
    return 0;
}
