// pbkdf2_gfx950.hip -- the product PBKDF2 kernel.  Compiled device-only to gfx950 assembly, passed through the
// VALU issue pass (gen/issue_pass.py, the Makefile's ISSUE_RULE), assembled to a code object and embedded in
// libdwpa22000.so (see Makefile); launched with hipModuleLaunchKernel (pbkdf2_module.cpp).
//
// These multi-wave kernels take the j = 2 schedule forms from round 73 on (crypto_dev.hpp sched_w: 1,116 VALU per
// loop iteration, 64 VGPRs, no spill): with the issue pass's list scheduler they measured -0.9 % at 8 waves per SIMD
// and -0.3 % at 6 against j <= 1 (profiles/r05/sched_identities/).  The lone-wave kernels in kernels.hip keep
// j <= 1, which is faster there (one-key call 8.17 against 8.29 ms).
#ifndef DWPA_SCHED_WIDE
#define DWPA_SCHED_WIDE 2
#endif
#ifndef DWPA_SCHED_J2_MIN
#define DWPA_SCHED_J2_MIN 73
#endif
#include <hip/hip_runtime.h>

#include "pbkdf2_dev.hpp"

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_gfx950(const uint32_t* __restrict__ mid, uint32_t cap,
                                                                  uint32_t base, uint32_t count,
                                                                  const uint32_t* __restrict__ counter,
                                                                  const uint32_t* __restrict__ salt, uint32_t nsalt,
                                                                  uint32_t* __restrict__ pmk) {
    dwpa::pbkdf2_body(mid, cap, base, count, counter, salt, nsalt, pmk);
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_gfx950_ms(const uint32_t* __restrict__ mid, uint32_t cap,
                                                                     uint32_t count,
                                                                     const uint32_t* __restrict__ pool,
                                                                     const uint32_t* __restrict__ sref,
                                                                     uint32_t* __restrict__ pmk) {
    dwpa::pbkdf2_body_ms(mid, cap, count, pool, sref, pmk);
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_gfx950_mg(const uint32_t* __restrict__ mid, uint32_t cap,
                                                                     const uint32_t* __restrict__ counter,
                                                                     uint32_t ngroups,
                                                                     const uint32_t* __restrict__ salt,
                                                                     const uint32_t* __restrict__ gsalt,
                                                                     uint32_t* __restrict__ pmk, uint32_t pstride) {
    dwpa::pbkdf2_body_mg(mid, cap, counter, ngroups, salt, gsalt, pmk, pstride);
}

// Progress-ordered priority variants (pbkdf2_dev.hpp, PRIO): selected per launch by pbkdf2_module.cpp.
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_gfx950_p(const uint32_t* __restrict__ mid, uint32_t cap,
                                                                    uint32_t base, uint32_t count,
                                                                    const uint32_t* __restrict__ counter,
                                                                    const uint32_t* __restrict__ salt, uint32_t nsalt,
                                                                    uint32_t* __restrict__ pmk) {
    dwpa::pbkdf2_body<true>(mid, cap, base, count, counter, salt, nsalt, pmk);
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_gfx950_ms_p(
    const uint32_t* __restrict__ mid, uint32_t cap, uint32_t count, const uint32_t* __restrict__ pool,
    const uint32_t* __restrict__ sref, uint32_t* __restrict__ pmk) {
    dwpa::pbkdf2_body_ms<true>(mid, cap, count, pool, sref, pmk);
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_gfx950_mg_p(
    const uint32_t* __restrict__ mid, uint32_t cap, const uint32_t* __restrict__ counter, uint32_t ngroups,
    const uint32_t* __restrict__ salt, const uint32_t* __restrict__ gsalt, uint32_t* __restrict__ pmk,
    uint32_t pstride) {
    dwpa::pbkdf2_body_mg<true>(mid, cap, counter, ngroups, salt, gsalt, pmk, pstride);
}

// Work-queue variant of k_pbkdf2_gfx950 (pbkdf2_dev.hpp pbkdf2_body_queue): XCD-balanced multi-round launches.
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_gfx950_q(
    const uint32_t* __restrict__ mid, uint32_t cap, uint32_t base, uint32_t count, const uint32_t* __restrict__ counter,
    const uint32_t* __restrict__ salt, uint32_t nsalt, uint32_t* __restrict__ pmk, uint32_t* __restrict__ work) {
    dwpa::pbkdf2_body_queue(mid, cap, base, count, counter, salt, nsalt, pmk, work);
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_pbkdf2_gfx950_mg_q(
    const uint32_t* __restrict__ mid, uint32_t cap, const uint32_t* __restrict__ counter, uint32_t ngroups,
    const uint32_t* __restrict__ salt, const uint32_t* __restrict__ gsalt, uint32_t* __restrict__ pmk,
    uint32_t pstride, uint32_t* __restrict__ work) {
    dwpa::pbkdf2_body_mg_queue(mid, cap, counter, ngroups, salt, gsalt, pmk, pstride, work);
}
