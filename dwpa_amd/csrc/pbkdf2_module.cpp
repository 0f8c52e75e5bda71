// pbkdf2_module.cpp -- loads the issue-pass PBKDF2 code object (embedded at build time) on each device and launches
// it.  Launches with at most one wave per SIMD (small server checks: C1) take the hipcc-scheduled k_pbkdf2 instead:
// the issue pass's s_nops only pay when several waves share a SIMD, and a lone wave runs its stream 1.55x slower
// with them (profiles/r01/partial_round/).  DWPA_PBKDF2_PLAIN=1 runs the plain kernel everywhere (a deployment's
// fallback to the compiler's own schedule); DWPA_PBKDF2_ISSUE=1 the issue-pass kernel everywhere (the test suite's
// switch to run the small parity cases on it).  The results are identical.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "kernels.hpp"

namespace dwpa {

extern const uint8_t pbkdf2_gfx950_hsaco[];
extern const size_t pbkdf2_gfx950_hsaco_size;

struct Fns {
    hipFunction_t one, ms, mg;  // k_pbkdf2_gfx950 (one ESSID), _ms (per-slot salt), _mg (ESSID groups x batch)
    hipFunction_t one_p, ms_p, mg_p;  // the same with progress-ordered wave priority (pbkdf2_dev.hpp PRIO)
    hipFunction_t one_q, mg_q;        // the one-ESSID and group kernels as work queues (pbkdf2_dev.hpp *_queue)
    uint64_t level_lanes;       // lanes that give every SIMD of the device one wave: CUs x 4 SIMDs x 64
};
static std::mutex g_mod_mu;
static std::map<int, Fns> g_fn;

static bool env_flag(const char* name) {
    const char* e = getenv(name);
    return e && *e && *e != '0';
}
static bool use_plain() {
    static const bool plain = env_flag("DWPA_PBKDF2_PLAIN");
    return plain;
}
static bool force_issue() {
    static const bool issue = env_flag("DWPA_PBKDF2_ISSUE");
    return issue;
}
// Progress-ordered priority (pbkdf2_dev.hpp PRIO) for launches of at most one wave round (<= 8 waves per SIMD):
// there the waves of a SIMD otherwise finish one after another and the last runs alone.  Measured on MI355X
// (profiles/r02/prio/): 6 waves/SIMD 43.0 -> 40.7 ms, 4 waves 29.4 -> 26.5 ms, the C5 call 58.0 -> 54.6 ms; level on
// 16-round launches (C2 844.3 vs 844.3 ms), so multi-round launches keep the plain-priority kernel.
static bool use_prio(const Fns& fn, uint64_t pmks) { return 2 * pmks <= 8 * fn.level_lanes; }

// Workgroup size of the issue-pass grid launches (64 and 128 measured level or slower on partial rounds).
constexpr uint32_t WG = 256;

static hipError_t tuned_functions(Fns* fn) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_mod_mu);
    auto it = g_fn.find(dev);
    if (it != g_fn.end()) {
        *fn = it->second;
        return hipSuccess;
    }
    hipModule_t mod;
    if ((e = hipModuleLoadData(&mod, pbkdf2_gfx950_hsaco)) != hipSuccess) return e;
    if ((e = hipModuleGetFunction(&fn->one, mod, "k_pbkdf2_gfx950")) != hipSuccess) return e;
    if ((e = hipModuleGetFunction(&fn->ms, mod, "k_pbkdf2_gfx950_ms")) != hipSuccess) return e;
    if ((e = hipModuleGetFunction(&fn->mg, mod, "k_pbkdf2_gfx950_mg")) != hipSuccess) return e;
    if ((e = hipModuleGetFunction(&fn->one_p, mod, "k_pbkdf2_gfx950_p")) != hipSuccess) return e;
    if ((e = hipModuleGetFunction(&fn->ms_p, mod, "k_pbkdf2_gfx950_ms_p")) != hipSuccess) return e;
    if ((e = hipModuleGetFunction(&fn->mg_p, mod, "k_pbkdf2_gfx950_mg_p")) != hipSuccess) return e;
    if ((e = hipModuleGetFunction(&fn->one_q, mod, "k_pbkdf2_gfx950_q")) != hipSuccess) return e;
    if ((e = hipModuleGetFunction(&fn->mg_q, mod, "k_pbkdf2_gfx950_mg_q")) != hipSuccess) return e;
    int cus = 0;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    fn->level_lanes = (uint64_t)(cus > 0 ? cus : 256) * 4 * 64;
    g_fn[dev] = *fn;
    return hipSuccess;
}

// At most one wave per SIMD (both output blocks counted): latency-bound, the plain schedule is faster.
static bool lone_waves(const Fns& fn, uint64_t pmks) { return !force_issue() && 2 * pmks <= fn.level_lanes; }

// Multi-round scan launches (one ESSID, ESSID groups) run as work queues: one resident round of 8 waves per SIMD
// taking 64-lane items from a counter, so a faster XCD takes more of them.  Measured (profiles/r02/queue/): C2
// 4.898 -> 4.907 M PMK/s, C4 4.980 -> 4.996 M.
hipError_t launch_pbkdf2(const uint32_t* mid, uint32_t cap, uint32_t base, uint32_t count, const uint32_t* counter,
                         const uint32_t* salt, uint32_t nsalt, uint32_t* pmk, hipStream_t s, uint32_t* work) {
    if (count == 0) return hipSuccess;
    if (use_plain()) return launch_pbkdf2_plain(mid, cap, base, count, counter, salt, nsalt, pmk, s);
    Fns fn;
    hipError_t e = tuned_functions(&fn);
    if (e != hipSuccess) return e;
    // with a device counter the host only knows the upper bound min(count, cap - base)
    if (lone_waves(fn, std::min<uint64_t>(count, cap > base ? cap - base : 0)))
        return launch_pbkdf2_plain(mid, cap, base, count, counter, salt, nsalt, pmk, s);
    const uint64_t pmks = std::min<uint64_t>(count, cap > base ? cap - base : 0);
    if (work && !use_prio(fn, pmks)) {
        // one resident round (8 waves per SIMD) that drains the item counter
        e = hipMemsetAsync(work, 0, 4, s);
        if (e != hipSuccess) return e;
        void* qargs[] = {(void*)&mid, (void*)&cap, (void*)&base, (void*)&count, (void*)&counter,
                         (void*)&salt, (void*)&nsalt, (void*)&pmk, (void*)&work};
        const uint32_t blocks = (uint32_t)(8 * fn.level_lanes / 256);
        return hipModuleLaunchKernel(fn.one_q, blocks, 1, 1, 256, 1, 1, 0, s, qargs, nullptr);
    }
    void* args[] = {(void*)&mid, (void*)&cap, (void*)&base, (void*)&count, (void*)&counter,
                    (void*)&salt, (void*)&nsalt, (void*)&pmk};
    const uint32_t wg = WG;
    return hipModuleLaunchKernel(use_prio(fn, std::min<uint64_t>(count, cap > base ? cap - base : 0)) ? fn.one_p : fn.one,
                                 (count + wg - 1) / wg, 2, 1, wg, 1, 1, 0, s, args,
                                 nullptr);
}

hipError_t launch_pbkdf2_ms(const uint32_t* mid, uint32_t cap, uint32_t count, const uint32_t* pool,
                            const uint32_t* sref, uint32_t* pmk, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (use_plain()) return launch_pbkdf2_ms_plain(mid, cap, count, pool, sref, pmk, s);
    Fns fn;
    hipError_t e = tuned_functions(&fn);
    if (e != hipSuccess) return e;
    if (lone_waves(fn, std::min(count, cap))) return launch_pbkdf2_ms_plain(mid, cap, count, pool, sref, pmk, s);
    void* args[] = {(void*)&mid, (void*)&cap, (void*)&count, (void*)&pool, (void*)&sref, (void*)&pmk};
    const uint32_t wg = WG;
    return hipModuleLaunchKernel(use_prio(fn, std::min(count, cap)) ? fn.ms_p : fn.ms, (count + wg - 1) / wg, 2, 1, wg, 1, 1, 0, s, args,
                                 nullptr);
}

hipError_t launch_pbkdf2_mg(const uint32_t* mid, uint32_t cap, const uint32_t* counter, uint32_t ngroups,
                            const uint32_t* salt, const uint32_t* gsalt, uint32_t* pmk, uint32_t pstride,
                            hipStream_t s, uint32_t* work) {
    if (ngroups == 0 || cap == 0) return hipSuccess;
    if (cap % 64) return hipErrorInvalidValue;  // chunk group must be wave-uniform
    if (use_plain()) return launch_pbkdf2_mg_plain(mid, cap, counter, ngroups, salt, gsalt, pmk, pstride, s);
    Fns fn;
    hipError_t e = tuned_functions(&fn);
    if (e != hipSuccess) return e;
    const uint64_t lanes = (uint64_t)ngroups * cap;
    if (lanes > 0xffffffffull - 255) return hipErrorInvalidValue;
    if (lone_waves(fn, lanes)) return launch_pbkdf2_mg_plain(mid, cap, counter, ngroups, salt, gsalt, pmk, pstride, s);
    if (work && !use_prio(fn, lanes)) {
        e = hipMemsetAsync(work, 0, 4, s);
        if (e != hipSuccess) return e;
        void* qargs[] = {(void*)&mid, (void*)&cap, (void*)&counter, (void*)&ngroups, (void*)&salt, (void*)&gsalt,
                         (void*)&pmk, (void*)&pstride, (void*)&work};
        const uint32_t blocks = (uint32_t)(8 * fn.level_lanes / 256);
        return hipModuleLaunchKernel(fn.mg_q, blocks, 1, 1, 256, 1, 1, 0, s, qargs, nullptr);
    }
    void* args[] = {(void*)&mid, (void*)&cap, (void*)&counter, (void*)&ngroups, (void*)&salt, (void*)&gsalt,
                    (void*)&pmk, (void*)&pstride};
    const uint32_t wg = WG;
    return hipModuleLaunchKernel(use_prio(fn, lanes) ? fn.mg_p : fn.mg, (uint32_t)((lanes + wg - 1) / wg), 2, 1, wg, 1, 1, 0, s,
                                 args, nullptr);
}

uint32_t pbkdf2_wave_unit() {
    Fns fn;
    if (tuned_functions(&fn) != hipSuccess) return 0;
    return (uint32_t)(fn.level_lanes / 2);
}

const char* pbkdf2_variant() {
    return use_plain() ? "k_pbkdf2 (hipcc schedule)"
                       : force_issue() ? "k_pbkdf2_gfx950 (issue pass)"
                                       : "k_pbkdf2_gfx950 (issue pass; hipcc schedule at <= 1 wave per SIMD)";
}

}  // namespace dwpa
