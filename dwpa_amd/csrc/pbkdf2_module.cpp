// pbkdf2_module.cpp -- loads the issue-pass PBKDF2 code object (embedded at build time) on each device and launches
// it.  DWPA_PBKDF2_PLAIN=1 selects the hipcc-scheduled k_pbkdf2 instead (A/B reference; identical results).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <map>
#include <mutex>

#include "kernels.hpp"

namespace dwpa {

extern const uint8_t pbkdf2_gfx950_hsaco[];
extern const size_t pbkdf2_gfx950_hsaco_size;

struct Fns {
    hipFunction_t one, ms, mg;  // k_pbkdf2_gfx950 (one ESSID), _ms (per-slot salt), _mg (ESSID groups x batch)
};
static std::mutex g_mod_mu;
static std::map<int, Fns> g_fn;

static bool use_plain() {
    static const bool plain = [] {
        const char* e = getenv("DWPA_PBKDF2_PLAIN");
        return e && *e && *e != '0';
    }();
    return plain;
}

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
    g_fn[dev] = *fn;
    return hipSuccess;
}

hipError_t launch_pbkdf2(const uint32_t* mid, uint32_t cap, uint32_t base, uint32_t count, const uint32_t* counter,
                         const uint32_t* salt, uint32_t nsalt, uint32_t* pmk, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (use_plain()) return launch_pbkdf2_plain(mid, cap, base, count, counter, salt, nsalt, pmk, s);
    Fns fn;
    hipError_t e = tuned_functions(&fn);
    if (e != hipSuccess) return e;
    void* args[] = {(void*)&mid, (void*)&cap, (void*)&base, (void*)&count, (void*)&counter,
                    (void*)&salt, (void*)&nsalt, (void*)&pmk};
    return hipModuleLaunchKernel(fn.one, (count + 255) / 256, 2, 1, 256, 1, 1, 0, s, args, nullptr);
}

hipError_t launch_pbkdf2_ms(const uint32_t* mid, uint32_t cap, uint32_t count, const uint32_t* pool,
                            const uint32_t* sref, uint32_t* pmk, hipStream_t s) {
    if (count == 0) return hipSuccess;
    if (use_plain()) return launch_pbkdf2_ms_plain(mid, cap, count, pool, sref, pmk, s);
    Fns fn;
    hipError_t e = tuned_functions(&fn);
    if (e != hipSuccess) return e;
    void* args[] = {(void*)&mid, (void*)&cap, (void*)&count, (void*)&pool, (void*)&sref, (void*)&pmk};
    return hipModuleLaunchKernel(fn.ms, (count + 255) / 256, 2, 1, 256, 1, 1, 0, s, args, nullptr);
}

hipError_t launch_pbkdf2_mg(const uint32_t* mid, uint32_t cap, const uint32_t* counter, uint32_t ngroups,
                            const uint32_t* salt, const uint32_t* gsalt, uint32_t* pmk, uint32_t pstride,
                            hipStream_t s) {
    if (ngroups == 0 || cap == 0) return hipSuccess;
    if (cap % 64) return hipErrorInvalidValue;  // chunk group must be wave-uniform
    if (use_plain()) return launch_pbkdf2_mg_plain(mid, cap, counter, ngroups, salt, gsalt, pmk, pstride, s);
    Fns fn;
    hipError_t e = tuned_functions(&fn);
    if (e != hipSuccess) return e;
    const uint64_t lanes = (uint64_t)ngroups * cap;
    if (lanes > 0xffffffffull - 255) return hipErrorInvalidValue;
    void* args[] = {(void*)&mid, (void*)&cap, (void*)&counter, (void*)&ngroups, (void*)&salt, (void*)&gsalt,
                    (void*)&pmk, (void*)&pstride};
    return hipModuleLaunchKernel(fn.mg, (uint32_t)((lanes + 255) / 256), 2, 1, 256, 1, 1, 0, s, args, nullptr);
}

const char* pbkdf2_variant() { return use_plain() ? "k_pbkdf2 (hipcc schedule)" : "k_pbkdf2_gfx950 (issue pass)"; }

}  // namespace dwpa
