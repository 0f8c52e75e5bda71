// engine.hpp -- internal interfaces of libdwpa22000.so shared by engine.cpp and crack.cpp.
#pragma once
#include <stdint.h>

#include <functional>
#include <new>
#include <stdexcept>
#include <vector>

#include "dwpa22000.h"
#include "tables.hpp"

namespace dwpa {

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes);
    void release();
};

// Per-batch device working set (cap candidate slots).
struct Batch {
    uint32_t cap = 0, hitcap = 0;
    DevBuf mid;       // [10][cap] u32 HMAC key midstates
    DevBuf pmk;       // [8][cap]  u32 PMKs
    DevBuf ids;       // [cap]     u64 candidate ids
    DevBuf hits;      // [hitcap]  HitDev
    DevBuf counters;  // [0] loaded slots, [1] hit count, [2] PBKDF2 work-queue counter
    int reserve(uint32_t cap, uint32_t hitcap);
};

// A field of the caller's dwpa_config counts only if its struct_size covers it (an older, shorter struct leaves the
// later fields at their documented defaults).  struct_size 0 = the full current struct.
#define DWPA_CFG_HAS(cfg, field) \
    ((cfg) && (!(cfg)->struct_size || (cfg)->struct_size >= offsetof(dwpa_config, field) + sizeof((cfg)->field)))

// No C++ exception crosses the C ABI (a PHP-FPM worker or a Python process would be aborted): every entry point that
// allocates host memory runs its body through guarded(), which maps std::bad_alloc / std::length_error (a host table
// for an input too large for the machine) to `nomem` and any other exception to `other`.  Locks, call contexts and
// in-flight device work are held by RAII objects in the bodies, so an unwound call leaves the library usable.
template <class F>
inline int guarded(F&& body, int nomem = DWPA_E_NOMEM, int other = DWPA_E_ARG) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return nomem;
    } catch (const std::length_error&) {
        return nomem;
    } catch (...) {
        return other;
    }
}

// The check path's host worker pool (engine.cpp HostPool): threads for n items of at least min_per_thread each (at
// most DWPA_HOST_THREADS), and fn(0..T-1) with part 0 on the calling thread.
size_t host_threads_for(size_t n, size_t min_per_thread);
void host_parallel(size_t T, const std::function<void(size_t)>& fn);

// Host (CPU) backend, host_check.cpp.  host_cost: the work of a check call in PMK-equivalents (PBKDF2 derives plus
// the nonce-correction attempts' verify compressions / 16,388), estimated from the jobs without parsing them.
struct HostCost {
    uint64_t keys = 0;      // non-null keys
    uint64_t derives = 0;   // keys whose PMK is derived (not the caller's $pmk)
    double pmk_equiv = 0;   // derives + verify work
};
HostCost host_cost(const dwpa_job* jobs, size_t njobs);
int host_check_batch(const dwpa_job* jobs, size_t njobs, dwpa_result* out, int* rcs, dwpa_check_stats& stats);
int host_pbkdf2(const dwpa_bytes* keys, size_t nkeys, const uint8_t* essid, size_t essid_len, uint8_t* out);
// PMKs the host backend derives in `seconds` on this CPU over `threads` threads (its measured per-chunk costs).
double host_pmks_in(double seconds, size_t threads);
// PBKDF2 of n keys on the host backend into SoA rows: pmk[w * stride + i] = big-endian word w of key i's PMK; key i
// salted with salt[i] (build_salt_blocks layout, nblk[i] blocks).  The device check path's remainder helper.
void host_derive_soa(size_t n, const uint8_t* const* key, const uint32_t* len, const uint32_t* const* salt,
                     const uint32_t* nblk, uint32_t* pmk, size_t stride);

// Pinned host memory (hipHostMalloc) counted in dwpa_resource_stats.pinned_host_bytes; free with the same size.
int pinned_alloc(void** p, size_t bytes);
void pinned_free(void* p, size_t bytes);

int engine_init();
// Rule-file loader mode of the process: dwpa_init's cfg->rule_mode when given, else DWPA_RULE_MODE=full|hashcat
// from the environment, else DWPA_RULES_HASHCAT.  Host only (no device needed).
int engine_rule_mode();
std::vector<int> engine_devices(uint32_t mask);  // mask 0 = the dwpa_init() selection
uint32_t engine_batch();

int scan_create(int device, const char* const* lines, const size_t* lens, size_t nlines, int nc, int nc_mode,
                uint32_t batch, dwpa_scan** out);
void scan_destroy(dwpa_scan* sc);
// fill = true (crack_files): count may exceed the batch; candidates beyond it are dropped by the compaction and
// counted, and scan_counter_raw tells the caller to retry with fewer words.
int scan_counter_raw(dwpa_scan* sc, void* stream, uint32_t* raw);
int scan_load_dict(dwpa_scan* sc, const uint64_t* off, const uint8_t* bytes, uint64_t first, uint32_t count,
                   uint32_t minlen, uint32_t maxlen, void* stream, bool fill = false);
int scan_load_numeric(dwpa_scan* sc, uint64_t first, uint32_t count, uint32_t digits, void* stream);
int scan_pbkdf2(dwpa_scan* sc, int group, void* stream);
int scan_verify(dwpa_scan* sc, int group, void* stream);
int scan_run(dwpa_scan* sc, void* stream);
int scan_hits_raw(dwpa_scan* sc, std::vector<HitDev>& out, void* stream);
void hit_to_public(const dwpa_scan* sc, const HitDev& h, dwpa_hit& o);
void scan_mark_cracked(dwpa_scan* sc, uint32_t input_line);
uint32_t scan_batch_cap(const dwpa_scan* sc);
Batch& scan_batch_ref(dwpa_scan* sc);
int scan_device(const dwpa_scan* sc);
void scan_rules_drop(const dwpa_scan* scan);

}  // namespace dwpa
