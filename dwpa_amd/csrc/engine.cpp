// engine.cpp -- libdwpa22000.so: device contexts, the server-side check path (routed to the host backend in
// host_check.cpp for small calls, and without a device when allowed; a device call derives its PBKDF2 remainder on
// the host beside the GPU head when that fits), the device-resident scan API and the C-ABI exports declared in
// include/dwpa22000.h.
//
// Process model: one process may drive every visible MI355X.  crack_files (crack.cpp) runs a stager and a scanner
// thread per device worker over ONE shared dictionary stream, cut into work items by guided self-scheduling
// (dict_reader.hpp ItemQueue) -- no collective, workers never exchange data; hits are gathered on the host.
// bench.py's scan workloads run one process per GPU (torch.distributed launch) on the scan API instead.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <deque>
#include <exception>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <unordered_map>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <thread>
#include <vector>

#include "dwpa22000.h"
#include "engine.hpp"
#include "kernels.hpp"
#include "m22000_host.hpp"

namespace dwpa {

static thread_local hipError_t t_last_hip = hipSuccess;

// DWPA_TRACE=1: host phase timings of the check path on stderr (what the PCIe-inclusive FFI rate is made of).
struct PhaseTrace {
    bool on;
    std::chrono::steady_clock::time_point t;
    PhaseTrace() : on(getenv("DWPA_TRACE") && *getenv("DWPA_TRACE") == '1'), t(std::chrono::steady_clock::now()) {}
    void mark(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[dwpa] %-22s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

#define HIPCHK(x)                                                                                            \
    do {                                                                                                     \
        hipError_t e_ = (x);                                                                                 \
        if (e_ != hipSuccess) {                                                                              \
            t_last_hip = e_;                                                                                 \
            return DWPA_E_HIP;                                                                               \
        }                                                                                                    \
    } while (0)
#define RCHK(x)                    \
    do {                           \
        int r_ = (x);              \
        if (r_ < 0) return r_;     \
    } while (0)

// What the library holds right now (dwpa_resource_stats): device buffers and pinned host memory.
std::atomic<uint64_t> g_dev_bytes{0}, g_pinned_bytes{0};

int DevBuf::ensure(size_t bytes) {
    if (n >= bytes && p) return 0;
    release();
    if (bytes == 0) bytes = 16;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        p = nullptr;
        return DWPA_E_NOMEM;
    }
    n = bytes;
    g_dev_bytes += n;
    return 0;
}
void DevBuf::release() {
    if (p) {
        (void)hipFree(p);
        g_dev_bytes -= n;
    }
    p = nullptr;
    n = 0;
}

int pinned_alloc(void** p, size_t bytes) {
    if (hipHostMalloc(p, bytes, hipHostMallocDefault) != hipSuccess) {
        *p = nullptr;
        return DWPA_E_NOMEM;
    }
    g_pinned_bytes += bytes;
    return 0;
}
void pinned_free(void* p, size_t bytes) {
    if (!p) return;
    (void)hipHostFree(p);
    g_pinned_bytes -= bytes;
}

// Pinned host staging (hipHostMalloc): uploads from it are plain DMA, unlike pageable copies, which HIP stages
// through its own buffers on the calling thread.  One arena per device, carved per call; the caller synchronises
// the stream before the arena is reused.
struct PinnedArena {
    uint8_t* p = nullptr;
    size_t cap = 0, used = 0;
    int reset(size_t bytes) {
        used = 0;
        if (cap >= bytes) return 0;
        release();
        if (hipHostMalloc((void**)&p, bytes, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return DWPA_E_NOMEM;
        }
        cap = bytes;
        g_pinned_bytes += cap;
        return 0;
    }
    template <typename T>
    T* take(size_t n) {
        const size_t off = (used + 63) & ~(size_t)63;
        used = off + n * sizeof(T);
        return (T*)(p + off);
    }
    void release() {
        if (p) {
            (void)hipHostFree(p);
            g_pinned_bytes -= cap;
        }
        p = nullptr;
        cap = used = 0;
    }
};

// ---------------------------------------------------------------------------------------------------------
// global state
// ---------------------------------------------------------------------------------------------------------
// The check path's candidate slots (explicit keys) in slot order: ESSID groups in first-seen order, jobs in input
// order within a group, keys in order within a job.  Flat arrays that keep their capacity (and their pages)
// between calls; the key bytes ($HEX[] decoded) sit in pinned memory, so they go up with one DMA and the unique
// keys are never copied on the host (k_prep_keys reads them through uslot).
constexpr uint32_t SLOT_CALLER = 0x80000000u;  // ord flag: the PMK comes from the caller (common.php:178)
struct SlotTable {
    std::vector<uint32_t> job;   // slot -> job
    std::vector<uint32_t> ord;   // key ordinal among the job's non-null keys (selects its attempt list) | SLOT_CALLER
    std::vector<uint64_t> hash;  // hash_key of the key, taken while its bytes are in cache
    std::vector<uint32_t> kidx;  // the key's index in the caller's key list (null keys included)
    PinnedArena mem;             // koff[n], klen[n], key bytes
    uint64_t* koff = nullptr;
    uint32_t* klen = nullptr;
    uint8_t* kbytes = nullptr;
    size_t n = 0, nbytes = 0;    // slots; capacity of kbytes (upper bound of the decoded bytes)
    int reserve(size_t slots, size_t bytes) {
        RCHK(mem.reset(12 * slots + bytes + 16 + 4 * 64));
        koff = mem.take<uint64_t>(slots);
        klen = mem.take<uint32_t>(slots);
        kbytes = mem.take<uint8_t>(bytes + 16);  // + 16: load_key_block reads whole dwords
        memset(kbytes + bytes, 0, 16);
        job.resize(slots);
        ord.resize(slots);
        hash.resize(slots);
        kidx.resize(slots);
        n = slots;
        nbytes = bytes;
        return 0;
    }
    std::string_view key(size_t i) const { return {(const char*)kbytes + koff[i], klen[i]}; }
};

// Per-run dedup output of one host thread (derive_slots); kept in the call context so its vectors keep capacity.
struct DedupPart {
    std::vector<uint32_t> uslot, sref, spool, cpmk, table, sb;  // sref: offsets into this part's spool
    std::vector<uint64_t> uhash;
    size_t rb = 0, re = 0, ubase = 0, sbase = 0, cbase = 0;
};

// Per-job scratch of the check path's host phases (capacity kept between calls).
struct CheckScratch {
    std::vector<ParsedLine> parsed;
    std::vector<uint32_t> nnz;          // non-null keys of a job that can match (0: no slots)
    std::vector<uint64_t> jbytes;       // their raw bytes (upper bound of the decoded bytes)
    std::vector<uint32_t> jslot;        // first slot of a job
    std::vector<uint64_t> jbyte;        // first key byte of a job
    std::vector<uint32_t> gid, order;   // job -> ESSID group; jobs in slot order (group-major)
    std::vector<uint32_t> gstart, gslot, gfill;  // per group: first entry of `order`, first slot
    std::vector<const uint8_t*> job_pmk;
    std::unordered_map<std::string_view, uint32_t> essid_id;
};

// Host-mapped pinned buffer that kernels write directly (hit copy-out, k_hits_out).
struct MappedHost {
    uint8_t* p = nullptr;
    void* dev = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (cap >= bytes && p) return 0;
        release();
        if (hipHostMalloc((void**)&p, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            p = nullptr;
            return DWPA_E_NOMEM;
        }
        cap = bytes;
        g_pinned_bytes += cap;
        if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess) {
            release();
            return DWPA_E_NOMEM;
        }
        return 0;
    }
    void release() {
        if (p) {
            (void)hipHostFree(p);
            g_pinned_bytes -= cap;
        }
        p = nullptr;
        dev = nullptr;
        cap = 0;
    }
};

struct Device {
    int id = 0;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;   // check path: table uploads while PBKDF2 runs on `stream`
    hipEvent_t side_done = nullptr;
    hipStream_t tail = nullptr;   // check path: the PBKDF2 remainder (< one wave per SIMD) + its verify
    hipEvent_t vs_go = nullptr, vs_done = nullptr;  // check path: fan-out of the keyver-3 verify onto `side`
    hipEvent_t head_done = nullptr, tail_done = nullptr, prep_done = nullptr;
    hipEvent_t head_end = nullptr;  // check path: this context's last PBKDF2 head (the device's head fence)
    double tail_share = 0.75;     // check path: share of the head's time the host tail may take (host_tail_fits)
    PinnedArena stage;            // check path: host staging of the derive uploads
    MappedHost hits_host;         // check path: hit count + hits written by k_hits_out
    TableBuilder tb;              // check path: line and attempt tables of the current call (capacity kept)
    std::mutex mu;
    Batch batch;
    DevBuf lines, atts, pool, segs, segs_tail, salt;
    DevBuf koff, klen, kbytes, uslot;  // check path: the call's key bytes by slot, unique key -> its first slot
    DevBuf keys, keys_tail;        // check path: per-key EapolKey scratch of the attempt-parallel verify
    DevBuf first_hit;              // check path: per line (= job), the smallest slot with a hit so far (~0u: none)
    DevBuf upmk, sref, src, cpmk;  // run_slots: unique-pair PMKs, their salt refs, slot -> PMK source
    SlotTable slots;               // check path: the call's slots (capacity kept between calls)
    CheckScratch cs;               // check path: host-phase scratch
    std::vector<DedupPart> parts;  // check path: dedup output per host thread
    dwpa_check_stats stats{};      // check path: the current call's statistics (dwpa_check_last_stats)
    std::atomic<bool> used{false}; // its streams exist (a call ran on it); read by dwpa_resource_stats
};

static std::mutex g_mu;
static bool g_init = false;
static int g_ndev = 0;
static uint32_t g_mask = 0;
static uint32_t g_batch = 0;
static int g_rule_mode = DWPA_RULES_DEFAULT;  // dwpa_init's cfg->rule_mode
static int g_cpu_fallback = 0;                // dwpa_init's cfg->allow_cpu_fallback (0: DWPA_CPU_FALLBACK)
static int g_host_max = 0;                    // dwpa_init's cfg->host_max_pmks (0: DWPA_HOST_MAX_PMKS, else default)
static bool g_nodev = false;                  // hipGetDeviceCount found no device (not asked again)
// A device call has completed in this process.  Until then the small-call threshold is COLD_FACTOR times larger:
// the first device call also starts the HIP runtime, loads the code objects and creates the call context (0.2-0.7 s
// in a fresh PHP-FPM worker, profiles/r05/c1cold/), which a few hundred host PBKDF2s undercut.
static std::atomic<bool> g_device_warm{false};
constexpr double COLD_FACTOR = 8.0;
static std::vector<std::unique_ptr<Device>> g_dev;  // call contexts: [device * calls_per_device() + k]

// Head fence of one physical device: concurrent calls launch their PBKDF2 heads one after another (each head
// stream waits for the previous head's end event), so two heads never split the SIMDs' wave slots; a call's tail
// and verify then run beside the next call's head.  Wait + launch + publish happen under the mutex, so a context
// re-recording its event for a later head can never be waited on by an earlier one (no cycle).
struct HeadFence {
    std::mutex mu;
    hipEvent_t last = nullptr;
};
static std::vector<std::unique_ptr<HeadFence>> g_fence;  // [device]
static std::atomic<uint32_t> g_rr{0};

static uint32_t default_batch() { return g_batch ? g_batch : (1u << 20); }

// Check-path calls in flight per device (DWPA_CALLS_PER_DEVICE, 1..8, default 2).  Each call context has its own
// streams and buffers, so concurrent callers (PHP ZTS threads, a threaded Python server) overlap on one GPU: one
// call's host phases, lone-wave PBKDF2 remainder and verify run beside the next call's PBKDF2 head instead of
// leaving SIMDs idle.  With one caller only context 0 is used.
static int calls_per_device() {
    static const int k = [] {
        const char* e = getenv("DWPA_CALLS_PER_DEVICE");
        const int v = e ? atoi(e) : 2;
        return v < 1 ? 1 : v > 8 ? 8 : v;
    }();
    return k;
}

static int init_locked(const dwpa_config* cfg, bool probe = true) {
    if (cfg) {
        g_mask = cfg->device_mask;
        g_batch = cfg->batch;
        if (DWPA_CFG_HAS(cfg, rule_mode)) g_rule_mode = cfg->rule_mode;
        if (DWPA_CFG_HAS(cfg, allow_cpu_fallback)) g_cpu_fallback = cfg->allow_cpu_fallback;
        if (DWPA_CFG_HAS(cfg, host_max_pmks)) g_host_max = cfg->host_max_pmks;
    }
    if (g_init || !probe) return 0;
    if (g_nodev) return DWPA_E_NODEV;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        g_nodev = true;
        return DWPA_E_NODEV;
    }
    g_ndev = n;
    g_dev.clear();
    g_fence.clear();
    for (int d = 0; d < n; d++) g_fence.push_back(std::make_unique<HeadFence>());
    for (int d = 0; d < n; d++)
        for (int k = 0; k < calls_per_device(); k++) {
            auto dev = std::make_unique<Device>();
            dev->id = d;
            g_dev.push_back(std::move(dev));
        }
    g_init = true;
    return 0;
}

static int ensure_init() {
    std::lock_guard<std::mutex> lk(g_mu);
    return init_locked(nullptr);
}

// Host backend switches (host_check.cpp).  allow_cpu_fallback: dwpa_init's value when set (1 on, -1 off), else
// DWPA_CPU_FALLBACK=1 from the environment; off by default, so a box without a device says DWPA_E_NODEV unless the
// caller asked for the host backend.  host_max_pmks: calls of at most this many PMK-equivalents with at least one
// PBKDF2 derive run on the host (dwpa_init's value, else DWPA_HOST_MAX_PMKS, else what the host pool derives in
// HOST_BUDGET_S on this CPU, at least HOST_MIN_PMKS; <= 0 from either = never).  The budget is a quarter of the GPU's
// one lone-wave PBKDF2 round (~8.2 ms): on the MI355X box's EPYC 9575F a host thread derives ~14,400 PMK/s on
// AVX-512, so the default is ~460 PMKs on 16 threads (profiles/r06/).
static size_t host_threads(size_t n, size_t min_per_thread);
constexpr double HOST_BUDGET_S = 0.002, HOST_MIN_PMKS = 8.0;
static bool cpu_fallback_on() {
    int v;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        v = g_cpu_fallback;
    }
    if (v) return v > 0;
    const char* e = getenv("DWPA_CPU_FALLBACK");
    return e && *e == '1';
}
static double host_max_pmks() {
    int v;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        v = g_host_max;
    }
    if (v) return v < 0 ? 0.0 : (double)v;
    const char* e = getenv("DWPA_HOST_MAX_PMKS");
    if (e && *e) return std::max(0.0, atof(e));
    static const double dflt = std::max(HOST_MIN_PMKS, std::floor(host_pmks_in(HOST_BUDGET_S, host_threads(SIZE_MAX, 1))));
    return dflt;
}
// Device-side failures a call may retry on the host backend (allow_cpu_fallback): no device, a HIP error, a device or
// pinned allocation that failed, a hit buffer that overflowed.
static bool host_retry_code(int rc) {
    return rc == DWPA_E_NODEV || rc == DWPA_E_HIP || rc == DWPA_E_NOMEM || rc == DWPA_E_OVERFLOW;
}

// Devices selected by `mask` (0 = the dwpa_init() mask; that one 0 = every visible device).
static std::vector<int> active_devices(uint32_t mask = 0) {
    if (!mask) mask = g_mask;
    std::vector<int> v;
    for (int d = 0; d < g_ndev; d++)
        if (!mask || (mask >> d & 1u)) v.push_back(d);
    return v;
}

// The priority the PBKDF2 tail raises itself to once the head has ended (pbkdf2_dev.hpp pbkdf2_lane_tail): above
// the verify waves that share its SIMDs.  (The other scheduling choices of the check path -- post-derive and keyver-3
// kernels at priority 0, head fence, keyver-3 fan-out, verify order -- are fixed at their measured best: DESIGN.md 4,
// CHANGELOG.md.)
constexpr uint32_t TAIL_PRIO = 2;

static int device_stream(Device& d) {
    if (!d.stream) {
        HIPCHK(hipSetDevice(d.id));
        HIPCHK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&d.side, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&d.side_done, hipEventDisableTiming));
        HIPCHK(hipStreamCreateWithFlags(&d.tail, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&d.head_done, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.tail_done, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.prep_done, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.head_end, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.vs_go, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&d.vs_done, hipEventDisableTiming));
        d.used.store(true, std::memory_order_release);
    }
    return 0;
}

int Batch::reserve(uint32_t want_cap, uint32_t want_hitcap) {
    if (cap < want_cap) {
        RCHK(mid.ensure((size_t)MID_WORDS * want_cap * 4));
        RCHK(pmk.ensure((size_t)PMK_WORDS * want_cap * 4));
        RCHK(ids.ensure((size_t)want_cap * 8));
        cap = want_cap;
    }
    if (hitcap < want_hitcap) {
        RCHK(hits.ensure((size_t)want_hitcap * sizeof(HitDev)));
        hitcap = want_hitcap;
    }
    RCHK(counters.ensure(32));  // [3] check path: head-done flag, [4] tail waves that raised their priority
    return 0;
}

template <typename T>
static int upload(DevBuf& b, const std::vector<T>& v, hipStream_t s) {
    RCHK(b.ensure(std::max<size_t>(v.size() * sizeof(T), 16)));
    if (!v.empty()) HIPCHK(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    return 0;
}

static void pmk_bytes(const uint32_t w[8], uint8_t out[32]) {
    for (int k = 0; k < 8; k++) {
        out[4 * k] = (uint8_t)(w[k] >> 24);
        out[4 * k + 1] = (uint8_t)(w[k] >> 16);
        out[4 * k + 2] = (uint8_t)(w[k] >> 8);
        out[4 * k + 3] = (uint8_t)w[k];
    }
}

// ---------------------------------------------------------------------------------------------------------
// explicit keys -> slots (server-side check path and dwpa_pbkdf2_pmk)
// ---------------------------------------------------------------------------------------------------------

// 64-bit hash of a key (8-byte multiply-xor rounds) for the (ESSID run, key) dedup table.  Reads only the key's
// own bytes, with overlapping loads for the tail: it runs on the caller's buffers, before the bytes are copied
// (hashing the fresh copy would stall on store-to-load forwarding).
static uint64_t hash_key(const uint8_t* p, size_t n) {
    uint64_t h = n * 0x9e3779b97f4a7c15ull, w;
    if (n >= 8) {
        const uint8_t* end = p + n;
        for (; p + 8 <= end; p += 8) {
            memcpy(&w, p, 8);
            h = (h ^ w) * 0xff51afd7ed558ccdull;
            h ^= h >> 32;
        }
        if (p == end) return h ^ (h >> 29);
        memcpy(&w, end - 8, 8);  // the last 8 bytes (overlapping the previous block)
    } else if (n >= 4) {
        uint32_t a, b;
        memcpy(&a, p, 4);
        memcpy(&b, p + n - 4, 4);
        w = (uint64_t)b << 32 | a;
    } else {
        w = 0;
        for (size_t k = 0; k < n; k++) w |= (uint64_t)p[k] << (8 * k);
    }
    h = (h ^ w) * 0xc4ceb9fe1a85ec53ull;
    return h ^ (h >> 29);
}

// Host threads for the check path's host work: at least `min_per_thread` items each, at most DWPA_HOST_THREADS
// (default 16, the MI355X box's host share per GPU; 8 measured ~1 ms slower per C5 call).  hardware_concurrency()
// reports the whole machine, so it only caps this.
static size_t host_threads(size_t n, size_t min_per_thread) {
    static const size_t cap = [] {
        const char* e = getenv("DWPA_HOST_THREADS");
        const int v = e && *e ? atoi(e) : 16;
        return (size_t)(v < 1 ? 1 : v > 64 ? 64 : v);
    }();
    const unsigned hw = std::thread::hardware_concurrency();
    return std::max<size_t>(1, std::min<size_t>({cap, hw ? hw : 1, n / std::max<size_t>(1, min_per_thread)}));
}

// Host worker pool of the check path: a C5 call runs four parallel phases, and spawning 7 threads per phase cost
// more than the smaller phases themselves.  Workers live for the process; concurrent calls (one per device) share
// them, and a caller waiting for its tasks runs queued tasks itself, so waiting never blocks progress.
class HostPool {
  public:
    static HostPool& get() {
        static HostPool* pool = new HostPool();  // never destroyed: workers may outlive static destructors
        return *pool;
    }
    // fn(0..T-1), part 0 on the calling thread.  An exception of any part (std::bad_alloc on a huge input) is
    // rethrown here once every part has ended -- the queued parts reference this frame -- so that it reaches the
    // entry point's guarded() instead of terminating a worker thread.
    template <typename F>
    void run(size_t T, const F& fn) {
        std::atomic<size_t> left{T - 1};
        std::exception_ptr err;
        std::mutex err_mu;
        auto part = [&](size_t t) {
            try {
                fn(t);
            } catch (...) {
                std::lock_guard<std::mutex> lk(err_mu);
                if (!err) err = std::current_exception();
            }
        };
        size_t queued = 0;
        {
            std::lock_guard<std::mutex> lk(mu_);
            try {
                grow_locked(T - 1);
            } catch (...) {  // fewer workers: the caller runs what they do not take
            }
            try {
                for (; queued + 1 < T; queued++)
                    q_.push_back([&part, &left, t = queued + 1] {
                        part(t);
                        left.fetch_sub(1, std::memory_order_acq_rel);
                    });
            } catch (...) {  // the parts that could not be queued run below
            }
        }
        cv_.notify_all();
        part(0);
        for (size_t t = queued + 1; t < T; t++) {
            part(t);
            left.fetch_sub(1, std::memory_order_acq_rel);
        }
        while (left.load(std::memory_order_acquire)) {
            std::function<void()> task;
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (!q_.empty()) {
                    task = std::move(q_.front());
                    q_.pop_front();
                }
            }
            if (task) task();
            else std::this_thread::yield();
        }
        if (err) std::rethrow_exception(err);
    }

    size_t workers() {
        std::lock_guard<std::mutex> lk(mu_);
        return workers_;
    }

  private:
    void grow_locked(size_t want) {
        while (workers_ < want) {
            std::thread([this] { loop(); }).detach();
            workers_++;
        }
    }
    void loop() {
        for (;;) {
            std::function<void()> task;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return !q_.empty(); });
                task = std::move(q_.front());
                q_.pop_front();
            }
            task();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    size_t workers_ = 0;
};

// fn(t) for t in [0, T) on up to T threads (the calling thread runs t = 0, pool workers the rest).
template <typename F>
static void parallel_for(size_t T, const F& fn) {
    if (T <= 1) {
        if (T == 1) fn(0);
        return;
    }
    HostPool::get().run(T, fn);
}

size_t host_threads_for(size_t n, size_t min_per_thread) { return host_threads(n, min_per_thread); }
void host_parallel(size_t T, const std::function<void(size_t)>& fn) { parallel_for(T, fn); }

// A typed view of pinned staging memory.
template <typename T>
struct Span {
    T* p = nullptr;
    size_t n = 0;
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
    T* data() const { return p; }
    size_t size() const { return n; }
};
template <typename T>
static Span<T> take(PinnedArena& a, size_t n) {
    return Span<T>{a.take<T>(n), n};
}
template <typename T>
static int upload_span(DevBuf& b, const Span<T>& v, hipStream_t s) {
    RCHK(b.ensure(std::max<size_t>(v.n * sizeof(T), 16)));
    if (v.n) HIPCHK(hipMemcpyAsync(b.p, v.p, v.n * sizeof(T), hipMemcpyHostToDevice, s));
    return 0;
}

// A host thread deriving the PBKDF2 remainder of a check call on the host backend while the head runs on the GPU
// (derive_slots); joined by finish_derive, or at the latest when the stage goes out of scope.
struct HostTailJob {
    std::thread t;
    int rc = 0;
    ~HostTailJob() {
        if (t.joinable()) t.join();
    }
};

// Host staging of one derive step in the device's pinned arena; valid until the stream is synchronised.
struct DeriveStage {
    Span<uint64_t> ids;
    Span<uint32_t> src, sref, spool, cpmk, uslot;
    uint32_t split = 0;  // slots [0, split) read d.stream's PMKs; [split, n) d.tail's (== n: no tail)
    uint32_t n = 0, nh = 0, nu = 0;
    bool host_tail = false;  // unique PMKs [nh, nu) come from the host (htail, SoA rows of nu - nh words)
    Span<uint32_t> htail;
    HostTailJob job;
};

// DWPA_HOST_TAIL=0 keeps the check path's PBKDF2 remainder on the GPU (a test switch: test_batch_host_tail_switch_off).
static bool host_tail_knob() {
    static const bool on = [] {
        const char* e = getenv("DWPA_HOST_TAIL");
        return !(e && *e == '0');
    }();
    return on;
}

// The PBKDF2 remainder below one wave per SIMD (the tail) goes to the host backend when the host derives it well
// within the head's time: the head then fills whole waves on every SIMD and no lone tail wave outlasts it.  A head
// wave time is ~6.5-7 ms (C2 6.50 ms, the C5 head 7.03 ms per wave per SIMD, CHANGELOG.md round 4/5); the host gets
// a share of the head's estimated time (d.tail_share, at most 3/4), so the GPU does not wait for it on a host with
// the measured speed.  A host busier than measured (other workers on the same cores) is caught by finish_derive: a
// tail that came after the head halves the share, and every later tail brings it back by a quarter.
constexpr double HEAD_WAVE_S = 6.5e-3, HOST_TAIL_SHARE = 0.75;
static bool host_tail_fits(Device& d, uint32_t nt, uint32_t nh) {
    if (!host_tail_knob() || !nt) return false;
    const double head_s = (double)nh / (double)std::max<uint32_t>(1, pbkdf2_wave_unit()) * HEAD_WAVE_S;
    const double share = d.tail_share;
    d.tail_share = std::min(HOST_TAIL_SHARE, d.tail_share * 1.25);
    return (double)nt <= host_pmks_in(share * head_s, host_threads(SIZE_MAX, 1));
}

// Head/tail split of one derive.  PBKDF2 is issue-bound, so a launch takes as long as its fullest SIMD: nu unique
// PMKs at k.f waves per SIMD cost k + 1 whole wave times (~7 ms each at C5 size), the last one with 1 - f of the
// chip idle.  The head (k whole waves per SIMD) runs at wave priority 3..1 (pbkdf2_dev.hpp PRIO); the tail
// (< one wave per SIMD, the latency-bound plain kernel, priority 0) is launched beside it on d.tail and takes only
// the issue slots the head leaves, then finishes alone while the head's verify runs.  From 2 whole waves per SIMD
// up (the head's PRIO kernel; below that both kernels are lone-wave plain kernels) the split pays.
static uint32_t head_pmks(uint32_t nu) {
    const uint32_t unit = pbkdf2_wave_unit();
    if (!unit || nu < 2 * unit) return nu;
    return nu / unit * unit;
}

// T's key bytes and their offsets/lengths (every slot of the call) up d.stream.
static int upload_slot_keys(Device& d, const SlotTable& T) {
    RCHK(upload_span(d.koff, Span<uint64_t>{T.koff, T.n}, d.stream));
    RCHK(upload_span(d.klen, Span<uint32_t>{T.klen, T.n}, d.stream));
    RCHK(upload_span(d.kbytes, Span<uint8_t>{T.kbytes, T.nbytes + 16}, d.stream));
    return 0;
}

// Derive the PMKs of slots [b, e) of T into batch.pmk (slot order) and their key ordinals into batch.ids.  Unique
// (ESSID, key) pairs are derived once, all ESSIDs in one PBKDF2 launch (server batches fan one key out to every
// net of an ESSID, common.php:879-902); each slot then gathers its PMK from them or from the caller's $pmk
// (common.php:178).  Slots arrive grouped by ESSID: `runs` holds the starts of the ESSID runs relative to b plus
// n = e - b, run_essid each run's ESSID.  upload_keys: send T's key bytes (every slot of the call) up first.  The
// uploads are queued ahead of the launches: a pageable upload queued behind a running kernel would block the host
// until that kernel ends.
static int derive_slots(Device& d, const SlotTable& T, size_t b, size_t e, const std::vector<const uint8_t*>& job_pmk,
                        const std::vector<uint32_t>& runs, const std::vector<const std::string*>& run_essid,
                        bool upload_keys, DeriveStage& st, bool allow_host_tail = false) {
    PhaseTrace tr;
    hipStream_t s = d.stream;
    const uint32_t n = (uint32_t)(e - b);
    RCHK(d.batch.reserve(n, 2 * n + 64));  // attempt-parallel verify: <= 2 matching attempts per (key, line)
    size_t saltwords = 0;
    const size_t nruns = runs.size() - 1;
    for (size_t r = 0; r < nruns; r++)  // count word + [2][nblk][16], nblk = SHA-1 blocks of ESSID || INT(i) || pad
        saltwords += 1 + 32 * ((run_essid[r]->size() + 4 + 9 + 63) / 64);
    // pinned staging, sized by upper bounds: <= n unique keys, <= n caller PMKs, <= n host-derived PMKs
    RCHK(d.stage.reset(12 * (size_t)n + 8 * (size_t)n + 4 * saltwords + 64 * (size_t)n + 9 * 64));
    st.src = take<uint32_t>(d.stage, n);
    st.ids = take<uint64_t>(d.stage, n);
    // Runs are deduplicated independently (one small open-addressing table per run keeps it cache-resident), on
    // up to 16 host threads that each take a contiguous block of runs; the parts are then concatenated.
    const size_t T_ = host_threads(n, 8192);
    const size_t np = std::max<size_t>(1, std::min(T_, nruns));
    if (d.parts.size() < np) d.parts.resize(np);
    for (size_t t = 0; t < np; t++) {  // split runs so that parts hold about equal slot counts
        DedupPart& P = d.parts[t];
        P.rb = t ? d.parts[t - 1].re : 0;
        const uint64_t goal = (uint64_t)n * (t + 1) / np;
        size_t r = P.rb;
        while (r < nruns && (runs[r + 1] <= goal || r == P.rb)) r++;
        P.re = t + 1 == np ? nruns : r;
    }
    parallel_for(np, [&](size_t t) {
        DedupPart& P = d.parts[t];
        P.uslot.clear();
        P.sref.clear();
        P.spool.clear();
        P.cpmk.clear();
        for (size_t r = P.rb; r < P.re; r++) {
            const uint32_t i0 = runs[r], i1 = runs[r + 1];
            size_t tcap = 16;
            while (tcap < 2 * (size_t)(i1 - i0)) tcap <<= 1;
            P.table.assign(tcap, UINT32_MAX);
            P.uhash.clear();
            const size_t u0 = P.uslot.size();
            uint32_t cur_ref = UINT32_MAX;
            for (uint32_t i = i0; i < i1; i++) {
                const size_t si = b + i;
                const uint32_t ord = T.ord[si];
                st.ids[i] = ord & ~SLOT_CALLER;  // selects the PHP attempt list of the key
                if (ord & SLOT_CALLER) {
                    const uint8_t* p = job_pmk[T.job[si]];
                    st.src[i] = GATHER_CALLER | (uint32_t)(P.cpmk.size() / 8);
                    for (int k = 0; k < 8; k++)
                        P.cpmk.push_back((uint32_t)p[4 * k] << 24 | (uint32_t)p[4 * k + 1] << 16 |
                                         (uint32_t)p[4 * k + 2] << 8 | p[4 * k + 3]);
                    continue;
                }
                if (cur_ref == UINT32_MAX) {
                    P.sb.clear();
                    const uint32_t nb = build_salt_blocks(*run_essid[r], P.sb);
                    cur_ref = (uint32_t)P.spool.size();
                    P.spool.push_back(nb);
                    P.spool.insert(P.spool.end(), P.sb.begin(), P.sb.end());
                }
                const uint64_t h = T.hash[si];
                size_t pos = h & (tcap - 1);
                uint32_t u;
                while ((u = P.table[pos]) != UINT32_MAX && !(P.uhash[u - u0] == h && T.key(P.uslot[u]) == T.key(si)))
                    pos = (pos + 1) & (tcap - 1);
                if (u == UINT32_MAX) {
                    u = (uint32_t)P.uslot.size();
                    P.table[pos] = u;
                    P.uslot.push_back((uint32_t)si);
                    P.uhash.push_back(h);
                    P.sref.push_back(cur_ref);
                }
                st.src[i] = u;  // part-local; rebased below
            }
        }
    });
    tr.mark("  dedup tables");
    size_t nu_total = 0, nsp = 0, ncp = 0;
    for (size_t t = 0; t < np; t++) {
        DedupPart& P = d.parts[t];
        P.ubase = nu_total;
        P.sbase = nsp;
        P.cbase = ncp;
        nu_total += P.uslot.size();
        nsp += P.spool.size();
        ncp += P.cpmk.size() / 8;
    }
    const uint32_t nu = (uint32_t)nu_total;
    st.sref = take<uint32_t>(d.stage, nu);
    st.uslot = take<uint32_t>(d.stage, nu);
    st.spool = take<uint32_t>(d.stage, nsp);
    st.cpmk = take<uint32_t>(d.stage, ncp * 8);
    if (d.stage.used > d.stage.cap) return DWPA_E_ARG;  // the bounds above are exact upper bounds
    parallel_for(np, [&](size_t t) {  // rebase and concatenate (no key bytes move: k_prep_keys reads them by slot)
        const DedupPart& P = d.parts[t];
        for (uint32_t i = runs[P.rb]; i < runs[P.re]; i++)
            st.src[i] = (st.src[i] & GATHER_CALLER) ? st.src[i] + (uint32_t)P.cbase : st.src[i] + (uint32_t)P.ubase;
        for (size_t u = 0; u < P.uslot.size(); u++) st.sref[P.ubase + u] = P.sref[u] + (uint32_t)P.sbase;
        std::copy(P.uslot.begin(), P.uslot.end(), st.uslot.data() + P.ubase);
        std::copy(P.spool.begin(), P.spool.end(), st.spool.data() + P.sbase);
        std::copy(P.cpmk.begin(), P.cpmk.end(), st.cpmk.data() + 8 * P.cbase);
    });
    tr.mark("  concat");

    RCHK(d.upmk.ensure((size_t)PMK_WORDS * d.batch.cap * 4));
    // head = unique PMKs [0, nh); unique ids are numbered in first-occurrence slot order, so slots [0, split) only
    // read head PMKs (or caller PMKs) and the slots after it wait for the tail
    const uint32_t nh = head_pmks(nu);
    st.split = n;
    st.n = n;
    st.nh = nh;
    st.nu = nu;
    if (allow_host_tail && nh < nu && host_tail_fits(d, nu - nh, nh)) {
        // the remainder on the host backend, beside the head: its keys' bytes (T), salt blocks (spool) and SoA rows
        // in pinned memory, uploaded by finish_derive once the thread is done
        const uint32_t nt = nu - nh;
        st.htail = take<uint32_t>(d.stage, 8 * (size_t)nt);
        if (d.stage.used > d.stage.cap) return DWPA_E_ARG;
        const uint8_t* kb = T.kbytes;
        const uint64_t* ko = T.koff;
        const uint32_t* kl = T.klen;
        const uint32_t* us = st.uslot.data() + nh;
        const uint32_t* sr = st.sref.data() + nh;
        const uint32_t* sp = st.spool.data();
        uint32_t* out = st.htail.data();
        HostTailJob& job = st.job;
        try {
            job.t = std::thread([=, &job] {
                job.rc = guarded([&]() -> int {
                    std::vector<const uint8_t*> key(nt);
                    std::vector<uint32_t> len(nt), nblk(nt);
                    std::vector<const uint32_t*> salt(nt);
                    for (uint32_t u = 0; u < nt; u++) {
                        key[u] = kb + ko[us[u]];
                        len[u] = kl[us[u]];
                        nblk[u] = sp[sr[u]];
                        salt[u] = sp + sr[u] + 1;
                    }
                    host_derive_soa(nt, key.data(), len.data(), salt.data(), nblk.data(), out, nt);
                    return 0;
                });
            });
            st.host_tail = true;
        } catch (...) {  // no thread: the GPU derives the remainder as a tail, as without the host backend
            st.host_tail = false;
        }
    }
    if (nh < nu && !st.host_tail)
        for (uint32_t i = 0; i < n; i++)
            if (!(st.src[i] & GATHER_CALLER) && st.src[i] >= nh) {
                st.split = i;
                break;
            }
    if (upload_keys) RCHK(upload_slot_keys(d, T));
    if (nu) {
        RCHK(upload_span(d.uslot, st.uslot, s));
        RCHK(upload_span(d.salt, st.spool, s));
        RCHK(upload_span(d.sref, st.sref, s));
    }
    RCHK(upload_span(d.cpmk, st.cpmk, s));
    RCHK(upload_span(d.src, st.src, s));
    HIPCHK(hipMemcpyAsync(d.batch.ids.p, st.ids.data(), n * 8, hipMemcpyHostToDevice, s));
    // hit counter reset ahead of every kernel of this derive (the tail's verify may run before the head's)
    HIPCHK(hipMemsetAsync(d.batch.counters.p, 0, 32, s));
    tr.mark("  stage+upload");
    const uint32_t cap = d.batch.cap;
    const uint32_t* mid = (const uint32_t*)d.batch.mid.p;
    const uint32_t* sref = (const uint32_t*)d.sref.p;
    uint32_t* upmk = (uint32_t*)d.upmk.p;
    if (nu) {
        HIPCHK(launch_prep_keys((const uint64_t*)d.koff.p, (const uint32_t*)d.klen.p, (const uint8_t*)d.kbytes.p,
                                (const uint32_t*)d.uslot.p, nu, (uint32_t*)d.batch.mid.p, cap, s));
        HeadFence& f = *g_fence[d.id];
        std::lock_guard<std::mutex> fl(f.mu);
        if (f.last && f.last != d.head_end) HIPCHK(hipStreamWaitEvent(s, f.last, 0));
        uint32_t* head_flag = (uint32_t*)d.batch.counters.p + 3;  // zeroed with the counters above
        uint32_t* raised = (uint32_t*)d.batch.counters.p + 4;     // likewise; read back by collect_hits
        d.stats.pmks += nu;
        if (st.host_tail) d.stats.tail_pmks += nu - nh;
        if (nh < nu && !st.host_tail) {  // the tail first, beside the head (priority 0 until the head has ended)
            HIPCHK(hipEventRecord(d.prep_done, s));
            HIPCHK(hipStreamWaitEvent(d.tail, d.prep_done, 0));
            HIPCHK(launch_pbkdf2_ms_tail(mid + nh, cap, nu - nh, (const uint32_t*)d.salt.p, sref + nh, upmk + nh,
                                         head_flag, TAIL_PRIO, raised, d.tail));
            d.stats.tail_pmks += nu - nh;
            d.stats.tail_waves += 2 * ((nu - nh + 63) / 64);  // two output-block lanes per PMK
        }
        HIPCHK(launch_pbkdf2_ms(mid, cap, nh, (const uint32_t*)d.salt.p, sref, upmk, s));
        if (nh < nu && !st.host_tail) HIPCHK(launch_set_flag(head_flag, s));
        HIPCHK(hipEventRecord(d.head_end, s));
        f.last = d.head_end;
    }
    if (st.host_tail) return 0;  // finish_derive gathers once the host's PMKs are up
    // SoA rows keep their stride (cap), so a sub-range is the same launch on offset base pointers
    const uint32_t sp = st.split;
    if (sp)
        HIPCHK(launch_gather_pmk(upmk, cap, (const uint32_t*)d.cpmk.p, (const uint32_t*)d.src.p, sp,
                                 (uint32_t*)d.batch.pmk.p, cap, s));
    if (sp < n) {  // tail slots may also read head PMKs: their gather waits for both derives
        HIPCHK(hipEventRecord(d.head_done, s));
        HIPCHK(hipStreamWaitEvent(d.tail, d.head_done, 0));
        HIPCHK(launch_gather_pmk(upmk, cap, (const uint32_t*)d.cpmk.p, (const uint32_t*)d.src.p + sp, n - sp,
                                 (uint32_t*)d.batch.pmk.p + sp, cap, d.tail));
    }
    return 0;
}

// The end of a derive whose remainder the host backend computes (derive_slots): wait for the host thread, upload its
// PMKs next to the head's, then gather every slot.  The host thread ran while the GPU derived the head, so the upload
// is normally queued well before the head ends.  Should the thread have failed (an allocation), the GPU derives the
// remainder after the head instead.
static int finish_derive(Device& d, DeriveStage& st) {
    if (!st.host_tail) return 0;
    if (st.job.t.joinable()) st.job.t.join();
    // the head had already ended: the GPU waited for the host, so give later tails less of the head's time
    if (hipEventQuery(d.head_end) == hipSuccess) {
        d.tail_share = std::max(0.05, d.tail_share * 0.5);
        if (PhaseTrace().on) fprintf(stderr, "[dwpa] host tail after the head: share now %.3f\n", d.tail_share);
    }
    const uint32_t cap = d.batch.cap, nh = st.nh, nt = st.nu - st.nh;
    uint32_t* upmk = (uint32_t*)d.upmk.p;
    if (st.job.rc == 0) {
        HIPCHK(hipMemcpy2DAsync(upmk + nh, (size_t)cap * 4, st.htail.data(), (size_t)nt * 4, (size_t)nt * 4, 8,
                                hipMemcpyHostToDevice, d.stream));
    } else {
        HIPCHK(launch_pbkdf2_ms((const uint32_t*)d.batch.mid.p + nh, cap, nt, (const uint32_t*)d.salt.p,
                                (const uint32_t*)d.sref.p + nh, upmk + nh, d.stream));
    }
    HIPCHK(launch_gather_pmk(upmk, cap, (const uint32_t*)d.cpmk.p, (const uint32_t*)d.src.p, st.n,
                             (uint32_t*)d.batch.pmk.p, cap, d.stream));
    return 0;
}

// DWPA_FIRST_KEY_EXIT=0 verifies every key of a job even after an earlier key matched: a test switch
// (tests/test_gpu_parity.py::test_first_key_exit_across_chunks runs both ways; the results are the same).
static bool first_key_exit_knob() {
    static const bool on = [] {
        const char* e = getenv("DWPA_FIRST_KEY_EXIT");
        return !(e && *e == '0');
    }();
    return on;
}

// Keys per attempt-parallel segment when the first-key early exit is on: a later segment of the same job can skip
// itself once an earlier one matched.
constexpr uint32_t ATT_SEG_KEYS = 16;

// d.stream waits for everything queued on d.tail so far.
static int join_tail(Device& d) {
    HIPCHK(hipEventRecord(d.tail_done, d.tail));
    HIPCHK(hipStreamWaitEvent(d.stream, d.tail_done, 0));
    return 0;
}

// Queue the verification of derived slots [b, e) (batch rows from b - base) against their jobs' lines on stream
// s.  The line tables go up on the side stream (while PBKDF2 may still run) and s waits for them.  EAPOL lines with
// wide nonce windows use the attempt-parallel kernel (a wave per key, lanes = attempts), the rest the key-parallel
// one; segments are runs of <= 64 consecutive slots of one job.  Hits are appended on the device (collect_hits).
static int queue_verify(Device& d, const SlotTable& T, size_t base, size_t b, size_t e,
                        const std::vector<uint32_t>& job_line, const TableBuilder& tb, bool upload_tables,
                        hipStream_t s, DevBuf& segbuf, DevBuf& keybuf, bool fanout) {
    const uint32_t n = (uint32_t)(e - b), row0 = (uint32_t)(b - base);
    if (!n && !upload_tables) return 0;
    // bucket = mode * 4 + class index; mode 1 = attempt-parallel (EAPOL lines with >= ATT_PARALLEL_MIN attempts).
    // Attempt-parallel keyver 1 and 2 share bucket 5 (one launch of the combined kernel): every verify launch that
    // runs while the PBKDF2 tail holds some SIMDs ends only with the tail, so fewer launches in a row end sooner.
    std::vector<SegDev> bucket[8];
    auto bucket_vc = [](int k) { return k == 5 ? (uint32_t)(VC_KV1 | VC_KV2) : 1u << (k & 3); };
    const uint32_t att_seg = first_key_exit_knob() ? ATT_SEG_KEYS : 64;
    for (uint32_t i = 0; i < n;) {
        uint32_t j = i;
        const uint32_t job = T.job[b + i];
        const uint32_t li = job_line[job];
        const LineDev& L = tb.lines[li];
        const bool att = L.kind == LINE_EAPOL && L.natt >= ATT_PARALLEL_MIN;
        // attempt-parallel segments are cut shorter: the early exit below skips whole segments dispatched after a
        // job's hit, so the finer the cut, the fewer keys past the hit are verified
        const uint32_t segmax = att ? att_seg : 64;
        while (j < n && T.job[b + j] == job && j - i < segmax) j++;
        // the key-parallel kernel reads every attempt's KW blocks (built for lines under ATT_PARALLEL_MIN)
        if (L.kind == LINE_EAPOL && !att && tb.atts[L.list_off].kw_off == NO_KW) return DWPA_E_ARG;
        if (!tb.never[li]) {
            const int k = (att ? 4 : 0) + __builtin_ctz(verify_class(L));
            bucket[k == 6 ? 5 : k].push_back({li, row0 + i, j - i, 0});
        }
        i = j;
    }
    // attempt-parallel buckets in rank order: every job's first 64 keys, then every job's next 64, ... .  The check
    // wants only the first key in input order with a hit (common.php:170-189,238-306), so a wave whose keys all come
    // after a key already found for its job exits at once (k_verify_att, first_hit); with a job's segments a whole
    // pass over the other jobs apart, the hit of an early segment is known before its later segments are dispatched.
    // A segment of S keys spans S * natt / 64 waves (at nc = 128, 261 attempts: 65.25 waves for S = 16, one partial
    // wave per segment).
    if (first_key_exit_knob())
        for (int k = 4; k < 8; k++) {
            std::vector<SegDev>& v = bucket[k];
            if (v.size() < 2) continue;
            std::vector<std::pair<uint32_t, uint32_t>> key(v.size());  // (rank within its line, position)
            std::unordered_map<uint32_t, uint32_t> rank;
            for (size_t i = 0; i < v.size(); i++) key[i] = {rank[v[i].line]++, (uint32_t)i};
            std::sort(key.begin(), key.end());
            std::vector<SegDev> w(v.size());
            for (size_t i = 0; i < v.size(); i++) w[i] = v[key[i].second];
            v.swap(w);
        }
    // attempt-parallel buckets: pad = the segment's first wave in its launch (ceil(count * natt / 64) waves each)
    uint32_t nwaves[8] = {0};
    for (int k = 4; k < 8; k++)
        for (SegDev& sg : bucket[k]) {
            sg.pad = nwaves[k];
            nwaves[k] += (uint32_t)(((uint64_t)sg.count * tb.lines[sg.line].natt + 63) / 64);
        }
    // per-key EapolKey state scratch of the attempt-parallel launches: one region per class (the classes may run
    // on parallel streams), class k's stride = att_seg (the most keys an attempt-parallel segment holds) x its
    // segments
    size_t koff[8] = {0}, ktotal = 0;
    for (int k = 4; k < 8; k++) {
        koff[k] = ktotal;
        ktotal += (size_t)eapol_key_words(bucket_vc(k)) * bucket[k].size() * att_seg;
    }
    if (ktotal) RCHK(keybuf.ensure(ktotal * 4));
    std::vector<SegDev> segs;
    size_t bstart[9];
    for (int k = 0; k < 8; k++) {
        bstart[k] = segs.size();
        segs.insert(segs.end(), bucket[k].begin(), bucket[k].end());
    }
    bstart[8] = segs.size();
    if (upload_tables) {
        RCHK(upload(d.lines, tb.lines, d.side));
        RCHK(upload(d.atts, tb.atts, d.side));
        RCHK(upload(d.pool, tb.pool, d.side));
    }
    RCHK(upload(segbuf, segs, d.side));
    HIPCHK(hipEventRecord(d.side_done, d.side));
    HIPCHK(hipStreamWaitEvent(s, d.side_done, 0));
    // fan-out: the keyver-3 launches (the longest class) on the side stream, idle once the tables are up, beside
    // the other classes on s, which then waits for them.  Verify waves that land on the SIMDs of the tail's lone
    // waves hold back only their own stream.  (A fourth stream of its own would share a hardware queue with the
    // tail's: a process gets GPU_MAX_HW_QUEUES = 4, one of them the null stream's.)
    const bool fan = fanout && (!bucket[3].empty() || !bucket[7].empty());
    if (fan) {
        HIPCHK(hipEventRecord(d.vs_go, s));
        HIPCHK(hipStreamWaitEvent(d.side, d.vs_go, 0));
    }
    uint32_t* hitcnt = (uint32_t*)d.batch.counters.p + 1;
    for (int k = 0; k < 8; k++) {
        const uint32_t nb = (uint32_t)(bstart[k + 1] - bstart[k]), vc = bucket_vc(k);
        const SegDev* sg = (const SegDev*)segbuf.p + bstart[k];
        if (!nb) continue;
        hipStream_t vsk = fan && (k & 3) == 3 ? d.side : s;
        if (k < 4)
            HIPCHK(launch_verify((const uint32_t*)d.batch.pmk.p, d.batch.cap, (const uint64_t*)d.batch.ids.p, nullptr,
                                 sg, nb, 0, 1, (const LineDev*)d.lines.p, (const uint32_t*)d.pool.p,
                                 (const AttDev*)d.atts.p, (HitDev*)d.batch.hits.p, hitcnt, d.batch.hitcap, vc, vsk));
        else
            HIPCHK(launch_verify_att((const uint32_t*)d.batch.pmk.p, d.batch.cap, (const uint64_t*)d.batch.ids.p, sg,
                                     nb, nwaves[k], (uint32_t*)keybuf.p + koff[k], (uint32_t)bucket[k].size() * att_seg,
                                     att_seg, (const LineDev*)d.lines.p, (const uint32_t*)d.pool.p, (const AttDev*)d.atts.p,
                                     (HitDev*)d.batch.hits.p, hitcnt, d.batch.hitcap,
                                     first_key_exit_knob() ? (uint32_t*)d.first_hit.p : nullptr, vc, vsk));
    }
    if (fan) {
        HIPCHK(hipEventRecord(d.vs_done, d.side));
        HIPCHK(hipStreamWaitEvent(s, d.vs_done, 0));
    }
    return 0;
}

// Wait for the derive + verify kernels of one chunk (both streams) and append their hits.
static int collect_hits(Device& d, std::vector<HitDev>& hits_out) {
    PhaseTrace tr;
    hipStream_t s = d.stream;
    RCHK(join_tail(d));
    const uint32_t* hitcnt = (const uint32_t*)d.batch.counters.p + 1;
    RCHK(d.hits_host.ensure(16 + (size_t)d.batch.hitcap * sizeof(HitDev)));
    HIPCHK(launch_hits_out(hitcnt, (const HitDev*)d.batch.hits.p, d.batch.hitcap, (uint32_t*)d.hits_host.dev,
                           (const uint32_t*)d.batch.counters.p + 4, s));
    HIPCHK(hipStreamSynchronize(s));
    tr.mark("  device wait");
    const uint32_t nh = *(volatile const uint32_t*)d.hits_host.p;
    d.stats.tail_waves_raised += *((volatile const uint32_t*)d.hits_host.p + 1);
    if (nh > d.batch.hitcap) return DWPA_E_OVERFLOW;
    size_t old = hits_out.size();
    hits_out.resize(old + nh);
    if (nh) memcpy(hits_out.data() + old, d.hits_host.p + 16, nh * sizeof(HitDev));
    return 0;
}

// Declared right after a call context's lock: when the call returns -- above all on an error after its first
// launch -- every stream of the context has drained before the lock is released, so the next call on this context
// never overwrites staging or device buffers that queued copies and kernels of this one still use.
// The success paths have synchronised already and disarm it.
struct DrainOnExit {
    Device& d;
    bool armed = true;
    ~DrainOnExit() {
        if (!armed) return;
        (void)hipSetDevice(d.id);
        for (hipStream_t s : {d.stream, d.side, d.tail})
            if (s) (void)hipStreamSynchronize(s);
    }
};

// A call context, locked: an idle one of the device with the fewest calls in flight (ties: round-robin from
// g_rr; within a device the lowest context, so one caller keeps reusing context 0's buffers), else wait for the
// first context of the next device in round-robin order.
static Device* pick_device() {
    std::vector<int> act = active_devices();
    if (act.empty()) return nullptr;
    const int K = calls_per_device();
    const uint32_t r0 = g_rr++;
    for (int busy = 0; busy < K; busy++)  // first pass: devices with no call in flight, then one, ...
        for (size_t k = 0; k < act.size(); k++) {
            const int dev = act[(r0 + k) % act.size()];
            int n_busy = 0;
            Device* idle = nullptr;
            for (int c = 0; c < K; c++) {
                Device* d = g_dev[(size_t)dev * K + c].get();
                if (d->mu.try_lock()) {
                    if (!idle) idle = d;
                    else d->mu.unlock();
                } else {
                    n_busy++;
                }
            }
            if (idle && n_busy <= busy) return idle;
            if (idle) idle->mu.unlock();
        }
    Device* d = g_dev[(size_t)act[r0 % act.size()] * K].get();
    d->mu.lock();
    return d;
}

// dwpa_check_last_stats: the calling thread's last check call
static thread_local dwpa_check_stats g_check_stats;
static thread_local bool g_have_check_stats = false;

static int check_batch_body(Device& d, const dwpa_job* jobs, size_t njobs, dwpa_result* out, int* rcs,
                            DrainOnExit& drain);

// The host backend answers the whole call (backend DWPA_BACKEND_HOST_SMALL or _HOST_FALLBACK).
static int check_batch_host(const dwpa_job* jobs, size_t njobs, dwpa_result* out, int* rcs, uint32_t backend,
                            std::chrono::steady_clock::time_point t0) {
    dwpa_check_stats st{};
    st.jobs = (uint32_t)std::min<size_t>(njobs, UINT32_MAX);
    st.backend = backend;
    const int rc = host_check_batch(jobs, njobs, out, rcs, st);
    g_check_stats = st;
    g_check_stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

static int check_batch_device(const dwpa_job* jobs, size_t njobs, dwpa_result* out, int* rcs,
                              std::chrono::steady_clock::time_point t0) {
    RCHK(ensure_init());
    Device* dp = pick_device();
    if (!dp) return DWPA_E_NODEV;
    std::lock_guard<std::mutex> lk(dp->mu, std::adopt_lock);
    DrainOnExit drain{*dp};
    Device& d = *dp;
    d.stats = dwpa_check_stats{};
    d.stats.jobs = (uint32_t)std::min<size_t>(njobs, UINT32_MAX);
    d.stats.backend = DWPA_BACKEND_DEVICE;
    const int rc = check_batch_body(d, jobs, njobs, out, rcs, drain);
    if (rc >= 0) g_device_warm.store(true, std::memory_order_relaxed);
    g_check_stats = d.stats;
    g_check_stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

// Routing: a small call runs on the host without touching the device -- one with PBKDF2 derives and at most
// host_max_pmks PMK-equivalents, or one without derives (caller-PMK checks, common.php:592,606,919) whose verify work
// the host does in tens of microseconds (HOST_VERIFY_MAX compressions: a PMKID check, or an EAPOL window of a few
// dozen attempts; a GPU call costs ~0.1 ms however little it does) -- both 8x larger before the process's first device
// call; every other call on the device, and on the host after a device-side failure when allow_cpu_fallback is on.
// host_max_pmks <= 0 turns both off.
constexpr double HOST_VERIFY_MAX = 1000.0;
static int check_batch_impl(const dwpa_job* jobs, size_t njobs, dwpa_result* out, int* rcs) {
    const auto t0 = std::chrono::steady_clock::now();
    g_check_stats = dwpa_check_stats{};
    g_have_check_stats = true;
    const HostCost hc = host_cost(jobs, njobs);
    const double cold = g_device_warm.load(std::memory_order_relaxed) ? 1.0 : COLD_FACTOR;
    const double thr = host_max_pmks() * cold;
    if (thr > 0 && (hc.derives ? hc.pmk_equiv <= thr : hc.pmk_equiv * 16388.0 <= HOST_VERIFY_MAX * cold))
        return check_batch_host(jobs, njobs, out, rcs, DWPA_BACKEND_HOST_SMALL, t0);
    const int rc = check_batch_device(jobs, njobs, out, rcs, t0);
    if (host_retry_code(rc) && cpu_fallback_on())
        return check_batch_host(jobs, njobs, out, rcs, DWPA_BACKEND_HOST_FALLBACK, t0);
    return rc;
}

static int check_batch_body(Device& d, const dwpa_job* jobs, size_t njobs, dwpa_result* out, int* rcs,
                            DrainOnExit& drain) {
    HIPCHK(hipSetDevice(d.id));
    RCHK(device_stream(d));

    PhaseTrace tr;
    CheckScratch& cs = d.cs;
    cs.parsed.resize(njobs);
    cs.nnz.assign(njobs, 0);
    cs.jbytes.assign(njobs, 0);
    cs.jslot.resize(njobs);
    cs.jbyte.resize(njobs);
    cs.job_pmk.assign(njobs, nullptr);
    // phase 1, per job: parse (PHP rules), count the non-null keys and their bytes
    const size_t TP = host_threads(njobs, 64);
    parallel_for(TP, [&](size_t t) {
        for (size_t j = njobs * t / TP; j < njobs * (t + 1) / TP; j++) {
            out[j].key_index = -1;
            out[j].nc = 0;
            out[j].endian = 0;
            out[j].nc_valid = 0;
            memset(out[j].pmk, 0, 32);
            ParsedLine& pl = cs.parsed[j];
            parse_m22000_into(jobs[j].line, jobs[j].line_len, pl);
            rcs[j] = pl.status;
            if (pl.status) continue;
            rcs[j] = DWPA_MISS;
            cs.job_pmk[j] = jobs[j].pmk;
            if (!line_can_match(pl)) continue;  // PMKID/MIC shorter than 16 bytes never verifies
            if (pl.kind == LINE_EAPOL && jobs[j].nc > DWPA_NC_MAX) {  // attempt tables beyond the documented bound
                rcs[j] = DWPA_E_ARG;
                continue;
            }
            if (jobs[j].nkeys > UINT32_MAX) {      // key indices are 32-bit (SlotTable::kidx)
                rcs[j] = DWPA_E_ARG;
                continue;
            }
            uint32_t c = 0;
            uint64_t by = 0;
            for (size_t k = 0; k < jobs[j].nkeys; k++)
                if (jobs[j].keys[k].ptr) {  // is_null($key): skipped (common.php:172,240)
                    c++;
                    by += jobs[j].keys[k].len;
                }
            cs.nnz[j] = c;
            cs.jbytes[j] = by;
        }
    });
    tr.mark("parse");
    // phase 2: ESSID groups in first-seen order, jobs in input order within a group -> slot and byte bases
    cs.essid_id.clear();
    cs.gid.assign(njobs, UINT32_MAX);
    cs.gstart.clear();
    for (size_t j = 0; j < njobs; j++) {
        if (!cs.nnz[j]) continue;
        auto ins = cs.essid_id.try_emplace(std::string_view(cs.parsed[j].essid), (uint32_t)cs.gstart.size());
        if (ins.second) cs.gstart.push_back(0);
        cs.gid[j] = ins.first->second;
        cs.gstart[cs.gid[j]]++;  // count for now
    }
    const size_t G = cs.gstart.size();
    cs.gstart.push_back(0);
    for (size_t g = 0, acc = 0; g <= G; g++) {  // counts -> starts
        const size_t c = cs.gstart[g];
        cs.gstart[g] = (uint32_t)acc;
        acc += c;
    }
    cs.order.resize(cs.gstart[G]);
    cs.gfill.assign(cs.gstart.begin(), cs.gstart.end() - 1);
    for (size_t j = 0; j < njobs; j++)
        if (cs.gid[j] != UINT32_MAX) cs.order[cs.gfill[cs.gid[j]]++] = (uint32_t)j;
    cs.gslot.resize(G + 1);
    size_t nslots = 0, nbytes = 0;
    for (size_t g = 0; g < G; g++) {
        cs.gslot[g] = (uint32_t)nslots;
        for (uint32_t q = cs.gstart[g]; q < cs.gstart[g + 1]; q++) {
            const uint32_t j = cs.order[q];
            cs.jslot[j] = (uint32_t)nslots;
            cs.jbyte[j] = nbytes;
            nslots += cs.nnz[j];
            nbytes += cs.jbytes[j];
        }
    }
    cs.gslot[G] = (uint32_t)nslots;
    d.stats.slots = (uint32_t)std::min<size_t>(nslots, UINT32_MAX);
    if (!nslots) return 0;
    if (nslots >= SLOT_CALLER) return DWPA_E_ARG;
    tr.mark("essid groups");
    // phase 3, per job: the job's keys ($HEX[] decoded) into its byte range of the pinned key bytes, slot records
    SlotTable& T = d.slots;
    RCHK(T.reserve(nslots, nbytes));
    const size_t TS = host_threads(nslots, 8192);
    parallel_for(TS, [&](size_t t) {
        std::string dec;
        const size_t q0 = std::upper_bound(cs.order.begin(), cs.order.end(), nslots * t / TS,
                                           [&](size_t v, uint32_t j) { return v < cs.jslot[j]; }) - cs.order.begin();
        const size_t q1 = std::upper_bound(cs.order.begin(), cs.order.end(), nslots * (t + 1) / TS,
                                           [&](size_t v, uint32_t j) { return v < cs.jslot[j]; }) - cs.order.begin();
        // thread t takes the jobs whose first slot s has lo_t < s <= lo_{t+1} (lo_t = nslots * t / TS; thread 0
        // also slot 0): contiguous runs of `order` with about nslots / TS slots each
        for (size_t q = t ? q0 : 0; q < (t + 1 == TS ? cs.order.size() : q1); q++) {
            const uint32_t j = cs.order[q];
            const dwpa_job& J = jobs[j];
            size_t si = cs.jslot[j];
            uint64_t pos = cs.jbyte[j];
            uint32_t o = 0;
            for (size_t k = 0; k < J.nkeys; k++) {
                // caller keys are scattered (one PHP string / Python bytes object each): prefetch ahead
                if (k + 16 < J.nkeys && J.keys[k + 16].ptr) __builtin_prefetch(J.keys[k + 16].ptr);
                const dwpa_bytes& kb = J.keys[k];
                if (!kb.ptr) continue;
                const uint8_t* src = kb.ptr;
                size_t len = kb.len;
                if (starts_hex(kb.ptr, kb.len)) {
                    dec = hc_unhex(std::string((const char*)kb.ptr, kb.len));
                    src = (const uint8_t*)dec.data();
                    len = dec.size();  // <= kb.len
                }
                T.hash[si] = hash_key(src, len);
                memcpy(T.kbytes + pos, src, len);
                T.koff[si] = pos;
                T.klen[si] = (uint32_t)len;
                T.job[si] = j;
                T.ord[si] = o | (o == 0 && cs.job_pmk[j] ? SLOT_CALLER : 0u);
                T.kidx[si] = (uint32_t)k;
                pos += len;
                si++;
                o++;
            }
        }
    });
    // the key bytes go up now, while the host deduplicates (derive_slots): the first kernel waits for them
    RCHK(upload_slot_keys(d, T));
    tr.mark("slots");

    // The first chunk's PBKDF2 is queued before the line tables exist: the host builds them while the GPU derives.
    // The builder is the context's (cleared, capacity kept): a fresh one per call mapped and zero-faulted its
    // ~7 MB of attempt records every call and unmapped them on return.
    TableBuilder& tb = d.tb;
    tb.lines.clear();
    tb.atts.clear();
    tb.pool.clear();
    tb.never.clear();
    tb.att_kw_all = false;
    std::vector<uint32_t> job_line(njobs, 0);
    std::vector<HitDev> hits;
    const size_t chunk = default_batch();
    // first-key early exit of the attempt-parallel verify (queue_verify): one word per line, reset before the first
    // kernel of the call; the tail stream's kernels wait for this stream's prep event, queued after it
    RCHK(d.first_hit.ensure(std::max<size_t>(njobs, 1) * 4));
    HIPCHK(hipMemsetAsync(d.first_hit.p, 0xff, njobs * 4, d.stream));
    for (size_t b = 0; b < nslots; b += chunk) {
        const size_t e = std::min(nslots, b + chunk);
        // the ESSID runs of [b, e) are the groups' slot ranges clipped to it
        std::vector<uint32_t> runs{0};
        std::vector<const std::string*> run_essid;
        for (size_t g = 0; g < G; g++) {
            if (cs.gslot[g + 1] <= b || cs.gslot[g] >= e) continue;
            if (cs.gslot[g] > b) runs.push_back((uint32_t)(cs.gslot[g] - b));
            run_essid.push_back(&cs.parsed[cs.order[cs.gstart[g]]].essid);
        }
        runs.push_back((uint32_t)(e - b));
        DeriveStage st;
        RCHK(derive_slots(d, T, b, e, cs.job_pmk, runs, run_essid, false, st, true));
        if (b == 0) {
            for (uint32_t j : cs.order) job_line[j] = tb.add_line(cs.parsed[j], jobs[j].nc, DWPA_NC_PHP, 0);
            tr.mark("tables (overlapped)");
        }
        RCHK(finish_derive(d, st));
        // the tail slots' verify first: its segment upload goes up the side stream ahead of the head's keyver-3
        // verify, which that stream then runs (fan-out)
        RCHK(queue_verify(d, T, b, b + st.split, e, job_line, tb, b == 0, d.tail, d.segs_tail, d.keys_tail, false));
        RCHK(queue_verify(d, T, b, b, b + st.split, job_line, tb, false, d.stream, d.segs, d.keys, true));
        tr.mark("  verify queued");
        RCHK(collect_hits(d, hits));
    }
    tr.mark("device");

    // first key in input order wins, then the first attempt in PHP order (common.php:186,280-289)
    std::unordered_map<uint32_t, uint32_t> line_job;
    for (uint32_t j : cs.order) line_job[job_line[j]] = j;
    std::vector<int64_t> best(njobs, -1);
    std::vector<uint32_t> best_att(njobs, 0);
    std::vector<const HitDev*> best_hit(njobs, nullptr);
    for (const HitDev& h : hits) {
        auto it = line_job.find(h.line);
        if (it == line_job.end()) continue;
        const size_t j = it->second;
        if (best[j] < 0 || (int64_t)h.cand < best[j] || ((int64_t)h.cand == best[j] && h.attempt < best_att[j])) {
            best[j] = (int64_t)h.cand;
            best_att[j] = h.attempt;
            best_hit[j] = &h;
        }
    }
    for (size_t j = 0; j < njobs; j++) {
        if (best[j] < 0) continue;
        const LineDev& L = tb.lines[job_line[j]];
        rcs[j] = DWPA_HIT;
        d.stats.hits++;
        out[j].key_index = (int32_t)T.kidx[cs.jslot[j] + (size_t)best[j]];  // ordinal -> the caller's index
        pmk_bytes(best_hit[j]->pmk, out[j].pmk);
        if (L.kind == LINE_PMKID) {
            out[j].nc_valid = 0;
        } else {
            const uint32_t list = (uint32_t)std::min<int64_t>(best[j], (int64_t)L.nlists - 1);
            const AttDev& at = tb.atts[L.list_off + list * L.natt + best_att[j]];
            out[j].nc_valid = 1;
            out[j].nc = at.nc;
            out[j].endian = (int8_t)at.endian;
        }
    }
    tr.mark("results");
    drain.armed = false;  // collect_hits synchronised every stream of this call
    return 0;
}

static int pbkdf2_device(const dwpa_bytes* keys, size_t nkeys, const uint8_t* essid, size_t essid_len, uint8_t* out);

// dwpa_pbkdf2_pmk: the check path's routing (a small derive on the host, the device otherwise, the host again after a
// device-side failure when allow_cpu_fallback is on).
static int pbkdf2_impl(const dwpa_bytes* keys, size_t nkeys, const uint8_t* essid, size_t essid_len, uint8_t* out) {
    const double thr = host_max_pmks() * (g_device_warm.load(std::memory_order_relaxed) ? 1.0 : COLD_FACTOR);
    if ((double)nkeys <= thr) return host_pbkdf2(keys, nkeys, essid, essid_len, out);
    const int rc = pbkdf2_device(keys, nkeys, essid, essid_len, out);
    if (rc >= 0) g_device_warm.store(true, std::memory_order_relaxed);
    if (host_retry_code(rc) && cpu_fallback_on()) return host_pbkdf2(keys, nkeys, essid, essid_len, out);
    return rc;
}

static int pbkdf2_device(const dwpa_bytes* keys, size_t nkeys, const uint8_t* essid, size_t essid_len, uint8_t* out) {
    RCHK(ensure_init());
    Device* dp = pick_device();
    if (!dp) return DWPA_E_NODEV;
    std::lock_guard<std::mutex> lk(dp->mu, std::adopt_lock);
    DrainOnExit drain{*dp};
    Device& d = *dp;
    HIPCHK(hipSetDevice(d.id));
    RCHK(device_stream(d));
    if (nkeys >= SLOT_CALLER) return DWPA_E_ARG;
    const std::string es((const char*)essid, essid_len);
    SlotTable& T = d.slots;
    size_t nbytes = 0;
    for (size_t i = 0; i < nkeys; i++) nbytes += keys[i].ptr ? keys[i].len : 0;
    RCHK(T.reserve(nkeys, nbytes));
    uint64_t pos = 0;
    for (size_t i = 0; i < nkeys; i++) {  // a null key derives as the empty key
        const size_t len = keys[i].ptr ? keys[i].len : 0;
        T.hash[i] = hash_key(keys[i].ptr, len);
        if (len) memcpy(T.kbytes + pos, keys[i].ptr, len);
        T.koff[i] = pos;
        T.klen[i] = (uint32_t)len;
        T.job[i] = 0;
        T.ord[i] = (uint32_t)i;
        T.kidx[i] = (uint32_t)i;
        pos += len;
    }
    const size_t chunk = default_batch();
    std::vector<const uint8_t*> jp(1, nullptr);
    for (size_t b = 0; b < nkeys; b += chunk) {
        const size_t e = std::min(nkeys, b + chunk);
        DeriveStage st;
        RCHK(derive_slots(d, T, b, e, jp, {0u, (uint32_t)(e - b)}, {&es}, b == 0, st, true));
        RCHK(finish_derive(d, st));
        RCHK(join_tail(d));
        std::vector<uint32_t> w((size_t)PMK_WORDS * d.batch.cap);
        HIPCHK(hipMemcpyAsync(w.data(), d.batch.pmk.p, w.size() * 4, hipMemcpyDeviceToHost, d.stream));
        HIPCHK(hipStreamSynchronize(d.stream));
        for (size_t i = 0; i < e - b; i++) {
            uint32_t pw[8];
            for (int k = 0; k < 8; k++) pw[k] = w[(size_t)k * d.batch.cap + i];
            pmk_bytes(pw, out + 32 * (b + i));
        }
    }
    return 0;
}

// ---------------------------------------------------------------------------------------------------------
// scan API
// ---------------------------------------------------------------------------------------------------------
struct ScanGroup {
    std::string essid;
    uint32_t line_begin = 0, line_end = 0;  // contiguous in the line table
    uint32_t salt_off = 0, nsalt = 0;
};

}  // namespace dwpa

struct dwpa_scan {
    int device = 0;
    int nc_mode = 0;
    dwpa::TableBuilder tb;
    std::vector<int> status;              // per input line
    std::vector<uint32_t> line_of;        // input line -> table line (valid when status == 0)
    std::vector<uint32_t> input_of;       // table line -> input line
    std::vector<dwpa::ScanGroup> groups;
    std::vector<uint8_t> cracked;         // per table line (crack_files stops re-checking cracked lines)
    dwpa::DevBuf lines, atts, pool, salt, segs;
    dwpa::Batch batch;
    uint32_t batch_cap = 0;
    // scan_run (many ESSID groups per PBKDF2 launch): rebuilt when the set of uncracked lines changes
    struct Chunk {
        uint32_t g0, ngroups, list0, nlines;
        uint32_t cls[5];  // the chunk's lines of verify class index c are list[list0 + cls[c], list0 + cls[c+1])
    };
    bool mg_dirty = true;
    uint32_t mg_stride = 0;                // PMK SoA stride = (most groups in one launch) x batch_cap
    std::vector<Chunk> mg_chunks;
    std::vector<uint32_t> mg_gsalt_h, mg_list_h, mg_poff_h;
    dwpa::DevBuf mg_pmk, mg_gsalt, mg_list, mg_poff;
};

namespace dwpa {

static hipStream_t as_stream(void* s) { return (hipStream_t)s; }

int scan_create(int device, const char* const* lines, const size_t* lens, size_t nlines, int nc, int nc_mode,
                uint32_t batch, dwpa_scan** out) {
    RCHK(ensure_init());
    if (device < 0 || device >= g_ndev || !out || batch == 0 || nc > DWPA_NC_MAX) return DWPA_E_ARG;
    HIPCHK(hipSetDevice(device));
    auto sc = std::make_unique<dwpa_scan>();
    sc->device = device;
    sc->nc_mode = nc_mode;
    sc->status.resize(nlines);
    sc->line_of.assign(nlines, 0);
    std::vector<ParsedLine> parsed(nlines);
    std::map<std::string, std::vector<size_t>> by_essid;
    sc->tb.att_kw_all = true;  // scans verify key-parallel only: every attempt needs its KW blocks
    for (size_t i = 0; i < nlines; i++) {
        parsed[i] = parse_m22000(lines[i], lens[i]);
        sc->status[i] = parsed[i].status;
        if (!parsed[i].status) by_essid[parsed[i].essid].push_back(i);
    }
    std::vector<uint32_t> salts;
    for (auto& kv : by_essid) {
        ScanGroup g;
        g.essid = kv.first;
        g.line_begin = (uint32_t)sc->tb.lines.size();
        // lines of a group ordered by verify class, so that each class is one contiguous run (one kernel each)
        auto cls = [&](size_t i) {
            return parsed[i].kind == LINE_PMKID ? 0 : parsed[i].keyver;
        };
        std::stable_sort(kv.second.begin(), kv.second.end(), [&](size_t x, size_t y) { return cls(x) < cls(y); });
        for (size_t i : kv.second) {
            sc->line_of[i] = sc->tb.add_line(parsed[i], nc, nc_mode, nc);
            sc->input_of.push_back((uint32_t)i);
        }
        g.line_end = (uint32_t)sc->tb.lines.size();
        std::vector<uint32_t> sb;
        g.nsalt = build_salt_blocks(g.essid, sb);
        g.salt_off = (uint32_t)salts.size();
        salts.insert(salts.end(), sb.begin(), sb.end());
        sc->groups.push_back(g);
    }
    sc->cracked.assign(sc->tb.lines.size(), 0);
    for (size_t l = 0; l < sc->tb.never.size(); l++)
        if (sc->tb.never[l]) sc->cracked[l] = 1;  // can never match: never verified
    RCHK(upload(sc->lines, sc->tb.lines, nullptr));
    RCHK(upload(sc->atts, sc->tb.atts, nullptr));
    RCHK(upload(sc->pool, sc->tb.pool, nullptr));
    RCHK(upload(sc->salt, salts, nullptr));
    batch = (batch + 63) & ~63u;
    RCHK(sc->batch.reserve(batch, std::max<uint32_t>(batch, 1u << 16)));
    sc->batch_cap = batch;
    HIPCHK(hipMemset(sc->batch.counters.p, 0, 16));
    HIPCHK(hipDeviceSynchronize());
    *out = sc.release();
    return 0;
}

void scan_destroy(dwpa_scan* sc) {
    if (!sc) return;
    scan_rules_drop(sc);
    (void)hipSetDevice(sc->device);
    (void)hipDeviceSynchronize();
    sc->lines.release(); sc->atts.release(); sc->pool.release(); sc->salt.release(); sc->segs.release();
    sc->mg_pmk.release(); sc->mg_gsalt.release(); sc->mg_list.release(); sc->mg_poff.release();
    sc->batch.mid.release(); sc->batch.pmk.release(); sc->batch.ids.release(); sc->batch.hits.release();
    sc->batch.counters.release();
    delete sc;
}

int scan_load_dict(dwpa_scan* sc, const uint64_t* off, const uint8_t* bytes, uint64_t first, uint32_t count,
                   uint32_t minlen, uint32_t maxlen, void* stream, bool fill) {
    if (!sc || count > (fill ? 16 * (uint64_t)sc->batch_cap : sc->batch_cap)) return DWPA_E_ARG;
    HIPCHK(hipSetDevice(sc->device));
    hipStream_t s = as_stream(stream);
    HIPCHK(hipMemsetAsync(sc->batch.counters.p, 0, 4, s));
    HIPCHK(launch_prep_dict(off, bytes, first, count, minlen, maxlen, (uint32_t*)sc->batch.mid.p,
                            (uint64_t*)sc->batch.ids.p, (uint32_t*)sc->batch.counters.p, sc->batch_cap, true, s));
    return 0;
}

int scan_counter_raw(dwpa_scan* sc, void* stream, uint32_t* raw) {
    HIPCHK(hipSetDevice(sc->device));
    hipStream_t s = as_stream(stream);
    HIPCHK(hipMemcpyAsync(raw, sc->batch.counters.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

int scan_load_numeric(dwpa_scan* sc, uint64_t first, uint32_t count, uint32_t digits, void* stream) {
    if (!sc || count > sc->batch_cap || digits == 0 || digits > 20) return DWPA_E_ARG;
    HIPCHK(hipSetDevice(sc->device));
    hipStream_t s = as_stream(stream);
    HIPCHK(hipMemcpyAsync(sc->batch.counters.p, &count, 4, hipMemcpyHostToDevice, s));
    HIPCHK(launch_prep_numeric(first, count, digits, (uint32_t*)sc->batch.mid.p, (uint64_t*)sc->batch.ids.p,
                               sc->batch_cap, s));
    HIPCHK(hipStreamSynchronize(s));  // `count` lives on this host stack frame
    return 0;
}

int scan_pbkdf2(dwpa_scan* sc, int group, void* stream) {
    if (!sc || group < 0 || group >= (int)sc->groups.size()) return DWPA_E_ARG;
    HIPCHK(hipSetDevice(sc->device));
    const ScanGroup& g = sc->groups[group];
    bool any = false;
    for (uint32_t l = g.line_begin; l < g.line_end; l++) any |= !sc->cracked[l];
    if (!any) return 0;
    HIPCHK(launch_pbkdf2((const uint32_t*)sc->batch.mid.p, sc->batch_cap, 0, sc->batch_cap,
                         (const uint32_t*)sc->batch.counters.p, (const uint32_t*)sc->salt.p + g.salt_off, g.nsalt,
                         (uint32_t*)sc->batch.pmk.p, as_stream(stream), (uint32_t*)sc->batch.counters.p + 2));
    return 0;
}

int scan_verify(dwpa_scan* sc, int group, void* stream) {
    if (!sc || group < 0 || group >= (int)sc->groups.size()) return DWPA_E_ARG;
    HIPCHK(hipSetDevice(sc->device));
    const ScanGroup& g = sc->groups[group];
    const uint32_t nsegs = sc->batch_cap / 64;
    // contiguous runs of uncracked lines of one verify class -> implicit-segment launches
    for (uint32_t l = g.line_begin; l < g.line_end;) {
        if (sc->cracked[l]) { l++; continue; }
        const uint32_t vc = verify_class(sc->tb.lines[l]);
        uint32_t e = l;
        while (e < g.line_end && !sc->cracked[e] && verify_class(sc->tb.lines[e]) == vc) e++;
        HIPCHK(launch_verify((const uint32_t*)sc->batch.pmk.p, sc->batch_cap, (const uint64_t*)sc->batch.ids.p,
                             (const uint32_t*)sc->batch.counters.p, nullptr, nsegs, l, e - l,
                             (const LineDev*)sc->lines.p, (const uint32_t*)sc->pool.p, (const AttDev*)sc->atts.p,
                             (HitDev*)sc->batch.hits.p, (uint32_t*)sc->batch.counters.p + 1, sc->batch.hitcap,
                             vc, as_stream(stream)));
        l = e;
    }
    return 0;
}

// Candidate slots per multi-group PBKDF2 launch (x2 lanes for the two output blocks).  The 1024 SIMDs hold 512K
// lanes at 8 waves, and every lane runs the same 4096 iterations, so a launch takes ceil(lanes / 512K) wave
// rounds: 16M slots = 64 rounds keeps a partial last round under ~2 %, and bounds the group-major PMK buffer
// at 512 MiB of the 288 GB.
constexpr uint64_t MG_SLOTS = 1u << 24;

static int scan_mg_rebuild(dwpa_scan* sc, hipStream_t s) {
    const uint32_t cap = sc->batch_cap;
    HIPCHK(hipStreamSynchronize(s));  // the previous tables may still be read by queued launches
    const uint32_t per = (uint32_t)std::max<uint64_t>(1, MG_SLOTS / cap);
    std::vector<const ScanGroup*> act;
    for (const ScanGroup& g : sc->groups) {
        bool any = false;
        for (uint32_t l = g.line_begin; l < g.line_end; l++) any |= !sc->cracked[l];
        if (any) act.push_back(&g);
    }
    // spread the active groups evenly over the launches: sizes differ by at most one (no small last launch)
    const uint32_t nact = (uint32_t)act.size();
    const uint32_t launches = (nact + per - 1) / per;
    sc->mg_chunks.clear();
    sc->mg_gsalt_h.clear();
    sc->mg_list_h.clear();
    sc->mg_poff_h.assign(std::max<size_t>(sc->tb.lines.size(), 1), 0);
    uint32_t most = 0, next = 0;
    for (uint32_t c = 0; c < launches; c++) {
        const uint32_t size = nact / launches + (c < nact % launches ? 1u : 0u);
        dwpa::ScanGroup const* const* grp = act.data() + next;
        dwpa_scan::Chunk ch{(uint32_t)sc->mg_gsalt_h.size() / 2, size, (uint32_t)sc->mg_list_h.size(), 0, {}};
        for (uint32_t k = 0; k < size; k++) {
            sc->mg_gsalt_h.push_back(grp[k]->salt_off);
            sc->mg_gsalt_h.push_back(grp[k]->nsalt);
        }
        for (uint32_t vc = 0; vc < 4; vc++) {
            ch.cls[vc] = (uint32_t)sc->mg_list_h.size() - ch.list0;
            for (uint32_t k = 0; k < size; k++)
                for (uint32_t l = grp[k]->line_begin; l < grp[k]->line_end; l++) {
                    if (sc->cracked[l] || verify_class(sc->tb.lines[l]) != (1u << vc)) continue;
                    sc->mg_list_h.push_back(l);
                    sc->mg_poff_h[l] = k * cap;
                }
        }
        next += size;
        ch.nlines = (uint32_t)sc->mg_list_h.size() - ch.list0;
        ch.cls[4] = ch.nlines;
        most = std::max(most, size);
        sc->mg_chunks.push_back(ch);
    }
    sc->mg_stride = most * cap;
    if (most) RCHK(sc->mg_pmk.ensure((size_t)PMK_WORDS * sc->mg_stride * 4));
    RCHK(upload(sc->mg_gsalt, sc->mg_gsalt_h, s));
    RCHK(upload(sc->mg_list, sc->mg_list_h, s));
    RCHK(upload(sc->mg_poff, sc->mg_poff_h, s));
    sc->mg_dirty = false;
    return 0;
}

int scan_run(dwpa_scan* sc, void* stream) {
    if (!sc) return DWPA_E_ARG;
    HIPCHK(hipSetDevice(sc->device));
    hipStream_t s = as_stream(stream);
    if (sc->mg_dirty) RCHK(scan_mg_rebuild(sc, s));
    const uint32_t cap = sc->batch_cap;
    const uint32_t pstride = sc->mg_stride;
    for (const dwpa_scan::Chunk& ch : sc->mg_chunks) {
        // every (group, slot) PMK of this launch must land inside mg_pmk: [8][pstride] words
        if ((uint64_t)ch.ngroups * cap > pstride || sc->mg_pmk.n < (size_t)PMK_WORDS * pstride * 4) return DWPA_E_ARG;
        HIPCHK(launch_pbkdf2_mg((const uint32_t*)sc->batch.mid.p, cap, (const uint32_t*)sc->batch.counters.p,
                                ch.ngroups, (const uint32_t*)sc->salt.p, (const uint32_t*)sc->mg_gsalt.p + 2 * ch.g0,
                                (uint32_t*)sc->mg_pmk.p, pstride, s, (uint32_t*)sc->batch.counters.p + 2));
        for (uint32_t c = 0; c < 4; c++)  // one launch per verify class (grid.y <= 65535 lines)
            for (uint32_t l = ch.cls[c]; l < ch.cls[c + 1]; l += 65535u) {
                const uint32_t nl = std::min<uint32_t>(65535u, ch.cls[c + 1] - l);
                HIPCHK(launch_verify((const uint32_t*)sc->mg_pmk.p, cap, (const uint64_t*)sc->batch.ids.p,
                                     (const uint32_t*)sc->batch.counters.p, nullptr, cap / 64, ch.list0 + l, nl,
                                     (const LineDev*)sc->lines.p, (const uint32_t*)sc->pool.p,
                                     (const AttDev*)sc->atts.p, (HitDev*)sc->batch.hits.p,
                                     (uint32_t*)sc->batch.counters.p + 1, sc->batch.hitcap, 1u << c, s,
                                     (const uint32_t*)sc->mg_list.p, (const uint32_t*)sc->mg_poff.p, pstride));
            }
    }
    return 0;
}

int scan_hits_raw(dwpa_scan* sc, std::vector<HitDev>& out, void* stream) {
    HIPCHK(hipSetDevice(sc->device));
    hipStream_t s = as_stream(stream);
    uint32_t nh = 0;
    HIPCHK(hipMemcpyAsync(&nh, (uint32_t*)sc->batch.counters.p + 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (nh > sc->batch.hitcap) return DWPA_E_OVERFLOW;
    out.resize(nh);
    if (nh) HIPCHK(hipMemcpyAsync(out.data(), sc->batch.hits.p, nh * sizeof(HitDev), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemsetAsync((uint32_t*)sc->batch.counters.p + 1, 0, 4, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

void hit_to_public(const dwpa_scan* sc, const HitDev& h, dwpa_hit& o) {
    const LineDev& L = sc->tb.lines[h.line];
    memset(&o, 0, sizeof(o));
    o.cand = h.cand;
    o.line = sc->input_of[h.line];
    pmk_bytes(h.pmk, o.pmk);
    if (L.kind == LINE_EAPOL) {
        const uint32_t list = (uint32_t)std::min<uint64_t>(h.cand, (uint64_t)L.nlists - 1);
        const AttDev& at = sc->tb.atts[L.list_off + list * L.natt + h.attempt];
        o.nc_valid = 1;
        o.nc = at.nc;
        o.endian = (int8_t)at.endian;
    }
}

void scan_mark_cracked(dwpa_scan* sc, uint32_t input_line) {
    if (input_line < sc->status.size() && sc->status[input_line] == 0 && !sc->cracked[sc->line_of[input_line]]) {
        sc->cracked[sc->line_of[input_line]] = 1;
        sc->mg_dirty = true;
    }
}
uint32_t scan_batch_cap(const dwpa_scan* sc) { return sc->batch_cap; }
Batch& scan_batch_ref(dwpa_scan* sc) { return sc->batch; }
int scan_device(const dwpa_scan* sc) { return sc->device; }

// ---------------------------------------------------------------------------------------------------------
// helpers for crack.cpp
// ---------------------------------------------------------------------------------------------------------
int engine_init() { return ensure_init(); }
int engine_rule_mode() {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (g_rule_mode == DWPA_RULES_HASHCAT || g_rule_mode == DWPA_RULES_FULL) return g_rule_mode;
    }
    const char* e = getenv("DWPA_RULE_MODE");
    return e && strcmp(e, "full") == 0 ? DWPA_RULES_FULL : DWPA_RULES_HASHCAT;
}
std::vector<int> engine_devices(uint32_t mask) { return active_devices(mask); }
uint32_t engine_batch() { return default_batch(); }

}  // namespace dwpa

// =========================================================================================================
// C ABI
// =========================================================================================================
using namespace dwpa;

extern "C" {

int dwpa_abi_version(void) { return DWPA_ABI_VERSION; }

int dwpa_init(const dwpa_config* cfg) {
    return guarded([&]() -> int {
        if (cfg && cfg->struct_size && cfg->struct_size < sizeof(uint32_t) * 3) return DWPA_E_ARG;
        if (DWPA_CFG_HAS(cfg, rule_mode) && (cfg->rule_mode < DWPA_RULES_DEFAULT || cfg->rule_mode > DWPA_RULES_FULL))
            return DWPA_E_ARG;
        if (DWPA_CFG_HAS(cfg, allow_cpu_fallback) && (cfg->allow_cpu_fallback < -1 || cfg->allow_cpu_fallback > 1))
            return DWPA_E_ARG;
        {
            std::lock_guard<std::mutex> lk(g_mu);
            init_locked(cfg, false);
        }
        // With the host backend allowed the library answers check and PBKDF2 calls with or without a device, so the
        // device is probed at the first call that needs it: a PHP-FPM worker whose calls all stay on the host backend
        // never starts the HIP runtime (0.1-0.2 s and ~60 MiB of RSS, more once queues exist).
        if (cpu_fallback_on()) return 0;
        std::lock_guard<std::mutex> lk(g_mu);
        return init_locked(nullptr);
    });
}

int dwpa_device_count(void) {
    return guarded([&]() -> int {
        int r = ensure_init();
        return r < 0 ? r : g_ndev;
    });
}

const char* dwpa_strerror(int code) {
    switch (code) {
    case DWPA_MISS: return "no match";
    case DWPA_HIT: return "match";
    case DWPA_E_FORMAT: return "malformed hashline (need 9 '*'-separated fields starting with WPA)";
    case DWPA_E_HEX: return "hashline field is not valid hex";
    case DWPA_E_TYPE: return "hashline type is neither 01 (PMKID) nor 02 (EAPOL)";
    case DWPA_E_KEYVER: return "unsupported EAPOL key version";
    case DWPA_E_NODEV: return "no usable gfx950 device";
    case DWPA_E_HIP: return hipGetErrorString(t_last_hip);
    case DWPA_E_ARG: return "invalid argument";
    case DWPA_E_NOMEM: return "out of memory";
    case DWPA_E_IO: return "I/O error";
    case DWPA_E_OVERFLOW: return "hit buffer overflow";
    case DWPA_E_RULE: return "unsupported or malformed rule";
    default: return "unknown error";
    }
}

void dwpa_shutdown(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto& d : g_dev) {
        std::lock_guard<std::mutex> dl(d->mu);
        (void)hipSetDevice(d->id);
        (void)hipDeviceSynchronize();
        for (DevBuf* b : {&d->lines, &d->atts, &d->pool, &d->segs, &d->segs_tail, &d->keys, &d->keys_tail, &d->salt,
                          &d->first_hit,
                          &d->koff, &d->klen, &d->kbytes, &d->uslot, &d->upmk, &d->sref, &d->src, &d->cpmk,
                          &d->batch.mid, &d->batch.pmk, &d->batch.ids, &d->batch.hits, &d->batch.counters})
            b->release();
        d->batch.cap = d->batch.hitcap = 0;
        d->stage.release();
        d->slots.mem.release();
        d->slots.n = d->slots.nbytes = 0;
        d->hits_host.release();
        if (d->head_end) (void)hipEventDestroy(d->head_end);
        d->head_end = nullptr;
        if (d->vs_go) (void)hipEventDestroy(d->vs_go);
        if (d->vs_done) (void)hipEventDestroy(d->vs_done);
        d->vs_go = d->vs_done = nullptr;
        if (d->stream) (void)hipStreamDestroy(d->stream);
        if (d->side) (void)hipStreamDestroy(d->side);
        if (d->side_done) (void)hipEventDestroy(d->side_done);
        if (d->tail) (void)hipStreamDestroy(d->tail);
        if (d->head_done) (void)hipEventDestroy(d->head_done);
        if (d->tail_done) (void)hipEventDestroy(d->tail_done);
        if (d->prep_done) (void)hipEventDestroy(d->prep_done);
        d->stream = d->side = d->tail = nullptr;
        d->side_done = d->head_done = d->tail_done = d->prep_done = nullptr;
    }
    g_dev.clear();
    g_fence.clear();
    g_init = false;
}

int dwpa_check_m22000(const char* line, size_t line_len, const dwpa_bytes* keys, size_t nkeys, const uint8_t* pmk,
                      int nc, dwpa_result* out) {
    return guarded([&]() -> int {
        if (!line || (!keys && nkeys) || !out) return DWPA_E_ARG;
        dwpa_job j{line, line_len, keys, nkeys, pmk, nc};
        int rc = 0;
        int r = check_batch_impl(&j, 1, out, &rc);
        return r < 0 ? r : rc;
    });
}

int dwpa_check_batch(const dwpa_job* jobs, size_t njobs, dwpa_result* out, int* rcs) {
    return guarded([&]() -> int {
        if ((!jobs || !out || !rcs) && njobs) return DWPA_E_ARG;
        if (njobs == 0) return 0;
        return check_batch_impl(jobs, njobs, out, rcs);
    });
}

int dwpa_resource_stats(dwpa_resources* out) {
    return guarded([&]() -> int {
        if (!out) return DWPA_E_ARG;
        memset(out, 0, sizeof(*out));
        out->device_bytes = g_dev_bytes.load();
        out->pinned_host_bytes = g_pinned_bytes.load();
        out->host_pool_threads = (uint32_t)HostPool::get().workers();
        std::lock_guard<std::mutex> lk(g_mu);
        out->devices = (uint32_t)g_ndev;
        for (auto& d : g_dev)
            if (d->used.load(std::memory_order_acquire)) out->call_contexts_used++;
        out->call_contexts = (uint32_t)g_dev.size();
        return 0;
    });
}

int dwpa_check_last_stats(dwpa_check_stats* out) {
    if (!out || !dwpa::g_have_check_stats) return DWPA_E_ARG;
    *out = dwpa::g_check_stats;
    return 0;
}

int dwpa_pbkdf2_pmk(const dwpa_bytes* keys, size_t nkeys, const uint8_t* essid, size_t essid_len, uint8_t* pmks_out) {
    return guarded([&]() -> int {
        if ((!keys && nkeys) || (!essid && essid_len) || (!pmks_out && nkeys)) return DWPA_E_ARG;
        if (nkeys == 0) return 0;
        return pbkdf2_impl(keys, nkeys, essid, essid_len, pmks_out);
    });
}

int dwpa_parse_m22000(const char* line, size_t line_len, int nc, int nc_mode, dwpa_line_info* out) {
    return guarded([&]() -> int {
        if (!line || !out) return DWPA_E_ARG;
        memset(out, 0, sizeof(*out));
        ParsedLine p = parse_m22000(line, line_len);
        if (p.status) return p.status;
        if (p.kind == LINE_EAPOL && nc > DWPA_NC_MAX) return DWPA_E_ARG;
        TableBuilder tb;
        const uint32_t li = tb.add_line(p, nc, nc_mode, nc);
        const LineDev& L = tb.lines[li];
        out->type = p.kind;
        out->keyver = p.keyver;
        out->essid_len = (uint32_t)p.essid.size();
        out->mac_ap_len = (uint32_t)p.mac_ap.size();
        out->mac_sta_len = (uint32_t)p.mac_sta.size();
        out->target_len = (uint32_t)(p.kind == LINE_PMKID ? p.pmkid.size() : p.keymic.size());
        out->attempts = p.kind == LINE_PMKID ? 1 : L.natt;
        out->lists = p.kind == LINE_PMKID ? 1 : L.nlists;
        out->never_matches = tb.never[li];
        memcpy(out->essid, p.essid.data(), std::min<size_t>(32, p.essid.size()));
        memcpy(out->mac_ap, p.mac_ap.data(), std::min<size_t>(16, p.mac_ap.size()));
        memcpy(out->mac_sta, p.mac_sta.data(), std::min<size_t>(16, p.mac_sta.size()));
        dwpa_hash_m22000(line, line_len, out->hash_m22000);
        return 0;
    });
}

int dwpa_hc_unhex(const uint8_t* in, size_t in_len, uint8_t* out, size_t* out_len) {
    return guarded([&]() -> int {
        if ((!in && in_len) || !out || !out_len) return DWPA_E_ARG;
        std::string r = hc_unhex(std::string((const char*)in, in_len));
        memcpy(out, r.data(), r.size());
        *out_len = r.size();
        return 0;
    });
}

int dwpa_scan_create(int device, const char* const* lines, const size_t* line_lens, size_t nlines, int nc,
                     int nc_mode, uint32_t batch, dwpa_scan** out) {
    return guarded([&]() -> int {
        if ((!lines || !line_lens) && nlines) return DWPA_E_ARG;
        return scan_create(device, lines, line_lens, nlines, nc, nc_mode, batch, out);
    });
}
int dwpa_scan_num_groups(const dwpa_scan* scan) { return scan ? (int)scan->groups.size() : DWPA_E_ARG; }
int dwpa_scan_line_status(const dwpa_scan* scan, size_t line) {
    if (!scan || line >= scan->status.size()) return DWPA_E_ARG;
    return scan->status[line];
}
int dwpa_scan_load_dict(dwpa_scan* scan, const uint64_t* d_offsets, const uint8_t* d_bytes, uint64_t first,
                        uint32_t count, uint32_t minlen, uint32_t maxlen, void* hip_stream) {
    return guarded([&]() -> int {
        return scan_load_dict(scan, d_offsets, d_bytes, first, count, minlen, maxlen, hip_stream);
    });
}
int dwpa_scan_load_numeric(dwpa_scan* scan, uint64_t first, uint32_t count, uint32_t digits, void* hip_stream) {
    return guarded([&]() -> int {
        return scan_load_numeric(scan, first, count, digits, hip_stream);
    });
}
int dwpa_scan_pbkdf2(dwpa_scan* scan, int group, void* hip_stream) {
    return guarded([&]() -> int { return scan_pbkdf2(scan, group, hip_stream); });
}
int dwpa_scan_verify(dwpa_scan* scan, int group, void* hip_stream) {
    return guarded([&]() -> int { return scan_verify(scan, group, hip_stream); });
}
int dwpa_scan_run(dwpa_scan* scan, void* hip_stream) {
    return guarded([&]() -> int { return scan_run(scan, hip_stream); });
}
int dwpa_scan_hits(dwpa_scan* scan, dwpa_hit* out, size_t cap, size_t* nhits, void* hip_stream) {
    return guarded([&]() -> int {
        if (!scan || !nhits || (!out && cap)) return DWPA_E_ARG;
        std::vector<HitDev> raw;
        RCHK(scan_hits_raw(scan, raw, hip_stream));
        *nhits = raw.size();
        for (size_t i = 0; i < raw.size() && i < cap; i++) hit_to_public(scan, raw[i], out[i]);
        return raw.size() > cap ? DWPA_E_OVERFLOW : 0;
    });
}
int dwpa_scan_loaded(dwpa_scan* scan, uint32_t* count, void* hip_stream) {
    return guarded([&]() -> int {
        if (!scan || !count) return DWPA_E_ARG;
        HIPCHK(hipSetDevice(scan->device));
        hipStream_t s = as_stream(hip_stream);
        HIPCHK(hipMemcpyAsync(count, scan->batch.counters.p, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (*count > scan->batch_cap) *count = scan->batch_cap;
        return 0;
    });
}
void dwpa_scan_destroy(dwpa_scan* scan) { scan_destroy(scan); }

static int set_dev(int device) {
    RCHK(ensure_init());
    if (device < 0 || device >= g_ndev) return DWPA_E_ARG;
    HIPCHK(hipSetDevice(device));
    return 0;
}
int dwpa_dev_alloc(int device, size_t bytes, void** out) {
    return guarded([&]() -> int {
        if (!out) return DWPA_E_ARG;
        RCHK(set_dev(device));
        if (hipMalloc(out, bytes ? bytes : 16) != hipSuccess) return DWPA_E_NOMEM;
        return 0;
    });
}
int dwpa_dev_free(int device, void* p) {
    return guarded([&]() -> int {
        RCHK(set_dev(device));
        if (p) HIPCHK(hipFree(p));
        return 0;
    });
}
int dwpa_dev_upload(int device, void* dst, const void* src, size_t bytes) {
    return guarded([&]() -> int {
        RCHK(set_dev(device));
        if (bytes) HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
        return 0;
    });
}
int dwpa_dev_download(int device, void* dst, const void* src, size_t bytes) {
    return guarded([&]() -> int {
        RCHK(set_dev(device));
        if (bytes) HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
        return 0;
    });
}
int dwpa_stream_create(int device, void** out) {
    return guarded([&]() -> int {
        if (!out) return DWPA_E_ARG;
        RCHK(set_dev(device));
        hipStream_t s;
        HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        *out = (void*)s;
        return 0;
    });
}
int dwpa_stream_sync(void* stream) {
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    return 0;
}
int dwpa_stream_destroy(void* stream) {
    if (stream) HIPCHK(hipStreamDestroy((hipStream_t)stream));
    return 0;
}
int dwpa_event_create(int device, void** out) {
    return guarded([&]() -> int {
        if (!out) return DWPA_E_ARG;
        RCHK(set_dev(device));
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        *out = (void*)e;
        return 0;
    });
}
int dwpa_event_record(void* event, void* stream) {
    HIPCHK(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
    return 0;
}
int dwpa_event_elapsed_ms(void* start, void* stop, float* ms) {
    if (!ms) return DWPA_E_ARG;
    HIPCHK(hipEventSynchronize((hipEvent_t)stop));
    HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return 0;
}
int dwpa_event_destroy(void* event) {
    if (event) HIPCHK(hipEventDestroy((hipEvent_t)event));
    return 0;
}

}  // extern "C"
