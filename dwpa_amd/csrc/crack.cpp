// crack.cpp -- dwpa_crack_files(): the in-process replacement of help_crack.py's hashcat subprocess
// (run_cracker, help_crack/help_crack.py:765-802; command line :773; rc handling :776-786; outfile parsed by
// get_key :804-879).
//
// Work distribution: the dictionary stream is cut into chunks; each chunk is split into contiguous, equal
// shards, one per active device, and every device thread scans its shard in batches (load -> per-ESSID PBKDF2 ->
// verify).  There is no device-to-device traffic: hits (a few bytes) are gathered on the host, where the first
// hit of each hashline is written to the outfile and the line is retired on every device (hashcat reports each
// hash once).  Rules (hashcat -r, help_crack.py:445-447,931-933) are applied on the GPU (rules.cpp).
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dwpa22000.h"
#include "engine.hpp"
#include "m22000_host.hpp"
#include "dict_reader.hpp"
#include "rules.hpp"

namespace dwpa {

struct CrackShared {
    std::mutex mu;
    std::vector<uint8_t> cracked;         // per input line (1: cracked, or never usable)
    std::vector<ParsedLine> parsed;
    FILE* out = nullptr;
    size_t valid = 0, ncracked = 0;
    std::atomic<uint32_t> version{0};     // bumped for every newly cracked line: workers re-sync their scans
    std::atomic<bool> stop{false};        // every usable line cracked, or an error
    std::atomic<int> error{0};
};

static std::string outfile_record(const ParsedLine& p, const std::string& psk) {
    const std::string& target = p.kind == LINE_PMKID ? p.pmkid : p.keymic;
    return hex_lower(target.substr(0, 16)) + ":" + hex_lower(p.mac_ap) + ":" + hex_lower(p.mac_sta) + ":" +
           hashcat_plain(p.essid) + ":" + hashcat_plain(psk) + "\n";
}

// One shard worker (one per device, or DWPA_CRACK_SHARDS_PER_DEVICE per device).  Its stager thread uploads the
// next item into the free one of two buffer slots on the `up` stream while its scanner thread scans the other.
struct DevWork {
    int device = 0;
    dwpa_scan* scan = nullptr;
    DevRules rules;
    DevBuf off[2], bytes[2];
    std::vector<uint64_t> hoff[2];  // host staging of the rebased offsets (alive until the upload completes)
    hipStream_t stream = nullptr, up = nullptr;
    hipEvent_t staged[2] = {nullptr, nullptr};
    double keep = 1.0;              // surviving candidates per (word x rule), carried from item to item
    uint32_t seen_version = 0;      // sh.version this scan's retired lines reflect
    size_t items = 0, words = 0;    // statistics (DWPA_TRACE, dwpa_crack_last_stats)
    uint64_t cands = 0;             // candidates loaded inside the 8..63 filter (after rules)
    double wait_s = 0;              // scanner time spent waiting for a staged item
    double scan_s = 0;              // scanner time spent scanning items
    // stager -> scanner hand-over
    std::mutex mu;
    std::condition_variable cv;
    WorkItem slot_item[2];
    bool slot_full[2] = {false, false};
    std::deque<int> ready;
    bool staging_done = false;
};

// Upload words [b, e) of chunk c (offsets rebased to the item) into slot `slot` of worker w.
static int stage_shard(DevWork& w, const Chunk& c, size_t b, size_t e, int slot) {
    if (hipSetDevice(w.device) != hipSuccess) return DWPA_E_HIP;
    std::vector<uint64_t>& off = w.hoff[slot];
    off.resize(e - b + 1);
    for (size_t i = b; i <= e; i++) off[i - b] = c.off[i] - c.off[b];
    const size_t nbytes = c.off[e] - c.off[b];
    DevBuf& ob = w.off[slot];
    DevBuf& bb = w.bytes[slot];
    if ((ob.n < off.size() * 8 && ob.ensure(off.size() * 8 * 3 / 2)) || (bb.n < nbytes + 64 && bb.ensure((nbytes + 64) * 3 / 2)))
        return DWPA_E_NOMEM;
    if (hipMemcpyAsync(ob.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, w.up) != hipSuccess ||
        (nbytes && hipMemcpyAsync(bb.p, c.bytes.data() + c.off[b], nbytes, hipMemcpyHostToDevice, w.up) != hipSuccess) ||
        hipEventRecord(w.staged[slot], w.up) != hipSuccess || hipStreamSynchronize(w.up) != hipSuccess)
        return DWPA_E_HIP;
    return 0;
}

// Retire on w's scan every line cracked anywhere so far (hashcat reports each hash once).
static void sync_retired(DevWork& w, CrackShared& sh) {
    const uint32_t v = sh.version.load(std::memory_order_acquire);
    if (v == w.seen_version) return;
    std::lock_guard<std::mutex> lk(sh.mu);
    for (size_t i = 0; i < sh.cracked.size(); i++)
        if (sh.cracked[i]) scan_mark_cracked(w.scan, (uint32_t)i);
    w.seen_version = v;
}

static int scan_shard(DevWork& w, CrackShared& sh, const Chunk& c, size_t b, size_t e, const RuleSet* rules,
                      int slot) {
    if (e <= b) return 0;
    if (hipSetDevice(w.device) != hipSuccess) return DWPA_E_HIP;
    if (hipStreamWaitEvent(w.stream, w.staged[slot], 0) != hipSuccess) return DWPA_E_HIP;
    const DevBuf& woff = w.off[slot];
    const DevBuf& wbytes = w.bytes[slot];
    const uint32_t cap = scan_batch_cap(w.scan);
    const size_t words = e - b;
    const uint64_t nrules = rules ? rules->size() : 1;
    // candidate id = word * nrules + rule; batches walk the candidate space in order.  Every PBKDF2 lane runs the
    // same 4096 iterations, so a batch costs ceil(candidates / 256K) wave rounds whatever its fill: the words per
    // batch follow the observed fraction of candidates that survive the 8..63 filter (and the rules), aiming at
    // 99.5 % of the batch.  A load that overflows the batch (the compaction drops and counts the excess) is
    // repeated with fewer words before anything is derived.
    double& keep = w.keep;
    for (size_t wb = 0; wb < words && !sh.stop.load(std::memory_order_relaxed);) {
        // keep == 1 (nothing filtered so far): exactly one batch of candidates, which cannot overflow
        const double want = (keep >= 1.0 ? 1.0 : 0.995) * cap / ((double)nrules * keep);
        const uint64_t most = 16ull * cap / nrules;  // kernel-side bound on a fill-mode load
        const uint32_t nw = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)want, most, words - wb}));
        int r;
        if (rules)
            r = rules_load(w.scan, &w.rules, (const uint64_t*)woff.p, (const uint8_t*)wbytes.p, wb, nw, w.stream, true);
        else
            r = scan_load_dict(w.scan, (const uint64_t*)woff.p, (const uint8_t*)wbytes.p, wb, nw, 8, 63, w.stream,
                               true);
        if (r < 0) return r;
        uint32_t raw = 0;
        if ((r = scan_counter_raw(w.scan, w.stream, &raw)) < 0) return r;
        const double seen = (double)raw / ((double)nw * nrules);
        if (raw > cap) {  // overflow: nothing derived yet, retry these words in a smaller batch
            if (nw == 1) return DWPA_E_OVERFLOW;
            keep = std::max(seen, keep * 1.05);
            continue;
        }
        if (raw > 0) keep = std::min(1.0, std::max(0.01, seen));
        if (raw == 0) {
            wb += nw;
            continue;
        }
        sync_retired(w, sh);
        if ((r = scan_run(w.scan, w.stream)) < 0) return r;  // all ESSID groups, grouped per launch
        wb += nw;
        w.cands += raw;
        std::vector<HitDev> hits;
        if ((r = scan_hits_raw(w.scan, hits, w.stream)) < 0) return r;
        if (hits.empty()) continue;
        std::sort(hits.begin(), hits.end(), [](const HitDev& x, const HitDev& y) { return x.cand < y.cand; });
        std::lock_guard<std::mutex> lk(sh.mu);
        for (const HitDev& h : hits) {
            dwpa_hit ph;
            hit_to_public(w.scan, h, ph);
            if (sh.cracked[ph.line]) continue;
            const uint64_t word = h.cand / nrules, rule = h.cand % nrules;
            std::string plain(c.bytes.data() + c.off[b + word], c.off[b + word + 1] - c.off[b + word]);
            if (rules && !rules->apply_host((size_t)rule, plain, &plain)) continue;  // cannot happen: the GPU kept it
            sh.cracked[ph.line] = 1;
            sh.ncracked++;
            sh.version.fetch_add(1, std::memory_order_acq_rel);
            const std::string rec = outfile_record(sh.parsed[ph.line], plain);
            fwrite(rec.data(), 1, rec.size(), sh.out);
            fflush(sh.out);
        }
        if (sh.ncracked == sh.valid) sh.stop = true;
    }
    return 0;
}

// DWPA_CRACK_SHARDS_PER_DEVICE=k runs k shard workers per selected device (default 1).  On a one-GPU box k = 2
// rehearses the multi-device path -- per-worker queues, shard scans and cross-worker line retirement -- that a
// volunteer's 8-GPU node runs (hashcat uses every device, help_crack.py:773).
static size_t shards_per_device() {
    const char* e = getenv("DWPA_CRACK_SHARDS_PER_DEVICE");
    const long k = e ? strtol(e, nullptr, 10) : 1;
    return (size_t)std::min<long>(8, std::max<long>(1, k));
}

// dwpa_crack_last_stats / dwpa_crack_worker_stats: the calling thread's last crack call
static thread_local dwpa_crack_stats g_last_stats;
static thread_local std::vector<dwpa_crack_worker> g_last_workers;
static thread_local bool g_have_stats = false;

static bool trace_on() {
    const char* e = getenv("DWPA_TRACE");
    return e && *e == '1';
}

static int crack_impl(const char* hash_file, const char* const* dicts, size_t ndicts, const char* rules_file, int nec,
                      const char* out_file, const dwpa_config* cfg, int32_t* dict_status) {
    const auto t_call = std::chrono::steady_clock::now();
    g_last_stats = dwpa_crack_stats{};  // an early return reports zeros, never the previous call
    g_last_workers.clear();
    g_have_stats = true;
    if (dict_status)
        for (size_t i = 0; i < ndicts; i++) dict_status[i] = DWPA_DICT_OK;
    if (!hash_file || !out_file || (!dicts && ndicts)) return DWPA_RC_ERROR;
    if (cfg && cfg->struct_size && cfg->struct_size < offsetof(dwpa_config, batch)) return DWPA_RC_ERROR;
    if (nec > DWPA_NC_MAX) {
        fprintf(stderr, "[dwpa] --nonce-error-corrections=%d is above the supported %d\n", nec, DWPA_NC_MAX);
        return DWPA_RC_ERROR;
    }
    // hashcat refuses to start when a wordlist cannot be opened; so does this call, before touching a device, and it
    // names the file (DWPA_E_IO in dict_status): a deterministic input error, which help_crack's drop-in does not retry
    bool unreadable = false;
    for (size_t i = 0; i < ndicts; i++) {
        FILE* f = dicts[i] ? fopen(dicts[i], "rb") : nullptr;
        if (!f) {
            unreadable = true;
            if (dict_status) dict_status[i] = DWPA_E_IO;
            fprintf(stderr, "[dwpa] dictionary %s: cannot be opened\n", dicts[i] ? dicts[i] : "(null)");
        } else {
            fclose(f);
        }
    }
    if (unreadable) return DWPA_RC_ERROR;
    // the config applies to this call only (dwpa_init's process-wide selection stays as it is)
    if (engine_init() < 0) return DWPA_RC_ERROR;
    std::vector<int> devs = engine_devices(DWPA_CFG_HAS(cfg, device_mask) ? cfg->device_mask : 0);
    if (devs.empty()) return DWPA_RC_ERROR;
    const int nc_mode = DWPA_CFG_HAS(cfg, nc_mode) ? cfg->nc_mode : DWPA_NC_HASHCAT;

    // hash file
    std::vector<std::string> lines;
    {
        FILE* f = fopen(hash_file, "rb");
        if (!f) return DWPA_RC_ERROR;
        std::string cur;
        int ch;
        while ((ch = fgetc(f)) != EOF) {
            if (ch == '\n') {
                if (!cur.empty() && cur.back() == '\r') cur.pop_back();
                if (!cur.empty()) lines.push_back(cur);
                cur.clear();
            } else cur.push_back((char)ch);
        }
        if (!cur.empty() && cur.back() == '\r') cur.pop_back();
        if (!cur.empty()) lines.push_back(cur);
        fclose(f);
    }
    CrackShared sh;
    sh.parsed.resize(lines.size());
    sh.cracked.assign(lines.size(), 0);
    for (size_t i = 0; i < lines.size(); i++) {
        sh.parsed[i] = parse_m22000(lines[i].data(), lines[i].size());
        // rejected by the parser (hashcat: token exception), or a PMKID/MIC shorter than 16 bytes that can never
        // verify (hashcat refuses such a hash at load time): neither is counted, so rc 0 stays reachable
        if (sh.parsed[i].status || !line_can_match(sh.parsed[i])) sh.cracked[i] = 1;
        else sh.valid++;
    }
    if (sh.valid == 0) return DWPA_RC_ERROR;  // hashcat: "No hashes loaded"

    // hashcat -r: lines that do not parse -- and, in the default DWPA_RULES_HASHCAT mode, lines using reject or
    // memory functions, which hashcat's -r loader skips too -- are skipped with a message each (RuleSet::add_line)
    // and counted in dwpa_crack_last_stats; a file with no rule left fails the call, as hashcat refuses to start
    RuleSet rules;
    const int want = DWPA_CFG_HAS(cfg, rule_mode) ? cfg->rule_mode : DWPA_RULES_DEFAULT;
    if (want != DWPA_RULES_DEFAULT && want != DWPA_RULES_HASHCAT && want != DWPA_RULES_FULL) return DWPA_RC_ERROR;
    rules.mode = want == DWPA_RULES_DEFAULT ? engine_rule_mode() : want;
    const RuleSet* rp = nullptr;
    if (rules_file) {
        const int lr = rules.load_file(rules_file);
        g_last_stats.rules = (uint32_t)rules.size();
        g_last_stats.rules_skipped = (uint32_t)rules.skipped.size();
        g_last_stats.rules_rejmem = rules.rejmem;
        if (lr < 0) return DWPA_RC_ERROR;
        if (!rules.all_noop()) rp = &rules;
    }

    sh.out = fopen(out_file, "ab");
    if (!sh.out) return DWPA_RC_ERROR;

    std::vector<const char*> lp(lines.size());
    std::vector<size_t> ll(lines.size());
    for (size_t i = 0; i < lines.size(); i++) { lp[i] = lines[i].data(); ll[i] = lines[i].size(); }
    const uint32_t batch = DWPA_CFG_HAS(cfg, batch) && cfg->batch ? cfg->batch : engine_batch();
    const size_t spd = shards_per_device();
    std::vector<std::unique_ptr<DevWork>> work;
    int rc = 0;
    for (int dev : devs)
        for (size_t k = 0; k < spd && rc >= 0; k++) {
            work.push_back(std::make_unique<DevWork>());
            DevWork& w = *work.back();
            w.device = dev;
            (void)hipSetDevice(dev);
            if (hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking) != hipSuccess ||
                hipStreamCreateWithFlags(&w.up, hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&w.staged[0], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&w.staged[1], hipEventDisableTiming) != hipSuccess)
                rc = DWPA_E_HIP;
            if (rc >= 0) rc = scan_create(dev, lp.data(), ll.data(), lines.size(), nec, nc_mode, batch, &w.scan);
            if (rc >= 0 && rp) rc = rules_upload(dev, rules, &w.rules);
        }
    const size_t G = work.size();

    std::vector<std::string> dpaths;
    for (size_t i = 0; i < ndicts; i++) dpaths.push_back(dicts[i]);
    // Items: the first is 1/16 of a batch of candidates (a device starts after ~1M words have been read, not a
    // whole 16M-word batch: on a dictionary's first pass that read took ~0.5 s of a 21 s C2 pass), doubling to
    // 16 batches (a partial last batch per item then costs ~1 % of its wave rounds).  The reader's chunks start at
    // one item per worker and grow to two full items per worker, so reading stays ahead of the scans without
    // holding much more than that in memory.
    const size_t nr = rp ? rp->size() : 1;
    const size_t first_item = std::max<size_t>(1, batch / nr / 16), most_item = std::max<size_t>(1, 16 * (size_t)batch / nr);
    ChunkSource source(dpaths, first_item * G, 2 * most_item * G);
    // several workers: items of at most 2 batches, so an item handed out just before the readers reach the end
    // cannot outlast the balanced tail by more than that
    ItemQueue items(source, first_item, G > 1 ? std::min(most_item, std::max<size_t>(first_item, 2 * (size_t)batch / nr))
                                              : most_item, G);
    const auto t0 = std::chrono::steady_clock::now();

    auto stop_all = [&]() {
        sh.stop = true;
        source.cancel();  // a stager blocked on the reader returns at once
        for (auto& wp : work) {
            std::lock_guard<std::mutex> lk(wp->mu);
            wp->cv.notify_all();
        }
    };
    auto fail = [&](int r) {
        int z = 0;
        sh.error.compare_exchange_strong(z, r);
        stop_all();
    };
    std::vector<std::thread> th;
    // A worker thread that cannot start (std::system_error, e.g. under RLIMIT_NPROC) stops the ones that did and
    // fails the call; the vector never unwinds with joinable threads in it.
    if (rc >= 0) try {
        for (size_t k = 0; k < G; k++) {
            th.emplace_back([&, k] {  // stager
                DevWork& w = *work[k];
                for (int slot = 0;; slot ^= 1) {
                    {
                        std::unique_lock<std::mutex> lk(w.mu);
                        w.cv.wait(lk, [&] { return !w.slot_full[slot] || sh.stop; });
                    }
                    WorkItem it;
                    if (sh.stop || !items.next(it)) break;
                    const int r = guarded([&] { return stage_shard(w, *it.chunk, it.b, it.e, slot); });
                    if (r < 0) {
                        fail(r);
                        break;
                    }
                    std::lock_guard<std::mutex> lk(w.mu);
                    w.slot_item[slot] = std::move(it);
                    w.slot_full[slot] = true;
                    w.ready.push_back(slot);
                    w.cv.notify_all();
                }
                std::lock_guard<std::mutex> lk(w.mu);
                w.staging_done = true;
                w.cv.notify_all();
            });
            th.emplace_back([&, k] {  // scanner
                DevWork& w = *work[k];
                for (;;) {
                    int slot;
                    WorkItem it;
                    {
                        const auto tw = std::chrono::steady_clock::now();
                        std::unique_lock<std::mutex> lk(w.mu);
                        w.cv.wait(lk, [&] { return !w.ready.empty() || w.staging_done || sh.stop; });
                        w.wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count();
                        if (w.ready.empty() || sh.stop) break;
                        slot = w.ready.front();
                        w.ready.pop_front();
                        it = w.slot_item[slot];
                    }
                    const auto ts = std::chrono::steady_clock::now();
                    const int r = guarded([&] { return scan_shard(w, sh, *it.chunk, it.b, it.e, rp, slot); });
                    w.scan_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
                    w.items++;
                    w.words += it.e - it.b;
                    {
                        std::lock_guard<std::mutex> lk(w.mu);
                        w.slot_item[slot] = WorkItem();
                        w.slot_full[slot] = false;
                        w.cv.notify_all();
                    }
                    if (r < 0) {
                        fail(r);
                        break;
                    }
                    if (sh.stop) {
                        stop_all();
                        break;
                    }
                }
            });
        }
    } catch (...) {
        fail(DWPA_E_NOMEM);
    }
    for (auto& t : th) t.join();
    source.finish();
    const bool ioerr = items.io_error();
    const std::vector<int> fst = source.file_status();
    for (size_t i = 0; i < ndicts; i++) {
        if (fst[i] == ChunkSource::FILE_DAMAGED)
            fprintf(stderr, "[dwpa] dictionary %s: damaged gzip stream (truncated or corrupt); scanned up to the damage, "
                            "as hashcat's gzread does\n", dicts[i]);
        else if (fst[i] == ChunkSource::FILE_UNREADABLE)
            fprintf(stderr, "[dwpa] dictionary %s: read error\n", dicts[i]);
        if (dict_status)
            dict_status[i] = fst[i] == ChunkSource::FILE_DAMAGED ? DWPA_DICT_DAMAGED
                             : fst[i] == ChunkSource::FILE_UNREADABLE ? DWPA_E_IO : DWPA_DICT_OK;
    }
    if (trace_on()) {
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        fprintf(stderr, "[dwpa] crack dictionary cache: %zu files replayed from memory so far\n", DictCache::get().hits());
        for (size_t k = 0; k < G; k++)
            fprintf(stderr, "[dwpa] crack worker %zu (device %d): %zu items, %zu words, %.3f s waiting for input of %.3f s\n",
                    k, work[k]->device, work[k]->items, work[k]->words, work[k]->wait_s, el);
    }
    for (auto& wp : work) {
        DevWork& w = *wp;
        if (w.scan) scan_destroy(w.scan);
        (void)hipSetDevice(w.device);
        for (int q = 0; q < 2; q++) {
            w.off[q].release();
            w.bytes[q].release();
            if (w.staged[q]) (void)hipEventDestroy(w.staged[q]);
        }
        rules_release(&w.rules);
        if (w.stream) (void)hipStreamDestroy(w.stream);
        if (w.up) (void)hipStreamDestroy(w.up);
    }
    fclose(sh.out);
    for (auto& wp : work) {
        g_last_stats.words += wp->words;
        g_last_stats.candidates += wp->cands;
        g_last_workers.push_back(dwpa_crack_worker{wp->device, (uint32_t)wp->items, (uint64_t)wp->words, wp->cands,
                                                   wp->wait_s, wp->scan_s});
    }
    g_last_stats.hashes = (uint32_t)sh.valid;
    g_last_stats.cracked = (uint32_t)sh.ncracked;
    g_last_stats.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_call).count();
    if (rc < 0 || sh.error.load() < 0 || ioerr) return DWPA_RC_ERROR;
    return sh.ncracked == sh.valid ? DWPA_RC_CRACKED : DWPA_RC_EXHAUSTED;
}

// `hashcat --stdout -r rules_file sources... -o out_path` (help_crack.py:508 expandcracked, :575 prdict): the words
// of the sources (plain or gzip, one per line, $HEX[] decoded, as hashcat reads wordlists) x every rule, expanded on
// the GPU in sub-batches of ~1M candidates (k_rules_expand into 256-byte slots), and packed on the GPU too
// (k_text_*: a scan of every candidate's text length, then each candidate copied to its offset): word-major order,
// rejected candidates skipped, raw bytes and '\n' as hashcat's --stdout writes them, $HEX[..] for a candidate holding
// '\n' or '\r'.  Only the packed text (~14 bytes per candidate) crosses PCIe -- round 4 copied the 256-byte slots
// back (189 GB for 740M candidates) and packed them on one host thread.  Two sets on two streams: the GPU expands and
// packs sub-batch i+1 while the host writes sub-batch i.
static int rules_expand_file_impl(int device, const char* rules_file, const char* const* sources, size_t nsources,
                                  const char* out_path, int gzip_level, uint64_t* words_out, uint64_t* cands_out) {
    if (!rules_file || !out_path || (!sources && nsources)) return DWPA_E_ARG;
    for (size_t i = 0; i < nsources; i++) {
        FILE* f = sources[i] ? fopen(sources[i], "rb") : nullptr;
        if (!f) return DWPA_E_IO;
        fclose(f);
    }
    RuleSet rs;
    rs.mode = engine_rule_mode();
    int rc = rs.load_file(rules_file);
    if (rc < 0) return rc;
    if ((rc = engine_init()) < 0) return rc;
    if (hipSetDevice(device) != hipSuccess) return DWPA_E_NODEV;
    FILE* fo = nullptr;
    gzFile gz = nullptr;
    if (gzip_level > 0) {
        char mode[8];
        snprintf(mode, sizeof mode, "wb%d", std::min(9, gzip_level));
        gz = gzopen(out_path, mode);
        if (!gz) return DWPA_E_IO;
        gzbuffer(gz, 1 << 20);
    } else if (!(fo = fopen(out_path, "wb"))) {
        return DWPA_E_IO;
    }
    // The text packer's offsets and totals are 32-bit: one word's candidates (nr of them, at most TEXT_MAX bytes each
    // as $HEX[..]) must fit 4 GiB, which bounds a rules file here to ~8.27M rules (bestWPA.rule has 145).
    constexpr size_t TEXT_MAX = 5 + 2 * (size_t)RP_PASSWORD_SIZE + 2;
    if (rs.size() > (size_t)UINT32_MAX / TEXT_MAX) {
        fprintf(stderr, "[dwpa] %zu rules: more than the %zu one expansion packs\n", rs.size(), (size_t)UINT32_MAX / TEXT_MAX);
        return DWPA_E_RULE;
    }
    DevRules dr;
    rc = rules_upload(device, rs, &dr);
    const size_t nr = rs.size();
    const size_t wpb = std::max<size_t>(1, (1u << 20) / nr);  // words per sub-batch: ~1M candidate slots
    const size_t ncap = wpb * nr;
    const size_t nblk = text_pack_blocks((uint32_t)ncap);
    struct Set {
        DevBuf off, bytes, out, len, tlen, bsum, bcnt, tot, text;
        uint32_t* h_tot = nullptr;  // pinned: text bytes, kept candidates
        uint8_t* h_text = nullptr;  // pinned, h_cap bytes (== text.n)
        size_t h_cap = 0;
        hipStream_t s = nullptr;
        hipEvent_t done = nullptr, up = nullptr;  // expansion + pack done and totals copied back / inputs uploaded
        std::vector<uint64_t> hoff;
        size_t words = 0;  // words of the sub-batch
        bool busy = false;
        int grow(size_t want) {  // device text buffer and its pinned host mirror, both `want` bytes
            pinned_free(h_text, h_cap);
            h_text = nullptr;
            h_cap = 0;
            if (text.ensure(want) || pinned_alloc((void**)&h_text, want) < 0) return DWPA_E_NOMEM;
            h_cap = want;
            return 0;
        }
    } set[2];
    for (Set& S : set) {
        if (rc < 0) break;
        if (S.out.ensure(ncap * 256) || S.len.ensure(ncap * 4) || S.tlen.ensure(ncap * 4) ||
            S.off.ensure((wpb + 1) * 8) || S.bsum.ensure(nblk * 4) || S.bcnt.ensure(nblk * 4) || S.tot.ensure(8) ||
            S.grow(ncap * 24) || pinned_alloc((void**)&S.h_tot, 8) < 0)
            rc = DWPA_E_NOMEM;
        else if (hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking) != hipSuccess ||
                 hipEventCreateWithFlags(&S.done, hipEventDisableTiming) != hipSuccess ||
                 hipEventCreateWithFlags(&S.up, hipEventDisableTiming) != hipSuccess)
            rc = DWPA_E_HIP;
    }
    uint64_t words = 0, cands = 0;
    auto pack = [&](Set& S) -> int {  // pack S's expansion into its text buffer, copy the totals back
        const uint32_t n = (uint32_t)(S.words * nr);
        if (launch_text_pack((const uint8_t*)S.out.p, (const uint32_t*)S.len.p, (const uint32_t*)S.tlen.p, n,
                             (uint32_t*)S.bsum.p, (uint32_t*)S.bcnt.p, (uint32_t*)S.tot.p, (uint8_t*)S.text.p, S.h_cap,
                             S.s) != hipSuccess ||
            hipMemcpyAsync(S.h_tot, S.tot.p, 8, hipMemcpyDeviceToHost, S.s) != hipSuccess ||
            hipEventRecord(S.done, S.s) != hipSuccess)
            return DWPA_E_HIP;
        return 0;
    };
    auto drain = [&](Set& S) -> int {  // wait for S's text, copy it back and write it
        if (!S.busy) return 0;
        S.busy = false;
        if (hipEventSynchronize(S.done) != hipSuccess) return DWPA_E_HIP;
        size_t bytes = S.h_tot[0];
        if (bytes > S.h_cap) {  // longer candidates than budgeted: a bigger buffer, and the same slots packed again
            if (S.grow(bytes + bytes / 4) < 0) return DWPA_E_NOMEM;
            int r = pack(S);
            if (r < 0) return r;
            if (hipEventSynchronize(S.done) != hipSuccess) return DWPA_E_HIP;
            bytes = S.h_tot[0];
        }
        if (bytes && (hipMemcpyAsync(S.h_text, S.text.p, bytes, hipMemcpyDeviceToHost, S.s) != hipSuccess ||
                      hipStreamSynchronize(S.s) != hipSuccess))
            return DWPA_E_HIP;
        cands += S.h_tot[1];
        const size_t put = gz ? (size_t)gzwrite(gz, S.h_text, (unsigned)bytes) : fwrite(S.h_text, 1, bytes, fo);
        return put == bytes ? 0 : DWPA_E_IO;
    };
    if (rc >= 0) {
        std::vector<std::string> paths(sources, sources + nsources);
        DictReader reader(paths);
        Chunk c;
        bool err = false;
        int cur = 0;
        auto uploads_done = [&]() {  // the chunk's bytes may change only when no upload still reads them
            for (Set& S : set)
                if (S.busy && hipEventSynchronize(S.up) != hipSuccess) return false;
            return true;
        };
        while (rc >= 0 && uploads_done() && reader.next(c, 16 * wpb, 64u << 20, err)) {
            for (size_t b = 0; b < c.words() && rc >= 0; b += wpb) {
                Set& S = set[cur];
                if ((rc = drain(S)) < 0) break;  // its previous sub-batch, two sub-batches ago
                const size_t e = std::min(c.words(), b + wpb);
                S.words = e - b;
                S.hoff.resize(S.words + 1);
                for (size_t i = b; i <= e; i++) S.hoff[i - b] = c.off[i] - c.off[b];
                const size_t nbytes = c.off[e] - c.off[b];
                if (S.bytes.n < nbytes + 16 && S.bytes.ensure(nbytes + 16 + (nbytes >> 1))) { rc = DWPA_E_NOMEM; break; }
                if (hipMemcpyAsync(S.off.p, S.hoff.data(), S.hoff.size() * 8, hipMemcpyHostToDevice, S.s) != hipSuccess ||
                    (nbytes && hipMemcpyAsync(S.bytes.p, c.bytes.data() + c.off[b], nbytes, hipMemcpyHostToDevice,
                                              S.s) != hipSuccess) ||
                    hipEventRecord(S.up, S.s) != hipSuccess ||
                    launch_rules_expand((const uint64_t*)S.off.p, (const uint8_t*)S.bytes.p, (uint32_t)S.words,
                                        (const uint32_t*)dr.offs, (const uint32_t*)dr.code, (uint32_t)nr,
                                        (uint8_t*)S.out.p, (uint32_t*)S.len.p, S.s, (uint32_t*)S.tlen.p) != hipSuccess) {
                    rc = DWPA_E_HIP;
                    break;
                }
                if ((rc = pack(S)) < 0) break;
                S.busy = true;  // S.hoff is rewritten only after drain(S); the chunk only after uploads_done()
                words += S.words;
                cur ^= 1;
                if ((rc = drain(set[cur])) < 0) break;
            }
        }
        if (err && rc >= 0) rc = DWPA_E_IO;
        for (Set& S : set)
            if (rc >= 0) rc = drain(S);
    }
    for (Set& S : set) {
        if (S.s) (void)hipStreamSynchronize(S.s);
        for (DevBuf* b : {&S.off, &S.bytes, &S.out, &S.len, &S.tlen, &S.bsum, &S.bcnt, &S.tot, &S.text}) b->release();
        pinned_free(S.h_text, S.h_cap);
        pinned_free(S.h_tot, 8);
        if (S.done) (void)hipEventDestroy(S.done);
        if (S.up) (void)hipEventDestroy(S.up);
        if (S.s) (void)hipStreamDestroy(S.s);
    }
    rules_release(&dr);
    if (gz && gzclose(gz) != Z_OK && rc >= 0) rc = DWPA_E_IO;
    if (fo && fclose(fo) != 0 && rc >= 0) rc = DWPA_E_IO;
    if (words_out) *words_out = words;
    if (cands_out) *cands_out = cands;
    return rc < 0 ? rc : 0;
}

}  // namespace dwpa

extern "C" {

int dwpa_rules_expand_file(int device, const char* rules_file, const char* const* sources, size_t nsources,
                           const char* out_path, int gzip_level, uint64_t* words_out, uint64_t* cands_out) {
    return dwpa::guarded([&]() -> int {
        return dwpa::rules_expand_file_impl(device, rules_file, sources, nsources, out_path, gzip_level, words_out,
                                            cands_out);
    });
}

int dwpa_crack_files(const char* hash_file, const char* const* dicts, size_t ndicts, const char* rules_file,
                     int nonce_error_corrections, const char* out_file, const dwpa_config* cfg) {
    return dwpa::guarded([&]() -> int {
        return dwpa::crack_impl(hash_file, dicts, ndicts, rules_file, nonce_error_corrections, out_file, cfg, nullptr);
    }, DWPA_RC_ERROR, DWPA_RC_ERROR);
}

int dwpa_crack_last_stats(dwpa_crack_stats* out) {
    if (!out || !dwpa::g_have_stats) return DWPA_E_ARG;
    *out = dwpa::g_last_stats;
    return 0;
}

int dwpa_crack_worker_stats(dwpa_crack_worker* out, size_t cap, size_t* n) {
    if (!n || (!out && cap) || !dwpa::g_have_stats) return DWPA_E_ARG;
    *n = dwpa::g_last_workers.size();
    for (size_t i = 0; i < std::min(cap, *n); i++) out[i] = dwpa::g_last_workers[i];
    return 0;
}

int dwpa_crack_files_ex(const char* hash_file, const char* const* dicts, size_t ndicts, const char* rules_file,
                        int nonce_error_corrections, const char* out_file, const dwpa_config* cfg,
                        int32_t* dict_status) {
    return dwpa::guarded([&]() -> int {
        return dwpa::crack_impl(hash_file, dicts, ndicts, rules_file, nonce_error_corrections, out_file, cfg, dict_status);
    }, DWPA_RC_ERROR, DWPA_RC_ERROR);
}

// md5 over fields 1..7 of the hashline (web/common.php:310-315); a tiny host MD5 keeps this dependency-free.
static void md5_host(const uint8_t* msg, size_t len, uint8_t out[16]) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static const int S[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
    std::string b((const char*)msg, len);
    b.push_back((char)0x80);
    while (b.size() % 64 != 56) b.push_back('\0');
    const uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; i++) b.push_back((char)(bits >> (8 * i)));
    uint32_t h[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
    for (size_t o = 0; o < b.size(); o += 64) {
        uint32_t m[16];
        for (int j = 0; j < 16; j++)
            m[j] = (uint32_t)(uint8_t)b[o + 4 * j] | (uint32_t)(uint8_t)b[o + 4 * j + 1] << 8 |
                   (uint32_t)(uint8_t)b[o + 4 * j + 2] << 16 | (uint32_t)(uint8_t)b[o + 4 * j + 3] << 24;
        uint32_t a = h[0], bb = h[1], c = h[2], d = h[3];
        for (int i = 0; i < 64; i++) {
            uint32_t f;
            int g;
            if (i < 16) { f = (bb & c) | (~bb & d); g = i; }
            else if (i < 32) { f = (d & bb) | (~d & c); g = (5 * i + 1) & 15; }
            else if (i < 48) { f = bb ^ c ^ d; g = (3 * i + 5) & 15; }
            else { f = c ^ (bb | ~d); g = (7 * i) & 15; }
            uint32_t t = d;
            d = c;
            c = bb;
            uint32_t x = a + f + K[i] + m[g];
            int s = S[i >> 4][i & 3];
            bb = bb + ((x << s) | (x >> (32 - s)));
            a = t;
        }
        h[0] += a; h[1] += bb; h[2] += c; h[3] += d;
    }
    for (int k = 0; k < 4; k++)
        for (int i = 0; i < 4; i++) out[4 * k + i] = (uint8_t)(h[k] >> (8 * i));
}

int dwpa_hash_m22000(const char* line, size_t line_len, uint8_t out[16]) {
    return dwpa::guarded([&]() -> int {
        if (!line || !out) return DWPA_E_ARG;
        const char* f[9];
        size_t fl[9], cnt = 0, st = 0;
        for (size_t i = 0; i < line_len && cnt < 8; i++)
            if (line[i] == '*') { f[cnt] = line + st; fl[cnt] = i - st; cnt++; st = i + 1; }
        f[cnt] = line + st; fl[cnt] = line_len - st; cnt++;
        if (cnt != 9) return DWPA_E_FORMAT;
        std::string cat;
        for (int i = 1; i <= 7; i++) cat.append(f[i], fl[i]);
        md5_host((const uint8_t*)cat.data(), cat.size(), out);
        return 0;
    });
}

}  // extern "C"
