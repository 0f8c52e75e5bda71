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
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dwpa22000.h"
#include "engine.hpp"
#include "m22000_host.hpp"
#include "rules.hpp"

namespace dwpa {

struct Chunk {
    std::vector<uint64_t> off;  // words+1 offsets
    std::string bytes;          // concatenated words (decoded)
    size_t words() const { return off.empty() ? 0 : off.size() - 1; }
};

// Dictionary reader: plain or gzip (zlib reads both), one word per line, "\n" or "\r\n", $HEX[] decoded.  Lines
// are cut straight out of the inflate buffer with memchr and appended to the chunk (no per-line allocation): the
// reader has to keep up with 8 GPUs at ~5 M words/s each when a work unit has one ESSID and no rules.
class DictReader {
  public:
    explicit DictReader(const std::vector<std::string>& paths) : paths_(paths) {}
    // Returns false at the end of all files; sets err on I/O failure.
    bool next(Chunk& c, size_t max_words, size_t max_bytes, bool& err) {
        c.off.clear();
        c.bytes.clear();
        c.off.push_back(0);
        while (c.words() < max_words && c.bytes.size() < max_bytes) {
            if (!gz_) {
                if (idx_ >= paths_.size()) break;
                gz_ = gzopen(paths_[idx_].c_str(), "rb");
                if (!gz_) { err = true; return false; }
                gzbuffer(gz_, 1 << 20);
                pos_ = len_ = 0;
            }
            if (pos_ >= len_) {
                const int r = gzread(gz_, buf_, sizeof(buf_));
                if (r < 0) { err = true; return false; }
                if (r == 0) {  // end of this file: a last line without '\n' is still a word
                    if (!partial_.empty()) emit(c, partial_.data(), partial_.size());
                    partial_.clear();
                    gzclose(gz_);
                    gz_ = nullptr;
                    idx_++;
                    continue;
                }
                pos_ = 0;
                len_ = (size_t)r;
            }
            const char* p = buf_ + pos_;
            const char* end = buf_ + len_;
            while (p < end && c.words() < max_words && c.bytes.size() < max_bytes) {
                const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
                if (!nl) {
                    partial_.append(p, (size_t)(end - p));
                    p = end;
                    break;
                }
                if (!partial_.empty()) {
                    partial_.append(p, (size_t)(nl - p));
                    emit(c, partial_.data(), partial_.size());
                    partial_.clear();
                } else {
                    emit(c, p, (size_t)(nl - p));
                }
                p = nl + 1;
            }
            pos_ = (size_t)(p - buf_);
        }
        return c.words() > 0;
    }
    ~DictReader() {
        if (gz_) gzclose(gz_);
    }

  private:
    static void emit(Chunk& c, const char* p, size_t k) {
        if (k && p[k - 1] == '\r') k--;
        if (k > 5 && p[0] == '$' && starts_hex((const uint8_t*)p, k)) c.bytes += hc_unhex(std::string(p, k));
        else c.bytes.append(p, k);
        c.off.push_back(c.bytes.size());
    }
    std::vector<std::string> paths_;
    size_t idx_ = 0;
    gzFile gz_ = nullptr;
    char buf_[1 << 16];
    size_t pos_ = 0, len_ = 0;
    std::string partial_;
};

// Dictionary chunks from several files at once: worker t reads files t, t+T, ... with its own DictReader and
// queues its chunks (first chunk small, then doubling to max_words), so inflating several gz dictionaries uses
// several host cores.  Chunks arrive in completion order; candidate order only decides which of two identical
// PSKs is written, so the outfile is the same as hashcat's.
class ChunkSource {
  public:
    ChunkSource(const std::vector<std::string>& paths, size_t first_words, size_t max_words) {
        const size_t T = std::max<size_t>(1, std::min<size_t>(paths.size(), 4));
        cap_ = T + 1;
        live_ = T;
        for (size_t t = 0; t < T; t++) {
            std::vector<std::string> mine;
            for (size_t i = t; i < paths.size(); i += T) mine.push_back(paths[i]);
            workers_.emplace_back([this, mine, first_words, max_words, T] { work(mine, first_words, std::max<size_t>(first_words, max_words / T)); });
        }
    }
    ~ChunkSource() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }
    // Blocks until a chunk is ready; false once every file is read (or on an I/O error: err is set).
    bool next(Chunk& c, bool& err) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty() || live_ == 0; });
        err = err || err_;
        if (q_.empty()) return false;
        c = std::move(q_.front());
        q_.pop_front();
        cv_.notify_all();
        return true;
    }

  private:
    void work(const std::vector<std::string>& paths, size_t words, size_t max_words) {
        DictReader reader(paths);
        bool err = false;
        for (;;) {
            Chunk c;
            const bool have = reader.next(c, words, (size_t)1 << 31, err);
            words = std::min(max_words, 2 * words);
            std::unique_lock<std::mutex> lk(mu_);
            if (!have || err || stop_) break;
            cv_.wait(lk, [&] { return q_.size() < cap_ || stop_; });
            if (stop_) break;
            q_.push_back(std::move(c));
            cv_.notify_all();
        }
        std::lock_guard<std::mutex> lk(mu_);
        err_ = err_ || err;
        live_--;
        cv_.notify_all();
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Chunk> q_;
    size_t cap_ = 2, live_ = 0;
    bool stop_ = false, err_ = false;
    std::vector<std::thread> workers_;
};

struct CrackShared {
    std::mutex mu;
    std::vector<uint8_t> cracked;         // per input line
    std::vector<ParsedLine> parsed;
    FILE* out = nullptr;
    size_t valid = 0, ncracked = 0;
    int error = 0;
};

static std::string outfile_record(const ParsedLine& p, const std::string& psk) {
    const std::string& target = p.kind == LINE_PMKID ? p.pmkid : p.keymic;
    return hex_lower(target.substr(0, 16)) + ":" + hex_lower(p.mac_ap) + ":" + hex_lower(p.mac_sta) + ":" +
           hashcat_plain(p.essid) + ":" + hashcat_plain(psk) + "\n";
}

// Per-device state.  Shards are uploaded into one of two buffer slots on the `up` stream by the thread that read
// the chunk, so the upload of chunk k+1 overlaps the scan of chunk k; the scan waits on `staged[slot]`.
struct DevWork {
    int device;
    dwpa_scan* scan = nullptr;
    DevBuf off[2], bytes[2];
    std::vector<uint64_t> hoff[2];  // host staging of the rebased offsets (alive until the upload completes)
    hipStream_t stream = nullptr, up = nullptr;
    hipEvent_t staged[2] = {nullptr, nullptr};
};

// Upload words [b, e) of chunk c (offsets rebased to the shard) into slot `slot` of device w.
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

static int scan_shard(DevWork& w, CrackShared& sh, const Chunk& c, size_t b, size_t e, const RuleSet* rules,
                      DevRules* drules, int slot) {
    if (e <= b) return 0;
    if (hipSetDevice(w.device) != hipSuccess) return DWPA_E_HIP;
    if (hipStreamWaitEvent(w.stream, w.staged[slot], 0) != hipSuccess) return DWPA_E_HIP;
    const DevBuf& woff = w.off[slot];
    const DevBuf& wbytes = w.bytes[slot];
    const uint32_t cap = scan_batch_cap(w.scan);
    const size_t words = e - b;
    const uint64_t nrules = rules ? rules->size() : 1;
    const uint64_t total = words * nrules;
    // candidate id = word * nrules + rule; batches walk the candidate space in order.  Every PBKDF2 lane runs the
    // same 4096 iterations, so a batch costs ceil(candidates / 256K) wave rounds whatever its fill: the words per
    // batch follow the observed fraction of candidates that survive the 8..63 filter (and the rules), aiming at
    // 99.5 % of the batch.  A load that overflows the batch (the compaction drops and counts the excess) is
    // repeated with fewer words before anything is derived.
    double keep = 1.0;  // surviving candidates per (word x rule)
    for (size_t wb = 0; wb < words;) {
        // keep == 1 (nothing filtered so far): exactly one batch of candidates, which cannot overflow
        const double want = (keep >= 1.0 ? 1.0 : 0.995) * cap / ((double)nrules * keep);
        const uint64_t most = 16ull * cap / nrules;  // kernel-side bound on a fill-mode load
        const uint32_t nw = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)want, most, words - wb}));
        int r;
        if (rules)
            r = rules_load(w.scan, drules, (const uint64_t*)woff.p, (const uint8_t*)wbytes.p, wb, nw, w.stream, true);
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
        if ((r = scan_run(w.scan, w.stream)) < 0) return r;  // all ESSID groups, grouped per launch
        wb += nw;
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
            if (rules) plain = rules->apply_host((size_t)rule, plain);
            sh.cracked[ph.line] = 1;
            sh.ncracked++;
            const std::string rec = outfile_record(sh.parsed[ph.line], plain);
            fwrite(rec.data(), 1, rec.size(), sh.out);
            fflush(sh.out);
        }
        (void)total;
    }
    return 0;
}

static int crack_impl(const char* hash_file, const char* const* dicts, size_t ndicts, const char* rules_file, int nec,
                      const char* out_file, const dwpa_config* cfg) {
    if (!hash_file || !out_file || (!dicts && ndicts)) return DWPA_RC_ERROR;
    if (cfg && dwpa_init(cfg) < 0) return DWPA_RC_ERROR;
    if (engine_init() < 0) return DWPA_RC_ERROR;
    std::vector<int> devs = engine_devices();
    if (devs.empty()) return DWPA_RC_ERROR;
    const int nc_mode = cfg ? cfg->nc_mode : DWPA_NC_HASHCAT;

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
        if (sh.parsed[i].status) sh.cracked[i] = 1;  // rejected by the parser (hashcat: token exception)
        else sh.valid++;
    }
    if (sh.valid == 0) return DWPA_RC_ERROR;  // hashcat: "No hashes loaded"

    RuleSet rules;
    const RuleSet* rp = nullptr;
    if (rules_file) {
        if (rules.load_file(rules_file) < 0) return DWPA_RC_ERROR;
        if (!rules.all_noop()) rp = &rules;
    }

    sh.out = fopen(out_file, "ab");
    if (!sh.out) return DWPA_RC_ERROR;

    std::vector<const char*> lp(lines.size());
    std::vector<size_t> ll(lines.size());
    for (size_t i = 0; i < lines.size(); i++) { lp[i] = lines[i].data(); ll[i] = lines[i].size(); }
    const uint32_t batch = cfg && cfg->batch ? cfg->batch : engine_batch();
    std::vector<DevWork> work(devs.size());
    std::vector<DevRules> drules(devs.size());
    int rc = 0;
    for (size_t k = 0; k < devs.size() && rc >= 0; k++) {
        work[k].device = devs[k];
        (void)hipSetDevice(devs[k]);
        if (hipStreamCreateWithFlags(&work[k].stream, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&work[k].up, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&work[k].staged[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&work[k].staged[1], hipEventDisableTiming) != hipSuccess)
            rc = DWPA_E_HIP;
        if (rc >= 0) rc = scan_create(devs[k], lp.data(), ll.data(), lines.size(), nec, nc_mode, batch, &work[k].scan);
        if (rc >= 0 && rp) rc = rules_upload(devs[k], rules, &drules[k]);
    }

    std::vector<std::string> dpaths;
    for (size_t i = 0; i < ndicts; i++) dpaths.push_back(dicts[i]);
    bool ioerr = false;
    const size_t chunk_words = (size_t)batch * devs.size() * 8;
    // double-buffered: the next chunk is read/inflated on a host thread while the devices scan this one.  The
    // first chunk is one batch per device, so the GPUs start after ~0.3 s of reading instead of a full chunk's.
    // Chunks then double until they reach chunk_words, so each read stays shorter than the previous chunk's scan.
    Chunk cur, nxt;
    ChunkSource source(dpaths, (size_t)batch * devs.size(), chunk_words);
    const size_t G = work.size();
    // contiguous, equal shards of a chunk, one per device, staged into buffer slot `slot`
    auto stage_all = [&](const Chunk& c, int slot) {
        int r = 0;
        for (size_t k = 0; k < G && r >= 0; k++) r = stage_shard(work[k], c, c.words() * k / G, c.words() * (k + 1) / G, slot);
        return r;
    };
    bool have = source.next(cur, ioerr);
    int slot = 0, stage_rc = 0;
    if (have && rc >= 0) rc = stage_all(cur, slot);
    while (rc >= 0 && have && sh.ncracked < sh.valid) {
        bool have_next = false;
        std::thread prefetch([&] {
            have_next = source.next(nxt, ioerr);
            if (have_next) stage_rc = stage_all(nxt, slot ^ 1);
        });
        {
            std::lock_guard<std::mutex> lk(sh.mu);  // retire lines cracked so far on every device
            for (size_t k = 0; k < work.size(); k++)
                for (size_t i = 0; i < lines.size(); i++)
                    if (sh.cracked[i]) scan_mark_cracked(work[k].scan, (uint32_t)i);
        }
        const size_t W = cur.words();
        std::vector<std::thread> th;
        std::vector<int> rcs(G, 0);
        for (size_t k = 0; k < G; k++) {
            const size_t b = W * k / G, e = W * (k + 1) / G;
            th.emplace_back([&, k, b, e] { rcs[k] = scan_shard(work[k], sh, cur, b, e, rp, &drules[k], slot); });
        }
        for (auto& t : th) t.join();
        prefetch.join();
        for (int r : rcs)
            if (r < 0) rc = r;
        if (stage_rc < 0) rc = stage_rc;
        std::swap(cur, nxt);
        slot ^= 1;
        have = have_next;
    }
    for (size_t k = 0; k < work.size(); k++) {
        if (work[k].scan) scan_destroy(work[k].scan);
        (void)hipSetDevice(work[k].device);
        for (int q = 0; q < 2; q++) {
            work[k].off[q].release();
            work[k].bytes[q].release();
            if (work[k].staged[q]) (void)hipEventDestroy(work[k].staged[q]);
        }
        rules_release(&drules[k]);
        if (work[k].stream) (void)hipStreamDestroy(work[k].stream);
        if (work[k].up) (void)hipStreamDestroy(work[k].up);
    }
    fclose(sh.out);
    if (rc < 0 || ioerr) return DWPA_RC_ERROR;
    return sh.ncracked == sh.valid ? DWPA_RC_CRACKED : DWPA_RC_EXHAUSTED;
}

}  // namespace dwpa

extern "C" {

int dwpa_crack_files(const char* hash_file, const char* const* dicts, size_t ndicts, const char* rules_file,
                     int nonce_error_corrections, const char* out_file, const dwpa_config* cfg) {
    return dwpa::crack_impl(hash_file, dicts, ndicts, rules_file, nonce_error_corrections, out_file, cfg);
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
}

}  // extern "C"
