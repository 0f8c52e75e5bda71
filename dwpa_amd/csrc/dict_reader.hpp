// dict_reader.hpp -- dictionary streaming for dwpa_crack_files (help_crack.py:520-552 hands hashcat plain or gzip
// wordlists, one candidate per line, $HEX[...] for non-printable words, maint.php:55-60).  Header-only so that
// tools/inflate_bench.cpp measures exactly the reader the library runs.
#pragma once
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "inflate.hpp"
#include "m22000_host.hpp"
#include "pinflate.hpp"

namespace dwpa {

struct Chunk {
    std::vector<uint64_t> off;  // words+1 offsets
    std::string bytes;          // concatenated words (decoded)
    size_t words() const { return off.empty() ? 0 : off.size() - 1; }
};

// Inflates files in order on a thread of its own into blocks of raw text, so that a single gz stream costs the line
// cutting no inflate time.  gzip files go through GzipDecoder (inflate.hpp: ~2x zlib 1.2.11's inflate on a host
// core; DWPA_INFLATE=zlib switches back to gzread for A/B), other files are read as they are.  A block with file_end
// set closes a file (its last line may lack the '\n').  Block buffers are recycled (next() hands the previous one
// back), so a 4 MiB block is neither allocated nor zero-filled per block.
class BlockInflater {
  public:
    static constexpr size_t BLOCK = 4u << 20, DEPTH = 4;
    struct Block {
        std::vector<uint8_t> buf;  // [0, WIN): history for back-references; text at [begin, end)
        size_t begin = 0, end = 0;
        bool file_end = false;
        bool err = false;      // the file could not be read (I/O error): the call fails
        bool damaged = false;  // on the file's last block: corrupt or truncated gzip, delivered up to the damage
        const char* data() const { return (const char*)buf.data() + begin; }
        size_t size() const { return end - begin; }
    };
    BlockInflater(std::vector<std::string> paths, const std::atomic<bool>* cancel)
        : paths_(std::move(paths)), cancel_(cancel) {
        const char* e = getenv("DWPA_INFLATE");
        zlib_ = e && !strcmp(e, "zlib");
        th_ = std::thread([this] { run(); });
    }
    ~BlockInflater() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        th_.join();
    }
    // ParallelGunzip workers this reader gives the gzip file `fd` (1: the single-stream GzipDecoder).
    static unsigned parallel_threads(int fd) { return parallel_threads_for(fd); }
    // Blocks until the next block (b's previous buffer goes back to the pool); false once every file is delivered.
    bool next(Block& b) {
        std::unique_lock<std::mutex> lk(mu_);
        if (!b.buf.empty()) free_.push_back(std::move(b.buf));
        cv_.wait(lk, [&] { return !q_.empty() || done_; });
        if (q_.empty()) return false;
        b = std::move(q_.front());
        q_.pop_front();
        cv_.notify_all();
        return true;
    }
    // Every file was delivered to its end (no cancel, no I/O error); valid once next() has returned false.
    bool complete() {
        std::lock_guard<std::mutex> lk(mu_);
        return done_ && complete_ && q_.empty();
    }

  private:
    static constexpr size_t BUFSZ = GzipDecoder::WIN + BLOCK + GzipDecoder::SLACK;
    bool push(Block&& b) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return q_.size() < DEPTH || stop_; });
        if (stop_) return false;
        q_.push_back(std::move(b));
        cv_.notify_all();
        return true;
    }
    Block fresh() {
        Block b;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!free_.empty()) {
                b.buf = std::move(free_.back());
                free_.pop_back();
            }
        }
        if (b.buf.size() != BUFSZ) b.buf.resize(BUFSZ);
        b.begin = b.end = GzipDecoder::WIN;
        return b;
    }
    bool cancelled() const { return (cancel_ && cancel_->load(std::memory_order_relaxed)); }
    bool error_block() {
        Block e;
        e.err = true;
        push(std::move(e));
        return false;
    }
    // one file; false ends the stream (error or cancel)
    bool file(const std::string& path) {
        const int fd = open(path.c_str(), O_RDONLY);
        if (fd < 0) return error_block();
        uint8_t magic[2] = {0, 0};
        const bool gz = pread(fd, magic, 2, 0) == 2 && magic[0] == 0x1f && magic[1] == 0x8b;
        bool ok = true;
        if (gz && zlib_) {
            ok = file_zlib(fd);
        } else if (gz && parallel_threads_for(fd) > 1) {
            ok = file_parallel(fd);
        } else if (gz) {
            GzipDecoder dec(fd);
            uint64_t delivered = 0;
            for (bool end = false; ok && !end && !cancelled();) {
                Block b = fresh();
                b.end = b.begin + dec.read(b.buf.data(), BLOCK);
                if (dec.failed()) {
                    // A damaged stream (truncated download, CRC error, bad code): deliver exactly what gzread
                    // would -- zlib decodes the file again from the start, the bytes this decoder already delivered
                    // are skipped, and what zlib yields up to the damage follows.  hashcat reads wordlists
                    // through gzread, scans that prefix and finishes normally (rc 0/1).
                    ok = file_zlib(fd, delivered, dec.error());
                    break;
                }
                delivered += b.size();
                end = dec.done();
                b.file_end = end;
                ok = push(std::move(b));
            }
        } else {
            for (bool end = false; ok && !end && !cancelled();) {
                Block b = fresh();
                while (b.end < b.begin + BLOCK) {
                    const ssize_t r = ::read(fd, b.buf.data() + b.end, b.begin + BLOCK - b.end);
                    if (r < 0) { b.err = true; break; }
                    if (r == 0) { end = true; break; }
                    b.end += (size_t)r;
                }
                b.file_end = end || b.err;
                const bool err = b.err;
                ok = push(std::move(b)) && !err;
            }
        }
        close(fd);
        return ok;
    }
    // Worker threads for one large gzip file (ParallelGunzip, pinflate.hpp): DWPA_INFLATE_THREADS, default
    // min(8, half the CPUs this process may use); files under 4 chunks (DWPA_INFLATE_CHUNK_MB, default 4) and
    // DWPA_INFLATE_THREADS=1 take the single-stream decoder.  DWPA_INFLATE_CHUNK_MB is the test suite's switch to run
    // the parallel decoder on small files (tests/test_dict_reader.py).
    static size_t chunk_bytes() {
        const char* e = getenv("DWPA_INFLATE_CHUNK_MB");
        const long mb = e && *e ? atol(e) : 4;
        return (size_t)std::max<long>(1, mb) << 20;
    }
    static unsigned parallel_threads_for(int fd) {
        struct stat st;
        if (fstat(fd, &st) != 0 || (size_t)st.st_size < 4 * chunk_bytes()) return 1;
        const char* e = getenv("DWPA_INFLATE_THREADS");
        if (e && *e) return (unsigned)std::max(1, atoi(e));
        cpu_set_t cs;
        const unsigned cpus = sched_getaffinity(0, sizeof(cs), &cs) == 0 ? (unsigned)CPU_COUNT(&cs)
                                                                          : std::thread::hardware_concurrency();
        return std::max(1u, std::min(8u, cpus / 2));
    }
    // One gzip file through ParallelGunzip into BLOCK-sized blocks.  If the parallel decode stops short (damage, or a
    // false block boundary), zlib's gzread continues from the bytes delivered and decides what the rest yields.
    bool file_parallel(int fd) {
        struct stat st;
        if (fstat(fd, &st) != 0) return error_block();
        Block b = fresh();
        bool ok = true;
        uint64_t pushed = 0;
        const char* perr = nullptr;
        ParallelGunzip::run(fd, (size_t)st.st_size, parallel_threads_for(fd), chunk_bytes(),
                            [&](const uint8_t* p, size_t k) {
                                while (k && ok) {
                                    const size_t t = std::min(b.begin + BLOCK - b.end, k);
                                    memcpy(b.buf.data() + b.end, p, t);
                                    b.end += t;
                                    p += t;
                                    k -= t;
                                    if (b.end == b.begin + BLOCK) {
                                        pushed += b.size();
                                        ok = push(std::move(b)) && !cancelled();
                                        b = fresh();
                                    }
                                }
                                return ok;
                            },
                            &perr);
        if (!ok || cancelled()) return false;
        if (perr) {  // damage (or a false boundary): gzread continues after the bytes delivered
            pushed += b.size();
            if (b.size() && !push(std::move(b))) return false;
            return file_zlib(fd, pushed, ParallelGunzip::false_boundary(perr) ? nullptr : perr);
        }
        b.file_end = true;
        return push(std::move(b));
    }
    // gzread over the whole file (DWPA_INFLATE=zlib), or over its rest after GzipDecoder failed (`skip` bytes
    // already delivered, `why` = the decoder's error).  gzread returns the data before a cut and then 0 (error
    // Z_BUF_ERROR), or -1 at a data error; either way the file's last block is marked damaged.
    bool file_zlib(int fd, uint64_t skip = 0, const char* why = nullptr) {
        if (lseek(fd, 0, SEEK_SET) != 0) return error_block();
        gzFile gz = gzdopen(dup(fd), "rb");
        if (!gz) return error_block();
        gzbuffer(gz, 1 << 20);
        bool ok = true, eof = false, damaged = false;
        std::vector<uint8_t> scratch;
        while (skip && !damaged) {  // the prefix GzipDecoder delivered (byte-identical to zlib's output)
            scratch.resize((size_t)std::min<uint64_t>(skip, 1u << 20));
            const int r = gzread(gz, scratch.data(), (unsigned)scratch.size());
            if (r <= 0) damaged = true;
            else skip -= (uint64_t)r;
        }
        if (damaged) {  // zlib failed inside the prefix already: close the file
            Block b = fresh();
            b.file_end = b.damaged = true;
            ok = push(std::move(b));
        }
        while (ok && !eof && !damaged && !cancelled()) {
            Block b = fresh();
            while (b.end < b.begin + BLOCK) {
                const int r = gzread(gz, b.buf.data() + b.end, (unsigned)(b.begin + BLOCK - b.end));
                if (r < 0) { damaged = true; break; }
                if (r == 0) { eof = true; break; }
                b.end += (size_t)r;
            }
            if (eof) {
                int zerr = Z_OK;
                gzerror(gz, &zerr);
                damaged = zerr == Z_BUF_ERROR;  // truncated: gzread delivered what it could
                // Only zlib's own verdict marks a file damaged (help_crack deletes and re-downloads those).  Our
                // decoder rejecting a stream that zlib reads to its end cleanly is a decoder divergence: report it,
                // keep the file.
                if (!damaged && why)
                    fprintf(stderr, "[dwpa] gzip decoder rejected a stream zlib reads cleanly (%s); zlib's output used\n",
                            why);
            }
            b.file_end = eof || damaged;
            b.damaged = damaged;
            ok = push(std::move(b));
        }
        gzclose(gz);
        return ok;
    }
    // The inflater thread.  No exception leaves it (that would terminate the caller's process): one that a file
    // raises (std::bad_alloc, a thread that cannot start) ends the stream as failed, and the reader reports an I/O
    // error for the call.
    void run() {
        bool all = true, failed = false;
        try {
            for (const std::string& path : paths_)
                if (!file(path) || cancelled()) {
                    all = false;
                    break;
                }
        } catch (...) {
            all = false;
            failed = true;
        }
        std::lock_guard<std::mutex> lk(mu_);
        complete_ = all && !cancelled();
        failed_ = failed;
        done_ = true;
        cv_.notify_all();
    }
    std::vector<std::string> paths_;
    const std::atomic<bool>* cancel_;
    bool zlib_ = false;
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Block> q_;
    std::vector<std::vector<uint8_t>> free_;
    bool stop_ = false, done_ = false, complete_ = false, failed_ = false;

  public:
    // The inflater thread failed (an exception inside it); valid once next() has returned false.
    bool failed() {
        std::lock_guard<std::mutex> lk(mu_);
        return failed_;
    }
};

// Dictionary reader: plain or gzip (zlib reads both), one word per line, "\n" or "\r\n", $HEX[] decoded.  Lines
// are cut straight out of the inflated blocks with memchr and appended to the chunk (no per-line allocation): the
// reader has to keep up with 8 GPUs at ~5 M words/s each when a work unit has one ESSID and no rules.
class DictReader {
  public:
    explicit DictReader(const std::vector<std::string>& paths, const std::atomic<bool>* cancel = nullptr)
        : src_(paths, cancel) {}
    // Returns false at the end of all files; sets err on I/O failure.  `cancel` (optional) ends the chunk early.
    bool next(Chunk& c, size_t max_words, size_t max_bytes, bool& err, const std::atomic<bool>* cancel = nullptr) {
        c.off.clear();
        c.bytes.clear();
        c.off.push_back(0);
        while (c.words() < max_words && c.bytes.size() < max_bytes) {
            if (cancel && cancel->load(std::memory_order_relaxed)) break;
            if (pos_ >= blk_.size()) {
                if (blk_.file_end) {  // end of a file: a last line without '\n' is still a word
                    if (!partial_.empty()) emit(c, partial_.data(), partial_.size());
                    partial_.clear();
                    blk_.file_end = false;
                    damaged_ = damaged_ || blk_.damaged;
                    continue;
                }
                if (!src_.next(blk_)) {
                    finished_ = true;
                    if (src_.failed()) {
                        err = true;
                        return false;
                    }
                    break;
                }
                if (blk_.err) { err = true; return false; }
                pos_ = 0;
                continue;
            }
            const char* base = blk_.data();
            const char* p = base + pos_;
            const char* end = base + blk_.size();
            while (p < end && c.words() < max_words && c.bytes.size() < max_bytes) {
                const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
                if (!nl) {
                    keep_partial(p, (size_t)(end - p));
                    p = end;
                    break;
                }
                if (!partial_.empty()) {
                    keep_partial(p, (size_t)(nl - p));
                    emit(c, partial_.data(), partial_.size());
                    partial_.clear();
                } else {
                    emit(c, p, (size_t)(nl - p));
                }
                p = nl + 1;
            }
            pos_ = (size_t)(p - base);
        }
        return c.words() > 0;
    }
    // A file of this reader was damaged (delivered up to the damage, as gzread does).
    bool damaged() const { return damaged_; }
    // The reader reached the end of every file: nothing was cut short by a cancel or an error.
    bool complete() { return finished_ && src_.complete(); }

    // A line is kept up to MAX_LINE bytes: every consumer rejects a word that long (the 8..63 PSK filter, the rule
    // engine's 256-byte words, hashcat's --stdout), a $HEX[] form cut short no longer decodes and stays as long, and
    // the line still counts as one word -- but a file of binary garbage without a '\n' no longer needs its whole
    // size in host memory.
    static constexpr size_t MAX_LINE = 1u << 20;

  private:
    void keep_partial(const char* p, size_t k) {
        if (partial_.size() < MAX_LINE) partial_.append(p, std::min(k, MAX_LINE - partial_.size()));
    }
    static void emit(Chunk& c, const char* p, size_t k) {
        k = std::min(k, MAX_LINE);
        if (k && p[k - 1] == '\r') k--;
        if (k > 5 && p[0] == '$' && starts_hex((const uint8_t*)p, k)) c.bytes += hc_unhex(std::string(p, k));
        else c.bytes.append(p, k);
        c.off.push_back(c.bytes.size());
    }
    BlockInflater src_;
    BlockInflater::Block blk_;
    size_t pos_ = 0;
    std::string partial_;
    bool damaged_ = false, finished_ = false;
};

// Decoded dictionaries kept in host memory between dwpa_crack_files calls of one process.  help_crack downloads a
// dictionary once and runs many work units over it (help_crack.py:520-552), and one gzip stream inflates at only
// ~28 M words/s -- under six GPUs' worth of one-ESSID candidates.  A file read to its end is kept
// whole (its chunks are shared with the work items that scan them), keyed by path, size, mtime and inode, so the
// next work unit over it streams from memory.  DWPA_DICT_CACHE_MB bounds the total (default 4096, 0 = off); the
// least recently used files go first.
class DictCache {
  public:
    using Chunks = std::vector<std::shared_ptr<const Chunk>>;
    static DictCache& get() {
        static DictCache* c = new DictCache();  // never destroyed: chunks may outlive static destructors
        return *c;
    }
    // "" when the file cannot be stat()ed or the cache is off (never cached then).
    std::string key(const std::string& path) const {
        struct stat st;
        if (budget_ == 0 || stat(path.c_str(), &st) != 0) return std::string();
        return path + '\0' + std::to_string((long long)st.st_size) + ':' + std::to_string((long long)st.st_mtim.tv_sec) +
               '.' + std::to_string((long long)st.st_mtim.tv_nsec) + ':' + std::to_string((unsigned long long)st.st_ino);
    }
    // The cached decode of `path` under its current key k.  Entries of the same path under another key (the file
    // was downloaded again: new size, mtime or inode) are dropped here, so a re-fetched cracked.txt.gz does not
    // leave its old decode behind until LRU eviction.
    std::shared_ptr<const Chunks> find(const std::string& path, const std::string& k) {
        if (k.empty()) return nullptr;
        std::lock_guard<std::mutex> lk(mu_);
        const std::string prefix = path + '\0';
        for (auto it = map_.lower_bound(prefix); it != map_.end() && it->first.compare(0, prefix.size(), prefix) == 0;) {
            if (it->first == k) {
                ++it;
                continue;
            }
            total_ -= it->second.bytes;
            lru_.erase(it->second.pos);
            it = map_.erase(it);
        }
        auto it = map_.find(k);
        if (it == map_.end()) return nullptr;
        lru_.splice(lru_.begin(), lru_, it->second.pos);
        hits_++;
        return it->second.chunks;
    }
    void put(const std::string& k, std::shared_ptr<const Chunks> chunks) {
        if (k.empty()) return;
        size_t bytes = 0;
        for (const auto& c : *chunks) bytes += c->off.size() * sizeof(uint64_t) + c->bytes.size();
        std::lock_guard<std::mutex> lk(mu_);
        if (bytes > budget_ || map_.count(k)) return;
        while (total_ + bytes > budget_ && !lru_.empty()) {  // evict least recently used
            auto it = map_.find(lru_.back());
            total_ -= it->second.bytes;
            map_.erase(it);
            lru_.pop_back();
        }
        lru_.push_front(k);
        map_[k] = Entry{std::move(chunks), bytes, lru_.begin()};
        total_ += bytes;
    }
    size_t budget() const { return budget_; }
    size_t entries() {
        std::lock_guard<std::mutex> lk(mu_);
        return map_.size();
    }
    bool can_hold(size_t bytes) const { return bytes <= budget_; }
    size_t hits() const { return hits_.load(); }

  private:
    // Budget: DWPA_DICT_CACHE_MB, else min(4 GiB, max(512 MiB, a quarter of MemAvailable when the library first
    // reads a dictionary)) -- a volunteer's help_crack process keeps this much host RAM between work units at most.
    // MemAvailable (/proc/meminfo) counts the reclaimable page cache; MemFree (_SC_AVPHYS_PAGES) does not, and on a
    // long-running host with a warm cache it can be a small fraction of what is really available.
    DictCache() {
        const char* e = getenv("DWPA_DICT_CACHE_MB");
        if (e && *e) {
            budget_ = (size_t)atoll(e) << 20;
        } else {
            size_t avail = mem_available();
            if (!avail) {
                const long pages = sysconf(_SC_AVPHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
                avail = pages > 0 && psz > 0 ? (size_t)pages * (size_t)psz : 0;
            }
            budget_ = std::min<size_t>((size_t)4096 << 20, std::max<size_t>((size_t)512 << 20, avail / 4));
        }
    }
    static size_t mem_available() {
        FILE* f = fopen("/proc/meminfo", "r");
        if (!f) return 0;
        char line[256];
        unsigned long long kb = 0;
        while (fgets(line, sizeof line, f))
            if (sscanf(line, "MemAvailable: %llu kB", &kb) == 1) break;
        fclose(f);
        return (size_t)kb << 10;
    }
    struct Entry {
        std::shared_ptr<const Chunks> chunks;
        size_t bytes;
        std::list<std::string>::iterator pos;
    };
    std::mutex mu_;
    std::map<std::string, Entry> map_;
    std::list<std::string> lru_;
    size_t total_ = 0, budget_ = 0;
    std::atomic<size_t> hits_{0};
};

// Dictionary chunks from several files at once: worker t reads files t, t+T, ... (one DictReader per file, so a
// chunk never spans two files) and queues its chunks (first chunk small, then doubling to max_words), so inflating
// several gz dictionaries uses several host cores.  A file in the DictCache is replayed from memory instead.
// Chunks arrive in completion order; candidate order only decides which of two identical PSKs is written, so the
// outfile is the same as hashcat's.
class ChunkSource {
  public:
    ChunkSource(const std::vector<std::string>& paths, size_t first_words, size_t max_words)
        : status_(paths.size(), FILE_OK) {
        const size_t T = std::max<size_t>(1, std::min<size_t>(paths.size(), 4));
        cap_ = T + 1;
        live_ = T;
        try {
            for (size_t t = 0; t < T; t++) {
                std::vector<size_t> mine;
                for (size_t i = t; i < paths.size(); i += T) mine.push_back(i);
                workers_.emplace_back([this, paths, mine, first_words, max_words, T] {
                    work(paths, mine, first_words, std::max<size_t>(first_words, max_words / T));
                });
            }
        } catch (...) {  // a reader thread that cannot start: stop and join the started ones, then report it
            finish();
            throw;
        }
    }
    ~ChunkSource() { finish(); }
    // Stops the readers (within one 64 KiB read) and makes next() return false.  cancel_ is raised before stop_:
    // a reader whose push() sees stop_ then also sees cancel_, so it never takes a cut-short file as complete.
    void cancel() {
        cancel_ = true;
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
    }
    // cancel() and wait for the reader threads; file_status() is final afterwards.
    void finish() {
        cancel();
        for (auto& w : workers_)
            if (w.joinable()) w.join();
    }
    enum { FILE_OK = 0, FILE_DAMAGED = 1, FILE_UNREADABLE = 2 };
    // Per input path: FILE_OK (read, or never reached), FILE_DAMAGED (corrupt or truncated gzip, delivered up to the
    // damage as gzread does) or FILE_UNREADABLE (open/read error: the call fails).
    std::vector<int> file_status() {
        std::lock_guard<std::mutex> lk(mu_);
        return status_;
    }
    // Blocks until a chunk is ready; false once every file is read (or on an I/O error: err is set).
    bool next(std::shared_ptr<const Chunk>& c, bool& err) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty() || live_ == 0 || stop_; });
        err = err || err_;
        if (q_.empty() || stop_) return false;
        c = std::move(q_.front());
        q_.pop_front();
        cv_.notify_all();
        return true;
    }
    // Words of the chunks read but not yet taken.
    size_t pending_words() {
        std::lock_guard<std::mutex> lk(mu_);
        size_t n = 0;
        for (const auto& c : q_) n += c->words();
        return n;
    }
    bool next(Chunk& c, bool& err) {  // by value (tools/inflate_bench)
        std::shared_ptr<const Chunk> p;
        if (!next(p, err)) return false;
        c = *p;
        return true;
    }

  private:
    bool push(std::shared_ptr<const Chunk> c) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return q_.size() < cap_ || stop_; });
        if (stop_) return false;
        q_.push_back(std::move(c));
        cv_.notify_all();
        return true;
    }
    // A reader thread.  No exception leaves it (std::terminate would end the caller's process): one raised while
    // reading (std::bad_alloc) fails the call like an I/O error.
    void work(const std::vector<std::string>& paths, const std::vector<size_t>& mine, size_t words,
              size_t max_words) {
        bool err = false;
        try {
            err = read_files(paths, mine, words, max_words);
        } catch (...) {
            err = true;
        }
        std::lock_guard<std::mutex> lk(mu_);
        err_ = err_ || err;
        live_--;
        cv_.notify_all();
    }
    // A chunk's byte capacity is reserved from the previous chunk's bytes per word (growing fresh 10-100 MB vectors
    // cost the crack path half its line-cutting rate), at most this much: a file of 1 MiB lines would otherwise ask
    // for words x 1 MiB.
    static constexpr size_t RESERVE_MAX = (size_t)256 << 20;
    bool read_files(const std::vector<std::string>& paths, const std::vector<size_t>& mine, size_t words,
                    size_t max_words) {
        DictCache& cache = DictCache::get();
        bool err = false;
        for (const size_t fi : mine) {
            const std::string& path = paths[fi];
            if (cancel_.load() || err) break;
            const std::string key = cache.key(path);
            if (auto hit = cache.find(path, key)) {  // decoded before: replay from memory
                for (const auto& c : *hit)
                    if (!push(c)) break;
                continue;
            }
            auto keep = std::make_shared<DictCache::Chunks>();
            size_t kept = 0;
            bool whole = !key.empty();
            DictReader reader({path}, &cancel_);
            size_t per_word = 16;  // decoded bytes per word, from the previous chunk (capacity reserved up front:
                                   // growing fresh 10-100 MB vectors cost the crack path half its line-cutting rate)
            for (;;) {
                auto c = std::make_shared<Chunk>();
                c->off.reserve(words + 1);
                c->bytes.reserve(std::min(words * (per_word + per_word / 8) + 64, RESERVE_MAX));
                const bool have = reader.next(*c, words, (size_t)1 << 31, err, &cancel_);
                if (c->words()) per_word = c->bytes.size() / c->words() + 1;
                words = std::min(max_words, 2 * words);
                if (!have || err) break;
                if (whole) {
                    kept += c->off.size() * sizeof(uint64_t) + c->bytes.size();
                    whole = cache.can_hold(kept);
                    if (whole) keep->push_back(c);
                    else keep->clear();
                }
                if (!push(std::move(c))) break;
            }
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (err) status_[fi] = FILE_UNREADABLE;
                else if (reader.damaged()) status_[fi] = FILE_DAMAGED;
            }
            // cached only when read to its very end, undamaged (a replay must be the whole dictionary)
            if (whole && !err && !reader.damaged() && reader.complete() && !cancel_.load())
                cache.put(key, std::move(keep));
        }
        return err;
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<const Chunk>> q_;
    size_t cap_ = 2, live_ = 0;
    bool stop_ = false, err_ = false;
    std::vector<int> status_;
    std::atomic<bool> cancel_{false};
    std::vector<std::thread> workers_;
};

// One contiguous word range of a dictionary chunk.  The chunk stays alive until its last range is scanned.
struct WorkItem {
    std::shared_ptr<const Chunk> chunk;
    size_t b = 0, e = 0;
};

// Cuts the reader's chunks into work items that every shard worker pulls for itself: a device that finishes its
// item early takes the next one, so no device waits for the slowest at a chunk boundary.  Items start at `first`
// words (a sixteenth of a batch of candidates, so every device starts after a short read) and double up to `most`
// once per round of the workers (every device ramps through the same sizes).
// With several workers the end of the work unit is balanced by guided self-scheduling: an item takes at most
// 1/(2 workers) of the words read and not yet handed out (each worker stages its next item while it scans the
// current one; never under `first`).  The readers run ahead of the devices, so mid-way that leaves the items at
// their doubling size, while at the end, when the last chunk holds all that remains, the items shrink and the
// devices finish within about one small item of each other.  Without it a 20M-word dictionary on 8 workers went
// out as items of 1, 2, 4, 1 and 11.6M words, three workers idle (profiles/r03/crack_balance/).
class ItemQueue {
  public:
    ItemQueue(ChunkSource& src, size_t first, size_t most, size_t workers)
        : src_(src), size_(std::max<size_t>(1, first)), first_(std::max<size_t>(1, first)),
          most_(std::max<size_t>(1, most)), workers_(std::max<size_t>(1, workers)) {}
    bool next(WorkItem& it) {
        std::lock_guard<std::mutex> lk(mu_);
        while (!cur_ || pos_ >= cur_->words()) {
            if (done_) return false;
            if (!src_.next(cur_, err_)) {
                done_ = true;
                cur_.reset();
                return false;
            }
            pos_ = 0;
        }
        size_t n = std::min(size_, cur_->words() - pos_);
        if (workers_ > 1) {  // the words read and not yet handed out (all that remains once the readers end)
            const size_t rem = cur_->words() - pos_ + src_.pending_words();
            n = std::min(n, std::max(first_, (rem + 2 * workers_ - 1) / (2 * workers_)));
        }
        it.chunk = cur_;
        it.b = pos_;
        it.e = pos_ + n;
        pos_ += n;
        if (++taken_ % workers_ == 0) size_ = std::min(most_, 2 * size_);  // one size per round of the workers
        return true;
    }
    bool io_error() {
        std::lock_guard<std::mutex> lk(mu_);
        return err_;
    }

  private:
    ChunkSource& src_;
    std::mutex mu_;
    std::shared_ptr<const Chunk> cur_;
    size_t pos_ = 0, size_, first_, most_, workers_, taken_ = 0;
    bool done_ = false, err_ = false;
};

}  // namespace dwpa
