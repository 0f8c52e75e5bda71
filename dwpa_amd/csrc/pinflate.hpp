// pinflate.hpp -- parallel inflate of ONE gzip stream for the dictionary reader (dict_reader.hpp).
//
// A gzip member is one DEFLATE stream, so the first pass over one large dictionary was bound by one host core's
// inflate (GzipDecoder, ~37 M words/s on random-looking words, 7.6 MI355X fed at ~4.9 M PMK/s each).
// This decodes the stream in parallel chunks, the way block-boundary-search decompressors do:
//   1. the compressed file is cut into C-byte chunks; in chunk j > 0 a worker searches the first bit position that
//      starts a dynamic-Huffman block (GzipDecoder::maybe_dynamic pre-test, then probe_block: valid code tables, the
//      block decodes to its end, a valid next block type follows);
//   2. chunk j is decoded from its boundary to chunk j+1's boundary.  Its preceding 32 KiB are unknown, so it first
//      decodes into 16-bit symbols where a back-reference into that window becomes a marker (GzipDecoder::read16),
//      and switches to the byte decoder as soon as its last 32 KiB hold no marker (for text, after a few tens of
//      KiB);
//   3. the caller's thread takes the chunks in order, replaces each chunk's markers from the previous chunk's last
//      32 KiB, checks every member's CRC-32 and ISIZE over the joined output, and hands the bytes on.
// A chunk whose end does not land exactly on the next chunk's boundary (a false find) or any decode error stops the
// parallel decode: the caller continues from the bytes delivered with zlib's gzread (dict_reader.hpp), which also
// decides what a damaged stream yields.  The input is read (pread, by a loader thread running ahead of the workers)
// into a zero-filled anonymous region, so every decoder can read GzipDecoder::PAD zero bytes past the end.  It is
// not memory-mapped: another help_crack in the same directory may truncate and rewrite a dictionary while it is read
// (cracked.txt.gz is re-downloaded every 100 work units), and a mapped page past the new end of file raises SIGBUS.
// A short read leaves zeros, which fail the decode and hand the file to zlib (a damaged-file outcome, not a crash).
#pragma once
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "inflate.hpp"

namespace dwpa {

class ParallelGunzip {
  public:
    static constexpr uint64_t NONE = ~0ull;
    static constexpr size_t OUT_BLOCK = 1u << 20;  // byte-decoder output per piece

    // sink(data, n) receives the output in order (n > 0); return false to stop (cancel).
    using Sink = std::function<bool(const uint8_t*, size_t)>;

    // Decodes the gzip file `fd` (size `n`) with `threads` workers and `chunk` compressed bytes per chunk.  Returns the
    // bytes handed to sink; *err is nullptr when the whole stream was decoded and checked, else the reason the
    // parallel decode stopped (the caller continues after the returned count).
    // The parallel decode stopped because a chunk boundary was a false find (the stream itself may be intact), not
    // because the stream is damaged.
    static bool false_boundary(const char* err) {
        return err && (!strcmp(err, "deflate block boundary mismatch") ||
                       !strcmp(err, "stream ended before the chunk boundary") || !strcmp(err, "mmap failed") ||
                       !strcmp(err, "short read"));
    }
    struct Stats {
        size_t chunks = 0;     // compressed chunks
        size_t decoded = 0;    // chunks decoded on their own (a boundary was found in them)
        size_t marker_syms = 0;  // symbols decoded in the marker phase (all chunks)
    };
    static uint64_t run(int fd, size_t n, unsigned threads, size_t chunk, const Sink& sink, const char** err,
                        Stats* stats = nullptr) {
        ParallelGunzip g(fd, n, threads, chunk);
        const uint64_t r = g.go(sink, err);
        if (stats) *stats = g.stats_;
        return r;
    }

  private:
    struct Piece {
        std::vector<uint8_t> buf;
        size_t begin = 0, end = 0;
    };
    struct Job {
        // boundary search
        bool found_done = false;
        uint64_t start = NONE;
        // decode
        bool submitted = false, decoded = false;
        const char* err = nullptr;
        std::vector<uint16_t> head;   // marker phase output
        std::vector<Piece> pieces;    // byte phase output
        std::vector<GzipDecoder::Trailer> trailers;
    };

    ParallelGunzip(int fd, size_t n, unsigned threads, size_t chunk)
        : n_(n), chunk_(std::max<size_t>(chunk, 1u << 16)), nthreads_(std::max(1u, threads)) {
        const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
        maplen_ = (n + GzipDecoder::PAD + 16 + pg - 1) / pg * pg + pg;
        void* area = mmap(nullptr, maplen_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (area == MAP_FAILED) return;
        data_ = (const uint8_t*)area;
        nchunks_ = (n + chunk_ - 1) / chunk_;
        jobs_.resize(nchunks_);
        try {
            loader_ = std::thread([this, fd, area] { load(fd, (uint8_t*)area); });
            for (unsigned t = 0; t < nthreads_; t++) pool_.emplace_back([this] { worker(); });
        } catch (...) {  // a thread that cannot start: stop and join the ones that did, then report it
            shutdown();
            throw;
        }
    }
    ~ParallelGunzip() { shutdown(); }
    void shutdown() {
        quit_flag_.store(true, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : pool_)
            if (t.joinable()) t.join();
        if (loader_.joinable()) loader_.join();
        if (data_) munmap((void*)data_, maplen_);
        data_ = nullptr;
    }

    // The loader: the file in order, LOAD_STEP bytes per pread, publishing how far it got (the ThreadSanitizer build
    // uses 16 KiB steps, so boundary probes keep running into bytes still being loaded).
#ifndef DWPA_PINFLATE_LOAD_STEP
#define DWPA_PINFLATE_LOAD_STEP (4u << 20)
#endif
    static constexpr size_t LOAD_STEP = DWPA_PINFLATE_LOAD_STEP;
    void load(int fd, uint8_t* area) {
        size_t pos = 0;
        while (pos < n_ && !quit_flag_.load(std::memory_order_relaxed)) {
            const ssize_t r = pread(fd, area + pos, std::min(LOAD_STEP, n_ - pos), (off_t)pos);
            if (r <= 0) {  // truncated (or unreadable) under us: the rest stays zero and fails the decode
                short_.store(true, std::memory_order_relaxed);
                break;
            }
            pos += (size_t)r;
            std::lock_guard<std::mutex> lk(load_mu_);
            loaded_.store(pos, std::memory_order_release);
            load_cv_.notify_all();
        }
        std::lock_guard<std::mutex> lk(load_mu_);
        loaded_.store(n_, std::memory_order_release);  // done (or given up): nothing more to wait for
        load_cv_.notify_all();
    }
    // Wait until bytes [0, min(end, n)) are loaded.
    void need(uint64_t end) {
        end = std::min<uint64_t>(end, n_);
        if (loaded_.load(std::memory_order_acquire) >= end) return;
        std::unique_lock<std::mutex> lk(load_mu_);
        load_cv_.wait(lk, [&] { return loaded_.load(std::memory_order_acquire) >= end; });
    }

    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            tasks_.push_back(std::move(f));
        }
        cv_.notify_all();
    }
    void worker() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return quit_ || !tasks_.empty(); });
                if (tasks_.empty()) return;
                f = std::move(tasks_.front());
                tasks_.pop_front();
                running_++;
            }
            f();
            std::lock_guard<std::mutex> lk(mu_);
            running_--;
            done_cv_.notify_all();
        }
    }

    // Input end a decoder may be given now: every byte it can read (its end plus GzipDecoder::PAD and a refill word)
    // is below what the loader has published, so no read races the loader's pread into the same bytes.
    size_t safe_end() const {
        const size_t l = loaded_.load(std::memory_order_acquire);
        constexpr size_t MARGIN = GzipDecoder::PAD + 16;
        return l >= n_ ? n_ : (l > MARGIN ? l - MARGIN : 0);
    }

    // first dynamic-block boundary in chunk j's bytes (NONE if there is none)
    uint64_t find(size_t j) {
        need((uint64_t)(j + 3) * chunk_);  // the chunk, and blocks probed from its end into the next ones
        const uint64_t b = (uint64_t)j * chunk_ * 8, e = (uint64_t)std::min(n_, (j + 1) * chunk_) * 8;
        size_t lim = safe_end();
        auto dec = std::make_unique<GzipDecoder>(data_, lim, true);
        std::vector<uint16_t> scratch;
        for (uint64_t p = b; p < e; p++) {
            if (!GzipDecoder::maybe_dynamic(data_, p)) continue;
            for (;;) {
                // a probe decodes a whole candidate block, which may run past the chunks loaded so far: the decoder
                // sees only [0, lim), and a probe that reached lim is no verdict -- wait for more input, probe again
                dec->start_block(p, nullptr, 0);
                if (dec->probe_block(scratch)) return p;
                if (lim >= n_ || dec->bit_pos() / 8 + 16 < lim) break;
                need(lim + GzipDecoder::PAD + 16 + LOAD_STEP);
                lim = safe_end();
                dec = std::make_unique<GzipDecoder>(data_, lim, true);
            }
        }
        return NONE;
    }

    // chunk j from bit `start` (0 = the file's gzip header) to bit `stop` (NONE = the end of the stream).  An
    // allocation that fails ends the chunk with an error: go() then hands the rest of the file to gzread.
    void decode(size_t j, uint64_t start, uint64_t stop) {
        try {
            decode_chunk(j, start, stop);
        } catch (...) {
            Job& J = jobs_[j];
            J.err = "out of memory in the parallel inflate";
            J.pieces.clear();
            J.trailers.clear();
        }
        std::lock_guard<std::mutex> lk(mu_);
        jobs_[j].decoded = true;
        done_cv_.notify_all();
    }
    void decode_chunk(size_t j, uint64_t start, uint64_t stop) {
        need(stop == NONE ? n_ : stop / 8 + 2 * chunk_);
        Job& J = jobs_[j];
        GzipDecoder dec(data_, n_, true);
        bool bytes = false;
        if (j == 0) {
            bytes = true;  // no unknown window before the stream's start
        } else {
            dec.start_block(start, nullptr, 0);
        }
        if (stop != NONE) dec.stop_at(stop);
        if (!bytes) {
            const int r = dec.read16(J.head);
            if (r == GzipDecoder::R16_ERR) J.err = dec.error();
            else if (r == GzipDecoder::R16_SWITCH) {
                std::vector<uint8_t> h(GzipDecoder::WIN);
                const uint16_t* src = J.head.data() + J.head.size() - GzipDecoder::WIN;
                for (size_t i = 0; i < GzipDecoder::WIN; i++) h[i] = (uint8_t)src[i];
                dec.set_history(h.data(), h.size());
                bytes = true;
            }
        }
        if (bytes && !J.err) {
            for (;;) {
                Piece pc;
                pc.buf.resize(GzipDecoder::WIN + OUT_BLOCK + GzipDecoder::SLACK);
                const size_t got = dec.read(pc.buf.data(), OUT_BLOCK);
                if (dec.failed()) {
                    J.err = dec.error();
                    break;
                }
                pc.begin = GzipDecoder::WIN;
                pc.end = pc.begin + got;
                if (got) J.pieces.push_back(std::move(pc));
                if (dec.done() || dec.stopped()) break;
            }
        }
        J.trailers = dec.trailers();
    }

    uint64_t wait_start(size_t j) {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return jobs_[j].found_done; });
        return jobs_[j].start;
    }

    uint64_t go(const Sink& sink, const char** err) {
        *err = nullptr;
        if (!data_) {
            *err = "mmap failed";
            return 0;
        }
        const size_t ahead = 2 * nthreads_;
        stats_.chunks = nchunks_;
        size_t next_find = 1, next_dec = 0;
        jobs_[0].found_done = true;
        jobs_[0].start = 0;
        auto submit_finds = [&](size_t upto) {
            for (; next_find < nchunks_ && next_find <= upto; next_find++) {
                const size_t j = next_find;
                submit([this, j] {
                    uint64_t s;
                    try {
                        s = find(j);
                    } catch (...) {  // no memory for the probe: no boundary, the previous chunk decodes through
                        s = NONE;
                    }
                    std::lock_guard<std::mutex> lk(mu_);
                    jobs_[j].start = s;
                    jobs_[j].found_done = true;
                    done_cv_.notify_all();
                });
            }
        };
        std::vector<uint8_t> window;  // the last <= 32 KiB delivered
        uint64_t delivered = 0;
        // member CRC-32 / ISIZE over the delivered bytes
        uint32_t crc = 0, isize = 0;
        std::vector<GzipDecoder::Trailer> pending;  // absolute ends, in order
        size_t tp = 0;
        bool stop = false;
        auto emit = [&](const uint8_t* p, size_t k) -> bool {
            while (k && !stop) {
                size_t take = k;
                if (tp < pending.size() && pending[tp].end - delivered < take) take = (size_t)(pending[tp].end - delivered);
                if (take) {
                    crc = Crc32::get()(crc, p, take);
                    isize += (uint32_t)take;
                    if (!sink(p, take)) {
                        stop = true;
                        return false;
                    }
                    delivered += take;
                    p += take;
                    k -= take;
                }
                while (tp < pending.size() && pending[tp].end == delivered) {
                    if (pending[tp].crc != crc || pending[tp].isize != isize) {
                        *err = pending[tp].crc != crc ? "gzip CRC-32 mismatch" : "gzip ISIZE mismatch";
                        stop = true;
                        return false;
                    }
                    crc = 0;
                    isize = 0;
                    tp++;
                }
            }
            return !stop;
        };
        auto keep_window = [&](const uint8_t* p, size_t k) {
            if (k >= GzipDecoder::WIN) {
                window.assign(p + k - GzipDecoder::WIN, p + k);
            } else {
                window.insert(window.end(), p, p + k);
                if (window.size() > GzipDecoder::WIN) window.erase(window.begin(), window.end() - GzipDecoder::WIN);
            }
        };
        size_t cur = 0;  // next chunk to deliver
        while (cur < nchunks_ && !stop) {
            submit_finds(cur + ahead + 1);
            // submit decodes of chunks whose both ends are known
            while (next_dec < nchunks_ && next_dec <= cur + ahead) {
                const size_t j = next_dec;
                const uint64_t s = wait_start(j);
                if (s == NONE) {  // no boundary in chunk j: the previous chunk decodes through it
                    next_dec++;
                    continue;
                }
                size_t k = j + 1;
                uint64_t e = NONE;
                for (; k < nchunks_; k++) {
                    submit_finds(k + 1);
                    if ((e = wait_start(k)) != NONE) break;
                }
                jobs_[j].submitted = true;
                submit([this, j, s, e] { decode(j, s, e); });
                next_dec = k;
            }
            Job& J = jobs_[cur];
            if (!J.submitted) {  // merged into an earlier chunk
                cur++;
                continue;
            }
            {
                std::unique_lock<std::mutex> lk(mu_);
                done_cv_.wait(lk, [&] { return J.decoded; });
            }
            stats_.decoded++;
            stats_.marker_syms += J.head.size();
            const uint64_t base = delivered;
            for (const auto& t : J.trailers) pending.push_back(GzipDecoder::Trailer{base + t.end, t.crc, t.isize});
            // markers -> bytes from the previous chunk's window
            if (!J.head.empty()) {
                std::vector<uint8_t> h(J.head.size());
                const size_t wsz = window.size();
                for (size_t i = 0; i < h.size(); i++) {
                    const uint16_t v = J.head[i];
                    if (v < 256) {
                        h[i] = (uint8_t)v;
                        continue;
                    }
                    const size_t w = (size_t)(v - GzipDecoder::MARK);  // WIN + offset before the chunk
                    if (w + wsz < GzipDecoder::WIN) {
                        *err = "distance too far back";
                        stop = true;
                        break;
                    }
                    h[i] = window[w + wsz - GzipDecoder::WIN];
                }
                if (stop) break;
                J.head.clear();
                J.head.shrink_to_fit();
                if (!emit(h.data(), h.size())) break;
                keep_window(h.data(), h.size());
            }
            for (auto& pc : J.pieces) {
                if (!emit(pc.buf.data() + pc.begin, pc.end - pc.begin)) break;
                keep_window(pc.buf.data() + pc.begin, pc.end - pc.begin);
                std::vector<uint8_t>().swap(pc.buf);
            }
            if (stop) break;
            if (J.err) {  // a decode error (or a false boundary) after the bytes delivered so far
                *err = J.err;
                break;
            }
            J.pieces.clear();
            cur++;
        }
        if (!stop && !*err && short_.load()) *err = "short read";  // the file shrank while it was read
        if (!stop && !*err && tp != pending.size()) *err = "member without its trailer";
        if (!stop && !*err && pending.empty()) *err = "truncated gzip stream";
        if (!stop && !*err && pending.back().end != delivered) *err = "truncated gzip stream";
        // drain: drop the queued tasks and let the running ones finish before the jobs go away; stop the loader
        quit_flag_.store(true, std::memory_order_relaxed);
        {
            std::unique_lock<std::mutex> lk(mu_);
            tasks_.clear();
            done_cv_.wait(lk, [&] { return running_ == 0; });
        }
        return delivered;
    }

    const uint8_t* data_ = nullptr;
    size_t n_ = 0, maplen_ = 0, chunk_, nchunks_ = 0;
    unsigned nthreads_;
    std::vector<Job> jobs_;
    std::vector<std::thread> pool_;
    std::thread loader_;
    std::mutex load_mu_;
    std::condition_variable load_cv_;
    std::atomic<size_t> loaded_{0};
    std::atomic<bool> short_{false}, quit_flag_{false};
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<std::function<void()>> tasks_;
    bool quit_ = false;
    unsigned running_ = 0;
    Stats stats_;
};

}  // namespace dwpa
