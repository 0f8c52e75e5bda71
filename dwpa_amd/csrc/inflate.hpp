// inflate.hpp -- gzip (RFC 1952) / DEFLATE (RFC 1951) decoder for the dictionary reader (dict_reader.hpp).
//
// help_crack hands hashcat gzip wordlists (help_crack.py:520-552).  With one ESSID and no rules an MI355X consumes
// ~4.9 M words/s, so one 8-GPU node needs ~40 M words/s from a dictionary's first pass, and a gzip member cannot be
// inflated in parallel.  zlib 1.2.11's inflate delivered ~320 MB/s (~28 M words/s) on the GPU box's EPYC.  This
// decoder is built for throughput on a host core:
//   * a 64-bit bit buffer refilled branch-free with one unaligned 8-byte load (input buffers carry a zero pad);
//   * one-lookup Huffman decoding: 11-bit literal/length and 8-bit distance primary tables whose entries carry the
//     symbol's base value and extra-bit count, plus second-level tables for longer codes;
//   * match copies in 8-byte words (distance >= 8) or a replicated pattern (distance < 8);
//   * CRC-32 by carry-less multiply folding (PCLMULQDQ), checked at start-up against a table CRC.
// It decodes into caller buffers that hold the last 32 KiB of output in front of the new bytes, so back-references
// never need a ring buffer.  Concatenated members are decoded in turn; bytes after the last member that do not start
// a gzip header end the stream (what gzread does).  Errors: bad header, invalid block or code, distance beyond the
// output so far, truncated input, CRC-32 or ISIZE mismatch.
#pragma once
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>
#include <wmmintrin.h>
#include <emmintrin.h>
#include <smmintrin.h>

#include <vector>

namespace dwpa {

// ---------------------------------------------------------------------------------------------------------
// CRC-32 (gzip, reflected polynomial 0xEDB88320)
// ---------------------------------------------------------------------------------------------------------
struct Crc32 {
    uint32_t t[8][256];
    bool clmul_ok = false;
    Crc32() {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = c & 1 ? (c >> 1) ^ 0xEDB88320u : c >> 1;
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; i++)
            for (int s = 1; s < 8; s++) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
        uint8_t probe[1024];
        for (int i = 0; i < 1024; i++) probe[i] = (uint8_t)(i * 131 + 7);
        clmul_ok = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
        if (clmul_ok) clmul_ok = fold(0, probe, 1024) == table(0, probe, 1024) &&
                                 fold(0x12345678u, probe + 3, 777) == table(0x12345678u, probe + 3, 777);
    }
    // slice-by-8 (short inputs, heads and tails, and the reference for the self-check)
    uint32_t table(uint32_t crc, const uint8_t* p, size_t n) const {
        crc = ~crc;
        for (; n >= 8; p += 8, n -= 8) {
            uint32_t a, b;
            memcpy(&a, p, 4);
            memcpy(&b, p + 4, 4);
            a ^= crc;
            crc = t[7][a & 0xff] ^ t[6][(a >> 8) & 0xff] ^ t[5][(a >> 16) & 0xff] ^ t[4][a >> 24] ^ t[3][b & 0xff] ^
                  t[2][(b >> 8) & 0xff] ^ t[1][(b >> 16) & 0xff] ^ t[0][b >> 24];
        }
        while (n--) crc = (crc >> 8) ^ t[0][(crc ^ *p++) & 0xff];
        return ~crc;
    }
    __attribute__((target("pclmul,sse4.1"))) static __m128i fold128(__m128i x, __m128i k, __m128i d) {
        return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), d);
    }
    // Carry-less multiply folding, four 128-bit lanes (64 bytes per step), then Barrett reduction.
    __attribute__((target("pclmul,sse4.1"))) uint32_t fold(uint32_t crc, const uint8_t* p, size_t n) const {
        if (n < 128) return table(crc, p, n);
        const __m128i k1k2 = _mm_set_epi64x(0x1c6e41596ll, 0x154442bd4ll);  // x^(4*128+32), x^(4*128-32) mod P
        const __m128i k3k4 = _mm_set_epi64x(0x0ccaa009ell, 0x1751997d0ll);  // x^(128+32), x^(128-32) mod P
        const __m128i k5 = _mm_set_epi64x(0, 0x163cd6124ll);
        const __m128i poly = _mm_set_epi64x(0x1f7011641ll, 0x1db710641ll);  // mu', P'
        const __m128i mask32 = _mm_set_epi32(0, 0, 0, -1);
        __m128i x0 = _mm_loadu_si128((const __m128i*)p), x1 = _mm_loadu_si128((const __m128i*)(p + 16)),
                x2 = _mm_loadu_si128((const __m128i*)(p + 32)), x3 = _mm_loadu_si128((const __m128i*)(p + 48));
        x0 = _mm_xor_si128(x0, _mm_cvtsi32_si128((int)~crc));
        p += 64;
        n -= 64;
        for (; n >= 64; p += 64, n -= 64) {
            x0 = fold128(x0, k1k2, _mm_loadu_si128((const __m128i*)p));
            x1 = fold128(x1, k1k2, _mm_loadu_si128((const __m128i*)(p + 16)));
            x2 = fold128(x2, k1k2, _mm_loadu_si128((const __m128i*)(p + 32)));
            x3 = fold128(x3, k1k2, _mm_loadu_si128((const __m128i*)(p + 48)));
        }
        x0 = fold128(x0, k3k4, x1);
        x0 = fold128(x0, k3k4, x2);
        x0 = fold128(x0, k3k4, x3);
        for (; n >= 16; p += 16, n -= 16) x0 = fold128(x0, k3k4, _mm_loadu_si128((const __m128i*)p));
        // 128 -> 64 bits, then 64 -> 32 (Barrett)
        __m128i x = _mm_xor_si128(_mm_clmulepi64_si128(x0, k3k4, 0x10), _mm_srli_si128(x0, 8));
        x = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x, mask32), k5, 0x00), _mm_srli_si128(x, 4));
        __m128i tt = _mm_clmulepi64_si128(_mm_and_si128(x, mask32), poly, 0x10);
        tt = _mm_clmulepi64_si128(_mm_and_si128(tt, mask32), poly, 0x00);
        const uint32_t c = (uint32_t)_mm_extract_epi32(_mm_xor_si128(x, tt), 1);
        return table(~c, p, n);
    }
    uint32_t operator()(uint32_t crc, const uint8_t* p, size_t n) const {
        return clmul_ok ? fold(crc, p, n) : table(crc, p, n);
    }
    static const Crc32& get() {
        static const Crc32 c;
        return c;
    }
};

// ---------------------------------------------------------------------------------------------------------
// DEFLATE decoder
// ---------------------------------------------------------------------------------------------------------
class GzipDecoder {
  public:
    static constexpr size_t WIN = 32768;  // history kept in front of every output block
    static constexpr size_t SLACK = 320;  // output room past the limit: one match (258) + an 8-byte word copy

    static constexpr size_t PAD = 64;     // zero bytes the input must carry past its end
    static constexpr uint16_t MARK = 0x8000;  // read16: MARK + w = byte w of the unknown window (0 = oldest)

    explicit GzipDecoder(int fd) : fd_(fd), in_(INCAP + PAD, 0) {
        base_ = in_ptr_ = in_end_ = in_.data();
        build_fixed();
    }
    // In-memory input data[0, n), followed by at least PAD readable zero bytes (parallel chunks, pinflate.hpp).  With
    // `chunk` set the decoder checks no CRC-32/ISIZE itself (its output is part of a stream decoded in pieces): member
    // trailers are recorded in trailers() for the caller, who checks them over the joined output.
    GzipDecoder(const uint8_t* data, size_t n, bool chunk) : fd_(-1), mem_(true), chunk_(chunk) {
        base_ = in_ptr_ = const_cast<uint8_t*>(data);  // never written: fill() does nothing in memory mode
        in_end_ = base_ + n;
        eof_ = true;
        build_fixed();
    }
    bool failed() const { return st_ == ERR; }
    bool done() const { return st_ == DONE; }
    bool stopped() const { return st_ == STOPPED; }
    const char* error() const { return err_; }

    struct Trailer {
        uint64_t end;  // output offset just past the member's last byte
        uint32_t crc, isize;
    };
    const std::vector<Trailer>& trailers() const { return trailers_; }
    uint64_t out_total() const { return out_total_; }
    // input bits consumed (memory mode)
    uint64_t bit_pos() const { return (uint64_t)(in_ptr_ - base_) * 8 - bc_; }
    // Memory mode: start at the deflate block header at bit `pos`, with `hlen` bytes of history (0: unknown window,
    // decode with read16 first).
    void start_block(uint64_t pos, const uint8_t* hist, size_t hlen) {
        in_ptr_ = base_ + pos / 8;
        bb_ = 0;
        bc_ = 0;
        refill();
        bb_ >>= pos & 7;
        bc_ -= (uint32_t)(pos & 7);
        hist_.assign(hist, hist + hlen);
        st_ = BLOCK;
        members_ = 1;
        err_ = nullptr;
    }
    // Stop (stopped()) at the block boundary at bit `pos`; running past it without landing on it is an error (the
    // next chunk's boundary was a false find).
    void stop_at(uint64_t pos) { stop_ = pos; }
    void set_history(const uint8_t* h, size_t n) { hist_.assign(h, h + n); }

    // Boundary probe (memory mode, right after start_block): the block there is a dynamic-Huffman block whose code
    // tables are valid and which decodes to its end-of-block (back-references into the unknown window allowed),
    // followed by a valid next block type or the member's end.
    bool probe_block(std::vector<uint16_t>& scratch) {
        scratch.clear();
        uint8_t* d = nullptr;
        step(d, d);
        if (st_ != HUFF || lt_ != dyn_l_.data()) return false;
        huff16(scratch);
        if (st_ == TRAILER) return !scratch.empty();
        if (st_ != BLOCK || scratch.empty()) return false;
        refill();
        return ((bb_ >> 1) & 3) != 3;
    }
    // Cheap pre-test of a dynamic block header at bit p of d (d padded): block type 2, HLIT/HDIST in range and a
    // complete code-length code (what build() demands) -- rejects all but a few per cent of bit positions.
    static bool maybe_dynamic(const uint8_t* d, uint64_t p) {
        uint64_t w0, w1;
        memcpy(&w0, d + p / 8, 8);
        memcpy(&w1, d + p / 8 + 8, 8);
        const uint32_t sh = (uint32_t)(p & 7);
        const uint64_t lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;  // 64 bits from p
        const uint64_t hi = w1 >> sh;                                     // bits 64.. (>= 56 of them)
        if (((lo >> 1) & 3) != 2) return false;
        if (((lo >> 3) & 31) > 29 || ((lo >> 8) & 31) > 29) return false;
        const uint32_t hclen = (uint32_t)((lo >> 13) & 15) + 4;
        uint32_t kraft = 0, nz = 0;
        for (uint32_t i = 0; i < hclen; i++) {
            const uint32_t b = 17 + 3 * i;
            const uint32_t l = b + 3 <= 64 ? (uint32_t)((lo >> b) & 7)
                               : b >= 64 ? (uint32_t)((hi >> (b - 64)) & 7)
                                         : (uint32_t)(((lo >> b) | (hi << (64 - b))) & 7);
            if (l) {
                kraft += 128u >> l;
                nz++;
            }
        }
        return kraft == 128 && nz >= 2;
    }

    // Marker phase of a chunk whose preceding 32 KiB are not known yet: appends 16-bit symbols to out, a byte value
    // (< 256) or MARK + w for byte w of that window.  Returns at a block boundary: R16_SWITCH once out holds >= WIN
    // symbols of which the last WIN are bytes (the caller continues with read() after set_history), R16_STOP at
    // stop_at's boundary, R16_END at the end of the stream, R16_ERR on an error.
    enum { R16_SWITCH, R16_STOP, R16_END, R16_ERR };
    int read16(std::vector<uint16_t>& out) {
        const size_t out0 = out.size();
        int r = R16_ERR;
        for (;;) {
            if (st_ == ERR) break;
            if (st_ == DONE) {
                if (stop_ != NO_STOP) fail("stream ended before the chunk boundary");
                else r = R16_END;
                break;
            }
            if (st_ == HEADER) {
                if (!read_header() && st_ != DONE) break;
                continue;
            }
            if (st_ == TRAILER) {
                cur_out_ = out_total_ + (out.size() - out0);
                finish_member();
                continue;
            }
            if (st_ == BLOCK) {
                if (stop_ != NO_STOP && bit_pos() >= stop_) {
                    if (bit_pos() == stop_) {
                        st_ = STOPPED;
                        r = R16_STOP;
                    } else {
                        fail("deflate block boundary mismatch");
                    }
                    break;
                }
                if (out.size() >= WIN && no_marker(out.data() + out.size() - WIN, WIN)) {
                    r = R16_SWITCH;
                    break;
                }
                uint8_t* d = nullptr;
                step(d, d);  // block header
                continue;
            }
            if (st_ == STORED) {
                while (stored_left_) {
                    const size_t k = (size_t)(in_end_ - in_ptr_) < stored_left_ ? (size_t)(in_end_ - in_ptr_) : stored_left_;
                    if (!k) break;
                    for (size_t i = 0; i < k; i++) out.push_back(in_ptr_[i]);
                    in_ptr_ += k;
                    stored_left_ -= (uint32_t)k;
                }
                if (stored_left_) {
                    fail("truncated stored block");
                    break;
                }
                end_block(nullptr);
                continue;
            }
            if (st_ == HUFF) {
                huff16(out);
                continue;
            }
            break;
        }
        out_total_ += out.size() - out0;
        return st_ == ERR ? R16_ERR : r;
    }

    // Decodes up to `want` new bytes into buf[WIN, WIN + want); buf must hold WIN + want + SLACK bytes.  The stream's
    // last <= 32 KiB of output is copied into buf[WIN - h, WIN) first.  Returns the new bytes (0: end of stream or
    // error -- see failed()).
    size_t read(uint8_t* buf, size_t want) {
        if (st_ == DONE || st_ == ERR || st_ == STOPPED) return 0;
        memcpy(buf + WIN - hist_.size(), hist_.data(), hist_.size());
        hist_start_ = buf + WIN - hist_.size();
        uint8_t* o = buf + WIN;
        uint8_t* const lim = o + want;
        uint8_t* seg = o;  // first byte of the current member in this call (CRC-32 / ISIZE)
        while (o < lim && st_ != DONE && st_ != ERR && st_ != STOPPED) {
            if (st_ == HEADER) {
                if (!read_header()) break;
                seg = o;
                continue;
            }
            o = step(o, lim);
            if (st_ == TRAILER) {  // the member's last block ended: check its trailer, then look for another member
                if (!chunk_) {
                    crc_ = Crc32::get()(crc_, seg, (size_t)(o - seg));
                    isize_ += (uint32_t)(o - seg);
                }
                seg = o;
                cur_out_ = out_total_ + (uint64_t)(o - (buf + WIN));
                finish_member();
            }
        }
        if (st_ != ERR && !chunk_) {
            crc_ = Crc32::get()(crc_, seg, (size_t)(o - seg));
            isize_ += (uint32_t)(o - seg);
        }
        if (st_ == DONE && stop_ != NO_STOP) fail("stream ended before the chunk boundary");
        // keep the last 32 KiB as the next block's history
        const size_t have = (size_t)(o - hist_start_), keep = have < WIN ? have : WIN;
        hist_.assign(o - keep, o);
        out_total_ += (uint64_t)(o - (buf + WIN));
        return st_ == ERR ? 0 : (size_t)(o - (buf + WIN));
    }

  private:
    static constexpr size_t INCAP = 4u << 20;
    static constexpr uint64_t NO_STOP = ~0ull;
    enum St { HEADER, BLOCK, STORED, HUFF, TRAILER, DONE, ERR, STOPPED };
    // table entry: bits 0-3 code length, 4-7 extra bits (SUB: index bits), 8-9 kind, 10 invalid, 16-31 value
    enum : uint32_t { K_LIT = 0, K_LEN = 1u << 8, K_EOB = 2u << 8, K_SUB = 3u << 8, K_MASK = 3u << 8, K_BAD = 1u << 10 };
    static constexpr int LBITS = 11, DBITS = 8, CBITS = 7;
    static constexpr size_t LSIZE = (1u << LBITS) + 288 * 16, DSIZE = (1u << DBITS) + 32 * 128;

    static uint32_t crc_update(uint32_t crc, const uint8_t* p, size_t n) { return Crc32::get()(crc, p, n); }

    // ---- input ----
    // Keeps the bytes from in_ptr_ - 8 on (a stored block or the trailer may step back over whole bytes that are
    // still in the bit buffer), reads more, zero-pads.
    void fill() {
        if (eof_ || mem_) return;
        uint8_t* keep = in_ptr_ - 8 > in_.data() ? in_ptr_ - 8 : in_.data();
        const size_t back = (size_t)(in_ptr_ - keep), tail = (size_t)(in_end_ - keep);
        memmove(in_.data(), keep, tail);
        in_ptr_ = in_.data() + back;
        in_end_ = in_.data() + tail;
        while (!eof_ && (size_t)(in_end_ - in_.data()) < INCAP) {
            const ssize_t r = ::read(fd_, in_end_, INCAP - (size_t)(in_end_ - in_.data()));
            if (r < 0) { fail("read error"); break; }
            if (r == 0) eof_ = true;
            in_end_ += r;
        }
        memset(in_end_, 0, PAD);
    }
    // at least n input bytes past in_ptr_ unless the file ends first
    void need(size_t n) {
        if ((size_t)(in_end_ - in_ptr_) < n) fill();
    }
    void refill() {  // bit buffer to 56..63 bits (reads the zero pad at the end of the file)
        uint64_t w;
        memcpy(&w, in_ptr_, 8);
        bb_ |= w << bc_;
        in_ptr_ += (63 - bc_) >> 3;
        bc_ |= 56;
    }
    uint32_t bits(int n) {  // n <= 32
        if (bc_ < (uint32_t)n) refill();
        const uint32_t v = (uint32_t)(bb_ & ((1ull << n) - 1));
        bb_ >>= n;
        bc_ -= n;
        return v;
    }
    void align_unread() {  // drop to a byte boundary and hand the whole bytes in the bit buffer back to the input
        bb_ >>= bc_ & 7;
        bc_ &= ~7u;
        in_ptr_ -= bc_ >> 3;
        bb_ = 0;
        bc_ = 0;
    }
    bool overrun() const { return eof_ && in_ptr_ - (bc_ >> 3) > in_end_; }
    void fail(const char* e) {
        st_ = ERR;
        err_ = e;
    }

    // ---- Huffman tables ----
    // Canonical code lengths -> lookup table of tb primary bits (+ second-level tables).  info[s] = value | extra << 4 |
    // kind for symbol s (K_BAD for symbols that must not occur).  Incomplete codes are accepted only with a single
    // code of length 1 (or none), as zlib does for literal/length and distance codes; code-length codes must be
    // complete.
    static bool build(const uint8_t* len, int n, const uint32_t* info, uint32_t* tab, int tb, bool complete) {
        uint16_t count[16] = {0}, offs[16], sorted[320];
        for (int s = 0; s < n; s++) count[len[s]]++;
        count[0] = 0;
        int left = 1, maxl = 0;
        for (int l = 1; l < 16; l++) {
            left = (left << 1) - count[l];
            if (left < 0) return false;  // over-subscribed
            if (count[l]) maxl = l;
        }
        if (left > 0 && (complete || maxl > 1)) return false;  // incomplete
        offs[1] = 0;
        for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + count[l];
        for (int s = 0; s < n; s++)
            if (len[s]) sorted[offs[len[s]]++] = (uint16_t)s;
        const uint32_t psize = 1u << tb;
        for (uint32_t i = 0; i < psize; i++) tab[i] = K_BAD;
        // second-level table sizes per primary prefix
        uint32_t code = 0, k = 0, next = psize;
        uint8_t subbits[1 << 11] = {0};
        uint32_t suboff[1 << 11];
        {
            uint32_t c = 0, kk = 0;
            for (int l = 1; l < 16; l++, c <<= 1)
                for (int j = 0; j < count[l]; j++, kk++, c++)
                    if (l > tb) {
                        const uint32_t r = rev(c, l) & (psize - 1);
                        if (l - tb > subbits[r]) subbits[r] = (uint8_t)(l - tb);
                    }
        }
        for (uint32_t r = 0; r < psize; r++)
            if (subbits[r]) {
                suboff[r] = next;
                tab[r] = K_SUB | (uint32_t)subbits[r] << 4 | next << 16;
                for (uint32_t i = 0; i < (1u << subbits[r]); i++) tab[next + i] = K_BAD;
                next += 1u << subbits[r];
            }
        for (int l = 1; l < 16; l++, code <<= 1)
            for (int j = 0; j < count[l]; j++, k++, code++) {
                const uint32_t s = sorted[k], r = rev(code, l), e = info[s] | (uint32_t)l;
                if (l <= tb) {
                    for (uint32_t i = r; i < psize; i += 1u << l) tab[i] = e;
                } else {
                    const uint32_t p = r & (psize - 1), sb = subbits[p];
                    for (uint32_t i = r >> tb; i < (1u << sb); i += 1u << (l - tb)) tab[suboff[p] + i] = e;
                }
            }
        return true;
    }
    static uint32_t rev(uint32_t c, int l) {
        uint32_t r = 0;
        for (int i = 0; i < l; i++, c >>= 1) r = r << 1 | (c & 1);
        return r;
    }
    static const uint32_t* litlen_info() {
        static uint32_t info[288];
        static bool init = [] {
            static const uint16_t base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                              31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
            static const uint8_t extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                              2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
            for (uint32_t s = 0; s < 256; s++) info[s] = K_LIT | s << 16;
            info[256] = K_EOB;
            for (uint32_t s = 257; s < 286; s++) info[s] = K_LEN | (uint32_t)extra[s - 257] << 4 | (uint32_t)base[s - 257] << 16;
            info[286] = info[287] = K_BAD;
            return true;
        }();
        (void)init;
        return info;
    }
    static const uint32_t* dist_info() {
        static uint32_t info[32];
        static bool init = [] {
            static const uint16_t base[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                              193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
            for (uint32_t s = 0; s < 30; s++) info[s] = K_LEN | (uint32_t)(s < 4 ? 0 : (s - 2) / 2) << 4 | (uint32_t)base[s] << 16;
            info[30] = info[31] = K_BAD;
            return true;
        }();
        (void)init;
        return info;
    }
    void build_fixed() {
        uint8_t l[288];
        for (int s = 0; s < 288; s++) l[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
        build(l, 288, litlen_info(), fixed_l_.data(), LBITS, true);
        uint8_t d[32];
        for (int s = 0; s < 32; s++) d[s] = 5;
        build(d, 32, dist_info(), fixed_d_.data(), DBITS, true);
    }
    bool read_dynamic() {
        need(512);
        const int hlit = (int)bits(5) + 257, hdist = (int)bits(5) + 1, hclen = (int)bits(4) + 4;
        if (hlit > 286 || hdist > 30) return false;
        static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        uint8_t cl[19] = {0};
        for (int i = 0; i < hclen; i++) cl[order[i]] = (uint8_t)bits(3);
        uint32_t cinfo[19], ctab[1 << CBITS];
        for (uint32_t s = 0; s < 19; s++) cinfo[s] = K_LIT | s << 16;
        if (!build(cl, 19, cinfo, ctab, CBITS, true)) return false;
        uint8_t lens[286 + 30];
        int i = 0;
        while (i < hlit + hdist) {
            if (bc_ < 16) refill();
            const uint32_t e = ctab[bb_ & ((1u << CBITS) - 1)];
            if (e & K_BAD) return false;
            bb_ >>= e & 15;
            bc_ -= e & 15;
            const uint32_t sym = e >> 16;
            if (sym < 16) {
                lens[i++] = (uint8_t)sym;
                continue;
            }
            uint8_t v = 0;
            int rep;
            if (sym == 16) {
                if (i == 0) return false;
                v = lens[i - 1];
                rep = 3 + (int)bits(2);
            } else if (sym == 17) {
                rep = 3 + (int)bits(3);
            } else {
                rep = 11 + (int)bits(7);
            }
            if (i + rep > hlit + hdist) return false;
            while (rep--) lens[i++] = v;
        }
        if (overrun()) return false;
        if (lens[256] == 0) return false;  // no end-of-block code
        return build(lens, hlit, litlen_info(), dyn_l_.data(), LBITS, false) &&
               build(lens + hlit, hdist, dist_info(), dyn_d_.data(), DBITS, false);
    }

    // ---- members ----
    bool read_header() {
        need(4096);
        if (in_end_ - in_ptr_ < 10) {
            if (in_end_ == in_ptr_ && members_) { st_ = DONE; return false; }
            if (members_) { st_ = DONE; return false; }  // trailing garbage after a member
            fail("truncated gzip header");
            return false;
        }
        const uint8_t* h = in_ptr_;
        if (h[0] != 0x1f || h[1] != 0x8b) {
            if (members_) { st_ = DONE; return false; }  // trailing garbage after a member: ignored, as gzread
            fail("not a gzip file");
            return false;
        }
        if (h[2] != 8 || (h[3] & 0xe0)) { fail("unsupported gzip header"); return false; }
        const uint8_t flg = h[3];
        size_t p = 10;
        auto avail = [&](size_t k) { return (size_t)(in_end_ - in_ptr_) >= p + k; };
        if (flg & 4) {  // FEXTRA
            if (!avail(2)) { fail("truncated gzip header"); return false; }
            p += 2 + (size_t)(h[p] | h[p + 1] << 8);
        }
        for (int f : {8, 16})  // FNAME, FCOMMENT: zero-terminated
            if (flg & f) {
                while (avail(1) && h[p]) p++;
                if (!avail(1)) { fail("truncated gzip header"); return false; }
                p++;
            }
        if (flg & 2) {  // FHCRC: low 16 bits of the CRC-32 of the header bytes before it (zlib checks it)
            if (!avail(2)) { fail("truncated gzip header"); return false; }
            if ((Crc32::get()(0, h, p) & 0xffff) != (uint32_t)(h[p] | h[p + 1] << 8)) {
                fail("gzip header CRC mismatch");
                return false;
            }
            p += 2;
        }
        if (!avail(0)) { fail("truncated gzip header"); return false; }
        in_ptr_ += p;
        bb_ = 0;
        bc_ = 0;
        crc_ = 0;
        isize_ = 0;
        members_++;
        st_ = BLOCK;
        return true;
    }
    void finish_member() {
        align_unread();
        need(8);
        if (in_end_ - in_ptr_ < 8) { fail("truncated gzip trailer"); return; }
        uint32_t c, s;
        memcpy(&c, in_ptr_, 4);
        memcpy(&s, in_ptr_ + 4, 4);
        in_ptr_ += 8;
        if (chunk_) {
            trailers_.push_back(Trailer{cur_out_, c, s});
        } else {
            if (c != crc_) { fail("gzip CRC-32 mismatch"); return; }
            if (s != isize_) { fail("gzip ISIZE mismatch"); return; }
        }
        st_ = HEADER;
    }

    // One state-machine step; returns the new output position.
    uint8_t* step(uint8_t* o, uint8_t* lim) {
        switch (st_) {
            case BLOCK: {
                if (stop_ != NO_STOP && bit_pos() >= stop_) {
                    if (bit_pos() == stop_) st_ = STOPPED;
                    else fail("deflate block boundary mismatch");
                    return o;
                }
                need(64);
                final_ = bits(1);
                const uint32_t type = bits(2);
                if (type == 0) {
                    align_unread();
                    need(4);
                    if (in_end_ - in_ptr_ < 4) { fail("truncated stored block"); return o; }
                    const uint32_t len = in_ptr_[0] | in_ptr_[1] << 8, nlen = in_ptr_[2] | in_ptr_[3] << 8;
                    if ((len ^ 0xffff) != nlen) { fail("invalid stored block length"); return o; }
                    in_ptr_ += 4;
                    stored_left_ = len;
                    st_ = STORED;
                } else if (type == 1) {
                    lt_ = fixed_l_.data();
                    dt_ = fixed_d_.data();
                    st_ = HUFF;
                } else if (type == 2) {
                    if (!read_dynamic()) { fail("invalid dynamic block"); return o; }
                    lt_ = dyn_l_.data();
                    dt_ = dyn_d_.data();
                    st_ = HUFF;
                } else {
                    fail("invalid block type");
                }
                if (overrun()) fail("truncated deflate stream");
                return o;
            }
            case STORED: {
                while (stored_left_ && o < lim) {
                    need(1);
                    size_t k = (size_t)(in_end_ - in_ptr_);
                    if (!k) { fail("truncated stored block"); return o; }
                    if (k > stored_left_) k = stored_left_;
                    if (k > (size_t)(lim - o)) k = (size_t)(lim - o);
                    memcpy(o, in_ptr_, k);
                    o += k;
                    in_ptr_ += k;
                    stored_left_ -= (uint32_t)k;
                }
                if (!stored_left_) end_block(o);
                return o;
            }
            case HUFF:
                return huff(o, lim);
            default:
                return o;
        }
    }
    void end_block(uint8_t*) { st_ = final_ ? TRAILER : BLOCK; }

    uint8_t* huff(uint8_t* o, uint8_t* lim) {
        const uint32_t* lt = lt_;
        const uint32_t* dt = dt_;
        uint64_t bb = bb_;
        uint32_t bc = bc_;
        uint8_t* in = in_ptr_;
        const uint8_t* const hist = hist_start_;
        // members are loaded once: the output stores are uint8_t and may alias them as far as the compiler knows.
        // Before the end of the file the loop stops 32 bytes short of the data (fill() between calls); at the end
        // it may read into the zero pad, and more than 16 bytes into it means the stream is truncated.
        const bool eof = eof_;
        const uint8_t* const in_stop = eof ? in_end_ + 16 : in_end_ - 32;
        for (;;) {
            if (o >= lim) break;
            if (in > in_stop) {
                if (!eof) break;
                bb_ = bb; bc_ = bc; in_ptr_ = in; fail("truncated deflate stream"); return o;
            }
            {   // refill to 56..63 bits
                uint64_t w;
                memcpy(&w, in, 8);
                bb |= w << bc;
                in += (63 - bc) >> 3;
                bc |= 56;
            }
            uint32_t e = lt[bb & ((1u << LBITS) - 1)];
            if ((e & K_MASK) == K_SUB) e = lt[(e >> 16) + ((bb >> LBITS) & ((1u << ((e >> 4) & 15)) - 1))];
            bb >>= e & 15;
            bc -= e & 15;
            if ((e & (K_MASK | K_BAD)) == K_LIT) {
                *o++ = (uint8_t)(e >> 16);
#pragma GCC unroll 5
                for (int r = 0; r < 5; r++) {  // more literals from this refill while >= 11 bits remain (the
                                               // output may run 5 bytes past lim: SLACK)
                    e = lt[bb & ((1u << LBITS) - 1)];
                    if ((e & (K_MASK | K_BAD)) != K_LIT || bc < 11) break;
                    bb >>= e & 15;
                    bc -= e & 15;
                    *o++ = (uint8_t)(e >> 16);
                }
                continue;
            }
            if (e & K_BAD) { bb_ = bb; bc_ = bc; in_ptr_ = in; fail("invalid literal/length code"); return o; }
            if ((e & K_MASK) == K_EOB) {
                bb_ = bb;
                bc_ = bc;
                in_ptr_ = in;
                end_block(o);
                if (overrun()) fail("truncated deflate stream");
                return o;
            }
            const uint32_t lx = (e >> 4) & 15;
            const uint32_t len = (e >> 16) + (uint32_t)(bb & ((1u << lx) - 1));
            bb >>= lx;
            bc -= lx;
            uint32_t d = dt[bb & ((1u << DBITS) - 1)];
            if ((d & K_MASK) == K_SUB) d = dt[(d >> 16) + ((bb >> DBITS) & ((1u << ((d >> 4) & 15)) - 1))];
            if (d & K_BAD) { bb_ = bb; bc_ = bc; in_ptr_ = in; fail("invalid distance code"); return o; }
            bb >>= d & 15;
            bc -= d & 15;
            const uint32_t dx = (d >> 4) & 15;
            const size_t dist = (d >> 16) + (uint32_t)(bb & ((1u << dx) - 1));
            bb >>= dx;
            bc -= dx;
            if (dist > (size_t)(o - hist)) { bb_ = bb; bc_ = bc; in_ptr_ = in; fail("distance too far back"); return o; }
            const uint8_t* src = o - dist;
            uint8_t* const end = o + len;
            if (dist >= 8) {  // 8-byte words; may write up to 7 bytes past end (SLACK)
                uint64_t w0, w1;
                memcpy(&w0, src, 8);
                memcpy(o, &w0, 8);
                memcpy(&w1, src + 8, 8);
                memcpy(o + 8, &w1, 8);
                src += 16;
                o += 16;
                while (o < end) {
                    uint64_t w;
                    memcpy(&w, src, 8);
                    memcpy(o, &w, 8);
                    src += 8;
                    o += 8;
                }
            } else if (dist == 1) {
                memset(o, *src, len);
            } else {
                do *o++ = *src++;
                while (o < end);
            }
            o = end;
        }
        bb_ = bb;
        bc_ = bc;
        in_ptr_ = in;
        if (in > in_stop && !eof) fill();
        return o;
    }

    static bool no_marker(const uint16_t* p, size_t n) {
        uint16_t acc = 0;
        for (size_t i = 0; i < n; i++) acc |= p[i];
        return !(acc & MARK);
    }
    // huff() for the marker phase: 16-bit output, references before the chunk's first symbol become markers.
    void huff16(std::vector<uint16_t>& out) {
        const uint32_t* lt = lt_;
        const uint32_t* dt = dt_;
        const uint8_t* const in_stop = in_end_ + 16;
        for (;;) {
            if (in_ptr_ > in_stop) { fail("truncated deflate stream"); return; }
            refill();
            uint32_t e = lt[bb_ & ((1u << LBITS) - 1)];
            if ((e & K_MASK) == K_SUB) e = lt[(e >> 16) + ((bb_ >> LBITS) & ((1u << ((e >> 4) & 15)) - 1))];
            if (e & K_BAD) { fail("invalid literal/length code"); return; }
            bb_ >>= e & 15;
            bc_ -= e & 15;
            if ((e & K_MASK) == K_LIT) {
                out.push_back((uint16_t)(e >> 16));
                continue;
            }
            if ((e & K_MASK) == K_EOB) {
                end_block(nullptr);
                if (overrun()) fail("truncated deflate stream");
                return;
            }
            const uint32_t lx = (e >> 4) & 15;
            const uint32_t len = (e >> 16) + (uint32_t)(bb_ & ((1u << lx) - 1));
            bb_ >>= lx;
            bc_ -= lx;
            uint32_t d = dt[bb_ & ((1u << DBITS) - 1)];
            if ((d & K_MASK) == K_SUB) d = dt[(d >> 16) + ((bb_ >> DBITS) & ((1u << ((d >> 4) & 15)) - 1))];
            if (d & K_BAD) { fail("invalid distance code"); return; }
            bb_ >>= d & 15;
            bc_ -= d & 15;
            const uint32_t dx = (d >> 4) & 15;
            const size_t dist = (d >> 16) + (uint32_t)(bb_ & ((1u << dx) - 1));
            bb_ >>= dx;
            bc_ -= dx;
            const size_t have = out.size();  // symbols of the chunk so far
            if (dist > have + WIN) { fail("distance too far back"); return; }
            for (uint32_t i = 0; i < len; i++) {
                const size_t at = out.size();
                out.push_back(at >= dist ? out[at - dist] : (uint16_t)(MARK + (WIN + at - dist)));
            }
        }
    }

    int fd_;
    bool mem_ = false, chunk_ = false;
    uint8_t* base_ = nullptr;  // start of the input (bit_pos)
    uint64_t stop_ = NO_STOP, out_total_ = 0, cur_out_ = 0;
    std::vector<Trailer> trailers_;
    std::vector<uint8_t> in_;
    uint8_t* in_ptr_;
    uint8_t* in_end_;
    bool eof_ = false;
    uint64_t bb_ = 0;
    uint32_t bc_ = 0;
    St st_ = HEADER;
    const char* err_ = nullptr;
    uint32_t final_ = 0, stored_left_ = 0, crc_ = 0, isize_ = 0, members_ = 0;
    const uint8_t* hist_start_ = nullptr;
    std::vector<uint8_t> hist_;
    std::vector<uint32_t> fixed_l_ = std::vector<uint32_t>(LSIZE), fixed_d_ = std::vector<uint32_t>(DSIZE),
                          dyn_l_ = std::vector<uint32_t>(LSIZE), dyn_d_ = std::vector<uint32_t>(DSIZE);
    const uint32_t* lt_ = nullptr;
    const uint32_t* dt_ = nullptr;
};

}  // namespace dwpa
