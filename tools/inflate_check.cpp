// inflate_check -- decodes each gzip file with dwpa::GzipDecoder (the dictionary reader's inflater) and with zlib's
// gzread, in blocks of a given size, and reports whether the outputs agree and each decoder's throughput.
// Used by tests/test_inflate.py (CPU) and on the GPU box's host to measure the single-stream feed rate.
//   inflate_check [-b block_bytes] [-r repeats] [-p threads -c chunk_bytes] file...
// With -p the fast side is ParallelGunzip (pinflate.hpp) continued by gzread after a stop, exactly as the dictionary
// reader runs it; the line then ends with "chunks <n> parallel <decoded> markers <symbols> stop <reason|none>".
// Per file one line: "<file> ok <bytes> fast_MBps zlib_MBps" | "<file> error <fast message> zlib_rc <n>" |
// "<file> mismatch at <offset>".  Exit 0 only if every file decodes identically with both (or fails with both).
#include <fcntl.h>
#include <sys/stat.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <zlib.h>

#include <chrono>
#include <string>
#include <vector>

#include "inflate.hpp"
#include "pinflate.hpp"

static double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

// keep = false: decode only (timing); out gets the byte count as its size
static bool fast_decode(const char* path, size_t block, std::string& out, std::string& err, bool keep = true) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) { err = "open"; return false; }
    dwpa::GzipDecoder dec(fd);
    std::vector<uint8_t> buf(dwpa::GzipDecoder::WIN + block + dwpa::GzipDecoder::SLACK);
    out.clear();
    size_t total = 0;
    for (;;) {
        const size_t n = dec.read(buf.data(), block);
        total += n;
        if (keep) out.append((const char*)buf.data() + dwpa::GzipDecoder::WIN, n);
        if (dec.failed()) { err = dec.error(); close(fd); return false; }
        if (dec.done()) break;
    }
    close(fd);
    if (!keep) out.assign(total, '\0');
    return true;
}

static int zlib_decode(const char* path, std::string& out, bool keep = true) {
    gzFile gz = gzopen(path, "rb");
    if (!gz) return -1;
    gzbuffer(gz, 1 << 20);
    out.clear();
    std::vector<char> b(1 << 22);
    size_t total = 0;
    for (;;) {
        const int r = gzread(gz, b.data(), (unsigned)b.size());
        if (r < 0) { gzclose(gz); return -2; }
        if (r == 0) break;
        total += (size_t)r;
        if (keep) out.append(b.data(), (size_t)r);
    }
    int e = 0;
    gzerror(gz, &e);
    gzclose(gz);
    if (!keep) out.assign(total, '\0');
    return e == Z_OK ? 0 : -3;  // Z_BUF_ERROR: truncated input ("unexpected end of file")
}

// ParallelGunzip, then gzread from the bytes delivered when it stops (dict_reader.hpp BlockInflater::file_parallel).
static bool parallel_decode(const char* path, unsigned threads, size_t chunk, std::string& out, std::string& info,
                            bool keep = true) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) { info = "open"; return false; }
    struct stat st;
    fstat(fd, &st);
    out.clear();
    size_t total = 0;
    const char* perr = nullptr;
    dwpa::ParallelGunzip::Stats ps;
    const uint64_t got = dwpa::ParallelGunzip::run(fd, (size_t)st.st_size, threads, chunk,
                                                   [&](const uint8_t* p, size_t k) {
                                                       if (keep) out.append((const char*)p, k);
                                                       total += k;
                                                       return true;
                                                   },
                                                   &perr, &ps);
    char buf[256];
    snprintf(buf, sizeof buf, "chunks %zu parallel %zu markers %zu stop %s", ps.chunks, ps.decoded, ps.marker_syms,
             perr ? perr : "none");
    info = buf;
    // a damaged stream stays damaged even where gzread, whose error reporting depends on its read sizes, ends cleanly
    bool ok = !perr || dwpa::ParallelGunzip::false_boundary(perr);
    if (perr) {  // continue with gzread after the delivered bytes
        gzFile gz = gzdopen(dup(fd), "rb");
        std::vector<char> b(1 << 20);
        uint64_t skip = got;
        while (skip) {
            const int r = gzread(gz, b.data(), (unsigned)std::min<uint64_t>(skip, b.size()));
            if (r <= 0) { ok = false; break; }
            skip -= (uint64_t)r;
        }
        for (bool more = true; more;) {
            const int r = gzread(gz, b.data(), (unsigned)b.size());
            if (r < 0) { ok = false; break; }
            if (r == 0) more = false;
            if (keep) out.append(b.data(), (size_t)r);
            total += (size_t)r;
        }
        int e = 0;
        gzerror(gz, &e);
        if (e != Z_OK) ok = false;
        gzclose(gz);
    }
    close(fd);
    if (!keep) out.assign(total, '\0');
    return ok;
}

int main(int argc, char** argv) {
    size_t block = 4u << 20, chunk = 4u << 20;
    unsigned threads = 0;
    int reps = 1, bad = 0;
    int i = 1;
    for (; i < argc && argv[i][0] == '-'; i += 2) {
        if (!strcmp(argv[i], "-b") && i + 1 < argc) block = strtoull(argv[i + 1], nullptr, 10);
        else if (!strcmp(argv[i], "-r") && i + 1 < argc) reps = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-p") && i + 1 < argc) threads = (unsigned)atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "-c") && i + 1 < argc) chunk = strtoull(argv[i + 1], nullptr, 10);
    }
    if (threads) {
        for (; i < argc; i++) {
            std::string a, b, info, scratch, i2;
            const bool okp = parallel_decode(argv[i], threads, chunk, a, info);
            const int rz = zlib_decode(argv[i], b);
            double tp = 1e30, tz = 1e30;
            for (int r = 0; r < reps && okp && !rz; r++) {
                double t0 = now_s();
                parallel_decode(argv[i], threads, chunk, scratch, i2, false);
                tp = std::min(tp, now_s() - t0);
                t0 = now_s();
                zlib_decode(argv[i], scratch, false);
                tz = std::min(tz, now_s() - t0);
            }
            // both failed: gzread may drop its failing read (data error), the reader keeps what decoded before it
            const bool both_failed = !okp && rz != 0 && a.size() >= b.size() && a.compare(0, b.size(), b) == 0;
            if (!both_failed && (a != b || okp != (rz == 0))) {
                size_t k = 0;
                while (k < a.size() && k < b.size() && a[k] == b[k]) k++;
                printf("%s mismatch at %zu (parallel %zu bytes ok %d, zlib %zu rc %d) %s\n", argv[i], k, a.size(),
                       (int)okp, b.size(), rz, info.c_str());
                bad++;
                continue;
            }
            if (!okp) {
                printf("%s error both %s\n", argv[i], info.c_str());
                continue;
            }
            printf("%s ok %zu %.1f %.1f %s\n", argv[i], a.size(), a.size() / tp / 1e6, b.size() / tz / 1e6, info.c_str());
        }
        return bad ? 1 : 0;
    }
    printf("crc32 %s\n", dwpa::Crc32::get().clmul_ok ? "pclmul" : "table");
    for (; i < argc; i++) {
        std::string a, b, err;
        double tf = 1e30, tz = 1e30;
        bool okf = false;
        int rz = 0;
        okf = fast_decode(argv[i], block, a, err);
        rz = zlib_decode(argv[i], b);
        std::string scratch, e2;
        for (int r = 0; r < reps && okf && !rz; r++) {  // timing: decode only
            double t0 = now_s();
            fast_decode(argv[i], block, scratch, e2, false);
            tf = std::min(tf, now_s() - t0);
            t0 = now_s();
            zlib_decode(argv[i], scratch, false);
            tz = std::min(tz, now_s() - t0);
        }
        if (!okf || rz) {
            printf("%s error %s zlib_rc %d\n", argv[i], okf ? "none" : err.c_str(), rz);
            if (okf != (rz == 0)) bad++;
            continue;
        }
        if (a != b) {
            size_t k = 0;
            while (k < a.size() && k < b.size() && a[k] == b[k]) k++;
            printf("%s mismatch at %zu (fast %zu bytes, zlib %zu)\n", argv[i], k, a.size(), b.size());
            bad++;
            continue;
        }
        printf("%s ok %zu %.1f %.1f\n", argv[i], a.size(), a.size() / tf / 1e6, b.size() / tz / 1e6);
    }
    return bad ? 1 : 0;
}
