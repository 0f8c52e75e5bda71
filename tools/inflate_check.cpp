// inflate_check -- decodes each gzip file with dwpa::GzipDecoder (the dictionary reader's inflater) and with zlib's
// gzread, in blocks of a given size, and reports whether the outputs agree and each decoder's throughput.
// Used by tests/test_inflate.py (CPU) and on the GPU box's host to measure the single-stream feed rate.
//   inflate_check [-b block_bytes] [-r repeats] file...
// Per file one line: "<file> ok <bytes> fast_MBps zlib_MBps" | "<file> error <fast message> zlib_rc <n>" |
// "<file> mismatch at <offset>".  Exit 0 only if every file decodes identically with both (or fails with both).
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <zlib.h>

#include <chrono>
#include <string>
#include <vector>

#include "inflate.hpp"

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

int main(int argc, char** argv) {
    size_t block = 4u << 20;
    int reps = 1, bad = 0;
    int i = 1;
    for (; i < argc && argv[i][0] == '-'; i += 2) {
        if (!strcmp(argv[i], "-b") && i + 1 < argc) block = strtoull(argv[i + 1], nullptr, 10);
        else if (!strcmp(argv[i], "-r") && i + 1 < argc) reps = atoi(argv[i + 1]);
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
