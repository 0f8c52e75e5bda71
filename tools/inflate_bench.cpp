// inflate_bench -- how fast the dwpa_crack_files dictionary reader (dwpa_amd/csrc/dict_reader.hpp, the exact
// code the library runs) turns gzip wordlists into candidate chunks on this host, i.e. how many GPUs one gz
// stream can feed in the rules-less first pass (help_crack.py:929; a GPU scans ~4.9 M words/s at C2).
//
//   inflate_bench FILE.gz [FILE2.gz ...]
//   inflate_bench --dump FILE... prints every word the reader yields, hex-encoded, one per line (tests/test_dict_reader.py)
//   inflate_bench --passes K FILE... reads the files K times through ChunkSource (the crack path, DictCache included):
//   per pass "#pass k cache_hits n", "#status s0 s1 ..." (per file: 0 ok, 1 damaged gzip, 2 unreadable), the words
//   inflate_bench --passes K FILE... runs crack_files' ChunkSource K times over the files in one process (the second
//     pass onwards replays the DictCache) and prints "#pass i cache_hits h" then that pass's words, hex-encoded
//
// Prints one JSON line: inflate-only throughput of the first file with zlib's gzread and with the reader's
// GzipDecoder (inflate.hpp), DictReader words/s on the first file (one stream: an inflate thread feeding the line
// cutting + $HEX[] decoding thread; DWPA_INFLATE=zlib runs it on gzread), and ChunkSource words/s over all files
// (up to 4 such streams, as crack_files runs them).
#include <fcntl.h>
#include <stdio.h>
#include <unistd.h>
#include <zlib.h>

#include <chrono>
#include <string>
#include <vector>

#include "dict_reader.hpp"

using clk = std::chrono::steady_clock;

static double since(clk::time_point t) { return std::chrono::duration<double>(clk::now() - t).count(); }

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s FILE.gz [FILE2.gz ...]\n", argv[0]);
        return 2;
    }
    auto hex_line = [](const dwpa::Chunk& c, size_t i, std::string& line) {
        line.clear();
        for (uint64_t k = c.off[i]; k < c.off[i + 1]; k++) {
            static const char* d = "0123456789abcdef";
            line.push_back(d[(uint8_t)c.bytes[k] >> 4]);
            line.push_back(d[(uint8_t)c.bytes[k] & 15]);
        }
        line.push_back('\n');
    };
    if (std::string(argv[1]) == "--passes" && argc > 3) {
        const int K = atoi(argv[2]);
        std::vector<std::string> paths(argv + 3, argv + argc);
        // DWPA_TEST_REWRITE=path: append one word to that (plain) file after every pass, as a re-download would
        // change it (the cache must drop the stale decode and read the new file)
        const char* rewrite = getenv("DWPA_TEST_REWRITE");
        std::string line;
        for (int pass = 0; pass < K; pass++) {
            dwpa::ChunkSource src(paths, 1000, 1 << 16);
            std::shared_ptr<const dwpa::Chunk> c;
            bool err = false;
            std::vector<std::shared_ptr<const dwpa::Chunk>> got;
            while (src.next(c, err)) got.push_back(c);
            src.finish();
            if (err) return 1;
            printf("#pass %d cache_hits %zu cache_entries %zu\n#status", pass, dwpa::DictCache::get().hits(),
                   dwpa::DictCache::get().entries());
            for (int st : src.file_status()) printf(" %d", st);  // ChunkSource::FILE_OK / _DAMAGED / _UNREADABLE
            printf("\n");
            for (const auto& ch : got)
                for (size_t i = 0; i < ch->words(); i++) {
                    hex_line(*ch, i, line);
                    fwrite(line.data(), 1, line.size(), stdout);
                }
            if (rewrite) {
                FILE* f = fopen(rewrite, "ab");
                if (!f) return 1;
                fprintf(f, "added-after-pass-%d\n", pass);
                fclose(f);
            }
        }
        return 0;
    }
    if (std::string(argv[1]) == "--dump") {
        dwpa::DictReader rd(std::vector<std::string>(argv + 2, argv + argc));
        dwpa::Chunk c;
        bool err = false;
        std::string line;
        while (rd.next(c, 1000, (size_t)1 << 20, err)) {
            for (size_t i = 0; i < c.words(); i++) {
                line.clear();
                for (uint64_t k = c.off[i]; k < c.off[i + 1]; k++) {
                    static const char* d = "0123456789abcdef";
                    line.push_back(d[(uint8_t)c.bytes[k] >> 4]);
                    line.push_back(d[(uint8_t)c.bytes[k] & 15]);
                }
                line.push_back('\n');
                fwrite(line.data(), 1, line.size(), stdout);
            }
        }
        return err ? 1 : 0;
    }
    std::vector<std::string> paths(argv + 1, argv + argc);
    // 1. inflate only
    gzFile gz = gzopen(paths[0].c_str(), "rb");
    if (!gz) return 1;
    gzbuffer(gz, 1 << 20);
    std::vector<char> buf(1 << 20);
    size_t raw = 0;
    auto t = clk::now();
    for (int r; (r = gzread(gz, buf.data(), (unsigned)buf.size())) > 0;) raw += (size_t)r;
    const double t_inflate = since(t);
    gzclose(gz);
    // 1b. inflate only, GzipDecoder
    size_t raw_fast = 0;
    double t_fast = 0;
    {
        const int fd = open(paths[0].c_str(), O_RDONLY);
        if (fd < 0) return 1;
        dwpa::GzipDecoder dec(fd);
        std::vector<uint8_t> ob(dwpa::GzipDecoder::WIN + (4u << 20) + dwpa::GzipDecoder::SLACK);
        t = clk::now();
        while (!dec.done() && !dec.failed()) raw_fast += dec.read(ob.data(), 4u << 20);
        t_fast = since(t);
        close(fd);
        if (dec.failed() || raw_fast != raw) raw_fast = 0;  // not gzip (plain file) or an error: no figure
    }
    // 2. one DictReader stream (what one dictionary costs one reader thread)
    size_t words1 = 0;
    {
        dwpa::DictReader rd({paths[0]});
        dwpa::Chunk c;
        bool err = false;
        t = clk::now();
        while (rd.next(c, 1 << 22, (size_t)1 << 31, err)) words1 += c.words();
        if (err) return 1;
    }
    const double t_reader = since(t);
    // 3. ChunkSource over every file (crack_files' reader threads)
    size_t words_all = 0;
    t = clk::now();
    {
        dwpa::ChunkSource src(paths, 1 << 20, 1 << 24);
        dwpa::Chunk c;
        bool err = false;
        while (src.next(c, err)) words_all += c.words();
        if (err) return 1;
    }
    const double t_all = since(t);
    std::string inflater = "GzipDecoder";
    {
        const int fd = open(paths[0].c_str(), O_RDONLY);
        const char* z = getenv("DWPA_INFLATE");
        if (z && !strcmp(z, "zlib")) inflater = "zlib";
        else if (fd >= 0 && dwpa::BlockInflater::parallel_threads(fd) > 1)
            inflater = "ParallelGunzip x" + std::to_string(dwpa::BlockInflater::parallel_threads(fd));
        if (fd >= 0) close(fd);
    }
    printf("{\"files\": %zu, \"raw_bytes\": %zu, \"inflate_MBps\": %.1f, \"fast_inflate_MBps\": %.1f, "
           "\"reader_inflater\": \"%s\", \"words\": %zu, "
           "\"reader_words_per_s\": %.0f, \"reader_MBps\": %.1f, \"chunk_source_threads\": %zu, "
           "\"chunk_source_words_per_s\": %.0f}\n",
           paths.size(), raw, raw / t_inflate / 1e6, raw_fast ? raw_fast / t_fast / 1e6 : 0.0,
           inflater.c_str(), words1, words1 / t_reader, raw / t_reader / 1e6,
           std::min<size_t>(paths.size(), 4), words_all / t_all);
    return 0;
}
