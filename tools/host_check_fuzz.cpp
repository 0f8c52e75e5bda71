// host_check_fuzz.cpp -- host fuzz of the host backend's check path under AddressSanitizer / UBSan.  The host backend
// (host_check.cpp, host_crypto.cpp) answers put_work's checks on the server, so it sees users' hashlines and keys.
// Batches of 1-8 jobs are built from a corpus of valid PMKID / EAPOL keyver 1-3 lines (tests/test_host_check_fuzz.py
// writes it), mutated as tools/parse_fuzz.cpp mutates them, with keys of 0..300 bytes (sometimes the corpus PSK,
// $HEX[...] forms, null keys, one of 64 KiB), caller PMKs or none, and nc from -9 to past DWPA_NC_MAX; each batch
// goes through host_cost and host_check_batch, and now and then a key list through host_pbkdf2.  Prints the counts;
// ASan/UBSan abort on a fault.  The engine's host thread pool is replaced by plain threads here (no HIP).
//   make tools/bin/host_check_fuzz_asan && tools/bin/host_check_fuzz_asan corpus.txt [batches]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <fstream>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "dwpa22000.h"
#include "engine.hpp"

namespace dwpa {
size_t host_threads_for(size_t n, size_t min_per_thread) {
    return std::max<size_t>(1, std::min<size_t>(4, n / std::max<size_t>(1, min_per_thread)));
}
void host_parallel(size_t T, const std::function<void(size_t)>& fn) {
    std::vector<std::thread> th;
    for (size_t t = 1; t < T; t++) th.emplace_back(fn, t);
    fn(0);
    for (auto& t : th) t.join();
}
}  // namespace dwpa

using namespace dwpa;

static std::string mutate(std::string s, std::mt19937_64& rng) {
    static const std::string hexd = "0123456789abcdefABCDEF";
    const int n = 1 + (int)(rng() % 3);
    for (int m = 0; m < n; m++) {
        const size_t at = s.empty() ? 0 : rng() % (s.size() + 1);
        switch (rng() % 9) {
        case 0: if (at < s.size()) s[at] = hexd[rng() % hexd.size()]; break;
        case 1: if (at < s.size()) s[at] = "*:$[]\r\n\0"[rng() % 8]; break;
        case 2: if (at < s.size()) s[at] = (char)(rng() % 256); break;
        case 3: s.insert(at, 1, hexd[rng() % hexd.size()]); break;
        case 4: if (at < s.size()) s.erase(at, 1 + rng() % 8); break;
        case 5: s.insert(at, std::string(2 * (1 + rng() % 600), hexd[rng() % 16])); break;  // a blown-up field
        case 6: {  // the type field
            static const char* t[] = {"01", "02", "1", "2", "03", "", " 02", "02 "};
            const size_t a = s.find('*'), b = a == std::string::npos ? a : s.find('*', a + 1);
            if (b != std::string::npos) s.replace(a + 1, b - a - 1, t[rng() % 8]);
            break;
        }
        case 7: s.resize(s.empty() ? 0 : rng() % s.size()); break;  // truncated
        default: s += s.substr(0, rng() % (s.size() + 1)); break;   // trailing garbage
        }
    }
    return s;
}

static std::string hex_of(const std::string& b) {
    static const char* d = "0123456789abcdef";
    std::string h;
    for (unsigned char c : b) {
        h += d[c >> 4];
        h += d[c & 15];
    }
    return h;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s corpus.txt [batches]\n", argv[0]);
        return 2;
    }
    // corpus lines: "<hashline>\t<psk>" (the PSK that verifies the line)
    std::vector<std::pair<std::string, std::string>> corpus;
    std::ifstream in(argv[1], std::ios::binary);
    for (std::string l; std::getline(in, l);) {
        const size_t tab = l.find('\t');
        if (tab != std::string::npos) corpus.emplace_back(l.substr(0, tab), l.substr(tab + 1));
    }
    if (corpus.empty()) return 2;
    const long batches = argc > 2 ? atol(argv[2]) : 1500;
    std::mt19937_64 rng(777);
    const int ncs[] = {-9, -1, 0, 1, 8, 17, 128, 131, 258, 1000, DWPA_NC_MAX, DWPA_NC_MAX + 1};
    long jobs_run = 0, hits = 0, errs = 0, pbkdf2_calls = 0;
    const std::string big(65536, 'k');
    for (long it = 0; it < batches; it++) {
        const size_t nj = 1 + rng() % 8;
        std::vector<std::string> lines(nj);
        std::vector<std::vector<std::string>> keys(nj);
        std::vector<std::vector<dwpa_bytes>> kb(nj);
        std::vector<std::string> pmks(nj);
        std::vector<dwpa_job> jobs(nj);
        for (size_t j = 0; j < nj; j++) {
            const auto& c = corpus[rng() % corpus.size()];
            lines[j] = rng() % 3 ? mutate(c.first, rng) : c.first;
            const size_t nk = rng() % 6;
            for (size_t k = 0; k < nk; k++) {
                switch (rng() % 7) {
                case 0: keys[j].push_back(c.second); break;
                case 1: keys[j].push_back("$HEX[" + hex_of(c.second) + "]"); break;
                case 2: keys[j].push_back("$HEX[" + hex_of(c.second).substr(0, rng() % 20) + "]"); break;
                case 3: keys[j].push_back(""); break;
                case 4: if (rng() % 40 == 0) keys[j].push_back(big); else keys[j].push_back("x"); break;
                default: {
                    std::string r(rng() % 300, '\0');
                    for (auto& ch : r) ch = (char)(rng() % 256);
                    keys[j].push_back(r);
                }
                }
            }
            for (size_t k = 0; k < keys[j].size(); k++) {
                const bool null_key = rng() % 10 == 0;
                kb[j].push_back(dwpa_bytes{null_key ? nullptr : (const uint8_t*)keys[j][k].data(),
                                           null_key ? 0 : keys[j][k].size()});
            }
            if (rng() % 4 == 0) {
                pmks[j].resize(32);
                for (auto& ch : pmks[j]) ch = (char)(rng() % 256);
            }
            jobs[j] = dwpa_job{lines[j].data(), lines[j].size(), kb[j].data(), kb[j].size(),
                               pmks[j].empty() ? nullptr : (const uint8_t*)pmks[j].data(), ncs[rng() % 12]};
        }
        (void)host_cost(jobs.data(), nj);
        std::vector<dwpa_result> out(nj);
        std::vector<int> rcs(nj);
        dwpa_check_stats st{};
        const int rc = host_check_batch(jobs.data(), nj, out.data(), rcs.data(), st);
        if (rc < 0) {
            errs++;
        } else {
            jobs_run += (long)nj;
            for (int r : rcs) hits += r == DWPA_HIT;
        }
        if (it % 25 == 0) {
            const std::string essid = mutate(corpus[rng() % corpus.size()].second, rng).substr(0, rng() % 300);
            std::vector<dwpa_bytes> ks;
            for (const auto& k : keys[0]) ks.push_back(dwpa_bytes{(const uint8_t*)k.data(), k.size()});
            std::vector<uint8_t> pm(32 * ks.size() + 1);
            if (host_pbkdf2(ks.data(), ks.size(), (const uint8_t*)essid.data(), essid.size(), pm.data()) < 0) errs++;
            pbkdf2_calls++;
        }
    }
    printf("batches %ld jobs %ld hits %ld errors %ld pbkdf2 %ld\n", batches, jobs_run, hits, errs, pbkdf2_calls);
    return 0;
}
