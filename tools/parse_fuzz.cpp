// parse_fuzz.cpp -- host fuzz of the check path's hashline handling under AddressSanitizer / UBSan.  Hashlines reach
// the server from users' uploads (put_work, submission), so parse_m22000 and the table builder see untrusted bytes.
// Each line of a corpus file (valid PMKID / EAPOL keyver 1-3 lines, tests/test_parse_fuzz.py writes it) is mutated
// -- bytes replaced by hex digits, separators or anything, inserted, deleted, fields duplicated, dropped or blown up
// to thousands of hex digits, the type field rewritten -- then parsed; an accepted line is added to a TableBuilder
// at several nonce-correction windows in both modes, with and without per-attempt KW blocks, and its salt blocks and
// outfile fields are built.  hc_unhex runs on mutated $HEX[] keys.  Prints the counts; ASan/UBSan abort on a fault.
//   make tools/bin/parse_fuzz_asan && tools/bin/parse_fuzz_asan corpus.txt [iterations]
#include <stdio.h>
#include <stdlib.h>

#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "dwpa22000.h"
#include "m22000_host.hpp"

using namespace dwpa;

static std::string mutate(std::string s, std::mt19937_64& rng) {
    static const std::string hexd = "0123456789abcdefABCDEF";
    const int n = 1 + (int)(rng() % 4);
    for (int m = 0; m < n; m++) {
        const size_t at = s.empty() ? 0 : rng() % (s.size() + 1);
        switch (rng() % 10) {
        case 0: if (at < s.size()) s[at] = hexd[rng() % hexd.size()]; break;
        case 1: if (at < s.size()) s[at] = "*:$[]\r\n\0"[rng() % 8]; break;
        case 2: if (at < s.size()) s[at] = (char)(rng() % 256); break;
        case 3: s.insert(at, 1, hexd[rng() % hexd.size()]); break;
        case 4: if (at < s.size()) s.erase(at, 1 + rng() % 8); break;
        case 5: s.insert(at, std::string(2 * (1 + rng() % 3000), hexd[rng() % 16])); break;  // a blown-up field
        case 6: {  // duplicate or drop a field
            std::vector<std::string> f;
            size_t st = 0;
            for (size_t i = 0; i <= s.size(); i++)
                if (i == s.size() || s[i] == '*') { f.push_back(s.substr(st, i - st)); st = i + 1; }
            const size_t k = rng() % f.size();
            if (rng() % 2) f.insert(f.begin() + (long)k, f[k]);
            else f.erase(f.begin() + (long)k);
            s.clear();
            for (size_t i = 0; i < f.size(); i++) s += (i ? "*" : "") + f[i];
            break;
        }
        case 7: {  // the type field
            static const char* t[] = {"01", "02", "1", "2", "03", "", "0x02", " 02", "2.0", "02 "};
            const size_t a = s.find('*'), b = a == std::string::npos ? a : s.find('*', a + 1);
            if (b != std::string::npos) s.replace(a + 1, b - a - 1, t[rng() % 10]);
            break;
        }
        case 8: s.resize(s.empty() ? 0 : rng() % s.size()); break;  // truncated
        default: s += s.substr(0, rng() % (s.size() + 1)); break;   // trailing garbage
        }
    }
    return s;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s corpus.txt [iterations]\n", argv[0]);
        return 2;
    }
    std::vector<std::string> corpus;
    std::ifstream in(argv[1], std::ios::binary);
    for (std::string l; std::getline(in, l);)
        if (!l.empty()) corpus.push_back(l);
    if (corpus.empty()) return 2;
    const long iters = argc > 2 ? atol(argv[2]) : 20000;
    std::mt19937_64 rng(4242);
    const int ncs[] = {-7, -1, 0, 1, 8, 16, 128, 131, 258};
    long accepted = 0, tables = 0, attempts = 0;
    for (long it = 0; it < iters; it++) {
        const std::string line = it % 8 ? mutate(corpus[rng() % corpus.size()], rng) : corpus[rng() % corpus.size()];
        ParsedLine p = parse_m22000(line.data(), line.size());
        ParsedLine q;
        parse_m22000_into(line.data(), line.size(), q);  // the reused-buffer form must agree
        if (p.status != q.status || p.kind != q.kind || p.essid != q.essid || p.eapol != q.eapol) {
            fprintf(stderr, "parse forms disagree on line %ld\n", it);
            return 1;
        }
        if (p.status) continue;
        accepted++;
        TableBuilder tb;
        tb.att_kw_all = rng() % 2;
        const int nc = ncs[rng() % 9];
        const int mode = (int)(rng() % 2) ? DWPA_NC_HASHCAT : DWPA_NC_PHP;
        const uint32_t li = tb.add_line(p, nc, mode, nc);
        tables++;
        attempts += tb.lines[li].natt;
        std::vector<uint32_t> salt;
        build_salt_blocks(p.essid, salt);
        (void)hex_lower(p.field2_hex);
        (void)hashcat_plain(p.essid);
        std::string key = "$HEX[" + hex_lower(p.essid) + "]";
        (void)hc_unhex(mutate(key, rng));
    }
    printf("lines %ld accepted %ld tables %ld attempts %ld\n", iters, accepted, tables, attempts);
    return 0;
}
