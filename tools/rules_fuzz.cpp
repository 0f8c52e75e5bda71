// rules_fuzz.cpp -- host fuzz of the rule engine under AddressSanitizer / UBSan (the interpreter in rules_apply.hpp is
// the same source the GPU runs, where an out-of-bounds write of a lane's 256-byte buffer would corrupt memory
// silently).  Random rule lines over the whole alphabet (valid and invalid) are parsed by RuleSet::add_line and
// applied to random words of 0..300 bytes by RuleSet::apply_host; the work and memory buffers are exactly
// RP_PASSWORD_SIZE + 4 bytes, as on the GPU.
//   make -C tools/.. tools/bin/rules_fuzz_asan && tools/bin/rules_fuzz_asan [iterations]
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <string>

#include "engine.hpp"
#include "rules.hpp"

// The device half of rules.cpp (uploads, scans) is linked but never called here.
namespace dwpa {
[[noreturn]] static void not_here() { abort(); }
uint32_t scan_batch_cap(const dwpa_scan*) { not_here(); }
Batch& scan_batch_ref(dwpa_scan*) { not_here(); }
int scan_device(const dwpa_scan*) { not_here(); }
int engine_init() { not_here(); }
hipError_t launch_rules_prep(const uint64_t*, const uint8_t*, uint64_t, uint32_t, const uint32_t*, const uint32_t*,
                             uint32_t, uint32_t, uint32_t, uint32_t*, uint64_t*, uint32_t*, uint32_t, hipStream_t) {
    not_here();
}
hipError_t launch_rules_expand(const uint64_t*, const uint8_t*, uint32_t, const uint32_t*, const uint32_t*, uint32_t,
                               uint8_t*, uint32_t*, hipStream_t, uint32_t*) {
    not_here();
}
}  // namespace dwpa

int main(int argc, char** argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 200000;
    std::mt19937_64 rng(12345);
    const std::string ops = ":lucCtrdf{}[]kKqEM46QTpDzZ'yYLR+-.,<>_$^@e!/()io=%3sxO*X";
    const std::string args = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ";
    long parsed = 0, applied = 0, rejected = 0;
    for (long it = 0; it < iters; it++) {
        std::string line;
        if (rng() % 10 < 3) {  // random characters: mostly lines that do not parse
            const int n = 1 + (int)(rng() % 24);
            for (int i = 0; i < n; i++) {
                const uint64_t r = rng() % 10;
                line.push_back(r < 5 ? ops[rng() % ops.size()] : r < 8 ? args[rng() % args.size()] : (char)(rng() % 256));
            }
        } else {  // 1..10 well-formed functions with random (often out-of-range) arguments
            static const std::string shape[] = {":lucCtrdf{}[]kKqEM46Q", "TpDzZ'yYLR+-.,<>_", "$^@e!/()", "io=%3", "s",
                                                "xO*", "X"};
            const int nf = 1 + (int)(rng() % 10);
            auto pos = [&] { return args[rng() % args.size()]; };
            auto chr = [&] { return (char)(rng() % 4 ? 'a' + rng() % 6 : rng() % 256); };
            for (int f = 0; f < nf; f++) {
                const int k = (int)(rng() % 7);
                line.push_back(shape[k][rng() % shape[k].size()]);
                if (k == 1) line.push_back(pos());
                if (k == 2) line.push_back(chr());
                if (k == 3) { line.push_back(pos()); line.push_back(chr()); }
                if (k == 4) { line.push_back(chr()); line.push_back(chr()); }
                if (k == 5) { line.push_back(pos()); line.push_back(pos()); }
                if (k == 6) { line.push_back(pos()); line.push_back(pos()); line.push_back(pos()); }
                if (rng() % 3 == 0) line.push_back(' ');
            }
        }
        while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.pop_back();
        for (auto& c : line)
            if (c == '\n' || c == '\r') c = 'x';
        dwpa::RuleSet rs;
        rs.quiet = true;
        if (rs.add_line(line, 1) != 1) continue;
        parsed++;
        for (int w = 0; w < 4; w++) {
            const size_t len = rng() % 8 == 0 ? 240 + rng() % 61 : rng() % 40;  // often near the 256-byte limit
            std::string word(len, 'a');
            for (auto& c : word) c = (char)(rng() % 4 == 0 ? rng() % 256 : 'a' + rng() % 6);
            std::string out;
            if (rs.apply_host(0, word, &out)) {
                applied++;
                if (out.size() > (size_t)dwpa::RP_PASSWORD_SIZE) {
                    fprintf(stderr, "candidate longer than %d bytes: rule '%s'\n", dwpa::RP_PASSWORD_SIZE, line.c_str());
                    return 1;
                }
            } else {
                rejected++;
            }
        }
    }
    printf("{\"iterations\": %ld, \"rules_parsed\": %ld, \"candidates\": %ld, \"rejected\": %ld}\n", iters, parsed,
           applied, rejected);
    return 0;
}
