// rules.cpp -- hashcat rule parsing (the whole rule language, rules.hpp), the device rule table, and host-side
// application for outfile reporting.  The candidates themselves are generated on the GPU (rules_dev.hip); the host
// runs the same interpreter (rules_apply.hpp) only to reconstruct the PSK of a hit for the outfile.  Lines that do
// not parse are reported on stderr and counted (RuleSet::skipped, dwpa_rules_count, dwpa_crack_last_stats).
#include "rules.hpp"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>

#include "engine.hpp"
#include "rules_apply.hpp"

namespace dwpa {

static int conv_pos(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'A' && c <= 'Z') return c - 'A' + 10;
    return -1;
}

// Argument shapes of the rule functions (rules.hpp lists them; oracle/rules.py is the same table).
enum ArgShape { A_NONE, A_POS, A_CHR, A_POS_CHR, A_CHR_CHR, A_POS_POS, A_POS3, A_BAD };
static ArgShape arg_shape(uint8_t op) {
    switch (op) {
    case ':': case 'l': case 'u': case 'c': case 'C': case 't': case 'r': case 'd': case 'f': case '{': case '}':
    case '[': case ']': case 'k': case 'K': case 'q': case 'E': case 'M': case '4': case '6': case 'Q':
        return A_NONE;
    case 'T': case 'p': case 'D': case 'z': case 'Z': case '\'': case 'y': case 'Y': case 'L': case 'R': case '+':
    case '-': case '.': case ',': case '<': case '>': case '_':
        return A_POS;
    case '$': case '^': case '@': case '!': case '/': case '(': case ')': case 'e':
        return A_CHR;
    case 'i': case 'o': case '=': case '%': case '3':
        return A_POS_CHR;
    case 's':
        return A_CHR_CHR;
    case 'x': case 'O': case '*':
        return A_POS_POS;
    case 'X':
        return A_POS3;
    default:
        return A_BAD;
    }
}

bool parse_rule(const std::string& line_in, std::vector<RuleOp>* ops, bool* is_rule) {
    std::string line = line_in;
    while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.pop_back();
    ops->clear();
    *is_rule = !(line.empty() || line[0] == '#');
    if (!*is_rule) return true;
    size_t i = 0;
    const size_t n = line.size();
    auto pos = [&](int* v) {
        if (i >= n) return false;
        *v = conv_pos((uint8_t)line[i++]);
        return *v >= 0;
    };
    auto chr = [&](int* v) {
        if (i >= n) return false;
        *v = (uint8_t)line[i++];
        return true;
    };
    while (i < n) {
        const uint8_t op = (uint8_t)line[i++];
        if (op == ' ') continue;  // separator between functions
        int a = 0, b = 0, c = 0;
        bool ok = true;
        switch (arg_shape(op)) {
        case A_NONE: break;
        case A_POS: ok = pos(&a); break;
        case A_CHR: ok = chr(&a); break;
        case A_POS_CHR: ok = pos(&a) && chr(&b); break;
        case A_CHR_CHR: ok = chr(&a) && chr(&b); break;
        case A_POS_POS: ok = pos(&a) && pos(&b); break;
        case A_POS3: ok = pos(&a) && pos(&b) && pos(&c); break;
        case A_BAD: ok = false; break;
        }
        if (!ok) {
            ops->clear();
            return false;
        }
        ops->push_back(RuleOp{op, (uint8_t)a, (uint8_t)b, (uint8_t)c});
    }
    if (ops->empty()) ops->push_back(RuleOp{':', 0, 0, 0});  // a line of spaces: the no-op rule
    return true;
}

bool rule_uses_rejmem(const std::vector<RuleOp>& ops) {
    for (const RuleOp& o : ops)
        switch (o.op) {
        case '<': case '>': case '_': case '!': case '/': case '(': case ')': case '=': case '%': case 'Q':  // reject
        case 'M': case '4': case '6': case 'X':                                                               // memory
            return true;
        default:
            break;
        }
    return false;
}

int RuleSet::add_line(const std::string& line_in, uint32_t lineno) {
    std::string line = line_in;
    while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.pop_back();
    std::vector<RuleOp> ops;
    bool is_rule = false;
    const bool ok = parse_rule(line, &ops, &is_rule);
    if (!is_rule) return 0;
    present++;
    if (!ok) {
        // hashcat prints "Skipping invalid or unsupported rule in file %s on line %u: %s" and goes on
        skipped.push_back(line);
        skipped_lines.push_back(lineno);
        if (!quiet)
            fprintf(stderr, "[dwpa] skipping invalid or unsupported rule in %s on line %u: %s\n", source.c_str(),
                    lineno, line.c_str());
        return -1;
    }
    if (mode == DWPA_RULES_HASHCAT && rule_uses_rejmem(ops)) {
        // hashcat's -r loader takes no reject / memory function (they work only with -j/-k): the same message
        skipped.push_back(line);
        skipped_lines.push_back(lineno);
        rejmem++;
        if (!quiet)
            fprintf(stderr,
                    "[dwpa] skipping invalid or unsupported rule in %s on line %u: %s (reject / memory functions "
                    "work only with -j/-k; DWPA_RULE_MODE=full runs them)\n",
                    source.c_str(), lineno, line.c_str());
        return -1;
    }
    rules.push_back(std::move(ops));
    text.push_back(line);
    return 1;
}

void RuleSet::load_text(const char* t, size_t len) {
    std::string cur;
    uint32_t lineno = 1;
    for (size_t i = 0; i < len; i++) {
        if (t[i] == '\n') {
            add_line(cur, lineno++);
            cur.clear();
        } else {
            cur.push_back(t[i]);
        }
    }
    if (!cur.empty()) add_line(cur, lineno);
}

int RuleSet::load_file(const char* path) {  // mode as set by the caller
    FILE* f = fopen(path, "rb");
    if (!f) return DWPA_E_IO;
    std::string all;
    char buf[65536];
    size_t got;
    while ((got = fread(buf, 1, sizeof buf, f)) > 0) all.append(buf, got);
    fclose(f);
    source = path;
    load_text(all.data(), all.size());
    if (!skipped.empty())
        fprintf(stderr, "[dwpa] %s: %zu of %u rules skipped (invalid or unsupported), %zu loaded\n", path,
                skipped.size(), present, rules.size());
    if (rules.empty()) {
        fprintf(stderr, "[dwpa] %s: no valid rules left\n", path);  // hashcat refuses to start likewise
        return DWPA_E_RULE;
    }
    return 0;
}

bool RuleSet::all_noop() const {
    for (auto& r : rules)
        for (auto& o : r)
            if (o.op != ':') return false;
    return true;
}

void RuleSet::flatten(std::vector<uint32_t>& offs, std::vector<uint32_t>& code) const {
    offs.clear();
    code.clear();
    for (auto& r : rules) {
        offs.push_back((uint32_t)code.size());
        for (auto& o : r)
            code.push_back((uint32_t)o.op | (uint32_t)o.p1 << 8 | (uint32_t)o.p2 << 16 | (uint32_t)o.p3 << 24);
    }
    offs.push_back((uint32_t)code.size());
    code.resize(code.size() + 4, 0);
}

// The device interpreter (rules_apply.hpp) run on the host: the PSK reported for a hit is the GPU's candidate.
bool RuleSet::apply_host(size_t ri, const std::string& word, std::string* out) const {
    if (word.empty() || word.size() > (size_t)RP_PASSWORD_SIZE) return false;
    uint8_t w[RULE_RP + 4], mem[RULE_RP + 4];
    memcpy(w, word.data(), word.size());
    std::vector<uint32_t> code;
    for (const RuleOp& o : rules[ri])
        code.push_back((uint32_t)o.op | (uint32_t)o.p1 << 8 | (uint32_t)o.p2 << 16 | (uint32_t)o.p3 << 24);
    const int len = rule_apply(w, (int)word.size(), mem, (const uint8_t*)word.data(), (int)word.size(), code.data(),
                               (uint32_t)code.size());
    if (len < 0) return false;
    out->assign((const char*)w, (size_t)len);
    return true;
}

int rules_upload(int device, const RuleSet& rs, DevRules* out) {
    std::vector<uint32_t> offs, code;
    rs.flatten(offs, code);
    if (hipSetDevice(device) != hipSuccess) return DWPA_E_HIP;
    out->device = device;
    out->nrules = (uint32_t)rs.size();
    if (hipMalloc(&out->offs, offs.size() * 4) != hipSuccess || hipMalloc(&out->code, code.size() * 4) != hipSuccess)
        return DWPA_E_NOMEM;
    if (hipMemcpy(out->offs, offs.data(), offs.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(out->code, code.data(), code.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return DWPA_E_HIP;
    return 0;
}

int rules_load(dwpa_scan* scan, const DevRules* r, const uint64_t* off, const uint8_t* bytes, uint64_t first,
               uint32_t nwords, hipStream_t s, bool fill) {
    if (!scan || !r || (uint64_t)nwords * r->nrules > (fill ? 16ull : 1ull) * scan_batch_cap(scan)) return DWPA_E_ARG;
    Batch& b = scan_batch_ref(scan);
    if (hipSetDevice(r->device) != hipSuccess) return DWPA_E_HIP;
    if (hipMemsetAsync(b.counters.p, 0, 4, s) != hipSuccess) return DWPA_E_HIP;
    if (launch_rules_prep(off, bytes, first, nwords, (const uint32_t*)r->offs, (const uint32_t*)r->code, r->nrules, 8,
                          63, (uint32_t*)b.mid.p, (uint64_t*)b.ids.p, (uint32_t*)b.counters.p, b.cap, s) != hipSuccess)
        return DWPA_E_HIP;
    return 0;
}

void rules_release(DevRules* r) {
    if (!r || r->device < 0) return;
    (void)hipSetDevice(r->device);
    if (r->offs) (void)hipFree(r->offs);
    if (r->code) (void)hipFree(r->code);
    r->offs = r->code = nullptr;
    r->device = -1;
}

// ---------------------------------------------------------------------------------------------------------
// scan-level rules (device-resident candidates x rules)
// ---------------------------------------------------------------------------------------------------------
struct ScanRules {
    RuleSet set;
    DevRules dev;
};
static std::mutex g_rules_mu;
static std::map<const dwpa_scan*, std::unique_ptr<ScanRules>> g_scan_rules;

void scan_rules_drop(const dwpa_scan* scan) {
    std::lock_guard<std::mutex> lk(g_rules_mu);
    auto it = g_scan_rules.find(scan);
    if (it != g_scan_rules.end()) {
        rules_release(&it->second->dev);
        g_scan_rules.erase(it);
    }
}

}  // namespace dwpa

extern "C" int dwpa_scan_set_rules(dwpa_scan* scan, const char* rules_text, size_t rules_len) {
    return dwpa::guarded([&]() -> int {
        using namespace dwpa;
        if (!scan || (!rules_text && rules_len)) return DWPA_E_ARG;
        scan_rules_drop(scan);
        auto sr = std::make_unique<ScanRules>();
        sr->set.load_text(rules_text, rules_len);
        if (sr->set.size() == 0) return DWPA_E_RULE;
        int rc = rules_upload(scan_device(scan), sr->set, &sr->dev);
        if (rc < 0) return rc;
        const int n = (int)sr->set.size();
        std::lock_guard<std::mutex> lk(g_rules_mu);
        g_scan_rules[scan] = std::move(sr);
        return n;
    });
}

extern "C" int dwpa_scan_load_rules(dwpa_scan* scan, const uint64_t* d_offsets, const uint8_t* d_bytes,
                                    uint64_t first_word, uint32_t nwords, void* hip_stream) {
    return dwpa::guarded([&]() -> int {
        using namespace dwpa;
        ScanRules* sr = nullptr;
        {
            std::lock_guard<std::mutex> lk(g_rules_mu);
            auto it = g_scan_rules.find(scan);
            if (it != g_scan_rules.end()) sr = it->second.get();
        }
        if (!sr) return DWPA_E_RULE;
        return rules_load(scan, &sr->dev, d_offsets, d_bytes, first_word, nwords, (hipStream_t)hip_stream);
    });
}

// ---------------------------------------------------------------------------------------------------------
// C ABI: rule counting (host only) and rule expansion on the GPU (replaces `hashcat --stdout -r rules`,
// help_crack.py:508,575)
// ---------------------------------------------------------------------------------------------------------
extern "C" int dwpa_rules_count(const char* rules_text, size_t rules_len, uint32_t* nrules_present,
                                uint32_t* nrules_parsed, uint32_t* first_skipped_line) {
    return dwpa::guarded([&]() -> int {
        using namespace dwpa;
        if (!rules_text && rules_len) return DWPA_E_ARG;
        RuleSet rs;
        rs.quiet = true;
        rs.load_text(rules_text, rules_len);
        if (nrules_present) *nrules_present = rs.present;
        if (nrules_parsed) *nrules_parsed = (uint32_t)rs.size();
        if (first_skipped_line)
            *first_skipped_line = rs.skipped_lines.empty() ? 0 : rs.skipped_lines[0];
        return 0;
    });
}

extern "C" int dwpa_rules_count_ex(const char* rules_text, size_t rules_len, dwpa_rules_counts* out) {
    return dwpa::guarded([&]() -> int {
        using namespace dwpa;
        if ((!rules_text && rules_len) || !out) return DWPA_E_ARG;
        RuleSet full;  // the interpreter's load; the hashcat loader keeps its parsed lines without reject / memory ones
        full.quiet = true;
        full.load_text(rules_text, rules_len);
        RuleSet hc;
        hc.quiet = true;
        hc.mode = DWPA_RULES_HASHCAT;
        hc.load_text(rules_text, rules_len);
        memset(out, 0, sizeof(*out));
        out->present = full.present;
        out->parsed = (uint32_t)full.size();
        out->loaded_hashcat = (uint32_t)hc.size();
        out->rejmem = hc.rejmem;
        out->invalid = (uint32_t)full.skipped.size();
        out->first_invalid_line = full.skipped_lines.empty() ? 0 : full.skipped_lines[0];
        for (size_t i = 0; i < hc.skipped_lines.size() && !out->first_rejmem_line; i++)
            if (std::find(full.skipped_lines.begin(), full.skipped_lines.end(), hc.skipped_lines[i]) ==
                full.skipped_lines.end())
                out->first_rejmem_line = hc.skipped_lines[i];
        return 0;
    });
}

extern "C" int dwpa_rules_expand(int device, const char* rules_text, size_t rules_len, const dwpa_bytes* words,
                                 size_t nwords, uint8_t* out /* nwords*nrules*256 */, uint32_t* out_len,
                                 uint32_t* nrules_out) {
    return dwpa::guarded([&]() -> int {
        using namespace dwpa;
        if ((!words && nwords) || !nrules_out || (!rules_text && rules_len)) return DWPA_E_ARG;
        RuleSet rs;
        rs.quiet = true;  // callers report skipped lines once per file through dwpa_rules_count, not per chunk
        rs.load_text(rules_text, rules_len);
        *nrules_out = (uint32_t)rs.size();
        if (!out || !out_len) return 0;
        if (rs.size() == 0 || nwords == 0) return 0;
        int rc = engine_init();
        if (rc < 0) return rc;
        if (hipSetDevice(device) != hipSuccess) return DWPA_E_NODEV;
        std::vector<uint64_t> off(nwords + 1, 0);
        std::string bytes;
        for (size_t i = 0; i < nwords; i++) {
            off[i] = bytes.size();
            if (words[i].ptr) bytes.append((const char*)words[i].ptr, words[i].len);
        }
        off[nwords] = bytes.size();
        bytes.append(16, '\0');
        DevRules dr;
        if ((rc = rules_upload(device, rs, &dr)) < 0) return rc;
        const size_t ncand = nwords * rs.size();
        void *d_off = nullptr, *d_bytes = nullptr, *d_out = nullptr, *d_len = nullptr;
        rc = 0;
        if (hipMalloc(&d_off, off.size() * 8) || hipMalloc(&d_bytes, bytes.size()) || hipMalloc(&d_out, ncand * 256) ||
            hipMalloc(&d_len, ncand * 4))
            rc = DWPA_E_NOMEM;
        if (!rc && (hipMemcpy(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice) ||
                    hipMemcpy(d_bytes, bytes.data(), bytes.size(), hipMemcpyHostToDevice)))
            rc = DWPA_E_HIP;
        if (!rc && launch_rules_expand((const uint64_t*)d_off, (const uint8_t*)d_bytes, (uint32_t)nwords,
                                       (const uint32_t*)dr.offs, (const uint32_t*)dr.code, dr.nrules, (uint8_t*)d_out,
                                       (uint32_t*)d_len, nullptr) != hipSuccess)
            rc = DWPA_E_HIP;
        if (!rc && (hipMemcpy(out, d_out, ncand * 256, hipMemcpyDeviceToHost) ||
                    hipMemcpy(out_len, d_len, ncand * 4, hipMemcpyDeviceToHost)))
            rc = DWPA_E_HIP;
        (void)hipFree(d_off); (void)hipFree(d_bytes); (void)hipFree(d_out); (void)hipFree(d_len);
        rules_release(&dr);
        return rc;
    });
}

// Host-only application of rule `rule_index` (0-based among the rules of rules_text that parse) to one word: the
// interpreter the GPU runs (rules_apply.hpp), compiled for the host.  *out_len = the candidate's length, or
// 0xFFFFFFFF when it is rejected.  For parity tests without a device and for reporting a hit's PSK.
extern "C" int dwpa_rules_apply_host(const char* rules_text, size_t rules_len, uint32_t rule_index, const uint8_t* word,
                                     size_t word_len, uint8_t* out /* 256 bytes */, uint32_t* out_len) {
    return dwpa::guarded([&]() -> int {
        using namespace dwpa;
        if ((!rules_text && rules_len) || (!word && word_len) || !out || !out_len) return DWPA_E_ARG;
        RuleSet rs;
        rs.quiet = true;
        rs.load_text(rules_text, rules_len);
        if (rule_index >= rs.size()) return DWPA_E_RULE;
        std::string cand;
        if (!rs.apply_host(rule_index, std::string((const char*)word, word_len), &cand)) {
            *out_len = 0xFFFFFFFFu;
            return 0;
        }
        memcpy(out, cand.data(), cand.size());
        *out_len = (uint32_t)cand.size();
        return 0;
    });
}
