// rules.cpp -- hashcat rule parsing, the device rule table, and host-side application for outfile reporting.
// The candidates themselves are generated on the GPU (rules_dev.hip); the host applies a rule only to reconstruct
// the PSK of a hit for the outfile, and the two are held identical by tests/test_rules*.py.
#include "rules.hpp"

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>

#include "engine.hpp"

namespace dwpa {

static int conv_pos(uint8_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'A' && c <= 'Z') return c - 'A' + 10;
    return -1;
}

int RuleSet::add_line(const std::string& line_in) {
    std::string line = line_in;
    while (!line.empty() && (line.back() == '\n' || line.back() == '\r')) line.pop_back();
    if (line.empty() || line[0] == '#') return 0;
    std::vector<RuleOp> ops;
    size_t i = 0;
    const size_t n = line.size();
    while (i < n) {
        const uint8_t op = (uint8_t)line[i++];
        RuleOp r{op, 0, 0};
        switch (op) {
        case ' ':
            continue;  // separator between ops
        case ':': case 'l': case 'u': case 'c': case 'C': case 't': case 'r': case 'd': case 'f':
        case '{': case '}': case '[': case ']': case 'q':
            break;
        case 'T': case 'p': case 'D': case '\'': case 'z': case 'Z': {
            if (i >= n) return 0;
            int p = conv_pos((uint8_t)line[i++]);
            if (p < 0) return 0;
            r.p1 = (uint8_t)p;
            break;
        }
        case '$': case '^': case '@':
            if (i >= n) return 0;
            r.p1 = (uint8_t)line[i++];
            break;
        case 's':
            if (i + 2 > n) return 0;
            r.p1 = (uint8_t)line[i++];
            r.p2 = (uint8_t)line[i++];
            break;
        default:
            return 0;  // unsupported op: skip this rule line
        }
        ops.push_back(r);
    }
    if (ops.empty()) return 0;
    rules.push_back(std::move(ops));
    text.push_back(line);
    return 1;
}

int RuleSet::load_file(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) return DWPA_E_IO;
    std::string cur;
    int ch;
    while ((ch = fgetc(f)) != EOF) {
        if (ch == '\n') {
            add_line(cur);
            cur.clear();
        } else {
            cur.push_back((char)ch);
        }
    }
    if (!cur.empty()) add_line(cur);
    fclose(f);
    return rules.empty() ? DWPA_E_RULE : 0;
}

bool RuleSet::all_noop() const {
    for (auto& r : rules)
        for (auto& o : r)
            if (o.op != ':') return false;
    return true;
}

void RuleSet::flatten(std::vector<uint32_t>& offs, std::vector<uint8_t>& code) const {
    offs.clear();
    code.clear();
    for (auto& r : rules) {
        offs.push_back((uint32_t)code.size());
        for (auto& o : r) {
            code.push_back(o.op);
            code.push_back(o.p1);
            code.push_back(o.p2);
        }
    }
    offs.push_back((uint32_t)code.size());
    code.resize(code.size() + 16, 0);
}

static inline bool is_lower(uint8_t c) { return c >= 'a' && c <= 'z'; }
static inline bool is_upper(uint8_t c) { return c >= 'A' && c <= 'Z'; }

// Host restatement of the device interpreter in rules_dev.hip (same op set and overflow rules).
std::string RuleSet::apply_host(size_t ri, const std::string& word) const {
    if (word.empty() || word.size() > (size_t)RP_PASSWORD_SIZE) return std::string();
    std::string w = word;
    for (const RuleOp& o : rules[ri]) {
        const size_t len = w.size();
        switch (o.op) {
        case ':': break;
        case 'l': for (auto& c : w) if (is_upper((uint8_t)c)) c ^= 0x20; break;
        case 'u': for (auto& c : w) if (is_lower((uint8_t)c)) c ^= 0x20; break;
        case 'c':
            for (auto& c : w) if (is_upper((uint8_t)c)) c ^= 0x20;
            if (len && is_lower((uint8_t)w[0])) w[0] ^= 0x20;
            break;
        case 'C':
            for (auto& c : w) if (is_lower((uint8_t)c)) c ^= 0x20;
            if (len && is_upper((uint8_t)w[0])) w[0] ^= 0x20;
            break;
        case 't': for (auto& c : w) if (is_lower((uint8_t)c) || is_upper((uint8_t)c)) c ^= 0x20; break;
        case 'T': if (o.p1 < len && (is_lower((uint8_t)w[o.p1]) || is_upper((uint8_t)w[o.p1]))) w[o.p1] ^= 0x20; break;
        case 'r': std::reverse(w.begin(), w.end()); break;
        case 'd': if (2 * len < (size_t)RP_PASSWORD_SIZE) w += w; break;
        case 'p': if (len * o.p1 + len < (size_t)RP_PASSWORD_SIZE) { std::string b = w; for (int k = 0; k < o.p1; k++) w += b; } break;
        case 'f': if (2 * len < (size_t)RP_PASSWORD_SIZE) { std::string b = w; std::reverse(b.begin(), b.end()); w += b; } break;
        case '{': if (len) { w = w.substr(1) + w[0]; } break;
        case '}': if (len) { w = w.back() + w.substr(0, len - 1); } break;
        case '[': if (len) w.erase(0, 1); break;
        case ']': if (len) w.pop_back(); break;
        case 'q': if (2 * len < (size_t)RP_PASSWORD_SIZE) { std::string b; for (char c : w) { b += c; b += c; } w = b; } break;
        case 'D': if (o.p1 < len) w.erase(o.p1, 1); break;
        case '\'': if (o.p1 < len) w.resize(o.p1); break;
        case 'z': if (len && len + o.p1 < (size_t)RP_PASSWORD_SIZE) w = std::string(o.p1, w[0]) + w; break;
        case 'Z': if (len && len + o.p1 < (size_t)RP_PASSWORD_SIZE) w += std::string(o.p1, w.back()); break;
        case '$': if (len + 1 < (size_t)RP_PASSWORD_SIZE) w.push_back((char)o.p1); break;
        case '^': if (len + 1 < (size_t)RP_PASSWORD_SIZE) w.insert(w.begin(), (char)o.p1); break;
        case 's': for (auto& c : w) if ((uint8_t)c == o.p1) c = (char)o.p2; break;
        case '@': w.erase(std::remove(w.begin(), w.end(), (char)o.p1), w.end()); break;
        default: break;
        }
    }
    return w;
}

int rules_upload(int device, const RuleSet& rs, DevRules* out) {
    std::vector<uint32_t> offs;
    std::vector<uint8_t> code;
    rs.flatten(offs, code);
    if (hipSetDevice(device) != hipSuccess) return DWPA_E_HIP;
    out->device = device;
    out->nrules = (uint32_t)rs.size();
    if (hipMalloc(&out->offs, offs.size() * 4) != hipSuccess || hipMalloc(&out->code, code.size()) != hipSuccess)
        return DWPA_E_NOMEM;
    if (hipMemcpy(out->offs, offs.data(), offs.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(out->code, code.data(), code.size(), hipMemcpyHostToDevice) != hipSuccess)
        return DWPA_E_HIP;
    return 0;
}

int rules_load(dwpa_scan* scan, const DevRules* r, const uint64_t* off, const uint8_t* bytes, uint64_t first,
               uint32_t nwords, hipStream_t s, bool fill) {
    if (!scan || !r || (uint64_t)nwords * r->nrules > (fill ? 16ull : 1ull) * scan_batch_cap(scan)) return DWPA_E_ARG;
    Batch& b = scan_batch_ref(scan);
    if (hipSetDevice(r->device) != hipSuccess) return DWPA_E_HIP;
    if (hipMemsetAsync(b.counters.p, 0, 4, s) != hipSuccess) return DWPA_E_HIP;
    if (launch_rules_prep(off, bytes, first, nwords, (const uint32_t*)r->offs, (const uint8_t*)r->code, r->nrules, 8,
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
    using namespace dwpa;
    if (!scan || (!rules_text && rules_len)) return DWPA_E_ARG;
    scan_rules_drop(scan);
    auto sr = std::make_unique<ScanRules>();
    std::string cur;
    for (size_t i = 0; i < rules_len; i++) {
        if (rules_text[i] == '\n') { sr->set.add_line(cur); cur.clear(); }
        else cur.push_back(rules_text[i]);
    }
    if (!cur.empty()) sr->set.add_line(cur);
    if (sr->set.size() == 0) return DWPA_E_RULE;
    int rc = rules_upload(scan_device(scan), sr->set, &sr->dev);
    if (rc < 0) return rc;
    const int n = (int)sr->set.size();
    std::lock_guard<std::mutex> lk(g_rules_mu);
    g_scan_rules[scan] = std::move(sr);
    return n;
}

extern "C" int dwpa_scan_load_rules(dwpa_scan* scan, const uint64_t* d_offsets, const uint8_t* d_bytes,
                                    uint64_t first_word, uint32_t nwords, void* hip_stream) {
    using namespace dwpa;
    ScanRules* sr = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_rules_mu);
        auto it = g_scan_rules.find(scan);
        if (it != g_scan_rules.end()) sr = it->second.get();
    }
    if (!sr) return DWPA_E_RULE;
    return rules_load(scan, &sr->dev, d_offsets, d_bytes, first_word, nwords, (hipStream_t)hip_stream);
}

// ---------------------------------------------------------------------------------------------------------
// C ABI: rule expansion on the GPU (replaces `hashcat --stdout -r rules` in help_crack.py:508,575)
// ---------------------------------------------------------------------------------------------------------
extern "C" int dwpa_rules_expand(int device, const char* rules_text, size_t rules_len, const dwpa_bytes* words,
                                 size_t nwords, uint8_t* out /* nwords*nrules*256 */, uint32_t* out_len,
                                 uint32_t* nrules_out) {
    using namespace dwpa;
    if ((!words && nwords) || !nrules_out) return DWPA_E_ARG;
    RuleSet rs;
    std::string cur;
    for (size_t i = 0; i < rules_len; i++) {
        if (rules_text[i] == '\n') { rs.add_line(cur); cur.clear(); }
        else cur.push_back(rules_text[i]);
    }
    if (!cur.empty()) rs.add_line(cur);
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
                                   (const uint32_t*)dr.offs, (const uint8_t*)dr.code, dr.nrules, (uint8_t*)d_out,
                                   (uint32_t*)d_len, nullptr) != hipSuccess)
        rc = DWPA_E_HIP;
    if (!rc && (hipMemcpy(out, d_out, ncand * 256, hipMemcpyDeviceToHost) ||
                hipMemcpy(out_len, d_len, ncand * 4, hipMemcpyDeviceToHost)))
        rc = DWPA_E_HIP;
    (void)hipFree(d_off); (void)hipFree(d_bytes); (void)hipFree(d_out); (void)hipFree(d_len);
    rules_release(&dr);
    return rc;
}
