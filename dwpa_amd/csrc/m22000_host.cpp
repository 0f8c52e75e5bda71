// m22000_host.cpp -- m22000 hashline parsing with PHP semantics and device-table building.
//
// Parsing follows web/common.php:157-237 exactly (PHP 8 quirks included, see ParsedLine).  The table builder
// expands the nonce-error-correction loop (common.php:237-300) into explicit attempt lists: every PRF message the
// PHP loop would hash is materialised here, pre-padded into SHA-1/SHA-256 blocks, so the GPU verifier only hashes
// wave-uniform data.  PHP's in-place mutation of $n across attempts *and keys* (substr_replace with offset
// clamping, :255-259) is simulated, which yields one list per key ordinal until the string reaches a fixed point.
#include "m22000_host.hpp"

#include <string.h>

#include <algorithm>
#include <map>

#include "dwpa22000.h"

namespace dwpa {

// ---------------------------------------------------------------------------------------------------------
// PHP helpers
// ---------------------------------------------------------------------------------------------------------
static bool is_xd(uint8_t c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
static int hv(uint8_t c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; }

static void hex2bin_into(const char* s, size_t n, std::string& o) {
    o.resize(n / 2);
    for (size_t i = 0; i < n / 2; i++) o[i] = (char)(hv((uint8_t)s[2 * i]) << 4 | hv((uint8_t)s[2 * i + 1]));
}
// valid_hex(s) then hex2bin(s) in one pass over a nibble table (16 = not a hex digit); false leaves o undefined
struct NibbleTable {
    uint8_t v[256];
    constexpr NibbleTable() : v() {
        for (int c = 0; c < 256; c++)
            v[c] = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : 16;
    }
};
static constexpr NibbleTable kNib;
static bool valid_hex_into(const char* s, size_t n, std::string& o) {
    if (n == 0 || (n & 1)) return false;
    o.resize(n / 2);
    uint32_t bad = 0;
    for (size_t i = 0; i < n / 2; i++) {
        const uint32_t hi = kNib.v[(uint8_t)s[2 * i]], lo = kNib.v[(uint8_t)s[2 * i + 1]];
        bad |= hi | lo;
        o[i] = (char)(hi << 4 | lo);
    }
    return bad < 16;
}
static std::string hex2bin(const char* s, size_t n) {
    std::string o;
    hex2bin_into(s, n, o);
    return o;
}

bool starts_hex(const uint8_t* p, size_t n) { return n >= 5 && memcmp(p, "$HEX[", 5) == 0; }

// hc_unhex(), common.php:3-25
std::string hc_unhex(const std::string& k) {
    if (k.size() <= 6) return k;
    const size_t in = k.size() - 6;  // substr($key, 5, -1)
    if (!(in & 1) && k.compare(0, 5, "$HEX[") == 0 && k.back() == ']') {
        bool xd = true;
        for (size_t i = 5; i < 5 + in && xd; i++) xd = is_xd((uint8_t)k[i]);
        if (xd) return hex2bin(k.data() + 5, in);
    }
    return k;
}

// zend_binary_strncmp
static int php_strncmp(const std::string& a, const std::string& b, size_t len) {
    size_t m = std::min(len, std::min(a.size(), b.size()));
    int r = memcmp(a.data(), b.data(), m);
    if (r) return r;
    size_t ma = std::min(len, a.size()), mb = std::min(len, b.size());
    return (ma > mb) - (ma < mb);
}

// PHP 8 `$field == '0N'`: numeric strings compare by value (" 1", "1.0", "+1e0" all equal '01').
static bool php_is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }
static bool php_eq_type(const char* s, size_t n, int target) {
    size_t i = 0;
    while (i < n && php_is_ws(s[i])) i++;
    const size_t st = i;
    if (i < n && (s[i] == '+' || s[i] == '-')) i++;
    size_t nd = 0, nf = 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') { i++; nd++; }
    if (i < n && s[i] == '.') {
        i++;
        while (i < n && s[i] >= '0' && s[i] <= '9') { i++; nf++; }
    }
    if (nd + nf == 0) return false;  // not numeric -> plain string compare with "0N" (which is numeric): unequal
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        size_t j = i + 1;
        if (j < n && (s[j] == '+' || s[j] == '-')) j++;
        size_t e0 = j;
        while (j < n && s[j] >= '0' && s[j] <= '9') j++;
        if (j > e0) i = j;
    }
    const size_t en = i;
    while (i < n && php_is_ws(s[i])) i++;
    if (i != n) return false;
    std::string num(s + st, en - st);
    return strtod(num.c_str(), nullptr) == (double)target;
}

// ---------------------------------------------------------------------------------------------------------
// parse
// ---------------------------------------------------------------------------------------------------------
ParsedLine parse_m22000(const char* s, size_t n) {
    ParsedLine p;
    parse_m22000_into(s, n, p);
    return p;
}

// The same into an existing ParsedLine: its strings keep their capacity (the check path re-parses a batch into
// the same objects on every call instead of allocating ~9 strings per line).
void parse_m22000_into(const char* s, size_t n, ParsedLine& p) {
    p.status = 0;
    p.kind = 0;
    p.keyver = 0;
    for (std::string* f : {&p.mac_ap, &p.mac_sta, &p.essid, &p.pmkid, &p.keymic, &p.nonce_ap, &p.eapol, &p.mp,
                           &p.field2_hex})
        f->clear();
    const char* f[9];
    size_t fl[9];
    size_t cnt = 0, st = 0;
    for (size_t i = 0; i < n && cnt < 8; i++)
        if (s[i] == '*') { f[cnt] = s + st; fl[cnt] = i - st; cnt++; st = i + 1; }
    f[cnt] = s + st; fl[cnt] = n - st; cnt++;            // explode('*', $hashline, 9)
    if (cnt != 9 || fl[0] != 3 || memcmp(f[0], "WPA", 3) != 0) { p.status = DWPA_E_FORMAT; return; }
    // the checks run in common.php's order (:159-164 before the type, :169/:192-195 after it), so the first failing
    // one sets the status
    if (!valid_hex_into(f[3], fl[3], p.mac_ap) || !valid_hex_into(f[4], fl[4], p.mac_sta) ||
        !valid_hex_into(f[5], fl[5], p.essid)) { p.status = DWPA_E_HEX; return; }
    p.field2_hex.assign(f[2], fl[2]);
    if (php_eq_type(f[1], fl[1], 1)) {
        p.kind = LINE_PMKID;
        if (!valid_hex_into(f[2], fl[2], p.pmkid)) { p.status = DWPA_E_HEX; return; }
    } else if (php_eq_type(f[1], fl[1], 2)) {
        p.kind = LINE_EAPOL;
        if (!valid_hex_into(f[2], fl[2], p.keymic) || !valid_hex_into(f[6], fl[6], p.nonce_ap) ||
            !valid_hex_into(f[7], fl[7], p.eapol) || !valid_hex_into(f[8], fl[8], p.mp)) { p.status = DWPA_E_HEX; return; }
        // unpack('x5/nkey_information/x10/a32nonce_sta', $eapol) needs 49 bytes, else null -> keyver 0
        if (p.eapol.size() >= 49) p.keyver = (((uint8_t)p.eapol[5] << 8) | (uint8_t)p.eapol[6]) & 3;
        if (p.keyver == 0) p.status = DWPA_E_KEYVER;  // common.php:274-276: unknown keyver -> False
    } else {
        p.status = DWPA_E_TYPE;
    }
}

// ---------------------------------------------------------------------------------------------------------
// padding helpers
// ---------------------------------------------------------------------------------------------------------
// SHA-1 / SHA-256 message stream of `msg` hashed after `prefix_len` bytes (the HMAC key block), big-endian words.
static std::vector<uint32_t> md_stream_be(const std::string& msg, uint64_t prefix_len) {
    std::string b = msg;
    b.push_back((char)0x80);
    while (b.size() % 64 != 56) b.push_back('\0');
    const uint64_t bits = (prefix_len + msg.size()) * 8;
    for (int i = 7; i >= 0; i--) b.push_back((char)(bits >> (8 * i)));
    std::vector<uint32_t> w(b.size() / 4);
    for (size_t i = 0; i < w.size(); i++)
        w[i] = (uint32_t)(uint8_t)b[4 * i] << 24 | (uint32_t)(uint8_t)b[4 * i + 1] << 16 |
               (uint32_t)(uint8_t)b[4 * i + 2] << 8 | (uint8_t)b[4 * i + 3];
    return w;
}
static std::vector<uint32_t> md5_stream_le(const std::string& msg, uint64_t prefix_len) {
    std::string b = msg;
    b.push_back((char)0x80);
    while (b.size() % 64 != 56) b.push_back('\0');
    const uint64_t bits = (prefix_len + msg.size()) * 8;
    for (int i = 0; i < 8; i++) b.push_back((char)(bits >> (8 * i)));
    std::vector<uint32_t> w(b.size() / 4);
    for (size_t i = 0; i < w.size(); i++)
        w[i] = (uint32_t)(uint8_t)b[4 * i] | (uint32_t)(uint8_t)b[4 * i + 1] << 8 |
               (uint32_t)(uint8_t)b[4 * i + 2] << 16 | (uint32_t)(uint8_t)b[4 * i + 3] << 24;
    return w;
}
static uint32_t be32(const std::string& s, size_t o) {
    return (uint32_t)(uint8_t)s[o] << 24 | (uint32_t)(uint8_t)s[o + 1] << 16 | (uint32_t)(uint8_t)s[o + 2] << 8 |
           (uint8_t)s[o + 3];
}
static uint32_t le32(const std::string& s, size_t o) {
    return (uint32_t)(uint8_t)s[o] | (uint32_t)(uint8_t)s[o + 1] << 8 | (uint32_t)(uint8_t)s[o + 2] << 16 |
           (uint32_t)(uint8_t)s[o + 3] << 24;
}

// ---------------------------------------------------------------------------------------------------------
// KW blocks (tables.hpp): host-expanded schedules of wave-uniform message blocks
// ---------------------------------------------------------------------------------------------------------
static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// SHA-1: kw[t] = K_t + W_t for the 16-word big-endian block m
static void sha1_kw(const uint32_t* m, std::vector<uint32_t>& out) {
    uint32_t w[80];
    for (int t = 0; t < 16; t++) w[t] = m[t];
    for (int t = 16; t < 80; t++) w[t] = rol(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    static const uint32_t K[4] = {0x5a827999u, 0x6ed9eba1u, 0x8f1bbcdcu, 0xca62c1d6u};
    for (int t = 0; t < 80; t++) out.push_back(K[t / 20] + w[t]);
}

// SHA-256: kw[t] = K_t + W_t (FIPS 180-4 round constants)
static void sha256_kw(const uint32_t* m, std::vector<uint32_t>& out) {
    static const uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    uint32_t w[64];
    for (int t = 0; t < 16; t++) w[t] = m[t];
    for (int t = 16; t < 64; t++) {
        const uint32_t s0 = ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3);
        const uint32_t s1 = ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    for (int t = 0; t < 64; t++) out.push_back(K[t] + w[t]);
}

// MD5: km[i] = K_i + M[g(i)] for the 16-word little-endian block m (RFC 1321, K_i = floor(2^32 |sin(i + 1)|))
static void md5_km(const uint32_t* m, std::vector<uint32_t>& out) {
    static const uint32_t K[64] = {
        0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
        0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
        0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
        0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
        0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
        0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
        0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
        0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};
    for (int i = 0; i < 64; i++) {
        const int g = i < 16 ? i : i < 32 ? (5 * i + 1) & 15 : i < 48 ? (3 * i + 5) & 15 : (7 * i) & 15;
        out.push_back(K[i] + m[g]);
    }
}

enum class Kw { Sha1, Sha256, Md5, Raw };
// Append blocks [b0, b1) of the 16-word-block stream w to the pool as KW blocks (Kw::Raw: as they are, 16 words
// each -- TableBuilder::raw); returns their word offset.
static uint32_t push_kw(std::vector<uint32_t>& pool, const uint32_t* w, size_t b0, size_t b1, Kw alg) {
    const uint32_t off = (uint32_t)pool.size();
    if (alg == Kw::Raw) {
        pool.insert(pool.end(), w + 16 * b0, w + 16 * b1);
        return off;
    }
    for (size_t b = b0; b < b1; b++) {
        if (alg == Kw::Sha1) sha1_kw(w + 16 * b, pool);
        else if (alg == Kw::Sha256) sha256_kw(w + 16 * b, pool);
        else md5_km(w + 16 * b, pool);
    }
    return off;
}

// PHP 8 substr_replace($s, $r, $off, $len) with offset/length clamping
static void php_substr_replace(std::string& s, const std::string& r, size_t off, size_t len) {
    if (off > s.size()) off = s.size();
    if (off + len > s.size()) len = s.size() - off;
    s.replace(off, len, r);
}

uint32_t build_salt_blocks(const std::string& essid, std::vector<uint32_t>& out) {
    out.clear();
    uint32_t nblk = 0;
    for (int i = 1; i <= 2; i++) {
        std::string m = essid;
        m.push_back('\0'); m.push_back('\0'); m.push_back('\0'); m.push_back((char)i);
        std::vector<uint32_t> w = md_stream_be(m, 64);
        nblk = (uint32_t)(w.size() / 16);
        out.insert(out.end(), w.begin(), w.end());
    }
    return nblk;
}

// ---------------------------------------------------------------------------------------------------------
// table builder
// ---------------------------------------------------------------------------------------------------------
namespace {
struct NcAtt {
    bool big;     // 'N' (big-endian) correction word, else 'V' (little-endian)
    int64_t off;
};
}  // namespace

// The 4 bytes one nonce-correction attempt writes into $n (common.php:255-259, pack('N'|'V', corr + off)).
static std::string nc_raw(const NcAtt& a, int64_t corrV, int64_t corrN) {
    const uint32_t v = (uint32_t)(uint64_t)((a.big ? corrN : corrV) + a.off);
    std::string r(4, '\0');
    for (int i = 0; i < 4; i++) r[i] = (char)(a.big ? v >> (24 - 8 * i) : v >> (8 * i));
    return r;
}

// Explicit attempt lists, used when an attempt can change the length of $n (short ANONCE: PHP's substr_replace
// then appends, and the state of $n carries over from key to key, common.php:255-259).  lists[k][a] = full PRF
// message of attempt a for the k-th non-null key; every attempt gets its own pre-padded blocks.
static void add_explicit_attempts(TableBuilder& tb, LineDev& L, const std::vector<NcAtt>& order, const std::string& n0,
                                  const std::string& pre, const std::string& post, size_t patch, int nc_mode,
                                  int64_t corrV, int64_t corrN, Kw alg, bool att_kw) {
    std::vector<std::vector<std::string>> lists;
    if (nc_mode == DWPA_NC_HASHCAT) {
        std::vector<std::string> lst;
        for (const NcAtt& a : order) {
            std::string nn = n0;
            php_substr_replace(nn, nc_raw(a, corrV, corrN), patch, 4);
            lst.push_back(pre + nn + post);
        }
        lists.push_back(std::move(lst));
    } else {
        std::string ns = n0;  // PHP's $n, carried across attempts and keys
        std::vector<std::string> starts;
        for (int q = 0; q < 256; q++) {
            starts.push_back(ns);
            std::vector<std::string> lst;
            for (const NcAtt& a : order) {
                php_substr_replace(ns, nc_raw(a, corrV, corrN), patch, 4);
                lst.push_back(pre + ns + post);
            }
            lists.push_back(std::move(lst));
            if (ns == starts.back()) break;  // fixed point: every later key sees this list again
        }
        while (lists.size() >= 2 && lists[lists.size() - 2] == lists.back()) lists.pop_back();
    }

    // pre-pad every attempt; share the leading blocks common to all of them
    std::vector<std::vector<std::vector<uint32_t>>> streams(lists.size());
    size_t minblk = SIZE_MAX;
    for (size_t k = 0; k < lists.size(); k++)
        for (const std::string& msg : lists[k]) {
            streams[k].push_back(md_stream_be(msg, 64));
            minblk = std::min(minblk, streams[k].back().size() / 16);
        }
    const std::vector<uint32_t>& ref = streams[0][0];
    size_t prefix = 0;
    while (prefix + 1 < minblk) {
        bool same = true;
        for (auto& lst : streams)
            for (auto& w : lst)
                if (!std::equal(w.begin() + 16 * prefix, w.begin() + 16 * (prefix + 1), ref.begin() + 16 * prefix)) same = false;
        if (!same) break;
        prefix++;
    }
    L.pre_off = push_kw(tb.pool, ref.data(), 0, prefix, tb.raw ? Kw::Raw : alg);
    L.pre_nblk = (uint32_t)prefix;
    L.list_off = (uint32_t)tb.atts.size();
    L.nlists = (uint32_t)lists.size();
    for (size_t k = 0; k < lists.size(); k++)
        for (size_t a = 0; a < order.size(); a++) {
            const std::vector<uint32_t>& w = streams[k][a];
            AttDev at;
            memset(&at, 0, sizeof(at));
            at.blk_off = (uint32_t)tb.pool.size();
            at.nblk = (uint32_t)(w.size() / 16 - prefix);
            at.nc = a == 0 ? 0 : (int32_t)order[a].off;
            at.endian = a == 0 ? 0u : (order[a].big ? 1u : 2u);
            tb.pool.insert(tb.pool.end(), w.begin() + 16 * prefix, w.end());
            at.kw_off = att_kw ? push_kw(tb.pool, w.data(), prefix, w.size() / 16, alg) : NO_KW;
            tb.atts.push_back(at);
        }

}

uint32_t TableBuilder::add_line(const ParsedLine& p, int nc, int nc_mode, int nec) {
    LineDev L;
    memset(&L, 0, sizeof(L));
    L.kind = (uint32_t)p.kind;
    const uint32_t idx = (uint32_t)lines.size();
    if (p.kind == LINE_PMKID) {
        std::string msg = std::string("PMK Name") + p.mac_ap + p.mac_sta;
        std::vector<uint32_t> w = md_stream_be(msg, 64);
        L.msg_nblk = (uint32_t)(w.size() / 16);
        L.msg_off = push_kw(pool, w.data(), 0, L.msg_nblk, raw ? Kw::Raw : Kw::Sha1);
        const bool ok = p.pmkid.size() >= 16;  // strncmp(20-byte digest, $pmkid, 16) needs >= 16 bytes
        for (int k = 0; k < 4; k++) L.target[k] = ok ? be32(p.pmkid, 4 * k) : 0;
        lines.push_back(L);
        never.push_back(ok ? 0 : 1);
        return idx;
    }

    // ---- EAPOL, common.php:192-300
    L.keyver = (uint32_t)p.keyver;
    const std::string nonce_sta = p.eapol.substr(17, 32);
    const std::string m = php_strncmp(p.mac_ap, p.mac_sta, 6) < 0 ? p.mac_ap + p.mac_sta : p.mac_sta + p.mac_ap;
    bool swap = false;
    std::string n0;
    if (php_strncmp(nonce_sta, p.nonce_ap, 6) < 0) n0 = nonce_sta + p.nonce_ap;
    else { n0 = p.nonce_ap + nonce_sta; swap = true; }
    int64_t corrV = 0, corrN = 0;  // unpack('x28/V'|'x28/N', $nonce_ap)[1], null -> 0 when < 32 bytes
    if (p.nonce_ap.size() >= 32) {
        corrV = le32(p.nonce_ap, 28);
        corrN = be32(p.nonce_ap, 28);
    }
    std::vector<NcAtt> order;
    order.push_back({true, 0});
    if (nc_mode == DWPA_NC_HASHCAT) {
        const uint8_t mp = p.mp.empty() ? 0 : (uint8_t)p.mp[0];
        const bool none = mp & 0x10, le_only = (mp & 0x20) && !(mp & 0x40), be_only = (mp & 0x40) && !(mp & 0x20);
        if (!none)
            for (int64_t k = 1; k <= nec; k++) {
                if (!be_only) { order.push_back({false, k}); order.push_back({false, -k}); }
                if (!le_only) { order.push_back({true, k}); order.push_back({true, -k}); }
            }
    } else {
        const int64_t halfnc = ((int64_t)nc >> 1) + 1;  // loop runs for offsets 1..halfnc (do/while, :293-300)
        for (int64_t k = 1; k <= halfnc; k++) {
            order.push_back({false, k}); order.push_back({false, -k});
            order.push_back({true, k}); order.push_back({true, -k});
        }
    }
    const bool kv3 = p.keyver == 3;
    const std::string pre = kv3 ? std::string("\x01\x00Pairwise key expansion", 24) + m
                                : std::string("Pairwise key expansion\0", 23) + m;
    const std::string post = kv3 ? std::string("\x80\x01", 2) : std::string("\0", 1);
    const size_t patch = swap ? 28 : 60;

    L.patch_w0 = L.patch_w1 = NO_PATCH;
    L.natt = (uint32_t)order.size();
    const Kw prf_alg = kv3 ? Kw::Sha256 : Kw::Sha1;
    const bool att_kw = !raw && (att_kw_all || L.natt < ATT_PARALLEL_MIN);
    if (n0.size() >= patch + 4) {
        // Every attempt rewrites exactly bytes [patch, patch+4) of $n (common.php:255-259) and never changes its
        // length, so all attempts of all keys share one message apart from those 4 bytes: one list, one shared
        // block stream, two patched words per attempt.
        const std::string base = pre + n0 + post;
        const size_t o = pre.size() + patch;  // first correction byte in the PRF message
        const std::vector<uint32_t> w = md_stream_be(base, 64);
        const uint32_t W0 = (uint32_t)(o >> 2), W1 = (uint32_t)((o + 3) >> 2);
        const uint32_t prefix = W0 / 16;
        L.pre_off = push_kw(pool, w.data(), 0, prefix, raw ? Kw::Raw : prf_alg);
        L.pre_nblk = prefix;
        const uint32_t blk_off = (uint32_t)pool.size();
        pool.insert(pool.end(), w.begin() + 16 * prefix, w.end());
        L.patch_w0 = W0 - 16 * prefix;
        L.patch_w1 = W1 - 16 * prefix;
        L.att_off = blk_off;
        L.att_nblk = (uint32_t)(w.size() / 16 - prefix);
        L.list_off = (uint32_t)atts.size();
        L.nlists = 1;
        for (size_t a = 0; a < order.size(); a++) {
            const NcAtt& na = order[a];
            const uint32_t cv = (uint32_t)(uint64_t)((na.big ? corrN : corrV) + na.off);
            uint8_t r[4];
            for (int i = 0; i < 4; i++) r[i] = (uint8_t)(na.big ? cv >> (24 - 8 * i) : cv >> (8 * i));
            uint32_t v[2] = {w[W0], w[W1]};
            for (int k = 0; k < 4; k++) {
                const size_t q = o + k;
                const int sh = 24 - 8 * (int)(q & 3);
                uint32_t& x = v[(q >> 2) == W0 ? 0 : 1];
                x = (x & ~(0xffu << sh)) | (uint32_t)r[k] << sh;
            }
            if (W0 == W1) v[1] = v[0];
            AttDev at;
            memset(&at, 0, sizeof(at));
            at.blk_off = blk_off;
            at.nblk = (uint32_t)(w.size() / 16 - prefix);
            at.nc = a == 0 ? 0 : (int32_t)order[a].off;
            at.endian = a == 0 ? 0u : (order[a].big ? 1u : 2u);
            at.v0 = v[0];
            at.v1 = v[1];
            at.kw_off = NO_KW;
            if (att_kw) {  // this attempt's blocks with its two words patched in, expanded
                std::vector<uint32_t> pw(w.begin() + 16 * prefix, w.end());
                pw[L.patch_w0] = v[0];
                pw[L.patch_w1] = v[1];
                at.kw_off = push_kw(pool, pw.data(), 0, pw.size() / 16, prf_alg);
            }
            atts.push_back(at);
        }
    } else {
        add_explicit_attempts(*this, L, order, n0, pre, post, patch, nc_mode, corrV, corrN, prf_alg, att_kw);
    }

    // MIC input
    L.mic_off = (uint32_t)pool.size();
    if (p.keyver == 1 || p.keyver == 2) {
        std::vector<uint32_t> w = p.keyver == 1 ? md5_stream_le(p.eapol, 64) : md_stream_be(p.eapol, 64);
        L.mic_nblk = (uint32_t)(w.size() / 16);
        L.mic_off = push_kw(pool, w.data(), 0, L.mic_nblk, raw ? Kw::Raw : p.keyver == 1 ? Kw::Md5 : Kw::Sha1);
    } else {
        const size_t len = p.eapol.size();
        const size_t nb = (len + 15) / 16;
        std::string b = p.eapol;
        L.cmac_complete = (len % 16 == 0) ? 1u : 0u;
        if (len % 16) {
            b.push_back((char)0x80);
            while (b.size() % 16) b.push_back('\0');
        }
        for (size_t i = 0; i < nb * 4; i++) pool.push_back(be32(b, 4 * i));
        L.mic_nblk = (uint32_t)nb;
    }
    const bool ok = p.keymic.size() >= 16;
    for (int k = 0; k < 4; k++) L.target[k] = !ok ? 0u : (p.keyver == 1 ? le32(p.keymic, 4 * k) : be32(p.keymic, 4 * k));
    lines.push_back(L);
    never.push_back(ok ? 0 : 1);
    return idx;
}

// ---------------------------------------------------------------------------------------------------------
// outfile helpers
// ---------------------------------------------------------------------------------------------------------
std::string hex_lower(const std::string& s) {
    static const char* d = "0123456789abcdef";
    std::string o;
    o.reserve(s.size() * 2);
    for (unsigned char c : s) { o.push_back(d[c >> 4]); o.push_back(d[c & 15]); }
    return o;
}

std::string hashcat_plain(const std::string& s) {
    bool hex = s.compare(0, 5, "$HEX[") == 0;
    for (unsigned char c : s)
        if (c < 0x20 || c > 0x7e || c == ':') hex = true;
    return hex ? "$HEX[" + hex_lower(s) + "]" : s;
}

}  // namespace dwpa
