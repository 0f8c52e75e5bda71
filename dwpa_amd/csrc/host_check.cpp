// host_check.cpp -- the host (CPU) backend behind the same C ABI ("the server may have no GPU, so the
// CPU backend is mandatory behind the same ABI").
//
// It answers dwpa_check_m22000 / dwpa_check_batch / dwpa_pbkdf2_pmk on the host's cores, with the library's own
// primitives (host_crypto.cpp: SHA-NI / AES-NI or scalar) -- never the oracle, never OpenSSL.  engine.cpp routes a
// call here in two cases:
//   * small calls: a call whose work is at most dwpa_config.host_max_pmks PMK-equivalents (put_work's one key per
//     check_key_m22000 call, common.php:902) -- one PBKDF2 chain on a lone GPU wave takes ~8 ms, on a SHA-NI core
//     well under one;
//   * no usable gfx950 device, or a device call that failed, when dwpa_config.allow_cpu_fallback (or
//     DWPA_CPU_FALLBACK=1) is set.
// Every call reports which backend answered it (dwpa_check_stats.backend).
//
// The semantics are the device path's, built from the same host pieces: parse_m22000 (PHP acceptance rules), the
// TableBuilder's attempt lists (common.php:237-300 nonce-correction order, PHP's $n mutation across attempts and
// keys) in raw-block form, first key in input order then first attempt in PHP order (common.php:186,280-289), and the
// caller's $pmk for the first non-null key only (:178,188,246,302).
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "dwpa22000.h"
#include "engine.hpp"
#include "host_crypto.hpp"
#include "m22000_host.hpp"

namespace dwpa {

using namespace hostc;

namespace {

constexpr uint32_t NO_UID = 0xffffffffu;  // slot whose PMK is the caller's

// HMAC midstates of a 32-byte PMK (key block = PMK || 0^32) for SHA-1 and SHA-256
void pmk_mid_sha1(const uint32_t pmk[8], uint32_t ip[5], uint32_t op[5]) {
    uint32_t wi[16], wo[16];
    for (int t = 0; t < 16; t++) {
        const uint32_t v = t < 8 ? pmk[t] : 0;
        wi[t] = v ^ 0x36363636u;
        wo[t] = v ^ 0x5c5c5c5cu;
    }
    memcpy(ip, SHA1_IV, 20);
    memcpy(op, SHA1_IV, 20);
    sha1_compress(ip, wi);
    sha1_compress(op, wo);
}
void pmk_mid_sha256(const uint32_t pmk[8], uint32_t ip[8], uint32_t op[8]) {
    uint32_t wi[16], wo[16];
    for (int t = 0; t < 16; t++) {
        const uint32_t v = t < 8 ? pmk[t] : 0;
        wi[t] = v ^ 0x36363636u;
        wo[t] = v ^ 0x5c5c5c5cu;
    }
    memcpy(ip, SHA256_IV, 32);
    memcpy(op, SHA256_IV, 32);
    sha256_compress(ip, wi);
    sha256_compress(op, wo);
}

inline uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }

// Block b of attempt `at`'s PRF blocks after the line's shared prefix, its two correction words patched in when the
// line shares one stream between all attempts (tables.hpp LineDev.patch_w0/_w1).
inline void att_block(const LineDev& L, const AttDev& at, const uint32_t* pool, uint32_t b, uint32_t w[16]) {
    memcpy(w, pool + at.blk_off + 16 * (size_t)b, 64);
    if (L.patch_w0 != NO_PATCH) {
        const uint32_t lo = 16 * b;
        if (L.patch_w0 >= lo && L.patch_w0 < lo + 16) w[L.patch_w0 - lo] = at.v0;
        if (L.patch_w1 >= lo && L.patch_w1 < lo + 16) w[L.patch_w1 - lo] = at.v1;
    }
}

// HMAC-SHA1 / HMAC-MD5 keyed with the 16-byte KCK (PTK words 0..3) over the EAPOL frame: the keyver 2 / 1 MIC
// (common.php:264,268).  mic[4]: SHA-1 words (big-endian) or MD5 words (little-endian), as LineDev.target.
void mic_sha1(const uint32_t kck[4], const uint32_t* blocks, uint32_t nblk, uint32_t mic[5]) {
    uint32_t ki[16], ko[16], st[5], w[16];
    for (int t = 0; t < 16; t++) {
        const uint32_t v = t < 4 ? kck[t] : 0;
        ki[t] = v ^ 0x36363636u;
        ko[t] = v ^ 0x5c5c5c5cu;
    }
    memcpy(st, SHA1_IV, 20);
    sha1_compress(st, ki);
    for (uint32_t b = 0; b < nblk; b++) sha1_compress(st, blocks + 16 * (size_t)b);
    memcpy(w, st, 20);
    w[5] = 0x80000000u;
    for (int t = 6; t < 15; t++) w[t] = 0;
    w[15] = (64 + 20) * 8;
    memcpy(mic, SHA1_IV, 20);
    sha1_compress(mic, ko);
    sha1_compress(mic, w);
}
void mic_md5(const uint32_t kck_be[4], const uint32_t* blocks, uint32_t nblk, uint32_t mic[4]) {
    uint32_t ki[16], ko[16], st[4], w[16];
    for (int t = 0; t < 16; t++) {
        const uint32_t v = t < 4 ? bswap(kck_be[t]) : 0;  // the KCK's bytes as little-endian words
        ki[t] = v ^ 0x36363636u;
        ko[t] = v ^ 0x5c5c5c5cu;
    }
    memcpy(st, MD5_IV, 16);
    md5_compress(st, ki);
    for (uint32_t b = 0; b < nblk; b++) md5_compress(st, blocks + 16 * (size_t)b);
    memcpy(w, st, 16);
    w[4] = 0x80u;
    for (int t = 5; t < 16; t++) w[t] = 0;
    w[14] = (64 + 16) * 8;
    memcpy(mic, MD5_IV, 16);
    md5_compress(mic, ko);
    md5_compress(mic, w);
}

// Keyver 1/2 attempts at[0..3] (equal block counts) against the line: the first of them whose MIC matches (0..3) or
// -1.  The PRF, the PTK's outer hash and the keyver 2 MIC run as four SHA-1 chains in lock step; keyver 1's HMAC-MD5
// per attempt.
int64_t verify_att4(const LineDev& L, const AttDev* at, const uint32_t* pool, const uint32_t pre[5],
                    const uint32_t op[5]) {
    uint32_t st[4][5], w[4][16];
    const uint32_t* wp[4] = {w[0], w[1], w[2], w[3]};
    for (int n = 0; n < 4; n++) memcpy(st[n], pre, 20);
    for (uint32_t b = 0; b < at[0].nblk; b++) {
        for (int n = 0; n < 4; n++) att_block(L, at[n], pool, b, w[n]);
        sha1_compress_x4(st, wp);
    }
    uint32_t ptk[4][5];
    for (int n = 0; n < 4; n++) {
        memcpy(w[n], st[n], 20);
        w[n][5] = 0x80000000u;
        for (int t = 6; t < 15; t++) w[n][t] = 0;
        w[n][15] = (64 + 20) * 8;
        memcpy(ptk[n], op, 20);
    }
    sha1_compress_x4(ptk, wp);
    uint32_t mic[4][5];
    if (L.keyver == 2) {  // HMAC-SHA1(KCK, EAPOL) (common.php:268), as mic_sha1
        uint32_t ko[4][16], mo[4][5];
        for (int n = 0; n < 4; n++)
            for (int t = 0; t < 16; t++) {
                const uint32_t v = t < 4 ? ptk[n][t] : 0;
                w[n][t] = v ^ 0x36363636u;
                ko[n][t] = v ^ 0x5c5c5c5cu;
            }
        for (int n = 0; n < 4; n++) memcpy(mic[n], SHA1_IV, 20);
        sha1_compress_x4(mic, wp);
        for (uint32_t b = 0; b < L.mic_nblk; b++) {
            const uint32_t* blk = pool + L.mic_off + 16 * (size_t)b;
            const uint32_t* bp[4] = {blk, blk, blk, blk};
            sha1_compress_x4(mic, bp);
        }
        const uint32_t* kop[4] = {ko[0], ko[1], ko[2], ko[3]};
        for (int n = 0; n < 4; n++) memcpy(mo[n], SHA1_IV, 20);
        sha1_compress_x4(mo, kop);
        for (int n = 0; n < 4; n++) {
            memcpy(w[n], mic[n], 20);
            w[n][5] = 0x80000000u;
            for (int t = 6; t < 15; t++) w[n][t] = 0;
            w[n][15] = (64 + 20) * 8;
        }
        sha1_compress_x4(mo, wp);
        for (int n = 0; n < 4; n++)
            if (memcmp(mo[n], L.target, 16) == 0) return n;
        return -1;
    }
    for (int n = 0; n < 4; n++) {  // keyver 1: HMAC-MD5(KCK, EAPOL) (common.php:264)
        mic_md5(ptk[n], pool + L.mic_off, L.mic_nblk, mic[n]);
        if (memcmp(mic[n], L.target, 16) == 0) return n;
    }
    return -1;
}

// The first attempt of the line's list for key ordinal `ord` under which `pmk` verifies, or -1 (PMKID lines: 0 / -1).
int64_t verify_pmk(const TableBuilder& tb, uint32_t li, uint32_t ord, const uint32_t pmk[8]) {
    const LineDev& L = tb.lines[li];
    if (tb.never[li]) return -1;
    const uint32_t* pool = tb.pool.data();
    if (L.kind == LINE_PMKID) {  // HMAC-SHA1(PMK, "PMK Name" || AP || STA)[0:16] (common.php:183-185)
        uint32_t ip[5], op[5], w[16];
        pmk_mid_sha1(pmk, ip, op);
        for (uint32_t b = 0; b < L.msg_nblk; b++) sha1_compress(ip, pool + L.msg_off + 16 * (size_t)b);
        memcpy(w, ip, 20);
        w[5] = 0x80000000u;
        for (int t = 6; t < 15; t++) w[t] = 0;
        w[15] = (64 + 20) * 8;
        sha1_compress(op, w);
        return memcmp(op, L.target, 16) == 0 ? 0 : -1;
    }
    const uint32_t list = std::min(ord, L.nlists - 1);
    const AttDev* at = tb.atts.data() + L.list_off + (size_t)list * L.natt;
    uint32_t w[16];
    if (L.keyver != 3) {
        // PTK = HMAC-SHA1(PMK, "Pairwise key expansion\0" || m || n || "\0") (common.php:263,267)
        uint32_t ip[5], op[5], pre[5];
        pmk_mid_sha1(pmk, ip, op);
        memcpy(pre, ip, 20);
        for (uint32_t b = 0; b < L.pre_nblk; b++) sha1_compress(pre, pool + L.pre_off + 16 * (size_t)b);
        uint32_t a = 0;
        // four attempts at a time, their SHA-1 compressions in lock step (a miss walks every attempt of the window)
        for (; a + 4 <= L.natt; a += 4) {
            if (at[a].nblk != at[a + 1].nblk || at[a].nblk != at[a + 2].nblk || at[a].nblk != at[a + 3].nblk) break;
            const int64_t r = verify_att4(L, at + a, pool, pre, op);
            if (r >= 0) return a + r;
        }
        for (; a < L.natt; a++) {
            uint32_t st[5], ptk[5], mic[5];
            memcpy(st, pre, 20);
            for (uint32_t b = 0; b < at[a].nblk; b++) {
                att_block(L, at[a], pool, b, w);
                sha1_compress(st, w);
            }
            memcpy(w, st, 20);
            w[5] = 0x80000000u;
            for (int t = 6; t < 15; t++) w[t] = 0;
            w[15] = (64 + 20) * 8;
            memcpy(ptk, op, 20);
            sha1_compress(ptk, w);
            if (L.keyver == 2) mic_sha1(ptk, pool + L.mic_off, L.mic_nblk, mic);
            else mic_md5(ptk, pool + L.mic_off, L.mic_nblk, mic);
            if (memcmp(mic, L.target, 16) == 0) return a;
        }
        return -1;
    }
    // keyver 3: PTK = HMAC-SHA256(PMK, "\1\0Pairwise key expansion" || m || n || "\x80\1"), MIC = AES-128-CMAC(KCK,
    // EAPOL) (common.php:271-272)
    uint32_t ip[8], op[8], pre[8];
    pmk_mid_sha256(pmk, ip, op);
    memcpy(pre, ip, 32);
    for (uint32_t b = 0; b < L.pre_nblk; b++) sha256_compress(pre, pool + L.pre_off + 16 * (size_t)b);
    std::vector<uint8_t> cm(16 * (size_t)L.mic_nblk);
    for (size_t i = 0; i < 4 * (size_t)L.mic_nblk; i++) {
        const uint32_t v = pool[L.mic_off + i];
        cm[4 * i] = (uint8_t)(v >> 24);
        cm[4 * i + 1] = (uint8_t)(v >> 16);
        cm[4 * i + 2] = (uint8_t)(v >> 8);
        cm[4 * i + 3] = (uint8_t)v;
    }
    uint8_t target[16];
    for (int k = 0; k < 4; k++) {
        target[4 * k] = (uint8_t)(L.target[k] >> 24);
        target[4 * k + 1] = (uint8_t)(L.target[k] >> 16);
        target[4 * k + 2] = (uint8_t)(L.target[k] >> 8);
        target[4 * k + 3] = (uint8_t)L.target[k];
    }
    for (uint32_t a = 0; a < L.natt; a++) {
        uint32_t st[8], ptk[8];
        memcpy(st, pre, 32);
        for (uint32_t b = 0; b < at[a].nblk; b++) {
            att_block(L, at[a], pool, b, w);
            sha256_compress(st, w);
        }
        memcpy(w, st, 32);
        w[8] = 0x80000000u;
        for (int t = 9; t < 15; t++) w[t] = 0;
        w[15] = (64 + 32) * 8;
        memcpy(ptk, op, 32);
        sha256_compress(ptk, w);
        uint8_t kck[16], mac[16];
        for (int k = 0; k < 4; k++) {
            kck[4 * k] = (uint8_t)(ptk[k] >> 24);
            kck[4 * k + 1] = (uint8_t)(ptk[k] >> 16);
            kck[4 * k + 2] = (uint8_t)(ptk[k] >> 8);
            kck[4 * k + 3] = (uint8_t)ptk[k];
        }
        aes128_cmac(kck, cm.data(), L.mic_nblk, L.cmac_complete != 0, mac);
        if (memcmp(mac, target, 16) == 0) return a;
    }
    return -1;
}

// One unique (ESSID, key) PMK to derive: its key bytes and its ESSID group's salt blocks.
struct Derive {
    const uint8_t* key;
    size_t len;
    uint32_t group;
};

// Keys per chunk for n derives over `threads` threads: the chunk size whose estimated makespan (rounds of chunks over
// the threads x one chunk's measured cost) is least -- 1 or 2 keys on SHA-NI chains for a few keys per thread
// (latency), 8 or 16 keys on AVX-512 once there are enough for the threads (throughput).
size_t derive_chunk(size_t n, size_t threads) {
    const Pbkdf2Costs& c = pbkdf2_costs();
    size_t per = 1;
    auto span = [&](size_t k, double cost) { return (double)(((n + k - 1) / k + threads - 1) / threads) * cost; };
    double best = span(1, c.ni1);
    if (span(2, c.ni) < best) best = span(2, c.ni), per = 2;
    if (c.avx1 > 0 && span(8, c.avx1) < best) best = span(8, c.avx1), per = 8;
    if (c.avx2 > 0 && span(16, c.avx2) < best) best = span(16, c.avx2), per = 16;
    return per;
}

// PBKDF2 of n keys over up to host_threads() threads: chunks of derive_chunk() keys handed out through an atomic
// counter, so uneven keys (a 64 KiB one) do not stall a part.  get(i, key, len, salt, nblk) describes key i (salt in
// build_salt_blocks layout), put(i, pmk) takes its PMK (8 big-endian words).
template <class Get, class Put>
void derive_each(size_t nkeys, Get get, Put put) {
    const size_t per = derive_chunk(nkeys, host_threads_for(SIZE_MAX, 1));
    const size_t nchunks = (nkeys + per - 1) / per;
    std::atomic<size_t> next{0};
    host_parallel(host_threads_for(nchunks, 1), [&](size_t) {
        std::vector<std::array<uint32_t, 10>> mid(per);
        std::vector<std::array<uint32_t, 8>> out(per);
        std::vector<const uint32_t*> sp(per);
        std::vector<uint32_t> nb(per);
        for (size_t c; (c = next.fetch_add(1, std::memory_order_relaxed)) < nchunks;) {
            const size_t i0 = c * per, n = std::min(per, nkeys - i0);
            for (size_t k = 0; k < n; k++) {
                const uint8_t* key;
                size_t len;
                get(i0 + k, key, len, sp[k], nb[k]);
                hmac_sha1_mid(key, len, mid[k].data(), mid[k].data() + 5);
            }
            pbkdf2_sha1(n, (const uint32_t(*)[10])mid.data(), sp.data(), nb.data(), (uint32_t(*)[8])out.data());
            for (size_t k = 0; k < n; k++) put(i0 + k, out[k].data());
        }
    });
}

// PBKDF2 of every entry of `dv` into pmk[i] (big-endian words).
void derive_all(const std::vector<Derive>& dv, const std::vector<std::vector<uint32_t>>& salt,
                const std::vector<uint32_t>& nblk, std::vector<std::array<uint32_t, 8>>& pmk) {
    pmk.resize(dv.size());
    derive_each(
        dv.size(),
        [&](size_t i, const uint8_t*& key, size_t& len, const uint32_t*& sp, uint32_t& nb) {
            key = dv[i].key;
            len = dv[i].len;
            sp = salt[dv[i].group].data();
            nb = nblk[dv[i].group];
        },
        [&](size_t i, const uint32_t* w) { memcpy(pmk[i].data(), w, 32); });
}

void pmk_bytes_out(const uint32_t w[8], uint8_t out[32]) {
    for (int k = 0; k < 8; k++) {
        out[4 * k] = (uint8_t)(w[k] >> 24);
        out[4 * k + 1] = (uint8_t)(w[k] >> 16);
        out[4 * k + 2] = (uint8_t)(w[k] >> 8);
        out[4 * k + 3] = (uint8_t)w[k];
    }
}

}  // namespace

HostCost host_cost(const dwpa_job* jobs, size_t njobs) {
    HostCost c;
    for (size_t j = 0; j < njobs; j++) {
        const dwpa_job& J = jobs[j];
        // the type field decides the verify work; a malformed line costs nothing (it fails the parse)
        const bool eapol = J.line && J.line_len > 6 && memcmp(J.line, "WPA*02*", 7) == 0;
        const int64_t nc = std::min<int64_t>(J.nc, DWPA_NC_MAX);
        const double att = eapol ? (double)(1 + 4 * std::max<int64_t>(0, (nc >> 1) + 1)) : 1.0;
        const double verify = eapol ? att * 9.0 : 4.0;  // compressions per key (PRF + MIC per attempt; PMKID)
        uint64_t nn = 0;
        for (size_t k = 0; k < J.nkeys; k++)
            if (J.keys[k].ptr) nn++;
        c.keys += nn;
        c.derives += nn - (nn && J.pmk ? 1 : 0);
        c.pmk_equiv += (double)nn * verify / 16388.0;
    }
    c.pmk_equiv += (double)c.derives;
    return c;
}

int host_check_batch(const dwpa_job* jobs, size_t njobs, dwpa_result* out, int* rcs, dwpa_check_stats& stats) {
    std::vector<ParsedLine> parsed(njobs);
    std::vector<uint32_t> nnz(njobs, 0);
    // parse (PHP acceptance rules) and count the non-null keys of every line that can match; the same per-job
    // validation as the device path (engine.cpp check_batch_body)
    const size_t TP = host_threads_for(njobs, 64);
    host_parallel(TP, [&](size_t t) {
        const size_t T = TP;
        for (size_t j = njobs * t / T; j < njobs * (t + 1) / T; j++) {
            out[j].key_index = -1;
            out[j].nc = 0;
            out[j].endian = 0;
            out[j].nc_valid = 0;
            memset(out[j].pmk, 0, 32);
            ParsedLine& pl = parsed[j];
            parse_m22000_into(jobs[j].line, jobs[j].line_len, pl);
            rcs[j] = pl.status;
            if (pl.status) continue;
            rcs[j] = DWPA_MISS;
            if (!line_can_match(pl)) continue;
            if ((pl.kind == LINE_EAPOL && jobs[j].nc > DWPA_NC_MAX) || jobs[j].nkeys > UINT32_MAX) {
                rcs[j] = DWPA_E_ARG;
                continue;
            }
            uint32_t c = 0;
            for (size_t k = 0; k < jobs[j].nkeys; k++)
                if (jobs[j].keys[k].ptr) c++;
            nnz[j] = c;
        }
    });

    // ESSID groups (first-seen order) with their salt blocks; the line tables (raw blocks, PHP nonce order)
    std::unordered_map<std::string_view, uint32_t> essid_id;
    std::vector<uint32_t> gid(njobs, 0), job_line(njobs, 0), jslot(njobs, 0);
    std::vector<std::vector<uint32_t>> salt;
    std::vector<uint32_t> nblk;
    TableBuilder tb;
    tb.raw = true;
    size_t nslots = 0;
    for (size_t j = 0; j < njobs; j++) {
        if (!nnz[j]) continue;
        auto ins = essid_id.try_emplace(std::string_view(parsed[j].essid), (uint32_t)salt.size());
        if (ins.second) {
            salt.emplace_back();
            nblk.push_back(build_salt_blocks(parsed[j].essid, salt.back()));
        }
        gid[j] = ins.first->second;
        job_line[j] = tb.add_line(parsed[j], jobs[j].nc, DWPA_NC_PHP, 0);
        jslot[j] = (uint32_t)nslots;
        nslots += nnz[j];
    }
    stats.slots = (uint32_t)std::min<size_t>(nslots, UINT32_MAX);
    if (!nslots) return 0;

    // slots: the job's non-null keys in order ($HEX[] decoded); unique (ESSID, key) pairs derived once
    std::vector<uint32_t> sjob(nslots), sord(nslots), skidx(nslots), suid(nslots);
    std::vector<std::string> dec;  // decoded $HEX[] keys (stable storage for the views below)
    size_t ndec = 0;
    for (size_t j = 0; j < njobs; j++)
        if (nnz[j])
            for (size_t k = 0; k < jobs[j].nkeys; k++)
                if (jobs[j].keys[k].ptr && starts_hex(jobs[j].keys[k].ptr, jobs[j].keys[k].len)) ndec++;
    dec.reserve(ndec);
    std::vector<std::unordered_map<std::string_view, uint32_t>> uniq(salt.size());
    std::vector<Derive> dv;
    for (size_t j = 0; j < njobs; j++) {
        if (!nnz[j]) continue;
        size_t s = jslot[j];
        uint32_t o = 0;
        for (size_t k = 0; k < jobs[j].nkeys; k++) {
            const dwpa_bytes& kb = jobs[j].keys[k];
            if (!kb.ptr) continue;  // is_null($key): skipped (common.php:172,240)
            sjob[s] = (uint32_t)j;
            sord[s] = o;
            skidx[s] = (uint32_t)k;
            if (o == 0 && jobs[j].pmk) {
                suid[s] = NO_UID;  // the caller's $pmk (common.php:178,246)
            } else {
                std::string_view key((const char*)kb.ptr, kb.len);
                if (starts_hex(kb.ptr, kb.len)) {
                    dec.push_back(hc_unhex(std::string(key)));
                    key = dec.back();
                }
                auto ins = uniq[gid[j]].try_emplace(key, (uint32_t)dv.size());
                if (ins.second) dv.push_back(Derive{(const uint8_t*)key.data(), key.size(), gid[j]});
                suid[s] = ins.first->second;
            }
            s++;
            o++;
        }
    }
    stats.pmks = (uint32_t)dv.size();
    std::vector<std::array<uint32_t, 8>> pmk;
    derive_all(dv, salt, nblk, pmk);

    // verify every slot; a job's slots beyond its first hit (in key order) are skipped once the hit is known
    std::vector<std::atomic<uint32_t>> best(njobs);
    for (auto& b : best) b.store(UINT32_MAX, std::memory_order_relaxed);
    std::vector<int32_t> satt(nslots, -1);
    std::vector<std::array<uint32_t, 8>> caller(njobs);
    for (size_t j = 0; j < njobs; j++)
        if (nnz[j] && jobs[j].pmk)
            for (int k = 0; k < 8; k++)
                caller[j][k] = (uint32_t)jobs[j].pmk[4 * k] << 24 | (uint32_t)jobs[j].pmk[4 * k + 1] << 16 |
                               (uint32_t)jobs[j].pmk[4 * k + 2] << 8 | jobs[j].pmk[4 * k + 3];
    const size_t chunk = 16, nchunks = (nslots + chunk - 1) / chunk;
    std::atomic<size_t> next{0};
    host_parallel(host_threads_for(nchunks, 1), [&](size_t) {
        for (size_t c; (c = next.fetch_add(1, std::memory_order_relaxed)) < nchunks;)
            for (size_t s = c * chunk; s < std::min(nslots, (c + 1) * chunk); s++) {
                const uint32_t j = sjob[s];
                if (sord[s] > best[j].load(std::memory_order_relaxed)) continue;
                const uint32_t* pw = suid[s] == NO_UID ? caller[j].data() : pmk[suid[s]].data();
                const int64_t a = verify_pmk(tb, job_line[j], sord[s], pw);
                if (a < 0) continue;
                satt[s] = (int32_t)a;
                uint32_t cur = best[j].load(std::memory_order_relaxed);
                while (sord[s] < cur && !best[j].compare_exchange_weak(cur, sord[s], std::memory_order_relaxed)) {
                }
            }
    });

    // first key in input order wins, then the first attempt in PHP order (common.php:186,280-289)
    for (size_t j = 0; j < njobs; j++) {
        const uint32_t o = best[j].load(std::memory_order_relaxed);
        if (o == UINT32_MAX) continue;
        const size_t s = jslot[j] + o;
        const LineDev& L = tb.lines[job_line[j]];
        rcs[j] = DWPA_HIT;
        stats.hits++;
        out[j].key_index = (int32_t)skidx[s];
        pmk_bytes_out(suid[s] == NO_UID ? caller[j].data() : pmk[suid[s]].data(), out[j].pmk);
        if (L.kind == LINE_PMKID) {
            out[j].nc_valid = 0;
        } else {
            const uint32_t list = std::min(o, L.nlists - 1);
            const AttDev& at = tb.atts[L.list_off + (size_t)list * L.natt + (size_t)satt[s]];
            out[j].nc_valid = 1;
            out[j].nc = at.nc;
            out[j].endian = (int8_t)at.endian;
        }
    }
    return 0;
}

void host_derive_soa(size_t n, const uint8_t* const* key, const uint32_t* len, const uint32_t* const* salt,
                     const uint32_t* nblk, uint32_t* pmk, size_t stride) {
    derive_each(
        n,
        [&](size_t i, const uint8_t*& k, size_t& l, const uint32_t*& sp, uint32_t& nb) {
            k = key[i];
            l = len[i];
            sp = salt[i];
            nb = nblk[i];
        },
        [&](size_t i, const uint32_t* w) {
            for (int k = 0; k < 8; k++) pmk[(size_t)k * stride + i] = w[k];
        });
}

double host_pmks_in(double seconds, size_t threads) {
    const Pbkdf2Costs& c = pbkdf2_costs();
    double rate = c.ni1 > 0 ? 1.0 / c.ni1 : 0.0;  // keys per second per thread on the best path
    if (c.ni > 0) rate = std::max(rate, 2.0 / c.ni);
    if (c.avx1 > 0) rate = std::max(rate, 8.0 / c.avx1);
    if (c.avx2 > 0) rate = std::max(rate, 16.0 / c.avx2);
    return rate * seconds * (double)threads;
}

int host_pbkdf2(const dwpa_bytes* keys, size_t nkeys, const uint8_t* essid, size_t essid_len, uint8_t* out) {
    std::vector<std::vector<uint32_t>> salt(1);
    std::vector<uint32_t> nblk{build_salt_blocks(std::string((const char*)essid, essid_len), salt[0])};
    std::vector<Derive> dv(nkeys);
    for (size_t i = 0; i < nkeys; i++)  // a null key derives as the empty key (as the device path)
        dv[i] = Derive{keys[i].ptr, keys[i].ptr ? keys[i].len : 0, 0};
    std::vector<std::array<uint32_t, 8>> pmk;
    derive_all(dv, salt, nblk, pmk);
    for (size_t i = 0; i < nkeys; i++) pmk_bytes_out(pmk[i].data(), out + 32 * i);
    return 0;
}

}  // namespace dwpa
