/*
 * m22000_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity oracle; never shipped, never on the product path).
 *
 * A literal CPU restatement of dwpa's PHP key check, /root/reference/web/common.php:
 *   hc_unhex()          common.php:3-25
 *   valid_hex()         common.php:28-36
 *   omac1_aes_128*()    common.php:56-112   (RFC 4493 CMAC built on AES-128-ECB)
 *   check_key_m22000()  common.php:157-307
 *   hash_m22000()       common.php:310-315
 * on top of OpenSSL libcrypto -- the same library PHP's openssl_pbkdf2()/openssl_encrypt() wrap
 * (PKCS5_PBKDF2_HMAC with EVP_sha1, HMAC over MD5/SHA1/SHA256, AES-128-ECB).
 *
 * PHP semantics are emulated on purpose, quirks included:
 *   - explode('*', $line, 9): the 9th field keeps any further '*' (common.php:159)
 *   - `$ahl[1] == '01'` is PHP-8 loose equality: numeric strings compare as numbers (common.php:167,190)
 *   - strncmp() is PHP's binary-safe zend_binary_strncmp (length difference decides on a common prefix)
 *   - unpack() failures on short EAPOL/ANONCE yield null -> keyver 0 / corr 0 (common.php:215-235)
 *   - $n is mutated in place by substr_replace() across attempts AND keys (common.php:255-259),
 *     including PHP's offset clamping when the nonce is shorter than expected
 *   - $pmk is used for the first non-null key only, then reset (common.php:178,188,246,302)
 *   - Null keys are skipped before the PMK logic (common.php:172,240)
 *
 * Parity pinning: see tests/test_oracle.py (challenge KAT help_crack.py:692-699, IEEE 802.11i H.4,
 * RFC 6070, RFC 4493) and tests/golden/.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <ctype.h>
#include <pthread.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>

#include "m22000_oracle.h"

/* ---------- small PHP helpers ---------- */

typedef struct { uint8_t *p; size_t n, cap; } buf_t;

static void buf_init(buf_t *b) { b->p = NULL; b->n = 0; b->cap = 0; }
static void buf_free(buf_t *b) { free(b->p); buf_init(b); }
static void buf_reserve(buf_t *b, size_t n) {
    if (n <= b->cap) return;
    size_t c = b->cap ? b->cap : 64;
    while (c < n) c *= 2;
    b->p = (uint8_t *)realloc(b->p, c);
    b->cap = c;
}
static void buf_set(buf_t *b, const uint8_t *p, size_t n) { buf_reserve(b, n + 1); if (n) memcpy(b->p, p, n); b->n = n; }
static void buf_cat(buf_t *b, const uint8_t *p, size_t n) { buf_reserve(b, b->n + n + 1); if (n) memcpy(b->p + b->n, p, n); b->n += n; }

/* PHP 8 substr_replace($s, $r, $off, $len) for non-negative off/len (clamping as in ext/standard/string.c) */
static void php_substr_replace(buf_t *s, const uint8_t *r, size_t rn, size_t off, size_t len) {
    if (off > s->n) off = s->n;
    if (off + len > s->n) len = s->n - off;
    size_t tail = s->n - off - len;
    buf_t out; buf_init(&out);
    buf_reserve(&out, off + rn + tail + 1);
    memcpy(out.p, s->p, off);
    memcpy(out.p + off, r, rn);
    memcpy(out.p + off + rn, s->p + off + len, tail);
    out.n = off + rn + tail;
    buf_free(s);
    *s = out;
}

/* zend_binary_strncmp */
static int php_strncmp(const uint8_t *a, size_t la, const uint8_t *b, size_t lb, size_t length) {
    size_t m = length;
    if (la < m) m = la;
    if (lb < m) m = lb;
    int r = memcmp(a, b, m);
    if (r) return r;
    size_t ma = la < length ? la : length;
    size_t mb = lb < length ? lb : length;
    return (ma > mb) - (ma < mb);
}

static int is_xdigit_c(uint8_t c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
static int hexval(uint8_t c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; }

/* common.php:28-36 -- even length and ctype_xdigit (which is false for "") */
int oracle_valid_hex(const uint8_t *s, size_t n) {
    if (n & 1) return 0;
    if (n == 0) return 0;
    for (size_t i = 0; i < n; i++) if (!is_xdigit_c(s[i])) return 0;
    return 1;
}

static void hex2bin(const uint8_t *s, size_t n, buf_t *out) {
    buf_reserve(out, n / 2 + 1);
    for (size_t i = 0; i < n / 2; i++) out->p[i] = (uint8_t)(hexval(s[2 * i]) << 4 | hexval(s[2 * i + 1]));
    out->n = n / 2;
}

/* common.php:3-25.  Writes the decoded key into out (may alias nothing). */
static void hc_unhex(const uint8_t *k, size_t n, buf_t *out) {
    if (n <= 6) { buf_set(out, k, n); return; }
    const uint8_t *in = k + 5;
    size_t in_n = n - 6;                    /* substr($key, 5, -1) */
    int starts = memcmp(k, "$HEX[", 5) == 0;
    int ends = k[n - 1] == ']';
    int xd = in_n > 0;
    for (size_t i = 0; i < in_n && xd; i++) if (!is_xdigit_c(in[i])) xd = 0;
    if (!(in_n & 1) && starts && ends && xd) { hex2bin(in, in_n, out); return; }
    /* common.php:17-22 (unreachable: n > 6 implies in_n >= 1) */
    buf_set(out, k, n);
}

int oracle_hc_unhex(const uint8_t *k, size_t n, uint8_t *out, size_t *out_n) {
    buf_t b; buf_init(&b);
    hc_unhex(k, n, &b);
    memcpy(out, b.p, b.n);
    *out_n = b.n;
    buf_free(&b);
    return 0;
}

/* PHP 8 numeric-string test + value (Zend/zend_operators.c _is_numeric_string_ex, allow_errors = false):
 * [ws]* [+-]? (digits [. digits*]? | . digits) ([eE][+-]?digits)? [ws]*    ws = " \t\n\r\v\f" */
static int php_numeric(const uint8_t *s, size_t n, double *val) {
    size_t i = 0;
    while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r' || s[i] == '\v' || s[i] == '\f')) i++;
    size_t st = i;
    if (i < n && (s[i] == '+' || s[i] == '-')) i++;
    size_t d0 = i;
    while (i < n && s[i] >= '0' && s[i] <= '9') i++;
    size_t nd = i - d0, nf = 0;
    if (i < n && s[i] == '.') {
        i++;
        size_t f0 = i;
        while (i < n && s[i] >= '0' && s[i] <= '9') i++;
        nf = i - f0;
    }
    if (nd == 0 && nf == 0) return 0;
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        size_t save = i;
        i++;
        if (i < n && (s[i] == '+' || s[i] == '-')) i++;
        size_t e0 = i;
        while (i < n && s[i] >= '0' && s[i] <= '9') i++;
        if (i == e0) i = save; /* not an exponent: then the 'e' is trailing garbage */
    }
    size_t en = i;
    while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r' || s[i] == '\v' || s[i] == '\f')) i++;
    if (i != n) return 0;
    char tmp[512];
    size_t L = en - st;
    if (L >= sizeof(tmp)) { *val = 0; return 1; } /* absurdly long: value irrelevant for ==1/==2 (never equal) */
    memcpy(tmp, s + st, L);
    tmp[L] = 0;
    *val = strtod(tmp, NULL);
    return 1;
}

/* `$field == '0N'` (PHP 8 loose string==string) */
static int php_eq_type(const uint8_t *s, size_t n, int target) {
    double v;
    if (php_numeric(s, n, &v)) return v == (double)target;
    char t[3] = {'0', (char)('0' + target), 0};
    return n == 2 && memcmp(s, t, 2) == 0;
}

/* ---------- crypto primitives (OpenSSL) ---------- */

void oracle_pbkdf2_sha1(const uint8_t *key, size_t klen, const uint8_t *salt, size_t slen, int iter, uint8_t *out, size_t olen) {
    static const char empty = 0;
    PKCS5_PBKDF2_HMAC(klen ? (const char *)key : &empty, (int)klen, slen ? salt : (const uint8_t *)&empty, (int)slen,
                      iter, EVP_sha1(), (int)olen, out);
}

static void hmac(const EVP_MD *md, const uint8_t *key, size_t kl, const uint8_t *msg, size_t ml, uint8_t *out) {
    unsigned int ol = 0;
    static const uint8_t z = 0;
    HMAC(md, kl ? key : &z, (int)kl, ml ? msg : &z, ml, out, &ol);
}

static void aes128_ecb_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int ol = 0;
    EVP_EncryptInit_ex(c, EVP_aes_128_ecb(), NULL, key, NULL);
    EVP_CIPHER_CTX_set_padding(c, 0);
    EVP_EncryptUpdate(c, out, &ol, in, 16);
    EVP_CIPHER_CTX_free(c);
}

/* common.php:56-68 */
static void omac_leftshift1(const uint8_t in[16], uint8_t out[16]) {
    uint8_t state = 0;
    for (int i = 15; i >= 0; i--) {
        uint8_t t = in[i];
        out[i] = (uint8_t)((t << 1) | state);
        state = (uint8_t)((t & 0x80) >> 7);
    }
}

/* common.php:72-112 */
void oracle_omac1_aes_128(const uint8_t *data, size_t n, const uint8_t key[16], uint8_t out[16]) {
    static const uint8_t zero[16] = {0};
    uint8_t L[16], K1[16], K2[16], c[16], blk[16];
    aes128_ecb_block(key, zero, L);
    omac_leftshift1(L, K1);
    if (L[0] > 127) K1[15] ^= 0x87;
    omac_leftshift1(K1, K2);
    if (K1[0] > 127) K2[15] ^= 0x87;
    /* str_split($data, 16): PHP >= 8.2 returns [] for "", older [""]; data is never empty on this path
     * (EAPOL >= 49 bytes), the [""] form is used here so the function is total. */
    size_t nb = n ? (n + 15) / 16 : 1;
    memset(c, 0, 16);
    for (size_t b = 0; b < nb; b++) {
        size_t off = b * 16, len = n - off < 16 ? n - off : 16;
        if (n == 0) len = 0;
        memset(blk, 0, 16);
        if (len) memcpy(blk, data + off, len);
        if (b == nb - 1) {
            if (len != 16) {
                blk[len] = 0x80;
                for (int i = 0; i < 16; i++) blk[i] ^= K2[i];
            } else {
                for (int i = 0; i < 16; i++) blk[i] ^= K1[i];
            }
        }
        for (int i = 0; i < 16; i++) blk[i] ^= c[i];
        aes128_ecb_block(key, blk, c);
    }
    memcpy(out, c, 16);
}

/* ---------- check_key_m22000 (common.php:157-307) ---------- */

typedef struct { const uint8_t *p; size_t n; } fld_t;

static int explode9(const uint8_t *s, size_t n, fld_t f[9]) {
    size_t cnt = 0, st = 0;
    for (size_t i = 0; i < n && cnt < 8; i++) {
        if (s[i] == '*') { f[cnt].p = s + st; f[cnt].n = i - st; cnt++; st = i + 1; }
    }
    f[cnt].p = s + st; f[cnt].n = n - st; cnt++;
    return (int)cnt;
}

static int hexfield(const fld_t *f, buf_t *out) {
    if (!oracle_valid_hex(f->p, f->n)) return 0;
    hex2bin(f->p, f->n, out);
    return 1;
}

static void put_u32(uint8_t *d, uint32_t v, int big) {
    if (big) { d[0] = v >> 24; d[1] = v >> 16; d[2] = v >> 8; d[3] = v; }
    else { d[0] = v; d[1] = v >> 8; d[2] = v >> 16; d[3] = v >> 24; }
}

/* The returned key (after hc_unhex): key_len is its full length, the buffer holds at most sizeof(out->key) bytes of
 * it (hash_pbkdf2 takes keys of any length; a caller reads a longer one from keys[key_index]). */
static void result_key(oracle_result *out, const buf_t *key) {
    memcpy(out->key, key->p, key->n < sizeof out->key ? key->n : sizeof out->key);
    out->key_len = key->n;
}

int oracle_check_m22000(const char *line, size_t len, const oracle_key *keys, size_t nkeys,
                        const uint8_t *pmk_in, int nc, oracle_result *out) {
    const uint8_t *s = (const uint8_t *)line;
    fld_t f[9];
    int rc = 0;
    memset(out, 0, sizeof(*out));
    out->key_index = -1;
    if (explode9(s, len, f) != 9) return 0;
    if (!(f[0].n == 3 && memcmp(f[0].p, "WPA", 3) == 0)) return 0;

    buf_t mac_ap, mac_sta, essid, key, pmkid, keymic, nonce_ap, eapol, mp, m, n, msg;
    buf_init(&mac_ap); buf_init(&mac_sta); buf_init(&essid); buf_init(&key); buf_init(&pmkid);
    buf_init(&keymic); buf_init(&nonce_ap); buf_init(&eapol); buf_init(&mp); buf_init(&m); buf_init(&n); buf_init(&msg);

    uint8_t pmk[32];
    int have_pmk = pmk_in != NULL;
    if (have_pmk) memcpy(pmk, pmk_in, 32);

    if (!hexfield(&f[3], &mac_ap) || !hexfield(&f[4], &mac_sta) || !hexfield(&f[5], &essid)) goto done;

    if (php_eq_type(f[1].p, f[1].n, 1)) {
        if (!hexfield(&f[2], &pmkid)) goto done;
        buf_set(&msg, (const uint8_t *)"PMK Name", 8);
        buf_cat(&msg, mac_ap.p, mac_ap.n);
        buf_cat(&msg, mac_sta.p, mac_sta.n);
        for (size_t i = 0; i < nkeys; i++) {
            if (keys[i].p == NULL) continue; /* is_null($key) */
            if (keys[i].n >= 5 && memcmp(keys[i].p, "$HEX[", 5) == 0) hc_unhex(keys[i].p, keys[i].n, &key);
            else buf_set(&key, keys[i].p, keys[i].n);
            if (!have_pmk) oracle_pbkdf2_sha1(key.p, key.n, essid.p, essid.n, 4096, pmk, 32);
            uint8_t test[20];
            hmac(EVP_sha1(), pmk, 32, msg.p, msg.n, test);
            if (php_strncmp(test, 20, pmkid.p, pmkid.n, 16) == 0) {
                out->key_index = (int32_t)i;
                out->nc_is_null = 1;
                out->endian = 0;
                memcpy(out->pmk, pmk, 32);
                result_key(out, &key);
                rc = 1;
                goto done;
            }
            have_pmk = 0;
        }
    } else if (php_eq_type(f[1].p, f[1].n, 2)) {
        if (!hexfield(&f[2], &keymic) || !hexfield(&f[6], &nonce_ap) || !hexfield(&f[7], &eapol) || !hexfield(&f[8], &mp))
            goto done;
        /* unpack('x5/nkey_information/x10/a32nonce_sta', $eapol): needs 49 bytes, else false -> null */
        int keyver = 0;
        uint8_t nonce_sta_buf[32];
        const uint8_t *nonce_sta = nonce_sta_buf;
        size_t nonce_sta_n = 0;
        if (eapol.n >= 49) {
            keyver = ((eapol.p[5] << 8) | eapol.p[6]) & 3;
            memcpy(nonce_sta_buf, eapol.p + 17, 32);
            nonce_sta_n = 32;
        }
        if (php_strncmp(mac_ap.p, mac_ap.n, mac_sta.p, mac_sta.n, 6) < 0) {
            buf_set(&m, mac_ap.p, mac_ap.n); buf_cat(&m, mac_sta.p, mac_sta.n);
        } else {
            buf_set(&m, mac_sta.p, mac_sta.n); buf_cat(&m, mac_ap.p, mac_ap.n);
        }
        int swap = 0;
        if (php_strncmp(nonce_sta, nonce_sta_n, nonce_ap.p, nonce_ap.n, 6) < 0) {
            buf_set(&n, nonce_sta, nonce_sta_n); buf_cat(&n, nonce_ap.p, nonce_ap.n);
        } else {
            buf_set(&n, nonce_ap.p, nonce_ap.n); buf_cat(&n, nonce_sta, nonce_sta_n);
            swap = 1;
        }
        /* unpack('x28/V'|'x28/N', $nonce_ap)[1]: null (-> 0) unless 32 bytes are there */
        int64_t corrV = 0, corrN = 0;
        if (nonce_ap.n >= 32) {
            const uint8_t *q = nonce_ap.p + 28;
            corrV = (int64_t)((uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24);
            corrN = (int64_t)((uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | (uint32_t)q[3]);
        }
        int64_t halfnc = ((int64_t)nc >> 1) + 1;

        for (size_t i = 0; i < nkeys; i++) {
            if (keys[i].p == NULL) continue;
            if (keys[i].n >= 5 && memcmp(keys[i].p, "$HEX[", 5) == 0) hc_unhex(keys[i].p, keys[i].n, &key);
            else buf_set(&key, keys[i].p, keys[i].n);
            if (!have_pmk) oracle_pbkdf2_sha1(key.p, key.n, essid.p, essid.n, 4096, pmk, 32);

            /* $ncarr as (endian, offset) pairs; 'N' = big endian, 'V' = little endian */
            int nj = 1;
            int jbig[4] = {1, 0, 0, 0};
            int64_t joff[4] = {0, 0, 0, 0};
            do {
                for (int jj = 0; jj < nj; jj++) {
                    uint8_t raw[4];
                    int64_t v = (jbig[jj] ? corrN : corrV) + joff[jj];
                    put_u32(raw, (uint32_t)(uint64_t)v, jbig[jj]);
                    php_substr_replace(&n, raw, 4, swap ? 28 : 60, 4);

                    uint8_t ptk[32], test[32];
                    switch (keyver) {
                    case 1:
                    case 2:
                        buf_set(&msg, (const uint8_t *)"Pairwise key expansion\0", 23);
                        buf_cat(&msg, m.p, m.n); buf_cat(&msg, n.p, n.n); buf_cat(&msg, (const uint8_t *)"\0", 1);
                        hmac(EVP_sha1(), pmk, 32, msg.p, msg.n, ptk);
                        if (keyver == 1) hmac(EVP_md5(), ptk, 16, eapol.p, eapol.n, test);
                        else hmac(EVP_sha1(), ptk, 16, eapol.p, eapol.n, test);
                        break;
                    case 3:
                        buf_set(&msg, (const uint8_t *)"\1\0Pairwise key expansion", 24);
                        buf_cat(&msg, m.p, m.n); buf_cat(&msg, n.p, n.n); buf_cat(&msg, (const uint8_t *)"\x80\1", 2);
                        hmac(EVP_sha256(), pmk, 32, msg.p, msg.n, ptk);
                        oracle_omac1_aes_128(eapol.p, eapol.n, ptk, test);
                        break;
                    default:
                        goto done; /* unknown keyver: return False */
                    }
                    if (php_strncmp(test, keyver == 2 ? 20 : 16, keymic.p, keymic.n, 16) == 0) {
                        out->key_index = (int32_t)i;
                        memcpy(out->pmk, pmk, 32);
                        result_key(out, &key);
                        out->nc_is_null = 0;
                        if (joff[0] == 0) { out->nc = 0; out->endian = 0; }
                        else { out->nc = (int32_t)joff[jj]; out->endian = jbig[jj] ? 1 : 2; }
                        rc = 1;
                        goto done;
                    }
                }
                if (joff[0] == 0) {
                    nj = 4;
                    jbig[0] = 0; joff[0] = 1;
                    jbig[1] = 0; joff[1] = -1;
                    jbig[2] = 1; joff[2] = 1;
                    jbig[3] = 1; joff[3] = -1;
                } else {
                    joff[0]++; joff[1]--; joff[2]++; joff[3]--;
                }
            } while (joff[0] <= halfnc);
            have_pmk = 0;
        }
    }
done:
    buf_free(&mac_ap); buf_free(&mac_sta); buf_free(&essid); buf_free(&key); buf_free(&pmkid); buf_free(&keymic);
    buf_free(&nonce_ap); buf_free(&eapol); buf_free(&mp); buf_free(&m); buf_free(&n); buf_free(&msg);
    return rc;
}

/* common.php:310-315: md5($ahl[1].$ahl[2]...$ahl[7]) raw; returns 0 if the line has != 9 fields */
int oracle_hash_m22000(const char *line, size_t len, uint8_t out[16]) {
    fld_t f[9];
    if (explode9((const uint8_t *)line, len, f) != 9) return 0;
    EVP_MD_CTX *c = EVP_MD_CTX_new();
    unsigned int ol = 0;
    EVP_DigestInit_ex(c, EVP_md5(), NULL);
    for (int i = 1; i <= 7; i++) EVP_DigestUpdate(c, f[i].p, f[i].n);
    EVP_DigestFinal_ex(c, out, &ol);
    EVP_MD_CTX_free(c);
    return 1;
}

/* ---------- multi-threaded drivers (CPU baseline timing) ---------- */

typedef struct {
    const char *line; size_t len;
    const oracle_key *keys; size_t nkeys;
    int nc;
    size_t begin, end;
    int64_t first_hit;
    oracle_result res;
} job_t;

static void *check_worker(void *arg) {
    job_t *j = (job_t *)arg;
    j->first_hit = -1;
    for (size_t i = j->begin; i < j->end; i++) {
        oracle_result r;
        if (oracle_check_m22000(j->line, j->len, &j->keys[i], 1, NULL, j->nc, &r) == 1) {
            j->first_hit = (int64_t)i;
            j->res = r;
            j->res.key_index = (int32_t)i;
            break;
        }
    }
    return NULL;
}

/* Runs check_key_m22000(line, [key]) for every key (one PHP request per key, as put_work does,
 * common.php:902) on `threads` threads.  Returns the lowest matching key index or -1. */
int64_t oracle_check_many(const char *line, size_t len, const oracle_key *keys, size_t nkeys, int nc, int threads,
                          oracle_result *out) {
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
    size_t per = (nkeys + (size_t)threads - 1) / (size_t)threads;
    for (int t = 0; t < threads; t++) {
        jobs[t].line = line; jobs[t].len = len; jobs[t].keys = keys; jobs[t].nkeys = nkeys; jobs[t].nc = nc;
        jobs[t].begin = (size_t)t * per < nkeys ? (size_t)t * per : nkeys;
        jobs[t].end = jobs[t].begin + per < nkeys ? jobs[t].begin + per : nkeys;
        pthread_create(&th[t], NULL, check_worker, &jobs[t]);
    }
    int64_t best = -1;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].first_hit >= 0 && (best < 0 || jobs[t].first_hit < best)) {
            best = jobs[t].first_hit;
            if (out) *out = jobs[t].res;
        }
    }
    free(th);
    free(jobs);
    return best;
}

typedef struct { const oracle_key *keys; const uint8_t *salt; size_t slen; uint8_t *out; size_t b, e; } pjob_t;
static void *pbkdf2_worker(void *arg) {
    pjob_t *j = (pjob_t *)arg;
    for (size_t i = j->b; i < j->e; i++) oracle_pbkdf2_sha1(j->keys[i].p, j->keys[i].n, j->salt, j->slen, 4096, j->out + 32 * i, 32);
    return NULL;
}

void oracle_pbkdf2_many(const oracle_key *keys, size_t n, const uint8_t *salt, size_t slen, uint8_t *out, int threads) {
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    pjob_t *jobs = (pjob_t *)calloc((size_t)threads, sizeof(pjob_t));
    size_t per = (n + (size_t)threads - 1) / (size_t)threads;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (pjob_t){keys, salt, slen, out, (size_t)t * per < n ? (size_t)t * per : n, 0};
        jobs[t].e = jobs[t].b + per < n ? jobs[t].b + per : n;
        pthread_create(&th[t], NULL, pbkdf2_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
}

/* exposed for the fixture cross-checks */
void oracle_hmac(int alg, const uint8_t *key, size_t kl, const uint8_t *msg, size_t ml, uint8_t *out) {
    hmac(alg == 0 ? EVP_md5() : alg == 1 ? EVP_sha1() : EVP_sha256(), key, kl, msg, ml, out);
}
