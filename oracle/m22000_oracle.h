/* m22000_oracle.h -- TEST INFRASTRUCTURE ONLY: CPU restatement of web/common.php's key check (parity oracle). */
#ifndef M22000_ORACLE_H
#define M22000_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct { const uint8_t *p; size_t n; } oracle_key; /* p == NULL models a PHP null key */

typedef struct {
    int32_t key_index;   /* index of the returned key in the input array */
    int32_t nc;          /* signed nonce correction (meaningful when nc_is_null == 0) */
    int32_t nc_is_null;  /* 1: PHP Null (PMKID lines) */
    int32_t endian;      /* 0: Null, 1: 'BE', 2: 'LE' */
    uint8_t pmk[32];
    uint8_t key[4096];   /* the key as returned by PHP (after hc_unhex), its first 4096 bytes */
    size_t key_len;      /* its full length */
} oracle_result;

int oracle_valid_hex(const uint8_t *s, size_t n);
int oracle_hc_unhex(const uint8_t *k, size_t n, uint8_t *out, size_t *out_n);
void oracle_pbkdf2_sha1(const uint8_t *key, size_t klen, const uint8_t *salt, size_t slen, int iter, uint8_t *out, size_t olen);
void oracle_omac1_aes_128(const uint8_t *data, size_t n, const uint8_t key[16], uint8_t out[16]);
void oracle_hmac(int alg /*0 md5, 1 sha1, 2 sha256*/, const uint8_t *key, size_t kl, const uint8_t *msg, size_t ml, uint8_t *out);

/* check_key_m22000($line, $keys, $pmk ?: False, $nc): 1 = hit (out filled), 0 = PHP False */
int oracle_check_m22000(const char *line, size_t len, const oracle_key *keys, size_t nkeys,
                        const uint8_t *pmk /* NULL = False */, int nc, oracle_result *out);
int oracle_hash_m22000(const char *line, size_t len, uint8_t out[16]);

int64_t oracle_check_many(const char *line, size_t len, const oracle_key *keys, size_t nkeys, int nc, int threads,
                          oracle_result *out);
void oracle_pbkdf2_many(const oracle_key *keys, size_t n, const uint8_t *salt, size_t slen, uint8_t *out, int threads);

#ifdef __cplusplus
}
#endif
#endif
