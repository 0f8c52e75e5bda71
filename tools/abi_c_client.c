/* abi_c_client.c -- the C ABI as a plain C caller sees it (what PHP FFI binds from include/dwpa22000.h): compile
 * against the header alone, link libdwpa22000.so, and check the reference's challenge (help_crack.py:692-699, PSK
 * aaaa1234) on both lines with dwpa_check_m22000 and dwpa_check_batch, with the host backend allowed (so it runs with
 * or without a GPU).  Lines come on argv[1], argv[2].  Prints the backend of each call; exit 0 when both hit.
 *   gcc -std=c99 -Wall -Iinclude tools/abi_c_client.c -Ldwpa_amd/lib -ldwpa22000 -o abi_c_client (tests/test_abi.py) */
#include <stdio.h>
#include <string.h>

#include "dwpa22000.h"

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    if (dwpa_abi_version() != DWPA_ABI_VERSION) return 3;
    dwpa_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.struct_size = sizeof cfg;
    cfg.allow_cpu_fallback = 1;
    if (dwpa_init(&cfg) != 0) return 4;
    const char *psk = "aaaa1234", *wrong = "wrongpass";
    dwpa_bytes keys[2] = {{(const uint8_t *)wrong, strlen(wrong)}, {(const uint8_t *)psk, strlen(psk)}};
    dwpa_job jobs[2];
    for (int i = 0; i < 2; i++) {
        dwpa_result r;
        const int rc = dwpa_check_m22000(argv[1 + i], strlen(argv[1 + i]), keys, 2, NULL, 8, &r);
        dwpa_check_stats st;
        dwpa_check_last_stats(&st);
        printf("line %d: rc %d key_index %d nc_valid %u nc %d endian %d backend %u\n", i, rc, r.key_index,
               (unsigned)r.nc_valid, r.nc, (int)r.endian, st.backend);
        if (rc != DWPA_HIT || r.key_index != 1) return 5;
        jobs[i].line = argv[1 + i];
        jobs[i].line_len = strlen(argv[1 + i]);
        jobs[i].keys = keys;
        jobs[i].nkeys = 2;
        jobs[i].pmk = NULL;
        jobs[i].nc = 8;
    }
    dwpa_result out[2];
    int rcs[2];
    if (dwpa_check_batch(jobs, 2, out, rcs) != 0 || rcs[0] != DWPA_HIT || rcs[1] != DWPA_HIT) return 6;
    if (memcmp(out[0].pmk, out[1].pmk, 32) != 0) return 7; /* same ESSID and PSK: one PMK */
    printf("batch: both hit, one PMK\n");
    return 0;
}
