// host_pbkdf2_paths -- one thread's time per call of each host PBKDF2 loop (host_crypto.cpp, included here so its
// static loops are visible): SHA-NI with 1, 2 and 4 chains in lock step, AVX-512 with 1, 2 and 3 registers of 16
// chains, the scalar loop.  Full 4,095-iteration chains, best of 5.  Prints one JSON object.
//   make tools/bin/host_pbkdf2_paths && tools/bin/host_pbkdf2_paths
#include "../dwpa_amd/csrc/host_crypto.cpp"

#include <chrono>
#include <cstdio>

using namespace dwpa::hostc;

template <class F>
static double best_of(F&& f) {
    double b = 1e30;
    for (int r = 0; r < 5; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        f();
        b = std::min(b, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    return b * 1e3;
}

int main() {
    static uint32_t mids[48][10], T[48][5];
    const uint32_t* cm[48];
    uint32_t* ct[48];
    for (int i = 0; i < 48; i++) {
        for (int k = 0; k < 10; k++) mids[i][k] = 0x9e3779b9u * (uint32_t)(10 * i + k + 1);
        cm[i] = mids[i];
        ct[i] = T[i];
    }
    const Caps& k = caps();
    printf("{\"sha_ni\": %d, \"avx512\": %d", k.sha_ni, k.avx512);
    if (k.sha_ni) {
        printf(", \"ni1_chain_ms\": %.4f", best_of([&] { pbkdf2_loop_ni<1>(cm, ct); }));
        printf(", \"ni2_chains_ms\": %.4f", best_of([&] { pbkdf2_loop_ni<2>(cm, ct); }));
        printf(", \"ni4_chains_ms\": %.4f", best_of([&] { pbkdf2_loop_ni<4>(cm, ct); }));
    }
    if (k.avx512) {
        printf(", \"avx16_chains_ms\": %.4f", best_of([&] { pbkdf2_loop_avx512<1>(cm, ct); }));
        printf(", \"avx32_chains_ms\": %.4f", best_of([&] { pbkdf2_loop_avx512<2>(cm, ct); }));
        printf(", \"avx48_chains_ms\": %.4f", best_of([&] { pbkdf2_loop_avx512<3>(cm, ct); }));
    }
    printf(", \"scalar_chain_ms\": %.4f}\n", best_of([&] { pbkdf2_loop_scalar(cm[0], ct[0]); }));
    return 0;
}
