// pinned_write -- host write and read rates into pinned staging (hipHostMalloc with the check path's flags) against
// plain pageable memory, single-threaded and from 16 threads, on the GPU box's host.  The check path writes every
// key of a call into pinned memory (engine.cpp, "slots"), so this bounds what that phase can gain.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

static double run(uint8_t* dst, const uint8_t* src, size_t n, int threads, int reps, bool read) {
    double best = 1e30;
    for (int r = 0; r < reps; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++)
            th.emplace_back([=] {
                const size_t b = n * t / threads, e = n * (t + 1) / threads;
                if (read) {
                    volatile uint64_t acc = 0;
                    uint64_t a = 0;
                    for (size_t i = b; i + 8 <= e; i += 8) {
                        uint64_t v;
                        memcpy(&v, dst + i, 8);
                        a += v;
                    }
                    acc = a;
                    (void)acc;
                } else {
                    // scattered-size copies like the keys of a call: 8..40-byte pieces
                    size_t i = b, k = 0;
                    while (i < e) {
                        const size_t len = std::min<size_t>(8 + (k++ * 7) % 33, e - i);
                        memcpy(dst + i, src + i, len);
                        i += len;
                    }
                }
            });
        for (auto& x : th) x.join();
        best = std::min(best, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    return best;
}

int main() {
    const size_t n = 8u << 20;
    std::vector<uint8_t> src(n, 7), plain(n, 0);
    uint8_t *pin_def = nullptr, *pin_wc = nullptr;
    if (hipHostMalloc((void**)&pin_def, n, hipHostMallocDefault) != hipSuccess) return 1;
    if (hipHostMalloc((void**)&pin_wc, n, hipHostMallocWriteCombined) != hipSuccess) return 1;
    memset(pin_def, 0, n);
    memset(pin_wc, 0, n);
    printf("{\"bytes\": %zu, \"results\": [\n", n);
    const char* names[] = {"pageable", "hipHostMallocDefault", "hipHostMallocWriteCombined"};
    uint8_t* bufs[] = {plain.data(), pin_def, pin_wc};
    bool first = true;
    for (int b = 0; b < 3; b++)
        for (int threads : {1, 16})
            for (int rd = 0; rd < 2; rd++) {
                const double ms = run(bufs[b], src.data(), n, threads, 7, rd);
                printf("%s  {\"memory\": \"%s\", \"threads\": %d, \"op\": \"%s\", \"ms\": %.3f, \"GBps\": %.2f}",
                       first ? "" : ",\n", names[b], threads, rd ? "read" : "write pieces", ms, n / ms / 1e6);
                first = false;
            }
    printf("\n]}\n");
    return 0;
}
