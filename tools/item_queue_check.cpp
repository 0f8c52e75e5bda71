// item_queue_check -- the crack path's work distribution without a GPU: ChunkSource + ItemQueue (dict_reader.hpp)
// over dictionary files, `workers` threads pulling items the way dwpa_crack_files' shard workers do (each holds one
// item while "scanning" it for a time proportional to its size).  Prints one JSON object: per-worker words and
// items, when it ran out of work (ms after the start), and whether every word of the input was handed out exactly
// once.
// Used by tests/test_dict_reader.py.
//   item_queue_check <workers> <first> <most> <us_per_mword> file...
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dict_reader.hpp"

int main(int argc, char** argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: item_queue_check workers first most us_per_mword file...\n");
        return 2;
    }
    const size_t W = (size_t)atol(argv[1]), first = (size_t)atol(argv[2]), most = (size_t)atol(argv[3]);
    const double us_per_mword = atof(argv[4]);
    std::vector<std::string> paths(argv + 5, argv + argc);
    setenv("DWPA_DICT_CACHE_MB", "0", 1);
    dwpa::ChunkSource source(paths, first * W, 2 * most * W);
    dwpa::ItemQueue items(source, first, most, W);
    std::mutex mu;
    std::vector<std::string> seen;  // every word handed out
    std::vector<size_t> words(W, 0), nitems(W, 0), largest(W, 0);
    std::vector<double> done_ms(W, 0);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    std::atomic<bool> tool_oom{false};
    for (size_t w = 0; w < W; w++)
        th.emplace_back([&, w] {
          try {
            dwpa::WorkItem it;
            while (items.next(it)) {
                const size_t n = it.e - it.b;
                std::vector<std::string> mine;
                for (size_t i = it.b; i < it.e; i++)
                    mine.emplace_back(it.chunk->bytes.data() + it.chunk->off[i], it.chunk->off[i + 1] - it.chunk->off[i]);
                std::this_thread::sleep_for(std::chrono::microseconds((long)(us_per_mword * (double)n / 1e6)));
                std::lock_guard<std::mutex> lk(mu);
                seen.insert(seen.end(), mine.begin(), mine.end());
                words[w] += n;
                nitems[w]++;
                largest[w] = std::max(largest[w], n);
            }
            std::lock_guard<std::mutex> lk(mu);
            done_ms[w] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
          } catch (const std::bad_alloc&) {  // this tool's own copies of the words; the library's threads catch theirs
            tool_oom = true;
          }
        });
    for (auto& t : th) t.join();
    size_t total = seen.size();
    std::sort(seen.begin(), seen.end());
    const bool unique = std::adjacent_find(seen.begin(), seen.end()) == seen.end();
    printf("{\"words_total\": %zu, \"unique\": %s, \"io_error\": %s, \"tool_oom\": %s, \"workers\": [", total,
           unique ? "true" : "false", items.io_error() ? "true" : "false", tool_oom.load() ? "true" : "false");
    for (size_t w = 0; w < W; w++)
        printf("%s{\"words\": %zu, \"items\": %zu, \"largest\": %zu, \"done_ms\": %.2f}", w ? ", " : "", words[w],
               nitems[w], largest[w], done_ms[w]);
    printf("]}\n");
    return 0;
}
