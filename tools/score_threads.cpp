// score() latency under concurrent C++ callers at C1 (1k synthetic rows, threshold 0, limit 100),
// with the server kernel (started by score() itself on a small library) and without it
// (ngsServe(h, 0)): tools/score_threads_probe.py without Python's interpreter lock between calls.
// T threads each make N score() calls; prints per-call p50 / p90 and all threads' calls per second.
// build + run (repo root): g++ -O2 -std=c++17 tools/score_threads.cpp -Iinclude
//   -Lstringsearchlib_amd/lib -lngram_search -lngs_synth -lpthread -Wl,-rpath,$PWD/stringsearchlib_amd/lib
//   -o /tmp/score_threads && /tmp/score_threads [calls per thread]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "ngram_search.h"

extern "C" int ngs_synth_corpus(uint64_t rows, uint64_t seed, uint32_t min_len, uint32_t span, uint32_t row_size,
                                char** blob_out, char*** words_out, float** weights_out, uint64_t* state_out);
extern "C" int ngs_synth_queries(char* const* words, uint64_t nwords, uint32_t row_size, uint64_t nq,
                                 uint64_t* state, uint32_t qlen, char** blob_out, uint64_t** off_out);

static void run(uint32_t h, const std::vector<std::string>& qs, int threads, int calls, const char* mode) {
    std::vector<std::vector<double>> lat(threads);
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    auto worker = [&](int i) {
        lat[i].reserve(calls);
        ready.fetch_add(1);
        while (!go.load()) std::this_thread::yield();
        for (int k = 0; k < calls; ++k) {
            const std::string& q = qs[(size_t)(i * calls + k) % qs.size()];
            char** res = nullptr;
            float* sc = nullptr;
            const auto t = std::chrono::steady_clock::now();
            score(h, q.c_str(), &res, &sc, 0.0f, 100);
            lat[i].push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count());
            release(h, res, sc);
        }
    };
    std::vector<std::thread> th;
    for (int i = 0; i < threads; ++i) th.emplace_back(worker, i);
    while (ready.load() < threads) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    go.store(true);
    for (auto& t : th) t.join();
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<double> all;
    for (auto& l : lat) all.insert(all.end(), l.begin(), l.end());
    std::sort(all.begin(), all.end());
    std::printf("%-9s threads %d: p50 %7.1f us  p90 %7.1f us  %9.0f calls/s\n", mode, threads, all[all.size() / 2],
                all[all.size() * 9 / 10], threads * calls / el);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    const int calls = argc > 1 ? std::atoi(argv[1]) : 2000;
    char* blob = nullptr;
    char** words = nullptr;
    float* weights = nullptr;
    uint64_t state = 0;
    if (ngs_synth_corpus(1000, 42, 8, 17, 1, &blob, &words, &weights, &state)) return 1;
    const uint32_t h = indexN(words, 1000, 1, nullptr);
    if (!h) return 1;
    char* qb = nullptr;
    uint64_t* qo = nullptr;
    if (ngs_synth_queries(words, 1000, 1, 4096, &state, 12, &qb, &qo)) return 1;
    std::vector<std::string> qs;
    for (int i = 0; i < 4096; ++i) qs.emplace_back(qb + qo[i], qb + qo[i + 1]);
    for (const char* mode : {"server", "no server"}) {
        if (std::string(mode) == "no server") ngsServe(h, 0);
        for (int threads : {1, 2, 4, 8, 16}) {
            run(h, qs, threads, 50, mode);  // warm
            run(h, qs, threads, calls, mode);
        }
    }
    dispose(h);
    return 0;
}
