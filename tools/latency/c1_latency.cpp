// score() latency through the C ABI alone (no Python / ctypes), on BASELINE configs[0]'s shape:
// a 1,000-row library of 8-24-character ASCII keys, one query per call (the reference's SearchTest
// harness times its CPU DLL the same way: 14.7 us per query).
// build: hipcc -O2 tools/latency/c1_latency.cpp -Iinclude -Lstringsearchlib_amd/lib -lngram_search -o c1_latency
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "ngram_search.h"

int main(int argc, char** argv) {
    const int rows = 1000, calls = argc > 1 ? std::atoi(argv[1]) : 5000;
    std::mt19937 rng(1);
    const char* alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
    std::vector<std::string> words(rows);
    for (auto& w : words) {
        const int n = 8 + (int)(rng() % 17);
        for (int i = 0; i < n; ++i) w.push_back(alpha[rng() % 36]);
    }
    std::vector<char*> ptrs(rows);
    for (int i = 0; i < rows; ++i) ptrs[i] = words[i].data();
    const uint32_t h = indexN(ptrs.data(), rows, 1, nullptr);
    if (!h) return 1;
    std::vector<std::string> qs(256);
    for (auto& q : qs) {
        const std::string& src = words[rng() % rows];
        const size_t l = std::min<size_t>(12, src.size()), o = rng() % (src.size() - l + 1);
        q = src.substr(o, l);
    }
    std::vector<double> us;
    for (int i = 0; i < calls + 50; ++i) {
        char** res = nullptr;
        float* sc = nullptr;
        const auto t0 = std::chrono::steady_clock::now();
        score(h, qs[i % 256].c_str(), &res, &sc, 0.3f, 100);
        release(h, res, sc);
        const auto t1 = std::chrono::steady_clock::now();
        if (i >= 50) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::sort(us.begin(), us.end());
    double sum = 0;
    for (double x : us) sum += x;
    std::printf("{\"c1_score_us_mean_c\": %.1f, \"c1_score_us_p50_c\": %.1f, \"calls\": %d}\n", sum / us.size(),
                us[us.size() / 2], calls);
    dispose(h);
    return 0;
}
