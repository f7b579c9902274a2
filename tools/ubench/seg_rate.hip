// Microbenchmark: the k_wave load shape on gfx950. Each wave repeatedly loads a "part":
// NSEG list segments of SEGLEN u32 entries at random 4-byte aligned places of a buffer of
// BUF bytes, the segments' 16-byte chunks packed across the wave (lane l: chunk l, 64 + l, ...),
// DEPTH parts in flight per wave (registers), then consumes the oldest.
// Reports posting throughput (u32 entries/s) and the cycles per wave-instruction per CU.
// `seg_rate c3`: only the C3 main launch's part shape (58 parts of ~434 postings per query over
// ~10 lists: segments of ~43 entries; 6 waves per SIMD = 24 per CU) over 512 MB and 2 GB buffers,
// one kernel per line so that rocprofv3 --pmc FETCH_SIZE gives each shape's fetch per posting.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NSEG, int SEGLEN, int DEPTH, int ROUNDS>
__global__ __launch_bounds__(64) void k_seg(const uint4* __restrict__ src, uint32_t mask, int iters,
                                            uint32_t* __restrict__ sink) {
    const uint32_t lane = threadIdx.x;
    uint64_t h = (blockIdx.x + 1) * 0x9E3779B97F4A7C15ull;
    constexpr int CH = (SEGLEN + 3) / 4 + 1;  // chunks per segment (unaligned start)
    uint32_t acc = 0;
    uint4 v[DEPTH][ROUNDS];
    uint32_t pc = blockIdx.x * 0x01000193u;
    auto issue = [&](int d) {
        // segment s owns chunks [s*CH, (s+1)*CH); its base is a cheap hash of (part, s) so the
        // address arithmetic stays a few VALU per round (no 64-bit division)
        ++pc;
#pragma unroll
        for (int r = 0; r < ROUNDS; ++r) {
            const uint32_t c = 64 * r + lane;
            const uint32_t s = c / CH;
            uint32_t x = (pc * 16 + s) * 0x9E3779B1u;
            x ^= x >> 15;
            x *= 0x85EBCA6Bu;
            x ^= x >> 13;
            const uint64_t b = (x & mask) * 4 + (x >> 30);  // 4-byte aligned segment start
            if (s < NSEG) v[d][r] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint32_t*>(src) + b + 4 * (c - s * CH));
        }
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) issue(d);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r) acc += v[d][r].x ^ v[d][r].y ^ v[d][r].z ^ v[d][r].w;
            issue(d);
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int NSEG, int SEGLEN, int DEPTH>
int run(const uint4* d, uint64_t n_chunks, uint32_t* sink, int waves_per_cu, const char* tag, int reps = 64) {
    constexpr int CH = (SEGLEN + 3) / 4 + 1;
    constexpr int ROUNDS = (NSEG * CH + 63) / 64;
    const int blocks = 256 * waves_per_cu, iters = reps / DEPTH;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k_seg<NSEG, SEGLEN, DEPTH, ROUNDS><<<blocks, 64>>>(d, (uint32_t)(n_chunks - 1), 2, sink);
    hipEventRecord(a);
    k_seg<NSEG, SEGLEN, DEPTH, ROUNDS><<<blocks, 64>>>(d, (uint32_t)(n_chunks - 1), iters, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    const double parts = (double)blocks * (iters * DEPTH + DEPTH);
    const double instr = parts * ROUNDS;
    const double posts = parts * NSEG * SEGLEN;
    printf("%-6s nseg %2d seglen %4d depth %d waves/CU %2d rounds %2d: %7.3f ms %7.1f Gpost/s (%6.0f GB/s) %6.1f cyc/instr/CU\n",
           tag, NSEG, SEGLEN, DEPTH, waves_per_cu, ROUNDS, ms, posts / ms / 1e6, posts * 4 / ms / 1e6,
           2.4e9 * (ms * 1e-3) / (instr / 256));
    return 0;
}

int main(int argc, char** argv) {
    const uint64_t big = (512ull << 20) / 16, small = (2ull << 20) / 16;  // chunks, powers of two
    uint4* d;
    uint32_t* sink;
    if (argc > 1 && argv[1][0] == 'c') {
        const uint64_t huge = (2048ull << 20) / 16;
        CHECK(hipMalloc(&d, huge * 16 + 4096));
        CHECK(hipMalloc(&sink, 64));
        CHECK(hipMemset(d, 1, huge * 16));
        for (uint64_t n : {big, huge}) {
            const char* tag = n == big ? "512MB" : "2GB";
            // the part shape of the main launch at its occupancy (24 waves per CU) ...
            run<10, 43, 1>(d, n, sink, 24, tag, 256);
            run<10, 43, 2>(d, n, sink, 24, tag, 256);
            run<12, 36, 1>(d, n, sink, 24, tag, 256);
            run<8, 54, 1>(d, n, sink, 24, tag, 256);
            // ... and parts twice as long, which need twice the LDS sketch: 12 or 16 waves per CU
            run<10, 86, 1>(d, n, sink, 24, tag, 256);
            run<10, 86, 1>(d, n, sink, 16, tag, 256);
            run<10, 86, 1>(d, n, sink, 12, tag, 256);
            run<10, 86, 2>(d, n, sink, 12, tag, 256);
            run<10, 128, 1>(d, n, sink, 24, tag, 256);
        }
        return 0;
    }
    CHECK(hipMalloc(&d, big * 16 + 4096));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(d, 1, big * 16));
    for (uint64_t n : {big, small}) {
        const char* tag = n == big ? "512MB" : "2MB";
        for (int w : {8, 16, 32}) {
            run<10, 64, 1>(d, n, sink, w, tag);
            run<10, 64, 2>(d, n, sink, w, tag);
        }
        for (int w : {16}) {
            run<10, 16, 2>(d, n, sink, w, tag);
            run<10, 32, 2>(d, n, sink, w, tag);
            run<10, 128, 2>(d, n, sink, w, tag);
            run<10, 256, 2>(d, n, sink, w, tag);
            run<5, 128, 2>(d, n, sink, w, tag);
            run<1, 1024, 2>(d, n, sink, w, tag);
            run<64, 16, 2>(d, n, sink, w, tag);
        }
    }
    return 0;
}
