// Microbenchmark: LDS-DMA vs register loads, per-instruction cost on gfx950.
// Each wave loops ITERS times: issue M loads of one form from pseudo-random 4 KiB-aligned
// places of a 1 GiB buffer, then wait. Reports wave-instructions/s and bytes/s chip-wide.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <int MODE, int M, int ACTIVE, uint64_t WIN = (1ull << 22)>
__global__ __launch_bounds__(64) void k_dma(const uint32_t* __restrict__ src, uint64_t n_words, int iters,
                                            uint32_t* __restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint32_t st[M * 256];
    const uint32_t lane = threadIdx.x;
    uint64_t h = blockIdx.x * 0x9E3779B97F4A7C15ull + 1;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        for (int m = 0; m < M; ++m) {
            h = h * 6364136223846793005ull + 1442695040888963407ull;
            const uint64_t base = ((h >> 20) % (n_words / 1024 - 1)) * 1024;  // 4 KiB aligned
            if (lane < ACTIVE) {
                if (MODE == 0) {  // LDS-DMA dword
                    const uint32_t* g = src + base + lane;
                    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g),
                                 "s"(lds_addr(st + m * 64)) : "memory", "m0");
                } else if (MODE == 1) {  // LDS-DMA dwordx4
                    const uint32_t* g = src + base + lane * 4;
                    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g),
                                 "s"(lds_addr(st + m * 256)) : "memory", "m0");
                } else if (MODE == 4) {  // LDS-DMA dwordx4, 16-byte chunks gathered from 5 segments
                    const uint32_t seg = lane / 13;
                    const uint64_t sb = ((h >> (8 + 4 * seg)) * 2654435761u % (n_words / 1024 - 1)) * 1024 + 4 * (seg * 7 % 5);
                    const uint32_t* g = src + sb + (lane % 13) * 4;
                    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g),
                                 "s"(lds_addr(st + m * 256)) : "memory", "m0");
                } else if (MODE == 5) {  // LDS-DMA dwordx4, contiguous but within a 64 MiB window
                    const uint32_t* g = src + base % (1u << 24) + lane * 4;
                    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g),
                                 "s"(lds_addr(st + m * 256)) : "memory", "m0");
                } else if (MODE == 6) {  // register dwordx4, 5-segment gather inside a small window
                    const uint32_t seg = lane / 13;
                    const uint64_t sb = (((h >> (8 + 4 * seg)) * 2654435761u) % (WIN / 64)) * 16 + 4 * (seg * 7 % 5);
                    const uint4 v = *reinterpret_cast<const uint4*>(src + sb + (lane % 13) * 4);
                    acc += v.x ^ v.y ^ v.z ^ v.w;
                } else if (MODE == 7) {  // register dwordx4, contiguous, inside a small window
                    const uint4 v = *reinterpret_cast<const uint4*>(src + (base % WIN) + lane * 4);
                    acc += v.x ^ v.y ^ v.z ^ v.w;
                } else if (MODE == 2) {  // register dword
                    acc += __builtin_nontemporal_load(src + base + lane);
                } else {  // register dwordx4
                    const uint4 v = *reinterpret_cast<const uint4*>(src + base + lane * 4);
                    acc += v.x ^ v.y ^ v.z ^ v.w;
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (MODE >= 2 && MODE != 4 && MODE != 5) { if (acc == 0x12345678u) sink[0] = acc; }
    else if (st[lane] == 0x12345678u) sink[1] = lane;
}

template <int MODE, int M, int ACTIVE, uint64_t WIN = (1ull << 22)>
int run(const char* name, const uint32_t* d, uint64_t n, uint32_t* sink, int waves_per_cu) {
    const int blocks = 256 * waves_per_cu, iters = 200;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k_dma<MODE, M, ACTIVE, WIN><<<blocks, 64>>>(d, n, 4, sink);
    hipEventRecord(a);
    k_dma<MODE, M, ACTIVE, WIN><<<blocks, 64>>>(d, n, iters, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    const double instr = (double)blocks * iters * M;
    const int bpl = (MODE == 1 || MODE == 3 || MODE >= 4) ? 16 : 4;
    const double bytes = instr * ACTIVE * bpl;
    printf("%-28s waves/CU %2d M %2d active %2d: %8.3f ms  %7.2f G wave-instr/s  %7.1f GB/s  %6.1f cyc/instr/CU\n",
           name, waves_per_cu, M, ACTIVE, ms, instr / ms / 1e6, bytes / ms / 1e6,
           2.4e9 * (ms * 1e-3) / (instr / 256));
    return 0;
}

int main() {
    const uint64_t n = 1ull << 28;  // 1 GiB of u32
    uint32_t *d, *sink;
    CHECK(hipMalloc(&d, n * 4));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(d, 1, n * 4));
    for (int w : {4, 8, 13, 16}) {
        run<3, 4, 64>("vgpr dwordx4 1GiB M=4", d, n, sink, w);
        run<7, 4, 64, (1ull << 20)>("vgpr dwordx4 4MiB win M=4", d, n, sink, w);
        run<6, 4, 64, (1ull << 20)>("vgpr x4 5-seg 4MiB win M=4", d, n, sink, w);
        run<6, 4, 64, (1ull << 14)>("vgpr x4 5-seg 64KiB win M=4", d, n, sink, w);
        run<6, 16, 64, (1ull << 20)>("vgpr x4 5-seg 4MiB win M=16", d, n, sink, w);
    }
    return 0;
}
