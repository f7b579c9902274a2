// Microbenchmark: wave64 VALU issue rate per SIMD on gfx950, alone and mixed with the scalar and
// LDS instructions the tier-1a kernel interleaves (per part it issues ~230 VALU, ~130 SALU,
// ~27 LDS). W waves per SIMD (blocks of 4 waves, W blocks per CU) each run `iters` iterations of
// 16 independent v_add_u32 (8 chains), plus per MODE:
//   0: nothing else
//   1: 8 dependent s_add_u32 (SALU : VALU = 0.5)
//   2: 8 s_add_u32 + 2 ds_add_rtn_u32 on random words of a 4 KB LDS table, results consumed
//   3: as 2, and the 16 VALU as 8 dependent pairs (each v_add reads the previous one's result)
// Reported: VALU instructions per SIMD per shader cycle, so the clock does not enter: each wave
// records its SIMD (HW_ID, XCC_ID) and the s_memtime ticks around its loop; per SIMD, the VALU
// its waves issued over the span from the first wave's start to the last wave's end, averaged
// over the SIMDs (with the mean number of waves that ran on a SIMD). Per the microarchitecture
// guide a wave64 VALU issues over 2 cycles: 0.5 per cycle would be the ceiling.
// build: hipcc -O3 --offload-arch=gfx950 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <array>
#include <map>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

#define V8(op) op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)

template <int MODE>
__global__ __launch_bounds__(256) void k_valu(uint32_t* __restrict__ out, int iters, unsigned long long* __restrict__ cyc) {
    // (size - 1) << 11 | offset << 6 | id: HW_REG_HW_ID (4) and HW_REG_XCC_ID (20), whole registers
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    constexpr uint32_t kTab = MODE >= 2 ? 1024 : 64;  // 4 KB per block for the LDS modes
    __shared__ uint32_t tab[kTab];
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    for (uint32_t i = tid; i < kTab; i += 256) tab[i] = 0;
    __syncthreads();
    uint32_t a0 = tid, a1 = tid + 1, a2 = tid + 2, a3 = tid + 3, a4 = tid + 4, a5 = tid + 5, a6 = tid + 6, a7 = tid + 7;
    const uint32_t b = tid * 0x9E3779B1u;
    uint32_t s0 = blockIdx.x;
    uint32_t h = tid * 0x85EBCA6Bu + blockIdx.x;
    uint32_t lsum = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 3) {
            asm volatile(
                "v_add_u32 %0, %0, %8\n v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %1, %1, %8\n"
                "v_add_u32 %2, %2, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %3, %3, %8\n"
                "v_add_u32 %4, %4, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %5, %5, %8\n"
                "v_add_u32 %6, %6, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n v_add_u32 %7, %7, %8\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(b));
        } else {
            asm volatile(
                "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
                "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(b));
        }
        if (MODE >= 1) {
            asm volatile(
                "s_add_u32 %0, %0, 3\n s_add_u32 %0, %0, 5\n s_add_u32 %0, %0, 7\n s_add_u32 %0, %0, 9\n"
                "s_add_u32 %0, %0, 11\n s_add_u32 %0, %0, 13\n s_add_u32 %0, %0, 15\n s_add_u32 %0, %0, 17\n"
                : "+s"(s0)
                :
                : "scc");
        }
        if (MODE >= 2) {
            h = h * 1664525u + 1013904223u;
            const uint32_t w0 = atomicAdd(&tab[(h >> 8) & (kTab - 1)], 1u);
            const uint32_t w1 = atomicAdd(&tab[(h >> 20) & (kTab - 1)], 1u);
            lsum += w0 + w1;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + tid] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s0 ^ lsum;
    if ((tid & 63) == 0) {
        const uint32_t simd = ((hw >> 4) & 3u) | ((hw >> 8) & 15u) << 2 | ((hw >> 12) & 15u) << 6 | (xcc & 15u) << 10;
        cyc[3 * (blockIdx.x * 4 + wave)] = t0;
        cyc[3 * (blockIdx.x * 4 + wave) + 1] = t1;
        cyc[3 * (blockIdx.x * 4 + wave) + 2] = simd;
    }
}

template <int MODE>
int run(int cus, int w, int iters) {
    const int blocks = cus * w;
    uint32_t* out;
    unsigned long long* cyc;
    CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * 256));
    CHECK(hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 4 * 3));
    hipLaunchKernelGGL(k_valu<MODE>, dim3(blocks), dim3(256), 0, 0, out, 10, cyc);  // warm-up
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_valu<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(blocks * 4 * 3);
    CHECK(hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    std::map<unsigned long long, std::array<unsigned long long, 3>> simd;  // key -> {first start, last end, waves}
    double span_sum = 0;
    for (int i = 0; i < blocks * 4; ++i) {
        const unsigned long long t0 = h[3 * i], t1 = h[3 * i + 1], k = h[3 * i + 2];
        span_sum += (double)(t1 - t0);
        auto it = simd.find(k);
        if (it == simd.end()) simd[k] = {t0, t1, 1};
        else it->second = {std::min(it->second[0], t0), std::max(it->second[1], t1), it->second[2] + 1};
    }
    double rate = 0, waves = 0;
    for (auto& [k, v] : simd) {
        rate += (double)v[2] * iters * 16.0 / (double)(v[1] - v[0]);
        waves += (double)v[2];
    }
    rate /= (double)simd.size();
    waves /= (double)simd.size();
    const double mean = span_sum / (blocks * 4);
    // per SIMD, first start to last end against one wave's span: 1.0 when its waves all ran together
    double stag = 0;
    for (auto& [k, v] : simd) stag += (double)(v[1] - v[0]);
    stag /= (double)simd.size() * mean;
    printf("mode %d, %d waves/SIMD: %.2f waves per SIMD, SIMD span / wave span %.2f; %.3f VALU per SIMD-cycle "
           "over SIMD spans, %.3f over wave spans (valid when the ratio is ~1); kernel %.3f ms\n", MODE, w, waves,
           stag, rate, waves * iters * 16.0 / mean, ms);
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("%s, %d CUs\n", p.gcnArchName, cus);
    const int iters = 20000;
    for (int w : {1, 2, 4, 6, 8}) {
        if (run<0>(cus, w, iters) || run<1>(cus, w, iters) || run<2>(cus, w, iters) || run<3>(cus, w, iters)) return 1;
    }
    return 0;
}
