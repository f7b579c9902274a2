// Host cost of queueing a C2-sized call: 10 small kernels launched one by one against the same
// 10 captured once into a hipGraph and replayed (hipGraphLaunch), each with 3 iterations in flight
// (a wait on the iteration 3 back), as bench.py's pipelined loop does. Prints host microseconds
// per iteration spent queueing and the iteration rate.
// build: hipcc -O2 --offload-arch=gfx950 graph_launch.hip -o graph_launch
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <deque>

__global__ void k_small(unsigned* p, unsigned n) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1u;
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                          \
        }                                                                      \
    } while (0)

static void queue_call(hipStream_t s, unsigned* buf, unsigned blocks) {
    for (int k = 0; k < 10; ++k)
        hipLaunchKernelGGL(k_small, dim3(blocks), dim3(64), 0, s, buf + k * 65536, 65536u);
}

int main() {
    constexpr int kIters = 2000, kDepth = 3, kCtx = 4;
    unsigned* buf = nullptr;
    CK(hipMalloc(&buf, sizeof(unsigned) * 65536 * 10 * kCtx));
    hipStream_t st[kCtx];
    hipEvent_t ev[kCtx];
    for (int c = 0; c < kCtx; ++c) {
        CK(hipStreamCreateWithFlags(&st[c], hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&ev[c], hipEventDisableTiming));
    }
    for (unsigned blocks : {64u, 1024u}) {
        for (int mode = 0; mode < 2; ++mode) {
            hipGraphExec_t ge[kCtx] = {};
            if (mode == 1) {
                for (int c = 0; c < kCtx; ++c) {
                    hipGraph_t g;
                    CK(hipStreamBeginCapture(st[c], hipStreamCaptureModeThreadLocal));
                    queue_call(st[c], buf + c * 65536 * 10, blocks);
                    CK(hipStreamEndCapture(st[c], &g));
                    CK(hipGraphInstantiate(&ge[c], g, nullptr, nullptr, 0));
                    CK(hipGraphDestroy(g));
                }
            }
            std::deque<int> inflight;
            double q_us = 0;
            CK(hipDeviceSynchronize());
            const auto t0 = std::chrono::steady_clock::now();
            for (int it = 0; it < kIters; ++it) {
                const int c = it % kCtx;
                const auto a = std::chrono::steady_clock::now();
                if (mode == 0) queue_call(st[c], buf + c * 65536 * 10, blocks);
                else CK(hipGraphLaunch(ge[c], st[c]));
                CK(hipEventRecord(ev[c], st[c]));
                q_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
                inflight.push_back(c);
                while ((int)inflight.size() >= kDepth) {
                    CK(hipEventSynchronize(ev[inflight.front()]));
                    inflight.pop_front();
                }
            }
            CK(hipDeviceSynchronize());
            const double el = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            std::printf("%-6s 10 kernels x %4u blocks: queue %6.1f us/call, %6.1f us/call overall\n",
                        mode ? "graph" : "plain", blocks, q_us / kIters, el / kIters);
            for (int c = 0; c < kCtx && mode == 1; ++c) CK(hipGraphExecDestroy(ge[c]));
        }
    }
    return 0;
}
