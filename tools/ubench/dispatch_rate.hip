// Kernel dispatch throughput with many streams: S streams (one hardware queue
// each when GPU_MAX_HW_QUEUES >= S + 1), each replaying a captured hipGraph of G
// tiny kernels (one 64-thread workgroup, ~1 us of work), round-robin, R replays
// per stream. Prints kernels/s and graphs/s: the command processor's ceiling for
// pipelines made of many short launches (the B=1 deconvolution is ~21 launches).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/dispatch_rate.hip -o tools/ubench/dispatch_rate
//   GPU_MAX_HW_QUEUES=32 tools/ubench/dispatch_rate [S] [G] [R] [spin]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                  \
            return 1;                                                                \
        }                                                                            \
    } while (0)

__global__ void tiny(double* p, int spin) {
    double v = p[threadIdx.x];
    for (int i = 0; i < spin; ++i) v = v * 1.0000001 + 1e-9;
    p[threadIdx.x] = v;
}

int main(int argc, char** argv) {
    const int S = argc > 1 ? atoi(argv[1]) : 16;
    const int G = argc > 2 ? atoi(argv[2]) : 20;
    const int R = argc > 3 ? atoi(argv[3]) : 200;
    const int spin = argc > 4 ? atoi(argv[4]) : 64;
    std::vector<hipStream_t> st(S);
    std::vector<hipGraphExec_t> ex(S);
    std::vector<double*> buf(S);
    for (int s = 0; s < S; ++s) {
        CHECK(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
        CHECK(hipMalloc(&buf[s], 64 * sizeof(double)));
        CHECK(hipMemset(buf[s], 0, 64 * sizeof(double)));
        hipGraph_t g;
        CHECK(hipStreamBeginCapture(st[s], hipStreamCaptureModeRelaxed));
        for (int k = 0; k < G; ++k) hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, st[s], buf[s], spin);
        CHECK(hipStreamEndCapture(st[s], &g));
        CHECK(hipGraphInstantiate(&ex[s], g, nullptr, nullptr, 0));
        CHECK(hipGraphDestroy(g));
    }
    for (int s = 0; s < S; ++s) CHECK(hipGraphLaunch(ex[s], st[s]));
    CHECK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < R; ++r)
        for (int s = 0; s < S; ++s) CHECK(hipGraphLaunch(ex[s], st[s]));
    const auto t1 = std::chrono::steady_clock::now();
    CHECK(hipDeviceSynchronize());
    const auto t2 = std::chrono::steady_clock::now();
    const double sec = std::chrono::duration<double>(t2 - t0).count();
    const double host = std::chrono::duration<double>(t1 - t0).count();
    printf("{\"streams\": %d, \"kernels_per_graph\": %d, \"replays_per_stream\": %d, \"spin\": %d, "
           "\"kernels_per_s\": %.0f, \"graphs_per_s\": %.0f, \"host_enqueue_s\": %.4f, \"total_s\": %.4f}\n",
           S, G, R, spin, (double)S * R * G / sec, (double)S * R / sec, host, sec);
    return 0;
}
