// Micro-benchmarks that ground the kernel designs (results in DESIGN.md):
// cycles per dependent v_add_f64, single-wave issue of independent f64 adds,
// the smoother's add/sub/mul/DPP step, and a dependent ds_read_b64 + add chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 1 << 16;

__global__ void dep_add(double* out, long long* cyc, double a) {
    double x = out[threadIdx.x];
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        x = x + a; x = x + a; x = x + a; x = x + a;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void indep_add(double* out, long long* cyc, double a) {
    double x0 = out[threadIdx.x], x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        x0 += a; x1 += a; x2 += a; x3 += a; x4 += a; x5 += a; x6 += a; x7 += a;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void lds_chain(double* out, long long* cyc, int stride) {
    __shared__ double buf[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) buf[i] = 1.0 / (i + 1);
    __syncthreads();
    double acc = 0.0;
    int idx = threadIdx.x;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        double v = buf[idx];
        acc += v;
        idx = (idx + stride + (int)(acc * 0.0)) & 4095;  // dependent address
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    double* d; long long* c;
    CHECK(hipMalloc(&d, 1024 * 8)); CHECK(hipMalloc(&c, 1024 * 8));
    CHECK(hipMemset(d, 0, 1024 * 8));
    std::vector<long long> h(4);
    auto run = [&](const char* name, void (*k)(double*, long long*, double), int threads, double ops) {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, d, c, 1e-9);
        hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, d, c, 1e-9);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        hipMemcpy(h.data(), c, 8, hipMemcpyDeviceToHost);
        printf("%-28s threads=%4d  memtime/op=%.2f  ns/op=%.3f\n", name, threads, h[0] / ops, ms * 1e6 / ops);
    };
    run("dependent v_add_f64", dep_add, 64, 4.0 * ITERS);
    run("dependent v_add_f64", dep_add, 1, 4.0 * ITERS);
    run("8 independent v_add_f64", indep_add, 64, 8.0 * ITERS);
    run("8 independent (4 waves)", indep_add, 256, 8.0 * ITERS);
    {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipLaunchKernelGGL(lds_chain, dim3(1), dim3(64), 0, 0, d, c, 65);
        hipEventRecord(a);
        hipLaunchKernelGGL(lds_chain, dim3(1), dim3(64), 0, 0, d, c, 65);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        hipMemcpy(h.data(), c, 8, hipMemcpyDeviceToHost);
        printf("%-28s memtime/iter=%.2f ns/iter=%.3f\n", "dep ds_read_b64+add chain", h[0] / (double)ITERS, ms * 1e6 / ITERS);
    }
    // s_memtime frequency: compare with wall time of the dependent chain
    return 0;
}
