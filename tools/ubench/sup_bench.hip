// Cycles per Lorentzian evaluation of mdg::superpose_t<true> (the lane = point
// superposition) for W waves per SIMD, parameters hot in the scalar cache.
#include "../../metabodecon-rust_amd/csrc/mdg_kernels.hip"
#include <cstdio>
using namespace mdg;

__global__ void k_sup(const double* x, const double* params, int P, double* out, long long* cyc) {
    const double xv = x[blockIdx.x * blockDim.x + threadIdx.x];
    double acc = superpose_t<true>(xv, params, P);  // warm the scalar cache
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    acc += superpose_t<true>(xv + 1e-3, params, P);
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k_sup2(const double* x, const double* params, int P, double* out) {
    const double xv = x[threadIdx.x];
    double acc = superpose_t<true>(xv, params, P);
    acc += superpose_t<true>(xv + 1e-3, params, P);
    out[threadIdx.x] = acc;
}

int main() {
    const int P = 2048, NT = 64 * 16;
    double *x, *params, *out; long long* cyc;
    (void)hipMalloc(&x, NT * 8); (void)hipMalloc(&params, P * 24); (void)hipMalloc(&out, NT * 8);
    (void)hipMalloc(&cyc, 64 * 8);
    double hp[3 * P], hx[NT];
    for (int j = 0; j < P; ++j) { hp[3 * j] = 1e3; hp[3 * j + 1] = 1e-6; hp[3 * j + 2] = -1.8 + j * 0.0064; }
    for (int i = 0; i < NT; ++i) hx[i] = 12.0 - i * 0.01;
    (void)hipMemcpy(params, hp, sizeof hp, hipMemcpyHostToDevice);
    (void)hipMemcpy(x, hx, sizeof hx, hipMemcpyHostToDevice);
    for (int wps : {1, 2, 4}) {  // waves per SIMD: one workgroup of 4*wps waves
        const int threads = 256 * wps;
        hipLaunchKernelGGL(k_sup, dim3(1), dim3(threads), 0, 0, x, params, P, out, cyc);
        long long c; (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("1 CU, waves/SIMD=%d: %.1f cycles per eval per wave (%.1f per eval per SIMD)\n", wps,
               (double)c / P, (double)c / P / wps);
    }
    // whole chip: 256 x k workgroups of 256 threads (k waves per SIMD), wall time
    for (int k : {1, 4, 6}) {
        const int blocks = 256 * k;
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        hipLaunchKernelGGL(k_sup2, dim3(blocks), dim3(256), 0, 0, x, params, P, out);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_sup2, dim3(blocks), dim3(256), 0, 0, x, params, P, out);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        const double evals = (double)blocks * 256 * P * 2;
        printf("chip, %d waves/SIMD: %.3f ms, %.2f T evals/s\n", k, ms, evals / ms / 1e9);
    }
    return 0;
}
