// Cycles per term of mdg::dpp_fold (ordered DPP row-broadcast fold) on an
// L2-resident buffer, one wave; plus variants isolating the chain and the loads.
#include "../../metabodecon-rust_amd/csrc/mdg_kernels.hip"
#include <cstdio>
using namespace mdg;

__global__ void k_fold(const double* t, int n, double* out, long long* cyc, int mode) {
    double acc = 0.0;
    // warm the lines into L2 / L1 first
    for (int k = threadIdx.x; k < n; k += 64) acc += t[k] * 0.0;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) {
        acc = dpp_fold(acc, t, n);
    } else if (mode == 1) {  // chain only: same 16-fmac groups on one register
        const double one = 1.0, v = t[threadIdx.x & 15];
        for (int g = 0; g < n / 16; ++g) fold16(acc, v, one);
    } else {  // loads only (8 in flight), no chain
        double s = 0.0;
        for (int g = 0; g < n / 16; g += 8) {
            double b[8];
#pragma unroll
            for (int d = 0; d < 8; ++d) b[d] = t[min(16 * (g + d) + (int)(threadIdx.x & 15), n - 1)];
#pragma unroll
            for (int d = 0; d < 8; ++d) s += b[d];
        }
        acc += s;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    const int n = 5120;
    double *t, *out; long long* cyc;
    (void)hipMalloc(&t, n * 8); (void)hipMalloc(&out, 64 * 8); (void)hipMalloc(&cyc, 8);
    double h[n]; for (int i = 0; i < n; ++i) h[i] = 1.0 / (i + 1);
    (void)hipMemcpy(t, h, n * 8, hipMemcpyHostToDevice);
    const char* names[3] = {"dpp_fold", "chain only", "loads only"};
    for (int mode = 0; mode < 3; ++mode)
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(k_fold, dim3(1), dim3(64), 0, 0, t, n, out, cyc, mode);
            long long c; (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("%-12s %.2f cycles/term\n", names[mode], (double)c / n);
        }
    return 0;
}
