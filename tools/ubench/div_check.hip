// Does one Newton step after v_rcp_f64 give the same correctly rounded quotient as
// the two steps of div_rn_fast? Random (n, d) with both in [2^-200, 2^200]
// (the FAST range), counting quotient mismatches and reciprocal mismatches.
// usage: div_check [log2 samples per launch] [launches]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double rnd(unsigned long long h, int mode) {
    // mantissa: random bits; exponent in [-200, 200]; mode 1: mantissa with long runs
    unsigned long long m = h & 0xfffffffffffffull;
    if (mode == 1) m = (h & 1) ? (0xfffffffffffffull >> (h >> 58)) : (1ull << ((h >> 52) & 51));
    const int e = (int)((h >> 12) % 401) - 200;
    return __longlong_as_double((long long)(((unsigned long long)(e + 1023) << 52) | m));
}
__global__ void k_check(unsigned long long seed, long long n, unsigned long long* bad) {
    unsigned long long nq = 0, nr = 0, nz = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long h1 = mix(seed ^ (2 * i)), h2 = mix(seed ^ (2 * i + 1));
        const int mode = (int)((h1 >> 63) & (h2 >> 63));
        const double num = rnd(h1, mode), d = rnd(h2, mode);
        const double r0 = __builtin_amdgcn_rcp(d);
        const double e0 = __builtin_fma(-d, r0, 1.0);
        const double r1 = __builtin_fma(r0, e0, r0);
        const double e1 = __builtin_fma(-d, r1, 1.0);
        const double r2 = __builtin_fma(r1, e1, r1);
        const double qa = num * r2, ra = __builtin_fma(-d, qa, num), QA = __builtin_fma(ra, r2, qa);
        const double qb = num * r1, rb = __builtin_fma(-d, qb, num), QB = __builtin_fma(rb, r1, qb);
        const double qc = num * r0, rc = __builtin_fma(-d, qc, num), QC = __builtin_fma(rc, r0, qc);
        const double Q = num / d;  // compiler IEEE division (reference)
        nz += __double_as_longlong(QC) != __double_as_longlong(Q);
        nq += (__double_as_longlong(QB) != __double_as_longlong(Q)) || (__double_as_longlong(QA) != __double_as_longlong(Q));
        nr += __double_as_longlong(r1) != __double_as_longlong(r2);
    }
    atomicAdd(&bad[0], nq);
    atomicAdd(&bad[1], nr);
    atomicAdd(&bad[2], nz);
}
int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 32;
    const int launches = argc > 2 ? atoi(argv[2]) : 4;
    unsigned long long* bad;
    (void)hipMalloc(&bad, 24);
    (void)hipMemset(bad, 0, 24);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int l = 0; l < launches; ++l) {
        hipLaunchKernelGGL(k_check, dim3(8192), dim3(256), 0, 0, 0x1234567ull + 977ull * l, 1ll << lg, bad);
        (void)hipDeviceSynchronize();
        unsigned long long h[3];
        (void)hipMemcpy(h, bad, 24, hipMemcpyDeviceToHost);
        printf("launch %d: %lld samples so far, quotient mismatches %llu, r1 != r2 %llu, no-Newton mismatches %llu\n", l,
               (long long)(l + 1) << lg, h[0], h[1], h[2]);
        fflush(stdout);
    }
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%.1f ms\n", ms);
    return 0;
}
