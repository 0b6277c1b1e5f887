// Shared-reciprocal seeds for the fit's correctly rounded division (experiment).
// div_rn starts its two Newton steps from v_rcp_f64(d) (16.5 issue cycles against
// 4 for a full-rate FP64 op). Two denominators can share one reciprocal:
// R = rcp(d0 d1), seeds R d1 ~ 1/d0 and R d0 ~ 1/d1 (two roundings on top of
// rcp's ~2^-26), four can share one through a product tree. After the two Newton
// steps the reciprocal's pre-rounding error is the square of the first step's
// (~2^-104) either way, so the quotient should round like '/'. This program
//   1. checks that on 2^32 random fast-range pairs and the constructed
//      near-midpoint family (mdg::division_hard_case) for each seed form, with
//      random partners, counting mismatches against IEEE '/';
//   2. compares the superposition sums of the variants bit for bit on a
//      synthetic spectrum (2048 Lorentzians, 1 M points);
//   3. times the variants on the whole chip.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o /tmp/seed_bench tools/ubench/seed_bench.hip
#include "../../metabodecon-rust_amd/csrc/mdg_kernels.hip"
#include <cstdio>
#include <vector>
#include <random>
#include <cstring>
using namespace mdg;

__device__ __forceinline__ double div_seeded(double n, double d, double r0) {
    const double e0 = __builtin_fma(-d, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-d, r1, 1.0);
    const double r2 = __builtin_fma(r1, e1, r1);
    const double q0 = n * r2;
    const double rem = __builtin_fma(-d, q0, n);
    return __builtin_fma(rem, r2, q0);
}

// form 0: own rcp; 1: pair seed (partner p1); 2: quad seed (partners p1..p3)
template <int FORM>
__device__ __forceinline__ double seeded(double n, double d, double p1, double p2, double p3) {
    if (FORM == 0) return div_rn(n, d);
    if (FORM == 1) return div_seeded(n, d, __builtin_amdgcn_rcp(d * p1) * p1);
    // quad: D = (d p1)(p2 p3); seed = R (p2 p3) p1, the order of the product tree
    const double a = d * p1, b = p2 * p3;
    const double R = __builtin_amdgcn_rcp(a * b);
    return div_seeded(n, d, (R * b) * p1);
}

template <int FORM>
__global__ void k_seed_check(unsigned long long seed, long long n, int cases, unsigned long long* out) {
    unsigned long long nb = 0, nt = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        double num, d;
        if (cases == 0) {
            const unsigned long long h1 = mix64(seed ^ (2 * i)), h2 = mix64(seed ^ (2 * i + 1));
            const bool runs = (h1 >> 63) & (h2 >> 63);
            num = fast_range_operand(h1, runs);
            d = fast_range_operand(h2, runs);
        } else {
            bool ok;
            division_hard_case(seed, (uint64_t)i, &num, &d, &ok);
            if (!ok) continue;
        }
        const unsigned long long h3 = mix64(seed ^ (0x5bd1e995ull * i + 7));
        const unsigned long long h4 = mix64(h3 + 1), h5 = mix64(h3 + 2);
        const double p1 = fabs(fast_range_operand(h3, false));
        const double p2 = fabs(fast_range_operand(h4, (h4 >> 61) == 7));
        const double p3 = fabs(fast_range_operand(h5, false));
        ++nt;
        nb += __double_as_longlong(seeded<FORM>(num, d, p1, p2, p3)) != __double_as_longlong(num / d);
    }
    if (nb) atomicAdd(out, nb);
    atomicAdd(out + 1, nt);
}

// superposition with GP-term groups (scalar parameters, prefetch as superpose_t)
template <int FORM>
__device__ __forceinline__ void group6(double x, double& acc, const double (&c)[18]) {
    double den[6], e[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const double dd = x - c[3 * k + 2];
        den[k] = c[3 * k + 1] + dd * dd;
    }
    if (FORM == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) e[k] = div_rn(c[3 * k], den[k]);
    } else if (FORM == 1) {
#pragma unroll
        for (int k = 0; k < 6; k += 2) {
            const double R = __builtin_amdgcn_rcp(den[k] * den[k + 1]);
            e[k] = div_seeded(c[3 * k], den[k], R * den[k + 1]);
            e[k + 1] = div_seeded(c[3 * k + 3], den[k + 1], R * den[k]);
        }
    } else {  // quad (0..3) + pair (4, 5)
        const double a = den[0] * den[1], b = den[2] * den[3];
        const double R = __builtin_amdgcn_rcp(a * b);
        const double Ra = R * b, Rb = R * a;
        e[0] = div_seeded(c[0], den[0], Ra * den[1]);
        e[1] = div_seeded(c[3], den[1], Ra * den[0]);
        e[2] = div_seeded(c[6], den[2], Rb * den[3]);
        e[3] = div_seeded(c[9], den[3], Rb * den[2]);
        const double R2 = __builtin_amdgcn_rcp(den[4] * den[5]);
        e[4] = div_seeded(c[12], den[4], R2 * den[5]);
        e[5] = div_seeded(c[15], den[5], R2 * den[4]);
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) acc += e[k];
}

template <int FORM>
__global__ void k_sup(const double* x, const double* params_g, int P, long long n, double* out) {
    const const_f64_ptr params = (const_f64_ptr)params_g;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const double xv = x[i];
        double acc = -0.0;
        double A[18], Bf[18];
#pragma unroll
        for (int k = 0; k < 18; ++k) A[k] = params[k];
        for (int g = 0; g + 1 < P / 6; g += 2) {
#pragma unroll
            for (int k = 0; k < 18; ++k) Bf[k] = params[18 * (g + 1) + k];
            group6<FORM>(xv, acc, A);
            if (g + 2 < P / 6) {
#pragma unroll
                for (int k = 0; k < 18; ++k) A[k] = params[18 * (g + 2) + k];
            }
            group6<FORM>(xv, acc, Bf);
        }
        out[i] = acc;
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
    const long long ncheck = argc > 1 ? atoll(argv[1]) : (1ll << 32);
    unsigned long long* cnt;
    CK(hipMalloc(&cnt, 16));
    const char* forms[] = {"own rcp", "pair seed", "quad seed"};
    for (int form = 0; form < 3; ++form) {
        for (int cases = 0; cases < 2; ++cases) {
            CK(hipMemset(cnt, 0, 16));
            const long long n = cases ? ncheck / 2 : ncheck;
            if (form == 0) hipLaunchKernelGGL(k_seed_check<0>, dim3(8192), dim3(256), 0, 0, 20261018ull, n, cases, cnt);
            if (form == 1) hipLaunchKernelGGL(k_seed_check<1>, dim3(8192), dim3(256), 0, 0, 20261018ull, n, cases, cnt);
            if (form == 2) hipLaunchKernelGGL(k_seed_check<2>, dim3(8192), dim3(256), 0, 0, 20261018ull, n, cases, cnt);
            CK(hipDeviceSynchronize());
            unsigned long long h[2];
            CK(hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost));
            printf("check %-9s %-12s: %llu mismatches in %llu\n", forms[form], cases ? "near-midpoint" : "random", h[0], h[1]);
            fflush(stdout);
        }
    }
    // superposition: 2048 Lorentzians over [0, 10] ppm, 1 M points
    const int P = 2046;  // multiple of 6 (the kernels take whole group pairs)
    const long long N = 1 << 20;
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::vector<double> hp(3 * P), hx(N);
    for (int j = 0; j < P; ++j) {
        hp[3 * j] = 1e2 * (0.01 + U(rng)) * 1e-3;        // sfhw
        hp[3 * j + 1] = 1e-6 * (0.05 + U(rng));            // hw2
        hp[3 * j + 2] = 10.0 * U(rng);                     // maxp
    }
    for (long long i = 0; i < N; ++i) hx[i] = 10.0 * (double)i / (double)N + 1e-9 * U(rng);
    double *x, *prm, *o0, *o1, *o2;
    CK(hipMalloc(&x, N * 8)); CK(hipMalloc(&prm, 3 * P * 8));
    CK(hipMalloc(&o0, N * 8)); CK(hipMalloc(&o1, N * 8)); CK(hipMalloc(&o2, N * 8));
    CK(hipMemcpy(x, hx.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(prm, hp.data(), 3 * P * 8, hipMemcpyHostToDevice));
    double* outs[3] = {o0, o1, o2};
    float ms[3] = {0, 0, 0};
    for (int rep = 0; rep < 3; ++rep) {
        for (int form = 0; form < 3; ++form) {
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            CK(hipEventRecord(e0));
            const dim3 g(4096), b(256);
            if (form == 0) hipLaunchKernelGGL(k_sup<0>, g, b, 0, 0, x, prm, P, N, outs[0]);
            if (form == 1) hipLaunchKernelGGL(k_sup<1>, g, b, 0, 0, x, prm, P, N, outs[1]);
            if (form == 2) hipLaunchKernelGGL(k_sup<2>, g, b, 0, 0, x, prm, P, N, outs[2]);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float t; CK(hipEventElapsedTime(&t, e0, e1));
            if (rep > 0) ms[form] += t / 2;
        }
    }
    std::vector<double> r0(N), r(N);
    CK(hipMemcpy(r0.data(), o0, N * 8, hipMemcpyDeviceToHost));
    for (int form = 0; form < 3; ++form) {
        CK(hipMemcpy(r.data(), outs[form], N * 8, hipMemcpyDeviceToHost));
        long long diff = 0;
        for (long long i = 0; i < N; ++i) diff += memcmp(&r[i], &r0[i], 8) != 0;
        printf("superposition %-9s: %.3f ms, %.3f T evals/s, %lld of %lld sums differ from own-rcp\n", forms[form],
               ms[form], (double)N * P / ms[form] / 1e9, diff, N);
    }
    return 0;
}
