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

// per-wave dependent chain; records the SIMD / CU each wave runs on (HW_REG_HW_ID)
__global__ void wave_chain(double* out, long long* cyc, int* ids, double a, unsigned active_mask, int lanes) {
    const int wv = threadIdx.x >> 6;
    double x = out[threadIdx.x];
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
    long long t0 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) < lanes && ((active_mask >> wv) & 1)) {
        for (int i = 0; i < ITERS; ++i) { x = x + a; x = x + a; x = x + a; x = x + a; }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) { cyc[wv] = t1 - t0; ids[wv] = (int)hw; }
}

// the smoother's tick (sum += in; sum -= pop; out = sum*div) on VGPR operands
template <int U>
__global__ void tick_chain(double* out, long long* cyc, int* ids, double div) {
    double v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = out[(threadIdx.x + k) & 1023];
    double sum = 0.0, f0 = 0.0, f1 = 0.0, f2 = 0.0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS / U; ++i) {
#pragma unroll
        for (int k = 0; k < U; k += 3) {
            sum += v[k]; sum -= f0; f0 = v[k]; v[k] = sum * div;
            sum += v[k + 1]; sum -= f1; f1 = v[k + 1]; v[k + 1] = sum * div;
            sum += v[k + 2]; sum -= f2; f2 = v[k + 2]; v[k + 2] = sum * div;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double t = 0; for (int k = 0; k < U; ++k) t += v[k];
    out[threadIdx.x] = t + sum;
    if ((threadIdx.x & 63) == 0) { cyc[threadIdx.x >> 6] = t1 - t0; ids[threadIdx.x >> 6] = 0; }
}

__device__ __forceinline__ double dpp_shr1_u(double v) {
    const long long b = __double_as_longlong(v);
    int lo = (int)(unsigned)(b & 0xffffffffll), hi = (int)(b >> 32);
    lo = __builtin_amdgcn_mov_dpp(lo, 0x138, 0xf, 0xf, true);
    hi = __builtin_amdgcn_mov_dpp(hi, 0x138, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}
// the lane-pipelined smoother step: feeder select, two adds, mul, DPP hand-off
template <int U>
__global__ void pipe_step(double* out, long long* cyc, int* ids, double div) {
    double v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = out[(threadIdx.x + k) & 1023];
    const bool feeder = (threadIdx.x % 3) == 0;
    double sum = 0.0, f[3] = {0, 0, 0}, rq[3] = {0, 0, 0}, ob[U];
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS / U; ++i) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const double in = feeder ? v[k] : rq[k % 3];
            sum += in; sum -= f[k % 3]; f[k % 3] = in;
            const double e = sum * div;
            ob[k] = e;
            rq[k % 3] = dpp_shr1_u(e);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = ob[k] + v[k];
        __builtin_amdgcn_sched_barrier(0);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double t = 0; for (int k = 0; k < U; ++k) t += v[k];
    out[threadIdx.x] = t + sum;
    if ((threadIdx.x & 63) == 0) { cyc[threadIdx.x >> 6] = t1 - t0; ids[threadIdx.x >> 6] = 0; }
}

// plain dependent chain with a VGPR operand
__global__ void vgpr_chain(double* out, long long* cyc, int* ids, double a) {
    double x = out[threadIdx.x], y = out[(threadIdx.x + 7) & 1023] + a;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) { x = x + y; x = x + y; x = x + y; x = x + y; }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) { cyc[threadIdx.x >> 6] = t1 - t0; ids[threadIdx.x >> 6] = 0; }
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
    {
        int* ids; CHECK(hipMalloc(&ids, 64 * 4));
        struct Cfg { int W; unsigned mask; int lanes; };
        Cfg cfgs[] = {{1, 1, 1}, {2, 3, 1}, {3, 7, 1}, {4, 15, 1}, {4, 7, 1}, {4, 1, 1}, {4, 5, 1},
                      {4, 3, 1}, {3, 7, 64}, {4, 15, 64}, {8, 0xff, 1}, {8, 0x0f, 1}, {2, 3, 64}};
        for (auto cf : cfgs) {
          for (int rep = 0; rep < 3; ++rep) {
            const int W = cf.W;
            hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
            hipLaunchKernelGGL(wave_chain, dim3(1), dim3(64 * W), 0, 0, d, c, ids, 1e-9, cf.mask, cf.lanes);
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(wave_chain, dim3(1), dim3(64 * W), 0, 0, d, c, ids, 1e-9, cf.mask, cf.lanes);
            (void)hipEventRecord(b); (void)hipEventSynchronize(b);
            float ms; (void)hipEventElapsedTime(&ms, a, b);
            std::vector<long long> cy(W); std::vector<int> hid(W);
            (void)hipMemcpy(cy.data(), c, 8 * W, hipMemcpyDeviceToHost);
            (void)hipMemcpy(hid.data(), ids, 4 * W, hipMemcpyDeviceToHost);
            printf("W=%d mask=%02x lanes=%2d: wall ns/op=%.3f |", W, cf.mask, cf.lanes, ms * 1e6 / (4.0 * ITERS));
            for (int k = 0; k < W; ++k) printf(" s%d:%.1f", (hid[k] >> 4) & 3, cy[k] / (4.0 * ITERS));
            printf("\n");
          }
        }
    }
    {
        int* ids; CHECK(hipMalloc(&ids, 64 * 4));
        auto rk = [&](const char* name, void (*k)(double*, long long*, int*, double), int W, double ops) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64 * W), 0, 0, d, c, ids, 0.3333);
            hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k, dim3(1), dim3(64 * W), 0, 0, d, c, ids, 0.3333);
            (void)hipEventRecord(b); (void)hipEventSynchronize(b);
            float ms; (void)hipEventElapsedTime(&ms, a, b);
            std::vector<long long> cy(W);
            (void)hipMemcpy(cy.data(), c, 8 * W, hipMemcpyDeviceToHost);
            printf("%-22s W=%d: wall ns/op=%.3f cyc/op(w0)=%.2f\n", name, W, ms * 1e6 / ops, cy[0] / ops);
        };
        for (int W : {1, 4}) {
            rk("vgpr dep add", vgpr_chain, W, 4.0 * ITERS);
            rk("tick U=33 (per f64 op)", tick_chain<33>, W, 3.0 * (ITERS / 33) * 33);
            rk("tick U=66 (per f64 op)", tick_chain<66>, W, 3.0 * (ITERS / 66) * 66);
            rk("pipe step U=33 (per step)", pipe_step<33>, W, 1.0 * (ITERS / 33) * 33);
        }
    }
    return 0;
}
