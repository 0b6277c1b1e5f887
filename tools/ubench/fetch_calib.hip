// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE per access width on gfx950.
// MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of the bytes of a 16-B/lane
// streaming read; other widths are uncalibrated. The engine's kernels read with
// 16-B, 8-B (plain and sc1) vector loads and wave-uniform scalar loads, so each
// width reads a known 1 GiB (4x the 256 MiB Infinity Cache, so nothing is
// served on-die) exactly once here, and writes likewise.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench/fetch_calib.hip -o tools/ubench/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d <dir> -o run -- tools/ubench/fetch_calib   (and WRITE_SIZE)
// prints the bytes each kernel moves; tools/pmc_summary.py calib turns the pair
// into per-width factors (profiles/<round>_fetch_calibration.json).
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                  \
            return 1;                                                                \
        }                                                                            \
    } while (0)

typedef const __attribute__((address_space(4))) double* const_f64_ptr;

__global__ __launch_bounds__(256) void read16(const double2* __restrict__ p, size_t n2, double* out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        const double2 v = p[i];
        s += v.x + v.y;
    }
    if (s == 1.2345) out[blockIdx.x] = s;  // keeps the loads, never stores
}

__global__ __launch_bounds__(256) void read8(const double* __restrict__ p, size_t n, double* out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += p[i];
    if (s == 1.2345) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void read8_sc1(const double* __restrict__ p, size_t n, double* out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        s += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 1.2345) out[blockIdx.x] = s;
}

// wave-uniform scalar loads (s_load_dwordx16 of 8 doubles): each wave streams its
// own contiguous chunk
__global__ __launch_bounds__(256) void read_scalar(const double* __restrict__ p, size_t n, double* out) {
    const size_t waves = (size_t)gridDim.x * 4;
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t chunk = n / waves;
    const const_f64_ptr q = (const_f64_ptr)(p + wave * chunk);
    double s = 0.0;
    for (size_t i = 0; i + 8 <= chunk; i += 8) {
        double t = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) t += q[i + k];
        s += t;
    }
    if (s == 1.2345) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void write16(double2* __restrict__ p, size_t n2) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256)
        p[i] = make_double2((double)i, 1.0);
}

__global__ __launch_bounds__(256) void write8(double* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (double)i;
}

__global__ __launch_bounds__(256) void write8_sc1(double* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        __hip_atomic_store(p + i, (double)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main() {
    const size_t bytes = 1ull << 30, n = bytes / 8;
    double *buf = nullptr, *out = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&out, 1 << 20));
    CHECK(hipMemset(buf, 0, bytes));
    const int grid = 4096;
    hipLaunchKernelGGL(write8, dim3(grid), dim3(256), 0, 0, buf, n);  // warm the pages
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(read16, dim3(grid), dim3(256), 0, 0, (const double2*)buf, n / 2, out);
    hipLaunchKernelGGL(read8, dim3(grid), dim3(256), 0, 0, buf, n, out);
    hipLaunchKernelGGL(read8_sc1, dim3(grid), dim3(256), 0, 0, buf, n, out);
    hipLaunchKernelGGL(read_scalar, dim3(grid), dim3(256), 0, 0, buf, n, out);
    hipLaunchKernelGGL(write16, dim3(grid), dim3(256), 0, 0, (double2*)buf, n / 2);
    hipLaunchKernelGGL(write8, dim3(grid), dim3(256), 0, 0, buf, n);
    hipLaunchKernelGGL(write8_sc1, dim3(grid), dim3(256), 0, 0, buf, n);
    CHECK(hipDeviceSynchronize());
    printf("{\"bytes_per_kernel\": %zu, \"kernels\": [\"read16\", \"read8\", \"read8_sc1\", "
           "\"read_scalar\", \"write16\", \"write8\", \"write8_sc1\"]}\n",
           bytes);
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
