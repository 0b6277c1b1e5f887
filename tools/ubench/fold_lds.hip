// LDS-fed ordered fold microbenchmark (gfx950): one wave folds 192-term rows with
// ds_read_b128 feeding dependent v_fmac_f64; variants separate the LDS read cost,
// the fmac chain and the waits (EXEC = 24 lanes: the term-fold fit's fold wave).
#include "../../metabodecon-rust_amd/csrc/mdg_kernels.hip"
#include <cstdio>
using namespace mdg;
constexpr int RS = 194;
// raw loop variants: 12 b128 reads + 24 fmacs per trip (192 terms = 8 trips)
#define RD(r, off) "ds_read_b128 v[" #r "], %[a] offset:" #off "\n"
#define FM(lo) "v_fmac_f64 %[acc], v[" #lo "], %[one]\n"
#define TRIP_BOTH RD(64:67,0) FM(64:65) FM(66:67) RD(68:71,16) FM(68:69) FM(70:71) RD(72:75,32) FM(72:73) FM(74:75) \
  RD(76:79,48) FM(76:77) FM(78:79) RD(80:83,64) FM(80:81) FM(82:83) RD(84:87,80) FM(84:85) FM(86:87) \
  RD(88:91,96) FM(88:89) FM(90:91) RD(92:95,112) FM(92:93) FM(94:95) RD(96:99,128) FM(96:97) FM(98:99) \
  RD(100:103,144) FM(100:101) FM(102:103) RD(104:107,160) FM(104:105) FM(106:107) RD(108:111,176) FM(108:109) FM(110:111)
#define TRIP_FMA FM(64:65) FM(66:67) FM(68:69) FM(70:71) FM(72:73) FM(74:75) FM(76:77) FM(78:79) FM(80:81) FM(82:83) FM(84:85) FM(86:87) \
  FM(88:89) FM(90:91) FM(92:93) FM(94:95) FM(96:97) FM(98:99) FM(100:101) FM(102:103) FM(104:105) FM(106:107) FM(108:109) FM(110:111)
#define TRIP_RD RD(64:67,0) RD(68:71,16) RD(72:75,32) RD(76:79,48) RD(80:83,64) RD(84:87,80) RD(88:91,96) RD(92:95,112) RD(96:99,128) RD(100:103,144) RD(104:107,160) RD(108:111,176)
#define CLOB12 "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79","v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95","v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111"
template <int V>
__global__ void k_raw(double* out, long long* cyc, int reps) {
    __shared__ __attribute__((aligned(16))) double T[24 * RS];
    for (int i = threadIdx.x; i < 24 * RS; i += blockDim.x) T[i] = 1.0 + i * 1e-9;
    __syncthreads();
    double acc = -0.0; const double one = 1.0;
    unsigned a = lds_offset(T) + (threadIdx.x & 63) * (RS * 8 % 4096 == 0 ? 16 : 0);
    if (V >= 4 && (threadIdx.x & 63) >= 24) return;  // EXEC = 24 lanes
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps * 8; ++r) {
        if (V == 0) asm volatile(TRIP_BOTH : [acc] "+v"(acc) : [a] "v"(a), [one] "v"(one) : CLOB12);
        if (V == 1) asm volatile(TRIP_FMA : [acc] "+v"(acc) : [a] "v"(a), [one] "v"(one) : CLOB12);
        if (V == 2) asm volatile(TRIP_RD "s_waitcnt lgkmcnt(0)\n" : [acc] "+v"(acc) : [a] "v"(a), [one] "v"(one) : CLOB12);
        if (V == 3 || V == 5) asm volatile(TRIP_RD : [acc] "+v"(acc) : [a] "v"(a), [one] "v"(one) : CLOB12);
        if (V == 4) asm volatile(TRIP_BOTH : [acc] "+v"(acc) : [a] "v"(a), [one] "v"(one) : CLOB12);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
    double* out; long long* cyc;
    (void)hipMalloc(&out, 4096 * 8); (void)hipMalloc(&cyc, 64);
    const int reps = 200;
    auto run = [&](auto kern, const char* name, int threads) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(threads), 0, 0, out, cyc, reps);
        (void)hipDeviceSynchronize();
        hipLaunchKernelGGL(kern, dim3(1), dim3(threads), 0, 0, out, cyc, reps);
        (void)hipDeviceSynchronize();
        long long c; (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-34s threads=%d  %.2f cycles/term\n", name, threads, (double)c / (reps * 192.0));
    };
    run(k_raw<0>, "raw: reads+fmacs no waits", 64);
    run(k_raw<1>, "raw: fmacs only", 64);
    run(k_raw<2>, "raw: 12 reads + wait0", 64);
    run(k_raw<3>, "raw: reads, no waits", 64);
    run(k_raw<4>, "raw: reads+fmacs, EXEC=24", 64);
    run(k_raw<5>, "raw: reads only, EXEC=24", 64);
    return 0;
}
