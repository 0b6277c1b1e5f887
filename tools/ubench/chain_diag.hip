// Timeline of k_smooth_chain<3> (3 passes) on synthetic 131072-point spectra:
// builds the library kernel source with -DMDG_DIAG; per (spectrum, pass) the
// chain wave's head / steady / tail stamps and the feeder/scaler round counts.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -DMDG_DIAG \
//       tools/ubench/chain_diag.hip -o tools/ubench/chain_diag
//   tools/ubench/chain_diag [B] [passes] [mode] [N]     (N: points, default 131072)
#include "../../metabodecon-rust_amd/csrc/mdg_kernels.hip"
#include <cstdio>
#include <vector>
using namespace mdg;
int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1, P = argc > 2 ? atoi(argv[2]) : 3, WS = 3;
    const int mode = argc > 3 ? atoi(argv[3]) : 0;
    const int N = argc > 4 ? atoi(argv[4]) : 131072;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_chain_mode), &mode, sizeof(mode));
    std::vector<double> h(N * (size_t)B);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000003) * 1e-3;
    double *y, *sm, *chain; int* status; long long* diag;
    const size_t cb = chain_bytes(B, N, WS, P);
    (void)hipMalloc(&y, h.size() * 8); (void)hipMalloc(&sm, h.size() * 8);
    (void)hipMalloc(&chain, cb); (void)hipMemset(chain, 0, cb);
    (void)hipMalloc(&status, 4 * B); (void)hipMemset(status, 0, 4 * B);
    (void)hipMalloc(&diag, (size_t)B * P * 32 * 8);
    (void)hipMemcpy(y, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag), &diag, sizeof(diag));
    BatchArgs a{}; a.B = B; a.N = N; a.y = y; a.y_stride = N;
    Workspace w{}; w.status = status; w.smooth = sm;
    const int64_t L = chain_stride_for(N, WS);
    w.chain_stride = L; w.chain_raw = chain; w.chain_tmp = chain + (size_t)P * B * L;
    w.chain_flags = (int32_t*)((char*)chain + (size_t)(2 * P - 1) * B * L * 8); w.chain_P = P;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipMemset(w.chain_flags, 0, (size_t)B * P * 128);
        (void)hipMemset(diag, 0, (size_t)B * P * 32 * 8);
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        launch_smooth(a, w, P, WS, EngineSwitches{}, 0);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("B=%d smooth %.3f ms (%s)\n", B, ms, hipGetErrorString(hipGetLastError()));
    }
    // check against a host moving average (3 passes, window 3)
    std::vector<double> hs(N), ref(h.begin(), h.begin() + N);
    (void)hipMemcpy(hs.data(), sm, N * 8, hipMemcpyDeviceToHost);
    for (int it = 0; it < P; ++it) {
        std::vector<double> src = ref;
        double sum = 0.0; sum += src[0];
        int len = 1;
        for (int i = 0; i < N - 1; ++i) {
            sum += src[i + 1];
            if (len < 3) { ++len; ref[i] = sum * (1.0 / len); }
            else { sum -= src[i + 1 - 3]; ref[i] = sum * (1.0 / 3); }
        }
        sum -= src[N - 3]; ref[N - 1] = sum * (1.0 / 2);
    }
    int bad = 0; for (int i = 0; i < N; ++i) bad += hs[i] != ref[i];
    printf("spectrum 0 mismatches vs host: %d\n", bad);
    std::vector<long long> d((size_t)B * P * 32);
    (void)hipMemcpy(d.data(), diag, d.size() * 8, hipMemcpyDeviceToHost);
    long long t0 = d[0];
    for (int s = 0; s < B && s < 4; ++s)
        for (int p = 0; p < P; ++p) {
            const long long* q = &d[((size_t)s * P + p) * 32];
            const double ticks = q[4] * 96.0;
            printf("s%d p%d chain: start %+lld head %lld steady %lld (%.2f cyc/tick over %lld blocks) tail %lld | "
                   "feeder %lld..%lld rounds %lld idle %lld | scaler %lld..%lld rounds %lld idle %lld\n",
                   s, p, q[0] - t0, q[1] - q[0], q[2] - q[1], (q[2] - q[1]) / (ticks > 0 ? ticks : 1), q[4],
                   q[3] - q[2], q[8] - t0, q[9] - t0, q[10], q[11], q[16] - t0, q[17] - t0, q[18], q[19]);
            printf("    scaler busy %lld cycles for %lld blocks (%.0f per block)\n", q[21], q[22],
                   q[22] ? (double)q[21] / q[22] : 0.0);
            printf("    scaler phases: loads+stage %lld replay %lld stores %lld vmcnt %lld\n", q[23], q[24], q[25], q[26]);
            printf("    chain in_ready waits %lld, sleeps %lld\n", q[6] >> 16, q[6] & 0xffff);
            for (int k : {5, 12, 20})
                printf("    HW_ID[%d]: wave %lld simd %lld cu %lld sh %lld se %lld\n", k, q[k] & 15,
                       (q[k] >> 4) & 3, (q[k] >> 8) & 15, (q[k] >> 12) & 1, (q[k] >> 13) & 7);
        }
    return 0;
}
