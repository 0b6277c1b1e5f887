// Phase breakdown of k_smooth_waves<3> on one synthetic 131072-point spectrum:
// builds the library kernel source with -DMDG_DIAG (stamps into a side buffer).
#include "../../metabodecon-rust_amd/csrc/mdg_kernels.hip"
#include <cstdio>
#include <vector>
using namespace mdg;
int main(int argc, char** argv) {
    const int N = 131072, B = argc > 1 ? atoi(argv[1]) : 1, P = 3;
    std::vector<double> h(N * (size_t)B);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000003) * 1e-3;
    double *y, *sm; int* status; long long* diag;
    (void)hipMalloc(&y, h.size() * 8); (void)hipMalloc(&sm, h.size() * 8);
    (void)hipMalloc(&status, 4 * B); (void)hipMemset(status, 0, 4 * B);
    (void)hipMalloc(&diag, (size_t)B * 16 * 8 * 8); (void)hipMemset(diag, 0, (size_t)B * 16 * 64);
    (void)hipMemcpy(y, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag), &diag, sizeof(diag));
    BatchArgs a{}; a.B = B; a.N = N; a.y = y; a.y_stride = N;
    Workspace w{}; w.status = status; w.smooth = sm;
    for (int rep = 0; rep < 2; ++rep) {
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        launch_smooth(a, w, P, 3, EngineSwitches{}, 0);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("B=%d smooth %.3f ms\n", B, ms);
    }
    std::vector<long long> d(16 * 8);
    (void)hipMemcpy(d.data(), diag, d.size() * 8, hipMemcpyDeviceToHost);
    const char* names[6] = {"dma-issue", "gather", "ticks", "vmcnt", "barrier", "copyout"};
    for (int wv = 0; wv < 4; ++wv) {
        long long tot = 0; for (int i = 0; i < 6; ++i) tot += d[wv * 8 + i];
        printf("wave %d total %lld cyc:", wv, tot);
        for (int i = 0; i < 6; ++i) printf(" %s=%.1f%%", names[i], 100.0 * d[wv * 8 + i] / (tot ? tot : 1));
        printf("\n");
    }
    return 0;
}
