// Phase breakdown and timing of the fit-superposition kernels on synthetic peak
// tables (P peaks, 3P reduced points per spectrum): builds the library kernel source
// with -DMDG_DIAG. usage: fit_diag [B] [P] [kinds, comma-separated; MDG_FITSUP names,
// '/noeval' suffix = tf without evaluation; "sQ.PB.PS@G" ("SQ.PB.PS@G": single
// buffer) = the term fold
// k_fit_sup_tw<TwShape<Q, PB, PS>> on a (G, B) grid, for the shapes listed in
// launch_shape (experiments: G workgroups per spectrum, tiles grid-strided)]
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -DMDG_DIAG \
//       tools/ubench/fit_diag.hip -o tools/ubench/fit_diag
#include "../../metabodecon-rust_amd/csrc/mdg_kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>
using namespace mdg;

// experimental term-fold shapes (not in the library): returns EW, or 0 if unknown
template <int Q, int PB, int PS, bool SB = false>
static int launch_one(const BatchArgs& a, const Workspace& w, int g) {
    using SH = TwShape<Q, PB, PS, SB>;
    hipLaunchKernelGGL((k_fit_sup_tw<SH>), dim3(g, a.B), dim3(64 * (SH::EW + 1)), 0, 0, a, w, 0);
    return SH::EW;
}
static int launch_shape(int q, int pb, int ps, const BatchArgs& a, const Workspace& w, int g, bool sb) {
    if (sb) {  // "Sq.pb.ps@g": single-buffered
        if (q == 63 && pb == 1 && ps == 3) return launch_one<63, 1, 3, true>(a, w, g);
        if (q == 63 && pb == 1 && ps == 7) return launch_one<63, 1, 7, true>(a, w, g);
        if (q == 63 && pb == 2 && ps == 3) return launch_one<63, 2, 3, true>(a, w, g);
        return 0;
    }
    if (q == 63 && pb == 1 && ps == 7) return launch_one<63, 1, 7>(a, w, g);
    if (q == 63 && pb == 2 && ps == 7) return launch_one<63, 2, 7>(a, w, g);
    if (q == 63 && pb == 1 && ps == 3) return launch_one<63, 1, 3>(a, w, g);
    if (q == 63 && pb == 2 && ps == 3) return launch_one<63, 2, 3>(a, w, g);
    if (q == 60 && pb == 1 && ps == 15) return launch_one<60, 1, 15>(a, w, g);
    if (q == 60 && pb == 2 && ps == 6) return launch_one<60, 2, 6>(a, w, g);
    if (q == 48 && pb == 1 && ps == 6) return launch_one<48, 1, 6>(a, w, g);
    if (q == 63 && pb == 1 && ps == 9) return launch_one<63, 1, 9>(a, w, g);
    return 0;
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1, P = argc > 2 ? atoi(argv[2]) : 2048;
    const int N = 131072, capD = N / 2 + 2;
    std::vector<double> par((size_t)B * capD * 3, 0.0), rx((size_t)B * capD * 3 + 64, 0.0),
        ry((size_t)B * capD * 3, 1.0);
    unsigned long long st = 12345;
    auto U = [&]() { st = st * 6364136223846793005ull + 1442695040888963407ull; return (double)(st >> 11) * 0x1p-53; };
    for (int s = 0; s < B; ++s)
        for (int p = 0; p < P; ++p) {
            const double m = -1.8 + 13.2 * U(), hw = 3e-4 + 5e-4 * U(), A = pow(10.0, 4.5 + 3.5 * U());
            double* L = &par[((size_t)s * capD + p) * 3];
            L[0] = A * hw * hw; L[1] = hw * hw; L[2] = m;
            for (int k = 0; k < 3; ++k) rx[(size_t)s * capD * 3 + 3 * p + k] = m + (k - 1) * 1.5e-4;
        }
    double *d_par, *d_rx, *d_ry, *d_ratio, *d_alt, *d_st; int32_t *status, *sel, *xok, *unsafe; long long* diag;
    (void)hipMalloc(&d_alt, par.size() * 8); (void)hipMalloc(&d_st, par.size() * 16);
    {
        std::vector<double> st6(par.size() * 2, 1.0);
        (void)hipMemcpy(d_st, st6.data(), st6.size() * 8, hipMemcpyHostToDevice);
    }
    (void)hipMalloc(&d_par, par.size() * 8); (void)hipMalloc(&d_rx, rx.size() * 8);
    (void)hipMalloc(&d_ry, ry.size() * 8); (void)hipMalloc(&d_ratio, ry.size() * 8);
    (void)hipMemcpy(d_par, par.data(), par.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_rx, rx.data(), rx.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_ry, ry.data(), ry.size() * 8, hipMemcpyHostToDevice);
    std::vector<int32_t> selv(B, P), ones(B, 1);
    (void)hipMalloc(&status, 4 * B); (void)hipMemset(status, 0, 4 * B);
    (void)hipMalloc(&sel, 4 * B); (void)hipMemcpy(sel, selv.data(), 4 * B, hipMemcpyHostToDevice);
    (void)hipMalloc(&xok, 4 * B); (void)hipMemcpy(xok, ones.data(), 4 * B, hipMemcpyHostToDevice);
    (void)hipMalloc(&unsafe, 16 * B); (void)hipMemset(unsafe, 0, 16 * B);
    // every DIAG_FLUSH record the guard allows, the KSTAMP slots and the placement records
    const size_t nd = kDiagStampBase + 4096 + ((size_t)1 << 20);
    (void)hipMalloc(&diag, nd * 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag), &diag, sizeof(diag));
    BatchArgs a{}; a.B = B; a.N = N;
    Workspace w{}; w.capD = capD; w.status = status; w.sel_count = sel; w.params = d_par;
    w.rx = d_rx; w.ry = d_ry; w.ratio = d_ratio; w.x_ok = xok; w.unsafe = unsafe;
    w.stencil = d_st; w.fit_iters = 10;
    {
        int cus = 0, dev = 0;
        (void)hipGetDevice(&dev);
        const hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        printf("device %d: %d CUs (rc %d)\n", dev, cus, (int)e);
    }
    std::vector<std::string> kinds;
    {
        std::string all = argc > 3 ? argv[3] : "dpp,plain,tf,tf/noeval";
        size_t p0 = 0;
        while (p0 <= all.size()) {
            const size_t p1 = all.find(',', p0);
            kinds.push_back(all.substr(p0, p1 == std::string::npos ? std::string::npos : p1 - p0));
            if (p1 == std::string::npos) break;
            p0 = p1 + 1;
        }
    }
    std::vector<double> ref;
    for (const std::string& ks : kinds) {
        const char* k = ks.c_str();
        const int mode = ks.find("/nostore") != std::string::npos ? 1 : ks.find("/noeval") != std::string::npos ? 2 : 0;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tf_mode), &mode, sizeof(mode));
        int sq = 0, spb = 0, sps = 0, sg = 0;
        const bool sbuf = ks[0] == 'S';
        const bool shape = (ks[0] == 's' || sbuf) && sscanf(k + 1, "%d.%d.%d@%d", &sq, &spb, &sps, &sg) == 4;
        // the engine's switches (normally read when a context is created): the kernel to run
        EngineSwitches sw;
        std::strncpy(sw.fitsup, shape ? "tw7" : ks.substr(0, ks.find('/')).c_str(), sizeof(sw.fitsup) - 1);
        if (const char* tg = std::getenv("MDG_TW_G")) sw.tw_g = std::max(1, std::atoi(tg));
        a.latency = 1;
        w.params_alt = fit_sup_fused(a, sw) ? d_alt : nullptr;
        float best = 1e30f;
        int shape_ew = 0;
        for (int rep = 0; rep < 6; ++rep) {
            (void)hipMemset(diag, 0, nd * 8);
            hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            if (shape) shape_ew = launch_shape(sq, spb, sps, a, w, sg, sbuf);
            else launch_fit_sup(a, w, 24, 0, sw, 0);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep > 0 && ms < best) best = ms;
        }
        std::vector<double> out(ry.size());
        (void)hipMemcpy(out.data(), d_ratio, out.size() * 8, hipMemcpyDeviceToHost);
        bool same = true;
        if (ref.empty()) ref = out;
        else if (!w.params_alt) for (int s = 0; s < B; ++s) for (int i = 0; i < 3 * P; ++i) same &= out[(size_t)s * capD * 3 + i] == ref[(size_t)s * capD * 3 + i];
        const double evals = 3.0 * P * P * B;
        printf("%-6s B=%d P=%d  %.2f us/launch  %.3f T evals/s  same_as_dpp=%d\n", k, B, P, best * 1e3,
               evals / (best * 1e-3) / 1e12, (int)same);
        if (shape && !shape_ew) { printf("%s: unknown shape\n", k); continue; }
        {
            // placement of the fold waves (wave EW of each block): HW_ID fields (gfx9:
            // wave 3:0, SIMD 5:4, CU 11:8, SH 12, SE 15:13, TG slot 19:16) and XCC_ID;
            // blocks sharing a CU whose fold waves share a SIMD compete for its issue
            std::vector<long long> d(nd);
            (void)hipMemcpy(d.data(), diag, nd * 8, hipMemcpyDeviceToHost);
            const int EWp = shape ? shape_ew : (ks.rfind("tf", 0) == 0 ? kTfEW : 7);
            std::map<long long, std::vector<int>> cu_fold;  // CU key -> fold SIMDs of its blocks
            int simd_hist[4] = {0, 0, 0, 0}, recs = 0;
            for (size_t b = 0; b < (1u << 16); ++b) {
                const long long v = d[kDiagStampBase + 4096 + b * 16 + EWp];
                if (!(v >> 62)) continue;
                const unsigned hw = (unsigned)v, xcc = (unsigned)((v >> 32) & 0xffff);
                const int simd = (hw >> 4) & 3;
                const long long cu = ((long long)xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
                cu_fold[cu].push_back(simd);
                simd_hist[simd] += 1;
                ++recs;
            }
            int shared = 0, pairs = 0;
            for (auto& kv : cu_fold) {
                const auto& v = kv.second;
                for (size_t i = 0; i < v.size(); ++i)
                    for (size_t j = i + 1; j < v.size(); ++j) { ++pairs; shared += v[i] == v[j]; }
            }
            printf("   fold waves: %d blocks on %zu CUs, SIMD histogram %d/%d/%d/%d, same-CU pairs %d, sharing a SIMD %d\n",
                   recs, cu_fold.size(), simd_hist[0], simd_hist[1], simd_hist[2], simd_hist[3], pairs, shared);
        }
        if (ks.rfind("tw7", 0) == 0 || shape) {
            // tw: waves 0..EW-1 evaluators, wave EW the fold wave; grid (g, B); a block
            // with blockIdx.x >= tiles has no work. Slots: see fit_tw_body.
            std::vector<long long> d(nd);
            (void)hipMemcpy(d.data(), diag, nd * 8, hipMemcpyDeviceToHost);
            const int EW = shape ? shape_ew : 7;
            const int QQ = shape ? sq : 63;
            const char* tg = std::getenv("MDG_TW_G");
            const int g = shape ? sg : tg ? std::max(1, std::atoi(tg)) : (3 * 2048 + 62) / 63;
            const int tiles = (3 * P + QQ - 1) / QQ, active = std::min(g, tiles);
            double ev[8] = {0}, fo[8] = {0};
            long long t0 = -1, t1 = 0;
            std::vector<long long> ends, starts;
            for (int s = 0; s < B; ++s)
                for (int b = 0; b < active; ++b) {
                    const long long* blk = &d[((size_t)(s * g + b) * 16) * 8];
                    long long life = 0;
                    for (int wv = 0; wv <= EW; ++wv) {
                        const long long* r = blk + wv * 8;
                        long long l = 0;
                        for (int i = 0; i < 7; ++i) { (wv < EW ? ev : fo)[i] += r[i]; l += r[i]; }
                        life = std::max(life, l);
                    }
                    const long long st = blk[7];
                    starts.push_back(st);
                    ends.push_back(st + life);
                    t0 = t0 < 0 ? st : std::min(t0, st);
                    t1 = std::max(t1, st + life);
                }
            const double nb = (double)B * active;
            printf("   %d blocks (%d per spectrum, %d tiles), span %.0f cycles\n", (int)nb, active, tiles, (double)(t1 - t0));
            printf("   evaluator wave avg: prologue %.0f  eval %.0f  barrier %.0f\n", ev[5] / nb / EW, ev[0] / nb / EW, ev[1] / nb / EW);
            printf("   fold wave avg: first-wait %.0f  fold %.0f  barrier %.0f  update %.0f\n", fo[6] / nb, fo[2] / nb, fo[3] / nb, fo[4] / nb);
            std::sort(starts.begin(), starts.end());
            std::sort(ends.begin(), ends.end());
            auto q = [&](std::vector<long long>& v, double f) { return (double)(v[(size_t)(f * (v.size() - 1))] - t0); };
            printf("   block start q0/25/50/75/100: %.0f %.0f %.0f %.0f %.0f\n", q(starts, 0), q(starts, .25), q(starts, .5), q(starts, .75), q(starts, 1));
            printf("   block end   q0/25/50/75/100: %.0f %.0f %.0f %.0f %.0f\n", q(ends, 0), q(ends, .25), q(ends, .5), q(ends, .75), q(ends, 1));
        } else if (k[0] == 't') {
            std::vector<long long> d(nd);
            (void)hipMemcpy(d.data(), diag, nd * 8, hipMemcpyDeviceToHost);
            const char* nm[5] = {"eval", "ev-barrier", "fold", "fold-barrier", "fold-other"};
            for (int wv = 0; wv < 4; ++wv) {
                printf("   wave %d (block 0):", wv);
                for (int i = 0; i < 5; ++i) printf(" %s=%lld", nm[i], d[wv * 8 + i]);
                printf("\n");
            }
        }
    }
    return 0;
}
