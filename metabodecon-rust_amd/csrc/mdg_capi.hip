// mdg_capi.hip -- host engine and C ABI of libmdgpu (see include/mdgpu.h).
//
// The engine replaces the body of Deconvoluter::deconvolute_spectrum
// (deconvoluter.rs:530-552) for a whole batch at once: every stage is one
// kernel launch over all B spectra, enqueued on one HIP stream with no host
// synchronisation between stages (the device API is graph-capturable).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <dlfcn.h>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <cstdlib>
#include <new>
#include <vector>

#include "../../include/mdgpu.h"
#include "mdg_common.hpp"
#include "mdg_kernels.hpp"

using namespace mdg;

namespace {

constexpr int kStages = 12;
enum Stage {
    ST_PREP = 0, ST_SMOOTH, ST_DETECT, ST_SELECT, ST_FIT_INIT, ST_FIT_SUP, ST_FIT_UPDATE,
    ST_RETAIN, ST_MSE, ST_MSE_REDUCE, ST_SUPVEC, ST_SYNTH
};

struct Pending {
    int stage;
    hipEvent_t a, b;
};

// roctx ranges around each pipeline stage (mdg_ctx_set_tracing / MDG_ROCTX=1), so a
// rocprofv3 trace (--marker-trace with --kernel-trace and --hip-trace) attributes
// every kernel to its stage through the host-side launch inside the range, without
// hipEvents in the stream. The roctx library is opened on first use (dlopen): a
// process that never traces does not load it.
const char* const kStageNames[kStages] = {"prep", "smooth", "detect", "select", "fit_init",
                                          "fit_superposition", "fit_update", "retain",
                                          "mse_superposition", "mse_reduce", "superposition_vec",
                                          "synth"};
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
};
const Roctx& roctx() {
    static const Roctx r = [] {
        Roctx t;
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            t.push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
            t.pop = (int (*)())dlsym(h, "roctxRangePop");
            if (!t.push || !t.pop) t.push = nullptr, t.pop = nullptr;
        }
        return t;
    }();
    return r;
}

struct Buffer {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace

struct mdg_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    // MDG_* switches, read when the context was created (mdg_ctx_reload_switches
    // re-reads them); the per-call paths read only this copy
    EngineSwitches sw;
    // latency mode (mdg_ctx_set_latency_mode): a B = 1 pipeline expects the GPU to
    // itself and takes the finer fit tiles (fit_choice)
    int latency = 1;
    // roctx ranges around the pipeline's stages (mdg_ctx_set_tracing, MDG_ROCTX=1)
    bool tracing = false;
    bool tracing_set = false;  // mdg_ctx_set_tracing was called (reloads keep its choice)
    std::mutex mu;
    // workspace arena
    Buffer arena;
    int ws_B = 0, ws_N = 0;
    Buffer chain;  // k_smooth_chain buffers (allocated on first use)
    // k_smooth_chain progress counters: one 128-byte slot per (spectrum, pass) at
    // a fixed place for every (B, P) the chain supports (B * P <= 2048), zeroed
    // once and left at zero by every run (k_flags), so no run has to clear them
    Buffer chain_flags;
    Buffer ign;  // the call's merged ignore regions (ppm pairs, device row)
    Buffer exact;  // MDG_OPTION_EXACT_MSE: B x N squared residuals (allocated on first use)
    std::vector<double> ign_last;  // the regions the device row holds now
    int ws_igcap = 0;  // ignore-region pairs per spectrum row of the arena
    // optimize_settings: per-spectrum overrides for the next run_pipeline, buffers
    const double* ovr_thr = nullptr;
    const int32_t* ovr_fit = nullptr;
    Buffer opt[12];
    // replayable pipelines of mdg_deconvolute_batch_device, keyed by every argument
    struct CachedGraph {
        std::vector<unsigned char> key;  // everything but the caller's array addresses
        hipGraph_t graph = nullptr;      // kept for its kernel nodes' argument copies
        hipGraphExec_t exec = nullptr;
        std::vector<hipGraphNode_t> knodes;  // kernel nodes, all (BatchArgs, Workspace, ...)
        BatchArgs cur;                   // the arguments the exec's nodes hold now
        const char* kernels[kStages];    // kernel names per stage of the captured pipeline
    };
    std::vector<CachedGraph> graphs;
    const char* stage_kernel[kStages] = {};  // kernels the last pipeline launched, per stage
    // bumped whenever the arena or the chain buffer is reallocated: cached graphs
    // bake their addresses and layout (ws_B/ws_N strides, counter offsets), so a
    // new generation drops every one of them before the next replay
    uint64_t ws_gen = 0, graphs_gen = 0;
    int last_B = 0, last_N = 0;  // shape of the last pipeline run
    bool last_smoothed = false;  // the last run used the moving average
    Workspace w{};
    // staging for the host-pointer API
    Buffer st_x, st_y, st_sb, st_out, st_cnt, st_mse, st_status, st_L, st_sup, st_flag;
    Buffer st_raw, st_desc;  // mdg_deconvolute_rows_i32: int32 rows and their descriptors
    // mdg_deconvolute_rows_i32 with page-locked rows: the chain launch decodes them
    // from host memory (BatchArgs::dec_rows); per-chunk flags, the call's generation
    Buffer dec_flags;
    int dec_gen = 0;
    bool dec_next = false;  // set by the upload: the next pipeline decodes the rows
    // batch_host: where this call's kernels read [sb][descriptors][row table] (the
    // page-locked scratch's device address, or st_sb after a copy when small_copy)
    const double* small_rd = nullptr;
    bool small_copy = true;
    // page-locked host ring for mdg_deconvolute_rows: the rows are gathered into a
    // slot and sent with one asynchronous DMA per slot (upload_rows)
    void* ring[2] = {nullptr, nullptr};
    size_t ring_bytes = 0;
    hipEvent_t ring_ev[2] = {nullptr, nullptr};
    bool ring_used[2] = {false, false};
    int ring_next = 0;  // the slot the next upload fills (uploads alternate slots)
    // page-locked scratch of the host-buffer calls: boundaries in, counts / statuses /
    // MSEs out (pageable small copies each cost a staged, host-blocking transfer)
    void* hsmall = nullptr;
    void* hsmall_dev = nullptr;  // its device address (null: kernels do not write it)
    size_t hsmall_bytes = 0;
    bool hsmall_busy = false;  // a call that failed midway may still have copies in flight
    size_t rows_guess = 0;     // batch_host: result rows fetched with the records (last count + 1/8)
    // profiling
    uint32_t profile_mask = 0;  // stages timed with hipEvents (bit = stage)
    std::vector<Pending> pending;
    std::vector<hipEvent_t> free_events;
    double stage_ms[kStages] = {0};
    uint64_t stage_launches[kStages] = {0};
};

namespace {

int hip_fail(hipError_t e) {
    if (e == hipErrorOutOfMemory) return MDG_ERR_OUT_OF_MEMORY;
    return MDG_ERR_HIP;
}

#define HIPCHK(expr)                              \
    do {                                          \
        hipError_t _e = (expr);                   \
        if (_e != hipSuccess) return hip_fail(_e); \
    } while (0)

int ensure(Buffer& b, size_t bytes) {
    if (b.bytes >= bytes) return MDG_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    size_t sz = std::max<size_t>(bytes, 256);
    HIPCHK(hipMalloc(&b.p, sz));
    b.bytes = sz;
    return MDG_OK;
}

hipEvent_t get_event(mdg_ctx* c) {
    if (!c->free_events.empty()) {
        hipEvent_t e = c->free_events.back();
        c->free_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// RAII stage timer: records events around a launch when profiling is on.
struct StageTimer {
    mdg_ctx* c;
    int stage;
    hipEvent_t a = nullptr;
    bool range = false;
    StageTimer(mdg_ctx* c_, int s) : c(c_), stage(s) {
        if (c->tracing && roctx().push) range = roctx().push(kStageNames[stage]) >= 0;
        if ((c->profile_mask >> stage) & 1u) {
            a = get_event(c);
            if (a) (void)hipEventRecord(a, c->stream);
        }
    }
    ~StageTimer() {
        if (range) roctx().pop();
        if (a) {
            hipEvent_t b = get_event(c);
            if (b) {
                (void)hipEventRecord(b, c->stream);
                c->pending.push_back({stage, a, b});
            }
        }
    }
};

void drain_timers(mdg_ctx* c) {
    if (c->pending.empty()) return;
    (void)hipStreamSynchronize(c->stream);
    for (auto& p : c->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            c->stage_ms[p.stage] += ms;
            c->stage_launches[p.stage] += 1;
        }
        c->free_events.push_back(p.a);
        c->free_events.push_back(p.b);
    }
    c->pending.clear();
}

size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

// ---- page-locked host blocks (mdg_host_alloc) ----------------------------------
// Blocks are carved from 64 MiB slabs (hipHostMalloc, portable) and kept on a free
// list per size when released; the slabs stay pinned for the process's life. The
// live map answers "is this row page-locked" for the host-buffer entry points,
// which then DMA straight from the caller's rows (upload_rows).
struct PinnedPool {
    std::mutex mu;
    std::map<uintptr_t, size_t> live;                  // block start -> bytes
    std::map<size_t, std::vector<void*>> free_blocks;  // bytes -> released blocks
    char* cur = nullptr;                                // bump pointer in the newest slab
    size_t cur_left = 0;
    size_t pinned = 0;                                  // bytes of all slabs
    bool uva = true;  // every slab's device address is its host address (kernels may read the rows)
};
PinnedPool& pinned_pool() {
    static PinnedPool* p = new PinnedPool();  // never destroyed: blocks may be freed at exit
    return *p;
}
constexpr size_t kPinnedSlab = 64u << 20;

// The environment, read in these two places only: the engine switches when a
// context is created (or mdg_ctx_reload_switches), and the pinned-memory cap once per
// process at its first page-locked allocation.
size_t env_pinned_max() {
    const char* e = std::getenv("MDGPU_PINNED_MAX");
    return e && *e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)8 << 30;
}

size_t pinned_limit() {
    static const size_t lim = env_pinned_max();
    return lim;
}

int pinned_alloc(int device, size_t bytes, void** out) {
    const size_t sz = (bytes + 4095) & ~size_t(4095);
    PinnedPool& P = pinned_pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.free_blocks.find(sz);
    if (it != P.free_blocks.end() && !it->second.empty()) {
        void* p = it->second.back();
        it->second.pop_back();
        P.live[(uintptr_t)p] = sz;
        *out = p;
        return MDG_OK;
    }
    if (P.cur_left < sz) {
        const size_t slab = std::max(sz, kPinnedSlab);
        if (P.pinned + slab > pinned_limit()) return MDG_ERR_OUT_OF_MEMORY;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MDG_ERR_NO_DEVICE;
        if (device < 0 || device >= n) return MDG_ERR_NO_DEVICE;
        int prev = 0;
        HIPCHK(hipGetDevice(&prev));
        HIPCHK(hipSetDevice(device));
        void* s = nullptr;
        const hipError_t e = hipHostMalloc(&s, slab, hipHostMallocPortable);
        (void)hipSetDevice(prev);
        if (e != hipSuccess) return MDG_ERR_OUT_OF_MEMORY;
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, s, 0) != hipSuccess || dp != s) P.uva = false;
        if (P.cur_left) P.free_blocks[P.cur_left].push_back(P.cur);  // the old slab's tail
        P.cur = (char*)s;
        P.cur_left = slab;
        P.pinned += slab;
    }
    void* p = P.cur;
    P.cur += sz;
    P.cur_left -= sz;
    P.live[(uintptr_t)p] = sz;
    *out = p;
    return MDG_OK;
}

int pinned_free(void* p) {
    if (!p) return MDG_OK;
    PinnedPool& P = pinned_pool();
    std::lock_guard<std::mutex> g(P.mu);
    auto it = P.live.find((uintptr_t)p);
    if (it == P.live.end()) return MDG_INVALID_ARGUMENT;
    P.free_blocks[it->second].push_back(p);
    P.live.erase(it);
    return MDG_OK;
}

// every [rows[i], rows[i] + bytes) inside one live page-locked block (and, with
// device_readable, the blocks readable by kernels at their host addresses)
bool pinned_rows(const void* const* rows, size_t b, size_t bytes, bool device_readable = false) {
    PinnedPool& P = pinned_pool();
    std::lock_guard<std::mutex> g(P.mu);
    if (P.live.empty() || (device_readable && !P.uva)) return false;
    for (size_t i = 0; i < b; ++i) {
        const uintptr_t a = (uintptr_t)rows[i];
        auto it = P.live.upper_bound(a);
        if (it == P.live.begin()) return false;
        --it;
        if (a + bytes > it->first + it->second) return false;
    }
    return true;
}

int ensure_workspace(mdg_ctx* c, int B, int N, int n_ignore) {
    const int igcap = std::max(kIgnoreRow, (n_ignore + kIgnoreRow - 1) / kIgnoreRow * kIgnoreRow);
    if (!(B <= c->ws_B && N <= c->ws_N && igcap <= c->ws_igcap && c->arena.p)) {
        const int nB = std::max(B, c->ws_B), nN = std::max(N, c->ws_N);
        const int nIg = std::max(igcap, c->ws_igcap);
        const size_t W = (size_t)(nN + 63) / 64;
        const size_t capD = (size_t)nN / 2 + 2;
        const size_t Bs = (size_t)nB;
        size_t off = 0;
        auto take = [&](size_t bytes) { size_t o = off; off = align256(off + bytes); return o; };
        const size_t o_smooth = take(Bs * nN * 8), o_tmp0 = take(Bs * nN * 8), o_tmp1 = take(Bs * nN * 8);
        const size_t o_masks = take(Bs * 3 * W * 8);
        const size_t o_dl = take(Bs * capD * 4), o_dc = take(Bs * capD * 4), o_dr = take(Bs * capD * 4);
        const size_t o_sl = take(Bs * capD * 4), o_sc = take(Bs * capD * 4), o_sr = take(Bs * capD * 4);
        const size_t o_scores = take(Bs * capD * 8);
        const size_t o_params = take(Bs * capD * 24), o_kept = take(Bs * capD * 24);
        const size_t o_st = take(Bs * capD * 48);
        const size_t o_rx = take(Bs * capD * 24), o_ry = take(Bs * capD * 24), o_ratio = take(Bs * capD * 24);
        const size_t o_msep = take(Bs * kMseMaxParts * 8);
        const size_t o_sfr = take(Bs * 16);
        const size_t o_sbi = take(Bs * 16);
        const size_t o_ig = take(Bs * 2 * (size_t)nIg * 8), o_igc = take(Bs * ((size_t)nIg + 2) * 8);
        const size_t o_nig = take(Bs * 4), o_panic = take(Bs * 4), o_status = take(Bs * 4);
        const size_t o_dcnt = take(Bs * 4), o_scnt = take(Bs * 4), o_kcnt = take(Bs * 4);
        const size_t o_xok = take(Bs * 4), o_unsafe = take(Bs * 16), o_uk = take(Bs * 4);
        const size_t o_pcnt = take(Bs * 2 * ((W + kPkSlotWords - 1) / kPkSlotWords) * 4);
        const size_t o_mcnt = take(Bs * 4);

        if (c->arena.p) (void)hipFree(c->arena.p);
        c->arena.p = nullptr;
        c->arena.bytes = 0;
        HIPCHK(hipMalloc(&c->arena.p, off));
        c->arena.bytes = off;
        char* base = (char*)c->arena.p;
        Workspace& w = c->w;
        w.smooth = (double*)(base + o_smooth);
        w.tmp0 = (double*)(base + o_tmp0);
        w.tmp1 = (double*)(base + o_tmp1);
        w.masks = (uint64_t*)(base + o_masks);
        w.det_l = (int32_t*)(base + o_dl);
        w.det_c = (int32_t*)(base + o_dc);
        w.det_r = (int32_t*)(base + o_dr);
        w.sel_l = (int32_t*)(base + o_sl);
        w.sel_c = (int32_t*)(base + o_sc);
        w.sel_r = (int32_t*)(base + o_sr);
        w.scores = (double*)(base + o_scores);
        w.params = (double*)(base + o_params);
        w.kept = (double*)(base + o_kept);
        w.stencil = (double*)(base + o_st);
        w.rx = (double*)(base + o_rx);
        w.ry = (double*)(base + o_ry);
        w.ratio = (double*)(base + o_ratio);
        w.mse_part = (double*)(base + o_msep);
        w.sfr_stats = (double*)(base + o_sfr);
        w.sbi = (int64_t*)(base + o_sbi);
        w.ig = (int64_t*)(base + o_ig);
        w.ig_cum = (int64_t*)(base + o_igc);
        w.ig_cap = nIg;
        w.n_ig = (int32_t*)(base + o_nig);
        w.mse_panic = (int32_t*)(base + o_panic);
        w.status = (int32_t*)(base + o_status);
        w.det_count = (int32_t*)(base + o_dcnt);
        w.sel_count = (int32_t*)(base + o_scnt);
        w.kept_count = (int32_t*)(base + o_kcnt);
        w.x_ok = (int32_t*)(base + o_xok);
        w.unsafe = (int32_t*)(base + o_unsafe);
        w.unsafe_kept = (int32_t*)(base + o_uk);
        w.peak_cnt = (int32_t*)(base + o_pcnt);
        w.mse_done = (int32_t*)(base + o_mcnt);
        // k_mse_local's arrival counters start (and are always left) at zero
        HIPCHK(hipMemset(w.mse_done, 0, Bs * 4));

        c->ws_B = nB;
        c->ws_N = nN;
        c->ws_igcap = nIg;
        ++c->ws_gen;
    }
    return MDG_OK;
}

// the exact-order MSE's residual rows (B x N doubles), bumping the workspace
// generation when the buffer moves (cached graphs bake its address)
int ensure_exact(mdg_ctx* c, int B, int N) {
    const void* old = c->exact.p;
    const int rc = ensure(c->exact, (size_t)B * (size_t)N * 8);
    if (c->exact.p != old) ++c->ws_gen;
    return rc;
}

// ensure() for the chain smoother buffer, bumping the workspace generation when
// the buffer moves
int ensure_chain(mdg_ctx* c, size_t bytes) {
    const void* old = c->chain.p;
    int rc = ensure(c->chain, bytes);
    if (c->chain.p != old) ++c->ws_gen;
    if (rc == MDG_OK && !c->chain_flags.p) {
        rc = ensure(c->chain_flags, (size_t)2048 * 128);
        if (rc == MDG_OK) HIPCHK(hipMemsetAsync(c->chain_flags.p, 0, c->chain_flags.bytes, c->stream));
        ++c->ws_gen;
    }
    return rc;
}

void destroy_graph(mdg_ctx::CachedGraph& ge) {
    (void)hipGraphExecDestroy(ge.exec);
    (void)hipGraphDestroy(ge.graph);
}

void drop_graphs(mdg_ctx* c) {
    for (auto& ge : c->graphs) destroy_graph(ge);
    c->graphs.clear();
}

int validate_common(const mdg_settings* s, size_t n_ignore, const double* ignore) {
    if (!s) return MDG_INVALID_ARGUMENT;
    int v = mdg_settings_validate(s);
    if (v) return v;
    if (n_ignore > (size_t)(INT32_MAX / 4)) return MDG_INVALID_ARGUMENT;
    if (n_ignore > 0 && !ignore) return MDG_INVALID_ARGUMENT;
    return MDG_OK;
}

// Runs the whole pipeline for a device-resident batch. Caller holds c->mu.
int run_pipeline(mdg_ctx* c, BatchArgs& a, const mdg_settings* s) {
    a.det_only = s->selector == MDG_SELECT_DETECTOR_ONLY;
    int rc = ensure_workspace(c, a.B, a.N, a.n_ignore);
    if (rc) return rc;
    // Row strides follow the current shape; the arena is sized for the largest
    // (B, N) seen so far, so every current-shape row fits.
    Workspace w = c->w;
    w.W = (a.N + 63) / 64;
    w.capD = a.N / 2 + 2;
    c->last_B = a.B;
    c->last_N = a.N;
    hipStream_t st = c->stream;
    const bool ma = s->smoother == MDG_SMOOTH_MOVING_AVERAGE;
    c->last_smoothed = ma;
    for (auto& k : c->stage_kernel) k = nullptr;
    const char** kn = c->stage_kernel;
    if (ma) {
        w.smooth_ptr = w.smooth;
        w.smooth_stride = a.N;
    } else {
        w.smooth_ptr = a.y;
        w.smooth_stride = a.y_stride;
    }
    const int det_only = s->selector == MDG_SELECT_DETECTOR_ONLY;
    // the term-fold fit kernel also updates the stencils; its parameter versions
    // alternate between params and the (then unused) ratio buffer
    const EngineSwitches& sw = c->sw;
    const bool fused = fit_sup_fused(a, sw);
    w.params_alt = fused ? w.ratio : nullptr;
    w.fit_iters = (int)s->fit_iterations;
    const int gfit = sw.gfit;  // k_fit_sup workgroups per spectrum (3 * 2048 / 256; MDG_GFIT: tuning)
    const int gupd = std::max(1, std::min(16, 1024 / std::max(1, a.B)));
    const int nparts = mse_nparts(a, sw);
    // chain smoother buffers: raw sums of every pass, scaled outputs of passes
    // 0..P-2 and one 128-byte progress counter per (spectrum, pass)
    w.thr_s = c->ovr_thr;
    w.fit_iters_s = c->ovr_fit;
    w.chain_P = 0;
    w.chain_raw = w.chain_tmp = nullptr;
    w.chain_flags = nullptr;
    if (ma) {
        const int P = (int)s->smooth_iterations, ws = (int)s->smooth_window;
        if ((sw.smooth == EngineSwitches::SM_DEFAULT || sw.smooth == EngineSwitches::SM_CHAIN) &&
            !smooth_uses_small(a, P, ws, sw) && chain_supported(a.B, a.N, P, ws) &&
            ensure_chain(c, chain_bytes(a.B, a.N, ws, P)) == MDG_OK) {
            const int64_t L = chain_stride_for(a.N, ws);
            char* base = (char*)c->chain.p;
            w.chain_stride = L;
            w.chain_raw = (double*)base;
            w.chain_tmp = w.chain_raw + (size_t)P * a.B * L;
            w.chain_flags = (int32_t*)c->chain_flags.p;
            w.chain_P = P;
        }
    }
#ifdef MDG_DIAG
    // diagnostic builds only (make diag; tools/stream_diag.py): MDG_DIAG_SKIP=smooth,mse
    // skips those stages (their outputs are stale, results wrong); MDG_DIAG_DUP=prep,
    // smooth,detect,select,retain,mse launches those stages twice (each is idempotent;
    // smooth adds a k_flags), for their marginal cost in stream mode
    const bool skip_smooth = std::strstr(sw.diag_skip, "smooth"), skip_mse = std::strstr(sw.diag_skip, "mse");
    auto reps = [&](const char* stage) { return std::strstr(sw.diag_dup, stage) ? 2 : 1; };
#else
    constexpr bool skip_smooth = false, skip_mse = false;
    auto reps = [](const char*) { return 1; };
#endif
    const int sm_it = (int)s->smooth_iterations, sm_ws = (int)s->smooth_window;
    const bool panic_shape = ma && (int64_t)(s->smooth_window / 2) > a.N;
    // the chain smoother does k_prep's work itself (MDG_PREP=separate: not)
    const bool fused_prep = ma && !panic_shape && !skip_smooth && !sw.prep_separate && reps("prep") == 1 &&
                            smooth_fuses_prep(a, w, sm_it, sm_ws, sw);
    if (a.dec_rows) {
        // rows still in host memory (mdg_deconvolute_rows_i32): the chain launch
        // decodes them while it smooths (flags of this call's generation), any other
        // smoother after a decode launch of their own
        const size_t need = (size_t)a.B * kDecChunks * 4;
        if (c->dec_flags.bytes < need || c->dec_gen >= INT32_MAX - 1) {
            if ((rc = ensure(c->dec_flags, need))) return rc;
            HIPCHK(hipMemsetAsync(c->dec_flags.p, 0, c->dec_flags.bytes, st));
            c->dec_gen = 0;
        }
        a.dec_gen = ++c->dec_gen;
        w.dec_flags = (int32_t*)c->dec_flags.p;
        // the chain launch's hand-off needs rows of whole 128-byte lines (batch_host
        // pads them; chain_decode): other rows are decoded by a launch of their own
        const bool lines_owned = a.y_stride % kDecRowAlign == 0 && ((uintptr_t)a.y & 127) == 0;
        if (!fused_prep || !lines_owned) {
            StageTimer t(c, ST_PREP);
            launch_decode_rows_zc(a, st);
            a.dec_rows = nullptr;  // decoded: the smoother reads y (the prep still takes the axis from dec_desc)
        }
    }
    if (!fused_prep) {
        StageTimer t(c, ST_PREP);
        for (int r = reps("prep"); r > 0; --r) launch_prep(a, w, st);
        kn[ST_PREP] = "k_prep";
    }
#ifdef MDG_DIAG
    for (int k = sw.diag_pad; k > 0; --k) launch_diag_nop(a, w, sw, st);
#endif
    if (ma) {
        if (panic_shape) {
            // moving_average.rs:63 `values_len - self.right` underflows: reference panics
            std::vector<int32_t> pan(a.B, MDG_REFERENCE_PANIC);
            HIPCHK(hipMemcpyAsync(w.status, pan.data(), sizeof(int32_t) * a.B, hipMemcpyHostToDevice, st));
            HIPCHK(hipStreamSynchronize(st));
        } else if (!skip_smooth) {
            StageTimer t(c, ST_SMOOTH);
            if (reps("smooth") == 2) {  // k_flags resets the chain's progress counters
                launch_smooth(a, w, sm_it, sm_ws, sw, st, fused_prep ? 1 : 0);
                launch_flags(a, w, st);
            }
            kn[ST_SMOOTH] = launch_smooth(a, w, sm_it, sm_ws, sw, st, fused_prep ? 1 : 0);
        }
    }
    // small spectra: the detection runs inside the selection's workgroup
    const bool det_fused = detect_fused(a, det_only, sw);
    if (!det_fused) {
        StageTimer t(c, ST_DETECT);
        for (int r = reps("detect"); r > 0; --r) {
            if (!peaks_fuse_flags(a, w, sw)) launch_flags(a, w, st);
            kn[ST_DETECT] = launch_peaks(a, w, det_only, sw, st);
        }
    }
    {
        StageTimer t(c, ST_SELECT);
        for (int r = reps("select"); r > 0; --r)
            kn[ST_SELECT] = launch_select(a, w, det_only, s->threshold, st, det_fused);
        if (det_fused) kn[ST_DETECT] = kn[ST_SELECT];
    }
    const bool small_fit = fit_is_small(a, sw);
    if (small_fit) {  // every iteration in one launch
        StageTimer t(c, ST_FIT_SUP);
        kn[ST_FIT_SUP] = launch_fit_small(a, w, st);
    }
    for (uint32_t it = 0; it < (small_fit ? 0u : s->fit_iterations); ++it) {
        {
            StageTimer t(c, ST_FIT_SUP);
            kn[ST_FIT_SUP] = launch_fit_sup(a, w, gfit, (int)it, sw, st);
        }
        if (!fused) {
            StageTimer t(c, ST_FIT_UPDATE);
            launch_fit_update(a, w, gupd, (int)it, st);
            kn[ST_FIT_UPDATE] = "k_fit_update";
        }
    }
    // k_mse_local compacts the retained Lorentzians itself; k_retain only when the MSE
    // is skipped or the retain duplicated (diagnostic builds)
    if (skip_mse || reps("retain") == 2) {
        StageTimer t(c, ST_RETAIN);
        launch_retain(a, w, st);
        kn[ST_RETAIN] = "k_retain<1024>";
    }
    if (!skip_mse) {
        StageTimer t(c, ST_MSE);
        for (int r = reps("mse"); r > 0; --r) kn[ST_MSE] = launch_mse(a, w, nparts, sw, st);
    }
    if (!skip_mse && (s->options & MDG_OPTION_EXACT_MSE)) {
        // the reference's summation order (deconvoluter.rs:828-862), over the retained
        // Lorentzians k_mse_local compacted; replaces its MSE
        if ((rc = ensure_exact(c, a.B, a.N))) return rc;
        StageTimer t(c, ST_MSE_REDUCE);
        launch_mse_exact_batch(a, w, (double*)c->exact.p, a.N, st);
        kn[ST_MSE_REDUCE] = "k_mse_exact_res+k_mse_exact_fold";
    }
    HIPCHK(hipGetLastError());
    return MDG_OK;
}

// The per-call arguments. The ignore regions (host memory, any number of merged
// pairs) go to the context's device row on its stream, ahead of the pipeline, so
// the kernels' argument block stays small (every launch copies it). The row is
// uploaded only when the regions differ from the ones it holds (the usual caller
// passes the same Deconvoluter's regions every call): no host-to-device copy, and
// no pageable-copy stall, in a stream of calls.
int fill_args(mdg_ctx* c, BatchArgs& a, size_t b, size_t n, const double* x, size_t xs, const double* y,
              size_t ys, const double* sb, const double* ignore, size_t n_ignore, double* out,
              size_t cap, int32_t* cnt, double* mse, int32_t* status) {
    std::memset(&a, 0, sizeof(a));  // padding too: graph keys compare the bytes
    a.B = (int)b;
    a.N = (int)n;
    a.x = x;
    a.x_stride = (int64_t)xs;
    a.y = y;
    a.y_stride = (int64_t)ys;
    a.sb = sb;
    a.sb_step = 2;
    a.n_ignore = (int)n_ignore;
    a.latency = c->latency;
    a.ignore = nullptr;
    if (n_ignore > 0) {
        const size_t cnt = 2 * n_ignore;
        const bool same = c->ign.p && c->ign_last.size() == cnt &&
                          std::memcmp(c->ign_last.data(), ignore, cnt * sizeof(double)) == 0;
        if (!same) {
            const void* old = c->ign.p;
            int rc = ensure(c->ign, std::max<size_t>(cnt, 2 * kIgnoreRow) * sizeof(double));
            if (rc) return rc;
            if (c->ign.p != old) ++c->ws_gen;  // graphs bake the row's address
            HIPCHK(hipMemcpyAsync(c->ign.p, ignore, cnt * sizeof(double), hipMemcpyHostToDevice, c->stream));
            c->ign_last.assign(ignore, ignore + cnt);
        }
        a.ignore = (const double*)c->ign.p;
    }
    a.out = out;
    a.cap = (int)std::min<size_t>(cap, (size_t)INT32_MAX);
    a.out_count = cnt;
    a.out_mse = mse;
    a.out_status = status;
    return MDG_OK;
}

}  // namespace

// =====================================================================================
// C ABI
// =====================================================================================
extern "C" {

int mdg_abi_version(void) { return MDG_ABI_VERSION; }

#ifndef MDG_SOURCE_HASH
#define MDG_SOURCE_HASH "unknown"
#endif
#ifndef MDG_FLAGS_HASH
#define MDG_FLAGS_HASH "unknown"
#endif
// build provenance: the Makefile's sha256 (16 hex digits) of the engine sources this
// library was compiled from, and of its compile flags; metabodecon/_native.py refuses
// a library whose source hash does not match the tree next to it
const char* mdg_build_info(void) {
    return "src=" MDG_SOURCE_HASH " flags=" MDG_FLAGS_HASH " compiler=" __clang_version__;
}

const char* mdg_strerror(int st) {
    // messages of deconvolution/error.rs:105-168 where the kind exists there
    switch (st) {
        case MDG_OK: return "ok";
        case MDG_NO_PEAKS_DETECTED: return "no peaks detected in the spectrum";
        case MDG_EMPTY_SIGNAL_REGION: return "no peaks found in the signal region of the spectrum";
        case MDG_EMPTY_SIGNAL_FREE_REGION: return "no peaks found in the signal-free region of the spectrum";
        case MDG_INVALID_SMOOTHING: return "invalid smoothing settings";
        case MDG_INVALID_SELECTION: return "invalid selection settings";
        case MDG_INVALID_FITTING: return "invalid fitting settings";
        case MDG_INVALID_IGNORE_REGION: return "invalid ignore region";
        case MDG_INVALID_ARGUMENT: return "invalid argument";
        case MDG_CAPACITY: return "output capacity too small";
        case MDG_REFERENCE_PANIC: return "input on which the reference implementation panics";
        case MDG_ERR_HIP: return "HIP runtime error";
        case MDG_ERR_NO_DEVICE: return "no HIP device";
        case MDG_ERR_OUT_OF_MEMORY: return "device out of memory";
        default: return "unknown status";
    }
}

void mdg_settings_default(mdg_settings* s) {
    if (!s) return;
    std::memset(s, 0, sizeof(*s));
    s->smoother = MDG_SMOOTH_MOVING_AVERAGE;  // smoother.rs:58-65
    s->smooth_iterations = 3;
    s->smooth_window = 3;
    s->selector = MDG_SELECT_NOISE_SCORE;  // selector.rs:59-66
    s->scoring = MDG_SCORE_MINIMUM_SUM;
    s->threshold = 5.0;
    s->fitter = MDG_FIT_ANALYTICAL;  // fitter.rs:59-63
    s->fit_iterations = 10;
}

int mdg_settings_validate(const mdg_settings* s) {
    if (!s) return MDG_INVALID_ARGUMENT;
    if (s->smoother == MDG_SMOOTH_MOVING_AVERAGE) {  // smoother.rs:84-100
        if (s->smooth_iterations == 0 || s->smooth_window <= 1) return MDG_INVALID_SMOOTHING;
    } else if (s->smoother != MDG_SMOOTH_IDENTITY) {
        return MDG_INVALID_SMOOTHING;
    }
    if (s->selector == MDG_SELECT_NOISE_SCORE) {  // selector.rs:85-98
        if (s->threshold <= 0.0 || !std::isfinite(s->threshold) || s->scoring != MDG_SCORE_MINIMUM_SUM)
            return MDG_INVALID_SELECTION;
    } else if (s->selector != MDG_SELECT_DETECTOR_ONLY) {
        return MDG_INVALID_SELECTION;
    }
    if (s->fitter != MDG_FIT_ANALYTICAL || s->fit_iterations == 0) return MDG_INVALID_FITTING;  // fitter.rs:80-90
    if (s->options & ~(int32_t)MDG_OPTION_EXACT_MSE) return MDG_INVALID_ARGUMENT;
    return MDG_OK;
}

int mdg_ignore_region_add(double* r, size_t n, size_t cap, double a, double b, size_t* n_out) {
    // deconvoluter.rs:438-472
    if (!std::isfinite(a) || !std::isfinite(b) || std::fabs(a - b) < kCheckPrecision)
        return MDG_INVALID_IGNORE_REGION;
    if (!r || !n_out || n + 1 > cap) return MDG_INVALID_ARGUMENT;
    r[2 * n] = std::fmin(a, b);
    r[2 * n + 1] = std::fmax(a, b);
    ++n;
    for (size_t i = 1; i < n; ++i) {  // sort by start
        const double s0 = r[2 * i], s1 = r[2 * i + 1];
        size_t j = i;
        while (j > 0 && r[2 * (j - 1)] > s0) {
            r[2 * j] = r[2 * (j - 1)];
            r[2 * j + 1] = r[2 * (j - 1) + 1];
            --j;
        }
        r[2 * j] = s0;
        r[2 * j + 1] = s1;
    }
    for (;;) {  // merge overlapping / adjacent (within CHECK_PRECISION) neighbours
        size_t pos = n;
        for (size_t i = 0; i + 1 < n; ++i) {
            if (r[2 * (i + 1)] < r[2 * i + 1] ||
                std::fabs(r[2 * i + 1] - r[2 * (i + 1)]) < kCheckPrecision) {
                pos = i;
                break;
            }
        }
        if (pos == n) break;
        const double lo = std::fmin(r[2 * pos], r[2 * (pos + 1)]);
        const double hi = std::fmax(r[2 * pos + 1], r[2 * (pos + 1) + 1]);
        r[2 * pos] = lo;
        r[2 * pos + 1] = hi;
        for (size_t i = pos + 1; i + 1 < n; ++i) {
            r[2 * i] = r[2 * (i + 1)];
            r[2 * i + 1] = r[2 * (i + 1) + 1];
        }
        --n;
    }
    *n_out = n;
    return MDG_OK;
}

int mdg_synth_lorentzians(uint64_t seed, size_t n_peaks, double lo, double hi, mdg_lorentzian* out) {
    return mdg_synth_lorentzians_hw(seed, n_peaks, lo, hi, 1.0, out);
}

int mdg_synth_lorentzians_hw(uint64_t seed, size_t n_peaks, double lo, double hi, double hw_scale,
                             mdg_lorentzian* out) {
    if (!out && n_peaks) return MDG_INVALID_ARGUMENT;
    const uint64_t key = stream_key(seed, kStreamPeaks);
    const double delta = (hi - lo) / (double)n_peaks;
    for (size_t p = 0; p < n_peaks; ++p) {
        const double u1 = u53(draw(key, 3 * p)), u2 = u53(draw(key, 3 * p + 1)),
                     u3 = u53(draw(key, 3 * p + 2));
        const double maxp = lo + ((double)p + 0.5) * delta + (u1 - 0.5) * 0.5 * delta;
        const double hw = (3.0e-4 + u2 * 5.0e-4) * hw_scale;  // x 1.0 is exact
        const double amp = std::pow(10.0, 4.5 + 3.5 * u3);
        const double hw2 = hw * hw;
        out[p].sfhw = amp * hw2;
        out[p].hw2 = hw2;
        out[p].maxp = maxp;
    }
    return MDG_OK;
}

int mdg_synth_noise(uint64_t seed, size_t n, double sigma, double* out) {
    if (!out && n) return MDG_INVALID_ARGUMENT;
    const uint64_t key = stream_key(seed, kStreamNoise);
    for (size_t i = 0; i < n; ++i) out[i] = synth_noise(key, i, sigma);
    return MDG_OK;
}

int mdg_device_count(int* count) {
    if (!count) return MDG_INVALID_ARGUMENT;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return MDG_OK;
}

int mdg_host_alloc(int device, size_t bytes, void** out) {
    if (!out || bytes == 0) return MDG_INVALID_ARGUMENT;
    *out = nullptr;
    return pinned_alloc(device, bytes, out);
}

int mdg_host_free(void* p) { return pinned_free(p); }

}  // extern "C"

EngineSwitches mdg::read_engine_switches() {
    EngineSwitches w;
    auto str = [](const char* name) -> std::string {
        const char* v = std::getenv(name);
        return v ? std::string(v) : std::string();
    };
    auto num = [&](const char* name, int dflt) {
        const std::string v = str(name);
        return v.empty() ? dflt : std::atoi(v.c_str());
    };
    auto copy = [](char* dst, size_t cap, const std::string& v) {
        std::memset(dst, 0, cap);
        std::strncpy(dst, v.c_str(), cap - 1);
    };
    const std::string sm = str("MDG_SMOOTH");
    w.smooth = sm.empty() ? EngineSwitches::SM_DEFAULT
               : sm == "chain" ? EngineSwitches::SM_CHAIN
               : sm == "pipe"  ? EngineSwitches::SM_PIPE
               : sm == "generic" ? EngineSwitches::SM_GENERIC
               : sm == "small" ? EngineSwitches::SM_SMALL
                                 : EngineSwitches::SM_OTHER;
    w.chain_excl = str("MDG_CHAIN_EXCL").substr(0, 1) != "0";
    w.chain_l2ahead = std::max(0, num("MDG_CHAIN_L2AHEAD", 0));
    const std::string pk = str("MDG_PEAKS");
    w.peaks = pk.empty() ? 0 : pk == "fine" ? 1 : 2;
    const std::string dt = str("MDG_DETECT");
    w.detect = dt == "separate" ? 1 : dt == "fused" ? 2 : 0;
    const std::string f = str("MDG_FITSUP");
    copy(w.fitsup, sizeof(w.fitsup), "");
    if (f == "tf" || f == "tf12" || f == "tw7" || f == "tw3s" || f == "twf" || f == "twf1" || f == "twf3s" ||
        f == "small" ||
        f == "plain")
        copy(w.fitsup, sizeof(w.fitsup), f);
#ifdef MDG_DIAG
    if (f == "mfma") copy(w.fitsup, sizeof(w.fitsup), f);  // the configs[2] experiment (not bit-exact)
#endif
    w.tw_g = std::max(0, num("MDG_TW_G", 0));
    if (!str("MDG_TW_G").empty()) w.tw_g = std::max(1, w.tw_g);
    w.gfit = std::max(1, num("MDG_GFIT", 24));
    w.mse_npt = str("MDG_MSE_NPT").empty() ? 0 : (num("MDG_MSE_NPT", 2) == 4 ? 4 : 2);
    w.mse_parts = str("MDG_MSE_PARTS").empty() ? 0 : std::max(1, num("MDG_MSE_PARTS", 1));
    w.mse_pk = str("MDG_MSE_PK").empty() ? 0 : (num("MDG_MSE_PK", 20) == 30 ? 30 : 20);
    w.mse_nearcap = str("MDG_MSE_NEARCAP").empty() ? -1 : std::max(0, num("MDG_MSE_NEARCAP", 0));
    w.prep_separate = str("MDG_PREP") == "separate";
    w.graphs = str("MDG_GRAPHS") == "1";
    w.host_direct = str("MDG_HOST_DIRECT").substr(0, 1) != "0";
    w.dec_overlap = str("MDG_DEC_OVERLAP").substr(0, 1) != "0";
    w.roctx = str("MDG_ROCTX") == "1";
#ifdef MDG_DIAG
    copy(w.diag_skip, sizeof(w.diag_skip), str("MDG_DIAG_SKIP"));
    copy(w.diag_dup, sizeof(w.diag_dup), str("MDG_DIAG_DUP"));
    w.diag_pad = std::max(0, num("MDG_DIAG_PAD", 0));
    w.diag_pad_small = !str("MDG_DIAG_PAD_SMALL").empty();
    w.diag_pad_wgs = std::max(0, num("MDG_DIAG_PAD_WGS", 0));
#else
    copy(w.diag_skip, sizeof(w.diag_skip), "");
    copy(w.diag_dup, sizeof(w.diag_dup), "");
#endif
    return w;
}

// the device's compute units (the batch-wide fit's grid; 256 on MI355X)
static int device_cus(int device) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
        cus = 256;
    return cus;
}

extern "C" {

int mdg_ctx_create(int device, mdg_ctx** out) {
    if (!out) return MDG_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MDG_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return MDG_ERR_NO_DEVICE;
    HIPCHK(hipSetDevice(device));
    mdg_ctx* c = new (std::nothrow) mdg_ctx();
    if (!c) return MDG_ERR_OUT_OF_MEMORY;
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hip_fail(e);
    }
    c->stream = c->own;
    c->sw = read_engine_switches();
    c->sw.cus = device_cus(device);
    c->tracing = c->sw.roctx != 0;
    *out = c;
    return MDG_OK;
}

int mdg_ctx_destroy(mdg_ctx* c) {
    if (!c) return MDG_OK;
    {
        std::lock_guard<std::mutex> g(c->mu);
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        for (auto& p : c->pending) {
            (void)hipEventDestroy(p.a);
            (void)hipEventDestroy(p.b);
        }
        for (auto e : c->free_events) (void)hipEventDestroy(e);
        drop_graphs(c);
        for (Buffer& b : c->opt)
            if (b.p) (void)hipFree(b.p);
        for (Buffer* b : {&c->arena, &c->chain, &c->chain_flags, &c->ign, &c->exact, &c->st_x, &c->st_y, &c->st_sb, &c->st_out, &c->st_cnt,
                          &c->st_mse, &c->st_status, &c->st_L, &c->st_sup, &c->st_flag, &c->st_raw,
                          &c->st_desc})
            if (b->p) (void)hipFree(b->p);
        for (int k = 0; k < 2; ++k) {
            if (c->ring[k]) (void)hipHostFree(c->ring[k]);
            if (c->ring_ev[k]) (void)hipEventDestroy(c->ring_ev[k]);
        }
        if (c->hsmall) (void)hipHostFree(c->hsmall);
        if (c->own) (void)hipStreamDestroy(c->own);
    }
    delete c;
    return MDG_OK;
}

int mdg_ctx_set_stream(mdg_ctx* c, void* stream) {
    if (!c) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    drain_timers(c);
    c->stream = stream ? (hipStream_t)stream : c->own;
    return MDG_OK;
}

int mdg_ctx_get_stream(mdg_ctx* c, void** stream) {
    if (!c || !stream) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    *stream = (void*)c->stream;
    return MDG_OK;
}

int mdg_ctx_synchronize(mdg_ctx* c) {
    if (!c) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    (void)hipSetDevice(c->device);
    HIPCHK(hipStreamSynchronize(c->stream));
    drain_timers(c);
    return MDG_OK;
}

int mdg_ctx_set_profiling(mdg_ctx* c, int enable) {
    if (!c) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    drain_timers(c);
    c->profile_mask = enable ? 0xffffffffu : 0u;
    return MDG_OK;
}

int mdg_ctx_set_profiling_mask(mdg_ctx* c, uint32_t mask) {
    if (!c) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    drain_timers(c);
    c->profile_mask = mask;
    return MDG_OK;
}

int mdg_ctx_stage_times(mdg_ctx* c, double* ms, uint64_t* launches, int n) {
    if (!c) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    (void)hipSetDevice(c->device);
    drain_timers(c);
    for (int i = 0; i < n && i < kStages; ++i) {
        if (ms) ms[i] = c->stage_ms[i];
        if (launches) launches[i] = c->stage_launches[i];
    }
    return MDG_OK;
}

int mdg_ctx_reset_stage_times(mdg_ctx* c) {
    if (!c) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    drain_timers(c);
    for (int i = 0; i < kStages; ++i) {
        c->stage_ms[i] = 0;
        c->stage_launches[i] = 0;
    }
    return MDG_OK;
}

int mdg_ctx_stage_kernel(mdg_ctx* c, int stage, const char** name) {
    if (!c || !name || stage < 0 || stage >= kStages) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    *name = c->stage_kernel[stage];
    return MDG_OK;
}

int mdg_ctx_set_latency_mode(mdg_ctx* c, int on) {
    if (!c || (on != 0 && on != 1)) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    c->latency = on;
    return MDG_OK;
}

int mdg_ctx_reload_switches(mdg_ctx* c) {
    if (!c) return MDG_INVALID_ARGUMENT;
    EngineSwitches w = read_engine_switches();
    std::lock_guard<std::mutex> g(c->mu);
    w.cus = c->sw.cus;
    c->sw = w;
    // MDG_ROCTX is the default of the tracing flag; an explicit mdg_ctx_set_tracing
    // stays in force across reloads
    if (!c->tracing_set) c->tracing = w.roctx != 0;
    return MDG_OK;
}

int mdg_ctx_set_tracing(mdg_ctx* c, int on) {
    if (!c || (on != 0 && on != 1)) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    c->tracing = on != 0;
    c->tracing_set = true;
    return c->tracing && !roctx().push ? MDG_ERR_HIP : MDG_OK;
}

int mdg_ctx_last_peaks(mdg_ctx* c, size_t spectrum, int which, int32_t* left, int32_t* center,
                       int32_t* right, size_t cap, size_t* count) {
    if (!c || !count || (which != 0 && which != 1)) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->arena.p || spectrum >= (size_t)c->last_B) return MDG_INVALID_ARGUMENT;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    const Workspace& w = c->w;
    const size_t capD = (size_t)c->last_N / 2 + 2;
    int32_t n = 0;
    HIPCHK(hipMemcpy(&n, (which ? w.sel_count : w.det_count) + spectrum, 4, hipMemcpyDeviceToHost));
    *count = (size_t)std::max(0, n);
    const size_t k = std::min(cap, (size_t)std::max(0, n));
    const size_t off = spectrum * capD;
    if (k) {
        if (left) HIPCHK(hipMemcpy(left, (which ? w.sel_l : w.det_l) + off, k * 4, hipMemcpyDeviceToHost));
        if (center) HIPCHK(hipMemcpy(center, (which ? w.sel_c : w.det_c) + off, k * 4, hipMemcpyDeviceToHost));
        if (right) HIPCHK(hipMemcpy(right, (which ? w.sel_r : w.det_r) + off, k * 4, hipMemcpyDeviceToHost));
    }
    return MDG_OK;
}

int mdg_ctx_last_smoothed(mdg_ctx* c, size_t spectrum, double* out, size_t n) {
    if (!c || !out) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->arena.p || !c->last_smoothed || spectrum >= (size_t)c->last_B ||
        n != (size_t)c->last_N)
        return MDG_INVALID_ARGUMENT;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(out, c->w.smooth + spectrum * (size_t)c->last_N, n * 8, hipMemcpyDeviceToHost));
    return MDG_OK;
}

int mdg_ctx_last_range_flags(mdg_ctx* c, size_t spectrum, int32_t* x_ok, uint32_t* slow_mask,
                              int32_t* unsafe_kept) {
    if (!c) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->arena.p || spectrum >= (size_t)c->last_B) return MDG_INVALID_ARGUMENT;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    const Workspace& w = c->w;
    int32_t v[3] = {0, 0, 0};
    HIPCHK(hipMemcpy(&v[0], w.x_ok + spectrum, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&v[1], w.unsafe + 4 * spectrum + 3, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&v[2], w.unsafe_kept + spectrum, 4, hipMemcpyDeviceToHost));
    if (x_ok) *x_ok = v[0];
    if (slow_mask) *slow_mask = (uint32_t)v[1];
    if (unsafe_kept) *unsafe_kept = v[2];
    return MDG_OK;
}

// the caller's array addresses in a BatchArgs (inputs and outputs): not part of a
// graph's key; a replay with other addresses rewrites them in the graph's nodes
void clear_io(BatchArgs& a) {
    a.x = a.y = a.sb = nullptr;
    a.y_rows = nullptr;
    a.out = nullptr;
    a.out_count = nullptr;
    a.out_mse = nullptr;
    a.out_status = nullptr;
}

bool same_io(const BatchArgs& p, const BatchArgs& q) {
    return p.x == q.x && p.y == q.y && p.y_rows == q.y_rows && p.sb == q.sb && p.out == q.out && p.out_count == q.out_count &&
           p.out_mse == q.out_mse && p.out_status == q.out_status;
}

// Point a cached graph at another call's arrays: every pipeline kernel takes
// (BatchArgs, Workspace, ...) by value (launch_k, mdg_kernels.hpp; a node whose
// kernel was not launched that way fails the call over to a new capture), so the
// node's copy of argument 0 is rewritten, and argument 1's smooth_ptr where it aliased y (the
// identity smoother), then the node's arguments are pushed into the exec.
int repoint_graph(mdg_ctx::CachedGraph& ge, const BatchArgs& a) {
    for (hipGraphNode_t nd : ge.knodes) {
        hipKernelNodeParams p{};
        HIPCHK(hipGraphKernelNodeGetParams(nd, &p));
        if (!is_pipeline_kernel(p.func) || !p.kernelParams || !p.kernelParams[0] || !p.kernelParams[1])
            return MDG_ERR_HIP;
        BatchArgs* na = (BatchArgs*)p.kernelParams[0];
        Workspace* nw = (Workspace*)p.kernelParams[1];
        if (nw->smooth_ptr == ge.cur.y) nw->smooth_ptr = a.y;
        std::memcpy(na, &a, sizeof(BatchArgs));
        HIPCHK(hipGraphExecKernelNodeSetParams(ge.exec, nd, &p));
    }
    ge.cur = a;
    return MDG_OK;
}

// run_pipeline through a cached hipGraph: the whole launch sequence (about 20
// kernels at B = 1 and the default settings) replays as one graph launch.
// Captured on the context's own stream, launched on the current one; keyed by
// the bytes of every argument except the caller's array addresses, the settings
// and the workspace addresses (a reallocation re-keys). A call with other arrays
// rewrites the nodes' arguments (repoint_graph) instead of capturing again, so
// a stream of calls on distinct device buffers replays one graph.
// Not used while stages are being timed, or for the reference-panic shape
// (host-synchronous path). Opt-in (MDG_GRAPHS=1): on ROCm 7 a replayed graph
// costs the GPU more per node than the same launches made directly -- 20
// concurrent B = 1 pipelines ran 7514-7576 spectra/s replayed against
// 7740-7766 launched directly, one spectrum alone 0.97-0.98 ms against 0.95
// (DESIGN.md §8); the host saves ≈10 µs per call.
int run_pipeline_graphed(mdg_ctx* c, BatchArgs& a, const mdg_settings* s) {
    const bool ma = s->smoother == MDG_SMOOTH_MOVING_AVERAGE;
    if (!c->sw.graphs || c->profile_mask ||
        (ma && (int64_t)(s->smooth_window / 2) > a.N))
        return run_pipeline(c, a, s);
    // size every buffer first: the capture must not allocate, and the key needs the
    // final addresses
    int rc = ensure_workspace(c, a.B, a.N, a.n_ignore);
    if (rc) return rc;
    if (ma && chain_supported(a.B, a.N, (int)s->smooth_iterations, (int)s->smooth_window) &&
        (c->sw.smooth == EngineSwitches::SM_DEFAULT || c->sw.smooth == EngineSwitches::SM_CHAIN))
        (void)ensure_chain(c, chain_bytes(a.B, a.N, (int)s->smooth_window, (int)s->smooth_iterations));
    if ((s->options & MDG_OPTION_EXACT_MSE) && (rc = ensure_exact(c, a.B, a.N))) return rc;
    if (c->graphs_gen != c->ws_gen) {  // buffers moved since these graphs were captured
        drop_graphs(c);
        c->graphs_gen = c->ws_gen;
    }
    a.det_only = s->selector == MDG_SELECT_DETECTOR_ONLY;
    BatchArgs ka = a;
    clear_io(ka);
    // the kernel-choice switches (tests, diagnostics) select other kernels, so they
    // are part of the key too (the struct is value-initialised: padding included)
    std::vector<unsigned char> key(sizeof(BatchArgs) + sizeof(mdg_settings) + 2 * sizeof(void*) +
                                   sizeof(size_t));
    {
        const unsigned char* sp = (const unsigned char*)&c->sw;
        key.insert(key.end(), sp, sp + sizeof(EngineSwitches));
    }
    unsigned char* k = key.data();
    std::memcpy(k, &ka, sizeof(BatchArgs));
    k += sizeof(BatchArgs);
    std::memcpy(k, s, sizeof(mdg_settings));
    k += sizeof(mdg_settings);
    std::memcpy(k, &c->arena.p, sizeof(void*));
    k += sizeof(void*);
    std::memcpy(k, &c->chain.p, sizeof(void*));
    k += sizeof(void*);
    std::memcpy(k, &c->chain.bytes, sizeof(size_t));
    // (the exact-MSE rows' address: a move bumps ws_gen, which drops every graph)
    mdg_ctx::CachedGraph* hit = nullptr;
    for (auto& ge : c->graphs)
        if (ge.key == key) hit = &ge;
    if (hit && !same_io(hit->cur, a) && repoint_graph(*hit, a)) {
        // a graph whose nodes could not be rewritten is captured again
        destroy_graph(*hit);
        c->graphs.erase(c->graphs.begin() + (hit - c->graphs.data()));
        hit = nullptr;
    }
    if (hit) {
        std::memcpy(c->stage_kernel, hit->kernels, sizeof(hit->kernels));
        // host-side state run_pipeline would have set
        c->last_B = a.B;
        c->last_N = a.N;
        c->last_smoothed = ma;
        HIPCHK(hipGraphLaunch(hit->exec, c->stream));
        return MDG_OK;
    }
    hipStream_t user = c->stream;
    c->stream = c->own;
    HIPCHK(hipStreamBeginCapture(c->own, hipStreamCaptureModeRelaxed));
    rc = run_pipeline(c, a, s);
    hipGraph_t graph = nullptr;
    const hipError_t e = hipStreamEndCapture(c->own, &graph);
    c->stream = user;
    if (rc || e != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc ? rc : hip_fail(e);
    }
    mdg_ctx::CachedGraph cg;
    cg.graph = graph;
    size_t nn = 0;
    hipError_t eg = hipGraphGetNodes(graph, nullptr, &nn);
    std::vector<hipGraphNode_t> nodes(nn);
    if (eg == hipSuccess && nn) eg = hipGraphGetNodes(graph, nodes.data(), &nn);
    for (size_t i = 0; eg == hipSuccess && i < nn; ++i) {
        hipGraphNodeType t;
        eg = hipGraphNodeGetType(nodes[i], &t);
        if (eg == hipSuccess && t == hipGraphNodeTypeKernel) cg.knodes.push_back(nodes[i]);
    }
    hipGraphExec_t exec = nullptr;
    if (eg == hipSuccess) eg = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    if (eg != hipSuccess) {
        (void)hipGraphDestroy(graph);
        return hip_fail(eg);
    }
    if (c->graphs.size() >= 8) {
        destroy_graph(c->graphs.front());
        c->graphs.erase(c->graphs.begin());
    }
    cg.key = std::move(key);
    cg.exec = exec;
    cg.cur = a;
    std::memcpy(cg.kernels, c->stage_kernel, sizeof(cg.kernels));
    c->graphs.push_back(std::move(cg));
    HIPCHK(hipGraphLaunch(exec, c->stream));
    return MDG_OK;
}

int mdg_deconvolute_batch_device(mdg_ctx* c, size_t b, size_t n, const double* d_x,
                                 size_t x_stride, const double* d_y, size_t y_stride,
                                 const double* d_sb, const mdg_settings* s, const double* ignore,
                                 size_t n_ignore, mdg_lorentzian* d_out, size_t cap,
                                 int32_t* d_counts, double* d_mse, int32_t* d_status) {
    if (!c) return MDG_INVALID_ARGUMENT;
    int v = validate_common(s, n_ignore, ignore);
    if (v) return v;
    if (b == 0) return MDG_OK;
    if (n < 2 || n > (size_t)INT32_MAX / 2 || b > (size_t)INT32_MAX) return MDG_INVALID_ARGUMENT;
    if (!d_x || !d_y || !d_sb || !d_counts || !d_mse || !d_status || (!d_out && cap)) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    BatchArgs a;
    int rc = fill_args(c, a, b, n, d_x, x_stride, d_y, y_stride, d_sb, ignore, n_ignore, (double*)d_out,
                       cap, d_counts, d_mse, d_status);
    if (rc) return rc;
    return run_pipeline_graphed(c, a, s);
}

}  // extern "C"

// Copies b host rows of `row_bytes` each (rows[i], anywhere in pageable memory) to
// the contiguous device range dst on st through the context's page-locked ring: a
// slot (<= kRingSlot bytes) is filled with memcpy, sent with one asynchronous DMA,
// and refilled once its event says the DMA has read it; the two slots alternate, so
// the host copy of one overlaps the DMA of the other. One pageable hipMemcpyAsync per
// row instead costs a host wait per row, and on a stream sharing its hardware queue
// with another lane's kernels each of those waits behind them (configs[4] at the
// default 4 queues: ~4.0k spectra/s with per-row copies against ~5.5-6.1k with one
// copy of a stacked buffer).
constexpr size_t kRingSlot = 32u << 20;
static int upload_rows(mdg_ctx* c, hipStream_t st, char* dst, const void* const* rows, size_t b,
                       size_t row_bytes) {
    const size_t total = b * row_bytes;
    if (total == 0) return MDG_OK;
    if (pinned_rows(rows, b, row_bytes)) {
        // rows in mdg_host_alloc memory: DMA straight from them, one copy per run of
        // adjacent rows (the call synchronises before it returns, so the rows are
        // read before the caller can release them)
        for (size_t r = 0; r < b;) {
            size_t e = r + 1;
            while (e < b && (const char*)rows[e] == (const char*)rows[e - 1] + row_bytes) ++e;
            HIPCHK(hipMemcpyAsync(dst + r * row_bytes, rows[r], (e - r) * row_bytes,
                                  hipMemcpyHostToDevice, st));
            r = e;
        }
        return MDG_OK;
    }
    const size_t want = std::min(kRingSlot, (total + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1));
    if (c->ring_bytes < want) {
        for (int k = 0; k < 2; ++k) {
            if (c->ring_used[k]) HIPCHK(hipEventSynchronize(c->ring_ev[k]));
            if (c->ring[k]) HIPCHK(hipHostFree(c->ring[k]));
            c->ring[k] = nullptr;
            c->ring_used[k] = false;
        }
        c->ring_bytes = 0;
        for (int k = 0; k < 2; ++k) {
            HIPCHK(hipHostMalloc(&c->ring[k], want, hipHostMallocDefault));
            if (!c->ring_ev[k]) HIPCHK(hipEventCreateWithFlags(&c->ring_ev[k], hipEventDisableTiming));
        }
        c->ring_bytes = want;
    }
    int slot = c->ring_next;
    for (size_t off = 0; off < total; off += c->ring_bytes) {
        const size_t len = std::min(c->ring_bytes, total - off);
        if (c->ring_used[slot]) HIPCHK(hipEventSynchronize(c->ring_ev[slot]));
        char* buf = (char*)c->ring[slot];
        // the rows overlapping [off, off + len)
        for (size_t r = off / row_bytes, done = 0; done < len; ++r) {
            const size_t in = (off + done) - r * row_bytes;
            const size_t k = std::min(row_bytes - in, len - done);
            std::memcpy(buf + done, (const char*)rows[r] + in, k);
            done += k;
        }
        HIPCHK(hipMemcpyAsync(dst + off, buf, len, hipMemcpyHostToDevice, st));
        HIPCHK(hipEventRecord(c->ring_ev[slot], st));
        c->ring_used[slot] = true;
        slot ^= 1;
    }
    c->ring_next = slot;
    return MDG_OK;
}

// Host-buffer batch: staging buffers, the caller's uploads (upload(dx, dy, st, &sent)
// enqueues the H2D copies of x and y into the staging rows; an upload with
// descriptors of its own sends them in the same copy as the signal boundaries and
// sets sent), the pipeline, and the results back in one round trip (the per-spectrum
// records and the first rows_guess rows of every table; more rows, if a spectrum has
// them, in a second copy). shared_x: one axis row.
template <typename Upload>
static int batch_host(mdg_ctx* c, size_t b, size_t n, bool shared_x, Upload upload, const double* sb,
                      const mdg_settings* s, const double* ignore, size_t n_ignore, mdg_lorentzian* out,
                      size_t cap, size_t* counts, double* mse, int* status) {
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const size_t xrows = shared_x ? 1 : b;
    int rc;
    if ((rc = ensure(c->st_x, xrows * n * 8))) return rc;
    // y rows the chain launch decodes while it smooths them (dec_next) are padded to
    // whole 128-byte lines (kDecRowAlign doubles): every line then belongs to one
    // decode chunk of one row (chain_decode), so no consumer can pull a line whose
    // bytes another decoder has yet to publish
    const size_t n_pad = (n + kDecRowAlign - 1) / kDecRowAlign * kDecRowAlign;
    if ((rc = ensure(c->st_y, b * n_pad * 8))) return rc;
    if ((rc = ensure(c->st_sb, b * 56))) return rc;  // [sb: 2b doubles][descriptors: 4b][row table: b]
    if ((rc = ensure(c->st_out, std::max<size_t>(1, b * cap) * 24))) return rc;
    // the per-spectrum results in one device row, [mse: 8 b][counts: 4 b][statuses:
    // 4 b] like the host scratch below, so they come back in one copy
    if ((rc = ensure(c->st_mse, b * 16))) return rc;
    double* d_mse = (double*)c->st_mse.p;
    int32_t* d_cnt = (int32_t*)(d_mse + b);
    int32_t* d_st = d_cnt + b;
    double* dx = (double*)c->st_x.p;
    double* dy = (double*)c->st_y.p;
    // the first rows_guess result rows of every spectrum come back with the records
    // (below); their count is known only after the pipeline
    // (above 64 MiB of guessed rows, every spectrum's rows are copied on their own)
    size_t guess = std::min(cap, c->rows_guess);
    if (b * guess * 24 > ((size_t)64 << 20)) guess = 0;
    // page-locked scratch: [sb: 16 b][the upload's own descriptors: 32 b and row
    // table: 8 b (mdg_deconvolute_rows_i32)][mse: 8 b][counts: 4 b][statuses: 4 b]
    // [the guessed result rows: 24 guess b]
    const size_t hs_need = b * 72 + b * guess * 24;
    if (c->hsmall_busy) {
        HIPCHK(hipStreamSynchronize(st));
        c->hsmall_busy = false;
    }
    if (c->hsmall_bytes < hs_need) {
        if (c->hsmall) {
            HIPCHK(hipHostFree(c->hsmall));
            c->hsmall = nullptr;
            c->hsmall_bytes = 0;
        }
        const size_t want = std::max<size_t>(hs_need, 64 * 64);
        HIPCHK(hipHostMalloc(&c->hsmall, want, hipHostMallocDefault));
        c->hsmall_bytes = want;
        void* dp = nullptr;
        c->hsmall_dev = hipHostGetDevicePointer(&dp, c->hsmall, 0) == hipSuccess ? dp : nullptr;
    }
    double* h_sb = (double*)c->hsmall;
    double* h_mse = h_sb + 7 * b;
    int32_t* h_cnt = (int32_t*)(h_mse + b);
    int32_t* h_st = h_cnt + b;
    mdg_lorentzian* h_rows = (mdg_lorentzian*)(h_sb + 9 * b);
    c->hsmall_busy = true;
    // From here on DMAs may read the caller's page-locked rows (upload_rows sends
    // mdg_host_alloc rows without copying them): a failure must not return while they
    // are in flight, or the caller could release and reuse the rows under the copy.
    auto fail = [&](int code) {
        (void)hipStreamSynchronize(st);
        c->hsmall_busy = false;
        return code;
    };
    // the kernels read the call's small inputs ([sb][descriptors][row table]) straight
    // from the page-locked scratch and write the records and the first guess rows of
    // every table into it (no copy either way, no copy-engine round trip;
    // MDG_HOST_DIRECT=0: device copies, as before round 4)
    const bool direct = c->hsmall_dev && c->sw.host_direct;
    c->small_rd = direct ? (const double*)c->hsmall_dev : (const double*)c->st_sb.p;
    c->small_copy = !direct;
    std::memcpy(h_sb, sb, b * 16);
    bool sent_sb = false;
    c->dec_next = false;
    if ((rc = upload(dx, dy, st, &sent_sb))) return fail(rc);
    hipError_t he = hipSuccess;
    if (!sent_sb && !direct) he = hipMemcpyAsync(c->st_sb.p, h_sb, b * 16, hipMemcpyHostToDevice, st);
    if (he != hipSuccess) return fail(hip_fail(he));
    BatchArgs a;
    if ((rc = fill_args(c, a, b, n, dx, shared_x ? 0 : n, dy, c->dec_next ? n_pad : n, c->small_rd, ignore,
                        n_ignore, (double*)c->st_out.p, cap, d_cnt, d_mse, d_st)))
        return fail(rc);
    if (c->dec_next) {  // the rows are decoded by the pipeline (run_pipeline)
        a.dec_rows = (const int32_t* const*)(c->small_rd + 6 * b);
        a.dec_desc = c->small_rd + 2 * b;
        c->dec_next = false;
    }
    // (writing a page-locked caller table in place instead measured no better:
    // configs[4] 13.9-14.1k against 14.0k, configs[0] alike, round 4)
    if (direct) {
        auto dev = [&](void* p) { return (char*)c->hsmall_dev + ((char*)p - (char*)c->hsmall); };
        a.out_mse = (double*)dev(h_mse);
        a.out_count = (int32_t*)dev(h_cnt);
        a.out_status = (int32_t*)dev(h_st);
        if (guess) {
            a.out_host = (double*)dev(h_rows);
            a.out_host_rows = (int)guess;
        }
    }
    if ((rc = run_pipeline(c, a, s))) return fail(rc);
    // Only the rows the spectra filled travel back (cap is usually N/2 + 2 rows, 1.5
    // MiB per 131072-point spectrum, against ~24 KiB of Lorentzians), and their count
    // is known only after the pipeline: the first rows_guess rows (the context's last
    // largest count and an eighth more) come back with the records, in the same round
    // trip, into the page-locked scratch, and each spectrum's own rows go on to `out`
    // from there (rows at and past counts[i] are never written: the device rows there
    // are stale); a spectrum with more rows than the guess has the rest copied after.
    if (!direct) {
        he = hipMemcpyAsync(h_mse, d_mse, b * 16, hipMemcpyDeviceToHost, st);
        if (he == hipSuccess && guess)
            he = hipMemcpy2DAsync(h_rows, guess * 24, c->st_out.p, cap * 24, guess * 24, b,
                                  hipMemcpyDeviceToHost, st);
        if (he != hipSuccess) return fail(hip_fail(he));
    }
    he = hipStreamSynchronize(st);
    if (he != hipSuccess) return fail(hip_fail(he));
    c->hsmall_busy = false;
    std::memcpy(mse, h_mse, b * 8);
    const int32_t* cnt = h_cnt;
    const int32_t* stv = h_st;
    size_t rows = 0;
    bool more = false;
    for (size_t i = 0; i < b; ++i) {
        const size_t r = std::min(cap, (size_t)std::max(0, cnt[i]));
        rows = std::max(rows, r);
        std::memcpy(out + i * cap, h_rows + i * guess, std::min(r, guess) * 24);
        if (r > guess) {
            more = true;
            HIPCHK(hipMemcpyAsync(out + i * cap + guess, (const mdg_lorentzian*)c->st_out.p + i * cap + guess,
                                  (r - guess) * 24, hipMemcpyDeviceToHost, st));
        }
    }
    if (more) HIPCHK(hipStreamSynchronize(st));
    c->rows_guess = rows + rows / 8 + 16;
    drain_timers(c);
    int first = MDG_OK;
    for (size_t i = 0; i < b; ++i) {
        counts[i] = (size_t)std::max(0, cnt[i]);
        status[i] = stv[i];
        if (first == MDG_OK && stv[i] != MDG_OK) first = stv[i];
    }
    return first;
}

extern "C" {

int mdg_deconvolute_batch(mdg_ctx* c, size_t b, size_t n, const double* x, size_t x_stride,
                          const double* y, size_t y_stride, const double* sb,
                          const mdg_settings* s, const double* ignore, size_t n_ignore,
                          mdg_lorentzian* out, size_t cap, size_t* counts, double* mse,
                          int* status) {
    if (!c) return MDG_INVALID_ARGUMENT;
    int v = validate_common(s, n_ignore, ignore);
    if (v) return v;
    if (b == 0) return MDG_OK;
    if (n < 2 || n > (size_t)INT32_MAX / 2 || b > (size_t)INT32_MAX) return MDG_INVALID_ARGUMENT;
    if (!x || !y || !sb || !counts || !mse || !status || (!out && cap)) return MDG_INVALID_ARGUMENT;
    const size_t xrows = x_stride ? b : 1;
    auto upload = [&](double* dx, double* dy, hipStream_t st, bool*) -> int {
        HIPCHK((x_stride == 0 || x_stride == n)
                   ? hipMemcpyAsync(dx, x, xrows * n * 8, hipMemcpyHostToDevice, st)
                   : hipMemcpy2DAsync(dx, n * 8, x, x_stride * 8, n * 8, b, hipMemcpyHostToDevice, st));
        HIPCHK(y_stride == n ? hipMemcpyAsync(dy, y, b * n * 8, hipMemcpyHostToDevice, st)
                             : hipMemcpy2DAsync(dy, n * 8, y, y_stride * 8, n * 8, b, hipMemcpyHostToDevice, st));
        return MDG_OK;
    };
    return batch_host(c, b, n, x_stride == 0, upload, sb, s, ignore, n_ignore, out, cap, counts, mse, status);
}

int mdg_deconvolute_rows(mdg_ctx* c, size_t b, size_t n, const double* const* x_rows,
                         const double* const* y_rows, const double* sb, const mdg_settings* s,
                         const double* ignore, size_t n_ignore, mdg_lorentzian* out, size_t cap,
                         size_t* counts, double* mse, int* status) {
    if (!c) return MDG_INVALID_ARGUMENT;
    int v = validate_common(s, n_ignore, ignore);
    if (v) return v;
    if (b == 0) return MDG_OK;
    if (n < 2 || n > (size_t)INT32_MAX / 2 || b > (size_t)INT32_MAX) return MDG_INVALID_ARGUMENT;
    if (!x_rows || !y_rows || !sb || !counts || !mse || !status || (!out && cap)) return MDG_INVALID_ARGUMENT;
    bool shared = true;
    for (size_t i = 0; i < b; ++i) {
        if (!x_rows[i] || !y_rows[i]) return MDG_INVALID_ARGUMENT;
        shared = shared && x_rows[i] == x_rows[0];
    }
    auto upload = [&](double* dx, double* dy, hipStream_t st, bool*) -> int {
        int rc = upload_rows(c, st, (char*)dx, (const void* const*)x_rows, shared ? 1 : b, n * 8);
        return rc ? rc : upload_rows(c, st, (char*)dy, (const void* const*)y_rows, b, n * 8);
    };
    return batch_host(c, b, n, shared, upload, sb, s, ignore, n_ignore, out, cap, counts, mse, status);
}

int mdg_deconvolute_rows_i32(mdg_ctx* c, size_t b, size_t n, const double* axes,
                             const int32_t* const* y_rows, const double* y_scale, const double* sb,
                             const mdg_settings* s, const double* ignore, size_t n_ignore,
                             mdg_lorentzian* out, size_t cap, size_t* counts, double* mse, int* status) {
    if (!c) return MDG_INVALID_ARGUMENT;
    int v = validate_common(s, n_ignore, ignore);
    if (v) return v;
    if (b == 0) return MDG_OK;
    if (n < 2 || n > (size_t)INT32_MAX / 2 || b > (size_t)INT32_MAX) return MDG_INVALID_ARGUMENT;
    if (!axes || !y_rows || !y_scale || !sb || !counts || !mse || !status || (!out && cap))
        return MDG_INVALID_ARGUMENT;
    if (b > 65535) return MDG_INVALID_ARGUMENT;  // the decode grid's y dimension
    bool shared = true;
    for (size_t i = 0; i < b; ++i) {
        if (!y_rows[i]) return MDG_INVALID_ARGUMENT;
        for (int k = 0; k < 3; ++k)
            if (!std::isfinite(axes[3 * i + k])) return MDG_INVALID_ARGUMENT;
        if (axes[3 * i + 2] == 0.0 || !std::isfinite(y_scale[i])) return MDG_INVALID_ARGUMENT;
        shared = shared && std::memcmp(axes + 3 * i, axes, 3 * sizeof(double)) == 0;
    }
    // rows in mdg_host_alloc memory are decoded by the pipeline straight from host
    // memory, the chain smoother starting on the first chunks while the rest are
    // read (chain_decode; MDG_DEC_OVERLAP=0: DMA and decode first, as other rows)
    const bool zc = c->sw.dec_overlap && pinned_rows((const void* const*)y_rows, b, n * 4, true);
    auto upload = [&](double* dx, double* dy, hipStream_t st, bool* sent_sb) -> int {
        int rc;
        // batch_host's scratch holds [sb: 2b][descriptors: 4b][row table: b] doubles:
        // one copy sends them all
        double* h = (double*)c->hsmall + 2 * b;
        for (size_t i = 0; i < b; ++i) {
            h[4 * i] = axes[3 * i];
            h[4 * i + 1] = axes[3 * i + 1];
            h[4 * i + 2] = axes[3 * i + 2];
            h[4 * i + 3] = y_scale[i];
        }
        if (zc) {
            const int32_t** tab = (const int32_t**)(h + 4 * b);
            for (size_t i = 0; i < b; ++i) tab[i] = y_rows[i];
            if (c->small_copy) HIPCHK(hipMemcpyAsync(c->st_sb.p, c->hsmall, b * 56, hipMemcpyHostToDevice, st));
            *sent_sb = true;
            c->dec_next = true;
            return MDG_OK;
        }
        if ((rc = ensure(c->st_raw, b * n * 4))) return rc;
        if ((rc = upload_rows(c, st, (char*)c->st_raw.p, (const void* const*)y_rows, b, n * 4))) return rc;
        if (c->small_copy) HIPCHK(hipMemcpyAsync(c->st_sb.p, c->hsmall, b * 48, hipMemcpyHostToDevice, st));
        *sent_sb = true;
        launch_decode_rows_i32((const int32_t*)c->st_raw.p, c->small_rd + 2 * b, (int)b,
                               (int64_t)n, shared ? 1 : 0, dx, dy, st);
        HIPCHK(hipGetLastError());
        return MDG_OK;
    };
    return batch_host(c, b, n, shared, upload, sb, s, ignore, n_ignore, out, cap, counts, mse, status);
}

int mdg_decode_rows_i32_device(mdg_ctx* c, size_t b, size_t n, const int32_t* d_raw,
                               const double* d_desc, double* d_x, double* d_y) {
    if (!c) return MDG_INVALID_ARGUMENT;
    if (b == 0) return MDG_OK;
    if (n < 2 || n > (size_t)INT32_MAX / 2 || b > 65535) return MDG_INVALID_ARGUMENT;
    if (!d_raw || !d_desc || !d_x || !d_y) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    launch_decode_rows_i32(d_raw, d_desc, (int)b, (int64_t)n, 0, d_x, d_y, c->stream);
    HIPCHK(hipGetLastError());
    return MDG_OK;
}

int mdg_deconvolute(mdg_ctx* c, const double* x, const double* y, size_t n, double sb0,
                    double sb1, const mdg_settings* s, const double* ignore, size_t n_ignore,
                    mdg_lorentzian* out, size_t cap, size_t* out_count, double* out_mse) {
    if (!out_count || !out_mse) return MDG_INVALID_ARGUMENT;
    if (!x || !y) return MDG_INVALID_ARGUMENT;
    const double sb[2] = {sb0, sb1};
    int status = 0;
    // through the page-locked ring (mdg_deconvolute_rows), not pageable copies
    const double* const xr[1] = {x};
    const double* const yr[1] = {y};
    return mdg_deconvolute_rows(c, 1, n, xr, yr, sb, s, ignore, n_ignore, out, cap, out_count, out_mse,
                                &status);
}

int mdg_superposition_vec_device(mdg_ctx* c, const double* d_x, size_t n, const mdg_lorentzian* d_L,
                                 size_t p, double* d_out) {
    if (!c || (!d_x && n) || (!d_L && p) || (!d_out && n)) return MDG_INVALID_ARGUMENT;
    if (p > (size_t)INT32_MAX) return MDG_INVALID_ARGUMENT;
    if (n == 0) return MDG_OK;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    int rc = ensure(c->st_flag, 256);
    if (rc) return rc;
    {
        StageTimer t(c, ST_SUPVEC);
        launch_superposition_vec(d_x, (int64_t)n, (const double*)d_L, (int)p, d_out,
                                 (int*)c->st_flag.p, c->stream);
    }
    HIPCHK(hipGetLastError());
    return MDG_OK;
}

int mdg_superposition_vec(mdg_ctx* c, const double* x, size_t n, const mdg_lorentzian* L, size_t p,
                          double* out) {
    if (!c || (!x && n) || (!L && p) || (!out && n)) return MDG_INVALID_ARGUMENT;
    if (p > (size_t)INT32_MAX) return MDG_INVALID_ARGUMENT;
    if (n == 0) return MDG_OK;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc;
    if ((rc = ensure(c->st_x, n * 8))) return rc;
    if ((rc = ensure(c->st_L, std::max<size_t>(p, 1) * 24))) return rc;
    if ((rc = ensure(c->st_sup, n * 8))) return rc;
    if ((rc = ensure(c->st_flag, 256))) return rc;
    HIPCHK(hipMemcpyAsync(c->st_x.p, x, n * 8, hipMemcpyHostToDevice, st));
    if (p) HIPCHK(hipMemcpyAsync(c->st_L.p, L, p * 24, hipMemcpyHostToDevice, st));
    {
        StageTimer t(c, ST_SUPVEC);
        launch_superposition_vec((const double*)c->st_x.p, (int64_t)n, (const double*)c->st_L.p,
                                 (int)p, (double*)c->st_sup.p, (int*)c->st_flag.p, st);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, c->st_sup.p, n * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    drain_timers(c);
    return MDG_OK;
}

int mdg_ordered_sum(mdg_ctx* c, const double* t, size_t n, double acc0, double* out) {
    if (!c || (!t && n) || !out || n > (size_t)INT32_MAX) return MDG_INVALID_ARGUMENT;
    for (size_t i = 0; i < n; ++i)
        if (!(t[i] >= 0.0) || std::signbit(t[i])) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc;
    if ((rc = ensure(c->st_x, std::max<size_t>(n, 1) * 8))) return rc;
    if ((rc = ensure(c->st_flag, 256))) return rc;
    if (n) HIPCHK(hipMemcpyAsync(c->st_x.p, t, n * 8, hipMemcpyHostToDevice, st));
    launch_ordered_sum((const double*)c->st_x.p, (int)n, acc0, (double*)c->st_flag.p, st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, c->st_flag.p, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MDG_OK;
}

int mdg_check_division(mdg_ctx* c, int variant, int cases, uint64_t seed, uint64_t n,
                       uint64_t* mismatches, uint64_t* tested) {
    if (!c || !mismatches || n > (uint64_t)INT64_MAX || (variant != 0 && variant != 1) ||
        (cases != 0 && cases != 1))
        return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    int rc;
    if ((rc = ensure(c->st_flag, 256))) return rc;
    HIPCHK(hipMemsetAsync(c->st_flag.p, 0, 16, st));
    launch_division_check(variant, cases, seed, (long long)n, (unsigned long long*)c->st_flag.p, st);
    HIPCHK(hipGetLastError());
    uint64_t res[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(res, c->st_flag.p, 16, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *mismatches = res[0];
    if (tested) *tested = res[1];
    return MDG_OK;
}

int mdg_check_fast_division(mdg_ctx* c, uint64_t seed, uint64_t n, uint64_t* mismatches) {
    return mdg_check_division(c, 0, 0, seed, n, mismatches, nullptr);
}

int mdg_division_hard_case(uint64_t seed, uint64_t i, double* n, double* d) {
    if (!n || !d) return MDG_INVALID_ARGUMENT;
    bool ok = false;
    division_hard_case(seed, i, n, d, &ok);
    return ok ? MDG_OK : MDG_INVALID_ARGUMENT;
}

int mdg_synth_batch_device(mdg_ctx* c, size_t b, size_t n, double xmax, double width,
                           uint64_t seed0, size_t n_peaks, double lo, double hi, double sigma,
                           double* d_x, double* d_y) {
    return mdg_synth_batch_device_hw(c, b, n, xmax, width, seed0, n_peaks, lo, hi, 1.0, sigma, d_x,
                                     d_y);
}

int mdg_synth_batch_device_hw(mdg_ctx* c, size_t b, size_t n, double xmax, double width,
                              uint64_t seed0, size_t n_peaks, double lo, double hi, double hw_scale,
                              double sigma, double* d_x, double* d_y) {
    if (!c || !d_x || !d_y || n < 2 || b == 0 || n_peaks > (size_t)INT32_MAX) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    std::vector<mdg_lorentzian> params(b * n_peaks);
    for (size_t s = 0; s < b; ++s)
        mdg_synth_lorentzians_hw(seed0 + s, n_peaks, lo, hi, hw_scale, params.data() + s * n_peaks);
    int rc;
    if ((rc = ensure(c->st_L, std::max<size_t>(1, params.size()) * 24))) return rc;
    HIPCHK(hipMemcpyAsync(c->st_L.p, params.data(), params.size() * 24, hipMemcpyHostToDevice, c->stream));
    {
        StageTimer t(c, ST_SYNTH);
        launch_synth(d_x, d_y, (int64_t)n, (int)b, xmax, width, (const double*)c->st_L.p,
                     (int)n_peaks, seed0, sigma, c->stream);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));  // params staging buffer is reused
    drain_timers(c);
    return MDG_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------
// Deconvoluter::optimize_settings (deconvoluter.rs:762-825) on the GPU.
// The reference deconvolutes the reference spectrum with every combination of
// 27 smoothing (iterations 2..=10 x windows 3, 5, 7), 10 noise-score thresholds
// (5 + c*3/9) and 3 fit iteration counts (5, 10, 15) and keeps the first minimum
// MSE. Here each smoothing setting is one batch of the 30 (threshold, fit)
// combinations (per-spectrum overrides; one shared input row). The batch MSE is
// a tree sum (<= 1e-12 relative from the reference's left fold), so every
// combination within 1e-9 of the minimum is re-run and its MSE recomputed in the
// reference's exact order; the first exact minimum in the reference's order wins.
// ------------------------------------------------------------------------------
extern "C" int mdg_optimize_settings(mdg_ctx* c, const double* x, const double* y, size_t n,
                                     double sb0, double sb1, const double* ignore,
                                     size_t n_ignore, mdg_settings* best, double* best_mse) {
    if (!c || !x || !y || !best || !best_mse) return MDG_INVALID_ARGUMENT;
    if (n < 2 || n > (size_t)INT32_MAX / 2) return MDG_INVALID_ARGUMENT;
    if (n_ignore > (size_t)(INT32_MAX / 4) || (n_ignore && !ignore)) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    constexpr int NSM = 27, NSEL = 10, NFIT = 3, NB = NSEL * NFIT;
    const size_t cap = n / 2 + 2;
    enum { BX, BY, BSB, BTHR, BFIT, BOUT, BCNT, BMSE, BST, BSUP, BSCR, BRES };
    const size_t sizes[12] = {n * 8, n * 8, NB * 16, NB * 8, NB * 4, NB * cap * 24, NB * 4,
                              NB * 8, NB * 4, n * 8, n * 8, 256};
    int rc;
    for (int k = 0; k < 12; ++k)
        if ((rc = ensure(c->opt[k], sizes[k]))) return rc;
    double* dx = (double*)c->opt[BX].p;
    double* dy = (double*)c->opt[BY].p;
    auto thr_of = [](int sel) { return 5.0 + ((double)sel * (8.0 - 5.0)) / 9.0; };
    std::vector<double> hsb(2 * NB), hthr(NB);
    std::vector<int32_t> hfit(NB);
    for (int k = 0; k < NB; ++k) {
        hsb[2 * k] = sb0;
        hsb[2 * k + 1] = sb1;
        hthr[k] = thr_of(k / NFIT);
        hfit[k] = 5 * (k % NFIT + 1);
    }
    HIPCHK(hipMemcpyAsync(dx, x, n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(dy, y, n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->opt[BSB].p, hsb.data(), NB * 16, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->opt[BTHR].p, hthr.data(), NB * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(c->opt[BFIT].p, hfit.data(), NB * 4, hipMemcpyHostToDevice, st));
    auto settings_of = [&](int sm, int sel, int fit) {
        mdg_settings s;
        mdg_settings_default(&s);
        s.smoother = MDG_SMOOTH_MOVING_AVERAGE;
        s.smooth_iterations = 2 + sm / 3;
        s.smooth_window = 3 + 2 * (sm % 3);
        s.selector = MDG_SELECT_NOISE_SCORE;
        s.scoring = MDG_SCORE_MINIMUM_SUM;
        s.threshold = thr_of(sel);
        s.fitter = MDG_FIT_ANALYTICAL;
        s.fit_iterations = (uint32_t)(5 * (fit + 1));
        return s;
    };
    std::vector<double> tree(NSM * NB);
    std::vector<int32_t> stat(NSM * NB);
    for (int sm = 0; sm < NSM; ++sm) {
        mdg_settings s = settings_of(sm, 0, NFIT - 1);  // 15 fit launches; per-spectrum counts
        BatchArgs a;
        if ((rc = fill_args(c, a, NB, n, dx, 0, dy, 0, (const double*)c->opt[BSB].p, ignore, n_ignore,
                            (double*)c->opt[BOUT].p, cap, (int32_t*)c->opt[BCNT].p,
                            (double*)c->opt[BMSE].p, (int32_t*)c->opt[BST].p)))
            return rc;
        c->ovr_thr = (const double*)c->opt[BTHR].p;
        c->ovr_fit = (const int32_t*)c->opt[BFIT].p;
        rc = run_pipeline(c, a, &s);
        c->ovr_thr = nullptr;
        c->ovr_fit = nullptr;
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(tree.data() + sm * NB, c->opt[BMSE].p, NB * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(stat.data() + sm * NB, c->opt[BST].p, NB * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    drain_timers(c);
    // the reference's `?` on the collected results: the first failure in its order
    for (int k = 0; k < NSM * NB; ++k)
        if (stat[k]) return stat[k];
    double m = tree[0];
    for (int k = 1; k < NSM * NB; ++k) m = std::min(m, tree[k]);
    const double tol = std::fabs(m) * 1e-9;
    int best_k = -1;
    double best_exact = 0.0;
    for (int k = 0; k < NSM * NB; ++k) {
        if (!(tree[k] <= m + tol)) continue;
        const int sm = k / NB, sel = (k % NB) / NFIT, fit = k % NFIT;
        mdg_settings s = settings_of(sm, sel, fit);
        BatchArgs a;
        if ((rc = fill_args(c, a, 1, n, dx, 0, dy, 0, (const double*)c->opt[BSB].p, ignore, n_ignore,
                            (double*)c->opt[BOUT].p, cap, (int32_t*)c->opt[BCNT].p,
                            (double*)c->opt[BMSE].p, (int32_t*)c->opt[BST].p)))
            return rc;
        if ((rc = run_pipeline(c, a, &s))) return rc;
        int32_t cnt = 0, sst = 0;
        HIPCHK(hipMemcpyAsync(&cnt, c->opt[BCNT].p, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&sst, c->opt[BST].p, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (sst) return sst;
        // the MSE regions come from the run's own workspace rows (on the device)
        launch_superposition_vec(dx, (int64_t)n, (const double*)c->opt[BOUT].p, cnt,
                                 (double*)c->opt[BSUP].p, (int*)c->opt[BRES].p + 8, st);
        launch_mse_exact((const double*)c->opt[BSUP].p, dy, (int64_t)n, c->w, (double*)c->opt[BSCR].p,
                         (double*)c->opt[BRES].p, st);
        HIPCHK(hipGetLastError());
        double exact = 0.0;
        HIPCHK(hipMemcpyAsync(&exact, c->opt[BRES].p, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (best_k < 0 || exact < best_exact) {  // min_by keeps the first minimum
            best_k = k;
            best_exact = exact;
        }
    }
    *best = settings_of(best_k / NB, (best_k % NB) / NFIT, best_k % NFIT);
    *best_mse = best_exact;
    return MDG_OK;
}

// ------------------------------------------------------------------------------
// Spectrum queue: the serving form of many concurrent deconvolute_spectrum calls
// (Deconvoluter is Send + Sync, deconvoluter.rs:913-917; par_deconvolute_spectra
// over an open-ended stream, :700-710). One submission is one spectrum with its
// own device arrays. Submissions are gathered into batches of up to max_batch
// spectra; each batch runs as one pipeline on the next of `lanes` engine contexts
// (own stream and workspace, round-robin), so a batch's sequential smoother
// overlaps the fits of the batch before it. Single spectra launched one by one use
// a B = 1 pipeline whose fit and smoother leave most of the chip idle, and
// concurrent B = 1 streams run out of hardware queues; a batch
// shares every launch among its spectra and needs one queue per lane.
// ------------------------------------------------------------------------------
struct mdg_queue {
    struct Lane {
        mdg_ctx* ctx = nullptr;
        Buffer x, y, sb, out, cnt, mse, st, table;
        QueueItem* host_table = nullptr;  // pinned: the upload of a batch's submission table
        hipEvent_t table_done = nullptr;  // that upload finished (the pinned rows are free)
        bool table_pending = false;
    };
    int device = 0;
    size_t n = 0;
    int max_batch = 0;
    mdg_settings s{};
    std::vector<double> ignore;
    std::mutex mu;
    std::vector<Lane> lanes;
    int next = 0;
    std::vector<QueueItem> open;  // the open batch
    uint64_t batches = 0, spectra = 0;
    int error = MDG_OK;  // first failure of an asynchronous batch launch (sticky)
    // flush deadline (mdg_queue_set_flush_us): a watcher thread launches the open
    // batch once its first submission has waited that long
    std::chrono::steady_clock::time_point open_since{};
    int64_t flush_us = 0;
    bool stop = false;
    std::condition_variable cv;
    std::thread watcher;
    uint64_t deadline_flushes = 0;
    int fail_next = 0;  // mdg_queue_fail_next_launch: status of the next launch (tests)
};

namespace {

int queue_launch(mdg_queue* q) {
    if (q->open.empty()) return MDG_OK;
    if (q->fail_next) {  // mdg_queue_fail_next_launch (tests): this launch fails
        const int rc = q->fail_next;
        q->fail_next = 0;
        return rc;
    }
    mdg_queue::Lane& L = q->lanes[q->next];
    q->next = (q->next + 1) % (int)q->lanes.size();
    const int B = (int)q->open.size();
    const size_t n = q->n, cap = n / 2 + 2;
    mdg_ctx* c = L.ctx;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    // the pinned table rows are rewritten only after their previous upload ran
    if (L.table_pending) HIPCHK(hipEventSynchronize(L.table_done));
    std::memcpy(L.host_table, q->open.data(), sizeof(QueueItem) * B);
    HIPCHK(hipMemcpyAsync(L.table.p, L.host_table, sizeof(QueueItem) * B, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(L.table_done, st));
    L.table_pending = true;
    // one shared axis (the usual case: every spectrum of a set on the same grid) is
    // read where it lies; otherwise the axes are gathered too
    const double* x0 = q->open[0].x;
    bool shared = true;
    for (const QueueItem& it : q->open) shared = shared && it.x == x0;
    const QueueItem* items = (const QueueItem*)L.table.p;
    // Each submission's intensity row is read where it lies, through the submission
    // table itself (BatchArgs::y_rows: row s = items[s].y; the signal boundaries
    // items[s].sb0 / sb1 likewise): no gather copy of 1 MiB per spectrum. The
    // identity smoother hands y to detection as the smoothed rows (one strided
    // base), and distinct axes need their rows side by side: those batches are
    // gathered as before.
    const bool in_place = shared && q->s.smoother == MDG_SMOOTH_MOVING_AVERAGE;
    if (!in_place)
        launch_queue_gather(items, B, (int64_t)n, shared ? 0 : 1, (double*)L.x.p, (double*)L.y.p, (double*)L.sb.p,
                            st);
    BatchArgs a;
    int rc = fill_args(c, a, B, n, shared ? x0 : (const double*)L.x.p, shared ? 0 : n, (const double*)L.y.p, n,
                       (const double*)L.sb.p, q->ignore.empty() ? nullptr : q->ignore.data(), q->ignore.size() / 2,
                       (double*)L.out.p, cap, (int32_t*)L.cnt.p, (double*)L.mse.p, (int32_t*)L.st.p);
    if (rc) return rc;
    if (in_place) {
        static_assert(sizeof(QueueItem) % 8 == 0 && offsetof(QueueItem, y) % 8 == 0 &&
                          offsetof(QueueItem, sb1) == offsetof(QueueItem, sb0) + 8,
                      "the submission table is read as rows of 8-byte words");
        a.y_rows = (const double* const*)((const char*)items + offsetof(QueueItem, y));
        a.rows_step = (int)(sizeof(QueueItem) / sizeof(void*));
        a.sb = (const double*)((const char*)items + offsetof(QueueItem, sb0));
        a.sb_step = (int)(sizeof(QueueItem) / sizeof(double));
    }
    if ((rc = run_pipeline(c, a, &q->s))) return rc;
    launch_queue_scatter(items, B, (const double*)L.out.p, (int64_t)cap, (const int32_t*)L.cnt.p,
                         (const double*)L.mse.p, (const int32_t*)L.st.p, st);
    HIPCHK(hipGetLastError());
    q->open.clear();
    q->batches += 1;
    q->spectra += (uint64_t)B;
    return MDG_OK;
}

}  // namespace

extern "C" {

int mdg_queue_create(int device, size_t n, size_t max_batch, int lanes, const mdg_settings* s,
                     const double* ignore, size_t n_ignore, mdg_queue** out) {
    if (!out) return MDG_INVALID_ARGUMENT;
    *out = nullptr;
    int v = validate_common(s, n_ignore, ignore);
    if (v) return v;
    if (n < 2 || n > (size_t)INT32_MAX / 2 || max_batch == 0 || max_batch > 4096 || lanes < 1 || lanes > 16)
        return MDG_INVALID_ARGUMENT;
    mdg_queue* q = new (std::nothrow) mdg_queue();
    if (!q) return MDG_ERR_OUT_OF_MEMORY;
    q->device = device;
    q->n = n;
    q->max_batch = (int)max_batch;
    q->s = *s;
    if (n_ignore) q->ignore.assign(ignore, ignore + 2 * n_ignore);
    q->open.reserve(max_batch);
    q->lanes.resize(lanes);
    const size_t cap = n / 2 + 2;
    int rc = MDG_OK;
    for (auto& L : q->lanes) {
        if ((rc = mdg_ctx_create(device, &L.ctx))) break;
        // lanes > 1: a B = 1 batch (a deadline flush, a flush per submit at low load)
        // shares the GPU with the other lanes' pipelines, so it takes tw7's fewer, wider
        // workgroups rather than latency mode's tf12
        if (lanes > 1) L.ctx->latency = 0;
        if ((rc = ensure(L.y, max_batch * n * 8)) || (rc = ensure(L.x, max_batch * n * 8)) ||
            (rc = ensure(L.sb, max_batch * 16)) || (rc = ensure(L.out, max_batch * cap * 24)) ||
            (rc = ensure(L.cnt, max_batch * 4)) || (rc = ensure(L.mse, max_batch * 8)) ||
            (rc = ensure(L.st, max_batch * 4)) || (rc = ensure(L.table, max_batch * sizeof(QueueItem))))
            break;
        if (hipHostMalloc((void**)&L.host_table, max_batch * sizeof(QueueItem), hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&L.table_done, hipEventDisableTiming) != hipSuccess) {
            rc = MDG_ERR_HIP;
            break;
        }
    }
    if (rc) {
        mdg_queue_destroy(q);
        return rc;
    }
    *out = q;
    return MDG_OK;
}

int mdg_queue_submit(mdg_queue* q, const double* d_x, const double* d_y, double sb0, double sb1,
                     mdg_lorentzian* d_out, size_t cap, int32_t* d_count, double* d_mse, int32_t* d_status) {
    if (!q || !d_x || !d_y || !d_count || !d_mse || !d_status || (!d_out && cap) || cap > (size_t)INT64_MAX / 24)
        return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(q->mu);
    if (q->error) return q->error;
    if (q->open.empty()) {
        q->open_since = std::chrono::steady_clock::now();
        if (q->flush_us > 0) q->cv.notify_one();
    }
    q->open.push_back({d_x, d_y, sb0, sb1, (double*)d_out, (int64_t)cap, d_count, d_mse, d_status});
    if ((int)q->open.size() >= q->max_batch) {
        const int rc = queue_launch(q);
        if (rc) q->error = rc;
        return rc;
    }
    return MDG_OK;
}

int mdg_queue_flush(mdg_queue* q) {
    if (!q) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(q->mu);
    if (q->error) return q->error;
    const int rc = queue_launch(q);
    if (rc) q->error = rc;
    return rc;
}

int mdg_queue_synchronize(mdg_queue* q) {
    if (!q) return MDG_INVALID_ARGUMENT;
    int rc = mdg_queue_flush(q);
    std::lock_guard<std::mutex> g(q->mu);
    for (auto& L : q->lanes) {
        const int r = mdg_ctx_synchronize(L.ctx);
        if (!rc) rc = r;
    }
    return rc;
}

int mdg_queue_set_flush_us(mdg_queue* q, int64_t us) {
    if (!q || us < 0) return MDG_INVALID_ARGUMENT;
    std::unique_lock<std::mutex> g(q->mu);
    q->flush_us = us;
    if (us > 0 && !q->watcher.joinable()) {
        q->watcher = std::thread([q] {
            std::unique_lock<std::mutex> lk(q->mu);
            while (!q->stop) {
                // nothing to launch: no deadline, an empty batch, or a queue whose
                // earlier launch failed (sticky error: the open batch never launches,
                // every call returns the error) -- wait, releasing q->mu
                if (q->flush_us <= 0 || q->open.empty() || q->error) {
                    q->cv.wait(lk);
                    continue;
                }
                const auto due = q->open_since + std::chrono::microseconds(q->flush_us);
                if (std::chrono::steady_clock::now() < due) {
                    q->cv.wait_until(lk, due);
                    continue;
                }
                const int rc = queue_launch(q);  // under q->mu, like a submit's launch
                if (rc) q->error = rc;
                ++q->deadline_flushes;
            }
        });
    }
    q->cv.notify_one();
    return MDG_OK;
}

int mdg_queue_fail_next_launch(mdg_queue* q, int status) {
    if (!q || status == MDG_OK) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(q->mu);
    q->fail_next = status;
    return MDG_OK;
}

int mdg_queue_lane(mdg_queue* q, int lane, mdg_ctx** ctx) {
    if (!q || !ctx || lane < 0 || lane >= (int)q->lanes.size()) return MDG_INVALID_ARGUMENT;
    *ctx = q->lanes[lane].ctx;
    return MDG_OK;
}

int mdg_queue_stats(mdg_queue* q, uint64_t* batches, uint64_t* spectra, size_t* open) {
    if (!q) return MDG_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> g(q->mu);
    if (batches) *batches = q->batches;
    if (spectra) *spectra = q->spectra;
    if (open) *open = q->open.size();
    return MDG_OK;
}

int mdg_queue_destroy(mdg_queue* q) {
    if (!q) return MDG_OK;
    if (q->watcher.joinable()) {
        {
            std::lock_guard<std::mutex> g(q->mu);
            q->stop = true;
        }
        q->cv.notify_one();
        q->watcher.join();
    }
    for (auto& L : q->lanes) {
        if (L.ctx) (void)mdg_ctx_synchronize(L.ctx);
        for (Buffer* b : {&L.x, &L.y, &L.sb, &L.out, &L.cnt, &L.mse, &L.st, &L.table})
            if (b->p) (void)hipFree(b->p);
        if (L.host_table) (void)hipHostFree(L.host_table);
        if (L.table_done) (void)hipEventDestroy(L.table_done);
        if (L.ctx) (void)mdg_ctx_destroy(L.ctx);
    }
    delete q;
    return MDG_OK;
}

}  // extern "C"
