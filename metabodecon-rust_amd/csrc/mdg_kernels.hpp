// mdg_kernels.hpp -- kernel argument blocks and launchers (internal to libmdgpu).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <tuple>
#include <utility>

#include "../../include/mdgpu.h"
#include "mdg_common.hpp"

namespace mdg {

// Per-call arguments: caller-owned device arrays (inputs resident in HBM).
struct BatchArgs {
    int B;                // spectra in the batch
    int N;                // points per spectrum
    const double* x;      // row s at x + s*x_stride (x_stride 0: shared axis)
    int64_t x_stride;
    const double* y;      // row s at y + s*y_stride (y_rows null)
    int64_t y_stride;
    // rows read in place through a table of row pointers (the spectrum queue: each
    // submission's own row, no gather copy): row s at y_rows[s * rows_step]
    const double* const* y_rows;
    int rows_step;        // pointers between consecutive rows' entries of y_rows
    int sb_step;          // doubles between consecutive spectra's signal-boundary pairs
    const double* sb;     // signal boundaries of spectrum s at sb[s*sb_step], sb[s*sb_step+1] (ppm, ordered as Spectrum stores them)
    int n_ignore;         // merged ignore regions (ppm), shared by the batch
    const double* ignore; // 2 * n_ignore doubles in device memory (null when none)
    double* out;          // B x cap x {sfhw, hw2, maxp}
    int cap;
    int32_t* out_count;
    double* out_mse;
    int32_t* out_status;
    int latency;          // the context's latency mode (mdg_ctx_set_latency_mode; kernel choice only)
    int det_only;         // the detector-only selector (run_pipeline; host-side kernel choice only)
    // mdg_deconvolute_rows_i32 with page-locked rows: the pipeline decodes the rows
    // into y / x itself, reading them from host memory (null: y and x hold them)
    const int32_t* const* dec_rows;  // B host-mapped int32 rows (device copy of the table)
    const double* dec_desc;          // B x {maximum, width, divisor, scale}
    int dec_gen;                     // a decoded chunk's flag value in this call (Workspace::dec_flags)
    // the host-buffer calls: the first out_host_rows rows of every spectrum's table go
    // straight to page-locked host memory (row s*out_host_rows + k), the rest to out
    double* out_host;
    int out_host_rows;               // <= cap; 0 when out_host is null
};

// Context-owned device workspace (sized for the worst case of the batch shape).
// Layout in HBM, all per-spectrum rows contiguous ("spectrum-major"):
//   smooth/tmp0/tmp1   B x N f64
//   masks              B x 3 x W u64   (center / right / left predicate bits)
//   det_* / sel_*      B x capD i32    (peak index triples, SoA)
//   scores             B x capD f64
//   params, kept       B x capD x 3 f64 (AoS {sfhw,hw2,maxp}: wave-uniform SMEM reads)
//   stencil            B x capD x 6 f64 (per spectrum: x plane 3 capD, then y plane 3 capD)
//   rx, ry, ratio      B x 3capD f64   (reduced spectrum, fitter order l,c,r)
struct Workspace {
    int W;                    // mask words per spectrum = ceil(N/64)
    int capD;                 // peak capacity per spectrum = N/2 + 2
    const double* smooth_ptr; // smoothed intensities (== y for the identity smoother)
    int64_t smooth_stride;
    double* smooth;
    double* tmp0;
    double* tmp1;
    uint64_t* masks;
    int32_t* det_l;
    int32_t* det_c;
    int32_t* det_r;
    int32_t* sel_l;
    int32_t* sel_c;
    int32_t* sel_r;
    double* scores;
    double* params;
    double* params_alt;       // k_fit_sup_tf: odd params versions (null: k_fit_update in place)
    int fit_iters;            // fit iterations launched for the batch
    double* kept;
    double* stencil;
    double* rx;
    double* ry;
    double* ratio;
    double* mse_part;         // B x nparts
    double* sfr_stats;        // B x {mean, sd}
    int64_t* sbi;             // B x 2
    int64_t* ig;              // B x 2*ig_cap: ignore-region index pairs
    int64_t* ig_cum;          // B x (ig_cap + 2): cumulative lengths of the MSE regions
    int ig_cap;               // pairs per spectrum the rows hold (>= the call's n_ignore)
    int32_t* n_ig;
    int32_t* mse_panic;
    int32_t* status;
    int32_t* det_count;
    int32_t* sel_count;
    int32_t* kept_count;
    int32_t* x_ok;            // B: axis inside the fast-division range
    int32_t* unsafe;          // B x 4: count of fit params outside it, per params version
                              // (k_fit_update path: version & 1; fused k_fit_sup_tf: version % 3);
                              // slot 3: the launches that took the plain division (mark_slow)
    int32_t* unsafe_kept;     // B: same for the retained Lorentzians
    int32_t* mse_done;        // B: k_mse_local workgroups finished (the last one folds, resets)
    int32_t* peak_cnt;        // B x ceil(W/64) u64: k_peaks slots {valid, bordered, kept} per mask chunk
    // k_smooth_chain (allocated on first use; null otherwise)
    double* chain_raw;        // P x B x chain_stride: raw running sums of every pass
    double* chain_tmp;        // (P-1) x B x chain_stride: scaled outputs of passes 0..P-2
    int32_t* chain_flags;     // B x P x 32: published output blocks of (s, p) (own 128-B line)
    int64_t chain_stride;
    int chain_P;              // passes the chain buffers hold (0 = not allocated)
    int32_t* dec_flags;       // B x kDecChunks: chunk c of row s decoded when == BatchArgs::dec_gen
    // per-spectrum overrides (optimize_settings batches; null = the batch settings)
    const double* thr_s;      // B noise-score thresholds
    const int32_t* fit_iters_s;  // B fit iteration counts (<= the launched count)
};

// row s of a batch's intensities (BatchArgs::y_rows or the strided rows)
__device__ __host__ inline const double* y_row(const BatchArgs& a, int s) {
    return a.y_rows ? a.y_rows[(size_t)s * a.rows_step] : a.y + (size_t)s * a.y_stride;
}

// Engine switches: the MDG_* environment variables that choose among the shipped,
// bit-exact kernels (tests, measurements). Read once per context, when it is created
// (mdg_ctx_create) or on an explicit mdg_ctx_reload_switches -- never on a call's
// path (a getenv there races a concurrent setenv, costs time every call, and makes a
// context's behaviour depend on when the variable was read).
// (ints and char arrays only: no padding, the bytes are part of the graph keys)
struct EngineSwitches {
    enum { SM_DEFAULT = 0, SM_CHAIN, SM_PIPE, SM_GENERIC, SM_OTHER, SM_SMALL };
    int smooth = SM_DEFAULT;     // MDG_SMOOTH = chain | pipe | generic (other values: the generic kernel)
    int chain_excl = 1;          // MDG_CHAIN_EXCL=0: never whole-CU chain workgroups
    int chain_l2ahead = 0;       // MDG_CHAIN_L2AHEAD: blocks each chain pulls into L2 ahead (0: by grid)
    int peaks = 0;               // MDG_PEAKS: 0 by batch size, 1 fine, 2 coarse (any other value)
    int detect = 0;              // MDG_DETECT: 0 by shape (N <= 4096: inside k_select, else k_flags +
                                 // k_peaks), 1 separate (k_flags + k_peaks at every N), 2 fused (also
                                 // the predicates inside k_peaks; measured slower, §5)
    char fitsup[8] = {};         // MDG_FITSUP: a shipped fit kernel's name ("": by batch size)
    int tw_g = 0;                // MDG_TW_G: term-fold workgroups (0: the kernel's default)
    int gfit = 24;               // MDG_GFIT: k_fit_sup workgroups per spectrum
    int mse_npt = 0;             // MDG_MSE_NPT = 2 | 4 (0: by batch size)
    int mse_parts = 0;           // MDG_MSE_PARTS (0: by shape)
    int mse_pk = 0;              // MDG_MSE_PK: 0 = 30 powers at radius 3 (every batch size);
                                 // 20 selects the round-4 radius-5 form
    int mse_nearcap = -1;        // MDG_MSE_NEARCAP (-1: kLocNear)
    int prep_separate = 0;      // MDG_PREP=separate
    int graphs = 0;              // MDG_GRAPHS=1
    int host_direct = 1;         // MDG_HOST_DIRECT=0: device copies of the small inputs / results
    int dec_overlap = 1;         // MDG_DEC_OVERLAP=0: compact rows by DMA + decode launch
    int roctx = 0;               // MDG_ROCTX=1: roctx ranges around the pipeline stages
    int cus = 256;               // not a switch: the device's CU count, set by mdg_ctx_create
                                 // (once per context, not per launch)
    // diagnostic builds only (make diag)
    char diag_skip[32] = {};
    char diag_dup[64] = {};
    int diag_pad = 0;
    int diag_pad_small = 0;
    int diag_pad_wgs = 0;
};
// the switches as the environment holds them now
EngineSwitches read_engine_switches();

// Bytes of the k_smooth_chain buffers for (B, N, passes) and their row stride.
int64_t chain_stride_for(int N, int ws);
size_t chain_bytes(int B, int N, int ws, int passes);
bool chain_supported(int B, int N, int iters, int ws);
// a.dec_rows decoded into a.y / a.x by a launch of its own (the pipeline does this
// when the chain smoother cannot decode them while it runs)
void launch_decode_rows_zc(const BatchArgs& a, hipStream_t st);

// exact-order MSE of spectrum 0 of the last pipeline run over its MSE regions
// (read on the device from the workspace: signal boundaries and ignore pairs)
void launch_mse_exact(const double* sup, const double* y, int64_t n, const Workspace& w,
                      double* scratch, double* out, hipStream_t st);

// Every pipeline kernel takes (BatchArgs, Workspace, ...) by value and is launched
// through launch_k, which the compiler holds to that signature and which records
// the kernel as one whose graph nodes may be re-pointed at another call's arrays
// (mdg_capi.hip repoint_graph rewrites argument 0 of such nodes only).
void note_pipeline_kernel(const void* f);
bool is_pipeline_kernel(const void* f);

template <class K, class T, size_t... I>
inline void launch_k_tuple(K k, dim3 g, dim3 b, size_t sh, hipStream_t st, const BatchArgs& a,
                           const Workspace& w, T& t, std::index_sequence<I...>) {
    void* args[] = {(void*)&a, (void*)&w, (void*)&std::get<I>(t)..., nullptr};
    (void)hipLaunchKernel((const void*)k, g, b, args, sh, st);
}

template <typename... P, typename... X>
inline void launch_k(void (*k)(BatchArgs, Workspace, P...), dim3 g, dim3 b, size_t sh, hipStream_t st,
                     const BatchArgs& a, const Workspace& w, X... x) {
    static_assert(sizeof...(P) == sizeof...(X), "kernel argument count");
    note_pipeline_kernel((const void*)k);
    std::tuple<P...> t{static_cast<P>(x)...};
    launch_k_tuple(k, g, b, sh, st, a, w, t, std::index_sequence_for<P...>{});
}

void launch_prep(const BatchArgs& a, const Workspace& w, hipStream_t st);
#ifdef MDG_DIAG
void launch_diag_nop(const BatchArgs& a, const Workspace& w, const EngineSwitches& sw, hipStream_t st);
#endif
bool smooth_uses_chain(const BatchArgs& a, const Workspace& w, int iters, int ws, const EngineSwitches& sw);
bool smooth_uses_small(const BatchArgs& a, int iters, int ws, const EngineSwitches& sw);
// the smoother launch runs k_prep's work itself (k_smooth_chain, k_smooth_small)
bool smooth_fuses_prep(const BatchArgs& a, const Workspace& w, int iters, int ws, const EngineSwitches& sw);
const char* launch_smooth(const BatchArgs& a, const Workspace& w, int iters, int ws, const EngineSwitches& sw,
                          hipStream_t st, int fused_prep = 0);
void launch_flags(const BatchArgs& a, const Workspace& w, hipStream_t st);
// k_peaks computes the detector's predicates itself (no k_flags launch)
bool peaks_fuse_flags(const BatchArgs& a, const Workspace& w, const EngineSwitches& sw);
const char* launch_peaks(const BatchArgs& a, const Workspace& w, int detector_only, const EngineSwitches& sw,
                         hipStream_t st);
// small spectra with the noise-score selector: detection inside k_select (no k_flags,
// no k_peaks launch)
bool detect_fused(const BatchArgs& a, int detector_only, const EngineSwitches& sw);
const char* launch_select(const BatchArgs& a, const Workspace& w, int detector_only,
                          double threshold, hipStream_t st, bool fused = false);
// returns true when the launched kernel also did the stencil update (no k_fit_update)
bool fit_sup_fused(const BatchArgs& a, const EngineSwitches& sw);
// small spectra (N <= kSmallN, or MDG_FITSUP=small): every fit iteration in one launch
bool fit_is_small(const BatchArgs& a, const EngineSwitches& sw);
const char* launch_fit_small(const BatchArgs& a, const Workspace& w, hipStream_t st);
const char* launch_fit_sup(const BatchArgs& a, const Workspace& w, int gx, int it, const EngineSwitches& sw,
                           hipStream_t st);
void launch_fit_update(const BatchArgs& a, const Workspace& w, int gx, int it, hipStream_t st);
void launch_retain(const BatchArgs& a, const Workspace& w, hipStream_t st);
// MSE tiles per spectrum for launch_mse (<= kMseMaxParts)
int mse_nparts(const BatchArgs& a, const EngineSwitches& sw);
// k_mse_local: the MSE and the retained Lorentzians (out rows, counts, statuses)
const char* launch_mse(const BatchArgs& a, const Workspace& w, int nparts, const EngineSwitches& sw,
                       hipStream_t st);
// exact-order MSE of every spectrum of the batch (MDG_OPTION_EXACT_MSE), after
// launch_mse: squared residuals into res (B rows of res_row >= N doubles), then the
// reference's left folds; overwrites out_mse
void launch_mse_exact_batch(const BatchArgs& a, const Workspace& w, double* res, int64_t res_row,
                            hipStream_t st);
// windowed left fold of n <= kWinMax non-negative terms (test support)
void launch_ordered_sum(const double* t, int n, double acc0, double* out, hipStream_t st);
// fast-range division variants against IEEE '/' (test support): variant 0 div_rn,
// 1 div_rn_1nr; cases 0 random pairs, 1 constructed near-midpoint pairs;
// out[0] += mismatches, out[1] += pairs tested
void launch_division_check(int variant, int cases, unsigned long long seed, long long n,
                           unsigned long long* out, hipStream_t st);
void launch_superposition_vec(const double* x, int64_t n, const double* params, int P,
                              double* out, int* flag, hipStream_t st);
void launch_synth(double* x, double* y, int64_t n, int B, double xmax, double width,
                  const double* params, int P, uint64_t seed0, double sigma, hipStream_t st);

// Spectrum queue (mdg_queue_*): one submission = one spectrum with its own device
// arrays. A batch of submissions is gathered into the lane's contiguous rows, runs
// as one pipeline, and its results are scattered back to each submission's arrays.
struct QueueItem {
    const double* x;      // n chemical shifts
    const double* y;      // n intensities
    double sb0, sb1;      // signal boundaries (ppm, as the Spectrum stores them)
    double* out;          // cap Lorentzians {sfhw, hw2, maxp}
    int64_t cap;
    int32_t* count;
    double* mse;
    int32_t* status;
};
// rows y (and x when gather_x) of the B items into y_rows / x_rows (B x n), sb pairs
void launch_queue_gather(const QueueItem* items, int B, int64_t n, int gather_x, double* x_rows,
                         double* y_rows, double* sb, hipStream_t st);
// the pipeline's B results (table rows of stage_cap) to each item's arrays: count,
// mse, status (MDG_CAPACITY when the item's cap is below the count) and min(count,
// cap) Lorentzians
void launch_queue_scatter(const QueueItem* items, int B, const double* out, int64_t stage_cap,
                          const int32_t* counts, const double* mse, const int32_t* status,
                          hipStream_t st);
// compact host rows (mdg_deconvolute_rows_i32) into B x n f64 staging rows: the
// Bruker axis from {maximum, width, divisor} and int32 samples times a power of two
void launch_decode_rows_i32(const int32_t* raw, const double* desc, int B, int64_t n, int shared_x,
                            double* x_rows, double* y_rows, hipStream_t st);

}  // namespace mdg
