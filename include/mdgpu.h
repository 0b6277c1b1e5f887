/*
 * mdgpu.h -- C ABI of the MI355X-native metabodecon deconvolution engine.
 *
 * Drop-in boundary for metabodecon's hot path. Each entry point replaces one
 * public reference interface (paths relative to SombkeMaximilian/metabodecon-rust):
 *
 *   mdg_deconvolute            <- Deconvoluter::deconvolute_spectrum
 *                                 metabodecon/src/deconvolution/deconvoluter.rs:530-552
 *                                 and par_deconvolute_spectrum (:591-613, same bits)
 *   mdg_deconvolute_batch      <- Deconvoluter::{deconvolute_spectra,par_deconvolute_spectra}
 *                                 deconvoluter.rs:651-661 / :700-710 (per-spectrum status;
 *                                 the caller reproduces the fail-fast Result collect)
 *   mdg_deconvolute_rows       same, one pointer per spectrum row (no caller-side stacking)
 *   mdg_deconvolute_rows_i32   same, rows in the Bruker reader's compact form (int32 samples,
 *                                axis formula; spectrum/formats/bruker.rs:278-280, :459-470)
 *   mdg_deconvolute_batch_device  same, inputs/outputs resident in HBM (no PCIe in the call)
 *   mdg_superposition_vec      <- Lorentzian::{superposition_vec,par_superposition_vec}
 *                                 deconvolution/lorentzian.rs:631-663
 *   mdg_settings_validate      <- SmoothingSettings/SelectionSettings/FittingSettings::validate
 *                                 smoother.rs:84-100, selector.rs:85-98, fitter.rs:80-90
 *   mdg_ignore_region_add      <- Deconvoluter::add_ignore_region  deconvoluter.rs:438-472
 *
 * Conventions: plain pointers and sizes, no C++/torch types; every function
 * returns an int status (0 = ok) and never throws/aborts across the boundary.
 * Host buffers are owned by the caller; device workspaces are owned by the
 * context and reused across calls. A context is internally locked, so one
 * context may be shared by threads (Deconvoluter is Send + Sync,
 * deconvoluter.rs:913-917); calls on one context serialise.
 *
 * Numerics: all arithmetic is IEEE binary64 with no FMA contraction and every
 * order-dependent sum evaluated in the reference's order, so peak index sets
 * and Lorentzian parameters are bit-identical to the reference CPU path; the
 * MSE reduction is a fixed-order tree (|rel err| < 1e-12).
 */
#ifndef MDGPU_H
#define MDGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDG_ABI_VERSION 1

/* Status codes (deconvolution/error.rs:39-95 kinds + engine failures). */
enum mdg_status {
    MDG_OK = 0,
    MDG_NO_PEAKS_DETECTED = 1,        /* Kind::NoPeaksDetected */
    MDG_EMPTY_SIGNAL_REGION = 2,      /* Kind::EmptySignalRegion */
    MDG_EMPTY_SIGNAL_FREE_REGION = 3, /* Kind::EmptySignalFreeRegion */
    MDG_INVALID_SMOOTHING = 10,       /* Kind::InvalidSmoothingSettings */
    MDG_INVALID_SELECTION = 11,       /* Kind::InvalidSelectionSettings */
    MDG_INVALID_FITTING = 12,         /* Kind::InvalidFittingSettings */
    MDG_INVALID_IGNORE_REGION = 13,   /* Kind::InvalidIgnoreRegion */
    MDG_INVALID_ARGUMENT = 20,        /* null pointer / bad size at the ABI */
    MDG_CAPACITY = 21,                /* out_cap smaller than the result (count still set) */
    MDG_REFERENCE_PANIC = 30,         /* input on which the reference panics (slice bounds) */
    MDG_ERR_HIP = 100,                /* HIP runtime failure */
    MDG_ERR_NO_DEVICE = 101,
    MDG_ERR_OUT_OF_MEMORY = 102
};

enum { MDG_SMOOTH_IDENTITY = 0, MDG_SMOOTH_MOVING_AVERAGE = 1 };
enum { MDG_SELECT_DETECTOR_ONLY = 0, MDG_SELECT_NOISE_SCORE = 1 };
enum { MDG_SCORE_MINIMUM_SUM = 0 };
enum { MDG_FIT_ANALYTICAL = 0 };

/* Deconvoluter settings (smoother.rs:27-65, selector.rs:21-66, fitter.rs:26-63). */
typedef struct mdg_settings {
    int32_t smoother;          /* MDG_SMOOTH_* */
    uint32_t smooth_iterations;
    uint32_t smooth_window;
    int32_t selector;          /* MDG_SELECT_* */
    int32_t scoring;           /* MDG_SCORE_* */
    uint32_t fit_iterations;
    int32_t fitter;            /* MDG_FIT_* */
    int32_t options;           /* MDG_OPTION_* bits (engine options; 0 = the defaults) */
    double threshold;
} mdg_settings;

/* mdg_settings.options. MDG_OPTION_EXACT_MSE: the MSE is computed in the reference's
 * operation order (compute_mse, deconvoluter.rs:828-862: each point's superposition
 * the in-order left fold of Lorentzian::superposition_vec, lorentzian.rs:606-611, the
 * squared residuals folded left to right per MSE region, the region sums in region
 * order), so Deconvolution::mse and the `mse` field of the serialized Deconvolution
 * (serialized_deconvolution.rs:18-31) equal the reference's bit for bit. Off: the
 * engine's MSE (local expansions and fixed-order trees), within 1e-12 relative of it
 *  and cheaper. Lorentzians, counts and statuses are the same either
 * way. Other bits must be 0 (MDG_INVALID_ARGUMENT). */
enum { MDG_OPTION_EXACT_MSE = 1 };

/* Lorentzian in transformed parameters (lorentzian.rs:138-145), repr(C). */
typedef struct mdg_lorentzian {
    double sfhw;
    double hw2;
    double maxp;
} mdg_lorentzian;

typedef struct mdg_ctx mdg_ctx;

/* ---- host-only helpers (no GPU needed) ---------------------------------- */
int mdg_abi_version(void);
/* Build provenance, "src=<sha256/16 of the engine sources> flags=<sha256/16 of the
 * compile flags> compiler=<hipcc clang>"
 * (no reference counterpart: lets a caller check the library matches its sources). */
const char* mdg_build_info(void);
const char* mdg_strerror(int status);
void mdg_settings_default(mdg_settings* s);
int mdg_settings_validate(const mdg_settings* s);
/* Merge (a,b) into the sorted ppm region list `regions` (n pairs, capacity cap
 * pairs) exactly like add_ignore_region; *n_out receives the new count. */
int mdg_ignore_region_add(double* regions, size_t n, size_t cap, double a, double b,
                          size_t* n_out);

/* Synthetic-workload generator (bench/test data, not the hot path):
 * n_peaks Lorentzians on a jittered grid over [lo, hi] ppm (SURVEY 8d recipe),
 * counter-based splitmix64 so host and device draw identical bits. */
int mdg_synth_lorentzians(uint64_t seed, size_t n_peaks, double lo, double hi,
                          mdg_lorentzian* out);
/* Same with every half width scaled by hw_scale (configs[3]: 2.0; 1.0 = the above). */
int mdg_synth_lorentzians_hw(uint64_t seed, size_t n_peaks, double lo, double hi, double hw_scale,
                             mdg_lorentzian* out);
/* Irwin-Hall(12) noise, exact in binary64: sigma * (sum of 12 u48 - 6). */
int mdg_synth_noise(uint64_t seed, size_t n, double sigma, double* out);

/* Host (no GPU): decode one JCAMP-DX data block (the text after ##XYDATA= / ##DATA TABLE=,
 * trimmed) into intensities times `factor` <- JcampDx::decode_asdf / decode_affn,
 * spectrum/formats/jcampdx.rs:892-1091 (the reference's rewriting passes, then every
 * line minus its first token). *n_out receives the value count; MDG_CAPACITY when it
 * exceeds cap (nothing written). MDG_INVALID_ARGUMENT for blocks it leaves to the
 * Python reader: non-ASCII text, or data the reference rejects (the reader then raises
 * the reference's error). */
int mdg_jcampdx_decode(const char* data, size_t len, double factor, double* out, size_t cap,
                       size_t* n_out);

/* ---- device contexts ------------------------------------------------------ */
int mdg_device_count(int* count);
/* Page-locked host memory for spectrum rows and result tables (the storage behind
 * the reference's Spectrum rows, Arc<[f64]> in spectrum.rs:101-105, and the
 * Deconvolution's Vec<Lorentzian>, deconvolution.rs:45-60): the host-buffer entry
 * points DMA straight from / into it instead of staging through a bounce buffer.
 * Blocks are carved from 64 MiB slabs pinned on `device` (portable to every device)
 * and reused by size after mdg_host_free; the total is capped by MDGPU_PINNED_MAX
 * (bytes, default 8 GiB): beyond it, and without a device, MDG_ERR_OUT_OF_MEMORY /
 * MDG_ERR_NO_DEVICE, and the caller keeps ordinary memory. */
int mdg_host_alloc(int device, size_t bytes, void** out);
int mdg_host_free(void* p);
int mdg_ctx_create(int device, mdg_ctx** out);
int mdg_ctx_destroy(mdg_ctx* ctx);
/* Run subsequent work on this hipStream_t (NULL = the context's own stream). */
int mdg_ctx_set_stream(mdg_ctx* ctx, void* hip_stream);
/* The hipStream_t work is enqueued on (the context's own one unless set). */
int mdg_ctx_get_stream(mdg_ctx* ctx, void** hip_stream);
int mdg_ctx_synchronize(mdg_ctx* ctx);
/* Per-stage device timing with hipEvents on the context stream (0 = off).
 * Stages: 0 prep, 1 smooth, 2 detect, 3 select, 4 fit_init, 5 fit_superposition,
 * 6 fit_update, 7 retain, 8 mse_superposition, 9 mse_reduce, 10 superposition_vec,
 * 11 synth. times_ms/launches receive accumulated values (arrays of n_stages). */
int mdg_ctx_set_profiling(mdg_ctx* ctx, int enable);
/* Same, for the stages whose bit (1 << stage) is set in mask only. */
int mdg_ctx_set_profiling_mask(mdg_ctx* ctx, uint32_t mask);
int mdg_ctx_stage_times(mdg_ctx* ctx, double* times_ms, uint64_t* launches, int n_stages);
int mdg_ctx_reset_stage_times(mdg_ctx* ctx);
/* Name of the kernel(s) the last pipeline run on this context launched for `stage`
 * (same numbering; "+"-joined when a stage launches several, NULL when the stage did
 * not run). The string is static. Lets benchmarks label measurements with what the
 * engine actually dispatched. */
int mdg_ctx_stage_kernel(mdg_ctx* ctx, int stage, const char** name);
/* Latency mode (default 1): a one-spectrum pipeline of this context expects the GPU to
 * itself (the reference's deconvolute_spectrum called from one thread,
 * deconvoluter.rs:530-552) and takes the fit tiling fastest alone; 0 = many contexts
 * run concurrently (par_ callers spread over contexts, deconvoluter.rs:591-613,
 * 913-917): the tiling that leaves room for the others. Results are bit-identical
 * either way; only which shipped kernel runs changes. */
int mdg_ctx_set_latency_mode(mdg_ctx* ctx, int on);
/* The engine's MDG_* switches (kernel choices for tests and measurements, all
 * bit-exact) are read from the environment once, when the context is created; this
 * reads them again (nothing else on a call's path reads the environment). */
int mdg_ctx_reload_switches(mdg_ctx* ctx);
/* roctx ranges ("prep", "smooth", "detect", "select", "fit_superposition", ...) around
 * every pipeline stage this context launches (default off; MDG_ROCTX=1 at context
 * creation turns it on): a rocprofv3 trace with --marker-trace --hip-trace
 * --kernel-trace attributes each kernel to its stage with no events in the stream.
 * MDG_ERR_HIP when the roctx library cannot be loaded (the ranges stay off). */
int mdg_ctx_set_tracing(mdg_ctx* ctx, int on);

/* ---- hot path: host buffers ------------------------------------------------
 * x, y: n chemical shifts / intensities of a validated Spectrum
 * (spectrum.rs:120-150 invariants). sb0/sb1: signal boundaries in ppm ordered
 * per monotonicity as Spectrum stores them (spectrum.rs:854-863). ignore:
 * n_ignore merged (lo,hi) ppm pairs from mdg_ignore_region_add (NULL/0 = None).
 * out: capacity `cap`; *out_count always receives P_kept; MDG_CAPACITY if it
 * exceeds cap. */
int mdg_deconvolute(mdg_ctx* ctx, const double* x, const double* y, size_t n, double sb0,
                    double sb1, const mdg_settings* s, const double* ignore, size_t n_ignore,
                    mdg_lorentzian* out, size_t cap, size_t* out_count, double* out_mse);

/* Batch of b spectra of n points. Row i of x is x + i*x_stride (x_stride 0 =
 * one shared axis), row i of y is y + i*y_stride. sb: b (sb0,sb1) pairs.
 * out: b*cap Lorentzians (row i at out + i*cap); only rows below counts[i] are
 * written. counts/mse/status: b each.
 * Returns the first nonzero status (the reference's fail-fast error) or 0. */
int mdg_deconvolute_batch(mdg_ctx* ctx, size_t b, size_t n, const double* x, size_t x_stride,
                          const double* y, size_t y_stride, const double* sb,
                          const mdg_settings* s, const double* ignore, size_t n_ignore,
                          mdg_lorentzian* out, size_t cap, size_t* counts, double* mse,
                          int* status);

/* Same, each spectrum's arrays where the caller keeps them: row i of x / y is
 * x_rows[i] / y_rows[i] (n doubles each; one pointer repeated = one shared axis,
 * uploaded once). Replaces the same reference interfaces as mdg_deconvolute_batch
 * (deconvoluter.rs:651-661 / :700-710 take &[Spectrum], each Spectrum holding its
 * rows as Arc<[f64]>, spectrum.rs:101-105, clones sharing one axis): the binding
 * passes those slices' pointers and no caller-side stacking copy is made; the
 * engine gathers the rows into its page-locked ring (two slots of up to 32 MiB per
 * context) and sends one asynchronous DMA per slot. When every row lies in memory
 * from mdg_host_alloc, the rows are sent straight from there (one DMA per run of
 * adjacent rows, no host copy); `out` from mdg_host_alloc is filled by DMA too. */
int mdg_deconvolute_rows(mdg_ctx* ctx, size_t b, size_t n, const double* const* x_rows,
                         const double* const* y_rows, const double* sb, const mdg_settings* s,
                         const double* ignore, size_t n_ignore, mdg_lorentzian* out, size_t cap,
                         size_t* counts, double* mse, int* status);

/* Same with the rows in the compact form the Bruker reader builds them from, decoded
 * on the device bit for bit (the reference builds the f64 rows on the host,
 * spectrum/formats/bruker.rs:278-280 and :459-470, then calls the same
 * deconvoluter.rs:651-661 / :700-710): spectrum i's axis is
 *   x_j = axes[3i] - ((double)j * axes[3i+1]) / axes[3i+2]   (maximum, width, SI - 1),
 * evaluated in that operation order, and its intensities y_j = (double)y_rows[i][j] *
 * y_scale[i] (the 1r int32 samples times 2^NC_proc). A quarter of the bytes of
 * mdg_deconvolute_rows cross PCIe (n int32 per spectrum, no axis row). Page-locked
 * rows (mdg_host_alloc) are not copied: the smoother's launch reads them from host
 * memory and smooths each chunk as soon as it is decoded (MDG_DEC_OVERLAP=0: one
 * DMA first, as for other rows). The call returns after every read of the rows. */
int mdg_deconvolute_rows_i32(mdg_ctx* ctx, size_t b, size_t n, const double* axes,
                             const int32_t* const* y_rows, const double* y_scale, const double* sb,
                             const mdg_settings* s, const double* ignore, size_t n_ignore,
                             mdg_lorentzian* out, size_t cap, size_t* counts, double* mse,
                             int* status);

/* The decode step of mdg_deconvolute_rows_i32 alone, device to device (for callers
 * that keep inputs and results in HBM, e.g. the multi-GPU path before
 * mdg_deconvolute_batch_device): d_raw b x n int32 samples, d_desc b x 4 doubles
 * {maximum, width, divisor, scale}; writes the b x n rows d_x and d_y. Enqueued on
 * the context stream, no host synchronisation. */
int mdg_decode_rows_i32_device(mdg_ctx* ctx, size_t b, size_t n, const int32_t* d_raw,
                               const double* d_desc, double* d_x, double* d_y);

/* Same, every array resident on the context's device (d_ prefix); enqueued on
 * the context stream without any host synchronisation (capturable). d_counts and
 * d_status are int32. Call mdg_ctx_synchronize before reading outputs. */
int mdg_deconvolute_batch_device(mdg_ctx* ctx, size_t b, size_t n, const double* d_x,
                                 size_t x_stride, const double* d_y, size_t y_stride,
                                 const double* d_sb, const mdg_settings* s,
                                 const double* ignore, size_t n_ignore,
                                 mdg_lorentzian* d_out, size_t cap, int32_t* d_counts,
                                 double* d_mse, int32_t* d_status);

/* Diagnostics: copy the peak index triples of spectrum `spectrum` from the last
 * batch run on this context. which = 0: detected peaks (after the detector and
 * ignore filters, detector.rs:168-182 + noise_score_filter.rs:41-48),
 * which = 1: selected peaks (input of the fitter). *count receives the total. */
int mdg_ctx_last_peaks(mdg_ctx* ctx, size_t spectrum, int which, int32_t* left,
                       int32_t* center, int32_t* right, size_t cap, size_t* count);

/* Diagnostics: the smoothed intensities (MovingAverage::smooth_values,
 * moving_average.rs:53-83) of spectrum `spectrum` from the last batch run on this
 * context; n must equal that run's point count, and the run must have used the
 * moving-average smoother. */
int mdg_ctx_last_smoothed(mdg_ctx* ctx, size_t spectrum, double* out, size_t n);

/* Test hook (no reference counterpart): the fast-division range flags of `spectrum`
 * in the context's last batch. x_ok: both axis ends within |x| <= 2^100.
 * slow_mask: bit it (it < 29; bit 29 for later iterations) = fit iteration it ran the
 * plain IEEE division (its parameters or the axis outside the fast ranges; DESIGN.md
 * §2), bit 30 = the MSE summed every term directly with `/`, bit 31 = the exact-order
 * MSE (MDG_OPTION_EXACT_MSE) did. unsafe_kept: retained Lorentzians outside the
 * ranges. The reference always divides with `/` (lorentzian.rs:546-548); these show
 * which of the engine's two bit-identical forms ran. */
int mdg_ctx_last_range_flags(mdg_ctx* ctx, size_t spectrum, int32_t* x_ok, uint32_t* slow_mask,
                             int32_t* unsafe_kept);

/* Deconvoluter::optimize_settings (deconvoluter.rs:762-825): grid search over 27
 * moving-average x 10 noise-score x 3 analytical-fit settings on the reference
 * spectrum (x, y: n host values; sb0/sb1 and ignore as for mdg_deconvolute).
 * *best receives the first setting of minimum MSE in the reference's order and
 * *best_mse its MSE, summed in the reference's order. A failing combination
 * returns its status (the reference's `?`). */
int mdg_optimize_settings(mdg_ctx* ctx, const double* x, const double* y, size_t n, double sb0,
                          double sb1, const double* ignore, size_t n_ignore, mdg_settings* best,
                          double* best_mse);

/* Lorentzian::superposition_vec: out[i] = sum_j L[j](x[i]) in slice order. */
int mdg_superposition_vec(mdg_ctx* ctx, const double* x, size_t n, const mdg_lorentzian* L,
                          size_t p, double* out);
int mdg_superposition_vec_device(mdg_ctx* ctx, const double* d_x, size_t n,
                                 const mdg_lorentzian* d_L, size_t p, double* d_out);

/* Test support: acc0 + t[0] + ... + t[n-1] as a left fold (one rounding per add),
 * computed on the device by the windowed parallel fold that k_select uses for the
 * signal-free-region statistics (noise_score_filter.rs:129-138). The terms must be
 * >= +0 (MDG_INVALID_ARGUMENT otherwise); the result is bit-identical to the
 * sequential fold whatever the data. */
int mdg_ordered_sum(mdg_ctx* ctx, const double* t, size_t n, double acc0, double* out);

/* Test support: the superposition's fast quotients (used when every operand lies
 * in [2^-200, 2^200]) against the IEEE division the reference performs
 * (lorentzian.rs:546-548). variant 0 = div_rn (v_rcp_f64 + two Newton steps +
 * residual correction: the compiler's own expansion without its no-op scaling
 * wrappers; fit and superposition_vec), variant 1 = div_rn_1nr (one Newton step;
 * MSE only, not bit-exact). cases 0 = n pseudo-random pairs drawn from seed,
 * cases 1 = candidates i < n of mdg_division_hard_case (quotients about 2^-53 ulp
 * from a rounding midpoint). *mismatches receives the pairs whose bits differ,
 * *tested (may be NULL) the pairs checked. */
int mdg_check_division(mdg_ctx* ctx, int variant, int cases, uint64_t seed, uint64_t n,
                       uint64_t* mismatches, uint64_t* tested);
/* mdg_check_division(ctx, 0, 0, seed, n, mismatches, NULL). */
int mdg_check_fast_division(mdg_ctx* ctx, uint64_t seed, uint64_t n, uint64_t* mismatches);
/* Host (no GPU): the i-th constructed near-midpoint operand pair of stream seed
 * (the generator mdg_check_division runs on the device); MDG_INVALID_ARGUMENT
 * when candidate i is rejected (its numerator does not fit 53 bits). */
int mdg_division_hard_case(uint64_t seed, uint64_t i, double* n, double* d);

/* Device synthetic batch: d_x (n, shared axis x_i = xmax - (i*width)/(n-1)) and
 * d_y (b x n): y_s = in-order superposition of mdg_synth_lorentzians(seed0+s) +
 * mdg_synth_noise(seed0+s). */
int mdg_synth_batch_device(mdg_ctx* ctx, size_t b, size_t n, double xmax, double width,
                           uint64_t seed0, size_t n_peaks, double lo, double hi, double sigma,
                           double* d_x, double* d_y);
/* Same with mdg_synth_lorentzians_hw's half-width scale. */
int mdg_synth_batch_device_hw(mdg_ctx* ctx, size_t b, size_t n, double xmax, double width,
                              uint64_t seed0, size_t n_peaks, double lo, double hi, double hw_scale,
                              double sigma, double* d_x, double* d_y);

/* ---- spectrum queue (serving form of many concurrent calls) ----------------
 * Replaces Deconvoluter::par_deconvolute_spectrum called by many concurrent
 * callers (Deconvoluter is Send + Sync, deconvoluter.rs:913-917) and
 * par_deconvolute_spectra over an open-ended stream of spectra (:700-710).
 * A queue owns `lanes` engine contexts on `device` (own HIP stream and workspace
 * each; lanes <= 16) and deconvolutes spectra of n points with the settings and
 * ignore regions given at creation. Each submission is ONE spectrum with its own
 * device arrays; the queue gathers submissions into batches of max_batch spectra
 * (a batch is launched when it is full, or by flush/synchronize) and runs each
 * batch as one pipeline on the next lane, so consecutive batches overlap. The
 * results of a submission (count, mse, status as in mdg_deconvolute_batch_device,
 * min(count, cap) Lorentzians) are bit-identical to a mdg_deconvolute_batch_device
 * call on that spectrum. Submissions are asynchronous: the input arrays must stay
 * unchanged, and the outputs are written, until mdg_queue_synchronize returns.
 * Thread-safe. A failed batch launch makes every later call return its status. */
typedef struct mdg_queue mdg_queue;
int mdg_queue_create(int device, size_t n, size_t max_batch, int lanes, const mdg_settings* s,
                     const double* ignore, size_t n_ignore, mdg_queue** out);
int mdg_queue_submit(mdg_queue* q, const double* d_x, const double* d_y, double sb0, double sb1,
                     mdg_lorentzian* d_out, size_t cap, int32_t* d_count, double* d_mse,
                     int32_t* d_status);
/* Launch the open (partial) batch. */
int mdg_queue_flush(mdg_queue* q);
/* Flush deadline: once the first submission of the open batch has waited `us`
 * microseconds, a watcher thread of the queue launches the batch however full it
 * is (0 = off, the default: batches launch when full or on flush). Bounds a
 * submission's wait under light load; under full load batches fill first. */
int mdg_queue_set_flush_us(mdg_queue* q, int64_t us);
/* Flush, then wait until every submitted spectrum's outputs are written. */
int mdg_queue_synchronize(mdg_queue* q);
/* The engine context of lane `lane` (stage timing, kernel names; owned by the queue). */
int mdg_queue_lane(mdg_queue* q, int lane, mdg_ctx** ctx);
/* Batches launched, spectra launched, submissions waiting in the open batch. */
int mdg_queue_stats(mdg_queue* q, uint64_t* batches, uint64_t* spectra, size_t* open);
int mdg_queue_destroy(mdg_queue* q);
/* Test support: the queue's next batch launch fails with `status` (nonzero) before
 * anything is enqueued, as an allocation or launch failure would; the failure is
 * then sticky like any other (every later call returns it, destroy still works). */
int mdg_queue_fail_next_launch(mdg_queue* q, int status);

#ifdef __cplusplus
}
#endif
#endif /* MDGPU_H */
