/*
 * md_oracle.h -- CPU restatement of metabodecon's Deconvoluter::deconvolute_spectrum
 * hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity oracle and the CPU baseline. Only tests/, the
 * smoke() check in __graft_entry__.py and bench.py's cpu_baseline leg may load
 * it. The product (libmdgpu.so) never links or calls it.
 *
 * Every function restates a reference function line by line (file:line cited
 * in md_oracle.c) with Rust's f64 semantics: no FMA contraction, left-fold sums
 * starting from -0.0, f64::max/min == fmax/fmin, `as usize` saturating.
 */
#ifndef MD_ORACLE_H
#define MD_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: identical numbering to include/mdgpu.h. */
enum {
    MDO_OK = 0,
    MDO_NO_PEAKS_DETECTED = 1,
    MDO_EMPTY_SIGNAL_REGION = 2,
    MDO_EMPTY_SIGNAL_FREE_REGION = 3,
    MDO_INVALID_SMOOTHING = 10,
    MDO_INVALID_SELECTION = 11,
    MDO_INVALID_FITTING = 12,
    MDO_INVALID_IGNORE_REGION = 13,
    MDO_INVALID_ARGUMENT = 20,
    MDO_CAPACITY = 21,
    MDO_REFERENCE_PANIC = 30
};

typedef struct mdo_settings {
    int32_t smoother;            /* 0 identity, 1 moving average */
    uint32_t smooth_iterations;
    uint32_t smooth_window;
    int32_t selector;            /* 0 detector only, 1 noise score filter */
    int32_t scoring;             /* 0 minimum sum */
    uint32_t fit_iterations;
    int32_t fitter;              /* 0 analytical */
    int32_t options;  /* mdgpu.h layout; the oracle always sums in the reference order */
    double threshold;
} mdo_settings;

typedef struct mdo_diag {
    /* optional intermediate outputs (may be NULL) */
    int64_t n_detected;          /* peaks after detect + ignore filter */
    int64_t n_selected;
    int64_t n_kept;
    int64_t sbi0, sbi1;
    double sfr_mean, sfr_sd;
    int64_t* sel_left;           /* capacity: sel_cap */
    int64_t* sel_center;
    int64_t* sel_right;
    size_t sel_cap;
    /* the engine's fast-division ranges (test hooks, mdgpu.h mdg_ctx_last_range_flags):
     * bit v of range_mask: some parameter of version v (0 = initial solve, v = after
     * iteration v-1's update) lies outside them; unsafe_kept: retained Lorentzians
     * outside them; x_ok: both axis ends inside |x| <= 2^100 */
    uint64_t range_mask;
    int64_t unsafe_kept;
    int32_t x_ok;
} mdo_diag;

void mdo_default_settings(mdo_settings* s);
int mdo_validate_settings(const mdo_settings* s);

/* smoothing/moving_average.rs:53-83 (in place) */
int mdo_moving_average(double* values, size_t n, size_t iterations, size_t window_size);

/* peak_selection/common.rs:5-10 ; out has n-2 entries */
void mdo_second_derivative(const double* y, size_t n, double* sd);

/* peak_selection/detector.rs:189-196 ; returns count, writes <= cap centers */
size_t mdo_find_peak_centers(const double* sd, size_t n_sd, int64_t* centers, size_t cap);
/* detector.rs:217-222 / :227-233 (slices given explicitly) */
size_t mdo_find_right_border(const double* sd_right, size_t len);
size_t mdo_find_left_border(const double* sd_left, size_t len);
/* detector.rs:168-182 ; returns count (0 => NoPeaksDetected) */
size_t mdo_detect_peaks(const double* sd, size_t n_sd, int64_t* left, int64_t* center,
                        int64_t* right, size_t cap);

/* scorer.rs:236-245 */
double mdo_score_minimum_sum(const double* abs_sd, int64_t left, int64_t center, int64_t right);
/* common.rs:26-40 */
void mdo_peak_region_boundaries(const int64_t* centers, size_t n, size_t sb0, size_t sb1,
                                size_t* out_left, size_t* out_right);
/* noise_score_filter.rs:129-138 */
void mdo_mean_sd(const double* scores, size_t n, double* mean, double* sd);

/* peak_stencil.rs:113-131 ; st = {x1,x2,x3,y1,y2,y3} */
void mdo_mirror_shoulder(double* st);
/* fitter_analytical.rs:147-172 */
void mdo_solve_stencil(const double* st, double* sfhw, double* hw2, double* maxp);

/* lorentzian.rs:606-663 ; params = {sfhw,hw2,maxp} x p (AoS) */
double mdo_superposition(double x, const double* params, size_t p);
void mdo_superposition_vec(const double* x, size_t n, const double* params, size_t p,
                           double* out, int threads);

/* deconvoluter.rs:865-904 ; returns number of index pairs written (pairs) or -1 */
long mdo_ignore_region_indices(const double* x, size_t n, double sb0, double sb1,
                               const double* regions, size_t n_regions, int64_t* pairs);
/* deconvoluter.rs:438-472 merge semantics; regions in/out as (lo,hi) pairs.
 * returns new count or -1 for InvalidIgnoreRegion */
long mdo_add_ignore_region(double* regions, size_t n_regions, size_t cap, double a, double b);

/* deconvoluter.rs:530-552 (threads>1 == par_deconvolute_spectrum, same bits) */
int mdo_deconvolute(const double* x, const double* y, size_t n, double sb0, double sb1,
                    const mdo_settings* s, const double* ignore, size_t n_ignore,
                    double* out_params, size_t cap, size_t* out_count, double* out_mse,
                    int threads, mdo_diag* diag);

/* deconvoluter.rs:651-710 ; per-spectrum status, parallel over spectra.
 * x, y: b rows of n (x_stride 0 => shared axis). out_params: b x cap x 3 */
int mdo_deconvolute_batch(size_t b, size_t n, const double* x, size_t x_stride,
                          const double* y, const double* sb, const mdo_settings* s,
                          const double* ignore, size_t n_ignore, double* out_params,
                          size_t cap, size_t* counts, double* mse, int* status, int threads);
int mdo_deconvolute_batch_nested(size_t b, size_t n, const double* x, size_t x_stride,
                          const double* y, const double* sb, const mdo_settings* s,
                          const double* ignore, size_t n_ignore, double* out_params,
                          size_t cap, size_t* counts, double* mse, int* status, int threads, int inner);

#ifdef __cplusplus
}
#endif
#endif
