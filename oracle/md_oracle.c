/*
 * md_oracle.c -- CPU restatement of the metabodecon deconvolution hot path.
 *
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY. Not part of the product: the HIP
 * library (libmdgpu.so) never links it. It is compiled with
 * -O3 -ffp-contract=off -fno-fast-math (oracle/Makefile) so that every f64 operation rounds
 * exactly like the Rust reference (rustc never contracts a*b+c into an FMA).
 *
 * Reference files are cited relative to metabodecon/src/ of
 * SombkeMaximilian/metabodecon-rust (snapshot 2025-07-04).
 *
 * Rust semantics reproduced:
 *   - Iterator::sum::<f64>() is a left fold starting at -0.0 (rustc >= 1.82);
 *   - powi(2) == x*x; f64::max/min == fmax/fmin (NaN-ignoring);
 *   - `f as usize` saturates (NaN/negative -> 0);
 *   - integer slicing that would panic in Rust returns MDO_REFERENCE_PANIC.
 */
#include "md_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* lib.rs:277 */
#define CHECK_PRECISION (1.0e+3 * DBL_EPSILON)

static size_t as_usize(double v) {
    /* Rust `f64 as usize`: saturating, NaN -> 0 */
    if (!(v > 0.0)) return 0;
    if (v >= 18446744073709551616.0) return SIZE_MAX;
    return (size_t)v;
}

void mdo_default_settings(mdo_settings* s) {
    /* smoother.rs:58-65, selector.rs:59-66, fitter.rs:59-63 */
    memset(s, 0, sizeof(*s));
    s->smoother = 1;
    s->smooth_iterations = 3;
    s->smooth_window = 3;
    s->selector = 1;
    s->scoring = 0;
    s->threshold = 5.0;
    s->fitter = 0;
    s->fit_iterations = 10;
}

int mdo_validate_settings(const mdo_settings* s) {
    /* smoother.rs:84-100 */
    if (s->smoother == 1) {
        if (s->smooth_iterations == 0 || s->smooth_window <= 1) return MDO_INVALID_SMOOTHING;
    } else if (s->smoother != 0) {
        return MDO_INVALID_SMOOTHING;
    }
    /* selector.rs:85-98 */
    if (s->selector == 1) {
        if (s->threshold <= 0.0 || !isfinite(s->threshold) || s->scoring != 0)
            return MDO_INVALID_SELECTION;
    } else if (s->selector != 0) {
        return MDO_INVALID_SELECTION;
    }
    /* fitter.rs:80-90 */
    if (s->fitter != 0 || s->fit_iterations == 0) return MDO_INVALID_FITTING;
    return MDO_OK;
}

/* ------------------------------------------------------------------------ */
/* smoothing/moving_average.rs:53-83 with circular_buffer.rs:34-59.
 * The FIFO holds the pass's pre-update values; we keep an explicit ring. */
int mdo_moving_average(double* values, size_t n, size_t iterations, size_t window_size) {
    size_t right = window_size / 2; /* moving_average.rs:114 */
    if (window_size == 0) return MDO_INVALID_SMOOTHING;
    if (right > n) return MDO_REFERENCE_PANIC; /* values_len - right underflows */
    double* ring = (double*)malloc(sizeof(double) * window_size);
    if (!ring) return MDO_INVALID_ARGUMENT;
    for (size_t it = 0; it < iterations; ++it) {
        size_t head = 0, len = 0; /* FIFO: oldest at ring[head] */
        double div = 1.0;
        double sum = 0.0; /* T::zero() */
        for (size_t k = 0; k < right; ++k) {
            /* cache.push(value) (never full here: right < window_size) */
            ring[(head + len) % window_size] = values[k];
            ++len;
            sum += values[k];
        }
        for (size_t i = 0; i < n - right; ++i) {
            double v = values[i + right];
            sum += v;
            if (len == window_size) {
                double popped = ring[head];
                head = (head + 1) % window_size;
                --len;
                ring[(head + len) % window_size] = v;
                ++len;
                sum -= popped;
            } else {
                ring[(head + len) % window_size] = v;
                ++len;
                div = 1.0 / (double)len;
            }
            values[i] = sum * div;
        }
        for (size_t i = n - right; i < n; ++i) {
            if (len > 0) {
                double popped = ring[head];
                head = (head + 1) % window_size;
                --len;
                sum -= popped;
                div = 1.0 / (double)len;
                values[i] = sum * div;
            }
        }
    }
    free(ring);
    return MDO_OK;
}

/* peak_selection/common.rs:5-10 */
void mdo_second_derivative(const double* y, size_t n, double* sd) {
    for (size_t k = 0; k + 2 < n; ++k) sd[k] = y[k] - 2.0 * y[k + 1] + y[k + 2];
}

/* peak_selection/detector.rs:189-196 */
size_t mdo_find_peak_centers(const double* sd, size_t n_sd, int64_t* centers, size_t cap) {
    size_t count = 0;
    for (size_t j = 0; j + 2 < n_sd; ++j) {
        double w0 = sd[j], w1 = sd[j + 1], w2 = sd[j + 2];
        if (w1 < 0. && w1 < w0 && w1 < w2) {
            if (count < cap) centers[count] = (int64_t)(j + 2);
            ++count;
        }
    }
    return count;
}

/* detector.rs:217-222 */
size_t mdo_find_right_border(const double* s, size_t len) {
    for (size_t p = 0; p + 2 < len; ++p) {
        double w0 = s[p], w1 = s[p + 1], w2 = s[p + 2];
        if (w1 > w0 && (w1 >= w2 || (w1 < 0. && w2 >= 0.))) return p + 1;
    }
    return len;
}

/* detector.rs:227-233 (windows().rev()) */
size_t mdo_find_left_border(const double* s, size_t len) {
    if (len < 3) return len;
    size_t p = 0;
    for (size_t q = len - 3 + 1; q-- > 0; ++p) {
        double w0 = s[q], w1 = s[q + 1], w2 = s[q + 2];
        if (w1 > w2 && (w1 >= w0 || (w1 < 0. && w0 >= 0.))) return p + 1;
    }
    return len;
}

/* detector.rs:168-182 + :202-212 */
size_t mdo_detect_peaks(const double* sd, size_t n_sd, int64_t* left, int64_t* center,
                        int64_t* right, size_t cap) {
    size_t count = 0;
    for (size_t j = 0; j + 2 < n_sd; ++j) {
        double w0 = sd[j], w1 = sd[j + 1], w2 = sd[j + 2];
        if (!(w1 < 0. && w1 < w0 && w1 < w2)) continue;
        size_t i = j + 2;
        size_t l = i - mdo_find_left_border(sd, i);
        size_t r = i + mdo_find_right_border(sd + (i - 1), n_sd - (i - 1));
        if (l != 0 && r != n_sd + 1) {
            if (count < cap) {
                left[count] = (int64_t)l;
                center[count] = (int64_t)i;
                right[count] = (int64_t)r;
            }
            ++count;
        }
    }
    return count;
}

/* scorer.rs:236-245 : min(sum |sd|[l-1..c], sum |sd|[c-1..r]) */
double mdo_score_minimum_sum(const double* abs_sd, int64_t l, int64_t c, int64_t r) {
    double a = -0.0, b = -0.0;
    for (int64_t k = l - 1; k < c; ++k) a += abs_sd[k];
    for (int64_t k = c - 1; k < r; ++k) b += abs_sd[k];
    return fmin(a, b);
}

/* common.rs:26-40 */
void mdo_peak_region_boundaries(const int64_t* centers, size_t n, size_t sb0, size_t sb1,
                                size_t* out_left, size_t* out_right) {
    size_t left = 0;
    for (size_t i = 0; i < n; ++i) {
        if ((size_t)centers[i] > sb0) { left = i; goto found_left; }
    }
    left = 0;
found_left:;
    size_t right = n - 1;
    for (size_t i = left; i < n; ++i) {
        if ((size_t)centers[i] > sb1) { right = i; break; }
    }
    *out_left = left;
    *out_right = right;
}

/* noise_score_filter.rs:129-138 */
void mdo_mean_sd(const double* scores, size_t n, double* mean_out, double* sd_out) {
    double sum = -0.0;
    for (size_t i = 0; i < n; ++i) sum += scores[i];
    double mean = sum / (double)n;
    double var = -0.0;
    for (size_t i = 0; i < n; ++i) {
        double d = scores[i] - mean;
        var += d * d;
    }
    var = var / (double)n;
    *mean_out = mean;
    *sd_out = sqrt(var);
}

/* ------------------------------------------------------------------------ */
/* fitting/peak_stencil.rs:113-131 ; st = {x1,x2,x3,y1,y2,y3} */
void mdo_mirror_shoulder(double* st) {
    int increasing = st[3] <= st[4] && st[4] <= st[5];
    int decreasing = st[3] >= st[4] && st[4] >= st[5];
    if (increasing) {
        st[5] = st[3];
        st[2] = 2.0 * st[1] - st[0];
    } else if (decreasing) {
        st[3] = st[5];
        st[0] = 2.0 * st[1] - st[2];
    }
}

/* fitting/fitter_analytical.rs:147-172 */
void mdo_solve_stencil(const double* st, double* sfhw, double* hw2, double* maxp) {
    double x1 = st[0], x2 = st[1], x3 = st[2], y1 = st[3], y2 = st[4], y3 = st[5];
    double numerator = x1 * x1 * y1 * (y2 - y3) + x2 * x2 * y2 * (y3 - y1)
                       + x3 * x3 * y3 * (y1 - y2);
    double divisor = 2.0 * (x1 - x2) * y1 * y2 + 2.0 * (x2 - x3) * y2 * y3
                     + 2.0 * (x3 - x1) * y3 * y1;
    double m = numerator / divisor;
    double t1 = x1 - m, t2 = x2 - m, t3 = x3 - m;
    double left = (y1 * (t1 * t1) - y2 * (t2 * t2)) / (y2 - y1);
    double right = (y2 * (t2 * t2) - y3 * (t3 * t3)) / (y3 - y2);
    double h = fmax((left + right) / 2.0, DBL_EPSILON);
    *maxp = m;
    *hw2 = h;
    *sfhw = y2 * (h + t2 * t2);
}

/* lorentzian.rs:546-548 + :606-611 */
double mdo_superposition(double x, const double* params, size_t p) {
    double acc = -0.0;
    for (size_t j = 0; j < p; ++j) {
        const double* L = params + 3 * j;
        double d = x - L[2];
        acc += L[0] / (L[1] + d * d);
    }
    return acc;
}

typedef struct {
    const double* x;
    const double* params;
    size_t p;
    double* out;
    size_t lo, hi;
} sup_job;

static void* sup_worker(void* arg) {
    sup_job* j = (sup_job*)arg;
    for (size_t i = j->lo; i < j->hi; ++i) j->out[i] = mdo_superposition(j->x[i], j->params, j->p);
    return NULL;
}

/* lorentzian.rs:631-663: rayon only distributes x, each sum stays in order */
void mdo_superposition_vec(const double* x, size_t n, const double* params, size_t p,
                           double* out, int threads) {
    if (threads <= 1 || n < 4096) {
        for (size_t i = 0; i < n; ++i) out[i] = mdo_superposition(x[i], params, p);
        return;
    }
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    sup_job jobs[256];
    size_t chunk = (n + (size_t)threads - 1) / (size_t)threads;
    int started = 0;
    for (int t = 0; t < threads; ++t) {
        size_t lo = (size_t)t * chunk, hi = lo + chunk;
        if (lo >= n) break;
        if (hi > n) hi = n;
        jobs[t] = (sup_job){x, params, p, out, lo, hi};
        if (pthread_create(&tid[t], NULL, sup_worker, &jobs[t]) != 0) {
            sup_worker(&jobs[t]);
            tid[t] = 0;
        }
        started = t + 1;
    }
    for (int t = 0; t < started; ++t)
        if (tid[t]) pthread_join(tid[t], NULL);
}

/* ------------------------------------------------------------------------ */
/* spectrum/spectrum.rs:633-635 (step) and :741-746 (signal_boundaries_indices) */
static void signal_boundaries_indices(const double* x, double sb0, double sb1, size_t* i0,
                                      size_t* i1) {
    double step = x[1] - x[0];
    *i0 = as_usize(floor((sb0 - x[0]) / step));
    *i1 = as_usize(ceil((sb1 - x[0]) / step));
}

/* deconvoluter.rs:865-904 */
long mdo_ignore_region_indices(const double* x, size_t n, double sb0, double sb1,
                               const double* regions, size_t n_regions, int64_t* pairs) {
    (void)n;
    double step = x[1] - x[0];
    double first = x[0];
    double lower_b = fmin(sb0, sb1), upper_b = fmax(sb0, sb1);
    size_t bi0, bi1;
    signal_boundaries_indices(x, sb0, sb1, &bi0, &bi1);
    size_t lower = bi0 < bi1 ? bi0 : bi1;
    size_t upper = bi0 < bi1 ? bi1 : bi0;
    long count = 0;
    for (size_t k = 0; k < n_regions; ++k) {
        double start = regions[2 * k], end = regions[2 * k + 1];
        if ((start < lower_b && end < lower_b) || (start > upper_b && end > upper_b)) continue;
        size_t fi = as_usize(floor((start - first) / step));
        if (fi < lower) fi = lower;
        size_t si = as_usize(ceil((end - first) / step));
        if (si > upper) si = upper;
        size_t b0 = fi < si ? fi : si;
        size_t b1 = fi < si ? si : fi;
        if (b0 < b1 - 1) { /* release-mode usize wrap when b1 == 0 */
            pairs[2 * count] = (int64_t)b0;
            pairs[2 * count + 1] = (int64_t)b1;
            ++count;
        }
    }
    return count;
}

/* deconvoluter.rs:438-472 */
long mdo_add_ignore_region(double* r, size_t n, size_t cap, double a, double b) {
    if (!isfinite(a) || !isfinite(b) || fabs(a - b) < CHECK_PRECISION) return -1;
    if (n + 1 > cap) return -2;
    r[2 * n] = fmin(a, b);
    r[2 * n + 1] = fmax(a, b);
    ++n;
    /* sort_unstable_by start (stable insertion sort gives the same order for
       distinct starts; equal starts are merged below anyway) */
    for (size_t i = 1; i < n; ++i) {
        double s0 = r[2 * i], s1 = r[2 * i + 1];
        size_t j = i;
        while (j > 0 && r[2 * (j - 1)] > s0) {
            r[2 * j] = r[2 * (j - 1)];
            r[2 * j + 1] = r[2 * (j - 1) + 1];
            --j;
        }
        r[2 * j] = s0;
        r[2 * j + 1] = s1;
    }
    for (;;) {
        size_t pos = n;
        for (size_t i = 0; i + 1 < n; ++i) {
            if (r[2 * (i + 1)] < r[2 * i + 1] || fabs(r[2 * i + 1] - r[2 * (i + 1)]) < CHECK_PRECISION) {
                pos = i;
                break;
            }
        }
        if (pos == n) break;
        double lo = fmin(r[2 * pos], r[2 * (pos + 1)]);
        double hi = fmax(r[2 * pos + 1], r[2 * (pos + 1) + 1]);
        r[2 * pos] = lo;
        r[2 * pos + 1] = hi;
        for (size_t i = pos + 1; i + 1 < n; ++i) {
            r[2 * i] = r[2 * (i + 1)];
            r[2 * i + 1] = r[2 * (i + 1) + 1];
        }
        --n;
    }
    return (long)n;
}

/* ------------------------------------------------------------------------ */
static int in_ignore(int64_t v, const int64_t* pairs, long n_pairs) {
    for (long k = 0; k < n_pairs; ++k)
        if (v >= pairs[2 * k] && v < pairs[2 * k + 1]) return 1;
    return 0;
}

/* The engine's fast-division range predicates (csrc/mdg_kernels.hip peak_fast_ok /
 * x_fast_ok), restated for the test hooks: a spectrum whose parameters or axis fail
 * them must take the plain IEEE division. Not part of the reference. */
static int fast_peak(const double* L) {
    double as = fabs(L[0]);
    return as >= 0x1p-200 && as <= 0x1p200 && L[1] >= 0x1p-200 && L[1] <= 0x1p200 &&
           fabs(L[2]) <= 0x1p100;
}
static uint64_t range_bit(const double* params, size_t P, unsigned v) {
    for (size_t p = 0; p < P; ++p)
        if (!fast_peak(params + 3 * p)) return (uint64_t)1 << (v < 63 ? v : 63);
    return 0;
}

/* deconvoluter.rs:530-552 (and par_deconvolute_spectrum :591-613) */
int mdo_deconvolute(const double* x, const double* y, size_t n, double sb0, double sb1,
                    const mdo_settings* s, const double* ignore, size_t n_ignore,
                    double* out_params, size_t cap, size_t* out_count, double* out_mse,
                    int threads, mdo_diag* diag) {
    int st = mdo_validate_settings(s);
    if (st) return st;
    if (n < 2) return MDO_INVALID_ARGUMENT;
    int rc = MDO_OK;
    double* work = (double*)malloc(sizeof(double) * n);
    double* sd = (double*)malloc(sizeof(double) * (n > 2 ? n - 2 : 1));
    size_t pcap = n / 2 + 2;
    int64_t* pl = (int64_t*)malloc(sizeof(int64_t) * pcap);
    int64_t* pc = (int64_t*)malloc(sizeof(int64_t) * pcap);
    int64_t* pr = (int64_t*)malloc(sizeof(int64_t) * pcap);
    int64_t* ig = (int64_t*)malloc(sizeof(int64_t) * (2 * n_ignore + 2));
    double* scores = NULL;
    double* params = NULL;
    double* st6 = NULL;
    double* rx = NULL;
    double* ry = NULL;
    double* sup = NULL;
    memcpy(work, y, sizeof(double) * n);

    /* deconvoluter.rs:531-532 */
    if (s->smoother == 1) {
        rc = mdo_moving_average(work, n, s->smooth_iterations, s->smooth_window);
        if (rc) goto done;
    }
    size_t sbi0, sbi1;
    signal_boundaries_indices(x, sb0, sb1, &sbi0, &sbi1);
    long n_ig = 0;
    if (n_ignore > 0) n_ig = mdo_ignore_region_indices(x, n, sb0, sb1, ignore, n_ignore, ig);
    if (diag) {
        diag->sbi0 = (int64_t)sbi0;
        diag->sbi1 = (int64_t)sbi1;
        diag->range_mask = 0;
        diag->unsafe_kept = 0;
        diag->x_ok = fabs(x[0]) <= 0x1p100 && fabs(x[n - 1]) <= 0x1p100;
    }

    /* selector.select_peaks */
    size_t n_sd = n >= 2 ? n - 2 : 0;
    mdo_second_derivative(work, n, sd);
    size_t np = mdo_detect_peaks(sd, n_sd, pl, pc, pr, pcap);
    if (np == 0) { rc = MDO_NO_PEAKS_DETECTED; goto done; }
    if (s->selector == 0) {
        /* detector_only.rs:305-315 */
        size_t k = 0;
        for (size_t i = 0; i < np; ++i) {
            if ((size_t)pl[i] >= sbi0 && (size_t)pr[i] <= sbi1) {
                pl[k] = pl[i]; pc[k] = pc[i]; pr[k] = pr[i]; ++k;
            }
        }
        np = k;
        if (n_ignore > 0) {
            k = 0;
            for (size_t i = 0; i < np; ++i) {
                if (!(in_ignore(pl[i], ig, n_ig) || in_ignore(pr[i], ig, n_ig))) {
                    pl[k] = pl[i]; pc[k] = pc[i]; pr[k] = pr[i]; ++k;
                }
            }
            np = k;
        }
        if (diag) diag->n_detected = (int64_t)np;
    } else {
        /* noise_score_filter.rs:41-48 */
        if (n_ignore > 0) {
            size_t k = 0;
            for (size_t i = 0; i < np; ++i) {
                if (!(in_ignore(pl[i], ig, n_ig) || in_ignore(pr[i], ig, n_ig))) {
                    pl[k] = pl[i]; pc[k] = pc[i]; pr[k] = pr[i]; ++k;
                }
            }
            np = k;
        }
        if (diag) diag->n_detected = (int64_t)np;
        /* :49-51 */
        for (size_t k = 0; k < n_sd; ++k) sd[k] = fabs(sd[k]);
        /* filter_peaks :91-126 */
        if (np == 0) { rc = MDO_REFERENCE_PANIC; goto done; } /* peaks.len()-1 underflow */
        size_t b0, b1;
        mdo_peak_region_boundaries(pc, np, sbi0, sbi1, &b0, &b1);
        if (b1 < b0) { rc = MDO_REFERENCE_PANIC; goto done; }
        if (b0 == 0 && b1 >= np) { rc = MDO_EMPTY_SIGNAL_FREE_REGION; goto done; }
        if (b0 == b1) { rc = MDO_EMPTY_SIGNAL_REGION; goto done; }
        size_t n_sfr = b0 + (np - b1);
        scores = (double*)malloc(sizeof(double) * (n_sfr + 1));
        size_t k = 0;
        for (size_t i = 0; i < b0; ++i) scores[k++] = mdo_score_minimum_sum(sd, pl[i], pc[i], pr[i]);
        for (size_t i = b1; i < np; ++i) scores[k++] = mdo_score_minimum_sum(sd, pl[i], pc[i], pr[i]);
        double mean, sdv;
        mdo_mean_sd(scores, n_sfr, &mean, &sdv);
        if (diag) { diag->sfr_mean = mean; diag->sfr_sd = sdv; }
        double thr = mean + s->threshold * sdv;
        k = 0;
        for (size_t i = b0; i < b1; ++i) {
            if (mdo_score_minimum_sum(sd, pl[i], pc[i], pr[i]) >= thr) {
                pl[k] = pl[i]; pc[k] = pc[i]; pr[k] = pr[i]; ++k;
            }
        }
        np = k;
        if (np == 0) { rc = MDO_EMPTY_SIGNAL_REGION; goto done; }
    }
    if (diag) {
        diag->n_selected = (int64_t)np;
        if (diag->sel_left && diag->sel_cap) {
            for (size_t i = 0; i < np && i < diag->sel_cap; ++i) {
                diag->sel_left[i] = pl[i];
                diag->sel_center[i] = pc[i];
                diag->sel_right[i] = pr[i];
            }
        }
    }

    /* fitter_analytical.rs:19-71 */
    {
        size_t P = np;
        params = (double*)malloc(sizeof(double) * 3 * (P + 1));
        st6 = (double*)malloc(sizeof(double) * 6 * (P + 1));
        rx = (double*)malloc(sizeof(double) * 3 * (P + 1));
        ry = (double*)malloc(sizeof(double) * 3 * (P + 1));
        sup = (double*)malloc(sizeof(double) * (3 * P > n ? 3 * P : n) + 8);
        for (size_t p = 0; p < P; ++p) {
            int64_t idx[3] = {pl[p], pc[p], pr[p]};
            for (int q = 0; q < 3; ++q) {
                rx[3 * p + q] = x[idx[q]];
                ry[3 * p + q] = y[idx[q]];
                st6[6 * p + q] = x[idx[q]];
                st6[6 * p + 3 + q] = y[idx[q]];
            }
            mdo_mirror_shoulder(st6 + 6 * p);
            mdo_solve_stencil(st6 + 6 * p, &params[3 * p], &params[3 * p + 1], &params[3 * p + 2]);
        }
        if (diag) diag->range_mask |= range_bit(params, P, 0);
        for (uint32_t it = 0; it < s->fit_iterations; ++it) {
            mdo_superposition_vec(rx, 3 * P, params, P, sup, threads);
            for (size_t p = 0; p < P; ++p) {
                double* q = st6 + 6 * p;
                q[3] = q[3] * (ry[3 * p] / sup[3 * p]);
                q[4] = q[4] * (ry[3 * p + 1] / sup[3 * p + 1]);
                q[5] = q[5] * (ry[3 * p + 2] / sup[3 * p + 2]);
                mdo_mirror_shoulder(q);
            }
            for (size_t p = 0; p < P; ++p)
                mdo_solve_stencil(st6 + 6 * p, &params[3 * p], &params[3 * p + 1], &params[3 * p + 2]);
            if (diag) diag->range_mask |= range_bit(params, P, it + 1);
        }
        size_t kept = 0;
        for (size_t p = 0; p < P; ++p) {
            if (params[3 * p] > CHECK_PRECISION && params[3 * p + 1] > CHECK_PRECISION) {
                params[3 * kept] = params[3 * p];
                params[3 * kept + 1] = params[3 * p + 1];
                params[3 * kept + 2] = params[3 * p + 2];
                ++kept;
            }
        }
        if (diag) {
            diag->n_kept = (int64_t)kept;
            for (size_t p = 0; p < kept; ++p) diag->unsafe_kept += !fast_peak(params + 3 * p);
        }
        if (out_count) *out_count = kept;
        if (kept > cap) { rc = MDO_CAPACITY; goto done; }
        if (out_params) memcpy(out_params, params, sizeof(double) * 3 * kept);

        /* deconvoluter.rs:540-543 + compute_mse :828-862 */
        mdo_superposition_vec(x, n, params, kept, sup, threads);
        size_t nreg = (size_t)n_ig + 1;
        double residuals = -0.0;
        size_t length = 0;
        for (size_t rgi = 0; rgi < nreg; ++rgi) {
            size_t a = rgi == 0 ? sbi0 : (size_t)ig[2 * (rgi - 1) + 1];
            size_t b = rgi + 1 == nreg ? sbi1 : (size_t)ig[2 * rgi];
            if (a > b || b > n) { rc = MDO_REFERENCE_PANIC; goto done; }
            double part = -0.0;
            for (size_t i = a; i < b; ++i) {
                double d = sup[i] - y[i];
                part += d * d;
            }
            residuals += part;
            length += b - a;
        }
        if (out_mse) *out_mse = residuals / (double)length;
    }

done:
    free(work); free(sd); free(pl); free(pc); free(pr); free(ig);
    free(scores); free(params); free(st6); free(rx); free(ry); free(sup);
    return rc;
}

typedef struct {
    size_t b, n;
    const double* x;
    size_t x_stride;
    const double* y;
    const double* sb;
    const mdo_settings* s;
    const double* ignore;
    size_t n_ignore;
    double* out;
    size_t cap;
    size_t* counts;
    double* mse;
    int* status;
    size_t next;
    pthread_mutex_t lock;
    int inner; /* threads per spectrum for its superpositions (rayon's nested par_iter) */
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    for (;;) {
        pthread_mutex_lock(&j->lock);
        size_t i = j->next++;
        pthread_mutex_unlock(&j->lock);
        if (i >= j->b) break;
        size_t cnt = 0;
        double m = 0.0;
        j->status[i] = mdo_deconvolute(j->x + i * j->x_stride, j->y + i * j->n, j->n,
                                       j->sb[2 * i], j->sb[2 * i + 1], j->s, j->ignore,
                                       j->n_ignore, j->out + i * j->cap * 3, j->cap, &cnt, &m,
                                       j->inner, NULL);
        j->counts[i] = cnt;
        j->mse[i] = m;
    }
    return NULL;
}

/* deconvoluter.rs:651-661 / :700-710 (fail-fast collect is done by the caller).
 * threads workers take spectra one at a time; each spectrum's superpositions use
 * inner threads (par_deconvolute_spectra maps par_deconvolute_spectrum, whose
 * par_fit_lorentzian / par_superposition_vec nest inside the outer par_iter). */
int mdo_deconvolute_batch_nested(size_t b, size_t n, const double* x, size_t x_stride,
                                 const double* y, const double* sb, const mdo_settings* s,
                                 const double* ignore, size_t n_ignore, double* out_params,
                                 size_t cap, size_t* counts, double* mse, int* status,
                                 int threads, int inner) {
    batch_job j = {b, n, x, x_stride, y, sb, s, ignore, n_ignore, out_params, cap,
                   counts, mse, status, 0, PTHREAD_MUTEX_INITIALIZER, inner < 1 ? 1 : inner};
    pthread_mutex_init(&j.lock, NULL);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    int started = 0;
    for (int t = 1; t < threads; ++t) {
        if (pthread_create(&tid[started], NULL, batch_worker, &j) == 0) ++started;
    }
    batch_worker(&j);
    for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
    pthread_mutex_destroy(&j.lock);
    for (size_t i = 0; i < b; ++i)
        if (status[i]) return status[i];
    return MDO_OK;
}

int mdo_deconvolute_batch(size_t b, size_t n, const double* x, size_t x_stride,
                          const double* y, const double* sb, const mdo_settings* s,
                          const double* ignore, size_t n_ignore, double* out_params,
                          size_t cap, size_t* counts, double* mse, int* status, int threads) {
    return mdo_deconvolute_batch_nested(b, n, x, x_stride, y, sb, s, ignore, n_ignore,
                                        out_params, cap, counts, mse, status, threads, 1);
}
