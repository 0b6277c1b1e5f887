// mdg_kernels.hip -- CDNA4 (gfx950) kernels of the metabodecon deconvolution hot path.
//
// One batch = B spectra of N points. Per-spectrum work is indexed by
// blockIdx.y (or by the block for the per-spectrum scan kernels), so every
// wave belongs to exactly one spectrum and all peak-parameter reads are
// wave-uniform: they compile to scalar (SMEM) loads that feed VALU operands
// straight from SGPRs -- no LDS traffic and no barriers in the O(N*P) loops.
//
// Numerics contract (DESIGN.md "Parity"): binary64 everywhere, compiled with
// -ffp-contract=off, correctly rounded '/' and sqrt, and every order-dependent
// sum evaluated in the reference's order (left folds starting at -0.0).
#include <hip/hip_runtime.h>

#include "mdg_common.hpp"
#include "mdg_kernels.hpp"
#include "mdg_chain_asm.inc"

#include <cstdlib>
#include <mutex>
#include <vector>
#include <string>
#include <type_traits>

namespace mdg {

// ----------------------------------------------------------------------------------
// small device helpers
// ----------------------------------------------------------------------------------
__device__ __forceinline__ double lorentz(double x, double sfhw, double hw2, double maxp) {
    // lorentzian.rs:546-548  sfhw / (hw2 + (x - maxp).powi(2))
    const double d = x - maxp;
    return sfhw / (hw2 + d * d);
}

// Correctly rounded binary64 quotient without the div_scale/div_fmas/div_fixup
// wrappers. hipcc expands `n / d` (LLVM's AMDGPU f64 fdiv lowering) to
//   s = div_scale(d), r0 = rcp(s), e0 = fma(-s, r0, 1), r1 = fma(r0, e0, r0),
//   e1 = fma(-s, r1, 1), r2 = fma(r1, e1, r1), t = div_scale(n), q0 = t * r2,
//   rem = fma(-s, q0, t), q = div_fmas(rem, r2, q0), div_fixup(q, d, n).
// When |n|, |d| lie in [2^-200, 2^200] div_scale returns its operand unchanged
// and clears VCC (no exponent gap >= 768, no denormal operand or quotient, n
// not below 2^-969), div_fmas is then a plain fma, and div_fixup returns its
// input for the resulting normal, finite quotient. div_rn is that sequence
// minus the three no-op wrappers -- the same operations on the same operands
// in the same order -- so it returns the bits of `/` by construction, not by
// measurement. Callers use it only for spectra whose flags prove
// the operand ranges (peak_fast_ok + x_ok below); everything else takes `/`.
__device__ __forceinline__ double div_rn(double n, double d) {
    const double r0 = __builtin_amdgcn_rcp(d);
    const double e0 = __builtin_fma(-d, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-d, r1, 1.0);
    const double r2 = __builtin_fma(r1, e1, r1);
    const double q0 = n * r2;
    const double rem = __builtin_fma(-d, q0, n);
    return __builtin_fma(rem, r2, q0);
}

// The same without the second Newton step. r1 is within about an ulp of 1/d
// (it differs from r2 in a third of the cases), so the corrected quotient is off
// by at most ~2^-52 ulp before its last rounding: it equals `/` except for
// quotients within that distance of a rounding midpoint. Such operand pairs
// exist (mdg_check_division's constructed cases hit them), so this variant is
// NOT bit-exact and is used only by the MSE superposition, whose result the
// tests compare at 1e-12 relative (one such term moves it by ~1e-16).
__device__ __forceinline__ double div_rn_1nr(double n, double d) {
    const double r0 = __builtin_amdgcn_rcp(d);
    const double e0 = __builtin_fma(-d, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double q0 = n * r1;
    const double rem = __builtin_fma(-d, q0, n);
    return __builtin_fma(rem, r1, q0);
}

// Ranges under which sfhw / (hw2 + (x - maxp)^2) may use div_rn_fast: with
// |x|, |maxp| <= 2^100 the denominator lies in [2^-200, 2^203) and the quotient
// in (2^-404, 2^400] -- no scaling, no denormals, no overflow.
__device__ __forceinline__ bool peak_fast_ok(double sfhw, double hw2, double maxp) {
    const double as = fabs(sfhw);
    return as >= 0x1p-200 && as <= 0x1p200 && hw2 >= 0x1p-200 && hw2 <= 0x1p200 &&
           fabs(maxp) <= 0x1p100;
}
__device__ __forceinline__ bool x_fast_ok(double x) { return fabs(x) <= 0x1p100; }

template <bool FAST>
__device__ __forceinline__ double lorentz_t(double x, double sfhw, double hw2, double maxp) {
    const double d = x - maxp;
    const double den = hw2 + d * d;
    return FAST ? div_rn(sfhw, den) : sfhw / den;
}

// MSE only (see div_rn_1nr): not bit-exact, within the MSE's tolerance
template <bool FAST>
__device__ __forceinline__ double lorentz_mse(double x, double sfhw, double hw2, double maxp) {
    const double d = x - maxp;
    const double den = hw2 + d * d;
    return FAST ? div_rn_1nr(sfhw, den) : sfhw / den;
}

// In-order superposition (lorentzian.rs:606-611) of P wave-uniform Lorentzians.
// params is AoS {sfhw, hw2, maxp}; the address is uniform so the compiler emits
// s_load_dwordx* and uses SGPR operands.
typedef const __attribute__((address_space(4))) double* const_f64_ptr;

// MDG_SUP_GP peaks per group: the prefetch of the next group covers one group's
// evaluations (~62 cycles each per wave), which must outlast an L2 hit when only
// one or two waves share a SIMD
// (bench, B = 1: MSE 174 us with 4, 134 with 6 or 8; B = 256: no change)
#ifndef MDG_SUP_GP
#define MDG_SUP_GP 6
#endif
constexpr int kSupGP = MDG_SUP_GP;

template <bool FAST>
__device__ __forceinline__ void sup_group(double x, double& acc, const double (&c)[3 * kSupGP],
                                          double (&n)[3 * kSupGP], const_f64_ptr next, bool load_next) {
    double e[kSupGP];
    e[0] = lorentz_t<FAST>(x, c[0], c[1], c[2]);
    // the wait for c precedes e0; the next group's loads go out only after it
    __builtin_amdgcn_sched_barrier(0);
    if (load_next) {
#pragma unroll
        for (int k = 0; k < 3 * kSupGP; ++k) n[k] = next[k];
    }
#pragma unroll
    for (int k = 1; k < kSupGP; ++k) e[k] = lorentz_t<FAST>(x, c[3 * k], c[3 * k + 1], c[3 * k + 2]);
#pragma unroll
    for (int k = 0; k < kSupGP; ++k) acc += e[k];
}

template <bool FAST>
__device__ __forceinline__ double superpose_t(double x, const double* __restrict__ params_g, int P,
                                              double acc = -0.0) {
    // Parameters are read-only for the whole launch: address space 4 (constant)
    // lets the backend issue s_load_dwordx* and feed SGPR operands to the VALU.
    // Groups of kSupGP Lorentzians alternate between two SGPR buffers (A, B): each
    // group's loads for the group after it are issued behind the group's first
    // evaluation, so their latency hides behind the rest of the group.
    constexpr int GW = 3 * kSupGP;
    const const_f64_ptr params = (const_f64_ptr)(params_g);
    const int G = P / kSupGP;  // full groups
    int g = 0;
    if (G > 0) {
        double A[GW], B[GW];
#pragma unroll
        for (int k = 0; k < GW; ++k) A[k] = params[k];
        for (; g + 2 < G; g += 2) {
            sup_group<FAST>(x, acc, A, B, params + GW * (g + 1), true);
            sup_group<FAST>(x, acc, B, A, params + GW * (g + 2), true);
        }
        if (g + 1 < G) {
            sup_group<FAST>(x, acc, A, B, params + GW * (g + 1), true);
            sup_group<FAST>(x, acc, B, A, params, false);
        } else {
            sup_group<FAST>(x, acc, A, B, params, false);
        }
    }
    for (int j = kSupGP * G; j < P; ++j) {
        const_f64_ptr L = params + 3 * j;
        acc += lorentz_t<FAST>(x, L[0], L[1], L[2]);
    }
    return acc;
}

__device__ __forceinline__ double superpose(double x, const double* __restrict__ params, int P,
                                            bool fast) {
    return fast ? superpose_t<true>(x, params, P) : superpose_t<false>(x, params, P);
}

// Diagnostic stamps (tools/ubench/smooth_diag.hip builds with -DMDG_DIAG): per-wave
// cycle sums of kernel phases, written to a side buffer only. Empty otherwise.
#ifdef MDG_DIAG
__device__ long long* g_diag = nullptr;
__device__ int g_tf_mode = 0;
__device__ int g_chain_mode = 0;  // chain_diag: 1 = feeder publishes everything at once, no scaler; 2 = no scaler; 3 = instant feeder; 4 = passes one after another  // fit_diag: 1 = evaluators skip LDS stores, 2 = skip evaluation
// g_diag layout: DIAG_FLUSH records in [0, kDiagStampBase), KSTAMP slots after it
constexpr size_t kDiagStampBase = (size_t)1 << 22;
#define KSTAMP(slot)                                                           \
    if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && g_diag)      \
        g_diag[kDiagStampBase + (slot)] = (long long)__builtin_amdgcn_s_memtime()
#define DIAG_DECL unsigned long long _d_t = __builtin_amdgcn_s_memtime(); unsigned long long _d_acc[8] = {0};
#define DIAG_STAMP(i)                                                       \
    do {                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                  \
        const unsigned long long _n = __builtin_amdgcn_s_memtime();         \
        _d_acc[i] += _n - _d_t;                                             \
        _d_t = _n;                                                          \
        __builtin_amdgcn_sched_barrier(0);                                  \
    } while (0)
#define DIAG_FLUSH()                                                        \
    do {                                                                    \
        const size_t _r = ((size_t)(blockIdx.y * gridDim.x + blockIdx.x) * 16 + (threadIdx.x >> 6)) * 8; \
        if ((threadIdx.x & 63) == 0 && g_diag && _r + 8 <= kDiagStampBase)  \
            for (int _i = 0; _i < 8; ++_i) g_diag[_r + _i] = (long long)_d_acc[_i]; \
    } while (0)
#else
#define KSTAMP(slot)
#define DIAG_DECL
#define DIAG_STAMP(i)
#define DIAG_FLUSH()
#endif

// Workgroup barrier that orders LDS only. __syncthreads() also waits vmcnt(0), i.e.
// for every global load/store the wave has in flight -- that would drain the
// HBM prefetches and the write-back stores these pipelines keep in flight across
// barriers. Register results of global loads are still waited for by the
// compiler at their first use.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// D[k] := sd[k-1] = (s[k-1] - 2*s[k]) + s[k+1]   (common.rs:5-10, intensity aligned)
__device__ __forceinline__ double dsd(const double* __restrict__ s, int k) {
    return s[k - 1] - 2.0 * s[k] + s[k + 1];
}

template <int BS>
__device__ __forceinline__ int block_exclusive_scan(int v, int* lds, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NW = BS / 64;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    if (wid == 0) {
        int t = lane < NW ? lds[lane] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(t, o, 64);
            if (lane >= o) t += y;
        }
        if (lane < NW) lds[lane] = t;
    }
    __syncthreads();
    const int prefix = wid > 0 ? lds[wid - 1] : 0;
    *total = lds[NW - 1];
    __syncthreads();
    return prefix + x - v;
}

template <int BS>
__device__ __forceinline__ long long block_sum_ll(long long v, long long* lds) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NW = BS / 64;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    long long t = 0;
    for (int w = 0; w < NW; ++w) t += lds[w];
    __syncthreads();
    return t;
}

// first set bit at position >= pos and <= limit, or -1
__device__ __forceinline__ int find_next_bit(const uint64_t* __restrict__ m, int pos, int limit) {
    if (pos > limit) return -1;
    int w = pos >> 6;
    const int lastw = limit >> 6;
    uint64_t bits = m[w] & (~0ull << (pos & 63));
    for (;;) {
        if (bits) {
            const int r = (w << 6) + __ffsll((unsigned long long)bits) - 1;
            return r <= limit ? r : -1;
        }
        if (++w > lastw) return -1;
        bits = m[w];
    }
}

// last set bit at position <= pos and >= lo, or -1
__device__ __forceinline__ int find_prev_bit(const uint64_t* __restrict__ m, int pos, int lo) {
    if (pos < lo || pos < 0) return -1;
    int w = pos >> 6;
    const int firstw = lo >> 6;
    const int b = pos & 63;
    uint64_t bits = m[w] & (b == 63 ? ~0ull : ((1ull << (b + 1)) - 1ull));
    for (;;) {
        if (bits) {
            const int r = (w << 6) + 63 - __clzll((long long)bits);
            return r >= lo ? r : -1;
        }
        if (--w < firstw) return -1;
        bits = m[w];
    }
}

// The border predicates of k_flags at position k (2 <= k <= N-3), from the row itself:
// first right border >= pos (<= limit), last left border <= pos (>= lo), or -1. For
// borders beyond a chunk's window of masks (k_peaks with the predicates fused).
__device__ __forceinline__ int next_fr_row(const double* __restrict__ sm, int N, int pos, int limit) {
    pos = max(pos, 2);
    limit = min(limit, N - 3);
    if (pos > limit) return -1;
    double dm = dsd(sm, pos - 1), d0 = dsd(sm, pos);
    for (int k = pos; k <= limit; ++k) {
        const double dp = dsd(sm, k + 1);
        if (d0 > dm && (d0 >= dp || (d0 < 0. && dp >= 0.))) return k;
        dm = d0;
        d0 = dp;
    }
    return -1;
}
__device__ __forceinline__ int prev_fl_row(const double* __restrict__ sm, int N, int pos, int lo) {
    pos = min(pos, N - 3);
    lo = max(lo, 2);
    if (pos < lo) return -1;
    double dp = dsd(sm, pos + 1), d0 = dsd(sm, pos);
    for (int k = pos; k >= lo; --k) {
        const double dm = dsd(sm, k - 1);
        if (d0 > dp && (d0 >= dm || (d0 < 0. && dm >= 0.))) return k;
        dp = d0;
        d0 = dm;
    }
    return -1;
}
// find_next_bit / find_prev_bit over a window of mask words [wlo, wlo + nw) held in LDS
// (m[0] = word wlo), continuing on the row (next_fr_row / prev_fl_row) past its ends
__device__ __forceinline__ int next_bit_win(const uint64_t* m, int wlo, int nw, int pos, int limit,
                                            const double* sm, int N) {
    if (pos > limit) return -1;
    int w = pos >> 6;
    const int lastw = limit >> 6, whi = wlo + nw - 1;
    if (w <= whi) {
        uint64_t bits = m[w - wlo] & (~0ull << (pos & 63));
        for (;;) {
            if (bits) {
                const int r = (w << 6) + __ffsll((unsigned long long)bits) - 1;
                return r <= limit ? r : -1;
            }
            if (++w > lastw) return -1;
            if (w > whi) break;
            bits = m[w - wlo];
        }
        pos = w << 6;
    }
    return next_fr_row(sm, N, pos, limit);
}
__device__ __forceinline__ int prev_bit_win(const uint64_t* m, int wlo, int nw, int pos, int lo,
                                            const double* sm, int N) {
    if (pos < lo || pos < 0) return -1;
    int w = pos >> 6;
    const int firstw = lo >> 6;
    if (w >= wlo) {
        const int b = pos & 63;
        uint64_t bits = m[w - wlo] & (b == 63 ? ~0ull : ((1ull << (b + 1)) - 1ull));
        for (;;) {
            if (bits) {
                const int r = (w << 6) + 63 - __clzll((long long)bits);
                return r >= lo ? r : -1;
            }
            if (--w < firstw) return -1;
            if (w < wlo) break;
            bits = m[w - wlo];
        }
        pos = (w << 6) + 63;
    }
    return prev_fl_row(sm, N, pos, lo);
}

// ----------------------------------------------------------------------------------
// K0  prep: signal-boundary indices, ignore-region indices, MSE regions
// spectrum.rs:633-635,741-746 ; deconvoluter.rs:828-904
// ----------------------------------------------------------------------------------
// Per-spectrum set-up of a pipeline run: signal boundary indices, ignore-region
// indices, MSE-region checks, range flags, counters and status. k_prep runs it for
// every spectrum; with the chain smoother the pass-0 workgroup of each spectrum
// runs it instead (one launch fewer), no other kernel of that launch reading it.
// x_i of a compact row (k_decode_rows_i32's operations): d = {maximum, width, divisor}
__device__ __forceinline__ double dec_x(const double* d, int64_t i) {
    return d[0] - ((double)i * d[1]) / d[2];
}

__device__ __forceinline__ void prep_spectrum(const BatchArgs& a, const Workspace& w, int s) {
    // k_peaks' look-back slots start empty (k_flags cleared them until round 6; with the
    // predicates inside k_peaks no launch runs between the smoother and it)
    {
        const int ns = (w.W + kPkSlotWords - 1) / kPkSlotWords;
        unsigned long long* slot = (unsigned long long*)w.peak_cnt + (size_t)s * ns;
        for (int k = 0; k < ns; ++k) slot[k] = 0;
    }
    // rows the chain launch is still decoding (a.dec_rows): the axis's end points from
    // its descriptor, the values the decoders write
    const double* x = a.x + (size_t)s * a.x_stride;
    const double* xd = a.dec_desc ? a.dec_desc + 4 * (a.x_stride ? s : 0) : nullptr;
    const double x0 = xd ? dec_x(xd, 0) : x[0];
    const double x1 = xd ? dec_x(xd, 1) : x[1];
    const double xl = xd ? dec_x(xd, a.N - 1) : x[a.N - 1];
    const double step = x1 - x0;
    const double sb0 = a.sb[(size_t)s * a.sb_step], sb1 = a.sb[(size_t)s * a.sb_step + 1];
    const int64_t bi0 = as_index(floor((sb0 - x0) / step));
    const int64_t bi1 = as_index(ceil((sb1 - x0) / step));
    w.sbi[2 * s] = bi0;
    w.sbi[2 * s + 1] = bi1;
    int nig = 0;
    int64_t* pairs = w.ig + (size_t)s * 2 * w.ig_cap;
    if (a.n_ignore > 0) {
        const double lower_b = fmin(sb0, sb1), upper_b = fmax(sb0, sb1);
        const int64_t lower = bi0 < bi1 ? bi0 : bi1, upper = bi0 < bi1 ? bi1 : bi0;
        for (int k = 0; k < a.n_ignore; ++k) {
            const double st = a.ignore[2 * k], en = a.ignore[2 * k + 1];
            if ((st < lower_b && en < lower_b) || (st > upper_b && en > upper_b)) continue;
            int64_t fi = as_index(floor((st - x0) / step));
            if (fi < lower) fi = lower;
            int64_t si = as_index(ceil((en - x0) / step));
            if (si > upper) si = upper;
            const int64_t b0 = fi < si ? fi : si, b1 = fi < si ? si : fi;
            // `boundaries.0 < boundaries.1 - 1` in usize (wraps in release when b1 == 0)
            if (b1 == 0 || b0 < b1 - 1) {
                pairs[2 * nig] = b0;
                pairs[2 * nig + 1] = b1;
                ++nig;
            }
        }
    }
    w.n_ig[s] = nig;
    // MSE regions (sbi.0, ig0.s), (ig0.e, ig1.s), ... (igk.e, sbi.1); Rust slicing
    // panics when start > end or end > len.
    // Their cumulative lengths (mse_index: virtual index -> point) as well.
    int panic = 0;
    int64_t* cum = w.ig_cum + (size_t)s * (w.ig_cap + 2);
    int64_t run = 0;
    cum[0] = 0;
    for (int r = 0; r <= nig; ++r) {
        const int64_t lo = r == 0 ? bi0 : pairs[2 * (r - 1) + 1];
        const int64_t hi = r == nig ? bi1 : pairs[2 * r];
        if (lo > hi || hi > (int64_t)a.N) panic = 1;
        run += hi - lo;
        cum[r + 1] = run;
    }
    w.mse_panic[s] = panic;
    // the axis is monotone (Spectrum invariant): its end points bound every x
    w.x_ok[s] = x_fast_ok(x0) && x_fast_ok(xl);
    w.unsafe[4 * s] = 0;
    w.unsafe[4 * s + 1] = 0;
    w.unsafe[4 * s + 2] = 0;
    w.unsafe[4 * s + 3] = 0;
    w.unsafe_kept[s] = 0;
    w.status[s] = (a.N < 2) ? MDG_INVALID_ARGUMENT : 0;
    w.det_count[s] = 0;
    w.sel_count[s] = 0;
    w.kept_count[s] = 0;
}

__global__ void k_prep(BatchArgs a, Workspace w) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.B) return;
    prep_spectrum(a, w, s);
    // the chain smoother's progress counters start at zero (k_flags leaves them so)
    for (int p = 0; p < w.chain_P; ++p) w.chain_flags[((size_t)s * w.chain_P + p) * 32] = 0;
}

// ----------------------------------------------------------------------------------
// K1  iterated moving average, exact running-sum recurrence
// smoothing/moving_average.rs:53-83, circular_buffer.rs:34-59
// One lane per spectrum: the recurrence is order dependent (hard part 2).
// ----------------------------------------------------------------------------------
__device__ void ma_pass(const double* __restrict__ src, double* __restrict__ dst, int N, int ws) {
    const int right = ws / 2;
    double sum = 0.0;  // T::zero()
    double div = 1.0;  // T::one()
    for (int k = 0; k < right; ++k) sum += src[k];
    int len = right;
    const int nmain = N - right;
    int i = 0;
    // steady state (window full) is the hot loop; growth phase first
    for (; i < nmain && len < ws; ++i) {
        sum += src[i + right];
        ++len;
        div = 1.0 / (double)len;
        dst[i] = sum * div;
    }
    constexpr int U = 8;
    for (; i + U <= nmain; i += U) {
        double add[U], sub[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            add[u] = src[i + u + right];
            sub[u] = src[i + u + right - ws];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            sum += add[u];
            sum -= sub[u];
            dst[i + u] = sum * div;
        }
    }
    for (; i < nmain; ++i) {
        sum += src[i + right];
        sum -= src[i + right - ws];
        dst[i] = sum * div;
    }
    // tail: the FIFO holds src[N-len .. N)
    int head = N - len;
    for (int t = nmain; t < N; ++t) {
        if (len > 0) {
            sum -= src[head];
            ++head;
            --len;
            div = 1.0 / (double)len;
            dst[t] = sum * div;
        } else {
            dst[t] = src[t];
        }
    }
}

// ----------------------------------------------------------------------------------
// K1b  lane-pipelined moving average (the fast path of K1)
//
// The recurrence of every pass is inherently sequential, so the parallelism is
// across (spectrum, pass) pairs: lane = g*P + p runs pass p of spectrum g of the
// wave. Pass p emits its output o[i] at its tick i+R (R = ws/2); a wave_shr:1 DPP
// move hands it to lane p+1, which runs D = R+WS ticks behind and consumes it WS
// steps later from a register ring (slot = step mod WS). The extra WS-1 ticks of
// lag take the DPP/select/multiply off the recurrence's critical path, which is
// then just the reference's two dependent adds per tick. No LDS, no barriers,
// one wave per floor(64/P) spectra; the latency of P passes is ~ one pass.
//
// Per tick q of one pass (moving_average.rs:53-83), with the FIFO of pushed
// values kept in registers at slot (global step mod WS):
//   q <  R        : push in, sum += in                          (prefill)
//   R <= q < N    : sum += in; pop if full (q >= WS) else div = 1/(q+1); emit sum*div
//   N <= q < N+R  : sum -= pop; div = 1/(N+WS-1-q); emit sum*div  (tail)
// The popped value is always the one pushed WS ticks earlier, in the tail too.
// ----------------------------------------------------------------------------------
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

#define MDG_FMAC_BCAST(k) "v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n"
__device__ __forceinline__ void fold16(double& acc, double t, double one) {
    // s_nop 1: a VALU write of t may precede this DPP read of it
    asm volatile("s_nop 1\n" MDG_FMAC_BCAST(0) MDG_FMAC_BCAST(1) MDG_FMAC_BCAST(2)
                 MDG_FMAC_BCAST(3) MDG_FMAC_BCAST(4) MDG_FMAC_BCAST(5) MDG_FMAC_BCAST(6)
                 MDG_FMAC_BCAST(7) MDG_FMAC_BCAST(8) MDG_FMAC_BCAST(9) MDG_FMAC_BCAST(10)
                 MDG_FMAC_BCAST(11) MDG_FMAC_BCAST(12) MDG_FMAC_BCAST(13) MDG_FMAC_BCAST(14)
                 MDG_FMAC_BCAST(15)
                 : "+v"(acc)
                 : "v"(t), "v"(one));
}

// eight moving-average ticks k0..k0+7 of a row-replicated operand group: for each
// tick, acc += A[k] then acc -= P[k] (fma(+-t, 1, acc) rounds as the add / sub)
#define MDG_TICK(k)                                                                        \
    "v_fmac_f64_dpp %0, %1, %3 row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n"           \
    "v_fmac_f64_dpp %0, -%2, %3 row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n"
template <int K0>
__device__ __forceinline__ void fold8_ticks(double& acc, double A, double P, double one);
template <>
__device__ __forceinline__ void fold8_ticks<0>(double& acc, double A, double P, double one) {
    asm volatile("s_nop 1\n" MDG_TICK(0) MDG_TICK(1) MDG_TICK(2) MDG_TICK(3) MDG_TICK(4)
                 MDG_TICK(5) MDG_TICK(6) MDG_TICK(7)
                 : "+v"(acc)
                 : "v"(A), "v"(P), "v"(one));
}
template <>
__device__ __forceinline__ void fold8_ticks<8>(double& acc, double A, double P, double one) {
    asm volatile("s_nop 1\n" MDG_TICK(8) MDG_TICK(9) MDG_TICK(10) MDG_TICK(11) MDG_TICK(12)
                 MDG_TICK(13) MDG_TICK(14) MDG_TICK(15)
                 : "+v"(acc)
                 : "v"(A), "v"(P), "v"(one));
}

__device__ __forceinline__ double dpp_shr1(double v) {
    const long long b = __double_as_longlong(v);
    int lo = (int)(unsigned)(b & 0xffffffffll), hi = (int)(b >> 32);
    lo = __builtin_amdgcn_mov_dpp(lo, 0x138, 0xf, 0xf, true);  // wave_shr:1, lane 0 <- 0
    hi = __builtin_amdgcn_mov_dpp(hi, 0x138, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

template <int WS>
struct MAState {
    double sum, div;
    double fifo[WS];
};

template <int WS>
__device__ __forceinline__ double ma_tick_generic(MAState<WS>& st, const int slot, int q, int N,
                                                  double in) {
    constexpr int R = WS / 2;
    double emit = 0.0;
    if (q >= 0 && q < N + R) {
        if (q < R) {
            st.sum += in;
            st.fifo[slot] = in;
        } else if (q < N) {
            st.sum += in;
            if (q >= WS) st.sum -= st.fifo[slot];
            else st.div = 1.0 / (double)(q + 1);
            st.fifo[slot] = in;
            emit = st.sum * st.div;
        } else {
            st.sum -= st.fifo[slot];
            st.div = 1.0 / (double)(N + WS - 1 - q);
            emit = st.sum * st.div;
        }
    }
    return emit;
}

template <int WS>
__device__ __forceinline__ double ma_tick_steady(MAState<WS>& st, const int slot, double in) {
    st.sum += in;
    st.sum -= st.fifo[slot];
    st.fifo[slot] = in;
    return st.sum * st.div;
}

template <int WS>
__global__ __launch_bounds__(64) void k_smooth_pipe(BatchArgs a, Workspace w, int P, int spw) {
    constexpr int R = WS / 2, D = R + WS;
    constexpr int U = WS * ((32 + WS - 1) / WS);  // steps per prefetch block (multiple of WS)
    const int lane = threadIdx.x;
    const int g = lane / P, p = lane - g * P;
    const int s = blockIdx.x * spw + g;
    const bool valid = g < spw && s < a.B;
    const bool ok = valid && w.status[valid ? s : 0] == 0;
    const int N = a.N;
    const double* yrow = y_row(a, valid ? s : 0);
    double* orow = w.smooth + (size_t)(valid ? s : 0) * N;
    const bool feeder = p == 0;
    const bool writer = ok && p == P - 1;
    const int off = p * D;  // tick = step - off
    MAState<WS> st;
    st.sum = 0.0;  // T::zero()
    st.div = 1.0;  // T::one()
#pragma unroll
    for (int k = 0; k < WS; ++k) st.fifo[k] = 0.0;
    double rq[WS];  // received emits of the previous pass, consumed WS steps later
#pragma unroll
    for (int k = 0; k < WS; ++k) rq[k] = 0.0;
    const int T = (P - 1) * D + N + R;
    int tA = ((P - 1) * D + WS + WS - 1) / WS * WS;
    const int nblk = N > tA ? (N - tA) / U : 0;
    int tB = tA + nblk * U;
    if (nblk == 0) tA = tB = 0;

    auto generic = [&](int t0, int t1) {
        for (int tt = t0; tt < t1; tt += WS) {
#pragma unroll
            for (int k = 0; k < WS; ++k) {
                const int q = tt + k - off;
                double in = rq[k];
                if (feeder) in = (q >= 0 && q < N) ? yrow[q] : 0.0;
                const double e = ma_tick_generic<WS>(st, k, q, N, in);
                if (writer && q >= R && q < N + R) orow[q - R] = e;
                rq[k] = dpp_shr1(e);
            }
        }
    };
    generic(0, tA);
    if (tB > tA) {
        double buf[U], nbuf[U], ob[U];
        if (feeder) {
#pragma unroll
            for (int k = 0; k < U; ++k) buf[k] = yrow[tA + k];
        } else {
#pragma unroll
            for (int k = 0; k < U; ++k) buf[k] = 0.0;
        }
        for (int t0 = tA; t0 < tB; t0 += U) {
            if (feeder && t0 + U < tB) {
#pragma unroll
                for (int k = 0; k < U; ++k) nbuf[k] = yrow[t0 + U + k];
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const double in = feeder ? buf[k] : rq[k % WS];
                const double e = ma_tick_steady<WS>(st, k % WS, in);
                ob[k] = e;
                rq[k % WS] = dpp_shr1(e);
            }
            if (writer) {  // one exec-masked burst of U stores per block
                double* o = orow + (t0 - off - R);
#pragma unroll
                for (int k = 0; k < U; ++k) o[k] = ob[k];
            }
#pragma unroll
            for (int k = 0; k < U; ++k) buf[k] = nbuf[k];
        }
    }
    generic(tB, T);
}

// ----------------------------------------------------------------------------------
// K1d  chain moving average: one workgroup per (spectrum, pass), passes on
// different CUs (the fast path for small and medium batches).
//
// Measured on gfx950 (tools/ubench/issue.hip): a dependent v_add_f64 costs ~4.8
// cycles, any other instruction of the same wave 3-10 more, an s_load_dwordx16
// plus its wait almost nothing when it feeds 8 ticks, and one CU issues one
// 16-byte vector store per ~16 cycles across all its waves. So each pass runs
// on its own CU, in four waves (one per SIMD):
//  * chain wave: issues little besides the reference's two dependent adds per
//    tick (moving_average.rs:69-80, in j = i + R form below) on SGPR operands,
//    and stores one checkpoint per kChainG = 48 ticks (the group's last raw sum);
//  * feeder wave: waits for the previous pass's published blocks (sc1 polls),
//    publishes them to the chain (in_ready in LDS), pulls them into L2 and
//    touches them into the scalar cache ahead of the chain;
//  * two scaler waves, batches of kChainScBatch output blocks round-robin: replay
//    each group of kChainG ticks from its checkpoint with the same two operations
//    (bit-identical sums), multiply by the reference's 1/len (moving_average.rs:
//    66-81: 1/len while the buffer grows, 1/ws, then 1/len in the tail) and
//    publish finished batches to the next pass in batch order (sc1 stores,
//    vmcnt(0), atomic-max counter; the consumer polls with sc1 loads --
//    MI355X_MICROARCH.md, cross-CU hand-offs).
//
// Per pass, in j = 0 .. N+R-1:  if j < N: sum += in[j];  if j >= WS: sum -= in[j-WS];
//                               raw[j] = sum  (= the reference's sum after tick j-R)
// out[i] = raw[i+R] * (1/len_i).  Blocks of CB ticks; the steady middle runs the
// generated asm of mdg_chain_asm.inc, the first and last blocks the code below.
// Every wait has a spin limit after which the spectrum reports MDG_ERR_HIP and
// all its waves drain (never expected; it bounds a protocol bug).
// ----------------------------------------------------------------------------------
constexpr int kChainCB = MDG_CHAIN_CB;
#ifndef MDG_CHAIN_PF
#define MDG_CHAIN_PF 8
#endif
constexpr int kChainScalers = 2;         // scaler waves (round-robin batches)
#ifndef MDG_CHAIN_SCB
#define MDG_CHAIN_SCB 8  // chain_diag ms: 2: 1.27, 4: 0.77, 8: 0.595, 12: 0.589, 16: 0.596; bench: 12 is 1% slower
#endif
constexpr int kChainScBatch = MDG_CHAIN_SCB;  // output blocks per scaler batch
// (round 6, measured and removed: batches of 1, 2, 4 blocks at the start and halving
// over the last 16 blocks, to shorten the three-pass pipeline's fill and drain.
// chain_diag, B = 1: 2048 points 46 -> 54 us, 131072 points 589 -> 603 us; the
// downstream chains ran 18-19 instead of 10.6-11 cycles per tick at 2048 points,
// starved by small batches whose fixed cost -- staging loads, the vmcnt drain, the
// ordered publication -- the scalers pay per batch.)
constexpr int kChainG = MDG_CHAIN_G;      // ticks per stored checkpoint in steady blocks
static_assert(kChainG % 8 == 0 && kChainCB % kChainG == 0, "checkpoint groups tile the blocks");
constexpr int kChainPrefetch = MDG_CHAIN_PF;  // input blocks touched into the scalar cache ahead
// Input blocks each chain pulls into L2 ahead of itself: at most 64, and about 1 MB
// of pulled lines per XCD in all (launch_chain). At B = 256 an XCD runs 96 chains, and
// 64 blocks (48 KB) ahead each was 4.6 MB against a 4 MB L2: lines were evicted before
// the chain and its scalers read them, and the scalers read them again from memory
// (round 5, queue 256 x 2: smoother reads 7.4 -> 4.3 MB per spectrum, headline
// 15.9k -> 16.5k spectra/s with 16 or 8 blocks; 32: 16.2k)
constexpr int kChainL2Ahead = 64;
constexpr int kChainL2Bytes = 1 << 20;
constexpr unsigned kChainSpins = 1u << 22;
// largest chain grid (workgroups, padded to 8 spectra x passes) launched with
// whole-CU workgroups: 8 spectra x 3 passes at the defaults, 232 CUs left free
constexpr int kChainExclMax = 24;

int64_t chain_stride_for(int N, int ws) {
    const int64_t span = (int64_t)N + ws / 2 + 2 * kChainCB;
    return (span + 63) / 64 * 64;
}

size_t chain_bytes(int B, int N, int ws, int passes) {
    const size_t row = (size_t)chain_stride_for(N, ws) * 8;
    return row * (size_t)B * (2 * (size_t)passes - 1) + (size_t)B * passes * 128 + 1024;
}

bool chain_supported(int B, int N, int iters, int ws) {
    return ws >= 2 && ws <= 8 && iters >= 1 && iters <= 16 && B >= 1 && B * iters <= 2048 &&
           N >= 4 * kChainCB + 16;
}

#ifdef MDG_DIAG
// (a diagnostic build run without a stamp buffer, mdg_debug_set_diag, writes nothing)
#define DIAGC(k, v) \
    if (lane == 0 && g_diag) g_diag[((size_t)s * P + p) * 32 + (k)] = (long long)(v)
#define DIAGC_ADD(k, v) \
    if (lane == 0 && g_diag) g_diag[((size_t)s * P + p) * 32 + (k)] += (long long)(v)
#else
#define DIAGC(k, v)
#define DIAGC_ADD(k, v)
#endif

struct ChainCtl {
    int in_ready;  // input blocks available in the scalar cache (helper -> chain)
    int raw_done;  // j-blocks whose raw sums are stored (chain -> helper)
    int abort;
    int pub;       // scaler batches published (scaler -> scaler)
};

// wave-uniform copies for "s" asm operands (values computed under a branch the
// compiler treats as divergent would otherwise land in VGPRs)
template <typename T>
__device__ __forceinline__ T* sgpr_ptr(T* p) {
    const uint64_t v = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int sgpr_int(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ unsigned lds_offset(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int WS>
__device__ __forceinline__ int chain_steady(const double* in_grp, double* raw, int blk, int cnt,
                                            int nib, unsigned lds, double& sum, int& stat);

#define MDG_CHAIN_CLOBBERS                                                                  \
    "s16", "s17", "s18", "s19", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", \
    "s29", "s30", "s31", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", \
    "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", \
    "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", \
    "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", \
    "s92", "s93", "s94", "s95", "s96", "s97", "s98", "s99", "v0", "v1", "v2", "v3", "v4", "v5",  \
    "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "scc", \
    "memory"

#define MDG_CHAIN_STEADY(WSV)                                                                \
    template <>                                                                              \
    __device__ __forceinline__ int chain_steady<WSV>(const double* in_grp, double* raw,     \
                                                     int blk, int cnt, int nib, unsigned lds, \
                                                     double& sum, int& stat) {              \
        int blk_out, st;                                                                     \
        asm volatile(MDG_CHAIN_ASM_##WSV                                                     \
                     : [sum] "+v"(sum), [blk_out] "=s"(blk_out), [stat] "=s"(st)             \
                     : [in] "s"(sgpr_ptr(in_grp)), [raw] "s"(sgpr_ptr(raw)),                 \
                       [blk] "s"(sgpr_int(blk)), [cnt] "s"(sgpr_int(cnt)),                  \
                       [nib] "s"(sgpr_int(nib)), [lds] "v"(lds)                              \
                     : MDG_CHAIN_CLOBBERS);                                                  \
        stat = st;                                                                           \
        return blk_out;                                                                      \
    }
MDG_CHAIN_STEADY(2)
MDG_CHAIN_STEADY(3)
MDG_CHAIN_STEADY(4)
MDG_CHAIN_STEADY(5)
MDG_CHAIN_STEADY(6)
MDG_CHAIN_STEADY(7)
MDG_CHAIN_STEADY(8)

// touch the 64-byte lines of cnt consecutive input blocks (scalar cache prefetch
// for the chain). All loads are in flight together and land in the same scratch
// SGPRs (their values are never used); one wait at the end, so no load is still
// outstanding when the compiler reuses those registers.
__device__ __forceinline__ void chain_touch(const double* p, int cnt) {
    static_assert(kChainCB == 96, "the touch loop below covers 12 lines per block");
#define MDG_TOUCH_LINE(k) "s_load_dwordx16 s[40:55], s[56:57], " #k "\n"
    asm volatile(
        "s_mov_b64 s[56:57], %0\n"
        "s_mov_b32 s58, %1\n"
        "Ltouch%=:\n" MDG_TOUCH_LINE(0) MDG_TOUCH_LINE(64) MDG_TOUCH_LINE(128) MDG_TOUCH_LINE(192)
            MDG_TOUCH_LINE(256) MDG_TOUCH_LINE(320) MDG_TOUCH_LINE(384) MDG_TOUCH_LINE(448)
                MDG_TOUCH_LINE(512) MDG_TOUCH_LINE(576) MDG_TOUCH_LINE(640) MDG_TOUCH_LINE(704)
        "s_add_u32 s56, s56, 768\n"
        "s_addc_u32 s57, s57, 0\n"
        "s_sub_u32 s58, s58, 1\n"
        "s_cmp_lg_u32 s58, 0\n"
        "s_cbranch_scc1 Ltouch%=\n"
        "s_waitcnt lgkmcnt(0)\n" ::"s"(sgpr_ptr(p)),
        "s"(sgpr_int(cnt))
        : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52",
          "s53", "s54", "s55", "s56", "s57", "s58", "scc", "memory");
#undef MDG_TOUCH_LINE
}


// load cnt consecutive blocks (this lane's 16 bytes of each) into L2 and wait:
// one asm statement, so no in-flight load can land in a register the compiler
// has reused
__device__ __forceinline__ void chain_l2_pull(const double* p, int cnt) {
    asm volatile(
        "v_mov_b64 v[24:25], %0\n"
        "s_mov_b32 s40, %1\n"
        "Lpull%=:\n"
        "global_load_dwordx4 v[20:23], v[24:25], off\n"
        "v_lshl_add_u64 v[24:25], v[24:25], 0, %2\n"
        "s_sub_u32 s40, s40, 1\n"
        "s_cmp_lg_u32 s40, 0\n"
        "s_cbranch_scc1 Lpull%=\n"
        "s_waitcnt vmcnt(0)\n" ::"v"(p),
        "s"(sgpr_int(cnt)), "s"((unsigned long long)(kChainCB * 8))
        : "v20", "v21", "v22", "v23", "v24", "v25", "s40", "scc", "memory");
}

// Rows decoded while the chain smooths them (mdg_deconvolute_rows_i32 with
// page-locked rows; y rows padded to whole 128-byte lines, kDecRowAlign, and a chunk
// is a whole number of 96-double blocks, 768 bytes, so every line belongs to one
// chunk of one row and one decoder): the chain launch's first ndec workgroups read the int32 rows
// straight from host memory and write y_i = raw_i * scale (k_decode_rows_i32's
// operation) chunk by chunk, kDecChunks chunks per row, chunk-major over the batch
// (the first chunks of every row first), each chunk published
// (Workspace::dec_flags = dec_gen) the way a chain pass publishes its output
// blocks: agent-scope stores, vmcnt(0), then the flag; pass 0's feeder polls the
// flags. The x rows follow (the chain does not read them; prep_spectrum takes the
// axis from its descriptor). Decoders wait for nothing, so they always finish;
// the chain waits for them within its spin limits.
__device__ __forceinline__ int dec_block_chunk(int nIB) { return (nIB + kDecChunks - 1) / kDecChunks; }
__device__ __forceinline__ void chain_decode(const BatchArgs& a, const Workspace& w, int d, int ndec) {
    const int N = a.N, B = a.B, NT = blockDim.x, tid = threadIdx.x;
    const int pts = dec_block_chunk((N + kChainCB - 1) / kChainCB) * kChainCB;  // a multiple of 4
    constexpr int U = 3;
    for (int t = d; t < kDecChunks * B; t += ndec) {
        const int c = t / B, s = t - c * B;
        const int lo = c * pts, hi = min(N, lo + pts);
        const int32_t* __restrict__ r = a.dec_rows[s];
        const double sc = a.dec_desc[4 * s + 3];
        double* yr = const_cast<double*>(a.y) + (size_t)s * a.y_stride;
        // 16-byte host reads where the row allows them (lo is a multiple of 4)
        const bool v4 = ((uintptr_t)r & 15) == 0;
        const int n4 = v4 && hi > lo ? (hi - lo) >> 2 : 0;
        for (int b4 = 0; b4 < n4; b4 += U * NT) {
            int4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {  // all host reads in flight together
                const int q = b4 + u * NT + tid;
                v[u] = q < n4 ? ((const int4*)(r + lo))[q] : make_int4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int q = b4 + u * NT + tid;
                if (q < n4) {
                    double* o = yr + lo + 4 * q;
                    __hip_atomic_store(o, (double)v[u].x * sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(o + 1, (double)v[u].y * sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(o + 2, (double)v[u].z * sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(o + 3, (double)v[u].w * sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        for (int i = lo + 4 * n4 + tid; i < hi; i += NT)  // the rest (unaligned rows, the row's tail)
            __hip_atomic_store(yr + i, (double)r[i] * sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // the whole of wave 0 publishes (a wave-uniform branch and value)
        if (tid < 64)
            __hip_atomic_store(w.dec_flags + (size_t)s * kDecChunks + c, a.dec_gen, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    // x rows (read only by later launches): one row when the axis is shared
    const int xrows = a.x_stride ? B : 1;
    double* xr0 = const_cast<double*>(a.x);
    for (int t = d; t < kDecChunks * xrows; t += ndec) {
        const int c = t / xrows, s = t % xrows;
        const int lo = c * pts, hi = min(N, lo + pts);
        const double* xd = a.dec_desc + 4 * s;
        double* xr = xr0 + (size_t)s * a.x_stride;
        for (int i = lo + tid; i < hi; i += NT) xr[i] = dec_x(xd, i);
    }
}

// EXCL: each wave claims the whole register file of its SIMD (256 arch + 256 acc
// VGPRs), so a chain workgroup owns its CU outright. Small batches only (the
// launcher requires B * passes <= kChainExclMax): with one workgroup per CU every
// pass must still find a CU of its own. Concurrent pipelines on other streams
// then never put waves next to the chain, feeder and scaler waves (which spin
// and would slow them, and whose neighbours they would slow: a stream's
// k_fit_sup_tf launch lasts as long as its slowest workgroup).
template <int WS, bool EXCL>
__global__ __launch_bounds__(64 * (2 + kChainScalers)) void k_smooth_chain(BatchArgs a, Workspace w, int P,
                                                                            int fused_prep, int ndec,
                                                                            int l2ahead) {
    if constexpr (EXCL) {
        asm volatile("v_mov_b32 v255, 0" ::: "v255");
        asm volatile("v_accvgpr_write_b32 a255, 0" ::: "a255");
    }
    // the first ndec workgroups (a multiple of 8) decode the rows (chain_decode)
    if ((int)blockIdx.x < ndec) {
        chain_decode(a, w, blockIdx.x, ndec);
        return;
    }
    // workgroup id -> (spectrum, pass): the P passes of a spectrum share id % 8
    // (the XCD of round-robin dispatch), so their hand-offs stay in one L2
    const int id = blockIdx.x - ndec;
    const int x8 = id & 7, j8 = id >> 3;
    const int p = j8 % P, s = (j8 / P) * 8 + x8;
    if (s >= a.B) return;
    if (fused_prep) {
        // k_prep's work; its status is 0 (N >= 2 is checked on the host), so no
        // pass of this launch needs to read it
        if (p == 0 && threadIdx.x == 0) prep_spectrum(a, w, s);
    } else if (w.status[s]) {
        return;  // uniform per spectrum
    }
    constexpr int R = WS / 2;
    constexpr int CB = kChainCB;
    const int N = a.N;
    const int nJ = N + R;
    const int nJB = (nJ + CB - 1) / CB;     // j-blocks of the chain
    const int nIB = (N + CB - 1) / CB;      // input blocks
    const int nOB = nIB;                    // output blocks
    const int64_t L = w.chain_stride;
    const double* in = p == 0 ? y_row(a, s)
                              : w.chain_tmp + ((size_t)(p - 1) * a.B + s) * L;
    double* out = p == P - 1 ? w.smooth + (size_t)s * N : w.chain_tmp + ((size_t)p * a.B + s) * L;
    double* raw = w.chain_raw + ((size_t)p * a.B + s) * L;
    int32_t* my_flag = w.chain_flags + ((size_t)s * w.chain_P + p) * 32;
    const int32_t* up_flag = p > 0 ? w.chain_flags + ((size_t)s * w.chain_P + p - 1) * 32 : nullptr;

    __shared__ ChainCtl ctl;
    // scaler staging (one wave): inputs and raw sums of one batch of output blocks
    // (one pad double per 32: the replay lanes, G doubles apart, hit distinct banks)
    constexpr int kScSpan = kChainScBatch * kChainCB + kChainG + 8;
    __shared__ double sc_in_all[kChainScalers][kScSpan + kScSpan / 32 + 1];
    __shared__ double sc_raw_all[kChainScalers][kScSpan + kScSpan / 32 + 1];
#define SCI(e) ((e) + ((e) >> 5))
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) {
        ctl.in_ready = 0;
        ctl.raw_done = 0;
        ctl.abort = 0;
        ctl.pub = 0;
    }
    __syncthreads();
    asm volatile("s_dcache_inv" ::: "memory");
    // LDS control words: workgroup-scope relaxed atomics lower to plain ds_ ops
#define CTL_LD(f) __hip_atomic_load(&ctl.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define CTL_ST(f, v) __hip_atomic_store(&ctl.f, (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)

    if (threadIdx.x < 64) {
        // ---------------------------- chain wave ----------------------------
        // top priority: the feeder and scaler share the CU's issue paths with it
        // (chain_diag: 13.0 -> 12.8 / 14.2 -> 13.6 cycles per tick, passes 1 / 3)
        __builtin_amdgcn_s_setprio(3);
        double sum = 0.0;  // T::zero()
        // first steady block: 1; steady blocks k need CB*(k+1) + 8 <= N (group prefetch);
        // the steady loop runs MDG_CHAIN_BPT blocks per trip, the rest go generic
        const int kA = 1;
        const int kB = kA + max(0, (N - 8) / CB - kA) / MDG_CHAIN_BPT * MDG_CHAIN_BPT;
        int avail = 0;
        auto wait_in = [&](int need) -> bool {
            unsigned spins = 0;
            while (avail < need) {
                avail = CTL_LD(in_ready);
                if (avail >= need) break;
                if (CTL_LD(abort)) return false;
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kChainSpins) return false;
            }
            return true;
        };
        // generic block (first and last blocks): the ticks as DPP row-broadcast fmacs
        // (fold8_ticks), operands zero-padded: the running sum starts at +0.0 and can
        // never become -0.0 (x + y is -0 only for -0 + -0, x - y only for -0 - +0),
        // so adding or subtracting +0.0 is exactly the reference's skipped term.
        // Checkpoints every 8 ticks are stored (a superset of the steady loop's).
        const double one = 1.0;
        auto generic = [&](int k) -> bool {
            if (!wait_in(min(k + 2, nIB))) return false;
            const int j0 = k * CB;
#pragma unroll 1
            for (int g16 = 0; g16 < CB / 16; ++g16) {
                const int j = j0 + 16 * g16 + (lane & 15);
                const double av = ld_sc1(in + min(j, N - 1));
                const double pv = ld_sc1(in + max(min(j - WS, N - 1), 0));
                const double A = j < N ? av : 0.0;
                const double Pm = j >= WS ? pv : 0.0;
                fold8_ticks<0>(sum, A, Pm, one);
                raw[j0 + 16 * g16 + 7] = sum;
                fold8_ticks<8>(sum, A, Pm, one);
                raw[j0 + 16 * g16 + 15] = sum;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            CTL_ST(raw_done, k + 1);
            return true;
        };
        bool ok = true;
        DIAGC(0, __builtin_amdgcn_s_memtime());
        DIAGC(5, __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11)));  // HW_ID: wave / SIMD / CU / SE
        for (int k = 0; ok && k < kA; ++k) ok = generic(k);
        DIAGC(1, __builtin_amdgcn_s_memtime());
        if (ok && kB > kA) {
            int stat = 0;
            const int done = chain_steady<WS>(in + (size_t)kA * CB - 8, raw + (size_t)kA * CB, kA,
                                              (kB - kA) / MDG_CHAIN_BPT, nIB,
                                              lds_offset(&ctl), sum, stat);
            ok = (stat & 1) == 0 && done == kB;  // stat >> 1: in_ready waits (diagnostic)
            DIAGC(6, stat >> 1);
            if (ok) CTL_ST(raw_done, kB);
        }
        DIAGC(2, __builtin_amdgcn_s_memtime());
        DIAGC(4, kB - kA);
        for (int k = kB; ok && k < nJB; ++k) ok = generic(k);
        DIAGC(3, __builtin_amdgcn_s_memtime());
        if (!ok) CTL_ST(abort, 1);
    } else if (threadIdx.x < 128) {
        // ---------------------------- feeder wave ----------------------------
        // polls the upstream pass, touches newly available input blocks into the
        // scalar cache (kChainPrefetch blocks ahead of the chain) and publishes them
        int pf = 0;     // next input block to touch
        int ready = 0;  // in_ready published
        // pass 0 of rows this launch decodes: the decoded chunks (dec_flags)
        int up = p == 0 && ndec == 0 ? nIB : 0;
        int l2 = 0;  // next input block pulled into L2
        unsigned idle = 0;
        bool ok = true;
        DIAGC(8, __builtin_amdgcn_s_memtime());
        DIAGC(12, __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11)));  // HW_ID: wave / SIMD / CU / SE
#ifdef MDG_DIAG
        if (g_chain_mode == 1 || g_chain_mode == 3) {
            CTL_ST(in_ready, nIB);
            pf = nIB;
        }
#endif
#ifdef MDG_DIAG
        if (g_chain_mode == 4 && p > 0)  // upstream pass finished before this one starts
            while (__hip_atomic_load(const_cast<int32_t*>(up_flag), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) < nOB)
                __builtin_amdgcn_s_sleep(8);
#endif
        while (pf < nIB) {
            if (CTL_LD(abort)) {
                ok = false;
                break;
            }
            const int rd = CTL_LD(raw_done);
            // learn what the upstream pass has published (pass 0: everything)
            if (p > 0 && up < min(nIB, rd + l2ahead))
                up = __hip_atomic_load(const_cast<int32_t*>(up_flag), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            if (p == 0 && ndec > 0 && up < min(nIB, rd + l2ahead)) {
                // lane c reads chunk c's flag; the decoded prefix is the run of set
                // flags from chunk 0 (kDecChunks == 64: one per lane)
                static_assert(kDecChunks == 64, "one flag per feeder lane");
                const int32_t f = __hip_atomic_load(w.dec_flags + (size_t)s * kDecChunks + lane, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t nm = ~__ballot(f == a.dec_gen);
                const int chunks = nm ? __builtin_ctzll(nm) : kDecChunks;
                const int nu = min(nIB, chunks * dec_block_chunk(nIB));
                if (nu > up) {
                    // consumer side of the decoders' hand-off (MI355X_MICROARCH.md,
                    // inter-workgroup visibility: one relaxed poll, one agent-scope
                    // acquire, its wait, then the loads): this CU's L1 is invalidated
                    // before the pulls, the touches and -- through in_ready, set after
                    // the wait -- the chain's loads of the new chunks. The rows are of
                    // whole 128-byte lines per chunk (kDecRowAlign; the host checks it),
                    // so no line read here holds bytes of a chunk not yet published,
                    // and the scalar cache (invalidated at this workgroup's start) only
                    // ever receives lines of published chunks.
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    up = nu;
                }
            }
            // pull published full input blocks into L2 (16 per wait), so the
            // scalar-cache touches below hit L2 instead of HBM / the MALL
            // (every pass: without it, 11.7 / 12.3 / 12.5 cycles per tick, passes 0..2)
            const int l2lim = min(min(N / CB, up), rd + l2ahead);
            bool prog = false;
            if (l2lim - l2 >= 16 || (l2lim > l2 && (l2lim == N / CB || l2 < pf + 4))) {
                const int cnt = min(16, l2lim - l2);
                if (lane < CB / 2) chain_l2_pull(in + (size_t)l2 * CB + 2 * lane, cnt);
                l2 += cnt;
                prog = true;
            }
            // the chain may read every published block (in_ready gates correctness
            // only); the touches run kChainPrefetch blocks ahead of it, in one batch
            if (min(up, nIB) > ready) {
                ready = min(up, nIB);
                CTL_ST(in_ready, ready);
                prog = true;
            }
            const int hi = min(min(up, nIB), rd + kChainPrefetch);
            if (hi > pf) {
                const int full = min(hi, N / CB) - pf;  // whole blocks only (no read past N)
                if (full > 0) chain_touch(in + (size_t)pf * CB, full);
                pf = hi;
                prog = true;
            }
            if (prog) {
                idle = 0;
                DIAGC_ADD(10, 1);
                continue;
            }
            DIAGC_ADD(11, 1);
            __builtin_amdgcn_s_sleep(1);
            if (++idle > kChainSpins) {
                ok = false;
                break;
            }
        }
        DIAGC(9, __builtin_amdgcn_s_memtime());
        if (!ok) CTL_ST(abort, 1);
    } else {
        // ---------------------------- scaler waves ---------------------------
        // batch b = output blocks [b*MB, b*MB + MB) goes to scaler wave b % kChainScalers;
        // each scales its batch, stores it (sc1), waits vmcnt(0) and then, in batch
        // order (ctl.pub), raises the pass's block counter (atomic max, so the order
        // the counter updates land in does not matter)
        const int sw = (threadIdx.x >> 6) - 2;
        double* sc_in = sc_in_all[sw];
        double* sc_raw = sc_raw_all[sw];
        // the reference's div = 1/len (moving_average.rs:66-81), one division per len
        double inv_len[WS + 1];
#pragma unroll
        for (int k = 0; k <= WS; ++k) inv_len[k] = 1.0 / (double)(k > 0 ? k : 1);
        double one = 1.0, mone = -1.0;  // opaque: keep the replay as VOP2 fmacs
        asm volatile("" : "+v"(one), "+v"(mone));
        constexpr int MB = kChainScBatch;
        const int nBatch = (nOB + MB - 1) / MB;
        unsigned idle = 0;
        bool ok = true;
        if (sw == 0) {
            DIAGC(16, __builtin_amdgcn_s_memtime());
            DIAGC(20, __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11)));  // HW_ID
        }
        int b = sw;
#ifdef MDG_DIAG
        if (g_chain_mode == 1 || g_chain_mode == 2) b = nBatch;
#endif
        while (b < nBatch) {
            if (CTL_LD(abort)) {
                ok = false;
                break;
            }
            const int sc = b * MB, hi = min(nOB, sc + MB);
            const int rd = CTL_LD(raw_done);
            // output block m needs raw j-blocks <= m+1: finished once raw_done >= m+2
            const int ready = rd >= nJB ? nOB : min(nOB, max(0, rd - 1));
            if (ready < hi) {
                if (sw == 0) DIAGC_ADD(19, 1);
                __builtin_amdgcn_s_sleep(1);
                if (++idle > kChainSpins) {
                    ok = false;
                    break;
                }
                continue;
            }
#ifdef MDG_DIAG
            const long long tr0 = __builtin_amdgcn_s_memtime();
            long long trp = tr0;
#define DIAG_PH(k)                                            \
    if (sw == 0) {                                            \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    \
        const long long tn = __builtin_amdgcn_s_memtime();    \
        DIAGC_ADD(k, tn - trp);                               \
        trp = tn;                                             \
    }
#else
#define DIAG_PH(k)
#endif
            const int i0 = sc * CB, i1 = min(hi * CB, N);
            // raw sums j = i + R of the batch, staged in LDS: groups of G ticks in
            // steady j-blocks [kA, kB) hold only their last sum (the checkpoint), so
            // one lane per group replays it from the previous checkpoint with the
            // chain's own two operations per tick; all HBM traffic is coalesced
            constexpr int G = kChainG;
            const int g0 = (i0 + R) / G, g1 = (i1 - 1 + R) / G + 1;
            const int base = G * g0 - 8;               // LDS index = j - base
            const int span = G * (g1 - g0) + 8;
            static_assert((MB * kChainCB) / G + 1 <= 64, "one replay group per lane");
            // lane g - g0: the checkpoint its group starts from (group 0: T::zero())
            const int gl = g0 + lane;
            const bool has_g = gl < g1;
            const double ck = has_g && gl > 0 ? ld_sc1(raw + (G * gl - 1)) : 0.0;
            {
                constexpr int SLOTS = (MB * kChainCB + G + 8 + 63) / 64;
                double vin[SLOTS];
#pragma unroll
                for (int k = 0; k < SLOTS; ++k) {  // all loads in flight together
                    const int e = 64 * k + lane, j = base + e;
                    vin[k] = (e < span && j >= 0 && j < N) ? ld_sc1(in + j) : 0.0;
                }
#pragma unroll
                for (int k = 0; k < SLOTS; ++k) {
                    const int e = 64 * k + lane;
                    if (e < span) sc_in[SCI(e)] = vin[k];
                }
            }
            DIAG_PH(23);
            if (has_g) {
                // replay the group from its checkpoint with the chain's own two
                // operations per tick (fma(x, +-1, s) rounds as s +- x; VOP2 fmacs)
                const int e0 = G * gl - base;
                double sum_g = ck;
                double xin[G + 8], rv[G];
#pragma unroll
                for (int u = -8; u < G; ++u) xin[u + 8] = sc_in[SCI(e0 + u)];
#pragma unroll
                for (int u = 0; u < G; ++u) {
                    sum_g = __builtin_fma(xin[u + 8], one, sum_g);
                    sum_g = __builtin_fma(xin[u + 8 - WS], mone, sum_g);
                    rv[u] = sum_g;
                }
#pragma unroll
                for (int u = 0; u < G; ++u) sc_raw[SCI(e0 + u)] = rv[u];
            }
            DIAG_PH(24);
            {
                constexpr int OSL = MB * kChainCB / 64;
                double ov[OSL];
#pragma unroll
                for (int k = 0; k < OSL; ++k) {  // LDS reads in flight together
                    const int i = i0 + 64 * k + lane;
                    ov[k] = i < i1 ? sc_raw[SCI(i + R - base)] : 0.0;
                }
#pragma unroll
                for (int k = 0; k < OSL; ++k) {
                    const int i = i0 + 64 * k + lane;
                    // len of the circular buffer after tick i (moving_average.rs:66-81)
                    const int len = i < N - R ? min(i + R + 1, WS) : WS - 1 - (i - (N - R));
                    if (i < i1)
                        __hip_atomic_store(out + i, ov[k] * inv_len[len], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            DIAG_PH(25);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            DIAG_PH(26);
            // publish in batch order: the batches before b are stored and counted
            unsigned spins = 0;
            while (CTL_LD(pub) != b) {
                if (CTL_LD(abort) || ++spins > kChainSpins) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) break;
            // the publication is issued by the whole wave with a wave-uniform value (no
            // lane-guarded branch around it; the compiler's atomic optimizer sends one
            // atomic): the round-3 lost-counter bug was a lane-guarded store in a
            // region with spilled SGPRs (publication audit)
            __hip_atomic_fetch_max(my_flag, __builtin_amdgcn_readfirstlane(hi), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            CTL_ST(pub, b + 1);
            if (sw == 0) {
                DIAGC_ADD(18, 1);
                DIAGC_ADD(21, __builtin_amdgcn_s_memtime() - tr0);
                DIAGC_ADD(22, hi - sc);
            }
            b += kChainScalers;
            idle = 0;
        }
        if (sw == 0) DIAGC(17, __builtin_amdgcn_s_memtime());
        if (!ok) {
            CTL_ST(abort, 1);
            w.status[s] = MDG_ERR_HIP;  // every lane, the same value
            // release every downstream pass so all waves drain (whole wave, as above)
            __hip_atomic_fetch_max(my_flag, 1 << 30, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
#undef CTL_LD
#undef CTL_ST
#undef SCI
#undef DIAG_PH
}

__global__ void k_smooth(BatchArgs a, Workspace w, int iters, int ws) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.B) return;
    if (w.status[s]) return;
    const int N = a.N;
    const double* src = y_row(a, s);
    double* out = w.smooth + (size_t)s * N;
    double* tmp0 = w.tmp0 + (size_t)s * N;
    double* tmp1 = w.tmp1 + (size_t)s * N;
    for (int it = 0; it < iters; ++it) {
        double* dst = (it == iters - 1) ? out : ((it & 1) ? tmp1 : tmp0);
        ma_pass(src, dst, N, ws);
        src = dst;
    }
}

// ----------------------------------------------------------------------------------
// K2  curvature flags: center / right-border / left-border predicates as bitmasks
// peak_selection/detector.rs:189-233 restated on intensity-aligned D[k]=sd[k-1]:
//   center c : D[c]<0 && D[c]<D[c-1] && D[c]<D[c+1]                    c in [2,N-3]
//   right  r : D[r]>D[r-1] && (D[r]>=D[r+1] || (D[r]<0 && D[r+1]>=0))
//   left   l : D[l]>D[l+1] && (D[l]>=D[l-1] || (D[l]<0 && D[l-1]>=0))
// The per-center border scans of the reference become next/previous-set-bit
// searches on these masks (K3): the predicates do not depend on the center.
// ----------------------------------------------------------------------------------
// ----------------------------------------------------------------------------------
// K1s  the moving average of a SMALL spectrum (N <= kSmallN, round 6) in ONE workgroup:
// one wave per pass, the passes pipelined through LDS (pass 0 reads the row staged in
// LDS, pass p > 0 a ring of pass p - 1's outputs, the last pass writes the smoothed
// row). moving_average.rs:53-83's recurrence exactly as k_smooth_chain runs it (sum +=
// in[i + R]; sum -= in[i + R - WS] once the FIFO is full; div = 1/len; out = sum *
// div): the scalar ticks (prefill, the FIFO filling, leftovers, the tail) in plain
// code, the steady ticks sixteen at a time as DPP row_newbcast fmacs on row-replicated
// operands (fma(+-t, 1, acc) rounds as the add / sub), tick k's sum captured into the
// lanes k, k + 16, ... of the block's output by a masked select. A 2048-point
// spectrum spent 46 us in k_smooth_chain, most of it filling and draining the
// three-CU pipeline (8-block scaler batches through L2); here
// the hand-off is a 16-tick block through LDS.
// MEASURED SLOWER, so not the default (MDG_SMOOTH=small selects it; bit-exact, tested):
// sim_01 (2048 points, three passes of width 3) 58-63 us against k_smooth_chain's 46-47.
// The steady loop runs ~32 cycles a tick in the DPP blocks and ~42 with the hand-offs
// (phase stamps, profiles/r06_smooth_small_stamps.txt) where the chain's folder runs
// ~10 with scalar operands: the two DPP adds alone issue at 7.75 cycles each, and a
// single workgroup cannot hide the per-pass lag of two superblocks.
constexpr int kSmallN = 4096;  // "small" spectra: k_smooth_small, k_fit_small
constexpr int kSmRing = 512;   // doubles per intermediate pass ring (a power of two)
constexpr int kSmMaxP = 15;    // passes = waves (+ one wave for the spectrum's prep)
constexpr int kSmMaxWS = 32;
constexpr int kSmSpins = 1 << 22;
constexpr int kSmStage = 16;  // row values per thread per staging round

__device__ __forceinline__ int lds_ld(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// 16 steady ticks: acc += A[k]; acc -= S[k] for k = 0..15 (lane k of each 16-lane row),
// hist lane (l & 15) += the sum after tick k times mk[k] (1.0 in lanes k, k + 16, ...,
// 0.0 elsewhere): with finite sums every other product is a zero and hist lane (l & 15)
// ends as that tick's sum exactly (the caller redoes a block whose sum went non-finite).
// The capture is an f64 fmac, not a select: a 32-bit select of the DPP fmac's result
// waited on it ~20 cycles a tick (46 cycles/tick measured, 15.5 for the two fmacs).
__device__ __forceinline__ void sm_block16(double& acc, double& hist, double A, double S, double one,
                                           const double (&mk)[16]) {
#define MDG_SMTICK(k)                                                                          \
    "v_fmac_f64_dpp %[acc], %[A], %[one] row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n"     \
    "v_fmac_f64_dpp %[acc], -%[S], %[one] row_newbcast:" #k " row_mask:0xf bank_mask:0xf\n"    \
    "v_fmac_f64 %[hist], %[acc], %[m" #k "]\n"
    hist = 0.0;
    asm volatile(
        "s_nop 4\n"
        MDG_SMTICK(0) MDG_SMTICK(1) MDG_SMTICK(2) MDG_SMTICK(3) MDG_SMTICK(4) MDG_SMTICK(5)
        MDG_SMTICK(6) MDG_SMTICK(7) MDG_SMTICK(8) MDG_SMTICK(9) MDG_SMTICK(10) MDG_SMTICK(11)
        MDG_SMTICK(12) MDG_SMTICK(13) MDG_SMTICK(14) MDG_SMTICK(15)
        : [acc] "+v"(acc), [hist] "+v"(hist)
        : [A] "v"(A), [S] "v"(S), [one] "v"(one), [m0] "v"(mk[0]), [m1] "v"(mk[1]), [m2] "v"(mk[2]),
          [m3] "v"(mk[3]), [m4] "v"(mk[4]), [m5] "v"(mk[5]), [m6] "v"(mk[6]), [m7] "v"(mk[7]),
          [m8] "v"(mk[8]), [m9] "v"(mk[9]), [m10] "v"(mk[10]), [m11] "v"(mk[11]), [m12] "v"(mk[12]),
          [m13] "v"(mk[13]), [m14] "v"(mk[14]), [m15] "v"(mk[15]));
#undef MDG_SMTICK
}

bool smooth_small_ok(int N, int iters, int ws) {
    return N <= kSmallN && N >= 4 * kSmMaxWS + 64 && iters >= 1 && iters <= kSmMaxP && ws >= 1 &&
           ws <= kSmMaxWS;
}

__global__ __launch_bounds__(64 * (kSmMaxP + 1)) void k_smooth_small(BatchArgs a, Workspace w, int P, int WS,
                                                             int fused_prep) {
    __shared__ double yl[kSmallN];
    __shared__ double ring[kSmMaxP - 1][kSmRing];
    __shared__ int prog[kSmMaxP];  // ticks (outputs) pass p has published
    __shared__ int fail;
    constexpr int RM = kSmRing - 1;
    const int s = blockIdx.x, N = a.N, tid = threadIdx.x, lane = tid & 63, p = tid >> 6;
    KSTAMP(88);
    // the row (decoded here from page-locked int32 rows for mdg_deconvolute_rows_i32:
    // y = raw * scale, the reader's operation; the x and y rows the later launches
    // read are written back)
    double* yg = const_cast<double*>(y_row(a, s));
    if (a.dec_rows) {
        const int32_t* __restrict__ r = a.dec_rows[s];
        const double sc = a.dec_desc[4 * s + 3];
        for (int b0 = 0; b0 < N; b0 += kSmStage * (int)blockDim.x) {
            double v[kSmStage];  // every load issued before the first store
#pragma unroll
            for (int j = 0; j < kSmStage; ++j) {
                const int i = b0 + j * blockDim.x + tid;
                v[j] = i < N ? (double)r[i] * sc : 0.0;
            }
#pragma unroll
            for (int j = 0; j < kSmStage; ++j) {
                const int i = b0 + j * blockDim.x + tid;
                if (i < N) {
                    yl[i] = v[j];
                    yg[i] = v[j];
                }
            }
        }
        if (a.x_stride || s == 0) {
            const double* xd = a.dec_desc + 4 * s;
            double* xr = const_cast<double*>(a.x) + (size_t)s * a.x_stride;
            for (int i = tid; i < N; i += blockDim.x) xr[i] = dec_x(xd, i);
        }
    } else {
        for (int b0 = 0; b0 < N; b0 += kSmStage * (int)blockDim.x) {
            double v[kSmStage];
#pragma unroll
            for (int j = 0; j < kSmStage; ++j) {
                const int i = b0 + j * blockDim.x + tid;
                v[j] = i < N ? yg[i] : 0.0;
            }
#pragma unroll
            for (int j = 0; j < kSmStage; ++j) {
                const int i = b0 + j * blockDim.x + tid;
                if (i < N) yl[i] = v[j];
            }
        }
    }
    if (tid < kSmMaxP) prog[tid] = 0;
    if (tid == 0) fail = 0;
    __syncthreads();
#ifdef MDG_DIAG
    // HW_ID of each wave (SIMD in bits 5:4): stage_diag.py prints slots 150 + wave
    if (lane == 0 && blockIdx.x == 0 && g_diag && p < 16)
        g_diag[kDiagStampBase + 150 + p] = 1 + (long long)(unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
#endif
    if (p >= P) {  // the extra wave: the spectrum's prep, off the passes' critical path
        if (lane == 0 && fused_prep) prep_spectrum(a, w, s);
        return;
    }
#ifdef MDG_DIAG
    // per-pass stamps (tools/stage_diag.py --sim): slots 90 + 4p + {0 start, 1 steady, 2 tail, 3 end}
#define SM_STAMP(k)                                                                           \
    if (lane == 0 && blockIdx.x == 0 && g_diag && p < 8)                                      \
    g_diag[kDiagStampBase + 90 + 4 * p + (k)] = (long long)__builtin_amdgcn_s_memtime()
#else
#define SM_STAMP(k)
#endif
    SM_STAMP(0);
    const int R = WS / 2;
    const double* in = p == 0 ? yl : ring[p - 1];
    const int im = p == 0 ? 0x7fffffff : RM;  // index mask of the input
    double* outr = p < P - 1 ? ring[p] : nullptr;
    double* outg = w.smooth + (size_t)s * N;
    int spins = 0;
    // wait until the input holds indices < need, and (a ring output) until the next
    // pass no longer needs the slots of indices < upto - kSmRing
    auto wait_for = [&](int need, int upto) {
        if (p > 0) {
            while (lds_ld(&prog[p - 1]) < need) {
                if (++spins > kSmSpins || lds_ld(&fail)) {
                    if (lane == 0) fail = 1;
                    return false;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (outr) {
            while (lds_ld(&prog[p + 1]) < upto - kSmRing + WS + 1) {
                if (++spins > kSmSpins || lds_ld(&fail)) {
                    if (lane == 0) fail = 1;
                    return false;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        return true;
    };
    // (a wave's LDS requests are served in order, so a reader that sees the count it
    // stores after the outputs also sees the outputs)
    auto publish = [&](int n) {
        if (lane == 0) __hip_atomic_store(&prog[p], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    auto emit = [&](int i, double v) {  // one output (scalar ticks)
        if (lane == 0) {
            if (outr) outr[i & RM] = v;
            else outg[i] = v;
        }
        publish(i + 1);
    };
    bool ok = true;
    double sum = 0.0, div = 1.0;
    int len = 0;
    // prefill: the first R values pushed (moving_average.rs:60-65)
    ok = wait_for(R, 0);
    for (int k = 0; ok && k < R; ++k) {
        sum += in[k & im];
        ++len;
    }
    const int nm = N - R;  // main ticks
    int i = 0;
    // the FIFO filling: no pop, div = 1/len
    for (; ok && i < nm && len < WS; ++i) {
        if (!(ok = wait_for(i + R + 1, i + 1))) break;
        sum += in[(i + R) & im];
        ++len;
        div = 1.0 / (double)len;
        emit(i, sum * div);
    }
    // steady: sixteen ticks per DPP block, kSmSuper blocks per wait and publication
    // (their operands loaded together: one round of LDS latency per 64 ticks)
    const double one = 1.0;
    const int l = lane & 15;
    double mk[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) mk[k] = l == k ? 1.0 : 0.0;
    // one 16-tick block from index b; a block whose sum went non-finite (the capture
    // multiplies every tick's sum by 0.0 or 1.0) is redone tick by tick
    auto block = [&](int b, double A, double S) {
        const double s0 = sum;
        double hist;
        sm_block16(sum, hist, A, S, one, mk);
        if (!__builtin_isfinite(sum)) {
            sum = s0;
            hist = 0.0;
            for (int k = 0; k < 16; ++k) {
                sum += in[(b + R + k) & im];
                sum -= in[(b + R - WS + k) & im];
                if (l == k) hist = sum;
            }
        }
        return hist;
    };
    SM_STAMP(1);
    constexpr int kSmSuper = 4;
#ifdef MDG_DIAG
    // one superblock of pass 0 (the eighth) split: slots 160 wait, 161 waited, 162 loaded, 163 blocks, 164 published
    int sbk = 0;
#define SB_STAMP(k)                                                                           \
    if (lane == 0 && blockIdx.x == 0 && g_diag && p == 0 && sbk == 8)                          \
    g_diag[kDiagStampBase + 160 + (k)] = (long long)__builtin_amdgcn_s_memtime()
#else
#define SB_STAMP(k)
#endif
    // the next superblock's operands are loaded before this one's blocks run when the
    // previous pass has already published them (no wait: a pass never blocks on its
    // input while holding outputs back)
    double A[kSmSuper], S[kSmSuper];
    bool have = false;
    auto load_super = [&](int b) {
#pragma unroll
        for (int u = 0; u < kSmSuper; ++u) {
            A[u] = in[(b + 16 * u + R + l) & im];
            S[u] = in[(b + 16 * u + R - WS + l) & im];
        }
    };
    for (; ok && i + 16 * kSmSuper <= nm; i += 16 * kSmSuper) {
        SB_STAMP(0);
        if (!(ok = wait_for(have ? 0 : i + 16 * kSmSuper + R, i + 16 * kSmSuper))) break;
        SB_STAMP(1);
        if (!have) load_super(i);
        double cA[kSmSuper], cS[kSmSuper];
#pragma unroll
        for (int u = 0; u < kSmSuper; ++u) {
            cA[u] = A[u];
            cS[u] = S[u];
        }
        const int nx = i + 32 * kSmSuper + R;
        have = i + 32 * kSmSuper <= nm && (p == 0 || lds_ld(&prog[p - 1]) >= nx);
        if (have) load_super(i + 16 * kSmSuper);
#pragma unroll
        for (int u = 0; u < kSmSuper; ++u) {
            if (u == 0) SB_STAMP(2);
            const double v = block(i + 16 * u, cA[u], cS[u]) * div;
            if (lane < 16) {
                if (outr) outr[(i + 16 * u + lane) & RM] = v;
                else outg[i + 16 * u + lane] = v;
            }
        }
        SB_STAMP(3);
        publish(i + 16 * kSmSuper);
        SB_STAMP(4);
#ifdef MDG_DIAG
        ++sbk;
#endif
    }
#undef SB_STAMP
    for (; ok && i + 16 <= nm; i += 16) {
        if (!(ok = wait_for(i + 16 + R, i + 16))) break;
        const double v = block(i, in[(i + R + l) & im], in[(i + R - WS + l) & im]) * div;
        if (lane < 16) {
            if (outr) outr[(i + lane) & RM] = v;
            else outg[i + lane] = v;
        }
        publish(i + 16);
    }
    for (; ok && i < nm; ++i) {  // leftover steady ticks
        if (!(ok = wait_for(i + R + 1, i + 1))) break;
        sum += in[(i + R) & im];
        sum -= in[(i + R - WS) & im];
        emit(i, sum * div);
    }
    SM_STAMP(2);
    // tail: pops only (moving_average.rs:76-81)
    for (; ok && i < N; ++i) {
        if (!(ok = wait_for(N, i + 1))) break;
        if (len > 0) {
            sum -= in[(i + R - WS) & im];
            --len;
            div = 1.0 / (double)len;
            emit(i, sum * div);
        }
    }
    if (!ok && lane == 0) w.status[s] = MDG_ERR_HIP;
    SM_STAMP(3);
#undef SM_STAMP
}

const char* launch_smooth_small(const BatchArgs& a, const Workspace& w, int iters, int ws, hipStream_t st,
                                int fused_prep) {
    launch_k(k_smooth_small, dim3(a.B), dim3(64 * (iters + 1)), 0, st, a, w, iters, ws, fused_prep);
    return "k_smooth_small";
}

// look-back slots of k_peaks per spectrum (one per kPkSlotWords mask words)
__device__ __forceinline__ int peak_slots(int W) { return (W + kPkSlotWords - 1) / kPkSlotWords; }
__global__ void k_flags(BatchArgs a, Workspace w) {
    const int s = blockIdx.y;
    // the smoother has finished: its progress counters go back to zero for the
    // next run (whatever this spectrum's status)
    if (blockIdx.x == 0 && (int)threadIdx.x < w.chain_P)
        w.chain_flags[((size_t)s * w.chain_P + threadIdx.x) * 32] = 0;
    // the status is loaded with the row (one memory round trip, not two); the row
    // of a failed spectrum is read and ignored
    const int st = w.status[s];
    const int N = a.N;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const double* sm = w.smooth_ptr + (size_t)s * w.smooth_stride;
    bool fc = false, fr = false, fl = false;
    if (k >= 2 && k <= N - 3) {
        const double dm = dsd(sm, k - 1), d0 = dsd(sm, k), dp = dsd(sm, k + 1);
        fc = d0 < 0. && d0 < dm && d0 < dp;
        fr = d0 > dm && (d0 >= dp || (d0 < 0. && dp >= 0.));
        fl = d0 > dp && (d0 >= dm || (d0 < 0. && dm >= 0.));
    }
    if (st) return;
    // k_peaks' per-chunk slots start empty
    if (k < peak_slots(w.W)) ((unsigned long long*)w.peak_cnt)[(size_t)s * peak_slots(w.W) + k] = 0;
    const uint64_t bc = __ballot(fc), br = __ballot(fr), bl = __ballot(fl);
    if ((threadIdx.x & 63) == 0 && k < N) {
        const int word = k >> 6;
        uint64_t* m = w.masks + (size_t)s * 3 * w.W;
        m[word] = bc;
        m[w.W + word] = br;
        m[2 * w.W + word] = bl;
    }
}

// ----------------------------------------------------------------------------------
// K3  peak list: borders, detector filter, ignore filter, ordered compaction
// detector.rs:168-212, noise_score_filter.rs:41-48, detector_only.rs:305-315
// One 1024-thread workgroup per spectrum; thread t owns a contiguous word range so
// the block scan preserves center order.
// ----------------------------------------------------------------------------------
__device__ __forceinline__ bool in_ignore(int v, const int64_t* pairs, int n) {
    if (n <= 8) {
        for (int k = 0; k < n; ++k)
            if (v >= pairs[2 * k] && v < pairs[2 * k + 1]) return true;
        return false;
    }
    // Many regions: the merged regions are sorted and disjoint in ppm, so both ends
    // of their index pairs are monotone in the same direction (ascending, or
    // descending for a descending axis; floor/ceil, the clamps and the filter keep
    // that). In ascending order the last pair starting at or before v has the
    // largest end of all such pairs, so v is ignored iff it lies before that end.
    const bool desc = pairs[0] > pairs[2 * (n - 1)] ||
                      (pairs[0] == pairs[2 * (n - 1)] && pairs[1] > pairs[2 * (n - 1) + 1]);
    int lo = 0, hi = n - 1, k = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const int q = desc ? n - 1 - mid : mid;
        if (pairs[2 * q] <= v) {
            k = q;
            lo = mid + 1;
        } else {
            hi = mid - 1;
        }
    }
    return k >= 0 && v < pairs[2 * k + 1];
}

// The peaks of one mask word (64 points) whose centre bits are in sel, in centre
// order: borders by bit scans, the detector-only and ignore-region filters. Counts
// the bordered peaks; returns the kept ones, writing them at out.. when WRITE.
// (LDSM: the masks are the caller's window of mask words [wlo, wlo + nw) in LDS, mlds:
// the centre words, then the right-border words, then the left-border ones; a border
// beyond the window is searched on the smoothed row smr itself. GOUT = false: WRITE
// fills only the pk copy, not the global peak rows)
template <bool WRITE, bool LDSM = false, bool GOUT = true>
__device__ __forceinline__ int word_peaks(const BatchArgs& a, const Workspace& w, int s, int wd, uint64_t sel,
                                          int detector_only, int* bordered, size_t out,
                                          int* pk = nullptr, int pcap = 0, int po = 0,
                                          const uint64_t* mlds = nullptr, int wlo = 0, int nw = 0,
                                          const double* smr = nullptr, int nig_in = -1) {
    const int N = a.N, W = w.W;
    const int mst = LDSM ? nw : W, off = LDSM ? wlo : 0;  // kind stride, first word held
    const uint64_t* mc = LDSM ? mlds : w.masks + (size_t)s * 3 * W;
    const uint64_t* mr = mc + mst;
    const uint64_t* ml = mc + 2 * mst;
    const int64_t* pairs = w.ig + (size_t)s * 2 * w.ig_cap;
    // (nig_in: the caller loaded the region count ahead, with its other head loads)
    const int nig = nig_in >= 0 ? nig_in : (a.n_ignore > 0 ? w.n_ig[s] : 0);
    const int64_t sbi0 = detector_only ? w.sbi[2 * s] : 0, sbi1 = detector_only ? w.sbi[2 * s + 1] : 0;
    // the word and its neighbours' border masks in one round trip; a border farther
    // than the neighbouring word falls back to the scans over memory
    uint64_t bits = mc[wd - off] & sel;
    const uint64_t r0 = mr[wd - off], r1 = wd + 1 < W ? mr[wd + 1 - off] : 0;
    const uint64_t l0 = ml[wd - off], l1 = wd > 0 ? ml[wd - 1 - off] : 0;
    const int lim_r = N - 3, lim_l = 2;
    int kept = 0;
    while (bits) {
        const int b = __ffsll((unsigned long long)bits) - 1;
        bits &= bits - 1;
        const int c = (wd << 6) + b;
        // first right-border bit > c (<= N-3): this word above b, then the next word
        int r;
        const uint64_t ra = b == 63 ? 0 : (r0 & (~0ull << (b + 1)));
        if (ra) r = (wd << 6) + __ffsll((unsigned long long)ra) - 1;
        else if (r1) r = ((wd + 1) << 6) + __ffsll((unsigned long long)r1) - 1;
        else r = LDSM ? next_bit_win(mr, wlo, nw, (wd + 2) << 6, lim_r, smr, N)
                      : find_next_bit(mr, (wd + 2) << 6, lim_r);
        if (r > lim_r) r = -1;
        // last left-border bit < c (>= 2): this word below b, then the previous word
        int l;
        const uint64_t la = b == 0 ? 0 : (l0 & ((1ull << b) - 1ull));
        if (la) l = (wd << 6) + 63 - __clzll((long long)la);
        else if (l1) l = ((wd - 1) << 6) + 63 - __clzll((long long)l1);
        else l = LDSM ? prev_bit_win(ml, wlo, nw, ((wd - 1) << 6) - 1, lim_l, smr, N)
                      : find_prev_bit(ml, ((wd - 1) << 6) - 1, lim_l);
        if (l < lim_l) l = -1;
        if (r < 0 || l < 0) continue;  // right == N-1 or left == 0: dropped
        ++*bordered;
        bool keep = true;
        if (detector_only) keep = (int64_t)l >= sbi0 && (int64_t)r <= sbi1;
        if (keep && a.n_ignore > 0) keep = !(in_ignore(l, pairs, nig) || in_ignore(r, pairs, nig));
        if (!keep) continue;
        if constexpr (WRITE) {
            if constexpr (GOUT) {
                w.det_l[out + kept] = l;
                w.det_c[out + kept] = c;
                w.det_r[out + kept] = r;
            }
            if (pk && po + kept < pcap) {  // the chunk's copy for its scoring (LDS)
                pk[po + kept] = l;
                pk[pcap + po + kept] = c;
                pk[2 * pcap + po + kept] = r;
            }
        }
        ++kept;
    }
    return kept;
}

// ScorerMinimumSum::score_peak (scorer.rs:65-75): min(sum |D[l..=c]|, sum
// |D[c..=r]|) with D[k] = (y[k-1] - 2 y[k]) + y[k+1] of the smoothed row, both
// sums left folds in k order. The values of a chunk of 16 ticks are loaded
// together (clamped addresses): one memory latency per 16 ticks, not per tick
// (p99 of a blood spectrum's peak widths is 12 ticks, its widest 63).
__device__ __forceinline__ double score_peak(const double* __restrict__ sm, int N, int l, int c, int r) {
    constexpr int CH = 16;
    double left = -0.0, right = -0.0;
    for (int k0 = l; k0 <= r; k0 += CH) {
        double y[CH + 2];  // y[k0-1 .. k0+CH]
#pragma unroll
        for (int u = 0; u < CH + 2; ++u) y[u] = sm[min(max(k0 - 1 + u, 0), N - 1)];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int k = k0 + u;
            if (k <= r) {
                const double d = fabs((y[u] - 2.0 * y[u + 1]) + y[u + 2]);
                if (k <= c) left += d;
                if (k >= c) right += d;
            }
        }
    }
    return fmin(left, right);
}

// score_peak over a staged copy of the row: ys[i] = sm[i + lo], l - 1 .. r + 1 inside
// it; the same operations in the same order
__device__ __forceinline__ double score_peak_lds(const double* ys, int lo, int l, int c, int r) {
    double left = -0.0, right = -0.0;
    double ym = ys[l - 1 - lo], y0 = ys[l - lo];
    for (int k = l; k <= r; ++k) {
        const double yp = ys[k + 1 - lo];
        const double d = fabs((ym - 2.0 * y0) + yp);
        if (k <= c) left += d;
        if (k >= c) right += d;
        ym = y0;
        y0 = yp;
    }
    return fmin(left, right);
}

// K3 per chunk of WORDS mask words (many workgroups per spectrum: a
// single-workgroup version took 46-53 us at N = 131072). Large batches take chunks
// of 256 words on 1024 threads; small ones chunks of 64 words on 256 threads, four
// times the workgroups per spectrum (a B = 1 launch is otherwise 8 workgroups on 8
// CUs, each scoring ~2000 peaks). The slots are laid out for the finer chunking
// (kPkSlotWords, mdg_common.hpp) whichever is launched.
// K3 in one pass (decoupled look-back): every chunk counts its peaks, publishes
// {bordered, kept} in its slot of w.peak_cnt (cleared by k_flags), then reads the
// slots of all chunks of its spectrum -- they publish before they wait, so one
// round of flag latency -- and compacts its peaks after the kept peaks of the
// chunks before it. Replaces k_peaks_count + k_peaks_write (one launch and one
// word scan fewer).
constexpr unsigned long long kPkValid = 1ull << 62;
// BS = 4 WORDS threads per chunk: four per mask word; all of them score the chunk's
// peaks afterwards
// FUSE (round 6): k_flags' predicates computed here, for the chunk's words and one word
// either side, into LDS (the row is read once, here, instead of by k_flags and again
// for the scores: one launch and ~0.74 MB per 128k-point spectrum fewer); a border
// beyond that window is found on the row itself (next_fr_row / prev_fl_row). k_flags'
// other duties move too: the chain's progress counters are reset here, the look-back
// slots are cleared by prep_spectrum.
template <int WORDS, int BS, bool FUSE = false>
__global__ __launch_bounds__(BS) void k_peaks(BatchArgs a, Workspace w, int detector_only, int score) {
    static_assert(WORDS % kPkSlotWords == 0 && BS == 4 * WORDS, "chunk shape");
    const int s = blockIdx.y, chunk = blockIdx.x;
    if (FUSE && chunk == 0 && (int)threadIdx.x < w.chain_P)  // (whatever the status, as k_flags)
        w.chain_flags[((size_t)s * w.chain_P + threadIdx.x) * 32] = 0;
    __shared__ int lds_i[BS / 64 + 1];
    __shared__ long long lds_l[BS / 64 + 1];
    // fine chunks (small batches, latency-bound) stage their stretch of the smoothed
    // row, MARG ticks either side, and their peaks in LDS for the scoring: its loads
    // then overlap the word pass instead of following the peak writes (round 4:
    // 12k of a B = 1 launch's 36k cycles were the scoring's two memory round trips)
    constexpr bool STAGE = WORDS == 64;
    // (FUSE: the predicates of the words either side of the chunk read 66 ticks beyond it)
    constexpr int SPAN = WORDS * 64, MARG = FUSE ? 128 : 64, SN = STAGE ? SPAN + 2 * MARG : 1;
    constexpr int PCAP = STAGE ? SPAN / 2 : 1;  // centres are strict minima: <= SPAN / 2
    constexpr int PER = STAGE ? (SN + BS - 1) / BS : 1;
    __shared__ double ys[SN];
    __shared__ int pk[3 * PCAP];
    const int st = w.status[s];  // (checked after the row's loads are issued)
    KSTAMP(0);
    const double* __restrict__ sm = w.smooth_ptr + (size_t)s * w.smooth_stride;
    const int lo = chunk * SPAN - MARG;
    double stv[PER];
    if constexpr (STAGE) {
#pragma unroll
        for (int u = 0; u < PER; ++u) stv[u] = sm[min(max(lo + u * BS + (int)threadIdx.x, 0), a.N - 1)];
    }
    if (st) return;  // uniform per spectrum: no chunk waits for a returned one
    constexpr int NWM = FUSE ? WORDS + 2 : 1;
    __shared__ uint64_t mw[3 * NWM];
    const int wlo = chunk * WORDS - 1;
    if constexpr (FUSE) {
        const int lane = threadIdx.x & 63, N = a.N, W = w.W;
        if constexpr (STAGE) {  // the staged row first: the predicates read it in LDS
#pragma unroll
            for (int u = 0; u < PER; ++u)
                if (u * BS + (int)threadIdx.x < SN) ys[u * BS + threadIdx.x] = stv[u];
            __syncthreads();
        }
        KSTAMP(5);
        // one word per wave and round, UW rounds' loads in flight together (a round
        // trip per word and wave otherwise: LDS for the staged fine chunks, memory for
        // the coarse ones)
        constexpr int NWV = BS / 64, UW = 4;
        for (int q0 = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6); q0 < NWM; q0 += UW * NWV) {
            double v[UW][5];
            bool val[UW];
#pragma unroll
            for (int u = 0; u < UW; ++u) {
                const int q = q0 + u * NWV, k = 64 * (wlo + q) + lane;
                val[u] = q < NWM && wlo + q >= 0 && wlo + q < W && k >= 2 && k <= N - 3;
                // unconditional loads (no exec-masked branch per value): the staged
                // window holds every index of the halo words; memory reads are clamped
#pragma unroll
                for (int d = 0; d < 5; ++d)
                    v[u][d] = STAGE ? ys[min(max(k - 2 + d - lo, 0), SN - 1)] : sm[min(max(k - 2 + d, 0), N - 1)];
            }
#pragma unroll
            for (int u = 0; u < UW; ++u) {
                const int q = q0 + u * NWV;
                if (q >= NWM) break;  // (wave-uniform)
                // dsd(., k - 1), dsd(., k), dsd(., k + 1): the same operations as k_flags
                const double dm = v[u][0] - 2.0 * v[u][1] + v[u][2];
                const double d0 = v[u][1] - 2.0 * v[u][2] + v[u][3];
                const double dp = v[u][2] - 2.0 * v[u][3] + v[u][4];
                const bool fc = val[u] && d0 < 0. && d0 < dm && d0 < dp;
                const bool fr = val[u] && d0 > dm && (d0 >= dp || (d0 < 0. && dp >= 0.));
                const bool fl = val[u] && d0 > dp && (d0 >= dm || (d0 < 0. && dm >= 0.));
                const uint64_t bc = __ballot(fc), br = __ballot(fr), bl = __ballot(fl);
                if (lane == 0) {
                    mw[q] = bc;
                    mw[NWM + q] = br;
                    mw[2 * NWM + q] = bl;
                }
            }
        }
        KSTAMP(6);
        __syncthreads();
    }
    const int nch = (w.W + WORDS - 1) / WORDS;
    unsigned long long* slot = (unsigned long long*)w.peak_cnt + (size_t)s * peak_slots(w.W);
    // four threads per mask word, each the peaks centred in 16 of its bits: thread
    // order is centre order, and the serial per-peak work a thread does is a
    // quarter of a word's (round 4: one thread per word, 4.5 us of a B = 1 launch)
    const int wd = chunk * WORDS + (threadIdx.x >> 2);
    const uint64_t sel = 0xffffull << (16 * (threadIdx.x & 3));
    int bordered = 0, kept = 0;
    if (wd < w.W)
        kept = word_peaks<false, FUSE>(a, w, s, wd, sel, detector_only, &bordered, 0, nullptr, 0, 0, mw, wlo, NWM, sm);
    if constexpr (STAGE && !FUSE) {
#pragma unroll
        for (int u = 0; u < PER; ++u)
            if (u * BS + (int)threadIdx.x < SN) ys[u * BS + threadIdx.x] = stv[u];
    }
    KSTAMP(1);
    int total;
    const int o = block_exclusive_scan<BS>(kept, lds_i, &total);
    const long long b_tot = block_sum_ll<BS>(bordered, lds_l);
    // published by the whole of wave 0 (a wave-uniform branch; the block sums are
    // uniform, read through readfirstlane), not by one lane (publication audit)
    if (threadIdx.x < 64) {
        const unsigned long long v = kPkValid | ((unsigned long long)__builtin_amdgcn_readfirstlane((int)b_tot) << 31) |
                                     (unsigned)__builtin_amdgcn_readfirstlane(total);
        __hip_atomic_store(slot + chunk, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    long long before = 0, k_all = 0, b_all = 0;
    bool ok = true;
    for (int k = threadIdx.x; k < nch; k += BS) {
        unsigned long long v;
        unsigned spins = 0;
        while (!((v = __hip_atomic_load(slot + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & kPkValid)) {
            if (++spins > (1u << 22)) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const long long kk = (long long)(v & 0x7fffffffull), bb = (long long)((v >> 31) & 0x7fffffffull);
        before += k < chunk ? kk : 0;
        k_all += kk;
        b_all += bb;
    }
    before = block_sum_ll<BS>(before, lds_l);
    k_all = block_sum_ll<BS>(k_all, lds_l);
    b_all = block_sum_ll<BS>(b_all, lds_l);
    const long long bad = block_sum_ll<BS>(ok ? 0 : 1, lds_l);
    if (bad) {
        if (threadIdx.x == 0) w.status[s] = MDG_ERR_HIP;
        return;
    }
    if (b_all == 0) {
        if (chunk == 0 && threadIdx.x == 0) w.status[s] = MDG_NO_PEAKS_DETECTED;
        return;
    }
    if (chunk == 0 && threadIdx.x == 0) w.det_count[s] = (int32_t)k_all;
    KSTAMP(2);
    const size_t b0 = (size_t)s * w.capD + before;
    if (kept)
        word_peaks<true, FUSE>(a, w, s, wd, sel, detector_only, &bordered, b0 + o, STAGE ? pk : nullptr, PCAP, o, mw,
                               wlo, NWM, sm);
    if (detector_only || !score) return;
    KSTAMP(3);
    // k_scores' work for this chunk's peaks, spread evenly over the block
    __syncthreads();  // the peaks above, written by other threads of the block
    if (STAGE && total <= PCAP) {
        for (int p = threadIdx.x; p < total; p += BS) {
            const int l = pk[p], c = pk[PCAP + p], r = pk[2 * PCAP + p];
            w.scores[b0 + p] = l - 1 >= lo && r + 1 < lo + SN ? score_peak_lds(ys, lo, l, c, r)
                                                               : score_peak(sm, a.N, l, c, r);
        }
    } else {
        for (int p = threadIdx.x; p < total; p += BS)
            w.scores[b0 + p] = score_peak(sm, a.N, w.det_l[b0 + p], w.det_c[b0 + p], w.det_r[b0 + p]);
    }
    KSTAMP(4);
}

// ----------------------------------------------------------------------------------
// K4  noise-score selection (noise_score_filter.rs:91-138, scorer.rs:65-75, common.rs:26-40)
// ----------------------------------------------------------------------------------

// Left fold over the signal-free-region scores peaks[..left] ++ peaks[right..P]
// in the reference's order (noise_score_filter.rs:129-138), by ONE wave. Terms
// come 16 at a time, lane l holding term l & 15 (each 16-lane row a copy), and
// every term is added with one v_fmac_f64 acc, term, 1.0 whose DPP row_newbcast:k
// hands row lane k to the whole row: fma(t, 1, acc) rounds exactly like acc + t
// (t*1 is exact), so the chain is the reference's adds, one instruction per
// term, no readlane. Four groups of loads stay in flight (in-order vmcnt).


// acc + t[0] + ... + t[n-1] (left to right) by one wave: groups of 16 terms loaded
// with lane l holding t[16g + (l & 15)], fold16-style DPP adds. The steady part is
// one asm loop with 12 load buffers: each group waits vmcnt(11) and, after its 16
// adds, reloads its buffer with the group 12 ahead -- loads never cross the loop's
// back-edge in a compiler-visible register (which forces vmcnt(0) there).
constexpr int kFoldD = 12;
__device__ __forceinline__ double dpp_fold_steady(double acc, const double* t, int iters) {
    const double one = 1.0;
    asm volatile(
        "v_mov_b64 v[44:45], %[addr]\n"
        "v_mov_b64 v[46:47], %[acc]\n"
        "v_mov_b64 v[48:49], %[one]\n"
        "s_mov_b32 s40, %[it]\n"
        "s_mov_b64 s[42:43], 1536\n"
        "global_load_dwordx2 v[20:21], v[44:45], off offset:0\n"
        "global_load_dwordx2 v[22:23], v[44:45], off offset:128\n"
        "global_load_dwordx2 v[24:25], v[44:45], off offset:256\n"
        "global_load_dwordx2 v[26:27], v[44:45], off offset:384\n"
        "global_load_dwordx2 v[28:29], v[44:45], off offset:512\n"
        "global_load_dwordx2 v[30:31], v[44:45], off offset:640\n"
        "global_load_dwordx2 v[32:33], v[44:45], off offset:768\n"
        "global_load_dwordx2 v[34:35], v[44:45], off offset:896\n"
        "global_load_dwordx2 v[36:37], v[44:45], off offset:1024\n"
        "global_load_dwordx2 v[38:39], v[44:45], off offset:1152\n"
        "global_load_dwordx2 v[40:41], v[44:45], off offset:1280\n"
        "global_load_dwordx2 v[42:43], v[44:45], off offset:1408\n"
        "Lfold%=:\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[20:21], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[20:21], v[44:45], off offset:1536\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[22:23], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[22:23], v[44:45], off offset:1664\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[24:25], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[24:25], v[44:45], off offset:1792\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[26:27], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[26:27], v[44:45], off offset:1920\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[28:29], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[28:29], v[44:45], off offset:2048\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[30:31], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[30:31], v[44:45], off offset:2176\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[32:33], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[32:33], v[44:45], off offset:2304\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[34:35], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[34:35], v[44:45], off offset:2432\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[36:37], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[36:37], v[44:45], off offset:2560\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[38:39], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[38:39], v[44:45], off offset:2688\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[40:41], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[40:41], v[44:45], off offset:2816\n"
        "s_waitcnt vmcnt(11)\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:0 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:10 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:11 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:12 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:13 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:14 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp v[46:47], v[42:43], v[48:49] row_newbcast:15 row_mask:0xf bank_mask:0xf\n"
        "global_load_dwordx2 v[42:43], v[44:45], off offset:2944\n"
        "v_lshl_add_u64 v[44:45], v[44:45], 0, s[42:43]\n"
        "s_sub_u32 s40, s40, 1\n"
        "s_cmp_lg_u32 s40, 0\n"
        "s_cbranch_scc1 Lfold%=\n"
        "s_waitcnt vmcnt(0)\n"
        "v_mov_b64 %[acc], v[46:47]\n"
        : [acc] "+v"(acc)
        : [addr] "v"(t + (threadIdx.x & 15)), [one] "v"(one), [it] "s"(sgpr_int(iters))
        : "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "s40", "s42", "s43", "scc", "memory");
    return acc;
}

__device__ double dpp_fold(double acc, const double* __restrict__ t, int n) {
    const int sub = threadIdx.x & 15;
    const double one = 1.0;
    const int G = n / 16;
    // steady asm loop: iterations of kFoldD groups whose prefetch stays below G
    const int it = G / kFoldD - 1;
    int g = 0;
    if (it > 0) {
        acc = dpp_fold_steady(acc, t, it);
        g = it * kFoldD;
    }
    for (; g < G; ++g) fold16(acc, t[16 * g + sub], one);
    const int r = n - 16 * G;
    if (r > 0) {
        const double v = t[min(16 * G + sub, n - 1)];
        for (int k = 0; k < r; ++k) acc += readlane_f64(v, k);
    }
    return acc;
}

// ----------------------------------------------------------------------------------
// Windowed fold: acc0 + t[0] + ... + t[n-1], left to right with a rounding per add,
// for NON-NEGATIVE terms, by the whole workgroup instead of one wave.
//
// The n terms (global memory, L2-resident) are cut into kWinSeg segments. A
// running sum of non-negative terms grows monotonically and stays close to the
// correctly rounded exact prefix sum (tools/probes/fold_window.py: at most 31
// ulps for the SFR scores and squared deviations of every probed spectrum). So:
//  A. the exact prefix sum at each segment start is estimated in double-double
//     and rounded: E_k;
//  B. each segment is folded from 64 candidate start values at once, lane j
//     starting from E_k stepped by (j - 32) ulps (consecutive doubles), with the
//     reference's additions (dpp_fold: every lane adds the same term, in order);
//  C. one wave walks the segments in order: the true value entering segment k is
//     one of its candidates (bit-equal) -> the true value leaving it is that
//     lane's result. A true value outside the window is not an error: that
//     segment is folded again from it.
// Every step of the returned value is an IEEE add in the reference's order, so
// the result is the reference's bits whatever the estimates (they only decide
// how often step C falls back).
// ----------------------------------------------------------------------------------
constexpr int kWinSeg = 16;  // one segment per wave of k_select (32: 6% slower, the walk is serial)
struct WinLds {
    double F[kWinSeg][64];
    double E[kWinSeg];
    double out;
};

__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
    s = a + b;
    const double bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}

// dpp_fold for one window segment (a few hundred terms): groups of 16 terms are
// loaded 8 groups at a time, the next 8 in flight while the current 8 are folded
// (dpp_fold's own steady loop starts at 24 groups; below that it waits on every load).
// The count is made wave-uniform (a call passes it in a VGPR), so the group loops are
// scalar branches, and only the last partial batch clamps its addresses: the
// per-group exec-mask branches and per-load clamps of the first version cost ~40% of
// stage B (18.4k cycles per fold on blood_01's 5116 SFR scores).
__device__ __noinline__ double seg_fold(double acc, const double* __restrict__ t, int n) {
    n = __builtin_amdgcn_readfirstlane(n);
    const int sub = threadIdx.x & 15;
    const double one = 1.0;
    const int G = n / 16;
    const double* tp = t + sub;
    int g = 0;
    if (G >= 8) {
        double cur[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) cur[u] = tp[16 * u];
        for (; g + 16 <= G; g += 8) {
            double nxt[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) nxt[u] = tp[16 * (g + 8 + u)];
#pragma unroll
            for (int u = 0; u < 8; ++u) fold16(acc, cur[u], one);
#pragma unroll
            for (int u = 0; u < 8; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) fold16(acc, cur[u], one);
        g += 8;
    }
    {  // the last < 8 groups: their loads issued together
        double tl[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (g + u < G) tl[u] = tp[16 * (g + u)];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (g + u < G) fold16(acc, tl[u], one);
    }
    const int r = n - 16 * G;
    if (r > 0) {
        const double v = t[min(16 * G + sub, n - 1)];
        for (int k = 0; k < r; ++k) acc += readlane_f64(v, k);
    }
    return acc;
}

// t: global memory or LDS (a generic pointer: the windowed fold of k_select reads its
// LDS-staged terms through it)
template <int BS>
__device__ __forceinline__ double window_fold(double acc0, WinLds& L, const double* __restrict__ t, int n,
                              int stamp = 40) {
    constexpr int NW = BS / 64;
    static_assert(kWinSeg <= 64, "one lane per segment in the prefix scan");
    KSTAMP(stamp + 5);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int seg = (n + kWinSeg - 1) / kWinSeg;
    // A. double-double sums of the segments (wave w: segments w, w+NW, ...); a
    // lane's terms of a segment are loaded 8 at a time (16: slower, 12k against 8k cycles)
    for (int k = wv; k < kWinSeg; k += NW) {
        double hi = 0.0, lo = 0.0;
        const int i0 = k * seg, i1 = min(n, (k + 1) * seg);
        for (int c = i0; c < i1; c += 8 * 64) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = c + 64 * u + lane;
                v[u] = i < i1 ? t[i] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                double e;
                two_sum(hi, v[u], hi, e);
                lo += e;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double h2 = __shfl_xor(hi, o, 64), l2 = __shfl_xor(lo, o, 64);
            double e;
            two_sum(hi, h2, hi, e);
            lo += l2 + e;
        }
        if (lane == 0) L.F[k][0] = hi, L.F[k][1] = lo;
    }
    __syncthreads();
    KSTAMP(stamp + 6);
    if (threadIdx.x < 64) {
        // exclusive prefix of the segment sums in double-double, by wave 0 as a
        // log-depth (Kogge-Stone) scan over lanes: the estimates only decide which
        // candidate windows step C tries, so their summation order is free
        double hi = lane < kWinSeg ? L.F[lane][0] : 0.0;
        double lo = lane < kWinSeg ? L.F[lane][1] : 0.0;
        if (lane == 0) {  // acc0 enters before segment 0
            double e;
            two_sum(acc0 == 0.0 ? 0.0 : acc0, hi, hi, e);
            lo += e;
        }
#pragma unroll
        for (int o = 1; o < kWinSeg; o <<= 1) {
            const double h2 = __shfl_up(hi, o, 64), l2 = __shfl_up(lo, o, 64);
            if (lane >= o) {
                double e;
                two_sum(hi, h2, hi, e);
                lo += l2 + e;
            }
        }
        // inclusive -> exclusive: segment k starts at the sum through segment k-1
        double ih, il;
        two_sum(hi, lo, ih, il);
        const double ex = __shfl_up(ih, 1, 64);
        if (lane < kWinSeg) L.E[lane] = lane == 0 ? (acc0 == 0.0 ? 0.0 : acc0) : ex;
    }
    __syncthreads();
    KSTAMP(stamp);
    // B. every segment from 64 candidates (segment 0 from acc0 itself, exactly)
    for (int k = wv; k < kWinSeg; k += NW) {
        double acc;
        if (k == 0) {
            acc = acc0;
        } else {
            const long long b = __double_as_longlong(L.E[k]) + (lane - 32);
            acc = __longlong_as_double(b < 0 ? 0ll : b);
        }
        const int i0 = min(n, k * seg), i1 = min(n, (k + 1) * seg);
        L.F[k][lane] = seg_fold(acc, t + i0, i1 - i0);
    }
    __syncthreads();
    KSTAMP(stamp + 1);
    // C. the true chain through the segments, by wave 0: the true value entering
    // segment k is candidate d = bits(tru) - bits(E_k) + 32 when that lies in
    // [0, 64) (clamped candidates below +0 only ever equal +0, which d then names),
    // and the value leaving it is that candidate's result, one LDS read away
    if (wv == 0) {
        const long long eb = lane < kWinSeg ? __double_as_longlong(L.E[lane]) : 0;
        double tru = L.F[0][0];
#pragma unroll 1
        for (int k = 1; k < kWinSeg; ++k) {
            const long long ek = ((long long)__builtin_amdgcn_readlane((int)(eb >> 32), k) << 32) |
                                 (long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(eb & 0xffffffffll), k);
            const long long d = __double_as_longlong(tru) - ek + 32;
            if (d >= 0 && d < 64) {
                tru = L.F[k][(int)d];
            } else {  // outside the window: this segment from the true value
                const int i0 = min(n, k * seg), i1 = min(n, (k + 1) * seg);
                tru = seg_fold(tru, t + i0, i1 - i0);
#ifdef MDG_DIAG
                if (lane == 0 && blockIdx.x == 0 && g_diag) g_diag[kDiagStampBase + stamp + 7] += 1;
#endif
            }
        }
        if (lane == 0) L.out = tru;
    }
    __syncthreads();
    KSTAMP(stamp + 2);
    return L.out;
}

// test support (mdg_ordered_sum): the windowed fold of k_select on caller data
__global__ __launch_bounds__(1024) void k_ordered_sum(const double* __restrict__ t, int n, double acc0,
                                                      double* out) {
    __shared__ WinLds wl;
    const double r = window_fold<1024>(acc0, wl, t, n);
    if (threadIdx.x == 0) out[0] = r;
}
void launch_ordered_sum(const double* t, int n, double acc0, double* out, hipStream_t st) {
    hipLaunchKernelGGL(k_ordered_sum, dim3(1), dim3(1024), 0, st, t, n, acc0, out);
}

// test support (mdg_check_fast_division): div_rn_fast against the compiler's IEEE
// division on n pseudo-random operand pairs of the FAST range [2^-200, 2^200]
// (random mantissas, and mantissas made of long runs of ones or zeros)
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ double fast_range_operand(unsigned long long h, bool runs) {
    unsigned long long m = h & 0xfffffffffffffull;
    if (runs) m = (h & 1) ? (0xfffffffffffffull >> (h >> 58)) : (1ull << ((h >> 52) & 51));
    const int e = (int)((h >> 12) % 401) - 200;
    return __longlong_as_double((long long)(((unsigned long long)(e + 1023) << 52) | m));
}
// variant 0: div_rn (fit, superposition_vec), 1: div_rn_1nr (MSE only).
// cases 0: random pairs, 1: constructed near-midpoint pairs (division_hard_case).
// out[0] += mismatches, out[1] += pairs tested.
template <int VARIANT>
__device__ __forceinline__ double div_variant(double n, double d) {
    return VARIANT == 0 ? div_rn(n, d) : div_rn_1nr(n, d);
}
template <int VARIANT>
__global__ void k_division_check(unsigned long long seed, long long n, int cases,
                                 unsigned long long* out) {
    unsigned long long nb = 0, nt = 0;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        double num, d;
        if (cases == 0) {
            const unsigned long long h1 = mix64(seed ^ (2 * i)), h2 = mix64(seed ^ (2 * i + 1));
            const bool runs = (h1 >> 63) & (h2 >> 63);
            num = fast_range_operand(h1, runs);
            d = fast_range_operand(h2, runs);
        } else {
            bool ok;
            division_hard_case(seed, (uint64_t)i, &num, &d, &ok);
            if (!ok) continue;
        }
        ++nt;
        nb += __double_as_longlong(div_variant<VARIANT>(num, d)) != __double_as_longlong(num / d);
    }
    if (nb) atomicAdd(out, nb);
    atomicAdd(out + 1, nt);
}
void launch_division_check(int variant, int cases, unsigned long long seed, long long n,
                           unsigned long long* out, hipStream_t st) {
    if (variant == 0)
        hipLaunchKernelGGL(k_division_check<0>, dim3(4096), dim3(256), 0, st, seed, n, cases, out);
    else
        hipLaunchKernelGGL(k_division_check<1>, dim3(4096), dim3(256), 0, st, seed, n, cases, out);
}

__device__ __forceinline__ void fit_init_peak(const BatchArgs& a, const Workspace& w, int s, size_t base,
                                              int p, int l, int c, int r);
__device__ __forceinline__ void fit_init_pair(const BatchArgs& a, const Workspace& w, int s, size_t base,
                                              int p1, int l1, int c1, int r1, int p2, int l2, int c2,
                                              int r2);

// k_select's LDS: the SFR terms of the two windowed folds (up to kSfrLds; more go
// through the workspace), reused afterwards for the selected peaks (up to kSelLds)
constexpr int kSfrLds = 12288;         // 96 KB
constexpr int kSelWinMin = 1024;       // signal-free-region terms from which the folds are windowed
constexpr int kSelLds = 4096;          // 3 ints each: 48 KB of the same buffer
// centers per thread counted directly: 1, i.e. only P <= 1024 (blood_01, P = 16100,
// stamps at B = 1: the two-level search 7.2-8.1k cycles, 16 direct loads per thread
// 11.2k strided and 12.1k coalesced)
constexpr int kSelCountDirect = 1;
constexpr int kSelPerThread = 16;      // candidates per thread compacted from registers
static_assert(3 * kSelLds * sizeof(int) <= kSfrLds * sizeof(double), "selection fits the SFR buffer");
// K3s  detection of a SMALL spectrum (N <= kSmallN) inside k_select's workgroup (DET):
// k_flags' predicates over the row staged in LDS (ys), the masks in LDS, k_peaks'
// word scans and scoring (word_peaks, score_peak_lds: the same operations in the same
// order), the peaks written where k_peaks writes them. Two launches and their
// boundaries fewer for the reference's own benchmark spectra (sim, 2048 points:
// k_flags 4.7 + k_peaks 10 us of dependent launches, round 6). Returns the kept
// count, or -1 with the status set (NoPeaksDetected) when no peak has both borders.
constexpr int kDetW = kSmallN / 64;  // mask words of a small spectrum
template <int BS>
__device__ __forceinline__ int detect_small(const BatchArgs& a, const Workspace& w, int s, double* ys, int* pk,
                                            int* park, double* scl, uint64_t* mlds, int* lds_i, long long* lds_l) {
    static_assert(BS >= 4 * kDetW, "four threads per mask word");
    const int N = a.N, W = w.W, tid = threadIdx.x, lane = tid & 63;
    const double* __restrict__ sm = w.smooth_ptr + (size_t)s * w.smooth_stride;
    KSTAMP(80);
    for (int k = tid; k < N; k += BS) ys[k] = sm[k];
    __syncthreads();
    KSTAMP(81);
    // k_flags: centre, right-border and left-border predicates, one ballot per word
    for (int k = tid; k < 64 * W; k += BS) {
        bool fc = false, fr = false, fl = false;
        if (k >= 2 && k <= N - 3) {
            const double dm = dsd(ys, k - 1), d0 = dsd(ys, k), dp = dsd(ys, k + 1);
            fc = d0 < 0. && d0 < dm && d0 < dp;
            fr = d0 > dm && (d0 >= dp || (d0 < 0. && dp >= 0.));
            fl = d0 > dp && (d0 >= dm || (d0 < 0. && dm >= 0.));
        }
        const uint64_t bc = __ballot(fc), br = __ballot(fr), bl = __ballot(fl);
        if (lane == 0) {
            mlds[k >> 6] = bc;
            mlds[W + (k >> 6)] = br;
            mlds[2 * W + (k >> 6)] = bl;
        }
    }
    __syncthreads();
    KSTAMP(82);
    // k_peaks: four threads per mask word in centre order, each thread's kept peaks
    // (at most 8 of its 16 centre bits: strict minima) parked in its own slots of
    // park and moved to their places after the scan (one word pass, not two)
    const int wd = tid >> 2;
    const uint64_t sel = 0xffffull << (16 * (tid & 3));
    constexpr int PARK = 4 * kDetW * 8;
    int bordered = 0, kept = 0;
    if (wd < W)
        kept = word_peaks<true, true, false>(a, w, s, wd, sel, 0, &bordered, 0, park, PARK, 8 * tid, mlds, 0, W, sm);
    int total;
    const int o = block_exclusive_scan<BS>(kept, lds_i, &total);
    const long long b_all = block_sum_ll<BS>(bordered, lds_l);
    if (b_all == 0) {
        if (tid == 0) w.status[s] = MDG_NO_PEAKS_DETECTED;
        return -1;
    }
    if (tid == 0) w.det_count[s] = total;
    KSTAMP(83);
    const size_t b0 = (size_t)s * w.capD;
    constexpr int PCAP = kSmallN / 2;  // centres are strict minima
    for (int i = 0; i < kept; ++i) {
        const int l = park[8 * tid + i], c = park[PARK + 8 * tid + i], r = park[2 * PARK + 8 * tid + i];
        w.det_l[b0 + o + i] = l;
        w.det_c[b0 + o + i] = c;
        w.det_r[b0 + o + i] = r;
        pk[o + i] = l;
        pk[PCAP + o + i] = c;
        pk[2 * PCAP + o + i] = r;
    }
    __syncthreads();
    KSTAMP(84);
    // l >= 2 and r <= N - 3: every score's ticks l - 1 .. r + 1 lie in the staged row;
    // the selection reads the LDS copies (scl over the parking slots, free by now)
    for (int p = tid; p < total; p += BS) {
        const double sc = score_peak_lds(ys, 0, pk[p], pk[PCAP + p], pk[2 * PCAP + p]);
        w.scores[b0 + p] = sc;
        scl[p] = sc;
    }
    __syncthreads();
    KSTAMP(85);
    return total;
}

template <int BS, bool DET = false>
__global__ __launch_bounds__(BS) void k_select(BatchArgs a, Workspace w, double threshold) {
    const int s = blockIdx.x;
    __shared__ int lds_i[BS / 64 + 1];
    __shared__ __attribute__((aligned(16))) double sfr_lds[kSfrLds];
    int* const sel_lds = (int*)sfr_lds;
    __shared__ long long lds_l[BS / 64 + 1];
    __shared__ double thr_sh;
    __shared__ WinLds wl;
    // the spectrum's scalars in one memory round trip (as fit_head)
    int st, P;
    const int64_t sbi0 = w.sbi[2 * s], sbi1 = w.sbi[2 * s + 1];
    // DET: the row, the peaks and the parking slots (then the scores) in the SFR buffer,
    // free until the staging; that overwrites the row only (n_sfr <= P <= kSmallN / 2)
    constexpr int kPk = 3 * (kSmallN / 2) / 2, kPark = 3 * (4 * kDetW * 8) / 2;  // doubles
    static_assert(kSmallN + kPk + kPark <= kSfrLds, "row and peaks in the SFR buffer");
    int* const dpk = (int*)(sfr_lds + kSmallN);
    double* const dsc = sfr_lds + kSmallN + kPk;
    if constexpr (DET) {
        __shared__ uint64_t mlds[3 * kDetW];
        st = w.status[s];
        // k_flags' duty: the smoother's progress counters back to zero (any status)
        if ((int)threadIdx.x < w.chain_P) w.chain_flags[((size_t)s * w.chain_P + threadIdx.x) * 32] = 0;
        if (st) return;
        P = detect_small<BS>(a, w, s, sfr_lds, dpk, (int*)dsc, dsc, mlds, lds_i, lds_l);
        if (P < 0) return;
    } else {
        st = w.status[s];
        P = w.det_count[s];
        asm volatile("" ::"s"(st), "s"(P), "s"(sbi0), "s"(sbi1));
        if (st) return;
    }
    if (P == 0) {  // peaks.len() - 1 underflows in peak_region_boundaries
        if (threadIdx.x == 0) w.status[s] = MDG_REFERENCE_PANIC;
        return;
    }
    const size_t base = (size_t)s * w.capD;
    const int* pl = DET ? dpk : w.det_l + base;
    const int* pc = DET ? dpk + kSmallN / 2 : w.det_c + base;
    const int* pr = DET ? dpk + kSmallN : w.det_r + base;
    const double* scores = DET ? dsc : w.scores + base;
    KSTAMP(10);
    // #(center <= sbi0) and #(center <= sbi1) over the ascending centers (scores:
    // k_peaks), both counts packed in one sum: up to kSelCountDirect centers per
    // thread counted at once (their loads in flight together); beyond, a two-level
    // search (every step-th center first, then the step-1 centers after the last
    // sampled one that passed)
    const int step = (P + BS - 1) / BS;
    long long cnt0, cnt1;
    if (step <= kSelCountDirect) {
        // thread t counts centers t, t + BS, ...: each load instruction is coalesced
        long long v = 0;
#pragma unroll
        for (int u = 0; u < kSelCountDirect; ++u) {
            const int i = (int)threadIdx.x + BS * u;
            const int64_t c = pc[min(i, P - 1)];
            if (i < P) v += ((long long)(c <= sbi0) << 32) | (long long)(c <= sbi1);
        }
        const long long k01 = block_sum_ll<BS>(v, lds_l);
        cnt0 = k01 >> 32;
        cnt1 = k01 & 0xffffffffll;
    } else {
        long long k01;
        {
            const int i = threadIdx.x * step;
            long long v = 0;
            if (i < P) {
                const int64_t c = pc[i];
                v = ((long long)(c <= sbi0) << 32) | (long long)(c <= sbi1);
            }
            k01 = block_sum_ll<BS>(v, lds_l);
        }
        const long long k0 = k01 >> 32, k1 = k01 & 0xffffffffll;
        cnt0 = k0 > 0 ? (k0 - 1) * step + 1 : 0;
        cnt1 = k1 > 0 ? (k1 - 1) * step + 1 : 0;
        if (2 * (step - 1) > BS) {  // more than 2 * 513 * BS / 2 peaks: plain count
            long long c0 = 0, c1 = 0;
            for (int p = threadIdx.x; p < P; p += BS) {
                const int64_t c = pc[p];
                c0 += c <= sbi0;
                c1 += c <= sbi1;
            }
            cnt0 = block_sum_ll<BS>(c0, lds_l);
            cnt1 = block_sum_ll<BS>(c1, lds_l);
        } else if (step > 1) {
            const int t = threadIdx.x;
            long long v = 0;
            if (t < step - 1 && k0 > 0) {
                const long long i = (k0 - 1) * step + 1 + t;
                if (i < P) v += (long long)(pc[i] <= sbi0) << 32;
            } else if (t >= step - 1 && t < 2 * (step - 1) && k1 > 0) {
                const long long i = (k1 - 1) * step + 1 + (t - (step - 1));
                if (i < P) v += (long long)(pc[i] <= sbi1);
            }
            const long long r = block_sum_ll<BS>(v, lds_l);
            cnt0 += r >> 32;
            cnt1 += r & 0xffffffffll;
        }
    }
    // centers ascend: position(center > sb) == #(center <= sb)
    const int left = cnt0 < P ? (int)cnt0 : 0;
    const long long r1 = cnt1 > left ? cnt1 : left;
    const int right = r1 < P ? (int)r1 : P - 1;
    if (left == 0 && right >= P) {
        if (threadIdx.x == 0) w.status[s] = MDG_EMPTY_SIGNAL_FREE_REGION;
        return;
    }
    if (left == right) {
        if (threadIdx.x == 0) w.status[s] = MDG_EMPTY_SIGNAL_REGION;
        return;
    }
    __syncthreads();  // scores visible to the whole block
    KSTAMP(11);
    // mean_sd_scores (noise_score_filter.rs:129-138): left folds over the SFR =
    // peaks[..left] ++ peaks[right..], staged contiguously (all threads) and folded
    // by wave 0; then the squared deviations, staged in place, folded the same way
    const int n_sfr = left + (P - right);
    // scores and squared deviations are >= +0: the windowed fold applies. One wave folds
    // short sets itself (seg_fold: any address space), below kSelWinMin terms: its
    // fixed phases -- the double-double segment sums, 64 candidate folds per segment,
    // the walk, their barriers -- cost a 208-term set (sim_01) ~13k cycles per fold
    // against ~1.7k for the direct left fold (round 6, k_select's phase stamps)
    const bool win = n_sfr >= kSelWinMin;
    // staged in LDS when they fit (the folds' loads are then LDS reads, not L2 round
    // trips; the windowed fold's DPP segment folds measured 18.4k cycles against 29k
    // with scalar-loaded terms and 38k with LDS broadcast reads, blood_01, round 4);
    // the short-set dpp_fold stays off its asm global-load loop (n_sfr < 4 * kWinSeg)
    double* sfr = n_sfr <= kSfrLds ? sfr_lds : w.tmp0 + (size_t)s * a.N;
    for (int k = threadIdx.x; k < n_sfr; k += BS) sfr[k] = scores[k < left ? k : right + (k - left)];
    __syncthreads();
    KSTAMP(15);
    if (win) {
        const double sum = window_fold<BS>(-0.0, wl, sfr, n_sfr);  // every thread: barriers inside
        if (threadIdx.x == 0) thr_sh = sum / (double)n_sfr;
    } else if (threadIdx.x < 64) {
        const double mean = seg_fold(-0.0, sfr, n_sfr) / (double)n_sfr;
        if (threadIdx.x == 0) thr_sh = mean;
    }
    __syncthreads();
    KSTAMP(16);
    const double mean = thr_sh;
    for (int k = threadIdx.x; k < n_sfr; k += BS) {
        const double d = sfr[k] - mean;
        sfr[k] = d * d;
    }
    __syncthreads();
    double var = 0.0;
    if (win) var = window_fold<BS>(-0.0, wl, sfr, n_sfr, 50) / (double)n_sfr;
    else if (threadIdx.x < 64) var = seg_fold(-0.0, sfr, n_sfr) / (double)n_sfr;
    KSTAMP(17);
    if (threadIdx.x == 0) {
        const double sd = __builtin_sqrt(var);
        thr_sh = mean + (w.thr_s ? w.thr_s[s] : threshold) * sd;
        w.sfr_stats[2 * s] = mean;
        w.sfr_stats[2 * s + 1] = sd;
    }
    KSTAMP(13);
    __syncthreads();
    const double thr = thr_sh;
    // ordered compaction of peaks[left..right] with score >= thr
    const int len = right - left;
    const int per = (len + BS - 1) / BS;
    const int q0 = left + threadIdx.x * per;
    const int q1 = min(right, q0 + per);
    if (per <= kSelPerThread) {
        // up to kSelPerThread candidates per thread (len <= 16384), owned wave by
        // wave: wave v holds the contiguous range [left + 64·per·v, +64·per), lane l
        // its candidates 64u + l (u < per), so every score load is coalesced and the
        // order within the wave is (u, lane). The keep flags of round u are a ballot;
        // a kept candidate's position is its wave's offset (a scan over the waves),
        // the kept ones of the wave's earlier rounds and its lanes below it in round u
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        const int wbase = left + 64 * per * wv;
        // the rounds this wave has candidates in (wave-uniform): a short candidate range
        // (the sim spectra: ~100) leaves most waves none and the others one round, and
        // each skipped round is 4 loads per lane fewer (sim_01: compaction 13.4k cycles)
        const int nu = min(per, max(0, (right - wbase + 63) >> 6));
        double sc[kSelPerThread];  // the scores stay in VGPRs; the ballots are redone
#pragma unroll
        for (int u = 0; u < kSelPerThread; ++u) {
            sc[u] = 0.0;
            if (u < nu) sc[u] = scores[min(wbase + 64 * u + lane, P - 1)];
        }
        auto kept = [&](int u) { return u < nu && wbase + 64 * u + lane < right && sc[u] >= thr; };
        int wcount = 0;
#pragma unroll
        for (int u = 0; u < kSelPerThread; ++u) wcount += __popcll(__ballot(kept(u)));
        int total;
        KSTAMP(12);
        const int woff = block_exclusive_scan<BS>(lane == 0 ? wcount : 0, lds_i, &total);
        KSTAMP(19);
        const int wstart = __shfl(woff, 0, 64);  // lane 0's exclusive prefix: the wave's offset
        // the kept candidates' borders, every load issued before the first is used
        int lv[kSelPerThread], cv[kSelPerThread], rv[kSelPerThread];
#pragma unroll
        for (int u = 0; u < kSelPerThread; ++u) {
            const int q = min(wbase + 64 * u + lane, P - 1);
            lv[u] = cv[u] = rv[u] = 0;
            if (u < nu) {
                lv[u] = kept(u) ? pl[q] : 0;
                cv[u] = kept(u) ? pc[q] : 0;
                rv[u] = kept(u) ? pr[q] : 0;
            }
        }
        int o = wstart;
#pragma unroll
        for (int u = 0; u < kSelPerThread; ++u) {
            if (u >= nu) continue;  // (not break: the loop must unroll, or the arrays go to scratch)
            const uint64_t bu = __ballot(kept(u));
            if (bu >> lane & 1) {
                const int pos = o + __builtin_amdgcn_mbcnt_hi((unsigned)(bu >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((unsigned)bu, 0u));
                const int l = lv[u], c = cv[u], r = rv[u];
                w.sel_l[base + pos] = l;
                w.sel_c[base + pos] = c;
                w.sel_r[base + pos] = r;
                if (pos < kSelLds) {
                    sel_lds[3 * pos] = l;
                    sel_lds[3 * pos + 1] = c;
                    sel_lds[3 * pos + 2] = r;
                }
            }
            o += __popcll(bu);
        }
        if (threadIdx.x == 0) {
            w.sel_count[s] = total;
            if (total == 0) w.status[s] = MDG_EMPTY_SIGNAL_REGION;
        }
        KSTAMP(14);
        const bool in_lds = total <= kSelLds;
        if (in_lds) lds_barrier();
        else __syncthreads();
        for (int p = threadIdx.x; p < total; p += 2 * BS) {
            const int p2 = p + BS < total ? p + BS : p;
            int l1, c1, r1, l2, c2, r2;
            if (in_lds) {
                l1 = sel_lds[3 * p]; c1 = sel_lds[3 * p + 1]; r1 = sel_lds[3 * p + 2];
                l2 = sel_lds[3 * p2]; c2 = sel_lds[3 * p2 + 1]; r2 = sel_lds[3 * p2 + 2];
            } else {
                l1 = w.sel_l[base + p]; c1 = w.sel_c[base + p]; r1 = w.sel_r[base + p];
                l2 = w.sel_l[base + p2]; c2 = w.sel_c[base + p2]; r2 = w.sel_r[base + p2];
            }
            fit_init_pair(a, w, s, base, p, l1, c1, r1, p2, l2, c2, r2);
        }
        KSTAMP(18);
        return;
    }
    int keep = 0;
    for (int q = q0; q < q1; ++q) keep += scores[q] >= thr;
    int total;
    int out = block_exclusive_scan<BS>(keep, lds_i, &total);
    for (int q = q0; q < q1; ++q) {
        if (scores[q] >= thr) {
            const size_t o = base + out;
            const int l = pl[q], c = pc[q], r = pr[q];
            w.sel_l[o] = l;
            w.sel_c[o] = c;
            w.sel_r[o] = r;
            if (out < kSelLds) {  // the fit initialisation below reads them from LDS
                sel_lds[3 * out] = l;
                sel_lds[3 * out + 1] = c;
                sel_lds[3 * out + 2] = r;
            }
            ++out;
        }
    }
    if (threadIdx.x == 0) {
        w.sel_count[s] = total;
        if (total == 0) w.status[s] = MDG_EMPTY_SIGNAL_REGION;
    }
    KSTAMP(14);
    // the fit's initial state (k_fit_init's work), spread evenly over the block:
    // selected peaks p and p + BS per thread, their loads in flight together. The
    // selection comes from LDS (a barrier that does not wait for the global
    // stores above), or from memory after a full barrier when it does not fit
    const bool in_lds = total <= kSelLds;
    if (in_lds) lds_barrier();
    else __syncthreads();
    for (int p = threadIdx.x; p < total; p += 2 * BS) {
        const int p2 = p + BS < total ? p + BS : p;
        int l1, c1, r1, l2, c2, r2;
        if (in_lds) {
            l1 = sel_lds[3 * p]; c1 = sel_lds[3 * p + 1]; r1 = sel_lds[3 * p + 2];
            l2 = sel_lds[3 * p2]; c2 = sel_lds[3 * p2 + 1]; r2 = sel_lds[3 * p2 + 2];
        } else {
            l1 = w.sel_l[base + p]; c1 = w.sel_c[base + p]; r1 = w.sel_r[base + p];
            l2 = w.sel_l[base + p2]; c2 = w.sel_c[base + p2]; r2 = w.sel_r[base + p2];
        }
        fit_init_pair(a, w, s, base, p, l1, c1, r1, p2, l2, c2, r2);
    }
    KSTAMP(18);
}

// DetectorOnly: the detector output is the selection (detector_only.rs:17-39)
__global__ void k_select_detector_only(BatchArgs a, Workspace w) {
    const int s = blockIdx.y;
    if (w.status[s]) return;
    const int P = w.det_count[s];
    if (blockIdx.x == 0 && threadIdx.x == 0) w.sel_count[s] = P;
    const size_t base = (size_t)s * w.capD;
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
        const int l = w.det_l[base + p], c = w.det_c[base + p], r = w.det_r[base + p];
        w.sel_l[base + p] = l;
        w.sel_c[base + p] = c;
        w.sel_r[base + p] = r;
        fit_init_peak(a, w, s, base, p, l, c, r);
    }
}

// ----------------------------------------------------------------------------------
// K5  fit: stencil gather, shoulder mirroring, closed-form 3x3 solve
// fitting/fitter_analytical.rs:19-37,147-172, peak_stencil.rs:27-36,113-131,
// reduced_spectrum.rs:16-43. Fitting uses the RAW intensities.
// ----------------------------------------------------------------------------------
struct Stencil {
    double x1, x2, x3, y1, y2, y3;
};

__device__ __forceinline__ void mirror_shoulder(Stencil& q) {
    const bool increasing = q.y1 <= q.y2 && q.y2 <= q.y3;
    const bool decreasing = q.y1 >= q.y2 && q.y2 >= q.y3;
    if (increasing) {
        q.y3 = q.y1;
        q.x3 = 2.0 * q.x2 - q.x1;
    } else if (decreasing) {
        q.y1 = q.y3;
        q.x1 = 2.0 * q.x2 - q.x3;
    }
}

__device__ __forceinline__ void solve(const Stencil& q, double* out3) {
    const double x1 = q.x1, x2 = q.x2, x3 = q.x3, y1 = q.y1, y2 = q.y2, y3 = q.y3;
    const double numerator =
        x1 * x1 * y1 * (y2 - y3) + x2 * x2 * y2 * (y3 - y1) + x3 * x3 * y3 * (y1 - y2);
    const double divisor =
        2.0 * (x1 - x2) * y1 * y2 + 2.0 * (x2 - x3) * y2 * y3 + 2.0 * (x3 - x1) * y3 * y1;
    const double m = numerator / divisor;
    const double t1 = x1 - m, t2 = x2 - m, t3 = x3 - m;
    const double left = (y1 * (t1 * t1) - y2 * (t2 * t2)) / (y2 - y1);
    const double right = (y2 * (t2 * t2) - y3 * (t3 * t3)) / (y3 - y2);
    const double h = fmax((left + right) / 2.0, kEpsilon);
    out3[0] = y2 * (h + t2 * t2);
    out3[1] = h;
    out3[2] = m;
}

// Stencil rows (round 6): per spectrum an x plane (x1 x2 x3 of each peak, 3 capD
// doubles) followed by a y plane (y1 y2 y3). An update rewrites the three y values
// and, of the x values, only the one mirror_shoulder replaced (x2 never changes):
// with the six values of a peak in one 48-byte record the unchanged x values shared
// the written lines, so every update rewrote all of them (k_fit_update: 144 bytes per
// peak and iteration moved)
__device__ __forceinline__ double* stencil_x(const Workspace& w, size_t base, int p) {
    return w.stencil + 6 * base + 3 * (size_t)p;
}
__device__ __forceinline__ double* stencil_y(const Workspace& w, size_t base, int p) {
    return w.stencil + 6 * base + 3 * (size_t)w.capD + 3 * (size_t)p;
}
__device__ __forceinline__ Stencil load_stencil(const Workspace& w, size_t base, int p) {
    const double* sx = stencil_x(w, base, p);
    const double* sy = stencil_y(w, base, p);
    return Stencil{sx[0], sx[1], sx[2], sy[0], sy[1], sy[2]};
}
__device__ __forceinline__ void store_stencil(const Workspace& w, size_t base, int p, const Stencil& q) {
    double* sx = stencil_x(w, base, p);
    double* sy = stencil_y(w, base, p);
    sx[0] = q.x1; sx[1] = q.x2; sx[2] = q.x3;
    sy[0] = q.y1; sy[1] = q.y2; sy[2] = q.y3;
}
// q: the updated stencil of peak p, x1 / x3 as it held them before (old1 / old3)
__device__ __forceinline__ void store_updated_stencil(const Workspace& w, size_t base, int p, const Stencil& q,
                                                      double old1, double old3) {
    double* sx = stencil_x(w, base, p);
    double* sy = stencil_y(w, base, p);
    if (__double_as_longlong(q.x1) != __double_as_longlong(old1)) sx[0] = q.x1;
    if (__double_as_longlong(q.x3) != __double_as_longlong(old3)) sx[2] = q.x3;
    sy[0] = q.y1; sy[1] = q.y2; sy[2] = q.y3;
}

// selected peak p of spectrum s with borders (l, c, r): its reduced points, the
// mirrored stencil and the initial parameters (version 0)
__device__ __forceinline__ void fit_init_peak(const BatchArgs& a, const Workspace& w, int s, size_t base,
                                              int p, int l, int c, int r) {
    const double* x = a.x + (size_t)s * a.x_stride;
    const double* y = y_row(a, s);
    Stencil q{x[l], x[c], x[r], y[l], y[c], y[r]};
    double* rx = w.rx + 3 * base + 3 * (size_t)p;
    double* ry = w.ry + 3 * base + 3 * (size_t)p;
    rx[0] = q.x1; rx[1] = q.x2; rx[2] = q.x3;
    ry[0] = q.y1; ry[1] = q.y2; ry[2] = q.y3;
    mirror_shoulder(q);
    store_stencil(w, base, p, q);
    double* L = w.params + 3 * base + 3 * (size_t)p;
    solve(q, L);
    if (!peak_fast_ok(L[0], L[1], L[2])) atomicAdd(&w.unsafe[4 * s], 1);
}

// two peaks (p2 == p1 for one): both stencils' loads in flight together
__device__ __forceinline__ void fit_init_pair(const BatchArgs& a, const Workspace& w, int s, size_t base,
                                              int p1, int l1, int c1, int r1, int p2, int l2, int c2,
                                              int r2) {
    const double* x = a.x + (size_t)s * a.x_stride;
    const double* y = y_row(a, s);
    const double xa[6] = {x[l1], x[c1], x[r1], x[l2], x[c2], x[r2]};
    const double ya[6] = {y[l1], y[c1], y[r1], y[l2], y[c2], y[r2]};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (k == 1 && p2 == p1) break;
        const int p = k ? p2 : p1;
        Stencil q{xa[3 * k], xa[3 * k + 1], xa[3 * k + 2], ya[3 * k], ya[3 * k + 1], ya[3 * k + 2]};
        double* rx = w.rx + 3 * base + 3 * (size_t)p;
        double* ry = w.ry + 3 * base + 3 * (size_t)p;
        rx[0] = q.x1; rx[1] = q.x2; rx[2] = q.x3;
        ry[0] = q.y1; ry[1] = q.y2; ry[2] = q.y3;
        mirror_shoulder(q);
        store_stencil(w, base, p, q);
        double* L = w.params + 3 * base + 3 * (size_t)p;
        solve(q, L);
        if (!peak_fast_ok(L[0], L[1], L[2])) atomicAdd(&w.unsafe[4 * s], 1);
    }
}

// K6  fit superposition at the 3P reduced points + ratio (fitter_analytical.rs:40-47)
// Ping-pong range flags: iteration `it` reads unsafe[it&1] (written by the
// producer of its parameters) and clears unsafe[(it+1)&1] for k_fit_update(it).
// per-spectrum fit iteration counts (optimize_settings batches): a spectrum whose
// count is reached skips the remaining superposition/update launches
__device__ __forceinline__ bool fit_done(const Workspace& w, int s, int it) {
    return w.fit_iters_s && it >= w.fit_iters_s[s];
}

// Record that spectrum s took the plain-division path (slot 3 of its range flags,
// cleared by prep_spectrum): bit min(it, 29) for fit iteration it, kSlowMse for
// k_mse_local's direct sums, kSlowMseExact for k_mse_exact_res. One lane of one
// workgroup per launch and spectrum, and only on the slow path, so the fast path
// pays a branch. mdg_ctx_last_range_flags reads it back: the tests' proof that a
// spectrum outside the fast ranges really ran the IEEE division.
constexpr int kSlowMse = 30, kSlowMseExact = 31;
__device__ __forceinline__ void mark_slow(const Workspace& w, int s, int bit) {
    atomicOr(&w.unsafe[4 * s + 3], (int)(1u << bit));
}
__device__ __forceinline__ int slow_bit(int it) { return it < 29 ? it : 29; }

// What a term-fold launch needs of spectrum s before its first parameter load, read
// together: one memory round trip. Written as branches (status, then fit_iters_s,
// then sel_count, then x_ok and unsafe) they were a chain of dependent loads, each
// waited for before the next was issued (the ISA of k_fit_sup_tf: six waits before
// the first parameter load), which a B = 1 launch of a few microseconds pays in full.
struct FitHead {
    bool live;  // neither failed nor past its own iteration count
    bool fast;  // x_ok and no parameter outside the fast ranges (slot it % 3)
    int P;
};
__device__ __forceinline__ FitHead fit_head(const Workspace& w, int s, int it) {
    const int st = w.status[s], P = w.sel_count[s], xo = w.x_ok[s], un = w.unsafe[4 * s + it % 3];
    const int fi = w.fit_iters_s ? w.fit_iters_s[s] : 0x7fffffff;
    // every value used here, so the compiler cannot sink a load behind the branch on
    // another (it did: status first, the rest after its wait)
    asm volatile("" ::"v"(st), "v"(P), "v"(xo), "v"(un), "v"(fi));
    return {st == 0 && it < fi, xo != 0 && un == 0, P};
}

// K6e  fit superposition + stencil update, term-fold form (small batches). A
// workgroup owns Q = 24 reduced points = 8 peaks of one spectrum. EW evaluator
// waves compute the terms of a chunk of J = 64*EW peaks (lane = peak, parameters
// in VGPRs; the Q x values are wave-uniform and sit in SGPRs) into LDS T[q][j].
// One fold wave (lane = point, raised priority) adds the chunk into each point's
// running sum in peak order -- the reference's left fold (lorentzian.rs:606-611),
// so the sums equal K6's bit for bit -- while the evaluators produce the next
// chunk into the other buffer (one barrier per chunk). The fold wave then owns
// whole peaks, so it also does k_fit_update's work for its 8 peaks
// (fitter_analytical.rs:48-65): ratio = y/sup, scale, mirror, re-solve. The new
// parameters go to the other parameter buffer (version it+1; odd versions in
// params_alt) because other workgroups still read version it; the range flags
// rotate over three slots (read it%3, count (it+1)%3, clear (it+2)%3).
// Measured (bench, P = 2048): 20.7 us per iteration at B = 1 against 28.0 for
// the DPP fold, 36 against 42 at B = 2; the DPP fold and one thread per point
// win from B = 4 (tools/fit_sweep.sh).
constexpr int kTfQ = 24, kTfEW = 3;
constexpr int kTfPad = 2;  // row padding (doubles): 16-byte aligned rows
template <int Q>
constexpr int tf_lds() { return 2 * Q * (64 * kTfEW + kTfPad); }

__device__ __forceinline__ const double* params_version(const Workspace& w, size_t base, int v) {
    return ((v & 1) ? w.params_alt : w.params) + 3 * base;
}

template <bool FAST, int QT = kTfQ>
__device__ __forceinline__ void fit_tf_body(const Workspace& w, int s, int P, int it, double* T) {
    constexpr int Q = QT, EW = kTfEW, J = 64 * EW;
    constexpr int RS = J + kTfPad;  // row stride of T (doubles)
    static_assert(Q % 3 == 0 && Q / 3 <= 64, "whole peaks per tile");
    const size_t base = (size_t)s * w.capD;
    const int npts = 3 * P;
    const int tiles = (npts + Q - 1) / Q;
    const int nch = (P + J - 1) / J;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const double* __restrict__ params = params_version(w, base, it);
    const bool folder = wv == EW;
    if (folder) __builtin_amdgcn_s_setprio(3);
    DIAG_DECL
    for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const int p0 = tile * Q;
        if (!folder) {
            // wave-uniform x of the tile's points; a tail tile reads past 3P into the
            // arena (ry follows rx), and those points are never used
            const const_f64_ptr rx = (const_f64_ptr)(w.rx + 3 * base + p0);
            double xq[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) xq[q] = rx[q];
            const int jl = wv * 64 + lane;
            int j = min(jl, P - 1);
            double f = params[3 * j], h = params[3 * j + 1], m = params[3 * j + 2];
            for (int c = 0; c <= nch; ++c) {
#ifdef MDG_DIAG
                if (c < nch && g_tf_mode == 2) {
                } else
#endif
                if (c < nch) {
                    double* Tb = T + (c & 1) * Q * RS + jl;
                    const double cf = f, ch = h, cm = m;
                    j = min((c + 1) * J + jl, P - 1);  // prefetch the next chunk's peak
                    f = params[3 * j];
                    h = params[3 * j + 1];
                    m = params[3 * j + 2];
#pragma unroll
                    for (int q = 0; q < Q; ++q) Tb[q * RS] = lorentz_t<FAST>(xq[q], cf, ch, cm);
                }
                DIAG_STAMP(0);
                lds_barrier();
                DIAG_STAMP(1);
            }
        } else {
            double acc = -0.0;
            const int q = lane < Q ? lane : Q - 1;
            // the stencil update's operands, loaded before the fold so their latency
            // hides behind it (this tile's stencils are only written below, by this wave)
            const double yq = w.ry[3 * base + min(p0 + q, npts - 1)];
            const int kq = lane < Q / 3 ? lane : 0;
            const int pkq = min(p0 / 3 + kq, P - 1);
            const Stencil sq0 = load_stencil(w, base, pkq);
            // acc = fma(t, 1, acc) rounds as acc + t; the VOP2 v_fmac_f64 chain issues
            // a cycle faster per term than dependent v_add_f64 (eval_cost.hip)
            double one = 1.0;
            asm volatile("" : "+v"(one));
            DIAG_STAMP(4);
            lds_barrier();  // chunk 0 written
            DIAG_STAMP(3);
            for (int c = 0; c < nch; ++c) {
                const double2* row = (const double2*)(T + (c & 1) * Q * RS + q * RS);
                const int cn = min(J, P - c * J);
                if (cn == J) {
                    // (round 5: a software-pipelined asm form, eight 16-byte reads kept in
                    // flight, was slower than this schedule -- ten tf12 launches 113 against
                    // 95 us at B = 1, twf1 385 against 370 at B = 16)
#pragma unroll 16
                    for (int k = 0; k < J / 2; ++k) {
                        const double2 v = row[k];
                        acc = __builtin_fma(v.x, one, acc);
                        acc = __builtin_fma(v.y, one, acc);
                    }
                } else {
                    const double* r1 = (const double*)row;
                    for (int k = 0; k < cn; ++k) acc = __builtin_fma(r1[k], one, acc);
                }
                DIAG_STAMP(2);
                lds_barrier();
                DIAG_STAMP(3);
            }
            // stencil update of the tile's peaks (k_fit_update): lane k gathers the
            // ratios y/sup of its peak's three points from lanes 3k..3k+2
            const double ratio = yq / acc;
            const int k = kq;
            const double r0 = __shfl(ratio, 3 * k, 64);
            const double r1 = __shfl(ratio, 3 * k + 1, 64);
            const double r2 = __shfl(ratio, 3 * k + 2, 64);
            const int pk = p0 / 3 + lane;
            if (lane < Q / 3 && pk < P) {
                Stencil sq = sq0;
                sq.y1 = sq.y1 * r0;
                sq.y2 = sq.y2 * r1;
                sq.y3 = sq.y3 * r2;
                mirror_shoulder(sq);
                store_updated_stencil(w, base, pk, sq, sq0.x1, sq0.x3);
                double* L = (((it + 1) & 1) ? w.params_alt : w.params) + 3 * base + 3 * (size_t)pk;
                solve(sq, L);
                if (!peak_fast_ok(L[0], L[1], L[2])) atomicAdd(&w.unsafe[4 * s + (it + 1) % 3], 1);
            }
            DIAG_STAMP(4);
        }
    }
    DIAG_FLUSH();
}

template <int Q>
__global__ __launch_bounds__(64 * (kTfEW + 1)) void k_fit_sup_tf(BatchArgs a, Workspace w, int it) {
    __shared__ __attribute__((aligned(16))) double T[tf_lds<Q>()];
    const int s = blockIdx.y;
    const FitHead h = fit_head(w, s, it);
    if (!h.live) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        w.unsafe[4 * s + (it + 2) % 3] = 0;
        if (!h.fast) mark_slow(w, s, slow_bit(it));
    }
    if (h.fast) fit_tf_body<true, Q>(w, s, h.P, it, T);
    else fit_tf_body<false, Q>(w, s, h.P, it, T);
}

// K6h  term-fold fit, wide tiles ("tw"): Q = 63 points (21 peaks) per workgroup
// instead of 24, so the fold wave's LDS reads serve 63 lanes, not 24 (a
// ds_read_b128 costs its wave 8 cycles of issue whatever EXEC holds,
// tools/ubench/fold_lds). The PB x PS evaluator waves split a chunk of J = 64 PB
// peaks into PB blocks (lane = peak, parameters in VGPRs) and the tile's points
// into PS subsets of Q / PS points (x wave-uniform in SGPRs), so a wave writes
// Q / PS terms per lane per chunk. Fold, stencil update and parameter versions as
// in k_fit_sup_tf, so the sums are the same left folds, bit for bit. A spectrum
// needs 98 workgroups instead of 256 at P = 2048: the same latency on fewer CUs,
// which is what concurrent pipelines need.
//
// SB (single buffer): one LDS chunk buffer instead of two, half the LDS (33 KB at
// Q = 63), so four workgroups fit a CU where two did. The evaluators compute chunk
// c + 1 into registers while the fold wave reads chunk c, wait for it to finish,
// store, and release it (two barriers per chunk instead of one). With three
// evaluator waves a workgroup is four waves, and four of them -- 16 waves, VGPRs
// for 4 per SIMD -- make 1024 tile slots: a B = 16 batch of ~1000-peak spectra
// (768 tiles) runs in one round instead of 1.5.
// (round 6, measured and removed: "twh", chunks of 32 peaks with an evaluator lane =
// (peak, half of its wave's points), 34 KB of LDS at Q = 60, four 7-wave workgroups per
// CU -- 1024 tile slots, so a B = 16 blood batch's 800 tiles in one round instead of
// two. Bit-exact, 69 VGPRs at occupancy 7, but slower: ten launches 405 against 366 us
// at B = 16, 295 against 263 at B = 8; PMC (profiles/r06_pmc_fit_b16_twh_rejected.json)
// waits 48% against 45%, VALU active 16% against 19%, LDS bank conflicts 8% against 1%:
// seven waves per SIMD leave the fold wave less issue, and the chunks' barriers double.)
template <int Q_, int PB, int PS, bool SB_ = false>
struct TwShape {
    static constexpr int Q = Q_;
    static constexpr bool SB = SB_;
    static constexpr int EW = PB * PS, J = 64 * PB, RS = J + kTfPad, QS = Q / PS;
    static constexpr int LDS = (SB ? 1 : 2) * Q * RS;
    static_assert(Q % 3 == 0 && Q / 3 <= 64 && Q <= 64 && Q % PS == 0, "tile shape");
};


template <bool FAST, class SH>
__device__ __forceinline__ void fit_tw_body(const Workspace& w, int s, int P, int it, double* T,
                                            int tile0, int tstep) {
    constexpr int QQ = SH::Q, EW = SH::EW, J = SH::J, RS = SH::RS, QS = SH::QS;
    constexpr int PB = J / 64;
    const size_t base = (size_t)s * w.capD;
    const int npts = 3 * P;
    const int tiles = (npts + QQ - 1) / QQ;
    const int nch = (P + J - 1) / J;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const double* __restrict__ params = params_version(w, base, it);
    const bool folder = wv == EW;
    if (folder) __builtin_amdgcn_s_setprio(3);
    // diagnostic builds (tools/ubench/fit_diag.hip): per-wave cycle sums -- evaluator
    // 0 eval, 1 barrier, 5 prologue loads; fold wave 2 fold, 3 barrier, 6 first wait,
    // 4 stencil update; slot 7 = the wave's start time
    DIAG_DECL
#ifdef MDG_DIAG
    _d_acc[7] = _d_t;
    // where the wave runs (fit_diag's placement analysis): HW_ID (wave / SIMD / CU / SE /
    // workgroup slot) and XCC_ID, one record per (block, wave) after the KSTAMP slots
    if (lane == 0 && g_diag) {
        const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
        const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((16 - 1) << 11));
        const size_t r = kDiagStampBase + 4096 + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 16 + wv;
        g_diag[r] = (long long)(((unsigned long long)xcc << 32) | hw) | (1ll << 62);
    }
#endif
    for (int tile = tile0; tile < tiles; tile += tstep) {
        const int p0 = tile * QQ;
        if (!folder) {
            const int pb = wv % PB, ps = wv / PB;
            // this wave's points: p0 + ps*QS .. +QS-1 (wave-uniform x; a tail tile
            // reads past 3P into the arena, and those points are never used)
            const const_f64_ptr rx = (const_f64_ptr)(w.rx + 3 * base + p0 + ps * QS);
            double xq[QS];
#pragma unroll
            for (int q = 0; q < QS; ++q) xq[q] = rx[q];
            const int jl = pb * 64 + lane;
            int j = min(jl, P - 1);
            double f = params[3 * j], h = params[3 * j + 1], m = params[3 * j + 2];
#ifdef MDG_DIAG
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::"v"(f), "v"(h), "v"(m), "s"(xq[0]));
            DIAG_STAMP(5);
#endif
            if constexpr (SH::SB) {
                // chunk c into registers while the fold wave reads chunk c - 1; then
                // A: it has finished, store; B: chunk c is in LDS
                double* Tb = T + ps * QS * RS + jl;
                for (int c = 0; c < nch; ++c) {
                    const double cf = f, ch = h, cm = m;
                    j = min((c + 1) * J + jl, P - 1);
                    f = params[3 * j];
                    h = params[3 * j + 1];
                    m = params[3 * j + 2];
                    double tv[QS];
#pragma unroll
                    for (int q = 0; q < QS; ++q) tv[q] = lorentz_t<FAST>(xq[q], cf, ch, cm);
                    DIAG_STAMP(0);
                    lds_barrier();  // A
                    DIAG_STAMP(1);
#pragma unroll
                    for (int q = 0; q < QS; ++q) Tb[q * RS] = tv[q];
                    lds_barrier();  // B
                    DIAG_STAMP(1);
                }
                lds_barrier();  // A: the fold wave has read the last chunk
                DIAG_STAMP(1);
            } else
            for (int c = 0; c <= nch; ++c) {
                if (c < nch) {
                    double* Tb = T + (c & 1) * QQ * RS + ps * QS * RS + jl;
                    const double cf = f, ch = h, cm = m;
                    // the next chunk's peak, in flight while this chunk is evaluated; the
                    // compiler copies it into f/h/m at the loop's back edge, so the copy
                    // waits for it there (the small-batch fit is bound by
                    // this load's latency, not by its FP64 issue)
                    j = min((c + 1) * J + jl, P - 1);
                    f = params[3 * j];
                    h = params[3 * j + 1];
                    m = params[3 * j + 2];
#pragma unroll
                    for (int q = 0; q < QS; ++q) Tb[q * RS] = lorentz_t<FAST>(xq[q], cf, ch, cm);
                }
                DIAG_STAMP(0);
                lds_barrier();
                DIAG_STAMP(1);
            }
        } else {
            double acc = -0.0;
            const int q = lane < QQ ? lane : QQ - 1;
            // the stencil update's operands, loaded before the fold so their latency
            // hides behind it (this tile's stencils are only written below, by this wave)
            const double yq = w.ry[3 * base + min(p0 + q, npts - 1)];
            const int kq = lane < QQ / 3 ? lane : 0;
            const int pkq = min(p0 / 3 + kq, P - 1);
            const Stencil sq0 = load_stencil(w, base, pkq);
            double one = 1.0;
            asm volatile("" : "+v"(one));
            if constexpr (!SH::SB) lds_barrier();  // chunk 0 written
            DIAG_STAMP(6);
            for (int c = 0; c < nch; ++c) {
                if constexpr (SH::SB) {
                    lds_barrier();  // A
                    lds_barrier();  // B: chunk c written
                    DIAG_STAMP(3);
                }
                const double2* row = (const double2*)(T + (SH::SB ? 0 : (c & 1) * QQ * RS) + q * RS);
                const int cn = min(J, P - c * J);
                if (cn == J) {
                    // (round 5: a software-pipelined asm form, eight 16-byte reads kept in
                    // flight, was slower than this schedule -- ten tf12 launches 113 against
                    // 95 us at B = 1, twf1 385 against 370 at B = 16)
#pragma unroll 16
                    for (int k = 0; k < J / 2; ++k) {
                        const double2 v = row[k];
                        acc = __builtin_fma(v.x, one, acc);
                        acc = __builtin_fma(v.y, one, acc);
                    }
                } else {
                    const double* r1 = (const double*)row;
                    for (int k = 0; k < cn; ++k) acc = __builtin_fma(r1[k], one, acc);
                }
                DIAG_STAMP(2);
                if constexpr (!SH::SB) {
                    lds_barrier();
                    DIAG_STAMP(3);
                }
            }
            if constexpr (SH::SB) {
                lds_barrier();  // A: the evaluators may refill the buffer
                DIAG_STAMP(3);
            }
            // stencil update of the tile's peaks: lane k gathers the ratios y/sup of
            // its peak's three points from lanes 3k..3k+2
            const double ratio = yq / acc;
            const int k = kq;
            const double r0 = __shfl(ratio, 3 * k, 64);
            const double r1 = __shfl(ratio, 3 * k + 1, 64);
            const double r2 = __shfl(ratio, 3 * k + 2, 64);
            const int pk = p0 / 3 + lane;
            if (lane < QQ / 3 && pk < P) {
                Stencil sq = sq0;
                sq.y1 = sq.y1 * r0;
                sq.y2 = sq.y2 * r1;
                sq.y3 = sq.y3 * r2;
                mirror_shoulder(sq);
                store_updated_stencil(w, base, pk, sq, sq0.x1, sq0.x3);
                double* L = (((it + 1) & 1) ? w.params_alt : w.params) + 3 * base + 3 * (size_t)pk;
                solve(sq, L);
                if (!peak_fast_ok(L[0], L[1], L[2])) atomicAdd(&w.unsafe[4 * s + (it + 1) % 3], 1);
            }
            DIAG_STAMP(4);
        }
    }
    DIAG_FLUSH();
}

template <class SH>
__global__ __launch_bounds__(64 * (SH::EW + 1)) void k_fit_sup_tw(BatchArgs a, Workspace w, int it) {
    __shared__ __attribute__((aligned(16))) double T[SH::LDS];
    const int s = blockIdx.y;
    const FitHead h = fit_head(w, s, it);
    if (!h.live) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        w.unsafe[4 * s + (it + 2) % 3] = 0;
        if (!h.fast) mark_slow(w, s, slow_bit(it));
    }
    if (h.fast) fit_tw_body<true, SH>(w, s, h.P, it, T, blockIdx.x, gridDim.x);
    else fit_tw_body<false, SH>(w, s, h.P, it, T, blockIdx.x, gridDim.x);
}

#ifdef MDG_DIAG
// EXPERIMENT, diagnostic builds only (make diag; BASELINE configs[2], "superposition
// recast as MFMA outer product"): the fit superposition with every
// denominator hw2 + (x - maxp)^2 taken from v_mfma_f64_16x16x4_f64 as the product
// [x'^2, x', 1, 0] . [1, -2m', m'^2 + hw2, 0] with x' = x - c, m' = maxp - c centred
// on the tile's first point (to keep the cancellation near a peak small). A wave
// owns 16 points (A rows) and walks the peaks 16 at a time (B columns); lane l then
// holds the denominators of peak 16t + (l & 15) at points (l >> 4) + 4r, r = 0..3,
// divides sfhw by them (div_rn under the fast flags) and accumulates per lane; the
// 16 lanes of a row then add their partial sums. NOT bit-identical (the
// denominators round differently and the sum is reordered), so never in the
// product library: MDG_FITSUP=mfma selects it in the diagnostic build, and
// tools/mfma_experiment.py measures it against the exact kernel and the oracle
// (round 2: 1.87 against 1.395 ms per launch at B = 256, 3.7e-4 relative deviation
// of the fitted parameters).
template <bool FAST>
__device__ __forceinline__ void fit_mfma_tile(const Workspace& w, size_t base, int P, int p0, int npts,
                                              const double* __restrict__ params) {
    typedef double v4d __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x & 63;
    const int col = lane & 15, kk = lane >> 4;
    const double* rx = w.rx + 3 * base;
    const double c = rx[min(p0, npts - 1)];
    const double xa = rx[min(p0 + col, npts - 1)] - c;  // A: row = point p0 + col
    const double av = kk == 0 ? xa * xa : kk == 1 ? xa : kk == 2 ? 1.0 : 0.0;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j0 = 0; j0 < P; j0 += 16) {
        const int j = min(j0 + col, P - 1);
        const double f = params[3 * j], h = params[3 * j + 1], m = params[3 * j + 2] - c;
        const double bv = kk == 0 ? 1.0 : kk == 1 ? -2.0 * m : kk == 2 ? m * m + h : 0.0;
        v4d d = {0.0, 0.0, 0.0, 0.0};
        d = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, d, 0, 0, 0);
        if (j0 + col < P) {
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] += FAST ? div_rn(f, d[r]) : f / d[r];
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) acc[r] += __shfl_xor(acc[r], o, 16);
    }
    if (col == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = p0 + kk + 4 * r;
            if (i < npts) w.ratio[3 * base + i] = w.ry[3 * base + i] / acc[r];  // fitter_analytical.rs:42-47
        }
    }
}

__global__ __launch_bounds__(256) void k_fit_sup_mfma(BatchArgs a, Workspace w, int it) {
    const int s = blockIdx.x % a.B, part = blockIdx.x / a.B, parts = gridDim.x / a.B;
    if (w.status[s] || fit_done(w, s, it)) return;
    const int P = w.sel_count[s];
    const size_t base = (size_t)s * w.capD;
    const double* __restrict__ params = w.params + 3 * base;
    if (part == 0 && threadIdx.x == 0) w.unsafe[4 * s + ((it + 1) & 1)] = 0;
    const bool fast = w.x_ok[s] && w.unsafe[4 * s + (it & 1)] == 0;
    const int npts = 3 * P, wv = threadIdx.x >> 6;
    for (int p0 = (part * 4 + wv) * 16; p0 < npts; p0 += parts * 64) {
        if (fast) fit_mfma_tile<true>(w, base, P, p0, npts, params);
        else fit_mfma_tile<false>(w, base, P, p0, npts, params);
    }
}
#endif

// K6i  the same term-fold tiles over ONE batch-wide list ("twf"): the tiles of all
// spectra, spectrum after spectrum, grid-strided over a 1-D grid of about one
// workgroup per slot of the chip. A (G, B) grid with a fixed G per spectrum leaves
// a tail whenever the batch's tiles are not a multiple of the slots (B = 16 at
// P = 992: 768 tiles of 63 points on 512 slots, 1.5 rounds); one list spreads them
// evenly whatever B and the spectra's peak counts. Each workgroup reads the
// batch's per-spectrum state once (B <= kTwfMaxB, one lane per spectrum) into LDS.
constexpr int kTwfMaxB = 64;
template <class SH>
__global__ __launch_bounds__(64 * (SH::EW + 1)) void k_fit_sup_twf(BatchArgs a, Workspace w, int it) {
    __shared__ __attribute__((aligned(16))) double T[SH::LDS];
    __shared__ int first[kTwfMaxB + 1];  // first list item of spectrum s; first[B] = items
    __shared__ int pk[kTwfMaxB];         // peaks of spectrum s
    __shared__ int fastf[kTwfMaxB];
    constexpr int QQ = SH::Q;
    if (threadIdx.x < 64) {
        const int s = threadIdx.x;
        int tiles = 0, P = 0, fast = 0;
        if (s < a.B) {
            const FitHead h = fit_head(w, s, it);
            if (h.live) {
                P = h.P;
                tiles = (3 * P + QQ - 1) / QQ;
                fast = h.fast;
                if (blockIdx.x == 0) {
                    w.unsafe[4 * s + (it + 2) % 3] = 0;
                    if (!h.fast) mark_slow(w, s, slow_bit(it));
                }
            }
        }
        int x = tiles;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (s >= o) x += y;
        }
        first[s + 1] = x;
        if (s == 0) first[0] = 0;
        pk[s] = P;
        fastf[s] = fast;
    }
    __syncthreads();
    const int items = first[a.B];
    int s = 0;
    for (int item = blockIdx.x; item < items; item += gridDim.x) {
        while (first[s + 1] <= item) ++s;  // items ascend: the search resumes
        // LDS values are uniform here, but the compiler cannot know it: readfirstlane
        // puts the spectrum, its tile and its peak count in SGPRs, so the body's
        // addresses and x values are scalar (as under k_fit_sup_tw's blockIdx.y) and
        // the FAST branch is a scalar branch
        s = __builtin_amdgcn_readfirstlane(s);
        const int tile = __builtin_amdgcn_readfirstlane(item - first[s]);
        const int P = __builtin_amdgcn_readfirstlane(pk[s]);
        if (__builtin_amdgcn_readfirstlane(fastf[s])) fit_tw_body<true, SH>(w, s, P, it, T, tile, 1 << 20);
        else fit_tw_body<false, SH>(w, s, P, it, T, tile, 1 << 20);
    }
}

// 1-D grid, spectrum = block % B (as k_mse_partial): round-robin dispatch puts the
// workgroups a CU holds at once on the same spectrum, so they share its Lorentzians
// in the scalar cache instead of each streaming another spectrum's table
__global__ void k_fit_sup(BatchArgs a, Workspace w, int it) {
    const int s = blockIdx.x % a.B, part = blockIdx.x / a.B, parts = gridDim.x / a.B;
    if (w.status[s] || fit_done(w, s, it)) return;
    const int P = w.sel_count[s];
    const size_t base = (size_t)s * w.capD;
    const double* __restrict__ params = w.params + 3 * base;
    const bool fast = w.x_ok[s] && w.unsafe[4 * s + (it & 1)] == 0;
    if (part == 0 && threadIdx.x == 0) {
        w.unsafe[4 * s + ((it + 1) & 1)] = 0;
        if (!fast) mark_slow(w, s, slow_bit(it));
    }
    for (int i = part * blockDim.x + threadIdx.x; i < 3 * P; i += parts * blockDim.x) {
        const double sup = superpose(w.rx[3 * base + i], params, P, fast);
        w.ratio[3 * base + i] = w.ry[3 * base + i] / sup;
    }
}

// K7  stencil update + re-solve (fitter_analytical.rs:48-65)
__global__ void k_fit_update(BatchArgs a, Workspace w, int it) {
    const int s = blockIdx.y;
    if (w.status[s] || fit_done(w, s, it)) return;
    const int P = w.sel_count[s];
    const size_t base = (size_t)s * w.capD;
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
        const double* ra = w.ratio + 3 * base + 3 * (size_t)p;
        const Stencil q0 = load_stencil(w, base, p);
        Stencil q = q0;
        q.y1 = q.y1 * ra[0];
        q.y2 = q.y2 * ra[1];
        q.y3 = q.y3 * ra[2];
        mirror_shoulder(q);
        store_updated_stencil(w, base, p, q, q0.x1, q0.x3);
        double* L = w.params + 3 * base + 3 * (size_t)p;
        solve(q, L);
        if (!peak_fast_ok(L[0], L[1], L[2])) atomicAdd(&w.unsafe[4 * s + ((it + 1) & 1)], 1);
    }
}

// K6s  the whole fit of a small spectrum in ONE workgroup ("small": N <= kSmallN, one
// workgroup per spectrum, all iterations in one launch). Each iteration: the
// superposition at the 3P reduced points, one thread per point, the reference's left
// fold over the peaks in their order (lorentzian.rs:606-611: the same adds as every
// fit kernel, so the same bits); the ratios y/sup (fitter_analytical.rs:40-47); the
// stencil update, mirror and re-solve of each peak (:48-65) -- with __syncthreads
// between the phases instead of kernel boundaries. Measured before it (sim_01, 2048
// points, 26 peaks; the reference's own benchmark case): ten k_fit_sup_tf<12>
// launches of 4.6 us each whose work is a few hundred cycles. Parameters, stencils and
// ratios stay in LDS for P <= kSmallP; a larger P (a small spectrum with that many
// selected peaks is pathological) runs the same loops over the global rows (params /
// params_alt versions, the stencil rows in place, the kept rows as ratio scratch):
// bit-identical, but one CU does all of it. Range flags per iteration from the version
// the iteration reads (every parameter through peak_fast_ok, and x_ok), as the tile
// kernels count them; slow iterations recorded by mark_slow. The retain and the MSE
// stay with k_mse_local (many workgroups): an exact-order MSE inside this one
// workgroup (38k evaluations and a 1468-term windowed fold for sim_01) measured 41
// against 23 + 11 us for the fit here and k_mse_local after it (round 6).
// Superposition per iteration: with 3 P^2 <= kSmallT terms (P <= 45: the sim spectra)
// every (point, peak) term is evaluated by its own thread into LDS and each point's
// thread then folds its row in peak order; otherwise each point's thread evaluates and
// folds its P terms itself (fold_small).
constexpr int kSmallP = 512, kSmallBS = 512, kSmallT = 6144;

// acc + sum_j<P sfhw_j / (hw2_j + (x - maxp_j)^2), a left fold in j order (the adds
// stay in order: the reference's bits); eight Lorentzians' parameters are read (LDS
// broadcasts, or wave-uniform global loads) and their eight divisions issued together
// before the eight adds. Folding term by term, each division waited on its own loads
// and latency chain: ~230 cycles per term (k_fit_small's phase stamps, round 6).
template <bool FAST>
__device__ __forceinline__ double fold_small(double x, const double* prm, int P, double acc = -0.0) {
    int j = 0;
    for (; j + 8 <= P; j += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            t[u] = lorentz_t<FAST>(x, prm[3 * (j + u)], prm[3 * (j + u) + 1], prm[3 * (j + u) + 2]);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += t[u];
    }
    for (; j < P; ++j) acc += lorentz_t<FAST>(x, prm[3 * j], prm[3 * j + 1], prm[3 * j + 2]);
    return acc;
}

template <int BS, class PT, class ST, class RT>
__device__ __forceinline__ void fit_small_body(const Workspace& w, int s, int P, int iters, int xok,
                                               PT prm_in, PT prm_out, ST stn, RT rat, bool lds,
                                               size_t ps) {  // ps: stencil y plane - x plane (doubles)
    const size_t base = (size_t)s * w.capD;
    const double* __restrict__ rx = w.rx + 3 * base;
    const double* __restrict__ ry = w.ry + 3 * base;
    const int tid = threadIdx.x, npts = 3 * P;
    KSTAMP(71);
    for (int it = 0; it < iters; ++it) {
        // LDS: one parameter row updated in place; global: versions it (read) and it + 1
        PT prm = lds ? prm_in : (PT)params_version(w, base, it);
        PT nxt = lds ? prm_in : (PT)params_version(w, base, it + 1);
        int bad = 0;
        for (int p = tid; p < P; p += BS) bad |= !peak_fast_ok(prm[3 * p], prm[3 * p + 1], prm[3 * p + 2]);
        const bool fast = xok && !__syncthreads_or(bad);
        if (!fast && tid == 0) mark_slow(w, s, slow_bit(it));
        for (int i = tid; i < npts; i += BS) {
            const double x = rx[i];
            const double acc = fast ? fold_small<true>(x, prm, P) : fold_small<false>(x, prm, P);
            rat[i] = ry[i] / acc;
        }
        __syncthreads();
        if (it == 0) KSTAMP(72);
        for (int p = tid; p < P; p += BS) {
            Stencil q{stn[3 * p], stn[3 * p + 1], stn[3 * p + 2], stn[ps + 3 * p], stn[ps + 3 * p + 1],
                      stn[ps + 3 * p + 2]};
            q.y1 = q.y1 * rat[3 * p];
            q.y2 = q.y2 * rat[3 * p + 1];
            q.y3 = q.y3 * rat[3 * p + 2];
            mirror_shoulder(q);
            stn[3 * p] = q.x1; stn[3 * p + 1] = q.x2; stn[3 * p + 2] = q.x3;
            stn[ps + 3 * p] = q.y1; stn[ps + 3 * p + 1] = q.y2; stn[ps + 3 * p + 2] = q.y3;
            double L[3];
            solve(q, L);
            nxt[3 * p] = L[0]; nxt[3 * p + 1] = L[1]; nxt[3 * p + 2] = L[2];
        }
        __syncthreads();
        if (it == 0) KSTAMP(73);
    }
    KSTAMP(74);
}

// k_fit_small for 3 P^2 <= kSmallT (P <= 45): the iteration's 3 P^2 terms are spread
// over the workgroup, kSmallT / BS per thread, every (point, peak) assignment and its x
// fixed in registers before the first iteration, all their LDS parameter reads issued
// together; each point's thread then folds its row of T in peak order (eight reads
// ahead of the adds), divides its y by the sum, and the peaks' threads update the
// stencils and re-solve; the range check of the new parameters rides on that update's
// barrier. The same operations as every fit kernel, so the same bits.
template <int BS>
__device__ __forceinline__ void fit_small_terms(const Workspace& w, int s, int P, int iters, int xok,
                                                double* prm, double* stn, double* rat, double* T) {
    constexpr int U = kSmallT / BS;
    constexpr int ps = 3 * kSmallP;  // the LDS stencil planes
    const size_t base = (size_t)s * w.capD;
    const int tid = threadIdx.x, npts = 3 * P, nt = npts * P;
    const int nu = __builtin_amdgcn_readfirstlane((nt + BS - 1) / BS);  // term slots in use
    const int RS = P | 1;  // row stride of T (odd: fewer bank conflicts in the folds)
    // term e = tid + u * BS is (point i, peak j) = (e % npts, e / npts): the lanes of a
    // wave share a peak, so its three parameters are LDS broadcasts (one address per
    // wave, not 64: the point-major order cost sim_01's terms ~1.9k cycles an iteration)
    double xu[U];
    int ju[U], eu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = tid + u * BS;
        const bool ok = e < nt;
        const int j = ok ? e / npts : 0, i = ok ? e - j * npts : 0;
        xu[u] = w.rx[3 * base + i];
        ju[u] = j;
        eu[u] = ok ? i * RS + j : -1;
    }
    const double yq = tid < npts ? w.ry[3 * base + tid] : 1.0;
    __shared__ int badf[2];
    int bad = 0;
    for (int p = tid; p < P; p += BS) bad |= !peak_fast_ok(prm[3 * p], prm[3 * p + 1], prm[3 * p + 2]);
    bool fast = xok && !__syncthreads_or(bad);
    if (tid == 0) badf[0] = 0;  // iteration 0's flags (read after its update's barrier)
    KSTAMP(71);
    for (int it = 0; it < iters; ++it) {
        if (!fast && tid == 0) mark_slow(w, s, slow_bit(it));
        // only the nu slots that hold terms (wave-uniform; sim_01: 4 of 12) -- evaluating
        // all twelve tripled the iteration's division work
        double t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = 0.0;
        if (fast) {  // (one uniform branch around the loop: per term, both forms were computed)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (u < nu) t[u] = lorentz_t<true>(xu[u], prm[3 * ju[u]], prm[3 * ju[u] + 1], prm[3 * ju[u] + 2]);
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (u < nu) t[u] = lorentz_t<false>(xu[u], prm[3 * ju[u]], prm[3 * ju[u] + 1], prm[3 * ju[u] + 2]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < nu && eu[u] >= 0) T[eu[u]] = t[u];
        if (it == 1) KSTAMP(76);
        lds_barrier();
        if (it == 1) KSTAMP(77);
        if (tid < npts) {
            const double* row = T + tid * RS;
            double acc = -0.0;
            int k = 0;
            for (; k + 8 <= P; k += 8) {
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = row[k + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += v[u];
            }
            for (; k < P; ++k) acc += row[k];
            rat[tid] = yq / acc;
        }
        if (it == 1) KSTAMP(78);
        lds_barrier();
        if (it == 0) KSTAMP(72);
        if (it == 1) KSTAMP(79);
        bad = 0;
        if (tid < P) {
            const int p = tid;
            Stencil q{stn[3 * p], stn[3 * p + 1], stn[3 * p + 2], stn[ps + 3 * p], stn[ps + 3 * p + 1],
                      stn[ps + 3 * p + 2]};
            q.y1 = q.y1 * rat[3 * p];
            q.y2 = q.y2 * rat[3 * p + 1];
            q.y3 = q.y3 * rat[3 * p + 2];
            mirror_shoulder(q);
            stn[3 * p] = q.x1; stn[3 * p + 1] = q.x2; stn[3 * p + 2] = q.x3;
            stn[ps + 3 * p] = q.y1; stn[ps + 3 * p + 1] = q.y2; stn[ps + 3 * p + 2] = q.y3;
            double L[3];
            solve(q, L);
            prm[3 * p] = L[0]; prm[3 * p + 1] = L[1]; prm[3 * p + 2] = L[2];
            bad = !peak_fast_ok(L[0], L[1], L[2]);
        }
        // the range check's reduction: the flags of iteration parity it & 1 set by the
        // peaks out of range, the other parity's cleared for the next iteration (its
        // last readers passed two barriers ago), one barrier -- __syncthreads_or here
        // cost ~1.3k cycles an iteration (its own barriers and LDS reduction; phase
        // stamps, sim_01)
        if (bad) badf[it & 1] = 1;
        if (tid == 0) badf[(it + 1) & 1] = 0;
        if (it == 1) KSTAMP(86);
        lds_barrier();
        fast = xok && !badf[it & 1];
        if (it == 0) KSTAMP(73);
        if (it == 1) KSTAMP(87);
    }
    KSTAMP(74);
}

// K8  retain sfhw > CHECK_PRECISION && hw2 > CHECK_PRECISION, order preserving
// (fitter_analytical.rs:67-69); copies min(count, cap) rows to the caller's output.
// the fitted parameters of spectrum s: k_fit_sup_tf / _tw leave version
// min(iterations) in the buffer of its parity; the k_fit_update path updates in place
__device__ __forceinline__ const double* final_params(const Workspace& w, int s, size_t base) {
    const int ver = w.params_alt ? (w.fit_iters_s ? min(w.fit_iters_s[s], w.fit_iters) : w.fit_iters) : 0;
    return params_version(w, base, ver);
}

// retain predicate (fitter_analytical.rs:67-69)
__device__ __forceinline__ bool retained(double sfhw, double hw2) {
    return sfhw > kCheckPrecision && hw2 > kCheckPrecision;
}

template <int BS>
__device__ __forceinline__ void retain_body(const BatchArgs& a, const Workspace& w, int s, int* lds_i);

template <int BS>
__global__ __launch_bounds__(BS) void k_retain(BatchArgs a, Workspace w) {
    const int s = blockIdx.x;
    __shared__ int lds_i[BS / 64 + 1];
    if (w.status[s]) {
        if (threadIdx.x == 0) {
            a.out_count[s] = 0;
            a.out_mse[s] = 0.0;
            a.out_status[s] = w.status[s];
        }
        return;
    }
    retain_body<BS>(a, w, s, lds_i);
}

// row o of spectrum s's result table: page-locked host rows first (out_host_rows
// of them, host-buffer calls), the caller's device rows after them, none past cap
__device__ __forceinline__ void put_row(const BatchArgs& a, int s, int o, double f, double h, double m) {
    double* q = o < a.out_host_rows ? a.out_host + 3 * ((size_t)s * a.out_host_rows + o)
              : o < a.cap           ? a.out + 3 * ((size_t)s * a.cap + o)
                                    : nullptr;
    if (q) {
        q[0] = f;
        q[1] = h;
        q[2] = m;
    }
}

// ordered compaction of the retained Lorentzians into kept and the caller's rows
// (k_retain; k_mse_local's first workgroup of each spectrum)
template <int BS>
__device__ __forceinline__ void retain_body(const BatchArgs& a, const Workspace& w, int s, int* lds_i) {
    const int P = w.sel_count[s];
    const size_t base = (size_t)s * w.capD;
    const double* params = final_params(w, s, base);
    const int per = (P + BS - 1) / BS;
    const int p0 = threadIdx.x * per, p1 = min(P, p0 + per);
    double* kept = w.kept + 3 * base;
    // up to R parameters per thread stay in registers (one load round): 4096
    // Lorentzians at 1024 threads, 2048 at 256
    constexpr int R = BS >= 1024 ? 4 : 8;
    if (per <= R) {
        double v[R][3];
        int keep = 0;
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const int p = min(p0 + u, P - 1);
            v[u][0] = params[3 * p];
            v[u][1] = params[3 * p + 1];
            v[u][2] = params[3 * p + 2];
        }
#pragma unroll
        for (int u = 0; u < R; ++u)
            keep += p0 + u < p1 && v[u][0] > kCheckPrecision && v[u][1] > kCheckPrecision;
        int total;
        int o = block_exclusive_scan<BS>(keep, lds_i, &total);
        int unsafe = 0;
#pragma unroll
        for (int u = 0; u < R; ++u) {
            if (p0 + u < p1 && v[u][0] > kCheckPrecision && v[u][1] > kCheckPrecision) {
                kept[3 * o] = v[u][0];
                kept[3 * o + 1] = v[u][1];
                kept[3 * o + 2] = v[u][2];
                unsafe += !peak_fast_ok(v[u][0], v[u][1], v[u][2]);
                put_row(a, s, o, v[u][0], v[u][1], v[u][2]);
                ++o;
            }
        }
        if (unsafe) atomicAdd(&w.unsafe_kept[s], unsafe);
        if (threadIdx.x == 0) {
            w.kept_count[s] = total;
            a.out_count[s] = total;
        }
        return;
    }
    int keep = 0;
    for (int p = p0; p < p1; ++p)
        keep += (params[3 * p] > kCheckPrecision && params[3 * p + 1] > kCheckPrecision);
    int total;
    int o = block_exclusive_scan<BS>(keep, lds_i, &total);
    for (int p = p0; p < p1; ++p) {
        if (params[3 * p] > kCheckPrecision && params[3 * p + 1] > kCheckPrecision) {
            kept[3 * o] = params[3 * p];
            kept[3 * o + 1] = params[3 * p + 1];
            kept[3 * o + 2] = params[3 * p + 2];
            if (!peak_fast_ok(params[3 * p], params[3 * p + 1], params[3 * p + 2]))
                atomicAdd(&w.unsafe_kept[s], 1);
            put_row(a, s, o, params[3 * p], params[3 * p + 1], params[3 * p + 2]);
            ++o;
        }
    }
    if (threadIdx.x == 0) {
        w.kept_count[s] = total;
        a.out_count[s] = total;
    }
}

// ----------------------------------------------------------------------------------
// K9  superposition over the MSE regions + squared residual, fixed-order tree
// (deconvoluter.rs:540-543, compute_mse :828-862). Regions are walked as one
// virtual concatenation so overlapping regions count twice, like the reference.
// ----------------------------------------------------------------------------------
__device__ __forceinline__ void mse_region(const Workspace& w, int s, int r, int nig, int64_t* lo,
                                           int64_t* hi) {
    const int64_t* pairs = w.ig + (size_t)s * 2 * w.ig_cap;
    *lo = r == 0 ? w.sbi[2 * s] : pairs[2 * (r - 1) + 1];
    *hi = r == nig ? w.sbi[2 * s + 1] : pairs[2 * r];
}

// Point of virtual index v (0 <= v < mse_len) of the concatenated MSE regions:
// the first region whose cumulative end exceeds v (empty regions are skipped).
// A walk for a few regions, a binary search over prep's cumulative lengths for many.
__device__ __forceinline__ int64_t mse_index(const Workspace& w, int s, int nig, int64_t v) {
    if (nig <= 8) {
        int64_t rem = v;
        for (int r = 0; r <= nig; ++r) {
            int64_t lo, hi;
            mse_region(w, s, r, nig, &lo, &hi);
            if (rem < hi - lo) return lo + rem;
            rem -= hi - lo;
        }
        return 0;
    }
    const int64_t* cum = w.ig_cum + (size_t)s * (w.ig_cap + 2);
    int lo = 0, hi = nig;  // the largest r with cum[r] <= v
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (cum[mid] <= v) lo = mid;
        else hi = mid - 1;
    }
    int64_t rlo, rhi;
    mse_region(w, s, lo, nig, &rlo, &rhi);
    return rlo + (v - cum[lo]);
}

// points in the MSE regions of spectrum s (their total length)
__device__ __forceinline__ int64_t mse_len(const Workspace& w, int s) {
    return w.ig_cum[(size_t)s * (w.ig_cap + 2) + w.n_ig[s] + 1];  // prep_spectrum
}

template <int BS>
__device__ __forceinline__ void mse_publish_fold(const BatchArgs& a, const Workspace& w, int s, int part,
                                                 int nparts, double acc, int kept_n, double* parts);
__device__ __forceinline__ void mse_panic_out(const BatchArgs& a, int s);

// ----------------------------------------------------------------------------------
// MSE superposition with one division per four Lorentzians (k_mse_quad).
// compute_mse (deconvoluter.rs:828-862) only needs the MSE within the tests'
// 1e-12 relative tolerance: the summation order inside a point's superposition is
// free there, and so is the rounding of each term. The retained Lorentzians have
// sfhw > 0 and hw2 > 0 (fitter_analytical.rs:67-69), so every term is positive and
// four of them combine without cancellation:
//   f0/b0 + f1/b1 = (f0 b1 + f1 b0) / (b0 b1),   b = hw2 + (x - maxp)^2 (one fma),
// two such pairs again into N/D, then one reciprocal with one Newton step and one
// residual correction. About seven issue slots per term against thirteen for a
// term with its own division; the relative error of a quad stays within ~8 ulp.
// Ranges: under the FAST flags (peak_fast_ok, x_ok) b lies in [2^-200, 2^203), so
// D (four b) in [2^-800, 2^812) and every product stays normal and finite; spectra
// outside them take the IEEE '/' per term.
// A workgroup's four waves share its 64 * NPT points and split the Lorentzians into
// four contiguous ranges (more waves per SIMD to hide the scalar loads at small B);
// the partial sums meet in LDS, then the residuals, the tree and the last-workgroup
// fold of k_mse_partial_n.
// ----------------------------------------------------------------------------------
__device__ __forceinline__ double quad_term(double x, const double (&c)[12]) {
    const double d0 = x - c[2], d1 = x - c[5], d2 = x - c[8], d3 = x - c[11];
    const double b0 = __builtin_fma(d0, d0, c[1]);
    const double b1 = __builtin_fma(d1, d1, c[4]);
    const double b2 = __builtin_fma(d2, d2, c[7]);
    const double b3 = __builtin_fma(d3, d3, c[10]);
    const double n01 = __builtin_fma(c[3], b0, c[0] * b1);
    const double n23 = __builtin_fma(c[9], b2, c[6] * b3);
    const double d01 = b0 * b1, d23 = b2 * b3;
    const double N = __builtin_fma(n01, d23, n23 * d01);
    const double D = d01 * d23;
    const double r0 = __builtin_amdgcn_rcp(D);
    const double r1 = __builtin_fma(r0, __builtin_fma(-D, r0, 1.0), r0);
    const double q0 = N * r1;
    return __builtin_fma(__builtin_fma(-D, q0, N), r1, q0);
}

// Thread 0's acc is this workgroup's partial of spectrum s: publish it, count the
// arrival, and let the last workgroup of the spectrum fold the nparts partials left
// to right from +0.0 (fixed order: deterministic) into out_mse / out_status.
template <int BS>
__device__ __forceinline__ void mse_publish_fold(const BatchArgs& a, const Workspace& w, int s, int part,
                                                 int nparts, double acc, int kept_n, double* parts) {
    __shared__ int last;
    if (threadIdx.x == 0) {
        __hip_atomic_store(w.mse_part + (size_t)s * nparts + part, acc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int done = __hip_atomic_fetch_add(w.mse_done + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = done == nparts - 1;
        if (last) __hip_atomic_store(w.mse_done + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    for (int k = threadIdx.x; k < nparts; k += BS) parts[k] = ld_sc1(w.mse_part + (size_t)s * nparts + k);
    __syncthreads();
    if (threadIdx.x < 64) {
        const int sub = threadIdx.x & 15;
        const double one = 1.0;
        double t = 0.0;
        const int G = nparts / 16;
        for (int g = 0; g < G; ++g) fold16(t, parts[16 * g + sub], one);
        const int r = nparts - 16 * G;
        if (r > 0) {
            const double v = parts[min(16 * G + sub, nparts - 1)];
            for (int k = 0; k < r; ++k) t += readlane_f64(v, k);
        }
        if (threadIdx.x == 0) {
            a.out_mse[s] = t / (double)mse_len(w, s);
            a.out_status[s] = (kept_n > a.cap) ? MDG_CAPACITY : MDG_OK;
        }
    }
}

// ----------------------------------------------------------------------------------
// K9d  MSE superposition by local expansions (default MSE kernel).
// compute_mse (deconvoluter.rs:828-862) needs sup(x) = sum_j sfhw_j / (hw2_j +
// (x - maxp_j)^2) at every signal-region point. With s_j = sqrt(hw2_j) and the
// complex pole z_j = maxp_j + i s_j, each term is Im[a_j / (x - z_j)] with
// a_j = sfhw_j / s_j. A tile of 256 consecutive points (centre t, half range r)
// splits the Lorentzians into
//   - near ones, |z_j - t| <= R r: summed directly per point (quad_term);
//   - far ones: their sum is a power series in u = (x - t) / r,
//       sum_j a_j / (x - z_j) = -sum_k [sum_j a_j w_j (r w_j)^k] u^k,  w_j = 1 / (z_j - t),
//     |u| <= 1 and |r w_j| < 1 / R, so PK terms leave ~R^-PK of each far term
//     (R = 3 with 30 terms, or R = 5 with 20); only the imaginary parts are needed
//     (u is real).
// Per point that is PK Horner steps plus a few % of the Lorentzians directly, and
// per tile one pass over the Lorentzians (~3 instructions per term and power)
// instead of 256 x P divisions. The radius trades the two: the near terms cost ~25
// issue slots per four per point, the far ones ~3 per power per tile, so at
// throughput (large batches) a smaller radius with more powers wins while the near
// list dominates; a small batch waits on a tile's latency instead, which the longer
// far-field recurrence adds to. Round 5, MSE us per spectrum in the queue (256 x 2):
// R = 5 / 20 powers 3.52-3.57, R = 4 / 30 3.48, R = 3 / 30 3.07-3.12, R = 2.5 / 40
// 3.76-3.82 (204 VGPRs, occupancy 2); blood, us per launch: B = 16 53.4 against 56.8,
// B = 1 17.2 either way. So PK = 30 (MDG_MSE_PK=20 selects the round-4 form). The
// <4, 30> form needs 168 VGPRs, the most that keeps 3 waves per SIMD: at 188 (an asm
// use-point on its head loads) it ran 3.7 us per spectrum. Measured against a
// long-double direct sum
// (tools/mse_local_error.py): the MSE within a few 1e-15 relative on the
// synthetic and blood spectra, the order of the direct f64 sum's own error; against
// the oracle 1.34e-14 at most for either order (tools/mse_error.py); the
// tests hold it to MSE_RTOL = 1e-12 like every MSE kernel. Every reduction has a
// fixed order, so results are deterministic. Spectra outside the fast ranges
// (x_ok, unsafe_kept) and tiles with more near Lorentzians than the list holds
// (kLocNear) sum every term directly.
// ----------------------------------------------------------------------------------
template <int PK>
constexpr double loc_radius() { return PK >= 30 ? 3.0 : 5.0; }  // far: |z - t| > R * r
constexpr int kLocNear = 512;     // near Lorentzians kept per tile (LDS)
constexpr int kLocTP = 256;       // points per tile (one per thread)

__device__ __forceinline__ double rcp_nr2(double d) {
    const double r0 = __builtin_amdgcn_rcp(d);
    const double r1 = __builtin_fma(r0, __builtin_fma(-d, r0, 1.0), r0);
    return __builtin_fma(r1, __builtin_fma(-d, r1, 1.0), r1);
}

// sum over the retained Lorentzians among params[0, P) at x, every term
// (wave-uniform parameters: scalar loads); FAST: div_rn_1nr, else '/'
template <bool FAST>
__device__ __forceinline__ double sup_retained_direct(double x, const_f64_ptr prm, int P) {
    double acc = 0.0;
    for (int j = 0; j < P; ++j) {
        const double f = prm[3 * j], h = prm[3 * j + 1], m = prm[3 * j + 2];
        if (retained(f, h)) acc += lorentz_mse<FAST>(x, f, h, m);
    }
    return acc;
}

// NPT points per thread: a tile of kLocTP * NPT points shares one coefficient pass
template <int NPT, int PK>
__global__ __launch_bounds__(256) void k_mse_local(BatchArgs a, Workspace w, int nparts, int near_cap) {
    constexpr int BS = 256, NW = BS / 64, TP = kLocTP * NPT, PH = 10, NH = PK / PH;
    constexpr double kLocR = loc_radius<PK>();
    static_assert(kLocTP == BS && PK % PH == 0 && PH * 16 <= BS, "tile shape");
    const int s = blockIdx.x % a.B, part = blockIdx.x / a.B;
    // LDS: the coefficient reduction (PH x BS) and, after the tile loop, the
    // partials of the final fold share one buffer
    constexpr int RED = PH * BS > kMseMaxParts ? PH * BS : kMseMaxParts;
    __shared__ double red[RED];
    __shared__ double coef[PK];
    __shared__ double nearp[3 * kLocNear];
    __shared__ double wmin[NW], wmax[NW], wacc[NW];
    __shared__ int wcnt[NW];
    __shared__ int lds_i[NW + 1];
    const int tid = threadIdx.x, wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    // the spectrum's scalars, loaded together (one memory round trip; behind the
    // branches below they were a chain of dependent loads, as in fit_head)
    const int st = w.status[s], panic = w.mse_panic[s], P = w.sel_count[s], nig = w.n_ig[s],
              xok = w.x_ok[s], fis = w.fit_iters_s ? w.fit_iters_s[s] : 0x7fffffff;
    // (no asm use-point as in fit_head: pinning them cost the <4, 30> form 20 VGPRs and
    // so a wave per SIMD; the compiler issues most of them together anyway)
    // k_retain's work, fused: one extra workgroup per spectrum (part == nparts)
    // reports a failed spectrum or compacts its retained Lorentzians into the
    // caller's rows, beside the tiles; the last tile workgroup reports the MSE
    if (part == nparts) {
        if (st) {
            if (tid == 0) {
                a.out_count[s] = 0;
                a.out_mse[s] = 0.0;
                a.out_status[s] = w.status[s];
            }
            return;
        }
        retain_body<BS>(a, w, s, lds_i);
        return;
    }
    if (st) return;
    if (panic) {
        if (part == 0) mse_panic_out(a, s);
        return;
    }
    KSTAMP(30);
    const size_t pbase = (size_t)s * w.capD;
    // final_params with the preloaded iteration count
    const double* __restrict__ prmv = params_version(w, pbase, w.params_alt ? min(fis, w.fit_iters) : 0);
    const const_f64_ptr prm = (const_f64_ptr)prmv;
    const double* x = a.x + (size_t)s * a.x_stride;
    const double* y = y_row(a, s);
    const int64_t total = w.ig_cum[(size_t)s * (w.ig_cap + 2) + nig + 1];  // mse_len
    // every workgroup counts the retained Lorentzians (the last one reports the
    // capacity status) and checks their fast ranges (k_retain's unsafe_kept)
    int cnt = 0, uns = 0;
#pragma unroll 4
    for (int j = tid; j < P; j += BS) {
        const double f = prmv[3 * j], h = prmv[3 * j + 1], m = prmv[3 * j + 2];
        const bool r = retained(f, h);
        cnt += r;
        uns |= r && !peak_fast_ok(f, h, m);
    }
    int kept_n;
    (void)block_exclusive_scan<BS>(cnt, lds_i, &kept_n);
    const bool fast = xok && !__syncthreads_or(uns);
    if (!fast && part == 0 && tid == 0) mark_slow(w, s, kSlowMse);
    KSTAMP(31);
    double acc = 0.0;
    for (int64_t v0 = (int64_t)part * TP; v0 < total; v0 += (int64_t)nparts * TP) {
        double xv[NPT], yv[NPT], sup[NPT];
        bool ok[NPT];
#pragma unroll
        for (int i = 0; i < NPT; ++i) {  // point v0 + tid + i * BS: lanes stay consecutive
            const int64_t v = v0 + tid + (int64_t)i * BS;
            ok[i] = v < total;
            const int64_t idx = mse_index(w, s, nig, ok[i] ? v : 0);
            xv[i] = x[idx];
            yv[i] = y[idx];
        }
        if (!fast) {
#pragma unroll
            for (int i = 0; i < NPT; ++i) sup[i] = sup_retained_direct<false>(xv[i], prm, P);
        } else {
            // (round 6: every term directly for up to 48 retained Lorentzians measured
            // slower on the sim spectra -- 13.4 against 11.8 us at B = 1, 22.0 against
            // 12.7 at B = 16: 26 divisions a point cost more than the far-field pass)
            // tile centre and half range over its valid points
            double lo = INFINITY, hi = -INFINITY;
#pragma unroll
            for (int i = 0; i < NPT; ++i) {
                lo = ok[i] ? fmin(lo, xv[i]) : lo;
                hi = ok[i] ? fmax(hi, xv[i]) : hi;
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                lo = fmin(lo, __shfl_xor(lo, o, 64));
                hi = fmax(hi, __shfl_xor(hi, o, 64));
            }
            if (lane == 0) {
                wmin[wv] = lo;
                wmax[wv] = hi;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                lo = fmin(lo, wmin[k]);
                hi = fmax(hi, wmax[k]);
            }
            const double t = 0.5 * lo + 0.5 * hi;
            const double rt = 0.5 * hi - 0.5 * lo;
            const double lim = kLocR * rt, lim2 = lim * lim;
            // far Lorentzians -> imaginary parts of the series coefficients (per
            // thread, then summed over the block); near ones -> the LDS list in
            // index order (ballot compaction)
            double L[PK];
#pragma unroll
            for (int k = 0; k < PK; ++k) L[k] = 0.0;
            int nnear = 0;
            // the next round's Lorentzian is loaded while this one is expanded
            const int j1 = max(0, min(tid, P - 1));  // P = 0: a harmless in-bounds read
            double fn = prmv[3 * j1], hn = prmv[3 * j1 + 1], mn = prmv[3 * j1 + 2];
            for (int j0 = 0; j0 < P; j0 += BS) {
                const int j = j0 + tid;
                const double f = fn, h = hn, m = mn;
                {
                    const int jn = min(j + BS, P - 1);
                    fn = prmv[3 * jn];
                    hn = prmv[3 * jn + 1];
                    mn = prmv[3 * jn + 2];
                }
                const bool have = j < P && retained(f, h);
                const double dm = m - t;
                const double d2 = __builtin_fma(dm, dm, h);  // |z - t|^2
                const bool nr = have && !(d2 > lim2);
                if (have && !nr) {
                    // w = (dm - i sg) / d2;  c = a w = (f / d2) (dm / sg - i);  q = r w
                    const double id2 = rcp_nr2(d2);
                    const double sg = __builtin_sqrt(h);
                    const double isg = rcp_nr2(sg);
                    const double fq = f * id2;
                    const double cr = fq * (dm * isg), ci = -fq;
                    const double rq = rt * id2;
                    const double qr = rq * dm, qi = -(rq * sg);
                    // y_k = Im(c q^k) by the real recurrence y_{k+2} = 2 Re(q) y_{k+1}
                    // - |q|^2 y_k (roots q and conj(q), one modulus < 1/kLocR: an error
                    // decays like the terms themselves; tools/mse_local_error.py 'rec'
                    // matches the complex product to the last digit): 3 instructions
                    // per power instead of the complex product's 5
                    const double a2 = 2.0 * qr, b = __builtin_fma(qr, qr, qi * qi);
                    double y0 = ci, y1 = __builtin_fma(cr, qi, ci * qr);
                    L[0] += y0;
                    L[1] += y1;
#pragma unroll
                    for (int k = 2; k < PK; ++k) {
                        const double y2 = __builtin_fma(a2, y1, -(b * y0));
                        L[k] += y2;
                        y0 = y1;
                        y1 = y2;
                    }
                }
                const uint64_t bal = __ballot(nr);
                const int pre = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
                if (lane == 0) wcnt[wv] = __popcll(bal);
                __syncthreads();
                int base = nnear, all = 0;
#pragma unroll
                for (int k = 0; k < NW; ++k) {
                    const int c = wcnt[k];
                    base += k < wv ? c : 0;
                    all += c;
                }
                if (nr && base + pre < near_cap) {
                    nearp[3 * (base + pre)] = f;
                    nearp[3 * (base + pre) + 1] = h;
                    nearp[3 * (base + pre) + 2] = m;
                }
                nnear += all;
                __syncthreads();
            }
            KSTAMP(32);
            // sum the coefficients over the block, PH at a time: 16 threads per
            // coefficient, 16 values each, then a butterfly over the 16 lanes
#pragma unroll
            for (int hf = 0; hf < NH; ++hf) {
#pragma unroll
                for (int k = 0; k < PH; ++k) red[k * BS + tid] = L[hf * PH + k];
                __syncthreads();
                if (tid < PH * 16) {
                    const int k = tid >> 4, g = tid & 15;
                    double sm = 0.0;
#pragma unroll
                    for (int i = 0; i < 16; ++i) sm += red[k * BS + g * 16 + i];
#pragma unroll
                    for (int o = 8; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 16);
                    if (g == 0) coef[hf * PH + k] = -sm;
                }
                __syncthreads();
            }
            KSTAMP(33);
            if (nnear > near_cap) {
#pragma unroll
                for (int i = 0; i < NPT; ++i) sup[i] = sup_retained_direct<true>(xv[i], prm, P);
            } else {
                double nsum[NPT];
#pragma unroll
                for (int i = 0; i < NPT; ++i) {
                    const double u = rt > 0.0 ? (xv[i] - t) / rt : 0.0;
                    double S = coef[PK - 1];
#pragma unroll
                    for (int k = PK - 2; k >= 0; --k) S = __builtin_fma(S, u, coef[k]);
                    sup[i] = S;
                    nsum[i] = 0.0;
                }
                // near Lorentzians: four per division (quad_term), the rest one by one
                int j = 0;
                for (; j + 4 <= nnear; j += 4) {
                    double c[12];
#pragma unroll
                    for (int k = 0; k < 12; ++k) c[k] = nearp[3 * j + k];
#pragma unroll
                    for (int i = 0; i < NPT; ++i) nsum[i] += quad_term(xv[i], c);
                }
                for (; j < nnear; ++j)
#pragma unroll
                    for (int i = 0; i < NPT; ++i)
                        nsum[i] += lorentz_mse<true>(xv[i], nearp[3 * j], nearp[3 * j + 1], nearp[3 * j + 2]);
#pragma unroll
                for (int i = 0; i < NPT; ++i) sup[i] = nsum[i] + sup[i];
            }
        }
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            const double d = sup[i] - yv[i];
            if (ok[i]) acc += d * d;
        }
        __syncthreads();  // LDS reuse by the next tile
    }
    KSTAMP(34);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (lane == 0) wacc[wv] = acc;
    __syncthreads();
    double tot = 0.0;
    if (tid == 0) {
#pragma unroll
        for (int k = 0; k < NW; ++k) tot += wacc[k];
    }
    mse_publish_fold<BS>(a, w, s, part, nparts, tot, kept_n, red);
    KSTAMP(35);
}

__device__ __forceinline__ void mse_panic_out(const BatchArgs& a, int s) {
    if (threadIdx.x == 0) {
        a.out_status[s] = MDG_REFERENCE_PANIC;
        a.out_mse[s] = 0.0;
    }
}

// ----------------------------------------------------------------------------------
// standalone Lorentzian::superposition_vec (lorentzian.rs:631-663)
// ----------------------------------------------------------------------------------
// range pre-pass: flag[0] = number of Lorentzians / x values outside the fast ranges
// ----------------------------------------------------------------------------------
// Exact MSE (deconvoluter.rs:846-861 in the reference's order): squared residuals,
// then one wave folds each region left to right (dpp_fold) and the region sums in
// region order. Used by optimize_settings to settle near-ties of the tree MSE.
// ----------------------------------------------------------------------------------
__global__ void k_sq_residuals(const double* __restrict__ sup, const double* __restrict__ y,
                               int64_t n, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const double d = sup[i] - y[i];
        out[i] = d * d;
    }
}

__global__ __launch_bounds__(64) void k_exact_fold(const double* __restrict__ t, Workspace w,
                                                   double* __restrict__ out) {
    const int nig = w.n_ig[0];
    double total = -0.0;
    int64_t len = 0;
    for (int k = 0; k <= nig; ++k) {
        int64_t lo, hi;
        mse_region(w, 0, k, nig, &lo, &hi);
        total += dpp_fold(-0.0, t + lo, (int)(hi - lo));
        len += hi - lo;
    }
    if (threadIdx.x == 0) out[0] = total / (double)len;
}

// Exact-order MSE of a whole batch (mdg_settings.options & MDG_OPTION_EXACT_MSE),
// after k_mse_local has compacted the retained Lorentzians: compute_mse
// (deconvoluter.rs:828-862) in the reference's operation order.
// k_mse_exact_res: the squared residual of every MSE-region point, in the regions'
// virtual concatenation order (row s of res, res_row doubles apart): the point's
// superposition is superposition_vec's in-order left fold over the retained
// Lorentzians (lorentzian.rs:606-611; superpose, bit-identical to the oracle --
// the fit's exact division), then (sup - y)^2 (`.powi(2)` is one multiply).
// 1-D grid, spectrum = block % B (k_fit_sup's layout: workgroups resident on a CU at
// once share one spectrum's Lorentzians in the scalar cache).
__global__ void k_mse_exact_res(BatchArgs a, Workspace w, double* res, int64_t res_row) {
    const int s = blockIdx.x % a.B, part = blockIdx.x / a.B, parts = gridDim.x / a.B;
    if (w.status[s] || w.mse_panic[s]) return;
    const int P = w.kept_count[s];
    const double* __restrict__ kept = w.kept + 3 * (size_t)s * w.capD;
    const double* x = a.x + (size_t)s * a.x_stride;
    const double* y = y_row(a, s);
    const int nig = w.n_ig[s];
    const int64_t total = mse_len(w, s);
    const bool fast = w.x_ok[s] && w.unsafe_kept[s] == 0;
    if (!fast && part == 0 && threadIdx.x == 0) mark_slow(w, s, kSlowMseExact);
    double* r = res + (size_t)s * res_row;
    for (int64_t v = (int64_t)part * blockDim.x + threadIdx.x; v < total; v += (int64_t)parts * blockDim.x) {
        const int64_t idx = mse_index(w, s, nig, v);
        const double d = superpose(x[idx], kept, P, fast) - y[idx];
        r[v] = d * d;
    }
}

// k_mse_exact_fold: one workgroup per spectrum folds each region's squared residuals
// left to right from -0.0 (`.sum::<f64>()`), adds the region sums in region order (the
// outer `.sum::<f64>()`) and divides by the regions' total length; it overwrites the
// MSE k_mse_local wrote (its status stays). The squared residuals are >= +0, so a
// region of 64 or more terms takes k_select's windowed fold (every add the
// reference's, in its order; §2): one wave alone folded the ~91k terms of a
// 131072-point spectrum in ~300 us.
constexpr int kExactFoldBS = 1024;
__global__ __launch_bounds__(kExactFoldBS) void k_mse_exact_fold(BatchArgs a, Workspace w, const double* res,
                                                                 int64_t res_row) {
    __shared__ WinLds wl;
    __shared__ double part_sh;
    const int s = blockIdx.x;
    if (w.status[s] || w.mse_panic[s]) return;
    const int nig = w.n_ig[s];
    const int64_t* cum = w.ig_cum + (size_t)s * (w.ig_cap + 2);
    const double* r = res + (size_t)s * res_row;
    double total = -0.0;
    for (int k = 0; k <= nig; ++k) {
        const int n = (int)(cum[k + 1] - cum[k]);
        double part;
        if (n >= 4 * kWinSeg) {
            part = window_fold<kExactFoldBS>(-0.0, wl, r + cum[k], n, 60);  // barriers inside
        } else {
            if (threadIdx.x < 64) {
                const double v = dpp_fold(-0.0, r + cum[k], n);
                if (threadIdx.x == 0) part_sh = v;
            }
            __syncthreads();
            part = part_sh;
            __syncthreads();
        }
        total += part;
    }
    if (threadIdx.x == 0) a.out_mse[s] = total / (double)cum[nig + 1];
}

template <int BS>
__global__ __launch_bounds__(BS) void k_fit_small(BatchArgs a, Workspace w) {
    __shared__ double prm[3 * kSmallP];
    __shared__ double buf[9 * kSmallP];  // stencil x and y planes (3 per peak each), ratios (3 per point)
    __shared__ double T[kSmallT];        // the terms of one iteration (3 P^2 <= kSmallT)
    double* const stn = buf;
    double* const rat = buf + 6 * kSmallP;
    const int s = blockIdx.x;
    KSTAMP(70);
    const int st = w.status[s], P = w.sel_count[s], xok = w.x_ok[s];
    const int fis = w.fit_iters_s ? w.fit_iters_s[s] : 0x7fffffff;
    if (st) return;
    const int iters = min(fis, w.fit_iters);
    const size_t base = (size_t)s * w.capD;
    if (P <= kSmallP) {
        for (int k = threadIdx.x; k < 3 * P; k += BS) prm[k] = w.params[3 * base + k];
        for (int k = threadIdx.x; k < 3 * P; k += BS) {
            stn[k] = w.stencil[6 * base + k];
            stn[3 * kSmallP + k] = w.stencil[6 * base + 3 * (size_t)w.capD + k];
        }
        __syncthreads();
        if (P > 0 && 3 * P * (P | 1) <= kSmallT && P <= BS) {
            static_assert(kSmallT % BS == 0, "whole term slots per thread");
            fit_small_terms<BS>(w, s, P, iters, xok, prm, stn, rat, T);
        } else {
            fit_small_body<BS>(w, s, P, iters, xok, (double*)prm, (double*)prm, stn, rat, true, 3 * kSmallP);
        }
        // the version k_mse_local's retain reads (final_params)
        double* out = (double*)params_version(w, base, iters);
        for (int k = threadIdx.x; k < 3 * P; k += BS) out[k] = prm[k];
    } else {
        fit_small_body<BS>(w, s, P, iters, xok, (double*)nullptr, (double*)nullptr, w.stencil + 6 * base,
                           w.kept + 3 * base, false, 3 * (size_t)w.capD);
    }
    KSTAMP(75);
}

__global__ void k_range_check(const double* __restrict__ x, int64_t n,
                              const double* __restrict__ params, int P, int* flag) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P;
         i += (int64_t)gridDim.x * blockDim.x)
        if (!peak_fast_ok(params[3 * i], params[3 * i + 1], params[3 * i + 2])) atomicAdd(flag, 1);
    if (blockIdx.x == 0 && threadIdx.x == 0 && n > 0)
        if (!x_fast_ok(x[0]) || !x_fast_ok(x[n - 1])) atomicAdd(flag, 1);
}

__global__ void k_superposition_vec(const double* __restrict__ x, int64_t n,
                                    const double* __restrict__ params, int P,
                                    double* __restrict__ out, const int* flag) {
    // x need not be monotone here: lanes check their own x
    const bool fast_peaks = *flag == 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double xi = x[i];
        out[i] = superpose(xi, params, P, fast_peaks && x_fast_ok(xi));
    }
}

// synthetic batch: x shared, y_s = superposition(params_s) + noise(seed_s)
__global__ void k_synth_x(double* x, int64_t n, double xmax, double width) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = xmax - ((double)i * width) / ((double)n - 1.0);
}

__global__ void k_synth_y(const double* __restrict__ x, int64_t n,
                          const double* __restrict__ params, int P, uint64_t seed0,
                          double sigma, double* __restrict__ y) {
    const int s = blockIdx.y;
    const uint64_t key = stream_key(seed0 + (uint64_t)s, kStreamNoise);
    const double* ps = params + 3 * (size_t)s * P;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[(size_t)s * n + i] = superpose(x[i], ps, P, false) + synth_noise(key, (uint64_t)i, sigma);
}

// ----------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------
static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

namespace {
std::mutex g_pk_mu;
std::vector<const void*> g_pk;  // pipeline kernels launched so far (a few dozen)
}  // namespace

void note_pipeline_kernel(const void* f) {
    std::lock_guard<std::mutex> g(g_pk_mu);
    if (std::find(g_pk.begin(), g_pk.end(), f) == g_pk.end()) g_pk.push_back(f);
}

bool is_pipeline_kernel(const void* f) {
    std::lock_guard<std::mutex> g(g_pk_mu);
    return std::find(g_pk.begin(), g_pk.end(), f) != g_pk.end();
}

void launch_prep(const BatchArgs& a, const Workspace& w, hipStream_t st) {
    launch_k(k_prep, dim3(cdiv(a.B, 64)), dim3(64), 0, st, a, w);
}

#ifdef MDG_DIAG
// throughput diagnostic (MDG_DIAG_PAD, mdg_capi.hip; diagnostic builds only): a
// launch that does nothing, with the pipeline's kernel arguments
__global__ void k_diag_nop(BatchArgs a, Workspace w) {
    if (a.B < 0) w.status[0] = 0;
}
__global__ void k_diag_nop_small(int32_t* p, int b) {
    if (b < 0) p[0] = 0;
}
void launch_diag_nop(const BatchArgs& a, const Workspace& w, const EngineSwitches& sw, hipStream_t st) {
    if (sw.diag_pad_small) hipLaunchKernelGGL(k_diag_nop_small, dim3(1), dim3(64), 0, st, w.status, a.B);
    else {
        // MDG_DIAG_PAD_WGS: workgroups of the no-op (the cost of workgroup dispatch)
        const int g = sw.diag_pad_wgs;
        launch_k(k_diag_nop, dim3(g ? std::max(1, g) : 1), dim3(g ? 256 : 64), 0, st, a, w);
    }
}
#endif
template <int WS>
static const char* launch_pipe(const BatchArgs& a, const Workspace& w, int iters, hipStream_t st) {
    const int spw = 64 / iters;
    launch_k(k_smooth_pipe<WS>, dim3(cdiv(a.B, spw)), dim3(64), 0, st, a, w, iters, spw);
    static const char* names[] = {"", "", "k_smooth_pipe<2>", "k_smooth_pipe<3>", "k_smooth_pipe<4>",
                                  "k_smooth_pipe<5>", "k_smooth_pipe<6>", "k_smooth_pipe<7>",
                                  "k_smooth_pipe<8>", "k_smooth_pipe<9>", "", "k_smooth_pipe<11>"};
    return names[WS];
}

template <int WS>
static const char* launch_chain(const BatchArgs& a, const Workspace& w, int iters, const EngineSwitches& sw,
                                hipStream_t st, int fused_prep) {
    const unsigned grid = 8u * (unsigned)iters * cdiv(a.B, 8);
    const bool excl = (int)grid <= kChainExclMax && sw.chain_excl;  // MDG_CHAIN_EXCL=0: never (measurements)
    // rows still in host memory (a.dec_rows; the pipeline fuses the prep then): 32
    // decoders up to 4 spectra, 64 beyond (chain_decode; a multiple of 8 keeps the
    // chain workgroups' XCD mapping)
    const int ndec = a.dec_rows && fused_prep ? (a.B <= 4 ? 32 : 64) : 0;
    // input blocks pulled into L2 ahead of each chain (MDG_CHAIN_L2AHEAD: measurements)
    const int per_xcd = (int)cdiv((int)grid, 8);
    const int l2ahead = sw.chain_l2ahead > 0
                            ? sw.chain_l2ahead
                            : std::max(8, std::min(kChainL2Ahead, kChainL2Bytes / (per_xcd * kChainCB * 8)));
    if (excl) {
        launch_k((k_smooth_chain<WS, true>), dim3(grid + ndec), dim3(64 * (2 + kChainScalers)), 0, st,
                           a, w, iters, fused_prep, ndec, l2ahead);
    } else {
        launch_k((k_smooth_chain<WS, false>), dim3(grid + ndec), dim3(64 * (2 + kChainScalers)), 0, st,
                           a, w, iters, fused_prep, ndec, l2ahead);
    }
    static const char* names[2][9] = {
        {"", "", "k_smooth_chain<2, false>", "k_smooth_chain<3, false>", "k_smooth_chain<4, false>",
         "k_smooth_chain<5, false>", "k_smooth_chain<6, false>", "k_smooth_chain<7, false>",
         "k_smooth_chain<8, false>"},
        {"", "", "k_smooth_chain<2, true>", "k_smooth_chain<3, true>", "k_smooth_chain<4, true>",
         "k_smooth_chain<5, true>", "k_smooth_chain<6, true>", "k_smooth_chain<7, true>",
         "k_smooth_chain<8, true>"}};
    return names[excl ? 1 : 0][WS];
}
// chain kernel (one CU per pass) for windows <= 8 and batches <= 512 (B * iters
// <= 2048) when its buffers are set up and MDG_SMOOTH does not force another
// small spectra (N <= kSmallN): k_smooth_small, one workgroup per spectrum (MDG_SMOOTH=small
// forces it wherever its shape limits allow)
bool smooth_uses_small(const BatchArgs& a, int iters, int ws, const EngineSwitches& sw) {
    const bool ok = smooth_small_ok(a.N, iters, ws);
    return ok && sw.smooth == EngineSwitches::SM_SMALL;  // MDG_SMOOTH=small only (slower, K1s)
}
bool smooth_uses_chain(const BatchArgs& a, const Workspace& w, int iters, int ws, const EngineSwitches& sw) {
    const bool chain = sw.smooth == EngineSwitches::SM_DEFAULT || sw.smooth == EngineSwitches::SM_CHAIN;
    return chain && !smooth_uses_small(a, iters, ws, sw) && w.chain_P >= iters &&
           chain_supported(a.B, a.N, iters, ws);
}
bool smooth_fuses_prep(const BatchArgs& a, const Workspace& w, int iters, int ws, const EngineSwitches& sw) {
    return smooth_uses_small(a, iters, ws, sw) || smooth_uses_chain(a, w, iters, ws, sw);
}
const char* launch_smooth(const BatchArgs& a, const Workspace& w, int iters, int ws, const EngineSwitches& sw,
                          hipStream_t st, int fused_prep) {
    // the chain kernel; then lane-pipelined (window fits the register FIFO); the
    // one-lane-per-spectrum kernel otherwise; small spectra k_smooth_small.
    // MDG_SMOOTH = chain | pipe | generic | small forces one (tests); an
    // unsupported shape falls through. fused_prep (chain and small only): the kernel
    // runs k_prep's work itself.
    if (smooth_uses_small(a, iters, ws, sw)) return launch_smooth_small(a, w, iters, ws, st, fused_prep);
    if (smooth_uses_chain(a, w, iters, ws, sw)) {
        switch (ws) {
            case 2: return launch_chain<2>(a, w, iters, sw, st, fused_prep);
            case 3: return launch_chain<3>(a, w, iters, sw, st, fused_prep);
            case 4: return launch_chain<4>(a, w, iters, sw, st, fused_prep);
            case 5: return launch_chain<5>(a, w, iters, sw, st, fused_prep);
            case 6: return launch_chain<6>(a, w, iters, sw, st, fused_prep);
            case 7: return launch_chain<7>(a, w, iters, sw, st, fused_prep);
            case 8: return launch_chain<8>(a, w, iters, sw, st, fused_prep);
            default: break;
        }
    }
    // beyond the chain's batch limit the lane-pipelined kernel (tools/smooth_sweep.sh:
    // 131072 points, B = 1024: 4.8 ms; configs[3], 4096 x 65536: 2.7 ms; round 2's
    // wave-per-pass kernel took 9.9 and 17.0); windows outside its
    // register FIFO the one-lane-per-spectrum kernel
    const bool pipe = sw.smooth == EngineSwitches::SM_DEFAULT || sw.smooth == EngineSwitches::SM_PIPE;
    if (pipe && iters >= 1 && iters <= 32 && a.N > ws + 1) {
        switch (ws) {
            case 2: return launch_pipe<2>(a, w, iters, st);
            case 3: return launch_pipe<3>(a, w, iters, st);
            case 4: return launch_pipe<4>(a, w, iters, st);
            case 5: return launch_pipe<5>(a, w, iters, st);
            case 6: return launch_pipe<6>(a, w, iters, st);
            case 7: return launch_pipe<7>(a, w, iters, st);
            case 8: return launch_pipe<8>(a, w, iters, st);
            case 9: return launch_pipe<9>(a, w, iters, st);
            case 11: return launch_pipe<11>(a, w, iters, st);
            default: break;
        }
    }
    launch_k(k_smooth, dim3(cdiv(a.B, 64)), dim3(64), 0, st, a, w, iters, ws);
    return "k_smooth";
}
// fine (staged) chunks up to 512 workgroups of 64-word chunks (launch_peaks)
static bool peaks_fine(const BatchArgs& a, const Workspace& w, const EngineSwitches& sw) {
    return sw.peaks ? sw.peaks == 1 : (size_t)cdiv(w.W, 64) * a.B <= 512;
}
// the predicates inside k_peaks only with MDG_DETECT=fused (bit-exact, tested): measured
// slower (round 6) -- the fine chunks' predicate pass took 13.5k cycles per chunk
// (stamps, B = 1: k_peaks 20 us against k_flags 4.8 + k_peaks 13.5), and the coarse
// chunks at the headline saved only 0.19 MB per spectrum (k_peaks 1.91 MB against
// k_flags 0.74 + k_peaks 1.36: the scores' row reads did not hit the lines the
// predicates had just read) while the queue ran 16.0k against 16.6-16.7k spectra/s
bool peaks_fuse_flags(const BatchArgs& a, const Workspace& w, const EngineSwitches& sw) {
    (void)a, (void)w;
    return sw.detect == 2;
}
void launch_flags(const BatchArgs& a, const Workspace& w, hipStream_t st) {
    launch_k(k_flags, dim3(cdiv(a.N, 256), a.B), dim3(256), 0, st, a, w);
}
const char* launch_peaks(const BatchArgs& a, const Workspace& w, int detector_only, const EngineSwitches& sw,
                         hipStream_t st) {
    // k_peaks scores the peaks it writes (scorer.rs:65-75) for the selector. Fine
    // (staged) chunks up to 512 workgroups of 64-word chunks (B <= 16 at N = 131072:
    // blood, 13.2 / 12.9 / 15.4 / 17.5 us at B = 1 / 4 / 8 / 16 against the coarse
    // chunks' 21.3 / 21.9 / 22.9 / 23.1; synthetic B = 64: 59.8 against 52.6, B = 256:
    // 230 against 216); MDG_PEAKS = fine | coarse forces one (tests)
    const bool fine = peaks_fine(a, w, sw);
    if (peaks_fuse_flags(a, w, sw)) {
        if (fine) {
            launch_k(k_peaks<64, 256, true>, dim3(cdiv(w.W, 64), a.B), dim3(256), 0, st, a, w, detector_only, 1);
            return "k_peaks<64, flags>";
        }
        launch_k(k_peaks<256, 1024, true>, dim3(cdiv(w.W, 256), a.B), dim3(1024), 0, st, a, w, detector_only, 1);
        return "k_peaks<256, flags>";
    }
    if (fine) {
        launch_k(k_peaks<64, 256>, dim3(cdiv(w.W, 64), a.B), dim3(256), 0, st, a, w, detector_only, 1);
        return "k_flags+k_peaks<64>";
    }
    launch_k(k_peaks<256, 1024>, dim3(cdiv(w.W, 256), a.B), dim3(1024), 0, st, a, w, detector_only, 1);
    return "k_flags+k_peaks<256>";
}
// detection inside k_select (k_select<1024, true>): small spectra, the noise-score
// selector (MDG_DETECT = separate | fused forces either where the shape allows)
bool detect_fused(const BatchArgs& a, int detector_only, const EngineSwitches& sw) {
    return !detector_only && a.N <= kSmallN && sw.detect != 1;
}
const char* launch_select(const BatchArgs& a, const Workspace& w, int detector_only,
                          double threshold, hipStream_t st, bool fused) {
    if (detector_only) {
        launch_k(k_select_detector_only, dim3(16, a.B), dim3(256), 0, st, a, w);
        return "k_select_detector_only";
    }
    if (fused) {  // (256 threads measured slower: 19.0 against 15.7 us on sim_01)
        launch_k(k_select<1024, true>, dim3(a.B), dim3(1024), 0, st, a, w, threshold);
        return "k_select<1024, det>";
    }
    launch_k(k_select<1024>, dim3(a.B), dim3(1024), 0, st, a, w, threshold);
    return "k_select<1024>";
}
// Fit kernel choice by batch size. B = 1: the term fold over 12-point
// tiles ("tf12": blood, ten launches 95.4 against 100.7 us; equal at B = 2, worse at
// 4; 6-point tiles: 112-113 us); B <= 4: the 24-point term fold over one workgroup per tile ("tf"); B <= 24: the 63-point term fold over one
// batch-wide tile list on two workgroups per CU ("twf1"; blood set, ten launches:
// 373 us at B = 16 against 403 for the (98, B) grid "tw7", 270 / 268 at B = 8, 204
// against tf's 185 at B = 4); beyond, one point per lane with the update separate
// ("plain": 79 / 57 us per spectrum at B = 32 / 256). When other engine contexts on
// the device run pipelines concurrently, B = 1 keeps "tw7": "tf"'s lead alone is gone
// as soon as a second context runs, and 18 concurrent B = 1 pipelines run 6.6k
// spectra/s with "tf" against 7.8-8.1k with "tw7". Which of the two a context takes
// is its latency mode (mdg_ctx_set_latency_mode: on by default -- one spectrum at a
// time with the GPU to itself; callers running many contexts at once turn it off).
// MDG_FITSUP = tf | tf12 | tw7 | tw3s | twf | twf1 | twf3s | plain forces one (all
// bit-identical; tests, measurements; read into the context's switches, where any
// other value is ignored).
static std::string fit_choice(const BatchArgs& a, const EngineSwitches& sw) {
    if (sw.fitsup[0]) return sw.fitsup;
    // small spectra: the whole fit in one workgroup per spectrum (k_fit_small). Not with
    // the detector-only selector: it keeps every detected peak (~250 in a 2048-point sim
    // spectrum), and one workgroup cannot evaluate 3 P^2 terms per iteration as fast as
    // the tile fits' hundreds (P ~ 100 is about even, measured at P = 26: 2.3 against
    // 4.6 us per iteration). A noise-score selection keeps ~25-35 peaks of the sims.
    if (a.N <= kSmallN && !a.det_only) return "small";
    if (a.B == 1) return a.latency ? "tf12" : "tw7";
    return a.B <= 4 ? "tf" : a.B <= 24 ? "twf1" : "plain";
}
bool fit_sup_fused(const BatchArgs& a, const EngineSwitches& sw) {
    const std::string f = fit_choice(a, sw);
    return f != "plain" && f != "mfma";  // those two leave the stencil update to k_fit_update
}
bool fit_is_small(const BatchArgs& a, const EngineSwitches& sw) { return fit_choice(a, sw) == "small"; }
const char* launch_fit_small(const BatchArgs& a, const Workspace& w, hipStream_t st) {
    launch_k(k_fit_small<kSmallBS>, dim3(a.B), dim3(kSmallBS), 0, st, a, w);
    return "k_fit_small";
}
const char* launch_fit_sup(const BatchArgs& a, const Workspace& w, int gx, int it, const EngineSwitches& sw,
                           hipStream_t st) {
    const std::string f = fit_choice(a, sw);
    // MDG_TW_G (tuning): workgroups per spectrum; tiles beyond them grid-stride
    const int tg = sw.tw_g;
#ifdef MDG_DIAG
    if (f == "mfma") {
        // experiment only (diagnostic builds; not bit-exact): 64 points per workgroup
        const int g = std::max(1, std::min(2048, (3 * (a.N / 2 + 2) + 63) / 64));
        const int parts = std::max(1, std::min(g, 8192 / a.B));
        launch_k(k_fit_sup_mfma, dim3(parts * a.B), dim3(256), 0, st, a, w, it);
        return "k_fit_sup_mfma";
    }
#endif
    if (f == "tw7") {
        // 7 evaluator waves: 1 peak block x 7 point subsets, 63 points per workgroup:
        // one workgroup per tile of a 2048-peak spectrum (98)
        using SH = TwShape<63, 1, 7>;
        const int g = tg ? tg : (3 * 2048 + 62) / 63;
        launch_k(k_fit_sup_tw<SH>, dim3(g, a.B), dim3(64 * (SH::EW + 1)), 0, st, a, w, it);
        return "k_fit_sup_tw<63, 1, 7>";
    }
    if (f == "tw3s") {
        // single-buffered 63-point tiles, 3 evaluator waves: four workgroups per CU
        using SH = TwShape<63, 1, 3, true>;
        const int g = tg ? tg : (3 * 2048 + 62) / 63;
        launch_k(k_fit_sup_tw<SH>, dim3(g, a.B), dim3(64 * (SH::EW + 1)), 0, st, a, w, it);
        return "k_fit_sup_tw<63, 1, 3, SB>";
    }
    if ((f == "twf" || f == "twf1" || f == "twf3s") && a.B <= kTwfMaxB) {
        // one list of the batch's tiles over about one workgroup per slot: <63, 2, 7>
        // (15 waves, 131 KB of LDS) one per CU, <63, 1, 7> (8 waves, 66 KB) two
        const int cus = sw.cus;
        if (f == "twf3s") {
            using SH = TwShape<63, 1, 3, true>;
            const int g = tg ? tg : 4 * cus;
            launch_k(k_fit_sup_twf<SH>, dim3(g), dim3(64 * (SH::EW + 1)), 0, st, a, w, it);
            return "k_fit_sup_twf<63, 1, 3, SB>";
        }
        if (f == "twf") {
            using SH = TwShape<63, 2, 7>;
            const int g = tg ? tg : cus;
            launch_k(k_fit_sup_twf<SH>, dim3(g), dim3(64 * (SH::EW + 1)), 0, st, a, w, it);
            return "k_fit_sup_twf<63, 2, 7>";
        }
        using SH = TwShape<63, 1, 7>;
        const int g = tg ? tg : 2 * cus;
        launch_k(k_fit_sup_twf<SH>, dim3(g), dim3(64 * (SH::EW + 1)), 0, st, a, w, it);
        return "k_fit_sup_twf<63, 1, 7>";
    }
    if (f == "tf12") {
        // 12-point tiles: twice the workgroups, half the evaluation per workgroup
        const int g = tg ? tg : (3 * 2048 + 11) / 12;
        launch_k(k_fit_sup_tf<12>, dim3(g, a.B), dim3(64 * (kTfEW + 1)), 0, st, a, w, it);
        return "k_fit_sup_tf<12>";
    }
    if (f == "tf" || f == "twf" || f == "twf1" || f == "twf3s") {
        // 24 points per workgroup: one workgroup per tile of a 2048-peak spectrum (256)
        const int g = tg ? tg : (3 * 2048 + 23) / 24;
        launch_k(k_fit_sup_tf<kTfQ>, dim3(g, a.B), dim3(64 * (kTfEW + 1)), 0, st, a, w, it);
        return "k_fit_sup_tf";
    }
    // gx 256-thread workgroups per spectrum (24: one point per thread at P = 2048)
    launch_k(k_fit_sup, dim3(gx * a.B), dim3(256), 0, st, a, w, it);
    return "k_fit_sup";
}
void launch_fit_update(const BatchArgs& a, const Workspace& w, int gx, int it, hipStream_t st) {
    launch_k(k_fit_update, dim3(gx, a.B), dim3(256), 0, st, a, w, it);
}
void launch_retain(const BatchArgs& a, const Workspace& w, hipStream_t st) {
    launch_k(k_retain<1024>, dim3(a.B), dim3(1024), 0, st, a, w);
}
// The MSE kernel is k_mse_local<2> (local expansions of the far Lorentzians, tiles of
// 512 points; it compacts the retained Lorentzians itself, so no k_retain launch).
// Round 3 measured it against the 256-point tiles (k_mse_local<1>) and the earlier
// k_mse_quad / k_mse_partial_n / k_mse_partial; those are not in the
// library any more.
constexpr int kLocNPT = 2;
// MDG_MSE_NPT = 2 | 4 (points per thread) and MDG_MSE_PARTS (tile workgroups per
// spectrum, <= kMseMaxParts): measurement knobs for small batches
// Default: 4 points per thread from B = 8 (blood set, B = 16: 55 against 81 us per
// launch; the headline queue, B = 256: 3.6 against 3.8 us per spectrum, 15.76-15.78k
// against 15.67-15.68k spectra/s; B = 1: 24 against 18 -- a single spectrum wants the
// finer tiles)
static int mse_npt(const BatchArgs& a, const EngineSwitches& sw) {
    if (sw.mse_npt) return sw.mse_npt == 4 ? 4 : kLocNPT;
    return a.B >= 8 ? 4 : kLocNPT;
}
int mse_nparts(const BatchArgs& a, const EngineSwitches& sw) {
    if (sw.mse_parts) return std::max(1, std::min(kMseMaxParts, sw.mse_parts));
    const int tp = kLocTP * mse_npt(a, sw);
    return std::max(1, std::min({kMseMaxParts, (a.N + tp - 1) / tp, std::max(1, 8192 / a.B)}));
}
const char* launch_mse(const BatchArgs& a, const Workspace& w, int nparts, const EngineSwitches& sw,
                       hipStream_t st) {
    // MDG_MSE_NEARCAP (tests): a smaller near-list capacity, to exercise the kernel's
    // own direct fallback for crowded tiles
    const int cap = sw.mse_nearcap >= 0 ? std::min(kLocNear, sw.mse_nearcap) : kLocNear;
    // nparts tile workgroups per spectrum plus its retain workgroup
    const dim3 g((nparts + 1) * a.B);
    const int npt = mse_npt(a, sw);
    const bool pk30 = sw.mse_pk != 20;  // 30 powers unless MDG_MSE_PK=20 (round 5)
    if (npt == 4) {
        if (pk30) {
            launch_k(k_mse_local<4, 30>, g, dim3(256), 0, st, a, w, nparts, cap);
            return "k_mse_local<4, 30>";
        }
        launch_k(k_mse_local<4, 20>, g, dim3(256), 0, st, a, w, nparts, cap);
        return "k_mse_local<4, 20>";
    }
    if (pk30) {
        launch_k(k_mse_local<kLocNPT, 30>, g, dim3(256), 0, st, a, w, nparts, cap);
        return "k_mse_local<2, 30>";
    }
    launch_k(k_mse_local<kLocNPT, 20>, g, dim3(256), 0, st, a, w, nparts, cap);
    return "k_mse_local<2, 20>";
}
void launch_mse_exact(const double* sup, const double* y, int64_t n, const Workspace& w,
                      double* scratch, double* out, hipStream_t st) {
    hipLaunchKernelGGL(k_sq_residuals, dim3(cdiv(n, 256)), dim3(256), 0, st, sup, y, n, scratch);
    hipLaunchKernelGGL(k_exact_fold, dim3(1), dim3(64), 0, st, scratch, w, out);
}
void launch_mse_exact_batch(const BatchArgs& a, const Workspace& w, double* res, int64_t res_row,
                            hipStream_t st) {
    // one point per thread (every SIMD gets waves even for one spectrum: each thread's
    // in-order superposition is a dependent chain), fewer workgroups per spectrum for
    // larger batches (the grid-stride loop covers the rest)
    const int parts = std::max(1, std::min<int>(cdiv(res_row, 256), std::max(1, 65536 / a.B)));
    launch_k(k_mse_exact_res, dim3(parts * a.B), dim3(256), 0, st, a, w, res, res_row);
    launch_k(k_mse_exact_fold, dim3(a.B), dim3(kExactFoldBS), 0, st, a, w, (const double*)res, res_row);
}
void launch_superposition_vec(const double* x, int64_t n, const double* params, int P,
                              double* out, int* flag, hipStream_t st) {
    (void)hipMemsetAsync(flag, 0, sizeof(int), st);
    hipLaunchKernelGGL(k_range_check, dim3(std::max(1u, std::min(cdiv(P, 256), 1024u))), dim3(256),
                       0, st, x, n, params, P, flag);
    const unsigned g = std::max(1u, std::min(cdiv(n, 256), 65535u));
    hipLaunchKernelGGL(k_superposition_vec, dim3(g), dim3(256), 0, st, x, n, params, P, out,
                       (const int*)flag);
}
void launch_synth(double* x, double* y, int64_t n, int B, double xmax, double width,
                  const double* params, int P, uint64_t seed0, double sigma, hipStream_t st) {
    hipLaunchKernelGGL(k_synth_x, dim3(cdiv(n, 256)), dim3(256), 0, st, x, n, xmax, width);
    const unsigned g = std::max(1u, std::min(cdiv(n, 256), 2048u));
    hipLaunchKernelGGL(k_synth_y, dim3(g, B), dim3(256), 0, st, x, n, params, P, seed0, sigma, y);
}


// ----------------------------------------------------------------------------------
// Spectrum queue: gather the submissions' rows, scatter the results (HBM copies)
// ----------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_queue_gather(const QueueItem* __restrict__ items,
                                                      int64_t n, int gather_x,
                                                      double* __restrict__ x_rows,
                                                      double* __restrict__ y_rows,
                                                      double* __restrict__ sb) {
    const int s = blockIdx.y;
    const QueueItem it = items[s];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        sb[2 * s] = it.sb0;
        sb[2 * s + 1] = it.sb1;
    }
    double* yr = y_rows + (size_t)s * n;
    double* xr = x_rows + (size_t)s * n;
    // consecutive threads copy consecutive points: every load and store coalesces
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        yr[i] = it.y[i];
        if (gather_x) xr[i] = it.x[i];
    }
}

__global__ __launch_bounds__(256) void k_queue_scatter(const QueueItem* __restrict__ items,
                                                       const double* __restrict__ out,
                                                       int64_t stage_cap,
                                                       const int32_t* __restrict__ counts,
                                                       const double* __restrict__ mse,
                                                       const int32_t* __restrict__ status) {
    const int s = blockIdx.x;
    const QueueItem it = items[s];
    const int32_t cnt = counts[s];
    const int64_t rows = cnt < 0 ? 0 : (cnt < it.cap ? cnt : it.cap);
    if (threadIdx.x == 0) {
        *it.count = cnt;
        *it.mse = mse[s];
        const int32_t st = status[s];
        *it.status = (st == MDG_OK && cnt > it.cap) ? MDG_CAPACITY : st;
    }
    const double* src = out + 3 * (size_t)s * stage_cap;
    for (int64_t i = threadIdx.x; i < 3 * rows; i += blockDim.x) it.out[i] = src[i];
}

void launch_queue_gather(const QueueItem* items, int B, int64_t n, int gather_x, double* x_rows,
                         double* y_rows, double* sb, hipStream_t st) {
    const unsigned gx = std::max(1u, std::min(cdiv(n, 1024), 64u));
    hipLaunchKernelGGL(k_queue_gather, dim3(gx, B), dim3(256), 0, st, items, n, gather_x, x_rows,
                       y_rows, sb);
}
void launch_queue_scatter(const QueueItem* items, int B, const double* out, int64_t stage_cap,
                          const int32_t* counts, const double* mse, const int32_t* status,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_queue_scatter, dim3(B), dim3(256), 0, st, items, out, stage_cap, counts,
                       mse, status);
}

// Compact host rows (mdg_deconvolute_rows_i32) decoded into the staging rows, bit for
// bit what the Bruker reader builds on the host (bruker.rs:278-280, :459-470):
// x_i = maximum - (i * width) / divisor in that operation order (three IEEE
// operations, none contracted: the build has -ffp-contract=off), and y_i = raw_i *
// scale (int32 -> f64 exact, scale a power of two: exact). desc holds per spectrum
// {maximum, width, divisor, scale}; only the first spectrum's axis when shared_x.
__global__ __launch_bounds__(256) void k_decode_rows_i32(const int32_t* __restrict__ raw,
                                                         const double* __restrict__ desc, int64_t n,
                                                         int shared_x, double* __restrict__ x_rows,
                                                         double* __restrict__ y_rows) {
    const int s = blockIdx.y;
    const double mx = desc[4 * s], wd = desc[4 * s + 1], dv = desc[4 * s + 2], sc = desc[4 * s + 3];
    const int32_t* r = raw + (size_t)s * n;
    double* yr = y_rows + (size_t)s * n;
    double* xr = x_rows + (size_t)s * n;
    const bool do_x = !shared_x || s == 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        yr[i] = (double)r[i] * sc;
        if (do_x) xr[i] = mx - ((double)i * wd) / dv;
    }
}
void launch_decode_rows_i32(const int32_t* raw, const double* desc, int B, int64_t n, int shared_x,
                            double* x_rows, double* y_rows, hipStream_t st) {
    const unsigned gx = std::max(1u, std::min(cdiv(n, 1024), 128u));
    hipLaunchKernelGGL(k_decode_rows_i32, dim3(gx, B), dim3(256), 0, st, raw, desc, n, shared_x,
                       x_rows, y_rows);
}
// the same decode from the rows in host memory (BatchArgs::dec_rows), for pipelines
// whose smoother cannot decode them while it runs (chain_decode)
__global__ __launch_bounds__(256) void k_decode_rows_zc(BatchArgs a) {
    const int s = blockIdx.y;
    const double* d = a.dec_desc + 4 * s;
    const int32_t* __restrict__ r = a.dec_rows[s];
    double* yr = const_cast<double*>(a.y) + (size_t)s * a.y_stride;
    double* xr = const_cast<double*>(a.x) + (size_t)s * a.x_stride;
    const bool do_x = a.x_stride != 0 || s == 0;
    constexpr int U = 8;
    for (int64_t b0 = (int64_t)blockIdx.x * 256 * U; b0 < a.N; b0 += (int64_t)gridDim.x * 256 * U) {
        int32_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // host reads in flight together
            const int64_t i = b0 + u * 256 + threadIdx.x;
            v[u] = i < a.N ? r[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = b0 + u * 256 + threadIdx.x;
            if (i < a.N) {
                yr[i] = (double)v[u] * d[3];
                if (do_x) xr[i] = dec_x(d, i);
            }
        }
    }
}
void launch_decode_rows_zc(const BatchArgs& a, hipStream_t st) {
    const unsigned gx = std::max(1u, std::min(cdiv(a.N, 2048), 64u));
    hipLaunchKernelGGL(k_decode_rows_zc, dim3(gx, a.B), dim3(256), 0, st, a);
}

}  // namespace mdg

#ifdef MDG_DIAG
// diagnostic builds only (make diag): device buffer for kernel phase stamps
extern "C" int mdg_debug_set_diag(void* dev_ptr) {
    return hipMemcpyToSymbol(HIP_SYMBOL(mdg::g_diag), &dev_ptr, sizeof(dev_ptr)) == hipSuccess ? 0
                                                                                                : 100;
}
#endif
