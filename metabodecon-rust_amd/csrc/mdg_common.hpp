// mdg_common.hpp -- helpers shared by host and device code of libmdgpu.
//
// Everything here is exact integer work or single IEEE-754 binary64 operations,
// so host and device produce identical bits. The library is compiled with
// -ffp-contract=off: rustc never contracts a*b+c into an FMA, so neither may we.
#pragma once

#include <cstddef>
#include <cstdint>

#ifndef MDG_HD
#if defined(__HIPCC__)
#define MDG_HD __host__ __device__
#else
#define MDG_HD
#endif
#endif

namespace mdg {

// lib.rs:277  CHECK_PRECISION = 1.0e+3 * f64::EPSILON
constexpr double kCheckPrecision = 1.0e+3 * 2.220446049250313080847e-16;
constexpr double kEpsilon = 2.220446049250313080847e-16;  // f64::EPSILON
constexpr int kIgnoreRow = 64;  // ignore-region pairs per spectrum row, grown in steps of this
constexpr int kPkSlotWords = 64;   // k_peaks: mask words per look-back slot (the finest chunk)
constexpr int kDecRowAlign = 16;  // doubles: decoded staging rows start on 128-byte lines (chain_decode)
constexpr int kDecChunks = 64;     // chunks per row the chain launch's decoders publish (Workspace::dec_flags)
constexpr int kMseMaxParts = 2048;  // MSE partial sums per spectrum (workspace rows)

// ---- counter-based splitmix64 (synthetic workload only) ----------------------
MDG_HD inline uint64_t mix64(uint64_t z) {
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}
MDG_HD inline uint64_t stream_key(uint64_t seed, uint64_t stream) {
    return mix64(seed * 0x9E3779B97F4A7C15ull + stream * 0xD1B54A32D192ED03ull + 1ull);
}
MDG_HD inline uint64_t draw(uint64_t key, uint64_t counter) {
    return mix64(key + (counter + 1ull) * 0x9E3779B97F4A7C15ull);
}
MDG_HD inline double u53(uint64_t r) { return (double)(r >> 11) * 0x1.0p-53; }
MDG_HD inline double u48(uint64_t r) { return (double)(r >> 16) * 0x1.0p-48; }

// Irwin-Hall(12) approximate normal; exact in binary64 (12 * 2^48 < 2^53).
MDG_HD inline double synth_noise(uint64_t key, uint64_t i, double sigma) {
    double s = 0.0;
    for (int k = 0; k < 12; ++k) s += u48(draw(key, i * 12ull + (uint64_t)k));
    return sigma * (s - 6.0);
}

constexpr uint64_t kStreamPeaks = 1;
constexpr uint64_t kStreamNoise = 2;

// ---- division hard cases (test support) ---------------------------------------
// Operand pairs whose exact quotient lies as close to a rounding midpoint as two
// binary64 values allow (|n/d - m| = ulp(q) / (2 D) with D the divisor's 53-bit
// odd significand, i.e. about 2^-53 ulp). For odd D and r = +-1, the odd M
// solving M*D == r (mod 2^k) gives N = (M*D - r) / 2^k, so N/D = M/2^k - r/(D 2^k)
// with M/2^k a midpoint of the quotient's binade. k = 54 puts the quotient in
// [1/2, 1) (M in [2^53, 2^54)), k = 53 in [1, 2) (M = u + 2^53). Candidates
// whose N does not fit 53 bits are reported as invalid (*ok = false).
MDG_HD inline uint64_t inv_odd64(uint64_t d) {  // d^-1 mod 2^64 (Newton, d odd)
    uint64_t x = d;                              // correct to 3 bits
    for (int i = 0; i < 5; ++i) x *= 2ull - d * x;
    return x;
}
MDG_HD inline uint64_t umulhi64(uint64_t a, uint64_t b) {
    const uint64_t a0 = a & 0xffffffffull, a1 = a >> 32, b0 = b & 0xffffffffull, b1 = b >> 32;
    const uint64_t p00 = a0 * b0, p01 = a0 * b1, p10 = a1 * b0, p11 = a1 * b1;
    const uint64_t mid = (p00 >> 32) + (p01 & 0xffffffffull) + (p10 & 0xffffffffull);
    return p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
}
MDG_HD inline double ldexp_int(uint64_t m, int e) {  // m < 2^53, |e| <= 1000: exact
    double v = (double)m;
    while (e > 500) { v *= 0x1p500; e -= 500; }
    while (e < -500) { v *= 0x1p-500; e += 500; }
    const uint64_t bits = (uint64_t)(e + 1023) << 52;
    double s;
    __builtin_memcpy(&s, &bits, 8);
    return v * s;
}
// The i-th hard pair of stream `seed`; exponents keep n, d and n/d inside the
// fast-division range [2^-200, 2^200] (no div_scale scaling).
MDG_HD inline void division_hard_case(uint64_t seed, uint64_t i, double* n, double* d, bool* ok) {
    const uint64_t h0 = mix64(seed * 0x9E3779B97F4A7C15ull + 2ull * i + 1ull);
    const uint64_t h1 = mix64(h0 ^ 0xD1B54A32D192ED03ull);
    const uint64_t D = (1ull << 52) | (h0 & ((1ull << 52) - 1)) | 1ull;  // odd, 53 bits
    const bool neg = (h1 & 1) != 0;                                       // r = -1 or +1
    const bool k54 = (h1 & 2) != 0;
    const int k = k54 ? 54 : 53;
    const uint64_t mask = (1ull << k) - 1;
    const uint64_t inv = inv_odd64(D);
    const uint64_t u = (neg ? (0ull - inv) : inv) & mask;  // u*D == r (mod 2^k)
    uint64_t M;
    if (k54) {
        if (u < (1ull << 53)) { *ok = false; *n = *d = 1.0; return; }
        M = u;
    } else {
        M = u + (1ull << 53);
    }
    // M*D - r as a 128-bit value (hi, lo); its low k bits are zero
    uint64_t lo = M * D, hi = umulhi64(M, D);
    if (neg) { lo += 1; if (lo == 0) hi += 1; } else { if (lo == 0) hi -= 1; lo -= 1; }
    const uint64_t N = (hi << (64 - k)) | (lo >> k);
    if (N >= (1ull << 53) || N == 0) { *ok = false; *n = *d = 1.0; return; }
    const int ed = (int)((h1 >> 8) % 301) - 150 - 52;  // d in [2^-150, 2^151)
    const int eq = (int)((h1 >> 24) % 61) - 30;         // quotient scale 2^eq
    *d = ldexp_int(D, ed);
    *n = ldexp_int(N, ed + eq);
    *ok = true;
}

// ---- Rust `f64 as usize` (saturating, NaN -> 0) -------------------------------
MDG_HD inline int64_t as_index(double v) {
    if (!(v > 0.0)) return 0;
    if (v >= 9.2e18) return INT64_MAX;
    return (int64_t)v;
}

}  // namespace mdg
