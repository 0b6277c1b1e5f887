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
constexpr int kMaxIgnore = 16;                               // ignore regions per call

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

// ---- Rust `f64 as usize` (saturating, NaN -> 0) -------------------------------
MDG_HD inline int64_t as_index(double v) {
    if (!(v > 0.0)) return 0;
    if (v >= 9.2e18) return INT64_MAX;
    return (int64_t)v;
}

}  // namespace mdg
