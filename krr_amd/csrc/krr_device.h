// krr_device.h — wave64 device primitives shared by the KRR hot-path kernels (gfx950).
//
// Everything here is written for one 64-lane wavefront that owns one segment:
// cross-lane work uses ballot / mbcnt / shuffles, never warp-32 idioms.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace krr {

constexpr int kWave = 64;
constexpr uint64_t kSignBit = 0x8000000000000000ull;
constexpr uint64_t kQuietNaN = 0x7FF8000000000000ull;

__device__ __forceinline__ uint64_t dbits(double v) { return (uint64_t)__double_as_longlong(v); }
__device__ __forceinline__ double bitsd(uint64_t u) { return __longlong_as_double((long long)u); }

// NaN <=> exponent all ones and mantissa non-zero.
__device__ __forceinline__ bool is_nan_bits(uint64_t u) { return (u << 1) > 0xFFE0000000000000ull; }
// +0.0 or -0.0
__device__ __forceinline__ bool is_zero_bits(uint64_t u) { return (u << 1) == 0; }

// Order-preserving key: for non-NaN a, b:  a <_IEEE b  <=>  okey(a) < okey(b), with -0 < +0.
__device__ __forceinline__ uint64_t okey(uint64_t u) { return (u & kSignBit) ? ~u : (u | kSignBit); }
__device__ __forceinline__ uint64_t okey_inv(uint64_t k) { return (k & kSignBit) ? (k ^ kSignBit) : ~k; }

// Force a value the program knows is wave-uniform into scalar registers.
__device__ __forceinline__ uint32_t uni32(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Number of set bits of m in lanes strictly below this lane.
__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o);
    return uni32(x);
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint64_t y = (uint64_t)__shfl_xor((unsigned long long)x, o);
        x = y > x ? y : x;
    }
    return uni64(x);
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint64_t y = (uint64_t)__shfl_xor((unsigned long long)x, o);
        x = y < x ? y : x;
    }
    return uni64(x);
}
// Inclusive suffix sum over lanes: lane l gets sum_{m >= l} x_m.
__device__ __forceinline__ uint32_t wave_suffix_incl(uint32_t x, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t y = (uint32_t)__shfl_down((int)x, d);
        if (lane + d < kWave) x += y;
    }
    return x;
}

// k = floor((n-1) * p_num / (100 * p_den)) exactly (n >= 1, 0 < p <= 100, p_den <= 1e15).
// This is the reference's int((len(data_) - 1) * cpu_percentile / 100) (simple.py:36)
// evaluated without rounding.
__device__ __forceinline__ int64_t exact_rank(int64_t n, int64_t p_num, int64_t p_den) {
    const uint64_t a = (uint64_t)(n - 1);
    const uint64_t den = 100ull * (uint64_t)p_den;
    const unsigned __int128 num = (unsigned __int128)a * (uint64_t)p_num;
    uint64_t k = (uint64_t)((double)a * ((double)p_num / (double)den));
    if (k > a) k = a;
    while (k < a && (unsigned __int128)(k + 1) * den <= num) ++k;
    while (k > 0 && (unsigned __int128)k * den > num) --k;
    return (int64_t)k;
}

}  // namespace krr
