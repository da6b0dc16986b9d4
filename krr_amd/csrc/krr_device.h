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
__device__ __forceinline__ uint64_t okey(uint64_t u) {
    // x ^ (sign ? all ones : sign bit only): one arithmetic shift, one or, two xors
    const uint32_t hi = (uint32_t)(u >> 32);
    const uint32_t m = (uint32_t)((int32_t)hi >> 31);
    return ((uint64_t)(hi ^ (m | 0x80000000u)) << 32) | (uint32_t)((uint32_t)u ^ m);
}
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

// ---- wave64 DPP primitives -------------------------------------------------
// Inclusive scans run on DPP row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast15 / row_bcast31 carry row totals across rows (GFX9-family DPP, which
// gfx950 keeps); broadcasts from a uniform lane are v_readlane.  Nothing here
// needs a ds_bpermute address register, so no lane-address VGPRs get hoisted
// into the kernels' loops.
constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114, kDppRowShr8 = 0x118;
constexpr int kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143;

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp32(uint32_t ident, uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)x, CTRL, ROW_MASK, 0xF, false);
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp64(uint64_t ident, uint64_t x) {
    const uint32_t lo = dpp32<CTRL, ROW_MASK>((uint32_t)ident, (uint32_t)x);
    const uint32_t hi = dpp32<CTRL, ROW_MASK>((uint32_t)(ident >> 32), (uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

struct OpAdd32 {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};
struct OpMinU64 {
    __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return b < a ? b : a; }
};
struct OpMaxU64 {
    __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return b > a ? b : a; }
};

// Inclusive scan over lanes 0..63 (lane l gets op over lanes 0..l).
template <class Op>
__device__ __forceinline__ uint32_t wave_scan32(uint32_t x, uint32_t ident, Op op) {
    x = op(x, dpp32<kDppRowShr1, 0xF>(ident, x));
    x = op(x, dpp32<kDppRowShr2, 0xF>(ident, x));
    x = op(x, dpp32<kDppRowShr4, 0xF>(ident, x));
    x = op(x, dpp32<kDppRowShr8, 0xF>(ident, x));
    x = op(x, dpp32<kDppRowBcast15, 0xA>(ident, x));
    x = op(x, dpp32<kDppRowBcast31, 0xC>(ident, x));
    return x;
}
template <class Op>
__device__ __forceinline__ uint64_t wave_scan64(uint64_t x, uint64_t ident, Op op) {
    x = op(x, dpp64<kDppRowShr1, 0xF>(ident, x));
    x = op(x, dpp64<kDppRowShr2, 0xF>(ident, x));
    x = op(x, dpp64<kDppRowShr4, 0xF>(ident, x));
    x = op(x, dpp64<kDppRowShr8, 0xF>(ident, x));
    x = op(x, dpp64<kDppRowBcast15, 0xA>(ident, x));
    x = op(x, dpp64<kDppRowBcast31, 0xC>(ident, x));
    return x;
}

// Value of x in (wave-uniform) lane src, as a scalar.
__device__ __forceinline__ uint32_t lane_bcast32(uint32_t x, int src) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, src);
}
__device__ __forceinline__ uint64_t lane_bcast64(uint64_t x, int src) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
    return lane_bcast32(wave_scan32(x, 0u, OpAdd32{}), kWave - 1);
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
    return lane_bcast64(wave_scan64(x, 0ull, OpMaxU64{}), kWave - 1);
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t x) {
    return lane_bcast64(wave_scan64(x, ~0ull, OpMinU64{}), kWave - 1);
}
// Inclusive suffix sum over lanes: lane l gets sum_{m >= l} x_m.
__device__ __forceinline__ uint32_t wave_suffix_incl(uint32_t x, int lane) {
    (void)lane;
    const uint32_t incl = wave_scan32(x, 0u, OpAdd32{});
    return lane_bcast32(incl, kWave - 1) - incl + x;
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

// The index rule k(n) of krr_percentile_params: the caller's k_table entry (the
// reference's own int((n-1) * p / 100) for p whose product it rounds), clamped into
// [0, n-1], else the exact floor.  n past the table: the table's last entry (the ABI
// checks the longest segment against the table; queries flag it, rule_covers).
__device__ __forceinline__ int64_t rule_rank(int64_t n, int64_t p_num, int64_t p_den, const int64_t* tab,
                                             int64_t tab_len) {
    if (!tab) return exact_rank(n, p_num, p_den);
    int64_t k = tab[n < tab_len ? n : tab_len - 1];
    k = k < 0 ? 0 : k;
    return k > n - 1 ? n - 1 : k;
}
__device__ __forceinline__ bool rule_covers(int64_t n, const int64_t* tab, int64_t tab_len) {
    return !tab || n < tab_len;
}

}  // namespace krr
