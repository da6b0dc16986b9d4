// krr_kll.h — KLL sketch, row format 2: a compactor hierarchy with a DETERMINISTIC schedule,
// an exact top tail, and a bounded fold (config 5 sketch mode; included by krr_kernels.hip after
// the streaming skeleton).  The specification, word for word, is oracle/kll_ref.py; rows and
// answers are compared with it bit for bit (tests/test_gpu_kll.py).
//
// north_star names "an optional mergeable t-digest/KLL sketch mode" whose rank error is
// reported.  Three properties make it fit for that:
//  * deterministic schedule — a compaction takes an EVEN number of equal-weight keys (an odd
//    largest key is SET ASIDE in its level's odd slot first), so every level's key count, and
//    sum w^2, depend on the presence pattern only, never on coins or values: the Azuma-Hoeffding
//    bound holds as written, and weight is conserved exactly (body weight == n);
//  * exact tail — the `tail` largest present keys are kept exactly, so any rank within `tail`
//    of the top (p99 of 172,800 samples needs 1,729) is answered with no error;
//  * bounded fold — krr_kll_merge folds W rows into ONE row of the same size (tails: the largest
//    `tail` of the union; body: levels unioned, then compacted from level 0 up until `budget`
//    keys remain), so a new slice folds into an old state without the old data.
//
// Build, one wave per series slice, one HBM pass (1,024-slot chunks; lane l holds slots
// u*128 + 2l + h):
//   level 0  every chunk, per lane: slot pair u (a double2 load) with both samples present ->
//            one 2-key compaction (coin bit u); a lone present sample -> the lane's level-0 odd slot;
//   level 1  odd chunks: the lane's pending 8 and new 8 weight-2 keys sorted (16-key bitonic
//            network), odd largest set aside, compacted -> <= 8 weight-4 keys;
//   level 2, 3  every 4th / 8th chunk: two runs of <= 8 merged (bitonic merge 16), compacted;
//   level 4  every 8th chunk, the wave: 64 lanes x 8 weight-16 keys sorted across the wave
//            (DPP / swizzle exchanges), compacted into a run of <= 256 weight-32 keys;
//   h >= 5   one LDS run per level; a run pushed onto an occupied level is merged with it
//            (merge-path positions), the odd largest set aside, compacted and carried up.
// An odd slot that receives a second key makes a 2-key compaction whose kept key goes to the
// next level's slot (per lane below level 4, per wave above).  The tail: candidates above a
// running threshold tau are appended to an LDS buffer; when it fills, tau rises to a sampled
// pivot that keeps >= `tail` keys (counted exactly, ties kept by count).  At the end: flush by
// all-absent chunks to a multiple of 8, the tail sorted and its top `tail` exported, the body
// compacted from level 0 up until `budget` keys remain, each level exported ascending.
#pragma once

#ifndef KRR_KLL_STREAM
#define KRR_KLL_STREAM 0  // streaming loop form (kll_stream): 0 one chunk ahead, 1 ping-pong, 2 two ahead
#endif

namespace krr {

constexpr int kKllHdr = 16;
constexpr int kKllLevels = 24;
constexpr int kKllRun = 256;
constexpr int kKllFirstRun = 5;
constexpr uint32_t kKllTailSlack = 128;  // a refresh leaves <= tail + slack keys in the buffer
constexpr uint32_t kKllWsWords = 576;     // final stage: one level's keys (<= 513)
constexpr uint32_t kKllFinalWords = kKllWsWords + 256;  // + the carry (<= 256), from tmp on
// coin tags (oracle/kll_ref.py T_*)
constexpr uint32_t kT_L0 = 0x100, kT_L1 = 0x200, kT_L2 = 0x300, kT_L3 = 0x400, kT_LODD = 0x800, kT_WAVE = 0x1000,
                   kT_RUN = 0x1100, kT_WODD = 0x1200, kT_FINAL = 0x1300, kT_FOLD = 0x2000;
constexpr uint64_t kKllInfBits = 0x7FF0000000000000ull;
// row flags (word 15)
constexpr uint64_t kKllRowOverflow = 1;  // a level past the provisioned runs (never expected): row unusable

__host__ __device__ inline uint64_t kll_mix64(uint64_t z) {  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t kll_slice_base(uint64_t seed, uint64_t series, uint64_t slc) {
    return kll_mix64(seed + 0x9E3779B97F4A7C15ull * (series + 1) + 0xD1B54A32D192ED03ull * (slc + 1));
}
__host__ __device__ inline uint32_t kll_fmix32(uint32_t h) {  // murmur3 finaliser
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    return h ^ (h >> 16);
}
// 32 coin bits of event (tag, idx) of the slice (or fold epoch) keyed by `base`.
__host__ __device__ inline uint32_t kll_coin32(uint64_t base, uint32_t tag, uint32_t idx) {
    return kll_fmix32((uint32_t)base ^ kll_fmix32((uint32_t)(base >> 32) + tag * 0x9E3779B9u + idx * 0x85EBCA6Bu));
}

// Chunks stream_segment delivers for [beg, end) (the same arithmetic).
__host__ __device__ inline int64_t kll_nchunks(int64_t beg, int64_t end) {
    int64_t a0 = (beg + 1) & ~(int64_t)1;
    if (a0 > end) a0 = end;
    int64_t a1 = end & ~(int64_t)1;
    if (a1 < a0) a1 = a0;
    const int64_t nunits = (a1 - a0) >> 1, CH = (int64_t)kUnroll * kWave;
    const int64_t nfull = nunits / CH, rem = nunits - nfull * CH;
    return nfull + ((rem > 0 || a0 > beg || a1 < end) ? 1 : 0);
}

// Run levels (5 ..) a segment of `len` slots can fill: one push at level 5 per 8 chunks,
// a binary counter above it.
__host__ __device__ inline int kll_run_levels(int64_t len) {
    const int64_t pushes = (kll_nchunks(0, len) + 7) / 8;
    int lg = 0;
    while ((int64_t(1) << (lg + 1)) <= pushes) ++lg;
    return lg + 1;
}

// ---- sorting networks on f64 keys (no NaN; -0 folded into +0, so min/max order totally) ----
__device__ __forceinline__ void kll_cxd(double& a, double& b) {  // ascending
    const double lo = fmin(a, b), hi = fmax(a, b);
    a = lo;
    b = hi;
}

// c ? b : a as a bit blend: a select between two adjacent array elements would otherwise be
// folded into a dynamically indexed load (an array in scratch memory).
__device__ __forceinline__ double kll_pick(bool c, double a, double b) {
    uint64_t m = c ? ~0ull : 0ull;
    asm volatile("" : "+v"(m));
    return bitsd((dbits(a) & ~m) | (dbits(b) & m));
}

// x of lane ^ M (M in {1, 2, 4, 8, 16}: never across the 32-lane halves): DPP quad_perm for
// 1 and 2, DPP row_ror:8 for 8 (a rotation by 8 in a 16-lane row is lane ^ 8), ds_swizzle
// (bit mode, xor mask) for 4 and 16 — no address registers, no bpermute.
template <int M>
__device__ __forceinline__ uint32_t kll_xor32(uint32_t v) {
    if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);
    else if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false);
    else if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x128, 0xF, 0xF, false);
    else return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (M << 10));
}
template <int M>
__device__ __forceinline__ double kll_xord(double d) {
    const uint64_t x = dbits(d);
    if constexpr (M == 32) {  // across the 32-lane halves
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, 32, kWave);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), 32, kWave);
        return bitsd(((uint64_t)hi << 32) | lo);
    }
    return bitsd(((uint64_t)kll_xor32<M>((uint32_t)(x >> 32)) << 32) | kll_xor32<M>((uint32_t)x));
}
#ifndef KRR_KLL_X_SLOWCROSS
// (key of the pair's lower lane, key of its upper lane) in every lane, for the pairs
// lane ^ 16 and lane ^ 32, by gfx950's v_permlane16_swap / v_permlane32_swap: a VALU row swap
// of a register with itself — no LDS, no address registers.
template <int M>
__device__ __forceinline__ void kll_pair_swap(double x, double& a, double& b) {
    const uint64_t u = dbits(x);
    const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    if constexpr (M == 32) {
        const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        a = bitsd(((uint64_t)h[0] << 32) | l[0]);
        b = bitsd(((uint64_t)h[1] << 32) | l[1]);
    } else {
        const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        a = bitsd(((uint64_t)h[0] << 32) | l[0]);
        b = bitsd(((uint64_t)h[1] << 32) | l[1]);
    }
}
#endif
template <int M, int N>
__device__ __forceinline__ void kll_cross(double (&x)[N], bool take_min) {
#ifndef KRR_KLL_X_SLOWCROSS
    if constexpr (M == 16 || M == 32) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double a, b;
            kll_pair_swap<M>(x[i], a, b);
            x[i] = ((b < a) != take_min) ? a : b;  // take_min: the smaller of the pair
        }
        return;
    }
#endif
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double o = kll_xord<M>(x[i]);
#ifndef KRR_KLL_X_SLOWCROSS
        // one compare and a select: keep x when (o < x) differs from take_min (keys hold no NaN
        // and no -0, so either side of a tie is the same key)
        x[i] = ((o < x[i]) != take_min) ? x[i] : o;
#else
        x[i] = take_min ? fmin(x[i], o) : fmax(x[i], o);
#endif
    }
}

#ifndef KRR_KLL_BATCHER
#define KRR_KLL_BATCHER 1  // Batcher's odd-even networks (63 / 25 compare-exchanges) instead of bitonic (80 / 32)
#endif
#if KRR_KLL_BATCHER
// Batcher's odd-even merge sort of 16 and odd-even merge of two sorted 8-runs, as (i, j)
// compare-exchange pairs (scripts-free: both checked on all 2^16 0-1 inputs, the 0-1 principle).
// Any sorting network leaves the same ascending keys (no NaN, -0 folded), so rows do not change.
constexpr int kKllSort16[126] = {0, 1, 2, 3, 0, 2, 1, 3, 1, 2, 4, 5, 6, 7, 4, 6, 5, 7, 5, 6, 0, 4, 2, 6, 2, 4, 1, 5, 3, 7, 3, 5, 1, 2, 3, 4, 5, 6, 8, 9, 10, 11, 8, 10, 9, 11, 9, 10, 12, 13, 14, 15, 12, 14, 13, 15, 13, 14, 8, 12, 10, 14, 10, 12, 9, 13, 11, 15, 11, 13, 9, 10, 11, 12, 13, 14, 0, 8, 4, 12, 4, 8, 2, 10, 6, 14, 6, 10, 2, 4, 6, 8, 10, 12, 1, 9, 5, 13, 5, 9, 3, 11, 7, 15, 7, 11, 3, 5, 7, 9, 11, 13, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14};
constexpr int kKllMerge16[50] = {0, 8, 4, 12, 4, 8, 2, 10, 6, 14, 6, 10, 2, 4, 6, 8, 10, 12, 1, 9, 5, 13, 5, 9, 3, 11, 7, 15, 7, 11, 3, 5, 7, 9, 11, 13, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14};
__device__ __forceinline__ void kll_sort16(double (&x)[16]) {
#pragma unroll
    for (int c = 0; c < 63; ++c) kll_cxd(x[kKllSort16[2 * c]], x[kKllSort16[2 * c + 1]]);
}
__device__ __forceinline__ void kll_merge16(double (&z)[16]) {
#pragma unroll
    for (int c = 0; c < 25; ++c) kll_cxd(z[kKllMerge16[2 * c]], z[kKllMerge16[2 * c + 1]]);
}
#else
// The lane's 16 keys ascending (a full bitonic sort in registers).
__device__ __forceinline__ void kll_sort16(double (&x)[16]) {
#pragma unroll
    for (int k = 2; k <= 16; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (!(i & j)) {
                    if (k == 16 || (i & k) == 0) kll_cxd(x[i], x[i + j]);
                    else kll_cxd(x[i + j], x[i]);
                }
        }
    }
}

// z[0, 8) and z[8, 16) ascending -> z ascending (reverse the second half: bitonic; clean).
__device__ __forceinline__ void kll_merge16(double (&z)[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double t = z[8 + i];
        z[8 + i] = z[15 - i];
        z[15 - i] = t;
    }
#pragma unroll
    for (int j = 8; j > 0; j >>= 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (!(i & j)) kll_cxd(z[i], z[i + j]);
    }
}
#endif

// 512 keys ascending across the wave: lane l holds positions 8l .. 8l+7, each lane's 8
// already ascending (odd lanes' runs are reversed first, so stage 16 starts bitonic).
__device__ __forceinline__ void kll_sort512(double (&y)[8], int lane) {
    if (lane & 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const double t = y[i];
            y[i] = y[7 - i];
            y[7 - i] = t;
        }
    }
#pragma unroll 1
    for (uint32_t k = 16; k <= 512; k <<= 1) {
        const bool asc = k >= 512 || (((uint32_t)lane * 8u) & k) == 0;
#ifndef KRR_KLL_X_NONEG
        // a descending block is sorted ascending on negated keys (the sign bit flipped, and
        // flipped back after the stage): every compare-exchange of the stage is ascending
        const uint32_t neg = asc ? 0u : 0x80000000u;
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = bitsd(dbits(y[i]) ^ ((uint64_t)neg << 32));
#endif
#pragma unroll 1
        for (uint32_t j = k >> 1; j >= 8; j >>= 1) {
            const int m = (int)(j >> 3);
#ifndef KRR_KLL_X_NONEG
            const bool take_min = (lane & m) == 0;
#else
            const bool take_min = ((lane & m) == 0) == asc;
#endif
            switch (m) {  // wave-uniform
                case 1: kll_cross<1, 8>(y, take_min); break;
                case 2: kll_cross<2, 8>(y, take_min); break;
                case 4: kll_cross<4, 8>(y, take_min); break;
                case 8: kll_cross<8, 8>(y, take_min); break;
                case 16: kll_cross<16, 8>(y, take_min); break;
                default: kll_cross<32, 8>(y, take_min); break;
            }
        }
#pragma unroll
        for (int j = 4; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (!(i & j)) {
#ifndef KRR_KLL_X_NONEG
                    kll_cxd(y[i], y[i + j]);
#else
                    if (asc) kll_cxd(y[i], y[i + j]);
                    else kll_cxd(y[i + j], y[i]);
#endif
                }
        }
#ifndef KRR_KLL_X_NONEG
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = bitsd(dbits(y[i]) ^ ((uint64_t)neg << 32));
#endif
    }
}

// One key per lane, ascending over the 64 lanes (refresh samples).
__device__ __forceinline__ double kll_sort64(double v, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t x = dbits(v);
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, j, kWave);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), j, kWave);
            const double o = bitsd(((uint64_t)hi << 32) | lo);
            const bool asc = (lane & k) == 0 || k == 64;
            const bool lower = (lane & j) == 0;
            v = (lower == asc) ? fmin(v, o) : fmax(v, o);
        }
    }
    return v;
}

// Ascending sort of a[0, n) in LDS by one wave, any n: bitonic with the flip first step (every
// block sorted ascending), so the virtual +inf past n never moves and its pairs are skipped.
__device__ void kll_lds_sort(uint64_t* a, uint32_t n, int lane) {
    if (n < 2) return;
    uint32_t P = 1;
    while (P < n) P <<= 1;
#pragma unroll 1
    for (uint32_t k = 2; k <= P; k <<= 1) {
#pragma unroll 1
        for (uint32_t j = k >> 1; j >= 1; j >>= 1) {
            const bool flip = j == (k >> 1);
#pragma unroll 1
            for (uint32_t t = lane; t < (P >> 1); t += kWave) {
                const uint32_t i = ((t & ~(j - 1)) << 1) | (t & (j - 1));
                const uint32_t p = flip ? (i ^ (k - 1)) : (i + j);
                if (p < n) {
                    const double x = bitsd(a[i]), y = bitsd(a[p]);
                    a[i] = dbits(fmin(x, y));
                    a[p] = dbits(fmax(x, y));
                }
            }
            __syncthreads();
        }
    }
}

// #{i < n : a[i] < v} (STRICT) or #{a[i] <= v} of an ascending LDS / global array.
template <bool STRICT>
__device__ __forceinline__ uint32_t kll_bound(const uint64_t* a, uint32_t n, double v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const double y = bitsd(a[mid]);
        if (STRICT ? y < v : y <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Merge-compaction step: every key X[i] (i = lane + 64 q, i < nx <= 256) lands at merged
// position p = i + #(Y < X[i]) (STRICT: X's keys go first among equal keys) or i + #(Y <= X[i]);
// positions p < lim with p = off, off + 2, ... are kept at O[(p - off) / 2].  The four binary
// searches of a lane advance together (their LDS reads overlap), 9 halvings each (ny <= 256).
template <bool STRICT>
__device__ __forceinline__ void kll_merge_half(const uint64_t* X, uint32_t nx, const uint64_t* Y, uint32_t ny,
                                               uint32_t off, uint32_t lim, uint64_t* O, int lane) {
    constexpr int Q = kKllRun / kWave;
    uint64_t v[Q];
    uint32_t lo[Q], hi[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint32_t i = (uint32_t)lane + (uint32_t)q * kWave;
        v[q] = i < nx ? X[i] : 0ull;
        lo[q] = 0;
        hi[q] = i < nx ? ny : 0u;
    }
    if (ny) {
        const uint32_t last = ny - 1;
#pragma unroll
        for (int step = 0; step < 9; ++step) {
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const uint32_t mid = (lo[q] + hi[q]) >> 1;
                const double y = bitsd(Y[mid < last ? mid : last]), vq = bitsd(v[q]);
                const bool active = lo[q] < hi[q];
                const bool go = STRICT ? y < vq : y <= vq;
                lo[q] = (active && go) ? mid + 1 : lo[q];
                hi[q] = (active && !go) ? mid : hi[q];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint32_t i = (uint32_t)lane + (uint32_t)q * kWave;
        const uint32_t p = i + lo[q];
        if (i < nx && p < lim && p >= off && ((p - off) & 1u) == 0) O[(p - off) >> 1] = v[q];
    }
}

// Full merge of ascending X (nx) and Y (ny), any sizes, into O (X first among equal keys;
// equal keys have equal bits, so the order is immaterial to the result).
__device__ void kll_lds_merge(const uint64_t* X, uint32_t nx, const uint64_t* Y, uint32_t ny, uint64_t* O,
                              int lane) {
#pragma unroll 1
    for (uint32_t i = lane; i < nx; i += kWave) O[i + kll_bound<true>(Y, ny, bitsd(X[i]))] = X[i];
#pragma unroll 1
    for (uint32_t j = lane; j < ny; j += kWave) O[j + kll_bound<false>(X, nx, bitsd(Y[j]))] = Y[j];
}

// Merge-compaction of two ascending runs (a, t <= 256 keys) in registers: lane l holds merged
// positions 8l .. 8l + 7 of the bitonic sequence L ascending (+inf padded to 256) followed by T
// descending (+inf first), cleaned by one bitonic merge (6 cross-lane and 3 in-lane stages);
// positions p < lim with p = off, off + 2, ... are written to O[(p - off) / 2].  Equal keys have
// equal bits (no -0: keys are folded where kept), so the order among them is immaterial, and a
// padding +inf is the same key as a real one: the first a + t positions are the merge.
__device__ __forceinline__ void kll_reg_merge(const uint64_t* L, uint32_t a, const uint64_t* T, uint32_t t,
                                              uint32_t off, uint32_t lim, uint64_t* O, int lane) {
    double x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t p = (uint32_t)lane * 8u + (uint32_t)i;
        const uint32_t q = 511u - p;
        const bool inL = p < (uint32_t)kKllRun;
        const bool have = inL ? p < a : q < t;
        x[i] = have ? bitsd(inL ? L[p] : T[q]) : __builtin_inf();
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const bool take_min = (lane & m) == 0;
        switch (m) {
            case 32: kll_cross<32, 8>(x, take_min); break;
            case 16: kll_cross<16, 8>(x, take_min); break;
            case 8: kll_cross<8, 8>(x, take_min); break;
            case 4: kll_cross<4, 8>(x, take_min); break;
            case 2: kll_cross<2, 8>(x, take_min); break;
            default: kll_cross<1, 8>(x, take_min); break;
        }
    }
#pragma unroll
    for (int j = 4; j > 0; j >>= 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (!(i & j)) kll_cxd(x[i], x[i + j]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t p = (uint32_t)lane * 8u + (uint32_t)i;
        if (p < lim && p >= off && ((p - off) & 1u) == 0) O[(p - off) >> 1] = dbits(x[i]);
    }
}

// Uniform build state in LDS.
struct KllShared {
    uint64_t* lv;    // runs, level h at lv + (h - kKllFirstRun) * kKllRun
    uint64_t* tmp;   // two work runs of kKllRun keys
    uint64_t* tb;    // tail buffer (tcap keys); the final compression's workspace at the end
    uint64_t* wk;    // [kKllLevels] wave odd-slot keys
    uint32_t* lens;  // [kKllLevels] run lengths
    uint32_t* rcnt;  // [kKllLevels] run merge-compactions per level
    uint32_t* wcnt;  // [kKllLevels] wave odd-pair compactions per level
    uint32_t* misc;  // [0] wave odd-slot presence bits  [1] overflow
};

struct KllBuildArgs {
    const double* vals;
    const int64_t* offs;
    int64_t S;
    int32_t gaps;
    int32_t budget;
    int32_t tail;
    int32_t nrl;      // run levels in LDS: kKllFirstRun .. kKllFirstRun + nrl - 1
    uint32_t tcap;    // tail buffer / workspace keys
    uint32_t slice;
    uint64_t seed;
    int64_t seg_base;
    uint64_t* rows;   // [S][kKllHdr + budget + tail]
    int32_t tail_pass;  // the tail is left to k_kll_tail (zero tail words, word 6 = 0)
    uint32_t* lines;    // LINES builds: per series, per chunk, 64 line maxima (kll_line_key)
    int64_t line_stride;  // u32 words per series in `lines`
};

// ---- line maxima: where the exact tail's keys can be (the sparse tail pass) ----
// A "line" is 16 slots = 128 contiguous bytes = the double2 of 8 consecutive lanes in one row
// u of a chunk.  Its key: the top 32 bits of the ordered key (okey) of the line's largest
// sample, plus one — an upper bound of okey(x) >> 32 for every x in the line, in 5 VALU (no
// rounding test, no NaN test: a NaN slot only makes its line's key large, so the tail pass
// reads that line and finds no candidate in the NaN).  A line whose key is below
// okey(tau) >> 32 holds no sample > tau.  (+1 wraps to 0 only for NaN bit patterns, and a
// wrapped lane never lowers its line's maximum below a real sample's key.)
__device__ __forceinline__ uint32_t kll_line_key(double hi) {
    const uint32_t h = (uint32_t)(dbits(hi) >> 32);
    const uint32_t m = (uint32_t)((int32_t)h >> 31);
    return (h ^ (m | 0x80000000u)) + 1u;
}

// max over each group of 8 consecutive lanes, in every lane of the group (DPP quad_perm
// [1,0,3,2], [2,3,0,1], then row_half_mirror: lane i <-> 7 - i within 8)
__device__ __forceinline__ uint32_t kll_max8(uint32_t k) {
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0xB1, 0xF, 0xF, false));
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0x4E, 0xF, 0xF, false));
    k = max(k, (uint32_t)__builtin_amdgcn_update_dpp((int)k, (int)k, 0x141, 0xF, 0xF, false));
    return k;
}

// ---- wave-level pieces, free functions of value arguments (the per-wave state below stays in
// registers: nothing of it is ever address-taken) ----

// A set-aside key at wave level h (>= 4): stored in the level's odd slot, or compacted with the
// key already there (coin) and carried up.  Returns the sum of w^2 it added.
__device__ uint64_t kll_wave_odd(KllShared sh, uint64_t base, uint32_t h, double v, int lane) {
    uint64_t w2 = 0;
#pragma unroll 1
    while (true) {
        if (h >= (uint32_t)kKllLevels) {
            if (lane == 0) sh.misc[1] = 1;
            __syncthreads();
            return w2;
        }
        const uint32_t pm = uni32(sh.misc[0]);
        if (!((pm >> h) & 1u)) {
            if (lane == 0) {
                sh.wk[h] = dbits(v);
                sh.misc[0] = pm | (1u << h);
            }
            __syncthreads();
            return w2;
        }
        const double k = bitsd(uni64(sh.wk[h]));
        const uint32_t c = uni32(sh.wcnt[h]);
        const uint32_t bit = kll_coin32(base, kT_WODD + h, c) & 1u;
        v = bit ? fmax(k, v) : fmin(k, v);
        w2 += 1ull << (2 * h);
        __syncthreads();
        if (lane == 0) {
            sh.wcnt[h] = c + 1;
            sh.misc[0] = pm & ~(1u << h);
        }
        __syncthreads();
        ++h;
    }
}

// Push the run tmp[t_sel][0, t) at level h (>= 5): store it, or merge-compact and carry up.
// Returns the sum of w^2 it added.
__device__ uint64_t kll_push(KllShared sh, uint64_t base, int32_t nrl, uint32_t t_sel, uint32_t t, uint32_t h,
                             int lane) {
    uint64_t w2 = 0;
#pragma unroll 1
    while (t) {
        if ((int)h >= kKllFirstRun + nrl) {
            if (lane == 0) sh.misc[1] = 1;
            __syncthreads();
            return w2;
        }
        const uint32_t a = uni32(sh.lens[h]);
        const uint64_t* T = sh.tmp + (size_t)t_sel * kKllRun;
        uint64_t* L = sh.lv + (size_t)(h - kKllFirstRun) * kKllRun;
        if (a == 0) {
            for (uint32_t i = lane; i < t; i += kWave) L[i] = T[i];
            __syncthreads();
            if (lane == 0) sh.lens[h] = t;
            __syncthreads();
            return w2;
        }
        const uint32_t m = a + t, lim = m & ~1u;
        if (m & 1u)  // the largest key of the merge is set aside at level h
            w2 += kll_wave_odd(sh, base, h, fmax(bitsd(L[a - 1]), bitsd(T[t - 1])), lane);
        const uint32_t c = uni32(sh.rcnt[h]);
        const uint32_t off = kll_coin32(base, kT_RUN + h, c) & 1u;
        uint64_t* O = sh.tmp + (size_t)(t_sel ^ 1) * kKllRun;
#ifdef KRR_KLL_X_REGMERGE  // A/B: the register bitonic merge (same speed, more VGPRs; profiles/r04/s)
        kll_reg_merge(L, a, T, t, off, lim, O, lane);
#else  // merge-path: positions by binary searches in LDS
        kll_merge_half<true>(L, a, T, t, off, lim, O, lane);  // the run's keys before T's equal keys
        kll_merge_half<false>(T, t, L, a, off, lim, O, lane);
#endif
        w2 += 1ull << (2 * h);
        __syncthreads();
        if (lane == 0) {
            sh.lens[h] = 0;
            sh.rcnt[h] = c + 1;
        }
        __syncthreads();
        t = lim >> 1;
        t_sel ^= 1;
        ++h;
    }
    return w2;
}

// The tail buffer's uniform state.
struct KllTail {
    uint32_t tl;    // keys in the buffer
    uint32_t full;  // tau is active
    double tau;     // keys <= tau are not candidates
#ifdef KRR_KLL_X_STATS  // profiling variant: refreshes / counting passes / sort fallbacks -> row word 14
    uint32_t nref = 0, npass = 0, nfall = 0;
#endif
};
#ifdef KRR_KLL_X_STATS
#define KLL_STAT_COPY(dst, src) ((dst).nref = (src).nref, (dst).npass = (src).npass, (dst).nfall = (src).nfall)
#define KLL_STAT_ADD(t, f) ((t).f += 1u)
#else
#define KLL_STAT_COPY(dst, src) ((void)0)
#define KLL_STAT_ADD(t, f) ((void)0)
#endif

// In-place stable compaction: keep keys > v and the first `eq` copies of v.  Four keys per
// lane per round, their LDS reads issued together.
__device__ KllTail kll_tail_keep(KllShared sh, KllTail ts, double v, uint32_t eq, int lane) {
    uint32_t out = 0;
#pragma unroll 1
    for (uint32_t r = 0; r < ts.tl; r += 4 * kWave) {
        double x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = r + (uint32_t)q * kWave + (uint32_t)lane;
            x[q] = i < ts.tl ? bitsd(sh.tb[i]) : -__builtin_inf();
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // in buffer order: q-th group of 64 after the (q-1)-th
            const uint32_t i = r + (uint32_t)q * kWave + (uint32_t)lane;
            const uint64_t em = ballot(i < ts.tl && x[q] == v);
            const bool keep = (i < ts.tl && x[q] > v) || (((em >> lane) & 1ull) && lane_prefix(em) < eq);
            const uint64_t km = ballot(keep);
            const uint32_t ne = popc64(em);
            eq -= ne < eq ? ne : eq;
            if (keep) sh.tb[out + lane_prefix(km)] = dbits(x[q]);
            out += popc64(km);
        }
    }
    __syncthreads();
    KllTail r{out, 1u, v};
    KLL_STAT_COPY(r, ts);
    return r;
}

// (#keys > v, #keys >= v) of the tail buffer, eight LDS reads per lane in flight.
__device__ __forceinline__ void kll_tail_count(const uint64_t* tb, uint32_t m, double v, uint32_t& gt, uint32_t& ge,
                                               int lane) {
    uint32_t g = 0, e = 0;
#pragma unroll 1
    for (uint32_t r = 0; r < m; r += 8 * kWave) {
        double x[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t i = r + (uint32_t)q * kWave + (uint32_t)lane;
            x[q] = i < m ? bitsd(tb[i]) : -__builtin_inf();
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            g += x[q] > v ? 1u : 0u;
            e += x[q] >= v ? 1u : 0u;
        }
    }
    gt = wave_sum_u32(g);
    ge = wave_sum_u32(e);
}

// Keep the buffer's largest keys: raise tau to a sampled pivot v that leaves between `tail`
// and tail + slack keys (> v, plus copies of v to reach `tail` when ties straddle it), all
// counted exactly.  The first pivot is where 64 strided samples put the cut; a miss jumps by
// the counted distance.  If no sample does, sort the buffer and keep exactly `tail`.
#ifdef KRR_KLL_X_REFRESH_NOINLINE
__device__ __attribute__((noinline))
#else
__device__ __forceinline__
#endif
KllTail kll_tail_refresh(KllShared sh, KllTail ts, uint32_t tail, int lane) {
    const uint32_t m = ts.tl;
    if (m <= tail) return ts;  // nothing to drop (callers refresh a buffer of > tail keys)
    KLL_STAT_ADD(ts, nref);
    double s = bitsd(sh.tb[(uint32_t)(((uint64_t)(uint32_t)lane * m) >> 6)]);
    s = kll_sort64(s, lane);
    const uint32_t want = tail + kKllTailSlack / 2;
    int idx = (int)(((uint64_t)(m - want) * 64u) / m);
    idx = idx < 0 ? 0 : (idx > 63 ? 63 : idx);
    int lo = -1, hi = 64;  // samples known too low (keep too many) / too high
#pragma unroll 1
    for (int it = 0; it < 6 && hi - lo > 1; ++it) {
        const double v = bitsd(lane_bcast64(dbits(s), idx));
        uint32_t gt, ge;
        kll_tail_count(sh.tb, m, v, gt, ge, lane);
        KLL_STAT_ADD(ts, npass);
        if (gt >= tail && gt <= tail + kKllTailSlack) return kll_tail_keep(sh, ts, v, 0, lane);
        if (gt < tail && ge >= tail) return kll_tail_keep(sh, ts, v, tail - gt, lane);
        // jump by the counted distance (about m / 64 keys between neighbouring samples)
        const int step = (int)(((int64_t)ge - (int64_t)want) * 64 / (int64_t)m);
        if (ge < tail) {  // pivot too high
            hi = idx;
            idx += step < -1 ? step : -1;
        } else {  // keeps too many
            lo = idx;
            idx += step > 1 ? step : 1;
        }
        idx = idx <= lo ? lo + 1 : (idx >= hi ? hi - 1 : idx);
    }
    kll_lds_sort(sh.tb, m, lane);  // exact fallback
    for (uint32_t i = lane; i < tail; i += kWave) sh.tb[i] = sh.tb[m - tail + i];
    __syncthreads();
    KllTail r{tail, 1u, bitsd(uni64(sh.tb[0]))};
    KLL_STAT_COPY(r, ts);
    KLL_STAT_ADD(r, nfall);
    return r;
}

// 2,048 keys ascending across the wave in registers (lane l holds positions 32 l .. 32 l + 31):
// bitonic with the flip first step of every stage, so every compare-exchange is ascending.
__device__ __forceinline__ void kll_regsort2048(double (&x)[32], int lane) {
#pragma unroll
    for (int k = 2; k <= 32; k <<= 1) {  // in-lane stages
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const int p = i ^ (k - 1);
            if ((i & (k >> 1)) == 0 && p > i) kll_cxd(x[i], x[p]);
        }
#pragma unroll
        for (int j = k >> 2; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < 32; ++i)
                if (!(i & j)) kll_cxd(x[i], x[i + j]);
        }
    }
#pragma unroll 1
    for (int k = 64; k <= 2048; k <<= 1) {
        // flip: position p pairs with p ^ (k - 1) = lane ^ ((k - 1) >> 5), slot 31 - i
        const int mk = (k - 1) >> 5;
        const bool lower = (lane & ((k >> 1) >> 5)) == 0;
        double o[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const uint64_t xb = dbits(x[31 - i]);
            const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)xb, mk, kWave);
            const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(xb >> 32), mk, kWave);
            o[i] = bitsd(((uint64_t)hi << 32) | lo);
        }
#pragma unroll
        for (int i = 0; i < 32; ++i) x[i] = lower ? fmin(x[i], o[i]) : fmax(x[i], o[i]);
        // half-cleaners across lanes (j >= 32), then in-lane
#pragma unroll 1
        for (int j = k >> 2; j >= 32; j >>= 1) {
            const int mj = j >> 5;
            const bool low = (lane & mj) == 0;
            switch (mj) {  // wave-uniform
                case 1: kll_cross<1, 32>(x, low); break;
                case 2: kll_cross<2, 32>(x, low); break;
                case 4: kll_cross<4, 32>(x, low); break;
                case 8: kll_cross<8, 32>(x, low); break;
                case 16: kll_cross<16, 32>(x, low); break;
                default: kll_cross<32, 32>(x, low); break;
            }
        }
#pragma unroll
        for (int j = 16; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < 32; ++i)
                if (!(i & j)) kll_cxd(x[i], x[i + j]);
        }
    }
}

// The tail buffer tb[0, m) (m <= 2,048) ascending in place, through registers.
__device__ void kll_tail_sort(uint64_t* tb, uint32_t m, int lane) {
    double x[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t p = (uint32_t)lane * 32u + (uint32_t)i;
        x[i] = p < m ? bitsd(tb[p]) : __builtin_inf();
    }
    __syncthreads();
    kll_regsort2048(x, lane);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t p = (uint32_t)lane * 32u + (uint32_t)i;
        if (p < m) tb[p] = dbits(x[i]);
    }
    __syncthreads();
}

// ---- the exact tail's candidate filter (the build's, and the tail pass's) ----
// Candidates: keys > tau (every present key until the buffer first fills).  A pair whose
// larger key is no candidate has none, so the per-slot tests run for hit pair columns only.
// The chunk's candidates are counted first and the buffer refreshed only when they do not
// fit: a refresh leaves <= tail + slack keys, so about 1,024 candidates arrive between two
// refreshes (refreshing whenever fewer than 1,024 slots were left made it one per ~64).
template <bool FULL>
__device__ __forceinline__ bool kll_cand(const KllTail& ts, double x) {
    return FULL ? x > ts.tau : x == x;
}
#ifndef KRR_KLL_LANE_APPEND
#define KRR_KLL_LANE_APPEND 1  // candidates that fit go in lane-major by one wave scan (else column by column)
#endif
template <bool FULL>
__device__ __forceinline__ void kll_tail_append(KllShared sh, KllTail& ts, uint32_t tail, uint32_t tcap, int lane,
                                                const double (&a)[8], const double (&b)[8], const double (&hi)[8]) {
#if KRR_KLL_LANE_APPEND
    {
        // the lane's candidates counted, one wave scan places them: when they all fit, each lane
        // writes its own after the keys of the lanes below it (the buffer is a set: the export
        // sorts it and a refresh keeps every key above its pivot, so the order is free)
        uint32_t mine = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool ca = kll_cand<FULL>(ts, a[u]), cb = kll_cand<FULL>(ts, b[u]);
            mine += (ca ? 1u : 0u) + (cb ? 1u : 0u);
        }
        const uint32_t incl = wave_scan32(mine, 0u, OpAdd32{});
        const uint32_t total = lane_bcast32(incl, kWave - 1);
        if (total == 0) return;
        if (ts.tl + total <= tcap) {
            uint32_t pos = ts.tl + incl - mine;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (kll_cand<FULL>(ts, a[u])) sh.tb[pos++] = dbits(a[u] + 0.0);  // -0 -> +0
                if (kll_cand<FULL>(ts, b[u])) sh.tb[pos++] = dbits(b[u] + 0.0);
            }
            ts.tl += total;
            return;
        }
    }
#endif
    uint64_t pm[8], any = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        pm[u] = ballot(kll_cand<FULL>(ts, hi[u]));
        any |= pm[u];
    }
    if (!any) return;
    // the chunk's candidates: at most two per hit pair; counted exactly (ballots recomputed
    // below: no masks kept) only when that bound does not fit
    uint32_t add = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) add += 2u * popc64(pm[u]);
    if (ts.tl + add > tcap) {
        add = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (pm[u]) add += popc64(ballot(kll_cand<FULL>(ts, a[u]))) + popc64(ballot(kll_cand<FULL>(ts, b[u])));
    }
    bool column_wise = false;
    if (ts.tl + add > tcap) {
        if (ts.tl > tail + kKllTailSlack) {  // a refresh leaves <= tail + slack: only then can it help
            ts = kll_tail_refresh(sh, ts, tail, lane);  // tau rises: recheck the keys
#pragma unroll
            for (int u = 0; u < 8; ++u) pm[u] = ballot(hi[u] > ts.tau);
        }
        // a buffer with less room than a whole chunk (the tail pass's): columns of <= 128 keys
        // one by one, refreshing when one does not fit (the buffer then holds > tail keys)
        column_wise = tcap < tail + kKllTailSlack + 16u * kWave;
    }
    uint32_t tl = ts.tl;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        if (pm[u]) {
            uint64_t ma = ballot(ts.full ? a[u] > ts.tau : a[u] == a[u]);
            uint64_t mb = ballot(ts.full ? b[u] > ts.tau : b[u] == b[u]);
            if (column_wise && tl + popc64(ma) + popc64(mb) > tcap) {  // <= 128 keys: fits after it
                ts.tl = tl;
                ts = kll_tail_refresh(sh, ts, tail, lane);
                tl = ts.tl;
                ma = ballot(a[u] > ts.tau);
                mb = ballot(b[u] > ts.tau);
            }
            if ((ma >> lane) & 1ull) sh.tb[tl + lane_prefix(ma)] = dbits(a[u] + 0.0);  // -0 -> +0
            tl += popc64(ma);
            if ((mb >> lane) & 1ull) sh.tb[tl + lane_prefix(mb)] = dbits(b[u] + 0.0);
            tl += popc64(mb);
        }
    }
    ts.tl = tl;
}
__device__ __forceinline__ void kll_tail_filter(KllShared sh, KllTail& ts, uint32_t tail, uint32_t tcap, int lane,
                                                const double (&a)[8], const double (&b)[8], const double (&hi)[8]) {
    if (ts.full) kll_tail_append<true>(sh, ts, tail, tcap, lane, a, b, hi);
    else kll_tail_append<false>(sh, ts, tail, tcap, lane, a, b, hi);
}

// The buffer's top min(n, tail) keys, ascending, into the row's tail words; returns how many.
__device__ __forceinline__ uint32_t kll_tail_export(KllShared sh, KllTail ts, uint32_t tail, uint64_t* row_tail, int lane) {
    // a buffer the register sort holds (<= 2,048 keys) is sorted as it is: the top `tail` of it are
    // the same keys a refresh would have kept
#ifdef KRR_KLL_X_OLDEXPORT
    if (ts.tl > tail + kKllTailSlack || (ts.tl > 2048 && ts.tl > tail)) ts = kll_tail_refresh(sh, ts, tail, lane);
#else
    if (ts.tl > 2048 && ts.tl > tail) ts = kll_tail_refresh(sh, ts, tail, lane);
#endif
#ifndef KRR_KLL_X_NOREGSORT
    if (ts.tl <= 2048) kll_tail_sort(sh.tb, ts.tl, lane);
    else
#endif
        kll_lds_sort(sh.tb, ts.tl, lane);
    const uint32_t tl_out = ts.tl < tail ? ts.tl : tail;
    for (uint32_t i = lane; i < tl_out; i += kWave) row_tail[i] = sh.tb[ts.tl - tl_out + i];
    for (uint32_t i = tl_out + lane; i < tail; i += kWave) row_tail[i] = 0;  // canonical rows
    __syncthreads();
    return tl_out;
}

// Per-wave build state; one instance per series slice (by value: nothing is address-taken).
// TAIL: the one-pass tail buffer is part of this build; LINES: the build also writes each
// chunk's 64 line maxima (kll_line_key) to lm[ci * 64 ...] for the sparse tail pass
template <bool TAIL, bool LINES = false>
struct KllProc {
    KllShared sh;
    uint32_t* lm;      // LINES: this series' line maxima
    uint64_t base;
    uint64_t w2u;      // sum w^2 of the wave-level compactions (uniform)
    uint32_t ci;       // chunk index (uniform)
    int lane;
    int32_t nrl;
    uint32_t tail, tcap;
    KllTail ts;
    // per lane
    double pend1[8], pend2[8], pend3[8];
    uint32_t cp1, cp2, cp3;
    double K[4];
    uint32_t kmask;
    uint32_t kcnt[4];
    double arr;
    bool has_arr;
    uint32_t w2l, pres;
    double kmin, kmax;

    // ---- per-lane odd slots (levels 0..3); a carry past level 3 arrives at the wave ----
    // Branch-free over the levels (a per-level early return would be merged into one store
    // through a dynamic index, putting K in scratch memory).
    template <int H0>
    __device__ __forceinline__ void lane_odd(double v, bool active = true) {
#pragma unroll
        for (int h = H0; h < 4; ++h) {
            const bool occ = (kmask >> h) & 1u;
            const bool here = active && !occ, comp = active && occ;
            const uint32_t bit = kll_coin32(base, kT_LODD + 4u * (uint32_t)lane + (uint32_t)h, kcnt[h]) & 1u;
            const double kept = bit ? fmax(K[h], v) : fmin(K[h], v);
            K[h] = kll_pick(here, K[h], v);
            kcnt[h] += comp ? 1u : 0u;
            kmask = here ? (kmask | (1u << h)) : (comp ? (kmask & ~(1u << h)) : kmask);
            w2l += comp ? (1u << (2 * h)) : 0u;
            v = kll_pick(comp, v, kept);
            active = comp;
        }
        arr = kll_pick(active, arr, v);
        has_arr = has_arr || active;
    }

    __device__ __forceinline__ void arrivals() {
        uint64_t am = ballot(has_arr);
        if (am) {  // rare: a per-lane odd carry reached level 4
#pragma unroll 1
            while (am) {
                const int l = __ffsll((long long)am) - 1;
                w2u += kll_wave_odd(sh, base, 4, bitsd(lane_bcast64(dbits(arr), l)), lane);
                am &= am - 1;
            }
            has_arr = false;
        }
    }

    // Odd largest set aside (slow path), then every other key from the coin: z (16, ascending,
    // absent keys +inf at the end, c present) -> y (8), cy.
    template <int H>
    __device__ __forceinline__ void lane_level(double (&z)[16], uint32_t c, uint32_t tag, uint32_t idx, double (&y)[8],
                                               uint32_t& cy) {
        if (ballot(c & 1u)) {
            const bool odd = c & 1u;
            double v = z[0];
#pragma unroll
            for (int i = 1; i < 16; ++i) v = kll_pick((uint32_t)i == c - 1, v, z[i]);
#pragma unroll
            for (int i = 0; i < 16; ++i) z[i] = kll_pick(odd && (uint32_t)i == c - 1, z[i], bitsd(kKllInfBits));
            lane_odd<H>(v, odd);
            c -= odd ? 1u : 0u;
        }
        const uint32_t off = kll_coin32(base, tag + (uint32_t)lane, idx) & 1u;
#pragma unroll
        for (int k = 0; k < 8; ++k) y[k] = kll_pick(off != 0, z[2 * k], z[2 * k + 1]);
        cy = c >> 1;
        w2l += c >= 2 ? (1u << (2 * H)) : 0u;
    }

    // ---- level 4: the wave ----
    __device__ __forceinline__ void wave_stage(double (&y)[8], uint32_t cy) {
        uint32_t C = wave_sum_u32(cy);
        if (C == 0) return;
        kll_sort512(y, lane);
        if (C & 1u) {  // the largest present key (position C - 1) is set aside at level 4
            const uint32_t src = (C - 1) >> 3, slot = (C - 1) & 7u;
            double v = y[0];
#pragma unroll
            for (int i = 1; i < 8; ++i) v = kll_pick((uint32_t)i == slot, v, y[i]);
            w2u += kll_wave_odd(sh, base, 4, bitsd(lane_bcast64(dbits(v), (int)src)), lane);
            C -= 1;
        }
        const uint32_t off = kll_coin32(base, kT_WAVE, ci >> 3) & 1u;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t p = (uint32_t)lane * 8u + (uint32_t)i;
            if (p < C && p >= off && ((p - off) & 1u) == 0) sh.tmp[(p - off) >> 1] = dbits(y[i]);
        }
        if (C >= 2) w2u += 1ull << 8;
        __syncthreads();
#ifndef KRR_KLL_X_NOPUSH  // profiling variant: no run push (rows are not valid)
        w2u += kll_push(sh, base, nrl, 0, C >> 1, kKllFirstRun, lane);
#endif
    }

    __device__ __forceinline__ void tail_filter(const double (&a)[8], const double (&b)[8], const double (&hi)[8]) {
        kll_tail_filter(sh, ts, tail, tcap, lane, a, b, hi);
    }

    // ---- one chunk ----
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
        // keys are folded (-0 -> +0) where they are kept: the selected pair key, lone and tail
        // keys, min / max at the end; compares treat -0 and +0 alike
        double a[8], b[8], lo[8], hi[8];
        uint64_t nanm = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a[u] = c[u].x;
            b[u] = c[u].y;
            nanm |= ballot(__builtin_isunordered(a[u], b[u]));
            lo[u] = fmin(a[u], b[u]);  // one NaN: both are the present sample
            hi[u] = fmax(a[u], b[u]);
        }
        if constexpr (LINES) {
            // lane 8g + j stores line (u = j, g) of this chunk: index u * 8 + g
            const uint32_t j = (uint32_t)lane & 7u;
            uint32_t mine = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t k = kll_max8(kll_line_key(hi[u]));
                mine = j == (uint32_t)u ? k : mine;
            }
            lm[(size_t)ci * 64u + j * 8u + ((uint32_t)lane >> 3)] = mine;
        }
#ifndef KRR_KLL_X_NOTAIL
        if constexpr (TAIL) {
            if (tail) tail_filter(a, b, hi);
        }
#endif
        double out[8];
        uint32_t c0 = 0;
        if (nanm == 0) {  // every slot present: 8 two-key compactions per lane
            const uint32_t bits = kll_coin32(base, kT_L0 + (uint32_t)lane, ci);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                out[u] = (((bits >> u) & 1u) ? hi[u] : lo[u]) + 0.0;
                kmin = fmin(kmin, lo[u]);
                kmax = fmax(kmax, hi[u]);
            }
            c0 = 8;
            w2l += 8;
            pres += 16;
        } else {
            bool any = false;
#pragma unroll
            for (int u = 0; u < 8; ++u) any |= hi[u] == hi[u];
            if (ballot(any)) {
                const uint32_t bits = kll_coin32(base, kT_L0 + (uint32_t)lane, ci);
                uint32_t lone = 0;  // pairs with one present sample, bit u
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const bool pa = !__builtin_isnan(a[u]), pb = !__builtin_isnan(b[u]);
                    kmin = fmin(kmin, lo[u]);
                    kmax = fmax(kmax, hi[u]);
                    pres += (pa ? 1u : 0u) + (pb ? 1u : 0u);
                    out[u] = (pa && pb) ? ((((bits >> u) & 1u) ? hi[u] : lo[u]) + 0.0) : bitsd(kKllInfBits);
                    c0 += (pa && pb) ? 1u : 0u;
                    lone |= (pa != pb) ? (1u << u) : 0u;
                }
                w2l += c0;
                // lone samples into the level-0 odd slot, in pair order (one slot update per round)
#pragma unroll 1
                while (ballot(lone != 0)) {
                    const uint32_t u0 = lone ? (uint32_t)__builtin_ctz(lone) : 0u;
                    double v = lo[0];
#pragma unroll
                    for (int u = 1; u < 8; ++u) v = kll_pick((uint32_t)u == u0, v, lo[u]);
                    lane_odd<0>(v + 0.0, lone != 0);
                    lone &= lone - 1;
                }
                arrivals();
            } else {
#pragma unroll
                for (int u = 0; u < 8; ++u) out[u] = bitsd(kKllInfBits);
            }
        }
#if defined(KRR_KLL_X_CUT) && KRR_KLL_X_CUT == 1  // profiling variant: level 0 only (rows not valid)
#pragma unroll
        for (int u = 0; u < 8; ++u) kmax = fmax(kmax, out[u]);
        if (true) {
#else
        if ((ci & 1u) == 0) {
#endif
#pragma unroll
            for (int u = 0; u < 8; ++u) pend1[u] = out[u];
            cp1 = c0;
        } else {
            double z[16], y[8];
            uint32_t cy;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                z[u] = pend1[u];
                z[8 + u] = out[u];
            }
            kll_sort16(z);
            lane_level<1>(z, cp1 + c0, kT_L1, ci >> 1, y, cy);
            arrivals();
#if defined(KRR_KLL_X_CUT) && KRR_KLL_X_CUT == 2  // profiling variant: levels 0-1 only
#pragma unroll
            for (int u = 0; u < 8; ++u) kmax = fmax(kmax, y[u]);
            if (true) {
#else
            if (((ci >> 1) & 1u) == 0) {
#endif
#pragma unroll
                for (int u = 0; u < 8; ++u) pend2[u] = y[u];
                cp2 = cy;
            } else {
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    z[u] = pend2[u];
                    z[8 + u] = y[u];
                }
                kll_merge16(z);
                lane_level<2>(z, cp2 + cy, kT_L2, ci >> 2, y, cy);
                arrivals();
                if (((ci >> 2) & 1u) == 0) {
#pragma unroll
                    for (int u = 0; u < 8; ++u) pend3[u] = y[u];
                    cp3 = cy;
                } else {
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        z[u] = pend3[u];
                        z[8 + u] = y[u];
                    }
                    kll_merge16(z);
                    lane_level<3>(z, cp3 + cy, kT_L3, ci >> 3, y, cy);
                    arrivals();
#ifndef KRR_KLL_X_NOWAVE  // profiling variant: no wave stage (rows are not valid)
                    wave_stage(y, cy);
#else
                    kmax = fmax(kmax, y[0]);
#endif
                }
            }
        }
        ++ci;
    }
};

// The streaming loop of stream_segment (ONE_SITE, one chunk in flight), run for npad chunks:
// chunks past the segment's last are all NaN (the flush), and the head / tail slots ride the
// last real chunk only.
template <class Proc, int MODE = KRR_KLL_STREAM>
__device__ __forceinline__ void kll_stream(const double* __restrict__ vals, int64_t beg, int64_t end, int64_t npad,
                                           Proc& proc, int lane) {
    int64_t a0 = (beg + 1) & ~(int64_t)1;
    if (a0 > end) a0 = end;
    int64_t a1 = end & ~(int64_t)1;
    if (a1 < a0) a1 = a0;
    const double2* __restrict__ v2 = reinterpret_cast<const double2*>(vals);
    const int64_t i0 = a0 >> 1;
    const int64_t nunits = (a1 >> 1) - i0;
    constexpr int CH = kUnroll * kWave;
    const int64_t nfull = nunits / CH;
    const bool head = a0 > beg, tail = a1 < end;
    const int64_t nch = nfull + ((nunits - nfull * CH) > 0 || head || tail ? 1 : 0);
    if (npad == 0) return;
    const double2* __restrict__ p = v2 + i0 + lane;
    const double qnan = __builtin_nan("");
    double hv = qnan, tv = qnan;
    if (head) hv = vals[beg];
    if (tail) tv = vals[a1];
    const double2* __restrict__ zp = g_zero_chunk + lane;
    auto fill_u = [&](double2 (&c)[kUnroll], int64_t ci) __attribute__((always_inline)) {
        if (ci < nfull) {
            load_chunk(c, p + ci * CH);
        } else {
            const double2* zpl = zp;
            int ln = lane;
            asm volatile("" : "+v"(zpl), "+v"(ln));
            const double2* q[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int64_t j = ci * CH + u * kWave + ln;
                q[u] = (ci < nch && j < nunits) ? v2 + i0 + j : zpl + u * kWave;
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) c[u] = load16(q[u]);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int64_t j = ci * CH + u * kWave + ln;
                if (j >= nunits) c[u] = make_double2(qnan, qnan);
            }
            if (lane == kWave - 1 && ci == nch - 1) {
                c[kUnroll - 1].x = hv;
                c[kUnroll - 1].y = tv;
            }
        }
    };
    if constexpr (MODE == 1) {
    // two chunks per iteration, ping-pong buffers: chunk ci + 1 in flight while ci is processed,
    // no register copies (npad is a multiple of 8)
    double2 A[kUnroll], B[kUnroll];
    fill_u(A, 0);
#pragma unroll 1
    for (int64_t ci = 0; ci < npad; ci += 2) {
        fill_u(B, ci + 1);
        proc.chunk(A);
        fill_u(A, ci + 2);
        proc.chunk(B);
    }
    } else if constexpr (MODE == 3) {
    // two chunks in flight, three buffers rotated by unrolling by 3 (no register copies);
    // npad is a multiple of 3
    double2 A[kUnroll], B[kUnroll], C[kUnroll];
    fill_u(A, 0);
    fill_u(B, 1);
#pragma unroll 1
    for (int64_t ci = 0; ci < npad; ci += 3) {
        fill_u(C, ci + 2);
        proc.chunk(A);
        fill_u(A, ci + 3);
        proc.chunk(B);
        fill_u(B, ci + 4);
        proc.chunk(C);
    }
    } else if constexpr (MODE == 2) {
    // two chunks in flight: ci + 1 and ci + 2 while ci is processed
    double2 A[kUnroll], B[kUnroll], C[kUnroll];
    fill_u(A, 0);
    fill_u(B, 1);
#pragma unroll 1
    for (int64_t ci = 0; ci < npad; ci += 2) {
        fill_u(C, ci + 2);
        proc.chunk(A);
        fill_u(A, ci + 3);
        proc.chunk(B);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            B[u] = A[u];
            A[u] = C[u];
        }
    }
    } else {
    double2 cur[kUnroll], nxt[kUnroll];
    fill_u(nxt, 0);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        double x = nxt[u].x, y = nxt[u].y;
        asm volatile("" : "+v"(x), "+v"(y));
        cur[u] = make_double2(x, y);
    }
#pragma unroll 1
    for (int64_t ci = 0; ci < npad; ++ci) {
        fill_u(nxt, ci + 1);
        proc.chunk(cur);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) cur[u] = nxt[u];
    }
    }
}

// Level h's keys after the build (per-lane odd slots below 4: `has` / `kv` of this lane, the
// wave slot, the run) plus `carry` (ascending, nc) gathered into ws, ascending; returns how many.
__device__ uint32_t kll_gather_level(const KllShared& sh, int32_t nrl, uint32_t h, bool has, double kv,
                                     const uint64_t* carry, uint32_t nc, uint64_t* ws, int lane) {
    const uint32_t a = (h >= (uint32_t)kKllFirstRun && (int)h < kKllFirstRun + nrl) ? uni32(sh.lens[h]) : 0u;
#ifndef KRR_KLL_X_SORTGATHER
    if (!ballot(has)) {
        // no lane odd slots: the run, the carry and the wave slot are each ascending — place
        // every key at its merged position (binary searches) instead of sorting the union
        const uint64_t* R = sh.lv + (size_t)(h >= (uint32_t)kKllFirstRun ? h - kKllFirstRun : 0u) * kKllRun;
        const bool wk = (uni32(sh.misc[0]) >> h) & 1u;
        const uint64_t kb = wk ? uni64(sh.wk[h]) : 0ull;
        const double k = bitsd(kb);
#pragma unroll 1
        for (uint32_t i = lane; i < a; i += kWave) {
            const double x = bitsd(R[i]);
            ws[i + kll_bound<true>(carry, nc, x) + (wk && k < x ? 1u : 0u)] = R[i];
        }
#pragma unroll 1
        for (uint32_t j = lane; j < nc; j += kWave) {
            const double x = bitsd(carry[j]);
            ws[j + kll_bound<false>(R, a, x) + (wk && k < x ? 1u : 0u)] = carry[j];
        }
        if (wk && lane == 0) ws[kll_bound<false>(R, a, k) + kll_bound<false>(carry, nc, k)] = kb;
        __syncthreads();
        return a + nc + (wk ? 1u : 0u);
    }
#endif
    uint32_t m = 0, sources = 0;
    if (a) {
        const uint64_t* R = sh.lv + (size_t)(h - kKllFirstRun) * kKllRun;
        for (uint32_t i = lane; i < a; i += kWave) ws[i] = R[i];
        m = a;
        ++sources;
    }
    if (nc) {
        for (uint32_t i = lane; i < nc; i += kWave) ws[m + i] = carry[i];
        m += nc;
        ++sources;
    }
    const uint64_t km = ballot(has);
    if (km) {
        if (has) ws[m + lane_prefix(km)] = dbits(kv);
        m += popc64(km);
        sources += 2;  // unsorted
    }
    if ((uni32(sh.misc[0]) >> h) & 1u) {
        if (lane == 0) ws[m] = sh.wk[h];
        m += 1;
        ++sources;
    }
    __syncthreads();
    if (sources > 1) kll_lds_sort(ws, m, lane);
    return m;
}

#ifndef KRR_KLL_BODY_WAVES_PER_SIMD
#define KRR_KLL_BODY_WAVES_PER_SIMD 2  // the body-only build: two waves per SIMD (LDS allows 9 per CU)
#endif
#ifndef KRR_KLL_WAVES_PER_SIMD
#define KRR_KLL_WAVES_PER_SIMD 1  // the build's LDS (runs + tail buffer) allows one wave per SIMD anyway
#endif
// TAIL = false: no tail (tail == 0) or the tail left to k_kll_tail (A.tail_pass); the build then
// holds none of the tail buffer's code or state.
template <bool TAIL, bool LINES = false>
__global__ __launch_bounds__(64, TAIL ? KRR_KLL_WAVES_PER_SIMD : KRR_KLL_BODY_WAVES_PER_SIMD) void k_kll_build(
    KllBuildArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    KllShared sh;
    sh.lv = reinterpret_cast<uint64_t*>(smem);
    sh.tmp = sh.lv + (size_t)A.nrl * kKllRun;
    sh.tb = sh.tmp + 2 * kKllRun;
    sh.wk = sh.tb + A.tcap;
    sh.lens = reinterpret_cast<uint32_t*>(sh.wk + kKllLevels);
    sh.rcnt = sh.lens + kKllLevels;
    sh.wcnt = sh.rcnt + kKllLevels;
    sh.misc = sh.wcnt + kKllLevels;
    const uint32_t budget = (uint32_t)A.budget, tail = (uint32_t)A.tail;
    const uint32_t RW = (uint32_t)kKllHdr + budget + tail;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        if (lane < kKllLevels) {
            sh.lens[lane] = 0;
            sh.rcnt[lane] = 0;
            sh.wcnt[lane] = 0;
        }
        if (lane < 2) sh.misc[lane] = 0;
        __syncthreads();
        const uint64_t series = (uint64_t)(A.seg_base + s);
        uint64_t* row = A.rows + (size_t)s * RW;
        const int64_t nch = kll_nchunks(beg, end);
        const int64_t npad = (nch + 7) & ~(int64_t)7;
        KllProc<TAIL, LINES> P;
        P.sh = sh;
        P.lm = LINES ? A.lines + (size_t)s * (size_t)A.line_stride : nullptr;
        P.base = kll_slice_base(A.seed, series, A.slice);
        P.w2u = 0;
        P.ci = 0;
        P.lane = lane;
        P.nrl = A.nrl;
        P.tail = A.tail_pass ? 0u : tail;
        P.tcap = A.tcap;
        P.ts = KllTail{0u, 0u, 0.0};
#pragma unroll
        for (int u = 0; u < 8; ++u) P.pend1[u] = P.pend2[u] = P.pend3[u] = bitsd(kKllInfBits);
        P.cp1 = P.cp2 = P.cp3 = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            P.K[h] = 0.0;
            P.kcnt[h] = 0;
        }
        P.kmask = 0;
        P.arr = 0.0;
        P.has_arr = false;
        P.w2l = 0;
        P.pres = 0;
        P.kmin = P.kmax = bitsd(kQuietNaN);
        kll_stream(A.vals, beg, end, npad, P, lane);

        const uint32_t kmask = P.kmask;
        const double K0[4] = {P.K[0], P.K[1], P.K[2], P.K[3]};
        const uint64_t n_pres = lane_bcast64(wave_scan64((uint64_t)P.pres, 0ull, OpAdd64{}), kWave - 1);
        const uint64_t w2lanes = lane_bcast64(wave_scan64((uint64_t)P.w2l, 0ull, OpAdd64{}), kWave - 1);
        const uint64_t gmin = dbits(bitsd(lane_bcast64(wave_scan64(dbits(P.kmin), kQuietNaN, OpMinF64Bits{}), kWave - 1)) + 0.0);
        const uint64_t gmax = dbits(bitsd(lane_bcast64(wave_scan64(dbits(P.kmax), kQuietNaN, OpMaxF64Bits{}), kWave - 1)) + 0.0);

        // tail: the min(n, tail) largest present keys, ascending
        // tail: the min(n, tail) largest present keys, ascending (the tail pass writes them
        // instead when A.tail_pass: this launch leaves them zero)
        uint32_t tl_out = 0;
        if constexpr (TAIL) {
            if (tail && !A.tail_pass) tl_out = kll_tail_export(sh, P.ts, tail, row + kKllHdr + budget, lane);
        }

        // body: from level 0 up, while more than `budget` keys remain, compact each level of
        // >= 2 keys once (odd largest set aside) into the next; export every level ascending
        // level keys: a run (<= 256) + the carry (<= 256) + lane odd slots (<= 64, levels < 4) or
        // the wave slot (1): <= 513; carry <= 256.  They start at tmp (free after the stream)
        // and run into the tail buffer (already exported): kKllFinalWords in all.
        uint64_t* ws = sh.tmp;
        uint64_t* cbuf = sh.tmp + kKllWsWords;
        uint64_t total = 0;
#pragma unroll 1
        for (uint32_t h = 0; h < (uint32_t)kKllLevels; ++h) {
            uint32_t n_h = 0;
            if (h < 4) n_h = popc64(ballot((kmask >> h) & 1u));
            if (h >= (uint32_t)kKllFirstRun && (int)h < kKllFirstRun + A.nrl) n_h += uni32(sh.lens[h]);
            n_h += (uni32(sh.misc[0]) >> h) & 1u;
            total += n_h;
        }
        uint32_t nc = 0, pos = 0;
        uint64_t lw[6] = {0, 0, 0, 0, 0, 0};
        uint64_t weight = 0, w2f = 0;
#pragma unroll 1
#ifdef KRR_KLL_X_NOFINAL  // profiling variant: no final compression / export (rows are not valid)
        for (uint32_t h = 0; h < 0u; ++h) {
#else
        for (uint32_t h = 0; h < (uint32_t)kKllLevels; ++h) {
#endif
            const bool has = h < 4 && ((kmask >> h) & 1u);
            const double kv = h == 0 ? K0[0] : (h == 1 ? K0[1] : (h == 2 ? K0[2] : K0[3]));
            const uint32_t m = kll_gather_level(sh, A.nrl, h, has, kv, cbuf, nc, ws, lane);
            uint32_t keep = m;  // keys exported at level h
            nc = 0;
            if (total > budget && m >= 2) {
                if (h + 1 >= (uint32_t)kKllLevels) {
                    if (lane == 0) sh.misc[1] = 1;
                    __syncthreads();
                    break;
                }
                const uint32_t me = m & ~1u;
                const uint32_t off = kll_coin32(P.base, kT_FINAL + h, 0) & 1u;
                for (uint32_t k = lane; k < (me >> 1); k += kWave) cbuf[k] = ws[off + 2 * k];
                nc = me >> 1;
                w2f += 1ull << (2 * h);
                total -= me - nc;
                keep = m - me;  // the set-aside key, ws[m - 1]
                if (keep && lane == 0) ws[0] = ws[m - 1];
                __syncthreads();
            }
            if (keep) {
                if (pos + keep > budget) {  // only after an overflow
                    if (lane == 0) sh.misc[1] = 1;
                    __syncthreads();
                    break;
                }
                for (uint32_t i = lane; i < keep; i += kWave) row[kKllHdr + pos + i] = ws[i];
                pos += keep;
                weight += (uint64_t)keep << h;
                lw[h >> 2] |= (uint64_t)keep << (16 * (h & 3));
            }
            __syncthreads();
        }
        const bool overflow = uni32(sh.misc[1]) != 0;
        for (uint32_t i = pos + lane; i < budget; i += kWave) row[kKllHdr + i] = 0;  // canonical rows: unused words 0
        if (A.tail_pass)
            for (uint32_t i = lane; i < tail; i += kWave) row[kKllHdr + budget + i] = 0;
        if (lane == 0) {
            row[0] = n_pres;
            row[1] = A.gaps ? 0ull : (uint64_t)(end - beg) - n_pres;
            row[2] = n_pres ? gmin : kQuietNaN;
            row[3] = n_pres ? gmax : kQuietNaN;
            row[4] = P.w2u + w2lanes + w2f;
            row[5] = weight;
            row[6] = tl_out;
            row[7] = ((uint64_t)budget << 32) | tail;
#pragma unroll
            for (int w = 0; w < 6; ++w) row[8 + w] = lw[w];
#ifdef KRR_KLL_X_STATS
            row[14] = ((uint64_t)P.ts.nfall << 48) | ((uint64_t)P.ts.npass << 24) | P.ts.nref;
#else
            row[14] = 0;
#endif
            row[15] = overflow ? kKllRowOverflow : 0ull;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// Fold / merge / query.  A row image in LDS: header, body, tail words exactly as in memory.

__device__ __forceinline__ uint32_t kll_len(const uint64_t* row, uint32_t h) {
    return (uint32_t)(row[8 + (h >> 2)] >> (16 * (h & 3))) & 0xFFFFu;
}

__device__ void kll_copy_row(const uint64_t* src, uint64_t* dst, uint32_t RW, int lane) {
    for (uint32_t i = lane; i < RW; i += kWave) dst[i] = src[i];
    __syncthreads();
}

// Three ascending lists merged into O (A, then C, then K among equal keys).
__device__ void kll_merge3(const uint64_t* A, uint32_t na, const uint64_t* C, uint32_t nc, const uint64_t* K,
                           uint32_t nk, uint64_t* O, int lane) {
#pragma unroll 1
    for (uint32_t i = lane; i < na; i += kWave) {
        const double x = bitsd(A[i]);
        O[i + kll_bound<true>(C, nc, x) + kll_bound<true>(K, nk, x)] = A[i];
    }
#pragma unroll 1
    for (uint32_t j = lane; j < nc; j += kWave) {
        const double x = bitsd(C[j]);
        O[j + kll_bound<false>(A, na, x) + kll_bound<true>(K, nk, x)] = C[j];
    }
#pragma unroll 1
    for (uint32_t k = lane; k < nk; k += kWave) {
        const double x = bitsd(K[k]);
        O[k + kll_bound<false>(A, na, x) + kll_bound<false>(C, nc, x)] = K[k];
    }
    __syncthreads();
}

// O = fold(A, C): A, C, O row images in LDS (the same budget / tail cap); S scratch
// (>= 3 budget keys), CB carry (>= 2 budget keys).  Coins: (base, kT_FOLD + h, idx).
__device__ void kll_fold(const uint64_t* A, const uint64_t* C, uint64_t* O, uint64_t* S, uint64_t* CB, uint64_t base,
                         uint32_t idx, uint32_t budget, uint32_t tail, int lane) {
    const uint64_t na = A[0], ncn = C[0];
    const uint32_t ta = (uint32_t)A[6], tc = (uint32_t)C[6];
    const uint64_t n = na + ncn;
    const uint32_t tn = (uint64_t)tail < n ? tail : (uint32_t)n;  // min(tail, n) <= ta + tc
    // tail: the tn largest of the union (merged positions >= ta + tc - tn)
    {
        const uint64_t* X = A + kKllHdr + budget;
        const uint64_t* Y = C + kKllHdr + budget;
        uint64_t* Z = O + kKllHdr + budget;
        const uint32_t drop = ta + tc - tn;
        for (uint32_t i = lane; i < ta; i += kWave) {
            const uint32_t p = i + kll_bound<true>(Y, tc, bitsd(X[i]));
            if (p >= drop) Z[p - drop] = X[i];
        }
        for (uint32_t j = lane; j < tc; j += kWave) {
            const uint32_t p = j + kll_bound<false>(X, ta, bitsd(Y[j]));
            if (p >= drop) Z[p - drop] = Y[j];
        }
    }
    // body
    uint64_t total = 0;
    for (uint32_t h = 0; h < (uint32_t)kKllLevels; ++h) total += kll_len(A, h) + kll_len(C, h);
    uint32_t offA = 0, offC = 0, pos = 0, ncarry = 0;
    uint64_t lw[6] = {0, 0, 0, 0, 0, 0};
    uint64_t weight = 0, w2 = 0;
    bool bad = (A[15] | C[15]) != 0;
#pragma unroll 1
    for (uint32_t h = 0; h < (uint32_t)kKllLevels; ++h) {
        const uint32_t la = kll_len(A, h), lc = kll_len(C, h);
        kll_merge3(A + kKllHdr + offA, la, C + kKllHdr + offC, lc, CB, ncarry, S, lane);
        offA += la;
        offC += lc;
        const uint32_t m = la + lc + ncarry;
        uint32_t keep = m;
        ncarry = 0;
        if (total > budget && m >= 2) {
            if (h + 1 >= (uint32_t)kKllLevels) {
                bad = true;
                break;
            }
            const uint32_t me = m & ~1u;
            const uint32_t off = kll_coin32(base, kT_FOLD + h, idx) & 1u;
            for (uint32_t k = lane; k < (me >> 1); k += kWave) CB[k] = S[off + 2 * k];
            ncarry = me >> 1;
            w2 += 1ull << (2 * h);
            total -= me - ncarry;
            keep = m - me;
            if (keep && lane == 0) S[0] = S[m - 1];
            __syncthreads();
        }
        if (keep) {
            if (pos + keep > budget) {
                bad = true;
                break;
            }
            for (uint32_t i = lane; i < keep; i += kWave) O[kKllHdr + pos + i] = S[i];
            pos += keep;
            weight += (uint64_t)keep << h;
            lw[h >> 2] |= (uint64_t)keep << (16 * (h & 3));
        }
        __syncthreads();
    }
    for (uint32_t i = pos + lane; i < budget; i += kWave) O[kKllHdr + i] = 0;  // canonical rows: unused words 0
    for (uint32_t i = tn + lane; i < tail; i += kWave) O[kKllHdr + budget + i] = 0;
    if (lane == 0) {
        O[0] = n;
        O[1] = A[1] + C[1];
        O[2] = dbits(fmin(bitsd(A[2]), bitsd(C[2])));  // fmin / fmax: the non-NaN operand wins
        O[3] = dbits(fmax(bitsd(A[3]), bitsd(C[3])));
        O[4] = A[4] + C[4] + w2;
        O[5] = weight;
        O[6] = tn;
        O[7] = A[7];
#pragma unroll
        for (int w = 0; w < 6; ++w) O[8 + w] = lw[w];
        O[14] = 0;
        O[15] = (bad || A[7] != C[7]) ? kKllRowOverflow : 0ull;
    }
    __syncthreads();
}

struct KllMergeArgs {
    int64_t S;
    int32_t W;
    int32_t budget, tail;
    uint32_t epoch;
    uint64_t seed;
    int64_t series_base;
    const uint64_t* rows;  // [S][W][RW]
    uint64_t* out;         // [S][RW] (merge)
    int32_t mode;          // query
    int64_t p_num, p_den;
    double q;
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
    const int64_t* ktab = nullptr;  // query: krr_percentile_params.k_table
    int64_t ktab_len = 0;
};

// The series' W rows folded left to right into the image returned (LDS).
__device__ uint64_t* kll_fold_rows(const KllMergeArgs& A, int64_t s, unsigned char* smem, int lane) {
    const uint32_t budget = (uint32_t)A.budget, tail = (uint32_t)A.tail;
    const uint32_t RW = (uint32_t)kKllHdr + budget + tail;
    uint64_t* im0 = reinterpret_cast<uint64_t*>(smem);
    uint64_t* im1 = im0 + RW;
    uint64_t* imc = im1 + RW;
    uint64_t* S = imc + RW;
    uint64_t* CB = S + 3 * (size_t)budget;
    const uint64_t* rows = A.rows + (size_t)s * A.W * RW;
    kll_copy_row(rows, im0, RW, lane);
    const uint64_t base = kll_slice_base(A.seed, (uint64_t)(A.series_base + s), A.epoch);
#pragma unroll 1
    for (int w = 1; w < A.W; ++w) {
        kll_copy_row(rows + (size_t)w * RW, imc, RW, lane);
        kll_fold(im0, imc, im1, S, CB, base, (uint32_t)w, budget, tail, lane);
        uint64_t* t = im0;
        im0 = im1;
        im1 = t;
    }
    return im0;
}

__global__ __launch_bounds__(64) void k_kll_merge(KllMergeArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const uint32_t RW = (uint32_t)kKllHdr + (uint32_t)A.budget + (uint32_t)A.tail;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const uint64_t* im = kll_fold_rows(A, s, smem, lane);
        uint64_t* o = A.out + (size_t)s * RW;
        for (uint32_t i = lane; i < RW; i += kWave) o[i] = im[i];
        __syncthreads();
    }
}

// Smallest body key K with (weight of body keys <= K) > r: bisection of the 64-bit
// order-preserving key space over the image's keys.
__device__ uint64_t kll_body_select(const uint64_t* im, const uint8_t* lvl, uint32_t m, uint64_t r, int lane) {
    uint64_t lo = 0, hi = ~0ull;
#pragma unroll 1
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        uint64_t c = 0;
        for (uint32_t i = lane; i < m; i += kWave) c += okey(im[kKllHdr + i]) <= mid ? (uint64_t)1 << lvl[i] : 0ull;
        c = lane_bcast64(wave_scan64(c, 0ull, OpAdd64{}), kWave - 1);
        lo = c > r ? lo : mid + 1;
        hi = c > r ? mid : hi;
    }
    return lo;
}

// A 32-bit value of lane ^ M (M a power of two < 64).
template <int M>
__device__ __forceinline__ uint32_t kll_lane_xor(uint32_t v) {
    if constexpr (M == 32) return (uint32_t)__shfl_xor((int)v, 32, kWave);
    else return kll_xor32<M>(v);
}
template <int M>
__device__ __forceinline__ void kll_kw_cross(uint64_t (&k)[8], uint32_t (&w)[8], bool take_min) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint64_t ok = ((uint64_t)kll_lane_xor<M>((uint32_t)(k[i] >> 32)) << 32) | kll_lane_xor<M>((uint32_t)k[i]);
        const uint32_t ow = kll_lane_xor<M>(w[i]);
        const bool mine = (k[i] < ok) == take_min || k[i] == ok;  // equal keys: either is the key
        k[i] = mine ? k[i] : ok;
        w[i] = mine ? w[i] : ow;
    }
}
__device__ __forceinline__ void kll_kw_cx(uint64_t& ka, uint32_t& wa, uint64_t& kb, uint32_t& wb, bool asc) {
    const bool sw = asc ? kb < ka : ka < kb;
    const uint64_t k0 = sw ? kb : ka, k1 = sw ? ka : kb;
    const uint32_t w0 = sw ? wb : wa, w1 = sw ? wa : wb;
    ka = k0; kb = k1; wa = w0; wb = w1;
}

// Weighted select over a row's body (m <= 512 keys, im[kKllHdr + i] with level lvl[i]) by ONE
// sort of (ordered key, weight 2^level) pairs across the wave and one prefix sum: for r0 and r1
// the smallest key whose weighted count of keys <= it exceeds r (the bisection's answer, bit for
// bit: inside a run of equal keys any order gives the same key).  Ordered-key space (okey).
template <int NQ>
__device__ __forceinline__ void kll_body_select2(const uint64_t* im, const uint8_t* lvl, uint32_t m, uint64_t r0,
                                                 uint64_t r1, int lane, uint64_t& out0, uint64_t& out1) {
    uint64_t k[8];
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t p = (uint32_t)lane * 8u + (uint32_t)i;
        k[i] = p < m ? okey(im[kKllHdr + p]) : ~0ull;
        w[i] = p < m ? (1u << lvl[p]) : 0u;
    }
#pragma unroll
    for (int kk = 2; kk <= 512; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j >= 8) {
                const int mm = j >> 3;
                const bool asc = (((uint32_t)lane * 8u) & (uint32_t)kk) == 0;
                const bool take_min = ((lane & mm) == 0) == asc;
                switch (mm) {
                    case 1: kll_kw_cross<1>(k, w, take_min); break;
                    case 2: kll_kw_cross<2>(k, w, take_min); break;
                    case 4: kll_kw_cross<4>(k, w, take_min); break;
                    case 8: kll_kw_cross<8>(k, w, take_min); break;
                    case 16: kll_kw_cross<16>(k, w, take_min); break;
                    default: kll_kw_cross<32>(k, w, take_min); break;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (!(i & j)) {
                        const bool asc = ((((uint32_t)lane * 8u + (uint32_t)i)) & (uint32_t)kk) == 0;
                        kll_kw_cx(k[i], w[i], k[i + j], w[i + j], asc);
                    }
            }
        }
    }
    uint64_t c[8], acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        acc += w[i];
        c[i] = acc;
    }
    const uint64_t base = wave_scan64(acc, 0ull, OpAdd64{}) - acc;  // exclusive over lanes
#pragma unroll 1
    for (int q = 0; q < NQ; ++q) {
        const uint64_t r = q ? r1 : r0;
        uint64_t sel = ~0ull;
        bool hit = false;
#pragma unroll
        for (int i = 7; i >= 0; --i) {
            const bool h = base + c[i] > r;
            sel = h ? k[i] : sel;
            hit = hit || h;
        }
        const uint64_t hm = ballot(hit);
        const uint64_t key = hm ? lane_bcast64(sel, __ffsll((long long)hm) - 1) : ~0ull;
        if (q) out1 = key;
        else out0 = key;
    }
}

__global__ __launch_bounds__(64) void k_kll_query(KllMergeArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const uint32_t budget = (uint32_t)A.budget;
    const uint32_t RW = (uint32_t)kKllHdr + budget + (uint32_t)A.tail;
    // W == 1: nothing to fold — the header and the tail are read from the row itself, and only
    // a body rank stages the body in LDS (the launch's LDS is then a body, not three rows)
    const bool direct = A.W == 1;
    uint64_t* bodyb = reinterpret_cast<uint64_t*>(smem);
    uint8_t* lvl = direct ? reinterpret_cast<uint8_t*>(bodyb + kKllHdr + budget)
                          : reinterpret_cast<uint8_t*>(reinterpret_cast<uint64_t*>(smem) + 3 * (size_t)RW +
                                                       5 * (size_t)budget);
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const uint64_t* im = direct ? A.rows + (size_t)s * RW : kll_fold_rows(A, s, smem, lane);
        const uint64_t n = im[0], nan = im[1];
        const uint32_t tl = (uint32_t)im[6];
        uint32_t m = 0;
        for (uint32_t h = 0; h < (uint32_t)kKllLevels; ++h) {
            const uint32_t l = kll_len(im, h);
            for (uint32_t i = lane; i < l; i += kWave) lvl[m + i] = (uint8_t)h;
            m += l;
        }
        __syncthreads();
        uint32_t flags = 0;
        double result = bitsd(kQuietNaN);
        if (im[15] != 0 || im[7] != (((uint64_t)budget << 32) | (uint32_t)A.tail)) {
            flags = KRR_FLAG_CAPACITY;
        } else if (nan) {
            flags = KRR_FLAG_NAN;
        } else if (n == 0) {
            flags = KRR_FLAG_EMPTY;
        } else {
            int64_t r0, r1;
            double gamma = 0.0;
            if (A.mode == KRR_PCT_SORTED_LOWER) {
                r0 = r1 = rule_rank((int64_t)n, A.p_num, A.p_den, A.ktab, A.ktab_len);
                if (!rule_covers((int64_t)n, A.ktab, A.ktab_len)) flags |= KRR_FLAG_CAPACITY;
            } else {
                const double vidx = __dmul_rn((double)(n - 1), A.q);
                if (vidx >= (double)(n - 1)) {
                    r0 = r1 = (int64_t)n - 1;
                    gamma = __dsub_rn(vidx, -1.0);
                } else {
                    const double fl = floor(vidx);
                    r0 = (int64_t)fl;
                    r1 = r0 + 1;
                    gamma = __dsub_rn(vidx, fl);
                }
            }
            double v[2];
            bool staged = false;
#ifndef KRR_KLL_X_BISECT
            // both ranks in the body: one sort of the body answers both
            const bool body0 = r0 != 0 && r0 != (int64_t)n - 1 && n - (uint64_t)r0 > tl;
            const bool body1 = r1 != 0 && r1 != (int64_t)n - 1 && n - (uint64_t)r1 > tl;
            uint64_t bk0 = 0, bk1 = 0;
            if ((body0 || body1) && m <= 512u)
                kll_body_select2<2>(im, lvl, m, (uint64_t)r0, (uint64_t)r1, lane, bk0, bk1);
#endif
#pragma unroll 1
            for (int qi = 0; qi < 2; ++qi) {
                const uint64_t r = (uint64_t)(qi ? r1 : r0);
                if (qi && r1 == r0) {
                    v[1] = v[0];
                    continue;
                }
                if (r == 0) v[qi] = bitsd(im[2]);
                else if (r == n - 1) v[qi] = bitsd(im[3]);
                else if (n - r <= tl) v[qi] = bitsd(im[kKllHdr + budget + tl - (n - r)]);
#ifndef KRR_KLL_X_BISECT
                else if (m <= 512u) v[qi] = bitsd(okey_inv(qi ? bk1 : bk0));
#endif
                else if (!direct) v[qi] = bitsd(okey_inv(kll_body_select(im, lvl, m, r, lane)));
                else {  // stage the body once (uniform branch: r is the same in every lane)
                    if (!staged) {
                        for (uint32_t i = lane; i < m; i += kWave) bodyb[kKllHdr + i] = im[kKllHdr + i];
                        __syncthreads();
                        staged = true;
                    }
                    v[qi] = bitsd(okey_inv(kll_body_select(bodyb, lvl, m, r, lane)));
                }
            }
            result = A.mode == KRR_PCT_SORTED_LOWER ? v[0] : np_lerp(v[0], v[1], gamma);
        }
        if (lane == 0) {
            A.out_v[s] = result;
            A.out_n[s] = (int64_t)n;
            A.out_f[s] = flags;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// The exact tail in a pass of its own (the default when tail > 0): k_kll_build runs without the
// tail buffer (A.tail_pass: fewer VGPRs live, the LDS of a tail-less build, so more waves per
// CU), then this pass streams each series slice again and keeps the keys >= a threshold tau0
// read from the row's own body: the body key at estimated rank q = n - tail - 1 - M, M the
// row's rank bound sqrt(2 ln(4/delta) sum w^2) at delta = 1e-3.  Every key >= tau0 is a
// candidate, so the buffer holds at least tail keys unless the body's estimate was off by more
// than M; then the slice is streamed once more with every present key a candidate.  Refreshes
// (tau rising, as in the build) keep the buffer within its capacity.  Either way the tail words
// are the top min(n, tail) present keys, exactly what the one-pass build writes: rows are the
// same bit for bit (oracle/kll_ref.py does not depend on how the tail is found).
#ifndef KRR_KLL_TAIL_MARGIN
#define KRR_KLL_TAIL_MARGIN 0.5  // the threshold's margin, in units of the rank bound at delta = 1e-3
#endif
#ifndef KRR_KLL_SPARSE_MARGIN
#define KRR_KLL_SPARSE_MARGIN 0.125  // the sparse pass's first margin (a miss retries at KRR_KLL_TAIL_RETRY x)
#endif
// The tail pass's threshold from the row's own body: the body key t0 at estimated rank
// q = n - tail - 1 - M (M = KRR_KLL_TAIL_MARGIN x the rank bound at delta = 1e-3); candidates are
// the keys > *tau (the next double below t0).  false: no usable threshold (every present key is
// a candidate).  im / lvl: LDS work space (the body keys and their levels).
__device__ bool kll_tail_tau(const uint64_t* row, uint32_t budget, uint32_t tail, double two_ln, uint64_t* im,
                             uint8_t* lvl, int lane, double* tau, double margin = KRR_KLL_TAIL_MARGIN) {
    const uint64_t n = uni64(row[0]);
    const double M = ceil(margin * sqrt(two_ln * (double)uni64(row[4])));
    const double qd = (double)n - (double)tail - 1.0 - M;
    bool full0 = false;
    *tau = 0.0;
    if (qd >= 0.0) {
        uint32_t m = 0;
        for (uint32_t h = 0; h < (uint32_t)kKllLevels; ++h) {
            const uint32_t l = kll_len(row, h);
            for (uint32_t i = lane; i < l; i += kWave) {
                lvl[m + i] = (uint8_t)h;
                im[kKllHdr + m + i] = row[kKllHdr + m + i];
            }
            m += l;
        }
        __syncthreads();
#ifndef KRR_KLL_X_BISECT
        uint64_t tk = 0, tk1 = 0;
        if (m <= 512u) kll_body_select2<1>(im, lvl, m, (uint64_t)qd, 0, lane, tk, tk1);
        else tk = kll_body_select(im, lvl, m, (uint64_t)qd, lane);
        const double t0 = bitsd(okey_inv(tk));
#else
        const double t0 = bitsd(okey_inv(kll_body_select(im, lvl, m, (uint64_t)qd, lane)));
#endif
        __syncthreads();
        if (t0 > -__builtin_inf()) {  // candidates: keys >= t0 (t0 == -inf: every present key)
            full0 = true;
            // the next double below t0 (bit arithmetic: no libm call in the kernel)
            const uint64_t tb0 = dbits(t0);
            *tau = t0 == 0.0 ? bitsd(0x8000000000000001ull) : bitsd(t0 > 0.0 ? tb0 - 1u : tb0 + 1u);
        }
    }
    return full0;
}

struct KllTailArgs {
    const double* vals;
    const int64_t* offs;
    int64_t S;
    int32_t budget;
    int32_t tail;
    uint32_t tcap;
    double two_ln;    // 2 ln(4 / delta)
    uint64_t* rows;
    const uint32_t* lines;  // the sparse pass: the body build's line maxima
    int64_t line_stride;
    const uint32_t* mask;   // optional: only series with mask[s] != 0 (the sparse pass's leftovers)
};

struct KllTailProc {
    KllShared sh;
    KllTail ts;
    uint32_t tail, tcap;
    int lane;
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
        double a[8], b[8], hi[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a[u] = c[u].x;
            b[u] = c[u].y;
            hi[u] = fmax(a[u], b[u]);  // one NaN: the present sample
        }
        kll_tail_filter(sh, ts, tail, tcap, lane, a, b, hi);
    }
};

#ifndef KRR_KLL_TAIL_STREAM
#define KRR_KLL_TAIL_STREAM 2  // kll_stream form of the tail pass (2: two ahead, copies; 3: unrolled by 3)
#endif
#ifndef KRR_KLL_TAIL_WAVES_PER_SIMD
#define KRR_KLL_TAIL_WAVES_PER_SIMD 2
#endif
__global__ __launch_bounds__(64, KRR_KLL_TAIL_WAVES_PER_SIMD) void k_kll_tail(KllTailArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const uint32_t budget = (uint32_t)A.budget, tail = (uint32_t)A.tail;
    const uint32_t RW = (uint32_t)kKllHdr + budget + tail;
    KllShared sh{};
    sh.tb = reinterpret_cast<uint64_t*>(smem);
    uint64_t* im = sh.tb;  // body keys at im[kKllHdr + i] (kll_body_select's layout), before the stream
    uint8_t* lvl = reinterpret_cast<uint8_t*>(im + kKllHdr + budget);
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        if (A.mask && !A.mask[s]) continue;
        uint64_t* row = A.rows + (size_t)s * RW;
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        double tau = 0.0;
        bool full0 = kll_tail_tau(row, budget, tail, A.two_ln, im, lvl, lane, &tau);
        const int64_t nch = kll_nchunks(beg, end);
        const int64_t npad = KRR_KLL_TAIL_STREAM == 3 ? (nch + 2) / 3 * 3 : (nch + 1) & ~(int64_t)1;
        KllTailProc P{sh, KllTail{0u, full0 ? 1u : 0u, tau}, tail, A.tcap, lane};
        uint32_t restreams = 0;
#pragma unroll 1
        for (int pass = 0; pass < 2; ++pass) {
            kll_stream<KllTailProc, KRR_KLL_TAIL_STREAM>(A.vals, beg, end, npad, P, lane);
            if (!(full0 && P.ts.tl < tail)) break;
            full0 = false;  // the estimate missed: once more, every present key a candidate
            P.ts = KllTail{0u, 0u, 0.0};
            ++restreams;
        }
        (void)restreams;
        const uint32_t tl_out = kll_tail_export(sh, P.ts, tail, row + kKllHdr + budget, lane);
        if (lane == 0) row[6] = tl_out;
#ifdef KRR_KLL_X_STATS  // refreshes | counting passes << 24 | (full restreams << 8 | sort fallbacks) << 48
        if (lane == 0)
            row[14] = ((uint64_t)((restreams << 8) | P.ts.nfall) << 48) | ((uint64_t)P.ts.npass << 24) | P.ts.nref;
#endif
        __syncthreads();
    }
}

}  // namespace krr
namespace krr {

// ---------------------------------------------------------------------------------------------
// The sparse tail pass (round 5): candidates are the keys > tau, and a line (16 slots, 128 B)
// whose maximum from the body build (k_kll_build<false, true>: kll_line_key per line) is below
// tau holds none — so only the lines that can hold a candidate are read.  Their ids queue in
// LDS (64 per virtual chunk: row r of the virtual chunk = 8 queued lines, 8 lanes each) and
// each virtual chunk goes through the same candidate filter as a streamed chunk.  The tail is a
// set (the top min(n, tail) present keys, exported sorted), so the order lines arrive in does
// not change it: the rows equal k_kll_tail's bit for bit.  If the threshold missed (fewer than
// `tail` candidates) the slice is streamed whole with every present key a candidate, as there.
// Reads: the line maxima (1/32 of the slice) + the flagged lines (~20% at p99 of 30d@15s).
#ifndef KRR_KLL_TAIL_RETRY
#define KRR_KLL_TAIL_RETRY 4.0  // a sparse attempt that missed is retried at this many margins
#endif
#ifndef KRR_KLL_SPARSE_PIPE
#define KRR_KLL_SPARSE_PIPE 1  // one batch of flagged lines in flight while the previous one is filtered
#endif
struct KllLineTailArgs {
    KllTailArgs T;
    uint32_t queue_off;     // byte offset of the 128-entry line queue in LDS
    uint32_t* lines_read;   // optional: per series, the lines this pass read (its bytes / 128)
};

__global__ __launch_bounds__(64, KRR_KLL_TAIL_WAVES_PER_SIMD) void k_kll_tail_lines(KllLineTailArgs LA) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const KllTailArgs& A = LA.T;
    const int lane = threadIdx.x;
    const uint32_t budget = (uint32_t)A.budget, tail = (uint32_t)A.tail;
    const uint32_t RW = (uint32_t)kKllHdr + budget + tail;
    KllShared sh{};
    sh.tb = reinterpret_cast<uint64_t*>(smem);
    uint64_t* im = sh.tb;
    uint8_t* lvl = reinterpret_cast<uint8_t*>(im + kKllHdr + budget);
    uint32_t* q = reinterpret_cast<uint32_t*>(smem + LA.queue_off);
    const double2* __restrict__ v2 = reinterpret_cast<const double2*>(A.vals);
    const double qnan = __builtin_nan("");
    constexpr int64_t CH = (int64_t)kUnroll * kWave;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        uint64_t* row = A.rows + (size_t)s * RW;
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        const int64_t nch = kll_nchunks(beg, end);
        double tau = 0.0;
        bool full0 = kll_tail_tau(row, budget, tail, A.two_ln, im, lvl, lane, &tau, KRR_KLL_SPARSE_MARGIN);
        KllTailProc P{sh, KllTail{0u, full0 ? 1u : 0u, tau}, tail, A.tcap, lane};
        bool dense = !full0;
        uint32_t nread = 0;  // lines read (uniform)
#ifdef KRR_KLL_X_SPARSE_NOFILTER  // profiling variant: the lines are loaded, not filtered (rows not valid)
        double xsink = 0.0;
#define KLL_SPARSE_CHUNK(c)                                                  \
    do {                                                                     \
        _Pragma("unroll") for (int r_ = 0; r_ < kUnroll; ++r_) xsink = fmax(xsink, fmax((c)[r_].x, (c)[r_].y)); \
    } while (0)
#else
#define KLL_SPARSE_CHUNK(c) P.chunk(c)
#endif
        // sparse attempts: the threshold at the margin, then (a miss: fewer than `tail` keys above
        // it) at KRR_KLL_TAIL_RETRY margins; then the whole slice, every present key a candidate
#pragma unroll 1
        for (int attempt = 0; attempt < 2 && full0 && nch > 0; ++attempt) {
            if (attempt == 1) {
                __syncthreads();
                full0 = kll_tail_tau(row, budget, tail, A.two_ln, im, lvl, lane, &tau,
                                     KRR_KLL_TAIL_RETRY * KRR_KLL_SPARSE_MARGIN);
                __syncthreads();
                P.ts = KllTail{0u, full0 ? 1u : 0u, tau};
                if (!full0) break;
            }
            // kll_stream's layout of this slice
            int64_t a0 = (beg + 1) & ~(int64_t)1;
            if (a0 > end) a0 = end;
            int64_t a1 = end & ~(int64_t)1;
            if (a1 < a0) a1 = a0;
            const int64_t i0 = a0 >> 1, nunits = (a1 >> 1) - i0, nfull = nunits / CH;
            const double hv = a0 > beg ? A.vals[beg] : qnan, tv = a1 < end ? A.vals[a1] : qnan;
            const uint32_t t32 = (uint32_t)(okey(dbits(tau)) >> 32);
            const uint32_t* L = A.lines + (size_t)s * (size_t)A.line_stride;
            // the lines of queue slots [0, cnt) loaded into c (row r = slots 8r .. 8r + 7)
            auto load_batch = [&](uint32_t cnt, double2 (&c)[kUnroll]) __attribute__((always_inline)) {
#pragma unroll
                for (int r = 0; r < kUnroll; ++r) {
                    const uint32_t slot = (uint32_t)r * 8u + ((uint32_t)lane >> 3);
                    const uint32_t id = slot < cnt ? q[slot] : 0xFFFFFFFFu;
                    c[r] = make_double2(qnan, qnan);
                    if (id != 0xFFFFFFFFu) {
                        const int64_t ci = id >> 6;
                        const uint32_t u = (id >> 3) & 7u, ln = (id & 7u) * 8u + ((uint32_t)lane & 7u);
                        const int64_t j = ci * CH + (int64_t)u * kWave + ln;
                        if (ci < nfull || j < nunits) c[r] = load16(v2 + i0 + j);
                        if (ci >= nfull && ci == nch - 1 && u == (uint32_t)kUnroll - 1 && ln == (uint32_t)kWave - 1)
                            c[r] = make_double2(hv, tv);  // the head / tail slots ride the last chunk
                    }
                }
                __syncthreads();  // the queue entries are read: the caller may shift it
            };
            uint32_t qn = 0;  // queued lines (uniform)
#if KRR_KLL_SPARSE_PIPE
            // one batch in flight: a full batch's lines are loaded when it fills and filtered
            // when the next one fills (or at the end), so the loads overlap the scan of the
            // maxima and the previous batch's filter; the batches keep their order
            double2 cp[kUnroll];
            bool pend = false;
#endif
            // the line maxima of 8 chunks at a time, the next 8 in flight while these are queued
            uint32_t nk[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) nk[c] = c < nch ? L[(size_t)c * 64u + lane] : 0u;
#pragma unroll 1
            for (int64_t cb = 0; cb < nch; cb += 8) {
                uint32_t lk[8];
#pragma unroll
                for (int c = 0; c < 8; ++c) lk[c] = nk[c];
#pragma unroll
                for (int c = 0; c < 8; ++c) nk[c] = cb + 8 + c < nch ? L[(size_t)(cb + 8 + c) * 64u + lane] : 0u;
#pragma unroll
                for (int c = 0; c < 8; ++c) {
#ifndef KRR_KLL_X_SPARSE_NOLOAD
                    const uint64_t m = ballot(cb + c < nch && lk[c] >= t32);
#else  // profiling variant: the maxima are scanned, no line is read (rows not valid)
                    const uint64_t m = ballot(cb + c < nch && lk[c] >= t32 && t32 == 0xFFFFFFFFu);
#endif
                    if (!m) continue;
                    if ((m >> lane) & 1ull) q[qn + lane_prefix(m)] = (uint32_t)((cb + c) * 64 + lane);
                    qn += popc64(m);
                    nread += popc64(m);
                    __syncthreads();
                    if (qn >= 64u) {
#if KRR_KLL_SPARSE_PIPE
                        double2 cn[kUnroll];
                        load_batch(64u, cn);
                        if (pend) KLL_SPARSE_CHUNK(cp);
#pragma unroll
                        for (int r = 0; r < kUnroll; ++r) cp[r] = cn[r];
                        pend = true;
#else
                        double2 cn[kUnroll];
                        load_batch(64u, cn);
                        KLL_SPARSE_CHUNK(cn);
#endif
                        const uint32_t rest = qn - 64u;  // < 64
                        const uint32_t v = (uint32_t)lane < rest ? q[64 + lane] : 0u;
                        __syncthreads();
                        if ((uint32_t)lane < rest) q[lane] = v;
                        __syncthreads();
                        qn = rest;
                    }
                }
            }
#if KRR_KLL_SPARSE_PIPE
            if (pend) KLL_SPARSE_CHUNK(cp);
#endif
            if (qn) {
                double2 cn[kUnroll];
                load_batch(qn, cn);
                KLL_SPARSE_CHUNK(cn);
            }
            dense = P.ts.tl < tail;  // a miss
#if defined(KRR_KLL_X_SPARSE_NOFILTER) || defined(KRR_KLL_X_SPARSE_NOLOAD)
            dense = false;  // profiling variants: no retry, no restream
#endif
            if (!dense) break;
        }
        if (dense) P.ts = KllTail{0u, 0u, 0.0};  // the whole slice, every present key a candidate
        if (dense) {
            const int64_t npad = KRR_KLL_TAIL_STREAM == 3 ? (nch + 2) / 3 * 3 : (nch + 1) & ~(int64_t)1;
            kll_stream<KllTailProc, KRR_KLL_TAIL_STREAM>(A.vals, beg, end, npad, P, lane);
            nread += (uint32_t)nch * 64u;
        }
#ifndef KRR_KLL_X_SPARSE_NOEXPORT
        const uint32_t tl_out = kll_tail_export(sh, P.ts, tail, row + kKllHdr + budget, lane);
#else  // profiling variant: no sort / export (rows not valid)
        const uint32_t tl_out = P.ts.tl;
#endif
        if (lane == 0) {
            row[6] = tl_out;
            if (LA.lines_read) LA.lines_read[s] = nread;
        }
#ifdef KRR_KLL_X_SPARSE_NOFILTER
        if (lane == 0) row[15] = dbits(xsink);
#endif
        __syncthreads();
    }
}

}  // namespace krr
