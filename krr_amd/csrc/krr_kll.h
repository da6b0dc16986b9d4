// krr_kll.h — KLL-style compactor sketch with a data-independent rank-error bound
// (config 5, sketch-only mode; included by krr_kernels.hip after the streaming skeleton).
//
// north_star names "an optional mergeable t-digest/KLL sketch mode" whose rank error is
// reported.  The log-linear histogram (k_sketch_build) bounds the VALUE error only; this
// one bounds the RANK error whatever the data (low dispersion, heavy quantisation, ties).
//
// One wave per series slice streams it once (stream_segment, 1,024 slots per chunk).  A
// COMPACTION keeps the keys at sorted positions off, off+2, ... (off a coin from a counter
// hash of (seed, series, slice, level, count)) and doubles their weight:
//   * level 0, per lane: the lane's 16 slots of a chunk are sorted in registers (NaN slots
//     sort last and are dropped) and compacted to <= 8 keys of weight 2;
//   * level 1, per lane: the runs of two consecutive chunks are merged in registers and
//     compacted to <= 8 keys of weight 4;
//   * level 2, per wave (every other chunk): the 64 lanes' weight-4 keys are sorted across
//     the wave (bitonic network: DPP / ds_swizzle exchanges) and compacted to a run of
//     <= 256 keys of weight 8, pushed to level 3;
//   * level h >= 3 holds at most one sorted run (LDS).  Pushing a run onto a full level
//     merges the two runs (merge-path positions by binary search) and compacts the merge:
//     <= 256 keys of weight 2^(h+1) go up — a binary counter of runs;
//   * at the end, while more than `budget` keys remain, the lowest run is compacted alone
//     and pushed up; the runs are exported as one fixed-size row.
// A slice of <= budget present samples that fits one chunk is exported whole (weight 1):
// short series are exact.
//
// Rank error: a compaction of weight-w keys moves the weighted rank of any fixed value by
// 0 or +-w, zero-mean over its coin, independently; so |error| <= sqrt(2 ln(2/delta) sum w^2)
// with probability >= 1 - delta (Hoeffding), plus one key's weight for the answer's own
// granularity.  sum w^2 is exported per row and merged by addition: the bound depends on
// n and the compaction schedule only, never on the values.
//
// Rows merge across time slices by concatenation (all-to-all to the series' owner, as the
// window export); k_kll_query stages a series' W rows in LDS and bisects the 64-bit key
// space for the smallest key whose weighted count passes rank r * total_weight / n.
#pragma once

namespace krr {

constexpr int kKllBlock = 512;   // level-0 block (half a streaming chunk)
constexpr int kKllRun = 256;     // keys per run at levels >= 1
constexpr int kKllLevels = 16;   // run slots: level 0 (whole short slices) .. 15
constexpr int kKllHdr = 10;      // header words of an exported row
constexpr uint64_t kKllNanKey = ~0ull;  // okey space: above every key (query bisection bound)
constexpr uint64_t kKllAbsent = 0x7FF0000000000000ull;  // +inf: an absent (NaN) slot sorts last
constexpr uint32_t kKllFirst = 3;  // first LDS run level (levels 0-2 are the lane and wave stages)
constexpr uint32_t kKllLane0 = 32, kKllLane1 = 96;  // coin "levels" of lane l's compactions: 32 + l, 96 + l

// Row layout (uint64 words): [0] present samples  [1] NaN samples (compact layout; 0 with
// gaps)  [2] min  [3] max (f64 bits, NaN when empty)  [4..7] run lengths, u16 x 16, level
// h at bits 16(h & 3) of word 4 + h/4  [8] sum over compactions of w^2  [9] total weight
// (sum of len_h 2^h)  [10 ..] keys (f64 bits), level 0 first, then level 1, 2, ...
// Keys are the sample values with -0 folded into +0 (the sketch keeps no zero sign), so
// f64 min / max and compares order them totally (NaN slots are absent and never kept).
// Within a run the keys ascend, except level 0 = block 0's keys then block 1's.

__host__ __device__ inline uint64_t kll_mix(uint64_t z) {  // splitmix64 finaliser
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// Compaction offset (0 or 1) of the `cnt`-th compaction at `level` of a series' slice.
__host__ __device__ inline uint32_t kll_coin(uint64_t seed, uint64_t series, uint32_t slice, uint32_t level,
                                             uint32_t cnt) {
    const uint64_t x = seed + 0x9E3779B97F4A7C15ull * (series + 1) + 0xD1B54A32D192ED03ull * ((uint64_t)slice + 1) +
                       0x8CB92BA72F3D8DD7ull * (((uint64_t)level << 32) | cnt);
    return (uint32_t)(kll_mix(x) >> 63);
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

// Highest run level a segment of `len` slots can reach: level 3 receives one run per two
// chunks, the runs form a binary counter, the final compression may carry one level more.
__host__ __device__ inline int kll_levels(int64_t len) {
    const int64_t pushes = (kll_nchunks(0, len) + 2) / 2 + 1;
    int lg = 0;
    while ((int64_t(1) << (lg + 1)) <= pushes) ++lg;
    return (int)kKllFirst + lg + 1;
}

struct KllBuildArgs {
    const double* vals;
    const int64_t* offs;
    int64_t S;
    int32_t gaps;
    int32_t budget;
    int32_t levels;   // highest run level (LDS slots for levels kKllFirst..levels)
    uint32_t slice;
    uint64_t seed;
    int64_t seg_base;
    uint64_t* rows;   // [S][kKllHdr + budget]
};

// Compare-exchange of two keys (f64 bits; no NaN, no -0): after it, a holds the min if asc,
// else the max — v_min_f64 / v_max_f64, two instructions when asc is known at compile time.
__device__ __forceinline__ void kll_cx(uint64_t& a, uint64_t& b, bool asc) {
    const double x = bitsd(a), y = bitsd(b);
    const double lo = fmin(x, y), hi = fmax(x, y);
    a = dbits(asc ? lo : hi);
    b = dbits(asc ? hi : lo);
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
__device__ __forceinline__ uint64_t kll_xor64(uint64_t x) {
    if constexpr (M == 32) {  // across the 32-lane halves
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)x, 32, kWave);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), 32, kWave);
        return ((uint64_t)hi << 32) | lo;
    }
    return ((uint64_t)kll_xor32<M>((uint32_t)(x >> 32)) << 32) | kll_xor32<M>((uint32_t)x);
}

template <int M, int N>
__device__ __forceinline__ void kll_cross(uint64_t (&x)[N], bool take_min) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const double o = bitsd(kll_xor64<M>(x[i])), v = bitsd(x[i]);
        x[i] = dbits(take_min ? fmin(v, o) : fmax(v, o));
    }
}

// In-lane substeps j = J, J/2, .., 1 of bitonic stage k on the lane's 16 keys
// (position = lane * 16 + i; direction from bit k of the position, all ascending at k = 512).
template <int J>
__device__ __forceinline__ void kll_inlane(uint64_t (&x)[16], uint32_t k, int lane) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i & J) continue;
        const uint32_t pos = (uint32_t)lane * 16u + (uint32_t)i;
        const bool asc = k >= (uint32_t)kKllBlock || (pos & k) == 0;
        kll_cx(x[i], x[i + J], asc);
    }
    if constexpr (J > 1) kll_inlane<J / 2>(x, k, lane);
}

// Sort each 512-key block (lanes 0-31: block 0, lanes 32-63: block 1) ascending.
__device__ __forceinline__ void kll_sort_blocks(uint64_t (&x)[16], int lane) {
    kll_inlane<1>(x, 2, lane);
    kll_inlane<2>(x, 4, lane);
    kll_inlane<4>(x, 8, lane);
    kll_inlane<8>(x, 16, lane);
#pragma unroll 1
    for (uint32_t k = 32; k <= (uint32_t)kKllBlock; k <<= 1) {
        const bool asc = k >= (uint32_t)kKllBlock || (((uint32_t)lane * 16u) & k) == 0;
#pragma unroll 1
        for (uint32_t j = k >> 1; j >= 16; j >>= 1) {
            const int m = (int)(j >> 4);
            const bool take_min = ((lane & m) == 0) == asc;  // the lower lane of the pair keeps the min if ascending
            switch (m) {  // wave-uniform
                case 1: kll_cross<1, 16>(x, take_min); break;
                case 2: kll_cross<2, 16>(x, take_min); break;
                case 4: kll_cross<4, 16>(x, take_min); break;
                case 8: kll_cross<8, 16>(x, take_min); break;
                default: kll_cross<16, 16>(x, take_min); break;
            }
        }
        kll_inlane<8>(x, k, lane);
    }
}

// The lane's 16 keys ascending (a full bitonic sort in registers).
__device__ __forceinline__ void kll_sort16(uint64_t (&x)[16]) {
#pragma unroll
    for (int k = 2; k <= 16; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (!(i & j)) kll_cx(x[i], x[i + j], k == 16 || (i & k) == 0);
        }
    }
}

// z[0, 8) and z[8, 16) ascending -> z ascending (reverse the second half: bitonic; clean).
__device__ __forceinline__ void kll_merge16(uint64_t (&z)[16]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t t = z[8 + i];
        z[8 + i] = z[15 - i];
        z[15 - i] = t;
    }
#pragma unroll
    for (int j = 8; j > 0; j >>= 1) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (!(i & j)) kll_cx(z[i], z[i + j], true);
    }
}

// 512 keys ascending across the wave: lane l holds positions 8l .. 8l+7, each lane's 8
// already ascending (odd lanes' runs are reversed first, so stage 16 starts bitonic).
__device__ __forceinline__ void kll_sort512(uint64_t (&y)[8], int lane) {
    if (lane & 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t t = y[i];
            y[i] = y[7 - i];
            y[7 - i] = t;
        }
    }
#pragma unroll 1
    for (uint32_t k = 16; k <= 512; k <<= 1) {
        const bool asc = k >= 512 || (((uint32_t)lane * 8u) & k) == 0;
#pragma unroll 1
        for (uint32_t j = k >> 1; j >= 8; j >>= 1) {
            const int m = (int)(j >> 3);
            const bool take_min = ((lane & m) == 0) == asc;
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
                if (!(i & j)) kll_cx(y[i], y[i + j], asc);
        }
    }
}

// Merge-path step of a merge-compaction: every key X[i] (i = lane + 64 q, i < nx <= 256)
// lands at merged position p = i + #(Y < X[i]) (STRICT: X's keys go before Y's equal keys)
// or i + #(Y <= X[i]); positions off, off + 2, ... are kept, at O[(p - off) / 2].  The four
// binary searches of a lane advance together (their LDS reads overlap), 9 halvings each
// (ny <= 256).
template <bool STRICT>
__device__ __forceinline__ void kll_merge_half(const uint64_t* X, uint32_t nx, const uint64_t* Y, uint32_t ny,
                                               uint32_t off, uint64_t* O, int lane) {
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
        if (i < nx && p >= off && ((p - off) & 1u) == 0) O[(p - off) >> 1] = v[q];
    }
}

struct KllState {
    uint64_t* tmp;      // two LDS runs of kKllRun keys (tb(0), tb(1))
    uint64_t* lv;       // LDS runs, level h at lv + (h - 1) * kKllRun
    uint32_t* lens;     // LDS [kKllLevels]
    uint32_t* cnt;      // LDS [kKllLevels] compactions done per level
    uint64_t seed, series;
    uint32_t slice;
    uint64_t sum_w2;    // wave-uniform
    uint32_t overflow;  // a run above the provisioned levels (never expected)
    int lane;

    __device__ __forceinline__ uint64_t* run(uint32_t h) const { return lv + (size_t)(h - kKllFirst) * kKllRun; }
    __device__ __forceinline__ uint64_t* tb(uint32_t sel) const { return tmp + (size_t)sel * kKllRun; }

    // Level 2: the lanes' weight-4 keys (y ascending per lane, NaN keys past cy) sorted
    // across the wave, compacted to <= 256 keys of weight 8, pushed to level 3.
    __device__ void wave_stage(uint64_t (&y)[8], uint32_t cy, int levels) {
        const uint32_t C = wave_sum_u32(cy);
        if (C == 0) return;
        kll_sort512(y, lane);
        const uint32_t c = uni32(cnt[2]);
        const uint32_t off = kll_coin(seed, series, slice, 2, c);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t p = (uint32_t)lane * 8u + (uint32_t)i;
            if (p < C && p >= off && ((p - off) & 1u) == 0) tb(0)[(p - off) >> 1] = y[i];
        }
        sum_w2 += 16;
        __syncthreads();
        if (lane == 0) cnt[2] = c + 1;
        __syncthreads();
        push(0, C > off ? (C - off + 1) >> 1 : 0u, kKllFirst, levels);
    }

    // Push the run tmp[t_sel][0, t) at level h (>= kKllFirst): store it, or merge-compact and carry.
    __device__ void push(uint32_t t_sel, uint32_t t, uint32_t h, int levels) {
        while (t) {  // an empty run changes nothing
            if ((int)h > levels) {
                overflow = 1;
                return;
            }
            const uint32_t a = uni32(lens[h]);
            const uint64_t* T = tb(t_sel);
            if (a == 0) {
                uint64_t* L = run(h);
                for (uint32_t i = lane; i < t; i += kWave) L[i] = T[i];
                __syncthreads();
                if (lane == 0) lens[h] = t;
                __syncthreads();
                return;
            }
            const uint32_t c = uni32(cnt[h]);
            const uint32_t off = kll_coin(seed, series, slice, h, c);
            const uint64_t* A = run(h);
            uint64_t* O = tb(t_sel ^ 1);
            kll_merge_half<true>(A, a, T, t, off, O, lane);  // A's keys before T's equal keys
            kll_merge_half<false>(T, t, A, a, off, O, lane);
            sum_w2 += (uint64_t)1 << (2 * h);
            __syncthreads();
            if (lane == 0) {
                lens[h] = 0;
                cnt[h] = c + 1;
            }
            __syncthreads();
            t = (a + t > off) ? (a + t - off + 1) >> 1 : 0;
            t_sel ^= 1;
            ++h;
        }
    }
};

__global__ __launch_bounds__(64) void k_kll_build(KllBuildArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    KllState K;
    K.tmp = reinterpret_cast<uint64_t*>(smem);
    K.lv = K.tmp + 2 * kKllRun;
    K.lens = reinterpret_cast<uint32_t*>(K.lv + (size_t)(A.levels - (int)kKllFirst + 1) * kKllRun);
    K.cnt = K.lens + kKllLevels;
    K.seed = A.seed;
    K.slice = A.slice;
    K.lane = lane;
    const uint32_t RW = (uint32_t)(kKllHdr + A.budget);
    const int blk = lane >> 5;                 // this lane's level-0 block
    const uint32_t bpos = (uint32_t)(lane & 31) * 16u;  // its first position in the block
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        if (lane < kKllLevels) {
            K.lens[lane] = 0;
            K.cnt[lane] = 0;
        }
        __syncthreads();
        K.series = (uint64_t)(A.seg_base + s);
        K.sum_w2 = 0;
        K.overflow = 0;
        const bool whole = kll_nchunks(beg, end) <= 1;  // one chunk: kept exactly if it fits the budget
        uint64_t* row = A.rows + (size_t)s * RW;

        struct Proc {  // by value: nothing here is address-taken (no scratch)
            KllState K;
            int budget, levels;
            uint64_t* row;
            int lane, blk;
            uint32_t bpos;
            bool whole;
            uint32_t nan_l, pres_l;
            uint32_t c_whole[2];
            double kmin, kmax;   // NaN until a present sample
            bool have;           // a level-1 run is pending in pend (wave-uniform)
            uint32_t cpend;      // its present keys
            uint32_t ci;         // chunks seen
            uint64_t pend[8];
            __device__ void chunk(const double2 (&c)[kUnroll]) {
                uint64_t x[16];
                uint32_t valid = 0;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const double d = slot_val(c, j);
                    const bool nan = __builtin_isnan(d);
                    const double v = d == 0.0 ? 0.0 : d;  // -0 -> +0
                    x[j] = nan ? kKllAbsent : dbits(v);
                    valid += nan ? 0u : 1u;
                    kmin = fmin(kmin, d == 0.0 ? 0.0 : d);  // fmin / fmax skip NaN
                    kmax = fmax(kmax, d == 0.0 ? 0.0 : d);
                }
                nan_l += 16u - valid;
                pres_l += valid;
                if (whole) {  // the only chunk: kept whole if it fits the budget
                    // present keys per block (lanes 0-31 / 32-63)
                    const uint32_t incl = wave_scan32(valid, 0u, OpAdd32{});
                    const uint32_t c0 = lane_bcast32(incl, 31), c1 = lane_bcast32(incl, kWave - 1) - c0;
                    c_whole[0] = c0;
                    c_whole[1] = c1;
                    if (c0 + c1 <= (uint32_t)budget) {  // level 0, block 0's keys then block 1's, sorted
                        kll_sort_blocks(x, lane);
                        const uint32_t base = blk ? c0 : 0u, cb = blk ? c1 : c0;
#pragma unroll
                        for (int i = 0; i < 16; ++i)
                            if (bpos + (uint32_t)i < cb) row[kKllHdr + base + bpos + i] = x[i];
                        return;
                    }
                }
                // level 0 (per lane): sort the lane's 16 slots, keep every other from a coin
                kll_sort16(x);
                const uint32_t off = kll_coin(K.seed, K.series, K.slice, kKllLane0 + lane, ci);
                uint64_t y[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) y[m] = off ? x[2 * m + 1] : x[2 * m];  // NaN keys stay past cy
                const uint32_t cy = valid > off ? (valid - off + 1) >> 1 : 0u;
                K.sum_w2 += popc64(ballot(valid > 0));
                if (!have) {
#pragma unroll
                    for (int m = 0; m < 8; ++m) pend[m] = y[m];
                    cpend = cy;
                    have = true;
                } else {  // level 1 (per lane): merge with the pending run, compact
                    uint64_t z[16];
#pragma unroll
                    for (int m = 0; m < 8; ++m) {
                        z[m] = pend[m];
                        z[8 + m] = y[m];
                    }
                    kll_merge16(z);
                    const uint32_t cz = cpend + cy;
                    const uint32_t off1 = kll_coin(K.seed, K.series, K.slice, kKllLane1 + lane, ci >> 1);
                    uint64_t y2[8];
#pragma unroll
                    for (int m = 0; m < 8; ++m) y2[m] = off1 ? z[2 * m + 1] : z[2 * m];
                    K.sum_w2 += 4ull * popc64(ballot(cz > 0));
                    have = false;
                    K.wave_stage(y2, cz > off1 ? (cz - off1 + 1) >> 1 : 0u, levels);
                }
                ++ci;
            }
        } P{K, A.budget, A.levels, row, lane, blk, bpos, whole, 0u, 0u, {0u, 0u}, bitsd(kQuietNaN), bitsd(kQuietNaN),
            false, 0u, 0u, {}};

        const uint32_t pad = stream_segment<true>(A.vals, beg, end, P, lane);
        if (P.have) {  // an odd last chunk: its level-1 run is compacted alone
            const uint32_t off1 = kll_coin(P.K.seed, P.K.series, P.K.slice, kKllLane1 + lane, P.ci >> 1);
            uint64_t y2[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) y2[m] = (m < 4) ? (off1 ? P.pend[2 * m + 1] : P.pend[2 * m]) : kKllAbsent;
            P.K.sum_w2 += 4ull * popc64(ballot(P.cpend > 0));
            P.K.wave_stage(y2, P.cpend > off1 ? (P.cpend - off1 + 1) >> 1 : 0u, A.levels);
        }
        K = P.K;
        const uint32_t nan_l = P.nan_l, pres_l = P.pres_l, c_whole[2] = {P.c_whole[0], P.c_whole[1]};
        const uint64_t n_nan = (uint64_t)wave_sum_u32(nan_l) - pad;
        const uint64_t n_pres = wave_sum_u32(pres_l);
        const uint64_t gmin = lane_bcast64(wave_scan64(dbits(P.kmin), kQuietNaN, OpMinF64Bits{}), kWave - 1);
        const uint64_t gmax = lane_bcast64(wave_scan64(dbits(P.kmax), kQuietNaN, OpMaxF64Bits{}), kWave - 1);
        const bool exact0 = whole && c_whole[0] + c_whole[1] <= (uint32_t)A.budget;
        // final compression: the lowest run alone, until the budget holds
        if (!exact0) {
#pragma unroll 1
            while (true) {
                uint32_t total = 0, low = 0;
#pragma unroll 1
                for (int h = A.levels; h >= (int)kKllFirst; --h) {
                    const uint32_t l = uni32(K.lens[h]);
                    total += l;
                    low = l ? (uint32_t)h : low;
                }
                if (total <= (uint32_t)A.budget || low == 0 || K.overflow) break;
                const uint32_t a = uni32(K.lens[low]);
                const uint32_t c = uni32(K.cnt[low]);
                const uint32_t off = kll_coin(K.seed, K.series, K.slice, low, c);
                const uint64_t* L = K.run(low);
                uint64_t keep[kKllRun / kWave / 2];
#pragma unroll
                for (int q = 0; q < kKllRun / kWave / 2; ++q) {
                    const uint32_t p = off + 2u * ((uint32_t)lane + (uint32_t)q * kWave);  // output index -> position
                    keep[q] = p < a ? L[p] : 0ull;
                }
                K.sum_w2 += (uint64_t)1 << (2 * low);
                __syncthreads();
                const uint32_t t = a > off ? (a - off + 1) >> 1 : 0u;
#pragma unroll
                for (int q = 0; q < kKllRun / kWave / 2; ++q) {
                    const uint32_t m = (uint32_t)lane + (uint32_t)q * kWave;
                    if (m < t) K.tb(0)[m] = keep[q];
                }
                if (lane == 0) {
                    K.lens[low] = 0;
                    K.cnt[low] = c + 1;
                }
                __syncthreads();
                K.push(0, t, low + 1, A.levels);
            }
        }
        // export: header, then the runs in level order
        uint64_t wtot = 0, lw0 = 0, lw1 = 0, lw2 = 0, lw3 = 0;  // run lengths, u16 x 4 per word
        uint32_t pos = 0;
        if (exact0) {
            wtot = c_whole[0] + c_whole[1];
            lw0 = wtot;
            pos = (uint32_t)wtot;
        } else {
#pragma unroll 1
            for (int h = (int)kKllFirst; h <= A.levels && h < kKllLevels; ++h) {
                const uint32_t l = uni32(K.lens[h]);
                if (!l) continue;
                if (pos + l > (uint32_t)A.budget) {  // only after an overflow
                    K.overflow = 1;
                    break;
                }
                const uint64_t* L = K.run((uint32_t)h);
                for (uint32_t i = lane; i < l; i += kWave) row[kKllHdr + pos + i] = L[i];
                pos += l;
                wtot += (uint64_t)l << h;
                const uint64_t f = (uint64_t)l << (16 * (h & 3));
                lw0 |= (h >> 2) == 0 ? f : 0ull;
                lw1 |= (h >> 2) == 1 ? f : 0ull;
                lw2 |= (h >> 2) == 2 ? f : 0ull;
                lw3 |= (h >> 2) == 3 ? f : 0ull;
            }
        }
        if (lane == 0) {
            row[0] = n_pres;
            row[1] = A.gaps ? 0ull : n_nan;
            row[2] = n_pres ? gmin : kQuietNaN;
            row[3] = n_pres ? gmax : kQuietNaN;
            row[4] = lw0;
            row[5] = lw1;
            row[6] = lw2;
            row[7] = lw3;
            row[8] = K.overflow ? ~0ull : K.sum_w2;
            row[9] = wtot;
        }
        __syncthreads();
    }
}

struct KllQueryArgs {
    int64_t S;
    int32_t W;        // rows per series (time slices)
    int32_t budget;
    const uint64_t* rows;  // [S][W][kKllHdr + budget]
    int32_t mode;
    int64_t p_num, p_den;
    double q;
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
};

// Smallest key K with (weighted count of keys <= K) * n > r * wtot (an item's key).
__device__ uint64_t kll_select(const uint64_t* key, const uint8_t* lvl, uint32_t m, uint64_t r, uint64_t n,
                               uint64_t wtot, int lane) {
    uint64_t lo = 0, hi = kKllNanKey;
#pragma unroll 1
    while (lo < hi) {
        const uint64_t mid = lo + ((hi - lo) >> 1);
        uint64_t c = 0;
        for (uint32_t i = lane; i < m; i += kWave) c += key[i] <= mid ? (uint64_t)1 << lvl[i] : 0ull;
        c = lane_bcast64(wave_scan64(c, 0ull, OpAdd64{}), kWave - 1);
        const bool ok = (unsigned __int128)c * n > (unsigned __int128)r * wtot;
        lo = ok ? lo : mid + 1;
        hi = ok ? mid : hi;
    }
    return lo;
}

__global__ __launch_bounds__(64) void k_kll_query(KllQueryArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const uint32_t RW = (uint32_t)(kKllHdr + A.budget);
    uint64_t* key = reinterpret_cast<uint64_t*>(smem);
    uint8_t* lvl = reinterpret_cast<uint8_t*>(key + (size_t)A.W * A.budget);
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const uint64_t* rows = A.rows + (size_t)s * A.W * RW;
        uint64_t n = 0, nan = 0, wtot = 0;
        double mn = bitsd(kQuietNaN), mx = bitsd(kQuietNaN);
        bool bad = false;
        uint32_t m = 0;
#pragma unroll 1
        for (int w = 0; w < A.W; ++w) {
            const uint64_t* row = rows + (size_t)w * RW;
            n += row[0];
            nan += row[1];
            mn = fmin(mn, bitsd(row[2]));
            mx = fmax(mx, bitsd(row[3]));
            bad = bad || row[8] == ~0ull;
            wtot += row[9];
            uint32_t pos = 0;
#pragma unroll 1
            for (int h = 0; h < kKllLevels; ++h) {
                const uint32_t l = (uint32_t)(row[4 + (h >> 2)] >> (16 * (h & 3))) & 0xFFFFu;
                if (pos + l > (uint32_t)A.budget) {  // not a row krr_kll_build wrote: never stage past it
                    bad = true;
                    break;
                }
                for (uint32_t i = lane; i < l; i += kWave) {
                    key[m + i] = okey(row[kKllHdr + pos + i]);  // f64 bits -> order-preserving
                    lvl[m + i] = (uint8_t)h;
                }
                pos += l;
                m += l;
            }
        }
        __syncthreads();
        uint32_t flags = 0;
        double result = bitsd(kQuietNaN);
        if (bad) {
            flags = KRR_FLAG_CAPACITY;
        } else if (nan) {
            flags = KRR_FLAG_NAN;
        } else if (n == 0) {
            flags = KRR_FLAG_EMPTY;
        } else {
            int64_t r0, r1;
            double gamma = 0.0;
            if (A.mode == KRR_PCT_SORTED_LOWER) {
                r0 = r1 = exact_rank((int64_t)n, A.p_num, A.p_den);
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
#pragma unroll 1
            for (int qi = 0; qi < 2; ++qi) {
                const uint64_t r = (uint64_t)(qi ? r1 : r0);
                if (qi && r1 == r0) {
                    v[1] = v[0];
                    continue;
                }
                // every kept key compacted away (a few samples spread over several chunks):
                // only the exact min / max remain
                v[qi] = r == 0 ? mn : (r == n - 1 ? mx : (wtot == 0 ? (2 * r < n ? mn : mx)
                                                                     : bitsd(okey_inv(kll_select(key, lvl, m, r, n,
                                                                                                 wtot, lane)))));
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

}  // namespace krr
