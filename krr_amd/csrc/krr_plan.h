// krr_plan.h — host+device planning shared by the ABI and the kernels.
#pragma once

#include <stdint.h>
#include <math.h>

#include "krr_amd.h"

namespace krr {

#if defined(__HIPCC__)
#define KRR_HD __host__ __device__
#else
#define KRR_HD
#endif

// Exact floor((n-1) * p_num / (100 * p_den)), host side (device side: krr_device.h).
KRR_HD inline int64_t exact_rank_hd(int64_t n, int64_t p_num, int64_t p_den) {
    const uint64_t a = (uint64_t)(n - 1);
    const uint64_t den = 100ull * (uint64_t)p_den;
    const unsigned __int128 num = (unsigned __int128)a * (uint64_t)p_num;
    uint64_t k = (uint64_t)((double)a * ((double)p_num / (double)den));
    if (k > a) k = a;
    while (k < a && (unsigned __int128)(k + 1) * den <= num) ++k;
    while (k > 0 && (unsigned __int128)k * den > num) --k;
    return (int64_t)k;
}

// Which extreme of a segment of L slots the selection keeps, and how many keys.
// The kernel needs ranks r1 (and r1+1 for LINEAR) of the n <= L present samples.
// Keeping the top T = L - k(L) + 2 keys (or the bottom k(L) + 4) covers every
// n <= L, because n - k(n) and k(n) are non-decreasing in n; the +2/+4 margins
// absorb the +-1 floor error of the float64 LINEAR index.  `table`: k(n) comes from
// krr_percentile_params.k_table, which is within [k_exact(n), k_exact(n) + 1] of the exact
// floor of p while p_num / p_den is within 1e-15 of p: two more keys on each side cover it
// (n - k(n) may then step down by one, and k(L) may exceed the plan's estimate by two).
struct SidePlan {
    uint32_t tkeep;
    uint32_t bottom;  // 1: keep the smallest keys (flip the order)
};

KRR_HD inline SidePlan plan_side(int64_t L, int32_t mode, int64_t p_num, int64_t p_den, double q,
                                 bool table = false) {
    SidePlan sp;
    if (L <= 0) {
        sp.tkeep = 1;
        sp.bottom = 0;
        return sp;
    }
    int64_t k;
    if (mode == KRR_PCT_LINEAR) {
        double v = (double)(L - 1) * q;
        k = (int64_t)floor(v);
        if (k > L - 1) k = L - 1;
        if (k < 0) k = 0;
    } else {
        k = exact_rank_hd(L, p_num, p_den);
    }
    const int64_t wide = (table && mode != KRR_PCT_LINEAR) ? 2 : 0;
    int64_t top = L - k + 2 + wide;
    int64_t bot = k + 4 + wide;
    if (top > L) top = L;
    if (bot > L) bot = L;
    if (top <= bot) {
        sp.tkeep = (uint32_t)top;
        sp.bottom = 0;
    } else {
        sp.tkeep = (uint32_t)bot;
        sp.bottom = 1;
    }
    return sp;
}

// Fixed LDS of the select kernel ahead of the candidate keys: 256-bin
// histogram (1 KiB) and the 64-key gather area (512 B).
constexpr uint32_t kSelectLdsFixed = 1536;

// Elements one streaming iteration can append (U double2 per lane, 64 lanes).
constexpr int kUnroll = 8;
constexpr uint32_t kChunkElems = 2u * kUnroll * 64u;

// LDS key capacity for a launch whose largest segment keeps tkeep keys.
// After a compaction at most tstop = cap - kChunkElems/2 keys remain, so half a
// chunk always fits; the 128-key margin above tkeep is what a histogram cut may
// keep beyond tkeep before the exact fallback is needed.  The first chunk of a
// segment (every sample a candidate) must fit an empty buffer.
#ifndef KRR_CAP_MARGIN
#define KRR_CAP_MARGIN 128
#endif
KRR_HD inline uint32_t capacity_for(uint32_t tkeep_max) {
    uint64_t c = (uint64_t)tkeep_max + kChunkElems / 2 + KRR_CAP_MARGIN;
    if (c < kChunkElems + 64) c = kChunkElems + 64;
    c = (c + 63) & ~63ull;
    return (uint32_t)c;
}

// Largest single-pass candidate capacity (keys); a segment needing more is
// selected by hselect (histogram pass + collect pass) instead.
#ifndef KRR_SINGLE_CAP_MAX
#define KRR_SINGLE_CAP_MAX 2048
#endif
constexpr uint32_t kSingleCapMax = KRR_SINGLE_CAP_MAX;
// ... up to this many keys when the kept tail is a small fraction of the segment
// (long series at tail percentiles: few inserts, so the single pass beats hselect's
// two passes even at the lower occupancy the bigger buffer allows; measured: 30d@15s
// p99 1.45x, 50,400-slot p97 1.08x, but p96.5 (3.5% kept) 0.92x — hence the fraction).
#ifndef KRR_SINGLE_CAP_LONG
#define KRR_SINGLE_CAP_LONG 2560
#endif
#ifndef KRR_LONG_KEEP_PERMILLE
#define KRR_LONG_KEEP_PERMILLE 30
#endif
constexpr uint32_t kSingleCapLong = KRR_SINGLE_CAP_LONG;

// ... and up to this many keys when the longest segment is at least
// KRR_PROBE_LEN_RATIO x the capacity: the start-threshold probe (krr_kernels.hip,
// KRR_SELECT_PROBE) keeps such a buffer at ~1.5x the kept tail without
// compactions.  A/B (profiles/r01/v16/ab_bigcap*.log, v17/ab_cap2.log): config 2 p94 +6%,
// p95 +5%, p97 +7%; 4,224 keys (p93) loses to hselect;
// launches of mixed lengths (config 3 p90, Lmax / need = 7.5) lose 4%, hence the ratio.
#ifndef KRR_SINGLE_CAP_PROBE
#define KRR_SINGLE_CAP_PROBE 3712
#endif
#ifndef KRR_PROBE_LEN_RATIO
#define KRR_PROBE_LEN_RATIO 12
#endif

// The start-threshold probe pays when the inserts past a full buffer (~tkeep
// ln(L/cap), a record-breaking count) would need several compactions of
// (cap - tkeep - 128) free keys each; for short tails (p99 of a week) it would
// only add a round trip.  Top side only.
#ifndef KRR_PROBE_MIN_COMPACT
#define KRR_PROBE_MIN_COMPACT 0.25f  // ... when tkeep * ln(L / cap) >= this x (cap - tkeep - 128) free keys
#endif
KRR_HD inline bool select_probe_pays(int64_t L, uint32_t tkeep, uint32_t cap) {
    if (L < 4 * (int64_t)cap || cap <= tkeep + 128) return false;
#if defined(__HIP_DEVICE_COMPILE__)
    const float inserts = (float)tkeep * __logf((float)L / (float)cap);
#else
    const float inserts = (float)tkeep * logf((float)L / (float)cap);
#endif
    return inserts >= KRR_PROBE_MIN_COMPACT * (float)(cap - tkeep - 128);
}

// `bottom`: the plan keeps the smallest keys.  The start-threshold probe only
// runs for the top side (krr_kernels.hip select_segment_with), so the probe-backed
// capacity is top-side only; a low percentile of a long series (p5 of 50,400
// slots keeps ~2,500 keys) would otherwise stream from the lowest key into a big
// buffer and compact a dozen times per segment.
KRR_HD inline bool single_pass_ok(uint32_t need, uint32_t tkeep, int64_t L, uint32_t bottom) {
    if (need <= kSingleCapMax) return true;
    if (need <= kSingleCapLong && (int64_t)tkeep * 1000 <= (int64_t)KRR_LONG_KEEP_PERMILLE * L) return true;
#if !defined(KRR_SELECT_PROBE) || KRR_SELECT_PROBE
    return !bottom && need <= KRR_SINGLE_CAP_PROBE && L >= (int64_t)KRR_PROBE_LEN_RATIO * need;
#else
    (void)bottom;
    return false;
#endif
}

// The launch's selection path: single pass (its candidate set fits LDS) or the window
// select (wselect, hselect for its misses).  The window select also takes launches the
// single pass could hold when their kept tail is a large share of the segment (more than
// KRR_WSEL_KEEP_PERMILLE) and the single-pass buffer would exceed KRR_WSEL_MIN_NEED keys:
// there the single pass pays compactions (or the probe-backed big buffer's lower
// occupancy) that the window's shrinking key range avoids.  Same-process A/B, fused
// launch (profiles/r02/ab18, ab19): config 2 p94 1.288 -> 1.220 ms, p95 1.221 -> 1.180,
// p96 1.189 -> 1.184; config 3 p95 2.56 -> 2.44, p96 2.46 -> 2.43; p97 and up (<= 3%
// kept) and the 10,080-slot config-4 shape equal or better on the single pass.
//
// (Tried in round 2: every fused buffer above 1,200 keys to the window, with gapped long
// segments on the 16-waves/CU kernel — faster in the A/B (config 2 p97 1.206 -> 1.186 ms),
// but on the bench's data one 50,400-slot segment per launch missed the window, and a miss
// there is finished by ONE wave in the separate miss pass: +150 us, config 2 p97 1.29 ms.
// Long segments keep the kernel whose misses run inline, beside the other waves.)
// Round 2, v21 (profiles/r02/q, same-process A/B of the percentile pass alone and of the
// fused launch): a percentile-only launch (krr_segmented_percentile) gains from the window
// down to 0.5% kept — 30d@15s (172,800 slots) p99 4.42 -> 4.23 ms, 50,400-slot p98 0.684 ->
// 0.646, p97 0.797 -> 0.625, 100,800-slot p97 4.46 -> 3.66 — while in the fused launch the
// window kernel's 2 waves per SIMD also carry the memory half, so there it only pays against
// the probe-backed big buffers (more than KRR_WSEL_FUSED_NEED keys: 100,800-slot p97 fused
// 7.71 -> 7.13 ms; 172,800-slot p99 8.09 vs 8.30 and 50,400-slot p97 / p98 1.170 / 1.162 vs
// 1.192 / 1.188 stay on the single pass).
#ifndef KRR_WSEL_KEEP_PERMILLE
#define KRR_WSEL_KEEP_PERMILLE 35
#endif
#ifndef KRR_WSEL_KEEP_PERMILLE_SOLO
#define KRR_WSEL_KEEP_PERMILLE_SOLO 5
#endif
#ifndef KRR_WSEL_FUSED_NEED
#define KRR_WSEL_FUSED_NEED 2560
#endif
#ifndef KRR_WSEL_SOLO_NEED
#define KRR_WSEL_SOLO_NEED 1600  // the measured gains: buffers of 1,664 keys and more
#endif
#ifndef KRR_WSEL_MIN_NEED
#define KRR_WSEL_MIN_NEED 1200
#endif
KRR_HD inline bool window_select(uint32_t need, uint32_t tkeep, int64_t L, uint32_t bottom, bool fused) {
    if (!single_pass_ok(need, tkeep, L, bottom)) return true;
    const int64_t kept = (int64_t)tkeep * 1000;  // vs permille of L
    if (need > (uint32_t)KRR_WSEL_MIN_NEED && kept > (int64_t)KRR_WSEL_KEEP_PERMILLE * L) return true;
    if (fused) return need > (uint32_t)KRR_WSEL_FUSED_NEED;
    return need > (uint32_t)KRR_WSEL_SOLO_NEED && kept > (int64_t)KRR_WSEL_KEEP_PERMILLE_SOLO * L;
}

// hselect LDS after kSelectLdsFixed: histogram + collect buffer.
#ifndef KRR_HIST_BITS
#define KRR_HIST_BITS 10
#endif
constexpr int kHistBits = KRR_HIST_BITS;
constexpr uint32_t kHistBins = 1u << kHistBits;
// 1,792 keys: hselect's LDS (1.5 + 4 + 14 KiB) x 8 waves still fits a CU's 160 KiB.
// (A/B against 2,048 bins + 1,280 keys: the wider band wins p50 +4.8%, p75 +4.2%.)
#ifndef KRR_COLLECT_CAP
#define KRR_COLLECT_CAP 1792
#endif
constexpr uint32_t kCollectCap = KRR_COLLECT_CAP;
constexpr size_t kHselectLds = (size_t)kHistBins * 4 + (size_t)kCollectCap * 8;

}  // namespace krr
