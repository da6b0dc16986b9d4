// krr_kernels.hip — CDNA4 (gfx950) kernels of the KRR SimpleStrategy hot path.
//
// Layout in HBM: one float64 CSR buffer per resource,
// values[] + offsets[S+1]; segment s = one object's pods concatenated in
// K8sObjectData.pods order (reference prometheus.py:150-155).
//
// Kernels (all HBM-bound streaming; no MFMA, nothing here is a contraction):
//   k_select        one wave64 per segment: single HBM pass, exact order statistic
//                   via a threshold-filtered candidate buffer in LDS + MSD radix
//                   select on order-preserving uint64 keys (SORTED_LOWER, LINEAR).
//   k_refindex_gaps one wave64 per segment: count present samples, then locate the
//                   k-th present one from the nearer end (REF_INDEX, NaN-gapped layout).
//   k_refindex_dense one thread per segment: X[k] gather (REF_INDEX, compact CSR).
//   k_max           one wave64 per segment: max + count (memory proposal).
//   k_synth         counter-hash synthetic series (bench / test data).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <dlfcn.h>
#include <sched.h>
#include <time.h>
#include <unistd.h>
#include <rccl/rccl.h>  // types only: RCCL is resolved with dlopen/dlsym (krr_comm_*)

#include <new>
#include <type_traits>

#include "krr_amd.h"
#include "krr_device.h"
#include "krr_plan.h"
#include "krr_json.h"

#ifndef KRR_STREAM_DEPTH
#define KRR_STREAM_DEPTH 2  // chunks in flight per wave
#endif
#ifndef KRR_WSEL_LONG_DEPTH
#define KRR_WSEL_LONG_DEPTH 2  // chunks in flight beyond the one processed, long-segment window kernels (v27)
#endif
#ifndef KRR_ONE_SITE_DEPTH
#define KRR_ONE_SITE_DEPTH 1  // chunks in flight beyond the one processed, single-call-site streaming loop
#endif
#ifndef KRR_LDS_BATCH
#define KRR_LDS_BATCH 4  // keys per lane read before use in the buffer passes (minmax, histogram, filter, gather)
#endif
#ifndef KRR_LDS_MIN
#define KRR_LDS_MIN 0  // experiments: minimum dynamic LDS per select workgroup (caps waves per CU)
#endif
#ifndef KRR_SELECT_WAVES_PER_SIMD
#define KRR_SELECT_WAVES_PER_SIMD 3  // __launch_bounds__ occupancy hint for the single-pass select
#endif
#ifndef KRR_MAX_DEPTH
#define KRR_MAX_DEPTH 2  // chunks in flight in the multi-site streaming loop (k_max): 1 or 2
#endif
#ifndef KRR_LANE_INSERT
#define KRR_LANE_INSERT 1  // select fast path: per-lane masks + one scan (0: per-slot ballot insert)
#endif
#ifndef KRR_PAIR_RANKS
#define KRR_PAIR_RANKS 1  // LINEAR's two adjacent ranks from one locate (0: two locates)
#endif
#ifndef KRR_HSEL_WAVES_PER_SIMD
#define KRR_HSEL_WAVES_PER_SIMD 2  // ... and for hselect (LDS allows ~9 waves per CU)
#endif
#ifndef KRR_WSEL_WAVES_PER_SIMD
#define KRR_WSEL_WAVES_PER_SIMD 4  // ... and for the window select (wselect) of short segments
#endif
#ifndef KRR_WSEL_CAP
#define KRR_WSEL_CAP 1088  // wselect's LDS keys: 1.5 + 8.5 KiB per wave -> 16 waves per CU (v23)
#endif
#ifndef KRR_WSEL_CAP_LONG
#define KRR_WSEL_CAP_LONG 2304  // ... for launches of long segments (1.5 + 18 KiB -> 8 waves per CU)
#endif
#ifndef KRR_WSEL_LONG
#define KRR_WSEL_LONG 32768  // longest segment from which a launch takes KRR_WSEL_CAP_LONG
#endif
#ifndef KRR_FALLBACK_GRID
#define KRR_FALLBACK_GRID 1024  // workgroups of the hselect pass over the segments wselect missed
#endif
#ifndef KRR_HSEL_BAND
#define KRR_HSEL_BAND 1  // hselect's first pass also collects a probe-estimated key band (0: off)
#endif
#ifndef KRR_PROBE_BATCH
#define KRR_PROBE_BATCH 8  // probe blocks (per 8 lanes) loaded per round trip
#endif
#ifndef KRR_HSEL_BAND_MIN
#define KRR_HSEL_BAND_MIN 16384  // ... for segments of at least this many slots (the probe's fixed cost)
#endif
#ifndef KRR_SELECT_PROBE
#define KRR_SELECT_PROBE 1  // single-pass select: probe-estimated start threshold when compactions would pile up (0: off)
#endif
#ifndef KRR_PROBE_MARGIN_X4
#define KRR_PROBE_MARGIN_X4 6  // ... aiming the start threshold at (this / 4) x the kept tail
#endif
// (KRR_PROBE_MIN_COMPACT, the rule for when the start-threshold probe pays: krr_plan.h)

namespace krr {

constexpr int kLdsBatch = KRR_LDS_BATCH;
#ifdef KRR_WEXP_DEBUG
__device__ unsigned long long g_wdbg[5 * 1024];
__device__ unsigned int g_wdbg_n = 0;
__device__ unsigned int g_wdbg_on = 1;
#endif

// Diagnostic build (-DKRR_DIAG): per-segment cycle and event counters written
// to a buffer attached with krr_diag_attach(); never compiled into the product.
#ifdef KRR_DIAG
__device__ unsigned long long* g_diag = nullptr;
enum { D_TOTAL, D_COMPACT, D_FINAL, D_NCOMPACT, D_NFALLBACK, D_ACTIVE_SLOTS, D_INSERTED, D_CHUNKS, D_WORDS };
#define KRR_DIAG_T0(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define KRR_DIAG_ADD(field, val) \
    do { diag[field] += (val); } while (0)
#else
#define KRR_DIAG_T0(v)
#define KRR_DIAG_ADD(field, val) \
    do {                          \
    } while (0)
#endif

#ifndef KRR_XCD_REMAP
#define KRR_XCD_REMAP 1  // per-XCD contiguous segment ranges (0: block i -> segment i)
#endif
// ... for launches whose longest segment is shorter than this (a per-launch flag): with
// segments of 172,800 slots (config 5) block i -> segment i streamed 3.7% faster in a
// same-process A/B (scripts/ab_variants.py, profiles/r03/l), with 50,400 ones 2.5% slower
#ifndef KRR_XCD_REMAP_MAXLEN
#define KRR_XCD_REMAP_MAXLEN 100000
#endif
// Workgroups are dispatched round-robin over the 8 XCDs (block i on XCD i % 8),
// so block i -> segment i leaves every XCD's L2 fetching a fresh offsets line
// per segment start.  Remap so that the blocks of one XCD (i, i+8, i+16, …)
// walk one contiguous eighth of the items: their offsets (and result records)
// share L2 lines.  A bijection of [0, n): the n % 8 trailing items map to
// themselves.
__device__ __forceinline__ int64_t xcd_item(int64_t i, int64_t n, int32_t remap) {
    if constexpr (!KRR_XCD_REMAP) return i;
    if (!remap) return i;
    const int64_t q = n >> 3;
    if (i >= (q << 3)) return i;
    return (i & 7) * q + (i >> 3);
}

// ---------------------------------------------------------------------------
// Streaming skeleton.  One wave walks values[beg, end): the 16-byte aligned
// body in chunks of kUnroll x 16 B per lane (8 KiB per wave), the next chunk
// in flight while this one is processed.  The partial last chunk is padded
// with NaN and carries the unaligned head/tail elements in its last slot
// (lane 63, which a partial chunk never fills), so every chunk goes through
// the same `proc.chunk(c)` body: a NaN is never a candidate, never a tie and is
// ignored by fmax, and the padding count is returned so NaN counts can be
// corrected.  ONE_SITE keeps a single inlined chunk body (register rotation,
// one 64-bit move per slot) for processors whose body is large.
// ---------------------------------------------------------------------------
#ifndef KRR_NT_LOADS
#define KRR_NT_LOADS 1  // nontemporal (streaming) policy on the once-read value stream (0: default policy)
#endif
typedef double v2f64 __attribute__((ext_vector_type(2)));

// A chunk of zeros: the target of the prefetch loads that have no real slot
// (partial chunk lanes, the prefetch past a segment's last chunk).  L2-resident.
__device__ double2 g_zero_chunk[kUnroll * kWave];

__device__ __forceinline__ double2 load16(const double2* p) {
    if constexpr (KRR_NT_LOADS) {
        const v2f64 v = __builtin_nontemporal_load(reinterpret_cast<const v2f64*>(p));
        return make_double2(v.x, v.y);
    } else {
        return *p;
    }
}

__device__ __forceinline__ void load_chunk(double2 (&c)[kUnroll], const double2* __restrict__ p) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) c[u] = load16(p + u * kWave);
}

template <bool ONE_SITE, class Proc, int DEPTH = KRR_ONE_SITE_DEPTH>
__device__ __forceinline__ uint32_t stream_segment(const double* __restrict__ vals, int64_t beg,
                                                   int64_t end, Proc& proc, int lane) {
    int64_t a0 = (beg + 1) & ~(int64_t)1;
    if (a0 > end) a0 = end;
    int64_t a1 = end & ~(int64_t)1;
    if (a1 < a0) a1 = a0;
    const double2* __restrict__ v2 = reinterpret_cast<const double2*>(vals);
    const int64_t i0 = a0 >> 1;
    const int64_t nunits = (a1 >> 1) - i0;
    constexpr int CH = kUnroll * kWave;  // double2 units per chunk
    const int64_t nfull = nunits / CH;
    const int64_t rem = nunits - nfull * CH;
    const bool head = a0 > beg, tail = a1 < end;
    const bool partial = rem > 0 || head || tail;
    const int64_t nch = nfull + (partial ? 1 : 0);
    if (nch == 0) return 0;
    const double2* __restrict__ p = v2 + i0 + lane;
    const double qnan = __builtin_nan("");
    auto fill = [&](double2 (&c)[kUnroll], int64_t ci) {
        if (ci < nfull) {
            load_chunk(c, p + ci * CH);
        } else {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int64_t j = ci * CH + u * kWave + lane;
                c[u] = j < nunits ? v2[i0 + j] : make_double2(qnan, qnan);
            }
            if (lane == kWave - 1) {
                if (head) c[kUnroll - 1].x = vals[beg];
                if (tail) c[kUnroll - 1].y = vals[a1];
            }
        }
    };
    if constexpr (ONE_SITE) {
        // Every in-loop fill issues exactly kUnroll 16-byte loads, unconditionally
        // (partial-chunk lanes and the prefetch past the last chunk read the
        // zero chunk instead, and are then replaced by NaN), so the compiler's
        // wait before proc.chunk(cur) is vmcnt(kUnroll) — the next chunk stays
        // in flight while this one is processed — instead of vmcnt(0).
        double hv = qnan, tv = qnan;
        if (head) hv = vals[beg];
        if (tail) tv = vals[a1];
        const double2* __restrict__ zp = g_zero_chunk + lane;
        auto fill_u = [&](double2 (&c)[kUnroll], int64_t ci) {
            if (ci < nfull) {
                load_chunk(c, p + ci * CH);
            } else {
                // opaque base: the 8 per-u zero-chunk addresses are rebuilt here, not
                // hoisted to kernel entry and held in 16 VGPRs for the whole kernel
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
                if (lane == kWave - 1) {
                    c[kUnroll - 1].x = hv;
                    c[kUnroll - 1].y = tv;
                }
            }
        };
        // cur only ever receives register copies of nxt (here and at the bottom of
        // the loop), so on every path into proc.chunk(cur) the only loads in
        // flight are nxt's and the wait the compiler places is for nothing.
        // KRR_ONE_SITE_DEPTH > 1: a ring of that many chunks in flight (for launches
        // whose LDS budget leaves few waves per CU to cover HBM latency).
        double2 cur[kUnroll];
        if constexpr (DEPTH <= 1) {
            double2 nxt[kUnroll];
            fill_u(nxt, 0);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                double x = nxt[u].x, y = nxt[u].y;
                asm volatile("" : "+v"(x), "+v"(y));
                cur[u] = make_double2(x, y);
            }
#pragma unroll 1
            for (int64_t ci = 0; ci < nch; ++ci) {
                fill_u(nxt, ci + 1);
                proc.chunk(cur);
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) cur[u] = nxt[u];
            }
        } else {
            // Ring of D buffers with compile-time roles: the loop body is unrolled D
            // times, so at sub-step k buffer (k + D - 1) % D takes chunk ci + k + D
            // and cur receives buffer k — the OLDEST group in flight, so the wait
            // before that copy leaves the D - 1 newer chunks' loads outstanding.
            // (Register shifting would wait for every load.)  D call sites of
            // proc.chunk.
            constexpr int D = DEPTH;
            double2 ring[D][kUnroll];
            {
                double2 first[kUnroll];
                fill_u(first, 0);
#pragma unroll
                for (int d = 0; d + 1 < D; ++d) fill_u(ring[d], d + 1);
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    double x = first[u].x, y = first[u].y;
                    asm volatile("" : "+v"(x), "+v"(y));
                    cur[u] = make_double2(x, y);
                }
            }
#pragma unroll 1
            for (int64_t ci = 0; ci < nch; ci += D) {
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    if (ci + k >= nch) break;  // wave-uniform
                    fill_u(ring[(k + D - 1) % D], ci + k + D);
                    proc.chunk(cur);
#pragma unroll
                    for (int u = 0; u < kUnroll; ++u) cur[u] = ring[k][u];
                }
            }
        }
    } else if constexpr (KRR_MAX_DEPTH >= 2) {
        // three buffers with fixed roles: two chunks stay in flight while one is processed
        double2 b0[kUnroll], b1[kUnroll], b2[kUnroll];
        fill(b0, 0);
        if (nch > 1) fill(b1, 1);
        if (nch > 2) fill(b2, 2);
        for (int64_t ci = 0; ci < nch; ci += 3) {
            proc.chunk(b0);
            if (ci + 3 < nch) fill(b0, ci + 3);
            if (ci + 1 < nch) proc.chunk(b1);
            if (ci + 4 < nch) fill(b1, ci + 4);
            if (ci + 2 < nch) proc.chunk(b2);
            if (ci + 5 < nch) fill(b2, ci + 5);
        }
    } else {
        double2 b0[kUnroll], b1[kUnroll];
        fill(b0, 0);
        if (nch > 1) fill(b1, 1);
        for (int64_t ci = 0; ci < nch; ci += 2) {
            proc.chunk(b0);
            if (ci + 2 < nch) fill(b0, ci + 2);
            if (ci + 1 < nch) proc.chunk(b1);
            if (ci + 3 < nch) fill(b1, ci + 3);
        }
    }
    return partial ? (uint32_t)(2 * CH - 2 * rem - (head ? 1 : 0) - (tail ? 1 : 0)) : 0u;
}

__device__ __forceinline__ double slot_val(const double2 (&c)[kUnroll], int j) {
    return (j & 1) ? c[j >> 1].y : c[j >> 1].x;
}

__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__popcll((long long)m); }

// Find the digit bin holding the R-th largest (1-based) of a 256-bin histogram
// (bins ordered by key), given `above0` elements already known to be larger.
struct BinHit {
    uint32_t b;      // bin index
    uint32_t above;  // elements in higher bins (+ above0)
    uint32_t cnt;    // elements in bin b
    uint32_t found;
};

__device__ __forceinline__ BinHit find_bin_desc(const uint32_t* hist, uint32_t R, uint32_t above0, int lane) {
    uint32_t hb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) hb[j] = hist[4 * lane + j];
    const uint32_t t = hb[0] + hb[1] + hb[2] + hb[3];
    const uint32_t incl = wave_suffix_incl(t, lane);
    uint32_t run = above0 + (incl - t);
    int fb = -1;
    uint32_t fab = 0, fcb = 0;
#pragma unroll
    for (int j = 3; j >= 0; --j) {
        if (fb < 0 && run < R && run + hb[j] >= R) {
            fb = 4 * lane + j;
            fab = run;
            fcb = hb[j];
        }
        run += hb[j];
    }
    const uint64_t m = ballot(fb >= 0);
    BinHit h;
    h.found = m != 0;
    const int src = m ? __ffsll((long long)m) - 1 : 0;
    h.b = lane_bcast32((uint32_t)fb, src);
    h.above = lane_bcast32(fab, src);
    h.cnt = lane_bcast32(fcb, src);
    return h;
}

// ---------------------------------------------------------------------------
// Threshold-filtered candidate buffer (one wave per segment).
//
// Invariant over the present non-NaN samples seen so far, in (possibly
// flipped) key order, in one of two modes:
//   inclusive (incl = 1): buf holds exactly those with key >= thr; every other
//                         one is < thr ("below", implied by n);
//   strict    (incl = 0): buf holds exactly those with key > thr, `eqs` counts
//                         those with key == thr, the rest are below.
// A segment starts inclusive at thr = 0 (every key).  Strict mode is entered
// only when one key value is so crowded that cutting at it inclusively would
// keep too many (e.g. a mostly-zero series); the next cut returns to inclusive.
// When a chunk's candidates do not fit, compact() raises thr so that at least
// tkeep keys stay in buf (+ ties) and at most tstop stay in buf, then the chunk
// is re-classified.  The segment's needed ranks lie in its top tkeep keys
// (krr_plan.h), so they are never dropped.
//
// Fast path (inclusive, top side, thr = key of a non-negative number t): "key >=
// thr" for a sample with bits x is the single unsigned range test
//   x - bits(t) < bits(+inf) - bits(t) + 1
// which also rejects every NaN and every negative number, and no tie count is
// needed.  NaN slots are counted for every chunk up front (independent of thr).
//
// Insertion is kept minimal (ballot + mbcnt position + one ds_write): with a
// ~1-3% candidate rate nearly every 64-wide slot has a candidate, so every
// VALU spent per insert is spent on most slots.  A compaction instead builds a
// 256-bin histogram of the buffer over [min, max] and reads the cut off it,
// re-histogramming a crowded bin's range if needed (locate), then filters
// once.  The final rank queries locate the rank the same way down to <= 64
// keys, gather them and rank them in registers.
// ---------------------------------------------------------------------------
struct SelectProc {
    uint64_t* buf;
    uint32_t* H;      // 256-bin histogram of buf (also select_desc's scratch)
    uint64_t* small;  // 64-key gather area
    int lane;
    uint32_t cap, tkeep, tstop;
    uint64_t flip;
    uint64_t thr;
    uint32_t incl;             // 1: inclusive mode (buf = keys >= thr), 0: strict
    uint32_t cnt, eqs;
    uint32_t nnan_lane;        // this lane's NaN slots (reduced at the end)
    uint32_t fast;             // inclusive, top side, thr = key of a number in [+0, +inf]
    uint64_t tb, tlim;         // fast-path constants
    uint32_t bad;
#ifdef KRR_DIAG
    unsigned long long diag[D_WORDS];
#endif

    __device__ __forceinline__ void set_thr(uint64_t t, uint32_t inclusive) {
        thr = uni64(t);
        incl = uni32(inclusive);
        fast = (incl && !flip && (thr & kSignBit) && (thr ^ kSignBit) <= 0x7FF0000000000000ull) ? 1u : 0u;
        tb = thr ^ kSignBit;
        tlim = 0x7FF0000000000001ull - tb;
    }

    template <bool FAST>
    __device__ __forceinline__ bool is_cand(double d, uint64_t& key) const {
        const uint64_t x = dbits(d);
        if (FAST) {
            key = x | kSignBit;
            return (x - tb) < tlim;
        }
        key = okey(x) ^ flip;
        return !__builtin_isnan(d) && (incl ? key >= thr : key > thr);
    }

    // NaN slots of a whole chunk (absent samples in the gapped layout), counted
    // per lane in a VGPR (no 16 live lane masks); reduced once per segment.
    __device__ __forceinline__ void count_nan(const double2 (&c)[kUnroll]) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) nnan_lane += __builtin_isnan(slot_val(c, j)) ? 1u : 0u;
    }

    // Count candidates (C) and, in strict mode, ties with thr (E) among the slots
    // in smask; jm = bit j set if slot j has a candidate in some lane.
    // OPAQUE: re-materialise each slot value (general path inside the step loop),
    // so the compiler cannot hoist 16 slots' keys and masks out of that loop.
    template <bool FAST, bool OPAQUE = true>
    __device__ __forceinline__ void classify(const double2 (&c)[kUnroll], uint32_t smask, uint32_t& C,
                                             uint32_t& E, uint32_t& jm) const {
        C = E = jm = 0;
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            if ((smask >> j) & 1u) {  // wave-uniform
                double d = slot_val(c, j);
                if (OPAQUE) asm volatile("" : "+v"(d));
                uint64_t key;
                const bool cand = is_cand<FAST>(d, key);
                const uint64_t m = ballot(cand);
                C += popc64(m);
                jm |= m ? (1u << j) : 0u;
                if (!FAST && !incl) E += popc64(ballot(!__builtin_isnan(d) && key == thr));
            }
        }
    }

    template <bool FAST>
    __device__ __forceinline__ void insert(const double2 (&c)[kUnroll], uint32_t jm) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            if ((jm >> j) & 1u) {
                // Opaque copy: recompute the test here instead of letting the
                // compiler keep classify's 16 keys/masks alive across compact().
                double d = slot_val(c, j);
                asm volatile("" : "+v"(d));
                uint64_t key;
                const bool cand = is_cand<FAST>(d, key);
                const uint64_t m = ballot(cand);
                if (cand) buf[cnt + lane_prefix(m)] = key;
                cnt = uni32(cnt + popc64(m));
            }
        }
    }

    // Classify the slots in smask, compact once if needed, insert.  Returns false
    // (nothing inserted, nothing counted) if the candidates still do not fit.
    __device__ __forceinline__ bool try_slots(const double2 (&c)[kUnroll], uint32_t smask) {
        uint32_t C, E, jm;
        if (uni32(fast)) classify<true>(c, smask, C, E, jm);
        else classify<false>(c, smask, C, E, jm);
        if (cnt + C > cap) {
            compact();
            if (uni32(fast)) classify<true>(c, smask, C, E, jm);
            else classify<false>(c, smask, C, E, jm);
            if (cnt + C > cap) return false;
        }
        eqs += E;
        KRR_DIAG_ADD(D_ACTIVE_SLOTS, __popc(jm));
        KRR_DIAG_ADD(D_INSERTED, C);
        if (jm) {
            if (uni32(fast)) insert<true>(c, jm);
            else insert<false>(c, jm);
        }
        return true;
    }

    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
        KRR_DIAG_ADD(D_CHUNKS, 1);
        count_nan(c);
        // Steady state: fast inclusive threshold, the whole chunk fits.
        if (uni32(fast)) {
#if KRR_LANE_INSERT
            // Per-lane candidate mask (slot j -> bit 15 - j) built in VGPRs, ONE wave
            // scan for every lane's write position, then predicated LDS writes
            // (non-candidates write a per-lane scratch slot): ~4 VALU + 1 LDS per
            // slot and no per-slot ballot/SALU work — with a 1-3% candidate rate
            // nearly every 64-wide slot holds a candidate, so per-slot scalar
            // bookkeeping was paid on most slots.
            uint32_t vm = 0;
#pragma unroll
            for (int j = 0; j < 2 * kUnroll; ++j) {
                const uint64_t x = dbits(slot_val(c, j));
                vm = (vm << 1) + ((x - tb) < tlim ? 1u : 0u);
            }
            const uint32_t vc = __popc(vm);
            const uint32_t incl_c = wave_scan32(vc, 0u, OpAdd32{});
            const uint32_t C = lane_bcast32(incl_c, kWave - 1);
            if (cnt + C <= cap) {
                KRR_DIAG_ADD(D_INSERTED, C);
                if (C) {
                    uint32_t pos = cnt + incl_c - vc;
                    uint64_t* const scratch = small + lane;
#pragma unroll
                    for (int j = 0; j < 2 * kUnroll; ++j) {
                        const uint64_t x = dbits(slot_val(c, j));
                        const uint32_t bit = (vm >> (2 * kUnroll - 1 - j)) & 1u;
                        uint64_t* const dst = bit ? buf + pos : scratch;
                        *dst = x | kSignBit;
                        pos += bit;
                    }
                    cnt = uni32(cnt + C);
                }
                return;
            }
#else
            uint32_t C, E, jm;
            classify<true, false>(c, 0xFFFFu, C, E, jm);
            if (cnt + C <= cap) {
                KRR_DIAG_ADD(D_ACTIVE_SLOTS, __popc(jm));
                KRR_DIAG_ADD(D_INSERTED, C);
                if (jm) insert<true>(c, jm);
                return;
            }
#endif
        }
        chunk_general(c);
    }

    // Compaction, general (slow) threshold test, insertion in halves.
    // After a compaction at most tstop = cap - kChunkElems/2 keys remain, so half a
    // chunk always fits: a chunk with more candidates than the free space (the
    // first chunks of a segment, or a monotone series) goes in as two halves.
    // The halves run through the same inlined body (a 3-iteration loop).
    __device__ __forceinline__ void chunk_general(const double2 (&c)[kUnroll]) {
        uint32_t smask = 0xFFFFu;
#pragma unroll 1
        for (int step = 0; step < 3; ++step) {
            if (try_slots(c, smask)) {
                if (smask != 0x00FFu) return;  // whole chunk, or second half done
                smask = 0xFF00u;
                continue;
            }
            if (smask != 0xFFFFu) {
                bad |= 2u;
                return;
            }
            smask = 0x00FFu;
        }
    }

    // min and max key of buf; four LDS reads in flight per lane.
    __device__ __forceinline__ void buf_minmax(uint64_t& mn_out, uint64_t& mx_out) const {
        uint64_t mn = ~0ull, mx = 0;
        for (uint32_t base = 0; base < cnt; base += kLdsBatch * kWave) {
            uint64_t x[kLdsBatch];
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const uint32_t i = base + t * kWave + lane;
                x[t] = i < cnt ? buf[i] : buf[0];
            }
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                mn = x[t] < mn ? x[t] : mn;
                mx = x[t] > mx ? x[t] : mx;
            }
        }
        mn_out = wave_min_u64(mn);
        mx_out = wave_max_u64(mx);
    }

    // Histogram of the keys of buf inside [lo, hi] (256 bins of width 2^hsh from
    // lo; the range always fits 256 bins), four LDS reads in flight per lane.
    __device__ __forceinline__ uint32_t hist_range(uint64_t lo, uint64_t hi) {
        const uint64_t range = hi - lo;
        const int bits = range ? 64 - __clzll((long long)range) : 0;
        const uint32_t sh = uni32(bits > 8 ? (uint32_t)(bits - 8) : 0u);
        for (uint32_t i = lane; i < 256; i += kWave) H[i] = 0;
        __syncthreads();
        for (uint32_t base = 0; base < cnt; base += kLdsBatch * kWave) {
            uint64_t x[kLdsBatch];
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const uint32_t i = base + t * kWave + lane;
                x[t] = i < cnt ? buf[i] : 0ull;
            }
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t)
                if (base + t * kWave + lane < cnt && x[t] >= lo && x[t] <= hi)
                    atomicAdd(&H[(uint32_t)((x[t] - lo) >> sh)], 1u);
        }
        __syncthreads();
        return sh;
    }

    // Locate the R-th largest key of buf (all keys in [mn, mx]) to a key range
    // [lo, hi] holding `cnt` keys with `above` larger ones: histogram, pick the
    // bin, re-histogram that bin's range, until `good(above, cnt)` or the range
    // is a single key.  Each level is one pass over buf (an MSD radix select
    // whose digits adapt to the remaining range).
    struct Cut {
        uint64_t lo, hi;
        uint32_t above, cnt, ok;
    };
    template <class Good>
    __device__ __forceinline__ Cut locate(uint32_t R, uint64_t mn, uint64_t mx, Good good) {
        Cut c;
        c.lo = mn;
        c.hi = mx;
        c.above = 0;
        c.cnt = cnt;
        c.ok = 1;
#pragma unroll 1
        for (int level = 0; level < 9; ++level) {
            const uint32_t sh = hist_range(c.lo, c.hi);
            const BinHit bh = find_bin_desc(H, R, c.above, lane);
            __syncthreads();
            if (!bh.found) {
                c.ok = 0;
                return c;
            }
            const uint64_t blo = uni64(c.lo + ((uint64_t)bh.b << sh));
            const uint64_t span = (1ull << sh) - 1;
            const uint64_t bhi = uni64(c.hi - blo <= span ? c.hi : blo + span);
            c.lo = blo;
            c.hi = bhi;
            c.above = bh.above;
            c.cnt = bh.cnt;
            if (good(c.above, c.cnt) || blo == bhi) return c;
        }
        return c;
    }

    // Raise thr to nt: keep keys >= nt (inclusive) or keys > nt (strict; keys == nt
    // are counted into eqs) in buf, in place.  A block of 4 x 64 keys is read
    // before any of its survivors is written, and survivors land at or below the
    // block start, so nothing unread is overwritten.
    __device__ __forceinline__ void filter(uint64_t nt, uint32_t inclusive) {
        uint32_t w = 0, e = 0;
        for (uint32_t base = 0; base < cnt; base += kLdsBatch * kWave) {
            uint64_t x[kLdsBatch];
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const uint32_t i = base + t * kWave + lane;
                x[t] = i < cnt ? buf[i] : 0ull;
            }
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const bool in = base + t * kWave + lane < cnt;
                const bool keep = in && (inclusive ? x[t] >= nt : x[t] > nt);
                e += popc64(ballot(in && x[t] == nt));
                const uint64_t m = ballot(keep);
                if (keep) buf[w + lane_prefix(m)] = x[t];
                w += popc64(m);
            }
        }
        cnt = uni32(w);
        eqs = inclusive ? 0u : uni32(e);
        set_thr(nt, inclusive);
    }

    // Cut at the low edge lo of the key range holding the tkeep-th largest, so
    // that >= tkeep and <= tstop keys stay >= lo (inclusive), or, when that range
    // is one crowded key, strictly above it with its copies counted in eqs (then
    // fewer than tkeep stay in buf).  With cnt <= tstop there is nothing to gain;
    // the caller inserts in halves.
    __device__ __forceinline__ void compact() {
        if (cnt <= tstop) return;
        KRR_DIAG_T0(t0);
        __syncthreads();
        uint64_t mn, mx;
        buf_minmax(mn, mx);
        const uint32_t ts = tstop;
        const Cut ct = locate(tkeep, mn, mx, [ts](uint32_t above, uint32_t c) { return above + c <= ts; });
        const uint32_t inclusive = ct.above + ct.cnt <= ts ? 1u : 0u;
        // progress (cannot fail while cnt > tstop >= tkeep; flagged if it does)
        if (!ct.ok || !(ct.lo > thr || (incl && !inclusive && ct.lo == thr))) {
            bad |= 1u;
            return;
        }
        filter(ct.lo, inclusive);
        __syncthreads();
        KRR_DIAG_ADD(D_NCOMPACT, 1);
#ifdef KRR_DIAG
        KRR_DIAG_ADD(D_COMPACT, __builtin_amdgcn_s_memtime() - t0);
#endif
    }

    // The R-th largest key (1-based) of buf: locate it to a range of <= 64 keys
    // (or one key), gather those, rank them in registers.
    __device__ __forceinline__ uint64_t kth_largest(uint32_t R, uint64_t mn, uint64_t mx) {
        const Cut ct = locate(R, mn, mx, [](uint32_t, uint32_t c) { return c <= (uint32_t)kWave; });
        if (!ct.ok) {
            bad |= 16u;
            return 0;
        }
        if (ct.lo == ct.hi) return ct.lo;
        uint32_t w = 0;
        for (uint32_t base = 0; base < cnt; base += kLdsBatch * kWave) {
            uint64_t x[kLdsBatch];
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const uint32_t i = base + t * kWave + lane;
                x[t] = i < cnt ? buf[i] : 0ull;
            }
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const bool inb = base + t * kWave + lane < cnt && x[t] >= ct.lo && x[t] <= ct.hi;
                const uint64_t m = ballot(inb);
                if (inb) small[w + lane_prefix(m)] = x[t];
                w += popc64(m);
            }
        }
        __syncthreads();
        const uint32_t R2 = R - ct.above;
        const uint64_t v = (uint32_t)lane < w ? small[lane] : 0ull;
        uint32_t gt = 0, ge = 0;
        for (uint32_t j = 0; j < w; ++j) {
            const uint64_t y = small[j];
            gt += y > v ? 1u : 0u;
            ge += y >= v ? 1u : 0u;
        }
        const uint64_t sel = ballot((uint32_t)lane < w && gt < R2 && R2 <= ge);
        __syncthreads();
        if (!sel) {
            bad |= 8u;
            return 0;
        }
        return lane_bcast64(v, __ffsll((long long)sel) - 1);
    }

    // Smallest key of buf above hi / largest below lo (one pass; ~0 / 0 if none).
    __device__ __forceinline__ uint64_t min_above(uint64_t hi) const {
        uint64_t m = ~0ull;
        for (uint32_t i = lane; i < cnt; i += kWave) {
            const uint64_t x = buf[i];
            m = (x > hi && x < m) ? x : m;
        }
        return wave_min_u64(m);
    }
    __device__ __forceinline__ uint64_t max_below(uint64_t lo) const {
        uint64_t m = 0;
        for (uint32_t i = lane; i < cnt; i += kWave) {
            const uint64_t x = buf[i];
            m = (x < lo && x > m) ? x : m;
        }
        return wave_max_u64(m);
    }

    // The R-th largest key (ka) and its neighbour the (R + dir)-th largest (kb;
    // dir = -1: the next larger key, +1: the next smaller) from ONE locate: LINEAR
    // needs two adjacent ranks, which a second locate would find in the same range.
    __device__ __forceinline__ void kth_pair(uint32_t R, int dir, uint64_t mn, uint64_t mx, uint64_t& ka,
                                             uint64_t& kb) {
        const Cut ct = locate(R, mn, mx, [](uint32_t, uint32_t c) { return c <= (uint32_t)kWave; });
        ka = kb = 0;
        if (!ct.ok) {
            bad |= 16u;
            return;
        }
        const uint32_t R2 = R - ct.above;  // 1-based rank inside [lo, hi]
        const int64_t Rb = (int64_t)R2 + dir;
        if (ct.lo == ct.hi) {
            ka = ct.lo;
            kb = (Rb >= 1 && Rb <= (int64_t)ct.cnt) ? ct.lo : (dir < 0 ? min_above(ct.hi) : max_below(ct.lo));
            return;
        }
        uint32_t w = 0;
        for (uint32_t base = 0; base < cnt; base += kLdsBatch * kWave) {
            uint64_t x[kLdsBatch];
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const uint32_t i = base + t * kWave + lane;
                x[t] = i < cnt ? buf[i] : 0ull;
            }
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const bool inb = base + t * kWave + lane < cnt && x[t] >= ct.lo && x[t] <= ct.hi;
                const uint64_t m = ballot(inb);
                if (inb) small[w + lane_prefix(m)] = x[t];
                w += popc64(m);
            }
        }
        __syncthreads();
        const uint64_t v = (uint32_t)lane < w ? small[lane] : 0ull;
        uint32_t gt = 0, ge = 0;
        for (uint32_t j = 0; j < w; ++j) {
            const uint64_t y = small[j];
            gt += y > v ? 1u : 0u;
            ge += y >= v ? 1u : 0u;
        }
        const uint64_t sa = ballot((uint32_t)lane < w && gt < R2 && R2 <= ge);
        const bool inside = Rb >= 1 && Rb <= (int64_t)w;
        const uint64_t sb = ballot(inside && (uint32_t)lane < w && (int64_t)gt < Rb && Rb <= (int64_t)ge);
        __syncthreads();
        if (!sa || (inside && !sb)) {
            bad |= 8u;
            return;
        }
        ka = lane_bcast64(v, __ffsll((long long)sa) - 1);
        kb = inside ? lane_bcast64(v, __ffsll((long long)sb) - 1) : (dir < 0 ? min_above(ct.hi) : max_below(ct.lo));
    }

    // Keys of ascending ranks r and r + 1 (LINEAR's pair) among nsel present samples.
    __device__ __forceinline__ void rank_key_pair(uint64_t r, uint64_t nsel, uint64_t mn, uint64_t mx, uint64_t& k0,
                                                  uint64_t& k1) {
        const uint64_t rr0 = flip ? (nsel - 1 - r) : r;
        const uint64_t rr1 = flip ? rr0 - 1 : rr0 + 1;
        const uint64_t ties = incl ? 0u : eqs;
        const uint64_t below = nsel - cnt - ties;
        if ((rr0 < rr1 ? rr0 : rr1) < below + ties) {  // a rank among the ties / below: one by one
            k0 = rank_key(r, nsel, mn, mx);
            k1 = rank_key(r + 1, nsel, mn, mx);
            return;
        }
        const uint32_t idx0 = (uint32_t)(rr0 - below - ties);
        kth_pair(cnt - idx0, flip ? 1 : -1, mn, mx, k0, k1);
    }

    // Key of the element with ascending rank r (0-based) among nsel present samples.
    __device__ __forceinline__ uint64_t rank_key(uint64_t r, uint64_t nsel, uint64_t mn, uint64_t mx) {
        const uint64_t rr = flip ? (nsel - 1 - r) : r;
        const uint64_t ties = incl ? 0u : eqs;
        const uint64_t below = nsel - cnt - ties;
        if (rr < below) {
            bad |= 4u;
            return 0;
        }
        if (rr < below + ties) return thr;
        const uint32_t idx = (uint32_t)(rr - below - ties);
        return kth_largest(cnt - idx, mn, mx);
    }

    // Speculative start threshold for a long segment whose kept tail is large
    // (e.g. p95 of 20,160 slots keeps ~1,000 keys: ~T ln(L/cap) inserts and ~5
    // compactions from thr = lowest).  16 evenly spread blocks of 64 consecutive
    // slots (1,024 samples, 8 KiB, all loads in flight) are ranked in buf; the
    // key with ~1.5x the needed tail fraction above it becomes thr.  The buffer
    // then only takes keys >= thr, which is exact whenever the needed ranks end
    // up at or above thr; the caller checks that and re-streams from the lowest
    // key otherwise.  Returns 0 (no speculation) when the probe cannot decide.
    __device__ __forceinline__ uint64_t probe_threshold(const double* __restrict__ vals, int64_t beg, int64_t L) {
        constexpr int kBlocks = 16;
        double v[kBlocks];
#pragma unroll
        for (int b = 0; b < kBlocks; ++b) v[b] = vals[beg + ((int64_t)b * (L - kWave)) / (kBlocks - 1) + lane];
        uint32_t m = 0;
#pragma unroll
        for (int b = 0; b < kBlocks; ++b) {
            const bool ok = !__builtin_isnan(v[b]);
            const uint64_t msk = ballot(ok);
            if (ok) buf[m + lane_prefix(msk)] = okey(dbits(v[b]));
            m += popc64(msk);
        }
        cnt = uni32(m);
        __syncthreads();
        // rank (from the top) of the probe key: 1.5x (KRR_PROBE_MARGIN_X4 / 4) the kept fraction of slots, + 4
        const uint64_t j = ((uint64_t)m * tkeep * KRR_PROBE_MARGIN_X4 + 4 * (uint64_t)L - 1) / (4 * (uint64_t)L) + 4;
        uint64_t t = 0;
        if (m >= (uint32_t)kWave && j < m) {
            uint64_t mn, mx;
            buf_minmax(mn, mx);
            t = kth_largest((uint32_t)j, mn, mx);
            if (bad) t = 0;
        }
        __syncthreads();
        cnt = 0;
        bad = 0;
        return uni64(t);
    }
};


// Count present, numerically negative samples (x < -0.0) of [beg, end).
__device__ uint64_t count_negative(const double* __restrict__ vals, int64_t beg, int64_t end, int lane) {
    uint32_t c = 0;
    for (int64_t base = beg; base < end; base += kWave) {
        const int64_t i = base + lane;
        if (i < end) {
            const uint64_t u = dbits(vals[i]);
            c += ((u & kSignBit) && !is_zero_bits(u) && !is_nan_bits(u)) ? 1u : 0u;
        }
    }
    return wave_sum_u32(c);
}

// Bits of the j-th (0-based, position order) sample equal to +-0.0 in [beg, end).
__device__ uint64_t nth_zero_bits(const double* __restrict__ vals, int64_t beg, int64_t end, uint64_t j,
                                  int lane) {
    uint64_t run = 0;
    for (int64_t base = beg; base < end; base += kWave) {
        const int64_t i = base + lane;
        const bool in = i < end;
        const uint64_t u = in ? dbits(vals[i]) : 1ull;
        const bool z = in && is_zero_bits(u);
        const uint64_t m = ballot(z);
        const uint32_t c = popc64(m);
        if (run + c > j) {
            const uint32_t want = (uint32_t)(j - run);
            const uint64_t sel = ballot(z && lane_prefix(m) == want);
            const int src = __ffsll((long long)sel) - 1;
            return lane_bcast64(u, src);
        }
        run += c;
    }
    return 0;
}

// numpy _lerp (numpy/lib/_function_base_impl.py, numpy 2.2.6) with no FMA contraction.
__device__ __forceinline__ double np_lerp(double a, double b, double t) {
#pragma clang fp contract(off)
    const double d = __dsub_rn(b, a);
    if (t >= 0.5) return __dsub_rn(b, __dmul_rn(d, __dsub_rn(1.0, t)));
    return __dadd_rn(a, __dmul_rn(d, t));
}

struct SelectArgs {
    const double* vals;
    const int64_t* offs;
    int64_t S;
    int32_t mode;
    int32_t gaps;
    int64_t p_num, p_den;
    double q;
    const int64_t* ktab;  // krr_percentile_params.k_table (null: the exact floor)
    int64_t ktab_len;
    uint32_t cap;        // single-pass candidate capacity (keys); longer segments use hselect
    uint32_t wcap;       // window select (wselect) capacity (keys)
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
    int64_t* rec = nullptr;  // optional 32-B result records (k_pack_records layout), CPU half
    unsigned long long* stats = nullptr;  // optional: [0] += segments wselect handed to hselect
    // wselect misses: segment ids for the hselect pass that follows (k_hselect_list)
    int64_t* fail_list = nullptr;
    unsigned int* fail_count = nullptr;   // this launch's list length
    unsigned int* fail_reset = nullptr;   // the previous launch's counter: zeroed for the next one
    int32_t remap = 1;   // xcd_item: per-XCD segment ranges (KRR_XCD_REMAP_MAXLEN)
};

// One half of an object's 32-B record (k_pack_records layout): half 0 = CPU, 1 = memory.
__device__ __forceinline__ void put_record(int64_t* rec, int64_t s, int half, double v, uint64_t n, uint32_t f) {
    if (rec) {
        rec[4 * s + half] = (int64_t)dbits(v);
        rec[4 * s + 2 + half] = (int64_t)(n | ((uint64_t)f << 48));
    }
}

// Ranks a SORTED_LOWER / LINEAR result needs among n present samples (ascending,
// 0-based): SORTED_LOWER r0 = r1 = k; LINEAR numpy's prev/next with its gamma.
struct Ranks {
    int64_t r0, r1;
    double gamma;
};

__device__ __forceinline__ Ranks ranks_for(const SelectArgs& A, uint64_t n) {
    Ranks R;
    R.gamma = 0.0;
    if (A.mode == KRR_PCT_SORTED_LOWER) {
        R.r0 = R.r1 = rule_rank((int64_t)n, A.p_num, A.p_den, A.ktab, A.ktab_len);
    } else {  // KRR_PCT_LINEAR, numpy method="linear"
        const double vidx = __dmul_rn((double)(n - 1), A.q);
        if (vidx >= (double)(n - 1)) {
            R.r0 = R.r1 = (int64_t)n - 1;
            R.gamma = __dsub_rn(vidx, -1.0);  // numpy subtracts the clipped index -1
        } else {
            const double fl = floor(vidx);
            R.r0 = (int64_t)fl;
            R.r1 = R.r0 + 1;
            R.gamma = __dsub_rn(vidx, fl);
        }
    }
    return R;
}

// Result from the ascending keys k0 (rank r0) and k1 (rank r1).
__device__ __forceinline__ double finish_value(const SelectArgs& A, const Ranks& R, uint64_t k0, uint64_t k1,
                                               int64_t beg, int64_t end, int lane) {
    const double a = bitsd(okey_inv(k0));
    if (A.mode == KRR_PCT_SORTED_LOWER) {
        uint64_t bits = dbits(a);
        if (is_zero_bits(bits)) {
            // Python sorted() is stable and -0 == +0: the zero at rank r is the
            // (r - #negatives)-th zero in position order.
            const uint64_t neg = count_negative(A.vals, beg, end, lane);
            bits = nth_zero_bits(A.vals, beg, end, (uint64_t)R.r0 - neg, lane);
        }
        return bitsd(bits);
    }
    const double b = R.r1 != R.r0 ? bitsd(okey_inv(k1)) : a;
    return np_lerp(a, b, R.gamma);
}

__device__ __forceinline__ void write_result(const SelectArgs& A, int64_t s, double v, uint64_t n, uint32_t flags,
                                             int lane) {
    if (lane == 0) {
        A.out_v[s] = v;
        A.out_n[s] = (int64_t)n;
        A.out_f[s] = flags;
        put_record(A.rec, s, 0, v, n, flags);
    }
}

// LDS of the select kernels: [H 1 KiB][gather 512 B] then, from kSelectLdsFixed,
// either the single-pass candidate keys (cap x 8 B) or hselect's histogram
// (kHistBins x 4 B) + collect buffer (kCollectCap x 8 B).

// One CPU segment (SORTED_LOWER / LINEAR) by one wave, single HBM pass.
// `stream(P)` runs the segment's samples through P and returns the NaN padding.
template <class Streamer>
__device__ __forceinline__ void select_segment_with(const SelectArgs& A, int64_t s, unsigned char* smem, int lane,
                                                    Streamer stream) {
    {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        const int64_t L = end - beg;
        const SidePlan sp = plan_side(L, A.mode, A.p_num, A.p_den, A.q, A.ktab != nullptr);
        SelectProc P;
        P.buf = reinterpret_cast<uint64_t*>(smem + kSelectLdsFixed);
        P.H = reinterpret_cast<uint32_t*>(smem);
        P.small = reinterpret_cast<uint64_t*>(smem + 1024);
        P.lane = lane;
        P.cap = A.cap;
        P.tkeep = sp.tkeep;
        P.tstop = A.cap - kChunkElems / 2;
        P.flip = sp.bottom ? ~0ull : 0ull;
        P.cnt = 0;
        P.bad = 0;
#ifdef KRR_DIAG
        for (int d = 0; d < D_WORDS; ++d) P.diag[d] = 0;
        KRR_DIAG_T0(t_begin);
#endif
        uint64_t thr0 = 0;  // inclusive at the lowest key: every sample is a candidate
#if KRR_SELECT_PROBE
        if (!sp.bottom && A.cap && select_probe_pays(L, sp.tkeep, A.cap)) thr0 = P.probe_threshold(A.vals, beg, L);
#endif
        uint32_t pad;
        uint64_t nnan, n;
#pragma unroll 1
        for (;;) {
            P.cnt = 0;
            P.eqs = 0;
            P.nnan_lane = 0;
            P.bad = 0;
            P.set_thr(thr0, 1u);
            pad = stream(P);  // NaN padding slots
            __syncthreads();
            nnan = wave_sum_u32(P.nnan_lane) - pad;
            n = A.gaps ? (uint64_t)L - nnan : (uint64_t)L;  // present samples
            if (thr0 == 0 || n == 0 || (nnan && !A.gaps)) break;
            // Speculative start: exact iff the lowest needed rank is held in buf
            // (ranks below n - cnt - ties lie under thr0); else stream again from
            // the lowest key.
            const uint64_t ties = P.incl ? 0u : P.eqs;
            if (!P.bad && (uint64_t)ranks_for(A, n).r0 >= n - P.cnt - ties) break;
            thr0 = 0;
        }
#ifdef KRR_DIAG
        KRR_DIAG_T0(t_final);
#endif
        uint64_t bmn = 0, bmx = 0;
        if (P.cnt) P.buf_minmax(bmn, bmx);

        uint32_t flags = 0;
        double result = bitsd(kQuietNaN);
        if (n == 0) {
            flags |= KRR_FLAG_EMPTY;
        } else if (nnan && !A.gaps) {
            flags |= KRR_FLAG_NAN;
        } else {
            const Ranks R = ranks_for(A, n);
            uint64_t k0 = 0, k1 = 0;
#if KRR_PAIR_RANKS
            if (R.r1 != R.r0) {  // LINEAR: both adjacent ranks from one locate
                P.rank_key_pair((uint64_t)R.r0, n, bmn, bmx, k0, k1);
                k0 ^= P.flip;
                k1 ^= P.flip;
            } else {
                k0 = P.rank_key((uint64_t)R.r0, n, bmn, bmx) ^ P.flip;
            }
#else
            // one rank-query body serves both ranks (a 1-2 iteration loop keeps it inlined once)
            const int nq = R.r1 != R.r0 ? 2 : 1;
#pragma unroll 1
            for (int qi = 0; qi < nq; ++qi) {
                const uint64_t kq = P.rank_key((uint64_t)(qi ? R.r1 : R.r0), n, bmn, bmx) ^ P.flip;
                if (qi) k1 = kq;
                else k0 = kq;
            }
#endif
            result = finish_value(A, R, k0, k1, beg, end, lane);
        }
        if (P.bad) flags |= KRR_FLAG_CAPACITY | (P.bad << 8);  // reason bits (diagnostic)
#ifdef KRR_DIAG
        {
            const unsigned long long t_end = __builtin_amdgcn_s_memtime();
            P.diag[D_TOTAL] = t_end - t_begin;
            P.diag[D_FINAL] = t_end - t_final;
            if (lane == 0 && g_diag)
                for (int d = 0; d < D_WORDS; ++d) g_diag[(size_t)s * D_WORDS + d] = P.diag[d];
        }
#endif
        write_result(A, s, result, n, flags, lane);
        __syncthreads();
    }
}

__device__ __forceinline__ void select_segment(const SelectArgs& A, int64_t s, unsigned char* smem, int lane) {
    const int64_t beg = A.offs[s], end = A.offs[s + 1];
    select_segment_with(A, s, smem, lane,
                        [&](SelectProc& P) {
                            // opaque bounds: the speculative start's retry loop must not
                            // hoist the stream's address set-up and keep it live throughout
                            int64_t b = beg, e = end;
                            asm volatile("" : "+s"(b), "+s"(e));
                            return stream_segment<true>(A.vals, b, e, P, lane);
                        });
}

// ---------------------------------------------------------------------------
// hselect: exact order statistics of a segment whose candidate set would not
// fit LDS (mid percentiles of long series: p50 of 50,400 samples needs 25k
// keys).  A streaming histogram pass over a key range [lo, hi] (kHistBins
// bins, LDS atomics) locates the bin holding the needed ranks, counting the
// keys below lo; a second streaming pass collects that bin's keys (expected
// ~100) into LDS, where the ranks are selected exactly.  The first range comes
// from a 64-sample strided probe of the segment widened 16x each way in value
// (4 exponents in key space), so two HBM passes are the common case; a rank
// that falls outside [lo, hi] or into a bin with more than kCollectCap keys
// refines the range and repeats (bounded).  Zeros are counted apart when they
// lie below lo, so a mostly-zero series resolves in the first pass.
// ---------------------------------------------------------------------------
constexpr uint64_t kKeyNegInf = 0x000FFFFFFFFFFFFFull;  // okey(-inf)
constexpr uint64_t kKeyPosInf = 0xFFF0000000000000ull;  // okey(+inf)
constexpr uint64_t kKeyNegZero = 0x7FFFFFFFFFFFFFFFull; // okey(-0)
constexpr uint64_t kKeyPosZero = 0x8000000000000000ull; // okey(+0)

template <bool FIRST, bool ZSPLIT, bool BAND = false>
struct HistProc {
    uint32_t* hist;
    uint64_t lo, span;
    uint32_t sh;
    uint32_t below_l, zb_l, z0_l, nan_l, nneg_l;  // per-lane counters
    // BAND: keys in [blo, blo + bspan] are also appended to bbuf (the first bcap of
    // them; bcnt counts all), keys below blo counted per lane (+ negative NaNs).
    uint64_t* bbuf;
    uint64_t blo, bspan;
    uint32_t bcnt, bbelow_l;

    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const double d = slot_val(c, j);
            const uint64_t x = dbits(d);
            const uint64_t key = okey(x);
            below_l += key < lo ? 1u : 0u;  // + negative NaNs (key < okey(-inf)); removed later
            if (BAND) {
                // the band lies inside [okey(-inf), okey(+inf)]: no NaN key enters it
                bbelow_l += key < blo ? 1u : 0u;
                const bool inb = key - blo <= bspan;
                const uint64_t m = ballot(inb);
                if (m) {
                    const uint32_t at = bcnt + lane_prefix(m);
                    if (inb && at < kCollectCap) bbuf[at] = key;
                    bcnt = uni32(bcnt + popc64(m));
                }
            }
            if (ZSPLIT) {
                zb_l += key <= kKeyPosZero ? 1u : 0u;  // negatives, -0, +0 (+ negative NaNs)
                z0_l += x == 0 ? 1u : 0u;
            }
            if (FIRST) {
                const bool nan = __builtin_isnan(d);
                nan_l += nan ? 1u : 0u;
                nneg_l += (nan && (x & kSignBit)) ? 1u : 0u;
            }
            const uint64_t t = key - lo;
            if (t <= span) atomicAdd(&hist[(uint32_t)(t >> sh)], 1u);
            // one slot at a time: nothing of this slot stays live into the next
            asm volatile("" ::: "memory");
        }
    }
};

struct HistCounts {
    uint32_t pad, below_l, zb_l, z0_l, nan_l, nneg_l;
    uint32_t bcnt, bbelow_l;  // band (first pass with a band only)
};

template <bool FIRST, bool ZSPLIT, bool BAND = false>
__device__ __forceinline__ HistCounts hist_pass(const double* vals, int64_t beg, int64_t end, uint32_t* hist,
                                                uint64_t lo, uint64_t span, uint32_t sh, int lane,
                                                uint64_t* bbuf = nullptr, uint64_t blo = 0, uint64_t bspan = 0) {
    HistProc<FIRST, ZSPLIT, BAND> HP;
    HP.hist = hist;
    HP.lo = lo;
    HP.span = span;
    HP.sh = sh;
    HP.below_l = HP.zb_l = HP.z0_l = HP.nan_l = HP.nneg_l = 0;
    HP.bbuf = bbuf;
    HP.blo = blo;
    HP.bspan = bspan;
    HP.bcnt = HP.bbelow_l = 0;
    HistCounts hc;
    hc.pad = stream_segment<true>(vals, beg, end, HP, lane);
    hc.below_l = HP.below_l;
    hc.zb_l = HP.zb_l;
    hc.z0_l = HP.z0_l;
    hc.nan_l = HP.nan_l;
    hc.nneg_l = HP.nneg_l;
    hc.bcnt = HP.bcnt;
    hc.bbelow_l = HP.bbelow_l;
    return hc;
}

struct CollectProc {
    uint64_t* buf;
    uint64_t lo, span;
    uint32_t cnt;
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const uint64_t key = okey(dbits(slot_val(c, j)));
            const bool in = key - lo <= span;  // NaN keys lie outside [okey(-inf), okey(+inf)]
            const uint64_t m = ballot(in);
            if (m) {
                if (in) buf[cnt + lane_prefix(m)] = key;
                cnt = uni32(cnt + popc64(m));
            }
        }
    }
};

// Lane l's share of the histogram is bins [32 l, 32 l + 32): its total and the
// inclusive prefix of the totals over lanes.
struct HistScan {
    uint32_t t, incl, total;
};

__device__ __forceinline__ HistScan hist_scan(const uint32_t* hist, int lane) {
    constexpr uint32_t per = kHistBins / kWave;
    static_assert(per % 4 == 0, "bins per lane");
    const uint4* h4 = reinterpret_cast<const uint4*>(hist + (uint32_t)lane * per);
    uint32_t t = 0;
#pragma unroll
    for (uint32_t j = 0; j < per / 4; ++j) {
        const uint4 v = h4[j];
        t += v.x + v.y + v.z + v.w;
    }
    const uint32_t incl = wave_scan32(t, 0u, OpAdd32{});
    HistScan hs;
    hs.t = t;
    hs.incl = incl;
    hs.total = lane_bcast32(incl, kWave - 1);
    return hs;
}

// Bin holding ascending rank r (0-based, r < total, relative to the histogram's
// first key): bin index, keys in earlier bins, keys in the bin.
__device__ __forceinline__ void hist_find(const uint32_t* hist, const HistScan& hs, uint64_t r, int lane,
                                          uint32_t& b, uint64_t& before, uint32_t& cnt) {
    constexpr uint32_t per = kHistBins / kWave;
    const uint32_t rr = (uint32_t)r;
    const uint64_t m = ballot(rr < hs.incl);
    const int src = __ffsll((long long)m) - 1;
    const uint32_t base = lane_bcast32(hs.incl - hs.t, src);
    // second level: lane j < per looks at bin src * per + j
    const uint32_t h = (uint32_t)lane < per ? hist[(uint32_t)src * per + (uint32_t)lane] : 0u;
    const uint32_t incl = wave_scan32(h, 0u, OpAdd32{});
    const uint64_t m2 = ballot((uint32_t)lane < per && rr - base < incl);
    const int sel = __ffsll((long long)m2) - 1;
    b = (uint32_t)src * per + (uint32_t)sel;
    cnt = lane_bcast32(h, sel);
    before = base + lane_bcast32(incl - h, sel);
}

// A resolved rank: either an exact key or a key range [lo, hi] holding `count`
// keys with `below` keys smaller than lo.
struct RankLoc {
    uint64_t lo, hi, below, count;
    uint32_t exact;
};

// hselect's band (KRR_HSEL_BAND): 16 consecutive samples from each of ~L/400 evenly
// spread blocks (16 to 128 blocks: ~4% of the segment's bytes) are ranked in LDS, and the keys around the
// needed ranks' estimated position among them, sized to ~3/4 of the collect buffer,
// become [blo, bhi].  The first streaming pass then collects that band beside its
// histogram; when the exact counts show both ranks inside it, the segment is done in
// one HBM pass.  Otherwise nothing changes: the pass's histogram drives the usual
// collect pass.  Returns false when the segment is too short or too long for a band.
// at most 128 (and what hselect's LDS holds); ~L/400 blocks (probe = ~4% of the segment)
constexpr int kProbeBlocks = (int)((kHselectLds / (16 * 8) < 128 ? kHselectLds / (16 * 8) : 128) & ~(size_t)7);
constexpr int kProbeSamples = kProbeBlocks * 16;

__device__ __forceinline__ bool hselect_band(const SelectArgs& A, int64_t beg, int64_t L, unsigned char* smem,
                                             int lane, uint64_t& blo, uint64_t& bhi) {
    static_assert(KRR_HSEL_BAND_MIN >= 16 * 16 * 2, "probe blocks must not overlap");
    if (L < KRR_HSEL_BAND_MIN || !(A.q >= 0.0 && A.q <= 1.0)) return false;
    int64_t nb = (L / 400) & ~(int64_t)7;
    nb = nb < 16 ? 16 : (nb > kProbeBlocks ? kProbeBlocks : nb);
    // sample ranks one band may span: ~0.75 * kCollectCap keys, L / (16 nb) keys per sample
    const int64_t width = ((int64_t)kCollectCap * 3 * 16 * nb) / (4 * L);
    const int64_t delta = width / 2 - 1;
    if (delta < 2) return false;
    uint64_t* pbuf = reinterpret_cast<uint64_t*>(smem + kSelectLdsFixed);  // hist + collect area
    static_assert(kProbeSamples * 8 <= kHselectLds, "probe keys fit hselect's LDS");
    // KRR_PROBE_BATCH blocks' loads in flight at a time (registers: 2 doubles per block)
    const int64_t sub = (lane & 7) * 2;
    const int nrounds = (int)(nb / 8);
    uint32_t cnt = 0;
#pragma unroll 1
    for (int it0 = 0; it0 < nrounds; it0 += KRR_PROBE_BATCH) {
        double v[2 * KRR_PROBE_BATCH];
#pragma unroll
        for (int it = 0; it < KRR_PROBE_BATCH; ++it) {
            const bool live = it0 + it < nrounds;  // wave-uniform
            const int64_t b = live ? (int64_t)(it0 + it) * 8 + (lane >> 3) : 0;  // always a real slot
            const int64_t i = beg + (b * (L - 16)) / (nb - 1) + sub;
            v[2 * it] = live ? A.vals[i] : __builtin_nan("");
            v[2 * it + 1] = live ? A.vals[i + 1] : __builtin_nan("");
        }
#pragma unroll
        for (int j = 0; j < 2 * KRR_PROBE_BATCH; ++j) {
            const bool ok = !__builtin_isnan(v[j]);
            const uint64_t m = ballot(ok);
            if (ok) pbuf[cnt + lane_prefix(m)] = okey(dbits(v[j]));
            cnt = uni32(cnt + popc64(m));
        }
    }
    __syncthreads();
    if (cnt < (uint32_t)(2 * nb)) return false;  // mostly gaps: no estimate worth a band
    SelectProc P;
    P.buf = pbuf;
    P.H = reinterpret_cast<uint32_t*>(smem);
    P.small = reinterpret_cast<uint64_t*>(smem + 1024);
    P.lane = lane;
    P.cnt = cnt;
    P.bad = 0;
    uint64_t mn, mx;
    P.buf_minmax(mn, mx);
    const int64_t rho = (int64_t)floor(A.q * (double)(cnt - 1));
    const int64_t alo = rho - delta, ahi = rho + 1 + delta;  // ascending sample ranks
    // R-th largest (1-based) of cnt keys = ascending rank cnt - R
    blo = alo <= 0 ? kKeyNegInf : P.kth_largest((uint32_t)((int64_t)cnt - alo), mn, mx);
    bhi = ahi >= (int64_t)cnt - 1 ? kKeyPosInf : P.kth_largest((uint32_t)((int64_t)cnt - ahi), mn, mx);
    __syncthreads();
    if (P.bad) return false;
    blo = blo < kKeyNegInf ? kKeyNegInf : blo;
    bhi = bhi > kKeyPosInf ? kKeyPosInf : bhi;
    return blo <= bhi;
}

__device__ __forceinline__ void hselect_segment(const SelectArgs& A, int64_t s, unsigned char* smem, int lane) {
    {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        const int64_t L = end - beg;
        uint32_t* hist = reinterpret_cast<uint32_t*>(smem + kSelectLdsFixed);
        uint64_t* cbuf = reinterpret_cast<uint64_t*>(smem + kSelectLdsFixed + kHistBins * 4);
        uint32_t bad = 0;

        // 64-sample strided probe -> first key range
        uint64_t kmn = ~0ull, kmx = 0;
        if (L > 0) {
            const int64_t i = L >= kWave ? ((int64_t)lane * L) / kWave : (lane < L ? lane : 0);
            const uint64_t x = dbits(A.vals[beg + i]);
            const bool ok = !is_nan_bits(x) && !is_zero_bits(x);
            const uint64_t k = okey(x);
            kmn = ok ? k : ~0ull;
            kmx = ok ? k : 0ull;
        }
        kmn = wave_min_u64(kmn);
        kmx = wave_max_u64(kmx);
        constexpr uint64_t kWiden = 4ull << 52;  // 16x in value
        uint64_t lo = kKeyNegInf, hi = kKeyPosInf;
        if (kmn <= kmx) {
            lo = kmn >= kKeyNegInf + kWiden ? kmn - kWiden : kKeyNegInf;
            hi = kmx <= kKeyPosInf - kWiden ? kmx + kWiden : kKeyPosInf;
        }

        uint64_t n = 0, nneg = 0;
        uint32_t flags = 0;
        double result = bitsd(kQuietNaN);
        Ranks R;
        R.r0 = R.r1 = 0;
        R.gamma = 0.0;
        RankLoc loc0, loc1;
        loc0.lo = loc0.hi = loc1.lo = loc1.hi = 0;
        loc0.exact = loc1.exact = 0;
        uint32_t done = 0;
        uint64_t blo = 0, bhi = 0;
        const bool band = KRR_HSEL_BAND && hselect_band(A, beg, L, smem, lane, blo, bhi);
#pragma unroll 1
        for (int pass = 0; pass < 10 && !done; ++pass) {
            // ---- histogram pass over [lo, hi]
            const uint64_t span = hi - lo;
            const int bits = span ? 64 - __clzll((long long)span) : 0;
            const uint32_t sh = bits > kHistBits ? (uint32_t)(bits - kHistBits) : 0u;
            for (uint32_t i = lane; i < kHistBins; i += kWave) hist[i] = 0;
            __syncthreads();
            const uint32_t zsplit = lo > kKeyPosZero ? 1u : 0u;
            HistCounts HP;
            if (pass == 0 && band) {
                if (zsplit)
                    HP = hist_pass<true, true, true>(A.vals, beg, end, hist, lo, span, sh, lane, cbuf, blo, bhi - blo);
                else
                    HP = hist_pass<true, false, true>(A.vals, beg, end, hist, lo, span, sh, lane, cbuf, blo, bhi - blo);
            } else if (pass == 0) {
                if (zsplit) HP = hist_pass<true, true>(A.vals, beg, end, hist, lo, span, sh, lane);
                else HP = hist_pass<true, false>(A.vals, beg, end, hist, lo, span, sh, lane);
            } else {
                if (zsplit) HP = hist_pass<false, true>(A.vals, beg, end, hist, lo, span, sh, lane);
                else HP = hist_pass<false, false>(A.vals, beg, end, hist, lo, span, sh, lane);
            }
            const uint32_t pad = HP.pad;
            __syncthreads();
            if (pass == 0) {
                const uint64_t nnan = wave_sum_u32(HP.nan_l) - pad;
                nneg = wave_sum_u32(HP.nneg_l);
                n = A.gaps ? (uint64_t)L - nnan : (uint64_t)L;
                if (n == 0) {
                    flags |= KRR_FLAG_EMPTY;
                    break;
                }
                if (nnan && !A.gaps) {
                    flags |= KRR_FLAG_NAN;
                    break;
                }
                R = ranks_for(A, n);
                if (band && HP.bcnt <= kCollectCap) {
                    // both ranks inside the collected band: select there, one HBM pass in all
                    const uint64_t bb = wave_sum_u32(HP.bbelow_l) - nneg;
                    if (bb <= (uint64_t)R.r0 && (uint64_t)R.r1 < bb + HP.bcnt) {
                        SelectProc P;
                        P.buf = cbuf;
                        P.H = reinterpret_cast<uint32_t*>(smem);
                        P.small = reinterpret_cast<uint64_t*>(smem + 1024);
                        P.lane = lane;
                        P.cnt = HP.bcnt;
                        P.bad = 0;
                        uint64_t mn, mx;
                        P.buf_minmax(mn, mx);
                        loc0.lo = P.kth_largest((uint32_t)(HP.bcnt - ((uint64_t)R.r0 - bb)), mn, mx);
                        loc1.lo = R.r1 == R.r0 ? loc0.lo
                                               : P.kth_largest((uint32_t)(HP.bcnt - ((uint64_t)R.r1 - bb)), mn, mx);
                        bad |= P.bad;
                        done = 1;
                        break;
                    }
                }
            }
            const uint64_t below = wave_sum_u32(HP.below_l) - nneg;
            const uint64_t zb = zsplit ? wave_sum_u32(HP.zb_l) - nneg : 0;
            const uint64_t z0 = zsplit ? wave_sum_u32(HP.z0_l) : 0;
            const HistScan hs = hist_scan(hist, lane);
            const uint64_t inr = hs.total;
            // locate both ranks
            // two named locations (not an indexed array: that would live in scratch)
            auto locate_rank = [&](uint64_t r) {
                RankLoc l;
                l.exact = 0;
                l.below = l.count = 0;
                if (r < below) {
                    if (zsplit && r >= zb - z0 && r < zb) {
                        l.exact = 1;
                        l.lo = l.hi = kKeyPosZero;
                    } else if (zsplit && r < zb) {
                        l.lo = kKeyNegInf;
                        l.hi = kKeyNegZero;
                        l.below = 0;
                        l.count = zb - z0;
                    } else if (zsplit) {
                        l.lo = kKeyPosZero + 1;
                        l.hi = lo - 1;
                        l.below = zb;
                        l.count = below - zb;
                    } else {
                        l.lo = kKeyNegInf;
                        l.hi = lo - 1;
                        l.below = 0;
                        l.count = below;
                    }
                } else if (r < below + inr) {
                    uint32_t b, c;
                    uint64_t before;
                    hist_find(hist, hs, r - below, lane, b, before, c);
                    l.lo = lo + ((uint64_t)b << sh);
                    const uint64_t w = (1ull << sh) - 1;
                    l.hi = hi - l.lo <= w ? hi : l.lo + w;
                    l.below = below + before;
                    l.count = c;
                } else {
                    l.lo = hi + 1;
                    l.hi = kKeyPosInf;
                    l.below = below + inr;
                    l.count = n - below - inr;
                }
                if (!l.exact && l.lo == l.hi) l.exact = 1;
                return l;
            };
            loc0 = locate_rank((uint64_t)R.r0);
            loc1 = R.r1 != R.r0 ? locate_rank((uint64_t)R.r1) : loc0;
            __syncthreads();
            if (loc0.exact && loc1.exact) {
                done = 1;
                break;
            }
            // the key range still to resolve (one range, or the union of two)
            RankLoc u = loc0.exact ? loc1 : loc0;
            if (!loc0.exact && !loc1.exact && (loc1.lo != loc0.lo || loc1.hi != loc0.hi)) {
                u.lo = loc0.lo;
                u.hi = loc1.hi;
                u.below = loc0.below;
                u.count = loc1.below + loc1.count - loc0.below;
            }
            if (u.count <= kCollectCap) {
                // ---- collect pass: the range's keys into LDS, select there
                CollectProc CP;
                CP.buf = cbuf;
                CP.lo = u.lo;
                CP.span = u.hi - u.lo;
                CP.cnt = 0;
                stream_segment<true>(A.vals, beg, end, CP, lane);
                __syncthreads();
                if (CP.cnt != (uint32_t)u.count) {
                    bad |= 32u;
                    break;
                }
                SelectProc P;
                P.buf = cbuf;
                P.H = reinterpret_cast<uint32_t*>(smem);
                P.small = reinterpret_cast<uint64_t*>(smem + 1024);
                P.lane = lane;
                P.cnt = CP.cnt;
                P.bad = 0;
                uint64_t mn, mx;
                P.buf_minmax(mn, mx);
                // ascending index in the range -> R-th largest (1-based)
                if (!loc0.exact) loc0.lo = P.kth_largest((uint32_t)(u.count - ((uint64_t)R.r0 - u.below)), mn, mx);
                if (!loc1.exact)
                    loc1.lo = R.r1 == R.r0 ? loc0.lo
                                           : P.kth_largest((uint32_t)(u.count - ((uint64_t)R.r1 - u.below)), mn, mx);
                loc0.exact = loc1.exact = 1;
                bad |= P.bad;
                done = 1;
                break;
            }
            // ---- refine: histogram the range again
            lo = u.lo;
            hi = u.hi;
        }
        if (n && !(flags & (KRR_FLAG_EMPTY | KRR_FLAG_NAN))) {
            if (done) result = finish_value(A, R, loc0.lo, loc1.lo, beg, end, lane);
            else bad |= 64u;
        }
        if (bad) flags |= KRR_FLAG_CAPACITY | (bad << 8);
        write_result(A, s, result, n, flags, lane);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// wselect: the first choice for order statistics whose candidate set does not
// fit LDS (mid percentiles of long series), in ONE HBM pass.  The wave keeps an
// inclusive key window [lo, hi]: LDS holds every present sample seen so far
// whose key lies in it, and per-lane counters hold how many fell below it.  The
// window starts as every key; whenever the buffer fills it shrinks around the
// target's estimated rank among the samples seen so far (seen-rank):
//   S seen present samples, at most U unseen ones (unread slots), q = p / 100;
//   the target's seen-rank has mean ~ q (S - 1) and, for exchangeable samples,
//   standard deviation sqrt(q (1 - q) S U / (S + U)) (0 once nothing is unseen);
//   the new window spans KRR_WSEL_Z of those plus a few ranks each way.
// For config 2's p50 (50,400 slots) that is ~2 shrinks per segment and a final
// window of ~1,300 keys.  The window only ever narrows, so what it holds stays
// exact; nothing here is trusted: at the end the exact counts decide.  When both
// needed ranks lie inside the window they are selected there; otherwise (a
// trending series the estimate misjudged, a crowded key, a NaN in the compact
// layout) the segment runs hselect below (two passes), so the answer is exact
// whatever the data.  A window of one key (e.g. p50 of a mostly-zero series)
// only counts.  No histogram atomics and no probe: the per-slot work is the
// single-pass select's (a range test, a below count, a NaN count).
// ---------------------------------------------------------------------------
#ifndef KRR_WSEL
#define KRR_WSEL 1
#endif
#ifndef KRR_WSEL_Z
#define KRR_WSEL_Z 5.0  // v26: 4.5 left ~1 statistical miss per 100k short segments (a ~40 us serial tail)
#endif
#ifndef KRR_WSEL_BINS
#define KRR_WSEL_BINS 1  // shrink to histogram-bin edges (one pass) instead of exact keys (0)
#endif
// Window keys in LDS.  Misses are finished by a separate hselect launch
// (k_hselect_list), so the window kernel's LDS and registers are its own.
constexpr uint32_t kWselCap = (uint32_t)KRR_WSEL_CAP & ~63u;
constexpr uint32_t kWselCapLong = (uint32_t)KRR_WSEL_CAP_LONG & ~63u;
#ifndef KRR_WSEL_CAP_MIN_SLACK
#define KRR_WSEL_CAP_MIN_SLACK 64  // the first chunk (every present sample) fits an empty window
#endif
static_assert(kWselCap >= kChunkElems + KRR_WSEL_CAP_MIN_SLACK && kWselCapLong >= kWselCap,
              "the window buffer takes a chunk before its first shrink");
// Per launch: more waves per CU for shorter segments (their fixed per-segment work
// needs the overlap), a larger window for long ones (fewer shrinks).
// Long segments take the long-segment kernel in every layout: its rare window misses run
// hselect inline, beside the other waves.  (Gapped 50,400-slot segments on the 16-waves/CU
// kernel were 1.5% faster at p50/p95 in the A/B, profiles/r02/z, but a miss there goes to the
// separate miss pass, where ONE wave streams the whole segment twice: on the bench's data one
// miss per launch cost config 2 p97 +150 us.)
#ifndef KRR_WSEL_LONG_GAPS
#define KRR_WSEL_LONG_GAPS 1  // 0: gapped layouts keep the 16-waves/CU kernel at any length
#endif
KRR_HD inline uint32_t wsel_cap_for(int64_t Lmax, bool gaps = false) {
    return Lmax >= KRR_WSEL_LONG && (KRR_WSEL_LONG_GAPS || !gaps) ? kWselCapLong : kWselCap;
}
// Dynamic LDS past kSelectLdsFixed of a window launch: the window keys; the long
// kernels finish their misses inline, so hselect's LDS too.
KRR_HD inline size_t window_lds(uint32_t wcap) {
    const size_t w = (size_t)wcap * 8;
    return wcap == kWselCapLong && w < kHselectLds ? kHselectLds : w;
}

enum { WIN_GENERAL = 0, WIN_FAST = 1, WIN_FULL = 2 };  // window classify modes (WindowProc::classify)

// LANE_COUNTS: below / NaN counts per lane in VALU (the long-segment kernels: their
// gapped layouts put NaNs in many chunks, and at 2 waves per SIMD the stream, not
// the vector unit, bounds them); otherwise scalar ballot popcounts (see classify).
// EXPORT: the time-sharded window export (k_window_export): the segment is one time
// slice of a longer series, so the other slices' ext_u slots count as unseen too.
#ifndef KRR_WEXP_Z
#define KRR_WEXP_Z 6.0  // export windows: a miss costs a regather of the series, not a second pass
#endif
template <bool LANE_COUNTS, bool EXPORT = false>
struct WindowProc {
    SelectProc sp;            // buffer algebra (locate / kth / pair) over buf
    uint64_t* buf;
    int lane;
    uint32_t cap;
    uint32_t shrinks;
    uint64_t lo, hi, span;    // inclusive key window
    uint64_t lob;             // raw bits of lo (fast windows: inside [+0, +inf])
    uint32_t fast, full, point;
    uint32_t cnt;             // window keys seen (stored unless point)
    uint64_t below_u, nan_u;  // present samples below the window, NaN slots (committed chunks)
    uint32_t below_l, nan_l, negnan_l;  // LANE_COUNTS: per lane (below_l includes negative NaNs)
    uint64_t below_extra;     // keys dropped below lo by shrinks (uniform)
    uint64_t seen;            // slots of committed chunks (uniform; padding included)
    int64_t L;
    int64_t p_num, p_den;     // percentile p = p_num / p_den
    uint32_t fail;
    double ext_u;             // EXPORT: slots of the series held by the other slices
#ifdef KRR_DIAG
    unsigned long long diag[D_WORDS];
#endif

    __device__ __forceinline__ void set_window(uint64_t l, uint64_t h) {
        lo = uni64(l);
        hi = uni64(h);
        span = hi - lo;
        fast = (lo >= kKeyPosZero && hi <= kKeyPosInf) ? 1u : 0u;
        full = (lo <= kKeyNegInf && hi >= kKeyPosInf) ? 1u : 0u;
        lob = lo ^ kSignBit;
        point = lo == hi ? 1u : 0u;
    }

    // Classify a chunk: per-slot window bits (in[j] = 1: slot j's key is in the window)
    // and the chunk's below / NaN counts (not yet committed).  The counts are ballot
    // popcounts, so the scalar unit adds them up beside the vector work: the chunk loop
    // is what bounds mid percentiles of short series (VALU issue, not HBM).
    //   WIN_FULL     the window is every key (before the first shrink): in = not NaN;
    //   WIN_FAST     the window lies inside [+0, +inf]: one unsigned range test on the
    //                raw bits; "below" is a signed compare (every negative, negative
    //                NaNs too); NaN slots are only ORed into a mask, and a chunk that
    //                holds one is recounted (rare outside gapped layouts);
    //   WIN_GENERAL  order-preserving keys.
    template <int MODE>
    __device__ __forceinline__ void classify(const double2 (&c)[kUnroll], uint32_t (&in)[2 * kUnroll], uint32_t& b,
                                             uint32_t& nn) const {
        b = nn = 0;
        uint64_t anynan = 0;
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const double v = slot_val(c, j);
            const uint64_t x = dbits(v);
            bool w;
            if constexpr (MODE == WIN_FULL) {
                w = !__builtin_isnan(v);
                nn += popc64(ballot(!w));
            } else if constexpr (MODE == WIN_FAST) {
                w = (x - lob) <= span;                           // rejects negatives and NaNs
                b += popc64(ballot((int64_t)x < (int64_t)lob));  // negatives (incl. -0) are below
                anynan |= ballot(__builtin_isnan(v));
            } else {
                const bool nan = __builtin_isnan(v);
                const uint64_t key = okey(x);
                w = (key - lo) <= span;                          // NaN keys lie outside [okey(-inf), okey(+inf)]
                b += popc64(ballot(key < lo && !nan));
                nn += popc64(ballot(nan));
            }
            // materialised here: a mask held in scalar registers until after the
            // mode branches would be sixteen 64-bit SGPR pairs
            uint32_t t = w ? 1u : 0u;
            asm volatile("" : "+v"(t));
            in[j] = t;
        }
        if (MODE == WIN_FAST && anynan) {
#pragma unroll
            for (int j = 0; j < 2 * kUnroll; ++j) {
                const double v = slot_val(c, j);
                const bool nan = __builtin_isnan(v);
                nn += popc64(ballot(nan));
                b -= popc64(ballot(nan && (int64_t)dbits(v) < 0));  // negative NaNs were counted below
            }
        }
    }

    // Append the chunk's window keys (in[]) from buffer index pos on: predicated LDS
    // writes, a slot outside the window writes this lane's scratch slot (the address
    // is scratch + in * (next - scratch): one 24-bit multiply-add).  Keys of a fast
    // window are non-negative numbers: okey is the sign bit.
    template <int MODE>
    __device__ __forceinline__ void insert(const double2 (&c)[kUnroll], const uint32_t (&in)[2 * kUnroll],
                                           uint32_t pos) {
        unsigned char* const scratch = reinterpret_cast<unsigned char*>(sp.small + lane);
        uint32_t d = (uint32_t)(reinterpret_cast<unsigned char*>(buf + pos) - scratch);  // > 0: buf lies above small
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const uint64_t x = dbits(slot_val(c, j));
            *reinterpret_cast<uint64_t*>(scratch + __umul24(in[j], d)) = MODE == WIN_FAST ? (x | kSignBit) : okey(x);
            d += in[j] << 3;
            asm volatile("" : "+v"(d));  // a running offset: not re-derived from prefix sums of in[]
        }
    }

    // LANE_COUNTS classify: per-lane below / NaN / negative-NaN counts.
    template <bool FAST>
    __device__ __forceinline__ void classify_lanes(const double2 (&c)[kUnroll], uint32_t (&in)[2 * kUnroll],
                                                   uint32_t& b, uint32_t& nn, uint32_t& ng) const {
        b = nn = ng = 0;
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const uint64_t x = dbits(slot_val(c, j));
            const bool nan = is_nan_bits(x);
            bool w, below;
            if (FAST) {
                w = (x - lob) <= span;              // rejects negatives and NaNs
                below = (int64_t)x < (int64_t)lob;  // negatives (incl. -0, negative NaNs) are below
            } else {
                const uint64_t key = okey(x);
                w = (key - lo) <= span;             // NaN keys lie outside [okey(-inf), okey(+inf)]
                below = key < lo;                   // + negative NaNs, removed via ng
            }
            in[j] = w ? 1u : 0u;
            b += below ? 1u : 0u;
            nn += nan ? 1u : 0u;
            ng += (nan && (x >> 63)) ? 1u : 0u;
        }
    }

    // Present samples below the window and NaN slots of the committed chunks.
    __device__ __forceinline__ uint64_t below_total() const {
        if constexpr (LANE_COUNTS) return (uint64_t)wave_sum_u32(below_l) - wave_sum_u32(negnan_l) + below_extra;
        return below_u + below_extra;
    }
    __device__ __forceinline__ uint64_t nan_total() const {
        if constexpr (LANE_COUNTS) return wave_sum_u32(nan_l);
        return nan_u;
    }

    // Every chunk fits: the buffer is shrunk right after a chunk that leaves less than
    // a chunk of room (so the chunk's registers are dead during the shrink).  Only a
    // window crowded by a few repeated keys can overflow: then the segment falls back.
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
        if (uni32(fail)) return;
        uint32_t b, nn, ng = 0, vc = 0, mode;
        uint32_t in[2 * kUnroll];
        if constexpr (LANE_COUNTS) {
            mode = uni32(fast) ? WIN_FAST : WIN_GENERAL;
            if (mode == WIN_FAST) classify_lanes<true>(c, in, b, nn, ng);
            else classify_lanes<false>(c, in, b, nn, ng);
        } else {
            mode = uni32(full) ? WIN_FULL : (uni32(fast) ? WIN_FAST : WIN_GENERAL);
            if (mode == WIN_FAST) classify<WIN_FAST>(c, in, b, nn);
            else if (mode == WIN_FULL) classify<WIN_FULL>(c, in, b, nn);
            else classify<WIN_GENERAL>(c, in, b, nn);
        }
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) vc += in[j];
        const uint32_t incl = wave_scan32(vc, 0u, OpAdd32{});
        const uint32_t C = lane_bcast32(incl, kWave - 1);
        if (!point && cnt + C > cap) {
            // EXPORT: a window crowded by ONE repeated key (a constant stretch whose
            // window still reaches up to +inf) becomes that key's point window, and the
            // chunk is counted against it; anything else fails (the series is a miss)
#ifdef KRR_WEXP_DEBUG
            dbg(3, seen, cnt, C, lo);
#endif
            if constexpr (EXPORT) {
                if (point_rescue()) {
                    point_chunk(c);
                    return;
                }
            }
            fail = 1;
            return;
        }
        if (C && !point) {
            if (mode == WIN_FAST) insert<WIN_FAST>(c, in, cnt + incl - vc);
            else insert<WIN_GENERAL>(c, in, cnt + incl - vc);
        }
        cnt = uni32(cnt + C);
        if constexpr (LANE_COUNTS) {
            below_l += b;
            nan_l += nn;
            negnan_l += ng;
        } else {
            below_u += b;
            nan_u += nn;
        }
        seen += kChunkElems;
        // room for the next chunk: a whole chunk while every key is a candidate, then
        // twice this chunk's candidates (>= 256): the window's share of slots only falls
        const uint32_t room = shrinks == 0 ? kChunkElems : (2 * C > 256 ? 2 * C : 256u);
        if (!point && seen < (uint64_t)L && cnt + room > cap) shrink();
    }

    // Keep the buffer keys in [nl, nh] (in place); the dropped keys below nl join
    // below_extra.  A block of 4 x 64 keys is read before any survivor is written.
    __device__ __forceinline__ void filter_window(uint64_t nl, uint64_t nh) {
        uint32_t w = 0, dropped_below = 0;
        for (uint32_t base = 0; base < cnt; base += kLdsBatch * kWave) {
            uint64_t x[kLdsBatch];
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const uint32_t i = base + t * kWave + lane;
                x[t] = i < cnt ? buf[i] : 0ull;
            }
#pragma unroll
            for (int t = 0; t < kLdsBatch; ++t) {
                const bool inr = base + t * kWave + lane < cnt;
                const bool keep = inr && x[t] >= nl && x[t] <= nh;
                dropped_below += popc64(ballot(inr && x[t] < nl));
                const uint64_t m = ballot(keep);
                if (keep) buf[w + lane_prefix(m)] = x[t];
                w += popc64(m);
            }
        }
        __syncthreads();
        cnt = uni32(w);
        below_extra += uni32(dropped_below);
    }

#ifdef KRR_WEXP_DEBUG
    __device__ void dbg(uint64_t tag, uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
        if (lane == 0 && g_wdbg_on) {
            const unsigned i = atomicAdd(&g_wdbg_n, 1u);
            if (i < 1024) {
                g_wdbg[5 * i] = tag; g_wdbg[5 * i + 1] = a; g_wdbg[5 * i + 2] = b; g_wdbg[5 * i + 3] = c;
                g_wdbg[5 * i + 4] = d;
            }
        }
    }
#endif
    // Narrow the window around the target's estimated seen-rank (header comment).
    __device__ __forceinline__ void shrink() {
        if (point || cnt == 0) return;
        const uint64_t nanc = nan_total();
        const uint64_t below = below_total();
        const uint64_t S = seen - nanc;  // present samples seen
        double U = L > (int64_t)seen ? (double)(L - (int64_t)seen) : 0.0;
        if constexpr (EXPORT) U += ext_u;
        // q from the kernel's scalars here, not a per-segment value the compiler would
        // hoist to kernel entry and keep in registers for the whole launch
        int64_t pn = p_num, pd = p_den;
        asm volatile("" : "+s"(pn), "+s"(pd));
        const double qq = (double)pn / (100.0 * (double)pd);
        const double Sd = (double)S;
        const double c = qq * (Sd - 1.0);
        const double sig = (S > 0 && U > 0.0) ? sqrt(qq * (1.0 - qq) * Sd * U / (Sd + U)) : 0.0;
        const double w = (EXPORT ? KRR_WEXP_Z : KRR_WSEL_Z) * sig + 4.0;
        const int64_t jlo = (int64_t)floor(c - w);
        const int64_t jhi = (int64_t)ceil(c + w) + 1;
        int64_t ilo = jlo - (int64_t)below;  // ascending buffer indices
        int64_t ihi = jhi - (int64_t)below;
        const int64_t last = (int64_t)cnt - 1;
        ilo = ilo < 0 ? 0 : (ilo > last ? last : ilo);
        ihi = ihi < 0 ? 0 : (ihi > last ? last : ihi);
        __syncthreads();
        KRR_DIAG_T0(t0);
        sp.cnt = cnt;
        sp.bad = 0;
        uint64_t mn = lo, mx = hi;  // after a shrink the window is tight around the keys
        if (shrinks == 0) sp.buf_minmax(mn, mx);
        ++shrinks;
        uint64_t nl = lo, nh = hi;
#if KRR_WSEL_BINS
        // The bounds need not be the keys at ranks ilo / ihi: any window holding them
        // works.  One 256-bin histogram of the buffer gives the edges of the bins that
        // hold them (a bin is ~cnt / 256 keys wider than needed on each side).
        {
            const uint32_t sh = sp.hist_range(mn, mx);
            uint32_t keep_hi_side = cnt, keep_lo_side = 0;  // keys >= nl, keys > nh
            if (ilo > 0) {
                const BinHit bl = find_bin_desc(sp.H, (uint32_t)(cnt - ilo), 0u, lane);
                nl = uni64(mn + ((uint64_t)bl.b << sh));
                keep_hi_side = bl.above + bl.cnt;
            }
            if (ihi < last) {
                const BinHit bh = find_bin_desc(sp.H, (uint32_t)(cnt - ihi), 0u, lane);
                const uint64_t w1 = (1ull << sh) - 1, blo = mn + ((uint64_t)bh.b << sh);
                nh = uni64(mx - blo <= w1 ? mx : blo + w1);
                keep_lo_side = bh.above;
            }
            __syncthreads();
            // crowded bins leave too much: exact bounds instead.  EXPORT windows are also
            // held to a few times the ranks they need: a bin can span most of the data
            // when the keys straddle the sign (negatives and positives in one histogram),
            // and such a window would overflow on the next chunk and fail the series.
            uint32_t keep_limit = cap - kChunkElems / 2;
            if constexpr (EXPORT) {
                const uint32_t need = 2u * (uint32_t)(ihi - ilo + 1) + 256u;
                keep_limit = need < keep_limit ? need : keep_limit;
            }
            // ... and so is a window that keeps so large a share of the keys that the next
            // two chunks would overflow it (coarse bins: zeros in the data put the
            // histogram's range over many octaves, one bin over several of them)
            const uint64_t keep = keep_hi_side - keep_lo_side;
            if (keep > keep_limit || keep * (uint64_t)(cnt + 2 * kChunkElems) > (uint64_t)cap * cnt) {
                nl = ilo > 0 ? sp.kth_largest((uint32_t)(cnt - ilo), mn, mx) : lo;
                nh = ihi < last ? sp.kth_largest((uint32_t)(cnt - ihi), mn, mx) : hi;
            }
        }
#else
        // the R-th largest (1-based) is ascending index cnt - R
        nl = ilo > 0 ? sp.kth_largest((uint32_t)(cnt - ilo), mn, mx) : lo;
        nh = ihi < last ? sp.kth_largest((uint32_t)(cnt - ihi), mn, mx) : hi;
#endif
        __syncthreads();
#ifdef KRR_WEXP_DEBUG
        dbg(1, seen, below, cnt, ((uint64_t)ilo << 32) | (uint64_t)ihi);
        dbg(2, lo, hi, nl, nh);
#endif
        if (sp.bad || nl > nh) {
            fail = 1;
            return;
        }
        filter_window(nl, nh);
        set_window(nl, nh);
#ifdef KRR_DIAG
        diag[D_COMPACT] += __builtin_amdgcn_s_memtime() - t0;
        diag[D_NCOMPACT] += 1;
#endif
    }

    // EXPORT: the buffer holds one distinct key v (and none below lo): the window becomes
    // [v, v] (counted, not stored); later keys above v fall outside it.  Exact counts
    // decide at the merge whether the target really is v.
    __device__ __forceinline__ bool point_rescue() {
        if (cnt == 0) return false;
        __syncthreads();
        uint64_t mn, mx;
        sp.cnt = cnt;
        sp.buf_minmax(mn, mx);
        if (mn != mx) return false;
        set_window(mn, mn);
        return true;
    }

    // EXPORT: commit a chunk against a point window [lo, lo] (after point_rescue).
    __device__ __forceinline__ void point_chunk(const double2 (&c)[kUnroll]) {
        uint32_t bl = 0, nnc = 0, eq = 0;
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const uint64_t x = dbits(slot_val(c, j));
            const bool nan = is_nan_bits(x);
            const uint64_t key = okey(x);
            nnc += popc64(ballot(nan));
            bl += popc64(ballot(!nan && key < lo));
            eq += popc64(ballot(!nan && key == lo));
        }
        below_extra += bl;
        if constexpr (LANE_COUNTS) nan_l += lane == 0 ? nnc : 0u;
        else nan_u += nnc;
        cnt = uni32(cnt + eq);
        seen += kChunkElems;
    }

    // EXPORT, after the stream: narrow the window to the ranks the GLOBAL percentile can
    // need (unseen = the other slices only) with exact key bounds, so that the row the
    // series' owner receives holds at most key_cap keys.
    __device__ __forceinline__ void export_shrink(uint32_t key_cap) {
        if (point || cnt <= key_cap) return;
        const uint64_t nanc = nan_total();
        const uint64_t below = below_total();
        const uint64_t S = seen - nanc;
        const double qq = (double)p_num / (100.0 * (double)p_den);
        const double Sd = (double)S, U = ext_u;
        const double c = qq * (Sd - 1.0);
        const double sig = (S > 0 && U > 0.0) ? sqrt(qq * (1.0 - qq) * Sd * U / (Sd + U)) : 0.0;
        const double w = KRR_WEXP_Z * sig + 4.0;
        const int64_t last = (int64_t)cnt - 1;
        int64_t ilo = (int64_t)floor(c - w) - (int64_t)below;
        int64_t ihi = (int64_t)ceil(c + w) + 1 - (int64_t)below;
        ilo = ilo < 0 ? 0 : (ilo > last ? last : ilo);
        ihi = ihi < 0 ? 0 : (ihi > last ? last : ihi);
        __syncthreads();
        sp.cnt = cnt;
        sp.bad = 0;
        uint64_t mn = lo, mx = hi;
        if (shrinks == 0) sp.buf_minmax(mn, mx);
        ++shrinks;
        const uint64_t nl = ilo > 0 ? sp.kth_largest((uint32_t)(cnt - ilo), mn, mx) : lo;
        const uint64_t nh = ihi < last ? sp.kth_largest((uint32_t)(cnt - ihi), mn, mx) : hi;
        __syncthreads();
        if (sp.bad || nl > nh) {
            fail = 1;
            return;
        }
        filter_window(nl, nh);
        set_window(nl, nh);
    }
};

// One CPU segment by wselect.  A miss goes to hselect: inline (INLINE_FALLBACK,
// the long-segment kernels, whose register budget holds both paths and whose
// rare misses then overlap the other waves' work) or through the miss list that
// k_hselect_list finishes after the launch (the 3-waves-per-SIMD kernels).
template <bool INLINE_FALLBACK>
__device__ __forceinline__ void wselect_segment(const SelectArgs& A, int64_t s, unsigned char* smem, int lane) {
    const int64_t beg = A.offs[s], end = A.offs[s + 1];
    const int64_t L = end - beg;
    WindowProc<INLINE_FALLBACK> W;
    W.buf = reinterpret_cast<uint64_t*>(smem + kSelectLdsFixed);
    W.sp.buf = W.buf;
    W.sp.H = reinterpret_cast<uint32_t*>(smem);
    W.sp.small = reinterpret_cast<uint64_t*>(smem + 1024);
    W.sp.lane = lane;
    W.sp.flip = 0;
    W.sp.cnt = 0;
    W.sp.bad = 0;
    W.lane = lane;
    W.cap = A.wcap;
    W.shrinks = 0;
    W.cnt = 0;
    W.below_u = W.nan_u = 0;
    W.below_l = W.nan_l = W.negnan_l = 0;
    W.below_extra = 0;
    W.seen = 0;
    W.L = L;
    W.p_num = A.p_num;
    W.p_den = A.p_den;
    W.fail = 0;
    W.set_window(kKeyNegInf, kKeyPosInf);
#ifdef KRR_DIAG
    for (int d = 0; d < D_WORDS; ++d) W.diag[d] = 0;
    KRR_DIAG_T0(t_begin);
#endif
    // opaque bounds (see select_segment): no address set-up hoisted across the pass
    int64_t b = beg, e = end;
    asm volatile("" : "+s"(b), "+s"(e));
    const uint32_t pad =
        stream_segment<true, WindowProc<INLINE_FALLBACK>, INLINE_FALLBACK ? KRR_WSEL_LONG_DEPTH : KRR_ONE_SITE_DEPTH>(
            A.vals, b, e, W, lane);
    __syncthreads();
    const uint64_t nnan = W.nan_total() - pad;
    const uint64_t n = A.gaps ? (uint64_t)L - nnan : (uint64_t)L;
    uint32_t flags = 0;
    double result = bitsd(kQuietNaN);
    bool done = false;
#ifdef KRR_DIAG
    KRR_DIAG_T0(t_final);
#endif
    if (W.fail) {
        // a failed window stopped counting part-way: nothing above is meaningful
    } else if (n == 0) {
        flags = KRR_FLAG_EMPTY;
        done = true;
    } else if (nnan && !A.gaps) {
        flags = KRR_FLAG_NAN;
        done = true;
    } else {
        const Ranks R = ranks_for(A, n);
        const uint64_t below = W.below_total();
        if (below <= (uint64_t)R.r0 && (uint64_t)R.r1 < below + W.cnt) {
            uint64_t k0, k1;
            if (W.point) {
                k0 = k1 = W.lo;
            } else {
                W.sp.cnt = W.cnt;
                W.sp.bad = 0;
                uint64_t mn = W.lo, mx = W.hi;  // tight after a shrink
                if (W.shrinks == 0) W.sp.buf_minmax(mn, mx);
                const uint32_t Rt = (uint32_t)(W.cnt - ((uint64_t)R.r0 - below));  // R-th largest = rank r0
                if (R.r1 != R.r0) {
                    W.sp.kth_pair(Rt, -1, mn, mx, k0, k1);
                } else {
                    k0 = k1 = W.sp.kth_largest(Rt, mn, mx);
                }
            }
            if (!W.sp.bad) {
                result = finish_value(A, R, k0, k1, beg, end, lane);
                done = true;
            }
        }
    }
#ifdef KRR_DIAG
    {
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        W.diag[D_TOTAL] = t_end - t_begin;
        W.diag[D_FINAL] = t_end - t_final;
        W.diag[D_NFALLBACK] = done ? 0ull : 1ull;
        W.diag[D_INSERTED] = W.cnt;
        if (lane == 0 && g_diag)
            for (int d = 0; d < D_WORDS; ++d) g_diag[(size_t)s * D_WORDS + d] = W.diag[d];
    }
#endif
    __syncthreads();
    if (!done) {
        if (lane == 0 && A.stats) atomicAdd(A.stats, 1ull);
        if constexpr (INLINE_FALLBACK) {
            hselect_segment(A, s, smem, lane);
        } else if (lane == 0) {
            A.fail_list[atomicAdd(A.fail_count, 1u)] = s;  // finished by k_hselect_list
        }
        return;
    }
    write_result(A, s, result, n, flags, lane);
    __syncthreads();
}

template <bool LONG>
__device__ __forceinline__ void mid_select_segment(const SelectArgs& A, int64_t s, unsigned char* smem, int lane) {
    if constexpr (KRR_WSEL) wselect_segment<LONG>(A, s, smem, lane);
    else hselect_segment(A, s, smem, lane);
}

// The segments wselect missed, by hselect (launched right after the window kernel
// on the same stream).  With no misses every workgroup reads the count and exits.
// Nothing here resets the list: launches alternate between two counters, and the
// window kernel of launch k + 1 zeroes launch k's (this pass has finished by then:
// same stream, or the ctx's event when k + 1 comes on another stream), which launch
// k + 2 counts into — no extra memset or completion counter per launch.
__global__ __launch_bounds__(64, KRR_HSEL_WAVES_PER_SIMD) void k_hselect_list(SelectArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const unsigned int n = __builtin_nontemporal_load(A.fail_count);
    for (unsigned int i = blockIdx.x; i < n; i += gridDim.x) hselect_segment(A, A.fail_list[i], smem, threadIdx.x);
}

// k_select<SEL_SINGLE>: every segment in one pass (the launch's longest segment fits
// A.cap keys); k_select<SEL_WINDOW / SEL_WINDOW_LONG>: every segment through the
// window select (hselect when KRR_WSEL is 0).  Separate kernels keep each one's
// register allocation to its own path; the two window kernels differ only in their
// occupancy bound (long segments: a larger window at 2 waves per SIMD).
enum { SEL_SINGLE = 0, SEL_WINDOW = 1, SEL_WINDOW_LONG = 2 };
constexpr int window_waves(bool longseg) {
    return !KRR_WSEL ? KRR_HSEL_WAVES_PER_SIMD : (longseg ? KRR_HSEL_WAVES_PER_SIMD : KRR_WSEL_WAVES_PER_SIMD);
}
template <int KIND>
__global__ __launch_bounds__(64, KIND == SEL_SINGLE ? KRR_SELECT_WAVES_PER_SIMD : window_waves(KIND == SEL_WINDOW_LONG))
void k_select(SelectArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if (KIND != SEL_SINGLE && A.fail_reset && blockIdx.x == 0 && threadIdx.x == 0) *A.fail_reset = 0;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        if constexpr (KIND != SEL_SINGLE) mid_select_segment<KIND == SEL_WINDOW_LONG>(A, xcd_item(s, A.S, A.remap), smem, threadIdx.x);
        else select_segment(A, xcd_item(s, A.S, A.remap), smem, threadIdx.x);
    }
}

// ---------------------------------------------------------------------------
// Time-sharded exact percentiles in one HBM pass (config 5; include/krr_amd.h
// "window export").  Each rank streams its time slice of every series once through
// the window select, with the other slices' slots counted as unseen (EXPORT), and
// exports the window: its bounds, the exact count of present samples below it and
// its keys.  The owner of a series intersects the ranks' windows; exact counts
// decide whether the needed ranks lie inside, and if so they are selected there.
// ---------------------------------------------------------------------------
struct WindowExportArgs {
    SelectArgs A;         // vals, offs, S, mode, gaps, p, q, wcap (outputs unused)
    double ext;           // slots of each series held by the other slices
    uint32_t key_cap;     // keys per row
    krr_window_hdr* hdr;  // [S]
    uint64_t* keys;       // [S][key_cap]
};

template <bool LONG>
__device__ __forceinline__ void window_export_segment(const WindowExportArgs& X, int64_t s, unsigned char* smem,
                                                      int lane) {
    const SelectArgs& A = X.A;
    const int64_t beg = A.offs[s], end = A.offs[s + 1];
    const int64_t L = end - beg;
    WindowProc<LONG, true> W;
    W.buf = reinterpret_cast<uint64_t*>(smem + kSelectLdsFixed);
    W.sp.buf = W.buf;
    W.sp.H = reinterpret_cast<uint32_t*>(smem);
    W.sp.small = reinterpret_cast<uint64_t*>(smem + 1024);
    W.sp.lane = lane;
    W.sp.flip = 0;
    W.sp.cnt = 0;
    W.sp.bad = 0;
    W.lane = lane;
    W.cap = A.wcap;
    W.shrinks = 0;
    W.cnt = 0;
    W.below_u = W.nan_u = 0;
    W.below_l = W.nan_l = W.negnan_l = 0;
    W.below_extra = 0;
    W.seen = 0;
    W.L = L;
    W.p_num = A.p_num;
    W.p_den = A.p_den;
    W.fail = 0;
    W.ext_u = X.ext;
    W.set_window(kKeyNegInf, kKeyPosInf);
    int64_t b = (int64_t)uni64((uint64_t)beg), e = (int64_t)uni64((uint64_t)end);
    asm volatile("" : "+s"(b), "+s"(e));
    const uint32_t pad = stream_segment<true, WindowProc<LONG, true>, LONG ? KRR_WSEL_LONG_DEPTH : KRR_ONE_SITE_DEPTH>(
        A.vals, b, e, W, lane);
    __syncthreads();
    // a failed window stopped counting part-way: its counts mean nothing (no NaN flag)
    const uint64_t nnan = W.fail ? 0 : W.nan_total() - pad;
    const uint64_t n = A.gaps ? (uint64_t)L - nnan : (uint64_t)L;
    const bool has_nan = nnan && !A.gaps;
    if (!W.fail && n > 0 && !has_nan) W.export_shrink(X.key_cap);
    uint32_t flags = 0;
    if (W.fail || (!W.point && W.cnt > X.key_cap)) flags |= KRR_WIN_FAIL;
    if (has_nan) flags |= KRR_FLAG_NAN;
    if (W.point) flags |= KRR_WIN_POINT;
    if (!(flags & (KRR_WIN_FAIL | KRR_WIN_POINT))) {
        uint64_t* row = X.keys + (size_t)s * X.key_cap;
        for (uint32_t i = lane; i < W.cnt; i += kWave) row[i] = W.buf[i];
    }
    const uint64_t below = W.below_total();  // a wave reduction (LANE_COUNTS): every lane takes part
    if (lane == 0) {
        krr_window_hdr h;
        h.lo = W.lo;
        h.hi = W.hi;
        h.below = (int64_t)below;
        h.n = (int64_t)n;
        h.cnt = W.cnt;
        h.flags = flags;
        X.hdr[s] = h;
    }
    __syncthreads();
}

template <bool LONG>
__global__ __launch_bounds__(64, window_waves(LONG)) void k_window_export(WindowExportArgs X) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    for (int64_t s = blockIdx.x; s < X.A.S; s += gridDim.x) window_export_segment<LONG>(X, xcd_item(s, X.A.S, X.A.remap), smem, threadIdx.x);
}

struct OpAdd64 {
    __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
};
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
    return lane_bcast64(wave_scan64(x, 0ull, OpAdd64{}), kWave - 1);
}

struct WindowMergeArgs {
    SelectArgs A;                // mode, p, q; out_v / out_n / out_f; S = series
    int32_t slices;
    int64_t stride;              // header / row index of slice j of series i: j * stride + i
    const krr_window_hdr* hdr;
    const uint64_t* keys;
    int64_t key_cap;
    unsigned int* miss_count;    // may be null
};

// One wave per series: the slices' windows -> the exact result, or a miss.
__global__ __launch_bounds__(64) void k_window_merge(WindowMergeArgs M) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const SelectArgs& A = M.A;
    uint64_t* buf = reinterpret_cast<uint64_t*>(smem + kSelectLdsFixed);
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const bool has = lane < M.slices;
        krr_window_hdr h;
        if (has) {
            h = M.hdr[(int64_t)lane * M.stride + s];
        } else {
            h.lo = 0;
            h.hi = ~0ull;
            h.below = h.n = 0;
            h.cnt = h.flags = 0;
        }
        const uint64_t n = wave_sum_u64((uint64_t)h.n);
        const uint64_t Lk = wave_max_u64(h.lo), Hk = wave_min_u64(h.hi);
        const bool any_nan = ballot((h.flags & KRR_FLAG_NAN) != 0) != 0;
        // a row longer than key_cap cannot come from krr_window_export: no window
        const bool any_fail =
            ballot((h.flags & KRR_WIN_FAIL) != 0 || (!(h.flags & KRR_WIN_POINT) && h.cnt > M.key_cap)) != 0;
        uint32_t flags = 0;
        double result = bitsd(kQuietNaN);
        bool miss = false;
        if (any_nan) {
            flags = KRR_FLAG_NAN;  // a NaN sample (compact layout): NaN, as the whole-series select says
        } else if (n == 0) {
            flags = KRR_FLAG_EMPTY;
        } else if (!rule_covers((int64_t)n, A.ktab, A.ktab_len)) {
            flags = KRR_FLAG_CAPACITY;  // the caller's k_table stops short of the merged count
        } else if (any_fail || Lk > Hk) {
            miss = true;
        } else {
            const Ranks R = ranks_for(A, n);
            uint64_t cb = wave_sum_u64((uint64_t)h.below);  // present samples below Lk, all slices
            uint32_t inr = 0, inr_point = 0;
#pragma unroll 1
            for (int j = 0; j < M.slices; ++j) {
                const uint64_t loj = lane_bcast64(h.lo, j);
                const uint32_t cj = lane_bcast32(h.cnt, j), fj = lane_bcast32(h.flags, j);
                if (fj & KRR_WIN_POINT) {  // cj copies of loj (Lk >= loj >= Hk when it is in range)
                    if (loj < Lk) cb += cj;
                    else if (loj <= Hk) inr_point += cj;
                    continue;
                }
                const uint64_t* row = M.keys + ((int64_t)j * M.stride + s) * M.key_cap;
                uint32_t lt = 0;
                for (uint32_t base = 0; base < cj; base += kWave) {
                    const uint32_t i = base + lane;
                    const bool v = i < cj;
                    const uint64_t k = v ? row[i] : 0ull;
                    lt += popc64(ballot(v && k < Lk));
                    const bool in = v && k >= Lk && k <= Hk;
                    const uint64_t m = ballot(in);
                    if (in) buf[inr + lane_prefix(m)] = k;
                    inr += popc64(m);
                }
                cb += lt;
            }
            __syncthreads();
            const uint64_t tot = (uint64_t)inr + inr_point;
            if (cb <= (uint64_t)R.r0 && (uint64_t)R.r1 < cb + tot) {
                uint64_t k0 = Lk, k1 = Lk;
                bool bad = false;
                if (Lk != Hk && inr_point == 0) {
                    SelectProc sp;
                    sp.buf = buf;
                    sp.H = reinterpret_cast<uint32_t*>(smem);
                    sp.small = reinterpret_cast<uint64_t*>(smem + 1024);
                    sp.lane = lane;
                    sp.flip = 0;
                    sp.cnt = inr;
                    sp.bad = 0;
                    uint64_t mn, mx;
                    sp.buf_minmax(mn, mx);
                    const uint32_t Rt = (uint32_t)(inr - ((uint64_t)R.r0 - cb));  // R-th largest = rank r0
                    if (R.r1 != R.r0) sp.kth_pair(Rt, -1, mn, mx, k0, k1);
                    else k0 = k1 = sp.kth_largest(Rt, mn, mx);
                    bad = sp.bad != 0;
                }
                const double a = bitsd(okey_inv(k0));
                if (bad) {
                    miss = true;
                } else if (A.mode == KRR_PCT_SORTED_LOWER) {
                    // a zero's sign is the (r0 - #negatives)-th zero's in time order (sorted()
                    // is stable): not in the windows, so the whole series decides it
                    if (is_zero_bits(dbits(a))) miss = true;
                    else result = a;
                } else {
                    result = np_lerp(a, R.r1 != R.r0 ? bitsd(okey_inv(k1)) : a, R.gamma);
                }
            } else {
                miss = true;
            }
        }
        if (miss) {
            flags = KRR_FLAG_WINDOW_MISS;
            result = bitsd(kQuietNaN);
        }
        if (lane == 0) {
            A.out_v[s] = result;
            A.out_n[s] = (int64_t)n;
            A.out_f[s] = flags;
            if (miss && M.miss_count) atomicAdd(M.miss_count, 1u);
        }
        __syncthreads();
    }
}

// --------------------------- REF_INDEX ------------------------------------
struct NanCountProc {
    uint32_t nn;
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) nn += popc64(ballot(__builtin_isnan(slot_val(c, j))));
    }
};

constexpr int kRefBlock = 16;  // 64-slot blocks per REF_INDEX locate step

struct RefArgs {
    const double* vals;
    const int64_t* offs;
    int64_t S;
    int64_t p_num, p_den;
    const int64_t* ktab;  // krr_percentile_params.k_table (null: the exact floor)
    int64_t ktab_len;
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
    int64_t* rec = nullptr;  // optional records, CPU half
};

// NaN-gapped layout: the k-th PRESENT sample in position order.
// ONE_SITE: the fused kernel's register budget (KRR_SELECT_WAVES_PER_SIMD) only fits
// the one-site streaming loop; the standalone kernel uses the depth-2 loop.
template <bool ONE_SITE>
__device__ __forceinline__ void refindex_gaps_segment(const RefArgs& A, int64_t s, int lane) {
    {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        NanCountProc C{0};
        C.nn -= stream_segment<ONE_SITE>(A.vals, beg, end, C, lane);
        const uint64_t n = (uint64_t)(end - beg) - C.nn;
        double result = bitsd(kQuietNaN);
        uint32_t flags = 0;
        if (n == 0) {
            flags = KRR_FLAG_EMPTY;
        } else {
            const uint64_t k = (uint64_t)rule_rank((int64_t)n, A.p_num, A.p_den, A.ktab, A.ktab_len);
            // walk from the nearer end in blocks of 16 x 64 slots whose loads are all
            // in flight at once (one HBM round trip per 1,024 slots, not per 64)
            const bool back = k >= n / 2;
            const uint64_t want = back ? n - 1 - k : k;  // present samples to skip
            const int64_t step = back ? -1 : 1;
            uint64_t run = 0;
            uint64_t found = kQuietNaN;
            bool done = false;
            for (int64_t pos = back ? end - 1 : beg; !done && (back ? pos >= beg : pos < end);
                 pos += step * kRefBlock * kWave) {
                uint64_t u[kRefBlock];
#pragma unroll
                for (int b = 0; b < kRefBlock; ++b) {
                    const int64_t i = pos + step * (b * kWave + lane);
                    u[b] = (i >= beg && i < end) ? dbits(A.vals[i]) : kQuietNaN;
                }
#pragma unroll
                for (int b = 0; b < kRefBlock; ++b) {
                    if (done) break;
                    const bool p = !is_nan_bits(u[b]);
                    const uint64_t m = ballot(p);
                    const uint32_t c = popc64(m);
                    if (run + c > want) {
                        const uint64_t sel = ballot(p && lane_prefix(m) == (uint32_t)(want - run));
                        found = lane_bcast64(u[b], __ffsll((long long)sel) - 1);
                        done = true;
                    }
                    run += c;
                }
            }
            result = bitsd(found);
        }
        if (lane == 0) {
            A.out_v[s] = result;
            A.out_n[s] = (int64_t)n;
            A.out_f[s] = flags;
            put_record(A.rec, s, 0, result, n, flags);
        }
    }
}

__global__ __launch_bounds__(64) void k_refindex_gaps(RefArgs A) {
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) refindex_gaps_segment<false>(A, xcd_item(s, A.S, 1), threadIdx.x);
}

// Compact CSR (every slot is a sample, NaN included): X[k] is one gather.
__global__ __launch_bounds__(256) void k_refindex_dense(RefArgs A) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= A.S) return;
    const int64_t beg = A.offs[s], end = A.offs[s + 1];
    const int64_t n = end - beg;
    if (n <= 0) {
        A.out_v[s] = bitsd(kQuietNaN);
        A.out_n[s] = 0;
        A.out_f[s] = KRR_FLAG_EMPTY;
        return;
    }
    const int64_t k = rule_rank(n, A.p_num, A.p_den, A.ktab, A.ktab_len);
    A.out_v[s] = A.vals[beg + k];
    A.out_n[s] = n;
    A.out_f[s] = 0;
}

// ------------------------------- MAX --------------------------------------
// v_max_f64 returns the non-NaN operand, so NaN slots (gaps or padding) drop
// out of the running max for free; one VALU per sample plus one NaN test.
struct MaxProc {
    double mx;
    uint32_t nn;
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const double d = slot_val(c, j);
            mx = fmax(mx, d);
            nn += popc64(ballot(__builtin_isnan(d)));
        }
    }
};

struct OpMaxF64Bits {  // fmax on f64 bit patterns: the non-NaN operand wins
    __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return dbits(fmax(bitsd(a), bitsd(b))); }
};
__device__ __forceinline__ double wave_max_f64(double x) {
    return bitsd(lane_bcast64(wave_scan64(dbits(x), kQuietNaN, OpMaxF64Bits{}), kWave - 1));
}

struct MaxArgs {
    const double* vals;
    const int64_t* offs;
    int64_t S;
    int32_t gaps;
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
    int64_t* rec = nullptr;  // optional records, memory half
    // optional forward copy done by the fused launch (krr_simple_run_forward): fwd_units
    // 16-byte units from fwd_src to fwd_dst (device or mapped page-locked host memory),
    // split over fwd_items work items that precede the segments
    const double2* fwd_src = nullptr;
    double2* fwd_dst = nullptr;
    int64_t fwd_units = 0;
    int64_t fwd_items = 0;
    int32_t remap = 1;  // xcd_item: per-XCD segment ranges (KRR_XCD_REMAP_MAXLEN)
};

template <class Streamer>
__device__ __forceinline__ void max_segment_with(const MaxArgs& A, int64_t s, int lane, Streamer stream) {
    {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        MaxProc M{__builtin_nan(""), 0u};
        M.nn -= stream(M);
        const uint64_t L = (uint64_t)(end - beg);
        const uint64_t n = A.gaps ? L - M.nn : L;
        const double mx = wave_max_f64(M.mx);
        double result = bitsd(kQuietNaN);
        uint32_t flags = 0;
        if (n == 0) {
            flags = KRR_FLAG_EMPTY;
        } else if (M.nn && !A.gaps) {
            flags = KRR_FLAG_NAN;
        } else {
            uint64_t bits = uni64(dbits(mx));
            // Python max() keeps the FIRST maximal element; only +-0 compare equal
            // with different bits.
            if (is_zero_bits(bits)) bits = nth_zero_bits(A.vals, beg, end, 0, lane);
            result = bitsd(bits);
        }
        if (lane == 0) {
            A.out_v[s] = result;
            A.out_n[s] = (int64_t)n;
            A.out_f[s] = flags;
            put_record(A.rec, s, 1, result, n, flags);
        }
    }
}

template <bool ONE_SITE>
__device__ __forceinline__ void max_segment(const MaxArgs& A, int64_t s, int lane) {
    const int64_t beg = A.offs[s], end = A.offs[s + 1];
    max_segment_with(A, s, lane, [&](MaxProc& M) { return stream_segment<ONE_SITE>(A.vals, beg, end, M, lane); });
}

__global__ __launch_bounds__(64) void k_max(MaxArgs A) {
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) max_segment<false>(A, xcd_item(s, A.S, A.remap), threadIdx.x);
}

// ------------------------------ FUSED --------------------------------------
// SimpleStrategy.run for the whole fleet in ONE launch: work item b < S_cpu is
// CPU segment b (select or REF_INDEX-on-gaps), the rest are memory segments.
// The dispatcher hands out blocks in order, so the shorter memory-max blocks
// fill CUs as the CPU blocks drain instead of leaving a partly idle last round
// per kernel; one launch is also one roofline for the whole step.
enum { CPU_SELECT = 0, CPU_REF_GAPS = 1, CPU_HSELECT = 2, CPU_HSELECT_LONG = 3 };  // HSELECT: window select

// One forward work item: a contiguous kFwdItemUnits-unit share of the copy, 16 B per
// lane per store (posted writes when the destination is host memory).
constexpr int64_t kFwdItemUnits = 4096;  // 64 KiB per item
__device__ __forceinline__ void forward_item(const MaxArgs& M, int64_t i, int lane) {
    const int64_t a = i * kFwdItemUnits;
    const int64_t e = a + kFwdItemUnits < M.fwd_units ? a + kFwdItemUnits : M.fwd_units;
    // not unrolled: an unrolled copy keeps many 16-B loads in flight and lifts the fused
    // kernel's VGPR count (and so its occupancy) for every launch, forward or not
#pragma unroll 1
    for (int64_t u = a + lane; u < e; u += kWave) M.fwd_dst[u] = M.fwd_src[u];
}

// FWD: the launch also runs a forward copy (krr_simple_run_forward) as its first items.  A
// template parameter, not a runtime branch: the forward arguments would otherwise take
// scalar registers in every launch (SGPR spills into VGPR lanes: the CPU_SELECT kernel went
// from 126 to 131 VGPRs, the short window kernel from 129 to 133).
template <int CPU_KIND, bool FWD = false>
__global__ __launch_bounds__(64, CPU_KIND == CPU_HSELECT ? window_waves(false)
                                : CPU_KIND == CPU_HSELECT_LONG ? window_waves(true)
                                                               : KRR_SELECT_WAVES_PER_SIMD) void k_simple(SelectArgs A, RefArgs R, MaxArgs M) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int64_t S_cpu = CPU_KIND == CPU_REF_GAPS ? R.S : A.S;
    const int64_t F = FWD ? M.fwd_items : 0;  // forward-copy items first: short, done while the stream ramps up
    const int64_t total = F + S_cpu + M.S;
    constexpr bool kWindow = CPU_KIND == CPU_HSELECT || CPU_KIND == CPU_HSELECT_LONG;
    if (kWindow && A.fail_reset && blockIdx.x == 0 && threadIdx.x == 0) *A.fail_reset = 0;
    for (int64_t bb = blockIdx.x; bb < total; bb += gridDim.x) {
        if constexpr (FWD) {
            if (bb < F) {
                forward_item(M, bb, threadIdx.x);
                continue;
            }
        }
        const int64_t b = bb - F;  // F is a multiple of 8: blocks keep their XCD's eighth
        // remap within each resource's half, so the CPU items still all precede
        // the memory items in dispatch order
        if (b < S_cpu) {
            const int64_t s = xcd_item(b, S_cpu, A.remap);
            if constexpr (CPU_KIND == CPU_SELECT) select_segment(A, s, smem, threadIdx.x);
            else if constexpr (kWindow) mid_select_segment<CPU_KIND == CPU_HSELECT_LONG>(A, s, smem, threadIdx.x);
            else refindex_gaps_segment<true>(R, s, threadIdx.x);
        } else {
            max_segment<true>(M, xcd_item(b - S_cpu, M.S, M.remap), threadIdx.x);
        }
    }
}

// 32-byte result records for the multi-GPU gather (int64[4] per object):
// cpu bits, mem bits, cpu count | cpu flags << 48, mem count | mem flags << 48.
__global__ __launch_bounds__(256) void k_pack_records(int64_t S, const double* __restrict__ cv,
                                                      const int64_t* __restrict__ cn,
                                                      const uint32_t* __restrict__ cf,
                                                      const double* __restrict__ mv,
                                                      const int64_t* __restrict__ mn,
                                                      const uint32_t* __restrict__ mf,
                                                      int64_t* __restrict__ rec) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    longlong2 a, b;
    a.x = (long long)dbits(cv[s]);
    a.y = (long long)dbits(mv[s]);
    b.x = (long long)((uint64_t)cn[s] | ((uint64_t)cf[s] << 48));
    b.y = (long long)((uint64_t)mn[s] | ((uint64_t)mf[s] << 48));
    reinterpret_cast<longlong2*>(rec)[2 * s] = a;
    reinterpret_cast<longlong2*>(rec)[2 * s + 1] = b;
}

// Largest segment length (for planning when the caller did not pass it).
__global__ void k_maxlen(const int64_t* __restrict__ offs, int64_t S, unsigned long long* out) {
    uint64_t m = 0;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < S;
         s += (int64_t)gridDim.x * blockDim.x) {
        const int64_t L = offs[s + 1] - offs[s];
        m = (uint64_t)L > m ? (uint64_t)L : m;
    }
    m = wave_max_u64(m);
    if ((threadIdx.x & 63) == 0) atomicMax(out, (unsigned long long)m);
}

// ------------------------------ SKETCH -------------------------------------
// Mergeable log-linear histogram sketch (config 5: series too long for one
// GPU's time window, time-sharded over ranks).  Bins are data-independent, so
// the sketches of a series' time slices on different ranks merge EXACTLY by
// adding counts (one RCCL reduce-scatter); min/max merge by min/max.
// Bin layout per segment (ascending value order), width = nbins + 4 words:
//   [0] negative  [1] +-0  [2] (0, 2^e_lo)  [3 .. 3+nbins) log-linear bins
//   [3+nbins] >= 2^(e_lo + octaves) (incl. +inf)
// bin i covers [2^E (1 + j 2^-m), 2^E (1 + (j+1) 2^-m)) with E = e_lo + (i >> m),
// j = i & (2^m - 1): relative bin width <= 2^-m.  The query interpolates
// linearly inside the bin holding the rank; its rank error is measured against
// the exact path (bench.py config 5), not assumed.
struct SketchGeom {
    uint32_t m, nbins, width, base;  // base = (e_lo + 1023) << m
    uint64_t low_bits;               // bits of 2^e_lo
    int32_t e_lo;
};

__host__ __device__ inline SketchGeom sketch_geom(const krr_sketch_params& p) {
    SketchGeom g;
    g.m = (uint32_t)p.mantissa_bits;
    g.nbins = (uint32_t)p.octaves << g.m;
    g.width = g.nbins + 4;
    g.e_lo = p.min_exponent;
    g.base = (uint32_t)(p.min_exponent + 1023) << g.m;
    g.low_bits = (uint64_t)(p.min_exponent + 1023) << 52;
    return g;
}

// Bin of a non-NaN sample (bit pattern x); ascending in value.
__device__ __forceinline__ uint32_t sketch_bin(const SketchGeom& g, uint64_t x) {
    const uint64_t mag = x & ~kSignBit;
    const uint32_t u = (uint32_t)(mag >> (52 - g.m)) - g.base;
    uint32_t bin = u < g.nbins ? 3u + u : (mag < g.low_bits ? 2u : 3u + g.nbins);
    bin = (x & kSignBit) ? 0u : bin;
    bin = mag == 0 ? 1u : bin;
    return bin;
}

struct SketchProc {
    uint32_t* h;
    SketchGeom g;
    uint32_t nan_l;
    double vmin, vmax;
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const double d = slot_val(c, j);
            const uint64_t x = dbits(d);
            const bool nan = __builtin_isnan(d);
            nan_l += nan ? 1u : 0u;
            vmin = fmin(vmin, d);
            vmax = fmax(vmax, d);
            const uint32_t bin = sketch_bin(g, x);
            if (!nan) atomicAdd(&h[bin], 1u);
            asm volatile("" ::: "memory");
        }
    }
};

struct OpMinF64Bits {  // fmin on f64 bit patterns: the non-NaN operand wins
    __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return dbits(fmin(bitsd(a), bitsd(b))); }
};

struct SketchBuildArgs {
    const double* vals;
    const int64_t* offs;
    int64_t S;
    int32_t gaps;
    SketchGeom g;
    uint32_t* counts;  // [S][width]
    double* vmin;
    double* vmax;
    uint32_t* flags;
};

__global__ __launch_bounds__(64) void k_sketch_build(SketchBuildArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* h = reinterpret_cast<uint32_t*>(smem);
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        for (uint32_t i = lane; i < A.g.width; i += kWave) h[i] = 0;
        __syncthreads();
        SketchProc P;
        P.h = h;
        P.g = A.g;
        P.nan_l = 0;
        P.vmin = bitsd(kQuietNaN);
        P.vmax = bitsd(kQuietNaN);
        const uint32_t pad = stream_segment<true>(A.vals, beg, end, P, lane);
        __syncthreads();
        const uint64_t nnan = wave_sum_u32(P.nan_l) - pad;
        const double mn = bitsd(lane_bcast64(wave_scan64(dbits(P.vmin), kQuietNaN, OpMinF64Bits{}), kWave - 1));
        const double mx = bitsd(lane_bcast64(wave_scan64(dbits(P.vmax), kQuietNaN, OpMaxF64Bits{}), kWave - 1));
        uint4* dst = reinterpret_cast<uint4*>(A.counts + (size_t)s * A.g.width);
        const uint4* src = reinterpret_cast<const uint4*>(h);
        for (uint32_t i = lane; i < A.g.width / 4; i += kWave) dst[i] = src[i];
        if (lane == 0) {
            A.vmin[s] = mn;
            A.vmax[s] = mx;
            A.flags[s] = (nnan && !A.gaps) ? KRR_FLAG_NAN : 0u;
        }
        __syncthreads();
    }
}

struct SketchQueryArgs {
    int64_t S;
    SketchGeom g;
    const uint32_t* counts;
    const double* vmin;
    const double* vmax;
    int32_t mode;
    int64_t p_num, p_den;
    double q;
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
    const int64_t* ktab = nullptr;  // krr_percentile_params.k_table
    int64_t ktab_len = 0;
};

// Value estimate of ascending rank r inside bin b holding c keys, `before` below.
__device__ __forceinline__ double sketch_value(const SketchGeom& g, uint32_t b, uint64_t r, uint64_t before, uint32_t c,
                                               double mn, double mx, uint64_t n, uint32_t& flags) {
    if (r == 0) return mn;
    if (r == n - 1) return mx;
    const double f = ((double)(r - before) + 0.5) / (double)c;
    double lo, hi;
    if (b == 1) return 0.0;
    if (b == 0) {  // negatives: [min, 0)
        lo = mn;
        hi = 0.0;
        flags |= KRR_FLAG_SKETCH_RANGE;
    } else if (b == 2) {  // (0, 2^e_lo)
        lo = 0.0;
        hi = ldexp(1.0, g.e_lo);
        flags |= KRR_FLAG_SKETCH_RANGE;
    } else if (b == 3 + g.nbins) {  // [2^(e_lo + octaves), max]
        lo = ldexp(1.0, g.e_lo + (int)(g.nbins >> g.m));
        hi = mx;
        flags |= KRR_FLAG_SKETCH_RANGE;
    } else {
        const uint32_t i = b - 3;
        const int E = g.e_lo + (int)(i >> g.m);
        const double j = (double)(i & ((1u << g.m) - 1u));
        const double step = ldexp(1.0, E - (int)g.m);
        lo = ldexp(1.0, E) + j * step;
        hi = lo + step;
    }
    double v = lo + f * (hi - lo);
    v = v < mn ? mn : v;
    v = v > mx ? mx : v;
    return v;
}

__global__ __launch_bounds__(64) void k_sketch_query(SketchQueryArgs A) {
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const uint32_t* h = A.counts + (size_t)s * A.g.width;
        const uint32_t W = A.g.width;
        const uint32_t per = (W + kWave - 1) / kWave;
        const uint32_t b0 = (uint32_t)lane * per;
        uint32_t t = 0;
        for (uint32_t j = 0; j < per; ++j) t += b0 + j < W ? h[b0 + j] : 0u;
        const uint32_t incl = wave_scan32(t, 0u, OpAdd32{});
        const uint64_t n = lane_bcast32(incl, kWave - 1);
        uint32_t flags = 0;
        double result = bitsd(kQuietNaN);
        if (n == 0) {
            flags = KRR_FLAG_EMPTY;
        } else {
            Ranks R;
            R.gamma = 0.0;
            if (A.mode == KRR_PCT_SORTED_LOWER) {
                R.r0 = R.r1 = rule_rank((int64_t)n, A.p_num, A.p_den, A.ktab, A.ktab_len);
                if (!rule_covers((int64_t)n, A.ktab, A.ktab_len)) flags |= KRR_FLAG_CAPACITY;
            } else {
                const double vidx = __dmul_rn((double)(n - 1), A.q);
                if (vidx >= (double)(n - 1)) {
                    R.r0 = R.r1 = (int64_t)n - 1;
                    R.gamma = __dsub_rn(vidx, -1.0);
                } else {
                    const double fl = floor(vidx);
                    R.r0 = (int64_t)fl;
                    R.r1 = R.r0 + 1;
                    R.gamma = __dsub_rn(vidx, fl);
                }
            }
            double v[2];
#pragma unroll 1
            for (int qi = 0; qi < 2; ++qi) {
                const uint64_t r = (uint64_t)(qi ? R.r1 : R.r0);
                const uint64_t m = ballot(r < incl);
                const int src = __ffsll((long long)m) - 1;
                uint64_t run = lane_bcast32(incl - t, src);
                // walk the source lane's bins (per <= a few dozen)
                const uint32_t sb = (uint32_t)src * per;
                uint32_t fb = sb, fc = 0;
                uint64_t fbefore = run;
                for (uint32_t j = 0; j < per && sb + j < W; ++j) {
                    const uint32_t c = h[sb + j];
                    if (r < run + c) {
                        fb = sb + j;
                        fc = c;
                        fbefore = run;
                        break;
                    }
                    run += c;
                }
                v[qi] = sketch_value(A.g, fb, r, fbefore, fc, A.vmin[s], A.vmax[s], n, flags);
            }
            result = A.mode == KRR_PCT_SORTED_LOWER ? v[0] : np_lerp(v[0], v[1], R.gamma);
        }
        if (lane == 0) {
            A.out_v[s] = result;
            A.out_n[s] = (int64_t)n;
            A.out_f[s] = flags;
        }
    }
}

// Rank interval of a value per segment: #present samples < v and <= v (for
// measuring a sketch answer's rank error against the data).
struct RankOfProc {
    double v;
    uint32_t lt, le;
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll]) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const double d = slot_val(c, j);
            lt += d < v ? 1u : 0u;  // false for NaN
            le += d <= v ? 1u : 0u;
        }
    }
};

__global__ __launch_bounds__(64) void k_rank_of(const double* __restrict__ vals, const int64_t* __restrict__ offs,
                                                int64_t S, const double* __restrict__ v, int64_t* out_lt,
                                                int64_t* out_le) {
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        RankOfProc P{v[s], 0u, 0u};
        stream_segment<false>(vals, offs[s], offs[s + 1], P, lane);
        const uint32_t lt = wave_sum_u32(P.lt), le = wave_sum_u32(P.le);
        if (lane == 0) {
            out_lt[s] = lt;
            out_le[s] = le;
        }
    }
}

}  // namespace krr
#include "krr_kll.h"
namespace krr {

// The k[s]-th present sample (0-based, position order; NaN slots absent when
// gaps) of each segment, k[s] < 0 -> skipped.  The time-sharded REF_INDEX: the
// rank whose slice holds global index k selects it locally.
__global__ __launch_bounds__(64) void k_select_present(const double* __restrict__ vals,
                                                       const int64_t* __restrict__ offs, int64_t S, int32_t gaps,
                                                       const int64_t* __restrict__ ks, double* out) {
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        const int64_t k = ks[s];
        if (k < 0) continue;
        const int64_t beg = offs[s], end = offs[s + 1];
        uint64_t found = kQuietNaN;
        if (!gaps) {
            if (beg + k < end) found = dbits(vals[beg + k]);
        } else {
            uint64_t run = 0;
            for (int64_t base = beg; base < end; base += kWave) {
                const int64_t i = base + lane;
                const bool in = i < end;
                const uint64_t u = in ? dbits(vals[i]) : kQuietNaN;
                const bool p = in && !is_nan_bits(u);
                const uint64_t m = ballot(p);
                const uint32_t c = popc64(m);
                if (run + c > (uint64_t)k) {
                    const uint64_t sel = ballot(p && lane_prefix(m) == (uint32_t)((uint64_t)k - run));
                    found = lane_bcast64(u, __ffsll((long long)sel) - 1);
                    break;
                }
                run += c;
            }
        }
        if (lane == 0) out[s] = bitsd(found);
    }
}

// Where a selected value sits in its segment: lt = #samples < v, eq = #samples == v
// (float ==: -0 == +0, NaN never), pos = the slot offset of the j-th sample equal to v in
// position order, j = rank - lt (rank >= 0: the stable-sort rank of sorted(X)[rank]) or 0
// (rank == -1: the first maximal element Python's max() keeps), -1 when there is none.
// rank < -1: segment skipped, outputs untouched.  The HistoryData path resolves with it
// the reference's own sample object (simple.py:29 max(data_), :36 data_[k] of a sorted
// list) for segments whose Decimals differ in representation from their float64 images.
__global__ __launch_bounds__(64) void k_locate(const double* __restrict__ vals, const int64_t* __restrict__ offs,
                                               int64_t S, const double* __restrict__ v,
                                               const int64_t* __restrict__ rank, int64_t* out_lt,
                                               int64_t* out_eq, int64_t* out_pos) {
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        const int64_t r = rank[s];
        if (r < -1) continue;
        const double x = v[s];
        const int64_t beg = offs[s], end = offs[s + 1];
        RankOfProc P{x, 0u, 0u};
        stream_segment<false>(vals, beg, end, P, lane);
        const int64_t lt = wave_sum_u32(P.lt), eq = (int64_t)wave_sum_u32(P.le) - lt;
        const int64_t j = r >= 0 ? r - lt : 0;
        int64_t pos = -1;
        if (j >= 0 && j < eq) {
            int64_t run = 0;
            for (int64_t base = beg; base < end; base += kWave) {
                const int64_t i = base + lane;
                const bool hit = i < end && vals[i] == x;
                const uint64_t m = ballot(hit);
                const uint32_t c = popc64(m);
                if (run + c > j) {
                    const uint64_t sel = ballot(hit && lane_prefix(m) == (uint32_t)(j - run));
                    pos = base + (__ffsll((long long)sel) - 1) - beg;
                    break;
                }
                run += c;
            }
        }
        if (lane == 0) {
            out_lt[s] = lt;
            out_eq[s] = eq;
            out_pos[s] = pos;
        }
    }
}

// --------------------- exact refinement of merged sketches ---------------------
// Sketch counts are exact, so the merged sketch of a time-sharded series tells
// exactly which bin holds each needed rank and how many samples lie below it.
// Every rank then collects its samples in that bin range (k_sketch_collect), the
// owner gathers them (RCCL all-to-all) and selects the exact order statistics
// inside the small collected list (k_sketch_refine): results identical to the
// single-window select, with one extra HBM pass.

// Locate rank r among a segment's W bins (lane holds bins [lane*per, lane*per+per)
// with inclusive prefix `incl` and own total t): bin index and samples below it.
__device__ __forceinline__ void sketch_find(const uint32_t* h, uint32_t W, uint32_t per, uint32_t t, uint32_t incl,
                                            uint64_t r, uint32_t& bin, uint64_t& before) {
    const uint64_t m = ballot(r < incl);
    const int src = __ffsll((long long)m) - 1;
    uint64_t run = lane_bcast32(incl - t, src);
    const uint32_t sb = (uint32_t)src * per;
    bin = sb;
    before = run;
    for (uint32_t j = 0; j < per && sb + j < W; ++j) {
        const uint32_t c = h[sb + j];
        if (r < run + c) {
            bin = sb + j;
            before = run;
            return;
        }
        run += c;
    }
}

struct SketchLocateArgs {
    int64_t S;
    SketchGeom g;
    const uint32_t* counts;
    int32_t mode;
    int64_t p_num, p_den;
    double q;
    krr_sketch_loc* out;
    const int64_t* ktab = nullptr;  // krr_percentile_params.k_table
    int64_t ktab_len = 0;
};

__global__ __launch_bounds__(64) void k_sketch_locate(SketchLocateArgs A) {
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const uint32_t* h = A.counts + (size_t)s * A.g.width;
        const uint32_t W = A.g.width;
        const uint32_t per = (W + kWave - 1) / kWave;
        const uint32_t b0 = (uint32_t)lane * per;
        uint32_t t = 0;
        for (uint32_t j = 0; j < per; ++j) t += b0 + j < W ? h[b0 + j] : 0u;
        const uint32_t incl = wave_scan32(t, 0u, OpAdd32{});
        const uint64_t n = lane_bcast32(incl, kWave - 1);
        krr_sketch_loc L;
        L.n = (int64_t)n;
        L.r0 = L.r1 = -1;
        L.before = 0;
        L.gamma = 0.0;
        L.bin_lo = 1;
        L.bin_hi = 0;  // empty range: nothing to collect
        L.flags = 0;
        L.mode = A.mode;
        if (n == 0) {
            L.flags = KRR_FLAG_EMPTY;
        } else {
            if (A.mode == KRR_PCT_SORTED_LOWER) {
                L.r0 = L.r1 = rule_rank((int64_t)n, A.p_num, A.p_den, A.ktab, A.ktab_len);
                if (!rule_covers((int64_t)n, A.ktab, A.ktab_len)) L.flags |= KRR_FLAG_CAPACITY;
            } else {  // numpy method="linear" (ranks_for)
                const double vidx = __dmul_rn((double)(n - 1), A.q);
                if (vidx >= (double)(n - 1)) {
                    L.r0 = L.r1 = (int64_t)n - 1;
                    L.gamma = __dsub_rn(vidx, -1.0);
                } else {
                    const double fl = floor(vidx);
                    L.r0 = (int64_t)fl;
                    L.r1 = L.r0 + 1;
                    L.gamma = __dsub_rn(vidx, fl);
                }
            }
            uint32_t blo, bhi;
            uint64_t before, before_hi;
            sketch_find(h, W, per, t, incl, (uint64_t)L.r0, blo, before);
            if (L.r1 != L.r0) sketch_find(h, W, per, t, incl, (uint64_t)L.r1, bhi, before_hi);
            else bhi = blo;
            L.bin_lo = blo;
            L.bin_hi = bhi;
            L.before = (int64_t)before;
        }
        if (lane == 0) A.out[s] = L;
    }
}

// Per segment: samples of this rank's local sketch inside [bin_lo, bin_hi].
__global__ __launch_bounds__(64) void k_sketch_range_count(int64_t S, uint32_t W, const uint32_t* __restrict__ counts,
                                                           const krr_sketch_loc* __restrict__ loc,
                                                           int64_t* __restrict__ out) {
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        const uint32_t lo = loc[s].bin_lo, hi = loc[s].bin_hi;
        uint32_t c = 0;
        if (lo <= hi && hi < W)
            for (uint32_t b = lo + lane; b <= hi; b += kWave) c += counts[(size_t)s * W + b];
        const uint32_t tot = wave_sum_u32(c);
        if (lane == 0) out[s] = (int64_t)tot;
    }
}

// Per segment: append, in position order, every present sample whose bin lies in
// [bin_lo, bin_hi] to out_vals[out_offs[s] ...]; out_n[s] = how many (optional).
__global__ __launch_bounds__(64) void k_sketch_collect(const double* __restrict__ vals,
                                                       const int64_t* __restrict__ offs, int64_t S, SketchGeom g,
                                                       const krr_sketch_loc* __restrict__ loc,
                                                       const int64_t* __restrict__ out_offs,
                                                       double* __restrict__ out_vals, int64_t* __restrict__ out_n) {
    constexpr int U = 8;
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        const uint32_t lo = loc[s].bin_lo, hi = loc[s].bin_hi;
        uint64_t run = 0;
        if (lo <= hi) {
            const int64_t beg = offs[s], end = offs[s + 1];
            double* __restrict__ dst = out_vals + out_offs[s];
            for (int64_t base = beg; base < end; base += (int64_t)U * kWave) {
                uint64_t x[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int64_t i = base + u * kWave + lane;
                    x[u] = i < end ? dbits(__builtin_nontemporal_load(vals + i)) : kQuietNaN;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t b = sketch_bin(g, x[u]);
                    const bool hit = !is_nan_bits(x[u]) && b >= lo && b <= hi;
                    const uint64_t m = ballot(hit);
                    if (m) {
                        if (hit) dst[run + lane_prefix(m)] = bitsd(x[u]);
                        run += popc64(m);
                    }
                }
            }
        }
        if (lane == 0 && out_n) out_n[s] = (int64_t)run;
    }
}

// Key for the refinement's ordering: numeric order with -0 == +0 (Python's
// sorted() and numpy compare the zeros equal; SORTED_LOWER resolves which zero by
// position afterwards, exactly as finish_value does).
__device__ __forceinline__ uint64_t refine_key(uint64_t u) { return okey(is_zero_bits(u) ? 0ull : u); }

// Key of ascending rank j among vals[beg, end) (no NaN): 8-bit MSD radix select,
// eight passes over the (small, L2-resident) list.
__device__ uint64_t radix_select(const double* __restrict__ vals, int64_t beg, int64_t end, uint64_t j,
                                 uint32_t* hist, int lane) {
    uint64_t prefix = 0, mask = 0;
#pragma unroll 1
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int b = lane; b < 256; b += kWave) hist[b] = 0;
        __syncthreads();
        for (int64_t i = beg + lane; i < end; i += kWave) {
            const uint64_t k = refine_key(dbits(vals[i]));
            if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
        }
        __syncthreads();
        uint32_t c4[4], t = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            c4[q] = hist[lane * 4 + q];
            t += c4[q];
        }
        const uint32_t incl = wave_scan32(t, 0u, OpAdd32{});
        const uint64_t m = ballot(j < incl);
        const int src = __ffsll((long long)m) - 1;
        uint64_t run = lane_bcast32(incl - t, src);
        uint32_t digit = (uint32_t)src * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t c = lane_bcast32(c4[q], src);
            if (j >= run + c && q < 3) {
                run += c;
                digit = (uint32_t)src * 4 + q + 1;
            } else {
                break;
            }
        }
        j -= run;
        prefix |= (uint64_t)digit << shift;
        mask |= 255ull << shift;
        __syncthreads();
    }
    return prefix;
}

struct SketchRefineArgs {
    const double* vals;  // collected samples, CSR by series, position (time) order within a series
    const int64_t* offs;
    int64_t S;
    const krr_sketch_loc* loc;
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
};

__global__ __launch_bounds__(64) void k_sketch_refine(SketchRefineArgs A) {
    __shared__ uint32_t hist[256];
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const krr_sketch_loc L = A.loc[s];
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        uint32_t flags = L.flags;
        double result = bitsd(kQuietNaN);
        if (L.n > 0) {
            const int64_t j0 = L.r0 - L.before, j1 = L.r1 - L.before;
            if (j0 < 0 || j1 < j0 || j1 >= end - beg) {
                flags |= KRR_FLAG_CAPACITY;  // collected list inconsistent with the sketch
            } else {
                const uint64_t k0 = radix_select(A.vals, beg, end, (uint64_t)j0, hist, lane);
                const uint64_t k1 = j1 != j0 ? radix_select(A.vals, beg, end, (uint64_t)j1, hist, lane) : k0;
                const double a = bitsd(okey_inv(k0));
                if (L.mode == KRR_PCT_SORTED_LOWER) {
                    uint64_t bits = dbits(a);
                    if (is_zero_bits(bits)) {  // the (j0 - #negatives)-th zero in time order
                        const uint64_t neg = count_negative(A.vals, beg, end, lane);
                        bits = nth_zero_bits(A.vals, beg, end, (uint64_t)j0 - neg, lane);
                    }
                    result = bitsd(bits);
                } else {
                    result = np_lerp(a, bitsd(okey_inv(k1)), L.gamma);
                }
            }
        }
        if (lane == 0) {
            A.out_v[s] = result;
            A.out_n[s] = L.n;
            A.out_f[s] = flags;
        }
        __syncthreads();
    }
}

// ------------------------------ SYNTH --------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t hash4(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    return mix64(mix64(mix64(mix64(a) ^ b) ^ c) ^ d);
}
// uniform in (0, 1]
__device__ __forceinline__ double unit01(uint64_t h) { return ((double)(h >> 11) + 1.0) * 0x1.0p-53; }

__global__ __launch_bounds__(256) void k_synth(double* __restrict__ vals, const int64_t* __restrict__ offs,
                                              int64_t S, uint64_t seed, int kind, int64_t pod_len,
                                              int gaps, int64_t seg_base, int64_t t0, int64_t total_len) {
    // Slot i of segment s is global time index t = t0 + i of a series of
    // total_len slots (0: the segment itself), so time slices generated on
    // different ranks concatenate to exactly the series one rank would generate.
    // Segment s is global segment g = seg_base + s, so object shards generated on
    // different ranks are exactly the fleet one rank would generate.
    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        const int64_t beg = offs[s], Lloc = offs[s + 1] - beg;
        const uint64_t g = (uint64_t)(seg_base + s);
        const int64_t L = total_len > 0 ? total_len : Lloc;
        const int64_t plen = pod_len > 0 ? pod_len : (L > 0 ? L : 1);
        for (int64_t i = threadIdx.x; i < Lloc; i += blockDim.x) {
            const int64_t t = t0 + i;
            const int64_t pod = t / plen;
            const int64_t tp = t - pod * plen;
            const int64_t pl = (L - pod * plen) < plen ? (L - pod * plen) : plen;
            bool gap = false;
            if (gaps) {
                const uint64_t hp = hash4(seed, g, (uint64_t)pod, 0xA11CEull);
                int64_t start = 0;
                if ((hp & 0xFFFF) < 19661 && pl > 1440)  // p = 0.3: the pod started late
                    start = (int64_t)((hp >> 16) % (uint64_t)(pl - 1440 + 1));
                const double f = 0.2 * unit01(hash4(seed, g, (uint64_t)pod, 0xF00Dull));
                const double ub = unit01(hash4(seed ^ 0x5EEDull, g, (uint64_t)pod, (uint64_t)(tp / 30)));
                gap = tp < start || (tp >= start + 1440 && ub <= f);
            }
            double v;
            if (gap) {
                v = bitsd(kQuietNaN);
            } else {
                const uint64_t h1 = hash4(seed, g, (uint64_t)t, (uint64_t)kind);
                const uint64_t h2 = mix64(h1 ^ 0xD1B54A32D192ED03ull);
                if (kind == 0) {  // Gamma(k=2, theta=0.05) cores = sum of two exponentials
                    v = -0.05 * (log(unit01(h1)) + log(unit01(h2)));
                } else {  // floor(Normal(2e8, 2e7)) bytes, Box-Muller
                    const double z = sqrt(-2.0 * log(unit01(h1))) * cospi(2.0 * unit01(h2));
                    v = floor(2.0e8 + 2.0e7 * z);
                    if (v < 0.0) v = 0.0;
                }
            }
            vals[beg + i] = v;
        }
    }
}

}  // namespace krr

// ============================== C ABI =======================================
using namespace krr;

struct krr_ctx {
    int device;
    int num_cus;
    size_t max_lds;
    unsigned long long* d_tmp;    // [0] scratch (max segment length), [1] stats: wselect fallbacks
    unsigned int* d_fail_count;   // wselect miss list lengths: [epoch & 1]
    unsigned int fail_epoch;      // advanced only after a window launch + its miss pass were enqueued
    int64_t* d_fail_list;         // segment ids (capacity fail_cap)
    int64_t fail_cap;
    // The miss list and its counters are shared by every stream the ctx is used on:
    // the miss pass of the last window launch is recorded here, and a window launch on
    // another stream first waits for it (same stream: stream order already does).
    hipEvent_t fail_ev;
    hipStream_t fail_stream;
    bool fail_ev_valid;
    char err[512];
};

static int set_err(krr_ctx* c, int code, const char* fmt, const char* a = "", long long b = 0) {
    if (c) snprintf(c->err, sizeof(c->err), fmt, a, b);
    return code;
}

#define KRR_HIP(ctx, call)                                                                      \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess) return set_err((ctx), KRR_E_HIP, "HIP error %s (%lld) at " #call, \
                                             hipGetErrorString(e_), (long long)e_);             \
    } while (0)

namespace {

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int grid_for(int64_t S) {
    const int64_t cap = 2147483647LL;
    return (int)(S < cap ? S : cap);
}

int resolve_maxlen(krr_ctx* ctx, const krr_series* s, hipStream_t st, int64_t* out) {
    if (s->max_segment_len > 0) {
        *out = s->max_segment_len;
        return KRR_OK;
    }
    if (s->n_segments == 0) {
        *out = 0;
        return KRR_OK;
    }
    KRR_HIP(ctx, hipMemsetAsync(ctx->d_tmp, 0, sizeof(unsigned long long), st));
    int blocks = (int)((s->n_segments + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_maxlen, dim3(blocks), dim3(256), 0, st, s->offsets, s->n_segments, ctx->d_tmp);
    KRR_HIP(ctx, hipGetLastError());
    unsigned long long h = 0;
    KRR_HIP(ctx, hipMemcpyAsync(&h, ctx->d_tmp, sizeof(h), hipMemcpyDeviceToHost, st));
    KRR_HIP(ctx, hipStreamSynchronize(st));
    *out = (int64_t)h;
    return KRR_OK;
}

// A launch reading krr_percentile_params.k_table: every segment's count must index it.
int check_table(krr_ctx* ctx, const krr_series* s, const krr_percentile_params* p, hipStream_t st) {
    if (!p->k_table || p->mode == KRR_PCT_LINEAR) return KRR_OK;
    int64_t Lmax = 0;
    int rc = resolve_maxlen(ctx, s, st, &Lmax);
    if (rc) return rc;
    if (Lmax >= p->k_table_len)
        return set_err(ctx, KRR_E_INVALID, "k_table holds %s%lld entries, segments reach more slots", "",
                       (long long)p->k_table_len);
    return KRR_OK;
}

int check_series(krr_ctx* ctx, const krr_series* s) {
    if (!s) return set_err(ctx, KRR_E_INVALID, "null series%s", "");
    if (s->n_segments < 0) return set_err(ctx, KRR_E_INVALID, "negative n_segments%s", "");
    if (s->n_segments > 0 && (!s->offsets || (!s->values && s->n_values > 0)))
        return set_err(ctx, KRR_E_INVALID, "null values/offsets%s", "");
    return KRR_OK;
}

// Plan a SORTED_LOWER / LINEAR launch: single-pass candidate capacity from the
// longest segment, or (when that exceeds kSingleCapMax keys) the hselect path
// for every segment (A->cap = 0), and the LDS bytes.
int plan_select(krr_ctx* ctx, const krr_series* series, const krr_percentile_params* params,
                hipStream_t st, double* ov, int64_t* on, uint32_t* of, SelectArgs* A, size_t* lds, bool fused) {
    int64_t Lmax = 0;
    int rc = resolve_maxlen(ctx, series, st, &Lmax);
    if (rc) return rc;
    if (params->k_table && params->mode != KRR_PCT_LINEAR && Lmax >= params->k_table_len)
        return set_err(ctx, KRR_E_INVALID, "k_table holds %s%lld entries, segments reach more slots", "",
                       (long long)params->k_table_len);
    const SidePlan sp = plan_side(Lmax, params->mode, params->p_num, params->p_den, params->q,
                                  params->k_table != nullptr);
    const uint32_t need = capacity_for(sp.tkeep);
    const bool hsel = window_select(need, sp.tkeep, Lmax, sp.bottom, fused);  // every segment through wselect
    const uint32_t cap = hsel ? 0u : need;
    *A = SelectArgs{};
    A->vals = series->values;
    A->offs = series->offsets;
    A->S = series->n_segments;
    A->mode = params->mode;
    A->gaps = series->gaps_are_nan;
    A->p_num = params->p_num;
    A->p_den = params->p_den;
    A->q = params->q;
    A->ktab = params->k_table;
    A->ktab_len = params->k_table_len;
    A->cap = cap;
    A->out_v = ov;
    A->out_n = on;
    A->out_f = of;
    A->stats = ctx->d_tmp + 1;
    A->wcap = wsel_cap_for(Lmax, series->gaps_are_nan != 0);
    A->remap = Lmax < KRR_XCD_REMAP_MAXLEN ? 1 : 0;
    if (hsel && KRR_WSEL && A->wcap != kWselCapLong) {  // misses: a list for the hselect launch that follows
        if (ctx->fail_cap < series->n_segments) {
            if (ctx->d_fail_list) KRR_HIP(ctx, hipFree(ctx->d_fail_list));
            ctx->d_fail_list = nullptr;
            ctx->fail_cap = 0;
            KRR_HIP(ctx, hipMalloc(&ctx->d_fail_list, (size_t)series->n_segments * sizeof(int64_t)));
            ctx->fail_cap = series->n_segments;
        }
    }
    *lds = kSelectLdsFixed + (hsel ? (KRR_WSEL ? window_lds(A->wcap) : kHselectLds) : (size_t)cap * 8);
    if (*lds < (size_t)KRR_LDS_MIN) *lds = (size_t)KRR_LDS_MIN;
    if (*lds > ctx->max_lds) return set_err(ctx, KRR_E_CAPACITY, "select needs %s%lld B of LDS", "", (long long)*lds);
    if (hsel && KRR_WSEL && A->wcap != kWselCapLong) {
        // launch k counts its misses into counter (k & 1) and zeroes counter ((k + 1) & 1),
        // which launch k - 1's miss pass has read by then (stream order, or the event below);
        // the epoch only advances once the launch is enqueued (commit_fail_list)
        if (ctx->fail_ev_valid && ctx->fail_stream != st) KRR_HIP(ctx, hipStreamWaitEvent(st, ctx->fail_ev, 0));
        A->fail_list = ctx->d_fail_list;
        const unsigned int e = ctx->fail_epoch & 1u;
        A->fail_count = ctx->d_fail_count + e;
        A->fail_reset = ctx->d_fail_count + (e ^ 1u);
    }
    return KRR_OK;
}

// After a window-select launch: hselect over the segments it missed (none, usually).
// Only then does the miss list's epoch advance, and the pass is recorded for window
// launches that come on another stream (plan_select).
int launch_fallback(krr_ctx* ctx, const SelectArgs& A, int64_t S, hipStream_t st) {
    if (!A.fail_list) return KRR_OK;
    const int64_t g = S < (int64_t)KRR_FALLBACK_GRID ? S : (int64_t)KRR_FALLBACK_GRID;
    hipLaunchKernelGGL(k_hselect_list, dim3((unsigned)g), dim3(64), kSelectLdsFixed + kHselectLds, st, A);
    KRR_HIP(ctx, hipGetLastError());
    ctx->fail_epoch++;
    KRR_HIP(ctx, hipEventRecord(ctx->fail_ev, st));
    ctx->fail_stream = st;
    ctx->fail_ev_valid = true;
    return KRR_OK;
}

int check_params(krr_ctx* ctx, const krr_percentile_params* p) {
    if (!p) return set_err(ctx, KRR_E_INVALID, "null params%s", "");
    if (p->mode < KRR_PCT_REF_INDEX || p->mode > KRR_PCT_LINEAR)
        return set_err(ctx, KRR_E_INVALID, "bad percentile mode %s%lld", "", p->mode);
    if (p->p_den <= 0 || p->p_den > 1000000000000000LL || p->p_num <= 0 || p->p_num > 100 * p->p_den)
        return set_err(ctx, KRR_E_INVALID, "percentile must be in (0, 100] with p_den <= 1e15%s", "");
    if ((p->k_table != nullptr) != (p->k_table_len > 0) || (p->k_table && p->k_table_len < 2))
        return set_err(ctx, KRR_E_INVALID, "k_table needs k_table_len >= 2 (and a table for a length)%s", "");
    if (p->mode == KRR_PCT_LINEAR && !(p->q > 0.0 && p->q <= 1.0))
        return set_err(ctx, KRR_E_INVALID, "LINEAR needs q = p/100 in (0, 1]%s", "");
    return KRR_OK;
}

}  // namespace

extern "C" {

int krr_abi_version(void) { return KRR_ABI_VERSION; }

int krr_create(int device, krr_ctx** out_ctx) {
    if (!out_ctx) return KRR_E_INVALID;
    *out_ctx = nullptr;
    krr_ctx* c = new (std::nothrow) krr_ctx();
    if (!c) return KRR_E_INVALID;
    c->device = device;
    c->d_tmp = nullptr;
    c->err[0] = 0;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        delete c;
        return KRR_E_HIP;
    }
    DeviceGuard g(device);
    hipDeviceProp_t prop;
    if (!g.ok || hipGetDeviceProperties(&prop, device) != hipSuccess) {
        delete c;
        return KRR_E_HIP;
    }
    c->num_cus = prop.multiProcessorCount;
    c->max_lds = prop.maxSharedMemoryPerMultiProcessor ? prop.maxSharedMemoryPerMultiProcessor : 65536;
    if (c->max_lds > 163840) c->max_lds = 163840;
    c->d_fail_count = nullptr;
    c->fail_epoch = 0;
    c->d_fail_list = nullptr;
    c->fail_cap = 0;
    c->fail_ev = nullptr;
    c->fail_stream = nullptr;
    c->fail_ev_valid = false;
    if (hipEventCreateWithFlags(&c->fail_ev, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return KRR_E_HIP;
    }
    if (hipMalloc(&c->d_tmp, 2 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_tmp, 0, 2 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->d_fail_count, 2 * sizeof(unsigned int)) != hipSuccess ||
        hipMemset(c->d_fail_count, 0, 2 * sizeof(unsigned int)) != hipSuccess) {
        if (c->d_tmp) (void)hipFree(c->d_tmp);
        if (c->d_fail_count) (void)hipFree(c->d_fail_count);
        (void)hipEventDestroy(c->fail_ev);
        delete c;
        return KRR_E_HIP;
    }

    for (const void* f : {(const void*)k_select<SEL_SINGLE>, (const void*)k_select<SEL_WINDOW>,
                          (const void*)k_select<SEL_WINDOW_LONG>, (const void*)k_simple<CPU_SELECT>,
                          (const void*)k_simple<CPU_HSELECT>, (const void*)k_simple<CPU_HSELECT_LONG>,
                          (const void*)k_simple<CPU_SELECT, true>, (const void*)k_simple<CPU_HSELECT, true>,
                          (const void*)k_simple<CPU_HSELECT_LONG, true>})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->max_lds);
    (void)hipFuncSetAttribute((const void*)k_sketch_build, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)c->max_lds);
    for (const void* f : {(const void*)k_hselect_list, (const void*)k_window_export<true>,
                          (const void*)k_window_export<false>, (const void*)k_window_merge,
                          (const void*)k_kll_build<false>, (const void*)k_kll_build<true>, (const void*)k_kll_tail,
                          (const void*)k_kll_build<false, true>, (const void*)k_kll_tail_lines,
                          (const void*)k_kll_merge,
                          (const void*)k_kll_query})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->max_lds);
    *out_ctx = c;
    return KRR_OK;
}

int krr_destroy(krr_ctx* ctx) {
    if (!ctx) return KRR_OK;
    DeviceGuard g(ctx->device);
    if (ctx->d_tmp) (void)hipFree(ctx->d_tmp);
    if (ctx->d_fail_count) (void)hipFree(ctx->d_fail_count);
    if (ctx->d_fail_list) (void)hipFree(ctx->d_fail_list);
    if (ctx->fail_ev) (void)hipEventDestroy(ctx->fail_ev);
    delete ctx;
    return KRR_OK;
}

const char* krr_last_error(const krr_ctx* ctx) { return ctx ? ctx->err : "null krr_ctx"; }

int krr_segmented_percentile(krr_ctx* ctx, const krr_series* series, const krr_percentile_params* params,
                             double* out_value, int64_t* out_count, uint32_t* out_flags, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    rc = check_params(ctx, params);
    if (rc) return rc;
    const int64_t S = series->n_segments;
    if (S == 0) return KRR_OK;
    if (!out_value || !out_count || !out_flags) return set_err(ctx, KRR_E_INVALID, "null outputs%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipStream_t st = (hipStream_t)stream;

    if (params->mode == KRR_PCT_REF_INDEX) {
        rc = check_table(ctx, series, params, st);
        if (rc) return rc;
        RefArgs A{series->values, series->offsets, S, params->p_num, params->p_den, params->k_table,
                  params->k_table_len, out_value, out_count, out_flags};
        if (series->gaps_are_nan) {
            hipLaunchKernelGGL(k_refindex_gaps, dim3(grid_for(S)), dim3(64), 0, st, A);
        } else {
            hipLaunchKernelGGL(k_refindex_dense, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, A);
        }
        KRR_HIP(ctx, hipGetLastError());
        return KRR_OK;
    }

    SelectArgs A;
    size_t lds = 0;
    rc = plan_select(ctx, series, params, st, out_value, out_count, out_flags, &A, &lds, false);
    if (rc) return rc;
    if (A.cap) hipLaunchKernelGGL(k_select<SEL_SINGLE>, dim3(grid_for(S)), dim3(64), lds, st, A);
    else if (A.wcap == kWselCapLong) hipLaunchKernelGGL(k_select<SEL_WINDOW_LONG>, dim3(grid_for(S)), dim3(64), lds, st, A);
    else hipLaunchKernelGGL(k_select<SEL_WINDOW>, dim3(grid_for(S)), dim3(64), lds, st, A);
    KRR_HIP(ctx, hipGetLastError());
    return launch_fallback(ctx, A, S, st);
}

int krr_segmented_max(krr_ctx* ctx, const krr_series* series, double* out_value, int64_t* out_count,
                      uint32_t* out_flags, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    const int64_t S = series->n_segments;
    if (S == 0) return KRR_OK;
    if (!out_value || !out_count || !out_flags) return set_err(ctx, KRR_E_INVALID, "null outputs%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    MaxArgs A{series->values, series->offsets, S, series->gaps_are_nan, out_value, out_count, out_flags};
    A.remap = series->max_segment_len > 0 && series->max_segment_len >= KRR_XCD_REMAP_MAXLEN ? 0 : 1;
    hipLaunchKernelGGL(k_max, dim3(grid_for(S)), dim3(64), 0, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_simple_run(krr_ctx* ctx, const krr_series* cpu, const krr_series* mem,
                   const krr_percentile_params* params, double* cpu_value, int64_t* cpu_count,
                   uint32_t* cpu_flags, double* mem_value, int64_t* mem_count, uint32_t* mem_flags,
                   void* stream) {
    return krr_simple_run_records(ctx, cpu, mem, params, cpu_value, cpu_count, cpu_flags, mem_value, mem_count,
                                  mem_flags, nullptr, stream);
}

int krr_simple_run_records(krr_ctx* ctx, const krr_series* cpu, const krr_series* mem,
                           const krr_percentile_params* params, double* cpu_value, int64_t* cpu_count,
                           uint32_t* cpu_flags, double* mem_value, int64_t* mem_count, uint32_t* mem_flags,
                           int64_t* records, void* stream) {
    return krr_simple_run_forward(ctx, cpu, mem, params, cpu_value, cpu_count, cpu_flags, mem_value, mem_count,
                                  mem_flags, records, nullptr, nullptr, 0, stream);
}

int krr_simple_run_forward(krr_ctx* ctx, const krr_series* cpu, const krr_series* mem,
                           const krr_percentile_params* params, double* cpu_value, int64_t* cpu_count,
                           uint32_t* cpu_flags, double* mem_value, int64_t* mem_count, uint32_t* mem_flags,
                           int64_t* records, const void* forward_src, void* forward_dst, int64_t forward_bytes,
                           void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (forward_bytes < 0 || forward_bytes % 16 != 0 || (forward_bytes > 0 && (!forward_src || !forward_dst)))
        return set_err(ctx, KRR_E_INVALID, "forward copy: a multiple of 16 bytes between non-null pointers%s", "");
    if (forward_bytes > 0 && (((uintptr_t)forward_src | (uintptr_t)forward_dst) & 15))
        return set_err(ctx, KRR_E_INVALID, "forward copy pointers must be 16-byte aligned%s", "");
    if (!cpu || !mem) return set_err(ctx, KRR_E_INVALID, "null series%s", "");
    if (cpu->n_segments != mem->n_segments)
        return set_err(ctx, KRR_E_INVALID, "cpu and mem need one segment per object each%s", "");
    int rc = check_series(ctx, cpu);
    if (!rc) rc = check_series(ctx, mem);
    if (!rc) rc = check_params(ctx, params);
    if (rc) return rc;
    const int64_t S = cpu->n_segments;
    if (S > 0 && (!cpu_value || !cpu_count || !cpu_flags || !mem_value || !mem_count || !mem_flags))
        return set_err(ctx, KRR_E_INVALID, "null outputs%s", "");
    const int64_t fwd_units = forward_bytes / 16;
    if (fwd_units > 0 && (S == 0 || (params->mode == KRR_PCT_REF_INDEX && !cpu->gaps_are_nan))) {
        // no fused launch to ride on: a plain copy on the stream
        DeviceGuard g(ctx->device);
        if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
        KRR_HIP(ctx, hipMemcpyAsync(forward_dst, forward_src, (size_t)forward_bytes, hipMemcpyDefault,
                                    (hipStream_t)stream));
    }
    if (S == 0) return KRR_OK;
    if (params->mode == KRR_PCT_REF_INDEX && !cpu->gaps_are_nan) {
        // compact REF_INDEX is one gather per segment: nothing to fuse with
        rc = krr_segmented_percentile(ctx, cpu, params, cpu_value, cpu_count, cpu_flags, stream);
        if (!rc) rc = krr_segmented_max(ctx, mem, mem_value, mem_count, mem_flags, stream);
        if (!rc && records)
            rc = krr_pack_records(ctx, S, cpu_value, cpu_count, cpu_flags, mem_value, mem_count, mem_flags,
                                  records, stream);
        return rc;
    }
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipStream_t st = (hipStream_t)stream;
    MaxArgs M{mem->values, mem->offsets, S, mem->gaps_are_nan, mem_value, mem_count, mem_flags, records};
    M.remap = mem->max_segment_len > 0 && mem->max_segment_len >= KRR_XCD_REMAP_MAXLEN ? 0 : 1;
    if (fwd_units > 0) {
        M.fwd_src = (const double2*)forward_src;
        M.fwd_dst = (double2*)forward_dst;
        M.fwd_units = fwd_units;
        M.fwd_items = ((fwd_units + kFwdItemUnits - 1) / kFwdItemUnits + 7) & ~(int64_t)7;
    }
    const int64_t items = M.fwd_items + 2 * S;
    RefArgs R{cpu->values, cpu->offsets, S, params->p_num, params->p_den, params->k_table, params->k_table_len,
              cpu_value, cpu_count, cpu_flags, records};
    SelectArgs A{};
    const bool fwd = M.fwd_items > 0;
    if (params->mode == KRR_PCT_REF_INDEX) {
        rc = check_table(ctx, cpu, params, st);
        if (rc) return rc;
        if (fwd) hipLaunchKernelGGL((k_simple<CPU_REF_GAPS, true>), dim3(grid_for(items)), dim3(64), 0, st, A, R, M);
        else hipLaunchKernelGGL((k_simple<CPU_REF_GAPS>), dim3(grid_for(items)), dim3(64), 0, st, A, R, M);
    } else {
        size_t lds = 0;
        rc = plan_select(ctx, cpu, params, st, cpu_value, cpu_count, cpu_flags, &A, &lds, true);
        if (rc) return rc;
        A.rec = records;
        const dim3 g(grid_for(items)), b(64);
        if (A.cap) {
            if (fwd) hipLaunchKernelGGL((k_simple<CPU_SELECT, true>), g, b, lds, st, A, R, M);
            else hipLaunchKernelGGL((k_simple<CPU_SELECT>), g, b, lds, st, A, R, M);
        } else if (A.wcap == kWselCapLong) {
            if (fwd) hipLaunchKernelGGL((k_simple<CPU_HSELECT_LONG, true>), g, b, lds, st, A, R, M);
            else hipLaunchKernelGGL((k_simple<CPU_HSELECT_LONG>), g, b, lds, st, A, R, M);
        } else {
            if (fwd) hipLaunchKernelGGL((k_simple<CPU_HSELECT, true>), g, b, lds, st, A, R, M);
            else hipLaunchKernelGGL((k_simple<CPU_HSELECT>), g, b, lds, st, A, R, M);
        }
        KRR_HIP(ctx, hipGetLastError());
        return launch_fallback(ctx, A, S, st);
    }
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_simple_run_host(krr_ctx* ctx, const double* cpu_values, const int64_t* cpu_offsets,
                        const double* mem_values, const int64_t* mem_offsets, int64_t n_objects,
                        int32_t gaps_are_nan, const krr_percentile_params* params, double* cpu_value,
                        int64_t* cpu_count, uint32_t* cpu_flags, double* mem_value, int64_t* mem_count,
                        uint32_t* mem_flags) {
    if (!ctx) return KRR_E_INVALID;
    if (n_objects < 0 || (n_objects > 0 && (!cpu_offsets || !mem_offsets)))
        return set_err(ctx, KRR_E_INVALID, "bad host arguments%s", "");
    if (n_objects == 0) return KRR_OK;
    int rc = check_params(ctx, params);
    if (rc) return rc;
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    const int64_t S = n_objects;
    const int64_t ncpu = cpu_offsets[S] - cpu_offsets[0];
    const int64_t nmem = mem_offsets[S] - mem_offsets[0];
    if (cpu_offsets[0] != 0 || mem_offsets[0] != 0)
        return set_err(ctx, KRR_E_INVALID, "offsets must start at 0%s", "");
    int64_t lc = 0, lm = 0;
    for (int64_t s = 0; s < S; ++s) {
        const int64_t a = cpu_offsets[s + 1] - cpu_offsets[s], b = mem_offsets[s + 1] - mem_offsets[s];
        if (a < 0 || b < 0) return set_err(ctx, KRR_E_INVALID, "offsets must be non-decreasing%s", "");
        lc = a > lc ? a : lc;
        lm = b > lm ? b : lm;
    }
    // one allocation: [cpu vals][mem vals][cpu offs][mem offs][outputs]
    const size_t bcv = (size_t)ncpu * 8, bmv = (size_t)nmem * 8, bo = (size_t)(S + 1) * 8;
    const size_t bout = (size_t)S * (8 + 8 + 4) * 2;
    const size_t total = bcv + bmv + 2 * bo + bout + 256;
    char* d = nullptr;
    KRR_HIP(ctx, hipMalloc(&d, total));
    char* p = d;
    auto take = [&](size_t n) {
        char* r = p;
        p += (n + 15) & ~(size_t)15;
        return r;
    };
    double* dcv = (double*)take(bcv);
    double* dmv = (double*)take(bmv);
    int64_t* dco = (int64_t*)take(bo);
    int64_t* dmo = (int64_t*)take(bo);
    double* o_cv = (double*)take((size_t)S * 8);
    int64_t* o_cn = (int64_t*)take((size_t)S * 8);
    uint32_t* o_cf = (uint32_t*)take((size_t)S * 4);
    double* o_mv = (double*)take((size_t)S * 8);
    int64_t* o_mn = (int64_t*)take((size_t)S * 8);
    uint32_t* o_mf = (uint32_t*)take((size_t)S * 4);
    hipError_t e = hipSuccess;
    if (bcv) e = hipMemcpy(dcv, cpu_values, bcv, hipMemcpyHostToDevice);
    if (e == hipSuccess && bmv) e = hipMemcpy(dmv, mem_values, bmv, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dco, cpu_offsets, bo, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dmo, mem_offsets, bo, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return set_err(ctx, KRR_E_HIP, "H2D copy failed: %s%lld", hipGetErrorString(e), 0);
    }
    krr_series cs{dcv, dco, S, ncpu, lc > 0 ? lc : 1, gaps_are_nan, 0};
    krr_series ms{dmv, dmo, S, nmem, lm > 0 ? lm : 1, gaps_are_nan, 0};
    rc = krr_simple_run(ctx, &cs, &ms, params, o_cv, o_cn, o_cf, o_mv, o_mn, o_mf, nullptr);
    if (rc == KRR_OK) {
        e = hipDeviceSynchronize();
        if (e == hipSuccess) e = hipMemcpy(cpu_value, o_cv, (size_t)S * 8, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(cpu_count, o_cn, (size_t)S * 8, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(cpu_flags, o_cf, (size_t)S * 4, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(mem_value, o_mv, (size_t)S * 8, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(mem_count, o_mn, (size_t)S * 8, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(mem_flags, o_mf, (size_t)S * 4, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = set_err(ctx, KRR_E_HIP, "D2H/sync failed: %s%lld", hipGetErrorString(e), 0);
    }
    (void)hipFree(d);
    return rc;
}

int krr_pack_records(krr_ctx* ctx, int64_t n_objects, const double* cpu_value, const int64_t* cpu_count,
                     const uint32_t* cpu_flags, const double* mem_value, const int64_t* mem_count,
                     const uint32_t* mem_flags, int64_t* records, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (n_objects < 0 || (n_objects > 0 && (!cpu_value || !cpu_count || !cpu_flags || !mem_value ||
                                            !mem_count || !mem_flags || !records)))
        return set_err(ctx, KRR_E_INVALID, "bad pack_records arguments%s", "");
    if (n_objects == 0) return KRR_OK;
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipLaunchKernelGGL(k_pack_records, dim3((unsigned)((n_objects + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, n_objects, cpu_value, cpu_count, cpu_flags, mem_value, mem_count,
                       mem_flags, records);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

#ifdef KRR_WEXP_DEBUG
int krr_wexp_debug_read(unsigned long long* out, unsigned int* n) {
    if (hipMemcpyFromSymbol(n, HIP_SYMBOL(krr::g_wdbg_n), sizeof(unsigned int)) != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(krr::g_wdbg), sizeof(unsigned long long) * 5 * 1024) != hipSuccess) return -2;
    unsigned int z = 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(krr::g_wdbg_n), &z, sizeof(z)) == hipSuccess ? 0 : -2;
}
#endif

#ifdef KRR_DIAG
int krr_diag_attach(void* dev_buffer) {
    return hipMemcpyToSymbol(HIP_SYMBOL(krr::g_diag), &dev_buffer, sizeof(void*)) == hipSuccess ? 0 : -2;
}
#endif

int krr_synth_fill_global(krr_ctx* ctx, double* values, const int64_t* offsets, int64_t n_segments, uint64_t seed,
                          int32_t kind, int64_t pod_len, int32_t gaps, int64_t seg_base, int64_t t0, int64_t total_len,
                          void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (n_segments < 0 || (n_segments > 0 && (!values || !offsets)) || kind < 0 || kind > 1 || t0 < 0 ||
        total_len < 0 || seg_base < 0)
        return set_err(ctx, KRR_E_INVALID, "bad synth arguments%s", "");
    if (n_segments == 0) return KRR_OK;
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    int64_t grid = n_segments < 65536 ? n_segments : 65536;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, values, offsets,
                       n_segments, seed, kind, pod_len, gaps, seg_base, t0, total_len);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_synth_fill_window(krr_ctx* ctx, double* values, const int64_t* offsets, int64_t n_segments, uint64_t seed,
                          int32_t kind, int64_t pod_len, int32_t gaps, int64_t t0, int64_t total_len, void* stream) {
    return krr_synth_fill_global(ctx, values, offsets, n_segments, seed, kind, pod_len, gaps, 0, t0, total_len,
                                 stream);
}

int krr_synth_fill(krr_ctx* ctx, double* values, const int64_t* offsets, int64_t n_segments, uint64_t seed,
                   int32_t kind, int64_t pod_len, int32_t gaps, void* stream) {
    return krr_synth_fill_window(ctx, values, offsets, n_segments, seed, kind, pod_len, gaps, 0, 0, stream);
}

int64_t krr_sketch_width(const krr_sketch_params* sp) {
    if (!sp || sp->mantissa_bits < 0 || sp->mantissa_bits > 10 || sp->octaves < 1 || sp->min_exponent < -1022 ||
        (int64_t)sp->min_exponent + sp->octaves > 1024)
        return -1;
    return ((int64_t)sp->octaves << sp->mantissa_bits) + 4;
}

int krr_sketch_build(krr_ctx* ctx, const krr_series* series, const krr_sketch_params* sp, uint32_t* counts,
                     double* vmin, double* vmax, uint32_t* flags, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    const int64_t W = krr_sketch_width(sp);
    if (W < 0) return set_err(ctx, KRR_E_INVALID, "bad sketch params%s", "");
    if ((size_t)W * 4 > ctx->max_lds || (W & 3)) return set_err(ctx, KRR_E_UNSUPPORTED, "sketch width %s%lld", "", W);
    const int64_t S = series->n_segments;
    if (S == 0) return KRR_OK;
    if (!counts || !vmin || !vmax || !flags) return set_err(ctx, KRR_E_INVALID, "null outputs%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    SketchBuildArgs A{series->values, series->offsets, S, series->gaps_are_nan, sketch_geom(*sp), counts, vmin, vmax,
                      flags};
    hipLaunchKernelGGL(k_sketch_build, dim3(grid_for(S)), dim3(64), (size_t)W * 4, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_sketch_query(krr_ctx* ctx, int64_t n_segments, const uint32_t* counts, const double* vmin,
                     const double* vmax, const krr_sketch_params* sp, const krr_percentile_params* params,
                     double* out_value, int64_t* out_count, uint32_t* out_flags, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_params(ctx, params);
    if (rc) return rc;
    if (params->mode == KRR_PCT_REF_INDEX)
        return set_err(ctx, KRR_E_UNSUPPORTED, "REF_INDEX has no sketch form: use krr_select_present%s", "");
    if (krr_sketch_width(sp) < 0) return set_err(ctx, KRR_E_INVALID, "bad sketch params%s", "");
    if (n_segments < 0) return set_err(ctx, KRR_E_INVALID, "negative n_segments%s", "");
    if (n_segments == 0) return KRR_OK;
    if (!counts || !vmin || !vmax || !out_value || !out_count || !out_flags)
        return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    SketchQueryArgs A{n_segments, sketch_geom(*sp), counts, vmin, vmax, params->mode, params->p_num,
                      params->p_den, params->q, out_value, out_count, out_flags, params->k_table,
                      params->k_table_len};
    hipLaunchKernelGGL(k_sketch_query, dim3(grid_for(n_segments)), dim3(64), 0, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int64_t krr_kll_row_words(const krr_kll_params* kp) {
    if (!kp || kp->budget < kKllRun || kp->budget > 4096 || (kp->budget & 63) || kp->tail < 0 || kp->tail > 4096)
        return -1;
    return (int64_t)kKllHdr + kp->budget + kp->tail;
}

// tail buffer keys: a refresh leaves <= tail + slack, a chunk adds <= 1,024; the final
// compression's workspace (1,024 level keys + 512 carry) reuses it
// Words of the region after tmp: the tail buffer (room for a chunk's 1,024 candidates past a
// refresh's tail + slack), at least what the final stage needs beyond tmp's 512 words.
#ifndef KRR_KLL_TAIL_ROOM
#define KRR_KLL_TAIL_ROOM 512u
#endif
static uint32_t kll_tcap(int32_t tail) {
    const uint32_t t = tail > 0 ? (uint32_t)tail + 1024u + kKllTailSlack : 0u;
    const uint32_t fin = kKllFinalWords - 2u * kKllRun;
    return t > fin ? t : fin;
}

static size_t kll_build_lds(int nrl, uint32_t tcap) {
    return ((size_t)(nrl + 2) * kKllRun + tcap + kKllLevels) * 8 + (3 * kKllLevels + 2) * 4;
}

static size_t kll_merge_lds(const krr_kll_params* kp, bool query) {
    const size_t rw = (size_t)kKllHdr + kp->budget + kp->tail;
    return (3 * rw + 5 * (size_t)kp->budget) * 8 + (query ? (size_t)kp->budget : 0);
}

// The tail pass's LDS: its buffer (tail + slack + room for KRR_KLL_TAIL_ROOM candidates between
// refreshes; columns of <= 128 keys go in one by one when a chunk brings more), which before the
// stream holds the body keys and their levels.
static void kll_tail_lds(const krr_kll_params* kp, uint32_t* tcap_t, size_t* lds_t) {
    *tcap_t = (uint32_t)kp->tail + kKllTailSlack + KRR_KLL_TAIL_ROOM;
    const size_t body_t = ((size_t)kKllHdr + kp->budget) * 8 + (size_t)kp->budget;
    *lds_t = (size_t)*tcap_t * 8 > body_t ? (size_t)*tcap_t * 8 : body_t;
}

static int kll_tail_launch(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, uint64_t* rows,
                           hipStream_t st) {
    uint32_t tcap_t;
    size_t lds_t;
    kll_tail_lds(kp, &tcap_t, &lds_t);
    const double two_ln = (kp->reserved & KRR_KLL_TAIL_NO_MARGIN) ? 0.0 : 2.0 * log(4.0 / 1e-3);
    KllTailArgs T{series->values, series->offsets, series->n_segments, kp->budget, kp->tail, tcap_t, two_ln, rows,
                  nullptr, 0, nullptr};
    hipLaunchKernelGGL(k_kll_tail, dim3(grid_for(series->n_segments)), dim3(64), lds_t, st, T);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

static int kll_build_common(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, int64_t seg_base,
                            uint64_t* rows, uint32_t* lines, int64_t line_stride, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    if (krr_kll_row_words(kp) < 0)
        return set_err(ctx, KRR_E_INVALID, "kll: budget in [256, 4096] (a multiple of 64), tail in [0, 4096]%s", "");
    if (seg_base < 0) return set_err(ctx, KRR_E_INVALID, "negative seg_base%s", "");
    const int64_t S = series->n_segments;
    if (S == 0) return KRR_OK;
    if (!rows) return set_err(ctx, KRR_E_INVALID, "null rows%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    int64_t maxlen = 0;
    rc = resolve_maxlen(ctx, series, (hipStream_t)stream, &maxlen);
    if (rc) return rc;
    const int nrl = kll_run_levels(maxlen);
    if (kKllFirstRun + nrl > kKllLevels - 1)
        return set_err(ctx, KRR_E_UNSUPPORTED, "kll: segments of %s%lld slots need more run levels", "",
                       (long long)maxlen);
    // tail > 0: by default the build leaves the tail to k_kll_tail (a second pass over the
    // slice, candidates above a threshold read from the row's body; KRR_KLL_BODY_ONLY: the
    // caller launches it, krr_kll_tail); KRR_KLL_ONE_PASS_TAIL keeps the running tail buffer
    // inside the build.  The rows are the same either way.
    const bool one_pass = kp->tail > 0 && (kp->reserved & KRR_KLL_ONE_PASS_TAIL);
    const bool tail_pass = kp->tail > 0 && !one_pass;
    const uint32_t tcap = kll_tcap(one_pass ? kp->tail : 0);
    const size_t lds = kll_build_lds(nrl, tcap);
    if (lds > ctx->max_lds) return set_err(ctx, KRR_E_CAPACITY, "kll build needs %s%lld B of LDS", "", (long long)lds);
    uint32_t tcap_t;
    size_t lds_t;
    kll_tail_lds(kp, &tcap_t, &lds_t);
    if (tail_pass && lds_t > ctx->max_lds)
        return set_err(ctx, KRR_E_CAPACITY, "kll tail pass needs %s%lld B of LDS", "", (long long)lds_t);
    if (lines) {  // the body-only build that also writes the line maxima (krr_kll_build_lines)
        if (!tail_pass) return set_err(ctx, KRR_E_INVALID, "kll line maxima need tail > 0 and the tail pass%s", "");
        if (line_stride < krr_kll_line_words(maxlen))
            return set_err(ctx, KRR_E_INVALID, "line_stride below krr_kll_line_words(max_segment_len) = %s%lld", "",
                           (long long)krr_kll_line_words(maxlen));
    }
    KllBuildArgs A{series->values, series->offsets, S, series->gaps_are_nan, kp->budget, kp->tail, nrl, tcap,
                   (uint32_t)kp->slice, kp->seed, seg_base, rows, tail_pass ? 1 : 0, lines, line_stride};
    if (lines) {
        hipLaunchKernelGGL((k_kll_build<false, true>), dim3(grid_for(S)), dim3(64), lds, (hipStream_t)stream, A);
        KRR_HIP(ctx, hipGetLastError());
        return KRR_OK;
    }
    if (one_pass)
        hipLaunchKernelGGL(k_kll_build<true>, dim3(grid_for(S)), dim3(64), lds, (hipStream_t)stream, A);
    else
        hipLaunchKernelGGL(k_kll_build<false>, dim3(grid_for(S)), dim3(64), lds, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    if (tail_pass && !(kp->reserved & KRR_KLL_BODY_ONLY)) return kll_tail_launch(ctx, series, kp, rows, (hipStream_t)stream);
    return KRR_OK;
}

int krr_kll_build(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, int64_t seg_base,
                  uint64_t* rows, void* stream) {
    return kll_build_common(ctx, series, kp, seg_base, rows, nullptr, 0, stream);
}

int64_t krr_kll_line_words(int64_t max_segment_len) {
    if (max_segment_len < 0) return -1;
    const int64_t nch = max_segment_len / ((int64_t)kUnroll * kWave * 2) + 2;  // 1,024-slot chunks, head/tail
    return 64 * ((nch + 7) & ~(int64_t)7);  // the build streams a multiple of 8 chunks
}

int krr_kll_build_lines(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, int64_t seg_base,
                        uint64_t* rows, uint32_t* lines, int64_t line_stride, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (!lines) return set_err(ctx, KRR_E_INVALID, "null lines%s", "");
    return kll_build_common(ctx, series, kp, seg_base, rows, lines, line_stride, stream);
}

int krr_kll_tail_lines(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, uint64_t* rows,
                       const uint32_t* lines, int64_t line_stride, uint32_t* lines_read, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    if (krr_kll_row_words(kp) < 0)
        return set_err(ctx, KRR_E_INVALID, "kll: budget in [256, 4096] (a multiple of 64), tail in [0, 4096]%s", "");
    if (series->n_segments == 0 || kp->tail == 0) return KRR_OK;
    if (!rows || !lines) return set_err(ctx, KRR_E_INVALID, "null rows / lines%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    int64_t maxlen = 0;
    rc = resolve_maxlen(ctx, series, (hipStream_t)stream, &maxlen);
    if (rc) return rc;
    if (line_stride < krr_kll_line_words(maxlen))
        return set_err(ctx, KRR_E_INVALID, "line_stride below krr_kll_line_words(max_segment_len) = %s%lld", "",
                       (long long)krr_kll_line_words(maxlen));
    uint32_t tcap_t;
    size_t lds_t;
    kll_tail_lds(kp, &tcap_t, &lds_t);
    const uint32_t qoff = (uint32_t)((lds_t + 15) & ~(size_t)15);
    const size_t lds = (size_t)qoff + 128 * sizeof(uint32_t);
    if (lds > ctx->max_lds)
        return set_err(ctx, KRR_E_CAPACITY, "kll tail pass needs %s%lld B of LDS", "", (long long)lds);
    const double two_ln = (kp->reserved & KRR_KLL_TAIL_NO_MARGIN) ? 0.0 : 2.0 * log(4.0 / 1e-3);
    KllLineTailArgs LA{{series->values, series->offsets, series->n_segments, kp->budget, kp->tail, tcap_t, two_ln, rows,
                        lines, line_stride, nullptr},
                       qoff, lines_read};
    hipLaunchKernelGGL(k_kll_tail_lines, dim3(grid_for(series->n_segments)), dim3(64), lds, (hipStream_t)stream, LA);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_kll_tail(krr_ctx* ctx, const krr_series* series, const krr_kll_params* kp, uint64_t* rows, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    if (krr_kll_row_words(kp) < 0)
        return set_err(ctx, KRR_E_INVALID, "kll: budget in [256, 4096] (a multiple of 64), tail in [0, 4096]%s", "");
    if (series->n_segments == 0 || kp->tail == 0) return KRR_OK;
    if (!rows) return set_err(ctx, KRR_E_INVALID, "null rows%s", "");
    uint32_t tcap_t;
    size_t lds_t;
    kll_tail_lds(kp, &tcap_t, &lds_t);
    if (lds_t > ctx->max_lds)
        return set_err(ctx, KRR_E_CAPACITY, "kll tail pass needs %s%lld B of LDS", "", (long long)lds_t);
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    return kll_tail_launch(ctx, series, kp, rows, (hipStream_t)stream);
}

static int kll_merge_common(krr_ctx* ctx, int64_t n_series, int32_t rows_per_series, const uint64_t* rows,
                            const krr_kll_params* kp, int64_t series_base, bool query, size_t* lds) {
    if (krr_kll_row_words(kp) < 0)
        return set_err(ctx, KRR_E_INVALID, "kll: budget in [256, 4096] (a multiple of 64), tail in [0, 4096]%s", "");
    if (n_series < 0 || rows_per_series < 1 || series_base < 0)
        return set_err(ctx, KRR_E_INVALID, "bad n_series / rows_per_series / series_base%s", "");
    if (n_series && !rows) return set_err(ctx, KRR_E_INVALID, "null rows%s", "");
    // a query over one row per series folds nothing: k_kll_query stages the body alone
    *lds = (query && rows_per_series == 1) ? ((size_t)kKllHdr + kp->budget) * 8 + (size_t)kp->budget
                                           : kll_merge_lds(kp, query);
    if (*lds > ctx->max_lds)
        return set_err(ctx, KRR_E_CAPACITY, "kll %s needs %lld B of LDS",
                       (query && rows_per_series == 1) ? "query of one row" : "fold of rows this wide",
                       (long long)*lds);
    return KRR_OK;
}

int krr_kll_merge(krr_ctx* ctx, int64_t n_series, int32_t rows_per_series, const uint64_t* rows,
                  const krr_kll_params* kp, int64_t series_base, uint64_t* out_rows, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    size_t lds = 0;
    int rc = kll_merge_common(ctx, n_series, rows_per_series, rows, kp, series_base, false, &lds);
    if (rc) return rc;
    if (n_series == 0) return KRR_OK;
    if (!out_rows) return set_err(ctx, KRR_E_INVALID, "null out_rows%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    KllMergeArgs A{n_series, rows_per_series, kp->budget, kp->tail, (uint32_t)kp->slice, kp->seed, series_base, rows,
                   out_rows, 0, 0, 1, 0.0, nullptr, nullptr, nullptr};
    hipLaunchKernelGGL(k_kll_merge, dim3(grid_for(n_series)), dim3(64), lds, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_kll_query(krr_ctx* ctx, int64_t n_series, int32_t rows_per_series, const uint64_t* rows,
                  const krr_kll_params* kp, int64_t series_base, const krr_percentile_params* params,
                  double* out_value, int64_t* out_count, uint32_t* out_flags, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_params(ctx, params);
    if (rc) return rc;
    if (params->mode == KRR_PCT_REF_INDEX)
        return set_err(ctx, KRR_E_UNSUPPORTED, "REF_INDEX has no sketch form: use krr_select_present%s", "");
    size_t lds = 0;
    rc = kll_merge_common(ctx, n_series, rows_per_series, rows, kp, series_base, true, &lds);
    if (rc) return rc;
    if (n_series == 0) return KRR_OK;
    if (!out_value || !out_count || !out_flags) return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    KllMergeArgs A{n_series, rows_per_series, kp->budget, kp->tail, (uint32_t)kp->slice, kp->seed, series_base, rows,
                   nullptr, params->mode, params->p_num, params->p_den, params->q, out_value, out_count, out_flags,
                   params->k_table, params->k_table_len};
    hipLaunchKernelGGL(k_kll_query, dim3(grid_for(n_series)), dim3(64), lds, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_sketch_locate(krr_ctx* ctx, int64_t n_segments, const uint32_t* counts, const krr_sketch_params* sp,
                      const krr_percentile_params* params, krr_sketch_loc* out, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_params(ctx, params);
    if (rc) return rc;
    if (params->mode == KRR_PCT_REF_INDEX)
        return set_err(ctx, KRR_E_UNSUPPORTED, "REF_INDEX has no sketch form: use krr_select_present%s", "");
    if (krr_sketch_width(sp) < 0) return set_err(ctx, KRR_E_INVALID, "bad sketch params%s", "");
    if (n_segments < 0) return set_err(ctx, KRR_E_INVALID, "negative n_segments%s", "");
    if (n_segments == 0) return KRR_OK;
    if (!counts || !out) return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    SketchLocateArgs A{n_segments, sketch_geom(*sp), counts, params->mode, params->p_num, params->p_den, params->q,
                       out, params->k_table, params->k_table_len};
    hipLaunchKernelGGL(k_sketch_locate, dim3(grid_for(n_segments)), dim3(64), 0, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_sketch_range_count(krr_ctx* ctx, int64_t n_segments, const uint32_t* counts, const krr_sketch_params* sp,
                           const krr_sketch_loc* loc, int64_t* out, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    const int64_t W = krr_sketch_width(sp);
    if (W < 0) return set_err(ctx, KRR_E_INVALID, "bad sketch params%s", "");
    if (n_segments < 0) return set_err(ctx, KRR_E_INVALID, "negative n_segments%s", "");
    if (n_segments == 0) return KRR_OK;
    if (!counts || !loc || !out) return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipLaunchKernelGGL(k_sketch_range_count, dim3(grid_for(n_segments)), dim3(64), 0, (hipStream_t)stream,
                       n_segments, (uint32_t)W, counts, loc, out);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_sketch_collect(krr_ctx* ctx, const krr_series* series, const krr_sketch_params* sp,
                       const krr_sketch_loc* loc, const int64_t* out_offsets, double* out_values,
                       int64_t* out_count, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    if (krr_sketch_width(sp) < 0) return set_err(ctx, KRR_E_INVALID, "bad sketch params%s", "");
    const int64_t S = series->n_segments;
    if (S == 0) return KRR_OK;
    if (!loc || !out_offsets) return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipLaunchKernelGGL(k_sketch_collect, dim3(grid_for(S)), dim3(64), 0, (hipStream_t)stream, series->values,
                       series->offsets, S, sketch_geom(*sp), loc, out_offsets, out_values, out_count);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_sketch_refine(krr_ctx* ctx, const krr_series* collected, const krr_sketch_loc* loc, double* out_value,
                      int64_t* out_count, uint32_t* out_flags, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, collected);
    if (rc) return rc;
    const int64_t S = collected->n_segments;
    if (S == 0) return KRR_OK;
    if (!loc || !out_value || !out_count || !out_flags) return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    SketchRefineArgs A{collected->values, collected->offsets, S, loc, out_value, out_count, out_flags};
    hipLaunchKernelGGL(k_sketch_refine, dim3(grid_for(S)), dim3(64), 0, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_rank_of(krr_ctx* ctx, const krr_series* series, const double* values, int64_t* out_lt, int64_t* out_le,
                void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    const int64_t S = series->n_segments;
    if (S == 0) return KRR_OK;
    if (!values || !out_lt || !out_le) return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipLaunchKernelGGL(k_rank_of, dim3(grid_for(S)), dim3(64), 0, (hipStream_t)stream, series->values,
                       series->offsets, S, values, out_lt, out_le);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_select_present(krr_ctx* ctx, const krr_series* series, const int64_t* k, double* out, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    const int64_t S = series->n_segments;
    if (S == 0) return KRR_OK;
    if (!k || !out) return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipLaunchKernelGGL(k_select_present, dim3(grid_for(S)), dim3(64), 0, (hipStream_t)stream, series->values,
                       series->offsets, S, series->gaps_are_nan, k, out);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_locate(krr_ctx* ctx, const krr_series* series, const double* values, const int64_t* rank, int64_t* out_lt,
               int64_t* out_eq, int64_t* out_pos, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, series);
    if (rc) return rc;
    const int64_t S = series->n_segments;
    if (S == 0) return KRR_OK;
    if (!values || !rank || !out_lt || !out_eq || !out_pos) return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    if (series->max_segment_len > (int64_t)UINT32_MAX)
        return set_err(ctx, KRR_E_UNSUPPORTED, "krr_locate counts in 32 bits%s: segment of %lld slots", "",
                       (long long)series->max_segment_len);
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipLaunchKernelGGL(k_locate, dim3(grid_for(S)), dim3(64), 0, (hipStream_t)stream, series->values,
                       series->offsets, S, values, rank, out_lt, out_eq, out_pos);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int64_t krr_window_key_cap(int64_t max_slice_len, int64_t ext_slots, const krr_percentile_params* params) {
    if (max_slice_len < 0 || ext_slots < 0 || check_params(nullptr, params) != KRR_OK ||
        params->mode == KRR_PCT_REF_INDEX)
        return 0;
    const double q = (double)params->p_num / (100.0 * (double)params->p_den);
    const double L = (double)max_slice_len, U = (double)ext_slots;
    const double sig = (L > 0 && U > 0) ? sqrt(q * (1.0 - q) * L * U / (L + U)) : 0.0;
    // export_shrink keeps ranks [c - w, c + w + 1] (w = z sig + 4): 2w + 2 keys, plus
    // room for keys equal to the bounds
    int64_t keys = 2 * (int64_t)ceil(KRR_WEXP_Z * sig + 4.0) + 2 + 64;
    keys = (keys + 63) & ~(int64_t)63;
    return keys;
}

int krr_window_export(krr_ctx* ctx, const krr_series* slices, const krr_percentile_params* params,
                      int64_t ext_slots, int64_t key_cap, krr_window_hdr* hdr, uint64_t* keys, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_series(ctx, slices);
    if (!rc) rc = check_params(ctx, params);
    if (rc) return rc;
    if (params->mode == KRR_PCT_REF_INDEX)
        return set_err(ctx, KRR_E_UNSUPPORTED, "REF_INDEX has no window form: use krr_select_present%s", "");
    if (ext_slots < 0 || key_cap < 1 || key_cap > (int64_t)kWselCapLong)
        return set_err(ctx, KRR_E_INVALID, "window export: ext_slots >= 0, 1 <= key_cap <= %s%lld", "",
                       (long long)kWselCapLong);
    const int64_t S = slices->n_segments;
    if (S == 0) return KRR_OK;
    if (!hdr || !keys) return set_err(ctx, KRR_E_INVALID, "null outputs%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipStream_t st = (hipStream_t)stream;
    int64_t Lmax = 0;
    rc = resolve_maxlen(ctx, slices, st, &Lmax);
    if (rc) return rc;
    WindowExportArgs X{};
    X.A.vals = slices->values;
    X.A.offs = slices->offsets;
    X.A.S = S;
    X.A.remap = Lmax < KRR_XCD_REMAP_MAXLEN ? 1 : 0;
    X.A.mode = params->mode;
    X.A.gaps = slices->gaps_are_nan;
    X.A.p_num = params->p_num;
    X.A.p_den = params->p_den;
    X.A.q = params->q;
    X.A.ktab = params->k_table;
    X.A.ktab_len = params->k_table_len;
    X.A.wcap = wsel_cap_for(Lmax, slices->gaps_are_nan != 0);
    X.ext = (double)ext_slots;
    X.key_cap = (uint32_t)key_cap;
    X.hdr = hdr;
    X.keys = keys;
    const size_t lds = kSelectLdsFixed + (size_t)X.A.wcap * 8;
    if (lds > ctx->max_lds) return set_err(ctx, KRR_E_CAPACITY, "window export needs %s%lld B of LDS", "", (long long)lds);
    if (X.A.wcap == kWselCapLong) hipLaunchKernelGGL(k_window_export<true>, dim3(grid_for(S)), dim3(64), lds, st, X);
    else hipLaunchKernelGGL(k_window_export<false>, dim3(grid_for(S)), dim3(64), lds, st, X);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_window_merge(krr_ctx* ctx, int64_t n_series, int32_t n_slices, int64_t slice_stride,
                     const krr_window_hdr* hdr, const uint64_t* keys, int64_t key_cap,
                     const krr_percentile_params* params, double* out_value, int64_t* out_count,
                     uint32_t* out_flags, uint32_t* miss_count, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    int rc = check_params(ctx, params);
    if (rc) return rc;
    if (params->mode == KRR_PCT_REF_INDEX)
        return set_err(ctx, KRR_E_UNSUPPORTED, "REF_INDEX has no window form: use krr_select_present%s", "");
    if (n_series < 0 || n_slices < 1 || n_slices > kWave || slice_stride < n_series || key_cap < 1 ||
        key_cap > (int64_t)kWselCapLong)
        return set_err(ctx, KRR_E_INVALID, "window merge: 1 <= n_slices <= 64, slice_stride >= n_series, "
                       "1 <= key_cap <= %s%lld", "", (long long)kWselCapLong);
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipStream_t st = (hipStream_t)stream;
    if (miss_count) KRR_HIP(ctx, hipMemsetAsync(miss_count, 0, sizeof(uint32_t), st));
    if (n_series == 0) return KRR_OK;
    if (!hdr || !keys || !out_value || !out_count || !out_flags) return set_err(ctx, KRR_E_INVALID, "null pointers%s", "");
    const size_t lds = kSelectLdsFixed + (size_t)n_slices * (size_t)key_cap * 8;
    if (lds > ctx->max_lds)
        return set_err(ctx, KRR_E_CAPACITY, "window merge needs %s%lld B of LDS (n_slices x key_cap keys)", "",
                       (long long)lds);
    WindowMergeArgs M{};
    M.A.S = n_series;
    M.A.mode = params->mode;
    M.A.p_num = params->p_num;
    M.A.p_den = params->p_den;
    M.A.q = params->q;
    M.A.ktab = params->k_table;
    M.A.ktab_len = params->k_table_len;
    M.A.out_v = out_value;
    M.A.out_n = out_count;
    M.A.out_f = out_flags;
    M.slices = n_slices;
    M.stride = slice_stride;
    M.hdr = hdr;
    M.keys = keys;
    M.key_cap = key_cap;
    M.miss_count = miss_count;
    hipLaunchKernelGGL(k_window_merge, dim3(grid_for(n_series)), dim3(64), lds, st, M);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_get_stats(krr_ctx* ctx, int64_t* wselect_fallbacks) {
    if (!ctx || !wselect_fallbacks) return KRR_E_INVALID;
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    unsigned long long h = 0;
    KRR_HIP(ctx, hipDeviceSynchronize());
    KRR_HIP(ctx, hipMemcpy(&h, ctx->d_tmp + 1, sizeof(h), hipMemcpyDeviceToHost));
    *wselect_fallbacks = (int64_t)h;
    return KRR_OK;
}

int krr_json_parse(krr_ctx* ctx, const krr_json_bodies* b, int64_t first, int64_t n, int32_t want_timestamps,
                   double* scratch_values, double* scratch_ts, int64_t* counts, int32_t* status, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (!b || b->n_bodies < 0 || first < 0 || n < 0 || first + n > b->n_bodies)
        return set_err(ctx, KRR_E_INVALID, "json: bad body range%s", "");
    if (n == 0) return KRR_OK;
    if (!b->bodies || !b->body_offsets || !scratch_values || !counts || !status || (want_timestamps && !scratch_ts))
        return set_err(ctx, KRR_E_INVALID, "json: null buffer%s", "");
    if (((uintptr_t)b->bodies & 15) != 0) return set_err(ctx, KRR_E_INVALID, "json: bodies not 16-byte aligned%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    json::JsonArgs A{b->bodies, b->body_offsets, first, n, want_timestamps ? 1 : 0, scratch_values,
                     want_timestamps ? scratch_ts : nullptr, counts, status};
    hipLaunchKernelGGL(json::k_json_parse, dim3(grid_for(n)), dim3(64), 0, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_json_compact(krr_ctx* ctx, const krr_json_bodies* b, const double* scratch_values,
                     const double* scratch_ts, const int64_t* counts, const int32_t* status,
                     const int64_t* out_pos, double* values, double* timestamps, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (!b || b->n_bodies < 0) return set_err(ctx, KRR_E_INVALID, "json: bad bodies%s", "");
    if (b->n_bodies == 0) return KRR_OK;
    if (!b->body_offsets || !scratch_values || !counts || !status || !out_pos || !values ||
        (timestamps && !scratch_ts))
        return set_err(ctx, KRR_E_INVALID, "json: null buffer%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    json::CompactArgs C{b->body_offsets, counts, status, out_pos, scratch_values, timestamps ? scratch_ts : nullptr,
                        values, timestamps, b->n_bodies};
    const int64_t grid = b->n_bodies < 65536 ? b->n_bodies : 65536;
    hipLaunchKernelGGL(json::k_json_compact, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, C);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_copy_h2d_batch(krr_ctx* ctx, int64_t n, void* const* dst, const void* const* src, const int64_t* bytes,
                       void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (n < 0 || (n > 0 && (!dst || !src || !bytes))) return set_err(ctx, KRR_E_INVALID, "copy: bad batch%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    for (int64_t i = 0; i < n; ++i) {
        if (bytes[i] < 0 || (bytes[i] > 0 && (!dst[i] || !src[i])))
            return set_err(ctx, KRR_E_INVALID, "copy: bad entry %s%lld", "", (long long)i);
        if (bytes[i] == 0) continue;
        KRR_HIP(ctx, hipMemcpyAsync(dst[i], src[i], (size_t)bytes[i], hipMemcpyHostToDevice, (hipStream_t)stream));
    }
    return KRR_OK;
}

int krr_json_find_series(krr_ctx* ctx, const krr_json_bodies* b, int64_t begin, int64_t end, int64_t limit,
                         int64_t* candidates, int64_t cap, uint64_t* n_candidates, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (!b || b->n_bodies < 0 || b->total_bytes < 0 || cap < 0 || begin < 0 || end > b->total_bytes ||
        limit > b->total_bytes || end > limit)
        return set_err(ctx, KRR_E_INVALID, "json: bad bodies or byte range%s", "");
    if (end <= begin) return KRR_OK;
    if (!b->bodies || !candidates || !n_candidates) return set_err(ctx, KRR_E_INVALID, "json: null buffer%s", "");
    if (((uintptr_t)b->bodies & 15) != 0) return set_err(ctx, KRR_E_INVALID, "json: bodies not 16-byte aligned%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    json::FindArgs F{b->bodies, begin, end, limit, candidates, cap, (unsigned long long*)n_candidates};
    const int64_t blocks = (end - (begin & ~(int64_t)15) + 4095) / 4096;
    hipLaunchKernelGGL(json::k_json_find_series, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(64), 0,
                       (hipStream_t)stream, F);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

static int json_segments_launch(krr_ctx* ctx, const krr_json_bodies* b, const int64_t* starts,
                                const int64_t* body_of, int64_t n, const char* label, int32_t want_timestamps,
                                double* scratch_values, double* scratch_ts, int64_t* segments, int64_t* workspace,
                                int64_t workspace_words, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (!b || n < 0) return set_err(ctx, KRR_E_INVALID, "json: bad arguments%s", "");
    if (!label) return set_err(ctx, KRR_E_INVALID, "json: null label%s", "");
    const size_t ll = strlen(label);
    if (ll >= (size_t)json::kMaxLabel) return set_err(ctx, KRR_E_INVALID, "json: label longer than 63 bytes%s", "");
    if (n == 0) return KRR_OK;
    if (!b->bodies || !b->body_offsets || !starts || !body_of || !scratch_values || !segments ||
        (want_timestamps && !scratch_ts))
        return set_err(ctx, KRR_E_INVALID, "json: null buffer%s", "");
    int64_t parts_cap = 0;
    if (workspace) {
        parts_cap = (workspace_words - 1 - n) / json::kPartWords;
        if (parts_cap < 1)
            return set_err(ctx, KRR_E_INVALID, "json: workspace of %s%lld words holds no part", "",
                           (long long)workspace_words);
    }
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipStream_t st = (hipStream_t)stream;
    // the label travels in the kernel arguments: a pageable hipMemcpyAsync here stalled the
    // calling thread behind the stream's earlier work (and raced across parse streams)
    json::SegArgs A{b->bodies, b->body_offsets, starts, body_of, n, want_timestamps ? 1 : 0, (int32_t)ll,
                    {}, scratch_values, want_timestamps ? scratch_ts : nullptr, segments,
                    nullptr, 0, nullptr, nullptr};
    memcpy(A.label_w, label, ll);
    if (workspace) {
        A.n_parts = (unsigned long long*)workspace;
        A.series_vend = workspace + 1;
        A.parts = workspace + 1 + n;
        A.parts_cap = parts_cap;
        KRR_HIP(ctx, hipMemsetAsync(workspace, 0, sizeof(int64_t), st));
    }
    hipLaunchKernelGGL(json::k_json_segments, dim3(grid_for(n)), dim3(64), 0, st, A);
    KRR_HIP(ctx, hipGetLastError());
    if (workspace) {
        json::PartArgs P{b->bodies, A.parts, A.n_parts, A.series_vend, parts_cap, want_timestamps ? 1 : 0,
                         scratch_values, want_timestamps ? scratch_ts : nullptr, segments};
        const int64_t grid = parts_cap < 8192 ? parts_cap : 8192;  // grid-stride past that
        hipLaunchKernelGGL(json::k_json_value_parts, dim3((unsigned)grid), dim3(64), 0, st, P);
        KRR_HIP(ctx, hipGetLastError());
    }
    return KRR_OK;
}

int krr_json_parse_segments(krr_ctx* ctx, const krr_json_bodies* b, const int64_t* starts, const int64_t* body_of,
                            int64_t n, const char* label, int32_t want_timestamps, double* scratch_values,
                            double* scratch_ts, int64_t* segments, void* stream) {
    return json_segments_launch(ctx, b, starts, body_of, n, label, want_timestamps, scratch_values, scratch_ts,
                                segments, nullptr, 0, stream);
}

int krr_json_parse_segments_split(krr_ctx* ctx, const krr_json_bodies* b, const int64_t* starts,
                                  const int64_t* body_of, int64_t n, const char* label, int32_t want_timestamps,
                                  double* scratch_values, double* scratch_ts, int64_t* segments, int64_t* workspace,
                                  int64_t workspace_words, void* stream) {
    if (ctx && !workspace) return set_err(ctx, KRR_E_INVALID, "json: null workspace%s", "");
    return json_segments_launch(ctx, b, starts, body_of, n, label, want_timestamps, scratch_values, scratch_ts,
                                segments, workspace, workspace_words, stream);
}

int krr_json_gather(krr_ctx* ctx, int64_t n_items, const int64_t* src, const int64_t* count, const int64_t* dst,
                    const double* scratch_values, const double* scratch_ts, double* values, double* timestamps,
                    void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (n_items < 0) return set_err(ctx, KRR_E_INVALID, "json: negative item count%s", "");
    if (n_items == 0) return KRR_OK;
    if (!src || !count || !dst || !scratch_values || !values || (timestamps && !scratch_ts))
        return set_err(ctx, KRR_E_INVALID, "json: null buffer%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    json::GatherArgs G{src, count, dst, scratch_values, timestamps ? scratch_ts : nullptr, values, timestamps, n_items};
    const int64_t grid = n_items < 65536 ? n_items : 65536;
    hipLaunchKernelGGL(json::k_json_gather, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, G);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_select_plan(int64_t max_segment_len, const krr_percentile_params* params, krr_select_plan_info* out) {
    if (!out || max_segment_len < 0) return KRR_E_INVALID;
    int rc = check_params(nullptr, params);
    if (rc) return rc;
    *out = krr_select_plan_info{};
    if (params->mode == KRR_PCT_REF_INDEX) return KRR_E_UNSUPPORTED;  // no selection: an index walk
    const int64_t Lmax = max_segment_len > 0 ? max_segment_len : 1;
    const SidePlan sp = plan_side(Lmax, params->mode, params->p_num, params->p_den, params->q,
                                  params->k_table != nullptr);
    const uint32_t need = capacity_for(sp.tkeep);
    const bool hsel = window_select(need, sp.tkeep, Lmax, sp.bottom, false);
    out->hselect = hsel ? 1 : 0;
    out->fused_hselect = window_select(need, sp.tkeep, Lmax, sp.bottom, true) ? 1 : 0;
    out->bottom = (int32_t)sp.bottom;
    out->tkeep = sp.tkeep;
    out->cap_keys = hsel ? 0 : need;
    out->lds_bytes = (int64_t)kSelectLdsFixed +
                     (int64_t)(hsel ? (KRR_WSEL ? window_lds(wsel_cap_for(Lmax)) : kHselectLds) : (size_t)need * 8);
#if KRR_SELECT_PROBE
    out->probe = (!hsel && !sp.bottom && select_probe_pays(Lmax, sp.tkeep, need)) ? 1 : 0;
#endif
    return KRR_OK;
}

}  // extern "C"

// ---- RCCL, resolved at run time --------------------------------------------
// The process may already hold a librccl.so.1 (PyTorch's); binding to that copy
// keeps communicators created by torch.distributed valid here.  Otherwise ROCm's
// is loaded (this library's RUNPATH holds /opt/rocm/lib).
namespace {
struct RcclApi {
    bool ok = false;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclCommUserRank) comm_user_rank = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;  // optional: nonblocking communicators
    decltype(&ncclCommInitRankConfig) init_config = nullptr;  // optional: bounded init
    decltype(&ncclCommAbort) abort = nullptr;
};

const RcclApi& rccl() {
    static const RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return a;
        bool all = true;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            all = all && fp != nullptr;
        };
        sym(a.get_unique_id, "ncclGetUniqueId");
        sym(a.comm_init_rank, "ncclCommInitRank");
        sym(a.comm_destroy, "ncclCommDestroy");
        sym(a.comm_count, "ncclCommCount");
        sym(a.comm_user_rank, "ncclCommUserRank");
        sym(a.send, "ncclSend");
        sym(a.recv, "ncclRecv");
        sym(a.group_start, "ncclGroupStart");
        sym(a.group_end, "ncclGroupEnd");
        sym(a.error_string, "ncclGetErrorString");
        a.ok = all;
        a.async_error = reinterpret_cast<decltype(a.async_error)>(dlsym(h, "ncclCommGetAsyncError"));
        a.init_config = reinterpret_cast<decltype(a.init_config)>(dlsym(h, "ncclCommInitRankConfig"));
        a.abort = reinterpret_cast<decltype(a.abort)>(dlsym(h, "ncclCommAbort"));
        return a;
    }();
    return api;
}

int nccl_err(krr_ctx* ctx, const char* what, ncclResult_t r) {
    return set_err(ctx, KRR_E_HIP, "RCCL %s failed (%lld)", what, (long long)r);
}
}  // namespace

extern "C" {

int krr_comm_unique_id(krr_ctx* ctx, void* unique_id) {
    if (!ctx) return KRR_E_INVALID;
    if (!unique_id) return set_err(ctx, KRR_E_INVALID, "null unique_id%s", "");
    const RcclApi& R = rccl();
    if (!R.ok) return set_err(ctx, KRR_E_UNSUPPORTED, "librccl.so.1 not loadable%s", "");
    ncclUniqueId id;
    const ncclResult_t r = R.get_unique_id(&id);
    if (r != ncclSuccess) return nccl_err(ctx, "ncclGetUniqueId", r);
    memcpy(unique_id, &id, sizeof(id));
    return KRR_OK;
}

int krr_comm_init(krr_ctx* ctx, int nranks, const void* unique_id, int rank, void** out_comm) {
    if (!ctx) return KRR_E_INVALID;
    if (!unique_id || !out_comm || nranks < 1 || rank < 0 || rank >= nranks)
        return set_err(ctx, KRR_E_INVALID, "bad comm arguments%s", "");
    *out_comm = nullptr;
    const RcclApi& R = rccl();
    if (!R.ok) return set_err(ctx, KRR_E_UNSUPPORTED, "librccl.so.1 not loadable%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = R.comm_init_rank(&comm, nranks, id, rank);
    if (r != ncclSuccess) return nccl_err(ctx, "ncclCommInitRank", r);
    *out_comm = comm;
    return KRR_OK;
}

int krr_comm_init_timeout(krr_ctx* ctx, int nranks, const void* unique_id, int rank, double timeout_s,
                          void** out_comm) {
    if (timeout_s <= 0) return krr_comm_init(ctx, nranks, unique_id, rank, out_comm);
    if (!ctx) return KRR_E_INVALID;
    if (!unique_id || !out_comm || nranks < 1 || rank < 0 || rank >= nranks)
        return set_err(ctx, KRR_E_INVALID, "bad comm arguments%s", "");
    *out_comm = nullptr;
    const RcclApi& R = rccl();
    if (!R.ok) return set_err(ctx, KRR_E_UNSUPPORTED, "librccl.so.1 not loadable%s", "");
    if (!R.init_config || !R.abort || !R.async_error)
        return set_err(ctx, KRR_E_UNSUPPORTED, "this RCCL has no nonblocking init%s", "");
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof(id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t comm = nullptr;
    ncclResult_t r = R.init_config(&comm, nranks, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) return nccl_err(ctx, "ncclCommInitRankConfig", r);
    timespec t0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (;;) {
        ncclResult_t st = ncclSuccess;
        r = R.async_error(comm, &st);
        if (r != ncclSuccess) st = r;
        if (st == ncclSuccess) break;
        if (st != ncclInProgress) {
            (void)R.abort(comm);
            return nccl_err(ctx, "ncclCommInitRankConfig", st);
        }
        timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        if ((double)(t.tv_sec - t0.tv_sec) + 1e-9 * (double)(t.tv_nsec - t0.tv_nsec) > timeout_s) {
            (void)R.abort(comm);
            return set_err(ctx, KRR_E_TIMEOUT, "ncclCommInitRankConfig: not every rank arrived within the timeout%s",
                           "");
        }
        usleep(1000);
    }
    *out_comm = comm;
    return KRR_OK;
}

int krr_comm_destroy(krr_ctx* ctx, void* comm) {
    if (!ctx) return KRR_E_INVALID;
    if (!comm) return KRR_OK;
    const RcclApi& R = rccl();
    if (!R.ok) return set_err(ctx, KRR_E_UNSUPPORTED, "librccl.so.1 not loadable%s", "");
    DeviceGuard g(ctx->device);
    const ncclResult_t r = R.comm_destroy((ncclComm_t)comm);
    return r == ncclSuccess ? KRR_OK : nccl_err(ctx, "ncclCommDestroy", r);
}

int krr_comm_info(krr_ctx* ctx, void* comm, int* nranks, int* rank) {
    if (!ctx) return KRR_E_INVALID;
    if (!comm || !nranks || !rank) return set_err(ctx, KRR_E_INVALID, "null comm / outputs%s", "");
    const RcclApi& R = rccl();
    if (!R.ok) return set_err(ctx, KRR_E_UNSUPPORTED, "librccl.so.1 not loadable%s", "");
    ncclResult_t r = R.comm_count((ncclComm_t)comm, nranks);
    if (r == ncclSuccess) r = R.comm_user_rank((ncclComm_t)comm, rank);
    return r == ncclSuccess ? KRR_OK : nccl_err(ctx, "ncclCommCount/UserRank", r);
}

int krr_gather_results(krr_ctx* ctx, void* comm, int root, const int64_t* records, int64_t n_local,
                       const int64_t* counts, int64_t* out, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (!comm || n_local < 0 || (n_local > 0 && !records))
        return set_err(ctx, KRR_E_INVALID, "bad gather arguments%s", "");
    const RcclApi& R = rccl();
    if (!R.ok) return set_err(ctx, KRR_E_UNSUPPORTED, "librccl.so.1 not loadable%s", "");
    ncclComm_t c = (ncclComm_t)comm;
    int nranks = 0, me = 0;
    ncclResult_t r = R.comm_count(c, &nranks);
    if (r == ncclSuccess) r = R.comm_user_rank(c, &me);
    if (r != ncclSuccess) return nccl_err(ctx, "ncclCommCount/UserRank", r);
    if (root < 0 || root >= nranks) return set_err(ctx, KRR_E_INVALID, "root %s%lld out of range", "", root);
    if (me == root) {
        if (!out) return set_err(ctx, KRR_E_INVALID, "null out on the root%s", "");
        if (counts && counts[root] != n_local)
            return set_err(ctx, KRR_E_INVALID, "counts[root] != n_local%s", "");
        for (int q = 0; q < nranks && counts; ++q)
            if (counts[q] < 0) return set_err(ctx, KRR_E_INVALID, "negative count for rank %s%lld", "", q);
    }
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    hipStream_t st = (hipStream_t)stream;
    constexpr size_t kWords = 4;  // int64 words per 32-B record
    r = R.group_start();
    if (r != ncclSuccess) return nccl_err(ctx, "ncclGroupStart", r);
    hipError_t he = hipSuccess;
    if (me == root) {
        int64_t off = 0;
        for (int q = 0; q < nranks; ++q) {
            const int64_t nq = counts ? counts[q] : n_local;
            if (nq > 0) {
                int64_t* dst = out + off * (int64_t)kWords;
                if (q == root) {
                    if (dst != records) he = hipMemcpyAsync(dst, records, (size_t)nq * kWords * 8,
                                                            hipMemcpyDeviceToDevice, st);
                } else if (r == ncclSuccess) {
                    r = R.recv(dst, (size_t)nq * kWords, ncclInt64, q, c, st);
                }
            }
            off += nq;
        }
    } else if (n_local > 0) {
        r = R.send(records, (size_t)n_local * kWords, ncclInt64, root, c, st);
    }
    ncclResult_t re = R.group_end();
    // A nonblocking communicator (ncclCommInitRankConfig with blocking = 0, e.g. PyTorch's
    // under TORCH_NCCL_USE_COMM_NONBLOCKING=1) may still be enqueueing when the group ends:
    // wait for its state to settle before the caller's next call on it.
    while (re == ncclInProgress && R.async_error) {
        ncclResult_t st = ncclSuccess;
        if (R.async_error(c, &st) != ncclSuccess) break;
        if (st != ncclInProgress) {
            re = st;
            break;
        }
        sched_yield();
    }
    if (he != hipSuccess) return set_err(ctx, KRR_E_HIP, "D2D copy failed: %s%lld", hipGetErrorString(he), 0);
    if (r != ncclSuccess) return nccl_err(ctx, "ncclSend/ncclRecv", r);
    if (re != ncclSuccess) return nccl_err(ctx, "ncclGroupEnd", re);
    return KRR_OK;
}

}  // extern "C"
