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

#include <new>

#include "krr_amd.h"
#include "krr_device.h"
#include "krr_plan.h"

#ifndef KRR_STREAM_DEPTH
#define KRR_STREAM_DEPTH 3  // chunks in flight per wave
#endif
#ifndef KRR_SELECT_WAVES_PER_SIMD
#define KRR_SELECT_WAVES_PER_SIMD 2  // __launch_bounds__ occupancy hint for k_select
#endif

namespace krr {

// ---------------------------------------------------------------------------
// Streaming skeleton.  One wave walks values[beg, end): the 16-byte aligned
// body in chunks of kUnroll x 16 B per lane (8 KiB per wave), three chunks in
// flight; the unaligned head/tail elements and the partial last chunk go
// through ONE guarded chunk call (the partial chunk never fills its last slot,
// so the head and tail elements ride in it).  A processor implements
//   template <bool GUARD> void chunk(const double2 (&c)[kUnroll], uint32_t vmask)
// where, with GUARD, bit (2u + h) of vmask says slot c[u].x (h=0) / .y (h=1)
// of this lane holds a sample.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_chunk(double2 (&c)[kUnroll], const double2* __restrict__ p) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) c[u] = p[u * kWave];
}

template <class Proc>
__device__ __forceinline__ void stream_segment(const double* __restrict__ vals, int64_t beg,
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
    if (nfull > 0) {
        const double2* __restrict__ p = v2 + i0 + lane;
        const int64_t last = nfull - 1;
        auto at = [&](int64_t c) { return p + (c < last ? c : last) * CH; };  // clamp: re-read, never overrun
#if KRR_STREAM_DEPTH == 2
        double2 b0[kUnroll], b1[kUnroll];
        load_chunk(b0, at(0));
        load_chunk(b1, at(1));
        for (int64_t c = 0; c < nfull; c += 2) {
            proc.template chunk<false>(b0, 0u);
            load_chunk(b0, at(c + 2));
            if (c + 1 < nfull) proc.template chunk<false>(b1, 0u);
            load_chunk(b1, at(c + 3));
        }
#else
        double2 b0[kUnroll], b1[kUnroll], b2[kUnroll];
        load_chunk(b0, at(0));
        load_chunk(b1, at(1));
        load_chunk(b2, at(2));
        for (int64_t c = 0; c < nfull; c += 3) {
            proc.template chunk<false>(b0, 0u);
            load_chunk(b0, at(c + 3));
            if (c + 1 < nfull) proc.template chunk<false>(b1, 0u);
            load_chunk(b1, at(c + 4));
            if (c + 2 < nfull) proc.template chunk<false>(b2, 0u);
            load_chunk(b2, at(c + 5));
        }
#endif
    }
    const int64_t r0 = nfull * CH;
    const bool head = a0 > beg, tail = a1 < end;
    if (r0 < nunits || head || tail) {
        double2 cur[kUnroll];
        uint32_t vmask = 0;
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t j = r0 + u * kWave + lane;
            const bool in = j < nunits;
            cur[u] = in ? v2[i0 + j] : make_double2(0.0, 0.0);
            vmask |= in ? (3u << (2 * u)) : 0u;
        }
        // nunits - r0 < CH, so the last slot (u = kUnroll-1, lane 63) is free
        if (lane == kWave - 1) {
            if (head) {
                cur[kUnroll - 1].x = vals[beg];
                vmask |= 1u << (2 * (kUnroll - 1));
            }
            if (tail) {
                cur[kUnroll - 1].y = vals[a1];
                vmask |= 2u << (2 * (kUnroll - 1));
            }
        }
        proc.template chunk<true>(cur, vmask);
    }
}

template <bool GUARD>
__device__ __forceinline__ bool slot_in(uint32_t vmask, int j) {
    return GUARD ? ((vmask >> j) & 1u) != 0 : true;
}

__device__ __forceinline__ double slot_val(const double2 (&c)[kUnroll], int j) {
    return (j & 1) ? c[j >> 1].y : c[j >> 1].x;
}

__device__ __forceinline__ uint32_t popc64(uint64_t m) { return (uint32_t)__popcll((long long)m); }

// ---------------------------------------------------------------------------
// MSD radix select over M = buf[0..cnt) U {xk repeated xc times}, in LDS or
// global scratch, by one wave.  Finds the R-th largest key (1-based):
// v with count(M > v) < R <= count(M >= v).  With `early`, it may stop at a
// digit-bin edge e > floor_key with count(M >= e) >= R and count(M > e) <= stop
// (good enough for a compaction threshold).  The first digit starts at the
// highest bit where min(M) and max(M) differ, so clustered keys (all samples
// in one binade) still split on their first level; <= 8 bits per level.
// Out of line: it is the rare fallback, and inlining it into every chunk call
// site costs registers and I-cache on the hot path.
// ---------------------------------------------------------------------------
struct SelHit {
    uint64_t key;
    uint32_t above;  // count(M > key)   (exact when !early)
    uint32_t ge;     // count(M >= key)  (upper bound when early-stopped)
    uint32_t ok;
};

__device__ __noinline__ SelHit select_desc(const uint64_t* buf, uint32_t cnt, uint64_t xk, uint32_t xc,
                                           uint32_t R, bool early, uint64_t floor_key, uint32_t stop,
                                           uint32_t* hist, int lane) {
    SelHit out;
    out.ok = 1;
    uint64_t mn = ~0ull, mx = 0;
    for (uint32_t i = lane; i < cnt; i += kWave) {
        const uint64_t x = buf[i];
        mn = x < mn ? x : mn;
        mx = x > mx ? x : mx;
    }
    mn = wave_min_u64(mn);
    mx = wave_max_u64(mx);
    if (xc) {
        mn = xk < mn ? xk : mn;
        mx = xk > mx ? xk : mx;
    }
    const uint32_t total = cnt + xc;
    if (R == 0 || R > total) {
        out.key = mx;
        out.above = 0;
        out.ge = total;
        out.ok = 0;
        return out;
    }
    uint64_t lo = mn, hi = mx;
    uint32_t above = 0, ge = total;
    while (lo != hi) {
        const int h = 63 - __clzll((long long)(lo ^ hi));
        const int s = h >= 7 ? h - 7 : 0;
        const uint32_t nb = 1u << (h - s + 1);
        const uint64_t pre = (h == 63) ? 0ull : ((lo >> (h + 1)) << (h + 1));
        for (uint32_t i = lane; i < 256; i += kWave) hist[i] = 0;
        __syncthreads();
        for (uint32_t i = lane; i < cnt; i += kWave) {
            const uint64_t x = buf[i];
            if (x >= lo && x <= hi) atomicAdd(&hist[(uint32_t)(x >> s) & (nb - 1)], 1u);
        }
        if (lane == 0 && xc && xk >= lo && xk <= hi) atomicAdd(&hist[(uint32_t)(xk >> s) & (nb - 1)], xc);
        __syncthreads();
        uint32_t hb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) hb[j] = hist[4 * lane + j];
        const uint32_t t = hb[0] + hb[1] + hb[2] + hb[3];
        const uint32_t incl = wave_suffix_incl(t, lane);
        uint32_t run = above + (incl - t);
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
        const int src = __ffsll((long long)m) - 1;
        const int b = __shfl(fb, src);
        const uint32_t ab = uni32((uint32_t)__shfl((int)fab, src));
        const uint32_t cb = uni32((uint32_t)__shfl((int)fcb, src));
        const uint64_t blo = pre | ((uint64_t)(uint32_t)b << s);
        const uint64_t bhi = blo | (s == 0 ? 0ull : ((1ull << s) - 1));
        const uint64_t nlo = uni64(blo > lo ? blo : lo);
        const uint64_t nhi = uni64(bhi < hi ? bhi : hi);
        __syncthreads();  // histogram reads done before the next level clears it
        if (early && nlo > floor_key && ab + cb <= stop) {
            out.key = nlo;
            out.above = ab;
            out.ge = ab + cb;
            return out;
        }
        lo = nlo;
        hi = nhi;
        above = ab;
        ge = ab + cb;
    }
    out.key = lo;
    out.above = above;
    out.ge = ge;
    return out;
}

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
    h.b = uni32((uint32_t)__shfl(fb, src));
    h.above = uni32((uint32_t)__shfl((int)fab, src));
    h.cnt = uni32((uint32_t)__shfl((int)fcb, src));
    return h;
}

// ---------------------------------------------------------------------------
// Threshold-filtered candidate buffer (one wave per segment).
//
// Invariant over the present non-NaN samples seen so far, in (possibly
// flipped) key order:  buf holds exactly those with key > thr, `eqs` counts
// those with key == thr, every other one is < thr ("below", implied by n).
// Before a chunk is inserted, its candidates are COUNTED (classify: a few VALU
// per sample, no branches, counts via ballot popcounts); if they do not fit,
// compact() raises thr so that at least tkeep keys stay >= thr and at most
// tstop = cap - kChunkElems stay > thr, then the chunk is re-classified and
// always fits.  The segment's needed ranks lie in its top tkeep keys
// (krr_plan.h), so they are never dropped.
//
// Fast path: once thr is a non-negative number t (top side), "key > thr" for a
// sample with bits x is the single unsigned range test
//   x - (bits(t)+1) < bits(+inf) - bits(t)
// which also rejects every NaN and every negative number.
//
// H is a 256-bin histogram of buf kept up to date on every insert (bins of
// width 2^hsh from hbase = thr + 1; bin 255 also takes everything above).  A
// compaction reads the new threshold off H and needs one filter pass over buf,
// which rebuilds H for the new range; select_desc is only the fallback when
// the cut falls into the overflow bin or a crowded bin.  The final rank
// queries use H the same way: locate the bin, gather its few members, rank
// them in registers.
// ---------------------------------------------------------------------------
struct SelectProc {
    uint64_t* buf;
    uint32_t* H;      // maintained histogram of buf
    uint32_t* scr;    // select_desc scratch histogram
    uint64_t* small;  // 64-key gather area
    int lane;
    uint32_t cap, tkeep, tstop;
    uint64_t flip;
    uint64_t thr;
    uint32_t cnt, eqs, nnan;
    uint64_t hbase;
    uint32_t hsh, hvalid;
    uint32_t fast;              // thr is a non-negative finite number or +0, top side
    uint64_t tbits, tb1, tlim;  // fast-path constants
    uint64_t mxk;               // per lane: largest key ever inserted
    uint32_t bad;

    __device__ __forceinline__ void set_thr(uint64_t t) {
        thr = uni64(t);
        fast = (!flip && (thr & kSignBit) && (thr ^ kSignBit) <= 0x7FF0000000000000ull) ? 1u : 0u;
        tbits = thr ^ kSignBit;
        tb1 = tbits + 1;
        tlim = 0x7FF0000000000000ull - tbits;
    }

    __device__ __forceinline__ uint32_t bin(uint64_t k) const {
        const uint64_t d = (k - hbase) >> hsh;
        return d > 255 ? 255u : (uint32_t)d;
    }

    template <bool GUARD, bool FAST>
    __device__ __forceinline__ bool is_cand(double d, uint32_t vmask, int j, uint64_t& key) const {
        const uint64_t x = dbits(d);
        if (FAST) {
            key = x | kSignBit;
            return slot_in<GUARD>(vmask, j) && (x - tb1) < tlim;
        }
        key = okey(x) ^ flip;
        return slot_in<GUARD>(vmask, j) && !__builtin_isnan(d) && key > thr;
    }

    // Count this chunk's candidates (C), ties with thr (E) and NaN slots (NN);
    // jm = bit j set if slot j has a candidate in some lane.
    template <bool GUARD, bool FAST>
    __device__ __forceinline__ void classify(const double2 (&c)[kUnroll], uint32_t vmask, uint32_t& C,
                                             uint32_t& E, uint32_t& NN, uint32_t& jm) const {
        C = E = NN = jm = 0;
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const double d = slot_val(c, j);
            uint64_t key;
            const bool cand = is_cand<GUARD, FAST>(d, vmask, j, key);
            const bool in = slot_in<GUARD>(vmask, j);
            const bool eq = FAST ? (in && dbits(d) == tbits) : (in && !__builtin_isnan(d) && key == thr);
            const uint64_t m = ballot(cand);
            C += popc64(m);
            jm |= m ? (1u << j) : 0u;
            E += popc64(ballot(eq));
            NN += popc64(ballot(in && __builtin_isnan(d)));
        }
    }

    template <bool GUARD, bool FAST>
    __device__ __forceinline__ void insert(const double2 (&c)[kUnroll], uint32_t vmask, uint32_t jm) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            if ((jm >> j) & 1u) {
                uint64_t key;
                const bool cand = is_cand<GUARD, FAST>(slot_val(c, j), vmask, j, key);
                const uint64_t m = ballot(cand);
                if (cand) {
                    buf[cnt + lane_prefix(m)] = key;
                    mxk = key > mxk ? key : mxk;
                    if (hvalid) atomicAdd(&H[bin(key)], 1u);
                }
                cnt = uni32(cnt + popc64(m));
            }
        }
    }

    template <bool GUARD>
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll], uint32_t vmask) {
        uint32_t C, E, NN, jm;
        if (fast) classify<GUARD, true>(c, vmask, C, E, NN, jm);
        else classify<GUARD, false>(c, vmask, C, E, NN, jm);
        if (cnt + C > cap) {
            compact();
            if (fast) classify<GUARD, true>(c, vmask, C, E, NN, jm);
            else classify<GUARD, false>(c, vmask, C, E, NN, jm);
            if (cnt + C > cap) {  // compaction failed (flagged): drop, never overrun
                bad = 1;
                return;
            }
        }
        eqs += E;
        nnan += NN;
        if (jm) {
            if (fast) insert<GUARD, true>(c, vmask, jm);
            else insert<GUARD, false>(c, vmask, jm);
        }
    }

    // Raise thr to nt and filter buf to keys > nt (counting keys == nt into eqs),
    // rebuilding H over (nt, mx].
    __device__ __forceinline__ void filter_rebuild(uint64_t nt, uint64_t mx) {
        hbase = uni64(nt + 1);
        const uint64_t range = mx > nt ? mx - hbase : 0ull;
        const int bits = range ? 64 - __clzll((long long)range) : 0;
        hsh = uni32(bits > 8 ? (uint32_t)(bits - 8) : 0u);
        for (uint32_t i = lane; i < 256; i += kWave) H[i] = 0;
        __syncthreads();
        uint32_t w = 0, e = 0;
        for (uint32_t base = 0; base < cnt; base += kWave) {
            const uint32_t i = base + lane;
            const bool in = i < cnt;
            const uint64_t x = in ? buf[i] : 0ull;
            const bool keep = in && x > nt;
            e += popc64(ballot(in && x == nt));
            const uint64_t m = ballot(keep);
            if (keep) {
                buf[w + lane_prefix(m)] = x;
                atomicAdd(&H[bin(x)], 1u);
            }
            w += popc64(m);
        }
        cnt = uni32(w);
        eqs = uni32(e);
        hvalid = 1;
        set_thr(nt);
    }

    __device__ __forceinline__ void compact() {
        __syncthreads();
        uint64_t nt = 0;
        bool have = false;
        if (hvalid) {
            const BinHit bh = find_bin_desc(H, tkeep, 0, lane);
            if (bh.found && bh.b < 255 && bh.above + bh.cnt <= tstop) {
                nt = uni64(hbase + ((uint64_t)bh.b << hsh));  // >= hbase > thr
                have = true;
            }
        }
        if (!have) {
            const SelHit hit = select_desc(buf, cnt, thr, eqs, tkeep, true, thr, tstop, scr, lane);
            nt = uni64(hit.key);
            if (!hit.ok || nt <= thr) {  // cannot happen while cnt > tstop; flag it
                bad = 1;
                return;
            }
        }
        filter_rebuild(nt, wave_max_u64(mxk));
        __syncthreads();
    }

    // The R-th largest key (1-based) of buf.
    __device__ __forceinline__ uint64_t kth_largest(uint32_t R) {
        if (hvalid) {
            const BinHit bh = find_bin_desc(H, R, 0, lane);
            if (bh.found && bh.b < 255 && bh.cnt <= kWave) {
                const uint64_t lo = hbase + ((uint64_t)bh.b << hsh);
                const uint64_t hi = lo + ((1ull << hsh) - 1);
                uint32_t w = 0;
                for (uint32_t base = 0; base < cnt; base += kWave) {
                    const uint32_t i = base + lane;
                    const bool in = i < cnt;
                    const uint64_t x = in ? buf[i] : 0ull;
                    const bool inb = in && x >= lo && x <= hi;
                    const uint64_t m = ballot(inb);
                    if (inb) small[w + lane_prefix(m)] = x;
                    w += popc64(m);
                }
                __syncthreads();
                const uint32_t R2 = R - bh.above;
                const uint64_t v = (uint32_t)lane < w ? small[lane] : 0ull;
                uint32_t gt = 0, ge = 0;
                for (uint32_t j = 0; j < w; ++j) {
                    const uint64_t y = small[j];
                    gt += y > v ? 1u : 0u;
                    ge += y >= v ? 1u : 0u;
                }
                const uint64_t sel = ballot((uint32_t)lane < w && gt < R2 && R2 <= ge);
                __syncthreads();
                if (sel) return uni64((uint64_t)__shfl((unsigned long long)v, __ffsll((long long)sel) - 1));
                bad = 1;
            }
        }
        const SelHit h = select_desc(buf, cnt, 0, 0, R, false, 0, 0, scr, lane);
        if (!h.ok) bad = 1;
        return h.key;
    }

    // Build H over the whole buffer (once at the end when no compaction ran).
    __device__ __forceinline__ void build_hist() {
        uint64_t mn = ~0ull, mx = 0;
        for (uint32_t i = lane; i < cnt; i += kWave) {
            const uint64_t x = buf[i];
            mn = x < mn ? x : mn;
            mx = x > mx ? x : mx;
        }
        mn = wave_min_u64(mn);
        mx = wave_max_u64(mx);
        hbase = mn;
        const uint64_t range = mx - mn;
        const int bits = range ? 64 - __clzll((long long)range) : 0;
        hsh = uni32(bits > 8 ? (uint32_t)(bits - 8) : 0u);
        for (uint32_t i = lane; i < 256; i += kWave) H[i] = 0;
        __syncthreads();
        for (uint32_t i = lane; i < cnt; i += kWave) atomicAdd(&H[bin(buf[i])], 1u);
        __syncthreads();
        hvalid = 1;
    }

    // Key of the element with ascending rank r (0-based) among nsel present samples.
    __device__ __forceinline__ uint64_t rank_key(uint64_t r, uint64_t nsel) {
        const uint64_t rr = flip ? (nsel - 1 - r) : r;
        const uint64_t below = nsel - cnt - eqs;
        if (rr < below) {
            bad = 1;
            return 0;
        }
        if (rr < below + eqs) return thr;
        const uint32_t idx = (uint32_t)(rr - below - eqs);
        return kth_largest(cnt - idx);
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
            return uni64((uint64_t)__shfl((unsigned long long)u, src));
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
    uint32_t cap;
    uint64_t* gscratch;  // non-null: candidate buffers live in HBM scratch, cap keys per block
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
};

// GBUF selects where candidate buffers live at COMPILE time, so the LDS variant
// emits ds_* (lgkmcnt) and never flat_* stores, which would force vmcnt(0)
// waits and serialise the prefetch pipeline.
template <bool GBUF>
__global__ __launch_bounds__(64, KRR_SELECT_WAVES_PER_SIMD) void k_select(SelectArgs A) {
    // LDS: [H 1 KiB][select scratch 1 KiB][gather 512 B][candidate keys cap x 8 B]
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t* buf;
    if constexpr (GBUF) {
        buf = A.gscratch + (size_t)blockIdx.x * A.cap;
    } else {
        buf = reinterpret_cast<uint64_t*>(smem + kSelectLdsFixed);
    }
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        const int64_t L = end - beg;
        const SidePlan sp = plan_side(L, A.mode, A.p_num, A.p_den, A.q);
        SelectProc P;
        P.buf = buf;
        P.H = reinterpret_cast<uint32_t*>(smem);
        P.scr = reinterpret_cast<uint32_t*>(smem + 1024);
        P.small = reinterpret_cast<uint64_t*>(smem + 2048);
        P.lane = lane;
        P.cap = A.cap;
        P.tkeep = sp.tkeep;
        P.tstop = A.cap - kChunkElems;
        P.flip = sp.bottom ? ~0ull : 0ull;
        P.cnt = 0;
        P.eqs = 0;
        P.nnan = 0;
        P.bad = 0;
        P.hbase = 0;
        P.hsh = 0;
        P.hvalid = 0;
        P.mxk = 0;
        P.set_thr(0);
        stream_segment(A.vals, beg, end, P, lane);
        __syncthreads();
        if (!P.hvalid && P.cnt > kWave) P.build_hist();

        const uint64_t nnan = P.nnan;
        const uint64_t n = A.gaps ? (uint64_t)L - nnan : (uint64_t)L;  // present samples
        uint32_t flags = 0;
        double result;
        if (n == 0) {
            result = bitsd(kQuietNaN);
            flags |= KRR_FLAG_EMPTY;
        } else if (nnan && !A.gaps) {
            result = bitsd(kQuietNaN);
            flags |= KRR_FLAG_NAN;
        } else if (A.mode == KRR_PCT_SORTED_LOWER) {
            const int64_t r = exact_rank(n, A.p_num, A.p_den);
            uint64_t bits = okey_inv(P.rank_key(r, n) ^ P.flip);
            if (is_zero_bits(bits)) {
                // Python sorted() is stable and -0 == +0: the zero at rank r is the
                // (r - #negatives)-th zero in position order.
                const uint64_t neg = count_negative(A.vals, beg, end, lane);
                bits = nth_zero_bits(A.vals, beg, end, (uint64_t)r - neg, lane);
            }
            result = bitsd(bits);
        } else {  // KRR_PCT_LINEAR, numpy method="linear"
            const double vidx = __dmul_rn((double)(n - 1), A.q);
            int64_t prev, next;
            double gamma;
            if (vidx >= (double)(n - 1)) {
                prev = next = (int64_t)n - 1;
                gamma = __dsub_rn(vidx, -1.0);  // numpy subtracts the clipped index -1
            } else {
                const double fl = floor(vidx);
                prev = (int64_t)fl;
                next = prev + 1;
                gamma = __dsub_rn(vidx, fl);
            }
            const double a = bitsd(okey_inv(P.rank_key(prev, n) ^ P.flip));
            const double b = (next == prev) ? a : bitsd(okey_inv(P.rank_key(next, n) ^ P.flip));
            result = np_lerp(a, b, gamma);
        }
        if (P.bad) flags |= KRR_FLAG_CAPACITY;
        if (lane == 0) {
            A.out_v[s] = result;
            A.out_n[s] = (int64_t)n;
            A.out_f[s] = flags;
        }
        __syncthreads();
    }
}

// --------------------------- REF_INDEX ------------------------------------
struct NanCountProc {
    uint32_t nn;
    template <bool GUARD>
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll], uint32_t vmask) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j)
            nn += popc64(ballot(slot_in<GUARD>(vmask, j) && __builtin_isnan(slot_val(c, j))));
    }
};

struct RefArgs {
    const double* vals;
    const int64_t* offs;
    int64_t S;
    int64_t p_num, p_den;
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
};

// NaN-gapped layout: the k-th PRESENT sample in position order.
__global__ __launch_bounds__(64) void k_refindex_gaps(RefArgs A) {
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        NanCountProc C{0};
        stream_segment(A.vals, beg, end, C, lane);
        const uint64_t n = (uint64_t)(end - beg) - C.nn;
        double result = bitsd(kQuietNaN);
        uint32_t flags = 0;
        if (n == 0) {
            flags = KRR_FLAG_EMPTY;
        } else {
            const uint64_t k = (uint64_t)exact_rank((int64_t)n, A.p_num, A.p_den);
            uint64_t run = 0;
            uint64_t found = kQuietNaN;
            if (k >= n / 2) {  // walk back from the end: j-th present from the end
                const uint64_t j = n - 1 - k;
                for (int64_t top = end; top > beg; top -= kWave) {
                    const int64_t i = top - 1 - lane;
                    const bool in = i >= beg;
                    const uint64_t u = in ? dbits(A.vals[i]) : kQuietNaN;
                    const bool p = in && !is_nan_bits(u);
                    const uint64_t m = ballot(p);
                    const uint32_t c = popc64(m);
                    if (run + c > j) {
                        const uint64_t sel = ballot(p && lane_prefix(m) == (uint32_t)(j - run));
                        found = uni64((uint64_t)__shfl((unsigned long long)u, __ffsll((long long)sel) - 1));
                        break;
                    }
                    run += c;
                }
            } else {
                for (int64_t base = beg; base < end; base += kWave) {
                    const int64_t i = base + lane;
                    const bool in = i < end;
                    const uint64_t u = in ? dbits(A.vals[i]) : kQuietNaN;
                    const bool p = in && !is_nan_bits(u);
                    const uint64_t m = ballot(p);
                    const uint32_t c = popc64(m);
                    if (run + c > k) {
                        const uint64_t sel = ballot(p && lane_prefix(m) == (uint32_t)(k - run));
                        found = uni64((uint64_t)__shfl((unsigned long long)u, __ffsll((long long)sel) - 1));
                        break;
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
        }
    }
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
    const int64_t k = exact_rank(n, A.p_num, A.p_den);
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
    template <bool GUARD>
    __device__ __forceinline__ void chunk(const double2 (&c)[kUnroll], uint32_t vmask) {
#pragma unroll
        for (int j = 0; j < 2 * kUnroll; ++j) {
            const double d = slot_val(c, j);
            const bool in = slot_in<GUARD>(vmask, j);
            mx = fmax(mx, in ? d : __builtin_nan(""));
            nn += popc64(ballot(in && __builtin_isnan(d)));
        }
    }
};

__device__ __forceinline__ double wave_max_f64(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o));
    return x;
}

struct MaxArgs {
    const double* vals;
    const int64_t* offs;
    int64_t S;
    int32_t gaps;
    double* out_v;
    int64_t* out_n;
    uint32_t* out_f;
};

__global__ __launch_bounds__(64) void k_max(MaxArgs A) {
    const int lane = threadIdx.x;
    for (int64_t s = blockIdx.x; s < A.S; s += gridDim.x) {
        const int64_t beg = A.offs[s], end = A.offs[s + 1];
        MaxProc M{__builtin_nan(""), 0u};
        stream_segment(A.vals, beg, end, M, lane);
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
        }
    }
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
                                              int gaps) {
    for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {
        const int64_t beg = offs[s], L = offs[s + 1] - beg;
        const int64_t plen = pod_len > 0 ? pod_len : (L > 0 ? L : 1);
        for (int64_t t = threadIdx.x; t < L; t += blockDim.x) {
            const int64_t pod = t / plen;
            const int64_t tp = t - pod * plen;
            const int64_t pl = (L - pod * plen) < plen ? (L - pod * plen) : plen;
            bool gap = false;
            if (gaps) {
                const uint64_t hp = hash4(seed, (uint64_t)s, (uint64_t)pod, 0xA11CEull);
                int64_t start = 0;
                if ((hp & 0xFFFF) < 19661 && pl > 1440)  // p = 0.3: the pod started late
                    start = (int64_t)((hp >> 16) % (uint64_t)(pl - 1440 + 1));
                const double f = 0.2 * unit01(hash4(seed, (uint64_t)s, (uint64_t)pod, 0xF00Dull));
                const double ub = unit01(hash4(seed ^ 0x5EEDull, (uint64_t)s, (uint64_t)pod, (uint64_t)(tp / 30)));
                gap = tp < start || (tp >= start + 1440 && ub <= f);
            }
            double v;
            if (gap) {
                v = bitsd(kQuietNaN);
            } else {
                const uint64_t h1 = hash4(seed, (uint64_t)s, (uint64_t)t, (uint64_t)kind);
                const uint64_t h2 = mix64(h1 ^ 0xD1B54A32D192ED03ull);
                if (kind == 0) {  // Gamma(k=2, theta=0.05) cores = sum of two exponentials
                    v = -0.05 * (log(unit01(h1)) + log(unit01(h2)));
                } else {  // floor(Normal(2e8, 2e7)) bytes, Box-Muller
                    const double z = sqrt(-2.0 * log(unit01(h1))) * cospi(2.0 * unit01(h2));
                    v = floor(2.0e8 + 2.0e7 * z);
                    if (v < 0.0) v = 0.0;
                }
            }
            vals[beg + t] = v;
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
    uint64_t* scratch;
    size_t scratch_bytes;
    unsigned long long* d_tmp;
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

int check_series(krr_ctx* ctx, const krr_series* s) {
    if (!s) return set_err(ctx, KRR_E_INVALID, "null series%s", "");
    if (s->n_segments < 0) return set_err(ctx, KRR_E_INVALID, "negative n_segments%s", "");
    if (s->n_segments > 0 && (!s->offsets || (!s->values && s->n_values > 0)))
        return set_err(ctx, KRR_E_INVALID, "null values/offsets%s", "");
    return KRR_OK;
}

int check_params(krr_ctx* ctx, const krr_percentile_params* p) {
    if (!p) return set_err(ctx, KRR_E_INVALID, "null params%s", "");
    if (p->mode < KRR_PCT_REF_INDEX || p->mode > KRR_PCT_LINEAR)
        return set_err(ctx, KRR_E_INVALID, "bad percentile mode %s%lld", "", p->mode);
    if (p->p_den <= 0 || p->p_den > 1000000000000000LL || p->p_num <= 0 || p->p_num > 100 * p->p_den)
        return set_err(ctx, KRR_E_INVALID, "percentile must be in (0, 100] with p_den <= 1e15%s", "");
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
    c->scratch = nullptr;
    c->scratch_bytes = 0;
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
    if (hipMalloc(&c->d_tmp, sizeof(unsigned long long)) != hipSuccess) {
        delete c;
        return KRR_E_HIP;
    }
    (void)hipFuncSetAttribute((const void*)k_select<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)c->max_lds);
    *out_ctx = c;
    return KRR_OK;
}

int krr_destroy(krr_ctx* ctx) {
    if (!ctx) return KRR_OK;
    DeviceGuard g(ctx->device);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->d_tmp) (void)hipFree(ctx->d_tmp);
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
        RefArgs A{series->values, series->offsets, S, params->p_num, params->p_den, out_value, out_count, out_flags};
        if (series->gaps_are_nan) {
            hipLaunchKernelGGL(k_refindex_gaps, dim3(grid_for(S)), dim3(64), 0, st, A);
        } else {
            hipLaunchKernelGGL(k_refindex_dense, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, st, A);
        }
        KRR_HIP(ctx, hipGetLastError());
        return KRR_OK;
    }

    int64_t Lmax = 0;
    rc = resolve_maxlen(ctx, series, st, &Lmax);
    if (rc) return rc;
    const SidePlan sp = plan_side(Lmax, params->mode, params->p_num, params->p_den, params->q);
    const uint32_t cap = capacity_for(sp.tkeep);
    SelectArgs A{};
    A.vals = series->values;
    A.offs = series->offsets;
    A.S = S;
    A.mode = params->mode;
    A.gaps = series->gaps_are_nan;
    A.p_num = params->p_num;
    A.p_den = params->p_den;
    A.q = params->q;
    A.cap = cap;
    A.gscratch = nullptr;
    A.out_v = out_value;
    A.out_n = out_count;
    A.out_f = out_flags;
    const size_t lds = kSelectLdsFixed + (size_t)cap * 8;
    if (lds <= ctx->max_lds) {
        hipLaunchKernelGGL(k_select<false>, dim3(grid_for(S)), dim3(64), lds, st, A);
    } else {
        // Candidate buffers too large for LDS (e.g. p near 50 on very long series):
        // same algorithm with per-block buffers in HBM scratch, persistent grid.
        int64_t grid = (int64_t)ctx->num_cus * 8;
        if (grid > S) grid = S;
        const size_t need = (size_t)grid * cap * 8;
        if (need > ctx->scratch_bytes) {
            if (ctx->scratch) KRR_HIP(ctx, hipFree(ctx->scratch));
            ctx->scratch = nullptr;
            ctx->scratch_bytes = 0;
            KRR_HIP(ctx, hipMalloc(&ctx->scratch, need));
            ctx->scratch_bytes = need;
        }
        A.gscratch = ctx->scratch;
        hipLaunchKernelGGL(k_select<true>, dim3((unsigned)grid), dim3(64), kSelectLdsFixed, st, A);
    }
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
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
    hipLaunchKernelGGL(k_max, dim3(grid_for(S)), dim3(64), 0, (hipStream_t)stream, A);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

int krr_simple_run(krr_ctx* ctx, const krr_series* cpu, const krr_series* mem,
                   const krr_percentile_params* params, double* cpu_value, int64_t* cpu_count,
                   uint32_t* cpu_flags, double* mem_value, int64_t* mem_count, uint32_t* mem_flags,
                   void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (!cpu || !mem) return set_err(ctx, KRR_E_INVALID, "null series%s", "");
    if (cpu->n_segments != mem->n_segments)
        return set_err(ctx, KRR_E_INVALID, "cpu and mem need one segment per object each%s", "");
    int rc = krr_segmented_percentile(ctx, cpu, params, cpu_value, cpu_count, cpu_flags, stream);
    if (rc) return rc;
    return krr_segmented_max(ctx, mem, mem_value, mem_count, mem_flags, stream);
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

int krr_synth_fill(krr_ctx* ctx, double* values, const int64_t* offsets, int64_t n_segments, uint64_t seed,
                   int32_t kind, int64_t pod_len, int32_t gaps, void* stream) {
    if (!ctx) return KRR_E_INVALID;
    if (n_segments < 0 || (n_segments > 0 && (!values || !offsets)) || kind < 0 || kind > 1)
        return set_err(ctx, KRR_E_INVALID, "bad synth arguments%s", "");
    if (n_segments == 0) return KRR_OK;
    DeviceGuard g(ctx->device);
    if (!g.ok) return set_err(ctx, KRR_E_HIP, "cannot select device%s", "");
    int64_t grid = n_segments < 65536 ? n_segments : 65536;
    hipLaunchKernelGGL(k_synth, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, values, offsets,
                       n_segments, seed, kind, pod_len, gaps);
    KRR_HIP(ctx, hipGetLastError());
    return KRR_OK;
}

}  // extern "C"
