// krr_json.h — the Prometheus query_range packer on the device (round 3).
//
// The host packer (krr_pack.cpp, include/krr_pack.h) parses response bodies at
// ~12 GB/s of JSON on 16 cores; the end-to-end path from bodies was bound by it
// (DESIGN.md §9).  Here the raw bodies go to HBM instead (PCIe moves ~55 GB/s) and
// every body is parsed by one wave:
//   * lane 0 reads the envelope up to data.result[0]["values"] (krr_json_parse.h
//     envelope_head: status, data, result, the series' other keys, validated);
//   * the values array — nearly all of the body — is parsed by all 64 lanes at once:
//     each lane owns 32 bytes of a 2-KiB block, parses the sample elements that start
//     in them (`[<time>,"<value>"]`, value -> float64 by Eisel-Lemire), and a wave
//     prefix sum over the lanes' element counts places each value;
//   * lane 0 validates the rest of the body (envelope_tail).
// Values land in a scratch array at slot (body byte offset / 8) + element index (an
// element takes at least 8 bytes, so bodies' slots never overlap); k_json_compact then
// moves each kept body's run to its place in the CSR (exclusive prefix of the counts).
// A body outside the canonical grammar is reported KRR_JSON_HOST, never as an error:
// the caller parses that batch with the host packer, which gives the reference's
// result or error for it (krr_json_parse.h header).
#pragma once

#include "krr_device.h"
#include "krr_json_parse.h"

namespace krr {
namespace json {

constexpr int kLaneBytes = 32;                  // bytes of a block each lane scans for '['
constexpr int kBlockBytes = kLaneBytes * kWave;  // 2 KiB per block
constexpr int kMaxPerLane = 4;                   // an element spans >= 8 bytes: <= 4 start in 32
constexpr int kStageBytes = 2 * kBlockBytes;     // LDS copy: the block and the next one

struct JsonArgs {
    const char* bodies;      // device: the bodies back to back (16-B aligned base)
    const int64_t* offs;     // device: [n_bodies + 1] byte offsets
    int64_t first;           // first body of this launch
    int64_t n;               // bodies in this launch
    int32_t want_ts;
    double* tmp_v;           // scratch [total_bytes / 8 + 1]
    double* tmp_t;           // scratch for timestamps (want_ts) or null
    int64_t* counts;         // [n_bodies] samples kept per body
    int32_t* status;         // [n_bodies] KRR_JSON_OK / DROPPED / HOST
};

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

// positions are >= 0 (INT64_MAX: none)
__device__ __forceinline__ int64_t wave_min_pos(int64_t x) { return (int64_t)wave_min_u64((uint64_t)x); }

// The json kernels run one wave per workgroup (__launch_bounds__(64)): a wave's LDS accesses
// complete in order, so lanes only need the compiler to keep the stores before the loads.  A
// workgroup barrier's release fence would also wait for every outstanding global load — the
// prefetched next block included.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Element bytes come from the wave's LDS copy of [blk, blk + kStageBytes) — an element
// starting in the block's first 2 KiB and shorter than 2 KiB lies inside it — and from
// global memory past it (long value strings only).
struct StagedLoad {
    const char* buf;           // the bodies buffer
    const unsigned char* lds;  // its bytes [blk, blk + kStageBytes)
    int64_t blk;
    __device__ char operator()(const char* p) const {
        const int64_t o = (p - buf) - blk;
        return (uint64_t)o < (uint64_t)kStageBytes ? (char)lds[o] : *p;
    }
};

// The values array from its first '[' (vs): returns false when the body goes to the
// host; else *count samples written at tv/tt[0 ..), *vend = one past the array's ']'.
// Per 2-KiB block: the wave stages the block and the next one in LDS (each lane 2 x 32
// bytes, 16-B loads; 64 readable bytes past every body make the loads safe), each lane
// finds the '[' in its own 32 bytes (a bit mask from registers) and parses the elements
// starting there from LDS, one at a time.
__device__ bool values_array(const char* const buf, bool want_ts, const char* vs, const char* e, double* tv, double* tt,
                             int lane, unsigned char* lds, int64_t* count, const char** vend) {
    const int64_t lo_abs = vs - buf, hi_abs = e - buf;
    int64_t blk = lo_abs & ~(int64_t)(kLaneBytes - 1);
    int64_t cnt = 0;
    // lane l's 32 bytes of the current block (x) and of the next one (y) stay in registers from
    // one block to the next: each block is read from memory once, and the block after next (z)
    // is requested before the current one is parsed, so its load overlaps the parse (a grouped
    // chunk's series give one wave each — too few waves per SIMD to hide a load otherwise)
    auto load32 = [&](int64_t at, v4u32& a, v4u32& b) {
        if (at < hi_abs) {
            const v4u32* q = reinterpret_cast<const v4u32*>(buf + at);
            a = q[0];
            b = q[1];
        }
    };
    const v4u32 zero = {0, 0, 0, 0};
    v4u32 x0 = zero, x1 = zero, y0 = zero, y1 = zero;
    load32(blk + (int64_t)lane * kLaneBytes, x0, x1);
    load32(blk + (int64_t)lane * kLaneBytes + kBlockBytes, y0, y1);
    for (; blk < hi_abs; blk += kBlockBytes) {
        // stage [blk, blk + 4 KiB): lane l's 32 bytes at 32 l and at 2 KiB + 32 l
        const int64_t r0 = blk + (int64_t)lane * kLaneBytes;
        uint32_t mine_w[8];
        {
            v4u32* d = reinterpret_cast<v4u32*>(lds + lane * kLaneBytes);
            d[0] = x0;
            d[1] = x1;
            v4u32* d2 = reinterpret_cast<v4u32*>(lds + kBlockBytes + lane * kLaneBytes);
            d2[0] = y0;
            d2[1] = y1;
            mine_w[0] = x0[0], mine_w[1] = x0[1], mine_w[2] = x0[2], mine_w[3] = x0[3];
            mine_w[4] = x1[0], mine_w[5] = x1[1], mine_w[6] = x1[2], mine_w[7] = x1[3];
        }
        v4u32 z0 = zero, z1 = zero;
        load32(r0 + 2 * kBlockBytes, z0, z1);
        wave_lds_sync();
        // '[' in this lane's 32 bytes that lie inside the array's span
        uint32_t starts = 0;
#pragma unroll
        for (int k = 0; k < kLaneBytes; ++k)
            starts |= (((mine_w[k >> 2] >> (8 * (k & 3))) & 0xFF) == '[' ? 1u : 0u) << k;
        if (r0 < lo_abs) {
            const int64_t d = lo_abs - r0;
            starts = d >= kLaneBytes ? 0u : (starts >> d) << d;
        }
        if (r0 + kLaneBytes > hi_abs) {
            const int64_t d = hi_abs - r0;
            starts = d <= 0 ? 0u : starts & (0xFFFFFFFFu >> (kLaneBytes - d));
        }
        double v[kMaxPerLane], t[kMaxPerLane];
        int64_t st[kMaxPerLane];
        int nok = 0;
        int64_t fail_min = INT64_MAX, last_start = INT64_MAX, last_next = 0;
        const StagedLoad ld{buf, lds, blk};
        while (starts) {
            const int k = __builtin_ctz(starts);
            starts &= starts - 1;
            const int64_t x = r0 + k;
            double vv = 0.0, tt2 = 0.0;
            const char* next = nullptr;
            bool last = false;
            if (nok == kMaxPerLane || !sample_element(buf + x, e, want_ts, &vv, &tt2, &next, &last, ld)) {
                fail_min = x < fail_min ? x : fail_min;  // (more than 4 starts: elements are >= 8 bytes)
                continue;
            }
            v[nok] = vv;
            t[nok] = tt2;
            st[nok] = x;
            ++nok;
            if (last && x < last_start) {
                last_start = x;
                last_next = next - buf;
            }
        }
        // the array's last element is the first one followed by ']'
        const int64_t end_start = wave_min_pos(last_start);
        if (wave_min_pos(fail_min) < (end_start == INT64_MAX ? INT64_MAX : end_start + 1)) return false;
        int mine = 0;
#pragma unroll
        for (int j = 0; j < kMaxPerLane; ++j) mine += (j < nok && st[j] <= end_start) ? 1 : 0;
        const uint32_t incl = wave_scan32((uint32_t)mine, 0u, OpAdd32{});
        const int64_t base = cnt + (int64_t)(incl - (uint32_t)mine);
#pragma unroll
        for (int j = 0; j < kMaxPerLane; ++j) {
            if (j < mine) {
                tv[base + j] = v[j];
                if (want_ts) tt[base + j] = t[j];
            }
        }
        cnt += (int64_t)lane_bcast32(incl, kWave - 1);
        if (end_start != INT64_MAX) {
            // the lane that holds the last element knows where the array ends
            const uint64_t nx = ballot(last_start == end_start);
            const int src = (int)__builtin_ctzll(nx);
            *vend = buf + (int64_t)lane_bcast64((uint64_t)last_next, src);
            *count = cnt;
            return true;
        }
        wave_lds_sync();  // every lane is done with the staged bytes
        x0 = y0, x1 = y1, y0 = z0, y1 = z1;
    }
    return false;  // no closing ']'
}

// One body per wave (grid-stride over the launch's bodies).
__global__ __launch_bounds__(64) void k_json_parse(JsonArgs A) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kStageBytes];
    const int lane = threadIdx.x;
    for (int64_t i = blockIdx.x; i < A.n; i += gridDim.x) {
        const int64_t bi = A.first + i;
        const int64_t ob = A.offs[bi], oe = A.offs[bi + 1];
        const char* s = A.bodies + ob;
        const char* e = A.bodies + oe;
        // phase 1 (lane 0): the envelope up to result[0]["values"]
        int code = 0;
        int64_t at = 0;
        Envelope env{0, 0};
        if (lane == 0) {
            Reader r{s, e};
            const char* p = nullptr;
            code = envelope_head(r, env, &p);
            if (code == 1) at = p - s;
        }
        code = (int)__builtin_amdgcn_readfirstlane(code);
        at = (int64_t)uni64((uint64_t)at);
        int32_t status = JSON_HOST;
        int64_t count = 0;
        if (code == 2) {
            status = JSON_DROPPED;
        } else if (code == 1) {
            const char* vs = s + at;
            const char* vend = nullptr;
            bool ok = false;
            if (vs < e && *vs == ']') {  // "values": []
                ok = true;
                vend = vs + 1;
            } else if (vs < e && *vs == '[') {
                // phase 2 (all lanes): the samples
                ok = values_array(A.bodies, A.want_ts != 0, vs, e, A.tmp_v + (ob >> 3),
                                  A.tmp_t ? A.tmp_t + (ob >> 3) : nullptr, lane, lds, &count, &vend);
            }
            // phase 3 (lane 0): the rest of the body
            if (ok) {
                int tail_ok = 0;
                if (lane == 0) {
                    Reader r{vend, e};
                    tail_ok = envelope_tail(r, env) ? 1 : 0;
                }
                ok = __builtin_amdgcn_readfirstlane(tail_ok) != 0;
            }
            if (ok) status = JSON_OK;
        }
        if (lane == 0) {
            A.status[bi] = status;
            A.counts[bi] = status == JSON_OK ? count : 0;
        }
    }
}

struct CompactArgs {
    const int64_t* offs;     // body byte offsets (scratch slot = offs[b] / 8)
    const int64_t* counts;
    const int32_t* status;
    const int64_t* out_pos;  // exclusive prefix of counts
    const double* tmp_v;
    const double* tmp_t;
    double* values;
    double* ts;
    int64_t n;
};

// Each kept body's run of values from its scratch slot to its CSR place.
__global__ __launch_bounds__(256) void k_json_compact(CompactArgs C) {
    for (int64_t b = blockIdx.x; b < C.n; b += gridDim.x) {
        if (C.status[b] != JSON_OK) continue;
        const int64_t n = C.counts[b], src = C.offs[b] >> 3, dst = C.out_pos[b];
        for (int64_t j = threadIdx.x; j < n; j += blockDim.x) {
            C.values[dst + j] = C.tmp_v[src + j];
            if (C.ts) C.ts[dst + j] = C.tmp_t[src + j];
        }
    }
}


// ---- grouped bodies ("sum by (pod) (...)"): one wave per SERIES ----
// A grouped body holds one series per pod (megabytes per body, a few bodies per fleet), so
// a wave per body would leave the GPU idle.  Instead:
//   k_json_find_series  every `{"metric":` after '[', ',' or whitespace in the bodies (a 32-bit
//                       window compare at each byte, 64 bytes per lane): the candidate series
//                       starts;
//   k_json_segments     one wave per candidate: the series object (GroupedWalker from
//                       SERIES_OPEN) — label span, values by the whole wave into scratch slot
//                       (array offset / 8), and where the object ends;
// and the host chains the segments body by body from the envelope head to its tail
// (krr_json_parse.h chain_grouped, in krr_pack_route_grouped): a candidate that is not a
// real series start is never reached by the chain, and a real series that is not a
// candidate (another key order) breaks it — that body goes to the host packer.
constexpr int kSegWords = 7;  // start, end (one past '}'), label offset (-1), label length, slot, count, ok
constexpr int kMaxLabel = 64;
constexpr uint32_t kMetricHead = (uint32_t)'{' | ((uint32_t)'"' << 8) | ((uint32_t)'m' << 16) | ((uint32_t)'e' << 24);

struct FindArgs {
    const char* bodies;
    int64_t begin, end;           // candidate positions searched: [begin, end)
    int64_t limit;                // bytes [0, limit) are in place (a pattern must end below it)
    int64_t* cand;                // absolute offsets of the candidates' '{'
    int64_t cap;
    unsigned long long* n_cand;
};

__global__ __launch_bounds__(64) void k_json_find_series(FindArgs F) {
    const int lane = threadIdx.x;
    constexpr int kLane = 64;
    const int64_t base = F.begin & ~(int64_t)15;  // 16-B aligned loads
    for (int64_t blk = base + (int64_t)blockIdx.x * kLane * kWave; blk < F.end;
         blk += (int64_t)gridDim.x * kLane * kWave) {
        const int64_t r0 = blk + (int64_t)lane * kLane;
        if (r0 >= F.end) continue;
        const v4u32* q = reinterpret_cast<const v4u32*>(F.bodies + r0);
        uint32_t w[20];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const v4u32 x = q[k];
            w[4 * k] = x[0], w[4 * k + 1] = x[1], w[4 * k + 2] = x[2], w[4 * k + 3] = x[3];
        }
#pragma unroll
        for (int k = 0; k < kLane; ++k) {
            const int s = 8 * (k & 3);
            const uint32_t win = s ? ((w[k >> 2] >> s) | (w[(k >> 2) + 1] << (32 - s))) : w[k >> 2];
            if (win != kMetricHead) continue;
            const int64_t x = r0 + k;
            if (x < F.begin || x >= F.end || x == 0 || x + 10 > F.limit) continue;
            const char* c = F.bodies + x;
            const char pre = c[-1];
            const bool pre_ok = pre == '[' || pre == ',' || pre == ' ' || pre == '\n' || pre == '\r' || pre == '\t';
            if (!pre_ok || c[4] != 't' || c[5] != 'r' || c[6] != 'i' || c[7] != 'c' ||
                c[8] != '"' || c[9] != ':')
                continue;
            const unsigned long long slot = atomicAdd(F.n_cand, 1ull);
            if ((int64_t)slot < F.cap) F.cand[slot] = x;
        }
    }
}

struct SegArgs {
    const char* bodies;
    const int64_t* offs;       // body byte offsets
    const int64_t* start;      // [n] candidate '{' (absolute)
    const int64_t* body;       // [n] its body
    int64_t n;
    int32_t want_ts;
    int32_t label_len;
    // the routing label key, by value in the kernel arguments (no per-launch copy into a
    // device buffer shared by the launches of several streams); NUL-padded to kMaxLabel
    uint64_t label_w[kMaxLabel / 8];
    double* tmp_v;
    double* tmp_t;
    int64_t* seg;              // [n][kSegWords]
    // split values parse (null: each series' values parsed by its own wave, values_array):
    // phase 1 (here) finds each values array's end and cuts it into parts, phase 2
    // (k_json_value_parts) parses the parts, one wave each
    int64_t* parts;                 // [parts_cap][kPartWords]
    int64_t parts_cap;
    unsigned long long* n_parts;    // device counter (zeroed by the caller)
    int64_t* series_vend;           // [n]: one past each split array's ']'
};

// ---- split values parse (round 6): a grouped chunk holds a few hundred series of ~10^4
// samples, one wave each — too few waves to hide a wave's serial element parse, so the
// last chunk's parse was the pipeline's tail.  Phase 1 scans each series' values array for
// its end (the last element's ']' followed by the array's ']') and counts the element
// starts ('[') per kPartBytes part; phase 2 parses every part with a wave of its own and
// writes its values at the series' slot + the elements before the part — the same slots,
// values and validation values_array gives (every element parsed by sample_element; the
// array's last element is the one followed by ']', at the end phase 1 found).
constexpr int kPartBytes = 8 * kBlockBytes;  // 16 KiB of a values array per phase-2 wave
constexpr int kPartWords = 6;                // series, first start, starts end, vend, slot, count

// Phase 1 scan over [vs, e) (vs = the first element's '['): *vend = one past the first "]]"
// at or after vs; per part [blk0 + k kPartBytes, +kPartBytes) the '[' count below the end.
// Returns the number of parts (lane-uniform) or -1: no "]]" below e (the caller falls back
// to values_array, which also accepts whitespace between the two brackets).  emit(k, lo,
// hi, base, count) runs on every lane with uniform arguments.
template <class Emit>
__device__ int64_t values_scan(const char* const buf, const char* vs, const char* e, int lane, int64_t* vend_out,
                               Emit emit) {
    const int64_t lo_abs = vs - buf, hi_abs = e - buf;
    const int64_t blk0 = lo_abs & ~(int64_t)(kLaneBytes - 1);
    auto load32 = [&](int64_t at, v4u32& a, v4u32& b) {
        if (at < hi_abs) {
            const v4u32* q = reinterpret_cast<const v4u32*>(buf + at);
            a = q[0];
            b = q[1];
        }
    };
    const v4u32 zero = {0, 0, 0, 0};
    v4u32 x0 = zero, x1 = zero;
    load32(blk0 + (int64_t)lane * kLaneBytes, x0, x1);
    bool prev_rb = false;      // the byte before this block is ']' (lane 63's last byte)
    int64_t base = 0, part_cnt = 0, part = 0;
    for (int64_t blk = blk0; blk < hi_abs; blk += kBlockBytes) {
        const int64_t r0 = blk + (int64_t)lane * kLaneBytes;
        v4u32 y0 = zero, y1 = zero;
        load32(r0 + kBlockBytes, y0, y1);  // the next block, requested before this one is scanned
        uint32_t w[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        uint32_t lb = 0, rb = 0, sb = 0;
#pragma unroll
        for (int k = 0; k < kLaneBytes; ++k) {
            const uint32_t c = (w[k >> 2] >> (8 * (k & 3))) & 0xFF;
            lb |= (c == '[' ? 1u : 0u) << k;
            rb |= (c == ']' ? 1u : 0u) << k;
            sb |= (c == '{' || c == '}' || c == ':' ? 1u : 0u) << k;  // never inside a values array
        }
        // bytes outside [lo_abs, hi_abs)
        uint32_t valid = 0xFFFFFFFFu;
        if (r0 < lo_abs) {
            const int64_t d = lo_abs - r0;
            valid = d >= kLaneBytes ? 0u : (valid >> d) << d;
        }
        if (r0 + kLaneBytes > hi_abs) {
            const int64_t d = hi_abs - r0;
            valid = d <= 0 ? 0u : valid & (0xFFFFFFFFu >> (kLaneBytes - d));
        }
        lb &= valid;
        rb &= valid;
        sb &= valid;
        // "]]": a ']' whose next byte is ']' (the next lane's first byte for bit 31); the
        // previous block's last ']' pairs with this block's first byte
        const uint32_t next_first = (uint32_t)__shfl_down((int)(rb & 1u), 1);
        const uint32_t nxt = (rb >> 1) | ((lane < kWave - 1 ? next_first : 0u) << 31);
        uint32_t pair = rb & nxt;
        int64_t my_end = INT64_MAX;  // position of the first ']' of the pair
        if (pair) my_end = r0 + __builtin_ctz(pair);
        if (lane == 0 && prev_rb && (rb & 1u)) my_end = r0 - 1;
        const int64_t end = wave_min_pos(my_end);
        // a byte no values array holds before any "]]": the array ends otherwise (whitespace
        // between its brackets) — values_array takes it, the scan stops here instead of
        // running on through the rest of the body
        const int64_t stop = wave_min_pos(sb ? r0 + __builtin_ctz(sb) : INT64_MAX);
        if (stop != INT64_MAX && (end == INT64_MAX || stop < end)) return -1;
        prev_rb = (lane_bcast32(rb, kWave - 1) >> 31) & 1u;
        // element starts below the end
        uint32_t mine = lb;
        if (end != INT64_MAX) {
            const int64_t d = end - r0;
            mine = d <= 0 ? 0u : (d >= kLaneBytes ? mine : mine & (0xFFFFFFFFu >> (kLaneBytes - d)));
        }
        part_cnt += (int64_t)wave_sum_u32((uint32_t)__builtin_popcount(mine));
        const bool part_full = blk + kBlockBytes >= blk0 + (part + 1) * (int64_t)kPartBytes;
        if (end != INT64_MAX) {
            *vend_out = end + 2;
            const int64_t plo = part == 0 ? lo_abs : blk0 + part * (int64_t)kPartBytes;
            emit(part, plo, end + 2, base, part_cnt);
            return part + 1;
        }
        if (part_full) {
            const int64_t plo = part == 0 ? lo_abs : blk0 + part * (int64_t)kPartBytes;
            emit(part, plo, blk0 + (part + 1) * (int64_t)kPartBytes, base, part_cnt);
            base += part_cnt;
            part_cnt = 0;
            ++part;
        }
        x0 = y0, x1 = y1;
    }
    return -1;
}

// Phase 2: the elements starting in [plo, phi) of one values array ending at vend (one past
// its ']'): parsed, checked (an element followed by ']' must end the array at vend, every
// other one must be followed by the next element before vend) and written at tv[0 ..) in
// order; true when all parse and their number is `expect`.
__device__ bool values_part(const char* const buf, bool want_ts, int64_t plo, int64_t phi, int64_t vend,
                            double* tv, double* tt, int64_t expect, int lane, unsigned char* lds) {
    const int64_t hi_abs = vend;  // nothing an element reads lies past the array
    const char* const e = buf + vend;
    auto load32 = [&](int64_t at, v4u32& a, v4u32& b) {
        if (at < hi_abs) {
            const v4u32* q = reinterpret_cast<const v4u32*>(buf + at);
            a = q[0];
            b = q[1];
        }
    };
    const v4u32 zero = {0, 0, 0, 0};
    int64_t blk = plo & ~(int64_t)(kLaneBytes - 1);
    v4u32 x0 = zero, x1 = zero, y0 = zero, y1 = zero;
    load32(blk + (int64_t)lane * kLaneBytes, x0, x1);
    load32(blk + (int64_t)lane * kLaneBytes + kBlockBytes, y0, y1);
    int64_t cnt = 0;
    bool bad = false;
    for (; blk < phi; blk += kBlockBytes) {
        const int64_t r0 = blk + (int64_t)lane * kLaneBytes;
        uint32_t mine_w[8];
        {
            v4u32* d = reinterpret_cast<v4u32*>(lds + lane * kLaneBytes);
            d[0] = x0;
            d[1] = x1;
            v4u32* d2 = reinterpret_cast<v4u32*>(lds + kBlockBytes + lane * kLaneBytes);
            d2[0] = y0;
            d2[1] = y1;
            mine_w[0] = x0[0], mine_w[1] = x0[1], mine_w[2] = x0[2], mine_w[3] = x0[3];
            mine_w[4] = x1[0], mine_w[5] = x1[1], mine_w[6] = x1[2], mine_w[7] = x1[3];
        }
        v4u32 z0 = zero, z1 = zero;
        load32(r0 + 2 * kBlockBytes, z0, z1);
        wave_lds_sync();
        uint32_t starts = 0;
#pragma unroll
        for (int k = 0; k < kLaneBytes; ++k)
            starts |= (((mine_w[k >> 2] >> (8 * (k & 3))) & 0xFF) == '[' ? 1u : 0u) << k;
        if (r0 < plo) {
            const int64_t d = plo - r0;
            starts = d >= kLaneBytes ? 0u : (starts >> d) << d;
        }
        if (r0 + kLaneBytes > phi) {
            const int64_t d = phi - r0;
            starts = d <= 0 ? 0u : starts & (0xFFFFFFFFu >> (kLaneBytes - d));
        }
        double v[kMaxPerLane], t[kMaxPerLane];
        int nok = 0;
        bool lane_bad = false;
        const StagedLoad ld{buf, lds, blk};
        while (starts) {
            const int k = __builtin_ctz(starts);
            starts &= starts - 1;
            double vv = 0.0, tt2 = 0.0;
            const char* next = nullptr;
            bool last = false;
            if (nok == kMaxPerLane || !sample_element(buf + r0 + k, e, want_ts, &vv, &tt2, &next, &last, ld) ||
                (last ? next != e : next >= e)) {
                lane_bad = true;
                continue;
            }
            v[nok] = vv;
            t[nok] = tt2;
            ++nok;
        }
        bad |= ballot(lane_bad) != 0;
        const uint32_t incl = wave_scan32((uint32_t)nok, 0u, OpAdd32{});
        const int64_t at = cnt + (int64_t)(incl - (uint32_t)nok);
        if (!bad && cnt + (int64_t)lane_bcast32(incl, kWave - 1) <= expect) {
#pragma unroll
            for (int j = 0; j < kMaxPerLane; ++j) {
                if (j < nok) {
                    tv[at + j] = v[j];
                    if (want_ts) tt[at + j] = t[j];
                }
            }
        }
        cnt += (int64_t)lane_bcast32(incl, kWave - 1);
        wave_lds_sync();  // every lane is done with the staged bytes
        x0 = y0, x1 = y1, y0 = z0, y1 = z1;
    }
    return !bad && cnt == expect;
}

__global__ __launch_bounds__(64) void k_json_segments(SegArgs A) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kStageBytes];
    __shared__ uint64_t label_lds[kMaxLabel / 8];
    const int lane = threadIdx.x;
    if (lane == 0) {
#pragma unroll
        for (int w = 0; w < kMaxLabel / 8; ++w) label_lds[w] = A.label_w[w];
    }
    __syncthreads();
    const char* label = reinterpret_cast<const char*>(label_lds);
    for (int64_t j = blockIdx.x; j < A.n; j += gridDim.x) {
        const int64_t x = A.start[j], bi = A.body[j];
        const char* e = A.bodies + A.offs[bi + 1];
        GroupedWalker W;
        if (lane == 0) {
            W.init(A.bodies + x, e, label, A.label_len);
            W.resume(A.bodies + x, GroupedWalker::SERIES_OPEN);
        }
        int ok = 0;
        for (;;) {
            int ev = W_HOST;
            int64_t at = 0;
            if (lane == 0) {
                ev = W.step();
                if (ev == W_VALUES) at = W.values_at - A.bodies;
            }
            ev = (int)__builtin_amdgcn_readfirstlane(ev);
            at = (int64_t)uni64((uint64_t)at);
            if (ev == W_SERIES) {
                ok = 1;
                break;
            }
            if (ev != W_VALUES) break;
            const char* vs = A.bodies + at;
            const char* vend = nullptr;
            int64_t count = 0;
            bool vok = false;
            if (vs < e && *vs == ']') {
                vok = true;
                vend = vs + 1;
            } else if (vs < e && *vs == '[') {
                int64_t np = -1;
                if (A.parts) {
                    // phase 1: the array's end and its parts (phase 2 parses them); a part that
                    // finds no room in the workspace fails the series (its batch goes to the host)
                    int64_t vend_abs = 0, total = 0;
                    bool room = true;
                    np = values_scan(A.bodies, vs, e, lane, &vend_abs,
                                     [&](int64_t k, int64_t plo, int64_t phi, int64_t base, int64_t c) {
                                         (void)k;
                                         total = base + c;
                                         if (lane == 0) {
                                             const unsigned long long q = atomicAdd(A.n_parts, 1ull);
                                             if ((int64_t)q < A.parts_cap) {
                                                 int64_t* P = A.parts + (int64_t)q * kPartWords;
                                                 P[0] = j;
                                                 P[1] = plo;
                                                 P[2] = phi;
                                                 P[3] = 0;
                                                 P[4] = (at >> 3) + base;
                                                 P[5] = c;
                                             } else {
                                                 room = false;
                                             }
                                         }
                                     });
                    room = __builtin_amdgcn_readfirstlane(room ? 1 : 0) != 0;
                    // the parts phase 2 may parse: only those of a finished scan (-1: the scan
                    // stopped — its parts so far are skipped, values_array below parses it all)
                    if (lane == 0) A.series_vend[j] = np >= 0 ? vend_abs : -1;
                    if (np >= 0) {
                        vok = room;
                        count = total;
                        vend = A.bodies + vend_abs;
                    }
                }
                if (np < 0)
                    vok = values_array(A.bodies, A.want_ts != 0, vs, e, A.tmp_v + (at >> 3),
                                       A.tmp_t ? A.tmp_t + (at >> 3) : nullptr, lane, lds, &count, &vend);
            }
            if (!vok) break;
            if (lane == 0) W.values_done(vend, count);
        }
        if (lane == 0) {
            int64_t* r = A.seg + j * kSegWords;
            r[0] = x;
            r[1] = ok ? (int64_t)(W.r.p - A.bodies) : -1;
            r[2] = (ok && W.lab) ? (int64_t)(W.lab - A.bodies) : -1;
            r[3] = ok ? W.lab_len : 0;
            r[4] = ok ? (int64_t)((W.values_at - A.bodies) >> 3) : 0;
            r[5] = ok ? W.count : 0;
            r[6] = ok;
        }
    }
}

struct PartArgs {
    const char* bodies;
    const int64_t* parts;              // [*n_parts][kPartWords] (phase 1)
    const unsigned long long* n_parts;
    const int64_t* series_vend;        // phase 1's array ends, by series
    int64_t parts_cap;
    int32_t want_ts;
    double* tmp_v;
    double* tmp_t;
    int64_t* seg;                      // a failed part clears its series' ok word
};

// Phase 2 of the split values parse: one part per wave (grid-stride over the parts phase 1
// recorded; the array's end from phase 1's series_vend).
__global__ __launch_bounds__(64) void k_json_value_parts(PartArgs A) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[kStageBytes];
    const int lane = threadIdx.x;
    const unsigned long long np_ = *A.n_parts;
    const int64_t np = (int64_t)np_ < A.parts_cap ? (int64_t)np_ : A.parts_cap;
    for (int64_t q = blockIdx.x; q < np; q += gridDim.x) {
        const int64_t* P = A.parts + q * kPartWords;
        const int64_t j = P[0], plo = P[1], phi = P[2], slot = P[4], c = P[5];
        const int64_t vend = A.series_vend[j];
        if (vend < 0) continue;  // the series' scan stopped: its own wave parsed it
        const bool ok = values_part(A.bodies, A.want_ts != 0, plo, phi, vend, A.tmp_v + slot,
                                    A.tmp_t ? A.tmp_t + slot : nullptr, c, lane, lds);
        if (!ok && lane == 0) {
            A.seg[j * kSegWords + 1] = -1;
            A.seg[j * kSegWords + 6] = 0;
        }
    }
}

struct GatherArgs {
    const int64_t* src;    // scratch slot of item j's first value
    const int64_t* count;  // its values (< 0: nothing)
    const int64_t* dst;    // its place in the CSR
    const double* tmp_v;
    const double* tmp_t;
    double* values;
    double* ts;
    int64_t n;
};

__global__ __launch_bounds__(256) void k_json_gather(GatherArgs G) {
    for (int64_t j = blockIdx.x; j < G.n; j += gridDim.x) {
        const int64_t n = G.count[j], src = G.src[j], dst = G.dst[j];
        for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
            G.values[dst + k] = G.tmp_v[src + k];
            if (G.ts) G.ts[dst + k] = G.tmp_t[src + k];
        }
    }
}

}  // namespace json
}  // namespace krr
