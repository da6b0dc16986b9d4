// krr_strip.h — the device packer's staging copy with the sample timestamps cut (round 5).
//
// The reference drops every sample's timestamp (robusta_krr/core/integrations/prometheus.py:152,
// `[Decimal(value) for _, value in ...]`), yet ~30-40% of a query_range body's bytes are
// timestamps, and the device packer's end-to-end rate is bound by the bytes crossing PCIe
// (DESIGN.md §9).  While staging a body this copy writes `[1700000000.25,"0.3"]` as
// `[1,"0.3"]`: the timestamp cut to its first digit — still a JSON number, so the device
// parser (krr_json.h) and the host packer read the stripped body unchanged, and neither reads
// a timestamp's value unless timestamps were asked for (then nothing is stripped).
//
// Contract.  Every maximal run of digits and '.' outside strings is cut to its first byte,
// and a body is stripped only when every such run is a whole JSON number token of the form
// (0|[1-9][0-9]*)(\.[0-9]+)? — no sign or exponent next to it (no e E + - ) / before it, no
// e E after it) — and the body holds no backslash (so the quotes delimit the strings
// exactly); anything else is copied unchanged.  Cutting a valid number token to one digit keeps every
// token of the body in place and every string byte for byte, so the host reader and the
// device parser walk the same structure, read the same value strings, and accept or reject
// the same bodies; the only numbers outside strings in a query_range body are the sample
// timestamps, whose values nobody reads unless timestamps were asked for (then nothing is
// stripped).  When the device rejects a stripped body its batch goes to the host packer,
// which parses the ORIGINAL bodies (krr_amd/core/device_pack.py).
//
// 64 bytes at a time (AVX-512BW masks + VBMI2 compress): the string mask by a carry-less
// prefix XOR of the quotes, runs by "preceded by" relations (bit 63 carried to the next
// block), the fraction digits by one 64-bit addition whose carry runs past them (the byte
// after them must not be a second '.'), the kept bytes by a masked compress store.  Without
// AVX-512 VBMI2 nothing is stripped.
#pragma once

#include <immintrin.h>
#include <stdint.h>
#include <string.h>

namespace krr {
namespace strip {

#define KRR_STRIP_TARGET __attribute__((target("avx512f,avx512bw,avx512vbmi2,bmi,bmi2,pclmul,popcnt")))

inline bool supported() {
    static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                           __builtin_cpu_supports("avx512vbmi2") && __builtin_cpu_supports("bmi2") &&
                           __builtin_cpu_supports("pclmul");
    return ok;
}

KRR_STRIP_TARGET inline uint64_t prefix_xor(uint64_t x) {
    const __m128i v = _mm_clmulepi64_si128(_mm_set_epi64x(0, (long long)x), _mm_set1_epi8((char)0xFF), 0);
    return (uint64_t)_mm_cvtsi128_si64(v);
}

// Carried from one 64-byte block to the next: inside a string, and bit 63 of the class
// masks the "preceded by" relations look back at.
#ifndef KRR_STRIP_MASKED_STORES
#define KRR_STRIP_MASKED_STORES 0  // 1: whole blocks stored with a byte mask too (scripts/strip_bench.cpp:
                                    // plain stores 8-26% faster on the EPYC 9575F host, masked faster on SPR)
#endif
struct StripState {
    uint64_t in_str = 0, cT = 0, cZ = 0, cDt = 0, cX = 0;
    unsigned char cadd = 0;
};

// One block x (bytes `valid`): false when a run breaks the contract, else *keep = the bytes
// the stripped copy keeps.
KRR_STRIP_TARGET __attribute__((always_inline)) inline bool strip_block(StripState& st, __m512i x, uint64_t valid,
                                                                        uint64_t* keep, int64_t* quotes = nullptr) {
    const __m512i kq = _mm512_set1_epi8('"'), kbs = _mm512_set1_epi8('\\'), kdt = _mm512_set1_epi8('.');
    const __m512i k0 = _mm512_set1_epi8('0'), k9 = _mm512_set1_epi8(9);
    const __m512i k20 = _mm512_set1_epi8(0x20), ke = _mm512_set1_epi8('e');
    const __m512i k06 = _mm512_set1_epi8(0x06), k2f = _mm512_set1_epi8(0x2F);
    if (_mm512_mask_cmpeq_epi8_mask(valid, x, kbs)) return false;
    const uint64_t qt = _mm512_mask_cmpeq_epi8_mask(valid, x, kq);
    if (quotes) *quotes += _mm_popcnt_u64(qt);
    const uint64_t dt = _mm512_mask_cmpeq_epi8_mask(valid, x, kdt);
    const uint64_t zr = _mm512_mask_cmpeq_epi8_mask(valid, x, k0);
    const uint64_t dg = _mm512_mask_cmple_epu8_mask(valid, _mm512_sub_epi8(x, k0), k9);
    // exponent letters e / E, and + - (with ) / : x | 6 == '/')
    const uint64_t ee = _mm512_mask_cmpeq_epi8_mask(valid, _mm512_or_si512(x, k20), ke);
    const uint64_t pm = _mm512_mask_cmpeq_epi8_mask(valid, _mm512_or_si512(x, k06), k2f);
    // strings: from an opening quote (set) to its closing quote (clear)
    const uint64_t instr = prefix_xor(qt) ^ st.in_str;
    const uint64_t outside = ~instr & ~qt;
    const uint64_t D = dg & outside, Dt = dt & outside, T = D | Dt;
    const uint64_t sT = (T << 1) | st.cT;
    const uint64_t first = T & ~sT;              // each run's first byte: kept
    const uint64_t Z = first & zr;
    const uint64_t sDt = (Dt << 1) | st.cDt;
    const uint64_t X = (ee | pm) & outside;
    unsigned long long run;                       // fraction digits: the carry runs past them
    const unsigned char cout = _addcarry_u64(st.cadd, D, sDt & D, &run);
    uint64_t bad = first & ~D;                    // a run starts with a digit,
    bad |= ((Z << 1) | st.cZ) & D;                // no leading zero,
    bad |= sDt & ~D;                              // '.' then a digit,
    bad |= run & ~D & Dt;                         // and one '.' at most;
    bad |= first & ((X << 1) | st.cX);            // a whole token: no sign or exponent before
    bad |= ee & outside & sT;                     // nor an exponent after
    if (bad & (valid | (valid + 1))) return false;  // (+ the byte after a partial block)
    *keep = valid & ~(T & sT);                    // a run's bytes after its first
    st.in_str = 0ull - (instr >> 63);
    st.cT = T >> 63, st.cZ = Z >> 63, st.cDt = Dt >> 63, st.cX = X >> 63;
    st.cadd = cout;
    return true;
}

// The span [p, e) stripped into out (e - p bytes of room): bytes written, or -1 when it is
// not strippable (out then holds garbage).  Whole blocks by plain loads and stores (the
// stripped copy never runs ahead of the input, so a 64-byte store stays inside out); the
// last partial block by a masked load and store (nothing read past e or written past the
// stripped end).
// `quotes` (optional): the quotes of [p, e) counted on the way (a local sum, written once: a
// pointer updated per block would alias the output stores and serialise the loop).
#ifndef KRR_STRIP_PREFETCH
#define KRR_STRIP_PREFETCH 0  // bytes ahead of the block to prefetch (0: none)
#endif
template <bool COUNT, int PF = KRR_STRIP_PREFETCH>
KRR_STRIP_TARGET inline int64_t strip_span_t(const char* p, const char* e, char* out, int64_t* quotes) {
    StripState st;
    int64_t nq = 0;
    int64_t* const qp = COUNT ? &nq : nullptr;
    char* o = out;
    while (e - p >= 64) {
        if (PF) _mm_prefetch(p + PF, _MM_HINT_T0);  // past a 4-KiB page the hardware prefetchers stop
        const __m512i x = _mm512_loadu_si512(p);
        uint64_t keep;
        if (!strip_block(st, x, ~0ull, &keep, qp)) return -1;
#if KRR_STRIP_MASKED_STORES
        const unsigned cnt = (unsigned)_mm_popcnt_u64(keep);
        _mm512_mask_storeu_epi8(o, _bzhi_u64(~0ull, cnt), _mm512_maskz_compress_epi8(keep, x));
        o += cnt;
#else
        _mm512_storeu_si512(o, _mm512_maskz_compress_epi8(keep, x));
        o += _mm_popcnt_u64(keep);
#endif
        p += 64;
    }
    if (p < e) {
        const uint64_t valid = _bzhi_u64(~0ull, (unsigned)(e - p));
        const __m512i x = _mm512_maskz_loadu_epi8(valid, p);
        uint64_t keep;
        if (!strip_block(st, x, valid, &keep, qp)) return -1;
        const unsigned cnt = (unsigned)_mm_popcnt_u64(keep);
        _mm512_mask_storeu_epi8(o, _bzhi_u64(~0ull, cnt), _mm512_maskz_compress_epi8(keep, x));
        o += cnt;
    } else if (st.cDt) {
        return -1;  // a '.' ends the body: nothing after it to look at
    }
    if (COUNT) *quotes = nq;
    return o - out;
}

KRR_STRIP_TARGET inline int64_t strip_span(const char* p, const char* e, char* out) {
    return strip_span_t<false>(p, e, out, nullptr);
}
KRR_STRIP_TARGET inline int64_t strip_span(const char* p, const char* e, char* out, int64_t* quotes) {
    return strip_span_t<true>(p, e, out, quotes);
}

inline int64_t strip_body(const char* s, int64_t n, char* out) {
    if (!supported() || n <= 0) return -1;
    return strip_span(s, s + n, out);
}

// ---- one large body stripped by several threads (grouped `sum by (pod)` bodies, ~100 MB each) ----
// A piece may start at a sample's '[' in a values array: `"],[` + a number + `,"` + a value's first
// byte ([0-9+-NI]).  In a valid body that quote CLOSES a string (were it an opening one, the quote
// before the value would close a string and be followed by a value byte, which JSON forbids).
// No token spans that point and the copy's state there is empty (outside a string, no digit,
// '.', sign or exponent before), so the pieces strip apart to what strip_span writes for the
// whole body.  The caller checks it anyway: a strippable body has no backslash, so every quote
// delimits a string, and the quotes each piece's copy counted must be even before every cut;
// when they are not the body is copied unchanged.

inline bool value_start(char c) {
    return (c >= '0' && c <= '9') || c == '+' || c == '-' || c == 'N' || c == 'I';
}

// The first piece start in [p, e) (a pointer to a sample's '['), or nullptr.
inline const char* next_split(const char* p, const char* e) {
    for (; p + 8 < e; ++p) {
        if (p[0] != '"' || p[1] != ']' || p[2] != ',' || p[3] != '[') continue;
        const char* q = p + 4;
        const char* d0 = q;
        while (q < e && *q >= '0' && *q <= '9') ++q;
        if (q == d0) continue;
        if (q < e && *q == '.') {
            const char* f0 = ++q;
            while (q < e && *q >= '0' && *q <= '9') ++q;
            if (q == f0) continue;
        }
        if (q + 2 < e && q[0] == ',' && q[1] == '"' && value_start(q[2])) return p + 3;
    }
    return nullptr;
}

}  // namespace strip
}  // namespace krr
