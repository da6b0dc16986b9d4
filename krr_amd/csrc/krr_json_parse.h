// krr_json_parse.h — Prometheus query_range parsing shared by the device packer
// (krr_json.h, one wave per response body) and its host-compiled checks.
//
// What the reference does per pod (robusta_krr/core/integrations/prometheus.py:147-155):
// keep ONLY data.result[0]["values"], drop a pod whose result list is empty, parse each
// sample's value string with Decimal().  The host packer (krr_pack.cpp) restates that
// with a recursive-descent reader and std::from_chars.  This header holds the pieces the
// device restates it with:
//   * decimal -> binary64, correctly rounded: Eisel-Lemire over a 128-bit table of
//     powers of five (krr_pow5.inc, scripts/gen_pow5.py).  With the decimal significand
//     exact in 64 bits (<= 19 significant digits) the 128-bit product always suffices
//     (N. Mushtak and D. Lemire, "Fast number parsing without fallback", Software:
//     Practice and Experience 53(6), 2023), so no big-integer path exists here; a
//     string with more significant digits is handed back to the host packer.
//   * one sample element `[<time>,"<value>"]` of a values array (JSON whitespace between
//     tokens as the host reader allows it);
//   * a small JSON reader for the envelope around that array.
// Contract with the host packer: whatever this code ACCEPTS it parses to exactly the
// bits krr_pack.cpp produces; anything else (whitespace inside a value string,
// escapes, "nan"/"infinity" spellings, > 19 digits, status != "success", a malformed
// body ...) is reported as JSON_HOST and the caller re-parses the batch on the host,
// which yields the host's own result or error.  So the device never invents an error.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define KRR_JHD __host__ __device__
#else
#define KRR_JHD
#endif

namespace krr {
namespace json {

enum : int32_t { JSON_OK = 0, JSON_DROPPED = 1, JSON_HOST = 2 };
enum : int { NUM_OK = 0, NUM_HOST = 1 };

#if defined(__HIP_DEVICE_COMPILE__)
__device__ static const uint64_t kPow5[] = {
#include "krr_pow5.inc"
};
#else
static const uint64_t kPow5[] = {
#include "krr_pow5.inc"
};
#endif

KRR_JHD inline uint64_t mul_hi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

KRR_JHD inline int clz64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __clzll((long long)x);
#else
    return __builtin_clzll(x);
#endif
}

KRR_JHD inline double from_bits(uint64_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double((long long)u);
#else
    double d;
    __builtin_memcpy(&d, &u, 8);
    return d;
#endif
}

// w * 10^q correctly rounded to binary64 (ties to even), w != 0 exact, as IEEE bits
// without the sign.  Eisel-Lemire (fast_float's compute_float restated).
KRR_JHD inline uint64_t eisel_lemire(uint64_t w, int64_t q) {
    if (w == 0 || q < -342) return 0;
    if (q > 308) return 0x7FF0000000000000ull;
    const int lz = clz64(w);
    w <<= lz;
    const int idx = 2 * (int)(q + 342);
    uint64_t hi = mul_hi64(w, kPow5[idx]);
    uint64_t lo = w * kPow5[idx];
    if ((hi & 0x1FF) == 0x1FF) {  // the 64-bit product leaves the rounding bits unsure
        const uint64_t hi2 = mul_hi64(w, kPow5[idx + 1]);
        lo += hi2;
        if (hi2 > lo) ++hi;
    }
    const int upper = (int)(hi >> 63);
    const int shift = upper + 9;
    uint64_t m = hi >> shift;
    // power(q) = floor(q * log2(10)) + 63
    int32_t p2 = (int32_t)((((152170 + 65536) * (int64_t)q) >> 16) + 63) + upper - lz + 1023;
    if (p2 <= 0) {  // subnormal (or zero)
        if (-p2 + 1 >= 64) return 0;
        m >>= -p2 + 1;
        m += m & 1;
        m >>= 1;
        p2 = m < (1ull << 52) ? 0 : 1;
        return ((uint64_t)p2 << 52) | (m & ((1ull << 52) - 1));
    }
    // an exact halfway case rounds to even (possible only for q in [-4, 23])
    if (lo <= 1 && q >= -4 && q <= 23 && (m & 3) == 1 && (m << shift) == hi) m &= ~1ull;
    m += m & 1;
    m >>= 1;
    if (m >= (2ull << 52)) {
        m = 1ull << 52;
        ++p2;
    }
    m &= ~(1ull << 52);
    if (p2 >= 0x7FF) return 0x7FF0000000000000ull;
    return ((uint64_t)p2 << 52) | m;
}

KRR_JHD inline bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }

// One pass over a number at p (advanced past it): a JSON number (the sample's timestamp;
// grammar of the host reader's Reader::num, -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?)
// or, with value_form, a sample value string's contents (krr_pack.cpp parse_value: an
// optional sign, then digits with an optional fraction and exponent, or "NaN" / "Inf" —
// Prometheus' spellings; std::from_chars' other spellings are the host's call).  The
// digits are read once: grammar, significand and exponent together.  false: not
// accepted here (more than 19 significant digits or 6 exponent digits included).
template <class Load>
KRR_JHD inline bool scan_number(const char*& p, const char* e, Load ld, bool value_form, uint64_t* out_bits) {
    uint64_t sign = 0;
    if (p < e) {
        const char c = ld(p);
        if (c == '-') {
            sign = 0x8000000000000000ull;
            ++p;
        } else if (c == '+' && value_form) {
            ++p;
        }
    }
    if (p >= e) return false;
    char c = ld(p);
    if (value_form && (c == 'N' || c == 'I')) {
        if (e - p < 3) return false;
        const char c1 = ld(p + 1), c2 = ld(p + 2);
        if (c == 'N' && c1 == 'a' && c2 == 'N') {
            *out_bits = 0x7FF8000000000000ull | sign;
        } else if (c == 'I' && c1 == 'n' && c2 == 'f') {
            *out_bits = 0x7FF0000000000000ull | sign;
        } else {
            return false;
        }
        p += 3;
        return true;
    }
    if (!is_digit((unsigned char)c)) return false;
    uint64_t w = 0;
    int nd = 0;          // significant digits taken into w
    int64_t drop = 0;    // power of ten of w's last digit
    bool lost = false;   // a nonzero digit beyond the 19th
    if (!value_form && c == '0') {  // JSON: a lone leading zero
        ++p;
        if (p < e && is_digit((unsigned char)ld(p))) return false;
    } else {
        for (; p < e; ++p) {
            c = ld(p);
            if (!is_digit((unsigned char)c)) break;
            const unsigned d = (unsigned)(c - '0');
            if (nd == 0 && d == 0) continue;  // leading zero
            if (nd < 19) {
                w = w * 10 + d;
                ++nd;
            } else {
                ++drop;
                lost |= d != 0;
            }
        }
    }
    if (p < e && ld(p) == '.') {
        ++p;
        if (p >= e || !is_digit((unsigned char)ld(p))) return false;
        for (; p < e; ++p) {
            c = ld(p);
            if (!is_digit((unsigned char)c)) break;
            const unsigned d = (unsigned)(c - '0');
            if (nd == 0 && d == 0) {
                --drop;
            } else if (nd < 19) {
                w = w * 10 + d;
                ++nd;
                --drop;
            } else {
                lost |= d != 0;
            }
        }
    }
    int64_t ex = 0;
    if (p < e && (ld(p) == 'e' || ld(p) == 'E')) {
        ++p;
        bool eneg = false;
        if (p < e && (ld(p) == '+' || ld(p) == '-')) {
            eneg = ld(p) == '-';
            ++p;
        }
        int ne = 0;
        for (; p < e; ++p) {
            c = ld(p);
            if (!is_digit((unsigned char)c)) break;
            ex = ex * 10 + (c - '0');
            if (++ne > 6) return false;
        }
        if (ne == 0) return false;
        if (eneg) ex = -ex;
    }
    if (lost) return false;
    *out_bits = eisel_lemire(w, drop + ex) | sign;
    return true;
}

struct PlainLoad {
    KRR_JHD char operator()(const char* q) const { return *q; }
};

// A JSON number's end (grammar only), or nullptr.
KRR_JHD inline const char* json_number_end(const char* p, const char* e) {
    if (p < e && *p == '-') ++p;
    if (p >= e) return nullptr;
    if (*p == '0') {
        ++p;
    } else if (*p >= '1' && *p <= '9') {
        while (p < e && is_digit((unsigned char)*p)) ++p;
    } else {
        return nullptr;
    }
    if (p < e && *p == '.') {
        ++p;
        if (p >= e || !is_digit((unsigned char)*p)) return nullptr;
        while (p < e && is_digit((unsigned char)*p)) ++p;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
        ++p;
        if (p < e && (*p == '+' || *p == '-')) ++p;
        if (p >= e || !is_digit((unsigned char)*p)) return nullptr;
        while (p < e && is_digit((unsigned char)*p)) ++p;
    }
    return p;
}

// A whole sample value string [b, e) -> float64 (NUM_OK), else NUM_HOST.
KRR_JHD inline int value_bits(const char* b, const char* e, double* out) {
    const char* p = b;
    uint64_t bits;
    if (!scan_number(p, e, PlainLoad{}, true, &bits) || p != e) return NUM_HOST;
    *out = from_bits(bits);
    return NUM_OK;
}

template <class Load>
KRR_JHD inline void skip_ws(const char*& p, const char* e, Load ld) {
    while (p < e) {
        const char c = ld(p);
        if (c != ' ' && c != '\n' && c != '\r' && c != '\t') break;
        ++p;
    }
}

// One element of a values array at p (which must be '['): `[<json number>,"<value>"]`
// followed by ',' + '[' (more follow) or ']' (the last one); JSON whitespace between the
// tokens as the host reader allows it (none inside the value string).  On success: *next =
// the following element's '[' or one past the array's ']', *last set.  Returns false for
// anything else (the caller hands the body to the host).  One pass: every byte is read
// once through ld.
template <class Load>
KRR_JHD inline bool sample_element(const char* p, const char* e, bool want_ts, double* value, double* ts,
                                   const char** next, bool* last, Load ld) {
    if (p >= e || ld(p) != '[') return false;
    ++p;
    skip_ws(p, e, ld);
    uint64_t tb;
    if (!scan_number(p, e, ld, false, &tb)) return false;
    skip_ws(p, e, ld);
    if (p >= e || ld(p) != ',') return false;
    ++p;
    skip_ws(p, e, ld);
    if (p >= e || ld(p) != '"') return false;
    ++p;
    uint64_t vb;
    if (!scan_number(p, e, ld, true, &vb)) return false;
    if (p >= e || ld(p) != '"') return false;
    ++p;
    skip_ws(p, e, ld);
    if (p >= e || ld(p) != ']') return false;
    ++p;
    skip_ws(p, e, ld);
    if (p >= e) return false;
    const char d = ld(p);
    if (d == ',') {
        ++p;
        skip_ws(p, e, ld);
        if (p >= e || ld(p) != '[') return false;
        *last = false;
        *next = p;
    } else if (d == ']') {
        *last = true;
        *next = p + 1;
    } else {
        return false;
    }
    *value = from_bits(vb);
    if (want_ts) *ts = from_bits(tb);
    return true;
}

// ---- the envelope: a small JSON reader ----------------------------------------
// Keys and the status value may not hold escapes here (the host decides those).
struct Reader {
    const char* p;
    const char* e;

    KRR_JHD void ws() {
        while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    KRR_JHD bool lit(char c) {
        ws();
        if (p < e && *p == c) {
            ++p;
            return true;
        }
        return false;
    }
    KRR_JHD bool peek(char c) {
        ws();
        return p < e && *p == c;
    }
    // A string; [*b, *n) = its raw bytes; *esc: it holds escapes.  Grammar as the host's.
    KRR_JHD bool str(const char** b, int64_t* n, bool* esc) {
        ws();
        if (p >= e || *p != '"') return false;
        const char* s = ++p;
        bool any = false;
        while (p < e && *p != '"') {
            const unsigned char c = (unsigned char)*p;
            if (c < 0x20) return false;
            if (c == '\\') {
                any = true;
                if (++p >= e) return false;
                if (*p == 'u') {
                    if (e - p < 5) return false;
                    for (int k = 1; k <= 4; ++k) {
                        const char h = p[k];
                        if (!((h >= '0' && h <= '9') || (h >= 'a' && h <= 'f') || (h >= 'A' && h <= 'F'))) return false;
                    }
                    p += 4;
                } else {
                    const char c2 = *p;
                    if (!(c2 == '"' || c2 == '\\' || c2 == '/' || c2 == 'b' || c2 == 'f' || c2 == 'n' || c2 == 'r' ||
                          c2 == 't'))
                        return false;
                }
            }
            ++p;
        }
        if (p >= e) return false;
        if (b) *b = s;
        if (n) *n = p - s;
        if (esc) *esc = any;
        ++p;
        return true;
    }
    // A key equal to k (no escapes): 1; another key without escapes: 0; escapes or a
    // malformed key: -1 (the host's call).
    KRR_JHD int key(const char* k) {
        const char* b;
        int64_t n;
        bool esc;
        if (!str(&b, &n, &esc) || esc) return -1;
        if (!lit(':')) return -1;
        int64_t i = 0;
        for (; k[i]; ++i)
            if (i >= n || b[i] != k[i]) return 0;
        return i == n ? 1 : 0;
    }
    KRR_JHD bool word(const char* w) {
        ws();
        int64_t n = 0;
        while (w[n]) ++n;
        if (e - p < n) return false;
        for (int64_t i = 0; i < n; ++i)
            if (p[i] != w[i]) return false;
        p += n;
        return true;
    }
    // Skip one JSON value, validating it (iterative: an explicit stack of up to 256
    // open containers, the host reader's depth bound).
    KRR_JHD bool skip() {
        uint64_t stk[5] = {0, 0, 0, 0, 0};  // bit d: container d is an object
        int d = 0;
        for (;;) {
            // a value
            ws();
            if (p >= e || d > 256) return false;
            const char c = *p;
            bool opened = false;
            if (c == '{' || c == '[') {
                ++p;
                const bool obj = c == '{';
                if (obj) stk[d >> 6] |= 1ull << (d & 63);
                else stk[d >> 6] &= ~(1ull << (d & 63));
                ++d;
                if (lit(obj ? '}' : ']')) {
                    --d;
                } else {
                    if (obj && (!str(nullptr, nullptr, nullptr) || !lit(':'))) return false;
                    opened = true;
                }
            } else if (c == '"') {
                if (!str(nullptr, nullptr, nullptr)) return false;
            } else if (c == 't') {
                if (!word("true")) return false;
            } else if (c == 'f') {
                if (!word("false")) return false;
            } else if (c == 'n') {
                if (!word("null")) return false;
            } else {
                const char* q = json_number_end(p, e);
                if (!q) return false;
                p = q;
            }
            if (opened) continue;  // its first member / element
            // after a value: close containers or move to the next member / element
            for (;;) {
                if (d == 0) return true;
                const bool obj = (stk[(d - 1) >> 6] >> ((d - 1) & 63)) & 1;
                if (lit(',')) {
                    if (obj && (!str(nullptr, nullptr, nullptr) || !lit(':'))) return false;
                    break;
                }
                if (!lit(obj ? '}' : ']')) return false;
                --d;
            }
        }
    }
};

// Where the envelope parse stands when it reaches result[0]'s "values" array.
struct Envelope {
    int32_t have_status, ok_status;
};

// From the body start to just inside result[0]["values"]'s '[' (returns 1, *at = that
// position), or through the whole body when the result list is empty (returns 2: a
// dropped pod, everything validated), or 0: the host decides.
KRR_JHD inline int envelope_head(Reader& r, Envelope& env, const char** at) {
    env.have_status = env.ok_status = 0;
    bool have_result = false, dropped = false;
    if (!r.lit('{') || r.peek('}')) return 0;
    for (;;) {
        const char* kb;
        int64_t kn;
        bool kesc;
        if (!r.str(&kb, &kn, &kesc) || kesc || !r.lit(':')) return 0;
        const bool is_status = kn == 6 && kb[0] == 's' && kb[1] == 't' && kb[2] == 'a' && kb[3] == 't' &&
                               kb[4] == 'u' && kb[5] == 's';
        const bool is_data = kn == 4 && kb[0] == 'd' && kb[1] == 'a' && kb[2] == 't' && kb[3] == 'a';
        if (is_status) {
            const char* vb;
            int64_t vn;
            bool vesc;
            if (!r.str(&vb, &vn, &vesc) || vesc) return 0;
            env.have_status = 1;
            env.ok_status = vn == 7 && vb[0] == 's' && vb[1] == 'u' && vb[2] == 'c' && vb[3] == 'c' && vb[4] == 'e' &&
                            vb[5] == 's' && vb[6] == 's';
        } else if (is_data) {
            if (have_result || dropped || !r.lit('{')) return 0;
            if (!r.lit('}')) {
                for (;;) {
                    const int k = r.key("result");
                    if (k < 0) return 0;
                    if (k == 0) {
                        if (!r.skip()) return 0;
                    } else {
                        if (have_result || !r.lit('[')) return 0;
                        have_result = true;
                        if (r.lit(']')) {
                            dropped = true;
                        } else {
                            if (!r.lit('{') || r.peek('}')) return 0;
                            for (;;) {
                                const int sk = r.key("values");
                                if (sk < 0) return 0;
                                if (sk == 1) {
                                    if (!r.lit('[')) return 0;
                                    r.ws();
                                    *at = r.p;
                                    return 1;
                                }
                                if (!r.skip() || !r.lit(',')) return 0;  // no "values" in result[0]: host
                            }
                        }
                    }
                    if (r.lit(',')) continue;
                    if (!r.lit('}')) return 0;
                    break;
                }
            }
        } else if (!r.skip()) {
            return 0;
        }
        if (r.lit(',')) continue;
        if (!r.lit('}')) return 0;
        break;
    }
    r.ws();
    if (r.p != r.e || !dropped || !env.have_status || !env.ok_status) return 0;
    return 2;
}

// From one past the values array's ']' to the end of the body: the rest of result[0],
// further series (validated, never read), the rest of data and of the response.
KRR_JHD inline bool envelope_tail(Reader& r, Envelope env) {
    // rest of result[0]
    while (r.lit(',')) {
        const int k = r.key("values");
        if (k != 0 || !r.skip()) return false;  // a second "values": the host's call
    }
    if (!r.lit('}')) return false;
    // further series
    while (r.lit(','))
        if (!r.skip()) return false;
    if (!r.lit(']')) return false;
    // rest of data
    while (r.lit(',')) {
        const int k = r.key("result");
        if (k != 0 || !r.skip()) return false;
    }
    if (!r.lit('}')) return false;
    // rest of the response
    while (r.lit(',')) {
        const char* kb;
        int64_t kn;
        bool kesc;
        if (!r.str(&kb, &kn, &kesc) || kesc || !r.lit(':')) return false;
        const bool is_status = kn == 6 && kb[0] == 's' && kb[1] == 't' && kb[2] == 'a' && kb[3] == 't' &&
                               kb[4] == 'u' && kb[5] == 's';
        const bool is_data = kn == 4 && kb[0] == 'd' && kb[1] == 'a' && kb[2] == 't' && kb[3] == 'a';
        if (is_data) return false;
        if (is_status) {
            const char* vb;
            int64_t vn;
            bool vesc;
            if (!r.str(&vb, &vn, &vesc) || vesc) return false;
            env.have_status = 1;
            env.ok_status = vn == 7 && vb[0] == 's' && vb[1] == 'u' && vb[2] == 'c' && vb[3] == 'c' && vb[4] == 'e' &&
                            vb[5] == 's' && vb[6] == 's';
        } else if (!r.skip()) {
            return false;
        }
    }
    if (!r.lit('}')) return false;
    r.ws();
    return r.p == r.e && env.have_status && env.ok_status;
}


// ---- grouped responses: every series of data.result, routed by a metric label ----
// ("sum by (pod) (...)" bodies, krr_amd.core.fleet_query; the host restatement is
// krr_pack.cpp parse_series_set).  A resumable walk over the envelope: step() runs until
// the next values array starts (W_VALUES: the caller parses it, then values_done()), a
// series ends (W_SERIES: its label span and values are final), or the body ends
// (W_DONE) / leaves the device grammar (W_HOST).
enum : int { W_HOST = 0, W_VALUES = 1, W_SERIES = 2, W_DONE = 3, W_AT_SERIES = 4 };

struct GroupedWalker {
    enum : int { TOP_OPEN, TOP_KEY, TOP_NEXT, DATA_KEY, DATA_NEXT, SERIES_OPEN, SERIES_KEY, SERIES_NEXT, RESULT_NEXT };
    Reader r;
    const char* label;   // the routing label key (no escapes)
    int64_t label_len;
    int state;
    bool have_status, ok_status, have_result, have_data;
    bool stop_at_series;  // step() returns W_AT_SERIES before each series object (r.p at its '{')
    // the current series
    int64_t index;        // 0-based position in data.result
    const char* lab;      // its label value (raw bytes, no escapes) or nullptr
    int64_t lab_len;
    bool have_values, have_metric;
    const char* values_at;  // its values array's first byte after '['
    int64_t count;

    KRR_JHD void init(const char* s, const char* e, const char* lbl, int64_t lbl_len) {
        r.p = s;
        r.e = e;
        label = lbl;
        label_len = lbl_len;
        state = TOP_OPEN;
        have_status = ok_status = have_result = have_data = false;
        stop_at_series = false;
        index = -1;
    }
    // Resume inside data.result: at a series object (SERIES_OPEN) or right after one
    // (RESULT_NEXT), at p.  The envelope flags are the head walk's.
    KRR_JHD void resume(const char* p, int st) {
        r.p = p;
        state = st;
    }
    KRR_JHD bool key_is(const char* kb, int64_t kn, const char* k, int64_t n) const {
        if (kn != n) return false;
        for (int64_t i = 0; i < n; ++i)
            if (kb[i] != k[i]) return false;
        return true;
    }
    KRR_JHD void values_done(const char* vend, int64_t n) {
        r.p = vend;
        count = n;
        state = SERIES_NEXT;
    }
    KRR_JHD int step() {
        for (;;) {
            switch (state) {
                case TOP_OPEN:
                    if (!r.lit('{') || r.peek('}')) return W_HOST;
                    state = TOP_KEY;
                    break;
                case TOP_KEY: {
                    const char* kb;
                    int64_t kn;
                    bool kesc;
                    if (!r.str(&kb, &kn, &kesc) || kesc || !r.lit(':')) return W_HOST;
                    if (key_is(kb, kn, "status", 6)) {
                        const char* vb;
                        int64_t vn;
                        bool vesc;
                        if (!r.str(&vb, &vn, &vesc) || vesc) return W_HOST;
                        have_status = true;
                        ok_status = key_is(vb, vn, "success", 7);
                        state = TOP_NEXT;
                    } else if (key_is(kb, kn, "data", 4)) {
                        if (have_data || !r.lit('{')) return W_HOST;
                        have_data = true;
                        state = r.lit('}') ? TOP_NEXT : DATA_KEY;
                    } else {
                        if (!r.skip()) return W_HOST;
                        state = TOP_NEXT;
                    }
                    break;
                }
                case TOP_NEXT:
                    if (r.lit(',')) {
                        state = TOP_KEY;
                        break;
                    }
                    if (!r.lit('}')) return W_HOST;
                    r.ws();
                    return (r.p == r.e && have_status && ok_status && have_result) ? W_DONE : W_HOST;
                case DATA_KEY: {
                    const int k = r.key("result");
                    if (k < 0) return W_HOST;
                    if (k == 0) {
                        if (!r.skip()) return W_HOST;
                        state = DATA_NEXT;
                        break;
                    }
                    if (have_result || !r.lit('[')) return W_HOST;
                    have_result = true;
                    state = r.lit(']') ? DATA_NEXT : SERIES_OPEN;
                    break;
                }
                case DATA_NEXT:
                    if (r.lit(',')) {
                        state = DATA_KEY;
                        break;
                    }
                    if (!r.lit('}')) return W_HOST;
                    state = TOP_NEXT;
                    break;
                case SERIES_OPEN:
                    if (stop_at_series) {
                        r.ws();
                        return W_AT_SERIES;
                    }
                    if (!r.lit('{') || r.peek('}')) return W_HOST;  // a series without values: the host's error
                    ++index;
                    lab = nullptr;
                    lab_len = 0;
                    have_values = have_metric = false;
                    values_at = nullptr;
                    count = 0;
                    state = SERIES_KEY;
                    break;
                case SERIES_KEY: {
                    const char* kb;
                    int64_t kn;
                    bool kesc;
                    if (!r.str(&kb, &kn, &kesc) || kesc || !r.lit(':')) return W_HOST;
                    if (key_is(kb, kn, "metric", 6)) {
                        if (have_metric || !r.lit('{')) return W_HOST;
                        have_metric = true;
                        if (!r.lit('}')) {
                            for (;;) {
                                const char* lb;
                                int64_t ln;
                                bool lesc;
                                if (!r.str(&lb, &ln, &lesc) || lesc || !r.lit(':')) return W_HOST;
                                if (key_is(lb, ln, label, label_len)) {
                                    const char* vb;
                                    int64_t vn;
                                    bool vesc;
                                    if (!r.str(&vb, &vn, &vesc) || vesc) return W_HOST;
                                    lab = vb;  // the last one, as the host keeps it
                                    lab_len = vn;
                                } else if (!r.skip()) {
                                    return W_HOST;
                                }
                                if (r.lit(',')) continue;
                                if (!r.lit('}')) return W_HOST;
                                break;
                            }
                        }
                        state = SERIES_NEXT;
                    } else if (key_is(kb, kn, "values", 6)) {
                        if (have_values || !r.lit('[')) return W_HOST;
                        have_values = true;
                        r.ws();
                        values_at = r.p;
                        return W_VALUES;  // the caller parses the array, then values_done()
                    } else {
                        if (!r.skip()) return W_HOST;
                        state = SERIES_NEXT;
                    }
                    break;
                }
                case SERIES_NEXT:
                    if (r.lit(',')) {
                        state = SERIES_KEY;
                        break;
                    }
                    if (!r.lit('}') || !have_values) return W_HOST;
                    state = RESULT_NEXT;
                    return W_SERIES;
                case RESULT_NEXT:
                    if (r.lit(',')) {
                        state = SERIES_OPEN;
                        break;
                    }
                    if (!r.lit(']')) return W_HOST;
                    state = DATA_NEXT;
                    break;
                default:
                    return W_HOST;
            }
        }
    }
};


// Chain check of one grouped body (host side of the device packer): the head walk finds
// data.result's first series; segment records (parsed on the device, one wave per series
// object, found by the `{"metric":` pattern) must then follow each other exactly — series
// k ends where series k + 1 starts (a ',' and whitespace between them) — until the one
// followed by ']';
// then the tail walk validates the rest.  seg[j] = {start, end, label_off, label_len,
// slot, count, ok} (absolute byte offsets, sorted by start); find(pos) returns the index of
// the segment starting at pos or -1.  Emits each chained series in order through emit(j).
// Returns false when the body is not canonical (the caller hands it to the host packer).
template <class Find, class Emit>
inline bool chain_grouped(const char* buf, int64_t ob, int64_t oe, const char* label, int64_t label_len,
                          const int64_t* seg, Find find, Emit emit) {
    GroupedWalker W;
    W.init(buf + ob, buf + oe, label, label_len);
    W.stop_at_series = true;
    int ev = W.step();
    if (ev == W_DONE) return true;   // no series (empty result)
    if (ev != W_AT_SERIES) return false;
    const char* p = W.r.p;
    for (;;) {
        const int64_t j = find((int64_t)(p - buf));
        if (j < 0 || !seg[7 * j + 6]) return false;
        emit(j);
        const char* q = buf + seg[7 * j + 1];  // one past the series' '}'
        skip_ws(q, buf + oe, PlainLoad{});
        if (q >= buf + oe) return false;
        if (*q == ',') {
            p = q + 1;
            skip_ws(p, buf + oe, PlainLoad{});
            if (p >= buf + oe || *p != '{') return false;
            continue;
        }
        if (*q != ']') return false;
        W.resume(q, GroupedWalker::RESULT_NEXT);
        W.stop_at_series = false;
        return W.step() == W_DONE;
    }
}

// chain_grouped over a staged copy in pieces (krr_pack_route_grouped_pieces): M.at(pos) = the
// byte at device position pos, M.end(pos) = one past the last position of pos's piece.  Pieces
// cut a body only inside values arrays, so the head walk (to the first series), the bytes after
// each series and the tail each lie inside one piece.
template <class Map, class Find, class Emit>
inline bool chain_grouped_mapped(const Map& M, int64_t ob, int64_t oe, const char* label, int64_t label_len,
                                 const int64_t* seg, Find find, Emit emit) {
    GroupedWalker W;
    const char* h = M.at(ob);
    const int64_t he = M.end(ob) < oe ? M.end(ob) : oe;
    W.init(h, h + (he - ob), label, label_len);
    W.stop_at_series = true;
    int ev = W.step();
    if (ev == W_DONE) return true;   // no series (empty result)
    if (ev != W_AT_SERIES) return false;
    int64_t pos = ob + (W.r.p - h);
    for (;;) {
        const int64_t j = find(pos);
        if (j < 0 || !seg[7 * j + 6]) return false;
        emit(j);
        const int64_t qp = seg[7 * j + 1];  // one past the series' '}'
        if (qp >= oe) return false;
        const char* q0 = M.at(qp);
        const int64_t qend = M.end(qp) < oe ? M.end(qp) : oe;
        const char* qe = q0 + (qend - qp);
        const char* q = q0;
        skip_ws(q, qe, PlainLoad{});
        if (q >= qe) return false;
        if (*q == ',') {
            const char* p = q + 1;
            skip_ws(p, qe, PlainLoad{});
            if (p >= qe || *p != '{') return false;
            pos = qp + (p - q0);
            continue;
        }
        if (*q != ']') return false;
        W.r.e = qe;
        W.resume(q, GroupedWalker::RESULT_NEXT);
        W.stop_at_series = false;
        return W.step() == W_DONE && qe == q0 + (oe - qp);  // the tail ends the body, in this piece
    }
}

}  // namespace json
}  // namespace krr
