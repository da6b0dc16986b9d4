// Host build of the device packer's parsing logic (krr_amd/csrc/krr_json_parse.h), for
// the CPU tests (tests/test_json_device_logic.py): the same envelope / element / number
// functions the device kernel runs, composed sequentially.  Test infrastructure only.
#include <stdint.h>

#include "krr_json_parse.h"

using namespace krr::json;

extern "C" int json_check_value(const char* s, int64_t n, double* out) { return value_bits(s, s + n, out); }

extern "C" int json_check_body(const char* s, int64_t n, int want_ts, double* v, double* t, int64_t cap,
                               int64_t* count) {
    Reader r{s, s + n};
    Envelope env{0, 0};
    const char* at = nullptr;
    *count = 0;
    const int code = envelope_head(r, env, &at);
    if (code == 2) return JSON_DROPPED;
    if (code != 1) return JSON_HOST;
    const char* e = s + n;
    const char* p = at;
    const char* vend = nullptr;
    int64_t k = 0;
    if (p < e && *p == ']') {
        vend = p + 1;
    } else if (p < e && *p == '[') {
        for (;;) {
            double vv = 0, tt = 0;
            const char* nx = nullptr;
            bool last = false;
            if (!sample_element(p, e, want_ts != 0, &vv, &tt, &nx, &last, [](const char* q) { return *q; }))
                return JSON_HOST;
            if (k < cap) {
                v[k] = vv;
                if (want_ts) t[k] = tt;
            }
            ++k;
            if (last) {
                vend = nx;
                break;
            }
            p = nx;
        }
    } else {
        return JSON_HOST;
    }
    Reader r2{vend, e};
    if (!envelope_tail(r2, env)) return JSON_HOST;
    *count = k;
    return JSON_OK;
}

// Grouped bodies: every series in order -> (label offset or -1, label length, values
// count) + the values, as the device walk produces them.  Returns JSON_OK / JSON_HOST.
extern "C" int json_check_grouped(const char* s, int64_t n, const char* label, int want_ts, int64_t* lab_off,
                                  int64_t* lab_len, int64_t* counts, int64_t max_series, double* v, double* t,
                                  int64_t cap, int64_t* n_series) {
    GroupedWalker W;
    int64_t ll = 0;
    while (label[ll]) ++ll;
    W.init(s, s + n, label, ll);
    const char* e = s + n;
    int64_t k = 0, ns = 0;
    for (;;) {
        const int ev = W.step();
        if (ev == W_HOST) return JSON_HOST;
        if (ev == W_DONE) break;
        if (ev == W_VALUES) {
            const char* p = W.values_at;
            int64_t c = 0;
            const char* vend = nullptr;
            if (p < e && *p == ']') {
                vend = p + 1;
            } else if (p < e && *p == '[') {
                for (;;) {
                    double vv = 0, tt = 0;
                    const char* nx = nullptr;
                    bool last = false;
                    if (!sample_element(p, e, want_ts != 0, &vv, &tt, &nx, &last, [](const char* q) { return *q; }))
                        return JSON_HOST;
                    if (k < cap) {
                        v[k] = vv;
                        if (want_ts) t[k] = tt;
                    }
                    ++k;
                    ++c;
                    if (last) {
                        vend = nx;
                        break;
                    }
                    p = nx;
                }
            } else {
                return JSON_HOST;
            }
            W.values_done(vend, c);
            continue;
        }
        // W_SERIES
        if (ns < max_series) {
            lab_off[ns] = W.lab ? (int64_t)(W.lab - s) : -1;
            lab_len[ns] = W.lab_len;
            counts[ns] = W.count;
        }
        ++ns;
    }
    *n_series = ns;
    return JSON_OK;
}
