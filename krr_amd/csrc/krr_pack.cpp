// krr_pack.cpp — native Prometheus query_range packer (host C++17, std::thread).
//
// The reference parses every pod's response in Python: response.json() in
// prometheus_api_client, then Decimal(value) per sample (prometheus.py:147-155),
// ~4.6 M samples/s on one core.  Here each body is scanned
// once by a small recursive-descent JSON reader that walks only the path it
// needs (status, data.result[0].values) and skips everything else (metric
// labels, further series) while still validating it; numbers go through
// std::from_chars.  Bodies are independent, so a pool of threads parses them in
// parallel, then the kept samples are copied into one CSR buffer.
#include "krr_pack.h"
#include "krr_json_parse.h"
#include "krr_strip.h"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <pthread.h>
#include <sched.h>
#include <cstdlib>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <new>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

double strtod_exact(const char* b, const char* e);

struct Reader {
    const char* p;
    const char* e;
    int depth = 0;

    void ws() {
        while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    bool lit(char c) {
        ws();
        if (p < e && *p == c) {
            ++p;
            return true;
        }
        return false;
    }
    bool peek(char c) {
        ws();
        return p < e && *p == c;
    }
    // A JSON string; *raw = its bytes between the quotes (escapes not decoded).
    bool str(std::string_view* raw, bool* esc) {
        ws();
        if (p >= e || *p != '"') return false;
        const char* b = ++p;
        bool any = false;
        while (p < e && *p != '"') {
            const unsigned char c = (unsigned char)*p;
            if (c < 0x20) return false;
            if (c == '\\') {
                any = true;
                if (++p >= e) return false;
                if (*p == 'u') {
                    if (e - p < 5) return false;
                    for (int k = 1; k <= 4; ++k)
                        if (!isxdigit((unsigned char)p[k])) return false;
                    p += 4;
                } else if (!strchr("\"\\/bfnrt", *p)) {
                    return false;
                }
            }
            ++p;
        }
        if (p >= e) return false;
        if (raw) *raw = std::string_view(b, (size_t)(p - b));
        if (esc) *esc = any;
        ++p;
        return true;
    }
    // JSON number (grammar checked), value via from_chars.
    bool num(double* out) {
        ws();
        const char* b = p;
        if (p < e && *p == '-') ++p;
        if (p >= e) return false;
        if (*p == '0') {
            ++p;
        } else if (*p >= '1' && *p <= '9') {
            while (p < e && isdigit((unsigned char)*p)) ++p;
        } else {
            return false;
        }
        if (p < e && *p == '.') {
            ++p;
            if (p >= e || !isdigit((unsigned char)*p)) return false;
            while (p < e && isdigit((unsigned char)*p)) ++p;
        }
        if (p < e && (*p == 'e' || *p == 'E')) {
            ++p;
            if (p < e && (*p == '+' || *p == '-')) ++p;
            if (p >= e || !isdigit((unsigned char)*p)) return false;
            while (p < e && isdigit((unsigned char)*p)) ++p;
        }
        if (out) {
            auto r = std::from_chars(b, p, *out);
            if (r.ec == std::errc::result_out_of_range) *out = strtod_exact(b, p);
            else if (r.ec != std::errc()) return false;
        }
        return true;
    }
    bool word(const char* w) {
        ws();
        const size_t n = strlen(w);
        if ((size_t)(e - p) < n || memcmp(p, w, n) != 0) return false;
        p += n;
        return true;
    }
    bool skip() {
        ws();
        if (p >= e || depth > 256) return false;
        switch (*p) {
            case '{': {
                ++p;
                ++depth;
                if (lit('}')) {
                    --depth;
                    return true;
                }
                do {
                    if (!str(nullptr, nullptr) || !lit(':') || !skip()) return false;
                } while (lit(','));
                --depth;
                return lit('}');
            }
            case '[': {
                ++p;
                ++depth;
                if (lit(']')) {
                    --depth;
                    return true;
                }
                do {
                    if (!skip()) return false;
                } while (lit(','));
                --depth;
                return lit(']');
            }
            case '"':
                return str(nullptr, nullptr);
            case 't':
                return word("true");
            case 'f':
                return word("false");
            case 'n':
                return word("null");
            default:
                return num(nullptr);
        }
    }
};

// Decode a JSON string body (escapes) for key comparison.
std::string unescape(std::string_view s) {
    std::string o;
    o.reserve(s.size());
    for (size_t i = 0; i < s.size(); ++i) {
        char c = s[i];
        if (c != '\\') {
            o.push_back(c);
            continue;
        }
        c = s[++i];
        switch (c) {
            case 'b': o.push_back('\b'); break;
            case 'f': o.push_back('\f'); break;
            case 'n': o.push_back('\n'); break;
            case 'r': o.push_back('\r'); break;
            case 't': o.push_back('\t'); break;
            case 'u': {
                unsigned v = 0;
                std::from_chars(s.data() + i + 1, s.data() + i + 5, v, 16);
                i += 4;
                if (v < 0x80) o.push_back((char)v);
                else o.push_back('?');  // non-ASCII never matches our keys
                break;
            }
            default: o.push_back(c);
        }
    }
    return o;
}

bool key_is(std::string_view raw, bool esc, const char* k) {
    return esc ? unescape(raw) == k : raw == k;
}

// from_chars leaves the value unspecified on a range error; strtod (C locale)
// returns the correctly rounded result there: +-HUGE_VAL, 0, or a subnormal.
double strtod_exact(const char* b, const char* e) {
    const std::string tmp(b, e);
    return strtod(tmp.c_str(), nullptr);
}

// Prometheus sample value string -> float64 (what Decimal(string) denotes, rounded).
bool parse_value(std::string_view s, double* out) {
    const char* b = s.data();
    const char* e = b + s.size();
    bool neg = false;
    if (b < e && (*b == '+' || *b == '-')) {
        neg = *b == '-';
        ++b;
    }
    if (b >= e || *b == '+' || *b == '-') return false;
    double v;
    auto r = std::from_chars(b, e, v);
    if (r.ptr != e) return false;
    if (r.ec == std::errc::result_out_of_range) {
        v = strtod_exact(b, e);  // overflow -> inf, underflow -> 0 or the subnormal
    } else if (r.ec != std::errc()) {
        return false;
    }
    *out = neg ? -v : v;
    return true;
}

struct Body {
    std::vector<double> v, t;
    // grouped packing: the samples live in the parsed series set (no copy)
    const std::vector<double>* pv = nullptr;
    const std::vector<double>* pt = nullptr;
    const std::vector<double>& V() const { return pv ? *pv : v; }
    const std::vector<double>& T() const { return pt ? *pt : t; }
    int status = KRR_PACK_OK;
    bool dropped = false;
    std::string err;
};

// One query_range response: {"status": "success", "data": {"resultType": ..., "result": [...]}}
void parse_body(const char* s, int64_t n, bool want_ts, Body& out) {
    Reader r{s, s + n};
    auto fail = [&](int code, const char* what) {
        out.status = code;
        char buf[160];
        snprintf(buf, sizeof(buf), "%s at byte %lld", what, (long long)(r.p - s));
        out.err = buf;
    };
    bool have_status = false, ok_status = false, have_result = false;
    if (!r.lit('{')) return fail(KRR_PACK_E_PARSE, "expected a JSON object");
    if (!r.peek('}')) {
        do {
            std::string_view k;
            bool esc;
            if (!r.str(&k, &esc) || !r.lit(':')) return fail(KRR_PACK_E_PARSE, "bad object key");
            if (key_is(k, esc, "status")) {
                std::string_view v;
                bool vesc;
                if (!r.str(&v, &vesc)) return fail(KRR_PACK_E_PARSE, "status is not a string");
                have_status = true;
                ok_status = key_is(v, vesc, "success");
            } else if (key_is(k, esc, "data")) {
                if (!r.lit('{')) return fail(KRR_PACK_E_PARSE, "data is not an object");
                if (!r.peek('}')) {
                    do {
                        std::string_view dk;
                        bool desc;
                        if (!r.str(&dk, &desc) || !r.lit(':')) return fail(KRR_PACK_E_PARSE, "bad data key");
                        if (!key_is(dk, desc, "result")) {
                            if (!r.skip()) return fail(KRR_PACK_E_PARSE, "malformed JSON");
                            continue;
                        }
                        if (!r.lit('[')) return fail(KRR_PACK_E_PARSE, "result is not an array");
                        have_result = true;
                        if (r.lit(']')) {
                            out.dropped = true;  // prometheus.py:154: a pod with no series is dropped
                            continue;
                        }
                        // result[0]: the only series the reference reads (pod_result[0]["values"])
                        if (!r.lit('{')) return fail(KRR_PACK_E_PARSE, "series is not an object");
                        bool have_values = false;
                        if (!r.peek('}')) {
                            do {
                                std::string_view sk;
                                bool sesc;
                                if (!r.str(&sk, &sesc) || !r.lit(':')) return fail(KRR_PACK_E_PARSE, "bad series key");
                                if (!key_is(sk, sesc, "values")) {
                                    if (!r.skip()) return fail(KRR_PACK_E_PARSE, "malformed JSON");
                                    continue;
                                }
                                have_values = true;
                                if (!r.lit('[')) return fail(KRR_PACK_E_PARSE, "values is not an array");
                                if (r.lit(']')) continue;
                                do {
                                    double ts, val;
                                    std::string_view vs;
                                    bool vesc;
                                    if (!r.lit('[') || !r.num(want_ts ? &ts : nullptr) || !r.lit(',') ||
                                        !r.str(&vs, &vesc) || !r.lit(']'))
                                        return fail(KRR_PACK_E_PARSE, "sample is not [time, \"value\"]");
                                    if (vesc || !parse_value(vs, &val))
                                        return fail(KRR_PACK_E_VALUE, "sample value is not a number");
                                    out.v.push_back(val);
                                    if (want_ts) out.t.push_back(ts);
                                } while (r.lit(','));
                                if (!r.lit(']')) return fail(KRR_PACK_E_PARSE, "unterminated values");
                            } while (r.lit(','));
                        }
                        if (!r.lit('}')) return fail(KRR_PACK_E_PARSE, "unterminated series");
                        if (!have_values) return fail(KRR_PACK_E_PARSE, "series without values");
                        while (r.lit(','))  // further series: never read by the reference; validated
                            if (!r.skip()) return fail(KRR_PACK_E_PARSE, "malformed JSON");
                        if (!r.lit(']')) return fail(KRR_PACK_E_PARSE, "unterminated result");
                    } while (r.lit(','));
                }
                if (!r.lit('}')) return fail(KRR_PACK_E_PARSE, "unterminated data");
            } else if (!r.skip()) {
                return fail(KRR_PACK_E_PARSE, "malformed JSON");
            }
        } while (r.lit(','));
    }
    if (!r.lit('}')) return fail(KRR_PACK_E_PARSE, "unterminated response");
    r.ws();
    if (r.p != r.e) return fail(KRR_PACK_E_PARSE, "trailing bytes");
    if (!have_status || !ok_status) return fail(KRR_PACK_E_STATUS, "status is not \"success\"");
    if (!have_result) return fail(KRR_PACK_E_PARSE, "no data.result");
}

// ---- grouped responses: "sum by (pod) (...)" returns one series per pod ----
struct Series {
    std::string label;  // the metric's `label` entry ("" when absent)
    bool has_label = false;
    std::vector<double> v, t;
};

struct SeriesSet {
    std::vector<Series> series;
    int status = KRR_PACK_OK;
    std::string err;
};

// Read a string value (escapes decoded) into *out.
bool read_string(Reader& r, std::string* out) {
    std::string_view raw;
    bool esc;
    if (!r.str(&raw, &esc)) return false;
    *out = esc ? unescape(raw) : std::string(raw);
    return true;
}

// {"status": "success", "data": {"result": [{"metric": {...}, "values": [...]}, ...]}}: every series.
void parse_series_set(const char* s, int64_t n, const char* label, bool want_ts, SeriesSet& out) {
    Reader r{s, s + n};
    auto fail = [&](int code, const char* what) {
        out.status = code;
        char buf[160];
        snprintf(buf, sizeof(buf), "%s at byte %lld", what, (long long)(r.p - s));
        out.err = buf;
    };
    bool have_status = false, ok_status = false, have_result = false;
    if (!r.lit('{')) return fail(KRR_PACK_E_PARSE, "expected a JSON object");
    if (!r.peek('}')) {
        do {
            std::string_view k;
            bool esc;
            if (!r.str(&k, &esc) || !r.lit(':')) return fail(KRR_PACK_E_PARSE, "bad object key");
            if (key_is(k, esc, "status")) {
                std::string v;
                if (!read_string(r, &v)) return fail(KRR_PACK_E_PARSE, "status is not a string");
                have_status = true;
                ok_status = v == "success";
            } else if (key_is(k, esc, "data")) {
                if (!r.lit('{')) return fail(KRR_PACK_E_PARSE, "data is not an object");
                if (!r.peek('}')) {
                    do {
                        std::string_view dk;
                        bool desc;
                        if (!r.str(&dk, &desc) || !r.lit(':')) return fail(KRR_PACK_E_PARSE, "bad data key");
                        if (!key_is(dk, desc, "result")) {
                            if (!r.skip()) return fail(KRR_PACK_E_PARSE, "malformed JSON");
                            continue;
                        }
                        if (!r.lit('[')) return fail(KRR_PACK_E_PARSE, "result is not an array");
                        have_result = true;
                        if (r.lit(']')) continue;
                        do {
                            Series S;
                            bool have_values = false;
                            if (!r.lit('{')) return fail(KRR_PACK_E_PARSE, "series is not an object");
                            if (!r.peek('}')) {
                                do {
                                    std::string_view sk;
                                    bool sesc;
                                    if (!r.str(&sk, &sesc) || !r.lit(':'))
                                        return fail(KRR_PACK_E_PARSE, "bad series key");
                                    if (key_is(sk, sesc, "metric")) {
                                        if (!r.lit('{')) return fail(KRR_PACK_E_PARSE, "metric is not an object");
                                        if (!r.peek('}')) {
                                            do {
                                                std::string_view lk;
                                                bool lesc;
                                                if (!r.str(&lk, &lesc) || !r.lit(':'))
                                                    return fail(KRR_PACK_E_PARSE, "bad label");
                                                if (key_is(lk, lesc, label)) {
                                                    if (!read_string(r, &S.label))
                                                        return fail(KRR_PACK_E_PARSE, "label value is not a string");
                                                    S.has_label = true;
                                                } else if (!r.skip()) {
                                                    return fail(KRR_PACK_E_PARSE, "malformed JSON");
                                                }
                                            } while (r.lit(','));
                                        }
                                        if (!r.lit('}')) return fail(KRR_PACK_E_PARSE, "unterminated metric");
                                    } else if (key_is(sk, sesc, "values")) {
                                        have_values = true;
                                        if (!r.lit('[')) return fail(KRR_PACK_E_PARSE, "values is not an array");
                                        if (r.lit(']')) continue;
                                        do {
                                            double ts, val;
                                            std::string_view vs;
                                            bool vesc;
                                            if (!r.lit('[') || !r.num(want_ts ? &ts : nullptr) || !r.lit(',') ||
                                                !r.str(&vs, &vesc) || !r.lit(']'))
                                                return fail(KRR_PACK_E_PARSE, "sample is not [time, \"value\"]");
                                            if (vesc || !parse_value(vs, &val))
                                                return fail(KRR_PACK_E_VALUE, "sample value is not a number");
                                            S.v.push_back(val);
                                            if (want_ts) S.t.push_back(ts);
                                        } while (r.lit(','));
                                        if (!r.lit(']')) return fail(KRR_PACK_E_PARSE, "unterminated values");
                                    } else if (!r.skip()) {
                                        return fail(KRR_PACK_E_PARSE, "malformed JSON");
                                    }
                                } while (r.lit(','));
                            }
                            if (!r.lit('}')) return fail(KRR_PACK_E_PARSE, "unterminated series");
                            if (!have_values) return fail(KRR_PACK_E_PARSE, "series without values");
                            out.series.push_back(std::move(S));
                        } while (r.lit(','));
                        if (!r.lit(']')) return fail(KRR_PACK_E_PARSE, "unterminated result");
                    } while (r.lit(','));
                }
                if (!r.lit('}')) return fail(KRR_PACK_E_PARSE, "unterminated data");
            } else if (!r.skip()) {
                return fail(KRR_PACK_E_PARSE, "malformed JSON");
            }
        } while (r.lit(','));
    }
    if (!r.lit('}')) return fail(KRR_PACK_E_PARSE, "unterminated response");
    r.ws();
    if (r.p != r.e) return fail(KRR_PACK_E_PARSE, "trailing bytes");
    if (!have_status || !ok_status) return fail(KRR_PACK_E_STATUS, "status is not \"success\"");
    if (!have_result) return fail(KRR_PACK_E_PARSE, "no data.result");
}

// threads = 0: the CPUs this process may run on (its affinity mask; hardware_concurrency counts
// the whole machine's, many times a GPU box's lease), capped by OMP_NUM_THREADS when set
int default_threads() {
    static const int n = [] {
        int c = (int)std::thread::hardware_concurrency();
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) c = CPU_COUNT(&set);
        if (const char* omp = std::getenv("OMP_NUM_THREADS")) {
            const int o = std::atoi(omp);
            if (o > 0 && o < c) c = o;
        }
        return c;
    }();
    return n;
}

int pool_size(int32_t threads, int64_t work) {
    int t = threads > 0 ? threads : default_threads();
    if (t < 1) t = 1;
    if ((int64_t)t > work) t = (int)std::max<int64_t>(work, 1);
    return t;
}

// Worker threads kept for the life of the process: the device packer stages a batch in ~20
// chunks, one parallel call each, and spawning 15 threads per call cost ~0.3 ms of the
// caller's time per chunk, with the link idle behind it.  A call hands `helpers` tickets of
// one job to the pool (spawning workers only when too few are idle) and works on the job
// itself; jobs of concurrent callers (the hybrid parser's two sides) queue side by side.
class WorkerPool {
  public:
    void run(int helpers, const std::function<void()>& work) {
        auto job = std::make_shared<Job>();
        job->work = &work;
        job->pending = helpers;
        {
            std::lock_guard<std::mutex> l(m_);
            for (int k = 0; k < helpers; ++k) queue_.push_back(job);
            for (int k = idle_; k < (int)queue_.size(); ++k) {
                std::thread(&WorkerPool::loop, this).detach();  // lives as long as the process
                ++idle_;
            }
        }
        cv_.notify_all();
        // `work` lives on this frame: whatever it throws here (e.g. std::bad_alloc from a
        // parse), the helpers still calling it must finish before the frame unwinds
        std::exception_ptr mine;
        try {
            work();
        } catch (...) {
            mine = std::current_exception();
        }
        std::unique_lock<std::mutex> l(job->m);
        job->done.wait(l, [&] { return job->pending == 0; });
        if (mine) std::rethrow_exception(mine);
        if (job->error) std::rethrow_exception(job->error);
    }

  private:
    struct Job {
        const std::function<void()>* work = nullptr;
        int pending = 0;
        std::exception_ptr error;  // the first a helper caught (rethrown by the caller)
        std::mutex m;
        std::condition_variable done;
    };
    void loop() {
        for (;;) {
            std::shared_ptr<Job> job;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return !queue_.empty(); });
                job = queue_.front();
                queue_.pop_front();
                --idle_;
            }
            std::exception_ptr err;
            try {
                (*job->work)();
            } catch (...) {  // a detached thread must not let it escape (std::terminate)
                err = std::current_exception();
            }
            {
                std::lock_guard<std::mutex> l(job->m);
                if (err && !job->error) job->error = err;
                if (--job->pending == 0) job->done.notify_all();
            }
            std::lock_guard<std::mutex> l(m_);
            ++idle_;
        }
    }
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<Job>> queue_;
    int idle_ = 0;
};

// Never destroyed: its threads outlive static destructors.  A child forked while the pool has
// workers (multiprocessing's fork start method) gets the pool's memory but none of its threads,
// and maybe a mutex another thread held: the child starts a fresh pool (the old one leaks).
WorkerPool* g_pool = nullptr;
std::once_flag g_pool_once;

void pool_after_fork_in_child() { g_pool = new WorkerPool(); }

WorkerPool& worker_pool() {
    std::call_once(g_pool_once, [] {
        g_pool = new WorkerPool();
        pthread_atfork(nullptr, nullptr, pool_after_fork_in_child);
    });
    return *g_pool;
}

template <class F>
void parallel_for(int64_t n, int32_t threads, F f) {
    const int t = pool_size(threads, n);
    if (t <= 1) {
        for (int64_t i = 0; i < n; ++i) f(i);
        return;
    }
    // chunks of up to 8 items, but at least ~4 chunks per thread so few large
    // items (grouped bodies) still spread over the pool
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(8, n / ((int64_t)t * 4)));
    std::atomic<int64_t> next{0};
    const std::function<void()> worker = [&]() {
        for (;;) {
            const int64_t b = next.fetch_add(chunk);
            if (b >= n) return;
            const int64_t e = std::min<int64_t>(b + chunk, n);
            for (int64_t i = b; i < e; ++i) f(i);
        }
    };
    worker_pool().run(t - 1, worker);
}

}  // namespace

struct krr_pack {
    std::vector<Body> bodies;
    std::vector<SeriesSet> sets;  // grouped packing only: bodies[] point into these
    std::vector<int64_t> obj;
    int64_t n_objects = 0;
    int64_t n_values = 0;
    int64_t max_len = 0;
    bool want_ts = false;
    std::string err;
};

extern "C" {

int krr_pack_abi_version(void) { return KRR_PACK_ABI_VERSION; }

int krr_pack_parse(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies, const int64_t* obj_of_body,
                   int64_t n_objects, int32_t want_timestamps, int32_t threads, krr_pack** out) {
    if (!out) return KRR_PACK_E_INVALID;
    *out = nullptr;
    if (n_bodies < 0 || n_objects < 0 || (n_bodies > 0 && (!bodies || !body_lens || !obj_of_body)))
        return KRR_PACK_E_INVALID;
    for (int64_t b = 0; b < n_bodies; ++b) {
        if (obj_of_body[b] < 0 || obj_of_body[b] >= n_objects || (b && obj_of_body[b] < obj_of_body[b - 1]) ||
            body_lens[b] < 0 || (body_lens[b] > 0 && !bodies[b]))
            return KRR_PACK_E_INVALID;
    }
    krr_pack* p = new (std::nothrow) krr_pack();
    if (!p) return KRR_PACK_E_INVALID;
    try {
        p->bodies.resize((size_t)n_bodies);
        p->obj.assign(obj_of_body, obj_of_body + n_bodies);
    } catch (...) {
        delete p;
        return KRR_PACK_E_INVALID;
    }
    p->n_objects = n_objects;
    p->want_ts = want_timestamps != 0;
    parallel_for(n_bodies, threads, [&](int64_t b) {
        try {
            parse_body(bodies[b], body_lens[b], p->want_ts, p->bodies[(size_t)b]);
        } catch (...) {
            p->bodies[(size_t)b].status = KRR_PACK_E_INVALID;
            p->bodies[(size_t)b].err = "out of memory";
        }
    });
    int rc = KRR_PACK_OK;
    std::vector<int64_t> seg((size_t)n_objects, 0);
    for (int64_t b = 0; b < n_bodies; ++b) {
        const Body& B = p->bodies[(size_t)b];
        if (B.status != KRR_PACK_OK) {
            if (rc == KRR_PACK_OK) {
                rc = B.status;
                p->err = "body " + std::to_string(b) + ": " + B.err;
            }
            continue;
        }
        seg[(size_t)p->obj[(size_t)b]] += (int64_t)B.V().size();
        p->n_values += (int64_t)B.V().size();
    }
    for (int64_t s : seg) p->max_len = std::max(p->max_len, s);
    *out = p;
    return rc;
}

int64_t krr_pack_n_values(const krr_pack* p) { return p ? p->n_values : -1; }
int64_t krr_pack_max_len(const krr_pack* p) { return p ? p->max_len : -1; }
const char* krr_pack_error(const krr_pack* p) { return p ? p->err.c_str() : "null krr_pack"; }
void krr_pack_free(krr_pack* p) { delete p; }

int krr_pack_copy(const krr_pack* p, double* values, int64_t* offsets, double* timestamps, int64_t* pod_counts,
                  int32_t threads) {
    if (!p || !offsets || (p->n_values > 0 && !values)) return KRR_PACK_E_INVALID;
    if (timestamps && !p->want_ts) return KRR_PACK_E_INVALID;
    if (!p->err.empty()) return KRR_PACK_E_PARSE;
    const int64_t nb = (int64_t)p->bodies.size();
    std::vector<int64_t> start((size_t)nb, 0);
    int64_t pos = 0;
    for (int64_t s = 0; s <= p->n_objects; ++s) offsets[s] = 0;
    for (int64_t b = 0; b < nb; ++b) {
        start[(size_t)b] = pos;
        const int64_t c = (int64_t)p->bodies[(size_t)b].V().size();
        pos += c;
        offsets[p->obj[(size_t)b] + 1] += c;
        if (pod_counts) pod_counts[b] = p->bodies[(size_t)b].dropped ? -1 : c;
    }
    for (int64_t s = 0; s < p->n_objects; ++s) offsets[s + 1] += offsets[s];
    parallel_for(nb, threads, [&](int64_t b) {
        const Body& B = p->bodies[(size_t)b];
        const std::vector<double>& v = B.V();
        if (v.empty()) return;
        memcpy(values + start[(size_t)b], v.data(), v.size() * sizeof(double));
        if (timestamps) memcpy(timestamps + start[(size_t)b], B.T().data(), B.T().size() * sizeof(double));
    });
    return KRR_PACK_OK;
}

struct krr_series_set {
    SeriesSet set;
};

int krr_pack_parse_grouped(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies, const char* label,
                           const int64_t* slot_body, const char* slot_names, const int64_t* slot_name_offsets,
                           const int64_t* obj_of_slot, int64_t n_slots, int64_t n_objects, int32_t want_timestamps,
                           int32_t threads, krr_pack** out) {
    if (!out) return KRR_PACK_E_INVALID;
    *out = nullptr;
    if (n_bodies < 0 || n_slots < 0 || n_objects < 0 || !label || (n_bodies > 0 && (!bodies || !body_lens)) ||
        (n_slots > 0 && (!slot_body || !slot_name_offsets || !obj_of_slot)))
        return KRR_PACK_E_INVALID;
    for (int64_t b = 0; b < n_bodies; ++b)
        if (body_lens[b] < 0 || (body_lens[b] > 0 && !bodies[b])) return KRR_PACK_E_INVALID;
    if (n_slots > 0 && (slot_name_offsets[0] < 0 || (slot_name_offsets[n_slots] > 0 && !slot_names)))
        return KRR_PACK_E_INVALID;
    for (int64_t s = 0; s < n_slots; ++s) {
        if (slot_body[s] < 0 || slot_body[s] >= n_bodies || obj_of_slot[s] < 0 || obj_of_slot[s] >= n_objects ||
            (s && obj_of_slot[s] < obj_of_slot[s - 1]) || slot_name_offsets[s + 1] < slot_name_offsets[s])
            return KRR_PACK_E_INVALID;
    }
    krr_pack* p = new (std::nothrow) krr_pack();
    if (!p) return KRR_PACK_E_INVALID;
    std::vector<SeriesSet>& sets = p->sets;
    // per body: label value -> first series carrying it (the reference reads result[0])
    std::vector<std::unordered_map<std::string_view, int64_t>> index;
    try {
        sets.resize((size_t)n_bodies);
        index.resize((size_t)n_bodies);
        p->bodies.resize((size_t)n_slots);
        p->obj.assign(obj_of_slot, obj_of_slot + n_slots);
    } catch (...) {
        delete p;
        return KRR_PACK_E_INVALID;
    }
    p->n_objects = n_objects;
    p->want_ts = want_timestamps != 0;
    parallel_for(n_bodies, threads, [&](int64_t b) {
        SeriesSet& S = sets[(size_t)b];
        try {
            parse_series_set(bodies[b], body_lens[b], label, p->want_ts, S);
            if (S.status != KRR_PACK_OK) return;
            auto& ix = index[(size_t)b];
            ix.reserve(S.series.size() * 2);
            for (size_t i = 0; i < S.series.size(); ++i)
                if (S.series[i].has_label) ix.emplace(std::string_view(S.series[i].label), (int64_t)i);
        } catch (...) {
            S.status = KRR_PACK_E_INVALID;
            S.err = "out of memory";
        }
    });
    int rc = KRR_PACK_OK;
    for (int64_t b = 0; b < n_bodies; ++b) {
        if (sets[(size_t)b].status != KRR_PACK_OK) {
            rc = sets[(size_t)b].status;
            p->err = "body " + std::to_string(b) + ": " + sets[(size_t)b].err;
            break;
        }
    }
    if (rc == KRR_PACK_OK) {
        parallel_for(n_slots, threads, [&](int64_t s) {
            Body& B = p->bodies[(size_t)s];
            const int64_t b = slot_body[s];
            const std::string_view name(slot_names + slot_name_offsets[s],
                                        (size_t)(slot_name_offsets[s + 1] - slot_name_offsets[s]));
            const auto& ix = index[(size_t)b];
            const auto it = ix.find(name);
            if (it == ix.end()) {
                B.dropped = true;  // no series for this pod: prometheus.py:154 drops it
                return;
            }
            const Series& src = p->sets[(size_t)b].series[(size_t)it->second];
            B.pv = &src.v;
            B.pt = &src.t;
        });
        std::vector<int64_t> seg((size_t)n_objects, 0);
        for (int64_t s = 0; s < n_slots; ++s) {
            const Body& B = p->bodies[(size_t)s];
            if (B.status != KRR_PACK_OK) {
                if (rc == KRR_PACK_OK) {
                    rc = B.status;
                    p->err = "slot " + std::to_string(s) + ": " + B.err;
                }
                continue;
            }
            seg[(size_t)p->obj[(size_t)s]] += (int64_t)B.V().size();
            p->n_values += (int64_t)B.V().size();
        }
        for (int64_t v : seg) p->max_len = std::max(p->max_len, v);
    }
    *out = p;
    return rc;
}

int krr_pack_parse_series(const char* body, int64_t len, const char* label, int32_t want_timestamps,
                          krr_series_set** out) {
    if (!out) return KRR_PACK_E_INVALID;
    *out = nullptr;
    if (len < 0 || (len > 0 && !body) || !label) return KRR_PACK_E_INVALID;
    krr_series_set* h = new (std::nothrow) krr_series_set();
    if (!h) return KRR_PACK_E_INVALID;
    try {
        parse_series_set(body, len, label, want_timestamps != 0, h->set);
    } catch (...) {
        h->set.status = KRR_PACK_E_INVALID;
        h->set.err = "out of memory";
    }
    *out = h;
    return h->set.status;
}

int64_t krr_series_count(const krr_series_set* h) { return h ? (int64_t)h->set.series.size() : -1; }

const char* krr_series_label(const krr_series_set* h, int64_t i, int64_t* len) {
    if (!h || i < 0 || i >= (int64_t)h->set.series.size()) return nullptr;
    const Series& S = h->set.series[(size_t)i];
    if (len) *len = S.has_label ? (int64_t)S.label.size() : -1;
    return S.label.c_str();
}

int64_t krr_series_len(const krr_series_set* h, int64_t i) {
    if (!h || i < 0 || i >= (int64_t)h->set.series.size()) return -1;
    return (int64_t)h->set.series[(size_t)i].v.size();
}

int krr_series_copy(const krr_series_set* h, int64_t i, double* values, double* timestamps) {
    if (!h || i < 0 || i >= (int64_t)h->set.series.size()) return KRR_PACK_E_INVALID;
    const Series& S = h->set.series[(size_t)i];
    if (!S.v.empty() && !values) return KRR_PACK_E_INVALID;
    if (timestamps && S.t.size() != S.v.size()) return KRR_PACK_E_INVALID;
    if (!S.v.empty()) memcpy(values, S.v.data(), S.v.size() * sizeof(double));
    if (timestamps && !S.t.empty()) memcpy(timestamps, S.t.data(), S.t.size() * sizeof(double));
    return KRR_PACK_OK;
}

const char* krr_series_error(const krr_series_set* h) { return h ? h->set.err.c_str() : "null krr_series_set"; }

void krr_series_free(krr_series_set* h) { delete h; }

int krr_pack_concat(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies,
                    const int64_t* dst_offsets, char* dst, int32_t threads) {
    if (n_bodies < 0 || (n_bodies > 0 && (!bodies || !body_lens || !dst_offsets || !dst))) return KRR_PACK_E_INVALID;
    for (int64_t b = 0; b < n_bodies; ++b)
        if (body_lens[b] < 0 || (body_lens[b] > 0 && !bodies[b]) ||
            dst_offsets[b + 1] - dst_offsets[b] != body_lens[b])
            return KRR_PACK_E_INVALID;
    const int64_t base = n_bodies > 0 ? dst_offsets[0] : 0;
    parallel_for(n_bodies, threads, [&](int64_t b) {
        if (body_lens[b]) memcpy(dst + (dst_offsets[b] - base), bodies[b], (size_t)body_lens[b]);
    });
    return KRR_PACK_OK;
}

int krr_pack_concat_strip(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies,
                          const int64_t* dst_offsets, char* dst, int32_t threads, int32_t max_runs,
                          int64_t* new_lens, int64_t* run_first, int32_t* n_runs) {
    if (n_bodies < 0 || max_runs < 1 || !run_first || !n_runs ||
        (n_bodies > 0 && (!bodies || !body_lens || !dst_offsets || !dst || !new_lens)))
        return KRR_PACK_E_INVALID;
    for (int64_t b = 0; b < n_bodies; ++b)
        if (body_lens[b] < 0 || (body_lens[b] > 0 && !bodies[b]) ||
            dst_offsets[b + 1] - dst_offsets[b] != body_lens[b])
            return KRR_PACK_E_INVALID;
    const int64_t base = n_bodies > 0 ? dst_offsets[0] : 0;
    const int64_t total = n_bodies > 0 ? dst_offsets[n_bodies] - base : 0;
    // runs of about equal bytes, each ending on a body boundary (a body never splits)
    int32_t R = 0;
    run_first[0] = 0;
    for (int64_t b = 0; b < n_bodies;) {
        const int64_t target = base + (total * (int64_t)(R + 1)) / max_runs;
        int64_t e = (int64_t)(std::lower_bound(dst_offsets + b + 1, dst_offsets + n_bodies + 1, target) - dst_offsets);
        e = std::min<int64_t>(std::max<int64_t>(e, b + 1), n_bodies);
        if (R + 1 == max_runs) e = n_bodies;
        run_first[++R] = e;
        b = e;
    }
    *n_runs = R;
    parallel_for(R, threads, [&](int64_t r) {
        char* o = dst + (dst_offsets[run_first[r]] - base);
        for (int64_t b = run_first[r]; b < run_first[r + 1]; ++b) {
            const int64_t n = body_lens[b];
            int64_t w = n ? krr::strip::strip_body(bodies[b], n, o) : 0;
            if (w < 0) {  // not strippable: unchanged (o never passes the body's own extent)
                memmove(o, bodies[b], (size_t)n);
                w = n;
            }
            new_lens[b] = w;
            o += w;
        }
    });
    return KRR_PACK_OK;
}

int krr_pack_concat_strip_pieces(const char* const* bodies, const int64_t* body_lens, int64_t n_bodies,
                                 const int64_t* dst_offsets, char* dst, int32_t threads, int32_t max_pieces,
                                 int64_t* new_lens, int64_t* piece_start, int64_t* piece_out, int32_t* n_pieces) {
    if (n_bodies < 0 || max_pieces < 1 || !piece_start || !piece_out || !n_pieces ||
        (n_bodies > 0 && (!bodies || !body_lens || !dst_offsets || !dst || !new_lens)))
        return KRR_PACK_E_INVALID;
    for (int64_t b = 0; b < n_bodies; ++b)
        if (body_lens[b] < 0 || (body_lens[b] > 0 && !bodies[b]) ||
            dst_offsets[b + 1] - dst_offsets[b] != body_lens[b])
            return KRR_PACK_E_INVALID;
    const int64_t base = n_bodies > 0 ? dst_offsets[0] : 0;
    const int64_t total = n_bodies > 0 ? dst_offsets[n_bodies] - base : 0;
    const int64_t P = std::max<int64_t>(1, (total + max_pieces - 1) / max_pieces);
    const bool simd = krr::strip::supported();
    // nominal pieces: runs of whole bodies of ~P bytes; a body of >= 2P bytes on its own, cut at
    // nominal offsets (moved to the next `"],[` below) into about len / P parts
    struct Nom {
        int64_t body, lo, hi;  // body (the first, for a run of whole bodies) and its bytes [lo, hi)
        int64_t last;          // one past the run's last body (whole-body runs), or body + 1
        const char* start = nullptr;  // the actual start after the split search
    };
    std::vector<Nom> nom;
    try {
        for (int64_t b = 0; b < n_bodies;) {
            const int64_t n = body_lens[b];
            if (n >= 2 * P && simd) {
                const int64_t k = (n + P - 1) / P;  // <= max_pieces + 1 (n <= total)
                for (int64_t i = 0; i < k; ++i) nom.push_back(Nom{b, n * i / k, n * (i + 1) / k, b + 1});
                ++b;
                continue;
            }
            int64_t e = b, bytes = 0;
            while (e < n_bodies && (e == b || (bytes + body_lens[e] <= P && body_lens[e] < 2 * P))) bytes += body_lens[e++];
            nom.push_back(Nom{b, 0, body_lens[b], e});
            b = e;
        }
    } catch (...) {
        return KRR_PACK_E_INVALID;
    }
    const int64_t N = (int64_t)nom.size();
    auto whole = [&](const Nom& u) { return u.last > u.body + 1 || (u.lo == 0 && u.hi == body_lens[u.body]); };
    // each cut part's start moved to the first sample boundary inside it
    parallel_for(N, threads, [&](int64_t i) {
        Nom& u = nom[(size_t)i];
        const char* s0 = bodies[u.body];
        u.start = (u.lo == 0) ? s0 : krr::strip::next_split(s0 + u.lo, s0 + u.hi);
    });
    // the pieces: cut parts without a split join the piece before them
    std::vector<int64_t> ps_body, ps_first, ps_last;
    std::vector<const char*> ps_p, ps_e;
    try {
        for (int64_t i = 0; i < N; ++i) {
            const Nom& u = nom[(size_t)i];
            if (!u.start) continue;
            if (whole(u)) {
                ps_body.push_back(u.body);
                ps_first.push_back(u.body);
                ps_last.push_back(u.last);
                ps_p.push_back(nullptr);
                ps_e.push_back(nullptr);
                continue;
            }
            if (!ps_p.empty() && ps_body.back() == u.body && ps_p.back()) ps_e.back() = u.start;
            ps_body.push_back(u.body);
            ps_first.push_back(u.body);
            ps_last.push_back(u.body + 1);
            ps_p.push_back(u.start);
            ps_e.push_back(bodies[u.body] + body_lens[u.body]);
        }
    } catch (...) {
        return KRR_PACK_E_INVALID;
    }
    const int64_t M = (int64_t)ps_body.size();
    if (M > 2 * n_bodies + (int64_t)max_pieces) return KRR_PACK_E_INVALID;  // (the documented capacity)
    std::vector<int64_t> out_len((size_t)M, 0), quotes((size_t)M, 0);
    std::vector<unsigned char> bad((size_t)n_bodies, 0);
    parallel_for(M, threads, [&](int64_t j) {
        if (!ps_p[(size_t)j]) {  // whole bodies back to back from the first one's extent
            char* o = dst + (dst_offsets[ps_first[(size_t)j]] - base);
            int64_t w_all = 0;
            for (int64_t b = ps_first[(size_t)j]; b < ps_last[(size_t)j]; ++b) {
                const int64_t n = body_lens[b];
                int64_t w = n ? krr::strip::strip_body(bodies[b], n, o) : 0;
                if (w < 0) {
                    memmove(o, bodies[b], (size_t)n);
                    w = n;
                }
                new_lens[b] = w;
                o += w;
                w_all += w;
            }
            out_len[(size_t)j] = w_all;
            return;
        }
        const int64_t b = ps_body[(size_t)j];
        const char* p = ps_p[(size_t)j];
        char* o = dst + (dst_offsets[b] - base) + (p - bodies[b]);
        // -1: not strippable; the quotes it saw check the cut (below)
        out_len[(size_t)j] = krr::strip::strip_span(p, ps_e[(size_t)j], o, &quotes[(size_t)j]);
    });
    {
        int64_t q = 0;
        for (int64_t j = 0; j < M; ++j) {
            if (!ps_p[(size_t)j]) continue;
            const int64_t b = ps_body[(size_t)j];
            if (ps_p[(size_t)j] == bodies[b]) q = 0;
            else if (q & 1) bad[(size_t)b] = 1;  // the cut was inside a string: not a sample boundary
            if (out_len[(size_t)j] < 0) bad[(size_t)b] = 1;
            q += quotes[(size_t)j];
        }
    }
    // a body with an unstrippable part is copied unchanged, part by part (its extents as they are)
    parallel_for(M, threads, [&](int64_t j) {
        if (!ps_p[(size_t)j] || !bad[(size_t)ps_body[(size_t)j]]) return;
        const int64_t b = ps_body[(size_t)j];
        const char* p = ps_p[(size_t)j];
        memmove(dst + (dst_offsets[b] - base) + (p - bodies[b]), p, (size_t)(ps_e[(size_t)j] - p));
        out_len[(size_t)j] = ps_e[(size_t)j] - p;
    });
    for (int64_t j = 0; j < M; ++j) {
        const int64_t b = ps_body[(size_t)j];
        piece_start[j] = ps_p[(size_t)j] ? dst_offsets[b] + (ps_p[(size_t)j] - bodies[b]) : dst_offsets[ps_first[(size_t)j]];
        piece_out[j] = out_len[(size_t)j];
        if (ps_p[(size_t)j]) new_lens[b] = (ps_p[(size_t)j] == bodies[b] ? 0 : new_lens[b]) + out_len[(size_t)j];
    }
    piece_start[M] = base + total;
    *n_pieces = (int32_t)M;
    return KRR_PACK_OK;
}

int64_t krr_pack_strip_body(const char* body, int64_t body_len, char* out) {
    if (body_len < 0 || (body_len > 0 && (!body || !out))) return -1;
    return krr::strip::strip_body(body, body_len, out);
}

int krr_pack_route_grouped(const char* bodies, const int64_t* body_offsets, int64_t n_bodies, const char* label,
                           const int64_t* segments, int64_t n_segments, const int64_t* slot_body,
                           const char* slot_names, const int64_t* slot_name_offsets, int64_t n_slots,
                           int64_t* slot_src, int64_t* slot_count, int32_t* body_ok, int32_t threads) {
    return krr_pack_route_grouped_pieces(bodies, body_offsets, n_bodies, nullptr, nullptr, 0, label, segments,
                                         n_segments, slot_body, slot_names, slot_name_offsets, n_slots, slot_src,
                                         slot_count, body_ok, threads);
}

int krr_pack_route_grouped_pieces(const char* bodies, const int64_t* body_offsets, int64_t n_bodies,
                                  const int64_t* piece_dev, const int64_t* piece_shift, int64_t n_pieces,
                                  const char* label, const int64_t* segments, int64_t n_segments,
                                  const int64_t* slot_body, const char* slot_names,
                                  const int64_t* slot_name_offsets, int64_t n_slots, int64_t* slot_src,
                                  int64_t* slot_count, int32_t* body_ok, int32_t threads) {
    if (n_bodies < 0 || n_segments < 0 || n_slots < 0 || n_pieces < 0 || !label ||
        (n_bodies > 0 && (!bodies || !body_offsets || !body_ok)) || (n_pieces > 0 && (!piece_dev || !piece_shift)) ||
        (n_segments > 0 && !segments) || (n_slots > 0 && (!slot_body || !slot_name_offsets || !slot_src ||
                                                          !slot_count)))
        return KRR_PACK_E_INVALID;
    for (int64_t j = 1; j < n_pieces; ++j)
        if (piece_dev[j] <= piece_dev[j - 1]) return KRR_PACK_E_INVALID;
    for (int64_t j = 1; j < n_segments; ++j)
        if (segments[7 * j] <= segments[7 * (j - 1)]) return KRR_PACK_E_INVALID;  // sorted, distinct starts
    for (int64_t s = 0; s < n_slots; ++s)
        if (slot_body[s] < 0 || slot_body[s] >= n_bodies || slot_name_offsets[s + 1] < slot_name_offsets[s])
            return KRR_PACK_E_INVALID;
    struct Map {
        const char* base;
        const int64_t *dev, *shift;
        int64_t n;
        int64_t piece(int64_t pos) const {  // the last piece starting at or before pos
            return (int64_t)(std::upper_bound(dev, dev + n, pos) - dev) - 1;
        }
        const char* at(int64_t pos) const {
            const int64_t j = n ? piece(pos) : -1;
            return base + pos + (j >= 0 ? shift[j] : 0);
        }
        int64_t end(int64_t pos) const {
            if (!n) return std::numeric_limits<int64_t>::max();
            const int64_t j = piece(pos);
            return j + 1 < n ? dev[j + 1] : std::numeric_limits<int64_t>::max();
        }
    } map{bodies, piece_dev, piece_shift, n_pieces};
    const int64_t ll = (int64_t)strlen(label);
    std::vector<std::unordered_map<std::string_view, int64_t>> index;
    try {
        index.resize((size_t)n_bodies);
    } catch (...) {
        return KRR_PACK_E_INVALID;
    }
    auto find = [&](int64_t pos) -> int64_t {
        int64_t lo = 0, hi = n_segments;
        while (lo < hi) {
            const int64_t mid = (lo + hi) / 2;
            if (segments[7 * mid] < pos) lo = mid + 1;
            else hi = mid;
        }
        return lo < n_segments && segments[7 * lo] == pos ? lo : -1;
    };
    parallel_for(n_bodies, threads, [&](int64_t b) {
        auto& ix = index[(size_t)b];
        const bool ok = krr::json::chain_grouped_mapped(
            map, body_offsets[b], body_offsets[b + 1], label, ll, segments, find, [&](int64_t j) {
                const int64_t* R = segments + 7 * j;
                if (R[2] >= 0)  // the first series with the label wins (a label never spans a piece cut)
                    ix.emplace(std::string_view(map.at(R[2]), (size_t)R[3]), j);
            });
        body_ok[b] = ok ? 1 : 0;
    });
    parallel_for(n_slots, threads, [&](int64_t s) {
        const std::string_view name(slot_names + slot_name_offsets[s],
                                    (size_t)(slot_name_offsets[s + 1] - slot_name_offsets[s]));
        const auto& ix = index[(size_t)slot_body[s]];
        const auto it = ix.find(name);
        if (it == ix.end()) {
            slot_src[s] = -1;
            slot_count[s] = -1;
        } else {
            slot_src[s] = segments[7 * it->second + 4];
            slot_count[s] = segments[7 * it->second + 5];
        }
    });
    return KRR_PACK_OK;
}

}  // extern "C"
