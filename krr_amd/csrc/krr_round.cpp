// krr_round.cpp — batched exact-decimal post-processing (host C++17).
//
// The reference rounds one object at a time with Python Decimals
// (strategies/simple.py:24-29, core/runner.py:49-86): ~60 us per object on this
// host, i.e. a 1M-container fleet spends a minute here after a
// 28 ms kernel pass.  This file does the same exact arithmetic on digit
// strings for every object in parallel and writes str(Decimal) of the
// reference's result, digits and exponent included.
#include "krr_round.h"

#include <sched.h>
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kFlagNan = 1u, kFlagCapacity = 2u, kFlagEmpty = 4u;  // krr_amd.h KRR_FLAG_*
constexpr int kPrec = 28;                                                 // the reference's decimal context

// A finite decimal: value = (-1)^neg * digits * 10^exp, digits most significant
// first, no leading zeros ("0" for zero).
struct Dec {
    bool neg = false;
    std::string d = "0";
    int exp = 0;
};

void strip_leading(std::string& d) {
    size_t i = 0;
    while (i + 1 < d.size() && d[i] == '0') ++i;
    d.erase(0, i);
}

bool is_zero(const Dec& a) { return a.d == "0"; }

// Parse str(Decimal)-style finite numbers: [-]digits[.digits][E[+-]n]
bool parse_dec(const char* s, Dec* out) {
    if (!s) return false;
    Dec r;
    const char* p = s;
    if (*p == '-' || *p == '+') r.neg = *p++ == '-';
    std::string digits;
    int frac = 0;
    bool seen_point = false, any = false;
    for (; *p; ++p) {
        if (*p >= '0' && *p <= '9') {
            digits.push_back(*p);
            any = true;
            if (seen_point) ++frac;
        } else if (*p == '.' && !seen_point) {
            seen_point = true;
        } else {
            break;
        }
    }
    if (!any) return false;
    int e = 0;
    if (*p == 'e' || *p == 'E') {
        ++p;
        auto res = std::from_chars(p + (*p == '+' ? 1 : 0), p + strlen(p), e);
        if (res.ec != std::errc() || *res.ptr) return false;
    } else if (*p) {
        return false;
    }
    strip_leading(digits);
    r.d = digits;
    r.exp = e - frac;
    *out = r;
    return true;
}

// The Decimal the reference parsed from Prometheus' string for sample x:
// shortest round-trip digits in positional form (utils/prom_decimal.py).
Dec prom_decimal(double x) {
    char buf[64];
    // shortest round-trip DIGITS: scientific form (the plain form prints large
    // integers with all their digits, e.g. 36792420997627696 for 3.67924209976277e+16)
    auto res = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);
    *res.ptr = 0;
    Dec r;
    parse_dec(buf, &r);
    if (r.exp > 0) {  // 'f' formatting never uses an exponent
        if (r.d != "0") r.d.append((size_t)r.exp, '0');
        r.exp = 0;
    }
    while (r.exp < 0 && r.d.size() > 1 && r.d.back() == '0') {
        r.d.pop_back();
        ++r.exp;
    }
    if (r.exp < 0 && r.d == "0") r.exp = 0;
    return r;
}

std::string mul_digits(const std::string& a, const std::string& b) {
    std::vector<uint32_t> acc(a.size() + b.size(), 0);
    for (size_t i = a.size(); i-- > 0;) {
        const uint32_t x = (uint32_t)(a[i] - '0');
        if (!x) continue;
        for (size_t j = b.size(); j-- > 0;) acc[i + j + 1] += x * (uint32_t)(b[j] - '0');
    }
    for (size_t k = acc.size(); k-- > 1;) {
        acc[k - 1] += acc[k] / 10;
        acc[k] %= 10;
    }
    std::string r(acc.size(), '0');
    for (size_t k = 0; k < acc.size(); ++k) r[k] = (char)('0' + acc[k]);
    strip_leading(r);
    return r;
}

Dec mul(const Dec& a, const Dec& b) {
    Dec r;
    r.d = mul_digits(a.d, b.d);
    r.exp = a.exp + b.exp;
    r.neg = a.neg != b.neg;
    return r;
}

// Add one unit in the last place of a digit string (carry may lengthen it).
void increment(std::string& d) {
    for (size_t i = d.size(); i-- > 0;) {
        if (d[i] != '9') {
            ++d[i];
            return;
        }
        d[i] = '0';
    }
    d.insert(d.begin(), '1');
}

// Round to prec significant digits, ROUND_HALF_EVEN (decimal context arithmetic).
Dec round_prec(Dec a, int prec) {
    if ((int)a.d.size() <= prec) return a;
    const size_t drop = a.d.size() - (size_t)prec;
    const std::string tail = a.d.substr((size_t)prec);
    std::string keep = a.d.substr(0, (size_t)prec);
    const char first = tail[0];
    bool rest_nonzero = tail.find_first_not_of('0', 1) != std::string::npos;
    bool up = first > '5' || (first == '5' && (rest_nonzero || ((keep.back() - '0') & 1)));
    if (up) {
        increment(keep);
        if ((int)keep.size() > prec) {  // 999.. -> 1000..: keep prec digits
            keep.pop_back();
            a.exp += 1;
        }
    }
    a.d = keep;
    a.exp += (int)drop;
    return a;
}

// ceil(a) as an integer Dec (exp 0).
Dec ceil_int(const Dec& a) {
    Dec r;
    if (a.exp >= 0) {
        r.d = a.d == "0" ? "0" : a.d + std::string((size_t)a.exp, '0');
        r.neg = a.neg && r.d != "0";
        return r;
    }
    const int nfrac = -a.exp;
    std::string ip, fp;
    if ((int)a.d.size() > nfrac) {
        ip = a.d.substr(0, a.d.size() - (size_t)nfrac);
        fp = a.d.substr(a.d.size() - (size_t)nfrac);
    } else {
        ip = "0";
        fp = a.d;
    }
    const bool frac_nonzero = fp.find_first_not_of('0') != std::string::npos;
    if (!a.neg && frac_nonzero) increment(ip);
    strip_leading(ip);
    r.d = ip;
    r.neg = a.neg && ip != "0";  // ceil toward +inf: negatives truncate
    return r;
}

// Numeric comparison: -1, 0, 1.
int cmp(const Dec& a, const Dec& b) {
    const bool za = is_zero(a), zb = is_zero(b);
    if (za && zb) return 0;
    const int sa = za ? 0 : (a.neg ? -1 : 1), sb = zb ? 0 : (b.neg ? -1 : 1);
    if (sa != sb) return sa < sb ? -1 : 1;
    // same sign, both non-zero: compare magnitudes
    const long adja = (long)a.exp + (long)a.d.size(), adjb = (long)b.exp + (long)b.d.size();
    int mag;
    if (adja != adjb) {
        mag = adja < adjb ? -1 : 1;
    } else {
        const size_t n = std::max(a.d.size(), b.d.size());
        std::string x = a.d, y = b.d;
        x.append(n - x.size(), '0');
        y.append(n - y.size(), '0');
        mag = x == y ? 0 : (x < y ? -1 : 1);
    }
    return sa > 0 ? mag : -mag;
}

// str(Decimal): Python's to-scientific-string.
std::string to_sci(const Dec& a) {
    const std::string& c = a.d;
    const long adjusted = (long)a.exp + (long)c.size() - 1;
    std::string s;
    if (a.exp <= 0 && adjusted >= -6) {
        if (a.exp == 0) {
            s = c;
        } else {
            const long point = (long)c.size() + a.exp;
            if (point > 0) s = c.substr(0, (size_t)point) + "." + c.substr((size_t)point);
            else s = "0." + std::string((size_t)(-point), '0') + c;
        }
    } else {
        s = c.substr(0, 1);
        if (c.size() > 1) s += "." + c.substr(1);
        s += adjusted >= 0 ? "E+" : "E-";
        s += std::to_string(adjusted >= 0 ? adjusted : -adjusted);
    }
    return (a.neg ? "-" : "") + s;
}

bool put(char* dst, int32_t width, const std::string& s) {
    if ((int32_t)s.size() + 1 > width) return false;
    memcpy(dst, s.c_str(), s.size() + 1);
    return true;
}

// Runner._round_value for CPU: Decimal(ceil(v * 10^3)) / Decimal(10^3), then max(., minimal).
bool round_cpu(double x, const Dec& minimal, std::string* out) {
    const Dec v = prom_decimal(x);
    Dec scaled = v;
    scaled.exp += 3;  // exact: the product keeps v's <= 17 significant digits
    Dec k = ceil_int(scaled);
    if ((int)k.d.size() > kPrec - 1) return false;
    // exact quotient k / 1000 at the ideal exponent 0: strip trailing zeros up to 3
    Dec q = k;
    q.exp = -3;
    while (q.exp < 0 && q.d.size() > 1 && q.d.back() == '0') {
        q.d.pop_back();
        ++q.exp;
    }
    if (q.d == "0") {
        q.exp = 0;
        q.neg = false;
    }
    *out = cmp(minimal, q) > 0 ? to_sci(minimal) : to_sci(q);
    return true;
}

// simple.py:29 then Runner._round_value for memory:
// raw = max * buffer (28-digit context); Decimal(ceil(raw * 10^-6)) / Decimal('0.000001'); max(., minimal).
bool round_mem(double x, const Dec& buffer, const Dec& minimal, std::string* out) {
    const Dec raw = round_prec(mul(prom_decimal(x), buffer), kPrec);
    Dec scaled = raw;
    scaled.exp -= 6;  // exact: raw has <= 28 digits
    Dec r = ceil_int(scaled);
    if ((int)r.d.size() > kPrec - 1) return false;
    Dec q = r;  // exact quotient r * 10^6 at the ideal exponent 6
    q.exp = 6;
    if (q.d == "0") q.neg = false;
    *out = cmp(minimal, q) > 0 ? to_sci(minimal) : to_sci(q);
    return true;
}

// ---- integer fast path ---------------------------------------------------------------
// The same arithmetic on 128-bit integers for the common case: the sample's shortest digits
// D (<= 17 of them) and, for memory, a buffer coefficient short enough that D * buffer has
// <= 28 digits (so the 28-digit context never rounds: the CLI path's Decimal('1.05'); the
// int-default path's 52-digit Decimal(1.05 float) takes the digit-string path above).
// Results are identical by construction (tests/test_fast_round.py pins both paths).
using u128 = unsigned __int128;
using i128 = __int128;

constexpr int kMaxInt = 38;  // decimal digits an i128 magnitude always holds (10^38 < 2^127)

struct Pow10 {
    u128 v[kMaxInt + 1];
    Pow10() {
        v[0] = 1;
        for (int i = 1; i <= kMaxInt; ++i) v[i] = v[i - 1] * 10;
    }
};
const Pow10 kPow10;

inline u128 pow10_u128(int e) { return kPow10.v[e]; }

// decimal digits of v (no divisions: compared against the powers of ten)
inline int ndigits(u128 v) {
    int n = 1;
    if (v >> 64 == 0) {
        const uint64_t w = (uint64_t)v;
        while (n < 20 && w >= (uint64_t)kPow10.v[n]) ++n;
        return n;
    }
    n = 20;
    while (n <= kMaxInt && v >= kPow10.v[n]) ++n;
    return n;
}

// q = m / 10^e and whether a remainder is left, 64-bit division when the operands fit
inline u128 div_pow10(u128 m, int e, bool* frac) {
    if (m >> 64 == 0 && e < 20) {
        const uint64_t w = (uint64_t)m, p = (uint64_t)kPow10.v[e];
        const uint64_t q = w / p;
        *frac = q * p != w;
        return q;
    }
    const u128 p = kPow10.v[e];
    const u128 q = m / p;
    *frac = q * p != m;
    return q;
}

// x's shortest round-trip digits: |x| = D * 10^E (D without trailing zeros; D = 0 for zero)
void shortest(double x, uint64_t* D, int* E) {
    char buf[48];
    auto res = std::to_chars(buf, buf + sizeof(buf), std::fabs(x), std::chars_format::scientific);
    *res.ptr = 0;
    uint64_t d = 0;
    int nd = 0;
    const char* p = buf;
    for (; *p && *p != 'e'; ++p)
        if (*p >= '0' && *p <= '9') {
            d = d * 10 + (uint64_t)(*p - '0');
            ++nd;
        }
    int e = (*p == 'e') ? atoi(p + 1) : 0;
    e -= nd - 1;
    while (d && d % 10 == 0) {
        d /= 10;
        ++e;
    }
    *D = d;
    *E = d ? e : 0;
}

// ceil((-1)^neg * m * 10^e) as a signed integer; false when it needs more than kMaxInt - 1 digits
bool ceil_scaled(bool neg, u128 m, int e, i128* out) {
    if (m == 0) {
        *out = 0;
        return true;
    }
    u128 q;
    bool frac = false;
    if (e >= 0) {
        if (ndigits(m) + e > kMaxInt - 1) return false;
        q = m * pow10_u128(e);
    } else if (-e >= kMaxInt) {
        q = 0;
        frac = true;
    } else {
        q = div_pow10(m, -e, &frac);
    }
    if (!neg && frac) ++q;  // toward +inf: a positive fraction rounds up, a negative one truncates
    if (ndigits(q) > kMaxInt - 1) return false;
    *out = neg ? -(i128)q : (i128)q;
    return true;
}

// The smallest integer t with k < t <=> k * 10^e < minimal (i.e. t = ceil(minimal * 10^-e))
bool threshold(const Dec& minimal, int e, i128* t) {
    if (minimal.d.size() > (size_t)kMaxInt - 1) {  // e.g. the CPU floor 0.0050000000000000001040834...
        Dec m = minimal;
        m.exp -= e;
        const Dec c = ceil_int(m);
        if (c.d.size() > (size_t)kMaxInt - 2) return false;
        u128 v = 0;
        for (char ch : c.d) v = v * 10 + (u128)(ch - '0');
        *t = c.neg ? -(i128)v : (i128)v;
        return true;
    }
    u128 v = 0;
    for (char ch : minimal.d) v = v * 10 + (u128)(ch - '0');
    return ceil_scaled(minimal.neg, v, minimal.exp - e, t);
}

// str(Decimal) of coefficient k (signed) at exponent exp into dst (NUL-terminated)
void put_sci(char* dst, i128 k, int exp) {
    char dig[48];
    int n = 0;
    const bool neg = k < 0;
    u128 v = neg ? (u128)(-k) : (u128)k;
    while (v >> 64) {
        dig[n++] = (char)('0' + (int)(v % 10));
        v /= 10;
    }
    uint64_t w = (uint64_t)v;
    do {
        dig[n++] = (char)('0' + (int)(w % 10));
        w /= 10;
    } while (w);
    char* o = dst;
    if (neg) *o++ = '-';
    const int adjusted = exp + n - 1;
    if (exp <= 0 && adjusted >= -6) {
        const int point = n + exp;  // digits before the point
        if (exp == 0) {
            for (int i = n; i-- > 0;) *o++ = dig[i];
        } else if (point > 0) {
            for (int i = n; i-- > 0;) {
                *o++ = dig[i];
                if (i == n - point) *o++ = '.';
            }
        } else {
            *o++ = '0';
            *o++ = '.';
            for (int z = 0; z < -point; ++z) *o++ = '0';
            for (int i = n; i-- > 0;) *o++ = dig[i];
        }
    } else {
        *o++ = dig[n - 1];
        if (n > 1) {
            *o++ = '.';
            for (int i = n - 1; i-- > 0;) *o++ = dig[i];
        }
        *o++ = 'E';
        *o++ = adjusted >= 0 ? '+' : '-';
        o += sprintf(o, "%d", adjusted >= 0 ? adjusted : -adjusted);
    }
    *o = 0;
}

struct Fast {
    bool cpu_ok = false, mem_ok = false;
    i128 cpu_t = 0, mem_t = 0;     // thresholds against the minimal (see threshold())
    std::string cpu_min_s, mem_min_s;
    u128 buf_c = 0;                // the memory buffer's coefficient and exponent
    int buf_e = 0;
    bool buf_neg = false;
    int buf_digits = 0;
};

// put_sci writes at most this many bytes (sign, 27 digits, point, "E+", exponent, NUL) for the
// coefficients the fast paths produce (< 10^27): any width >= 64 holds it
constexpr int32_t kFastMaxBytes = 40;

// Runner._round_value(CPU) of prom_decimal(x) into out (width bytes); false: not covered here
bool fast_cpu(double x, const Fast& F, char* out, int32_t width) {
    uint64_t D;
    int E;
    shortest(x, &D, &E);
    i128 k;  // ceil(v * 10^3)
    if (!ceil_scaled(std::signbit(x), D, E + 3, &k) || ndigits((u128)(k < 0 ? -k : k)) > kPrec - 1) return false;
    if (k < F.cpu_t) {
        if ((int32_t)F.cpu_min_s.size() + 1 > width) return false;
        memcpy(out, F.cpu_min_s.c_str(), F.cpu_min_s.size() + 1);
        return true;
    }
    if (width < kFastMaxBytes) return false;
    // k / 1000 at the ideal exponent 0: trailing zeros stripped up to 3
    int exp = -3;
    while (exp < 0 && k != 0 && (int)(k < 0 ? (uint64_t)(-k % 10) : (uint64_t)(k % 10)) == 0) {
        k /= 10;
        ++exp;
    }
    if (k == 0) exp = 0;
    put_sci(out, k, exp);
    return true;
}

// simple.py:29's max * buffer, then Runner._round_value(Memory); false: not covered here
bool fast_mem(double x, const Fast& F, char* out, int32_t width) {
    uint64_t D;
    int E;
    shortest(x, &D, &E);
    if (D && ndigits(D) + F.buf_digits > kPrec) return false;  // the 28-digit context would round
    const u128 P = (u128)D * F.buf_c;
    i128 r;  // ceil(raw * 10^-6)
    if (!ceil_scaled(std::signbit(x) != F.buf_neg && P != 0, P, E + F.buf_e - 6, &r) ||
        ndigits((u128)(r < 0 ? -r : r)) > kPrec - 1)
        return false;
    if (r < F.mem_t) {
        if ((int32_t)F.mem_min_s.size() + 1 > width) return false;
        memcpy(out, F.mem_min_s.c_str(), F.mem_min_s.size() + 1);
        return true;
    }
    if (width < kFastMaxBytes) return false;
    put_sci(out, r, 6);  // r * 10^6 at the ideal exponent 6
    return true;
}

// threads = 0: the CPUs of this process's affinity mask, capped by OMP_NUM_THREADS when set
// (hardware_concurrency counts the whole machine's CPUs, many times a GPU box's lease)
inline int default_threads() {
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

template <class F>
void parallel_for(int64_t n, int32_t threads, F f) {
    int t = threads > 0 ? threads : default_threads();
    if (t < 1) t = 1;
    if ((int64_t)t * 256 > n) t = (int)std::max<int64_t>(1, n / 256);
    if (t <= 1) {
        for (int64_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
        for (;;) {
            const int64_t b = next.fetch_add(256);
            if (b >= n) return;
            const int64_t e = std::min<int64_t>(b + 256, n);
            for (int64_t i = b; i < e; ++i) f(i);
        }
    };
    std::vector<std::thread> pool;
    for (int k = 1; k < t; ++k) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
}

}  // namespace

extern "C" int krr_round_simple(int64_t n, const double* cpu_value, const uint32_t* cpu_flags, const double* mem_value,
                                const uint32_t* mem_flags, const krr_round_params* params, char* cpu_out,
                                char* mem_out, int32_t width, uint8_t* status, int32_t threads) {
    if (n < 0 || !params || width < 64) return -1;
    if (n == 0) return 0;
    if (!cpu_value || !cpu_flags || !mem_value || !mem_flags || !cpu_out || !mem_out || !status) return -1;
    Dec buffer, cpu_min, mem_min;
    if (!parse_dec(params->mem_buffer, &buffer) || !parse_dec(params->cpu_minimal, &cpu_min) ||
        !parse_dec(params->mem_minimal, &mem_min))
        return -1;
    Fast F;
    F.cpu_min_s = to_sci(cpu_min);
    F.mem_min_s = to_sci(mem_min);
    F.cpu_ok = threshold(cpu_min, -3, &F.cpu_t) && params->fast_path != 0;
    F.mem_ok = buffer.d.size() < (size_t)kPrec && threshold(mem_min, 6, &F.mem_t) && params->fast_path != 0;
    if (F.mem_ok) {
        for (char ch : buffer.d) F.buf_c = F.buf_c * 10 + (u128)(ch - '0');
        F.buf_e = buffer.exp;
        F.buf_neg = buffer.neg;
        F.buf_digits = buffer.d == "0" ? 1 : (int)buffer.d.size();
    }
    parallel_for(n, threads, [&](int64_t i) {
        uint8_t st = 0;
        std::string s;
        char* co = cpu_out + (size_t)i * (size_t)width;
        char* mo = mem_out + (size_t)i * (size_t)width;
        const uint32_t cf = cpu_flags[i], mf = mem_flags[i];
        if (cf == kFlagEmpty) {
            put(co, width, "NaN");
        } else if (cf != 0 || !std::isfinite(cpu_value[i])) {
            st |= KRR_ROUND_CPU_FALLBACK;
        } else if (!(F.cpu_ok && fast_cpu(cpu_value[i], F, co, width)) &&
                   (!round_cpu(cpu_value[i], cpu_min, &s) || !put(co, width, s))) {
            st |= KRR_ROUND_CPU_FALLBACK;
        }
        if (mf == kFlagEmpty) {
            put(mo, width, "NaN");
        } else if (mf != 0 || !std::isfinite(mem_value[i])) {
            st |= KRR_ROUND_MEM_FALLBACK;
        } else if (!(F.mem_ok && fast_mem(mem_value[i], F, mo, width)) &&
                   (!round_mem(mem_value[i], buffer, mem_min, &s) || !put(mo, width, s))) {
            st |= KRR_ROUND_MEM_FALLBACK;
        }
        (void)kFlagNan;
        (void)kFlagCapacity;
        status[i] = st;
    });
    return 0;
}
