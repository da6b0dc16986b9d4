// krr_pydec.cpp — Decimal-level host work around the kernels (CPython C API, C++17).
//
// 1. pack_resource: the HistoryData packer.  The reference hands SimpleStrategy.run one
//    HistoryData per object: dict[ResourceType, dict[pod, list[Decimal]]]
//    (core/abstract/strategies.py:35-36), each Decimal parsed from a Prometheus sample
//    string (core/integrations/prometheus.py:152), and the strategy flattens the pods in
//    dict order (strategies/simple.py:25, 32).  pack_resource walks those lists once and
//    writes, for one resource of every object:
//      * the float64 CSR values (segment = the object's non-empty pods, dict order);
//      * per segment an exactness class — what the float64 values can stand for:
//          0 CANONICAL  every sample is the Decimal Prometheus' shortest round-trip string
//                       gives (prom_decimal of its float): rebuilding the Decimal from the
//                       kernel's float64 answer reproduces the reference's object;
//          1 FAITHFUL   every sample's VALUE is its float's shortest repr, but some
//                       representation differs ('0.10', '2.00E+7', '1E+2'): float order is
//                       Decimal order with the same ties, so the kernel's selection is the
//                       reference's, and the answer is the sample OBJECT at the located
//                       position (SimpleStrategy resolves it, krr_amd/core/exact.py);
//          2 INEXACT    some sample is not its float's shortest repr (more digits than a
//                       float64 holds, a non-Decimal, sNaN / -NaN): distinct values may
//                       share a float, so ties of the selected float are settled in Decimal;
//      * for class >= 1 segments, the tuple of the pod lists (positions index into them).
//    A sample's float64 is float(Decimal), correctly rounded (Eisel-Lemire for <= 19
//    significant digits, strtod beyond).
// 2. scan_fleet: Runner._collect_result's ResourceScan.calculate per object + Result's score
//    (core/runner.py:122-131, core/models/result.py:33-150) for a whole fleet: the four
//    Severity.calculate per object decided on float64 images, a pair whose margin to a
//    threshold float64 cannot be trusted settled by the caller's exact Decimal restatement,
//    and the reference's own pydantic-v1 model objects built in construct() layout.
//
// Decimal values are read from the C decimal object itself (CPython 3.10 _decimal: a
// libmpdec mpd_t inside the object; coefficient in base-10^19 words), a layout checked
// against Decimal.as_tuple() when the module loads — if it does not match, every sample
// goes through str(Decimal) instead (same results, slower).
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <vector>

#include "krr_json_parse.h"

namespace {

enum : uint8_t { kCanonical = 0, kFaithful = 1, kInexact = 2 };

bool is_digit(char c) { return c >= '0' && c <= '9'; }

// ---- the C decimal object ----------------------------------------------------------------
struct MpdT {  // libmpdec mpd_t
    uint8_t flags;
    Py_ssize_t exp;
    Py_ssize_t digits;
    Py_ssize_t len;
    Py_ssize_t alloc;
    uint64_t* data;
};
struct PyDecObj {  // CPython 3.10 Modules/_decimal/_decimal.c PyDecObject
    PyObject_HEAD
    Py_hash_t hash;
    MpdT dec;
};
constexpr uint8_t kMpdNeg = 1, kMpdInf = 2, kMpdNan = 4, kMpdSnan = 8, kMpdSpecial = kMpdInf | kMpdNan | kMpdSnan;

PyTypeObject* g_dec_type = nullptr;  // decimal.Decimal
bool g_layout_ok = false;            // the struct above checked against as_tuple()

// A finite Decimal whose coefficient fits one word (<= 19 digits): w * 10^exp, sign.
struct DecView {
    bool neg;
    uint8_t special;  // 0 finite, else kMpdInf / kMpdNan / kMpdSnan
    uint64_t w;
    int64_t exp;
    int64_t digits;
};

// true: *v describes x (a decimal.Decimal whose coefficient fits one word, or a special)
inline bool dec_view(PyObject* x, DecView* v) {
    if (!g_layout_ok || Py_TYPE(x) != g_dec_type) return false;
    const MpdT& m = reinterpret_cast<PyDecObj*>(x)->dec;
    v->neg = m.flags & kMpdNeg;
    v->special = m.flags & kMpdSpecial;
    if (v->special) {  // w: a NaN's payload (nonzero if any word is)
        v->w = (m.len > 1 || (m.len == 1 && m.data[0])) ? 1 : 0;
        return true;
    }
    if (m.len != 1) return false;
    v->w = m.data[0];
    v->exp = m.exp;
    v->digits = m.digits;
    return true;
}

// The class of a finite value given as (-1)^neg * ws * 10^es, ws without trailing zeros
// (sig digits, sig == 0 for zero), exp the raw exponent, tz the raw trailing zeros, f its
// correctly rounded magnitude as float64.
uint8_t classify_finite(bool neg, uint64_t ws, int sig, long long exp, int tz, double f, double* out) {
    if (sig == 0) {
        *out = neg ? -0.0 : 0.0;
        return exp == 0 ? kCanonical : kFaithful;  // Go prints "0" / "-0"
    }
    *out = neg ? -f : f;
    const long long es = exp + tz;
    bool faithful;
    if (sig > 17 || !std::isfinite(f)) {
        faithful = false;  // a shortest repr has <= 17 digits; inf: out of range
    } else if (sig <= 15 && f >= std::numeric_limits<double>::min()) {
        faithful = true;   // DBL_DIG: <= 15 digits round-trip through a normal float64
    } else {
        // compare with the float's shortest round-trip digits
        char buf[48];
        auto r = std::to_chars(buf, buf + sizeof(buf), f, std::chars_format::scientific);
        *r.ptr = 0;
        uint64_t dw = 0;
        int nd = 0;
        const char* q = buf;
        for (; *q && *q != 'e'; ++q)
            if (is_digit(*q)) {
                dw = dw * 10 + (uint64_t)(*q - '0');
                ++nd;
            }
        long long de = (*q == 'e') ? strtoll(q + 1, nullptr, 10) : 0;
        de -= nd - 1;
        while (dw && dw % 10 == 0) {
            dw /= 10;
            ++de;
        }
        faithful = dw == ws && de == es;
    }
    if (!faithful) return kInexact;
    // prom_decimal's form: positional, no trailing fraction zeros ('f', -1)
    return (es >= 0 ? exp == 0 : tz == 0) ? kCanonical : kFaithful;
}

using u128 = unsigned __int128;

struct Pow10 {
    u128 v[39];
    Pow10() {
        v[0] = 1;
        for (int i = 1; i < 39; ++i) v[i] = v[i - 1] * 10;
    }
};
const Pow10 kPow10;

inline u128 pow10_u128(int e) { return kPow10.v[e]; }

inline double w_pow10(uint64_t w, long long e) {
    if (w == 0) return 0.0;
    if (e <= -100000) return 0.0;
    if (e >= 100000) return HUGE_VAL;
    return krr::json::from_bits(krr::json::eisel_lemire(w, e));
}

// A view -> float64 and class (specials included).
uint8_t classify_view(const DecView& v, double* out) {
    if (v.special) {
        if (v.special == kMpdInf) {
            *out = v.neg ? -HUGE_VAL : HUGE_VAL;
            return kCanonical;  // "+Inf" / "-Inf"
        }
        *out = std::numeric_limits<double>::quiet_NaN();
        // Prometheus' "NaN" is Decimal('NaN'): no sign, no payload (coefficient 0), quiet
        return (v.special == kMpdNan && !v.neg && !v.w) ? kCanonical : kInexact;
    }
    uint64_t ws = v.w;
    int tz = 0;
    if (ws) {
        while (ws % 10 == 0) {
            ws /= 10;
            ++tz;
        }
    }
    const int sig = ws ? (int)v.digits - tz : 0;
    return classify_finite(v.neg, ws, sig, v.exp, tz, w_pow10(ws, v.exp + tz), out);
}

// str(Decimal) (its to_sci_string) -> float64 value and exactness class.
uint8_t classify(const char* s, Py_ssize_t n, double* out) {
    const char* p = s;
    const char* e = s + n;
    bool neg = false;
    if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
    const Py_ssize_t rest = e - p;
    if (rest >= 3 && (memcmp(p, "NaN", 3) == 0 || (rest >= 4 && memcmp(p, "sNaN", 4) == 0))) {
        *out = std::numeric_limits<double>::quiet_NaN();
        return (!neg && p == s && rest == 3) ? kCanonical : kInexact;
    }
    if (rest == 8 && memcmp(p, "Infinity", 8) == 0) {
        *out = neg ? -HUGE_VAL : HUGE_VAL;
        return kCanonical;
    }
    uint64_t w = 0;  // significant digits without trailing zeros (while <= 19 of them)
    int sig = 0, tz = 0, frac = 0;
    bool point = false, any = false;
    for (; p < e; ++p) {
        const char c = *p;
        if (is_digit(c)) {
            any = true;
            if (point) ++frac;
            if (c == '0') {
                if (sig) ++tz;
                continue;
            }
            for (int z = 0; z < tz; ++z) {  // the pending zeros become significant
                if (sig < 20) w = w * 10;
                ++sig;
            }
            tz = 0;
            if (sig < 20) w = w * 10 + (uint64_t)(c - '0');
            ++sig;
        } else if (c == '.' && !point) {
            point = true;
        } else {
            break;
        }
    }
    if (!any) {
        *out = std::numeric_limits<double>::quiet_NaN();
        return kInexact;
    }
    long long ex = 0;
    if (p < e && (*p == 'E' || *p == 'e')) {
        ++p;
        bool eneg = false;
        if (p < e && (*p == '-' || *p == '+')) eneg = *p++ == '-';
        for (; p < e && is_digit(*p); ++p)
            if (ex < 100000000) ex = ex * 10 + (*p - '0');
        if (eneg) ex = -ex;
    }
    const long long exp = ex - frac;
    if (sig == 0) return classify_finite(neg, 0, 0, exp, 0, 0.0, out);
    const double f = sig <= 19 ? w_pow10(w, exp + tz) : std::fabs(strtod(s, nullptr));  // s is NUL-terminated
    return classify_finite(neg, w, sig, exp, tz, f, out);
}

// One sample -> float64 and class; false with a Python error set.
bool sample_value(PyObject* x, double* v, uint8_t* cls) {
    DecView dv;
    if (dec_view(x, &dv)) {
        *cls = classify_view(dv, v);
        return true;
    }
    if (Py_TYPE(x) == g_dec_type) {
        PyObject* str = PyObject_Str(x);
        if (!str) return false;
        Py_ssize_t n;
        const char* b = PyUnicode_AsUTF8AndSize(str, &n);
        if (!b) {
            Py_DECREF(str);
            return false;
        }
        *cls = classify(b, n, v);
        Py_DECREF(str);
        return true;
    }
    // not a Decimal (a subclass, int, float ...): its own comparisons decide ties
    *v = PyFloat_AsDouble(x);
    if (*v == -1.0 && PyErr_Occurred()) return false;
    *cls = kInexact;
    return true;
}

// The layout check: views of probe Decimals against as_tuple().
bool check_layout(PyObject* dec_type) {
    static const char* probes[] = {"0", "-0", "123.45", "-1E+7", "0.10", "9999999999999999999", "1E-400",
                                   "-0.000001234", "42E+5", "NaN", "-Infinity", "sNaN"};
    for (const char* s : probes) {
        PyObject* d = PyObject_CallFunction(dec_type, "s", s);
        if (!d) return false;
        PyObject* t = PyObject_CallMethod(d, "as_tuple", nullptr);
        bool ok = t && PyTuple_Check(t) && PyTuple_GET_SIZE(t) == 3;
        if (ok) {
            const MpdT& m = reinterpret_cast<PyDecObj*>(d)->dec;
            const long sign = PyLong_AsLong(PyTuple_GET_ITEM(t, 0));
            PyObject* digits = PyTuple_GET_ITEM(t, 1);
            PyObject* expo = PyTuple_GET_ITEM(t, 2);
            ok = sign == (long)(m.flags & kMpdNeg);
            if (ok && PyUnicode_Check(expo)) {  // 'n' NaN, 'N' sNaN, 'F' Infinity
                const char* k = PyUnicode_AsUTF8(expo);
                const uint8_t want = k[0] == 'F' ? kMpdInf : (k[0] == 'n' ? kMpdNan : kMpdSnan);
                ok = (m.flags & kMpdSpecial) == want;
            } else if (ok) {
                ok = !(m.flags & kMpdSpecial) && PyLong_AsSsize_t(expo) == m.exp && m.len == 1 &&
                     PyTuple_GET_SIZE(digits) == m.digits;
                uint64_t w = 0;
                for (Py_ssize_t i = 0; ok && i < PyTuple_GET_SIZE(digits); ++i)
                    w = w * 10 + (uint64_t)PyLong_AsLong(PyTuple_GET_ITEM(digits, i));
                ok = ok && w == m.data[0];
            }
        }
        Py_XDECREF(t);
        Py_DECREF(d);
        if (PyErr_Occurred()) PyErr_Clear();
        if (!ok) return false;
    }
    return true;
}

// ---- pack_resource --------------------------------------------------------------------

// The resource's pod mapping of one HistoryData (`h.get(resource) or {}`), new reference.
PyObject* pods_of(PyObject* h, PyObject* resource) {
    PyObject* pods;
    if (PyDict_Check(h)) {
        pods = PyDict_GetItemWithError(h, resource);
        if (!pods) return PyErr_Occurred() ? nullptr : PyDict_New();
        Py_INCREF(pods);
    } else {
        pods = PyObject_CallMethod(h, "get", "O", resource);
        if (!pods) return nullptr;
    }
    int truth = PyObject_IsTrue(pods);
    if (truth < 0) {
        Py_DECREF(pods);
        return nullptr;
    }
    if (!truth) {
        Py_DECREF(pods);
        return PyDict_New();
    }
    return pods;
}

// list(pods.values()) as a new reference
PyObject* pod_values(PyObject* pods) {
    if (PyDict_Check(pods)) return PyDict_Values(pods);
    PyObject* v = PyObject_CallMethod(pods, "values", nullptr);
    if (!v) return nullptr;
    PyObject* l = PySequence_List(v);
    Py_DECREF(v);
    return l;
}

// pack_resource(histories, resource) -> (values: bytearray, lens: bytes, cls: bytes, sources: list)
PyObject* pack_resource(PyObject*, PyObject* args) {
    PyObject *histories, *resource;
    if (!PyArg_ParseTuple(args, "OO", &histories, &resource)) return nullptr;
    PyObject* hs = PySequence_Fast(histories, "histories must be a sequence");
    if (!hs) return nullptr;
    const Py_ssize_t S = PySequence_Fast_GET_SIZE(hs);
    // pass 1: every segment's pod lists (non-empty ones, dict order) and the total count
    std::vector<PyObject*> seg_pods(S, nullptr);  // owned: list of sample sequences
    std::vector<int64_t> lens(S, 0);
    std::vector<uint8_t> cls(S, kCanonical);
    Py_ssize_t total = 0;
    PyObject *values = nullptr, *sources = nullptr, *result = nullptr;
    for (Py_ssize_t s = 0; s < S; ++s) {
        PyObject* pods = pods_of(PySequence_Fast_GET_ITEM(hs, s), resource);
        if (!pods) goto done;
        PyObject* vals = pod_values(pods);
        Py_DECREF(pods);
        if (!vals) goto done;
        PyObject* kept = PyList_New(0);
        if (!kept) {
            Py_DECREF(vals);
            goto done;
        }
        seg_pods[s] = kept;
        for (Py_ssize_t i = 0; i < PyList_GET_SIZE(vals); ++i) {
            PyObject* fast = PySequence_Fast(PyList_GET_ITEM(vals, i), "pod samples must be a sequence");
            if (!fast) {
                Py_DECREF(vals);
                goto done;
            }
            const Py_ssize_t len = PySequence_Fast_GET_SIZE(fast);
            if (len && PyList_Append(kept, fast) < 0) {
                Py_DECREF(fast);
                Py_DECREF(vals);
                goto done;
            }
            Py_DECREF(fast);
            lens[s] += len;
            total += len;
        }
        Py_DECREF(vals);
    }
    values = PyByteArray_FromStringAndSize(nullptr, (Py_ssize_t)(8 * total));
    sources = PyList_New(S);
    if (!values || !sources) goto done;
    {
        double* out = reinterpret_cast<double*>(PyByteArray_AS_STRING(values));
        Py_ssize_t at = 0;
        for (Py_ssize_t s = 0; s < S; ++s) {
            PyObject* kept = seg_pods[s];
            uint8_t c = kCanonical;
            for (Py_ssize_t i = 0; i < PyList_GET_SIZE(kept); ++i) {
                PyObject* fast = PyList_GET_ITEM(kept, i);
                const Py_ssize_t len = PySequence_Fast_GET_SIZE(fast);
                PyObject** items = PySequence_Fast_ITEMS(fast);
                for (Py_ssize_t j = 0; j < len; ++j) {
                    uint8_t k;
                    if (!sample_value(items[j], &out[at++], &k)) goto done;
                    if (k > c) c = k;
                }
            }
            cls[s] = c;
            PyObject* src = Py_None;
            if (c != kCanonical) {
                src = PyList_AsTuple(kept);
                if (!src) goto done;
            } else {
                Py_INCREF(src);
            }
            PyList_SET_ITEM(sources, s, src);
        }
    }
    result = Py_BuildValue("(Oy#y#O)", values, reinterpret_cast<const char*>(lens.data()), (Py_ssize_t)(8 * S),
                           reinterpret_cast<const char*>(cls.data()), (Py_ssize_t)S, sources);
done:
    for (PyObject* k : seg_pods) Py_XDECREF(k);
    Py_XDECREF(values);
    Py_XDECREF(sources);
    Py_DECREF(hs);
    return result;
}

// classify(str) -> (float, class): one sample's string, for tests
PyObject* classify_str(PyObject*, PyObject* args) {
    const char* s;
    Py_ssize_t n;
    if (!PyArg_ParseTuple(args, "s#", &s, &n)) return nullptr;
    double v;
    const uint8_t c = classify(s, n, &v);
    return Py_BuildValue("(di)", v, (int)c);
}

// sample(x) -> (float, class): one sample object through the packer's own path
PyObject* sample_py(PyObject*, PyObject* x) {
    double v;
    uint8_t c;
    if (!sample_value(x, &v, &c)) return nullptr;
    return Py_BuildValue("(di)", v, (int)c);
}

// ---- scan_fleet -----------------------------------------------------------------------

// Severity codes in ResourceScan.calculate's precedence (result.py:83-87)
enum : int { kCritical = 0, kWarning = 1, kOk = 2, kGood = 3, kUnknown = 4 };
constexpr double kMargin = 1e-9;  // krr_amd/core/models/result.py _MARGIN

// The cyclic GC need not traverse the result graphs built here: they are trees (a scan ->
// its recommendation -> dicts -> Recommendation -> value / severity, and the caller's
// object), so no reference cycle runs through them as built.  Untracking them keeps the
// gen-0 collection the next allocation triggers from walking millions of fresh objects (a
// full traversal, ~3 us per scan, otherwise).  A dict that later receives a container is
// tracked again by CPython itself; a cycle a caller later builds through an instance is
// kept alive rather than collected.
inline void untrack(PyObject* o) {
    if (PyObject_IS_GC(o)) PyObject_GC_UnTrack(o);
}

// A model class built in pydantic v1 construct() layout: field names (dict order), one
// fields-set shared by its instances (see make()), and where the __fields_set__ slot lives.
struct Model {
    PyTypeObject* cls = nullptr;
    PyObject* names[3] = {nullptr, nullptr, nullptr};
    Py_hash_t hashes[3] = {0, 0, 0};
    int n = 0;
    PyObject* fields_set = nullptr;
    Py_ssize_t fs_offset = 0;
    bool skip_dict = false;  // profiling variant KRR_X_NODICT only: instances without a dict
    // A prototype instance dict (split table, field k's value at ma_values[k]): each new
    // instance's dict is PyDict_Copy of it (for a split table: the shared keys and a copy of
    // the values array) with the values then replaced in place — no key lookups.  Null when
    // the class's dicts are not laid out so (the SetItem path below is used).
    PyObject* proto = nullptr;

    ~Model() { Py_XDECREF(proto); }

    // Build `proto` from one instance made the slow way with the field names as sentinel
    // values, if its dict is a split table holding field k at value slot k.
    void init_proto() {
        PyObject* o = make_slow(names[0], names[1], n > 2 ? names[2] : nullptr);
        if (!o) {
            PyErr_Clear();
            return;
        }
        PyObject** dp = _PyObject_GetDictPtr(o);
        PyObject* d = dp ? *dp : nullptr;
        bool ok = d && PyDict_CheckExact(d) && reinterpret_cast<PyDictObject*>(d)->ma_values != nullptr &&
                  PyDict_GET_SIZE(d) == n;
        for (int k = 0; ok && k < n; ++k) ok = reinterpret_cast<PyDictObject*>(d)->ma_values[k] == names[k];
        if (ok) {
            Py_INCREF(d);
            proto = d;
        }
        Py_DECREF(o);
    }

    PyObject* make(PyObject* a, PyObject* b, PyObject* c = nullptr) const {
        if (!proto) return make_slow(a, b, c);
        PyObject* o = cls->tp_alloc(cls, 0);
        if (!o) return nullptr;
        PyObject** dp = _PyObject_GetDictPtr(o);
        PyObject* d = dp ? PyDict_Copy(proto) : nullptr;
        if (!d || reinterpret_cast<PyDictObject*>(d)->ma_values == nullptr) {  // (a combined copy: never)
            Py_XDECREF(d);
            Py_DECREF(o);
            return dp ? nullptr : make_slow(a, b, c);
        }
        PyObject** v = reinterpret_cast<PyDictObject*>(d)->ma_values;
        PyObject* vals[3] = {a, b, c};
        for (int k = 0; k < n; ++k) {
            PyObject* old = v[k];
            Py_INCREF(vals[k]);
            v[k] = vals[k];
            Py_DECREF(old);
        }
        untrack(d);
        *dp = d;
        untrack(o);
        Py_INCREF(fields_set);
        *reinterpret_cast<PyObject**>(reinterpret_cast<char*>(o) + fs_offset) = fields_set;
        return o;
    }

    PyObject* make_slow(PyObject* a, PyObject* b, PyObject* c = nullptr) const {
        PyObject* o = cls->tp_alloc(cls, 0);
        if (!o) return nullptr;
        // the instance dict as attribute assignment would create it: a split table sharing the
        // class's cached keys (the fields, in order), about half the size and time of a new dict
        PyObject* d = skip_dict ? nullptr : PyObject_GenericGetDict(o, nullptr);
        PyObject* vals[3] = {a, b, c};
        bool bad = !d && !skip_dict;
        for (int i = 0; !bad && d && i < n; ++i) bad = _PyDict_SetItem_KnownHash(d, names[i], vals[i], hashes[i]) < 0;
        if (!bad && d) untrack(d);
        Py_XDECREF(d);
        if (bad) {
            Py_DECREF(o);
            return nullptr;
        }
        untrack(o);
        // the class's fields-set, shared: it holds every field, so the add() pydantic's
        // __setattr__ does never changes it (these models forbid other names), and pydantic
        // itself shares a fields-set between a model and its validation copy
        // (pydantic/v1/main.py:729 _copy_and_set_values(value.__dict__, value.__fields_set__))
        Py_INCREF(fields_set);
        *reinterpret_cast<PyObject**>(reinterpret_cast<char*>(o) + fs_offset) = fields_set;
        return o;
    }
};

bool init_model(Model* m, PyObject* cls, PyObject* names, PyObject* fields_set, Py_ssize_t fs_offset) {
    if (!PyType_Check(cls) || !PyTuple_Check(names) || PyTuple_GET_SIZE(names) < 2 || PyTuple_GET_SIZE(names) > 3) {
        PyErr_SetString(PyExc_TypeError, "scan_fleet: bad model description");
        return false;
    }
    m->cls = reinterpret_cast<PyTypeObject*>(cls);
    m->n = (int)PyTuple_GET_SIZE(names);
    for (int i = 0; i < m->n; ++i) {
        m->names[i] = PyTuple_GET_ITEM(names, i);
        m->hashes[i] = PyObject_Hash(m->names[i]);
        if (m->hashes[i] == -1) return false;
    }
    m->fields_set = fields_set;
    m->fs_offset = fs_offset;
#ifndef KRR_X_NOPROTO
    m->init_proto();
#endif
    return true;
}

// x's float64 image when it is a finite decimal.Decimal (kind 0), else the kind:
// 1 None, 2 str ("?"), 3 other (NaN / Infinity Decimals, subclasses, numbers)
inline int value_kind(PyObject* x, double* f, DecView* v) {
    v->special = 1;  // no one-word view unless set below
    if (x == Py_None) return 1;
    if (PyUnicode_Check(x)) return 2;
    if (dec_view(x, v)) {
        if (v->special) return 3;
        const double m = w_pow10(v->w, v->exp);
        *f = v->neg ? -m : m;
        return 0;
    }
    v->special = 1;
    if (Py_TYPE(x) == g_dec_type) {  // a coefficient wider than one word
        PyObject* fin = PyObject_CallMethod(x, "is_finite", nullptr);
        const int finite = fin ? PyObject_IsTrue(fin) : -1;
        Py_XDECREF(fin);
        if (finite < 0) {
            PyErr_Clear();
            return 3;
        }
        if (!finite) return 3;
        *f = PyFloat_AsDouble(x);
        if (*f == -1.0 && PyErr_Occurred()) {
            PyErr_Clear();
            return 3;
        }
        return 0;
    }
    return 3;
}

// c == (1 + t) * r exactly, i.e. 4c == M r with M = 4 (1 + t), for one-word Decimals:
// 1 yes, 0 no, -1 cannot tell here (the aligned operands pass 37 digits)
int exact_tie(const DecView& c, const DecView& r, int M) {
    if (c.w == 0 || r.w == 0) return (c.w == 0 && r.w == 0) ? 1 : 0;
    if (c.neg != r.neg) return 0;  // M > 0
    const int64_t e = std::min(c.exp, r.exp);
    const int64_t da = c.exp - e, db = r.exp - e;
    if (da + 20 > 37 || db + 20 > 37) return -1;
    const u128 a = (u128)4 * c.w * pow10_u128((int)da), b = (u128)(unsigned)M * r.w * pow10_u128((int)db);
    return a == b ? 1 : 0;
}

inline int bucket(double diff) {
    if (diff > 1.0 || diff < -0.5) return kCritical;
    if (diff > 0.5 || diff < -0.25) return kWarning;
    return kGood;
}

// Severity.calculate(current, recommended) -> code, or -1 with an error set.  Decided on the
// float64 images; a diff within the margin of a threshold t is decided exactly when the
// values tie with it (current == (1 + t) * recommended: the reference's Decimal quotient is
// then exactly t, its subtraction exact); anything else near a threshold, and operands that
// are zero, subnormal, non-finite or not finite Decimals, go to `settle` (the Decimal
// restatement, which also raises what the reference raises).
int severity_code(PyObject* cur, PyObject* rec, PyObject* settle) {
    double c = 0.0, r = 1.0;
    DecView cv, rv;
    const int kc = value_kind(cur, &c, &cv), kr = value_kind(rec, &r, &rv);
    if (kc == 2 || kr == 2) return kUnknown;
    if (kc == 1 && kr == 1) return kOk;
    if (kc == 1 || kr == 1) return kWarning;
    bool exact = kc != 0 || kr != 0;
    if (!exact) {
        const double tiny = std::numeric_limits<double>::min();
        exact = !std::isfinite(c) || !std::isfinite(r) || std::fabs(r) < tiny || (c != 0 && std::fabs(c) < tiny);
    }
    if (!exact) {
        const double diff = (c - r) / r;
        const double scale = kMargin * (1.0 + std::fabs(c / r));
        static const double kT[4] = {1.0, -0.5, 0.5, -0.25};
        static const int kM[4] = {8, 2, 6, 3};
        int near = -1;
        for (int j = 0; j < 4; ++j)
            if (!(std::fabs(diff - kT[j]) > scale)) near = j;
        if (near < 0) return bucket(diff);
        if (cv.special == 0 && rv.special == 0 && exact_tie(cv, rv, kM[near]) == 1) return bucket(kT[near]);
        exact = true;
    }
    PyObject* code = PyObject_CallFunctionObjArgs(settle, cur, rec, nullptr);
    if (!code) return -1;
    const long k = PyLong_AsLong(code);
    Py_DECREF(code);
    return (k == -1 && PyErr_Occurred()) ? -1 : (int)k;
}

// attribute of a pydantic-v1 instance: its __dict__ entry, else the generic lookup (new ref)
inline PyObject* field(PyObject* o, PyObject* name, Py_hash_t h) {
    PyObject** dp = _PyObject_GetDictPtr(o);
    if (dp && *dp && PyDict_CheckExact(*dp)) {
        PyObject* v = _PyDict_GetItem_KnownHash(*dp, name, h);
        if (v) {
            Py_INCREF(v);
            return v;
        }
        if (PyErr_Occurred()) return nullptr;
    }
    return PyObject_GetAttr(o, name);
}

// d.get(k) with k's hash known; *present = whether k is a key (new reference)
inline PyObject* dict_get(PyObject* d, PyObject* k, Py_hash_t h, bool* present) {
    PyObject* v = nullptr;
    if (PyDict_Check(d)) {
        v = _PyDict_GetItem_KnownHash(d, k, h);
        if (!v && PyErr_Occurred()) return nullptr;
    } else {  // a Mapping
        v = PyObject_GetItem(d, k);
        if (!v) {
            if (!PyErr_ExceptionMatches(PyExc_KeyError)) return nullptr;
            PyErr_Clear();
        } else {
            Py_DECREF(v);  // borrowed semantics below; the mapping keeps it alive
        }
    }
    *present = v != nullptr;
    v = v ? v : Py_None;
    Py_INCREF(v);
    return v;
}

// The scan loop shared by scan_fleet and scan_columns.  `recommended(i, alloc_k, sel, rv_out)`
// gives object i's recommended value for resource type k under selector sel (0 requests,
// 1 limits) as a new reference and whether the key is present, or returns false with an error.
template <class RecOf>
PyObject* scan_loop(PyObject* ob, Py_ssize_t n, PyObject* rts, PyObject* sevs, PyObject* settle, Model* M,
                    RecOf recommended, bool* keys_ok) {
    const Py_ssize_t R = PyTuple_GET_SIZE(rts);
    PyObject* out = nullptr;
    PyObject* tmpl = nullptr;
    PyObject* s_alloc = PyUnicode_InternFromString("allocations");
    PyObject* s_req = PyUnicode_InternFromString("requests");
    PyObject* s_lim = PyUnicode_InternFromString("limits");
    Py_hash_t h_alloc = s_alloc ? PyObject_Hash(s_alloc) : -1, h_req = s_req ? PyObject_Hash(s_req) : -1,
              h_lim = s_lim ? PyObject_Hash(s_lim) : -1;
    Py_hash_t h_rt[8];
    bool ok = s_alloc && s_req && s_lim && h_alloc != -1 && h_req != -1 && h_lim != -1;
    for (Py_ssize_t k = 0; ok && k < R; ++k) ok = (h_rt[k] = PyObject_Hash(PyTuple_GET_ITEM(rts, k))) != -1;
    if (!ok) goto done;
    tmpl = _PyDict_NewPresized(R);
    for (Py_ssize_t k = 0; tmpl && k < R; ++k)
        if (_PyDict_SetItem_KnownHash(tmpl, PyTuple_GET_ITEM(rts, k), Py_None, h_rt[k]) < 0) Py_CLEAR(tmpl);
    if (!tmpl) goto done;
    out = PyList_New(n);
    if (!out) goto done;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* obj = PySequence_Fast_GET_ITEM(ob, i);
        PyObject* alloc = field(obj, s_alloc, h_alloc);
        PyObject* creq = alloc ? field(alloc, s_req, h_req) : nullptr;
        PyObject* clim = creq ? field(alloc, s_lim, h_lim) : nullptr;
        PyObject* dreq = clim ? PyDict_Copy(tmpl) : nullptr;  // {rt: None ...}: values replaced below
        PyObject* dlim = dreq ? PyDict_Copy(tmpl) : nullptr;
        bool bad = !dlim;
        int worst = kUnknown;
        for (Py_ssize_t k = 0; !bad && k < R; ++k) {
            PyObject* rt = PyTuple_GET_ITEM(rts, k);
            PyObject* sel_cur[2] = {creq, clim};
            PyObject* sel_out[2] = {dreq, dlim};
            for (int j = 0; !bad && j < 2; ++j) {
                bool pc = false, pr = false;
                PyObject* cv = dict_get(sel_cur[j], rt, h_rt[k], &pc);
                PyObject* rv = nullptr;
                if (cv && !recommended(i, k, j, h_rt[k], &rv, &pr)) rv = nullptr;
#ifndef KRR_X_NOSEV
                const int code = rv ? severity_code(cv, rv, settle) : -1;
#else  // profiling variant: no severity decided (scans not valid)
                const int code = rv ? kOk : -1;
#endif
                PyObject* r = code >= 0 ? M[0].make(rv, PyTuple_GET_ITEM(sevs, code)) : nullptr;
                bad = !r || _PyDict_SetItem_KnownHash(sel_out[j], rt, r, h_rt[k]) < 0;
                *keys_ok = *keys_ok && pc;  // Result's score indexes the current allocations (result.py:137-143)
                if (code >= 0 && code < worst) worst = code;
                Py_XDECREF(r);
                Py_XDECREF(cv);
                Py_XDECREF(rv);
            }
        }
        if (!bad) {
            untrack(dreq);
            untrack(dlim);
        }
        PyObject* rr = bad ? nullptr : M[1].make(dreq, dlim);
        PyObject* scan = rr ? M[2].make(obj, rr, PyTuple_GET_ITEM(sevs, worst)) : nullptr;
        Py_XDECREF(rr);
        Py_XDECREF(dreq);
        Py_XDECREF(dlim);
        Py_XDECREF(alloc);
        Py_XDECREF(creq);
        Py_XDECREF(clim);
        if (!scan) {
            Py_CLEAR(out);
            goto done;
        }
        PyList_SET_ITEM(out, i, scan);
    }
done:
    Py_XDECREF(tmpl);
    Py_XDECREF(s_alloc);
    Py_XDECREF(s_req);
    Py_XDECREF(s_lim);
    return out;
}

// The three models of a scan: (cls, field names, fields_set, slot offset) each.
bool init_scan_models(Model* M, PyObject* md_rec, PyObject* md_rr, PyObject* md_scan) {
    PyObject* mds[3] = {md_rec, md_rr, md_scan};
    for (int i = 0; i < 3; ++i) {
        PyObject* t = mds[i];
        if (PyTuple_GET_SIZE(t) != 4) {
            PyErr_SetString(PyExc_ValueError, "scan: model = (cls, names, fields_set, offset)");
            return false;
        }
        const Py_ssize_t off = PyLong_AsSsize_t(PyTuple_GET_ITEM(t, 3));
        if (off <= 0 || !init_model(&M[i], PyTuple_GET_ITEM(t, 0), PyTuple_GET_ITEM(t, 1), PyTuple_GET_ITEM(t, 2), off)) {
            if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "scan: bad slot offset");
            return false;
        }
    }
#ifdef KRR_X_NODICT  // profiling variant: the scan's models without instance dicts (not valid)
    for (int i = 0; i < 3; ++i) M[i].skip_dict = true;
#endif
    return true;
}

PyObject* scan_result(PyObject* out, bool keys_ok) {
    if (!out) return nullptr;
    PyObject* res = Py_BuildValue("(OO)", out, keys_ok ? Py_True : Py_False);
    Py_DECREF(out);
    return res;
}

// scan_fleet(objects, recommendations, rts, severities, settle, rec_model, rr_model, scan_model)
//   rts: tuple of ResourceType members; severities: the 5 Severity members in code order;
//   settle(current, recommended) -> code; *_model: (cls, field names, fields_set, slot offset)
// -> (scans, all_keys_present)
PyObject* scan_fleet(PyObject*, PyObject* args) {
    bool keys_ok = true;
    PyObject *objects, *recs, *rts, *sevs, *settle, *md_rec, *md_rr, *md_scan;
    if (!PyArg_ParseTuple(args, "OOO!O!OO!O!O!", &objects, &recs, &PyTuple_Type, &rts, &PyTuple_Type, &sevs, &settle,
                          &PyTuple_Type, &md_rec, &PyTuple_Type, &md_rr, &PyTuple_Type, &md_scan))
        return nullptr;
    if (PyTuple_GET_SIZE(sevs) != 5 || PyTuple_GET_SIZE(rts) < 1 || PyTuple_GET_SIZE(rts) > 8) {
        PyErr_SetString(PyExc_ValueError, "scan_fleet: 5 severities and 1..8 resource types");
        return nullptr;
    }
    Model M[3];
    if (!init_scan_models(M, md_rec, md_rr, md_scan)) return nullptr;
    PyObject* ob = PySequence_Fast(objects, "objects must be a sequence");
    if (!ob) return nullptr;
    PyObject* rb = PySequence_Fast(recs, "recommendations must be a sequence");
    if (!rb) {
        Py_DECREF(ob);
        return nullptr;
    }
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(ob);
    PyObject* out = nullptr;
    if (PySequence_Fast_GET_SIZE(rb) != n) {
        PyErr_SetString(PyExc_ValueError, "one recommendation per object");
    } else {
        PyObject* s_req = PyUnicode_InternFromString("requests");
        PyObject* s_lim = PyUnicode_InternFromString("limits");
        const Py_hash_t h_req = s_req ? PyObject_Hash(s_req) : -1, h_lim = s_lim ? PyObject_Hash(s_lim) : -1;
        if (h_req != -1 && h_lim != -1) {
            // the recommendation's selector dicts of the object in hand (fetched once per object)
            Py_ssize_t cur = -1;
            PyObject* sel[2] = {nullptr, nullptr};
            auto rec_of = [&](Py_ssize_t i, Py_ssize_t k, int j, Py_hash_t h, PyObject** rv, bool* present) {
                if (i != cur) {
                    Py_CLEAR(sel[0]);
                    Py_CLEAR(sel[1]);
                    cur = i;
                    PyObject* rec = PySequence_Fast_GET_ITEM(rb, i);
                    sel[0] = field(rec, s_req, h_req);
                    sel[1] = sel[0] ? field(rec, s_lim, h_lim) : nullptr;
                }
                if (!sel[1]) return false;
                *rv = dict_get(sel[j], PyTuple_GET_ITEM(rts, k), h, present);
                return *rv != nullptr;
            };
            out = scan_loop(ob, n, rts, sevs, settle, M, rec_of, &keys_ok);
            Py_XDECREF(sel[0]);
            Py_XDECREF(sel[1]);
        }
        Py_XDECREF(s_req);
        Py_XDECREF(s_lim);
    }
    Py_DECREF(ob);
    Py_DECREF(rb);
    return scan_result(out, keys_ok);
}

// scan_columns(objects, cpu_col, mem_col, rts, severities, settle, rec_model, rr_model, scan_model)
// -> (scans, all_keys_present): scan_fleet of the ResourceAllocations allocations() would build
// from the same columns (requests {cpu: c, mem: m}, limits {cpu: None, mem: m}; runner.py:113-120)
// without building them — Runner._collect_result only reads them (runner.py:122-131).
PyObject* scan_columns(PyObject*, PyObject* args) {
    bool keys_ok = true;
    PyObject *objects, *cl, *ml, *rts, *sevs, *settle, *md_rec, *md_rr, *md_scan;
    if (!PyArg_ParseTuple(args, "OO!O!O!O!OO!O!O!", &objects, &PyList_Type, &cl, &PyList_Type, &ml, &PyTuple_Type,
                          &rts, &PyTuple_Type, &sevs, &settle, &PyTuple_Type, &md_rec, &PyTuple_Type, &md_rr,
                          &PyTuple_Type, &md_scan))
        return nullptr;
    if (PyTuple_GET_SIZE(sevs) != 5 || PyTuple_GET_SIZE(rts) != 2) {
        PyErr_SetString(PyExc_ValueError, "scan_columns: 5 severities and the 2 resource types (CPU, Memory)");
        return nullptr;
    }
    Model M[3];
    if (!init_scan_models(M, md_rec, md_rr, md_scan)) return nullptr;
    PyObject* ob = PySequence_Fast(objects, "objects must be a sequence");
    if (!ob) return nullptr;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(ob);
    PyObject* out = nullptr;
    if (PyList_GET_SIZE(cl) != n || PyList_GET_SIZE(ml) != n) {
        PyErr_SetString(PyExc_ValueError, "one recommendation per object");
    } else {
        auto rec_of = [&](Py_ssize_t i, Py_ssize_t k, int j, Py_hash_t, PyObject** rv, bool* present) {
            PyObject* v = k == 0 ? (j == 0 ? PyList_GET_ITEM(cl, i) : Py_None) : PyList_GET_ITEM(ml, i);
            Py_INCREF(v);
            *rv = v;
            *present = true;
            return true;
        };
        out = scan_loop(ob, n, rts, sevs, settle, M, rec_of, &keys_ok);
    }
    Py_DECREF(ob);
    return scan_result(out, keys_ok);
}

// allocations(model, rts, cpu_list, mem_list) -> list: per object a ResourceAllocations
// (runner.py:113-120) in construct() layout — requests {cpu: c, mem: m}, limits
// {cpu: None, mem: m} — the values already what the model's validator leaves
// (allocations.py:33-51); model = (cls, field names, fields_set, slot offset).
PyObject* allocations(PyObject*, PyObject* args) {
    PyObject *md, *rts, *cl, *ml;
    if (!PyArg_ParseTuple(args, "O!O!O!O!", &PyTuple_Type, &md, &PyTuple_Type, &rts, &PyList_Type, &cl, &PyList_Type,
                          &ml))
        return nullptr;
    const Py_ssize_t n = PyList_GET_SIZE(cl);
    if (PyList_GET_SIZE(ml) != n || PyTuple_GET_SIZE(rts) != 2 || PyTuple_GET_SIZE(md) != 4) {
        PyErr_SetString(PyExc_ValueError, "allocations: two equal columns, two resource types, one model");
        return nullptr;
    }
    Model M;
    const Py_ssize_t off = PyLong_AsSsize_t(PyTuple_GET_ITEM(md, 3));
    if (off <= 0 || !init_model(&M, PyTuple_GET_ITEM(md, 0), PyTuple_GET_ITEM(md, 1), PyTuple_GET_ITEM(md, 2), off)) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_ValueError, "allocations: bad slot offset");
        return nullptr;
    }
    PyObject* ck = PyTuple_GET_ITEM(rts, 0);
    PyObject* mk = PyTuple_GET_ITEM(rts, 1);
    const Py_hash_t hc = PyObject_Hash(ck), hm = PyObject_Hash(mk);
    if (hc == -1 || hm == -1) return nullptr;
    PyObject* tmpl = _PyDict_NewPresized(2);
    if (!tmpl || _PyDict_SetItem_KnownHash(tmpl, ck, Py_None, hc) < 0 ||
        _PyDict_SetItem_KnownHash(tmpl, mk, Py_None, hm) < 0) {
        Py_XDECREF(tmpl);
        return nullptr;
    }
    PyObject* out = PyList_New(n);
    for (Py_ssize_t i = 0; out && i < n; ++i) {
        PyObject* c = PyList_GET_ITEM(cl, i);
        PyObject* m = PyList_GET_ITEM(ml, i);
        PyObject* req = PyDict_Copy(tmpl);
        PyObject* lim = req ? PyDict_Copy(tmpl) : nullptr;
        bool bad = !lim || _PyDict_SetItem_KnownHash(req, ck, c, hc) < 0 || _PyDict_SetItem_KnownHash(req, mk, m, hm) < 0 ||
                   _PyDict_SetItem_KnownHash(lim, mk, m, hm) < 0;
        if (!bad) {
            untrack(req);
            untrack(lim);
        }
        PyObject* o = bad ? nullptr : M.make(req, lim);
        Py_XDECREF(req);
        Py_XDECREF(lim);
        if (!o) {
            Py_CLEAR(out);
            break;
        }
        PyList_SET_ITEM(out, i, o);
    }
    Py_DECREF(tmpl);
    return out;
}

// slot_offset(member_descriptor) -> its byte offset in the instance (pydantic v1's
// BaseModel.__fields_set__ slot)
PyObject* slot_offset(PyObject*, PyObject* d) {
    if (Py_TYPE(d) != &PyMemberDescr_Type) {
        PyErr_SetString(PyExc_TypeError, "expected a member descriptor");
        return nullptr;
    }
    PyMemberDef* m = reinterpret_cast<PyMemberDescrObject*>(d)->d_member;
    if (m->type != T_OBJECT_EX && m->type != T_OBJECT) {
        PyErr_SetString(PyExc_TypeError, "not an object slot");
        return nullptr;
    }
    return PyLong_FromSsize_t(m->offset);
}

PyObject* layout_ok(PyObject*, PyObject*) { return PyBool_FromLong(g_layout_ok); }

// body_table(resources) -> (ptrs, lens, obj, obj_bytes): the device packer's flat body table in
// one pass over resources[r][o][i] (bytes bodies, objects of resource r numbered after those of
// r - 1): ptrs / lens / obj as int64 columns packed in bytes objects (the bodies' buffer
// addresses — valid while the caller holds `resources` — lengths and object ids), obj_bytes
// per object.  None when a body is not exactly bytes (the caller's Python path converts it).
PyObject* body_table(PyObject*, PyObject* resources) {
    PyObject* rs = PySequence_Fast(resources, "resources must be a sequence");
    if (!rs) return nullptr;
    std::vector<int64_t> ptrs, lens, obj, obj_bytes;
    bool ok = true, plain = true;
    int64_t base = 0;
    for (Py_ssize_t r = 0; ok && plain && r < PySequence_Fast_GET_SIZE(rs); ++r) {
        PyObject* objs = PySequence_Fast(PySequence_Fast_GET_ITEM(rs, r), "a resource must be a sequence");
        if (!objs) {
            ok = false;
            break;
        }
        const Py_ssize_t n = PySequence_Fast_GET_SIZE(objs);
        for (Py_ssize_t o = 0; ok && plain && o < n; ++o) {
            PyObject* bodies = PySequence_Fast(PySequence_Fast_GET_ITEM(objs, o), "an object's bodies must be a sequence");
            if (!bodies) {
                ok = false;
                break;
            }
            int64_t tot = 0;
            for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(bodies); ++i) {
                PyObject* b = PySequence_Fast_GET_ITEM(bodies, i);
                if (!PyBytes_CheckExact(b)) {
                    plain = false;
                    break;
                }
                ptrs.push_back((int64_t)(intptr_t)PyBytes_AS_STRING(b));
                lens.push_back((int64_t)PyBytes_GET_SIZE(b));
                obj.push_back(base + o);
                tot += (int64_t)PyBytes_GET_SIZE(b);
            }
            Py_DECREF(bodies);
            obj_bytes.push_back(tot);
        }
        base += n;
        Py_DECREF(objs);
    }
    Py_DECREF(rs);
    if (!ok) return nullptr;
    if (!plain) Py_RETURN_NONE;
    auto col = [](const std::vector<int64_t>& v) {
        return PyBytes_FromStringAndSize(reinterpret_cast<const char*>(v.data()), (Py_ssize_t)(v.size() * 8));
    };
    PyObject *a = col(ptrs), *l = col(lens), *ob = col(obj), *ob2 = col(obj_bytes);
    PyObject* res = (a && l && ob && ob2) ? PyTuple_Pack(4, a, l, ob, ob2) : nullptr;
    Py_XDECREF(a);
    Py_XDECREF(l);
    Py_XDECREF(ob);
    Py_XDECREF(ob2);
    return res;
}

PyMethodDef methods[] = {
    {"pack_resource", pack_resource, METH_VARARGS,
     "HistoryData list -> (float64 CSR values, lens, exactness class, pod lists) for one resource"},
    {"classify", classify_str, METH_VARARGS, "str(Decimal) -> (float64, exactness class)"},
    {"sample", sample_py, METH_O, "one sample object -> (float64, exactness class), the packer's path"},
    {"scan_fleet", scan_fleet, METH_VARARGS, "ResourceScan per object in construct() layout -> (scans, keys_ok)"},
    {"scan_columns", scan_columns, METH_VARARGS,
     "scan_fleet of the ResourceAllocations two value columns describe, without building them"},
    {"allocations", allocations, METH_VARARGS, "ResourceAllocations in construct() layout from value columns"},
    {"slot_offset", slot_offset, METH_O, "byte offset of an object slot (member descriptor)"},
    {"layout_ok", layout_ok, METH_NOARGS, "whether Decimals are read in place (else through str())"},
    {"body_table", body_table, METH_O, "resources[r][o][i] bytes -> (ptrs, lens, obj, obj_bytes) int64 columns"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_krr_pydec", nullptr, -1, methods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__krr_pydec(void) {
    PyObject* dec_mod = PyImport_ImportModule("decimal");
    if (!dec_mod) return nullptr;
    PyObject* dec_type = PyObject_GetAttrString(dec_mod, "Decimal");
    Py_DECREF(dec_mod);
    if (!dec_type || !PyType_Check(dec_type)) {
        Py_XDECREF(dec_type);
        return nullptr;
    }
    g_dec_type = reinterpret_cast<PyTypeObject*>(dec_type);  // kept for the module's lifetime
    // the C implementation (_decimal) only: _pydecimal objects have no mpd_t inside
    PyObject* cdec = PyImport_ImportModule("_decimal");
    bool is_c = false;
    if (cdec) {
        PyObject* t = PyObject_GetAttrString(cdec, "Decimal");
        is_c = t == dec_type;
        Py_XDECREF(t);
        Py_DECREF(cdec);
    }
    PyErr_Clear();
    g_layout_ok = is_c && g_dec_type->tp_basicsize >= (Py_ssize_t)sizeof(PyDecObj) && check_layout(dec_type);
    return PyModule_Create(&module);
}
