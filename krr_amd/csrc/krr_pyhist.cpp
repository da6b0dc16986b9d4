// krr_pyhist.cpp — the HistoryData packer (CPython C API, C++17).
//
// The reference hands SimpleStrategy.run one HistoryData per object:
// dict[ResourceType, dict[pod, list[Decimal]]] (core/abstract/strategies.py:35-36), each
// Decimal parsed from a Prometheus sample string (core/integrations/prometheus.py:152),
// and the strategy flattens the pods in dict order (strategies/simple.py:25, 32).
// pack_resource() walks those lists once and writes, for one resource of every object:
//   * the float64 CSR values (segment = the object's non-empty pods, dict order);
//   * per segment an exactness class — what the float64 values can stand for:
//       0 CANONICAL  every sample is the Decimal Prometheus' shortest round-trip string
//                    gives (prom_decimal of its float): rebuilding the Decimal from the
//                    kernel's float64 answer reproduces the reference's object;
//       1 FAITHFUL   every sample's VALUE is its float's shortest repr, but some
//                    representation differs ('0.10', '2.00E+7', '1E+2'): float order is
//                    Decimal order with the same ties, so the kernel's selection is the
//                    reference's, and the answer is the sample OBJECT at the located
//                    position (SimpleStrategy resolves it, krr_amd/core/exact.py);
//       2 INEXACT    some sample is not its float's shortest repr (more digits than a
//                    float64 holds, a non-Decimal, sNaN / -NaN): distinct values may share
//                    a float, so ties of the selected float are settled in Decimal;
//   * for class >= 1 segments, the tuple of the pod lists (positions index into them).
// A sample's float64 is float(Decimal) (correctly rounded: Eisel-Lemire for <= 19
// significant digits, strtod beyond).
#define PY_SSIZE_T_CLEAN
#include <Python.h>

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

// str(Decimal) (its to_sci_string) -> float64 value and exactness class.
uint8_t classify(const char* s, Py_ssize_t n, double* out) {
    const char* p = s;
    const char* e = s + n;
    bool neg = false;
    if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
    const Py_ssize_t rest = e - p;
    if (rest >= 3 && (memcmp(p, "NaN", 3) == 0 || (rest >= 4 && memcmp(p, "sNaN", 4) == 0))) {
        *out = std::numeric_limits<double>::quiet_NaN();
        // Prometheus' "NaN" parses to Decimal('NaN'); a sign, payload or sNaN did not come from it
        return (!neg && p == s && rest == 3) ? kCanonical : kInexact;
    }
    if (rest == 8 && memcmp(p, "Infinity", 8) == 0) {
        *out = neg ? -HUGE_VAL : HUGE_VAL;
        return kCanonical;  // "+Inf" / "-Inf"
    }
    // coefficient digits [. digits] [E [+-] digits]
    uint64_t w = 0;        // significant digits without trailing zeros (while <= 19 of them)
    int sig = 0;           // significant digits so far (leading zeros excluded)
    int tz = 0;            // trailing zeros of the coefficient
    int frac = 0;
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
            // a nonzero digit: the pending zeros become significant
            for (int z = 0; z < tz; ++z) {
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
    const long long exp = ex - frac;          // value = coefficient * 10^exp
    if (sig == 0) {                           // a zero
        *out = neg ? -0.0 : 0.0;
        return exp == 0 ? kCanonical : kFaithful;  // Go prints "0" / "-0"
    }
    const long long es = exp + tz;            // value = w * 10^es, w without trailing zeros
    double f;
    if (sig <= 19 && es > -100000 && es < 100000) {
        f = krr::json::from_bits(krr::json::eisel_lemire(w, es));
    } else {
        f = std::fabs(strtod(s, nullptr));  // s is NUL-terminated (PyUnicode_AsUTF8AndSize)
    }
    f = neg ? -f : f;
    *out = f;
    bool faithful;
    if (sig > 17 || !std::isfinite(f)) {
        faithful = false;  // a shortest repr has <= 17 digits; inf: out of range
    } else if (sig <= 15 && std::fabs(f) >= std::numeric_limits<double>::min()) {
        faithful = true;   // DBL_DIG: <= 15 digits round-trip through a normal float64
    } else {
        // compare with the float's shortest round-trip digits
        char buf[48];
        auto r = std::to_chars(buf, buf + sizeof(buf), std::fabs(f), std::chars_format::scientific);
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
        faithful = dw == w && de == es;
    }
    if (!faithful) return kInexact;
    // prom_decimal's form: positional, no trailing fraction zeros ('f', -1)
    const bool canonical = es >= 0 ? exp == 0 : tz == 0;
    return canonical ? kCanonical : kFaithful;
}

struct Out {
    std::vector<int64_t> lens;
    std::vector<uint8_t> cls;
};

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

// pack_resource(histories, resource, Decimal) -> (values: bytearray, lens: bytes, cls: bytes, sources: list)
PyObject* pack_resource(PyObject*, PyObject* args) {
    PyObject *histories, *resource, *dec_type;
    if (!PyArg_ParseTuple(args, "OOO", &histories, &resource, &dec_type)) return nullptr;
    PyObject* hs = PySequence_Fast(histories, "histories must be a sequence");
    if (!hs) return nullptr;
    const Py_ssize_t S = PySequence_Fast_GET_SIZE(hs);
    // pass 1: every segment's pod lists (non-empty ones, dict order) and the total count
    std::vector<PyObject*> seg_pods(S, nullptr);  // owned: list of sample sequences
    Py_ssize_t total = 0;
    Out o;
    o.lens.assign(S, 0);
    o.cls.assign(S, kCanonical);
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
        const Py_ssize_t np_ = PyList_GET_SIZE(vals);
        for (Py_ssize_t i = 0; i < np_; ++i) {
            PyObject* samples = PyList_GET_ITEM(vals, i);
            PyObject* fast = PySequence_Fast(samples, "pod samples must be a sequence");
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
            o.lens[s] += len;
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
                    PyObject* x = items[j];
                    double v;
                    if (Py_TYPE(x) == (PyTypeObject*)dec_type) {
                        PyObject* str = PyObject_Str(x);
                        if (!str) goto done;
                        Py_ssize_t n;
                        const char* b = PyUnicode_AsUTF8AndSize(str, &n);
                        if (!b) {
                            Py_DECREF(str);
                            goto done;
                        }
                        const uint8_t k = classify(b, n, &v);
                        Py_DECREF(str);
                        if (k > c) c = k;
                    } else {
                        // not a Decimal (a subclass, int, float ...): its own comparisons decide ties
                        v = PyFloat_AsDouble(x);
                        if (v == -1.0 && PyErr_Occurred()) goto done;
                        c = kInexact;
                    }
                    out[at++] = v;
                }
            }
            o.cls[s] = c;
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
    result = Py_BuildValue("(Oy#y#O)", values, reinterpret_cast<const char*>(o.lens.data()),
                           (Py_ssize_t)(8 * S), reinterpret_cast<const char*>(o.cls.data()), (Py_ssize_t)S,
                           sources);
done:
    for (PyObject* k : seg_pods) Py_XDECREF(k);
    Py_XDECREF(values);
    Py_XDECREF(sources);
    Py_DECREF(hs);
    return result;
}

// classify(str) -> (float, class): one sample, for tests and the Python-side checks
PyObject* classify_str(PyObject*, PyObject* args) {
    const char* s;
    Py_ssize_t n;
    if (!PyArg_ParseTuple(args, "s#", &s, &n)) return nullptr;
    double v;
    const uint8_t c = classify(s, n, &v);
    return Py_BuildValue("(di)", v, (int)c);
}

PyMethodDef methods[] = {
    {"pack_resource", pack_resource, METH_VARARGS,
     "HistoryData list -> (float64 CSR values, lens, exactness class, pod lists) for one resource"},
    {"classify", classify_str, METH_VARARGS, "str(Decimal) -> (float64, exactness class)"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module = {PyModuleDef_HEAD_INIT, "_krr_pyhist", nullptr, -1, methods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__krr_pyhist(void) { return PyModule_Create(&module); }
