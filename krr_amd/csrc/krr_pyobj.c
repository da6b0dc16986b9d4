/* krr_pyobj.c — bulk construction of the reference's result objects (CPython C API).
 *
 * The reference builds, per object, a RunResult of ResourceRecommendations
 * (strategies/simple.py:42-49, rounded by core/runner.py:57-86) and then a
 * ResourceAllocations (core/runner.py:113-120).  krr_amd.core.fast_round computes every
 * rounded value natively (include/krr_round.h); this module turns those columns into the
 * objects themselves without a per-object Python frame:
 *   decimal_column   fixed-width str(Decimal) strings -> one Decimal per distinct string
 *                    (a hash table over the raw bytes), as a list;
 *   allocations      per object a `model` instance whose fields are exactly what the model's
 *                    validator would leave (pydantic v1 construct layout: the field dict and
 *                    the fields-set, set through object.__setattr__);
 *   run_results      per object {cpu_key: rec(c, None), mem_key: rec(m, m)}.
 * Dict keys are the ResourceType members; their hashes are taken once (the enum's __hash__
 * is Python code) and every insertion passes them in (_PyDict_SetItem_KnownHash).
 * Loaded by krr_amd.core.fast_round when present; the pure-Python forms there are equal.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>
#include <string.h>

static PyObject* s_dict;    /* "__dict__" */
static PyObject* s_fields;  /* "__fields_set__" */

static int set_known(PyObject* d, PyObject* k, Py_hash_t h, PyObject* v) {
    return _PyDict_SetItem_KnownHash(d, k, v, h);
}

static uint64_t fnv(const unsigned char* p, Py_ssize_t n) {
    uint64_t h = 1469598103934665603ull;
    for (Py_ssize_t i = 0; i < n; ++i) {
        if (!p[i]) break;
        h = (h ^ p[i]) * 1099511628211ull;
    }
    return h;
}

/* decimal_column(buf, n, width, Decimal, empty, nan) -> list; "NaN" rows become `nan` */
static PyObject* decimal_column(PyObject* self, PyObject* args) {
    (void)self;
    Py_buffer buf;
    Py_ssize_t n, width;
    PyObject *dec_cls, *empty, *nan_obj;
    if (!PyArg_ParseTuple(args, "y*nnOOO", &buf, &n, &width, &dec_cls, &empty, &nan_obj)) return NULL;
    if (n < 0 || width <= 0 || buf.len < n * width) {
        PyBuffer_Release(&buf);
        PyErr_SetString(PyExc_ValueError, "buffer shorter than n * width");
        return NULL;
    }
    const unsigned char* base = (const unsigned char*)buf.buf;
    Py_ssize_t cap = 64;
    while (cap < 2 * n + 16) cap <<= 1;
    Py_ssize_t* slot_idx = PyMem_Malloc(sizeof(Py_ssize_t) * cap);  /* first row of a distinct string */
    PyObject** slot_val = PyMem_Calloc(cap, sizeof(PyObject*));
    PyObject* out = PyList_New(n);
    if (!slot_idx || !slot_val || !out) goto fail;
    for (Py_ssize_t i = 0; i < cap; ++i) slot_idx[i] = -1;
    for (Py_ssize_t i = 0; i < n; ++i) {
        const unsigned char* p = base + i * width;
        Py_ssize_t len = 0;
        while (len < width && p[len]) ++len;
        PyObject* v;
        if (len == 0) {
            v = empty;
        } else {
            Py_ssize_t s = (Py_ssize_t)(fnv(p, len) & (uint64_t)(cap - 1));
            for (;;) {
                if (slot_idx[s] < 0) {
                    PyObject* str = PyUnicode_DecodeASCII((const char*)p, len, NULL);
                    if (!str) goto fail;
                    PyObject* d;
                    if (len == 3 && memcmp(p, "NaN", 3) == 0 && nan_obj != Py_None) {
                        d = nan_obj;
                        Py_INCREF(d);
                    } else {
                        d = PyObject_CallOneArg(dec_cls, str);
                    }
                    Py_DECREF(str);
                    if (!d) goto fail;
                    slot_idx[s] = i;
                    slot_val[s] = d;  /* owned by the table */
                    break;
                }
                const unsigned char* q = base + slot_idx[s] * width;
                if (memcmp(p, q, (size_t)len) == 0 && (len == width || q[len] == 0)) break;
                s = (s + 1) & (cap - 1);
            }
            v = slot_val[s];
        }
        Py_INCREF(v);
        PyList_SET_ITEM(out, i, v);
    }
    for (Py_ssize_t i = 0; i < cap; ++i) Py_XDECREF(slot_val[i]);
    PyMem_Free(slot_idx);
    PyMem_Free(slot_val);
    PyBuffer_Release(&buf);
    return out;
fail:
    if (slot_val)
        for (Py_ssize_t i = 0; i < cap; ++i) Py_XDECREF(slot_val[i]);
    PyMem_Free(slot_idx);
    PyMem_Free(slot_val);
    Py_XDECREF(out);
    PyBuffer_Release(&buf);
    return NULL;
}

static PyObject* new_instance(PyTypeObject* cls) {
    PyObject* empty = PyTuple_New(0);
    if (!empty) return NULL;
    PyObject* o = PyBaseObject_Type.tp_new(cls, empty, NULL);  /* object.__new__(cls) */
    Py_DECREF(empty);
    return o;
}

static PyObject* two_key_dict(PyObject* k1, Py_hash_t h1, PyObject* v1, PyObject* k2, Py_hash_t h2, PyObject* v2) {
    PyObject* d = PyDict_New();
    if (!d) return NULL;
    if (set_known(d, k1, h1, v1) < 0 || set_known(d, k2, h2, v2) < 0) {
        Py_DECREF(d);
        return NULL;
    }
    return d;
}

/* allocations(model, fields_set, cpu_key, mem_key, cpu_list, mem_list) -> list */
static PyObject* allocations(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *model, *fields_set, *ck, *mk, *cl, *ml;
    if (!PyArg_ParseTuple(args, "O!OOOO!O!", &PyType_Type, &model, &fields_set, &ck, &mk, &PyList_Type, &cl,
                          &PyList_Type, &ml))
        return NULL;
    const Py_ssize_t n = PyList_GET_SIZE(cl);
    if (PyList_GET_SIZE(ml) != n) {
        PyErr_SetString(PyExc_ValueError, "cpu and memory columns differ in length");
        return NULL;
    }
    const Py_hash_t hc = PyObject_Hash(ck), hm = PyObject_Hash(mk);
    if (hc == -1 || hm == -1) return NULL;
    PyObject* s_requests = PyUnicode_InternFromString("requests");
    PyObject* s_limits = PyUnicode_InternFromString("limits");
    PyObject* out = NULL;
    if (!s_requests || !s_limits) goto fail;
    const Py_hash_t hreq = PyObject_Hash(s_requests), hlim = PyObject_Hash(s_limits);
    out = PyList_New(n);
    if (!out) goto fail;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* c = PyList_GET_ITEM(cl, i);
        PyObject* m = PyList_GET_ITEM(ml, i);
        PyObject* req = two_key_dict(ck, hc, c, mk, hm, m);
        PyObject* lim = req ? two_key_dict(ck, hc, Py_None, mk, hm, m) : NULL;
        PyObject* fd = lim ? PyDict_New() : NULL;
        /* a fields-set of its own per object: pydantic adds to it on attribute assignment */
        PyObject* fs = fd ? PySet_New(fields_set) : NULL;
        PyObject* o = fs ? new_instance((PyTypeObject*)model) : NULL;
        int bad = !o || set_known(fd, s_requests, hreq, req) < 0 || set_known(fd, s_limits, hlim, lim) < 0 ||
                  PyObject_GenericSetAttr(o, s_dict, fd) < 0 || PyObject_GenericSetAttr(o, s_fields, fs) < 0;
        Py_XDECREF(req);
        Py_XDECREF(lim);
        Py_XDECREF(fd);
        Py_XDECREF(fs);
        if (bad) {
            Py_XDECREF(o);
            goto fail;
        }
        PyList_SET_ITEM(out, i, o);
    }
    Py_DECREF(s_requests);
    Py_DECREF(s_limits);
    return out;
fail:
    Py_XDECREF(out);
    Py_XDECREF(s_requests);
    Py_XDECREF(s_limits);
    return NULL;
}

static PyObject* recommendation(PyTypeObject* rec_cls, PyObject* fields_keys, PyObject* s_request, Py_hash_t hr,
                                PyObject* s_limit, Py_hash_t hl, PyObject* request, PyObject* limit) {
    PyObject* fd = two_key_dict(s_request, hr, request, s_limit, hl, limit);
    if (!fd) return NULL;
    PyObject* fs = PySet_New(fields_keys);
    PyObject* o = fs ? new_instance(rec_cls) : NULL;
    int bad = !o || PyObject_GenericSetAttr(o, s_dict, fd) < 0 || PyObject_GenericSetAttr(o, s_fields, fs) < 0;
    Py_DECREF(fd);
    Py_XDECREF(fs);
    if (bad) {
        Py_XDECREF(o);
        return NULL;
    }
    return o;
}

/* run_results(rec_cls, cpu_key, mem_key, cpu_list, mem_list) -> list of dicts */
static PyObject* run_results(PyObject* self, PyObject* args) {
    (void)self;
    PyObject *rec_cls, *ck, *mk, *cl, *ml;
    if (!PyArg_ParseTuple(args, "O!OOO!O!", &PyType_Type, &rec_cls, &ck, &mk, &PyList_Type, &cl, &PyList_Type, &ml))
        return NULL;
    const Py_ssize_t n = PyList_GET_SIZE(cl);
    if (PyList_GET_SIZE(ml) != n) {
        PyErr_SetString(PyExc_ValueError, "cpu and memory columns differ in length");
        return NULL;
    }
    const Py_hash_t hc = PyObject_Hash(ck), hm = PyObject_Hash(mk);
    if (hc == -1 || hm == -1) return NULL;
    PyObject* s_request = PyUnicode_InternFromString("request");
    PyObject* s_limit = PyUnicode_InternFromString("limit");
    PyObject *keys = NULL, *out = NULL;
    if (!s_request || !s_limit) goto fail;
    keys = PyTuple_Pack(2, s_request, s_limit);
    const Py_hash_t hr = PyObject_Hash(s_request), hl = PyObject_Hash(s_limit);
    out = PyList_New(n);
    if (!out || !keys) goto fail;
    for (Py_ssize_t i = 0; i < n; ++i) {
        PyObject* c = PyList_GET_ITEM(cl, i);
        PyObject* m = PyList_GET_ITEM(ml, i);
        PyObject* rc = recommendation((PyTypeObject*)rec_cls, keys, s_request, hr, s_limit, hl, c, Py_None);
        PyObject* rm = rc ? recommendation((PyTypeObject*)rec_cls, keys, s_request, hr, s_limit, hl, m, m) : NULL;
        PyObject* d = rm ? two_key_dict(ck, hc, rc, mk, hm, rm) : NULL;
        Py_XDECREF(rc);
        Py_XDECREF(rm);
        if (!d) goto fail;
        PyList_SET_ITEM(out, i, d);
    }
    Py_DECREF(s_request);
    Py_DECREF(s_limit);
    Py_DECREF(keys);
    return out;
fail:
    Py_XDECREF(out);
    Py_XDECREF(keys);
    Py_XDECREF(s_request);
    Py_XDECREF(s_limit);
    return NULL;
}

static PyMethodDef methods[] = {
    {"decimal_column", decimal_column, METH_VARARGS, "fixed-width strings -> Decimal list (one per distinct)"},
    {"allocations", allocations, METH_VARARGS, "ResourceAllocations-layout models from value columns"},
    {"run_results", run_results, METH_VARARGS, "RunResult dicts of ResourceRecommendations from value columns"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_krr_pyobj", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__krr_pyobj(void) {
    s_dict = PyUnicode_InternFromString("__dict__");
    s_fields = PyUnicode_InternFromString("__fields_set__");
    if (!s_dict || !s_fields) return NULL;
    return PyModule_Create(&module);
}
