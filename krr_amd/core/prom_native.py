"""ctypes front-end of libkrr_host.so's packer: Prometheus query_range response bodies ->
CSR float64 (include/krr_pack.h).

The reference turns every pod's ``custom_query_range`` result into
``[Decimal(value) for _, value in pod_result[0]["values"]]`` and drops pods whose
result is empty (``core/integrations/prometheus.py:147-155``), one object and one
pod at a time in Python.  ``pack_query_range_bodies`` does the same for a whole
fleet's raw HTTP bodies at once, in parallel native code, and returns the packed
layout the kernels read (``krr_amd.core.packing.PackedSeries``).  Host-only: no
HIP, no torch.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional, Sequence

import numpy as np

from krr_amd.core.packing import PackedSeries

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("KRR_HOST_LIB", os.path.join(_HERE, "lib", "libkrr_host.so"))

KRR_PACK_OK = 0
KRR_PACK_E_INVALID = -1
KRR_PACK_E_PARSE = -2
KRR_PACK_E_STATUS = -3
KRR_PACK_E_VALUE = -4

EXPORTED_SYMBOLS = ("krr_pack_abi_version", "krr_pack_parse", "krr_pack_n_values", "krr_pack_max_len",
                    "krr_pack_copy", "krr_pack_error", "krr_pack_free", "krr_pack_parse_series", "krr_series_count",
                    "krr_series_label", "krr_series_len", "krr_series_copy", "krr_series_error", "krr_series_free",
                    "krr_pack_parse_grouped", "krr_round_simple", "krr_pack_concat", "krr_pack_route_grouped",
                    "krr_pack_concat_strip", "krr_pack_strip_body", "krr_pack_route_grouped_pieces",
                    "krr_pack_concat_strip_pieces")


class PackerUnavailable(RuntimeError):
    """libkrr_host.so is missing or does not load."""


class PrometheusResponseError(ValueError):
    """A response body is not a successful query_range result (the reference's
    prometheus_api_client / json would raise here too)."""

    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code


_lib = None
_lock = threading.Lock()


def load_library() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise PackerUnavailable(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; "
                                    f"g.build()'`")
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover
            raise PackerUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        lib.krr_pack_abi_version.argtypes = []
        lib.krr_pack_abi_version.restype = ctypes.c_int
        lib.krr_pack_parse.argtypes = [vp, vp, i64, vp, i64, i32, i32, ctypes.POINTER(vp)]
        lib.krr_pack_parse.restype = ctypes.c_int
        lib.krr_pack_n_values.argtypes = [vp]
        lib.krr_pack_n_values.restype = i64
        lib.krr_pack_max_len.argtypes = [vp]
        lib.krr_pack_max_len.restype = i64
        lib.krr_pack_copy.argtypes = [vp, vp, vp, vp, vp, i32]
        lib.krr_pack_copy.restype = ctypes.c_int
        lib.krr_pack_error.argtypes = [vp]
        lib.krr_pack_error.restype = ctypes.c_char_p
        lib.krr_pack_free.argtypes = [vp]
        lib.krr_pack_free.restype = None
        lib.krr_pack_parse_series.argtypes = [ctypes.c_char_p, i64, ctypes.c_char_p, i32, ctypes.POINTER(vp)]
        lib.krr_pack_parse_series.restype = ctypes.c_int
        lib.krr_series_count.argtypes = [vp]
        lib.krr_series_count.restype = i64
        lib.krr_series_label.argtypes = [vp, i64, ctypes.POINTER(i64)]
        lib.krr_series_label.restype = ctypes.c_void_p
        lib.krr_series_len.argtypes = [vp, i64]
        lib.krr_series_len.restype = i64
        lib.krr_series_copy.argtypes = [vp, i64, vp, vp]
        lib.krr_series_copy.restype = ctypes.c_int
        lib.krr_series_error.argtypes = [vp]
        lib.krr_series_error.restype = ctypes.c_char_p
        lib.krr_series_free.argtypes = [vp]
        lib.krr_series_free.restype = None
        lib.krr_pack_parse_grouped.argtypes = [vp, vp, i64, ctypes.c_char_p, vp, ctypes.c_char_p, vp, vp, i64, i64,
                                               i32, i32, ctypes.POINTER(vp)]
        lib.krr_pack_parse_grouped.restype = ctypes.c_int
        lib.krr_round_simple.argtypes = [i64, vp, vp, vp, vp, vp, vp, vp, i32, vp, i32]
        lib.krr_round_simple.restype = ctypes.c_int
        lib.krr_pack_concat.argtypes = [vp, vp, i64, vp, vp, i32]
        lib.krr_pack_concat.restype = ctypes.c_int
        lib.krr_pack_concat_strip.argtypes = [vp, vp, i64, vp, vp, i32, i32, vp, vp, ctypes.POINTER(i32)]
        lib.krr_pack_concat_strip.restype = ctypes.c_int
        lib.krr_pack_strip_body.argtypes = [ctypes.c_char_p, i64, vp]
        lib.krr_pack_strip_body.restype = i64
        lib.krr_pack_route_grouped.argtypes = [vp, vp, i64, ctypes.c_char_p, vp, i64, vp, ctypes.c_char_p, vp, i64,
                                               vp, vp, vp, i32]
        lib.krr_pack_route_grouped.restype = ctypes.c_int
        lib.krr_pack_route_grouped_pieces.argtypes = [vp, vp, i64, vp, vp, i64, ctypes.c_char_p, vp, i64, vp,
                                                      ctypes.c_char_p, vp, i64, vp, vp, vp, i32]
        lib.krr_pack_route_grouped_pieces.restype = ctypes.c_int
        lib.krr_pack_concat_strip_pieces.argtypes = [vp, vp, i64, vp, vp, i32, i32, vp, vp, vp, ctypes.POINTER(i32)]
        lib.krr_pack_concat_strip_pieces.restype = ctypes.c_int
        if lib.krr_pack_abi_version() != 1:
            raise PackerUnavailable("libkrr_host.so packer ABI version mismatch")
        _lib = lib
        return lib


def strip_body(body: bytes) -> Optional[bytes]:
    """``body`` with every number outside strings cut to its first digit (the device
    packer's staging form, krr_amd/csrc/krr_strip.h), or None when it is not strippable."""
    lib = load_library()
    out = ctypes.create_string_buffer(max(len(body), 1))
    n = lib.krr_pack_strip_body(body, len(body), ctypes.addressof(out))
    return None if n < 0 else out.raw[:n]


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def parse_series(body: bytes, label: str = "pod", *, want_timestamps: bool = False) -> list:
    """Every series of one query_range response body: [(label value or None,
    values float64[, timestamps float64])] in response order."""
    lib = load_library()
    body = body if isinstance(body, (bytes, bytearray)) else bytes(body)
    h = ctypes.c_void_p()
    rc = lib.krr_pack_parse_series(bytes(body), len(body), label.encode(), int(bool(want_timestamps)),
                                   ctypes.byref(h))
    try:
        if rc != KRR_PACK_OK:
            msg = lib.krr_series_error(h) if h else b""
            raise PrometheusResponseError(rc, (msg or b"invalid arguments").decode())
        out = []
        for i in range(int(lib.krr_series_count(h))):
            ln = ctypes.c_int64()
            ptr = lib.krr_series_label(h, i, ctypes.byref(ln))
            name = ctypes.string_at(ptr, ln.value).decode() if ln.value >= 0 else None
            v = np.empty(int(lib.krr_series_len(h, i)), dtype=np.float64)
            t = np.empty_like(v) if want_timestamps else None
            if lib.krr_series_copy(h, i, _ptr(v), _ptr(t) if t is not None else None) != KRR_PACK_OK:
                raise PrometheusResponseError(KRR_PACK_E_INVALID, "krr_series_copy failed")
            out.append((name, v, t) if want_timestamps else (name, v))
        return out
    finally:
        if h:
            lib.krr_series_free(h)


def pack_query_range_bodies(per_object_bodies: Sequence[Sequence[bytes]], *, want_timestamps: bool = False,
                            threads: int = 0, return_pod_counts: bool = False, alloc=None):
    """per_object_bodies[o][i] = the raw /api/v1/query_range response body (bytes)
    for pod i of object o (K8sObjectData.pods order), for ONE resource.

    Returns a PackedSeries (segment o = object o's kept pods concatenated), plus
    the timestamps (float64 seconds, same layout) if ``want_timestamps`` and the
    per-pod sample counts (-1 = dropped: empty result) if ``return_pod_counts``.
    Raises PrometheusResponseError naming the first bad body.  ``alloc(n)`` (optional)
    returns the float64 array the samples are written into — e.g.
    ``krr_amd.core.engine.pinned_alloc`` for page-locked memory the H2D copy reads
    by DMA at full PCIe rate.
    """
    lib = load_library()
    flat: list[bytes] = []
    obj: list[int] = []
    for o, bodies in enumerate(per_object_bodies):
        for b in bodies:
            flat.append(b if isinstance(b, bytes) else bytes(b))  # c_char_p takes bytes only
            obj.append(o)
    n_obj = len(per_object_bodies)
    nb = len(flat)
    ptrs = (ctypes.c_char_p * max(nb, 1))(*flat) if nb else (ctypes.c_char_p * 1)()
    lens = np.array([len(b) for b in flat] or [0], dtype=np.int64)
    obj_a = np.array(obj or [0], dtype=np.int64)
    h = ctypes.c_void_p()
    rc = lib.krr_pack_parse(ctypes.cast(ptrs, ctypes.c_void_p), _ptr(lens), nb, _ptr(obj_a), n_obj,
                            int(bool(want_timestamps)), int(threads), ctypes.byref(h))
    try:
        if rc != KRR_PACK_OK:
            msg = lib.krr_pack_error(h) if h else b""
            raise PrometheusResponseError(rc, (msg or b"invalid arguments").decode())
        n = int(lib.krr_pack_n_values(h))
        values = alloc(n) if alloc is not None else np.empty(n, dtype=np.float64)
        offsets = np.empty(n_obj + 1, dtype=np.int64)
        ts = np.empty(n, dtype=np.float64) if want_timestamps else None
        counts = np.empty(max(nb, 1), dtype=np.int64) if return_pod_counts else None
        rc = lib.krr_pack_copy(h, _ptr(values), _ptr(offsets), _ptr(ts) if ts is not None else None,
                               _ptr(counts) if counts is not None else None, int(threads))
        if rc != KRR_PACK_OK:
            raise PrometheusResponseError(rc, "krr_pack_copy failed")
        max_len = int(lib.krr_pack_max_len(h))
    finally:
        if h:
            lib.krr_pack_free(h)
    series = PackedSeries(values, offsets, max_len)
    out: list = [series]
    if want_timestamps:
        out.append(ts)
    if return_pod_counts:
        out.append(counts[:nb])
    return out[0] if len(out) == 1 else tuple(out)
