"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the CPU oracle (krr_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline.  The product path
(krr_amd/) never imports it.

Parity status: pinned against golden vectors generated from the reference
(tests/golden/make_golden.py); see krr_oracle.c for the restated semantics.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

REF_INDEX, SORTED_LOWER, LINEAR = 0, 1, 2
FLAG_NAN, FLAG_EMPTY = 1, 4


def build() -> str:
    """Compile the oracle (gcc, OpenMP) into oracle/build/liboracle.so."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        lib = ctypes.CDLL(_LIB)
        d, i64, u32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        lib.oracle_percentile.argtypes = [d, d, i64, u32, u32, i64, i64, ctypes.c_double, d, d, d, u32]
        lib.oracle_percentile.restype = ctypes.c_int
        lib.oracle_max.argtypes = [d, d, i64, u32, d, d, d, u32]
        lib.oracle_max.restype = ctypes.c_int
        lib.oracle_percentile_ktab.argtypes = [d, d, i64, ctypes.c_int, ctypes.c_int, i64, i64, d, i64,
                                               ctypes.c_double, d, d, d, ctypes.c_int]
        lib.oracle_percentile_ktab.restype = ctypes.c_int
        lib.oracle_exact_rank.argtypes = [i64, i64, i64]
        lib.oracle_exact_rank.restype = i64
        _lib = lib
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def percentile(values: np.ndarray, offsets: np.ndarray, mode: int, p_num: int, p_den: int,
               q: float, gaps: bool = False, nthreads: int = 0, k_table: np.ndarray = None):
    """Per-segment CPU proposal: returns (value f64[S], count i64[S], flags u32[S]).
    k_table (optional int64, longer than every segment): k(n) = k_table[n] instead of the
    exact floor of p_num / p_den (the reference's rounded index rule for long p)."""
    lib = _load()
    values = np.ascontiguousarray(values, dtype=np.float64)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    S = offsets.size - 1
    ov = np.empty(S, np.float64)
    on = np.empty(S, np.int64)
    of = np.empty(S, np.uint32)
    if k_table is not None:
        kt = np.ascontiguousarray(k_table, dtype=np.int64)
        rc = lib.oracle_percentile_ktab(_ptr(values), _ptr(offsets), S, mode, int(bool(gaps)), p_num, p_den,
                                        _ptr(kt), kt.size, q, _ptr(ov), _ptr(on), _ptr(of), nthreads)
    else:
        rc = lib.oracle_percentile(_ptr(values), _ptr(offsets), S, mode, int(bool(gaps)), p_num, p_den,
                                   q, _ptr(ov), _ptr(on), _ptr(of), nthreads)
    if rc != 0:
        raise RuntimeError(f"oracle_percentile failed: {rc}")
    return ov, on, of


def seg_max(values: np.ndarray, offsets: np.ndarray, gaps: bool = False, nthreads: int = 0):
    """Per-segment Python-max() restatement: returns (value, count, flags)."""
    lib = _load()
    values = np.ascontiguousarray(values, dtype=np.float64)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    S = offsets.size - 1
    ov = np.empty(S, np.float64)
    on = np.empty(S, np.int64)
    of = np.empty(S, np.uint32)
    lib.oracle_max(_ptr(values), _ptr(offsets), S, int(bool(gaps)), _ptr(ov), _ptr(on), _ptr(of), nthreads)
    return ov, on, of


def exact_rank(n: int, p_num: int, p_den: int) -> int:
    return int(_load().oracle_exact_rank(n, p_num, p_den))


def locate(values: np.ndarray, offsets: np.ndarray, v: np.ndarray, rank: np.ndarray):
    """krr_locate restated (include/krr_amd.h): per segment with rank >= -1, lt = #x < v,
    eq = #x == v, pos = offset of the j-th x == v (j = rank - lt, or 0 for rank -1), -1
    if none; other segments -1 everywhere.  Plain numpy, for the CPU stand-in tests."""
    S = offsets.size - 1
    lt, eq, pos = (np.full(S, -1, dtype=np.int64) for _ in range(3))
    for s in range(S):
        if rank[s] < -1:
            continue
        seg = values[offsets[s]:offsets[s + 1]]
        lt[s] = int(np.count_nonzero(seg < v[s]))
        hits = np.flatnonzero(seg == v[s])
        eq[s] = hits.size
        j = int(rank[s]) - int(lt[s]) if rank[s] >= 0 else 0
        pos[s] = int(hits[j]) if 0 <= j < hits.size else -1
    return lt, eq, pos
