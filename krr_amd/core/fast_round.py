"""Batched exact-decimal post-processing through libkrr_host.so (include/krr_round.h).

The reference computes, per object, the memory proposal ``max * Decimal(1 + b/100)``
(``strategies/simple.py:24-29``) and then ``Runner._format_result``
(``core/runner.py:49-86``) with Python Decimals — ~60 us per object here.
``format_simple_batch`` produces the same rounded RunResults for a whole fleet:
native code does the exact decimal arithmetic for every object and writes
``str(Decimal)`` (digits and exponent of the reference's result); objects it does
not cover (non-finite values, NaN-sample flags, absurd magnitudes) go through the
Python restatement (``krr_amd.core.rounding``), which also raises what the
reference raises.
"""
from __future__ import annotations

import gc
from decimal import Decimal

import numpy as np

from krr_amd.core.abstract.strategies import ResourceRecommendation, RunResult
from krr_amd.core.models.allocations import ResourceType
from krr_amd.core.prom_native import _ptr, load_library
from krr_amd.core.rounding import (
    DEFAULT_CPU_MIN_VALUE,
    DEFAULT_MEMORY_MIN_VALUE,
    resource_minimal,
    round_value,
)

WIDTH = 64
CPU_FALLBACK = 1
MEM_FALLBACK = 2


class _Params:
    def __init__(self, buffer: Decimal, cpu_min: Decimal, mem_min: Decimal):
        import ctypes

        class P(ctypes.Structure):
            _fields_ = [("mem_buffer", ctypes.c_char_p), ("cpu_minimal", ctypes.c_char_p),
                        ("mem_minimal", ctypes.c_char_p)]

        self._strs = [str(buffer).encode(), str(cpu_min).encode(), str(mem_min).encode()]
        self.struct = P(*self._strs)


def round_strings(cpu_value, cpu_flags, mem_value, mem_flags, buffer: Decimal,
                  cpu_min_value: int = DEFAULT_CPU_MIN_VALUE, memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE,
                  threads: int = 0):
    """Columnar form: (cpu strings, memory strings, status) as numpy arrays; str(Decimal)
    of the rounded CPU request and memory request (= limit) per object."""
    import ctypes

    lib = load_library()
    cv = np.ascontiguousarray(cpu_value, dtype=np.float64)
    mv = np.ascontiguousarray(mem_value, dtype=np.float64)
    cf = np.ascontiguousarray(cpu_flags, dtype=np.uint32)
    mf = np.ascontiguousarray(mem_flags, dtype=np.uint32)
    n = int(cv.size)
    cpu_out = np.zeros(max(n, 1), dtype=f"S{WIDTH}")
    mem_out = np.zeros(max(n, 1), dtype=f"S{WIDTH}")
    status = np.zeros(max(n, 1), dtype=np.uint8)
    params = _Params(buffer, resource_minimal(ResourceType.CPU, cpu_min_value, memory_min_value),
                     resource_minimal(ResourceType.Memory, cpu_min_value, memory_min_value))
    rc = lib.krr_round_simple(n, _ptr(cv), _ptr(cf), _ptr(mv), _ptr(mf), ctypes.byref(params.struct),
                              _ptr(cpu_out), _ptr(mem_out), WIDTH, _ptr(status), int(threads))
    if rc != 0:
        raise ValueError("krr_round_simple rejected its arguments")
    return cpu_out[:n], mem_out[:n], status[:n]


def format_simple_batch(raw, settings, cpu_min_value: int = DEFAULT_CPU_MIN_VALUE,
                        memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE, threads: int = 0) -> list[RunResult]:
    """Rounded RunResults (what format_result(SimpleStrategy.results_from_raw(raw)) gives),
    one per object.  ``settings`` is a SimpleStrategySettings (its memory buffer and
    the NaN rules of cpu_from_raw / memory_from_raw apply to the fallback objects)."""
    buffer = settings.memory_buffer()
    cs, ms, st = round_strings(raw.cpu_value, raw.cpu_flags, raw.mem_value, raw.mem_flags, buffer, cpu_min_value,
                               memory_min_value, threads)
    # Decimals are immutable: one object per distinct string (1m / 1M granularity
    # makes fleets highly repetitive).  Each object still gets its own models.
    cache: dict[bytes, Decimal] = {}

    def dec(b: bytes) -> Decimal:
        d = cache.get(b)
        if d is None:
            d = cache[b] = Decimal(b.decode())
        return d

    out: list[RunResult] = []
    cpu_rt, mem_rt = ResourceType.CPU, ResourceType.Memory
    # millions of small acyclic objects: keep the cyclic GC from rescanning them
    gc_was = gc.isenabled()
    gc.disable()
    try:
        _fill(out, st.tolist(), cs, ms, dec, raw, settings, buffer, cpu_min_value, memory_min_value, cpu_rt, mem_rt)
    finally:
        if gc_was:
            gc.enable()
    return out


def _fill(out, status, cs, ms, dec, raw, settings, buffer, cpu_min_value, memory_min_value, cpu_rt, mem_rt):
    for i, s in enumerate(status):
        if s & CPU_FALLBACK:
            cpu = round_value(settings.cpu_from_raw(raw, i), cpu_rt, cpu_min_value, memory_min_value)
        else:
            cpu = dec(cs[i])
        if s & MEM_FALLBACK:
            mem = round_value(settings.memory_from_raw(raw, i, buffer), mem_rt, cpu_min_value, memory_min_value)
        else:
            mem = dec(ms[i])
        out.append({cpu_rt: _recommendation(cpu, None), mem_rt: _recommendation(mem, mem)})


_FIELDS = ("request", "limit")


def _recommendation(request, limit) -> ResourceRecommendation:
    """ResourceRecommendation.construct(request=..., limit=...) without its per-call
    overhead (pydantic v1 construct = __dict__ + __fields_set__, no validation)."""
    m = object.__new__(ResourceRecommendation)
    object.__setattr__(m, "__dict__", {"request": request, "limit": limit})
    object.__setattr__(m, "__fields_set__", set(_FIELDS))
    return m


__all__ = ["format_simple_batch", "round_strings"]
