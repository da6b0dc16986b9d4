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
from typing import Optional

import numpy as np
try:
    import pydantic.v1 as pv1
except ImportError:  # a process that aliased pydantic -> pydantic.v1 (the reference's import recipe)
    import pydantic as pv1

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


def _load_pyobj():
    """krr_amd/lib/_krr_pyobj.so (krr_amd/csrc/krr_pyobj.c, built by __graft_entry__.build()):
    the per-object construction loops in C.  None when it is not built: the Python forms below
    build the same objects."""
    import importlib.machinery
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "_krr_pyobj.so")
    if not os.path.exists(path):
        return None
    try:
        loader = importlib.machinery.ExtensionFileLoader("_krr_pyobj", path)
        spec = importlib.util.spec_from_file_location("_krr_pyobj", path, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        return mod
    except ImportError:  # pragma: no cover - built for another interpreter
        return None


_PYOBJ = _load_pyobj()


class _Params:
    def __init__(self, buffer: Decimal, cpu_min: Decimal, mem_min: Decimal, fast_path: bool = True):
        import ctypes

        class P(ctypes.Structure):
            _fields_ = [("mem_buffer", ctypes.c_char_p), ("cpu_minimal", ctypes.c_char_p),
                        ("mem_minimal", ctypes.c_char_p), ("fast_path", ctypes.c_int32),
                        ("reserved", ctypes.c_int32)]

        self._strs = [str(buffer).encode(), str(cpu_min).encode(), str(mem_min).encode()]
        self.struct = P(*self._strs, int(bool(fast_path)), 0)


def round_strings(cpu_value, cpu_flags, mem_value, mem_flags, buffer: Decimal,
                  cpu_min_value: int = DEFAULT_CPU_MIN_VALUE, memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE,
                  threads: int = 0, fast_path: bool = True):
    """Columnar form: (cpu strings, memory strings, status) as numpy arrays; str(Decimal)
    of the rounded CPU request and memory request (= limit) per object.  ``fast_path``: the
    native code's 128-bit integer arithmetic where the operands fit (False: its digit-string
    arithmetic throughout; the results are the same)."""
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
                     resource_minimal(ResourceType.Memory, cpu_min_value, memory_min_value), fast_path)
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
    _route_exact(st, raw)
    # Decimals are immutable: one object per distinct string (1m / 1M granularity makes
    # fleets highly repetitive), found by a sort of the string columns, not per object.
    # Each object still gets its own models.
    cpu_col, mem_col = decimal_column(cs), decimal_column(ms)
    out: list[RunResult] = []
    cpu_rt, mem_rt = ResourceType.CPU, ResourceType.Memory
    # millions of small acyclic objects: keep the cyclic GC from rescanning them
    gc_was = gc.isenabled()
    gc.disable()
    try:
        _apply_fallbacks(cpu_col, mem_col, st, raw, settings, buffer, cpu_min_value, memory_min_value)
        if _PYOBJ is not None:
            out = _PYOBJ.run_results(ResourceRecommendation, cpu_rt, mem_rt, cpu_col, mem_col)
        else:
            rec = _recommendation
            out = [{cpu_rt: rec(c, None), mem_rt: rec(m, m)} for c, m in zip(cpu_col, mem_col)]
    finally:
        if gc_was:
            gc.enable()
    return out


def decimal_column(strings: np.ndarray, nan=None) -> list:
    """Decimal(s) for every string of a numpy bytes column, as a list: one Decimal object per
    distinct string (Decimal() runs once per distinct value); rows "NaN" become ``nan`` when
    given (e.g. the "?" ResourceAllocations shows), empty rows (fallback objects) None."""
    n = int(strings.size)
    if n == 0:
        return []
    if _PYOBJ is not None:
        col = np.ascontiguousarray(strings)
        return _PYOBJ.decimal_column(col.view(np.uint8).reshape(-1), n, col.dtype.itemsize, Decimal, None, nan)
    uniq, inv = np.unique(strings, return_inverse=True)
    decs = np.empty(uniq.size, dtype=object)
    decs[:] = [(nan if (nan is not None and u == b"NaN") else Decimal(u.decode())) if u else None
               for u in uniq.tolist()]  # '': a fallback object
    return decs[inv.reshape(-1)].tolist()


def _route_exact(status, raw) -> None:
    """Objects whose answer is the reference's own sample object (krr_amd.core.exact: HistoryData
    Decimals the float64 values do not reproduce) take the Python rounding of that object."""
    for name, bit in (("cpu_exact", CPU_FALLBACK), ("mem_exact", MEM_FALLBACK)):
        ex = getattr(raw, name, None)
        if ex:
            idx = np.fromiter(ex.keys(), dtype=np.int64, count=len(ex))
            status[idx] |= bit


def _apply_fallbacks(cpu_col, mem_col, status, raw, settings, buffer, cpu_min_value, memory_min_value) -> None:
    """The objects the native rounding did not cover, through the Python restatement (which
    raises what the reference raises)."""
    cpu_rt, mem_rt = ResourceType.CPU, ResourceType.Memory
    for i in np.nonzero(status)[0].tolist():
        s = int(status[i])
        if s & CPU_FALLBACK:
            cpu_col[i] = round_value(settings.cpu_from_raw(raw, i), cpu_rt, cpu_min_value, memory_min_value)
        if s & MEM_FALLBACK:
            mem_col[i] = round_value(settings.memory_from_raw(raw, i, buffer), mem_rt, cpu_min_value,
                                     memory_min_value)


def allocations_batch(raw, settings, cpu_min_value: int = DEFAULT_CPU_MIN_VALUE,
                      memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE, threads: int = 0, model=None,
                      resource_type=None, timings: Optional[dict] = None) -> list:
    """Runner._gather_objects_recommendations's list (runner.py:113-120) straight from raw kernel
    results: one ``ResourceAllocations`` per object, equal to
    ``ResourceAllocations(requests={rt: r[rt].request ...}, limits={rt: r[rt].limit ...})`` of the
    rounded RunResult r, built in bulk.  The values are what the model's validator would leave
    (allocations.py:33-51: Decimal unchanged, NaN -> "?", the CPU limit None), so each model is
    made without a per-object validation walk (pydantic v1 ``construct``'s layout: the field
    dict and the fields-set).  ``model`` / ``resource_type``: the reference's own classes
    (krr_amd.integration) or, by default, this package's mirror.  ``timings``: filled with the
    phases' seconds (round_s: native rounding, decimal_s: one Decimal per distinct string,
    models_s: the models)."""
    from krr_amd.core.models.allocations import ResourceAllocations

    model = model or ResourceAllocations
    rtypes = list(resource_type or ResourceType)
    cpu_k, mem_k = rtypes[0], rtypes[1]
    import time

    gc_was = gc.isenabled()
    gc.disable()
    try:
        cpu_col, mem_col = rounded_columns(raw, settings, cpu_min_value, memory_min_value, threads, timings)
        t1 = time.perf_counter()
        fields = {"requests", "limits"}
        if not _v1_construct_layout(model):  # e.g. a pydantic v2 model: its own constructor, per object
            return [model(requests={cpu_k: c, mem_k: m}, limits={cpu_k: None, mem_k: m})
                    for c, m in zip(cpu_col, mem_col)]
        from krr_amd.core.packing import _PYDEC

        if _PYDEC is not None and tuple(model.__fields__) == ("requests", "limits"):
            out = _PYDEC.allocations(_model_desc(model), (cpu_k, mem_k), cpu_col, mem_col)
            if timings is not None:
                timings["models_s"] = time.perf_counter() - t1
            return out
        if _PYOBJ is not None:
            return _PYOBJ.allocations(model, fields, cpu_k, mem_k, cpu_col, mem_col)
        new, setattr_ = object.__new__, object.__setattr__

        def mk(c, m):
            o = new(model)
            setattr_(o, "__dict__", {"requests": {cpu_k: c, mem_k: m}, "limits": {cpu_k: None, mem_k: m}})
            setattr_(o, "__fields_set__", set(fields))  # its own: pydantic adds to it on assignment
            return o

        return list(map(mk, cpu_col, mem_col))
    finally:
        if gc_was:
            gc.enable()


def rounded_columns(raw, settings, cpu_min_value: int = DEFAULT_CPU_MIN_VALUE,
                    memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE, threads: int = 0,
                    timings: Optional[dict] = None) -> tuple[list, list]:
    """The rounded CPU request and memory request / limit of every object as the
    ResourceAllocations validator leaves them (a Decimal, or "?" for NaN; allocations.py:33-51):
    Runner._format_result's values (runner.py:49-86) from raw kernel results, by the native
    rounding, with the reference's own arithmetic for what it does not cover.  ``timings``:
    round_s (native rounding), decimal_s (one Decimal per distinct string)."""
    import time

    t0 = time.perf_counter()
    buffer = settings.memory_buffer()
    cs, ms, st = round_strings(raw.cpu_value, raw.cpu_flags, raw.mem_value, raw.mem_flags, buffer, cpu_min_value,
                               memory_min_value, threads)
    _route_exact(st, raw)
    t1 = time.perf_counter()
    q = "?"
    cpu_col, mem_col = decimal_column(cs, q), decimal_column(ms, q)
    if timings is not None:
        timings.update(round_s=t1 - t0, decimal_s=time.perf_counter() - t1)
    fb = np.nonzero(st)[0].tolist()
    _apply_fallbacks(cpu_col, mem_col, st, raw, settings, buffer, cpu_min_value, memory_min_value)
    for i in fb:  # the validator's NaN -> "?" (allocations.py:40-41) for the Python-rounded ones
        if isinstance(cpu_col[i], Decimal) and cpu_col[i].is_nan():
            cpu_col[i] = q
        if isinstance(mem_col[i], Decimal) and mem_col[i].is_nan():
            mem_col[i] = q
    return cpu_col, mem_col


def result_batch(objects, raw, settings, cpu_min_value: int = DEFAULT_CPU_MIN_VALUE,
                 memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE, threads: int = 0, models=None,
                 timings: Optional[dict] = None):
    """Runner._collect_result (runner.py:122-131) from raw kernel results: the rounded values
    (rounded_columns) scanned straight into the Result — ResourceScan.calculate per object and
    the score (result.py:33-150) — without the ResourceAllocations list in between, which the
    reference builds only for the scan to read (runner.py:113-120).  Equal to
    collect_result(objects, allocations_batch(raw, ...)).  ``models``: the reference's result
    module (krr_amd.integration) or, by default, this package's mirror.  ``timings``: as
    rounded_columns, plus scan_s."""
    import time

    from krr_amd.core.models.result import collect_result_columns

    gc_was = gc.isenabled()
    gc.disable()
    try:
        cpu_col, mem_col = rounded_columns(raw, settings, cpu_min_value, memory_min_value, threads, timings)
        t0 = time.perf_counter()
        res = collect_result_columns(objects, cpu_col, mem_col, models)
        if timings is not None:
            timings["scan_s"] = time.perf_counter() - t0
        return res
    finally:
        if gc_was:
            gc.enable()


def _model_desc(model) -> tuple:
    """(class, field names, fields-set, __fields_set__ slot offset): how the native builders
    (krr_amd/csrc/krr_pydec.cpp) make pydantic-v1 instances in construct() layout.  Every
    instance of the class shares the one fields-set: it holds every field, so the add()
    pydantic's __setattr__ does never changes it (_v1_construct_layout admits only models
    that forbid other names), as pydantic itself shares one between a model and its
    validation copy (pydantic/v1/main.py _copy_and_set_values)."""
    from krr_amd.core.packing import _PYDEC

    names = tuple(model.__fields__)
    return (model, names, set(names), _PYDEC.slot_offset(pv1.BaseModel.__dict__["__fields_set__"]))


def _v1_construct_layout(model) -> bool:
    """True when instances of ``model`` are exactly pydantic v1's construct() layout (the field
    dict + __fields_set__): a pydantic.v1 BaseModel without private attributes, as the
    reference's models are (pydantic 1.10).  Anything else is built by its own constructor."""
    return (isinstance(model, type) and issubclass(model, pv1.BaseModel)
            and not getattr(model, "__private_attributes__", None)
            and model.__config__.extra is not pv1.Extra.allow)


_FIELDS = ("request", "limit")


def _recommendation(request, limit) -> ResourceRecommendation:
    """ResourceRecommendation.construct(request=..., limit=...) without its per-call
    overhead (pydantic v1 construct = __dict__ + __fields_set__, no validation)."""
    m = object.__new__(ResourceRecommendation)
    object.__setattr__(m, "__dict__", {"request": request, "limit": limit})
    object.__setattr__(m, "__fields_set__", set(_FIELDS))
    return m


__all__ = ["allocations_batch", "decimal_column", "format_simple_batch", "round_strings"]
