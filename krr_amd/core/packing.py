"""Fleet packer: every object's history -> one CSR float64 buffer per resource.

The reference builds, per object and resource, ``dict[pod, list[Decimal]]``
(robusta_krr/core/integrations/prometheus.py:147-155) and the strategy flattens
it in dict order (robusta_krr/strategies/simple.py:25, 32).  The packer keeps
exactly that order: segment s = object s's pods in dict (= K8sObjectData.pods)
order, pods without data already dropped by the loader, each pod's samples in
timestamp order.  Nothing is sorted or de-duplicated here.

Two input forms:
  * ``pack_histories``  — the reference's HistoryData (Decimal lists);
  * ``pack_prometheus`` — raw ``custom_query_range`` results (lists of
    ``{"values": [[ts, "str"], ...]}``), parsed straight to float64 with numpy,
    applying the reference's first-series / empty-pod rules (prometheus.py:147-155).
And one alternative layout:
  * ``pack_dense_grid`` — pods aligned on a fixed time grid, absent samples as NaN
    (``gaps_are_nan``), the layout the bench's NaN-gapped config uses.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from decimal import Decimal
from typing import Iterable, Mapping, Optional, Sequence

import numpy as np

from krr_amd.core.models.allocations import ResourceType


@dataclass
class PackedSeries:
    values: np.ndarray        # float64 [N]
    offsets: np.ndarray       # int64 [S+1]
    max_len: int              # max segment length (planning hint for the kernels)
    gaps_are_nan: bool = False
    # HistoryData path only (pack_resource): per segment the exactness class of its Decimals
    # (EXACT_* below; None = every sample came from a Prometheus string: canonical), and for
    # class >= 1 segments the tuple of its pod sample lists, which positions index into
    exact: Optional[np.ndarray] = None
    sources: Optional[list] = None

    @property
    def n_segments(self) -> int:
        return len(self.offsets) - 1  # numpy array, or a torch tensor in HBM (device packer)

    def segment(self, s: int) -> np.ndarray:
        return self.values[self.offsets[s]:self.offsets[s + 1]]


@dataclass
class PackedFleet:
    cpu: PackedSeries
    mem: PackedSeries

    @property
    def n_objects(self) -> int:
        return self.cpu.n_segments


def _from_chunks(chunks: list[np.ndarray], lens: list[int], gaps: bool = False) -> PackedSeries:
    offsets = np.zeros(len(lens) + 1, dtype=np.int64)
    if lens:
        np.cumsum(np.asarray(lens, dtype=np.int64), out=offsets[1:])
    values = np.concatenate(chunks) if chunks else np.zeros(0, dtype=np.float64)
    return PackedSeries(values.astype(np.float64, copy=False), offsets, int(max(lens, default=0)), gaps)


# Exactness class of a HistoryData segment — what its samples' float64 images stand for
# (krr_amd/csrc/krr_pydec.cpp holds the same rule natively):
EXACT_CANONICAL = 0  # every Decimal is prom_decimal(float(d)): the one Prometheus' string gives
EXACT_FAITHFUL = 1   # every VALUE is its float's shortest repr, some representation is not
EXACT_INEXACT = 2    # some sample is not (more digits than float64 holds, non-Decimal, sNaN)


def sample_class(x) -> tuple[float, int]:
    """(float64, exactness class) of one HistoryData sample (the packer's rule)."""
    if type(x) is not Decimal:
        return float(x), EXACT_INEXACT
    if x.is_nan():
        return math.nan, (EXACT_CANONICAL if str(x) == "NaN" else EXACT_INEXACT)
    f = float(x)
    if x.is_infinite():
        return f, EXACT_CANONICAL
    if math.isinf(f):
        return f, EXACT_INEXACT
    shortest = Decimal(repr(f))
    if shortest != x:
        return f, EXACT_INEXACT
    _, digits, exp = x.as_tuple()
    if not any(digits):
        return f, (EXACT_CANONICAL if exp == 0 else EXACT_FAITHFUL)
    tz = len(digits) - len("".join(map(str, digits)).rstrip("0"))
    es = exp + tz
    return f, (EXACT_CANONICAL if (exp == 0 if es >= 0 else tz == 0) else EXACT_FAITHFUL)


def _load_pydec():
    """krr_amd/lib/_krr_pydec.so (krr_amd/csrc/krr_pydec.cpp, built by __graft_entry__.build()):
    the per-sample walk in C++.  None when it is not built: the Python form below is equal."""
    import importlib.machinery
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "_krr_pydec.so")
    if not os.path.exists(path):
        return None
    try:
        loader = importlib.machinery.ExtensionFileLoader("_krr_pydec", path)
        spec = importlib.util.spec_from_file_location("_krr_pydec", path, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        return mod
    except ImportError:  # pragma: no cover - built for another interpreter
        return None


_PYDEC = _load_pydec()


def _pack_resource_py(histories: Sequence[Mapping], resource: ResourceType):
    values: list[float] = []
    lens: list[int] = []
    cls: list[int] = []
    sources: list = []
    for h in histories:
        pods = h.get(resource) or {}
        kept = [samples for samples in pods.values() if len(samples)]
        c = EXACT_CANONICAL
        for samples in kept:
            for x in samples:
                f, k = sample_class(x)
                values.append(f)
                c = max(c, k)
        lens.append(sum(len(s) for s in kept))
        cls.append(c)
        sources.append(tuple(kept) if c else None)
    return np.asarray(values, dtype=np.float64), lens, np.asarray(cls, dtype=np.uint8), sources


def pack_resource(histories: Sequence[Mapping], resource: ResourceType) -> PackedSeries:
    """One segment per history: its pods' samples concatenated in dict order, as float64
    (float(Decimal): correctly rounded, so Prometheus' shortest-repr strings give back the
    exact float the server formatted), plus each segment's exactness class.

    The reference returns the selected sample object itself (simple.py:36 ``data_[k]``,
    :29 ``max(data_)``).  For a CANONICAL segment (every Decimal is what the reference's
    loader parses from Prometheus' string, prometheus.py:152) the host rebuilds that object
    from the kernel's float64 answer (prom_decimal).  Other segments keep their pod lists
    (``sources``) and SimpleStrategy returns the reference's own object at the position the
    GPU located (krr_amd/core/exact.py), e.g. Decimal('0.10') or 25-digit values."""
    if _PYDEC is not None:
        vals, lens_b, cls_b, sources = _PYDEC.pack_resource(histories, resource)
        values = np.frombuffer(vals, dtype=np.float64) if len(vals) else np.zeros(0, dtype=np.float64)
        lens = np.frombuffer(lens_b, dtype=np.int64)
        cls = np.frombuffer(cls_b, dtype=np.uint8).copy()
    else:
        values, lens, cls, sources = _pack_resource_py(histories, resource)
        lens = np.asarray(lens, dtype=np.int64)
    offsets = np.zeros(lens.size + 1, dtype=np.int64)
    np.cumsum(lens, out=offsets[1:])
    exact = cls if cls.any() else None
    return PackedSeries(values, offsets, int(lens.max(initial=0)), False, exact,
                        sources if exact is not None else None)


def pack_histories(histories: Sequence[Mapping]) -> PackedFleet:
    return PackedFleet(pack_resource(histories, ResourceType.CPU), pack_resource(histories, ResourceType.Memory))


def _pod_values(pod_result) -> Optional[np.ndarray]:
    """prometheus.py:150-155: a pod with an empty result is dropped; otherwise only
    its FIRST series is used and timestamps are discarded."""
    if not pod_result:
        return None
    vals = [v for _, v in pod_result[0]["values"]]
    return np.asarray([float(v) for v in vals], dtype=np.float64) if vals else np.zeros(0, np.float64)


def pack_prometheus(per_object_pod_results: Iterable[Sequence]) -> PackedSeries:
    """per_object_pod_results[o][i] = the query_range result for pod i of object o
    (K8sObjectData.pods order), for ONE resource."""
    chunks: list[np.ndarray] = []
    lens: list[int] = []
    for pod_results in per_object_pod_results:
        n = 0
        for pr in pod_results:
            v = _pod_values(pr)
            if v is not None and v.size:
                chunks.append(v)
                n += v.size
        lens.append(n)
    return _from_chunks(chunks, lens)


def pack_dense_grid(per_object_pods: Sequence[Sequence[tuple[np.ndarray, np.ndarray]]], start: float,
                    step: float, slots: int) -> PackedSeries:
    """Time-aligned dense layout: each pod gets ``slots`` slots on the grid
    start + i*step; a pod sample lands in its slot, every other slot is NaN
    (absent).  per_object_pods[o] = [(timestamps, values) per pod].  Because each
    pod keeps its slots in time order and pods stay in order, the present samples
    of a segment are exactly the compact layout's samples, in the same order."""
    chunks: list[np.ndarray] = []
    lens: list[int] = []
    for pods in per_object_pods:
        n = 0
        for ts, vs in pods:
            grid = np.full(slots, np.nan, dtype=np.float64)
            idx = np.rint((np.asarray(ts, dtype=np.float64) - start) / step).astype(np.int64)
            ok = (idx >= 0) & (idx < slots)
            if np.any(np.diff(idx[ok]) <= 0):
                raise ValueError("pod timestamps must be strictly increasing on the grid")
            grid[idx[ok]] = np.asarray(vs, dtype=np.float64)[ok]
            chunks.append(grid)
            n += slots
        lens.append(n)
    return _from_chunks(chunks, lens, gaps=True)
