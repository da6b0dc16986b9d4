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


def _decimals_to_f64(xs: Sequence[Decimal]) -> np.ndarray:
    # float(Decimal) is correctly rounded; for Prometheus' shortest-repr strings it
    # recovers the exact float64 the server formatted.
    #
    # Contract of the HistoryData path: every Decimal is what the reference's loader
    # builds, Decimal(<Prometheus sample string>) (prometheus.py:152), and Prometheus
    # formats samples with Go's strconv.FormatFloat(v, 'f', -1, 64) — the shortest
    # string that round-trips — so prom_decimal(float(d)) == d.  A hand-made Decimal
    # with more significant digits than a float64 holds (e.g. 100000000.0000000000000001)
    # or a non-canonical form ('0.10') is NOT reproduced: the kernel selects float64
    # values and the host rebuilds the Decimal from the float's shortest repr.
    return np.fromiter((float(x) for x in xs), dtype=np.float64, count=len(xs))


def pack_resource(histories: Sequence[Mapping], resource: ResourceType) -> PackedSeries:
    """One segment per history: its pods' samples concatenated in dict order."""
    chunks: list[np.ndarray] = []
    lens: list[int] = []
    for h in histories:
        pods = h.get(resource) or {}
        n = 0
        for samples in pods.values():
            if len(samples):
                chunks.append(_decimals_to_f64(samples))
                n += len(samples)
        lens.append(n)
    return _from_chunks(chunks, lens)


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
