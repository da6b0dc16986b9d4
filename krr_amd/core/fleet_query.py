"""Fleet-level PromQL batching: one range query per
(namespace, container) group instead of one per pod, demultiplexed natively.

The reference issues ``sum(<metric>{namespace="ns", pod="p", container="c"})``
once per pod, per object, per resource (``PrometheusLoader.gather_data``,
``robusta_krr/core/integrations/prometheus.py:118-143``) — for a 10k-pod fleet
that is 20k HTTP round trips, each returning one series.  Here the pods of every
object that share a (namespace, container) pair go into one

    sum by (pod) (<metric>{<same matchers>, namespace="ns", pod=~"p1|p2|...", container="c"})

query, split when the pod regex grows past ``max_query_chars`` or the group's
expected samples (pods x ``series_per_pod`` x points per series) would pass
``max_query_samples`` — Prometheus refuses a query that loads more than its
``--query.max-samples`` (default 50,000,000) [external], where the per-pod queries
it replaces would each pass.  ``sum by (pod)``
evaluated over the same start/end/step yields, for every pod, exactly the series
the per-pod ``sum(...{pod="p"})`` yields (same matchers, same aggregation inputs,
same evaluation timestamps); a pod with no samples is absent from the grouped
result just as its per-pod result list is empty, and is dropped the same way
(prometheus.py:154).  ``krr_pack_parse_grouped`` (include/krr_pack.h) parses all
grouped bodies in parallel and routes each series by its ``pod`` label into the
fleet's (object, pod) order, producing the same CSR layout
``pack_query_range_bodies`` produces from per-pod bodies — bit-identical values
and offsets (tests/test_fleet_query.py).

Host-only: no HIP, no torch.  ``FleetQueryPlan.fetch`` takes any callable that
performs one query_range HTTP request and returns its raw body, so the plan works
with the reference's ``PrometheusConnect`` session or a test double.
"""
from __future__ import annotations

import ctypes
import datetime
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import Callable, Sequence

import numpy as np

from krr_amd.core.models.allocations import ResourceType
from krr_amd.core.packing import PackedFleet, PackedSeries
from krr_amd.core.prom_native import KRR_PACK_OK, PrometheusResponseError, _ptr, load_library

# The reference's selectors (prometheus.py:123 and :137), without the pod/ns/container matchers.
CPU_METRIC = "node_namespace_pod_container:container_cpu_usage_seconds_total:sum_irate"
CPU_MATCHERS = ""
MEMORY_METRIC = "container_memory_working_set_bytes"
MEMORY_MATCHERS = 'job="kubelet", metrics_path="/metrics/cadvisor", image!="", '

_METRIC = {ResourceType.CPU: (CPU_METRIC, CPU_MATCHERS), ResourceType.Memory: (MEMORY_METRIC, MEMORY_MATCHERS)}

# RE2 metacharacters (Prometheus' =~ is a fully anchored RE2 match).
_RE2_META = set("\\.+*?()|[]{}^$")


def step_string(timeframe: datetime.timedelta) -> str:
    """The reference's step argument (prometheus.py:126)."""
    return f"{int(timeframe.total_seconds()) // 60}m"


def pod_query(resource: ResourceType, namespace: str, pod: str, container: str) -> str:
    """The reference's per-pod query, character for character (prometheus.py:123, :137)."""
    metric, matchers = _resolve(resource)
    return f'sum({metric}{{{matchers}namespace="{namespace}", pod="{pod}", container="{container}"}})'


def pod_regex(pods: Sequence[str]) -> str:
    """RE2 alternation matching exactly ``pods``, as it appears inside a PromQL
    double-quoted string (every regex backslash doubled)."""
    parts = []
    for p in pods:
        esc = "".join("\\\\" + c if c in _RE2_META else c for c in p)
        parts.append(esc.replace('"', '\\"'))
    return "|".join(parts)


def group_query(resource: ResourceType, namespace: str, container: str, pods: Sequence[str]) -> str:
    metric, matchers = _resolve(resource)
    return (f'sum by (pod) ({metric}{{{matchers}namespace="{namespace}", pod=~"{pod_regex(pods)}", '
            f'container="{container}"}})')


def _resolve(resource) -> tuple[str, str]:
    try:
        return _METRIC[ResourceType(resource)]
    except (KeyError, ValueError):
        raise ValueError(f"Unknown resource type: {resource}") from None


@dataclass
class GroupQuery:
    """One grouped range query: the pods of one (namespace, container) it covers."""
    namespace: str
    container: str
    pods: list[str]

    def query(self, resource: ResourceType) -> str:
        return group_query(resource, self.namespace, self.container, self.pods)


# history_duration 336 h / timeframe_duration 15 min + 1 (SimpleStrategySettings defaults,
# robusta_krr/core/abstract/strategies.py:20-23; range query prometheus.py:124-126)
DEFAULT_POINTS_PER_SERIES = 336 * 60 // 15 + 1


@dataclass
class FleetQueryPlan:
    """Grouping of a fleet's (object, pod) pairs into grouped range queries.

    ``objects`` are K8sObjectData (anything with ``namespace``, ``container`` and
    ``pods``); their order is the fleet order of the packed segments.  Each
    object's pods are de-duplicated keeping first occurrence, as the reference's
    ``{pod: result[i] for i, pod in enumerate(object.pods)}`` does
    (prometheus.py:152).  A pod shared by several objects of the same group is
    queried once and routed to each of them.
    """
    objects: Sequence
    max_query_chars: int = 6000
    # evaluation timestamps per series.  Default: the reference's default settings (336 h
    # at 15 min: 1,345 points), so a plan built without settings still respects Prometheus'
    # sample limit; ``for_settings`` takes them from the strategy; 0 turns the bound off.
    points_per_series: int = DEFAULT_POINTS_PER_SERIES
    max_query_samples: int = 50_000_000  # Prometheus' default --query.max-samples [external]
    series_per_pod: int = 4              # raw series the selector may match per pod (restarts, ids)
    groups: list[GroupQuery] = field(init=False)
    slot_obj: np.ndarray = field(init=False)      # int64 [n_slots], non-decreasing
    slot_group: np.ndarray = field(init=False)    # int64 [n_slots]
    slot_pods: list[str] = field(init=False)

    def __post_init__(self):
        if self.max_query_chars < 1:
            raise ValueError("max_query_chars must be positive")
        if self.points_per_series < 0 or self.max_query_samples < 1 or self.series_per_pod < 1:
            raise ValueError("points_per_series must be >= 0, max_query_samples and series_per_pod positive")
        # pods one grouped query may hold under the sample bound (at least one)
        per_pod = self.points_per_series * self.series_per_pod
        max_pods = max(1, self.max_query_samples // per_pod) if per_pod else None
        self.groups = []
        open_group: dict[tuple[str, str], int] = {}   # (ns, container) -> index of the group being filled
        group_chars: list[int] = []
        pod_group: dict[tuple[str, str, str], int] = {}
        slot_obj, slot_group, slot_pods = [], [], []
        for o, obj in enumerate(self.objects):
            key = (obj.namespace, obj.container)
            for pod in dict.fromkeys(obj.pods):
                pk = (obj.namespace, obj.container, pod)
                g = pod_group.get(pk)
                if g is None:
                    cost = len(pod_regex([pod])) + 1
                    g = open_group.get(key)
                    if g is None or (self.groups[g].pods and (group_chars[g] + cost > self.max_query_chars or
                                                              (max_pods is not None and
                                                               len(self.groups[g].pods) >= max_pods))):
                        g = len(self.groups)
                        self.groups.append(GroupQuery(obj.namespace, obj.container, []))
                        group_chars.append(0)
                        open_group[key] = g
                    self.groups[g].pods.append(pod)
                    group_chars[g] += cost
                    pod_group[pk] = g
                slot_obj.append(o)
                slot_group.append(g)
                slot_pods.append(pod)
        self.slot_obj = np.asarray(slot_obj, dtype=np.int64)
        self.slot_group = np.asarray(slot_group, dtype=np.int64)
        self.slot_pods = slot_pods
        names = [p.encode() for p in slot_pods]
        self._names = b"".join(names)
        self._name_offsets = np.zeros(len(names) + 1, dtype=np.int64)
        if names:
            np.cumsum([len(n) for n in names], out=self._name_offsets[1:])

    @classmethod
    def for_settings(cls, objects: Sequence, settings, **kw) -> "FleetQueryPlan":
        """Sample-bounded plan for a strategy's settings: points per series = the range
        query's evaluation timestamps, history / step + 1 (prometheus.py:124-126)."""
        step_s = int(settings.timeframe_timedelta.total_seconds()) // 60 * 60
        points = int(settings.history_timedelta.total_seconds()) // max(step_s, 1) + 1
        return cls(objects, points_per_series=points, **kw)

    @property
    def n_objects(self) -> int:
        return len(self.objects)

    @property
    def n_slots(self) -> int:
        return len(self.slot_pods)

    def queries(self, resource: ResourceType) -> list[str]:
        return [g.query(resource) for g in self.groups]

    def pack(self, bodies: Sequence[bytes], *, want_timestamps: bool = False, threads: int = 0,
             return_pod_counts: bool = False, alloc=None):
        """bodies[g] = the raw query_range response body of ``queries(resource)[g]``.

        Returns a PackedSeries (segment o = object o's pods with data, concatenated
        in K8sObjectData.pods order), plus the timestamps if ``want_timestamps`` and
        the per-(object, pod) sample counts (-1: dropped) if ``return_pod_counts``.
        ``alloc(n)``: optional allocator of the float64 value array (pinned memory).
        """
        if len(bodies) != len(self.groups):
            raise ValueError(f"expected {len(self.groups)} bodies (one per group query), got {len(bodies)}")
        lib = load_library()
        flat = [b if isinstance(b, bytes) else bytes(b) for b in bodies]  # c_char_p takes bytes only
        nb, ns, no = len(flat), self.n_slots, self.n_objects
        ptrs = (ctypes.c_char_p * max(nb, 1))(*flat)
        lens = np.array([len(b) for b in flat] or [0], dtype=np.int64)
        slot_group = self.slot_group if ns else np.zeros(1, np.int64)
        slot_obj = self.slot_obj if ns else np.zeros(1, np.int64)
        h = ctypes.c_void_p()
        rc = lib.krr_pack_parse_grouped(ctypes.cast(ptrs, ctypes.c_void_p), _ptr(lens), nb, b"pod",
                                        _ptr(slot_group), self._names or b"\0", _ptr(self._name_offsets),
                                        _ptr(slot_obj), ns, no, int(bool(want_timestamps)), int(threads),
                                        ctypes.byref(h))
        try:
            if rc != KRR_PACK_OK:
                msg = lib.krr_pack_error(h) if h else b""
                raise PrometheusResponseError(rc, (msg or b"invalid arguments").decode())
            n = int(lib.krr_pack_n_values(h))
            values = alloc(n) if alloc is not None else np.empty(n, dtype=np.float64)
            offsets = np.empty(no + 1, dtype=np.int64)
            ts = np.empty(n, dtype=np.float64) if want_timestamps else None
            counts = np.empty(max(ns, 1), dtype=np.int64) if return_pod_counts else None
            rc = lib.krr_pack_copy(h, _ptr(values), _ptr(offsets), _ptr(ts) if ts is not None else None,
                                   _ptr(counts) if counts is not None else None, int(threads))
            if rc != KRR_PACK_OK:
                raise PrometheusResponseError(rc, "krr_pack_copy failed")
            max_len = int(lib.krr_pack_max_len(h))
        finally:
            if h:
                lib.krr_pack_free(h)
        out: list = [PackedSeries(values, offsets, max_len)]
        if want_timestamps:
            out.append(ts)
        if return_pod_counts:
            out.append(counts[:ns])
        return out[0] if len(out) == 1 else tuple(out)

    def group_sorted_slots(self):
        """The slots ordered by group (stable): (order int64 [n_slots], slot_group[order], the pod
        names blob in that order, its offsets int64 [n_slots + 1], group_start int64 [n_groups + 1]
        = where each group's slots begin in that order).  A run of whole groups is then one
        contiguous range — the device packer routes chunk by chunk over it.  Cached."""
        cached = getattr(self, "_group_sorted", None)
        if cached is not None:
            return cached
        order = np.argsort(self.slot_group, kind="stable").astype(np.int64)
        sgroup = np.ascontiguousarray(self.slot_group[order])
        names = [self.slot_pods[i].encode() for i in order.tolist()]
        offs = np.zeros(len(names) + 1, dtype=np.int64)
        if names:
            np.cumsum([len(n) for n in names], out=offs[1:])
        gstart = np.searchsorted(sgroup, np.arange(len(self.groups) + 1), side="left").astype(np.int64)
        self._group_sorted = (order, sgroup, b"".join(names), offs, gstart)
        return self._group_sorted

    def pack_group_slots(self, bodies: Sequence[bytes], g0: int, g1: int, *, threads: int = 0, alloc=None):
        """The slots of groups [g0, g1) alone, from their bodies (bodies[i] answers group g0 + i),
        one segment per SLOT instead of per object: returns (slot indices int64 [k], values,
        offsets int64 [k + 1], counts int64 [k], -1 = dropped) — the series ``pack`` would route
        to each of those (object, pod) slots (krr_pack_parse_grouped, first series with the pod
        label wins).  The hybrid grouped parser's host side (krr_amd.core.device_pack)."""
        if len(bodies) != g1 - g0:
            raise ValueError("one body per group of [g0, g1)")
        idx = np.flatnonzero((self.slot_group >= g0) & (self.slot_group < g1)).astype(np.int64)
        k = idx.size
        lib = load_library()
        flat = [b if isinstance(b, bytes) else bytes(b) for b in bodies]
        ptrs = (ctypes.c_char_p * max(len(flat), 1))(*flat)
        lens = np.array([len(b) for b in flat] or [0], dtype=np.int64)
        names = [self.slot_pods[i].encode() for i in idx.tolist()]
        blob = b"".join(names)
        name_offs = np.zeros(k + 1, dtype=np.int64)
        if k:
            np.cumsum([len(n) for n in names], out=name_offs[1:])
        sg = np.ascontiguousarray(self.slot_group[idx] - g0) if k else np.zeros(1, np.int64)
        so = np.arange(max(k, 1), dtype=np.int64)
        h = ctypes.c_void_p()
        rc = lib.krr_pack_parse_grouped(ctypes.cast(ptrs, ctypes.c_void_p), _ptr(lens), len(flat), b"pod", _ptr(sg),
                                        blob or b"\0", _ptr(name_offs), _ptr(so), k, k, 0, int(threads),
                                        ctypes.byref(h))
        try:
            if rc != KRR_PACK_OK:
                msg = lib.krr_pack_error(h) if h else b""
                raise PrometheusResponseError(rc, (msg or b"invalid arguments").decode())
            n = int(lib.krr_pack_n_values(h))
            values = alloc(n) if alloc is not None else np.empty(n, dtype=np.float64)
            offsets = np.empty(k + 1, dtype=np.int64)
            counts = np.empty(max(k, 1), dtype=np.int64)
            rc = lib.krr_pack_copy(h, _ptr(values), _ptr(offsets), None, _ptr(counts), int(threads))
            if rc != KRR_PACK_OK:
                raise PrometheusResponseError(rc, "krr_pack_copy failed")
        finally:
            if h:
                lib.krr_pack_free(h)
        return idx, values, offsets, counts[:k]

    def fetch(self, query_range: Callable[[str], bytes], *, max_workers: int = 16) -> dict:
        """Run every grouped query for both resources; ``query_range(query)``
        performs one /api/v1/query_range request (start, end and step — the
        reference's ``step_string(timeframe)`` — bound by the caller)
        and returns the raw body.  Returns {ResourceType: [body per group]}."""
        jobs = [(rt, g.query(rt)) for rt in ResourceType for g in self.groups]
        with ThreadPoolExecutor(max_workers=max(1, max_workers)) as ex:
            bodies = list(ex.map(lambda j: query_range(j[1]), jobs))
        n = len(self.groups)
        return {rt: bodies[i * n:(i + 1) * n] for i, rt in enumerate(ResourceType)}

    def pack_fleet(self, cpu_bodies: Sequence[bytes], mem_bodies: Sequence[bytes], threads: int = 0,
                   alloc=None) -> PackedFleet:
        return PackedFleet(self.pack(cpu_bodies, threads=threads, alloc=alloc),
                           self.pack(mem_bodies, threads=threads, alloc=alloc))


__all__ = ["FleetQueryPlan", "GroupQuery", "group_query", "pod_query", "pod_regex", "step_string"]
