"""Reference-side drop-in: route the reference Runner's fleet fan-out to the HIP path.

The reference's ``Runner`` (robusta_krr/core/runner.py:17-137) holds ``self._strategy``,
built by ``Config.create_strategy()`` (core/models/config.py:48-51) from the strategy
registry (core/abstract/strategies.py:58-73): the reference's own pure-Python
``SimpleStrategy`` (strategies/simple.py:39-49).  Handing that object to
``krr_amd.core.runner.BatchedRunner`` would run ``simple.py:42-49`` per object, so this
module does the translation a maintainer needs:

* ``hip_strategy(reference_strategy)`` — the reference's ``SimpleStrategy`` (exactly that
  class; a subclass overriding ``run()`` is the user's own code) becomes
  ``krr_amd.strategies.simple.SimpleStrategy`` with the SAME settings values.  Only the
  fields the caller set are copied (pydantic v1 ``__fields_set__``), so the two numeric
  paths of SURVEY §0.4 survive: the CLI path (every field set, Decimals) and the
  int-default path (nothing set: ``99`` / ``5`` stay ``int``).
* ``gather_objects_recommendations(runner, objects)`` — replaces
  ``Runner._gather_objects_recommendations`` (runner.py:109-120): the reference's loaders
  fetch every object's history exactly as ``_calculate_object_recommendations``
  (runner.py:88-102) does, then ONE packed kernel pass + native exact-decimal rounding
  (runner.py:49-86) run for the whole fleet, and the reference's own
  ``ResourceAllocations`` come back (NaN -> "?" by its validator, allocations.py:40-41).
  Any other strategy takes the reference's own per-object path unchanged.
* ``install(Runner, loader=..., scan=...)`` — patches that method on the reference's
  ``Runner`` class, with two opt-in switches that take the rest of the path native:

  ``loader="reference"`` (default)  the reference's own ``PrometheusLoader.gather_data``
      (prometheus.py:108-155: one query per pod, ``Decimal(value)`` per sample), then
      ``pack_histories``;
  ``loader="bodies"``  the SAME per-pod queries (prometheus.py:118-143, character for
      character), issued through the reference loader's own ``prometheus._session``, but
      the raw response bodies go straight to the native packer (``krr_pack_parse``): no
      ``Decimal(value)`` per sample (prometheus.py:152), no Python list per pod;
  ``loader="grouped"`` one ``sum by (pod)`` range query per (namespace, container) group
      (``FleetQueryPlan.for_settings``), demultiplexed natively by pod label
      (``krr_pack_parse_grouped``); same CSR, bit for bit;
  ``scan="fleet"``  ``Runner._collect_result`` (runner.py:122-131) keeps its
      cluster/object listing and calls the patched gather, but the per-object
      ``ResourceScan.calculate`` + ``Result`` validation become ``scan_fleet`` (one
      vectorised severity pass) building the reference's OWN ResourceScan / Result
      objects, so ``_process_result`` and the formatters take them unchanged.

Nothing here falls back to CPU arithmetic: without ``libkrr_amd.so`` or a HIP device the
kernel call raises ``krr_amd._native.NativeUnavailable``.
"""
from __future__ import annotations

import asyncio
import datetime
import sys
from typing import Any, Optional, Sequence

import numpy as np

from krr_amd.core.models.allocations import ResourceType as HipResourceType
from krr_amd.core.runner import BatchedRunner
from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

REFERENCE_SIMPLE = ("robusta_krr.strategies.simple", "SimpleStrategy")
_ORIGINAL_ATTR = "_krr_amd_original_gather"
_ORIGINAL_COLLECT_ATTR = "_krr_amd_original_collect"
_OPTIONS_ATTR = "_krr_amd_options"
_PATCHED_ATTR = "_krr_amd_gather"  # marks install()'s _gather_objects_recommendations
LOADERS = ("reference", "bodies", "grouped")
SCANS = ("reference", "fleet")


class PrometheusHTTPError(RuntimeError):
    """A query_range request did not return HTTP 200 — where prometheus-api-client 0.5.3's
    ``custom_query_range`` raises ``PrometheusApiClientException`` [external] (the
    reference lets it abort the run: nothing in prometheus.py:108-155 catches it)."""


def hip_strategy(reference_strategy: Any) -> Optional[SimpleStrategy]:
    """The HIP-backed SimpleStrategy equivalent to the reference's, or None for any other
    strategy (custom plugins keep the reference's per-object ``run()``)."""
    cls = type(reference_strategy)
    if (cls.__module__, cls.__name__) != REFERENCE_SIMPLE:
        return None
    settings = reference_strategy.settings
    explicit = {name: getattr(settings, name) for name in getattr(settings, "__fields_set__", ())}
    return SimpleStrategy(SimpleStrategySettings(**explicit))


def _reference_types(runner: Any):
    """The reference's ResourceType / ResourceAllocations, as its runner module imported them
    (runner.py:11), so the results are the reference's own model objects."""
    mod = sys.modules[type(runner).__module__]
    return mod.ResourceType, mod.ResourceAllocations


def _options(runner: Any) -> dict:
    return getattr(type(runner), _OPTIONS_ATTR, None) or {"loader": "reference", "scan": "reference"}


async def gather_objects_recommendations(runner: Any, objects: Sequence[Any]) -> list:
    """Drop-in body of the reference's ``Runner._gather_objects_recommendations``."""
    RefResourceType, RefResourceAllocations = _reference_types(runner)
    strategy = hip_strategy(runner._strategy)
    if strategy is None:  # the reference's own per-object path (runner.py:109-120)
        original = getattr(type(runner), _ORIGINAL_ATTR, None)
        if original is not None:
            return await original(runner, objects)
        recs = await asyncio.gather(*[runner._calculate_object_recommendations(o) for o in objects])
        return [RefResourceAllocations(requests={rt: r[rt].request for rt in RefResourceType},
                                       limits={rt: r[rt].limit for rt in RefResourceType}) for r in recs]

    batched = BatchedRunner(strategy, runner.config.cpu_min_value, runner.config.memory_min_value)
    fleet = await packed_fleet(runner, objects, strategy, batched)
    ref = dict(model=RefResourceAllocations, resource_type=RefResourceType)
    # one fleet-wide kernel pass + native rounding + bulk models, off the event loop like the
    # reference's to_thread (runner.py:106)
    return await asyncio.to_thread(batched.allocations_packed, fleet, **ref)


async def packed_fleet(runner: Any, objects: Sequence[Any], strategy: SimpleStrategy, batched: BatchedRunner):
    """The fleet's PackedFleet through the installed loader: the reference's own per-object
    gather_data (runner.py:88-102), per-pod bodies, or grouped bodies."""
    RefResourceType, _ = _reference_types(runner)
    settings = runner._strategy.settings
    loader = _options(runner)["loader"]
    if loader == "bodies":
        cpu_bodies, mem_bodies = await fetch_pod_bodies(runner, objects, settings)
        # native packer (device by default), off the event loop
        parser = _options(runner).get("parser", "device")
        return await asyncio.to_thread(batched.pack_from_bodies, cpu_bodies, mem_bodies, 0, parser)
    if loader == "grouped":
        return await fetch_grouped_fleet(runner, objects, settings, _options(runner).get("parser", "device"), batched)

    async def history(obj):  # runner.py:88-102, with the reference's own loaders
        lo = runner._get_prometheus_loader(obj.cluster)
        data = await asyncio.gather(*[
            lo.gather_data(obj, rt, settings.history_timedelta, timeframe=settings.timeframe_timedelta)
            for rt in RefResourceType])
        return {HipResourceType(rt.value): d for rt, d in zip(RefResourceType, data)}

    histories = await asyncio.gather(*[history(o) for o in objects])
    return strategy.pack(histories)


# ---- body-level loaders -------------------------------------------------------------------------

def query_window(settings, now: Optional[datetime.datetime] = None) -> tuple[int, int, str]:
    """(start, end, step) of the reference's range queries: ``now - history .. now`` at
    ``"{timeframe minutes}m"`` (prometheus.py:124-126), as prometheus-api-client 0.5.3 sends
    them (``round(datetime.timestamp())``) [external].  One window for the whole fleet;
    the reference evaluates ``datetime.now()`` per query, microseconds apart."""
    from krr_amd.core.fleet_query import step_string

    now = now or datetime.datetime.now()
    return (round((now - settings.history_timedelta).timestamp()), round(now.timestamp()),
            step_string(settings.timeframe_timedelta))


def query_range_fn(prometheus: Any, start: int, end: int, step: str):
    """One raw ``/api/v1/query_range`` request on the reference's ``CustomPrometheusConnect``
    (prometheus.py:41-53): its session, url, headers and TLS setting, the parameters
    ``custom_query_range`` sends [external]; returns the response body (bytes)."""
    session, url = prometheus._session, f"{prometheus.url}/api/v1/query_range"
    verify, headers = prometheus.ssl_verification, prometheus.headers

    def query_range(query: str) -> bytes:
        r = session.get(url, params={"query": query, "start": start, "end": end, "step": step},
                        verify=verify, headers=headers)
        if r.status_code != 200:
            raise PrometheusHTTPError(f"HTTP Status Code {r.status_code} ({r.content!r})")
        return r.content

    return query_range


async def fetch_pod_bodies(runner: Any, objects: Sequence[Any], settings) -> tuple[list, list]:
    """Every object's per-pod CPU and memory bodies, fleet order (what gather_data fetches,
    prometheus.py:118-143): one request per (object, pod, resource), each on an executor
    thread like the reference's ``asyncio.to_thread`` per pod."""
    from krr_amd.core.fleet_query import pod_query

    start, end, step = query_window(settings)
    fns: dict = {}

    def fn(cluster):
        if cluster not in fns:
            fns[cluster] = query_range_fn(runner._get_prometheus_loader(cluster).prometheus, start, end, step)
        return fns[cluster]

    async def one(obj, rt):
        q = fn(obj.cluster)
        return list(await asyncio.gather(*[
            asyncio.to_thread(q, pod_query(rt, obj.namespace, pod, obj.container)) for pod in obj.pods]))

    cpu = asyncio.gather(*[one(o, HipResourceType.CPU) for o in objects])
    mem = asyncio.gather(*[one(o, HipResourceType.Memory) for o in objects])
    return tuple(await asyncio.gather(cpu, mem))  # type: ignore[return-value]


async def fetch_grouped_fleet(runner: Any, objects: Sequence[Any], settings, parser: str = "host", batched=None):
    """The fleet's PackedFleet from grouped ``sum by (pod)`` queries: one FleetQueryPlan per
    cluster (each cluster has its own Prometheus), packed natively, then the clusters'
    segments put back in fleet order for ONE kernel pass."""
    from krr_amd.core.fleet_query import FleetQueryPlan
    from krr_amd.core.packing import PackedFleet
    from krr_amd.core.runner import _pinned_alloc_or_none

    start, end, step = query_window(settings)
    by_cluster: dict = {}
    for i, o in enumerate(objects):
        by_cluster.setdefault(o.cluster, []).append(i)
    parts = []
    for cluster, idx in by_cluster.items():
        plan = FleetQueryPlan.for_settings([objects[i] for i in idx], settings)
        q = query_range_fn(runner._get_prometheus_loader(cluster).prometheus, start, end, step)
        bodies = await asyncio.to_thread(plan.fetch, q)
        if parser in ("device", "hybrid") and batched is not None:  # parsed on the MI355X, routed by pod label
            fleet = await asyncio.to_thread(batched.pack_grouped, plan, bodies[HipResourceType.CPU],
                                            bodies[HipResourceType.Memory], 0, parser)
        else:
            fleet = await asyncio.to_thread(plan.pack_fleet, bodies[HipResourceType.CPU],
                                            bodies[HipResourceType.Memory])
        parts.append((idx, fleet))
    if len(parts) == 1 and parts[0][0] == list(range(len(objects))):
        return parts[0][1]
    alloc = _pinned_alloc_or_none()
    order = [i for idx, _ in parts for i in idx]  # segment j of the concatenation = object order[j]
    return PackedFleet(_reorder([f.cpu for _, f in parts], order, alloc),
                       _reorder([f.mem for _, f in parts], order, alloc))


def _reorder(series: list, order: list, alloc=None):
    """Concatenate PackedSeries whose segments are objects ``order`` and permute the segments
    into object order 0..n-1 (numpy on the host, or torch for series already in HBM)."""
    from krr_amd.core.packing import PackedSeries

    on_dev = [s for s in series if not isinstance(s.values, np.ndarray)]
    if on_dev:  # device packer output (torch, HBM) — one cluster's batch may have gone to the host packer
        import torch

        dev = on_dev[0].values.device
        series = [s if not isinstance(s.values, np.ndarray) else
                  PackedSeries(torch.from_numpy(np.ascontiguousarray(s.values, np.float64)).to(dev),
                               torch.from_numpy(np.ascontiguousarray(s.offsets, np.int64)).to(dev), s.max_len)
                  for s in series]
        lens = torch.cat([s.offsets[1:] - s.offsets[:-1] for s in series])
        bases = torch.tensor(np.cumsum([0] + [int(s.values.numel()) for s in series])[:-1], device=dev)
        srcs = torch.cat([s.offsets[:-1] + b for s, b in zip(series, bases)])
        flat = torch.cat([s.values for s in series])
        inv = torch.empty(len(order), dtype=torch.int64, device=dev)
        inv[torch.tensor(order, dtype=torch.int64, device=dev)] = torch.arange(len(order), device=dev)
        lens_o, srcs_o = lens[inv], srcs[inv]
        offsets = torch.zeros(len(order) + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens_o, 0, out=offsets[1:])
        total = int(offsets[-1].item())
        seg = torch.repeat_interleave(torch.arange(len(order), device=dev), lens_o)
        pos = torch.arange(total, device=dev) - offsets[:-1][seg] + srcs_o[seg]
        return PackedSeries(flat[pos], offsets, max(s.max_len for s in series))
    lens = np.concatenate([np.diff(s.offsets) for s in series]) if series else np.zeros(0, np.int64)
    srcs = np.concatenate([s.offsets[:-1] + base for s, base in
                           zip(series, np.cumsum([0] + [s.values.size for s in series])[:-1])]) \
        if series else np.zeros(0, np.int64)
    flat = np.concatenate([s.values for s in series]) if series else np.zeros(0, np.float64)
    inv = np.empty(len(order), dtype=np.int64)
    inv[np.asarray(order, dtype=np.int64)] = np.arange(len(order), dtype=np.int64)
    lens_o, srcs_o = lens[inv], srcs[inv]
    offsets = np.zeros(len(order) + 1, dtype=np.int64)
    np.cumsum(lens_o, out=offsets[1:])
    values = alloc(int(offsets[-1])) if alloc is not None else np.empty(int(offsets[-1]), dtype=np.float64)
    for j in range(len(order)):
        values[offsets[j]:offsets[j + 1]] = flat[srcs_o[j]:srcs_o[j] + lens_o[j]]
    return PackedSeries(values, offsets, int(lens.max(initial=0)))


# ---- Runner._collect_result with the fleet-vectorised scan ------------------------------------

async def collect_result(runner: Any):
    """Drop-in body of the reference's ``Runner._collect_result`` (runner.py:122-131): its own
    cluster and object listing, the (patched) gather, then ``scan_fleet`` + the score over
    the reference's own ResourceScan / Result models (core/models/result.py:63-150)."""
    from krr_amd.core.models.result import collect_result as fleet_collect

    clusters = await runner._k8s_loader.list_clusters()
    runner.debug(f'Using clusters: {clusters if clusters is not None else "inner cluster"}')
    objects = await runner._k8s_loader.list_scannable_objects(clusters)
    models = sys.modules[sys.modules[type(runner).__module__].Result.__module__]
    strategy = hip_strategy(runner._strategy)
    if strategy is not None and getattr(type(runner)._gather_objects_recommendations, _PATCHED_ATTR, False):
        # the gather is this module's: its ResourceAllocations would only be read by the scan, so
        # the rounded values go straight into it (fast_round.result_batch)
        from krr_amd.core.fast_round import result_batch

        batched = BatchedRunner(strategy, runner.config.cpu_min_value, runner.config.memory_min_value)
        fleet = await packed_fleet(runner, objects, strategy, batched)

        def run():
            raw = strategy.settings.run_fleet(fleet)
            return result_batch(objects, raw, strategy.settings, batched.cpu_min_value, batched.memory_min_value,
                                models=models)

        return await asyncio.to_thread(run)
    recommendations = await runner._gather_objects_recommendations(objects)
    return fleet_collect(objects, recommendations, models)


def install(runner_cls: Any = None, *, loader: str = "reference", scan: str = "reference",
            parser: str = "device") -> Any:
    """Route ``runner_cls._gather_objects_recommendations`` (default: the reference's
    ``robusta_krr.core.runner.Runner``) through ``gather_objects_recommendations``, loading
    histories with ``loader`` (see the module docstring), and with ``scan="fleet"`` also
    ``_collect_result`` through ``collect_result``.  ``parser`` (loader="bodies"): "device"
    parses the raw bodies on the MI355X (krr_amd.core.device_pack), "host" with the native
    host packer, "hybrid" both at once on disjoint object ranges
    (``BatchedRunner.pack_hybrid``; loader="grouped" parses as "device").  Calling it again
    changes the switches;
    ``uninstall`` restores the reference's methods.  Returns the class."""
    if loader not in LOADERS:
        raise ValueError(f"loader must be one of {LOADERS}")
    if scan not in SCANS:
        raise ValueError(f"scan must be one of {SCANS}")
    if parser not in ("device", "host", "hybrid"):
        raise ValueError("parser must be 'device', 'host' or 'hybrid'")
    if runner_cls is None:
        from robusta_krr.core.runner import Runner as runner_cls  # the reference, in its own process
    if getattr(runner_cls, _ORIGINAL_ATTR, None) is None:
        setattr(runner_cls, _ORIGINAL_ATTR, runner_cls._gather_objects_recommendations)

        async def _gather_objects_recommendations(self, objects):
            return await gather_objects_recommendations(self, objects)

        setattr(_gather_objects_recommendations, _PATCHED_ATTR, True)

        runner_cls._gather_objects_recommendations = _gather_objects_recommendations
    if scan == "fleet" and getattr(runner_cls, _ORIGINAL_COLLECT_ATTR, None) is None:
        setattr(runner_cls, _ORIGINAL_COLLECT_ATTR, runner_cls._collect_result)

        async def _collect_result(self):
            return await collect_result(self)

        runner_cls._collect_result = _collect_result
    elif scan == "reference" and getattr(runner_cls, _ORIGINAL_COLLECT_ATTR, None) is not None:
        runner_cls._collect_result = getattr(runner_cls, _ORIGINAL_COLLECT_ATTR)
        setattr(runner_cls, _ORIGINAL_COLLECT_ATTR, None)
    setattr(runner_cls, _OPTIONS_ATTR, {"loader": loader, "scan": scan, "parser": parser})
    return runner_cls


def uninstall(runner_cls: Any) -> Any:
    """Put back the reference's own methods patched by ``install``."""
    for attr, name in ((_ORIGINAL_ATTR, "_gather_objects_recommendations"),
                       (_ORIGINAL_COLLECT_ATTR, "_collect_result")):
        orig = getattr(runner_cls, attr, None)
        if orig is not None:
            setattr(runner_cls, name, orig)
            setattr(runner_cls, attr, None)
    setattr(runner_cls, _OPTIONS_ATTR, None)
    return runner_cls


__all__ = ["LOADERS", "PrometheusHTTPError", "SCANS", "collect_result", "fetch_grouped_fleet", "fetch_pod_bodies",
           "gather_objects_recommendations", "hip_strategy", "install", "query_range_fn", "query_window", "uninstall"]
