"""Batched runner: the fleet-wide replacement of the reference's per-object loop
(Runner._calculate_object_recommendations / _gather_objects_recommendations,
robusta_krr/core/runner.py:88-120).

  1. gather every object's HistoryData (loader I/O, concurrently as the reference does);
  2. strategies with ``run_batch`` (SimpleStrategy): pack once, ONE kernel pass;
     any other BaseStrategy subclass: the reference's per-object ``run()`` loop;
  3. exact-decimal rounding + minimum clamp (runner.py:49-86, krr_amd.core.rounding);
  4. ResourceAllocations (NaN -> "?", allocations.py:40-41).

Multi-GPU (one process per GPU, torch.distributed over RCCL): the fleet fan-out
(runner.py:109-120) becomes a contiguous, sample-balanced object shard per rank,
ONE fused kernel pass per rank writing 32-B result records, one gather of the
records to the destination rank, and the exact-decimal rounding there
(``recommend_shard`` / ``recommend_packed_sharded`` /
``gather_objects_recommendations_sharded``).
"""
from __future__ import annotations

import asyncio
import datetime
from typing import Optional, Protocol, Sequence

from krr_amd.core.abstract.strategies import (
    BaseStrategy,
    HistoryData,
    ResourceHistoryData,
    RunResult,
    run_each,
    supports_batch,
    supports_packed,
)
from krr_amd.core.models.allocations import ResourceAllocations, ResourceType
from krr_amd.core.models.objects import K8sObjectData
from krr_amd.core.rounding import DEFAULT_CPU_MIN_VALUE, DEFAULT_MEMORY_MIN_VALUE, format_result


class HistoryLoader(Protocol):
    """What the reference's PrometheusLoader.gather_data provides (prometheus.py:108-155)."""

    async def gather_data(self, object: K8sObjectData, resource: ResourceType, period: datetime.timedelta,
                          *, timeframe: datetime.timedelta) -> ResourceHistoryData: ...


class BatchedRunner:
    def __init__(self, strategy: BaseStrategy, cpu_min_value: int = DEFAULT_CPU_MIN_VALUE,
                 memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE):
        self.strategy = strategy
        self.cpu_min_value = cpu_min_value
        self.memory_min_value = memory_min_value

    @classmethod
    def from_config(cls, config) -> "BatchedRunner":
        return cls(config.create_strategy(), config.cpu_min_value, config.memory_min_value)

    def raw_results(self, objects: Sequence[K8sObjectData], histories: Sequence[HistoryData]) -> list[RunResult]:
        if len(objects) != len(histories):
            raise ValueError("one HistoryData per object")
        if supports_batch(self.strategy):
            return self.strategy.run_batch(histories, objects)  # type: ignore[attr-defined]
        return run_each(self.strategy, histories, objects)

    def recommend(self, objects: Sequence[K8sObjectData], histories: Sequence[HistoryData]) -> list[RunResult]:
        """Rounded RunResults, one per object (what _calculate_object_recommendations returns)."""
        if len(objects) != len(histories):
            raise ValueError("one HistoryData per object")
        if supports_packed(self.strategy):  # SimpleStrategy: pack once, native rounding
            return self.strategy.format_packed(self.strategy.pack(histories), self.cpu_min_value,
                                               self.memory_min_value)
        return [format_result(r, self.cpu_min_value, self.memory_min_value)
                for r in self.raw_results(objects, histories)]

    def recommend_packed(self, fleet) -> list[RunResult]:
        """Rounded RunResults for a PackedFleet (e.g. from recommend_from_bodies)."""
        self._require_packed()
        return self.strategy.format_packed(fleet, self.cpu_min_value, self.memory_min_value)

    def _require_packed(self) -> None:
        if not supports_packed(self.strategy):
            raise TypeError(f"{type(self.strategy).__name__} has no batched packed path; use recommend()")

    # --- multi-GPU: one process per GPU ------------------------------------------
    def recommend_shard(self, local_fleet, group=None, dst: int = 0, device: Optional[int] = None):
        """This rank's contiguous object shard -> ONE kernel pass (records written by the
        same launch) -> records gathered to rank ``dst`` of ``group`` (RCCL for "nccl",
        host tensors for gloo) -> the rounded RunResults of every rank's objects, in rank
        order, on ``dst``; None on the other ranks.  Collective: every rank calls it."""
        from krr_amd.core.distributed import collective_device, gather_records, local_device, raw_from_records

        import torch

        import numpy as np
        import torch.distributed as dist

        from krr_amd.core.distributed import record_counts, records_from_raw

        self._require_packed()
        dev = local_device() if device is None else int(device)
        settings = self.strategy.settings
        coll = collective_device(group, dev)
        objs = None
        if local_fleet.cpu.exact is not None or local_fleet.mem.exact is not None:
            # HistoryData whose Decimals the float64 images do not reproduce ('0.10', 25-digit
            # values ...): this rank locates and resolves its shard's sample objects
            # (krr_amd.core.exact, as run_fleet does on one GPU) and sends them to dst
            raw = settings.run_fleet(local_fleet, device=dev)
            rec = records_from_raw(raw, coll)
            objs = {"cpu": raw.cpu_exact or {}, "mem": raw.mem_exact or {}}
        else:
            rec = settings.run_fleet_records(local_fleet, dev)
        if coll.type == "cuda":
            # this may run on a worker thread (gather_objects_recommendations_sharded):
            # its current device is 0 until set, and RCCL enqueues on the current device
            torch.cuda.set_device(coll)
        counts = record_counts(rec.shape[0], coll, group)
        full = gather_records(rec.to(coll), dst=dst, group=group, counts=counts)
        # every rank says whether it holds such objects (one all_reduce of an int); only then
        # do the per-rank dicts travel (gather_object), keyed by global object index
        flag = torch.tensor([0 if objs is None else 1], dtype=torch.int64, device=coll)
        dist.all_reduce(flag, group=group)
        exact = None
        if int(flag.item()):
            rank = dist.get_rank(group)
            gdst = dist.get_global_rank(group, dst) if group is not None else dst
            got = [None] * dist.get_world_size(group) if rank == dst else None
            dist.gather_object(objs or {"cpu": {}, "mem": {}}, got, dst=gdst, group=group)
            if got is not None:
                base = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
                exact = {name: {int(base[r]) + i: v for r, o in enumerate(got) for i, v in o[name].items()}
                         for name in ("cpu", "mem")}
        if full is None:
            return None
        raw = raw_from_records(full)
        if exact is not None:
            raw.cpu_exact, raw.mem_exact = exact["cpu"] or None, exact["mem"] or None
        return self.strategy.format_raw(raw, self.cpu_min_value, self.memory_min_value)

    def recommend_bodies_shard(self, cpu_bodies: Sequence[Sequence[bytes]], mem_bodies: Sequence[Sequence[bytes]],
                               group=None, dst: int = 0, device: Optional[int] = None, parser: str = "device",
                               threads: int = 0):
        """This rank's objects' raw query_range bodies (its contiguous object range; rank order
        = fleet order, e.g. ``body_shard_bounds``) -> packed on this rank's GPU (the device
        packer by default: each GPU's own PCIe link carries its shard's JSON) -> one kernel
        pass -> the records gathered to ``dst``, which returns every rank's rounded RunResults
        in fleet order (None elsewhere).  Collective: every rank calls it."""
        from krr_amd.core.distributed import local_device
        from krr_amd.core.packing import PackedFleet
        from krr_amd.core.prom_native import pack_query_range_bodies

        if parser not in ("device", "host", "hybrid"):
            raise ValueError("parser must be 'device', 'host' or 'hybrid'")
        # ONE device for the pack and the kernel pass: this rank's GPU (LOCAL_RANK) unless
        # the caller names one — the packer's own default (settings.device) is GPU 0
        dev = local_device() if device is None else int(device)
        if parser == "hybrid":
            parts = self.pack_hybrid(cpu_bodies, mem_bodies, threads=threads, device=dev)
            fleet = parts[0] if len(parts) == 1 else _concat_fleets(parts, dev)
        elif parser == "device":
            fleet = self.pack_bodies_device(cpu_bodies, mem_bodies, threads=threads, device=dev)
        else:
            fleet = PackedFleet(pack_query_range_bodies(cpu_bodies, threads=threads),
                                pack_query_range_bodies(mem_bodies, threads=threads))
        return self.recommend_shard(fleet, group=group, dst=dst, device=dev)

    def recommend_packed_sharded(self, fleet, group=None, dst: int = 0, device: Optional[int] = None):
        """Every rank holds the same packed fleet: each runs its sample-balanced contiguous
        shard (``fleet_shard_bounds``) and ``dst`` receives the whole fleet's results."""
        import torch.distributed as dist

        from krr_amd.core.distributed import fleet_shard_bounds, slice_fleet

        lo, hi = fleet_shard_bounds(fleet, dist.get_world_size(group))[dist.get_rank(group)]
        return self.recommend_shard(slice_fleet(fleet, lo, hi), group=group, dst=dst, device=device)

    async def gather_objects_recommendations_sharded(self, objects: Sequence[K8sObjectData], loader: HistoryLoader,
                                                     group=None, dst: int = 0,
                                                     device: Optional[int] = None) -> Optional[list]:
        """The reference's fleet fan-out (runner.py:109-120) over ranks: every rank knows the
        object list, fetches ONLY its shard's histories (objects cut by expected samples =
        pod count), packs them, runs one kernel pass; ``dst`` gets every object's
        ResourceAllocations in object order, the other ranks None."""
        import torch.distributed as dist

        from krr_amd.core.distributed import shard_bounds

        self._require_packed()
        lo, hi = shard_bounds([max(len(o.pods), 1) for o in objects],
                              dist.get_world_size(group))[dist.get_rank(group)]
        histories = await self.gather_histories(objects[lo:hi], loader)
        fleet = self.strategy.pack(histories)
        res = await asyncio.to_thread(self.recommend_shard, fleet, group, dst, device)
        return None if res is None else [to_allocations(r) for r in res]

    def allocations_packed(self, fleet, model=None, resource_type=None) -> list:
        """Runner._gather_objects_recommendations's list (runner.py:113-120) for a PackedFleet:
        one kernel pass, native rounding, and the ResourceAllocations built in bulk
        (krr_amd.core.fast_round.allocations_batch; ``model`` / ``resource_type``: the
        reference's own classes, default this package's mirror)."""
        from krr_amd.core.fast_round import allocations_batch

        self._require_packed()
        raw = self.strategy.settings.run_fleet(fleet)
        return allocations_batch(raw, self.strategy.settings, self.cpu_min_value, self.memory_min_value, model=model,
                                 resource_type=resource_type)

    def result_packed(self, objects: Sequence[K8sObjectData], fleet, models=None, threads: int = 0):
        """Runner._collect_result's Result (runner.py:122-131) for a PackedFleet: one kernel pass,
        native rounding, and the ResourceScan per object + score built straight from the rounded
        values (krr_amd.core.fast_round.result_batch: the ResourceAllocations the reference builds
        in between are only read by the scan).  ``models``: the reference's result module
        (default this package's mirror)."""
        from krr_amd.core.fast_round import result_batch

        self._require_packed()
        raw = self.strategy.settings.run_fleet(fleet)
        return result_batch(objects, raw, self.strategy.settings, self.cpu_min_value, self.memory_min_value,
                            threads=threads, models=models)

    def pack_from_bodies(self, cpu_bodies, mem_bodies, threads: int = 0, parser: str = "device"):
        """The PackedFleet of raw per-pod query_range bodies (see recommend_from_bodies)."""
        from krr_amd.core.packing import PackedFleet
        from krr_amd.core.prom_native import pack_query_range_bodies

        if len(cpu_bodies) != len(mem_bodies):
            raise ValueError("cpu and memory bodies need one entry per object each")
        if parser not in ("device", "host", "hybrid"):
            raise ValueError("parser must be 'device', 'host' or 'hybrid'")
        if parser == "hybrid":
            parts = self.pack_hybrid(cpu_bodies, mem_bodies, threads=threads)
            if len(parts) == 1:
                return parts[0]
            return _concat_fleets(parts, self.strategy.settings.device)
        if parser == "device":
            return self.pack_bodies_device(cpu_bodies, mem_bodies, threads=threads)
        alloc = _pinned_alloc_or_none()
        return PackedFleet(pack_query_range_bodies(cpu_bodies, threads=threads, alloc=alloc),
                           pack_query_range_bodies(mem_bodies, threads=threads, alloc=alloc))

    def recommend_from_bodies(self, cpu_bodies: Sequence[Sequence[bytes]], mem_bodies: Sequence[Sequence[bytes]],
                              threads: int = 0, parser: str = "device") -> list[RunResult]:
        """The whole loader -> strategy -> rounding path from raw Prometheus query_range
        response bodies: bodies[o][i] = pod i of object o (K8sObjectData.pods order),
        as PrometheusLoader.gather_data would fetch them (prometheus.py:118-143).
        ``parser="device"`` (default): the bodies cross PCIe raw and the MI355X parses them
        (krr_amd.core.device_pack; a batch with bodies outside Prometheus' canonical form
        goes to the host packer); ``"host"``: the native host packer (libkrr_host.so);
        ``"hybrid"``: both at once on disjoint object ranges (``pack_hybrid``), one kernel
        pass per range.  No Decimal lists either way; native rounding."""
        self._require_packed()
        if parser == "hybrid":
            import threading

            import torch

            settings = self.strategy.settings
            lock = threading.Lock()  # one engine context: its passes one at a time

            import time

            done = {}

            def host_then(fleet):  # the host part's upload + kernel pass, while the device part packs
                with lock, torch.cuda.stream(torch.cuda.Stream(device=settings.device)):
                    r = settings.run_fleet(fleet)
                done["host"] = time.perf_counter()
                return r

            def device_then(fleet):  # the device part's kernel pass, before the host side is joined
                with lock:
                    r = settings.run_fleet(fleet)
                done["device"] = time.perf_counter()
                return r

            t0 = time.perf_counter()
            share = self.hybrid_share
            parts, (raw_host, raw_dev) = self._pack_hybrid(cpu_bodies, mem_bodies, threads=threads,
                                                           host_then=host_then, device_then=device_then)
            if len(parts) > 1:
                raws = [raw_dev, raw_host]
                # balance the whole critical paths (pack + kernel pass on each side), not the packs
                self.hybrid_share = _rebalance(share, done["device"] - t0, done.get("host", t0) - t0)
            else:
                with lock:
                    raws = [settings.run_fleet(parts[0])]
            raw = _concat_raw(raws)
            return self.strategy.format_raw(raw, self.cpu_min_value, self.memory_min_value)
        return self.recommend_packed(self.pack_from_bodies(cpu_bodies, mem_bodies, threads, parser))

    # parser="hybrid": the share of the JSON bytes the host packer takes, moved after every
    # call toward equal finishing times of the two sides (_rebalance)
    hybrid_share = 0.08
    # staging threads of the device side (0: three quarters of the threads when the device packer
    # strips timestamps while staging, a quarter for a plain copy; the host parser gets the rest)
    hybrid_device_threads = 0
    hybrid_last: Optional[dict] = None

    def pack_hybrid(self, cpu_bodies, mem_bodies, threads: int = 0, device: Optional[int] = None) -> list:
        """Raw bodies -> PackedFleets of consecutive object ranges, in object order: the LAST
        ``hybrid_share`` of the JSON bytes parsed by the host packer (libkrr_host.so, on a
        worker thread, most of the threads) WHILE the first part crosses PCIe raw and is
        parsed on the device (krr_amd.core.device_pack, the staging copy on the remaining
        threads).  Each part equals what its parser gives for that range alone, so the
        concatenation equals either parser on the whole batch; a body either parser rejects
        sends the whole batch to the host packer (its result, or its error naming the
        first bad body).  The share then moves toward r_host / (r_host + r_device)."""
        return self._pack_hybrid(cpu_bodies, mem_bodies, threads, device)[0]

    def _pack_hybrid(self, cpu_bodies, mem_bodies, threads: int = 0, device: Optional[int] = None,
                     host_then=None, device_then=None):
        """pack_hybrid, plus ``host_then(host_fleet)`` run on the worker thread as soon as the
        host part is packed (e.g. its upload and kernel pass, overlapping the device part's
        pack) and ``device_then(device_fleet)`` on the calling thread as soon as the device part
        is packed (before the host side is joined); returns (parts, (host_then's result,
        device_then's result)), None for a callback not run or whose part was discarded."""
        import os
        import threading
        import time

        import numpy as np

        from krr_amd.core.packing import PackedFleet
        from krr_amd.core.prom_native import PrometheusResponseError, pack_query_range_bodies

        if len(cpu_bodies) != len(mem_bodies):
            raise ValueError("cpu and memory bodies need one entry per object each")
        n = len(cpu_bodies)
        T = int(threads) or _host_threads()
        from krr_amd.core.device_pack import _body_table

        table = _body_table([cpu_bodies, mem_bodies])
        if table is not None:  # bytes per object from one native pass
            nb = table[3][:n] + table[3][n:]
        else:
            nb = np.fromiter((sum(len(b) for b in cb) + sum(len(b) for b in mb)
                              for cb, mb in zip(cpu_bodies, mem_bodies)), dtype=np.int64, count=n)
        cum = np.cumsum(nb)
        total = int(cum[-1]) if n else 0
        share = min(max(float(self.hybrid_share), 0.02), 0.8)
        k = int(np.searchsorted(cum, (1.0 - share) * total, side="left")) + 1 if n else 0
        k = min(max(k, 1), n - 1)
        if T < 3 or n < 2:
            return [self.pack_bodies_device(cpu_bodies, mem_bodies, threads=threads, device=device)], (None, None)
        # staging threads (hybrid_device_threads); the host parser gets the rest.  A stripping
        # staging thread moves 5-9x the JSON bytes per second of a host parser thread and keeps
        # fewer bytes on the link, so it gets three quarters of the threads — enough to keep
        # the link busy on a host whose cores strip only ~7 GB/s each (a plain copy: a quarter)
        strips = self._device_packer(threads, device).strip
        t_dev = max(1, min(T - 1, int(self.hybrid_device_threads or (3 * T // 4 if strips else T // 4))))
        t_host = max(1, T - t_dev)
        host_out: dict = {}
        alloc = _pinned_alloc_or_none()
        # set once the device side knows the batch goes to the host packer whole: host_then's
        # pass over the partial host fleet would be discarded, so it is not started after that
        device_fell_back = threading.Event()

        def host_part():
            t0 = time.perf_counter()
            try:
                host_out["fleet"] = PackedFleet(
                    pack_query_range_bodies(cpu_bodies[k:], threads=t_host, alloc=alloc),
                    pack_query_range_bodies(mem_bodies[k:], threads=t_host, alloc=alloc))
                if host_then is not None and not device_fell_back.is_set():
                    host_out["then"] = host_then(host_out["fleet"])
            except PrometheusResponseError as e:
                host_out["error"] = e
            except BaseException as e:  # noqa: BLE001 - re-raised on the calling thread
                host_out["exc"] = e
            host_out["s"] = time.perf_counter() - t0

        worker = threading.Thread(target=host_part, name="krr-hybrid-host", daemon=True)
        worker.start()
        t0 = time.perf_counter()
        dev_then = None
        try:
            dev_fleet = self.pack_bodies_device(cpu_bodies[:k], mem_bodies[:k], threads=t_dev, device=device)
            dev_via = self.last_pack_via
            if dev_via != ("device", "device"):
                device_fell_back.set()
            dev_s = time.perf_counter() - t0
            if device_then is not None and dev_via == ("device", "device"):
                dev_then = device_then(dev_fleet)
            self.last_pack_via = dev_via
        finally:
            worker.join()
        if "exc" in host_out:
            raise host_out["exc"]
        if "error" in host_out or self.last_pack_via != ("device", "device"):
            # a body one side rejected: the outcome is the host packer's on the whole batch
            self.last_pack_via = ("host", "host")
            return [PackedFleet(pack_query_range_bodies(cpu_bodies, threads=threads, alloc=alloc),
                                pack_query_range_bodies(mem_bodies, threads=threads, alloc=alloc))], (None, None)
        b_dev, b_host = int(cum[k - 1]), total - int(cum[k - 1])
        r_dev, r_host = b_dev / max(dev_s, 1e-9), b_host / max(host_out["s"], 1e-9)
        self.hybrid_last = {"share": share, "split_object": k, "device_s": dev_s, "host_s": host_out["s"],
                            "device_GBps": r_dev / 1e9, "host_GBps": r_host / 1e9,
                            "device_threads": t_dev, "host_threads": t_host,
                            "device_upload": self._device_packer(threads, device).last_upload}
        self.hybrid_share = _rebalance(share, dev_s, host_out["s"])
        self.hybrid_last.update(bytes_device=b_dev, bytes_host=b_host)
        self.last_pack_via = ("hybrid", "hybrid")
        return [dev_fleet, host_out["fleet"]], (host_out.get("then"), dev_then)

    @staticmethod
    def body_shard_bounds(objects: Sequence[K8sObjectData], world: int) -> list:
        """Contiguous object ranges per rank, cut by pod count (one query_range body per pod
        and resource): rank r fetches and packs objects[lo:hi] of its (lo, hi)."""
        from krr_amd.core.distributed import shard_bounds

        return shard_bounds([max(len(o.pods), 1) for o in objects], world)

    def pack_bodies_device(self, cpu_bodies, mem_bodies, threads: int = 0, device: Optional[int] = None):
        """PackedFleet in HBM from raw bodies, parsed on the device (krr_amd.core.device_pack)."""
        from krr_amd.core.packing import PackedFleet

        packer = self._device_packer(threads, device)
        cpu, mem = packer.pack_many([cpu_bodies, mem_bodies])  # one staging / copy / parse pipeline
        self.last_pack_via = (cpu.via, mem.via)
        return PackedFleet(cpu.series, mem.series)

    def recommend_from_grouped(self, plan, cpu_bodies: Sequence[bytes], mem_bodies: Sequence[bytes],
                               threads: int = 0, parser: str = "device") -> list[RunResult]:
        """As recommend_from_bodies, from fleet-batched responses: ``plan`` is a
        krr_amd.core.fleet_query.FleetQueryPlan and bodies[g] answers its g-th grouped
        ``sum by (pod)`` query (one per (namespace, container), not one per pod).
        ``parser="device"``: the MI355X parses the bodies and the host routes series to
        pods by label (krr_amd.core.device_pack); ``"host"``: krr_pack_parse_grouped;
        ``"hybrid"``: the device, with the last groups' bodies parsed by the host packer
        meanwhile (``DevicePacker.pack_grouped_many(hybrid=True)``)."""
        import time

        t0 = time.perf_counter()
        fleet = self.pack_grouped(plan, cpu_bodies, mem_bodies, threads=threads, parser=parser)
        t1 = time.perf_counter()
        out = self.recommend_packed(fleet)
        self.grouped_last = {"pack_s": t1 - t0, "kernel_round_s": time.perf_counter() - t1}
        return out

    def pack_grouped(self, plan, cpu_bodies, mem_bodies, threads: int = 0, parser: str = "device"):
        from krr_amd.core.packing import PackedFleet

        if parser not in ("device", "host", "hybrid"):
            raise ValueError("parser must be 'device', 'host' or 'hybrid'")
        if parser == "host":
            return plan.pack_fleet(cpu_bodies, mem_bodies, threads=threads, alloc=_pinned_alloc_or_none())
        packer = self._device_packer(threads)
        # hybrid: the last groups' bodies parsed by the host packer while the rest cross the link
        cpu, mem = packer.pack_grouped_many([(plan, cpu_bodies), (plan, mem_bodies)], hybrid=parser == "hybrid")
        self.last_pack_via = (cpu.via, mem.via)
        return PackedFleet(cpu.series, mem.series)

    def _device_packer(self, threads: int = 0, device: Optional[int] = None):
        from krr_amd.core.device_pack import default_packer

        dev = getattr(self.strategy.settings, "device", 0) if device is None else int(device)
        packer = default_packer(dev)  # NativeUnavailable without a GPU
        if threads:
            packer.threads = int(threads)
        return packer

    def allocations(self, objects: Sequence[K8sObjectData],
                    histories: Sequence[HistoryData]) -> list[ResourceAllocations]:
        if len(objects) != len(histories):
            raise ValueError("one HistoryData per object")
        if supports_packed(self.strategy):  # bulk-built models (fast_round.allocations_batch)
            return self.allocations_packed(self.strategy.pack(histories))
        return [to_allocations(r) for r in self.recommend(objects, histories)]

    def collect_result(self, objects: Sequence[K8sObjectData], histories: Sequence[HistoryData]):
        """Runner._collect_result's Result (runner.py:122-131) from already gathered
        histories: recommendations, then the fleet-vectorised ResourceScan/score."""
        from krr_amd.core.models.result import collect_result

        return collect_result(objects, self.allocations(objects, histories))

    async def gather_histories(self, objects: Sequence[K8sObjectData], loader: HistoryLoader) -> list[HistoryData]:
        settings = self.strategy.settings

        async def one(obj: K8sObjectData) -> HistoryData:
            data = await asyncio.gather(*[
                loader.gather_data(obj, resource, settings.history_timedelta, timeframe=settings.timeframe_timedelta)
                for resource in ResourceType
            ])
            return dict(zip(ResourceType, data))

        return list(await asyncio.gather(*[one(o) for o in objects]))

    async def gather_objects_recommendations(self, objects: Sequence[K8sObjectData],
                                             loader: HistoryLoader) -> list[ResourceAllocations]:
        histories = await self.gather_histories(objects, loader)
        # the kernel pass runs off the event loop, like the reference's to_thread (runner.py:106)
        return await asyncio.to_thread(self.allocations, objects, histories)


def _rebalance(share: float, t_device: float, t_host: float) -> float:
    """The hybrid parser's next host share: moved toward equal finishing times by the square
    root of their ratio, at most 25% per call, within [0.02, 0.8].  (Balancing the two sides'
    RATES instead runs away on a shared host: each side's rate depends on the other's load.)"""
    r = (max(t_device, 1e-9) / max(t_host, 1e-9)) ** 0.5
    return min(max(share * min(max(r, 0.8), 1.25), 0.02), 0.8)


def _host_threads() -> int:
    """Host threads this process may use: the affinity set, capped by OMP_NUM_THREADS when set
    (a GPU box may show every CPU of the machine but lease a few per GPU)."""
    import os

    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n)


def _concat_raw(raws):
    """RawResults of consecutive object ranges -> one RawResults."""
    import numpy as np

    from krr_amd.core.engine import RawResults

    if len(raws) == 1:
        return raws[0]
    return RawResults(*(np.concatenate([np.asarray(getattr(r, f)) for r in raws])
                        for f in ("cpu_value", "cpu_count", "cpu_flags", "mem_value", "mem_count", "mem_flags")))


def _concat_fleets(parts, device):
    """PackedFleets of consecutive object ranges (HBM and/or host) -> one PackedFleet in HBM."""
    import torch

    from krr_amd.core.packing import PackedFleet, PackedSeries

    dev = torch.device("cuda", int(device))

    def cat(series):
        vals, offs, base = [], [torch.zeros(1, dtype=torch.int64, device=dev)], 0
        for ps in series:
            v = ps.values if isinstance(ps.values, torch.Tensor) else torch.from_numpy(ps.values)
            o = ps.offsets if isinstance(ps.offsets, torch.Tensor) else torch.from_numpy(ps.offsets)
            vals.append(v.to(dev))
            offs.append(o[1:].to(dev) + base)
            base += int(o[-1])
        return PackedSeries(torch.cat(vals), torch.cat(offs), max(int(ps.max_len) for ps in series))

    return PackedFleet(cat([p.cpu for p in parts]), cat([p.mem for p in parts]))


def _pinned_alloc_or_none():
    """Page-locked packer output when a HIP device is present (the kernels need one anyway)."""
    try:
        import torch

        if torch.cuda.is_available():
            from krr_amd.core.engine import pinned_alloc

            return pinned_alloc
    except ImportError:  # pragma: no cover
        pass
    return None


def to_allocations(result: RunResult) -> ResourceAllocations:
    return ResourceAllocations(
        requests={rt: result[rt].request for rt in ResourceType},
        limits={rt: result[rt].limit for rt in ResourceType},
    )


__all__ = ["BatchedRunner", "HistoryLoader", "to_allocations"]
