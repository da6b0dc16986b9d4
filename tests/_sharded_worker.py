"""One rank of the multi-GPU BatchedRunner tests (started as a fresh interpreter per rank
by tests/test_distributed.py and tests/test_gpu_multirank.py; RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT come from the environment, backend gloo).

    python tests/_sharded_worker.py --compute oracle|gpu --entry packed|loader --path cli_99_5 --out rows.json

--compute oracle: the per-rank kernel pass is stood in for by the CPU oracle (test
infrastructure, so the sharding / gather / rounding logic runs on a GPU-less host);
--compute gpu: the real HIP path (ranks may share one GPU: LOCAL_RANK modulo devices).
Rank 0 writes the rounded rows of the whole config-1 fleet to --out.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(HERE, "golden"))

import numpy as np  # noqa: E402


def _oracle_records(settings, fleet):
    import torch

    from oracle import oracle

    p = settings.params()
    cv, cn, cf = oracle.percentile(fleet.cpu.values, fleet.cpu.offsets, p.mode, p.p_num, p.p_den, p.q,
                                   fleet.cpu.gaps_are_nan)
    mv, mn, mf = oracle.seg_max(fleet.mem.values, fleet.mem.offsets, fleet.mem.gaps_are_nan)
    rec = np.stack([cv.view(np.int64), mv.view(np.int64),
                    cn.astype(np.int64) | (cf.astype(np.int64) << 48),
                    mn.astype(np.int64) | (mf.astype(np.int64) << 48)], axis=1)
    return torch.from_numpy(np.ascontiguousarray(rec))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--compute", choices=("oracle", "gpu"), required=True)
    ap.add_argument("--entry", choices=("packed", "loader", "bodies", "exact"), default="packed")
    ap.add_argument("--path", default="cli_99_5")
    ap.add_argument("--out", required=True)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import config1
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.models.objects import K8sObjectData
    from krr_amd.core.packing import PackedFleet, PackedSeries
    from krr_amd.core.runner import BatchedRunner
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings
    from krr_amd.utils.prom_decimal import prom_format

    if args.compute == "oracle":
        SimpleStrategySettings.run_fleet_records = lambda self, fleet, device=None: _oracle_records(self, fleet)
        from _standin import oracle_run_packed
        from krr_amd.core.engine import SimpleEngine

        SimpleEngine.run_packed = oracle_run_packed  # the exact-HistoryData path (run_fleet + locate)
        SimpleEngine.context = lambda self: None
    else:
        from krr_amd.core.distributed import local_device

        torch.cuda.set_device(local_device())
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    kw = dict(cpu_percentile="99", memory_buffer_percentage="5") if args.path == "cli_99_5" else {}
    runner = BatchedRunner(SimpleStrategy(SimpleStrategySettings(**kw)))
    cpu, mem = config1.inputs()
    O, P, T = cpu.shape
    if args.entry == "exact":
        # HistoryData outside Prometheus' strings (tests/golden/simple_strategy_exact.json):
        # every rank packs the whole fleet and runs its shard; the sample objects resolved on
        # each rank must reach rank 0 (the reference returns the objects themselves)
        from decimal import Decimal

        with open(os.path.join(HERE, "golden", "simple_strategy_exact.json")) as fh:
            doc = json.load(fh)
        cases = [c for c in doc["cases"] if "rounded" in c["results"][args.path]]

        def hist(c):
            return {ResourceType.CPU: {k: [Decimal(x) for x in v] for k, v in c["cpu"].items() if v},
                    ResourceType.Memory: {k: [Decimal(x) for x in v] for k, v in c["mem"].items() if v}}

        fleet = runner.strategy.pack([hist(c) for c in cases])
        res = runner.recommend_packed_sharded(fleet)
        rows = None if res is None else [
            [str(r[ResourceType.CPU].request), str(r[ResourceType.Memory].request), str(r[ResourceType.Memory].limit)]
            for r in res]
    elif args.entry == "packed":
        offs = np.arange(0, O * P * T + 1, P * T, dtype=np.int64)
        fleet = PackedFleet(PackedSeries(cpu.reshape(-1).copy(), offs, P * T),
                            PackedSeries(mem.reshape(-1).copy(), offs.copy(), P * T))
        res = runner.recommend_packed_sharded(fleet)
        rows = None if res is None else [
            [str(r[ResourceType.CPU].request), str(r[ResourceType.Memory].request), str(r[ResourceType.Memory].limit)]
            for r in res]
    elif args.entry == "bodies":
        # every rank builds (as it would fetch) ONLY its shard's query_range bodies; the device
        # packer parses them on its GPU (--compute gpu), the host packer stands in otherwise
        class _O:
            def __init__(self, o):
                self.pods = config1.pod_names(o)

        lo, hi = BatchedRunner.body_shard_bounds([_O(o) for o in range(O)], dist.get_world_size())[rank]

        def body(xs):
            vals = ",".join(f'[{1700000000 + 60 * i},"{prom_format(float(x))}"]' for i, x in enumerate(xs))
            return ('{"status":"success","data":{"resultType":"matrix","result":[{"metric":{},"values":[' + vals +
                    ']}]}}').encode()

        cb = [[body(cpu[o, p]) for p in range(P)] for o in range(lo, hi)]
        mb = [[body(mem[o, p]) for p in range(P)] for o in range(lo, hi)]
        res = runner.recommend_bodies_shard(cb, mb, parser="device" if args.compute == "gpu" else "host")
        rows = None if res is None else [
            [str(r[ResourceType.CPU].request), str(r[ResourceType.Memory].request), str(r[ResourceType.Memory].limit)]
            for r in res]
    else:
        from decimal import Decimal

        from krr_amd.core.models.allocations import ResourceAllocations

        none = {ResourceType.CPU: None, ResourceType.Memory: None}
        objects = [K8sObjectData(cluster=None, name=f"app-{o:03d}", container="main", pods=config1.pod_names(o),
                                 namespace="default", kind="Deployment",
                                 allocations=ResourceAllocations(requests=none, limits=none)) for o in range(O)]
        index = {o.name: i for i, o in enumerate(objects)}
        fetched = []

        class Loader:  # what PrometheusLoader.gather_data returns, from the config-1 arrays
            async def gather_data(self, obj, resource, period, *, timeframe):
                i = index[obj.name]
                fetched.append(i)
                x = cpu if resource == ResourceType.CPU else mem
                return {pod: [Decimal(prom_format(float(v))) for v in x[i, p]] for p, pod in enumerate(obj.pods)}

        allocs = asyncio.run(runner.gather_objects_recommendations_sharded(objects, Loader()))
        # every rank fetched only its own shard
        counts = [None] * dist.get_world_size()
        dist.all_gather_object(counts, sorted(set(fetched)))
        if rank == 0:
            flat = sorted(i for c in counts for i in c)
            assert flat == list(range(O)), "shards must cover every object exactly once"
        rows = None if allocs is None else [
            [str(a.requests[ResourceType.CPU]), str(a.requests[ResourceType.Memory]),
             str(a.limits[ResourceType.Memory])] for a in allocs]
    if rank == 0:
        with open(args.out, "w") as fh:
            json.dump({"rows": rows, "world": dist.get_world_size()}, fh)
    else:
        assert rows is None
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
