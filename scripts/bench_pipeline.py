"""Whole-job host+device pipeline, stage by stage: Prometheus query_range bodies ->
native CSR packer -> H2D -> fused kernel -> D2H -> native exact-decimal rounding ->
RunResults.  Compared with the reference's per-object path (json + Decimal +
SimpleStrategy.run + _format_result) timed on a small sample of the same objects.

usage: python scripts/bench_pipeline.py [--objects 2000] [--pods 3] [--samples 10080]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=2000)
    ap.add_argument("--pods", type=int, default=3)
    ap.add_argument("--samples", type=int, default=10080)
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    import torch

    from krr_amd.core.fast_round import format_simple_batch
    from krr_amd.core.packing import PackedFleet
    from krr_amd.core.prom_native import pack_query_range_bodies
    from krr_amd.strategies.simple import SimpleStrategySettings

    rng = np.random.default_rng(0)
    ts = [[1.7e9 + 60.0 * i, None] for i in range(a.samples)]

    tstr = [repr(t) for t, _ in ts]

    def body(xs):  # the query_range JSON Prometheus sends (values as shortest-repr strings)
        vals = ",".join(f'[{t},"{x!r}"]' for t, x in zip(tstr, xs.tolist()))
        return ('{"status":"success","data":{"resultType":"matrix","result":[{"metric":{"pod":"p"},"values":['
                + vals + ']}]}}').encode()

    t0 = time.perf_counter()
    cpu_b = [[body(rng.gamma(2.0, 0.05, a.samples)) for _ in range(a.pods)] for _ in range(a.objects)]
    mem_b = [[body(np.floor(rng.normal(2e8, 2e7, a.samples))) for _ in range(a.pods)] for _ in range(a.objects)]
    t_gen = time.perf_counter() - t0
    st = SimpleStrategySettings(cpu_percentile="99", memory_buffer_percentage="5")
    from krr_amd.core.engine import pinned_alloc

    # warm-up (context, module load, allocator) on a slice of the fleet
    st.run_fleet(PackedFleet(pack_query_range_bodies(cpu_b[:8]), pack_query_range_bodies(mem_b[:8])))
    torch.cuda.synchronize()
    runs = {}
    for name, alloc in (("pageable", None), ("pinned", pinned_alloc)):
        t0 = time.perf_counter()
        fleet = PackedFleet(pack_query_range_bodies(cpu_b, threads=a.threads, alloc=alloc),
                            pack_query_range_bodies(mem_b, threads=a.threads, alloc=alloc))
        t1 = time.perf_counter()
        raw = st.run_fleet(fleet)  # H2D + fused kernel + D2H
        t2 = time.perf_counter()
        res = format_simple_batch(raw, st, threads=a.threads)
        t3 = time.perf_counter()
        runs[name] = ({"pack_ms": (t1 - t0) * 1e3, "device_ms": (t2 - t1) * 1e3, "round_ms": (t3 - t2) * 1e3},
                      t3 - t0)
        del fleet
    stages, total = runs["pinned"]
    stages["pageable_device_ms"] = runs["pageable"][0]["device_ms"]
    samples = 2 * a.objects * a.pods * a.samples
    # the reference's per-object path on a sample: json + Decimal + strategy + rounding
    from decimal import Decimal

    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.rounding import format_result

    m = min(20, a.objects)
    r0 = time.perf_counter()
    for o in range(m):
        hist = {}
        for rt, bodies in ((ResourceType.CPU, cpu_b[o]), (ResourceType.Memory, mem_b[o])):
            data = {}
            for i, b in enumerate(bodies):
                r = json.loads(b)["data"]["result"]
                if r:
                    data[f"p{i}"] = [Decimal(v) for _, v in r[0]["values"]]
            hist[rt] = data
        cpu_d = [x for v in hist[ResourceType.CPU].values() for x in v]
        mem_d = [x for v in hist[ResourceType.Memory].values() for x in v]
        cpu = cpu_d[int((len(cpu_d) - 1) * Decimal(99) / 100)]
        mem = max(mem_d) * Decimal(1 + Decimal(5) / 100)
        from krr_amd.core.abstract.strategies import ResourceRecommendation

        format_result({ResourceType.CPU: ResourceRecommendation(request=cpu, limit=None),
                       ResourceType.Memory: ResourceRecommendation(request=mem, limit=mem)})
    ref_s = (time.perf_counter() - r0) / m
    print(json.dumps({
        "objects": a.objects, "pods": a.pods, "samples_per_pod": a.samples, "total_samples": samples,
        "pipeline_objects_per_s": a.objects / total, "pipeline_samples_per_s": samples / total,
        "stages": stages, "host_threads": a.threads or os.cpu_count(),
        "reference_path_objects_per_s": 1.0 / ref_s, "reference_path_sample": m,
        "speedup": (a.objects / total) * ref_s, "json_gen_s": t_gen, "results": len(res)}))


if __name__ == "__main__":
    main()
