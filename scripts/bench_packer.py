"""Host packer throughput: native libkrr_pack (JSON bodies -> CSR) vs the reference's
per-pod path (json.loads + Decimal(value), prometheus.py:147-155).

usage: python scripts/bench_packer.py [--objects 300] [--pods 3] [--samples 10080] [--threads 0]
Prints one JSON line: samples/s for each path and the speed-up.
"""
import argparse
import json
import os
import sys
import time
from decimal import Decimal

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=300)
    ap.add_argument("--pods", type=int, default=3)
    ap.add_argument("--samples", type=int, default=10080)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--objects-per-group", type=int, default=10,
                    help="objects sharing one (namespace, container): one grouped query for all their pods")
    ap.add_argument("--ref-objects", type=int, default=20, help="objects timed through the reference path")
    a = ap.parse_args()
    from krr_amd.core.prom_native import pack_query_range_bodies

    rng = np.random.default_rng(0)
    per_obj = []
    for o in range(a.objects):
        pods = []
        for p in range(a.pods):
            xs = rng.gamma(2.0, 0.05, size=a.samples)
            ts = 1.7e9 + 60.0 * np.arange(a.samples)
            doc = {"status": "success", "data": {"resultType": "matrix", "result": [
                {"metric": {"namespace": "default", "pod": f"pod-{o}-{p}", "container": "app"},
                 "values": [[float(t), repr(float(x))] for t, x in zip(ts, xs)]}]}}
            pods.append(json.dumps(doc).encode())
        per_obj.append(pods)
    nbytes = sum(len(b) for pods in per_obj for b in pods)
    total = a.objects * a.pods * a.samples
    t0 = time.perf_counter()
    ps = pack_query_range_bodies(per_obj, threads=a.threads)
    t1 = time.perf_counter()
    ps1 = pack_query_range_bodies(per_obj, threads=1)
    t2 = time.perf_counter()
    assert ps.values.size == total and np.array_equal(ps.values, ps1.values)
    # the reference's path on a subset
    sub = per_obj[: a.ref_objects]
    t3 = time.perf_counter()
    n_ref = 0
    for pods in sub:
        for b in pods:
            res = json.loads(b)["data"]["result"]
            if res:
                vals = [Decimal(v) for _, v in res[0]["values"]]
                n_ref += len(vals)
    t4 = time.perf_counter()
    # fleet-batched form: one `sum by (pod)` body per (namespace, container) group
    from krr_amd.core.fleet_query import FleetQueryPlan

    class Obj:
        def __init__(self, o):
            self.namespace, self.container = "default", f"app-{o // a.objects_per_group}"
            self.pods = [f"pod-{o}-{p}" for p in range(a.pods)]

    objs = [Obj(o) for o in range(a.objects)]
    plan = FleetQueryPlan(objs)
    where = {(objs[o].container, pod): json.loads(b)["data"]["result"][0]
             for o, pods in enumerate(per_obj) for pod, b in zip(objs[o].pods, pods)}
    gbodies = [json.dumps({"status": "success", "data": {"resultType": "matrix", "result": [
        where[(g.container, pod)] for pod in reversed(g.pods)]}}).encode() for g in plan.groups]
    del where
    t5 = time.perf_counter()
    pg = plan.pack(gbodies, threads=a.threads)
    t6 = time.perf_counter()
    assert pg.values.tobytes() == ps.values.tobytes() and np.array_equal(pg.offsets, ps.offsets)
    threads = a.threads or os.cpu_count()
    out = {
        "grouped_queries": len(plan.groups), "per_pod_queries": a.objects * a.pods,
        "grouped_native_samples_per_s": total / (t6 - t5),
        "samples": total, "json_bytes": nbytes,
        "native_samples_per_s": total / (t1 - t0), "native_threads": threads,
        "native_1thread_samples_per_s": total / (t2 - t1),
        "native_GB_per_s": nbytes / (t1 - t0) / 1e9,
        "reference_path_samples_per_s": n_ref / (t4 - t3), "reference_path_threads": 1,
        "speedup_vs_reference_path": (total / (t1 - t0)) / (n_ref / (t4 - t3)),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
