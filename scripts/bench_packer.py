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
    threads = a.threads or os.cpu_count()
    out = {
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
