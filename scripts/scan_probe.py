"""Right-size / scan cost on the host this runs on (no GPU): allocations_batch + collect_result
over N synthetic config-4 records, with the native module loaded from a variant path (profiling
builds of krr_amd/csrc/krr_pydec.cpp: KRR_X_NOSEV, KRR_X_NODICT), best of 3.
usage: python scripts/scan_probe.py VARIANT_DIR [--n 1000000]"""
import argparse
import gc
import importlib.machinery
import importlib.util
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variant")
    ap.add_argument("--n", type=int, default=1_000_000)
    a = ap.parse_args()
    from krr_amd.core import packing

    path = os.path.join(a.variant, "_krr_pydec.so")
    loader = importlib.machinery.ExtensionFileLoader("_krr_pydec", path)
    spec = importlib.util.spec_from_file_location("_krr_pydec", path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    packing._PYDEC = mod
    import bench
    from krr_amd.core.distributed import raw_from_records
    from krr_amd.core.fast_round import allocations_batch
    from krr_amd.core.models.result import collect_result
    from krr_amd.strategies.simple import SimpleStrategySettings
    from test_bench_right_size import _records

    objs = bench.fleet_objects(a.n)
    st = SimpleStrategySettings(cpu_percentile="99", memory_buffer_percentage="5")
    raw = raw_from_records(_records(a.n))
    collect_result(objs[:1000], allocations_batch(raw_from_records(_records(1000)), st, threads=16))
    gc.collect()
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        al = allocations_batch(raw, st, threads=16)
        t1 = time.perf_counter()
        r = collect_result(objs, al)
        t2 = time.perf_counter()
        cur = (t2 - t0, t1 - t0, t2 - t1)
        best = cur if best is None or cur[0] < best[0] else best
        del r, al
        gc.collect()
    print(f"{os.path.basename(a.variant)}: right-size {best[0]:.3f} s (allocations {best[1]:.3f}, scan {best[2]:.3f}) "
          f"for {a.n} objects", flush=True)


if __name__ == "__main__":
    main()
