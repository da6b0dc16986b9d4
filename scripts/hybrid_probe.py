"""Hybrid parse A/B (GPU): BatchedRunner.recommend_from_bodies on bench.py's host-path fleet
(2,000 config-1-shaped objects) with parser='device' and parser='hybrid' at several staging
thread counts; best of 3 after the share settles.
usage: python scripts/hybrid_probe.py [--objects 2000] [--threads 16] [--dev-threads 2,3,4,6]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=2000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dev-threads", default="2,3,4,6")
    a = ap.parse_args()
    from bench import body_fleet
    from krr_amd.core.runner import BatchedRunner
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    _, _, cpu_b, mem_b = body_fleet(0, a.objects)
    runner = BatchedRunner(SimpleStrategy(SimpleStrategySettings(cpu_percentile=99, memory_buffer_percentage=5)))

    def best(parser, n=3):
        runner.recommend_from_bodies(cpu_b, mem_b, threads=a.threads, parser=parser)
        t = float("inf")
        for _ in range(n):
            t0 = time.perf_counter()
            runner.recommend_from_bodies(cpu_b, mem_b, threads=a.threads, parser=parser)
            t = min(t, time.perf_counter() - t0)
        return t

    td = best("device")
    print(f"device: {a.objects / td:.0f} objects/s ({td * 1e3:.1f} ms)", flush=True)
    for d in [int(x) for x in a.dev_threads.split(",")]:
        runner.hybrid_device_threads = d
        runner.hybrid_share = 0.2
        for _ in range(5):  # the share settles
            runner.recommend_from_bodies(cpu_b, mem_b, threads=a.threads, parser="hybrid")
        th = best("hybrid")
        h = runner.hybrid_last
        print(f"hybrid dev_threads={d}: {a.objects / th:.0f} objects/s ({th * 1e3:.1f} ms, +{td / th - 1:.1%}), "
              f"share {h['share']:.3f}, device {h['device_s'] * 1e3:.1f} ms {h['device_GBps']:.1f} GB/s, "
              f"host {h['host_s'] * 1e3:.1f} ms {h['host_GBps']:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
