"""Hybrid parse A/B (GPU): BatchedRunner.recommend_from_bodies on bench.py's host-path fleet
(2,000 config-1-shaped objects) with parser='device' and parser='hybrid' at several staging
thread counts; best of 3 after the share settles.
With --strip 0,1 the sweep runs with the device packer's staging copy plain and with the
timestamps cut (krr_amd/csrc/krr_strip.h).
usage: python scripts/hybrid_probe.py [--objects 2000] [--threads 16] [--dev-threads 2,3,4,6] [--strip 0,1]"""
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
    ap.add_argument("--strip", default="1")
    ap.add_argument("--cores", action="store_true", help="with --numa: one hardware thread per core")
    ap.add_argument("--numa", action="store_true", help="bind to the GPU-local NUMA node first (krr_amd.utils.numa)")
    ap.add_argument("--fixed-shares", default="", help="e.g. 0.05,0.1: time these host shares as set, no settling")
    a = ap.parse_args()
    if a.numa:
        from krr_amd.utils.numa import bind_local, gpu_numa_node

        cpus = bind_local(0, one_per_core=a.cores)
        print(f"numa: GPU 0 on node {gpu_numa_node(0)}, bound to {len(cpus) if cpus else 0} CPUs", flush=True)
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

    from krr_amd.core.device_pack import default_packer

    packer = default_packer(0)
    for strip in [int(x) for x in a.strip.split(",")]:
        packer.strip = bool(strip)
        td = best("device")
        up = packer.last_upload or {}
        print(f"strip={strip} device: {a.objects / td:.0f} objects/s ({td * 1e3:.1f} ms), link bytes "
              f"{up.get('bytes_sent', 0) / max(up.get('bytes', 1), 1):.3f} of the JSON", flush=True)
        if a.fixed_shares:
            for d in [int(x) for x in a.dev_threads.split(",")]:
                runner.hybrid_device_threads = d
                for sh in [float(x) for x in a.fixed_shares.split(",")]:
                    t = float("inf")
                    for _ in range(4):
                        runner.hybrid_share = sh
                        t0 = time.perf_counter()
                        runner.recommend_from_bodies(cpu_b, mem_b, threads=a.threads, parser="hybrid")
                        t = min(t, time.perf_counter() - t0)
                    h = runner.hybrid_last
                    print(f"strip={strip} fixed share {sh:.2f} dev_threads={d}: {a.objects / t:.0f} objects/s "
                          f"({t * 1e3:.1f} ms), device {h['device_s'] * 1e3:.1f} ms {h['device_GBps']:.1f} GB/s, "
                          f"host {h['host_s'] * 1e3:.1f} ms {h['host_GBps']:.1f} GB/s", flush=True)
            continue
        for d in [int(x) for x in a.dev_threads.split(",")]:
            runner.hybrid_device_threads = d
            runner.hybrid_share = 0.2
            for _ in range(5):  # the share settles
                runner.recommend_from_bodies(cpu_b, mem_b, threads=a.threads, parser="hybrid")
            th = best("hybrid")
            h = runner.hybrid_last
            print(f"strip={strip} hybrid dev_threads={d}: {a.objects / th:.0f} objects/s ({th * 1e3:.1f} ms, "
                  f"+{td / th - 1:.1%}), share {h['share']:.3f}, device {h['device_s'] * 1e3:.1f} ms "
                  f"{h['device_GBps']:.1f} GB/s, host {h['host_s'] * 1e3:.1f} ms {h['host_GBps']:.1f} GB/s", flush=True)

if __name__ == "__main__":
    main()
