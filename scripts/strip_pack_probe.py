"""Where the stripped device pack's time goes (GPU): DevicePacker.pack_many on bench.py's
host-path bodies (both resources), strip off / on, at several chunk sizes and runs per thread;
the C strip calls, the copy enqueues and the rest of the pipeline timed apart.
usage: python scripts/strip_pack_probe.py [--objects 2000] [--threads 16]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=2000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--cores", action="store_true", help="with --numa: one hardware thread per core")
    ap.add_argument("--numa", action="store_true")
    ap.add_argument("--only", default="", help="strip,chunk_mib,runs_per_thread: one configuration (for traces)")
    a = ap.parse_args()
    import torch

    if a.numa:
        from krr_amd.utils.numa import bind_local, gpu_numa_node

        cpus = bind_local(0, one_per_core=a.cores)
        print(f"numa: GPU 0 on node {gpu_numa_node(0)}, bound to {len(cpus) if cpus else 0} CPUs", flush=True)
    from bench import body_fleet
    from krr_amd import _native
    from krr_amd.core.device_pack import DevicePacker
    from krr_amd.core.prom_native import load_library

    _, _, cpu_b, mem_b = body_fleet(0, a.objects)
    ctx = _native.Context(0)
    host = load_library()
    raw_strip, raw_concat = host.krr_pack_concat_strip, host.krr_pack_concat
    acc = {"c": 0.0, "n": 0}

    def timed(f):
        def g(*args):
            t0 = time.perf_counter()
            r = f(*args)
            acc["c"] += time.perf_counter() - t0
            acc["n"] += 1
            return r
        return g

    host.krr_pack_concat_strip = timed(raw_strip)
    host.krr_pack_concat = timed(raw_concat)
    if a.only:
        s0, c0, r0 = (int(x) for x in a.only.split(","))
        configs = [(s0, c0, r0)]
    else:
        configs = [(s, c, r) for s in (0, 1) for c in (64, 256, 1024) for r in ((1, 2, 4) if s else (2,))]
    for strip, chunk, rpt in configs:
        if True:
            if True:
                p = DevicePacker(ctx, chunk_bytes=chunk << 20, threads=a.threads, strip=bool(strip))
                p.strip_runs_per_thread = rpt
                p.pack_many([cpu_b[:8], mem_b[:8]])
                best = None
                for _ in range(3):
                    acc["c"], acc["n"] = 0.0, 0
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    p.pack_many([cpu_b, mem_b])
                    torch.cuda.synchronize()
                    t = time.perf_counter() - t0
                    if best is None or t < best[0]:
                        best = (t, acc["c"], acc["n"])
                up = p.last_upload
                print(f"strip={strip} chunk={chunk:5d} MiB runs/thread={rpt}: pack {best[0] * 1e3:6.1f} ms "
                      f"({up['bytes'] / best[0] / 1e9:5.1f} GB/s of JSON), staging calls {best[1] * 1e3:6.1f} ms "
                      f"x{best[2]}, sent {up['bytes_sent'] / up['bytes']:.3f}", flush=True)


if __name__ == "__main__":
    main()
