"""Same-process probes of the device packer's grouped pipeline on bench.py's grouped workload
(2,000 objects x 3 pods x 10,080 samples as 20-namespace `sum by (pod)` bodies).

    python scripts/grouped_probe.py [--rounds R]

Prints the pinned->HBM copy rate for several copy sizes and stream counts (torch copies and
the library's krr_copy_h2d_batch), then, per packer variant (edit `variants`: round 6 compared
pieces per thread, chunk sizes, routing modes and the pipeline thread this way), the median
seconds of pack_grouped_many (both resources, to a synchronised CSR in HBM, checked against the
host plan once) with the packer's last phase split and the cgroup's throttled periods."""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from krr_amd.core.device_pack import default_packer  # noqa: E402
from krr_amd.core.fleet_query import FleetQueryPlan  # noqa: E402
from krr_amd.strategies.simple import SimpleStrategySettings  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--objects", type=int, default=2000)
    args = ap.parse_args()
    objects, pods, distinct = args.objects, 3, 48
    from krr_amd.utils.numa import bind_local

    bind_local(0)  # as bench.py: the GPU's NUMA node
    threads = bench.cpu_lease()["threads"]
    cpu_vals, mem_vals, _, _ = bench.body_fleet(0, objects, pods, distinct)

    class _Obj:
        def __init__(self, o):
            self.namespace, self.container = f"ns{o % 20}", "main"
            self.pods = [f"pod-{o}-{i}" for i in range(pods)]

    plan = FleetQueryPlan.for_settings([_Obj(o) for o in range(objects)], SimpleStrategySettings())

    def grouped(vals, shift):
        out_b = []
        for gq in plan.groups:
            parts = [f'{{"metric":{{"pod":"{pod}"}},"values":[{vals[(i + shift) % distinct]}]}}'
                     for i, pod in enumerate(reversed(gq.pods))]
            out_b.append((bench.BODY_HEAD + ",".join(parts) + ']}}').encode())
        return out_b

    g_cpu, g_mem = grouped(cpu_vals, 0), grouped(mem_vals, 7)
    print(f"{len(plan.groups)} bodies per resource, {sum(map(len, g_cpu)) / 1e9:.2f} GB CPU JSON", flush=True)
    from krr_amd.core.device_pack import DevicePacker

    base = default_packer(0)
    want = (plan.pack(g_cpu).values, plan.pack(g_mem).values)
    # the packer's streams (copy stream at construction, 3 parse streams at the first grouped
    # call) come from torch's stream pool in order: k dummy streams first shift which hardware
    # queues (GPU_MAX_HW_QUEUES) they land on
    # the link alone: the bench's pinned->HBM rate with copies of several sizes, one stream
    n = 1 << 28
    src = torch.empty(n * 10, dtype=torch.uint8, pin_memory=True)
    src.fill_(1)
    dst = torch.empty(n * 10, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(4)]
    for piece in (4 << 20, 10 << 20, 32 << 20, 128 << 20):
        for ns in (1, 2, 4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i, a in enumerate(range(0, src.numel(), piece)):
                with torch.cuda.stream(streams[i % ns]):
                    dst[a:a + piece].copy_(src[a:a + piece], non_blocking=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"H2D {piece >> 20} MiB pieces on {ns} streams: {src.numel() / dt / 1e9:.1f} GB/s", flush=True)
    # the library's batch call (one hipMemcpyAsync per piece, as the packer issues them)
    from krr_amd.core.device_pack import default_packer as _dp

    ctx = _dp(0).ctx
    for piece in (10 << 20, 128 << 20):
        k = src.numel() // piece
        d = np.array([dst.data_ptr() + i * piece for i in range(k)], dtype=np.int64)
        s_ = np.array([src.data_ptr() + i * piece for i in range(k)], dtype=np.int64)
        b = np.full(k, piece, dtype=np.int64)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.copy_h2d_batch(d, s_, b, stream=streams[0])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"copy_h2d_batch {piece >> 20} MiB pieces: {k * piece / dt / 1e9:.1f} GB/s", flush=True)
    del src, dst
    res = {}
    variants = [(16, 1), (15, 1), (16, 2), (14, 1), (16, 1), (15, 1), (16, 2), (14, 1)]
    for st_, ppt in variants:
        packer = DevicePacker(base.ctx, threads=threads)
        packer.strip_threads, packer.pieces_per_thread = st_, ppt
        out = packer.pack_grouped_many([(plan, g_cpu), (plan, g_mem)])
        torch.cuda.synchronize()
        assert all(np.array_equal(o.series.values.cpu().numpy(), w) for o, w in zip(out, want))
        ts = []
        for r in range(args.rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            packer.pack_grouped_many([(plan, g_cpu), (plan, g_mem)])
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ph = packer.last_grouped_phases
        print(f"strip threads {st_} pieces/thread {ppt}: median {np.median(ts) * 1e3:.2f} ms "
              f"runs {[round(t * 1e3, 2) for t in sorted(ts)]} strip {ph.get('strip')} "
              f"join {ph.get('pipeline_join_s')}", flush=True)
        packer.release()
        del packer


if __name__ == "__main__":
    main()
