"""PCIe-inclusive rate of the config-2 step: series in page-locked HOST memory, moved to HBM
chunk by chunk and reduced by the fused launch (`krr_simple_run_records`), records back to host.

Two schedules over the same chunks:
  serial     - H2D(chunk) -> kernel(chunk) -> records D2H, one stream;
  pipelined  - H2D of chunk i+1 on a copy stream overlaps chunk i's kernel (double-buffered).
Plus the device-resident rate of the same chunks (the bench.py `value` definition) for scale.
This is NOT bench.py's `value` (inputs already resident in HBM); DESIGN.md §4 quotes it.
usage: python scripts/bench_pcie.py [--containers 4000] [--chunk 500] [--reps 3]
"""
import argparse
import json
import os
import sys
import time
from decimal import Decimal

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--containers", type=int, default=4000)
    ap.add_argument("--chunk", type=int, default=500)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    dev = torch.device("cuda", 0)
    L, C = 5 * 10080, a.chunk
    n_chunks = a.containers // C
    n = n_chunks * C
    ctx = _native.Context(0)
    offs = torch.arange(C + 1, dtype=torch.int64, device=dev) * L
    # synthesise chunk by chunk on the device, park it in page-locked host memory
    host_cpu = torch.empty(n * L, dtype=torch.float64, pin_memory=True)
    host_mem = torch.empty(n * L, dtype=torch.float64, pin_memory=True)
    bufs = [(torch.empty(C * L, dtype=torch.float64, device=dev), torch.empty(C * L, dtype=torch.float64, device=dev))
            for _ in range(2)]
    for i in range(n_chunks):
        cpu, mem = bufs[0]
        ctx.synth_fill(cpu, offs, 7 + i, 0, 10080, True)
        ctx.synth_fill(mem, offs, 8 + i, 1, 10080, True)
        host_cpu[i * C * L:(i + 1) * C * L].copy_(cpu)
        host_mem[i * C * L:(i + 1) * C * L].copy_(mem)
    torch.cuda.synchronize()
    params = percentile_params(Decimal("99"), "linear")
    out = {k: torch.empty(C, dtype=dt, device=dev) for k, dt in
           (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
            ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
    rec = torch.empty(C, 4, dtype=torch.int64, device=dev)
    rec_host = torch.empty(n, 4, dtype=torch.int64, pin_memory=True)
    series = [(ctx.series(c, offs, L, True), ctx.series(m, offs, L, True)) for c, m in bufs]
    compute = torch.cuda.current_stream()
    copy = torch.cuda.Stream()

    def h2d(i, b, stream):
        with torch.cuda.stream(stream):
            bufs[b][0].copy_(host_cpu[i * C * L:(i + 1) * C * L], non_blocking=True)
            bufs[b][1].copy_(host_mem[i * C * L:(i + 1) * C * L], non_blocking=True)

    def run(i, b):
        ctx.simple_run(series[b][0], series[b][1], params, out, stream=compute, records=rec)
        rec_host[i * C:(i + 1) * C].copy_(rec, non_blocking=True)

    def serial():
        for i in range(n_chunks):
            h2d(i, 0, compute)
            run(i, 0)

    def pipelined():
        ready = [torch.cuda.Event(), torch.cuda.Event()]
        free = [torch.cuda.Event(), torch.cuda.Event()]
        h2d(0, 0, copy)
        ready[0].record(copy)
        for i in range(n_chunks):
            b = i & 1
            if i + 1 < n_chunks:
                copy.wait_event(free[b ^ 1]) if i >= 1 else None
                h2d(i + 1, b ^ 1, copy)
                ready[b ^ 1].record(copy)
            compute.wait_event(ready[b])
            run(i, b)
            free[b].record(compute)

    def resident():
        for i in range(n_chunks):
            run(i, i & 1)

    res = {}
    for name, fn in (("serial", serial), ("pipelined", pipelined), ("resident", resident)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = sorted(ts)[len(ts) // 2]
        res[name] = {"s": t, "containers_per_s": n / t, "host_GB_per_s": 2 * n * L * 8 / t / 1e9}
    print(json.dumps({"workload": f"config-2 shape from page-locked host memory: {n} containers x 5 pods x 10080 "
                                  f"slots per resource, chunks of {C}, linear p99 + max",
                      "bytes": 2 * n * L * 8, **res}))


if __name__ == "__main__":
    main()
