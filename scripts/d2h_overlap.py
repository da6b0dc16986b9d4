"""What a records D2H costs beside the fused launch (rank 0 of an N-rank bench copies
N x 320 KB of gathered records to the host every step).

Config 2 (10k containers) fused launches back to back, each followed by a D2H copy
of `--mb` MB from HBM to page-locked host memory: (a) no copy, (b) the copy on the
launch stream (serial), (c) the copy on a second stream, overlapping the next launch, (d) the copy done by the
launch itself as its first work items (krr_simple_run_forward).
usage: python scripts/d2h_overlap.py [--mb 2.56] [--steps 20]
"""
import argparse
import os
import sys
import time
from decimal import Decimal

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, nargs="+", default=[0.32, 1.28, 2.56])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    S, L = 10000, 50400
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    cpu = torch.empty(S * L, dtype=torch.float64, device=dev)
    mem = torch.empty(S * L, dtype=torch.float64, device=dev)
    ctx.synth_fill(cpu, offs, 7, 0, 10080, True)
    ctx.synth_fill(mem, offs, 8, 1, 10080, True)
    cs, ms = ctx.series(cpu, offs, L, True), ctx.series(mem, offs, L, True)
    params = percentile_params(Decimal("99"), "linear")
    out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
           (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
            ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
    rec = torch.empty((S, 4), dtype=torch.int64, device=dev)
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def run(mode, nbytes):
        src = torch.zeros(max(nbytes // 8, 1), dtype=torch.int64, device=dev)
        dst = torch.empty_like(src, device="cpu").pin_memory()
        done = torch.cuda.Event()
        for _ in range(3):
            ctx.simple_run(cs, ms, params, out, main_s, records=rec)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ctx.simple_run(cs, ms, params, out, main_s, records=rec,
                           forward=(src, dst) if mode == "fwd" else None)
            if mode == "serial":
                dst.copy_(src, non_blocking=True)
            elif mode == "fwd":  # the next launch forwards the copy as its first work items
                pass
            elif mode == "side":
                done.record(main_s)
                with torch.cuda.stream(side):
                    side.wait_event(done)
                    dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3

    for mb in a.mb:
        nb = int(mb * 1e6)
        res = {m: [] for m in ("none", "serial", "side", "fwd")}
        for _ in range(a.rounds):
            for m in res:
                res[m].append(run(m, nb))
        print(f"{mb:.2f} MB D2H per step: " + ", ".join(f"{m} {np.median(v):.4f} ms/step" for m, v in res.items()),
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
