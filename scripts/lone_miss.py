"""What one window miss costs a launch: the config-4 shape (100k x 10,080 compact, p50) with
and without a few regime-change series (the rank estimate from the first part of such a
series misses the window, the segment goes to the miss pass: one wave, two passes).
usage: python scripts/lone_miss.py [--bad 1] [--length 10080]
"""
import argparse
import os
import sys
from decimal import Decimal

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--containers", type=int, default=100_000)
    ap.add_argument("--length", type=int, default=10080)
    ap.add_argument("--bad", type=int, nargs="+", default=[0, 1, 4, 16])
    ap.add_argument("--percentile", default="50")
    a = ap.parse_args()
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    S, L = a.containers, a.length
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    cpu = torch.empty(S * L, dtype=torch.float64, device=dev)
    mem = torch.empty(S * L, dtype=torch.float64, device=dev)
    ctx.synth_fill(cpu, offs, 7, 0, 0, False)
    ctx.synth_fill(mem, offs, 8, 1, 0, False)
    regime = torch.from_numpy(np.concatenate([np.random.default_rng(1).random(int(0.6 * L)),
                                              np.random.default_rng(2).random(L - int(0.6 * L)) + 10.0])).to(dev)
    saved = cpu[: max(a.bad) * L].clone()
    params = percentile_params(Decimal(a.percentile), "linear")
    cs, ms = ctx.series(cpu, offs, L, False), ctx.series(mem, offs, L, False)
    out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
           (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
            ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
    for nb in a.bad:
        cpu[: max(a.bad) * L] = saved
        for j in range(nb):  # spread over the launch: every 100k / nb-th series
            s = (j * S) // max(nb, 1)
            cpu[s * L:(s + 1) * L] = regime
        torch.cuda.synchronize()
        f0 = ctx.wselect_fallbacks()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ctx.simple_run(cs, ms, params, out)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        f1 = ctx.wselect_fallbacks()
        print(f"{nb:3d} regime-change series: fused {np.median(ts):.4f} ms, misses/launch {(f1 - f0) / 7:.1f}",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
