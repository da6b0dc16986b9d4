"""Minimal driver for rocprofv3 passes: generate one workload on the device, then
run the percentile and max kernels `--reps` times (nothing else on the GPU)."""
import argparse
import os
import sys
from decimal import Decimal

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="linear")
    ap.add_argument("--percentile", default="99")
    ap.add_argument("--containers", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--separate", action="store_true")
    a = ap.parse_args()
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    n = a.containers
    if a.config == 5:  # sketch build over 30d@15s series (bench.py config 5 at N=1)
        from krr_amd.core import sketch

        T = 172_800
        offs = torch.arange(n + 1, dtype=torch.int64, device=dev) * T
        x = torch.empty(n * T, dtype=torch.float64, device=dev)
        ctx.synth_fill_window(x, offs, 1000003 * 6, 0, 0, False, 0, T)
        ser = ctx.series(x, offs, T, False)
        cfg = sketch.SketchConfig()
        for _ in range(a.reps):
            sketch.build(ctx, ser, cfg)
        torch.cuda.synchronize()
        print("done", n, n * T)
        return
    if a.config == 2:
        L, pod_len, gaps = 5 * 10080, 10080, True
        offs_np = np.arange(n + 1, dtype=np.int64) * L
    else:
        rng = np.random.default_rng(3)
        Ls = rng.integers(1, 15, size=n) * 1440
        offs_np = np.concatenate([[0], np.cumsum(Ls)]).astype(np.int64)
        pod_len, gaps = 0, False
    offs = torch.from_numpy(offs_np).to(dev)
    N = int(offs_np[-1])
    cpu = torch.empty(N, dtype=torch.float64, device=dev)
    mem = torch.empty(N, dtype=torch.float64, device=dev)
    ctx.synth_fill(cpu, offs, 7, 0, pod_len, gaps)
    ctx.synth_fill(mem, offs, 8, 1, pod_len, gaps)
    S = n
    maxlen = int(np.max(np.diff(offs_np)))
    cs = ctx.series(cpu, offs, maxlen, gaps)
    ms = ctx.series(mem, offs, maxlen, gaps)
    ov = torch.empty(S, dtype=torch.float64, device=dev)
    on = torch.empty(S, dtype=torch.int64, device=dev)
    of = torch.empty(S, dtype=torch.int32, device=dev)
    params = percentile_params(Decimal(a.percentile), a.mode)
    out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
           (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
            ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
    for _ in range(a.reps):
        if a.separate:
            ctx.segmented_percentile(cs, params, ov, on, of)
            ctx.segmented_max(ms, ov, on, of)
        else:
            ctx.simple_run(cs, ms, params, out)
    torch.cuda.synchronize()
    print("done", S, N)


if __name__ == "__main__":
    main()
