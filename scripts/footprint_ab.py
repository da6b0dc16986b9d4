"""Why big fleets stream slower on one GPU (config 4 at N = 1: 83.6% of peak at 700k
containers against 89.4% at 125k): the fused launch over the whole fleet, the same fleet
cut into launches of `--chunk` containers, and single chunks taken from the start and the
end of the allocation.  Offsets are absolute indices into the value buffers, so a chunk is
just a slice of the offsets.
usage: python scripts/footprint_ab.py [--containers 700000] [--chunk 125000] [--rounds 5]
"""
import argparse
import os
import sys
from decimal import Decimal

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--containers", type=int, default=700_000)
    ap.add_argument("--chunk", type=int, default=125_000)
    ap.add_argument("--length", type=int, default=10080)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--percentile", default="99")
    ap.add_argument("--separate", action="store_true",
                    help="allocate every chunk as buffers of its own instead of slicing one allocation")
    a = ap.parse_args()
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    dev = torch.device("cuda", 0)
    ctx = _native.Context(0)
    S, L = a.containers, a.length
    params = percentile_params(Decimal(a.percentile), "linear")
    stream = torch.cuda.current_stream()
    cuts = list(range(0, S, a.chunk)) + [S]
    out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
           (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
            ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
    if a.separate:  # one (cpu, mem, offsets) triple per chunk; chunk c = global containers [lo, hi)
        bufs = {}
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            o = torch.arange(hi - lo + 1, dtype=torch.int64, device=dev) * L
            c = torch.empty((hi - lo) * L, dtype=torch.float64, device=dev)
            m = torch.empty((hi - lo) * L, dtype=torch.float64, device=dev)
            ctx.synth_fill(c, o, 7, 0, 0, False, seg_base=lo)
            ctx.synth_fill(m, o, 8, 1, 0, False, seg_base=lo)
            bufs[(lo, hi)] = (c, m, o)
    else:
        offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
        cpu = torch.empty(S * L, dtype=torch.float64, device=dev)
        mem = torch.empty(S * L, dtype=torch.float64, device=dev)
        ctx.synth_fill(cpu, offs, 7, 0, 0, False)
        ctx.synth_fill(mem, offs, 8, 1, 0, False)
    torch.cuda.synchronize()

    def launch(lo, hi):
        if a.separate:
            c, m, o = bufs[(lo, hi)]
        else:
            c, m, o = cpu, mem, offs[lo:hi + 1]
        cs, ms = ctx.series(c, o, L, False), ctx.series(m, o, L, False)
        ctx.simple_run(cs, ms, params, {k: v[lo:hi] for k, v in out.items()}, stream)

    variants = {} if a.separate else {"whole": [(0, S)]}
    variants.update({
        f"chunks_of_{a.chunk}": list(zip(cuts[:-1], cuts[1:])),
        "first_chunk_only": [(0, min(a.chunk, S))],
        "last_chunk_only": [(cuts[-2], S)],
    })
    times = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, ranges in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for lo, hi in ranges:
                launch(lo, hi)
            e1.record(stream)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1))
    for k, ranges in variants.items():
        n = sum(hi - lo for lo, hi in ranges)
        by = 2 * (8 * n * L + 8 * (n + 1) + 20 * n)
        t = float(np.median(times[k]))
        print(f"{k:22s} {len(ranges):3d} launch(es) {n:8d} containers {t:9.3f} ms  {by / t / 1e6:6.0f} GB/s "
              f"({by / t / 1e6 / 8000:.1%})", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
