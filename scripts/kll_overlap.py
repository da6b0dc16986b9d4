"""GPU probe: does pipelining the KLL body pass and the tail pass over pieces of the series,
on two streams, beat running them one after the other?  The body pass (k_kll_build<false>) is
VALU-bound at ~60% of HBM peak, the tail pass (k_kll_tail) streams at ~74%; with pieces, the tail
of piece j can share the CUs with the body of piece j+1.  Rows must be identical either way.

usage: python scripts/kll_overlap.py [--series 20000] [--pieces 2 4 8 16] [--rounds 5]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from krr_amd import _native  # noqa: E402
from krr_amd.core.sketch import KllConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--series", type=int, default=20000)
    ap.add_argument("--length", type=int, default=172_800)
    ap.add_argument("--tail", type=int, default=1792)
    ap.add_argument("--pieces", type=int, nargs="+", default=[2, 4, 8, 16])
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    S, L = a.series, a.length
    ctx = _native.Context(0)
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    vals = torch.empty(S * L, dtype=torch.float64, device=dev)
    ctx.synth_fill_window(vals, offs, 1000003 * 6, 0, 0, False, 0, L)
    cfg = KllConfig(budget=512, tail=a.tail)
    kp = cfg.params(0)
    kb = cfg.params(0)
    kb.reserved |= _native.KRR_KLL_BODY_ONLY
    rw = cfg.row_words
    A = torch.cuda.current_stream(dev)
    B = torch.cuda.Stream(dev)
    whole = ctx.series(vals, offs, L, False)

    def sequential(rows):
        ctx.kll_build(whole, kp, rows, seg_base=0, stream=A)

    def pipelined(rows, P):
        bounds = [S * j // P for j in range(P + 1)]
        B.wait_stream(A)
        for j in range(P):
            lo, hi = bounds[j], bounds[j + 1]
            ser = ctx.series(vals, offs[lo:hi + 1], L, False)
            ctx.kll_build(ser, kb, rows[lo:hi], seg_base=lo, stream=A)
            ev = torch.cuda.Event()
            ev.record(A)
            B.wait_event(ev)
            ctx.kll_tail(ser, kp, rows[lo:hi], stream=B)
        A.wait_stream(B)

    ref = torch.empty((S, rw), dtype=torch.int64, device=dev)
    variants = [("sequential", lambda r: sequential(r))] + [(f"pieces={P}", (lambda P: lambda r: pipelined(r, P))(P))
                                                            for P in a.pieces]
    rows = {name: torch.empty((S, rw), dtype=torch.int64, device=dev) for name, _ in variants}
    times = {name: [] for name, _ in variants}
    for r in range(a.rounds + 1):
        for name, fn in variants:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn(rows[name])
            torch.cuda.synchronize()
            if r:
                times[name].append((time.perf_counter() - t0) * 1e3)
    sequential(ref)
    torch.cuda.synchronize()
    nbytes = 2 * 8 * S * L  # two passes over the slice
    for name, _ in variants:
        ms = sorted(times[name])[len(times[name]) // 2]
        print(f"{name}: median {ms:.3f} ms over {a.rounds} rounds ({nbytes / (ms * 1e-3) / 1e9:.0f} GB/s of the two passes' "
              f"reads), rows == sequential: {bool(torch.equal(rows[name], ref))}", flush=True)


if __name__ == "__main__":
    main()
