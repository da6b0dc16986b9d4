"""Same-process A/B of krr_kll_build across libkrr_amd build variants, on config-5-shaped data
(S series x L slots of the device synthetic CPU series, in one buffer).  Also the workload of
rocprofv3 --pmc passes on the KLL build kernel.
usage: python scripts/kll_probe.py lib1.so [lib2.so ...] [--series 20000] [--length 172800]
       [--budget 512] [--tail 1792] [--rounds 5] [--check]
--check compares every variant's rows with the first variant's (bit for bit)."""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--series", type=int, default=20000)
    ap.add_argument("--length", type=int, default=172_800)
    ap.add_argument("--budget", type=int, default=512)
    ap.add_argument("--tail", type=int, default=1792)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--gaps", action="store_true", help="config-2-style NaN gaps")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--one-pass", action="store_true", help="KRR_KLL_ONE_PASS_TAIL: the tail inside the build")
    a = ap.parse_args()
    import torch

    from krr_amd import _native

    dev = torch.device("cuda", 0)
    base = _native.load_library()
    libs = []
    for path in a.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        for name in ("krr_create", "krr_kll_build", "krr_kll_row_words"):
            getattr(lib, name).argtypes = getattr(base, name).argtypes
            getattr(lib, name).restype = getattr(base, name).restype
        h = ctypes.c_void_p()
        assert lib.krr_create(0, ctypes.byref(h)) == 0
        libs.append((os.path.basename(path), lib, h))
    S, L = a.series, a.length
    ctx = _native.Context(0)
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    vals = torch.empty(S * L, dtype=torch.float64, device=dev)
    if a.gaps:
        ctx.synth_fill(vals, offs, 1000003 * 2, 0, 10080, True)
    else:
        ctx.synth_fill_window(vals, offs, 1000003 * 6, 0, 0, False, 0, L)
    ser = ctx.series(vals, offs, L, a.gaps)
    kp = _native.KrrKllParams(a.budget, 0, 0x4B4C4C5345454431, a.tail, 1 if a.one_pass else 0)
    rw = int(base.krr_kll_row_words(ctypes.byref(kp)))
    rows = {name: torch.empty((S, rw), dtype=torch.int64, device=dev) for name, _, _ in libs}
    st = torch.cuda.current_stream()
    times = {name: [] for name, _, _ in libs}
    for r in range(a.rounds + 1):
        for name, lib, h in libs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)  # both launches when the tail has a pass of its own
            rc = lib.krr_kll_build(h, ctypes.byref(ser), ctypes.byref(kp), 0, rows[name].data_ptr(),
                                   ctypes.c_void_p(st.cuda_stream))
            e1.record(st)
            assert rc == 0, (name, rc)
            torch.cuda.synchronize()
            if r:  # round 0 warms up
                times[name].append(e0.elapsed_time(e1))
    nbytes = 8 * S * L + 8 * (S + 1) + 8 * rw * S
    for name, _, _ in libs:
        ms = sorted(times[name])[len(times[name]) // 2]
        gbs = nbytes / (ms * 1e-3) / 1e9
        print(f"{name}: krr_kll_build{' (one pass)' if a.one_pass else ''} median {ms:.3f} ms over {a.rounds} rounds, {gbs:.1f} GB/s "
              f"= {gbs / 8000:.3f} of 8 TB/s (S={S}, L={L}, budget={a.budget}, tail={a.tail})",
              flush=True)
    for name, _, _ in libs:  # a KRR_KLL_X_STATS build: tail refresh statistics in row word 14
        w = rows[name][:, 14].cpu().numpy().view(np.uint64).astype(np.int64)
        if w.any():
            nref, npass, nfall, nre = w & 0xFFFFFF, (w >> 24) & 0xFFFFFF, (w >> 48) & 0xFF, w >> 56
            print(f"{name}: per series: {nref.mean():.2f} tail refreshes, {npass.mean():.2f} counting passes, "
                  f"{nfall.mean():.3f} sort fallbacks, {nre.mean():.4f} tail-pass restreams "
                  f"(max {nref.max()}, {npass.max()}, {nfall.max()}, {nre.max()})", flush=True)
    if a.check and len(libs) > 1:
        ref = rows[libs[0][0]]
        for name, _, _ in libs[1:]:
            print(f"{name} rows == {libs[0][0]} rows: {bool(torch.equal(rows[name], ref))}", flush=True)


if __name__ == "__main__":
    main()
