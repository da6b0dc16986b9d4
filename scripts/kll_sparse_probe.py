"""Same-process A/B of the sparse two-pass KLL build (krr_kll_build_lines + krr_kll_tail_lines)
across libkrr_amd build variants, on config-5-shaped data (S series x L slots of the device
synthetic CPU series).  Times the body and the tail launches apart (HIP events), reports the
fraction of 128-B lines the tail read, and (--check) compares every variant's rows with the
first variant's bit for bit.
usage: python scripts/kll_sparse_probe.py lib1.so [lib2.so ...] [--series 20000] [--tail 1792]"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--series", type=int, default=20000)
    ap.add_argument("--length", type=int, default=172_800)
    ap.add_argument("--budget", type=int, default=512)
    ap.add_argument("--tail", type=int, default=1792)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    import torch

    from krr_amd import _native

    dev = torch.device("cuda", 0)
    base = _native.load_library()
    names = ("krr_create", "krr_kll_build_lines", "krr_kll_tail_lines", "krr_kll_row_words", "krr_kll_line_words")
    libs = []
    for path in a.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        for name in names:
            getattr(lib, name).argtypes = getattr(base, name).argtypes
            getattr(lib, name).restype = getattr(base, name).restype
        h = ctypes.c_void_p()
        assert lib.krr_create(0, ctypes.byref(h)) == 0
        libs.append((os.path.basename(path), lib, h))
    S, L = a.series, a.length
    ctx = _native.Context(0)
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    vals = torch.empty(S * L, dtype=torch.float64, device=dev)
    ctx.synth_fill_window(vals, offs, 1000003 * 6, 0, 0, False, 0, L)
    ser = ctx.series(vals, offs, L, False)
    kp = _native.KrrKllParams(a.budget, 0, 0x4B4C4C5345454431, a.tail, _native.KRR_KLL_BODY_ONLY)
    rw = int(base.krr_kll_row_words(ctypes.byref(kp)))
    stride = int(base.krr_kll_line_words(L))
    lines = torch.empty(S * stride, dtype=torch.int32, device=dev)
    read = torch.zeros(S, dtype=torch.int32, device=dev)
    rows = {name: torch.empty((S, rw), dtype=torch.int64, device=dev) for name, _, _ in libs}
    st = torch.cuda.current_stream()
    tb, tt = {n: [] for n, _, _ in libs}, {n: [] for n, _, _ in libs}
    reads = {}
    for r in range(a.rounds + 1):
        for name, lib, h in libs:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            s = ctypes.c_void_p(st.cuda_stream)
            ev[0].record(st)
            rc = lib.krr_kll_build_lines(h, ctypes.byref(ser), ctypes.byref(kp), 0, rows[name].data_ptr(),
                                         lines.data_ptr(), stride, s)
            ev[1].record(st)
            rc2 = lib.krr_kll_tail_lines(h, ctypes.byref(ser), ctypes.byref(kp), rows[name].data_ptr(),
                                         lines.data_ptr(), stride, read.data_ptr(), s)
            ev[2].record(st)
            assert rc == 0 and rc2 == 0, (name, rc, rc2)
            torch.cuda.synchronize()
            if r:
                tb[name].append(ev[0].elapsed_time(ev[1]))
                tt[name].append(ev[1].elapsed_time(ev[2]))
            reads[name] = int(read.sum().item())
    nch = (L // 1024) + 1
    for name, _, _ in libs:
        mb, mt = sorted(tb[name])[a.rounds // 2], sorted(tt[name])[a.rounds // 2]
        print(f"{name}: body {mb:.3f} ms ({8 * S * L / (mb * 1e-3) / 8e12:.3f} of 8 TB/s), tail {mt:.3f} ms, "
              f"both {mb + mt:.3f} ms = {S / ((mb + mt) * 1e-3) / 1e6:.2f} M series/s; tail read "
              f"{reads[name] / (S * nch * 64):.4f} of the lines (S={S}, L={L}, tail={a.tail})", flush=True)
    if a.check and len(libs) > 1:
        ref = rows[libs[0][0]]
        for name, _, _ in libs[1:]:
            print(f"{name} rows == {libs[0][0]} rows: {bool(torch.equal(rows[name], ref))}", flush=True)


if __name__ == "__main__":
    main()
