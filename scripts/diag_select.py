"""Per-segment cycle breakdown of k_select from the KRR_DIAG build.

usage: python scripts/diag_select.py krr_amd/lib/libkrr_amd_diag.so [--mode linear] [--containers 10000]
"""
import argparse
import ctypes
import os
import sys
from decimal import Decimal

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
NAMES = ["total", "compact", "final", "n_compact", "n_fallback", "active_slots", "inserted", "chunks"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--mode", default="linear")
    ap.add_argument("--percentile", default="99")
    ap.add_argument("--containers", type=int, default=10000)
    ap.add_argument("--length", type=int, default=5 * 10080, help="slots per segment")
    ap.add_argument("--compact", action="store_true", help="no NaN gaps (config 3/4 layout)")
    a = ap.parse_args()
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    base = _native.load_library()
    lib = ctypes.CDLL(os.path.abspath(a.lib))
    for name in ("krr_create", "krr_segmented_percentile", "krr_synth_fill"):
        getattr(lib, name).argtypes = getattr(base, name).argtypes
    lib.krr_diag_attach.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    h = ctypes.c_void_p()
    assert lib.krr_create(0, ctypes.byref(h)) == 0
    n = a.containers
    L = a.length
    offs_np = np.arange(n + 1, dtype=np.int64) * L
    offs = torch.from_numpy(offs_np).to(dev)
    N = int(offs_np[-1])
    cpu = torch.empty(N, dtype=torch.float64, device=dev)
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    gaps = 0 if a.compact else 1
    assert lib.krr_synth_fill(h, cpu.data_ptr(), offs.data_ptr(), n, 7, 0, 10080, gaps, sp) == 0
    diag = torch.zeros(n * 8, dtype=torch.int64, device=dev)
    assert lib.krr_diag_attach(ctypes.c_void_p(diag.data_ptr())) == 0
    ser = _native.KrrSeries(cpu.data_ptr(), offs.data_ptr(), n, N, L, gaps, 0)
    params = percentile_params(Decimal(a.percentile), a.mode)
    ov = torch.empty(n, dtype=torch.float64, device=dev)
    on = torch.empty(n, dtype=torch.int64, device=dev)
    of = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert lib.krr_segmented_percentile(h, ctypes.byref(ser), ctypes.byref(params), ov.data_ptr(),
                                            on.data_ptr(), of.data_ptr(), sp) == 0
        e1.record()
        torch.cuda.synchronize()
    print(f"kernel {e0.elapsed_time(e1):.3f} ms (diag build)")
    d = diag.view(n, 8).cpu().numpy().astype(np.float64)
    for i, nm in enumerate(NAMES):
        col = d[:, i]
        print(f"  {nm:13s} mean {col.mean():14.1f}  p50 {np.median(col):14.1f}  max {col.max():14.1f}")
    tot = d[:, 0].mean()
    print(f"  shares: compact {d[:, 1].mean() / tot:.3f}  final {d[:, 2].mean() / tot:.3f}  "
          f"stream(rest) {1 - (d[:, 1].mean() + d[:, 2].mean()) / tot:.3f}; memtime ticks/segment {tot:.0f}")


if __name__ == "__main__":
    main()
