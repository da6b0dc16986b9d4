"""Trace the window export's shrinks for one series of tests/test_gpu_window.py's fleet
(debug build: every shrink's seen / below / cnt / rank bounds / key bounds, and the
overflow that fails a window), to see why a series misses.

    bash scripts/build_variants.sh wdbg:"-DKRR_WEXP_DEBUG"
    python scripts/trace_window.py --gaps --mode linear --pct 50 --W 1 --series 17 27
"""
import argparse
import ctypes
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["KRR_AMD_LIB"] = os.path.join(ROOT, "krr_amd/lib/variants/lib_wdbg.so")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def key_value(u):
    import numpy as np

    u = int(u) % 2**64
    v = (u ^ 2**63) if u >> 63 else (~u) % 2**64
    return np.array([v], dtype=np.uint64).view(np.float64)[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaps", action="store_true")
    ap.add_argument("--mode", default="linear")
    ap.add_argument("--pct", default="50")
    ap.add_argument("--W", type=int, default=1)
    ap.add_argument("--series", type=int, nargs="+", default=[0])
    a = ap.parse_args()
    from decimal import Decimal

    import numpy as np
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params
    from test_gpu_window import _mixed

    ctx = _native.Context(0)
    lib = _native.load_library()
    lib.krr_wexp_debug_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(zlib.crc32(f"{a.gaps}{a.mode}{a.pct}{a.W}".encode()))
    S, L = 40, 12_000
    X = _mixed(rng, S, L)
    if a.gaps:
        X[rng.random(X.shape) < 0.15] = np.nan
        X[7, : L // 2] = np.nan
        X[8] = np.nan
    params = percentile_params(Decimal(a.pct), a.mode)
    for s in a.series:
        for j, c in enumerate(np.array_split(np.arange(L), a.W)):
            x = np.ascontiguousarray(X[s, c])
            xs = torch.from_numpy(x).to(dev)
            o = torch.tensor([0, x.size], dtype=torch.int64, device=dev)
            ser = ctx.series(xs, o, x.size, a.gaps)
            kc = _native.window_key_cap(x.size, L - x.size, params)
            hdr = torch.zeros((1, _native.HDR_WORDS), dtype=torch.int64, device=dev)
            keys = torch.zeros((1, kc), dtype=torch.int64, device=dev)
            ctx.window_export(ser, params, L - x.size, kc, hdr, keys)
            torch.cuda.synchronize()
            buf = (ctypes.c_ulonglong * 5120)()
            n = ctypes.c_uint()
            lib.krr_wexp_debug_read(buf, ctypes.byref(n))
            h = hdr.cpu().numpy()[0]
            print(f"== series {s} slice {j}: lo {key_value(h[0])} hi {key_value(h[1])} below {h[2]} n {h[3]} "
                  f"cnt {h[4] & 0xFFFFFFFF} flags {h[4] >> 32:#x}")
            for i in range(min(n.value, 200)):
                t, p, q, r, w = buf[5 * i:5 * i + 5]
                if t == 1:
                    print(f"  shrink seen {p} below {q} cnt {r} ilo {w >> 32} ihi {w & 0xFFFFFFFF}")
                elif t == 2:
                    print(f"    [{key_value(p)}, {key_value(q)}] -> [{key_value(r)}, {key_value(w)}]")
                else:
                    print(f"  overflow seen {p} cnt {q} C {r} lo {key_value(w)}")


if __name__ == "__main__":
    main()
