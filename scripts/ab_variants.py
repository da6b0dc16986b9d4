"""A/B timing of libkrr_amd build variants in ONE process (interleaved rounds).

Each variant is a separately built .so (different -D flags); all are loaded side by
side with ctypes and fed the same device-resident synthetic workload.  Times the
percentile kernel, the max kernel and the fused krr_simple_run launch per variant.
usage: python scripts/ab_variants.py lib1.so lib2.so ... [--mode linear] [--rounds 5]
"""
import argparse
import ctypes
import os
import sys
from decimal import Decimal

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--mode", default="linear")
    ap.add_argument("--percentile", default="99")
    ap.add_argument("--containers", type=int, default=10000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--pods", type=int, default=5, help="config 2: pods per container")
    ap.add_argument("--length", type=int, default=10080, help="config 4: slots per (compact) segment")
    a = ap.parse_args()
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params
    from oracle import oracle

    dev = torch.device("cuda", 0)
    torch.cuda.init()
    base = _native.load_library()
    names = ("krr_create", "krr_segmented_percentile", "krr_segmented_max", "krr_simple_run", "krr_get_stats")
    libs = []
    for path in a.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        for name in names:
            if not hasattr(lib, name):
                continue
            getattr(lib, name).argtypes = getattr(base, name).argtypes
            getattr(lib, name).restype = ctypes.c_int
        h = ctypes.c_void_p()
        assert lib.krr_create(0, ctypes.byref(h)) == 0
        libs.append((os.path.basename(path), lib, h))
    n = a.containers
    if a.config == 2:
        L, pod_len, gaps = a.pods * 10080, 10080, True
        offs_np = np.arange(n + 1, dtype=np.int64) * L
    elif a.config == 4:  # compact segments of --length samples (10,080: one shard of config 4)
        offs_np = np.arange(n + 1, dtype=np.int64) * a.length
        pod_len, gaps = 0, False
    else:
        rng = np.random.default_rng(3)
        offs_np = np.concatenate([[0], np.cumsum(rng.integers(1, 15, size=n) * 1440)]).astype(np.int64)
        pod_len, gaps = 0, False
    offs = torch.from_numpy(offs_np).to(dev)
    N = int(offs_np[-1])
    cpu = torch.empty(N, dtype=torch.float64, device=dev)
    mem = torch.empty(N, dtype=torch.float64, device=dev)
    ctx = _native.Context(0)
    ctx.synth_fill(cpu, offs, 7, 0, pod_len, gaps)
    ctx.synth_fill(mem, offs, 8, 1, pod_len, gaps)
    maxlen = int(np.max(np.diff(offs_np)))
    cs = ctx.series(cpu, offs, maxlen, gaps)
    ms = ctx.series(mem, offs, maxlen, gaps)
    params = percentile_params(Decimal(a.percentile), a.mode)
    S = n
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)

    def outs():
        return [torch.empty(S, dtype=dt, device=dev) for dt in
                (torch.float64, torch.int64, torch.int32, torch.float64, torch.int64, torch.int32)]

    o = {name: outs() for name, _, _ in libs}
    times = {name: {"pct": [], "max": [], "fused": []} for name, _, _ in libs}
    for r in range(a.rounds):
        for name, lib, h in libs:
            cv, cn, cf, mv, mn, mf = o[name]
            e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            e[0].record(stream)
            rc = lib.krr_segmented_percentile(h, ctypes.byref(cs), ctypes.byref(params), cv.data_ptr(),
                                              cn.data_ptr(), cf.data_ptr(), sp)
            e[1].record(stream)
            rc |= lib.krr_segmented_max(h, ctypes.byref(ms), mv.data_ptr(), mn.data_ptr(), mf.data_ptr(), sp)
            e[2].record(stream)
            rc |= lib.krr_simple_run(h, ctypes.byref(cs), ctypes.byref(ms), ctypes.byref(params),
                                     cv.data_ptr(), cn.data_ptr(), cf.data_ptr(), mv.data_ptr(), mn.data_ptr(),
                                     mf.data_ptr(), sp)
            e[3].record(stream)
            torch.cuda.synchronize()
            assert rc == 0
            times[name]["pct"].append(e[0].elapsed_time(e[1]))
            times[name]["max"].append(e[1].elapsed_time(e[2]))
            times[name]["fused"].append(e[2].elapsed_time(e[3]))
    # parity on a sample vs the oracle (outputs of the last fused launch)
    m = min(200, S)
    end = int(offs_np[m])
    ov, _, _ = oracle.percentile(cpu[:end].cpu().numpy(), offs_np[: m + 1], params.mode, params.p_num,
                                 params.p_den, params.q, gaps, 16)
    mvo, _, _ = oracle.seg_max(mem[:end].cpu().numpy(), offs_np[: m + 1], gaps, 16)
    seg_bytes = 8 * N + 8 * (S + 1) + 20 * S
    for name, _, _ in libs:
        t = {k: np.median(np.array(v)) for k, v in times[name].items()}
        got = o[name][0][:m].cpu().numpy()
        gm = o[name][3][:m].cpu().numpy()
        ok = bool(np.all((got.view(np.uint64) == ov.view(np.uint64)) | ((got == 0) & (ov == 0)))
                  and np.array_equal(gm, mvo, equal_nan=True))
        fb = ""
        lib_h = next((lb, hh) for nm, lb, hh in libs if nm == name)
        if hasattr(lib_h[0], "krr_get_stats"):
            v = ctypes.c_int64()
            lib_h[0].krr_get_stats(lib_h[1], ctypes.byref(v))
            fb = f" | fallbacks {v.value / (2 * a.rounds) / S:.4%}"
        print(f"{name:28s} pct {t['pct']:.4f} ms ({seg_bytes / t['pct'] / 1e6:.0f} GB/s) | "
              f"max {t['max']:.4f} ms ({seg_bytes / t['max'] / 1e6:.0f} GB/s) | "
              f"fused {t['fused']:.4f} ms ({2 * seg_bytes / t['fused'] / 1e6:.0f} GB/s) | parity {ok}{fb}", flush=True)


if __name__ == "__main__":
    main()
