"""A/B of the device allocation behind the value buffers: the PyTorch caching allocator
(hipMalloc) against hipExtMallocWithFlags(hipDeviceMallocContiguous) (physically
contiguous: the largest page fragments, fewest address-translation misses).

Same process, same data (counter hash), interleaved rounds; times the fused launch.
usage: python scripts/alloc_ab.py --config 2|3|4 [--containers N] [--rounds 5] [--percentile 99]
"""
import argparse
import ctypes
import os
import sys
from decimal import Decimal

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--containers", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--percentile", default="99")
    ap.add_argument("--mode", default="linear")
    ap.add_argument("--flags", type=lambda s: int(s, 0), default=HIP_DEVICE_MALLOC_CONTIGUOUS)
    a = ap.parse_args()
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    dev = torch.device("cuda", 0)
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    lib = _native.load_library()
    ctx = _native.Context(0)

    n = a.containers
    if a.config == 2:
        n = n or 10000
        offs_np = np.arange(n + 1, dtype=np.int64) * 50400
        pod_len, gaps = 10080, True
    elif a.config == 4:
        n = n or 1_000_000
        offs_np = np.arange(n + 1, dtype=np.int64) * 10080
        pod_len, gaps = 0, False
    else:
        n = n or 100_000
        rng = np.random.default_rng(3)
        offs_np = np.concatenate([[0], np.cumsum(rng.integers(1, 15, size=n) * 1440)]).astype(np.int64)
        pod_len, gaps = 0, False
    N = int(offs_np[-1])
    S = n
    offs = torch.from_numpy(offs_np).to(dev)
    maxlen = int(np.max(np.diff(offs_np)))
    params = percentile_params(Decimal(a.percentile), a.mode)
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)

    def fill(ptr_c, ptr_m):
        for ptr, seed, kind in ((ptr_c, 7, 0), (ptr_m, 8, 1)):
            rc = lib.krr_synth_fill_global(ctx._h, ptr, offs.data_ptr(), S, seed, kind, pod_len, int(gaps), 0, 0, 0,
                                           sp)
            assert rc == 0

    variants = {}
    # torch caching allocator
    tc = torch.empty(N, dtype=torch.float64, device=dev)
    tm = torch.empty(N, dtype=torch.float64, device=dev)
    variants["torch"] = (tc.data_ptr(), tm.data_ptr())
    # contiguous hipExtMallocWithFlags
    pc, pm = ctypes.c_void_p(), ctypes.c_void_p()
    e1 = hip.hipExtMallocWithFlags(ctypes.byref(pc), N * 8, a.flags)
    e2 = hip.hipExtMallocWithFlags(ctypes.byref(pm), N * 8, a.flags)
    print(f"hipExtMallocWithFlags(flags={a.flags:#x}) -> {e1}, {e2}", flush=True)
    if e1 == 0 and e2 == 0:
        variants["contig"] = (pc.value, pm.value)
    for name, (c, m) in variants.items():
        fill(c, m)
    torch.cuda.synchronize()

    def outs():
        return [torch.empty(S, dtype=dt, device=dev) for dt in
                (torch.float64, torch.int64, torch.int32, torch.float64, torch.int64, torch.int32)]

    o = {k: outs() for k in variants}
    ser = {k: (_native.KrrSeries(c, offs.data_ptr(), S, N, maxlen, int(gaps), 0),
               _native.KrrSeries(m, offs.data_ptr(), S, N, maxlen, int(gaps), 0)) for k, (c, m) in variants.items()}
    times = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k in variants:
            cv, cn, cf, mv, mn, mf = o[k]
            cs, ms = ser[k]
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record(stream)
            rc = lib.krr_simple_run(ctx._h, ctypes.byref(cs), ctypes.byref(ms), ctypes.byref(params),
                                    cv.data_ptr(), cn.data_ptr(), cf.data_ptr(), mv.data_ptr(), mn.data_ptr(),
                                    mf.data_ptr(), sp)
            e[1].record(stream)
            torch.cuda.synchronize()
            assert rc == 0
            times[k].append(e[0].elapsed_time(e[1]))
    seg_bytes = 8 * N + 8 * (S + 1) + 20 * S
    ref = None
    for k in variants:
        t = float(np.median(times[k]))
        got = torch.cat([o[k][0].view(torch.int64), o[k][3].view(torch.int64)]).cpu()
        same = "" if ref is None else f" | results equal to {next(iter(variants))}: {bool(torch.equal(got, ref))}"
        ref = got if ref is None else ref
        print(f"config {a.config} S={S} {k:7s} fused {t:.4f} ms ({2 * seg_bytes / t / 1e6:.0f} GB/s, "
              f"{2 * seg_bytes / t / 1e6 / 8000:.2%}) all {['%.4f' % x for x in times[k]]}{same}", flush=True)
    if "contig" in variants:
        hip.hipFree(pc)
        hip.hipFree(pm)
    ctx.close()


if __name__ == "__main__":
    main()
