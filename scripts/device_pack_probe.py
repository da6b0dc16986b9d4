"""Where the device packer's time goes, on bench.py's host-path bodies (2,000 objects x 3
pods x 10,080 samples, one resource): staging copy alone (krr_pack_concat into page-locked
memory, 16 threads), H2D alone (the staged bytes, 256-MiB copies), parse kernels alone (bodies
already in HBM), and the whole pipelined DevicePacker.pack.
usage: python scripts/device_pack_probe.py [--objects 2000] [--chunk-mib 256]"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=2000)
    ap.add_argument("--pods", type=int, default=3)
    ap.add_argument("--chunk-mib", type=int, default=256)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch

    from krr_amd import _native
    from krr_amd.core.device_pack import DevicePacker
    from krr_amd.core.prom_native import load_library

    rng = np.random.default_rng(0)
    L = 10080
    ts = [repr(1.7e9 + 60.0 * i) for i in range(L)]
    pool = []
    for _ in range(48):
        vals = ",".join(f'[{t},"{x!r}"]' for t, x in zip(ts, rng.gamma(2.0, 0.05, L).tolist()))
        pool.append(('{"status":"success","data":{"resultType":"matrix","result":[{"metric":{"pod":"p"},'
                     '"values":[' + vals + ']}]}}').encode())
    bodies = [[pool[(o * a.pods + i) % 48] for i in range(a.pods)] for o in range(a.objects)]
    flat = [b for bs in bodies for b in bs]
    nb = len(flat)
    lens = np.array([len(b) for b in flat], dtype=np.int64)
    offs = np.zeros(nb + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    total = int(offs[-1])
    ctx = _native.Context(0)
    packer = DevicePacker(ctx, chunk_bytes=a.chunk_mib << 20, threads=a.threads)
    packer.pack(bodies[:8])
    host = load_library()
    stage = torch.empty(total + 128, dtype=torch.uint8, pin_memory=True)
    ptrs = (ctypes.c_char_p * nb)(*flat)
    res = {}
    for rep in range(3):
        t0 = time.perf_counter()
        host.krr_pack_concat(ctypes.addressof(ptrs), lens.ctypes.data, nb, offs.ctypes.data, stage.data_ptr(),
                             a.threads)
        res.setdefault("stage_s", []).append(time.perf_counter() - t0)
        d = torch.empty(total + 128, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step = a.chunk_mib << 20
        for lo in range(0, total, step):
            d[lo:min(lo + step, total)].copy_(stage[lo:min(lo + step, total)], non_blocking=True)
        torch.cuda.synchronize()
        res.setdefault("h2d_s", []).append(time.perf_counter() - t0)
        d_offs = torch.from_numpy(offs).to("cuda:0")
        jb = ctx.json_bodies(d, d_offs, total)
        tmp = torch.empty(total // 8 + 1, dtype=torch.float64, device="cuda:0")
        cnt = torch.empty(nb, dtype=torch.int64, device="cuda:0")
        st = torch.empty(nb, dtype=torch.int32, device="cuda:0")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.json_parse(jb, 0, nb, False, tmp, None, cnt, st)
        torch.cuda.synchronize()
        res.setdefault("parse_all_s", []).append(time.perf_counter() - t0)
        del d, tmp
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        packer.pack(bodies)
        torch.cuda.synchronize()
        res.setdefault("pack_s", []).append(time.perf_counter() - t0)
    out = {k: min(v) for k, v in res.items()}
    out["bytes"] = total
    out.update({k.replace("_s", "_GBps"): total / out[k] / 1e9 for k in list(out) if k.endswith("_s")})
    print(out)


if __name__ == "__main__":
    main()
