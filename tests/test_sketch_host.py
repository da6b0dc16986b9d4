"""Sketch mode / time-sharded merges on CPU (no GPU): the numpy restatement of the
sketch, exact mergeability, rank-error bound, and the world-size-2 gloo merges
(reduce-scatter of sketches, time-ordered max, REF_INDEX location)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from krr_amd.core import sketch
from oracle import sketch_ref

M, ELO, OCT = 5, -24, 36


def test_bins_cover_specials():
    x = np.array([-1.0, -0.0, 0.0, 1e-300, 2.0**-24, 1.0, 1.5, 2.0**12 - 1e-9, 2.0**12, np.inf, 5e-324])
    b = sketch_ref.bins_of(x, M, ELO, OCT)
    nb = OCT << M
    assert list(b[:4]) == [0, 1, 1, 2]
    assert b[4] == 3  # first log-linear bin starts at 2^e_lo
    assert b[5] == 3 + (24 << M) and b[6] == 3 + (24 << M) + 16
    assert b[7] == 3 + nb - 1 and b[8] == 3 + nb and b[9] == 3 + nb
    assert b[10] == 2  # denormal


def test_merge_is_exact():
    rng = np.random.default_rng(0)
    x = rng.gamma(2.0, 0.05, size=172_800)
    x[rng.random(x.size) < 0.05] = np.nan
    whole, mn, mx = sketch_ref.build(x, M, ELO, OCT)
    parts = [sketch_ref.build(p, M, ELO, OCT) for p in np.array_split(x, 8)]
    assert np.array_equal(sum(p[0] for p in parts), whole)
    assert min(p[1] for p in parts) == mn and max(p[2] for p in parts) == mx


@pytest.mark.parametrize("pct", [99, 95, 50, 10])
def test_rank_error_bounded_by_bin_mass(pct):
    rng = np.random.default_rng(pct)
    x = rng.gamma(2.0, 0.05, size=50_000)
    counts, mn, mx = sketch_ref.build(x, M, ELO, OCT)
    v, n = sketch_ref.query(counts, mn, mx, M, ELO, OCT, "sorted_lower", pct, 1, pct / 100)
    k = ((n - 1) * pct) // 100
    srt = np.sort(x)
    exact = srt[k]
    lt, le = np.searchsorted(srt, v, "left"), np.searchsorted(srt, v, "right")
    err = max(0, lt - k, k - (le - 1)) / n
    b = sketch_ref.bins_of(np.array([exact]), M, ELO, OCT)[0]
    assert err <= counts[b] / n + 1e-12
    assert abs(v - exact) <= exact * 2.0**-M * 1.0001


def test_refindex_locate():
    all_n = np.array([[3, 0, 5, 10], [4, 0, 0, 10]])
    n, k, owner, kl0 = sketch.refindex_locate(all_n, 50, 1, 0)
    assert list(n) == [7, 0, 5, 20]
    assert list(k) == [3, -1, 2, 9]
    assert list(owner) == [1, -1, 0, 0]
    assert list(kl0) == [-1, -1, 2, 9]
    _, _, _, kl1 = sketch.refindex_locate(all_n, 50, 1, 1)
    assert list(kl1) == [0, -1, -1, -1]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _series(seed=5, S=13, L=4000):
    rng = np.random.default_rng(seed)
    x = rng.gamma(2.0, 0.05, size=(S, L))
    x[rng.random(x.shape) < 0.1] = np.nan
    x[3, :] = np.nan  # an empty series
    x[4, :2000] = np.nan  # empty in the first time slice only
    x[5] = np.where(rng.random(L) < 0.5, 0.0, -0.0)  # +-0 ties for max
    return x


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = _series()
        S, L = x.shape
        sl = np.array_split(np.arange(L), world)[rank]
        local = x[:, sl]
        built = [sketch_ref.build(local[s], M, ELO, OCT) for s in range(S)]
        sk = {"counts": torch.tensor(np.stack([b[0] for b in built]), dtype=torch.int32),
              "vmin": torch.tensor([b[1] for b in built], dtype=torch.float64),
              "vmax": torch.tensor([b[2] for b in built], dtype=torch.float64),
              "flags": torch.zeros(S, dtype=torch.int32)}
        merged = sketch.merge_time_sharded(sk)
        # memory max per slice (Python max() first-maximum rule within the slice)
        lv, lc = [], []
        for s in range(S):
            v = local[s][~np.isnan(local[s])]
            lc.append(v.size)
            if v.size:
                best = v[0]
                for y in v[1:]:
                    if y > best:
                        best = y
                lv.append(best)
            else:
                lv.append(np.nan)
        mx = sketch.max_time_sharded(torch.tensor(lv, dtype=torch.float64), torch.tensor(lc, dtype=torch.int64),
                                     torch.zeros(S, dtype=torch.int32))
        q.put((rank, {k: (v.numpy() if torch.is_tensor(v) else v) for k, v in merged.items()}, mx))
    finally:
        dist.destroy_process_group()


def test_time_sharded_merges_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (m, mx)) for r, m, mx in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x = _series()
    S = x.shape[0]
    for r in range(world):
        m, _ = res[r]
        lo, hi = m["block"]
        assert (lo, hi) == sketch.owner_blocks(S, world)[r]
        for s in range(lo, hi):
            c, mn, mx = sketch_ref.build(x[s], M, ELO, OCT)
            assert np.array_equal(m["counts"][s - lo], c)
            assert np.array_equal(m["vmin"][s - lo], mn, equal_nan=True)
            assert np.array_equal(m["vmax"][s - lo], mx, equal_nan=True)
    for r in range(world):
        _, mx = res[r]
        for s in range(S):
            v = x[s][~np.isnan(x[s])]
            if v.size == 0:
                assert np.isnan(mx["value"][s]) and mx["count"][s] == 0
                continue
            best = v[0]
            for y in v[1:]:
                if y > best:
                    best = y
            assert np.float64(mx["value"][s]).view(np.uint64) == np.float64(best).view(np.uint64), s
            assert mx["count"][s] == v.size


def _exact_worker(rank, world, port, q):
    """The exact refinement's host flow with the kernels replaced by oracle/sketch_ref:
    merged sketches (reduce-scatter) -> locate on the owner -> all-gather of the
    locations -> local collect -> exchange_to_owners (all-to-all) -> exact select."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = _series()
        S, L = x.shape
        local = x[:, np.array_split(np.arange(L), world)[rank]]
        built = [sketch_ref.build(local[s], M, ELO, OCT) for s in range(S)]
        sk = {"counts": torch.tensor(np.stack([b[0] for b in built]), dtype=torch.int32),
              "vmin": torch.tensor([b[1] for b in built], dtype=torch.float64),
              "vmax": torch.tensor([b[2] for b in built], dtype=torch.float64),
              "flags": torch.zeros(S, dtype=torch.int32)}
        merged = sketch.merge_time_sharded(sk)
        lo, hi = merged["block"]
        out = {}
        for mode, pn, pd in (("sorted_lower", 99, 1), ("linear", 99, 1), ("sorted_lower", 50, 1),
                             ("linear", 5, 1)):
            qv = pn / pd / 100
            locs = [sketch_ref.locate(c, mode, pn, pd, qv) for c in merged["counts"].numpy()]
            blk = torch.tensor([[n, r0, r1, bef, b0, b1] for n, r0, r1, bef, g, b0, b1 in locs],
                               dtype=torch.int64).reshape(-1, 6)
            every = sketch._all_gather_blocks(blk, S, None, world)
            assert every.shape == (S, 6)
            lists = [sketch_ref.collect(local[s], int(every[s, 4]), int(every[s, 5]), M, ELO, OCT) for s in range(S)]
            cnt = torch.tensor([len(v) for v in lists], dtype=torch.int64)
            vals = torch.tensor(np.concatenate(lists) if lists else np.zeros(0), dtype=torch.float64)
            gv, go = sketch.exchange_to_owners(vals, cnt, S, None)
            got = []
            for i, (n, r0, r1, bef, g, b0, b1) in enumerate(locs):
                lst = gv[int(go[i]):int(go[i + 1])].numpy()
                got.append(np.nan if n == 0 else sketch_ref.refine(lst, r0 - bef, r1 - bef, g, mode))
            out[(mode, pn)] = (lo, hi, got)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exact_refinement_host_flow(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_exact_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x = _series()
    for (mode, pn), _ in res[0].items():
        for r in range(world):
            lo, hi, got = res[r][(mode, pn)]
            for s in range(lo, hi):
                v = x[s][~np.isnan(x[s])]
                if v.size == 0:
                    assert np.isnan(got[s - lo])
                    continue
                if mode == "linear":
                    want = np.percentile(v, pn)
                else:
                    want = sorted(v.tolist())[((v.size - 1) * pn) // 100]
                assert got[s - lo] == want, (mode, pn, s)
                if mode == "sorted_lower":
                    assert np.signbit(got[s - lo]) == np.signbit(want), (mode, pn, s)
