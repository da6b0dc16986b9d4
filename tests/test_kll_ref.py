"""The KLL-style sketch's specification on the CPU (oracle/kll_ref.py): short series are
exact, and on every data shape the answer's rank error stays inside the data-independent
bound the rows carry (krr_amd.core.sketch.kll_rank_bound).  The GPU kernel is compared
with this model bit for bit in tests/test_gpu_kll.py."""
from __future__ import annotations

from decimal import Decimal

import numpy as np
import pytest

from krr_amd.core.engine import percentile_params
from oracle import kll_ref as M


def _shapes(n: int, rng):
    return {
        "gamma": rng.gamma(2.0, 0.05, n),
        "low_dispersion": 0.25 + rng.uniform(-0.002, 0.002, n),
        "quantized": rng.choice([0.1, 0.2, 0.3, 0.5], n, p=[0.5, 0.3, 0.15, 0.05]),
        "increasing": np.sort(rng.gamma(2.0, 0.05, n)),
        "decreasing": np.sort(rng.gamma(2.0, 0.05, n))[::-1].copy(),
        "constant": np.full(n, 0.125),
        "signed": rng.standard_normal(n),
    }


def _rank_error(x: np.ndarray, v: float, target: float) -> float:
    lt = int((x < v).sum())
    le = int((x <= v).sum())
    return max(0.0, lt - target, target - (le - 1)) / x.size


@pytest.mark.parametrize("n", [1, 7, 300, 511, 512, 1023])
def test_short_series_are_exact(n):
    rng = np.random.default_rng(n)
    x = rng.gamma(2.0, 0.05, n)
    row = M.build_row(x, 0, n, budget=1024)
    assert int(row[9]) == n and int(row[8]) == 0  # kept whole: weight n, no compaction
    for p, mode in (("99", "linear"), ("50", "sorted_lower"), ("95", "linear")):
        prm = percentile_params(Decimal(p), mode)
        v, cnt, fl = M.query(row[None], prm.mode, prm.p_num, prm.p_den, prm.q)
        want = np.percentile(x, float(p)) if mode == "linear" else np.sort(x)[(n - 1) * int(p) // 100]
        assert cnt == n and fl == 0 and v == want


@pytest.mark.parametrize("shape", ["gamma", "low_dispersion", "quantized", "increasing", "decreasing", "constant",
                                   "signed"])
@pytest.mark.parametrize("W", [1, 3])
def test_rank_error_within_bound(shape, W):
    rng = np.random.default_rng(7 + W)
    n = 43_200
    x = _shapes(n, rng)[shape]
    cuts = [n * w // W for w in range(W + 1)]
    rows = np.stack([M.build_row(x, cuts[w], cuts[w + 1], budget=512, seed=11, series=3, slc=w)
                     for w in range(W)])
    assert int(rows[:, 0].sum()) == n
    bound = M.rank_bound(rows, delta=0.01)
    assert bound < 0.05  # 43,200 samples into 512 keys per slice
    for p in ("50", "90", "99"):
        prm = percentile_params(Decimal(p), "sorted_lower")
        v, cnt, fl = M.query(rows, prm.mode, prm.p_num, prm.p_den, prm.q)
        assert cnt == n and fl == 0
        assert _rank_error(x, v, (n - 1) * int(p) // 100) <= bound, (shape, p)


def test_weight_and_nan_accounting():
    rng = np.random.default_rng(3)
    x = rng.gamma(2.0, 0.05, 20_000)
    x[::97] = np.nan
    row = M.build_row(x, 5, 19_999, budget=512, gaps=True)
    present = int((~np.isnan(x[5:19_999])).sum())
    assert int(row[0]) == present and int(row[1]) == 0
    w = int(row[9])
    assert abs(w - present) < 0.05 * present  # total weight tracks n (coins are zero-mean)
    keys, lvl = M.row_keys(row)
    assert keys.size <= 512 and np.all(np.diff(keys[lvl == lvl.max()].astype(np.float64)) >= 0)
    compact = M.build_row(x, 5, 19_999, budget=512, gaps=False)
    assert int(compact[1]) == int(np.isnan(x[5:19_999]).sum())
    prm = percentile_params(Decimal("99"), "linear")
    assert M.query(compact[None], prm.mode, prm.p_num, prm.p_den, prm.q)[2] == 1  # KRR_FLAG_NAN


def test_rank_bound_helper_matches_restatement():
    """krr_amd.core.sketch.kll_rank_bound (the bench's bound, from device rows) equals the
    restatement's per-series bound."""
    import torch

    from krr_amd.core import sketch

    rng = np.random.default_rng(12)
    W, rows = 3, []
    for s, n in enumerate((0, 900, 30_000, 90_000)):
        x = rng.gamma(2.0, 0.05, n)
        cuts = [n * w // W for w in range(W + 1)]
        rows.append(np.stack([M.build_row(x, cuts[w], cuts[w + 1], budget=256, seed=2, series=s, slc=w)
                              for w in range(W)]))
    got = sketch.kll_rank_bound(torch.from_numpy(np.concatenate(rows).view(np.int64)), W)
    assert np.isnan(got[0])
    for s in range(1, 4):
        assert got[s] == pytest.approx(M.rank_bound(rows[s]), rel=1e-12)


def _exchange_worker(rank, world, port, q, n_series, T, budget):
    import os

    import torch
    import torch.distributed as dist

    from krr_amd.core import sketch

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(0)
        x = rng.gamma(2.0, 0.05, (n_series, T))
        t0, t1 = T * rank // world, T * (rank + 1) // world
        rows = np.stack([M.build_row(x[s], t0, t1, budget=budget, seed=9, series=s, slc=rank)
                         for s in range(n_series)])
        merged, W = sketch.kll_exchange(torch.from_numpy(rows.view(np.int64)))
        lo, hi = sketch.owner_blocks(n_series, world)[rank]
        q.put((rank, lo, hi, W, merged.numpy().view(np.uint64)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_hands_each_owner_its_series_rows(world):
    """gloo: kll_exchange gives each rank the W slice rows of its owner block, series-major
    in slice (= time) order: the rows a single process builds for the same slices."""
    import multiprocessing as mp
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    n_series, T, budget = 7, 5000, 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q, n_series, T, budget))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x = np.random.default_rng(0).gamma(2.0, 0.05, (n_series, T))
    prm = percentile_params(Decimal("99"), "linear")
    for rank, lo, hi, W, merged in got:
        assert W == world and merged.shape[0] == (hi - lo) * world
        for s in range(lo, hi):
            want = np.stack([M.build_row(x[s], T * w // world, T * (w + 1) // world, budget=budget, seed=9, series=s,
                                         slc=w) for w in range(world)])
            have = merged[(s - lo) * world:(s - lo + 1) * world]
            assert np.array_equal(have, want)
            v, n, f = M.query(have, prm.mode, prm.p_num, prm.p_den, prm.q)
            assert n == T and f == 0 and np.isfinite(v)


def test_sparse_series_whose_keys_all_vanish():
    """Three present samples spread over many chunks (NaN gaps): every kept key can be
    compacted away; the answer then comes from the exact min / max, never a NaN."""
    x = np.full(5000, np.nan)
    x[[10, 2500, 4990]] = [0.3, 0.1, 0.2]
    prm = percentile_params(Decimal("50"), "sorted_lower")
    for seed in range(16):
        row = M.build_row(x, 0, x.size, budget=256, seed=seed, gaps=True)
        v, n, f = M.query(row[None], prm.mode, prm.p_num, prm.p_den, prm.q)
        assert n == 3 and f == 0 and v in (0.1, 0.2, 0.3)
