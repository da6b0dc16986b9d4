"""GPU: randomized parity sweep of the fused launch against the CPU oracle.

Many small launches, each with a random percentile (including 15-significant-digit
ones), a random segment-length mix (around the single-pass capacity boundaries, the
hselect switch and tiny segments), a random value generator (continuous, heavy
duplicates, two-valued, monotone up/down, sawtooth, ±0 heavy, negatives, ±inf,
subnormals) and both layouts (compact with NaN samples, NaN-gapped).  Every CPU
result must be bit-exact (LINEAR: up to the sign of a zero) and every memory max,
count and flag identical.  Seeds are fixed so a failure reproduces.
"""
import os

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _values(rng, n, kind):
    if kind == "gamma":
        return rng.gamma(2.0, 0.05, n)
    if kind == "dups":
        return rng.integers(0, 7, n).astype(np.float64) * 0.125
    if kind == "two":
        return np.where(rng.random(n) < 0.97, 0.25, 3.0)
    if kind == "up":
        return np.sort(rng.gamma(2.0, 0.05, n))
    if kind == "down":
        return np.sort(rng.gamma(2.0, 0.05, n))[::-1].copy()
    if kind == "saw":
        return (np.arange(n) % 97).astype(np.float64) + rng.random(n) * 1e-3
    if kind == "zeros":
        x = rng.gamma(2.0, 0.05, n)
        u = rng.random(n)
        x[u < 0.6] = 0.0
        x[u < 0.3] = -0.0
        return x
    if kind == "signed":
        return rng.normal(0.0, 1.0, n)
    if kind == "specials":
        x = rng.gamma(2.0, 0.05, n)
        u = rng.random(n)
        x[u < 0.01] = np.inf
        x[(u >= 0.01) & (u < 0.02)] = -np.inf
        x[(u >= 0.02) & (u < 0.03)] = 5e-324
        return x
    raise ValueError(kind)


KINDS = ["gamma", "dups", "two", "up", "down", "saw", "zeros", "signed", "specials"]


def _lengths(rng, S):
    pick = rng.integers(0, 6, S)
    lens = np.empty(S, dtype=np.int64)
    lens[pick == 0] = rng.integers(0, 4, (pick == 0).sum())
    lens[pick == 1] = rng.integers(1000, 1200, (pick == 1).sum())       # around cap for small tkeep
    lens[pick == 2] = rng.integers(8000, 12000, (pick == 2).sum())
    lens[pick == 3] = rng.integers(30000, 60000, (pick == 3).sum())
    lens[pick == 4] = rng.integers(1, 300, (pick == 4).sum())
    lens[pick == 5] = rng.integers(2000, 5000, (pick == 5).sum())
    return lens


def _pct(rng):
    r = rng.random()
    if r < 0.3:
        return int(rng.choice([99, 95, 90, 50, 100, 1])), 1
    if r < 0.6:
        return int(rng.integers(1, 1000)), 10
    den = 10 ** int(rng.integers(2, 14))
    return int(rng.integers(1, 100 * den + 1)), den


@pytest.mark.parametrize("seed", list(range(int(os.environ.get("KRR_STRESS_SEEDS", "40")))))
def test_random_sweep(seed):
    import torch

    from krr_amd import _native

    rng = np.random.default_rng(1000 + seed)
    S = int(rng.integers(20, 60))
    lens = _lengths(rng, S)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    N = int(offs[-1])
    gaps = bool(seed % 2)
    cpu = np.empty(N)
    mem = np.empty(N)
    for s in range(S):
        a, b = offs[s], offs[s + 1]
        cpu[a:b] = _values(rng, b - a, KINDS[int(rng.integers(0, len(KINDS)))])
        mem[a:b] = np.floor(_values(rng, b - a, KINDS[int(rng.integers(0, len(KINDS)))]) * 1e8)
    if gaps:
        cpu[rng.random(N) < rng.random() * 0.3] = np.nan
        mem[rng.random(N) < rng.random() * 0.3] = np.nan
    else:  # compact: a few segments carry real NaN samples
        for s in rng.choice(S, size=3, replace=False):
            if offs[s + 1] > offs[s]:
                cpu[offs[s]] = np.nan
                mem[offs[s + 1] - 1] = np.nan
    dev = torch.device("cuda:0")
    ctx = _native.Context(0)
    d_off = torch.from_numpy(offs).to(dev)
    cs = ctx.series(torch.from_numpy(cpu).to(dev), d_off, 0, gaps)
    ms = ctx.series(torch.from_numpy(mem).to(dev), d_off, 0, gaps)
    for rep in range(3):
        mode = [_native.KRR_PCT_REF_INDEX, _native.KRR_PCT_SORTED_LOWER, _native.KRR_PCT_LINEAR][rep]
        p_num, p_den = _pct(rng)
        q = p_num / p_den / 100.0
        out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
               (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
                ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
        rec = torch.empty((S, 4), dtype=torch.int64, device=dev)
        params = _native.KrrPercentileParams(mode, 0, p_num, p_den, q)
        ctx.simple_run(cs, ms, params, out, records=rec)
        if mode != _native.KRR_PCT_REF_INDEX and seed % 3 == 0:
            # the percentile-only launch (its own window-select rule, krr_plan.h) must agree
            pv = torch.empty(S, dtype=torch.float64, device=dev)
            pn = torch.empty(S, dtype=torch.int64, device=dev)
            pf = torch.empty(S, dtype=torch.int32, device=dev)
            ctx.segmented_percentile(cs, params, pv, pn, pf)
            torch.cuda.synchronize()
            a, b = pv.cpu().numpy(), out["cpu_value"].cpu().numpy()
            same = (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b)) | ((a == 0) & (b == 0))
            assert same.all() and torch.equal(pn, out["cpu_count"]) and torch.equal(pf, out["cpu_flags"]), \
                f"seed {seed}: percentile-only launch differs from the fused one"
        torch.cuda.synchronize()
        ov, on, of = oracle.percentile(cpu, offs, mode, p_num, p_den, q, gaps)
        mv, mn, mf = oracle.seg_max(mem, offs, gaps)
        gv = out["cpu_value"].cpu().numpy()
        same = (gv.view(np.uint64) == ov.view(np.uint64)) | (np.isnan(gv) & np.isnan(ov))
        if mode == _native.KRR_PCT_LINEAR:
            same |= (gv == 0) & (ov == 0)
        tag = f"seed {seed} mode {mode} p {p_num}/{p_den} gaps {gaps}"
        bad = np.nonzero(~same)[0]
        assert bad.size == 0, f"{tag}: cpu differs at {bad[:6]} got {gv[bad[:3]]} want {ov[bad[:3]]}"
        assert np.array_equal(out["cpu_count"].cpu().numpy(), on), tag
        assert np.array_equal(out["cpu_flags"].cpu().numpy().astype(np.uint32), of), tag
        gm = out["mem_value"].cpu().numpy()
        assert ((gm.view(np.uint64) == mv.view(np.uint64)) | (np.isnan(gm) & np.isnan(mv))).all(), tag
        assert np.array_equal(out["mem_count"].cpu().numpy(), mn), tag
        assert np.array_equal(out["mem_flags"].cpu().numpy().astype(np.uint32), mf), tag
        r = rec.cpu().numpy()
        assert np.array_equal(r[:, 0], gv.view(np.int64)) and np.array_equal(r[:, 1], gm.view(np.int64)), tag
    ctx.close()
