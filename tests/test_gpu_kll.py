"""GPU: the KLL-style compactor sketch (krr_kll_build / krr_kll_query) through the C ABI.

Rows and answers are compared bit for bit with the CPU restatement (oracle/kll_ref.py:
the same blocks, coins, merge/carry order and query rule); at full config-5 length the
answers' rank errors, measured against the exact order statistics, stay within the
data-independent bound the rows carry (krr_amd.core.sketch.kll_rank_bound), on the data
shapes where the log-linear histogram has no rank bound (low dispersion, quantised)."""
from decimal import Decimal

import numpy as np
import pytest

from oracle import kll_ref as R

pytestmark = pytest.mark.gpu
SEED = 0x5EED


@pytest.fixture(scope="module")
def ctx():
    from krr_amd import _native

    c = _native.Context(0)
    yield c
    c.close()


def _dev(a, dt=np.float64):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, dt)).to("cuda:0")


def _fleet(rng, lens):
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n = int(offs[-1])
    x = rng.gamma(2.0, 0.05, size=n)
    u = rng.random(n)
    x[u < 0.03] = 0.0
    x[(u >= 0.03) & (u < 0.04)] = -rng.random(int(((u >= 0.03) & (u < 0.04)).sum()))
    x[(u >= 0.04) & (u < 0.06)] = 0.25  # ties
    x[(u >= 0.06) & (u < 0.061)] = np.inf
    x[(u >= 0.061) & (u < 0.063)] = -0.0  # folded into +0 by the sketch (and the restatement)
    x[(u >= 0.063) & (u < 0.065)] = 5e-324 * rng.integers(1, 1000, int(((u >= 0.063) & (u < 0.065)).sum()))
    x[(u >= 0.065) & (u < 0.066)] = -np.inf
    return offs, x


LENS = [0, 1, 2, 3, 300, 511, 512, 513, 1023, 1024, 1025, 1026, 2047, 2048, 5000, 9999, 20_160, 43_200]


def _rows(ctx, x, offs, gaps, budget=512, slice_id=0, seg_base=0):
    import torch

    from krr_amd.core import sketch

    cfg = sketch.KllConfig(budget=budget, seed=SEED)
    ser = ctx.series(_dev(x), _dev(offs, np.int64), 0, gaps)
    rows = sketch.kll_build(ctx, ser, cfg, slice_id=slice_id, seg_base=seg_base)
    torch.cuda.synchronize()
    return cfg, rows.cpu().numpy().view(np.uint64)


def _check_rows(got, x, offs, gaps, budget, slice_id=0, seg_base=0):
    for s in range(offs.size - 1):
        want = R.build_row(x, int(offs[s]), int(offs[s + 1]), budget=budget, seed=SEED, series=seg_base + s,
                           slc=slice_id, gaps=gaps)
        used = R.HDR + sum((int(want[4 + (h >> 2)]) >> (16 * (h & 3))) & 0xFFFF for h in range(16))
        assert np.array_equal(got[s, :used], want[:used]), (s, int(offs[s + 1] - offs[s]),
                                                           got[s, :R.HDR].tolist(), want[:R.HDR].tolist())


@pytest.mark.parametrize("gaps", [False, True])
@pytest.mark.parametrize("budget", [256, 512, 1024])
def test_rows_match_restatement(ctx, gaps, budget):
    rng = np.random.default_rng(budget + gaps)
    lens = rng.permutation(np.array(LENS * 2))
    offs, x = _fleet(rng, lens)
    if gaps:
        x[rng.random(x.size) < 0.15] = np.nan
    _, got = _rows(ctx, x, offs, gaps, budget=budget, seg_base=17)
    _check_rows(got, x, offs, gaps, budget, seg_base=17)


def test_odd_offsets_and_heads(ctx):
    """Segments starting at odd slots (stream_segment's head/tail slots) and one long
    segment whose level counter carries to the top."""
    rng = np.random.default_rng(5)
    lens = np.array([3, 1025, 7, 1027, 1, 172_801, 2049])
    offs, x = _fleet(rng, lens)
    _, got = _rows(ctx, x, offs, False)
    _check_rows(got, x, offs, False, 512)


def _query(ctx, rows_u64, W, cfg, mode, p):
    import torch

    from krr_amd.core import sketch
    from krr_amd.core.engine import percentile_params

    prm = percentile_params(Decimal(p), mode)
    out = sketch.kll_query(ctx, _dev(rows_u64.view(np.int64), np.int64), W, cfg, prm)
    torch.cuda.synchronize()
    return prm, {k: v.cpu().numpy() for k, v in out.items()}


@pytest.mark.parametrize("W", [1, 3])
@pytest.mark.parametrize("mode,p", [("linear", "99"), ("sorted_lower", "99"), ("linear", "50"),
                                    ("sorted_lower", "95.5")])
def test_query_matches_restatement(ctx, W, mode, p):
    """W time slices of every series built as separate launches (slice ids 0..W-1), rows
    interleaved series-major as kll_exchange delivers them, queried together."""
    rng = np.random.default_rng(W * 10 + len(p))
    lens = np.array([0, 1, 5, 900, 3000, 20_000, 60_000, 1024, 4097])
    S = lens.size
    slices = []
    for w in range(W):
        offs, x = _fleet(rng, np.maximum(lens // W, np.minimum(lens, 1)))
        cfg, rows = _rows(ctx, x, offs, False, slice_id=w)
        slices.append(rows)
    merged = np.stack(slices, axis=1).reshape(S * W, -1)
    prm, out = _query(ctx, merged, W, cfg, mode, p)
    for s in range(S):
        v, n, f = R.query(merged[s * W:(s + 1) * W], prm.mode, prm.p_num, prm.p_den, prm.q)
        assert out["count"][s] == n and out["flags"][s] == f
        assert (np.isnan(v) and np.isnan(out["value"][s])) or out["value"][s] == v, (s, out["value"][s], v)


def test_short_series_exact_and_flags(ctx):
    rng = np.random.default_rng(9)
    lens = np.array([0, 1, 2, 100, 511])
    offs, x = _fleet(rng, lens)
    x[offs[3] + 4] = np.nan  # a NaN sample in the compact layout: KRR_FLAG_NAN
    cfg, rows = _rows(ctx, x, offs, False)
    prm, out = _query(ctx, rows, 1, cfg, "linear", "99")
    assert out["flags"][0] == 4 and np.isnan(out["value"][0])
    assert out["flags"][3] == 1 and np.isnan(out["value"][3])
    for s in (1, 2, 4):
        seg = x[offs[s]:offs[s + 1]]
        assert out["flags"][s] == 0 and out["value"][s] == np.percentile(seg, 99.0)


@pytest.mark.parametrize("shape", ["gamma", "low_dispersion", "quantized", "increasing"])
def test_full_length_rank_error_within_bound(ctx, shape):
    """Config-5 length (172,800 samples) over 1 and 8 emulated time slices: the measured
    rank error of p50/p90/p99 against the exact order statistic <= the rows' bound."""
    import torch

    from krr_amd.core import sketch
    from krr_amd.core.engine import percentile_params

    T, S = 172_800, 64
    rng = np.random.default_rng({"gamma": 1, "low_dispersion": 2, "quantized": 3, "increasing": 4}[shape])
    if shape == "gamma":
        x = rng.gamma(2.0, 0.05, (S, T))
    elif shape == "low_dispersion":
        x = 0.25 + rng.uniform(-0.002, 0.002, (S, T))
    elif shape == "quantized":
        x = rng.choice([0.1, 0.2, 0.3, 0.5], (S, T), p=[0.5, 0.3, 0.15, 0.05])
    else:
        x = np.sort(rng.gamma(2.0, 0.05, (S, T)), axis=1)
    xs = np.sort(x, axis=1)
    cfg = sketch.KllConfig(budget=512, seed=SEED)
    for W in (1, 8):
        cuts = [T * w // W for w in range(W + 1)]
        parts = []
        for w in range(W):
            sl = np.ascontiguousarray(x[:, cuts[w]:cuts[w + 1]])
            offs = (np.arange(S + 1) * sl.shape[1]).astype(np.int64)
            ser = ctx.series(_dev(sl.ravel()), _dev(offs, np.int64), sl.shape[1], False)
            parts.append(sketch.kll_build(ctx, ser, cfg, slice_id=w))
        merged = torch.stack(parts, dim=1).reshape(S * W, -1)
        bound = sketch.kll_rank_bound(merged, W)
        assert np.all(bound < (0.03 if W == 1 else 0.015))
        for p in ("50", "90", "99"):
            prm = percentile_params(Decimal(p), "sorted_lower")
            out = sketch.kll_query(ctx, merged, W, cfg, prm)
            v = out["value"].cpu().numpy()
            k = (T - 1) * int(p) // 100
            lt = np.array([np.searchsorted(xs[s], v[s], "left") for s in range(S)])
            le = np.array([np.searchsorted(xs[s], v[s], "right") for s in range(S)])
            err = np.maximum(0, np.maximum(lt - k, k - (le - 1))) / T
            assert np.all(err <= bound), (shape, W, p, float(err.max()), float(bound.min()))


def test_time_sharded_helper_world1(ctx):
    import torch

    from krr_amd.core import sketch
    from krr_amd.core.engine import percentile_params

    rng = np.random.default_rng(4)
    offs, x = _fleet(rng, np.array([10_080] * 8 + [0, 3]))
    ser = ctx.series(_dev(x), _dev(offs, np.int64), 0, False)
    cfg = sketch.KllConfig(budget=512, seed=SEED)
    prm = percentile_params(Decimal("99"), "linear")
    out = sketch.kll_time_sharded(ctx, ser, cfg, prm)
    torch.cuda.synchronize()
    assert out["block"] == (0, 10) and out["rows_per_series"] == 1
    rows = out["rows"].cpu().numpy().view(np.uint64)
    for s in range(10):
        v, n, f = R.query(rows[s:s + 1], prm.mode, prm.p_num, prm.p_den, prm.q)
        got = out["value"][s].item()
        assert out["count"][s].item() == n and (got == v or (np.isnan(got) and np.isnan(v)))


def test_sparse_gapped_series_match_restatement(ctx):
    """A few present samples spread over several chunks (NaN gaps), for many series: kept
    keys may all be compacted away, and the answer then comes from the exact min / max."""
    rng = np.random.default_rng(21)
    S, L = 64, 5000
    x = np.full(S * L, np.nan)
    for s in range(S):
        idx = rng.choice(L, size=int(rng.integers(1, 6)), replace=False)
        x[s * L + idx] = rng.gamma(2.0, 0.05, idx.size)
    offs = (np.arange(S + 1) * L).astype(np.int64)
    cfg, rows = _rows(ctx, x, offs, True, budget=256)
    _check_rows(rows, x, offs, True, 256)
    prm, out = _query(ctx, rows, 1, cfg, "sorted_lower", "50")
    for s in range(S):
        v, n, f = R.query(rows[s:s + 1], prm.mode, prm.p_num, prm.p_den, prm.q)
        assert out["count"][s] == n and out["flags"][s] == f == 0 and out["value"][s] == v and np.isfinite(v)
