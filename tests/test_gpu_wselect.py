"""wselect — the one-pass window select for mid percentiles (krr_kernels.hip
wselect_segment) — bit-exact against the oracle, and its fallback to the two-pass
hselect when the window misses (krr_get_stats counts those segments).

The window narrows around the target's estimated rank among the samples seen so far,
so exchangeable series (config 2 / config 3 data) must finish in one pass, while
series whose later half differs from the first (regime changes, monotone trends) may
miss and fall back — the answer is exact either way."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

MODES = {"sorted_lower": 1, "linear": 2}


@pytest.fixture(scope="module")
def ctx():
    from krr_amd import _native

    c = _native.Context(0)
    yield c
    c.close()


def _run(ctx, vals, offs, mode, p_num, p_den, gaps, fused=False):
    import torch

    from krr_amd import _native

    dev = torch.device("cuda:0")
    dv = torch.from_numpy(np.ascontiguousarray(vals, np.float64)).to(dev)
    do = torch.from_numpy(np.ascontiguousarray(offs, np.int64)).to(dev)
    S = offs.size - 1
    q = float(p_num) / float(p_den) / 100.0
    prm = _native.KrrPercentileParams(MODES[mode], 0, p_num, p_den, q)
    before = ctx.wselect_fallbacks()
    ser = ctx.series(dv, do, int(np.diff(offs).max()), gaps)
    if fused:
        out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
               (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
                ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
        ctx.simple_run(ser, ser, prm, out)
        ov, on, of = out["cpu_value"], out["cpu_count"], out["cpu_flags"]
    else:
        ov = torch.empty(S, dtype=torch.float64, device=dev)
        on = torch.empty(S, dtype=torch.int64, device=dev)
        of = torch.empty(S, dtype=torch.int32, device=dev)
        ctx.segmented_percentile(ser, prm, ov, on, of)
    torch.cuda.synchronize()
    fb = ctx.wselect_fallbacks() - before
    return (ov.cpu().numpy(), on.cpu().numpy(), of.cpu().numpy().astype(np.uint32)), fb


def _check(got, vals, offs, mode, p_num, p_den, gaps, tag):
    q = float(p_num) / float(p_den) / 100.0
    wv, wn, wf = oracle.percentile(vals, offs, MODES[mode], p_num, p_den, q, gaps)
    gv, gn, gf = got
    assert np.array_equal(gn, wn), f"{tag}: counts"
    assert np.array_equal(gf, wf), f"{tag}: flags {gf[gf != wf][:4]} vs {wf[gf != wf][:4]}"
    same = (gv.view(np.uint64) == wv.view(np.uint64)) | (np.isnan(gv) & np.isnan(wv))
    if mode == "linear":
        same |= (gv == 0) & (wv == 0)
    bad = np.nonzero(~same)[0]
    assert bad.size == 0, f"{tag}: values differ at {bad[:8]}: {gv[bad[:4]]} vs {wv[bad[:4]]}"


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
@pytest.mark.parametrize("pct", [(50, 1), (25, 1), (75, 1), (90, 1), (4999, 100), (10, 1)])
def test_exchangeable_series_finish_in_one_pass(ctx, mode, pct):
    """Config-2-shaped (5 x 10,080, NaN gaps) and config-3-shaped (1..14 days, compact)
    gamma series: exact, and (nearly) no segment falls back — the window spans 4 standard
    deviations of the rank estimate, a miss per shrink is a ~1e-4 event."""
    rng = np.random.default_rng(1000 + pct[0])
    S, L = 60, 50400
    v = rng.gamma(2.0, 0.05, size=S * L)
    gap = rng.random(S * L) < rng.uniform(0, 0.2, size=S).repeat(L)
    v[gap] = np.nan
    offs = (np.arange(S + 1) * L).astype(np.int64)
    for fused in (False, True):
        got, fb = _run(ctx, v, offs, mode, *pct, gaps=True, fused=fused)
        _check(got, v, offs, mode, *pct, True, f"config2-shape fused={fused}")
        assert fb <= 1, f"{fb} fallbacks on {S} exchangeable gapped series (p={pct})"
    lens = rng.integers(1, 15, size=300) * 1440
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    v = rng.gamma(2.0, 0.05, size=int(offs[-1]))
    got, fb = _run(ctx, v, offs, mode, *pct, gaps=False, fused=True)
    _check(got, v, offs, mode, *pct, False, "config3-shape")
    assert fb <= 3, f"{fb} fallbacks on 300 exchangeable compact series (p={pct})"


def _adversarial(L, rng):
    segs = {}
    r = rng.random(L)
    r[int(0.6 * L):] += 10.0  # regime change: the estimate from the first 60% is wrong
    segs["regime_change_up"] = r
    d = rng.random(L) + 10.0
    d[int(0.4 * L):] -= 10.0
    segs["regime_change_down"] = d
    segs["increasing"] = np.arange(L, dtype=np.float64)
    segs["decreasing"] = np.arange(L, 0, -1, dtype=np.float64)
    segs["sawtooth"] = np.tile(np.arange(1000, dtype=np.float64), L // 1000 + 1)[:L]
    z = rng.gamma(2.0, 0.05, size=L)
    z[rng.random(L) < 0.7] = 0.0  # the median is a crowded key: a one-key window (count only)
    segs["mostly_zero"] = z
    sz = rng.normal(size=L)
    u = rng.random(L)
    sz[u < 0.25] = 0.0
    sz[(u >= 0.25) & (u < 0.5)] = -0.0
    sz[(u >= 0.5) & (u < 0.53)] = np.inf
    sz[(u >= 0.53) & (u < 0.56)] = -np.inf
    segs["signed_zero_inf"] = sz
    segs["constant"] = np.full(L, 0.125)
    segs["two_values"] = np.where(rng.random(L) < 0.5, 1.0, 2.0)
    segs["negatives"] = -rng.gamma(2.0, 0.05, size=L)
    segs["log_uniform"] = np.exp(rng.uniform(-700, 700, size=L)) * np.where(rng.random(L) < 0.5, -1.0, 1.0)
    return segs


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_adversarial_orders_exact_with_fallback(ctx, mode):
    rng = np.random.default_rng(4242)
    for L in (50400, 20160, 7000):
        segs = _adversarial(L, rng)
        names = list(segs)
        vals = np.concatenate([segs[k] for k in names])
        offs = (np.arange(len(names) + 1) * L).astype(np.int64)
        fallbacks = 0
        for pct in [(50, 1), (30, 1), (70, 1), (90, 1)]:
            got, fb = _run(ctx, vals, offs, mode, *pct, gaps=False)
            fallbacks += fb
            wv, wn, wf = oracle.percentile(vals, offs, MODES[mode], pct[0], pct[1], pct[0] / pct[1] / 100, False)
            for i, nm in enumerate(names):
                one = tuple(a[i:i + 1] for a in got)
                _check(one, vals[offs[i]:offs[i + 1]], np.array([0, L], np.int64), mode, *pct, False,
                       f"{nm} L={L} p={pct}")
        if L == 50400:  # regime changes and trends do miss the window: the fallback ran
            assert fallbacks > 0


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
@pytest.mark.parametrize("lens", [(50400, 0, 30000, 50400, 17000, 50400), (20160, 0, 12000, 20160, 7000, 20160)],
                         ids=["long_kernel", "short_kernel"])
def test_gaps_nan_and_empty(ctx, mode, lens):
    """Gapped segments (incl. negative NaN gaps, all-gap and empty segments) and a real
    NaN sample in the compact layout (flagged) through the window select: the long-segment
    kernel (per-lane counts) and the 16-waves/CU kernel, whose scalar counts recount every
    chunk holding a NaN and take negative NaNs back out of "below"."""
    rng = np.random.default_rng(77)
    lens = np.array(lens, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    v = rng.gamma(2.0, 0.05, size=int(offs[-1]))
    v[rng.random(v.size) < 0.3] = np.nan
    neg_nan = np.frombuffer(np.uint64(0xFFF8000000000001).tobytes(), dtype=np.float64)[0]
    v[rng.random(v.size) < 0.02] = neg_nan
    v[offs[2]:offs[3]] = np.nan  # all gaps
    for pct in [(50, 1), (33, 1)]:
        got, _ = _run(ctx, v, offs, mode, *pct, gaps=True, fused=True)
        _check(got, v, offs, mode, *pct, True, f"gapped p={pct}")
    c = np.nan_to_num(v, nan=0.5)
    c[offs[4] + 1234] = np.nan  # a real NaN sample: KRR_FLAG_NAN
    got, _ = _run(ctx, c, offs, mode, 50, 1, gaps=False)
    _check(got, c, offs, mode, 50, 1, False, "compact with a NaN")


def _missing_fleet(L, rng, copies=6):
    """Short segments (the 16-waves/CU window kernel, whose misses go through the separate
    miss list + k_hselect_list) that the window cannot hold: monotone trends and regime
    changes, interleaved with exchangeable series that do not miss."""
    segs = []
    for _ in range(copies):
        segs.append(np.arange(L, dtype=np.float64) + rng.random())           # increasing
        r = rng.random(L)
        r[int(0.6 * L):] += 10.0
        segs.append(r)                                                      # regime change
        segs.append(rng.gamma(2.0, 0.05, size=L))                            # exchangeable
    return np.concatenate(segs), (np.arange(len(segs) + 1) * L).astype(np.int64)


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
@pytest.mark.parametrize("L", [20160, 7000])
def test_short_segment_miss_list_across_consecutive_launches(ctx, mode, L):
    """The miss-list path (segments < 32,768 slots): every launch misses some segments, and
    consecutive launches on one ctx alternate between the list's two counters (launch k
    zeroes launch k-1's) — five launches in a row, different data and percentiles each
    time, no sync in between; every one exact against the oracle and every one with misses."""
    import torch

    from krr_amd import _native

    rng = np.random.default_rng(L + MODES[mode])
    dev = torch.device("cuda:0")
    runs = []
    before = ctx.wselect_fallbacks()
    for i, pct in enumerate([(50, 1), (40, 1), (60, 1), (50, 1), (35, 1)]):
        vals, offs = _missing_fleet(L, rng)
        S = offs.size - 1
        dv = torch.from_numpy(vals).to(dev)
        do = torch.from_numpy(offs).to(dev)
        ser = ctx.series(dv, do, L, False)
        prm = _native.KrrPercentileParams(MODES[mode], 0, pct[0], pct[1], pct[0] / pct[1] / 100.0)
        out = [torch.empty(S, dtype=dt, device=dev) for dt in (torch.float64, torch.int64, torch.int32)]
        ctx.segmented_percentile(ser, prm, *out)
        runs.append((vals, offs, pct, out, dv, do, ser))
    torch.cuda.synchronize()
    total = ctx.wselect_fallbacks() - before
    assert total >= 5 * 2, f"only {total} misses over 5 launches of trend / regime-change series"
    for vals, offs, pct, out, *_ in runs:
        got = (out[0].cpu().numpy(), out[1].cpu().numpy(), out[2].cpu().numpy().astype(np.uint32))
        _check(got, vals, offs, mode, *pct, False, f"L={L} p={pct}")


def test_two_streams_share_one_ctx(ctx):
    """One ctx, window launches with misses on two streams, issued back to back with no
    host sync: the miss list and its counters are shared, so a launch on the other stream
    waits for the previous launch's miss pass (the ctx's event) — both results exact."""
    import torch

    from krr_amd import _native

    rng = np.random.default_rng(5)
    dev = torch.device("cuda:0")
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
    runs = []
    for i in range(6):
        L = (20160, 7000)[i % 2]
        vals, offs = _missing_fleet(L, rng, copies=4)
        S = offs.size - 1
        st = streams[i % 2]
        with torch.cuda.stream(st):
            dv = torch.from_numpy(vals).to(dev, non_blocking=False)
            do = torch.from_numpy(offs).to(dev, non_blocking=False)
            out = [torch.empty(S, dtype=dt, device=dev) for dt in (torch.float64, torch.int64, torch.int32)]
        st.synchronize()  # inputs in place; the launches below are not synchronised with each other
        runs.append((vals, offs, out, dv, do, st, ctx.series(dv, do, L, False)))
    for i, (vals, offs, out, dv, do, st, ser) in enumerate(runs):
        prm = _native.KrrPercentileParams(MODES["linear"], 0, 50, 1, 0.5)
        ctx.segmented_percentile(ser, prm, *out, st)
    torch.cuda.synchronize()
    for vals, offs, out, *_ in runs:
        got = (out[0].cpu().numpy(), out[1].cpu().numpy(), out[2].cpu().numpy().astype(np.uint32))
        _check(got, vals, offs, "linear", 50, 1, False, "two streams")
