"""GPU parity of the segmented kernels against the CPU oracle (bit-exact).

Calls go through the C ABI (krr_amd._native -> libkrr_amd.so).  The oracle is
pinned to the reference by tests/test_oracle_golden.py.
"""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

MODES = {"ref_index": 0, "sorted_lower": 1, "linear": 2}


@pytest.fixture(scope="module")
def ctx():
    from krr_amd import _native

    c = _native.Context(0)
    yield c
    c.close()


def _run_gpu(ctx, values, offsets, mode, p_num, p_den, gaps=False, maxlen=0):
    import torch

    from krr_amd import _native

    dev = torch.device("cuda:0")
    dv = torch.from_numpy(np.ascontiguousarray(values, np.float64)).to(dev)
    do = torch.from_numpy(np.ascontiguousarray(offsets, np.int64)).to(dev)
    S = offsets.size - 1
    ov = torch.empty(S, dtype=torch.float64, device=dev)
    on = torch.empty(S, dtype=torch.int64, device=dev)
    of = torch.empty(S, dtype=torch.int32, device=dev)
    ser = ctx.series(dv, do, maxlen, gaps)
    if mode == "max":
        ctx.segmented_max(ser, ov, on, of)
    else:
        q = float(p_num) / float(p_den) / 100.0
        ctx.segmented_percentile(ser, _native.KrrPercentileParams(MODES[mode], 0, p_num, p_den, q), ov, on, of)
    torch.cuda.synchronize()
    return ov.cpu().numpy(), on.cpu().numpy(), of.cpu().numpy().astype(np.uint32)


def _run_gpu_fused(ctx, values, offsets, mode, p_num, p_den, gaps=False):
    """The CPU half of krr_simple_run's fused launch (the memory half gets the same series)."""
    import torch

    from krr_amd import _native

    dev = torch.device("cuda:0")
    dv = torch.from_numpy(np.ascontiguousarray(values, np.float64)).to(dev)
    do = torch.from_numpy(np.ascontiguousarray(offsets, np.int64)).to(dev)
    S = offsets.size - 1
    out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
           (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
            ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
    q = float(p_num) / float(p_den) / 100.0
    ser = ctx.series(dv, do, 0, gaps)
    ctx.simple_run(ser, ser, _native.KrrPercentileParams(MODES[mode], 0, p_num, p_den, q), out)
    torch.cuda.synchronize()
    return (out["cpu_value"].cpu().numpy(), out["cpu_count"].cpu().numpy(),
            out["cpu_flags"].cpu().numpy().astype(np.uint32))


def _oracle(values, offsets, mode, p_num, p_den, gaps=False):
    if mode == "max":
        return oracle.seg_max(values, offsets, gaps)
    q = float(p_num) / float(p_den) / 100.0
    return oracle.percentile(values, offsets, MODES[mode], p_num, p_den, q, gaps)


def _assert_same(got, want, mode, tag=""):
    gv, gn, gf = got
    wv, wn, wf = want
    assert np.array_equal(gn, wn), f"{tag} counts differ at {np.nonzero(gn != wn)[0][:10]}"
    assert np.array_equal(gf, wf), f"{tag} flags differ at {np.nonzero(gf != wf)[0][:10]}"
    gb, wb = gv.view(np.uint64), wv.view(np.uint64)
    nan_both = np.isnan(gv) & np.isnan(wv)
    same = (gb == wb) | nan_both
    if mode == "linear":  # sign of a zero result is unspecified (numpy's partition is unstable)
        same |= (gv == 0) & (wv == 0)
    bad = np.nonzero(~same)[0]
    assert bad.size == 0, f"{tag} values differ at {bad[:10]}: got {gv[bad[:5]]} want {wv[bad[:5]]}"


def _ragged(rng, nseg, lo, hi):
    lens = rng.integers(lo, hi, size=nseg)
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)


PCTS = [(99, 1), (50, 1), (1, 10), (100, 1), (999, 10), (75, 1), (1, 1)]


@pytest.mark.parametrize("mode", ["ref_index", "sorted_lower", "linear", "max"])
@pytest.mark.parametrize("pct", PCTS)
def test_random_ragged(ctx, mode, pct):
    if mode == "max" and pct != PCTS[0]:
        pytest.skip("max has no percentile")
    rng = np.random.default_rng(hash((mode, pct)) & 0xFFFF)
    offs = _ragged(rng, 300, 0, 6000)
    offs[1:] += 0  # keep
    vals = rng.gamma(2.0, 0.05, size=int(offs[-1]))
    got = _run_gpu(ctx, vals, offs, mode, *pct)
    want = _oracle(vals, offs, mode, *pct)
    _assert_same(got, want, mode, f"{mode} p={pct}")


@pytest.mark.parametrize("mode", ["ref_index", "sorted_lower", "linear", "max"])
def test_gapped_dense(ctx, mode):
    rng = np.random.default_rng(11)
    S, L = 64, 5 * 2016
    vals = rng.gamma(2.0, 0.05, size=S * L)
    mask = rng.random(S * L) < 0.15
    vals[mask] = np.nan
    vals[3 * L:4 * L] = np.nan  # an all-gap segment
    offs = (np.arange(S + 1) * L).astype(np.int64)
    for pct in [(99, 1), (50, 1), (1, 10)]:
        got = _run_gpu(ctx, vals, offs, mode, *pct, gaps=True)
        want = _oracle(vals, offs, mode, *pct, gaps=True)
        _assert_same(got, want, mode, f"gaps {mode} p={pct}")


@pytest.mark.parametrize("mode", ["sorted_lower", "linear", "max", "ref_index"])
def test_ties_and_specials(ctx, mode):
    rng = np.random.default_rng(5)
    offs = _ragged(rng, 200, 0, 3000)
    N = int(offs[-1])
    vals = rng.integers(0, 3, size=N).astype(np.float64)  # heavy ties
    special = rng.random(N)
    vals[special < 0.02] = -0.0
    vals[(special >= 0.02) & (special < 0.025)] = np.inf
    vals[(special >= 0.025) & (special < 0.03)] = -np.inf
    for pct in [(99, 1), (50, 1), (1, 10), (100, 1)]:
        got = _run_gpu(ctx, vals, offs, mode, *pct)
        want = _oracle(vals, offs, mode, *pct)
        _assert_same(got, want, mode, f"ties {mode} p={pct}")


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_adversarial_order(ctx, mode):
    """Monotone and sawtooth series force a compaction on nearly every chunk."""
    L = 50400
    inc = np.arange(L, dtype=np.float64) * 1e-3
    dec = inc[::-1].copy()
    saw = np.tile(np.arange(1000, dtype=np.float64), L // 1000 + 1)[:L]
    const = np.full(L, 0.25)
    vals = np.concatenate([inc, dec, saw, const])
    offs = (np.arange(5) * L).astype(np.int64)
    for pct in [(99, 1), (50, 1), (1, 10), (9999, 100)]:
        got = _run_gpu(ctx, vals, offs, mode, *pct)
        want = _oracle(vals, offs, mode, *pct)
        _assert_same(got, want, mode, f"adversarial {mode} p={pct}")


def test_signed_zero_rules(ctx):
    """Python max() keeps the first of -0/+0; sorted() is stable for them."""
    segs = [[-0.0, 0.0], [0.0, -0.0], [-1.0, -0.0, 0.0, -0.0], [0.0, -0.0, -0.0, 0.0, -2.0]]
    vals = np.array([x for s in segs for x in s])
    offs = np.concatenate([[0], np.cumsum([len(s) for s in segs])]).astype(np.int64)
    for mode in ("max", "sorted_lower"):
        for pct in [(99, 1), (50, 1), (1, 10), (100, 1)]:
            got = _run_gpu(ctx, vals, offs, mode, *pct)
            want = _oracle(vals, offs, mode, *pct)
            _assert_same(got, want, mode, f"zeros {mode} p={pct}")


@pytest.mark.parametrize("mode", ["ref_index", "sorted_lower", "linear", "max"])
def test_nan_values_compact(ctx, mode):
    """Without gap masking a NaN is a sample: flags + NaN per the reference's rules."""
    rng = np.random.default_rng(9)
    offs = _ragged(rng, 50, 1, 500)
    vals = rng.gamma(2.0, 0.05, size=int(offs[-1]))
    vals[rng.random(vals.size) < 0.003] = np.nan
    got = _run_gpu(ctx, vals, offs, mode, 99, 1)
    want = _oracle(vals, offs, mode, 99, 1)
    _assert_same(got, want, mode, f"nan {mode}")


def test_unaligned_offsets(ctx):
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 2500, size=257) | 1  # odd lengths -> odd starts
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    vals = rng.normal(size=int(offs[-1]))
    for mode in ("ref_index", "sorted_lower", "linear", "max"):
        got = _run_gpu(ctx, vals, offs, mode, 99, 1)
        want = _oracle(vals, offs, mode, 99, 1)
        _assert_same(got, want, mode, f"unaligned {mode}")


def test_large_candidate_set_uses_hselect(ctx):
    """p=50 on 50,400-sample series would keep ~25k keys: the histogram + collect path."""
    rng = np.random.default_rng(21)
    S, L = 40, 50400
    vals = rng.gamma(2.0, 0.05, size=S * L)
    offs = (np.arange(S + 1) * L).astype(np.int64)
    for mode in ("sorted_lower", "linear"):
        got = _run_gpu(ctx, vals, offs, mode, 50, 1)
        want = _oracle(vals, offs, mode, 50, 1)
        _assert_same(got, want, mode, f"hselect {mode}")


def _hselect_segments(L, rng):
    """Series that stress hselect's range estimate, refinement and zero handling."""
    segs = {}
    segs["gamma"] = rng.gamma(2.0, 0.05, size=L)
    z = rng.gamma(2.0, 0.05, size=L)
    z[rng.random(L) < 0.7] = 0.0
    segs["mostly_zero"] = z
    m = rng.random(L) * 1e-9  # the strided probe sees only 1.0: ranks fall below its range
    m[(np.arange(64) * L) // 64] = 1.0
    segs["probe_misled_low"] = m
    h = 1.0 + rng.random(L) * 1e-3
    h[(np.arange(64) * L) // 64] = 1e-6  # ... and above it
    h[rng.random(L) < 0.4] = 1e12
    segs["probe_misled_high"] = h
    c = rng.gamma(2.0, 0.05, size=L)
    c[rng.random(L) < 0.6] = 0.5  # one crowded value in the middle
    segs["crowded_middle"] = c
    segs["normal_signed"] = rng.normal(size=L)
    sp = rng.normal(size=L)
    u = rng.random(L)
    sp[u < 0.2] = -0.0
    sp[(u >= 0.2) & (u < 0.4)] = 0.0
    sp[(u >= 0.4) & (u < 0.45)] = np.inf
    sp[(u >= 0.45) & (u < 0.5)] = -np.inf
    segs["signed_zero_inf"] = sp
    segs["log_uniform"] = np.exp(rng.uniform(-690, 690, size=L)) * np.where(rng.random(L) < 0.3, -1.0, 1.0)
    segs["increasing"] = np.arange(L, dtype=np.float64)
    segs["decreasing"] = np.arange(L, dtype=np.float64)[::-1].copy()
    segs["constant"] = np.full(L, 3.25)
    segs["two_values"] = np.where(rng.random(L) < 0.5, 1.0, 2.0)
    return segs


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_hselect_adversarial(ctx, mode):
    rng = np.random.default_rng(77)
    L = 50400
    segs = _hselect_segments(L, rng)
    names = list(segs)
    vals = np.concatenate([segs[k] for k in names])
    offs = (np.arange(len(names) + 1) * L).astype(np.int64)
    for pct in [(50, 1), (75, 1), (90, 1), (25, 1), (10, 1), (95, 1), (333, 10)]:
        got = _run_gpu(ctx, vals, offs, mode, *pct)
        want = _oracle(vals, offs, mode, *pct)
        for i, nm in enumerate(names):
            one = tuple(a[i:i + 1] for a in got), tuple(a[i:i + 1] for a in want)
            _assert_same(one[0], one[1], mode, f"hselect {nm} {mode} p={pct}")


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_hselect_gapped_and_ragged(ctx, mode):
    """Mixed single-pass / hselect segments in one launch, NaN gaps (incl. negative NaN)."""
    rng = np.random.default_rng(78)
    offs = _ragged(rng, 120, 0, 30000)
    N = int(offs[-1])
    vals = rng.gamma(2.0, 0.05, size=N)
    vals[rng.random(N) < 0.2] = np.nan
    neg_nan = np.frombuffer(np.uint64(0xFFF8000000000001).tobytes(), dtype=np.float64)[0]
    vals[rng.random(N) < 0.01] = neg_nan
    vals[rng.random(N) < 0.1] = 0.0
    for pct in [(50, 1), (80, 1), (20, 1), (99, 1)]:
        got = _run_gpu(ctx, vals, offs, mode, *pct, gaps=True)
        want = _oracle(vals, offs, mode, *pct, gaps=True)
        _assert_same(got, want, mode, f"hselect gapped {mode} p={pct}")
    vals_c = np.nan_to_num(vals, nan=0.25)
    vals_c[rng.random(N) < 0.00005] = neg_nan  # a few real NaN samples: flagged
    for pct in [(50, 1), (65, 1)]:
        got = _run_gpu(ctx, vals_c, offs, mode, *pct)
        want = _oracle(vals_c, offs, mode, *pct)
        _assert_same(got, want, mode, f"hselect compact {mode} p={pct}")


def test_maxlen_autodetect(ctx):
    rng = np.random.default_rng(4)
    offs = _ragged(rng, 100, 0, 3000)
    vals = rng.gamma(2.0, 0.05, size=int(offs[-1]))
    got = _run_gpu(ctx, vals, offs, "linear", 99, 1, maxlen=0)
    want = _oracle(vals, offs, "linear", 99, 1)
    _assert_same(got, want, "linear", "autodetect")


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_long_series_single_pass_large_buffer(ctx, mode):
    """30d@15s series (172,800 slots) at p99 keep 1,730 keys: the single pass with the
    larger (2,560-key) buffer, not hselect.  Adversarial orders included: increasing
    (every sample a candidate), decreasing, constant, two values, gapped, signed zeros."""
    rng = np.random.default_rng(31)
    L = 172_800
    segs = [rng.gamma(2.0, 0.05, L), np.arange(L, dtype=np.float64), np.arange(L, dtype=np.float64)[::-1].copy(),
            np.full(L, 0.5), np.where(rng.random(L) < 0.995, 1.0, 2.0)]
    g = rng.gamma(2.0, 0.05, L)
    g[rng.random(L) < 0.3] = np.nan
    segs.append(g)
    z = rng.normal(size=L)
    z[rng.random(L) < 0.5] = -0.0
    segs.append(z)
    vals = np.concatenate(segs)
    offs = (np.arange(len(segs) + 1) * L).astype(np.int64)
    for p_num, p_den in ((99, 1), (995, 10), (97, 1)):
        got = _run_gpu(ctx, vals, offs, mode, p_num, p_den, gaps=True)
        want = _oracle(vals, offs, mode, p_num, p_den, gaps=True)
        _assert_same(got, want, mode, f"long single pass {mode} p{p_num}/{p_den}")


def _probe_slots(L):
    """Slots hselect's band probe reads (KRR_HSEL_BAND): 16 from each of nb evenly
    spread blocks, nb = L/400 rounded down to a multiple of 8, within [16, 128]."""
    nb = min(max((L // 400) & ~7, 16), 128)
    starts = (np.arange(nb, dtype=np.int64) * (L - 16)) // (nb - 1)
    return (starts[:, None] + np.arange(16)[None, :]).ravel()


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_hselect_band(ctx, mode):
    """The one-pass band of hselect: hits, misses in both directions (the probe's blocks
    unrepresentative of the segment), overflow (a crowded value inside the band), probes
    that are mostly gaps, and lengths at the band's minimum (16,384 slots)."""
    rng = np.random.default_rng(91)
    segs = []
    for L in (4095, 4096, 8191, 16383, 16384, 20160, 50400, 172800):
        segs.append(("gamma", L, rng.gamma(2.0, 0.05, size=L), False))
    L = 50400
    ps = _probe_slots(L)
    lo = rng.random(L) + 10.0
    lo[ps] = rng.random(ps.size)  # the probe sees only small values: the band lies too low
    segs.append(("probe_low", L, lo, False))
    hi = rng.random(L)
    hi[ps] = 1e6 + rng.random(ps.size)  # ... and too high
    segs.append(("probe_high", L, hi, False))
    half = rng.random(L)
    half[ps[: ps.size // 2]] = -1.0  # half the probe below everything: band shifted
    segs.append(("probe_shifted", L, half, False))
    crowd = rng.gamma(2.0, 0.05, size=L)
    crowd[rng.random(L) < 0.3] = np.median(crowd)  # thousands of ties inside the band
    segs.append(("crowded_band", L, crowd, False))
    g = rng.gamma(2.0, 0.05, size=L)
    g[ps] = np.nan  # probe entirely in gaps: no band
    segs.append(("probe_in_gaps", L, g, True))
    g2 = rng.gamma(2.0, 0.05, size=L)
    g2[rng.random(L) < 0.5] = np.nan  # half gaps everywhere: the present count is estimated
    segs.append(("half_gaps", L, g2, True))
    sz = rng.normal(size=L)
    u = rng.random(L)
    sz[u < 0.3] = 0.0
    sz[(u >= 0.3) & (u < 0.5)] = -0.0
    sz[(u >= 0.5) & (u < 0.52)] = np.inf
    sz[(u >= 0.52) & (u < 0.54)] = -np.inf
    segs.append(("signed_zero_inf", L, sz, False))
    for gaps in (False, True):
        chosen = [(nm, v) for nm, _, v, g_ in segs if g_ == gaps]
        if not chosen:
            continue
        vals = np.concatenate([v for _, v in chosen])
        offs = np.concatenate([[0], np.cumsum([v.size for _, v in chosen])]).astype(np.int64)
        for pct in [(50, 1), (95, 1), (90, 1), (10, 1), (75, 1), (4999, 100), (1, 1)]:
            got = _run_gpu(ctx, vals, offs, mode, *pct, gaps=gaps)
            want = _oracle(vals, offs, mode, *pct, gaps=gaps)
            for i, (nm, _) in enumerate(chosen):
                one = tuple(a[i:i + 1] for a in got), tuple(a[i:i + 1] for a in want)
                _assert_same(one[0], one[1], mode, f"band {nm} gaps={gaps} {mode} p={pct}")


def _select_probe_slots(L):
    """Slots the single-pass select's start-threshold probe reads (KRR_SELECT_PROBE):
    64 consecutive slots from each of 16 evenly spread blocks."""
    starts = (np.arange(16, dtype=np.int64) * (L - 64)) // 15
    return (starts[:, None] + np.arange(64)[None, :]).ravel()


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_select_probe_start_threshold(ctx, mode):
    """Tail percentiles of long segments start the single-pass select at a probe-estimated
    threshold: hits, a probe that sees only huge values (threshold too high: the segment
    is streamed again from the lowest key), only tiny values (too low: compactions as
    before), a crowded value at the threshold, a probe in gaps, signed zeros and infinities,
    monotone series, and lengths on both sides of the probe's gate."""
    rng = np.random.default_rng(95)
    segs = []
    for L in (6000, 10080, 14000, 15000, 17280, 20160):
        segs.append(("gamma", L, rng.gamma(2.0, 0.05, size=L), False))
    L = 20160
    ps = _select_probe_slots(L)
    hi = rng.random(L)
    hi[ps] = 1e6 + rng.random(ps.size)
    segs.append(("probe_high", L, hi, False))
    lo = rng.random(L) + 10.0
    lo[ps] = rng.random(ps.size)
    segs.append(("probe_low", L, lo, False))
    crowd = rng.gamma(2.0, 0.05, size=L)
    crowd[rng.random(L) < 0.2] = np.quantile(crowd, 0.96)
    segs.append(("crowded_at_thr", L, crowd, False))
    segs.append(("constant", L, np.full(L, 0.25), False))
    segs.append(("increasing", L, np.arange(L, dtype=np.float64), False))
    segs.append(("decreasing", L, np.arange(L, 0, -1, dtype=np.float64), False))
    sz = rng.normal(size=L)
    u = rng.random(L)
    sz[u < 0.3] = 0.0
    sz[(u >= 0.3) & (u < 0.5)] = -0.0
    sz[(u >= 0.5) & (u < 0.56)] = np.inf
    sz[(u >= 0.56) & (u < 0.58)] = -np.inf
    segs.append(("signed_zero_inf", L, sz, False))
    g = rng.gamma(2.0, 0.05, size=L)
    g[ps] = np.nan
    segs.append(("probe_in_gaps", L, g, True))
    g2 = rng.gamma(2.0, 0.05, size=L)
    g2[rng.random(L) < 0.3] = np.nan
    g2[ps[::3]] = 50.0 + rng.random(ps[::3].size)
    segs.append(("gaps_probe_high", L, g2, True))
    g3 = rng.gamma(2.0, 0.05, size=L)
    g3[rng.random(L) < 0.15] = np.nan
    segs.append(("gaps", L, g3, True))
    for gaps in (False, True):
        chosen = [(nm, v) for nm, _, v, g_ in segs if g_ == gaps]
        vals = np.concatenate([v for _, v in chosen])
        offs = np.concatenate([[0], np.cumsum([v.size for _, v in chosen])]).astype(np.int64)
        for pct in [(95, 1), (96, 1), (97, 1), (98, 1), (99, 1), (9499, 100), (5, 1)]:
            got = _run_gpu(ctx, vals, offs, mode, *pct, gaps=gaps)
            want = _oracle(vals, offs, mode, *pct, gaps=gaps)
            for i, (nm, _) in enumerate(chosen):
                one = tuple(a[i:i + 1] for a in got), tuple(a[i:i + 1] for a in want)
                _assert_same(one[0], one[1], mode, f"probe {nm} gaps={gaps} {mode} p={pct}")


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
@pytest.mark.parametrize("L", [50400, 100800])
def test_select_probe_large_buffer(ctx, mode, L, fused):
    """Long launches at tail percentiles through both launch kinds: p94-p97 and p95.49
    (1,515-3,027 kept keys) take the window select (krr_plan.h single_pass_ok / window_select; the plan is pinned by
    tests/test_abi.py::test_select_plan_decisions; the biggest probe-backed buffers by
    test_select_probe_biggest_buffer): hits, a probe that sees only huge values (re-stream),
    only tiny values, gaps, and a short segment sharing the launch.  p5 / p6 keep the BOTTOM
    keys, for which there is no probe: window select."""
    rng = np.random.default_rng(97)
    ps = _select_probe_slots(L)
    segs = [("gamma", rng.gamma(2.0, 0.05, size=L), False), ("short", rng.gamma(2.0, 0.05, size=3000), False)]
    hi = rng.random(L)
    hi[ps] = 1e6 + rng.random(ps.size)
    segs.append(("probe_high", hi, False))
    lo = rng.random(L) + 10.0
    lo[ps] = rng.random(ps.size)
    segs.append(("probe_low", lo, False))
    crowd = rng.gamma(2.0, 0.05, size=L)
    crowd[rng.random(L) < 0.2] = np.quantile(crowd, 0.955)
    segs.append(("crowded_at_thr", crowd, False))
    g = rng.gamma(2.0, 0.05, size=L)
    g[rng.random(L) < 0.2] = np.nan
    segs.append(("gaps", g, True))
    g2 = rng.gamma(2.0, 0.05, size=L)
    g2[ps] = np.nan
    segs.append(("probe_in_gaps", g2, True))
    for gaps in (False, True):
        chosen = [(nm, v) for nm, v, g_ in segs if g_ == gaps]
        vals = np.concatenate([v for _, v in chosen])
        offs = np.concatenate([[0], np.cumsum([v.size for _, v in chosen])]).astype(np.int64)
        for pct in [(94, 1), (95, 1), (96, 1), (97, 1), (9549, 100), (5, 1), (6, 1)]:
            got = (_run_gpu_fused if fused else _run_gpu)(ctx, vals, offs, mode, *pct, gaps=gaps)
            want = _oracle(vals, offs, mode, *pct, gaps=gaps)
            for i, (nm, _) in enumerate(chosen):
                one = tuple(a[i:i + 1] for a in got), tuple(a[i:i + 1] for a in want)
                _assert_same(one[0], one[1], mode, f"probe-large {nm} gaps={gaps} {mode} p={pct}")


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_select_probe_biggest_buffer(ctx, mode):
    """A 500,000-slot series at p99.6 (2,001 kept keys, 0.4%): the percentile-only launch keeps
    the single pass behind the probe with a buffer above 2,560 keys (the biggest buffers the
    window-select rules still leave to it); parity with a probe that sees only huge values."""
    from decimal import Decimal

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    L = 500_000
    info = _native.select_plan(L, percentile_params(Decimal("99.6"), mode))
    assert info.hselect == 0 and info.probe == 1 and 2560 < info.cap_keys <= 3712, (info.tkeep, info.cap_keys)
    rng = np.random.default_rng(996)
    a = rng.gamma(2.0, 0.05, size=L)
    b = rng.random(L)
    b[_select_probe_slots(L)] = 1e6 + rng.random(_select_probe_slots(L).size)
    vals = np.concatenate([a, b])
    offs = np.array([0, L, 2 * L], dtype=np.int64)
    got = _run_gpu(ctx, vals, offs, mode, 996, 10)
    want = _oracle(vals, offs, mode, 996, 10)
    _assert_same(got, want, mode, f"biggest buffer {mode}")
