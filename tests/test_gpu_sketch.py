"""GPU: sketch mode and the time-sharded helpers (config 5), through the C ABI.

Build and query are checked bit-exactly against the numpy restatement
(oracle/sketch_ref.py); the exact time-sharded REF_INDEX / max against the C
oracle on the concatenated series; rank_of / select_present against numpy."""
import numpy as np
import pytest

from oracle import oracle, sketch_ref

pytestmark = pytest.mark.gpu
M, ELO, OCT = 5, -24, 36


@pytest.fixture(scope="module")
def ctx():
    from krr_amd import _native

    c = _native.Context(0)
    yield c
    c.close()


def _dev(a, dt=np.float64):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, dt)).to("cuda:0")


def _fleet(rng, S=40, lo=0, hi=9000):
    lens = rng.integers(lo, hi, size=S)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    x = rng.gamma(2.0, 0.05, size=int(offs[-1]))
    u = rng.random(x.size)
    x[u < 0.03] = 0.0
    x[(u >= 0.03) & (u < 0.04)] = -rng.random(int(((u >= 0.03) & (u < 0.04)).sum()))
    x[(u >= 0.04) & (u < 0.045)] = 1e-9
    x[(u >= 0.045) & (u < 0.05)] = 1e6
    x[(u >= 0.05) & (u < 0.052)] = np.inf
    return offs, x


def _build(ctx, x, offs, gaps):
    import torch

    from krr_amd.core import sketch

    cfg = sketch.SketchConfig(M, ELO, OCT)
    ser = ctx.series(_dev(x), _dev(offs, np.int64), 0, gaps)
    out = sketch.build(ctx, ser, cfg)
    torch.cuda.synchronize()
    return cfg, out


@pytest.mark.parametrize("gaps", [False, True])
def test_build_matches_restatement(ctx, gaps):
    rng = np.random.default_rng(1)
    offs, x = _fleet(rng)
    if gaps:
        x[rng.random(x.size) < 0.2] = np.nan
    _, out = _build(ctx, x, offs, gaps)
    counts = out["counts"].cpu().numpy().view(np.uint32)
    for s in range(offs.size - 1):
        c, mn, mx = sketch_ref.build(x[offs[s]:offs[s + 1]], M, ELO, OCT)
        assert np.array_equal(counts[s], c), s
        assert np.array_equal(out["vmin"][s].cpu().numpy(), mn, equal_nan=True)
        assert np.array_equal(out["vmax"][s].cpu().numpy(), mx, equal_nan=True)
    assert (out["flags"].cpu().numpy() == 0).all()


def test_build_flags_nan_in_compact(ctx):
    x = np.array([1.0, np.nan, 2.0, 3.0, 4.0])
    offs = np.array([0, 2, 5], dtype=np.int64)
    _, out = _build(ctx, x, offs, False)
    assert list(out["flags"].cpu().numpy()) == [1, 0]


@pytest.mark.parametrize("mode,pct", [("linear", 99), ("linear", 50), ("sorted_lower", 95), ("sorted_lower", 1),
                                      ("linear", 100), ("sorted_lower", 33)])
def test_query_matches_restatement(ctx, mode, pct):
    import torch

    from krr_amd.core import sketch
    from krr_amd.core.engine import percentile_params

    rng = np.random.default_rng(pct)
    offs, x = _fleet(rng)
    cfg, out = _build(ctx, x, offs, False)
    params = percentile_params(pct, mode)
    res = sketch.query(ctx, out, cfg, params)
    torch.cuda.synchronize()
    got = res["value"].cpu().numpy()
    counts = out["counts"].cpu().numpy().view(np.uint32)
    for s in range(offs.size - 1):
        want, n = sketch_ref.query(counts[s], float(out["vmin"][s]), float(out["vmax"][s]), M, ELO, OCT, mode,
                                   params.p_num, params.p_den, params.q)
        assert int(res["count"][s]) == n
        if n == 0:
            assert np.isnan(got[s]) and int(res["flags"][s]) & 4
        elif np.isnan(want):  # e.g. lerp of inf and inf: NaN, sign not specified
            assert np.isnan(got[s])
        else:
            assert np.float64(got[s]).view(np.uint64) == np.float64(want).view(np.uint64), (s, got[s], want)


def test_time_slices_merge_exactly(ctx):
    """Sketches of 8 time slices, summed, equal the sketch of the whole series."""
    import torch

    rng = np.random.default_rng(3)
    S, L, W = 16, 172_800 // 8, 8
    x = rng.gamma(2.0, 0.05, size=(S, L * W))
    whole_offs = (np.arange(S + 1) * L * W).astype(np.int64)
    _, whole = _build(ctx, x.ravel(), whole_offs, False)
    total = None
    for r in range(W):
        part = np.ascontiguousarray(x[:, r * L:(r + 1) * L])
        _, pr = _build(ctx, part.ravel(), (np.arange(S + 1) * L).astype(np.int64), False)
        total = pr["counts"].to(torch.int64) if total is None else total + pr["counts"].to(torch.int64)
    assert torch.equal(total, whole["counts"].to(torch.int64))


def test_rank_of_and_select_present(ctx):
    import torch

    rng = np.random.default_rng(4)
    offs, x = _fleet(rng, S=30)
    x[rng.random(x.size) < 0.1] = np.nan
    S = offs.size - 1
    probe = np.array([x[offs[s]] if offs[s + 1] > offs[s] else 0.1 for s in range(S)])
    probe = np.where(np.isnan(probe), 0.1, probe)
    ser = ctx.series(_dev(x), _dev(offs, np.int64), 0, True)
    lt = torch.empty(S, dtype=torch.int64, device="cuda:0")
    le = torch.empty_like(lt)
    ctx.rank_of(ser, _dev(probe), lt, le)
    ks = np.array([(s * 37) % max(1, offs[s + 1] - offs[s]) for s in range(S)], dtype=np.int64)
    ks[::7] = -1
    out = _dev(np.full(S, -5.0))
    ctx.select_present(ser, _dev(ks, np.int64), out)
    torch.cuda.synchronize()
    for s in range(S):
        seg = x[offs[s]:offs[s + 1]]
        pres = seg[~np.isnan(seg)]
        assert int(lt[s]) == int((pres < probe[s]).sum()) and int(le[s]) == int((pres <= probe[s]).sum())
        got = float(out[s])
        if ks[s] < 0:
            assert got == -5.0
        elif ks[s] < pres.size:
            assert np.float64(got).view(np.uint64) == np.float64(pres[ks[s]]).view(np.uint64)
        else:
            assert np.isnan(got)


@pytest.mark.parametrize("gaps", [False, True])
def test_time_sharded_exact_world1(ctx, gaps):
    import torch

    from krr_amd.core import sketch
    from krr_amd.core.engine import percentile_params

    rng = np.random.default_rng(6)
    offs, x = _fleet(rng, S=25)
    if gaps:
        x[rng.random(x.size) < 0.2] = np.nan
    ser = ctx.series(_dev(x), _dev(offs, np.int64), 0, gaps)
    params = percentile_params(99, "ref_index")
    res = sketch.refindex_time_sharded(ctx, ser, params)
    ov, on, of = oracle.percentile(x, offs, 0, 99, 1, 0.99, gaps)
    assert np.array_equal(res["value"].view(np.uint64), ov.view(np.uint64)) or \
        np.array_equal(res["value"], ov, equal_nan=True)
    assert np.array_equal(res["count"], on) and np.array_equal(res["flags"], of)
    S = offs.size - 1
    mv = torch.empty(S, dtype=torch.float64, device="cuda:0")
    mn = torch.empty(S, dtype=torch.int64, device="cuda:0")
    mf = torch.empty(S, dtype=torch.int32, device="cuda:0")
    ctx.segmented_max(ser, mv, mn, mf)
    m = sketch.max_time_sharded(mv, mn, mf)
    wv, wn, wf = oracle.seg_max(x, offs, gaps)
    assert np.array_equal(m["value"], wv, equal_nan=True) and np.array_equal(m["count"], wn)
    assert np.array_equal(m["flags"], wf)


def test_synth_window_concatenates(ctx):
    import torch

    S, L, W = 6, 7000, 4
    dev = torch.device("cuda:0")
    whole = torch.empty(S * L, dtype=torch.float64, device=dev)
    offs = torch.arange(S + 1, dtype=torch.int64, device=dev) * L
    ctx.synth_fill(whole, offs, 99, 0, 0, False)
    parts = []
    for r in range(W):
        n = L // W
        buf = torch.empty(S * n, dtype=torch.float64, device=dev)
        ctx.synth_fill_window(buf, torch.arange(S + 1, dtype=torch.int64, device=dev) * n, 99, 0, 0, False,
                              r * n, L)
        parts.append(buf.view(S, n))
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts, dim=1).reshape(-1), whole)


def _same(got, want):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    return np.array_equal(got.view(np.uint64), want.view(np.uint64)) or \
        (np.array_equal(got, want, equal_nan=True))


@pytest.mark.parametrize("gaps", [False, True])
@pytest.mark.parametrize("mode,pct", [("sorted_lower", "99"), ("linear", "99"), ("sorted_lower", "50"),
                                      ("linear", "5"), ("linear", "100"), ("sorted_lower", "0.1")])
def test_exact_refinement_world1(ctx, gaps, mode, pct):
    """locate -> collect -> refine on one rank equals the single-window select
    (krr_segmented_percentile path, C oracle) bit for bit, incl. zeros, negatives,
    +inf, tiny/huge values (lumped bins) and empty series."""
    import torch
    from decimal import Decimal

    from krr_amd.core import sketch
    from krr_amd.core.engine import percentile_params

    rng = np.random.default_rng(11)
    offs, x = _fleet(rng, S=30)
    if gaps:
        x[rng.random(x.size) < 0.2] = np.nan
    ser = ctx.series(_dev(x), _dev(offs, np.int64), 0, gaps)
    cfg = sketch.SketchConfig(M, ELO, OCT)
    params = percentile_params(Decimal(pct), mode)
    local = sketch.build(ctx, ser, cfg)
    merged = sketch.merge_time_sharded(local)
    res = sketch.exact_time_sharded(ctx, ser, local, merged, cfg, params)
    torch.cuda.synchronize()
    ov, on, of = oracle.percentile(x, offs, params.mode, params.p_num, params.p_den, params.q, gaps)
    got = res["value"].cpu().numpy()
    if mode == "linear":  # the zero sign of a LINEAR result is unspecified (numpy's partition)
        assert np.array_equal(got, ov, equal_nan=True)
    else:
        assert _same(got, ov)
    assert np.array_equal(res["count"].cpu().numpy(), on)
    assert np.array_equal(res["flags"].cpu().numpy().astype(np.uint32), of)
    assert res["collected"] < x.size // 4  # only the located bins travel


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_exact_refinement_emulated_ranks(ctx, mode):
    """Three time slices per series handled as three 'ranks' in one process: local
    sketches summed (the reduce-scatter), per-slice collect, lists concatenated in
    slice order (the all-to-all), refine — equals the select over whole series."""
    import torch
    from decimal import Decimal

    from krr_amd import _native
    from krr_amd.core import sketch
    from krr_amd.core.engine import percentile_params

    rng = np.random.default_rng(12)
    S, L, W = 20, 6000, 3
    x = rng.gamma(2.0, 0.05, size=(S, L))
    x[rng.random(x.shape) < 0.15] = np.nan
    x[2] = np.where(rng.random(L) < 0.5, 0.0, -0.0)  # all-zero series: the sign comes from position
    x[3, :4000] = np.nan                              # empty in the first two slices
    x[4] = np.nan                                     # empty
    x[5, ::7] = -x[5, ::7]
    cfg = sketch.SketchConfig(M, ELO, OCT)
    params = percentile_params(Decimal("99"), mode)
    cuts = np.array_split(np.arange(L), W)
    sers, locals_ = [], []
    for c in cuts:
        xs = np.ascontiguousarray(x[:, c]).ravel()
        o = (np.arange(S + 1) * c.size).astype(np.int64)
        ser = ctx.series(_dev(xs), _dev(o, np.int64), 0, True)
        sers.append(ser)
        locals_.append(sketch.build(ctx, ser, cfg))
    merged = {"counts": sum(l["counts"] for l in locals_), "flags": torch.zeros(S, dtype=torch.int32, device="cuda:0")}
    loc = sketch.locate(ctx, merged, cfg, params)
    lists = []
    for ser, l in zip(sers, locals_):
        cnt = torch.empty(S, dtype=torch.int64, device="cuda:0")
        ctx.sketch_range_count(l["counts"], cfg.params(), loc, cnt)
        off = torch.zeros(S + 1, dtype=torch.int64, device="cuda:0")
        off[1:] = torch.cumsum(cnt, 0)
        vals = torch.empty(max(int(off[-1]), 1), dtype=torch.float64, device="cuda:0")
        got_n = torch.empty(S, dtype=torch.int64, device="cuda:0")
        ctx.sketch_collect(ser, cfg.params(), loc, off, vals, got_n)
        assert torch.equal(got_n, cnt)
        lists.append((vals.cpu().numpy(), off.cpu().numpy()))
    cat, offs = [], [0]
    for s in range(S):
        for v, o in lists:
            cat.append(v[o[s]:o[s + 1]])
        offs.append(offs[-1] + sum(o[s + 1] - o[s] for _, o in lists))
    cser = ctx.series(_dev(np.concatenate(cat) if cat else np.zeros(1)), _dev(np.array(offs), np.int64), 0, False)
    ov_ = torch.empty(S, dtype=torch.float64, device="cuda:0")
    on_ = torch.empty(S, dtype=torch.int64, device="cuda:0")
    of_ = torch.empty(S, dtype=torch.int32, device="cuda:0")
    ctx.sketch_refine(cser, loc, ov_, on_, of_)
    full = x.ravel()
    fo = (np.arange(S + 1) * L).astype(np.int64)
    wv, wn, wf = oracle.percentile(full, fo, params.mode, params.p_num, params.p_den, params.q, True)
    got = ov_.cpu().numpy()
    if mode == "linear":
        assert np.array_equal(got, wv, equal_nan=True)
    else:
        assert _same(got, wv)
    assert np.array_equal(on_.cpu().numpy(), wn)
    assert np.array_equal(of_.cpu().numpy().astype(np.uint32), wf)
    assert (of_.cpu().numpy() & _native.KRR_FLAG_CAPACITY).sum() == 0
