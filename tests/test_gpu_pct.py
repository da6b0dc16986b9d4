"""cpu_percentile values whose Decimal index product rounds, on the MI355X.

The fixture runs of tests/golden/simple_strategy_pct.json (the reference's own outputs at
n in {1, 2, 3, 1001, 10080, 172800, 1000003}) through SimpleStrategy.run_batch / run,
BatchedRunner.recommend and krr_amd.integration.install() for the CLI and direct-construction
settings paths; the SORTED_LOWER / LINEAR rules against the fixture; and the kernels' k_table
path (REF_INDEX and SORTED_LOWER, compact and NaN-gapped layouts, fused and standalone) bit for
bit against oracle.percentile with the same table."""
import asyncio
import sys
import types
from decimal import Decimal

import numpy as np
import pytest

from test_gpu_exact import Runner
from test_index_rule import DOC, PATHS, history, runs_for, settings, strategy

pytestmark = pytest.mark.gpu


def rows(res):
    from krr_amd.core.models.allocations import ResourceType

    return (str(res[ResourceType.CPU].request), str(res[ResourceType.Memory].request))


@pytest.mark.parametrize("path", PATHS)
def test_gpu_pct_runs_match_reference(path):
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.rounding import format_result
    from krr_amd.core.runner import BatchedRunner
    from test_exact_history import obj

    runs = runs_for(path, 10**7)
    assert len(runs) == 70
    for p in sorted({r["p"] for r in runs}):
        mine = [r for r in runs if r["p"] == p]
        strat = strategy(path, p)
        hs = [history(r["n"]) for r in mine]
        got = strat.run_batch(hs)
        rec = BatchedRunner(strat, 5, 10).recommend([obj(f"o{i}") for i in range(len(hs))], hs)
        for r, g, rr in zip(mine, got, rec):
            want = (r["raw"]["cpu_request"], r["raw"]["mem_request"])
            assert rows(g) == want, (p, r["n"])
            assert rows(format_result(g)) == (r["rounded"]["cpu_request"], r["rounded"]["mem_request"])
            assert rows(rr) == (r["rounded"]["cpu_request"], r["rounded"]["mem_request"]), (p, r["n"])
            if r["n"] <= 172800:  # the per-object call (coalesced launch)
                assert rows(strat.run(history(r["n"]), None)) == want, (p, r["n"])
            assert str(rr[ResourceType.Memory].limit) == r["rounded"]["mem_limit"]


def test_gpu_pct_sorted_and_linear():
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.packing import pack_histories

    for r in runs_for("cli", 10**7):
        h = history(r["n"])
        st = settings("cli", r["p"], "sorted_lower")
        assert str(st.calculate_cpu_proposal(h[ResourceType.CPU])) == r["sorted"], (r["p"], r["n"])
        lin = settings("cli", r["p"], "linear")
        assert float(lin.run_fleet(pack_histories([h])).cpu_value[0]) == float.fromhex(r["linear_hex"])


@pytest.mark.parametrize("path", ["cli", "direct_decimal"])
def test_gpu_pct_through_integration_install(monkeypatch, path):
    from krr_amd import integration
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.utils.prom_decimal import prom_format
    from test_exact_history import obj

    from pct_inputs import cpu_values, mem_values, pods_of

    def case(n):
        c, m = cpu_values(n), mem_values(n)
        cpu, mem, o = {}, {}, 0
        for i, ln in enumerate(pods_of(n)):
            cpu[f"pod{i}"] = [prom_format(float(x)) for x in c[o:o + ln]]
            mem[f"pod{i}"] = [prom_format(float(x)) for x in m[o:o + ln]]
            o += ln
        return {"cpu": cpu, "mem": mem}

    mod = types.ModuleType("robusta_krr.strategies.simple")

    class SimpleStrategy:
        def __init__(self, settings):
            self.settings = settings

    SimpleStrategy.__module__ = mod.__name__
    mod.SimpleStrategy = SimpleStrategy
    monkeypatch.setitem(sys.modules, "robusta_krr.strategies.simple", mod)
    runs = [r for r in runs_for(path, 172800)]
    integration.install(Runner)
    try:
        for p in sorted({r["p"] for r in runs}):
            mine = [r for r in runs if r["p"] == p]
            ref = SimpleStrategy(settings(path, p))
            cases = [case(r["n"]) for r in mine]
            runner = Runner(ref, cases, 5, 10)
            objects = [obj(f"app-{i:03d}") for i in range(len(cases))]
            got = asyncio.run(runner._gather_objects_recommendations(objects))
            for r, a in zip(mine, got):
                assert str(a.requests[ResourceType.CPU]) == r["rounded"]["cpu_request"], (p, r["n"])
                assert str(a.requests[ResourceType.Memory]) == r["rounded"]["mem_request"], (p, r["n"])
    finally:
        integration.uninstall(Runner)


@pytest.mark.parametrize("gaps", [False, True])
@pytest.mark.parametrize("p", ["99.99999999999999999999999999", "33.33333333333333333333333333",
                               "50.00000000000000000000000001", "12.3456789012345678"])
def test_gpu_k_table_kernels_match_oracle(p, gaps):
    """krr_segmented_percentile and krr_simple_run with the reference's index table: every
    segment bit for bit against oracle.percentile reading the same table."""
    import torch

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params
    from oracle import oracle

    rng = np.random.default_rng(17)
    lens = rng.integers(0, 6000, 400)
    lens[:6] = [0, 1, 2, 3, 70000, 1440]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    x = np.round(rng.gamma(2.0, 0.05, int(offs[-1])), 4)
    if gaps:
        x[rng.random(x.size) < 0.1] = np.nan
    ctx = _native.Context(0)
    dev = torch.device("cuda:0")
    S = lens.size
    series = ctx.series(torch.from_numpy(x).to(dev), torch.from_numpy(offs).to(dev), int(lens.max()), gaps)
    for mode in ("ref_index", "sorted_lower"):
        prm = percentile_params(Decimal(p), mode)
        tab = prm.rule.table(int(lens.max()))
        want = oracle.percentile(x, offs, prm.mode, prm.p_num, prm.p_den, prm.q, gaps, k_table=tab)
        outs = []
        o1 = [torch.empty(S, dtype=dt, device=dev) for dt in (torch.float64, torch.int64, torch.int32)]
        ctx.segmented_percentile(series, prm, *o1)
        outs.append(o1)
        o2 = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
              (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
               ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
        ctx.simple_run(series, series, prm, o2)
        outs.append([o2["cpu_value"], o2["cpu_count"], o2["cpu_flags"]])
        torch.cuda.synchronize()
        for v, n, f in outs:
            v = v.cpu().numpy()
            same = (v.view(np.uint64) == want[0].view(np.uint64)) | (np.isnan(v) & np.isnan(want[0]))
            assert same.all(), (p, mode, gaps, np.flatnonzero(~same)[:5])
            assert np.array_equal(n.cpu().numpy(), want[1])
            assert np.array_equal(f.cpu().numpy().astype(np.uint32), want[2])
        # the table changes answers somewhere (else this test would not test it)
        if mode == "ref_index" and p.startswith("99.99"):
            exact = oracle.percentile(x, offs, prm.mode, prm.p_num, prm.p_den, prm.q, gaps)
            assert (exact[0].view(np.uint64) != want[0].view(np.uint64)).any()
    ctx.close()


def test_gpu_k_table_too_short_is_refused():
    import torch

    from krr_amd import _native

    ctx = _native.Context(0)
    dev = torch.device("cuda:0")
    offs = torch.tensor([0, 10, 30], dtype=torch.int64, device=dev)
    vals = torch.arange(30, dtype=torch.float64, device=dev)
    tab = torch.arange(16, dtype=torch.int64, device=dev)
    out = [torch.empty(2, dtype=dt, device=dev) for dt in (torch.float64, torch.int64, torch.int32)]
    for mode in (_native.KRR_PCT_REF_INDEX, _native.KRR_PCT_SORTED_LOWER):
        prm = _native.KrrPercentileParams(mode, 0, 99, 1, 0.99, tab.data_ptr(), tab.numel())
        with pytest.raises(_native.NativeError) as e:
            ctx.segmented_percentile(ctx.series(vals, offs, 20), prm, *out)
        assert e.value.code == _native.KRR_E_INVALID
    ctx.close()
