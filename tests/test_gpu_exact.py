"""HistoryData outside Prometheus' canonical strings on the MI355X: the
golden cases of tests/golden/simple_strategy_exact.json (the reference's own outputs for
'0.10', '2.00E+7', 25-digit values, float-colliding pairs ...) through the real engine —
the fused kernel pass, then krr_locate for the segments whose answer is a sample object —
via SimpleStrategy.run / run_batch, BatchedRunner.recommend / allocations, and
krr_amd.integration.install() on a Runner built like the reference's (the reference itself
is not on the GPU box: its strategy and runner classes are stood in for by objects of the
same shape; tests/test_integration.py runs the reference's own Runner in the build container)."""
import asyncio
import datetime
import sys
import types
from decimal import Decimal

import numpy as np
import pytest

from krr_amd.core.models.allocations import ResourceAllocations, ResourceType  # noqa: F401 (the stand-in runner's module types)
from test_exact_history import DOC, MINS, PATHS, check_against_golden, hist, obj, strategy

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("path", list(PATHS))
def test_gpu_exact_cases_match_reference(path):
    from krr_amd.core.runner import BatchedRunner

    strat = strategy(path)

    def recommend(objs, hs, cmin, mmin):
        return BatchedRunner(strat, cmin, mmin).recommend(objs, hs)

    def allocations(objs, hs, cmin, mmin):
        return BatchedRunner(strat, cmin, mmin).allocations(objs, hs)

    check_against_golden(path, strat.run_batch, strat.run, recommend, allocations)


def test_gpu_exact_sorted_lower_and_linear():
    import decimal
    import math

    from krr_amd.core.packing import pack_histories

    for path in PATHS:
        for mode in ("sorted_lower", "linear"):
            st = strategy(path, mode).settings
            for c in DOC["cases"]:
                want = c["results"][path]
                h = hist(c)
                if mode == "sorted_lower":
                    if "sorted_error" in want:
                        with pytest.raises(decimal.InvalidOperation):
                            st.calculate_cpu_proposal(h[ResourceType.CPU])
                        continue
                    got = st.calculate_cpu_proposal(h[ResourceType.CPU])
                    assert str(got) == want["sorted"], (path, c["name"])
                elif "linear_hex" in want:
                    got = float(st.run_fleet(pack_histories([h])).cpu_value[0])
                    assert math.isnan(got) if want["linear_hex"] == "nan" else got == float.fromhex(want["linear_hex"])


def test_gpu_locate_against_oracle():
    """krr_locate on random segments with heavy ties, both rank forms, against oracle.locate."""
    import torch

    from krr_amd import _native
    from oracle import oracle

    rng = np.random.default_rng(11)
    lens = rng.integers(0, 3000, 300)
    lens[:4] = [0, 1, 2, 70000]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    x = rng.integers(-3, 6, int(offs[-1])).astype(np.float64) * 0.5
    x[rng.random(x.size) < 0.01] = -0.0
    x[rng.random(x.size) < 0.003] = np.nan
    S = lens.size
    v = np.array([x[o + rng.integers(0, n)] if n else 0.0 for o, n in zip(offs[:-1], lens)])
    v[5] = 99.0  # absent value
    rank = np.where(rng.random(S) < 0.5, -1, np.array([rng.integers(0, n) if n else 0 for n in lens]))
    rank[7] = -2
    rank[8] = 10 ** 6  # past the equal group: pos -1
    ctx = _native.Context(0)
    dev = torch.device("cuda:0")
    series = ctx.series(torch.from_numpy(x).to(dev), torch.from_numpy(offs).to(dev), int(lens.max()))
    out = [torch.full((S,), -7, dtype=torch.int64, device=dev) for _ in range(3)]
    ctx.locate(series, torch.from_numpy(v).to(dev), torch.from_numpy(rank.astype(np.int64)).to(dev), *out)
    torch.cuda.synchronize()
    want = oracle.locate(x, offs, v, rank)
    for g, w in zip(out, want):
        g = g.cpu().numpy()
        keep = rank >= -1
        assert np.array_equal(g[keep], w[keep])
        assert (g[~keep] == -7).all()  # skipped segments untouched
    ctx.close()


# ---- krr_amd.integration.install() on a reference-shaped Runner -----------------------------

def _stand_in_reference_strategy(path):
    """An object of the reference SimpleStrategy's shape: class robusta_krr.strategies.simple.
    SimpleStrategy, pydantic-v1 settings whose __fields_set__ says which fields the CLI set."""
    from krr_amd.strategies.simple import SimpleStrategySettings

    mod = types.ModuleType("robusta_krr.strategies.simple")

    class SimpleStrategy:
        def __init__(self, settings):
            self.settings = settings

    SimpleStrategy.__module__ = mod.__name__
    mod.SimpleStrategy = SimpleStrategy
    kw = PATHS[path]
    return mod, SimpleStrategy(SimpleStrategySettings(**kw) if kw else SimpleStrategySettings())


class Runner:
    """runner.py:17-137's attributes that install() reads."""

    def __init__(self, strategy, cases, cmin, mmin):
        self._strategy = strategy
        self.config = types.SimpleNamespace(cpu_min_value=cmin, memory_min_value=mmin)
        self._cases = cases

    def _get_prometheus_loader(self, cluster):
        cases = self._cases

        class Loader:  # prometheus.py:108-155's output shape: {pod: [Decimal]}
            async def gather_data(self, obj, resource, period, *, timeframe):
                assert isinstance(period, datetime.timedelta)
                c = cases[int(obj.name.split("-")[1])]
                pods = c["cpu" if resource == ResourceType.CPU else "mem"]
                return {k: [Decimal(s) for s in v] for k, v in pods.items() if v}

        return Loader()

    async def _gather_objects_recommendations(self, objects):
        raise AssertionError("install() did not patch the runner")


@pytest.mark.parametrize("path", ["cli_99_5", "default_int"])
def test_gpu_exact_through_integration_install(monkeypatch, path):
    from krr_amd import integration

    mod, ref_strategy = _stand_in_reference_strategy(path)
    monkeypatch.setitem(sys.modules, "robusta_krr.strategies.simple", mod)
    cases = [c for c in DOC["cases"] if "rounded" in c["results"][path]]
    cmin, mmin = MINS.get(path, (5, 10))
    integration.install(Runner)
    try:
        runner = Runner(ref_strategy, cases, cmin, mmin)
        assert integration.hip_strategy(ref_strategy) is not None
        objects = [obj(f"app-{i:03d}") for i in range(len(cases))]
        got = asyncio.run(runner._gather_objects_recommendations(objects))
    finally:
        integration.uninstall(Runner)
    assert len(got) == len(cases) >= 30
    for c, a in zip(cases, got):
        want = c["results"][path]["rounded"]
        for rt, key in ((ResourceType.CPU, "cpu_request"), (ResourceType.Memory, "mem_request"),
                        (ResourceType.Memory, "mem_limit")):
            v = a.requests[rt] if key != "mem_limit" else a.limits[rt]
            assert (v == "?" and want[key] == "NaN") or str(v) == want[key], (c["name"], key, v, want[key])
