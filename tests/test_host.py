"""Host-side logic (no GPU): Prometheus decimals, packing, params, plugin registry,
batched runner fallback for custom strategies, and loud failure without HIP."""
import asyncio
import datetime
import math
from decimal import Decimal

import numpy as np
import pytest

from krr_amd.api.models import K8sObjectData, ResourceAllocations, ResourceRecommendation, ResourceType
from krr_amd.api.strategies import BaseStrategy, StrategySettings
from krr_amd.core.engine import percentile_params
from krr_amd.core.packing import pack_dense_grid, pack_histories, pack_prometheus
from krr_amd.core.rounding import round_value
from krr_amd.core.runner import BatchedRunner
from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings
from krr_amd.utils.prom_decimal import prom_decimal, prom_format


def _obj(pods=("p0", "p1")):
    return K8sObjectData(cluster=None, name="web", container="app", pods=list(pods), namespace="default",
                         kind="Deployment", allocations=ResourceAllocations(requests={}, limits={}))


def test_prom_decimal_random_roundtrip():
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.gamma(2, 0.05, 2000), np.floor(rng.normal(2e8, 2e7, 2000)),
                         rng.lognormal(0, 20, 2000), [0.0, -0.0, 1e22, 1e-300, 5e-324, 123.0]])
    for x in xs:
        s = prom_format(float(x))
        assert "e" not in s.lower() or s in ("+Inf", "-Inf")
        assert float(s) == x
        assert Decimal(s).as_tuple() == prom_decimal(float(x)).as_tuple()
    assert prom_format(2e8) == "200000000" and prom_format(-0.0) == "-0"


def test_round_value_decimal_not_float():
    # ceil(2.007 * 1000) is 2008 in float64 but 2007 in Decimal
    assert str(round_value(Decimal("2.007"), ResourceType.CPU)) == "2.007"
    assert str(round_value(Decimal("0.001"), ResourceType.CPU)) == "0.005000000000000000104083408559"
    assert str(round_value(Decimal("21000000.00"), ResourceType.Memory)) == "2.1E+7"
    assert round_value(None, ResourceType.CPU) is None
    assert round_value(Decimal("NaN"), ResourceType.Memory).is_nan()


def test_pack_histories_keeps_pod_order_and_drops_nothing_else():
    h = {ResourceType.CPU: {"b": [Decimal("0.2"), Decimal("0.1")], "a": [Decimal("0.9")]},
         ResourceType.Memory: {"a": [Decimal("5")]}}
    e = {ResourceType.CPU: {}, ResourceType.Memory: {}}
    f = pack_histories([h, e, h])
    assert f.cpu.offsets.tolist() == [0, 3, 3, 6]
    assert f.cpu.values.tolist() == [0.2, 0.1, 0.9, 0.2, 0.1, 0.9]
    assert f.mem.offsets.tolist() == [0, 1, 1, 2]
    assert f.cpu.max_len == 3


def test_pack_prometheus_first_series_and_empty_pods():
    pod_a = [{"values": [[1, "0.5"], [2, "NaN"]]}, {"values": [[1, "9"]]}]  # only the first series counts
    pod_b = []                                                             # no data: dropped
    pod_c = [{"values": [[1, "+Inf"], [2, "0.25"]]}]
    ps = pack_prometheus([[pod_a, pod_b, pod_c], [pod_b]])
    assert ps.offsets.tolist() == [0, 4, 4]
    v = ps.values
    assert v[0] == 0.5 and math.isnan(v[1]) and math.isinf(v[2]) and v[3] == 0.25


def test_pack_dense_grid_present_samples_equal_compact():
    rng = np.random.default_rng(2)
    pods = []
    for _ in range(3):
        ts = np.sort(rng.choice(100, size=60, replace=False)).astype(float) * 60.0
        pods.append((ts, rng.gamma(2, 0.05, ts.size)))
    dense = pack_dense_grid([pods], start=0.0, step=60.0, slots=100)
    assert dense.gaps_are_nan and dense.offsets.tolist() == [0, 300]
    present = dense.values[~np.isnan(dense.values)]
    assert np.array_equal(present, np.concatenate([v for _, v in pods]))


def test_percentile_params_exact_rationals():
    p = percentile_params(Decimal("99"), "ref_index")
    assert (p.p_num, p.p_den, p.mode) == (99, 1, 0)
    p = percentile_params(Decimal("99.9"), "sorted_lower")
    assert (p.p_num, p.p_den, p.mode) == (999, 10, 1)
    p = percentile_params(99, "linear")
    assert p.q == 0.99 and p.mode == 2
    p = percentile_params(Decimal(99.9), "ref_index")  # binary float made exact: 2^-k denominator
    assert p.p_den <= 10**15
    # more digits than the kernels' exact floor takes: an approximation that only sizes buffers,
    # and the reference's own index rule (a table bound at launch; tests/test_index_rule.py)
    p = percentile_params(Decimal("99.12345678901234567"), "ref_index")
    assert p.p_den <= 10**15 and p.rule.needs_table(2) and not p.k_table
    with pytest.raises(ValueError):
        percentile_params(Decimal("0"), "ref_index")
    with pytest.raises(ValueError):
        percentile_params(Decimal("100.5"), "ref_index")
    with pytest.raises(ValueError):
        percentile_params(Decimal("50"), "median")


def test_registry_and_settings_type():
    assert BaseStrategy.find("simple") is SimpleStrategy
    assert BaseStrategy.find("SIMPLE") is SimpleStrategy
    assert SimpleStrategy.get_settings_type() is SimpleStrategySettings
    assert str(SimpleStrategy(SimpleStrategySettings())) == "Simple"
    with pytest.raises(ValueError):
        BaseStrategy.find("nope")
    s = SimpleStrategySettings(cpu_percentile="99", memory_buffer_percentage="5")
    assert s.cpu_percentile == Decimal("99") and isinstance(s.cpu_percentile, Decimal)
    assert isinstance(SimpleStrategySettings().cpu_percentile, int)  # pydantic v1: defaults unvalidated
    assert s.memory_buffer() == Decimal("1.05")
    assert SimpleStrategySettings().memory_buffer() == Decimal(1.05)


class _CustomSettings(StrategySettings):
    param_1: Decimal = Decimal(99)
    param_2: Decimal = Decimal(105_000)


class MyCustomStrategy(BaseStrategy[_CustomSettings]):
    """examples/custom_strategy.py:13-29 shape: a plugin without run_batch."""

    def run(self, history_data, object_data):
        return {
            ResourceType.CPU: ResourceRecommendation(request=self.settings.param_1, limit=None),
            ResourceType.Memory: ResourceRecommendation(request=self.settings.param_2, limit=self.settings.param_2),
        }


def test_custom_strategy_runs_through_batched_runner():
    assert BaseStrategy.find("mycustom") is MyCustomStrategy
    runner = BatchedRunner(MyCustomStrategy(_CustomSettings()))
    objs = [_obj(), _obj()]
    allocs = runner.allocations(objs, [{}, {}])
    assert allocs[0].requests[ResourceType.CPU] == Decimal("99")
    assert allocs[0].requests[ResourceType.Memory] == Decimal("1E+7")  # clamped to 10 MB
    assert allocs[1].limits[ResourceType.CPU] is None


def test_async_gather_with_fake_loader():
    class Loader:
        async def gather_data(self, object, resource, period, *, timeframe):
            assert period == datetime.timedelta(hours=336) and timeframe == datetime.timedelta(minutes=15)
            return {p: [Decimal("1")] for p in object.pods}

    runner = BatchedRunner(MyCustomStrategy(_CustomSettings()))
    out = asyncio.run(runner.gather_objects_recommendations([_obj()], Loader()))
    assert out[0].requests[ResourceType.CPU] == Decimal("99")


def test_nan_becomes_question_mark():
    a = ResourceAllocations(requests={ResourceType.CPU: Decimal("NaN"), ResourceType.Memory: "1Gi"},
                            limits={ResourceType.CPU: None, ResourceType.Memory: Decimal("5")})
    assert a.requests[ResourceType.CPU] == "?"
    assert a.requests[ResourceType.Memory] == Decimal(2**30)


def test_simple_strategy_fails_loudly_without_hip():
    import torch

    from krr_amd import _native

    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    h = {ResourceType.CPU: {"p": [Decimal("0.1")]}, ResourceType.Memory: {"p": [Decimal("1")]}}
    with pytest.raises(_native.NativeUnavailable):
        SimpleStrategy(SimpleStrategySettings()).run(h, _obj())
