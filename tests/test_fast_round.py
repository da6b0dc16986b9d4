"""Native batched rounding (libkrr_host.so krr_round_simple) vs the Python
restatement of the reference's Decimal path (strategies/simple.py:24-29 +
core/runner.py:49-86, pinned by tests/test_oracle_golden.py): identical Decimal
objects — digits AND exponent — for every object, both settings paths."""
import decimal
import math
from decimal import Decimal

import numpy as np
import pytest

from krr_amd.core.engine import RawResults
from krr_amd.core.fast_round import format_simple_batch, round_strings
from krr_amd.core.models.allocations import ResourceType
from krr_amd.core.rounding import format_result
from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings


def _settings(path):
    if path == "cli":  # typer/click hand pydantic strings -> exact Decimal('1.05')
        return SimpleStrategySettings(cpu_percentile="99", memory_buffer_percentage="5")
    if path == "cli7":
        return SimpleStrategySettings(cpu_percentile="95", memory_buffer_percentage="7.5")
    return SimpleStrategySettings()  # int defaults: Decimal(1.05 as float)


def _raw(seed, n=20000):
    rng = np.random.default_rng(seed)
    cpu = rng.gamma(2.0, 0.05, n)
    k = rng.integers(0, 12, n)
    cpu[k == 0] = rng.integers(0, 5000, int((k == 0).sum())) / 1000.0  # exact thousandths: ceil() edge
    cpu[k == 1] = 0.0
    cpu[k == 2] = -0.0
    cpu[k == 3] = rng.random(int((k == 3).sum())) * 0.006  # near the 5m floor
    cpu[k == 4] = np.exp(rng.uniform(-40, 40, int((k == 4).sum())))
    cpu[k == 5] = -rng.random(int((k == 5).sum()))
    mem = np.floor(rng.normal(2e8, 2e7, n))
    j = rng.integers(0, 10, n)
    mem[j == 0] = rng.integers(0, 3, int((j == 0).sum())) * 1e6 + rng.integers(-1, 2, int((j == 0).sum()))
    mem[j == 1] = 9999999.0
    mem[j == 2] = 10000000.0
    mem[j == 3] = 0.0
    mem[j == 4] = np.exp(rng.uniform(0, 60, int((j == 4).sum())))
    mem[j == 5] = rng.integers(1, 10**6, int((j == 5).sum())) * 19047619.0 / 1e3
    cf = np.zeros(n, np.uint32)
    mf = np.zeros(n, np.uint32)
    cf[rng.random(n) < 0.02] = 4  # empty
    mf[rng.random(n) < 0.02] = 4
    cnt = np.full(n, 10080, np.int64)
    return RawResults(cpu, cnt, cf, mem, cnt.copy(), mf)


def _same(a, b):
    return (a is None and b is None) or (a.is_nan() and b.is_nan()) or (a == b and a.as_tuple() == b.as_tuple())


@pytest.mark.parametrize("path", ["cli", "default", "cli7"])
@pytest.mark.parametrize("threads", [1, 0])
def test_matches_python_restatement(path, threads):
    st = _settings(path)
    raw = _raw(hash(path) & 0xFFFF)
    want = [format_result(r) for r in SimpleStrategy(st).results_from_raw(raw)]
    got = format_simple_batch(raw, st, threads=threads)
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        for rt in ResourceType:
            assert _same(g[rt].request, w[rt].request), (i, rt, g[rt].request, w[rt].request, raw.cpu_value[i])
            assert _same(g[rt].limit, w[rt].limit), (i, rt)
            assert str(g[rt].request) == str(w[rt].request)


def test_strings_cover_most_objects():
    raw = _raw(3)
    cs, ms, st = round_strings(raw.cpu_value, raw.cpu_flags, raw.mem_value, raw.mem_flags, Decimal("1.05"))
    assert (st == 0).mean() > 0.95
    assert cs[np.nonzero(raw.cpu_flags == 4)[0][0]] == b"NaN"


def test_fallbacks_raise_like_the_reference():
    st = _settings("cli")
    raw = RawResults(np.array([np.inf, 0.1, 0.2]), np.array([5, 5, 3]), np.array([0, 0, 1], np.uint32),
                     np.array([1e8, np.nan, 5.0]), np.array([5, 5, 3]), np.array([0, 1, 0], np.uint32))
    with pytest.raises(OverflowError):  # math.ceil(Decimal('Infinity')) in Runner._round_value
        format_simple_batch(raw, st)
    raw2 = RawResults(raw.cpu_value[1:], raw.cpu_count[1:], raw.cpu_flags[1:], raw.mem_value[1:],
                      raw.mem_count[1:], raw.mem_flags[1:])
    with pytest.raises(decimal.InvalidOperation):  # max() over a NaN Decimal (simple.py:29)
        format_simple_batch(raw2, st)


def test_huge_values_fall_back_exactly():
    st = _settings("cli")
    raw = RawResults(np.array([1e30, 1.7976931348623157e308]), np.array([1, 1]), np.zeros(2, np.uint32),
                     np.array([1e40, 2.5e27]), np.array([1, 1]), np.zeros(2, np.uint32))
    want = [format_result(r) for r in SimpleStrategy(st).results_from_raw(raw)]
    got = format_simple_batch(raw, st)
    for g, w in zip(got, want):
        for rt in ResourceType:
            assert _same(g[rt].request, w[rt].request)


@pytest.mark.parametrize("path", ["cli", "default", "cli7"])
def test_allocations_batch_equals_validated_models(path):
    """allocations_batch (bulk, no per-object validation walk) == the reference's list
    [ResourceAllocations(requests=..., limits=...)] (runner.py:113-120) built through the
    model's validator from the rounded RunResults: same values, same exponents, same JSON."""
    from krr_amd.core.fast_round import allocations_batch
    from krr_amd.core.runner import to_allocations

    st = _settings(path)
    raw = _raw(7 + len(path), n=5000)
    want = [to_allocations(r) for r in format_simple_batch(raw, st)]
    got = allocations_batch(raw, st)
    assert len(got) == len(want)
    nq = 0
    for g, w in zip(got, want):
        assert type(g) is type(w) and g == w and g.json() == w.json()
        for part in ("requests", "limits"):
            gd, wd = getattr(g, part), getattr(w, part)
            assert list(gd) == list(wd)
            for k in gd:
                assert type(gd[k]) is type(wd[k]) and str(gd[k]) == str(wd[k])
                nq += gd[k] == "?"
    assert nq > 0  # empty series became "?"
    # construct() layout: every field set; assignment keeps it so, other names are refused
    got[0].requests = dict(got[0].requests)
    assert got[0].__fields_set__ == got[1].__fields_set__ == {"requests", "limits"}
    with pytest.raises(ValueError):
        got[0].scratch = 1


def test_allocations_batch_reference_model_types():
    """With the reference's classes passed in (krr_amd.integration does), the models and
    their dict keys are those classes' instances."""
    import enum

    import pydantic.v1 as pd

    from krr_amd.core.fast_round import allocations_batch

    class RT(str, enum.Enum):
        CPU = "cpu"
        Memory = "memory"

    class RA(pd.BaseModel):
        requests: dict
        limits: dict

    raw = _raw(11, n=50)
    got = allocations_batch(raw, _settings("cli"), model=RA, resource_type=RT)
    assert all(type(g) is RA and list(g.requests) == [RT.CPU, RT.Memory] for g in got)
    assert got[0].dict()["limits"][RT.CPU] is None
