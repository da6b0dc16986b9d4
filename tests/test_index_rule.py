"""The reference's CPU index rule for every cpu_percentile it accepts.

simple.py:36 evaluates int((n-1) * p / 100) in Decimal (28 digits): for p with many digits the
product rounds before the floor (p = 99.99999999999999999999999999 gives k(3) = 2).  Pinned by
tests/golden/simple_strategy_pct.json (make_golden.py pct, the reference imported) on the CLI
and direct-construction settings paths.  Kernels are stood in for by the oracle here
(tests/_standin.py, k_table honoured); tests/test_gpu_pct.py runs the same cases on the MI355X."""
import decimal
import functools
import json
import os
import sys
from decimal import Decimal
from fractions import Fraction

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from pct_inputs import PERCENTILES, RUN_NS, cpu_values, mem_values, pods_of  # noqa: E402
from _standin import oracle_run_packed  # noqa: E402

with open(os.path.join(HERE, "golden", "simple_strategy_pct.json")) as fh:
    DOC = json.load(fh)

PATHS = ("cli", "direct_decimal", "direct_float")


def settings(path, p, mode=None):
    from krr_amd.strategies.simple import PercentileMode, SimpleStrategySettings

    kw = {}
    if mode:
        kw["percentile_mode"] = PercentileMode(mode)
    if path == "cli":  # what typer hands pydantic: strings (main.py:29-36, 110)
        return SimpleStrategySettings(cpu_percentile=p, memory_buffer_percentage="5", **kw)
    return SimpleStrategySettings(cpu_percentile=Decimal(p) if path == "direct_decimal" else float(p), **kw)


def strategy(path, p, mode=None):
    from krr_amd.strategies.simple import SimpleStrategy

    return SimpleStrategy(settings(path, p, mode))


@functools.lru_cache(maxsize=None)
def history(n):
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.utils.prom_decimal import prom_format

    cs = [Decimal(prom_format(float(x))) for x in cpu_values(n)]
    ms = [Decimal(prom_format(float(x))) for x in mem_values(n)]
    cpu, mem, o = {}, {}, 0
    for i, ln in enumerate(pods_of(n)):
        cpu[f"pod{i}"], mem[f"pod{i}"] = cs[o:o + ln], ms[o:o + ln]
        o += ln
    return {ResourceType.CPU: cpu, ResourceType.Memory: mem}


def runs_for(path, max_n):
    return [r for r in DOC["runs"] if r["path"] == path and r["n"] <= max_n]


@pytest.fixture
def standin(monkeypatch):
    from krr_amd.core.engine import SimpleEngine

    monkeypatch.setattr(SimpleEngine, "run_packed", oracle_run_packed)
    monkeypatch.setattr(SimpleEngine, "context", lambda self: None)


def test_settings_objects_match_reference():
    """Our settings hold the same object the reference's pydantic built (type and digits)."""
    for row in DOC["index"]:
        st = settings(row["path"], row["p"])
        assert type(st.cpu_percentile).__name__ == row["setting_type"]
        assert str(st.cpu_percentile) == row["setting"], row


@pytest.mark.parametrize("path", PATHS)
def test_index_rule_equals_reference(path):
    for row in DOC["index"]:
        if row["path"] != path:
            continue
        rule = settings(path, row["p"]).params().rule
        ns = np.array(row["n"], dtype=np.int64)
        assert [rule.k(int(n)) for n in ns] == row["k"], row["p"]
        small = ns <= 200_000  # the table's build at 1 M entries is the GPU tests' (test_gpu_pct.py)
        want = np.array(row["k"])[small].tolist()
        assert rule.ks(ns[small]).tolist() == want, row["p"]
        assert rule.table(int(ns[small].max()))[ns[small]].tolist() == want, row["p"]


def test_default_int_rule_is_the_exact_floor():
    from krr_amd.strategies.simple import SimpleStrategySettings

    st = SimpleStrategySettings()
    assert type(st.cpu_percentile) is int
    rule = st.params().rule
    assert not rule.needs_table(10**9)
    ns = np.arange(1, 200_000, 997)
    assert rule.ks(ns).tolist() == [int((int(n) - 1) * 99 / 100) for n in ns]


@pytest.mark.parametrize("p", ["99.99999999999999999999999999", "33.33333333333333333333333333",
                               "0.0000000000000000000000000001", "12.3456789012345678", "1E-20",
                               "66.66666666666666666666666667", "99.9999999999999999"])
def test_table_equals_literal_expression(p):
    """The table's float-filtered build equals the reference's expression at every n."""
    from krr_amd.core.index_rule import IndexRule

    rule = IndexRule(Decimal(p))
    tab = rule.table(30_000)
    with decimal.localcontext(decimal.Context(prec=28)):
        want = [int((n - 1) * Decimal(p) / 100) for n in range(1, 30_001)]
    assert tab[1:].tolist() == want


def test_exact_floor_region_is_exact():
    """Where IndexRule claims the exact floor (exact_upto), the literal expression agrees."""
    from krr_amd.core.index_rule import IndexRule

    rng = np.random.default_rng(3)
    for _ in range(300):
        digits = int(rng.integers(1, 19))
        c = int(rng.integers(1, 10**digits))
        p = Decimal(c).scaleb(-int(rng.integers(0, digits + 1)))
        if not (0 < p <= 100):
            continue
        rule = IndexRule(p)
        top = min(rule.exact_upto, 10**15)
        for n in (2, 3, int(top), int(top) - 1, int(rng.integers(2, max(3, int(top))))):
            if n < 1:
                continue
            f = Fraction(p)
            assert rule.literal(n) == (n - 1) * f.numerator // (100 * f.denominator), (p, n)


def test_params_approximation_bounds():
    from krr_amd.strategies.simple import SimpleStrategySettings

    for p in PERCENTILES:
        prm = SimpleStrategySettings(cpu_percentile=p).params()
        assert 0 < prm.p_num <= 100 * prm.p_den and prm.p_den <= 10**15
        assert abs(Fraction(prm.p_num, prm.p_den) - Fraction(Decimal(p))) <= Fraction(1, 10**15)


@pytest.mark.parametrize("path", PATHS)
def test_pct_runs_match_reference(standin, path):
    """run_batch / run / format_result for every fixture run up to 172,800 samples (oracle stand-in)."""
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.rounding import format_result

    for r in runs_for(path, 172800):
        strat = strategy(path, r["p"])
        h = history(r["n"])
        got = strat.run_batch([h])[0]
        assert str(got[ResourceType.CPU].request) == r["raw"]["cpu_request"], (r["p"], r["n"])
        assert str(got[ResourceType.Memory].request) == r["raw"]["mem_request"], (r["p"], r["n"])
        rr = format_result(got)
        assert str(rr[ResourceType.CPU].request) == r["rounded"]["cpu_request"]
        assert str(rr[ResourceType.Memory].request) == r["rounded"]["mem_request"]
        if r["n"] <= 10080:
            one = strat.run(h, None)
            assert str(one[ResourceType.CPU].request) == r["raw"]["cpu_request"]


def test_pct_sorted_and_linear_match_reference(standin):
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.packing import pack_histories

    for r in runs_for("cli", 10080):
        h = history(r["n"])
        st = settings("cli", r["p"], "sorted_lower")
        assert str(st.calculate_cpu_proposal(h[ResourceType.CPU])) == r["sorted"], (r["p"], r["n"])
        lin = settings("cli", r["p"], "linear")
        assert float(lin.run_fleet(pack_histories([h])).cpu_value[0]) == float.fromhex(r["linear_hex"])


def test_no_accepted_percentile_raises(standin):
    """Every p in (0, 100] the reference's settings accept runs (no 'more than 15 digits' error)."""
    from krr_amd.core.models.allocations import ResourceType

    h = history(1001)
    for p in ["1E-100", "0.1234567890123456789012345678901234567890", "99.999999999999999999999999999999999",
              "100.0000000000000000000000000000", "7.5E-10"]:
        got = strategy("cli", p).run_batch([h])[0]
        assert got[ResourceType.CPU].request.is_finite()
