"""Pin the CPU oracle AND the host-side exact-decimal logic to the reference.

tests/golden/simple_strategy.json holds the outputs of the reference itself
(imported in the build container by tests/golden/make_golden.py).  Here the
oracle computes the raw per-segment results, the product's host code turns them
into RunResults exactly as it does for GPU results (SimpleStrategySettings
.cpu_from_raw / .memory_from_raw, krr_amd.core.rounding.format_result), and
every string is compared with the reference's.  No GPU needed.
"""
import decimal
import json
import math
import os
from decimal import Decimal

import numpy as np
import pytest

from krr_amd.core.abstract.strategies import ResourceType
from krr_amd.core.engine import RawResults, percentile_params
from krr_amd.core.rounding import format_result
from krr_amd.strategies.simple import PercentileMode, SimpleStrategy, SimpleStrategySettings
from krr_amd.utils.prom_decimal import prom_decimal
from oracle import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "simple_strategy.json")

with open(GOLDEN) as fh:
    DOC = json.load(fh)

PATHS = {
    "cli_99_5": dict(cpu_percentile="99", memory_buffer_percentage="5"),
    "cli_50_0.5": dict(cpu_percentile="50", memory_buffer_percentage="0.5"),
    "cli_99.9_100": dict(cpu_percentile="99.9", memory_buffer_percentage="100"),
    "cli_0.1_5": dict(cpu_percentile="0.1", memory_buffer_percentage="5"),
    "cli_100_5_min": dict(cpu_percentile="100", memory_buffer_percentage="5"),
    "default_int": None,
}
MINS = {"cli_100_5_min": (50, 300)}


def _settings(path, mode):
    kw = PATHS[path]
    s = SimpleStrategySettings() if kw is None else SimpleStrategySettings(**kw)
    return s.copy(update={"percentile_mode": PercentileMode(mode)})


def _segment(pods):
    vals = [float(Decimal(x)) for v in pods.values() for x in v]
    return np.array(vals, dtype=np.float64)


def _raw_from_oracle(case, settings, mode_code):
    cpu = _segment(case["cpu"])
    mem = _segment(case["mem"])
    co = np.array([0, cpu.size], dtype=np.int64)
    mo = np.array([0, mem.size], dtype=np.int64)
    pr = percentile_params(settings.cpu_percentile, settings.percentile_mode.value)
    assert pr.mode == mode_code
    cv, cn, cf = oracle.percentile(cpu, co, pr.mode, pr.p_num, pr.p_den, pr.q)
    mv, mn, mf = oracle.seg_max(mem, mo)
    return RawResults(cv, cn, cf, mv, mn, mf)


def _dstr(x):
    return None if x is None else str(x)


CASES = [(c["name"], p) for c in DOC["cases"] for p in DOC["settings_paths"]]
BY_NAME = {c["name"]: c for c in DOC["cases"]}


@pytest.mark.parametrize("name,path", CASES)
def test_ref_index_matches_reference(name, path):
    case = BY_NAME[name]
    want = case["results"][path]
    st = _settings(path, "ref_index")
    raw = _raw_from_oracle(case, st, 0)
    strat = SimpleStrategy(st)
    if "error" in want:
        with pytest.raises(getattr(decimal, want["error"], None) or Exception) as ei:
            strat.results_from_raw(raw)
        assert type(ei.value).__name__ == want["error"]
        return
    res = strat.results_from_raw(raw)[0]
    got_raw = {
        "cpu_request": _dstr(res[ResourceType.CPU].request),
        "cpu_limit": _dstr(res[ResourceType.CPU].limit),
        "mem_request": _dstr(res[ResourceType.Memory].request),
        "mem_limit": _dstr(res[ResourceType.Memory].limit),
    }
    assert got_raw == want["raw"]
    cmin, mmin = MINS.get(path, (5, 10))
    if "rounded_error" in want:
        with pytest.raises(Exception) as ei:
            format_result(res, cmin, mmin)
        assert type(ei.value).__name__ == want["rounded_error"]
        return
    rr = format_result(res, cmin, mmin)
    got_rounded = {
        "cpu_request": _dstr(rr[ResourceType.CPU].request),
        "cpu_limit": _dstr(rr[ResourceType.CPU].limit),
        "mem_request": _dstr(rr[ResourceType.Memory].request),
        "mem_limit": _dstr(rr[ResourceType.Memory].limit),
    }
    assert got_rounded == want["rounded"]


@pytest.mark.parametrize("name,path", CASES)
def test_sorted_lower_matches_reference_rule(name, path):
    case = BY_NAME[name]
    want = case["results"][path]
    st = _settings(path, "sorted_lower")
    raw = _raw_from_oracle(case, st, 1)
    if "sorted_error" in want:
        with pytest.raises(decimal.InvalidOperation):
            st.cpu_from_raw(raw, 0)
        return
    got = st.cpu_from_raw(raw, 0)
    assert str(got) == want["sorted"]
    if not got.is_nan():
        assert np.float64(raw.cpu_value[0]).view(np.uint64) == np.float64(float(Decimal(want["sorted"]))).view(np.uint64) \
            or float(got) == 0.0  # the Decimal already pins the sign of a zero


@pytest.mark.parametrize("name,path", CASES)
def test_linear_matches_numpy(name, path):
    case = BY_NAME[name]
    want = case["results"][path]
    if "linear_hex" not in want:
        pytest.skip("empty CPU segment")
    st = _settings(path, "linear")
    raw = _raw_from_oracle(case, st, 2)
    got = float(raw.cpu_value[0])
    if want["linear_hex"] == "nan":
        assert math.isnan(got)
    else:
        exp = float.fromhex(want["linear_hex"])
        assert got == exp and (got != 0.0 or True)
        if got != 0.0:
            assert got.hex() == exp.hex()


@pytest.mark.parametrize("row", DOC["index_table"], ids=lambda r: f"p{r['p']}-n{r['n']}")
def test_index_rule(row):
    p = 99 if row["p"] == "int99" else Decimal(row["p"])
    pr = percentile_params(p, "ref_index")
    assert oracle.exact_rank(row["n"], pr.p_num, pr.p_den) == row["k"]


def test_prom_decimal_roundtrip_of_fixture_strings():
    seen = 0
    for case in DOC["cases"]:
        for pods in (case["cpu"], case["mem"]):
            for vals in pods.values():
                for s in vals:
                    d = Decimal(s)
                    x = float(d)
                    if math.isnan(x):
                        assert prom_decimal(x).is_nan()
                        continue
                    # the reference's Decimal(s) is exactly what the host rebuilds from the f64
                    assert prom_decimal(x).as_tuple() == d.as_tuple(), s
                    seen += 1
    assert seen > 1000
