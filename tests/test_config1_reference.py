"""BASELINE.json configs[0] (config 1) against the REFERENCE's own outputs.

`tests/golden/config1_reference.json` holds what yonahd/krr 1.0.0's `SimpleStrategy.run()`
and `Runner._format_result()` return for the 100 synthetic containers of config 1 (generated
by `tests/golden/make_config1_golden.py`, which imports the reference in the build
container).  The inputs are regenerated here from PCG64 seed 0 and checked by sha256.

CPU tests: the oracle (`oracle/krr_oracle.c`, REF_INDEX + max) and the product's host rounding
(Python restatement and native `krr_round_simple`) reproduce every string.
GPU tests: the HIP path through the plugin API (`SimpleStrategy.run_batch`) and through the
whole loader path (`BatchedRunner.recommend_from_bodies`: Prometheus JSON bodies -> native
packer -> fused kernel -> native rounding) reproduce every string, for the CLI settings path
and the int-default path.
"""
import decimal
import json
import os
import sys
from decimal import Decimal

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import config1  # noqa: E402

with open(os.path.join(HERE, "golden", "config1_reference.json")) as fh:
    DOC = json.load(fh)

PATHS = {"cli_99_5": dict(cpu_percentile="99", memory_buffer_percentage="5"), "default_int": None}


@pytest.fixture(scope="module")
def data():
    cpu, mem = config1.inputs()
    assert config1.sha256(cpu, mem) == DOC["input_sha256"], "config-1 generator drifted from the fixture"
    return cpu, mem


def _strategy(path):
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    kw = PATHS[path]
    return SimpleStrategy(SimpleStrategySettings() if kw is None else SimpleStrategySettings(**kw))


def _csr(x):
    flat = np.ascontiguousarray(x.reshape(-1))
    offs = np.arange(0, flat.size + 1, x.shape[1] * x.shape[2], dtype=np.int64)
    return flat, offs


def _d(x):
    return None if x is None else str(x)


def _row(res):
    from krr_amd.core.models.allocations import ResourceType

    return {"cpu_request": _d(res[ResourceType.CPU].request), "cpu_limit": _d(res[ResourceType.CPU].limit),
            "mem_request": _d(res[ResourceType.Memory].request), "mem_limit": _d(res[ResourceType.Memory].limit)}


@pytest.mark.parametrize("path", list(PATHS))
def test_oracle_and_host_rounding_match_reference(data, path):
    """CPU only: oracle REF_INDEX + max, then the product's exact-decimal host code."""
    from oracle import oracle

    from krr_amd import _native
    from krr_amd.core.abstract.strategies import ResourceRecommendation
    from krr_amd.core.fast_round import round_strings
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.rounding import format_result, reference_context
    from krr_amd.utils.prom_decimal import prom_decimal

    cpu, mem = data
    cv, co = _csr(cpu)
    mv, mo = _csr(mem)
    pv, pn, pf = oracle.percentile(cv, co, _native.KRR_PCT_REF_INDEX, 99, 1, 0.99)
    xv, xn, xf = oracle.seg_max(mv, mo)
    assert (pn == config1.PODS * config1.SAMPLES).all() and (xn == pn).all()
    strat = _strategy(path)
    buffer = strat.settings.memory_buffer()
    want = DOC["results"][path]
    for o in range(config1.OBJECTS):
        c = prom_decimal(float(pv[o]))
        with decimal.localcontext(reference_context()):
            m = prom_decimal(float(xv[o])) * buffer
        raw = {ResourceType.CPU: ResourceRecommendation(request=c, limit=None),
               ResourceType.Memory: ResourceRecommendation(request=m, limit=m)}
        assert _row(raw) == want[o]["raw"], o
        assert _row(format_result(raw)) == want[o]["rounded"], o
    cs, ms, st = round_strings(pv, pf, xv, xf, buffer)
    assert (st == 0).all()
    assert [s.decode() for s in cs] == [w["rounded"]["cpu_request"] for w in want]
    assert [s.decode() for s in ms] == [w["rounded"]["mem_request"] for w in want]


def test_reference_index_rule_is_unsorted_position(data):
    """The fixture really is the reference's unsorted-position rule (simple.py:31-36), not a
    sorted percentile: the CPU answer is the sample at floor((n-1)*99/100) of the pod-ordered
    concatenation."""
    cpu, _ = data
    n = config1.PODS * config1.SAMPLES
    k = (n - 1) * 99 // 100
    for o in (0, 17, 99):
        x = cpu[o].reshape(-1)[k]
        assert Decimal(DOC["results"]["cli_99_5"][o]["raw"]["cpu_request"]) == Decimal(repr(float(x)))
        assert x != np.sort(cpu[o].reshape(-1))[k]


@pytest.mark.gpu
@pytest.mark.parametrize("path", list(PATHS))
def test_gpu_plugin_api_matches_reference(data, path):
    """SimpleStrategy.run_batch (HIP kernels) + format_result, string-for-string."""
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.rounding import format_result
    from krr_amd.utils.prom_decimal import prom_format

    cpu, mem = data
    hists = []
    for o in range(config1.OBJECTS):
        pods = config1.pod_names(o)
        hists.append({ResourceType.CPU: {pods[p]: [Decimal(prom_format(float(x))) for x in cpu[o, p]]
                                         for p in range(config1.PODS)},
                      ResourceType.Memory: {pods[p]: [Decimal(prom_format(float(x))) for x in mem[o, p]]
                                            for p in range(config1.PODS)}})
    got = _strategy(path).run_batch(hists)
    want = DOC["results"][path]
    for o, res in enumerate(got):
        assert _row(res) == want[o]["raw"], o
        assert _row(format_result(res)) == want[o]["rounded"], o


@pytest.mark.gpu
@pytest.mark.parametrize("path", list(PATHS))
def test_gpu_from_prometheus_bodies_matches_reference(data, path):
    """The loader path: one query_range JSON body per pod (as prometheus.py:118-143 fetches
    them) -> native packer -> fused kernel -> native rounding."""
    from krr_amd.core.runner import BatchedRunner
    from krr_amd.utils.prom_decimal import prom_format

    cpu, mem = data
    t0 = 1.7e9

    def body(pod, xs):
        vals = [[t0 + 60 * i, prom_format(float(x))] for i, x in enumerate(xs)]
        return json.dumps({"status": "success", "data": {"resultType": "matrix", "result": [
            {"metric": {"pod": pod}, "values": vals}]}}).encode()

    cb = [[body(p, cpu[o, i]) for i, p in enumerate(config1.pod_names(o))] for o in range(config1.OBJECTS)]
    mb = [[body(p, mem[o, i]) for i, p in enumerate(config1.pod_names(o))] for o in range(config1.OBJECTS)]
    got = BatchedRunner(_strategy(path)).recommend_from_bodies(cb, mb)
    want = DOC["results"][path]
    for o, res in enumerate(got):
        assert _row(res) == want[o]["rounded"], o
