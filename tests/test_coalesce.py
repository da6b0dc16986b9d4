"""Per-object SimpleStrategy.run() calls coalesced into fleet launches (krr_amd.core.coalesce).

The reference Runner calls strategy.run() once per object from its executor threads
(robusta_krr/core/runner.py:104-106).  These CPU tests pin the coalescer's contract — every
caller gets its own object's row, overlapping calls share launches, a launch failure reaches
exactly that launch's callers, per-object exceptions stay per object — and, with the device
pass stood in for by the C oracle (test infrastructure), that concurrent run() calls return
the reference's own strings (tests/golden/simple_strategy.json) for every settings path."""
import decimal
import json
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from decimal import Decimal

import numpy as np
import pytest

from krr_amd.core.coalesce import RunCoalescer

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "simple_strategy.json")
with open(GOLDEN) as fh:
    DOC = json.load(fh)

PATHS = {
    "cli_99_5": dict(cpu_percentile="99", memory_buffer_percentage="5"),
    "cli_50_0.5": dict(cpu_percentile="50", memory_buffer_percentage="0.5"),
    "cli_99.9_100": dict(cpu_percentile="99.9", memory_buffer_percentage="100"),
    "cli_0.1_5": dict(cpu_percentile="0.1", memory_buffer_percentage="5"),
    "default_int": None,
}


class _SlowSquare:
    """run_raw stand-in: squares its inputs after a delay, remembers batch sizes."""

    def __init__(self, delay=0.02, fail_on=None):
        self.delay, self.fail_on, self.batches = delay, fail_on, []
        self.lock = threading.Lock()

    def __call__(self, hs):
        with self.lock:
            self.batches.append(len(hs))
        time.sleep(self.delay)
        if self.fail_on is not None and self.fail_on in hs:
            raise RuntimeError(f"launch with {self.fail_on} failed")
        return [h * h for h in hs]


def _submit_all(co, items, workers=32):
    def one(x):
        raw, i = co.submit(x)
        return raw[i]

    with ThreadPoolExecutor(workers) as ex:
        return list(ex.map(one, items))


def test_lone_call_launches_at_once():
    run = _SlowSquare(delay=0.0)
    co = RunCoalescer(run)
    raw, i = co.submit(7)
    assert raw[i] == 49 and run.batches == [1] and co.launches == 1 and co.calls == 1


def test_overlapping_calls_share_launches_and_get_their_own_rows():
    run = _SlowSquare(delay=0.03)
    co = RunCoalescer(run)
    items = list(range(200))
    assert _submit_all(co, items, workers=64) == [x * x for x in items]
    assert co.calls == 200 and sum(run.batches) == 200
    assert co.launches == len(run.batches) < 40  # a burst batches itself behind the launch in flight
    assert max(run.batches) > 10


def test_max_batch_is_respected():
    run = _SlowSquare(delay=0.02)
    co = RunCoalescer(run, max_batch=5)
    items = list(range(60))
    assert _submit_all(co, items, workers=30) == [x * x for x in items]
    assert max(run.batches) <= 5 and sum(run.batches) == 60
    with pytest.raises(ValueError):
        RunCoalescer(run, max_batch=0)


def test_a_failed_launch_reaches_its_callers_only():
    run = _SlowSquare(delay=0.02, fail_on=13)
    co = RunCoalescer(run)
    out = {}

    def one(x):
        try:
            raw, i = co.submit(x)
            out[x] = raw[i]
        except RuntimeError as e:
            out[x] = e

    with ThreadPoolExecutor(32) as ex:
        list(ex.map(one, range(100)))
    failed = {x for x, v in out.items() if isinstance(v, RuntimeError)}
    assert 13 in failed and len(out) == 100
    assert all(out[x] == x * x for x in out if x not in failed)
    # the failed callers are exactly one launch's batch
    assert len(failed) in run.batches
    # the coalescer keeps working after a failure
    assert co.submit(3)[0][co.submit(3)[1]] == 9


def _oracle_run_fleet(self, fleet):
    from krr_amd.core.engine import RawResults
    from oracle import oracle

    p = self.params()
    cv, cn, cf = oracle.percentile(fleet.cpu.values, fleet.cpu.offsets, p.mode, p.p_num, p.p_den, p.q,
                                   fleet.cpu.gaps_are_nan)
    mv, mn, mf = oracle.seg_max(fleet.mem.values, fleet.mem.offsets, fleet.mem.gaps_are_nan)
    time.sleep(0.01)  # a launch takes time: let calls overlap
    return RawResults(cv, cn, cf.astype(np.uint32), mv, mn, mf.astype(np.uint32))


def _hist(case):
    from krr_amd.core.models.allocations import ResourceType

    return {ResourceType.CPU: {k: [Decimal(s) for s in v] for k, v in case["cpu"].items() if v},
            ResourceType.Memory: {k: [Decimal(s) for s in v] for k, v in case["mem"].items() if v}}


def _obj(name):
    from krr_amd.api.models import K8sObjectData, ResourceAllocations

    return K8sObjectData(cluster=None, name=name, container="c", pods=["p"], namespace="ns", kind="Deployment",
                         allocations=ResourceAllocations(requests={}, limits={}))


def _d(x):
    return None if x is None else str(x)


@pytest.mark.parametrize("path", list(PATHS))
def test_concurrent_run_calls_match_reference(path, monkeypatch):
    """Every golden case through SimpleStrategy.run() from 16 threads at once (the device
    pass stood in for by the oracle): each call returns the reference's own raw strings, or
    raises the reference's exception, and the calls share launches."""
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    monkeypatch.setattr(SimpleStrategySettings, "run_fleet", _oracle_run_fleet)
    kw = PATHS[path]
    strat = SimpleStrategy(SimpleStrategySettings() if kw is None else SimpleStrategySettings(**kw))
    cases = DOC["cases"] * 3

    def one(case):
        try:
            return strat.run(_hist(case), _obj(case["name"]))
        except decimal.DecimalException as e:
            return e

    with ThreadPoolExecutor(16) as ex:
        results = list(ex.map(one, cases))
    for case, res in zip(cases, results):
        want = case["results"][path]
        if "error" in want:
            assert isinstance(res, getattr(decimal, want["error"])), case["name"]
            continue
        got = {"cpu_request": _d(res[ResourceType.CPU].request), "cpu_limit": _d(res[ResourceType.CPU].limit),
               "mem_request": _d(res[ResourceType.Memory].request), "mem_limit": _d(res[ResourceType.Memory].limit)}
        assert got == want["raw"], case["name"]
    co = strat.coalescer()
    assert co.calls == len(cases) and co.launches < len(cases)
