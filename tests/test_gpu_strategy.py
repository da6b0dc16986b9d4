"""End-to-end GPU parity: the plugin API (SimpleStrategy.run / run_batch, BatchedRunner)
on the MI355X path against the REFERENCE's own outputs (tests/golden), plus the fused
krr_simple_run / krr_simple_run_host / krr_pack_records entries against the oracle."""
import ctypes
import decimal
import json
import os
from decimal import Decimal

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

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
def test_simple_strategy_gpu_matches_reference(path):
    """Every golden case through SimpleStrategy on the GPU (one batched kernel pass per
    settings path, failing cases one by one), compared string-for-string."""
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.rounding import format_result
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    kw = PATHS[path]
    strat = SimpleStrategy(SimpleStrategySettings() if kw is None else SimpleStrategySettings(**kw))
    cmin, mmin = MINS.get(path, (5, 10))
    ok_cases = [c for c in DOC["cases"] if "error" not in c["results"][path]]
    results = strat.run_batch([_hist(c) for c in ok_cases], [_obj(c["name"]) for c in ok_cases])
    for case, res in zip(ok_cases, results):
        want = case["results"][path]
        got = {"cpu_request": _d(res[ResourceType.CPU].request), "cpu_limit": _d(res[ResourceType.CPU].limit),
               "mem_request": _d(res[ResourceType.Memory].request), "mem_limit": _d(res[ResourceType.Memory].limit)}
        assert got == want["raw"], case["name"]
        if "rounded" in want:
            rr = format_result(res, cmin, mmin)
            got_r = {"cpu_request": _d(rr[ResourceType.CPU].request), "cpu_limit": _d(rr[ResourceType.CPU].limit),
                     "mem_request": _d(rr[ResourceType.Memory].request),
                     "mem_limit": _d(rr[ResourceType.Memory].limit)}
            assert got_r == want["rounded"], case["name"]
    for case in DOC["cases"]:
        want = case["results"][path]
        if "error" in want:
            with pytest.raises(getattr(decimal, want["error"])):
                strat.run(_hist(case), _obj(case["name"]))


@pytest.mark.parametrize("mode", ["sorted_lower", "linear"])
def test_percentile_modes_gpu_match_reference_rules(mode):
    from krr_amd.strategies.simple import PercentileMode, SimpleStrategySettings

    st = SimpleStrategySettings(cpu_percentile="99", memory_buffer_percentage="5",
                                percentile_mode=PercentileMode(mode))
    for case in DOC["cases"]:
        want = case["results"]["cli_99_5"]
        h = _hist(case)
        from krr_amd.core.models.allocations import ResourceType

        if mode == "sorted_lower":
            if "sorted_error" in want:
                with pytest.raises(decimal.InvalidOperation):
                    st.calculate_cpu_proposal(h[ResourceType.CPU])
                continue
            assert str(st.calculate_cpu_proposal(h[ResourceType.CPU])) == want["sorted"], case["name"]
        elif "linear_hex" in want:
            raw = st.run_fleet(__import__("krr_amd.core.packing", fromlist=["x"]).pack_histories([h]))
            got = float(raw.cpu_value[0])
            if want["linear_hex"] == "nan":
                assert np.isnan(got), case["name"]
            else:
                assert got == float.fromhex(want["linear_hex"]), case["name"]


def test_batched_runner_end_to_end():
    from krr_amd.core.models.config import Config
    from krr_amd.core.runner import BatchedRunner

    cfg = Config(other_args={"cpu_percentile": "99", "memory_buffer_percentage": "5"})
    runner = BatchedRunner.from_config(cfg)
    cases = [c for c in DOC["cases"] if "rounded" in c["results"]["cli_99_5"]]
    allocs = runner.allocations([_obj(c["name"]) for c in cases], [_hist(c) for c in cases])
    from krr_amd.core.models.allocations import ResourceType

    for c, a in zip(cases, allocs):
        want = c["results"]["cli_99_5"]["rounded"]
        cpu = a.requests[ResourceType.CPU]
        assert (cpu == "?" and want["cpu_request"] == "NaN") or str(cpu) == want["cpu_request"], c["name"]


@pytest.mark.parametrize("path", list(PATHS))
def test_batched_runner_recommend_and_bodies_match_reference(path):
    """BatchedRunner.recommend (native rounding) and recommend_from_bodies (native JSON
    packer + kernel + native rounding) against the reference's rounded outputs."""
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.runner import BatchedRunner
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings
    from krr_amd.utils.prom_decimal import prom_format

    kw = PATHS[path]
    strat = SimpleStrategy(SimpleStrategySettings() if kw is None else SimpleStrategySettings(**kw))
    cmin, mmin = MINS.get(path, (5, 10))
    runner = BatchedRunner(strat, cmin, mmin)
    cases = [c for c in DOC["cases"] if "rounded" in c["results"][path]]
    got = runner.recommend([_obj(c["name"]) for c in cases], [_hist(c) for c in cases])

    def body(vals):
        res = [] if not vals else [{"metric": {"pod": "p"}, "values": [[1.7e9 + i, v] for i, v in enumerate(vals)]}]
        return json.dumps({"status": "success", "data": {"resultType": "matrix", "result": res}}).encode()

    # Prometheus can only send shortest-repr strings: cases whose samples are not are skipped
    repr_ok = [all(prom_format(float(v)) == v for r in ("cpu", "mem") for vs in c[r].values() for v in vs)
               for c in cases]
    bc = [c for c, ok in zip(cases, repr_ok) if ok]
    got_b = runner.recommend_from_bodies([[body(v) for v in c["cpu"].values()] for c in bc],
                                         [[body(v) for v in c["mem"].values()] for c in bc])
    for c, r in zip(cases, got):
        want = c["results"][path]["rounded"]
        assert {"cpu_request": _d(r[ResourceType.CPU].request), "cpu_limit": _d(r[ResourceType.CPU].limit),
                "mem_request": _d(r[ResourceType.Memory].request),
                "mem_limit": _d(r[ResourceType.Memory].limit)} == want, c["name"]
    assert len(bc) > len(cases) // 2
    for c, r in zip(bc, got_b):
        want = c["results"][path]["rounded"]
        assert _d(r[ResourceType.CPU].request) == want["cpu_request"], c["name"]
        assert _d(r[ResourceType.Memory].request) == want["mem_request"], c["name"]

    # fleet-batched queries: one grouped body per (namespace, container), routed by pod label
    from krr_amd.core.fleet_query import FleetQueryPlan

    def grouped(per_pod):
        res = [{"metric": {"pod": pod}, "values": [[1.7e9 + i, v] for i, v in enumerate(vals)]}
               for pod, vals in reversed(list(per_pod.items())) if vals]
        return json.dumps({"status": "success", "data": {"resultType": "matrix", "result": res}}).encode()

    class _O:
        def __init__(self, c):
            self.namespace, self.container = "default", c["name"]
            self.pods = list(dict.fromkeys(list(c["cpu"]) + list(c["mem"])))

    plan = FleetQueryPlan([_O(c) for c in bc])
    by_name = {c["name"]: c for c in bc}
    assert len(by_name) == len(bc)
    got_g = runner.recommend_from_grouped(plan, [grouped(by_name[g.container]["cpu"]) for g in plan.groups],
                                          [grouped(by_name[g.container]["mem"]) for g in plan.groups])
    for rb, rg in zip(got_b, got_g):
        for rt in ResourceType:
            assert _d(rb[rt].request) == _d(rg[rt].request) and _d(rb[rt].limit) == _d(rg[rt].limit)


def _fleet(seed, gaps):
    rng = np.random.default_rng(seed)
    S = 300
    if gaps:
        L = 4 * 2016
        offs = (np.arange(S + 1) * L).astype(np.int64)
    else:
        offs = np.concatenate([[0], np.cumsum(rng.integers(0, 5000, size=S))]).astype(np.int64)
    N = int(offs[-1])
    cpu = rng.gamma(2.0, 0.05, N)
    mem = np.floor(rng.normal(2e8, 2e7, N))
    if gaps:
        cpu[rng.random(N) < 0.1] = np.nan
        mem[rng.random(N) < 0.1] = np.nan
    return offs, cpu, mem


@pytest.mark.parametrize("gaps", [False, True])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_fused_simple_run_and_records(mode, gaps):
    import torch

    from krr_amd import _native
    from krr_amd.core.distributed import unpack_records

    offs, cpu, mem = _fleet(10 + mode, gaps)
    S = offs.size - 1
    dev = torch.device("cuda:0")
    ctx = _native.Context(0)
    d_cpu, d_mem, d_offs = (torch.from_numpy(a).to(dev) for a in (cpu, mem, offs))
    cs = ctx.series(d_cpu, d_offs, 0, gaps)
    ms = ctx.series(d_mem, d_offs, 0, gaps)
    out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
           (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
            ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
    params = _native.KrrPercentileParams(mode, 0, 99, 1, 0.99)
    ctx.simple_run(cs, ms, params, out)
    rec = torch.empty((S, 4), dtype=torch.int64, device=dev)
    ctx.pack_records(out, rec)
    torch.cuda.synchronize()
    u = unpack_records(rec)
    ov, on, of = oracle.percentile(cpu, offs, mode, 99, 1, 0.99, gaps)
    mv, mn, mf = oracle.seg_max(mem, offs, gaps)
    gv = u["cpu_value"]
    same = (gv.view(np.uint64) == ov.view(np.uint64)) | (np.isnan(gv) & np.isnan(ov))
    if mode == 2:
        same |= (gv == 0) & (ov == 0)
    assert same.all()
    assert np.array_equal(u["cpu_count"], on) and np.array_equal(u["cpu_flags"], of)
    assert np.array_equal(u["mem_value"], mv, equal_nan=True) and np.array_equal(u["mem_count"], mn)
    assert np.array_equal(u["mem_flags"], mf)
    # the same launch writing the records itself (krr_simple_run_records) == k_pack_records
    rec2 = torch.full((S, 4), -7, dtype=torch.int64, device=dev)
    ctx.simple_run(cs, ms, params, out, records=rec2)
    torch.cuda.synchronize()
    assert torch.equal(rec2, rec)
    ctx.close()


def test_simple_run_host_entry():
    from krr_amd import _native

    offs, cpu, mem = _fleet(3, False)
    S = offs.size - 1
    lib = _native.load_library()
    ctx = _native.Context(0)
    outs = [np.empty(S, t) for t in (np.float64, np.int64, np.uint32, np.float64, np.int64, np.uint32)]
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    params = _native.KrrPercentileParams(2, 0, 99, 1, 0.99)
    rc = lib.krr_simple_run_host(ctx._h, p(cpu), p(offs), p(mem), p(offs), S, 0, ctypes.byref(params),
                                 *map(p, outs))
    assert rc == 0, lib.krr_last_error(ctx._h)
    ov, on, _ = oracle.percentile(cpu, offs, 2, 99, 1, 0.99)
    mv, mn, _ = oracle.seg_max(mem, offs)
    assert np.array_equal(outs[0], ov, equal_nan=True) and np.array_equal(outs[1], on)
    assert np.array_equal(outs[3], mv, equal_nan=True) and np.array_equal(outs[4], mn)
    ctx.close()


def test_batched_runner_collect_result_matches_per_object_scans():
    """BatchedRunner.collect_result (kernel + native rounding + vectorised scans) equals
    the reference's per-object ResourceScan.calculate over the same allocations."""
    from krr_amd.core.models.result import Result, ResourceScan
    from krr_amd.core.runner import BatchedRunner
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    runner = BatchedRunner(SimpleStrategy(SimpleStrategySettings()), 5, 10)
    cases = [c for c in DOC["cases"] if "rounded" in c["results"]["default_int"]]
    from krr_amd.api.models import K8sObjectData, ResourceAllocations
    quantities = [("100m", "128Mi"), ("1", "1Gi"), (None, "64Mi"), ("5m", None), ("250m", "10M")]
    objs = [K8sObjectData(cluster=None, name=c["name"], container="c", pods=["p"], namespace="ns", kind="Deployment",
                          allocations=ResourceAllocations(requests=dict(zip(["cpu", "memory"], quantities[i % 5])),
                                                          limits=dict(zip(["cpu", "memory"], quantities[(i + 2) % 5]))))
            for i, c in enumerate(cases)]
    hists = [_hist(c) for c in cases]
    result = runner.collect_result(objs, hists)
    allocs = runner.allocations(objs, hists)
    want = Result(scans=[ResourceScan.calculate(o, a) for o, a in zip(objs, allocs)])
    assert result.scans == want.scans and result.score == want.score


def test_concurrent_run_from_threads_matches_sequential():
    """The reference calls strategy.run from executor threads (runner.py:104-106): the
    ABI is reentrant per thread-local krr_ctx, so concurrent runs give the sequential
    results bit for bit."""
    from concurrent.futures import ThreadPoolExecutor

    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    strat = SimpleStrategy(SimpleStrategySettings(cpu_percentile="99", memory_buffer_percentage="5"))
    cases = [c for c in DOC["cases"] if "error" not in c["results"]["cli_99_5"]][:40]
    args = [(_hist(c), _obj(c["name"])) for c in cases]
    seq = [strat.run(h, o) for h, o in args]
    with ThreadPoolExecutor(max_workers=8) as ex:
        par = list(ex.map(lambda a: strat.run(*a), args * 3))
    for i, r in enumerate(par):
        s = seq[i % len(seq)]
        for rt in ResourceType:
            assert _d(r[rt].request) == _d(s[rt].request) and _d(r[rt].limit) == _d(s[rt].limit)


def test_concurrent_run_calls_share_launches_on_gpu():
    """The reference Runner's per-object calls (runner.py:104-106: strategy.run in executor
    threads) on the GPU: 16 threads calling SimpleStrategy.run() at once get the reference's
    own strings (or its exception) per object, from fewer launches than calls."""
    from concurrent.futures import ThreadPoolExecutor

    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    strat = SimpleStrategy(SimpleStrategySettings(**PATHS["cli_99_5"]))
    cases = DOC["cases"] * 4

    def one(case):
        try:
            return strat.run(_hist(case), _obj(case["name"]))
        except decimal.DecimalException as e:
            return e

    with ThreadPoolExecutor(16) as ex:
        results = list(ex.map(one, cases))
    for case, res in zip(cases, results):
        want = case["results"]["cli_99_5"]
        if "error" in want:
            assert isinstance(res, getattr(decimal, want["error"])), case["name"]
            continue
        got = {"cpu_request": _d(res[ResourceType.CPU].request), "cpu_limit": _d(res[ResourceType.CPU].limit),
               "mem_request": _d(res[ResourceType.Memory].request), "mem_limit": _d(res[ResourceType.Memory].limit)}
        assert got == want["raw"], case["name"]
    co = strat.coalescer()
    assert co.calls == len(cases) and co.launches < len(cases)


def test_engine_chunks_large_fleets(monkeypatch):
    """SimpleEngine runs a fleet of more than two chunks as chunks (uploads and launches of
    their own, records rows per chunk): with a 256-KiB chunk the golden cases come back
    identical to the one-launch run, through run_batch (host records) and the device-records
    path of the multi-GPU shard."""
    from krr_amd.core.distributed import unpack_records
    from krr_amd.core.engine import SimpleEngine
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    strat = SimpleStrategy(SimpleStrategySettings(**PATHS["cli_99_5"]))
    ok_cases = [c for c in DOC["cases"] if "error" not in c["results"]["cli_99_5"]] * 40
    fleet = strat.pack([_hist(c) for c in ok_cases])
    one = strat.settings.run_fleet(fleet)
    rec_one = strat.settings.run_fleet_records(fleet).cpu().numpy()
    assert 8 * (fleet.cpu.offsets[-1] + fleet.mem.offsets[-1]) > 6 * (256 << 10)
    monkeypatch.setattr(SimpleEngine, "chunk_bytes", 256 << 10)
    many = strat.settings.run_fleet(fleet)
    rec_many = strat.settings.run_fleet_records(fleet).cpu().numpy()
    for f in ("cpu_value", "mem_value"):
        assert np.array_equal(getattr(one, f).view(np.uint64), getattr(many, f).view(np.uint64)), f
    for f in ("cpu_count", "cpu_flags", "mem_count", "mem_flags"):
        assert np.array_equal(getattr(one, f), getattr(many, f)), f
    assert np.array_equal(rec_one, rec_many)
    u = unpack_records(rec_many)
    assert np.array_equal(u["cpu_value"].view(np.uint64), many.cpu_value.view(np.uint64))
