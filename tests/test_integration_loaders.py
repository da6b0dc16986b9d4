"""krr_amd.integration's body-level loaders without the reference (runs anywhere, CPU only).

A stand-in runner exposes what the loaders use of the reference's Runner:
``_get_prometheus_loader(cluster).prometheus`` with ``_session``, ``url``, ``headers`` and
``ssl_verification`` (prometheus.py:41-53, 88).  Objects of two clusters are interleaved, so
``fetch_grouped_fleet`` must pack each cluster's grouped bodies and put the segments back in
fleet order: the result must equal, value for value, the per-pod bodies packed directly."""
import asyncio
import datetime
import json
import re
from types import SimpleNamespace

import numpy as np
import pytest

from krr_amd import integration
from krr_amd.core.prom_native import pack_query_range_bodies
from krr_amd.strategies.simple import SimpleStrategySettings
from krr_amd.utils.prom_decimal import prom_format


class Session:
    def __init__(self, series):
        self.series, self.calls = series, []

    def get(self, url, params=None, verify=None, headers=None):
        q = params["query"]
        self.calls.append(q)
        rt = "cpu" if "cpu_usage" in q else "memory"
        m = re.search(r'pod=~"([^"]*)"', q)
        if m:
            pods = m.group(1).split("|")
            res = [{"metric": {"pod": p}, "values": [[i, prom_format(v)] for i, v in enumerate(self.series[(rt, p)])]}
                   for p in pods if (rt, p) in self.series]
        else:
            p = re.search(r'pod="([^"]*)"', q).group(1)
            res = ([{"metric": {}, "values": [[i, prom_format(v)] for i, v in enumerate(self.series[(rt, p)])]}]
                   if (rt, p) in self.series else [])
        body = json.dumps({"status": "success", "data": {"resultType": "matrix", "result": res}}).encode()
        return SimpleNamespace(status_code=200 if "bad" not in q else 503, content=body)


def _fleet(seed=3):
    rng = np.random.default_rng(seed)
    objects, series = [], {}
    for o in range(23):
        pods = [f"c{o % 2}-o{o}-p{p}" for p in range(int(rng.integers(0, 4)))]
        for p in pods:
            if rng.random() < 0.85:
                n = int(rng.integers(1, 60))
                series[("cpu", p)] = rng.gamma(2.0, 0.05, n)
                series[("memory", p)] = np.floor(rng.normal(2e8, 2e7, n))
        objects.append(SimpleNamespace(cluster=f"k{o % 2}", namespace="ns" if o % 3 else "other",
                                       container="main", pods=pods, name=f"o{o}"))
    return objects, series


def _runner(session):
    prom = SimpleNamespace(_session=session, url="http://p", headers={}, ssl_verification=True)
    return SimpleNamespace(_get_prometheus_loader=lambda cluster: SimpleNamespace(prometheus=prom))


def test_grouped_loader_equals_per_pod_bodies_across_clusters():
    objects, series = _fleet()
    settings = SimpleStrategySettings()
    session = Session(series)
    cpu_b, mem_b = asyncio.run(integration.fetch_pod_bodies(_runner(session), objects, settings))
    n_pod_queries = len(session.calls)
    assert n_pod_queries == 2 * sum(len(o.pods) for o in objects)
    want_cpu, want_mem = pack_query_range_bodies(cpu_b), pack_query_range_bodies(mem_b)
    session.calls.clear()
    got = asyncio.run(integration.fetch_grouped_fleet(_runner(session), objects, settings))
    assert len(session.calls) < n_pod_queries
    for g, w in ((got.cpu, want_cpu), (got.mem, want_mem)):
        assert np.array_equal(g.offsets, w.offsets)
        assert np.array_equal(g.values.view(np.int64), w.values.view(np.int64))
        assert g.max_len == w.max_len


def test_query_window_matches_reference_parameters():
    s = SimpleStrategySettings()
    now = datetime.datetime(2026, 1, 2, 3, 4, 5, 600000)
    start, end, step = integration.query_window(s, now)
    assert step == "15m" and end - start == 336 * 3600 and end == round(now.timestamp())


def test_http_error_raises():
    q = integration.query_range_fn(_runner(Session({})).__dict__["_get_prometheus_loader"](None).prometheus,
                                   0, 1, "1m")
    with pytest.raises(integration.PrometheusHTTPError):
        q('sum(bad{pod="x"})')


def test_install_rejects_unknown_switches():
    class R:
        async def _gather_objects_recommendations(self, objects):
            return []

        async def _collect_result(self):
            return None

    with pytest.raises(ValueError):
        integration.install(R, loader="nope")
    integration.install(R, loader="bodies", scan="fleet")
    assert R._collect_result.__qualname__.startswith("install")
    integration.install(R, loader="bodies", scan="reference")
    assert R._collect_result.__qualname__.endswith("R._collect_result")
    integration.uninstall(R)
    assert R._gather_objects_recommendations.__qualname__.endswith("R._gather_objects_recommendations")


def test_reorder_of_tensor_series_equals_numpy():
    """_reorder on series held as torch tensors (the device packer's output lives in HBM;
    here CPU tensors) gives the numpy path's CSR."""
    import torch

    from krr_amd.core.packing import PackedSeries

    rng = np.random.default_rng(4)
    parts = []
    for k in range(3):
        lens = rng.integers(0, 7, size=int(rng.integers(1, 6)))
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        parts.append(PackedSeries(rng.random(int(offs[-1])), offs, int(lens.max(initial=0))))
    n = sum(p.n_segments for p in parts)
    order = list(rng.permutation(n))
    want = integration._reorder(parts, order)
    tparts = [PackedSeries(torch.from_numpy(p.values), torch.from_numpy(p.offsets), p.max_len) for p in parts]
    got = integration._reorder(tparts, order)
    assert np.array_equal(got.offsets.numpy(), want.offsets)
    assert np.array_equal(got.values.numpy(), want.values)
    assert got.max_len == want.max_len


@pytest.mark.parametrize("host_part", [0, 1, 2])
def test_reorder_mixed_host_and_device_parts(host_part):
    """One cluster's batch fell back to the host packer (numpy) while the others came from
    the device packer (tensors): _reorder normalises to the device side instead of failing
    on torch.cat of numpy arrays (advisor round 3)."""
    import torch

    from krr_amd.core.packing import PackedSeries

    rng = np.random.default_rng(10 + host_part)
    parts = []
    for k in range(3):
        lens = rng.integers(0, 7, size=int(rng.integers(1, 6)))
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        parts.append(PackedSeries(rng.random(int(offs[-1])), offs, int(lens.max(initial=0))))
    n = sum(p.n_segments for p in parts)
    order = list(rng.permutation(n))
    want = integration._reorder(parts, order)
    mixed = [p if k == host_part else PackedSeries(torch.from_numpy(p.values), torch.from_numpy(p.offsets), p.max_len)
             for k, p in enumerate(parts)]
    got = integration._reorder(mixed, order)
    assert isinstance(got.values, torch.Tensor)
    assert np.array_equal(got.offsets.numpy(), want.offsets)
    assert np.array_equal(got.values.numpy(), want.values)
