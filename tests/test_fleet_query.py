"""Fleet-level PromQL batching (krr_amd.core.fleet_query).

A small in-process stand-in for Prometheus evaluates both query forms over the
same raw series: the reference's per-pod ``sum(<metric>{..., pod="p", ...})``
(prometheus.py:118-143) and the grouped ``sum by (pod) (...{pod=~"a|b"})``.
Packing the grouped responses through ``krr_pack_parse_grouped`` must give the
same float64 bits, offsets and pod drops as packing the per-pod responses with
``pack_query_range_bodies`` — and both must equal the reference's json + Decimal
semantics (tests/test_prom_native.ref_pack).  The fake evaluator matches pod
regexes with Python's ``re.fullmatch`` after PromQL string unescaping, so the
escaping of pod names is checked too.  Host-only: no GPU.
"""
import datetime
import json
import random
import re

import numpy as np
import pytest

from krr_amd.core.fleet_query import FleetQueryPlan, group_query, pod_query, pod_regex, step_string
from krr_amd.core.models.allocations import ResourceType
from krr_amd.core.prom_native import PrometheusResponseError, pack_query_range_bodies, parse_series
from tests.test_prom_native import go_format, ref_pack


class Obj:
    def __init__(self, namespace, container, pods):
        self.namespace, self.container, self.pods = namespace, container, list(pods)


# ---- the reference's query strings (prometheus.py:123, :126, :137) -------------------------------

def test_pod_query_strings_match_reference():
    assert pod_query(ResourceType.CPU, "ns1", "web-1", "app") == (
        'sum(node_namespace_pod_container:container_cpu_usage_seconds_total:sum_irate'
        '{namespace="ns1", pod="web-1", container="app"})')
    assert pod_query(ResourceType.Memory, "ns1", "web-1", "app") == (
        'sum(container_memory_working_set_bytes{job="kubelet", metrics_path="/metrics/cadvisor", image!="", '
        'namespace="ns1", pod="web-1", container="app"})')
    assert step_string(datetime.timedelta(minutes=15)) == "15m"
    assert step_string(datetime.timedelta(seconds=90)) == "1m"
    with pytest.raises(ValueError):
        pod_query("gpu", "n", "p", "c")


def test_group_query_form():
    q = group_query(ResourceType.Memory, "ns", "app", ["a.b", "c-1"])
    assert q == ('sum by (pod) (container_memory_working_set_bytes{job="kubelet", metrics_path="/metrics/cadvisor", '
                 'image!="", namespace="ns", pod=~"a\\\\.b|c-1", container="app"})')


# ---- a fake Prometheus --------------------------------------------------------------------------

_SEL = re.compile(r'^(sum|sum by \(pod\)) ?\((?P<metric>[^{]+)\{(?P<m>.*)\}\)$')
_MATCHER = re.compile(r'(\w+)(=~|!=|=)"((?:[^"\\]|\\.)*)"')


def _unquote(s):
    return re.sub(r'\\(.)', r'\1', s)


class FakePrometheus:
    """Raw series: (labels dict, {timestamp: value}).  Evaluates the two query
    shapes on a fixed step grid, summing matching series in storage order."""

    def __init__(self, series, grid):
        self.series, self.grid = series, grid
        self.calls = 0

    def _select(self, query):
        m = _SEL.match(query)
        assert m, query
        by_pod = m.group(1) != "sum"
        matchers = _MATCHER.findall(m.group("m"))
        out = []
        for labels, samples in self.series:
            if labels["__name__"] != m.group("metric"):
                continue
            ok = True
            for name, op, val in matchers:
                v, have = labels.get(name, ""), _unquote(val)
                if op == "=":
                    ok &= v == have
                elif op == "!=":
                    ok &= v != have
                else:
                    ok &= re.fullmatch(have, v) is not None
            if ok:
                out.append((labels, samples))
        return by_pod, out

    def query_range(self, query):
        self.calls += 1
        by_pod, sel = self._select(query)
        groups = {}
        for labels, samples in sel:
            key = labels.get("pod", "") if by_pod else None
            acc = groups.setdefault(key, {})
            for t in self.grid:
                if t in samples:
                    acc[t] = acc.get(t, 0.0) + samples[t]
        result = []
        for key, acc in groups.items():
            if not acc:
                continue
            metric = {"pod": key} if by_pod else {}
            result.append({"metric": metric, "values": [[t, go_format(acc[t])] for t in self.grid if t in acc]})
        if by_pod:
            random.Random(len(query)).shuffle(result)  # routing must go by label, not position
        return json.dumps({"status": "success", "data": {"resultType": "matrix", "result": result}}).encode()


def make_fleet(seed=0, n_ns=3, n_obj=12):
    rng = np.random.default_rng(seed)
    grid = [1700000000 + 60 * k for k in range(40)]
    objects, series = [], []
    pod_chars = ["web", "db.replica", "x+y", "a(b)", "q?[1]", "tail$", "plain"]
    for o in range(n_obj):
        ns = f"ns{o % n_ns}"
        container = ["app", "sidecar"][o % 2]
        pods = [f"{pod_chars[(o + k) % len(pod_chars)]}-{o}-{k}" for k in range(int(rng.integers(0, 5)))]
        objects.append(Obj(ns, container, pods))
        for k, pod in enumerate(pods):
            if (o + k) % 5 == 3:
                continue  # a pod with no samples: dropped by both forms
            for restart in range(1 + (k % 2)):  # container restarts: several series summed per pod
                present = rng.random(len(grid)) > 0.2
                cpu = {t: float(rng.gamma(2.0, 0.05)) for t, p in zip(grid, present) if p}
                mem = {t: float(rng.integers(10 ** 6, 10 ** 9)) for t, p in zip(grid, present) if p}
                base = {"namespace": ns, "pod": pod, "container": container, "restart": str(restart)}
                series.append(({**base, "__name__": "node_namespace_pod_container:container_cpu_usage_seconds_total:"
                                "sum_irate"}, cpu))
                series.append(({**base, "__name__": "container_memory_working_set_bytes", "job": "kubelet",
                                "metrics_path": "/metrics/cadvisor", "image": "img"}, mem))
                # a same-pod series in another container and a pause container (image="") must not leak in
                series.append(({**base, "container": "other", "__name__": "container_memory_working_set_bytes",
                                "job": "kubelet", "metrics_path": "/metrics/cadvisor", "image": "img"}, mem))
                series.append(({**base, "__name__": "container_memory_working_set_bytes", "job": "kubelet",
                                "metrics_path": "/metrics/cadvisor", "image": ""}, mem))
    # a duplicated pod inside one object and a pod listed by two objects of one group
    first = next(o for o in objects if o.pods and o.namespace == "ns0" and o.container == "app")
    objects.append(Obj("ns0", "app", first.pods[:1] * 2 + ["ghost"]))
    objects.append(Obj("ns0", "app", []))
    return objects, FakePrometheus(series, grid)


def per_pod_bodies(objects, prom, resource):
    return [[prom.query_range(pod_query(resource, o.namespace, p, o.container)) for p in dict.fromkeys(o.pods)]
            for o in objects]


@pytest.mark.parametrize("max_chars", [6000, 40, 1])
@pytest.mark.parametrize("resource", list(ResourceType))
def test_grouped_pack_equals_per_pod_pack(resource, max_chars):
    objects, prom = make_fleet()
    plan = FleetQueryPlan(objects, max_query_chars=max_chars)
    grouped = [prom.query_range(q) for q in plan.queries(resource)]
    ref_bodies = per_pod_bodies(objects, prom, resource)
    got, got_ts, got_counts = plan.pack(grouped, want_timestamps=True, return_pod_counts=True)
    exp, exp_ts, exp_counts = pack_query_range_bodies(ref_bodies, want_timestamps=True, return_pod_counts=True)
    np.testing.assert_array_equal(got.offsets, exp.offsets)
    assert got.values.tobytes() == exp.values.tobytes()
    assert got_ts.tobytes() == exp_ts.tobytes()
    np.testing.assert_array_equal(got_counts, exp_counts)
    assert got.max_len == exp.max_len
    rv, ro, rc = ref_pack(ref_bodies)  # the reference's json + Decimal semantics
    assert got.values.tobytes() == rv.tobytes()
    np.testing.assert_array_equal(got.offsets, ro)
    np.testing.assert_array_equal(got_counts, rc)
    assert (got_counts == -1).any() and (got_counts > 0).any()


def test_plan_grouping():
    objects, prom = make_fleet()
    plan = FleetQueryPlan(objects)
    n_pairs = len({(o.namespace, o.container) for o in objects if o.pods})
    assert len(plan.groups) == n_pairs
    n_unique = len({(o.namespace, o.container, p) for o in objects for p in o.pods})
    assert sum(len(g.pods) for g in plan.groups) == n_unique
    assert plan.n_slots == sum(len(dict.fromkeys(o.pods)) for o in objects)
    assert np.all(np.diff(plan.slot_obj) >= 0)
    split = FleetQueryPlan(objects, max_query_chars=1)
    assert len(split.groups) == n_unique  # every pod alone once the budget is exceeded
    for g in FleetQueryPlan(objects, max_query_chars=60).groups:
        assert len(g.pods) == 1 or len(pod_regex(g.pods)) < 60 + len(g.pods)
    with pytest.raises(ValueError):
        FleetQueryPlan(objects, max_query_chars=0)


def test_fetch_and_pack_fleet():
    objects, prom = make_fleet(seed=3)
    plan = FleetQueryPlan(objects)
    bodies = plan.fetch(prom.query_range, max_workers=4)
    assert prom.calls == 2 * len(plan.groups)
    fleet = plan.pack_fleet(bodies[ResourceType.CPU], bodies[ResourceType.Memory])
    for rt, packed in ((ResourceType.CPU, fleet.cpu), (ResourceType.Memory, fleet.mem)):
        exp = pack_query_range_bodies(per_pod_bodies(objects, prom, rt))
        assert packed.values.tobytes() == exp.values.tobytes()
        np.testing.assert_array_equal(packed.offsets, exp.offsets)
    reference_calls = 2 * sum(len(dict.fromkeys(o.pods)) for o in objects)
    assert len(plan.groups) * 2 < reference_calls


def test_errors_and_edge_cases():
    objects, prom = make_fleet()
    plan = FleetQueryPlan(objects)
    bodies = [prom.query_range(q) for q in plan.queries(ResourceType.CPU)]
    with pytest.raises(ValueError):
        plan.pack(bodies[:-1])
    bad = list(bodies)
    bad[1] = b'{"status": "error", "data": {"result": []}}'
    with pytest.raises(PrometheusResponseError, match="body 1"):
        plan.pack(bad)
    bad[1] = b'{"status": "success", "data": {"result": [{"metric": {}, "values": [[1, "x"]]}]}}'
    with pytest.raises(PrometheusResponseError, match="body 1"):
        plan.pack(bad)
    empty = FleetQueryPlan([])
    s = empty.pack([])
    assert s.values.size == 0 and list(s.offsets) == [0]
    nopods = FleetQueryPlan([Obj("n", "c", []), Obj("n", "c", [])])
    s = nopods.pack([])
    assert list(s.offsets) == [0, 0, 0]


def test_parse_series_labels_and_first_match():
    doc = {"status": "success", "data": {"resultType": "matrix", "result": [
        {"metric": {"pod": "a\"b"}, "values": [[1.5, "1"], [2.5, "2e-3"]]},
        {"metric": {}, "values": [[1, "NaN"]]},
        {"metric": {"pod": "a\"b"}, "values": [[1, "9"]]},
    ]}}
    out = parse_series(json.dumps(doc).encode(), want_timestamps=True)
    assert [o[0] for o in out] == ['a"b', None, 'a"b']
    assert out[0][1].tolist() == [1.0, 0.002] and out[0][2].tolist() == [1.5, 2.5]
    assert np.isnan(out[1][1][0])
    # a duplicated label keeps the first series (the reference reads result[0])
    plan = FleetQueryPlan([Obj("n", "c", ['a"b'])])
    s = plan.pack([json.dumps(doc).encode()])
    assert s.values.tolist() == [1.0, 0.002]


@pytest.mark.parametrize("max_samples", [10_000, 25_000, 1])
@pytest.mark.parametrize("resource", list(ResourceType))
def test_sample_bounded_groups_keep_the_per_pod_csr(resource, max_samples):
    """Groups split by expected samples (pods x series_per_pod x points <= max_query_samples)
    still pack to the per-pod CSR byte for byte."""
    objects, prom = make_fleet()
    points = 1000
    plan = FleetQueryPlan(objects, points_per_series=points, max_query_samples=max_samples, series_per_pod=2)
    cap = max(1, max_samples // (points * 2))
    assert all(1 <= len(g.pods) <= cap for g in plan.groups)
    grouped = [prom.query_range(q) for q in plan.queries(resource)]
    got = plan.pack(grouped)
    exp = pack_query_range_bodies(per_pod_bodies(objects, prom, resource))
    np.testing.assert_array_equal(got.offsets, exp.offsets)
    assert got.values.tobytes() == exp.values.tobytes()
    unbounded = FleetQueryPlan(objects, points_per_series=0)
    assert len(plan.groups) >= len(unbounded.groups)


def test_plan_for_settings_counts_points():
    from krr_amd.strategies.simple import SimpleStrategySettings

    objects, _ = make_fleet()
    plan = FleetQueryPlan.for_settings(objects, SimpleStrategySettings())  # 336 h @ 15 min
    assert plan.points_per_series == 336 * 4 + 1
    big = [Obj("ns", "c", [f"p{i}" for i in range(20_000)])]
    pods_per_group = [len(g.pods) for g in FleetQueryPlan.for_settings(big, SimpleStrategySettings(),
                                                                       max_query_chars=10**9).groups]
    assert max(pods_per_group) == 50_000_000 // (1345 * 4) and sum(pods_per_group) == 20_000
    with pytest.raises(ValueError):
        FleetQueryPlan(objects, points_per_series=-1)
    # without settings the plan still bounds samples, at the reference's default settings
    default = FleetQueryPlan(big, max_query_chars=10**9)
    assert default.points_per_series == 1345 and max(len(g.pods) for g in default.groups) == max(pods_per_group)


@pytest.mark.parametrize("max_chars", [6000, 40])
def test_group_sorted_slots_are_contiguous_per_group(max_chars):
    """The device packer routes a chunk of whole bodies over one range of this order."""
    objects, _ = make_fleet()
    plan = FleetQueryPlan(objects, max_query_chars=max_chars)
    order, sgroup, blob, offs, gstart = plan.group_sorted_slots()
    assert sorted(order.tolist()) == list(range(plan.n_slots))
    np.testing.assert_array_equal(sgroup, plan.slot_group[order])
    assert np.all(np.diff(sgroup) >= 0)
    for g in range(len(plan.groups)):
        idx = order[gstart[g]:gstart[g + 1]]
        np.testing.assert_array_equal(idx, np.flatnonzero(plan.slot_group == g))  # stable: plan order
    assert gstart[0] == 0 and gstart[-1] == plan.n_slots
    names = [blob[offs[i]:offs[i + 1]].decode() for i in range(plan.n_slots)]
    assert names == [plan.slot_pods[i] for i in order.tolist()]
    assert plan.group_sorted_slots() is plan.group_sorted_slots()  # cached


@pytest.mark.parametrize("resource", list(ResourceType))
def test_pack_group_slots_equals_the_plan_pack(resource):
    """The hybrid grouped parser's host side: groups [g0, g1) alone, one segment per slot, give
    each slot the series plan.pack routes to it (values and per-slot counts)."""
    objects, prom = make_fleet(seed=5)
    plan = FleetQueryPlan(objects, max_query_chars=40)
    bodies = [prom.query_range(q) for q in plan.queries(resource)]
    full, counts = plan.pack(bodies, return_pod_counts=True)
    ng = len(plan.groups)
    # the full plan's per-slot values: walk objects' segments in slot order (kept slots only)
    per_slot, pos = {}, 0
    for s in range(plan.n_slots):
        if counts[s] > 0:
            per_slot[s] = full.values[pos:pos + counts[s]]
            pos += counts[s]
    for g0, g1 in ((0, ng), (ng // 2, ng), (ng - 1, ng), (0, 1)):
        idx, values, offsets, cnt = plan.pack_group_slots(bodies[g0:g1], g0, g1)
        np.testing.assert_array_equal(idx, np.flatnonzero((plan.slot_group >= g0) & (plan.slot_group < g1)))
        np.testing.assert_array_equal(cnt, counts[idx])
        for j, s in enumerate(idx.tolist()):
            got = values[offsets[j]:offsets[j + 1]]
            if counts[s] > 0:
                assert got.tobytes() == per_slot[s].tobytes()
            else:
                assert got.size == 0
    with pytest.raises(ValueError):
        plan.pack_group_slots(bodies[:1], 0, 2)
