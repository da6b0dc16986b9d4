"""Device packer (include/krr_amd.h krr_json_parse / krr_json_compact, krr_amd/csrc/krr_json.h)
against the host packer (krr_pack_parse, itself pinned to json + Decimal by
tests/test_prom_native.py): values, offsets, pod drops and timestamps bit for bit.

Canonical bodies (what Prometheus writes: compact JSON) must be parsed on the device
(``via == "device"``); a batch holding a body outside that form goes to the host packer
and gives exactly the host's result or error."""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def packer():
    from krr_amd import _native
    from krr_amd.core.device_pack import DevicePacker

    ctx = _native.Context(0)
    yield DevicePacker(ctx, chunk_bytes=1 << 20)
    ctx.close()


def _compact(doc) -> bytes:
    return json.dumps(doc, separators=(",", ":")).encode()


def _host(per_obj, want_ts=True):
    from krr_amd.core.prom_native import pack_query_range_bodies

    return pack_query_range_bodies(per_obj, want_timestamps=want_ts, return_pod_counts=True)


def _same(dp, per_obj, want_ts=True):
    if want_ts:
        ps, ts, counts = _host(per_obj, want_ts)
    else:
        ps, counts = _host(per_obj, want_ts)
    got = dp.series
    v = got.values.cpu().numpy() if hasattr(got.values, "cpu") else got.values
    o = got.offsets.cpu().numpy() if hasattr(got.offsets, "cpu") else got.offsets
    assert np.array_equal(o, ps.offsets)
    assert np.array_equal(v.view(np.uint64), ps.values.view(np.uint64))
    assert got.max_len == ps.max_len
    pc = dp.pod_counts.cpu().numpy() if hasattr(dp.pod_counts, "cpu") else dp.pod_counts
    assert np.array_equal(pc, counts)
    if want_ts:
        t = dp.timestamps.cpu().numpy() if hasattr(dp.timestamps, "cpu") else dp.timestamps
        assert np.array_equal(t.view(np.uint64), ts.view(np.uint64))


def _fleet(seed, n_obj=80, max_samples=3000):
    from krr_amd.utils.prom_decimal import prom_format

    rng = np.random.default_rng(seed)
    per_obj = []
    for o in range(n_obj):
        pods = []
        for p in range(int(rng.integers(0, 5))):
            if rng.random() < 0.12:
                pods.append(_compact({"status": "success", "data": {"resultType": "matrix", "result": []}}))
                continue
            n = int(rng.integers(0, max_samples))
            xs = rng.gamma(2.0, 0.05, n)
            sp = rng.random(n)
            xs[sp < 0.01] = np.nan
            xs[(sp >= 0.01) & (sp < 0.015)] = np.inf
            xs[(sp >= 0.015) & (sp < 0.02)] = -np.inf
            m = (sp >= 0.02) & (sp < 0.1)
            xs[m] = np.floor(rng.normal(2e8, 2e7, int(m.sum())))
            m = (sp >= 0.1) & (sp < 0.105)
            xs[m] = 1e-300 * rng.random(int(m.sum()))
            m = (sp >= 0.105) & (sp < 0.11)
            xs[m] = 1e300 * rng.random(int(m.sum()))  # 300-digit strings: elements longer than a block's lane
            ts = 1.7e9 + 60.0 * np.arange(n) + 0.781
            res = [{"metric": {"pod": f"p{o}-{p}", "container": "c"},
                    "values": [[float(t), prom_format(float(x))] for t, x in zip(ts, xs)]}]
            if rng.random() < 0.3:
                res.append({"metric": {"pod": "x"}, "values": [[1.0, "7"]]})
            pods.append(_compact({"status": "success", "data": {"resultType": "matrix", "result": res}}))
        per_obj.append(pods)
    return per_obj


@pytest.mark.parametrize("seed", [1, 2])
def test_canonical_fleet_parsed_on_device(packer, seed):
    per_obj = _fleet(seed)
    dp = packer.pack(per_obj, want_timestamps=True, return_pod_counts=True)
    assert dp.via == "device" and dp.host_bodies == 0
    _same(dp, per_obj)


def test_prom_native_vectors_compacted(packer):
    """tests/test_prom_native.py's fleet (escaped label values, non-ASCII keys, extra
    series, NaN/Inf, subnormals), re-serialised compactly as Prometheus writes it."""
    from test_prom_native import _fleet as pn_fleet

    per_obj = [[json.dumps(json.loads(b), separators=(",", ":")).encode() for b in bodies]
               for bodies in pn_fleet(1)]
    dp = packer.pack(per_obj, want_timestamps=True, return_pod_counts=True)
    assert dp.via == "device"
    _same(dp, per_obj)


def test_prom_native_vectors_as_is(packer):
    """The same vectors as json.dumps writes them (', ' and ': ' between every token): parsed
    on the device too, with the host's bits."""
    from test_prom_native import _fleet as pn_fleet

    per_obj = pn_fleet(1)
    dp = packer.pack(per_obj, want_timestamps=True, return_pod_counts=True)
    assert dp.via == "device"
    _same(dp, per_obj)


def test_non_canonical_batch_goes_to_the_host(packer):
    """A body the device does not decide (an escaped key): the batch is the host packer's."""
    per_obj = _fleet(4, n_obj=12)
    per_obj[5] = per_obj[5] + [_compact({"status": "success", "data": {"resultType": "matrix", "result": [
        {"metric": {}, "values": [[1, "2"]]}]}}).replace(b'"status"', b'"st\\u0061tus"')]
    dp = packer.pack(per_obj, want_timestamps=True, return_pod_counts=True)
    assert dp.via == "host" and dp.host_bodies == 1
    _same(dp, per_obj)


def test_config2_sized_bodies_many_chunks(packer):
    """10,080-sample bodies (7d@1m), many per chunk and chunks of 1 MiB: the staged copy /
    parse pipeline and the block loop over long values arrays."""
    from krr_amd.utils.prom_decimal import prom_format

    rng = np.random.default_rng(5)
    per_obj = []
    for o in range(40):
        pods = []
        for p in range(3):
            xs = rng.gamma(2.0, 0.05, 10080)
            vals = ",".join(f'[{1700000000 + 60 * i},"{prom_format(float(x))}"]' for i, x in enumerate(xs))
            pods.append(('{"status":"success","data":{"resultType":"matrix","result":[{"metric":{},"values":['
                         + vals + ']}]}}').encode())
        per_obj.append(pods)
    dp = packer.pack(per_obj, want_timestamps=True, return_pod_counts=True)
    assert dp.via == "device"
    _same(dp, per_obj)


@pytest.mark.parametrize("bad", [b'{"status":"error","errorType":"bad_data","error":"x"}', b'{"status":"success"',
                                 b'not json'])
def test_error_bodies_raise_the_host_error(packer, bad):
    from krr_amd.core.prom_native import PrometheusResponseError

    per_obj = _fleet(3, n_obj=10)
    per_obj[4] = per_obj[4] + [bad]
    with pytest.raises(PrometheusResponseError) as dev_err:
        packer.pack(per_obj)
    with pytest.raises(PrometheusResponseError) as host_err:
        _host(per_obj)
    assert str(dev_err.value) == str(host_err.value) and dev_err.value.code == host_err.value.code


def test_empty_and_odd_layouts(packer):
    per_obj = [[], [_compact({"status": "success", "data": {"result": [{"metric": {}, "values": []}]}})],
               [_compact({"data": {"result": [{"values": [[1, "1"], [2, "2"]], "metric": {"a": "b"}}],
                                   "resultType": "matrix"}, "status": "success", "warnings": ["w"]})],
               []]
    dp = packer.pack(per_obj, want_timestamps=True, return_pod_counts=True)
    assert dp.via == "device"
    _same(dp, per_obj)
    dp = packer.pack([], want_timestamps=False, return_pod_counts=True)
    assert dp.series.offsets.numel() == 1


def test_recommend_from_bodies_device_equals_host():
    """The whole path from bodies: device parse -> kernel -> rounding equals the host
    packer's path, result for result."""
    from krr_amd.core.runner import BatchedRunner
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    cpu = _fleet(7, n_obj=60, max_samples=2000)
    mem = _fleet(8, n_obj=60, max_samples=2000)
    # finite samples only: the reference's rounding raises on +-Inf (math.ceil) and on a NaN
    # memory sample (max over Decimals) — both paths would raise the same there
    def finite(b):
        return b.replace(b'"NaN"', b'"1"').replace(b'"+Inf"', b'"2"').replace(b'"-Inf"', b'"3"')

    cpu = [[finite(b) for b in bodies] for bodies in cpu]
    mem = [[finite(b) for b in bodies] for bodies in mem]
    runner = BatchedRunner(SimpleStrategy(SimpleStrategySettings(cpu_percentile="99", memory_buffer_percentage="5")))
    a = runner.recommend_from_bodies(cpu, mem, parser="device")
    assert runner.last_pack_via == ("device", "device")
    b = runner.recommend_from_bodies(cpu, mem, parser="host")
    assert [{k: (str(v.request), str(v.limit)) for k, v in r.items()} for r in a] == \
           [{k: (str(v.request), str(v.limit)) for k, v in r.items()} for r in b]


@pytest.mark.parametrize("share", [0.02, 0.3, 0.8])
def test_recommend_from_bodies_hybrid_equals_host(share):
    """parser="hybrid": the last share of the objects parsed by the host packer while the
    first part is parsed on the device (one kernel pass each) equals the host packer's path
    result for result, at any split; the same through pack_from_bodies (one fleet in HBM);
    a malformed body in either part gives the host packer's error on the whole batch."""
    from krr_amd.core.prom_native import PrometheusResponseError
    from krr_amd.core.runner import BatchedRunner
    from krr_amd.strategies.simple import SimpleStrategy, SimpleStrategySettings

    def finite(b):
        return b.replace(b'"NaN"', b'"1"').replace(b'"+Inf"', b'"2"').replace(b'"-Inf"', b'"3"')

    cpu = [[finite(b) for b in bodies] for bodies in _fleet(17, n_obj=80, max_samples=1500)]
    mem = [[finite(b) for b in bodies] for bodies in _fleet(18, n_obj=80, max_samples=1500)]
    runner = BatchedRunner(SimpleStrategy(SimpleStrategySettings(cpu_percentile="95", memory_buffer_percentage="7")))
    want = [{k: (str(v.request), str(v.limit)) for k, v in r.items()}
            for r in runner.recommend_from_bodies(cpu, mem, parser="host")]
    runner.hybrid_share = share
    got = runner.recommend_from_bodies(cpu, mem, parser="hybrid", threads=8)
    assert runner.last_pack_via == ("hybrid", "hybrid") and 0 < runner.hybrid_last["split_object"] < 80
    assert [{k: (str(v.request), str(v.limit)) for k, v in r.items()} for r in got] == want
    fleet = runner.pack_from_bodies(cpu, mem, threads=8, parser="hybrid")
    assert fleet.cpu.values.is_cuda and fleet.n_objects == 80
    got2 = runner.recommend_packed(fleet)
    assert [{k: (str(v.request), str(v.limit)) for k, v in r.items()} for r in got2] == want
    for bad_at in (0, 79):  # device part / host part
        broken = [list(b) for b in cpu]
        broken[bad_at] = [b'{"status":"error","errorType":"bad_data","error":"boom"}'] + broken[bad_at]
        with pytest.raises(PrometheusResponseError) as e_h:
            runner.recommend_from_bodies(broken, mem, parser="host")
        runner.hybrid_share = share
        with pytest.raises(PrometheusResponseError) as e_y:
            runner.recommend_from_bodies(broken, mem, parser="hybrid", threads=8)
        assert str(e_y.value) == str(e_h.value)


# ---- grouped bodies (fleet PromQL batching): krr_json_parse_series + krr_pack_match_grouped ----

def _recompact(b: bytes) -> bytes:
    return json.dumps(json.loads(b), separators=(",", ":")).encode()


@pytest.fixture(params=[("chunk", True), ("end", True), ("chunk", False)], ids=["chunk-split", "end-split",
                                                                                   "chunk-wave"])
def route_mode(request, packer):
    """Both routings: chunk by chunk (segments written into page-locked host memory by the
    parse kernel) and once after the last parse (one device-to-host copy); the values arrays
    parsed in 16-KiB parts (krr_json_parse_segments_split) or one wave per series."""
    was = packer.grouped_route, packer.grouped_split_parse
    packer.grouped_route, packer.grouped_split_parse = request.param
    yield request.param
    packer.grouped_route, packer.grouped_split_parse = was


@pytest.mark.parametrize("max_chars", [6000, 40, 1])
@pytest.mark.parametrize("resource", ["cpu", "memory"])
def test_grouped_bodies_on_device_equal_host_plan(packer, resource, max_chars, route_mode):
    """tests/test_fleet_query.py's fleet (regex-metacharacter pod names, restarts summed per
    pod, decoy series, shuffled series order, duplicated and ghost pods): the device parse
    routed by pod label gives plan.pack's CSR, timestamps and pod counts bit for bit."""
    from test_fleet_query import make_fleet

    from krr_amd.core.fleet_query import FleetQueryPlan
    from krr_amd.core.models.allocations import ResourceType

    objects, prom = make_fleet()
    plan = FleetQueryPlan(objects, max_query_chars=max_chars)
    rt = ResourceType(resource)
    bodies = [_recompact(prom.query_range(q)) for q in plan.queries(rt)]
    want, want_ts, want_counts = plan.pack(bodies, want_timestamps=True, return_pod_counts=True)
    dp = packer.pack_grouped(plan, bodies, want_timestamps=True, return_pod_counts=True)
    assert dp.via == "device"
    assert np.array_equal(dp.series.offsets.cpu().numpy(), want.offsets)
    assert np.array_equal(dp.series.values.cpu().numpy().view(np.uint64), want.values.view(np.uint64))
    assert np.array_equal(dp.timestamps.cpu().numpy().view(np.uint64), want_ts.view(np.uint64))
    assert np.array_equal(np.asarray(dp.pod_counts), want_counts)
    assert dp.series.max_len == want.max_len
    # as json.dumps wrote them (', ' / ': ' between tokens): on the device too, same bits
    raw = [prom.query_range(q) for q in plan.queries(rt)]
    dh = packer.pack_grouped(plan, raw, want_timestamps=True, return_pod_counts=True)
    assert dh.via == "device"
    assert np.array_equal(dh.series.values.cpu().numpy().view(np.uint64), want.values.view(np.uint64))
    assert np.array_equal(dh.series.offsets.cpu().numpy(), want.offsets)
    # a body with an escaped series key: that batch is the host's
    bad = list(bodies)
    bad[0] = bad[0].replace(b'"values"', b'"v\\u0061lues"', 1)
    dh = packer.pack_grouped(plan, bad, want_timestamps=True, return_pod_counts=True)
    hv = plan.pack(bad, want_timestamps=True, return_pod_counts=True)[0]
    assert dh.via == "host" and np.array_equal(dh.series.values.view(np.uint64), hv.values.view(np.uint64))


def test_grouped_large_bodies(packer):
    """Groups of 40 pods x 10,080 samples per body (several MB per body, many blocks per
    series), pods listed in another order than the series."""
    from krr_amd.core.fleet_query import FleetQueryPlan
    from krr_amd.utils.prom_decimal import prom_format

    class Obj:
        def __init__(self, ns, c, pods):
            self.namespace, self.container, self.pods = ns, c, pods

    rng = np.random.default_rng(12)
    objects = [Obj(f"ns{g}", "app", [f"pod-{g}-{k}" for k in range(int(rng.integers(1, 4)))]) for g in range(40)]
    plan = FleetQueryPlan(objects, max_query_chars=400)
    bodies = []
    for grp in plan.groups:
        res = []
        for pod in reversed(grp.pods):
            xs = rng.gamma(2.0, 0.05, 10080)
            res.append({"metric": {"pod": pod}, "values": [[1700000000 + 60 * k, prom_format(float(x))]
                                                           for k, x in enumerate(xs)]})
        bodies.append(_compact({"status": "success", "data": {"resultType": "matrix", "result": res}}))
    want, want_counts = plan.pack(bodies, return_pod_counts=True)
    dp = packer.pack_grouped(plan, bodies, return_pod_counts=True)
    assert dp.via == "device"
    assert np.array_equal(dp.series.offsets.cpu().numpy(), want.offsets)
    assert np.array_equal(dp.series.values.cpu().numpy().view(np.uint64), want.values.view(np.uint64))
    assert np.array_equal(np.asarray(dp.pod_counts), want_counts)


@pytest.mark.parametrize("split", [True, False])
def test_grouped_split_parse_at_part_boundaries(packer, split):
    """Values arrays ending at every offset around the 16-KiB parts of the split parse (1 to
    4,000 samples, value strings of several lengths, NaN / Inf / signs), json.dumps spacing,
    end brackets the split scan cannot pair (`] ]` in the first or the last series: the scan
    stops at the series' `}` and the series' own wave parses it — on the device), and an
    indented body (the host's): the CSR is the host plan's."""
    from krr_amd.core.fleet_query import FleetQueryPlan

    class Obj:
        def __init__(self, ns, c, pods):
            self.namespace, self.container, self.pods = ns, c, pods

    rng = np.random.default_rng(31)
    lens = [1, 2, 3, 511, 512, 513, 700, 701, 1023, 1024, 1025, 1400, 2047, 2048, 2049, 4000]
    objects = [Obj("ns", "app", [f"pod-{k}" for k in range(len(lens))])]
    plan = FleetQueryPlan(objects, max_query_chars=10_000)
    assert len(plan.groups) == 1
    specials = ["NaN", "+Inf", "-Inf", "-0", "0", "1e-300", "123456789012345678"]

    def body(shift, dumps_kw):
        res = []
        for k, pod in enumerate(plan.groups[0].pods):
            n = lens[(k + shift) % len(lens)]
            vals = [specials[i % len(specials)] if i % 97 == 5 else repr(float(rng.gamma(2.0, 10.0 ** (i % 7 - 3))))
                    for i in range(n)]
            res.append({"metric": {"pod": pod, "container": "app"},
                        "values": [[1700000000 + 15 * i, v] for i, v in enumerate(vals)]})
        return json.dumps({"status": "success", "data": {"resultType": "matrix", "result": res}},
                          **dumps_kw).encode()

    p = packer
    was = p.grouped_split_parse
    p.grouped_split_parse = split
    try:
        for shift in range(0, len(lens), 5):
            cases = {"compact": ([body(shift, {"separators": (",", ":")})], True),
                     "dumps": ([body(shift, {})], True),
                     # (indented: `,\n  {"metric"` is no series candidate — the host's batch)
                     "indent": ([body(shift, {"indent": 1})], False)}
            b = cases["compact"][0][0]
            cut = b.index(b'"]]}') + 2  # the first series' "]]" -> "] ]"
            cases["spaced_end"] = ([b[:cut - 1] + b" " + b[cut - 1:]], True)
            last = b.rindex(b'"]]}') + 2  # and the last one's (no "]]" after it in the body)
            cases["spaced_last_end"] = ([b[:last - 1] + b" " + b[last - 1:]], True)
            for name, (bodies, on_device) in cases.items():
                want, want_counts = plan.pack(bodies, return_pod_counts=True)
                dp = p.pack_grouped(plan, bodies, return_pod_counts=True)
                if on_device:
                    assert dp.via == "device", name
                got = dp.series.values.cpu().numpy() if dp.via == "device" else dp.series.values
                offs = dp.series.offsets.cpu().numpy() if dp.via == "device" else dp.series.offsets
                assert np.array_equal(offs, want.offsets), name
                assert np.array_equal(np.asarray(got).view(np.uint64), want.values.view(np.uint64)), name
                assert np.array_equal(np.asarray(dp.pod_counts), want_counts), name
    finally:
        p.grouped_split_parse = was


def test_pack_many_equals_separate(packer):
    """CPU and memory bodies through one pipeline (pack_many) equal each packed alone; a
    resource with a non-canonical body goes to the host alone."""
    cpu = _fleet(21, n_obj=30)
    mem = _fleet(22, n_obj=30)
    a, b = packer.pack_many([cpu, mem], want_timestamps=True, return_pod_counts=True)
    assert a.via == b.via == "device"
    _same(a, cpu)
    _same(b, mem)
    mem_bad = [list(x) for x in mem]
    mem_bad[3] = mem_bad[3] + [_compact({"status": "success", "data": {"result": [  # an escaped key
        {"metric": {}, "values": [[1, "2"], [2, "3"]]}]}}).replace(b'"status"', b'"st\\u0061tus"')]
    a, b = packer.pack_many([cpu, mem_bad], want_timestamps=True, return_pod_counts=True)
    assert a.via == "device" and b.via == "host"
    _same(a, cpu)
    _same(b, mem_bad)


def test_grouped_many_and_small_chunks(packer, route_mode):
    """CPU and memory grouped bodies through one pipeline, with 1-MiB chunks: candidates
    near chunk ends are searched with the next chunk (the 16-byte carry)."""
    from test_fleet_query import make_fleet

    from krr_amd.core.device_pack import DevicePacker
    from krr_amd.core.fleet_query import FleetQueryPlan
    from krr_amd.core.models.allocations import ResourceType

    objects, prom = make_fleet(seed=3, n_obj=40)
    plan = FleetQueryPlan(objects, max_query_chars=60)
    bc = [_recompact(prom.query_range(q)) for q in plan.queries(ResourceType.CPU)]
    bm = [_recompact(prom.query_range(q)) for q in plan.queries(ResourceType.Memory)]
    small = DevicePacker(packer.ctx, chunk_bytes=4096)
    for p in (packer, small):
        a, b = p.pack_grouped_many([(plan, bc), (plan, bm)], want_timestamps=True, return_pod_counts=True)
        for dp, bodies in ((a, bc), (b, bm)):
            want, want_ts, want_counts = plan.pack(bodies, want_timestamps=True, return_pod_counts=True)
            assert dp.via == "device"
            assert np.array_equal(dp.series.offsets.cpu().numpy(), want.offsets)
            assert np.array_equal(dp.series.values.cpu().numpy().view(np.uint64), want.values.view(np.uint64))
            assert np.array_equal(dp.timestamps.cpu().numpy().view(np.uint64), want_ts.view(np.uint64))
            assert np.array_equal(np.asarray(dp.pod_counts), want_counts)


def _stripped_cases():
    import json as _json

    from test_prom_native import _fleet as pn_fleet

    compacted = [[_json.dumps(_json.loads(b), separators=(",", ":")).encode() for b in bodies]
                 for bodies in pn_fleet(1)]
    mixed = _fleet(6, n_obj=30)
    # bodies the strip leaves whole, beside stripped ones: an escape, an exponent and a
    # leading-zero timestamp (the device then parses the original bytes of those)
    mixed[3] = mixed[3] + [b'{"status":"success","data":{"resultType":"matrix","result":[{"metric":{"pod":"a\\"b"},'
                           b'"values":[[1700000000.5,"0.5"],[1700000060,"0.75"]]}]}}']
    mixed[7] = mixed[7] + [b'{"status":"success","data":{"resultType":"matrix","result":[{"metric":{},'
                           b'"values":[[1.7e9,"1"],[1.70000006e9,"2"]]}]}}']
    mixed[9] = mixed[9] + [b'{"status":"success","data":{"resultType":"matrix","result":[{"metric":{},'
                           b'"values":[[0.5,"3"],[10,"4"]]}]}}']
    return {"fleet1": _fleet(1), "fleet2": _fleet(2), "prom_native_compacted": compacted,
            "prom_native_as_is": pn_fleet(1), "mixed": mixed}


@pytest.mark.parametrize("case", ["fleet1", "fleet2", "prom_native_compacted", "prom_native_as_is", "mixed"])
@pytest.mark.parametrize("chunk", [1 << 20, 4096])
def test_stripped_staging_equals_host(packer, case, chunk):
    """Without timestamps the bodies are staged with their timestamps cut (krr_strip.h): fewer
    bytes cross PCIe and the CSR, the pod drops and the device/host decision are unchanged."""
    from krr_amd.core.device_pack import DevicePacker

    per_obj = _stripped_cases()[case]
    p = DevicePacker(packer.ctx, chunk_bytes=chunk)
    assert p.strip
    dp = p.pack(per_obj, want_timestamps=False, return_pod_counts=True)
    assert dp.via == "device"
    _same(dp, per_obj, want_ts=False)
    up = p.last_upload
    if case.startswith("prom_native"):  # escaped label values in every body: none stripped
        assert up["bodies_stripped"] == 0 and up["bytes_sent"] == up["bytes"]
    else:
        assert up["bodies_stripped"] > 0 and up["bytes_sent"] < 0.8 * up["bytes"]
    q = DevicePacker(packer.ctx, chunk_bytes=chunk, strip=False)
    dq = q.pack(per_obj, want_timestamps=False, return_pod_counts=True)
    assert q.last_upload["bytes_sent"] == q.last_upload["bytes"]
    assert np.array_equal(dq.series.values.cpu().numpy().view(np.uint64), dp.series.values.cpu().numpy().view(np.uint64))


def test_stripped_staging_error_and_host_batches(packer):
    """A batch the device hands to the host, and one with an error body, behave as without
    the strip: the host packer's result or error on the ORIGINAL bodies."""
    from krr_amd.core.prom_native import PrometheusResponseError

    per_obj = _fleet(4, n_obj=12)
    per_obj[5] = per_obj[5] + [_compact({"status": "success", "data": {"resultType": "matrix", "result": [
        {"metric": {}, "values": [[1, "2"]]}]}}).replace(b'"status"', b'"st\\u0061tus"')]
    dp = packer.pack(per_obj, want_timestamps=False, return_pod_counts=True)
    assert dp.via == "host" and dp.host_bodies == 1
    _same(dp, per_obj, want_ts=False)
    bad = _fleet(3, n_obj=10)
    bad[4] = bad[4] + [b'{"status":"success","data":{"resultType":"matrix","result":[{"metric":{},'
                       b'"values":[[1700000000,"1"],[1700000015,2]]}]}}']  # an unquoted value
    with pytest.raises(PrometheusResponseError) as dev_err:
        packer.pack(bad)
    with pytest.raises(PrometheusResponseError) as host_err:
        _host(bad)
    assert str(dev_err.value) == str(host_err.value) and dev_err.value.code == host_err.value.code


@pytest.mark.parametrize("share", [0.05, 0.3, 0.9])
def test_grouped_hybrid_equals_host_plan(packer, share):
    """The hybrid grouped parser (round 6): the last groups' bodies parsed by the host packer
    (FleetQueryPlan.pack_group_slots) while the rest are staged in pieces, parsed on the device
    and routed; the host slots' values join the device scratch and one gather builds the CSR —
    plan.pack's CSR and pod counts bit for bit, at any share; a body the host part rejects, or
    the device part, gives the host packer's error for the batch."""
    from test_fleet_query import make_fleet

    from krr_amd.core.device_pack import DevicePacker
    from krr_amd.core.fleet_query import FleetQueryPlan
    from krr_amd.core.models.allocations import ResourceType
    from krr_amd.core.prom_native import PrometheusResponseError

    objects, prom = make_fleet(seed=5, n_obj=60)
    plan = FleetQueryPlan(objects, max_query_chars=300)
    bc = [_recompact(prom.query_range(q)) for q in plan.queries(ResourceType.CPU)]
    bm = [_recompact(prom.query_range(q)) for q in plan.queries(ResourceType.Memory)]
    assert len(plan.groups) >= 4
    for p in (packer, DevicePacker(packer.ctx, chunk_bytes=8192)):
        p.grouped_share = share
        a, b = p.pack_grouped_many([(plan, bc), (plan, bm)], return_pod_counts=True, hybrid=True)
        assert getattr(p, "last_grouped_hybrid", None) and p.last_grouped_hybrid["host_bodies"] >= 1
        for dp, bodies in ((a, bc), (b, bm)):
            want, want_counts = plan.pack(bodies, return_pod_counts=True)
            assert dp.via == "device"
            assert np.array_equal(dp.series.offsets.cpu().numpy(), want.offsets)
            assert np.array_equal(dp.series.values.cpu().numpy().view(np.uint64), want.values.view(np.uint64))
            assert np.array_equal(np.asarray(dp.pod_counts), want_counts)
            assert dp.series.max_len == want.max_len
    err = b'{"status":"error","errorType":"bad_data","error":"boom"}'
    for at in (0, len(bm) - 1):  # the device part / the host part
        bad = list(bm)
        bad[at] = err
        with pytest.raises(PrometheusResponseError) as e_h:
            plan.pack(bad)
        packer.grouped_share = share
        with pytest.raises(PrometheusResponseError) as e_y:
            packer.pack_grouped_many([(plan, bc), (plan, bad)], hybrid=True)
        assert str(e_y.value) == str(e_h.value)


def test_grouped_large_bodies_in_pieces_and_hybrid(packer, route_mode):
    """~2.5 MB grouped bodies staged in pieces cut inside the bodies (`"],[`), parsed one chunk
    behind the search on the parse streams, with and without the host share: plan.pack's CSR."""
    from krr_amd.core.device_pack import DevicePacker
    from krr_amd.core.fleet_query import FleetQueryPlan
    from krr_amd.utils.prom_decimal import prom_format

    class Obj:
        def __init__(self, ns, c, pods):
            self.namespace, self.container, self.pods = ns, c, pods

    rng = np.random.default_rng(31)
    objects = [Obj(f"ns{g % 6}", "app", [f"pod-{g}-{k}" for k in range(int(rng.integers(1, 4)))]) for g in range(60)]
    plan = FleetQueryPlan(objects, max_query_chars=2000)
    bodies = []
    for grp in plan.groups:
        res = []
        for pod in reversed(grp.pods):
            xs = rng.gamma(2.0, 0.05, int(rng.integers(3000, 10081)))
            res.append({"metric": {"pod": pod, "note": "],[1,2"},  # cut-like bytes inside a string
                        "values": [[1700000000 + 60 * k + 0.25 * (k % 3), prom_format(float(x))]
                                   for k, x in enumerate(xs)]})
        bodies.append(_compact({"status": "success", "data": {"resultType": "matrix", "result": res}}))
    want, want_counts = plan.pack(bodies, return_pod_counts=True)
    for p in (packer, DevicePacker(packer.ctx, chunk_bytes=1 << 20, threads=5)):
        for hybrid in (False, True):
            p.grouped_share = 0.25
            dp = p.pack_grouped_many([(plan, bodies)], return_pod_counts=True, hybrid=hybrid)[0]
            assert dp.via == "device"
            n_dev = len(bodies) - (p.last_grouped_hybrid["host_bodies"] if hybrid else 0)
            if p is packer:  # its pieces (2 per staging thread) are smaller than a body: the bodies were cut
                assert p.last_upload["pieces"] > n_dev, (p.last_upload, n_dev)
            assert np.array_equal(dp.series.offsets.cpu().numpy(), want.offsets)
            assert np.array_equal(dp.series.values.cpu().numpy().view(np.uint64), want.values.view(np.uint64))
            assert np.array_equal(np.asarray(dp.pod_counts), want_counts)


def _fuzz_grouped_bodies(rng, plan):
    """One body per group of `plan`, each with random variations of what a query_range answer
    may hold: separators (compact, json.dumps, indented), key orders, extra keys, empty and long
    values arrays, value spellings (shortest reprs, integers, exponents, NaN / +Inf / -Inf, 19
    and 21 significant digits), a label value with an escape, and `] ]` at an array's end."""
    spellings = [lambda x: repr(x), lambda x: str(int(x * 1000)), lambda x: f"{x:.6e}", lambda x: "NaN",
                 lambda x: "+Inf", lambda x: "-Inf", lambda x: "1234567890123456789",
                 lambda x: "123456789012345678901", lambda x: f"{-x!r}"]
    bodies = []
    for grp in plan.groups:
        res = []
        for pod in rng.permutation(grp.pods).tolist():
            n = int(rng.choice([0, 1, 2, 3, 100, 2047, 2048, 5000]))
            xs = rng.gamma(2.0, 0.05, n)
            vals = [spellings[int(rng.integers(0, len(spellings)))](float(x)) if rng.random() < 0.05 else repr(float(x))
                    for x in xs]
            metric = {"pod": pod, "container": "app"}
            if rng.random() < 0.2:
                metric = dict(reversed(list(metric.items())))
            if rng.random() < 0.05:
                metric["note"] = 'a"b'  # an escape: this body is the host's
            series = {"metric": metric, "values": [[1700000000 + 15 * i, v] for i, v in enumerate(vals)]}
            if rng.random() < 0.2:
                series = {"values": series["values"], "metric": series["metric"]}
            if rng.random() < 0.1:
                series["extra"] = [1, {"k": "v"}]
            if n or rng.random() < 0.5:  # a series without samples now and then
                res.append(series)
        doc = {"status": "success", "data": {"resultType": "matrix", "result": res}}
        form = rng.random()
        if form < 0.6:
            b = json.dumps(doc, separators=(",", ":")).encode()
        elif form < 0.85:
            b = json.dumps(doc).encode()
        else:
            b = json.dumps(doc, indent=int(rng.integers(0, 3))).encode()
        if rng.random() < 0.1 and b'"]]' in b:
            i = b.index(b'"]]') + 2
            b = b[:i] + b" " + b[i:]
        bodies.append(b)
    return bodies


@pytest.mark.parametrize("seed", range(12))
def test_grouped_fuzz_equals_host(packer, route_mode, seed):
    """Randomly varied grouped bodies through the device pipeline (every routing / parse form of
    route_mode) give exactly the host plan's CSR and pod counts, or the host plan's error —
    whichever parser ends up deciding."""
    from krr_amd.core.fleet_query import FleetQueryPlan
    from krr_amd.core.prom_native import PrometheusResponseError

    class Obj:
        def __init__(self, ns, c, pods):
            self.namespace, self.container, self.pods = ns, c, pods

    rng = np.random.default_rng(1000 + seed)
    n_ns = int(rng.integers(2, 7))
    objects = [Obj(f"ns{g % n_ns}", f"c{g % 2}", [f"pod-{g}-{k}" for k in range(int(rng.integers(1, 5)))])
               for g in range(int(rng.integers(4, 16)))]
    plan = FleetQueryPlan(objects, max_query_chars=int(rng.choice([40, 200, 10_000])))
    bodies = _fuzz_grouped_bodies(rng, plan)
    try:
        want, want_counts = plan.pack(bodies, return_pod_counts=True)
    except PrometheusResponseError as e:
        with pytest.raises(PrometheusResponseError) as got:
            packer.pack_grouped(plan, bodies, return_pod_counts=True)
        assert got.value.code == e.code
        return
    dp = packer.pack_grouped(plan, bodies, return_pod_counts=True)
    vals = dp.series.values.cpu().numpy() if dp.via == "device" else np.asarray(dp.series.values)
    offs = dp.series.offsets.cpu().numpy() if dp.via == "device" else np.asarray(dp.series.offsets)
    assert np.array_equal(offs, want.offsets)
    assert np.array_equal(vals.view(np.uint64), want.values.view(np.uint64))
    assert np.array_equal(np.asarray(dp.pod_counts), want_counts)


def test_grouped_segment_rows_grow_mid_batch(packer):
    """More series than the page-locked segment-row buffer holds at first (16,384 rows): the
    buffer grows while earlier chunks' rows are still being parsed into and routed from the old
    one (their views keep it alive); the CSR is still the host plan's."""
    from krr_amd.core.device_pack import DevicePacker
    from krr_amd.core.fleet_query import FleetQueryPlan

    class Obj:
        def __init__(self, ns, c, pods):
            self.namespace, self.container, self.pods = ns, c, pods

    rng = np.random.default_rng(77)
    objects = [Obj(f"ns{o % 4}", "app", [f"p{o}-{k}" for k in range(100)]) for o in range(220)]
    plan = FleetQueryPlan(objects, max_query_chars=20_000)
    bodies = []
    for grp in plan.groups:
        res = [{"metric": {"pod": pod}, "values": [[1700000000 + 15 * i, repr(float(x))]
                                                   for i, x in enumerate(rng.gamma(2.0, 0.05, int(rng.integers(1, 4))))]}
               for pod in grp.pods]
        bodies.append(_compact({"status": "success", "data": {"resultType": "matrix", "result": res}}))
    want, want_counts = plan.pack(bodies, return_pod_counts=True)
    assert plan.n_slots > 16384
    p = DevicePacker(packer.ctx, chunk_bytes=64 << 10)
    dp = p.pack_grouped(plan, bodies, return_pod_counts=True)
    assert dp.via == "device"
    assert p._seg_rows.shape[0] > 16384  # grew during the batch
    assert np.array_equal(dp.series.offsets.cpu().numpy(), want.offsets)
    assert np.array_equal(dp.series.values.cpu().numpy().view(np.uint64), want.values.view(np.uint64))
    assert np.array_equal(np.asarray(dp.pod_counts), want_counts)


def test_split_parse_workspace_is_checked(packer):
    """krr_json_parse_segments_split refuses a workspace with no room for a part (the Python
    binding before the call, the C ABI for a raw call)."""
    import ctypes

    import torch

    from krr_amd import _native

    ctx = packer.ctx
    body = _compact({"status": "success", "data": {"resultType": "matrix", "result": [
        {"metric": {"pod": "a"}, "values": [[1, "0.5"], [2, "0.25"]]}]}})
    dev = torch.device("cuda", ctx.device)
    d_bodies = torch.zeros(len(body) + 128, dtype=torch.uint8, device=dev)
    d_bodies[:len(body)] = torch.frombuffer(bytearray(body), dtype=torch.uint8).to(dev)
    offs = torch.tensor([0, len(body)], dtype=torch.int64, device=dev)
    jb = ctx.json_bodies(d_bodies, offs, len(body))
    starts = torch.tensor([body.index(b'{"metric"')], dtype=torch.int64, device=dev)
    body_of = torch.zeros(1, dtype=torch.int64, device=dev)
    tmp_v = torch.zeros(len(body) // 8 + 1, dtype=torch.float64, device=dev)
    segs = torch.zeros(7, dtype=torch.int64, device=dev)
    with pytest.raises(ValueError):
        ctx.json_parse_segments(jb, starts, body_of, "pod", False, tmp_v, None, segs,
                                workspace=torch.zeros(4, dtype=torch.int64, device=dev))
    small = torch.zeros(1 + 1 + 5, dtype=torch.int64, device=dev)  # 1 + n + < 6: no part fits
    rc = ctx._lib.krr_json_parse_segments_split(ctx._h, ctypes.byref(jb), starts.data_ptr(), body_of.data_ptr(), 1,
                                                 b"pod", 0, tmp_v.data_ptr(), None, segs.data_ptr(),
                                                 small.data_ptr(), small.numel(), None)
    assert rc == _native.KRR_E_INVALID
    rc = ctx._lib.krr_json_parse_segments_split(ctx._h, ctypes.byref(jb), starts.data_ptr(), body_of.data_ptr(), 1,
                                                 b"pod", 0, tmp_v.data_ptr(), None, segs.data_ptr(), None, 0, None)
    assert rc == _native.KRR_E_INVALID
    # with room: the segment and its values, as the one-wave parse gives them
    ws = torch.zeros(1 + 1 + 6 * 4, dtype=torch.int64, device=dev)
    ctx.json_parse_segments(jb, starts, body_of, "pod", False, tmp_v, None, segs, workspace=ws)
    torch.cuda.synchronize()
    seg = segs.cpu().numpy()
    assert seg[6] == 1 and seg[5] == 2
    assert tmp_v.cpu().numpy()[seg[4]:seg[4] + 2].tolist() == [0.5, 0.25]
