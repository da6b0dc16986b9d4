"""Native query_range packer (libkrr_pack.so) vs the reference's semantics.

The reference (core/integrations/prometheus.py:147-155) keeps, per pod, only
result[0]["values"], drops a pod whose result list is empty, discards the
timestamps and parses each value with Decimal().  The oracle below restates that
with json + Decimal; the packer must give the same float64 bits, offsets and pod
drops.  (No reference test pins this boundary: SURVEY.md §8c, "parity unpinned"
by reference fixtures — these tests are the pin.)"""
import json
import math
from decimal import Decimal

import numpy as np
import pytest

from krr_amd.core.prom_native import PrometheusResponseError, pack_query_range_bodies


def go_format(x: float) -> str:
    """Prometheus' value formatting: strconv.FormatFloat(x, 'f', -1, 64), NaN/+Inf/-Inf."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "+Inf" if x > 0 else "-Inf"
    r = repr(x)  # shortest round-trip digits
    if "e" not in r and "E" not in r:
        return r[:-2] if r.endswith(".0") else r
    d = Decimal(r)
    s = format(d, "f")
    return s


def body(series, status="success", extra_series=0, rng=None):
    res = []
    for k in range(1 + extra_series if series is not None else 0):
        vals = series if k == 0 else [(1.0, "7")]
        res.append({"metric": {"pod": "p\"o\\d", "container": "c", "ünï": "x"},
                    "values": [[t, v] for t, v in vals]})
    doc = {"status": status, "data": {"resultType": "matrix", "result": res}}
    return json.dumps(doc).encode()


def ref_pack(per_object_bodies):
    """The reference's semantics (prometheus.py:147-155) + float()."""
    vals, offs, counts = [], [0], []
    for bodies in per_object_bodies:
        n = 0
        for b in bodies:
            result = json.loads(b)["data"]["result"]
            if result == []:
                counts.append(-1)
                continue
            v = [float(Decimal(x)) for _, x in result[0]["values"]]
            vals.extend(v)
            n += len(v)
            counts.append(len(v))
        offs.append(offs[-1] + n)
    return np.array(vals, dtype=np.float64), np.array(offs, dtype=np.int64), np.array(counts, dtype=np.int64)


def _fleet(seed, n_obj=60):
    rng = np.random.default_rng(seed)
    per_obj = []
    for o in range(n_obj):
        pods = []
        for p in range(int(rng.integers(0, 5))):
            kind = rng.random()
            if kind < 0.15:
                pods.append(body(None))  # empty result: dropped
                continue
            n = int(rng.integers(0, 400))
            xs = rng.gamma(2.0, 0.05, size=n)
            special = rng.random(n)
            xs[special < 0.01] = np.nan
            xs[(special >= 0.01) & (special < 0.015)] = np.inf
            xs[(special >= 0.015) & (special < 0.02)] = -np.inf
            xs[(special >= 0.02) & (special < 0.05)] = np.floor(rng.normal(2e8, 2e7, size=int(((special >= 0.02) & (special < 0.05)).sum())))
            xs[(special >= 0.05) & (special < 0.06)] = 1e-300 * rng.random(int(((special >= 0.05) & (special < 0.06)).sum()))
            ts = 1.7e9 + 60.0 * np.arange(n) + 0.781
            pods.append(body([(float(t), go_format(float(x))) for t, x in zip(ts, xs)],
                             extra_series=int(rng.integers(0, 2))))
        per_obj.append(pods)
    return per_obj


@pytest.mark.parametrize("threads", [1, 4, 0])
def test_matches_reference_semantics(threads):
    per_obj = _fleet(1)
    ps, ts, counts = pack_query_range_bodies(per_obj, want_timestamps=True, threads=threads, return_pod_counts=True)
    v, o, c = ref_pack(per_obj)
    assert np.array_equal(ps.offsets, o)
    assert np.array_equal(ps.values.view(np.uint64), v.view(np.uint64))
    assert np.array_equal(counts, c)
    assert ps.max_len == int(np.diff(o).max())
    want_ts = []
    for bodies in per_obj:
        for b in bodies:
            r = json.loads(b)["data"]["result"]
            if r:
                want_ts.extend(t for t, _ in r[0]["values"])
    assert np.array_equal(ts, np.array(want_ts, dtype=np.float64))


def test_shortest_repr_round_trip():
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.gamma(2.0, 0.05, 3000), np.exp(rng.uniform(-700, 700, 3000)),
                         rng.integers(0, 2**53, 1000).astype(np.float64), [5e-324, 2.2250738585072014e-308,
                                                                            1.7976931348623157e308, 0.0, -0.0]])
    strs = [repr(float(x)) for x in xs] + [go_format(float(x)) for x in xs]
    b = body([(0.0, s) for s in strs])
    ps = pack_query_range_bodies([[b]])
    want = np.array([float(s) for s in strs])
    assert np.array_equal(ps.values.view(np.uint64), want.view(np.uint64))


def test_layout_variants():
    vals = [(1.0, "1.5"), (2.0, "2.5")]
    a = body(vals)
    # reordered keys, whitespace, escaped key names, leading data before status
    b = (b'  {"data" : {"result":[ {"\\u0076alues": [[1, "1.5"] ,[2,"2.5"]], "metric":{"a":[1,{"b":null}]}} ],'
         b' "resultType":"matrix"}, "status":"success", "warnings": ["x"]} \n')
    ps = pack_query_range_bodies([[a], [b], []])
    assert list(ps.offsets) == [0, 2, 4, 4]
    assert list(ps.values) == [1.5, 2.5, 1.5, 2.5]


@pytest.mark.parametrize("bad,code", [
    (b'{"status":"error","errorType":"bad_data","error":"x"}', -3),
    (b'{"status":"success","data":{"result":[{"values":[[1,"abc"]]}]}}', -4),
    (b'{"status":"success","data":{"result":[{"values":[[1,1.5]]}]}}', -2),
    (b'{"status":"success","data":{"result":[{"values":[[1,"1.5"]]}]}', -2),
    (b'{"status":"success","data":{"resultType":"matrix"}}', -2),
    (b'{"status":"success","data":{"result":[{"metric":{}}]}}', -2),
    (b'not json', -2),
    (b'{"status":"success","data":{"result":[{"values":[[1,"1.5"]]}]}} trailing', -2),
    (b'{"status":"success","data":{"result":[{"values":[[1,"1_5"]]}]}}', -4),
])
def test_errors_name_the_body(bad, code):
    good = body([(1.0, "1")])
    with pytest.raises(PrometheusResponseError) as e:
        pack_query_range_bodies([[good], [good, bad]])
    assert e.value.code == code
    assert "body 2" in str(e.value)


def test_empty_fleet():
    ps = pack_query_range_bodies([])
    assert ps.values.size == 0 and list(ps.offsets) == [0]
    ps = pack_query_range_bodies([[], []])
    assert list(ps.offsets) == [0, 0, 0]


def _decimal_strings(seed, n):
    """Value strings over many forms and their rounding edges: shortest reprs and
    fixed/scientific forms over many magnitudes, random digit strings with up to 25
    digits and exponents to +-40, leading/trailing zeros, and exact ties between
    adjacent doubles (integers 2^53 + odd, halfway decimals with many digits)."""
    rng = np.random.default_rng(seed)
    out = []
    mags = np.exp(rng.uniform(np.log(1e-35), np.log(1e35), n))
    for x in mags:
        x = float(x)
        out.append(repr(x))
        out.append(go_format(x))
        out.append("%.*f" % (int(rng.integers(0, 26)), x))
        out.append("%.*e" % (int(rng.integers(0, 22)), x))
    for _ in range(n):
        nd = int(rng.integers(1, 26))
        digits = "".join(str(d) for d in rng.integers(0, 10, nd))
        dot = int(rng.integers(0, nd + 1))
        s = digits[:dot] + "." + digits[dot:] if rng.random() < 0.7 else digits
        if s.startswith("."):
            s = "0" + s
        if s.endswith("."):
            s += "0"
        if rng.random() < 0.4:
            s += "e%d" % int(rng.integers(-40, 41))
        out.append(s)
    for k in range(1, 400, 2):  # ties: 2^53 + k sits halfway between two doubles
        out.append(str(2**53 + k))
        out.append(str((2**53 + k) * 2**6))
        out.append("%de-3" % (2**53 + k))
    for x in rng.uniform(0.1, 1e6, 200):  # exact decimal midpoints (many digits -> fallback)
        x = float(x)
        out.append(format((Decimal(x) + Decimal(np.nextafter(x, np.inf))) / 2, "f"))
    out += ["0", "0.0", "000.000", "0e5000", "1e-27", "1e27", "1e-28", "1e28", "9999999999999999999",
            "99999999999999999999", "0.1000000000000000000000", "123456789012345678.9", "4.9e-324",
            "2.2250738585072011e-308", "1.7976931348623157e308", "1e309", "1e-400", "0.000012345678901234567"]
    return out


def test_values_are_correctly_rounded():
    strs = _decimal_strings(11, 3000)
    signed = strs + ["-" + s for s in strs[::7]] + ["+" + s for s in strs[::11]]
    b = body([(0.0, s) for s in signed])
    ps = pack_query_range_bodies([[b]])
    want = np.array([float(s) for s in signed])
    bad = np.nonzero(ps.values.view(np.uint64) != want.view(np.uint64))[0]
    assert bad.size == 0, [signed[i] for i in bad[:10]]


def test_timestamps_are_correctly_rounded():
    import re

    json_num = re.compile(r"-?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?$")
    strs = [s for s in _decimal_strings(12, 500) if json_num.match(s)]
    strs += ["-" + s for s in strs[::5]]
    assert len(strs) > 2000
    samples = [(float(s), "1") for s in strs]  # JSON numbers: the timestamp path (Reader::num)
    raw = ",".join("[%s,\"1\"]" % s for s in strs)
    b = ('{"status":"success","data":{"resultType":"matrix","result":[{"metric":{},"values":[%s]}]}}' % raw).encode()
    ps, ts = pack_query_range_bodies([[b]], want_timestamps=True)
    want = np.array([t for t, _ in samples])
    assert np.array_equal(ts.view(np.uint64), want.view(np.uint64))


def test_near_midpoint_short_strings_are_correctly_rounded():
    """The packer's fast path (one x87 extended multiply/divide, krr_pack.cpp fast_decimal)
    must hand every string it cannot round safely to from_chars: 17-19 significant digits
    lying within a few units of the last digit of a halfway point between two doubles, over
    the magnitudes Prometheus values take (CPU cores, bytes), plus exact short midpoints."""
    rng = np.random.default_rng(21)
    strs = []
    xs = np.concatenate([rng.gamma(2.0, 0.05, 1500), np.exp(rng.uniform(np.log(1e-12), np.log(1e18), 1500))])
    for x in xs:
        x = float(x)
        mid = (Decimal(x) + Decimal(float(np.nextafter(x, np.inf)))) / 2
        for sig in (17, 18, 19):
            q = mid.scaleb(-mid.adjusted()).quantize(Decimal(1).scaleb(-(sig - 1)))  # sig digits
            for d in (-2, -1, 0, 1, 2):
                v = (q + d * Decimal(1).scaleb(-(sig - 1))).scaleb(mid.adjusted())
                strs.append(format(v, "f"))
    for k in range(1, 200, 2):  # short exact midpoints: (2^53 + k) / 2^s * 10^... as decimals
        for s in (1, 2, 3):
            strs.append(format(Decimal(2**53 + k) / Decimal(2**s), "f"))
    b = body([(0.0, s) for s in strs])
    ps = pack_query_range_bodies([[b]])
    want = np.array([float(s) for s in strs])
    bad = np.nonzero(ps.values.view(np.uint64) != want.view(np.uint64))[0]
    assert bad.size == 0, [strs[i] for i in bad[:10]]
