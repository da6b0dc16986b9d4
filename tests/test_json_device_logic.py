"""The device packer's parsing logic (krr_amd/csrc/krr_json_parse.h), compiled for the
host (tests/native/json_check.cpp) and checked on the CPU:

* numbers: Eisel-Lemire over the 128-bit powers-of-five table against Python's float()
  (correctly rounded) on shortest-repr strings of every magnitude, subnormals, huge
  integers in Prometheus' 'f' format, and random 1-19 digit significands near rounding
  midpoints;
* bodies: whatever the device logic accepts it parses to the host packer's bits
  (krr_pack_parse), and every body it does not accept is reported JSON_HOST — never an
  error of its own — so the host decides (whitespace, escapes, other spellings, errors).
The GPU kernel (wave-parallel values array) is checked against the host packer in
tests/test_gpu_json.py."""
import ctypes
import json
import math
import os
import subprocess

import numpy as np
import pytest

from krr_amd.core.prom_native import PrometheusResponseError, pack_query_range_bodies

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JSON_OK, JSON_DROPPED, JSON_HOST = 0, 1, 2


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("jc") / "libjsoncheck.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I" + os.path.join(ROOT, "krr_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "json_check.cpp"), "-o", out], check=True)
    L = ctypes.CDLL(out)
    vp = ctypes.c_void_p
    L.json_check_value.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_double)]
    L.json_check_body.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int, vp, vp, ctypes.c_int64,
                                  ctypes.POINTER(ctypes.c_int64)]
    return L


def go_format(x: float) -> str:
    from krr_amd.utils.prom_decimal import prom_format

    return prom_format(x)


def _value(lib, s: str):
    out = ctypes.c_double()
    rc = lib.json_check_value(s.encode(), len(s), ctypes.byref(out))
    return rc, out.value


def _bits(x: float) -> int:
    return int(np.float64(x).view(np.uint64))


def test_shortest_repr_values_of_every_magnitude(lib):
    rng = np.random.default_rng(7)
    xs = np.concatenate([
        rng.gamma(2.0, 0.05, 20000),
        np.floor(rng.normal(2e8, 2e7, 5000)),
        np.exp(rng.uniform(-744, 709, 20000)),                       # every exponent, subnormals included
        rng.integers(0, 2**63, 2000).astype(np.float64) * 2.0 ** rng.integers(0, 900, 2000),
        np.array([5e-324, 2.2250738585072014e-308, 2.2250738585072009e-308, 1.7976931348623157e308, 0.0, 1.0,
                  0.1, 0.2, 0.3, 1e22, 1e23, 9007199254740993.0, 123456789012345678.0]),
    ])
    xs = np.concatenate([xs, -xs[:3000]])
    bad = []
    for x in xs:
        s = go_format(float(x))
        rc, v = _value(lib, s)
        if rc != 0 or _bits(v) != _bits(float(s)):
            bad.append((s, rc, v))
    assert not bad, bad[:5]


def test_random_significands_near_midpoints(lib):
    """1-19 digit significands with exponents over the whole range, plus decimal strings
    built from exact binary midpoints (the halfway cases the round-to-even branch
    decides) — against float(), correctly rounded."""
    from decimal import Decimal

    rng = np.random.default_rng(11)
    cases = []
    for _ in range(40000):
        nd = int(rng.integers(1, 20))
        digits = str(int(rng.integers(1, 10))) + "".join(str(int(d)) for d in rng.integers(0, 10, nd - 1))
        e = int(rng.integers(-360, 320))
        cases.append(f"{digits}e{e}")
        cases.append(f"0.{digits}")
    for _ in range(6000):  # midpoints between adjacent doubles, written exactly when short enough
        x = float(np.exp(rng.uniform(-50, 50)))
        lo = Decimal(x)
        hi = Decimal(float(np.nextafter(x, np.inf)))
        mid = (lo + hi) / 2
        s = format(mid, "f")
        if len(s.replace(".", "").lstrip("0")) <= 19:
            cases.append(s)
    bad = []
    for s in cases:
        rc, v = _value(lib, s)
        if rc == 0 and _bits(v) != _bits(float(s)):
            bad.append((s, v, float(s)))
        if rc != 0 and len(s.replace(".", "").replace("-", "").lstrip("0").split("e")[0]) <= 19:
            bad.append((s, "host"))
    assert not bad, bad[:5]


@pytest.mark.parametrize("s,want", [("NaN", 0x7FF8000000000000), ("-NaN", 0xFFF8000000000000),
                                    ("+NaN", 0x7FF8000000000000), ("+Inf", 0x7FF0000000000000),
                                    ("-Inf", 0xFFF0000000000000), ("Inf", 0x7FF0000000000000),
                                    ("-0", 0x8000000000000000), ("0", 0), ("1e400", 0x7FF0000000000000),
                                    ("-1e-400", 0x8000000000000000)])
def test_special_spellings(lib, s, want):
    rc, v = _value(lib, s)
    assert rc == 0 and _bits(v) == want
    # and the host packer agrees bit for bit
    b = json.dumps({"status": "success", "data": {"result": [{"metric": {}, "values": [[1, s]]}]}}).encode()
    assert _bits(pack_query_range_bodies([[b]]).values[0]) == want


@pytest.mark.parametrize("s", ["nan", "inf", "Infinity", ".5", "5.", "1e", "1e+", "--1", "+-1", "1.2.3", "0x10",
                               "12345678901234567890123", "1" * 25 + ".5", "1e1234567", " 1", "1 ", ""])
def test_other_spellings_go_to_the_host(lib, s):
    rc, _ = _value(lib, s)
    assert rc != 0


def _compact(doc) -> bytes:
    return json.dumps(doc, separators=(",", ":"), ensure_ascii=False).encode()


def _bodies(seed, n=300):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = rng.random()
        if k < 0.1:
            res = []
        else:
            m = int(rng.integers(0, 300))
            xs = rng.gamma(2.0, 0.05, m)
            sp = rng.random(m)
            xs[sp < 0.02] = np.nan
            xs[(sp >= 0.02) & (sp < 0.03)] = np.inf
            xs[(sp >= 0.03) & (sp < 0.1)] = np.floor(rng.normal(2e8, 2e7, int(((sp >= 0.03) & (sp < 0.1)).sum())))
            ts = 1.7e9 + 15.0 * np.arange(m) + (0.5 if rng.random() < 0.5 else 0.0)
            vals = [[float(t) if t != int(t) else int(t), go_format(float(x))] for t, x in zip(ts, xs)]
            res = [{"metric": {"pod": f"p{i}", "namespace": "n"}, "values": vals}]
            if rng.random() < 0.2:  # further series: validated, never read
                res.append({"metric": {"pod": "other"}, "values": [[1, "3"], [2, "4"]]})
            if rng.random() < 0.2:  # keys in another order
                res[0] = {"values": vals, "metric": res[0]["metric"]}
        doc = {"status": "success", "data": {"resultType": "matrix", "result": res}}
        if rng.random() < 0.1:
            doc = {"data": doc["data"], "status": "success", "warnings": ["w"]}
        out.append(_compact(doc))
    return out


def _check_body(lib, b, want_ts=0):
    cap = len(b) // 8 + 1
    v = np.empty(cap)
    t = np.empty(cap)
    cnt = ctypes.c_int64()
    rc = lib.json_check_body(b, len(b), want_ts, v.ctypes.data, t.ctypes.data, cap, ctypes.byref(cnt))
    return rc, v[:cnt.value], t[:cnt.value]


def test_canonical_bodies_parse_like_the_host_packer(lib):
    bodies = _bodies(3)
    vals, ts, counts = pack_query_range_bodies([[b] for b in bodies], want_timestamps=True, return_pod_counts=True)
    offs = vals.offsets
    for i, b in enumerate(bodies):
        rc, v, t = _check_body(lib, b, want_ts=1)
        if counts[i] < 0:
            assert rc == JSON_DROPPED
            continue
        assert rc == JSON_OK, b[:200]
        want = vals.values[offs[i]:offs[i + 1]]
        assert np.array_equal(v.view(np.uint64), want.view(np.uint64))
        assert np.array_equal(t.view(np.uint64), ts[offs[i]:offs[i + 1]].view(np.uint64))


def test_whitespace_between_tokens_is_parsed_like_the_host(lib):
    """json.dumps' default separators (', ' and ': ') and newlines / tabs between the tokens of
    the values array and the envelope: the device logic accepts them, with the host's bits."""
    from krr_amd.core.prom_native import pack_query_range_bodies

    rng = np.random.default_rng(17)
    xs = rng.gamma(2.0, 0.05, 40)
    vals = [[1.7e9 + 15 * k, go_format(float(x))] for k, x in enumerate(xs)]
    doc = {"status": "success", "data": {"resultType": "matrix", "result": [{"metric": {"pod": "a"}, "values": vals}]}}
    for b in (json.dumps(doc).encode(), json.dumps(doc, indent=2).encode(),
              json.dumps(doc, indent="\t").encode().replace(b"],", b"] \r\n,")):
        rc, v, t = _check_body(lib, b, want_ts=1)
        assert rc == JSON_OK, b[:120]
        ps, ts = pack_query_range_bodies([[b]], want_timestamps=True)
        assert np.array_equal(v.view(np.uint64), ps.values.view(np.uint64))
        assert np.array_equal(t.view(np.uint64), ts.view(np.uint64))


@pytest.mark.parametrize("kind", ["space_in_value", "escaped_key", "escaped_value", "status_error", "no_status",
                                  "two_values", "bad_json", "trailing", "nan_lower", "no_result", "truncated",
                                  "dup_result"])
def test_non_canonical_bodies_go_to_the_host(lib, kind):
    base = {"status": "success", "data": {"resultType": "matrix",
                                          "result": [{"metric": {}, "values": [[1, "0.5"], [2, "1"]]}]}}
    b = {
        "space_in_value": _compact(base).replace(b'"0.5"', b'" 0.5"'),
        "escaped_key": _compact(base).replace(b'"status"', b'"st\\u0061tus"'),
        "escaped_value": _compact(base).replace(b'"0.5"', b'"0\\u002e5"'),
        "status_error": _compact(dict(base, status="error")),
        "no_status": _compact({"data": base["data"]}),
        "two_values": _compact(base).replace(b'"metric":{}', b'"values":[[0,"9"]]'),
        "bad_json": _compact(base).replace(b'"metric":{}', b'"metric":{,}'),
        "trailing": _compact(base) + b"x",
        "nan_lower": _compact(base).replace(b'"0.5"', b'"nan"'),
        "no_result": _compact({"status": "success", "data": {"resultType": "matrix"}}),
        "truncated": _compact(base)[:-3],
        "dup_result": _compact(base)[:-2] + b',"result":[]}}',
    }[kind]
    rc, _, _ = _check_body(lib, b)
    assert rc == JSON_HOST
    # the host packer's own verdict stands: either a result or its error
    try:
        pack_query_range_bodies([[b]])
    except PrometheusResponseError:
        pass


def _grouped(lib, b, label="pod", want_ts=1):
    cap = len(b) // 8 + 1
    ms = len(b) // 20 + 2
    lo = np.empty(ms, np.int64)
    ll = np.empty(ms, np.int64)
    cn = np.empty(ms, np.int64)
    v = np.empty(cap)
    t = np.empty(cap)
    ns = ctypes.c_int64()
    lib.json_check_grouped.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int] + \
        [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                 ctypes.POINTER(ctypes.c_int64)]
    rc = lib.json_check_grouped(b, len(b), label.encode(), want_ts, lo.ctypes.data, ll.ctypes.data, cn.ctypes.data,
                                ms, v.ctypes.data, t.ctypes.data, cap, ctypes.byref(ns))
    n = ns.value
    return rc, [(None if lo[i] < 0 else b[lo[i]:lo[i] + ll[i]].decode(), int(cn[i])) for i in range(n)], v, t


def test_grouped_bodies_walk_like_the_host_packer(lib):
    """Every series of grouped (`sum by (pod)`) bodies, in order, with its pod label and
    values — against the host packer's parse_series (krr_pack_parse_series)."""
    from krr_amd.core.prom_native import parse_series

    rng = np.random.default_rng(9)
    for i in range(60):
        res = []
        for j in range(int(rng.integers(0, 6))):
            m = int(rng.integers(0, 50))
            xs = rng.gamma(2.0, 0.05, m)
            metric = {"pod": f"p{i}-{j % 3}", "namespace": "n"} if rng.random() < 0.85 else {"namespace": "n"}
            if rng.random() < 0.2:
                metric = {"zz": {"nested": [1, 2, {"a": None}]}, **metric}
            ser = {"metric": metric, "values": [[1.7e9 + 15 * k, go_format(float(x))] for k, x in enumerate(xs)]}
            if rng.random() < 0.2:
                ser = {"values": ser["values"], "metric": metric, "extra": True}
            res.append(ser)
        doc = {"status": "success", "data": {"resultType": "matrix", "result": res}}
        b = _compact(doc)
        rc, got, v, t = _grouped(lib, b)
        assert rc == JSON_OK, b[:300]
        want = parse_series(b, "pod", want_timestamps=True)
        assert [(g[0], g[1]) for g in got] == [(w[0], len(w[1])) for w in want]
        flat_v = np.concatenate([w[1] for w in want]) if want else np.zeros(0)
        flat_t = np.concatenate([w[2] for w in want]) if want else np.zeros(0)
        k = flat_v.size
        assert np.array_equal(v[:k].view(np.uint64), flat_v.view(np.uint64))
        assert np.array_equal(t[:k].view(np.uint64), flat_t.view(np.uint64))


@pytest.mark.parametrize("kind", ["escaped_label", "dup_metric", "dup_values", "no_values", "value_space", "status",
                                  "escaped_label_key", "empty_series"])
def test_grouped_non_canonical_go_to_the_host(lib, kind):
    base = {"status": "success", "data": {"resultType": "matrix", "result": [
        {"metric": {"pod": "a"}, "values": [[1, "1"]]}, {"metric": {"pod": "b"}, "values": [[1, "2"]]}]}}
    b = _compact(base)
    b = {
        "escaped_label": b.replace(b'"pod":"a"', b'"pod":"\\u0061"'),
        "dup_metric": b.replace(b'{"metric":{"pod":"a"},', b'{"metric":{"pod":"a"},"metric":{},'),
        "dup_values": b.replace(b'"values":[[1,"1"]]}', b'"values":[[1,"1"]],"values":[]}'),
        "no_values": b.replace(b',"values":[[1,"1"]]', b''),
        "value_space": b.replace(b'"2"', b'"2 "'),
        "status": b.replace(b'"success"', b'"error"'),
        "escaped_label_key": b.replace(b'{"pod":"a"}', b'{"p\\u006fd":"a"}'),
        "empty_series": b.replace(b'{"metric":{"pod":"a"},"values":[[1,"1"]]}', b'{}'),
    }[kind]
    rc, _, _, _ = _grouped(lib, b)
    assert rc == JSON_HOST
