"""The device packer's stripped staging (krr_amd/csrc/krr_strip.h, krr_pack_concat_strip):
every number outside strings cut to its first digit while the bodies are staged, so fewer
bytes cross PCIe.  The reference drops the timestamps (robusta_krr/core/integrations/
prometheus.py:152); what must hold is that the host packer (the parity restatement of that
loader) reads a stripped body exactly as the original: same values, same pod drops, or the
same error.  CPU only: the device parser's side is tests/test_gpu_json.py."""
import ctypes
import random
import re

import numpy as np
import pytest

from krr_amd.core import prom_native
from krr_amd.core.prom_native import PrometheusResponseError, pack_query_range_bodies, strip_body

HEAD = '{"status":"success","data":{"resultType":"matrix","result":['
_NUM = re.compile(rb"[0-9.]+")
_OK_RUN = re.compile(rb"(0|[1-9][0-9]*)(\.[0-9]+)?")


def _restated(body: bytes):
    """The strip restated in Python: None unless every run of digits / '.' outside strings
    is a whole number token (0|[1-9][0-9]*)(\\.[0-9]+)? (no e E + - ) / before it, no e E
    after it) and no backslash occurs; else each run cut to one byte."""
    if b"\\" in body:
        return None
    parts = body.split(b'"')
    for i in range(0, len(parts), 2):  # outside strings
        part = parts[i]
        for m in _NUM.finditer(part):
            if not _OK_RUN.fullmatch(m.group()):
                return None
            if m.start() > 0 and part[m.start() - 1:m.start()] in (b"e", b"E", b"+", b"-", b")", b"/"):
                return None                      # a sign or exponent before the run
            if part[m.end():m.end() + 1] in (b"e", b"E"):
                return None                      # an exponent after it
        parts[i] = _NUM.sub(lambda m: m.group()[:1], parts[i])
    return b'"'.join(parts)


def _body(values, ts=None, pod="p", extra=""):
    ts = ts if ts is not None else [f"{1.7e9 + 15 * i!r}" for i in range(len(values))]
    items = ",".join(f'[{t},"{v}"]' for t, v in zip(ts, values))
    return (HEAD + f'{{"metric":{{"pod":"{pod}"}},"values":[{items}]{extra}}}]}}}}').encode()


def _packed(bodies):
    try:
        ps, counts = pack_query_range_bodies([[b] for b in bodies], threads=2, return_pod_counts=True)
    except PrometheusResponseError as e:
        return ("error", e.code)
    return (np.asarray(ps.values).view(np.int64).tolist(), np.asarray(ps.offsets).tolist(),
            np.asarray(counts).tolist())


def _same_outcome(orig: bytes, stripped: bytes):
    return _packed([orig]) == _packed([stripped])


def test_bench_shaped_bodies_strip_to_a_third_less():
    rng = np.random.default_rng(1)
    for vals in ([repr(x) for x in rng.gamma(2.0, 0.05, 3000).tolist()],
                 [repr(x) for x in np.floor(rng.normal(2e8, 2e7, 3000)).tolist()]):
        b = _body(vals)
        s = strip_body(b)
        assert s is not None and s == _restated(b)
        assert len(s) < 0.72 * len(b)
        assert b'[1,"' in s and b"1700000" not in s
        assert _same_outcome(b, s)


TIMESTAMPS = ["1700000000", "1700000000.5", "1700000000.123", "0", "0.5", "7"]
NOT_STRIPPED = ["01700000000", "1700000000.", ".5", "1.2.3", "1e9", "1.7E9", "-5", "1700000000.5.5"]


@pytest.mark.parametrize("t", TIMESTAMPS + NOT_STRIPPED)
def test_timestamp_forms(t):
    b = _body(["0.25", "1", "NaN"], ts=[t, t, t])
    s = strip_body(b)
    assert s == _restated(b)
    if t in NOT_STRIPPED:
        assert s is None
    if s is not None:
        assert _same_outcome(b, s)


@pytest.mark.parametrize("body", [
    _body(["0.1"] * 5, pod='p\\"q'),                                   # a backslash: not stripped
    _body(["0.1", "0.2"]).replace(b",", b" , "),                        # whitespace between tokens
    (HEAD + "]}}").encode(),                                            # an empty result: dropped pod
    b'{"status":"error","errorType":"bad_data","error":"x 12.5"}',     # an error body
    _body(["0.1", "2"], extra=',"x":[1.25,2.5e3]'),                     # other numbers in result[0]
    _body(["0.1", "0.2"]).replace(b'"0.2"', b"0.2"),                    # an unquoted value
    _body(["1.5", "2"], pod="pod-123.45"),                              # digits inside strings stay
    _body([]),
])
def test_odd_bodies_keep_their_outcome(body):
    s = strip_body(body)
    assert s == _restated(body)
    if s is not None:
        assert _same_outcome(body, s)


def test_fuzzed_bodies_keep_their_outcome():
    """Byte mutations of a small body: whenever it strips, the host packer's outcome on the
    stripped body (values, drops, or error code) is the original's."""
    rng = random.Random(7)
    base = _body(["0.25", "1e-3", "NaN", "+Inf", "12"], ts=["1700000000", "1700000015.5", "0", "3", "99.25"])
    alphabet = b'0123456789.,[]{}"-+eE :\\ a'
    stripped = 0
    for _ in range(20000):
        b = bytearray(base)
        for _ in range(rng.randint(1, 3)):
            i = rng.randrange(len(b))
            op = rng.random()
            if op < 0.4:
                b[i] = rng.choice(alphabet)
            elif op < 0.7:
                b.insert(i, rng.choice(alphabet))
            else:
                del b[i]
        b = bytes(b)
        s = strip_body(b)
        assert s == _restated(b), b
        if s is not None:
            stripped += 1
            assert _same_outcome(b, s), b
    assert stripped > 5000


def test_block_boundaries():
    """Runs and strings crossing the 64-byte blocks, at every alignment."""
    for pad in range(0, 70):
        b = _body(["0.5", "17", "3.25"], ts=["1700000000.125", "1700000015", "1700000030.5"], pod="x" * pad)
        s = strip_body(b)
        assert s == _restated(b)
        assert _same_outcome(b, s)
        bad = _body(["0.5"], ts=["1700000000.1.5"], pod="x" * pad)
        assert strip_body(bad) is None
        bad = _body(["0.5"], ts=["1700000000."], pod="x" * pad)
        assert strip_body(bad) is None


def test_concat_strip_runs_lay_out_the_stripped_bodies():
    lib = prom_native.load_library()
    rng = np.random.default_rng(3)
    bodies = []
    for k in range(37):
        n = int(rng.integers(0, 400))
        b = _body([repr(x) for x in rng.gamma(2.0, 0.05, n).tolist()])
        if k % 9 == 4:
            b = b.replace(b'"metric":{', b'"metric":{"a":"\\"",')   # not strippable
        bodies.append(b)
    lens = np.array([len(b) for b in bodies], dtype=np.int64)
    offs = np.zeros(len(bodies) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    dst = ctypes.create_string_buffer(int(offs[-1]) + 64)
    new_lens = np.zeros(len(bodies), dtype=np.int64)
    for max_runs in (1, 3, 8, 64):
        runs = np.zeros(max_runs + 1, dtype=np.int64)
        nr = ctypes.c_int32()
        ptrs = (ctypes.c_char_p * len(bodies))(*bodies)
        rc = lib.krr_pack_concat_strip(ctypes.addressof(ptrs), lens.ctypes.data, len(bodies), offs.ctypes.data,
                                       ctypes.addressof(dst), 4, max_runs, new_lens.ctypes.data, runs.ctypes.data,
                                       ctypes.byref(nr))
        assert rc == 0 and 1 <= nr.value <= max_runs and runs[0] == 0 and runs[nr.value] == len(bodies)
        raw = dst.raw
        for r in range(nr.value):
            pos = int(offs[runs[r]])
            for i in range(int(runs[r]), int(runs[r + 1])):
                want = strip_body(bodies[i]) if bodies[i] else b""
                want = bodies[i] if want is None else want
                assert new_lens[i] == len(want)
                assert raw[pos:pos + len(want)] == want
                pos += len(want)
            assert pos <= offs[runs[r + 1]]


def test_body_table_matches_the_python_walk():
    """krr_pydec.cpp body_table (the device packer's flat table in one native pass) against the
    Python walk it replaces; None when a body is not bytes (the Python path converts those)."""
    from krr_amd.core.device_pack import _body_table
    from krr_amd.core.packing import _PYDEC

    if _PYDEC is None:
        pytest.skip("_krr_pydec.so not built")
    res = [[[b"ab", b"c"], [], [b"defg"]], [[b"", b"hi"], [b"j"], []]]
    ptrs, lens, obj, ob = _body_table(res)
    flat = [(b, r * 3 + o) for r, objs in enumerate(res) for o, bodies in enumerate(objs) for b in bodies]
    assert lens.tolist() == [len(b) for b, _ in flat]
    assert obj.tolist() == [o for _, o in flat]
    assert ob.tolist() == [sum(map(len, bodies)) for objs in res for bodies in objs]
    assert [ctypes.string_at(int(p), int(n)) for p, n in zip(ptrs, lens)] == [b for b, _ in flat]
    assert _body_table([[[b"x", bytearray(b"y")]]]) is None
    assert _body_table([]) is not None and len(_body_table([])[0]) == 0


# ---- pieces: one large body stripped by several threads (grouped bodies) ----------------------

@pytest.fixture
def lib():
    return prom_native.load_library()


def _grouped(rng, n_series, n_samples, pods=None, tricky=False):
    """A `sum by (pod)` body: n_series series of n_samples each (label values may hold `"],[`-like
    bytes, which must not be taken for a cut)."""
    parts = []
    for i in range(n_series):
        pod = pods[i] if pods else f"pod-{i}"
        if tricky and i % 3 == 0:
            pod = f'x],[1,"{i}'  # no backslash: still strippable
        ts = [f"{1.7e9 + 60 * j!r}" for j in range(n_samples)]
        vals = [repr(float(v)) for v in rng.gamma(2.0, 0.05, n_samples)]
        items = ",".join(f'[{t},"{v}"]' for t, v in zip(ts, vals))
        parts.append(f'{{"metric":{{"pod":"{pod}"}},"values":[{items}]}}')
    return (HEAD + ",".join(parts) + "]}}").encode()


def _strip_pieces(lib, bodies, max_pieces, threads=4):
    lens = np.array([len(b) for b in bodies], dtype=np.int64)
    offs = np.zeros(len(bodies) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    dst = ctypes.create_string_buffer(int(offs[-1]) + 64)
    new_lens = np.zeros(len(bodies), dtype=np.int64)
    cap = 2 * len(bodies) + max_pieces
    start = np.zeros(cap + 1, dtype=np.int64)
    out = np.zeros(cap, dtype=np.int64)
    n = ctypes.c_int32()
    ptrs = (ctypes.c_char_p * len(bodies))(*bodies)
    rc = lib.krr_pack_concat_strip_pieces(ctypes.addressof(ptrs), lens.ctypes.data, len(bodies), offs.ctypes.data,
                                          ctypes.addressof(dst), threads, max_pieces, new_lens.ctypes.data,
                                          start.ctypes.data, out.ctypes.data, ctypes.byref(n))
    assert rc == 0
    k = n.value
    return dst.raw, offs, new_lens, start[:k + 1].copy(), out[:k].copy()


def _whole(bodies):
    w = [strip_body(b) if b else b"" for b in bodies]
    return [b if s is None else s for b, s in zip(bodies, w)]


@pytest.mark.parametrize("max_pieces", [1, 2, 5, 16, 64])
def test_strip_pieces_equal_the_whole_body_copy(lib, max_pieces):
    """krr_pack_concat_strip_pieces: large bodies cut at `"],[` inside values arrays and stripped
    apart give, concatenated, exactly the whole-body stripped copy (or the original for a body
    with an unstrippable part); small bodies go in runs."""
    rng = np.random.default_rng(5)
    bodies = [_grouped(rng, 30, 400), _body(["0.1", "0.2"]), _grouped(rng, 8, 900, tricky=True),
              _grouped(rng, 40, 50), b"", _body(["1", "2"], ts=["1e9", "2"]),  # unstrippable: exponent
              _grouped(rng, 20, 300).replace(b'"pod-3"', b'"po\\\\d"'),       # a backslash: unchanged
              _grouped(rng, 1, 5000)]
    raw, offs, new_lens, start, out = _strip_pieces(lib, bodies, max_pieces)
    want = _whole(bodies)
    assert new_lens.tolist() == [len(w) for w in want]
    got = b"".join(raw[int(s - offs[0]):int(s - offs[0] + o)] for s, o in zip(start[:-1], out))
    assert got == b"".join(want)
    assert (np.diff(start) >= out).all() and start[-1] == offs[-1]
    if max_pieces >= 16:
        assert out.size > len(bodies)  # the large bodies were cut


def _segments(stripped: bytes, body_offs):
    """The device's series segments of a stripped concatenation (this generator's bodies only):
    start, end (one past '}'), label offset / length, scratch slot, count, ok."""
    segs = []
    for m in re.finditer(rb'[\[,](\{"metric":\{"pod":")', stripped):
        st = m.start(1)
        lab = m.end(1)
        lab_end = stripped.index(b'"}', lab)
        end = stripped.index(b"]}", stripped.index(b'"values":[', lab_end)) + 2
        cnt = stripped.count(b"],[", st, end) + 1
        segs.append([st, end, lab, lab_end - lab, st // 8, cnt, 1])
    return np.array(segs, dtype=np.int64).reshape(-1, 7)


@pytest.mark.parametrize("max_pieces", [1, 7, 32])
def test_route_over_pieces_equals_contiguous(lib, max_pieces):
    """krr_pack_route_grouped_pieces over the piecewise staged copy routes every slot as
    krr_pack_route_grouped does over the contiguous stripped bodies."""
    rng = np.random.default_rng(9)
    pods = [[f"pod-{b}-{i}" for i in range(n)] for b, n in enumerate((25, 6, 40))]
    bodies = [_grouped(rng, len(p), m, pods=p) for p, m in zip(pods, (300, 2000, 120))]
    raw, offs, new_lens, start, out = _strip_pieces(lib, bodies, max_pieces)
    dev_offs = np.zeros(len(bodies) + 1, dtype=np.int64)
    np.cumsum(new_lens, out=dev_offs[1:])
    contiguous = b"".join(raw[int(s - offs[0]):int(s - offs[0] + o)] for s, o in zip(start[:-1], out))
    segs = np.ascontiguousarray(_segments(contiguous, dev_offs))
    piece_dev = np.concatenate([[0], np.cumsum(out)[:-1]]).astype(np.int64)
    piece_shift = (start[:-1] - offs[0] - piece_dev).astype(np.int64)
    names = [n.encode() for p in pods for n in p] + [b"absent"]
    slot_body = np.array([b for b, p in enumerate(pods) for _ in p] + [1], dtype=np.int64)
    name_offs = np.concatenate([[0], np.cumsum([len(n) for n in names])]).astype(np.int64)
    blob = b"".join(names)
    res = []
    for pieces in (False, True):
        src, cnt = np.zeros(len(names), np.int64), np.zeros(len(names), np.int64)
        ok = np.zeros(len(bodies), np.int32)
        if pieces:
            buf = ctypes.create_string_buffer(raw, len(raw) + 128)
            rc = lib.krr_pack_route_grouped_pieces(ctypes.addressof(buf), dev_offs.ctypes.data, len(bodies),
                                                   piece_dev.ctypes.data, piece_shift.ctypes.data, len(out), b"pod",
                                                   segs.ctypes.data, len(segs), slot_body.ctypes.data, blob,
                                                   name_offs.ctypes.data, len(names), src.ctypes.data,
                                                   cnt.ctypes.data, ok.ctypes.data, 2)
        else:
            buf = ctypes.create_string_buffer(contiguous, len(contiguous) + 128)
            rc = lib.krr_pack_route_grouped(ctypes.addressof(buf), dev_offs.ctypes.data, len(bodies), b"pod",
                                            segs.ctypes.data, len(segs), slot_body.ctypes.data, blob,
                                            name_offs.ctypes.data, len(names), src.ctypes.data, cnt.ctypes.data,
                                            ok.ctypes.data, 2)
        assert rc == 0 and ok.all(), (pieces, ok)
        res.append((src.tolist(), cnt.tolist()))
    assert res[0] == res[1]
    assert res[0][1][:-1] == [m for p, m in zip(pods, (300, 2000, 120)) for _ in p] and res[0][1][-1] == -1
