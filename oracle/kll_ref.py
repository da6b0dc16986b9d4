"""CPU restatement of the KLL-style compactor sketch (krr_amd/csrc/krr_kll.h).

Test infrastructure only: imported by tests/ (and bench.py's checks after the timed
region), never by the product; the GPU rows and answers are compared with it bit for bit.

The sketch is a build-only extension (north_star: "an optional mergeable t-digest/KLL
sketch mode"); the reference has no sketch, so there is nothing of the reference to
restate here: this module pins the kernel to its own specification (the same blocks,
the same compaction coins, the same merge/carry order, the same query rule), and the
tests check the specification's rank-error bound against exact ranks.
"""
from __future__ import annotations

import math

import numpy as np

MASK = (1 << 64) - 1
SIGN = np.uint64(1 << 63)
HDR = 10
RUN = 256
LEVELS = 16
CH_UNITS = 512  # double2 units per streaming chunk (kUnroll x 64 lanes)


def mix(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def coin(seed: int, series: int, slc: int, level: int, cnt: int) -> int:
    x = (seed + 0x9E3779B97F4A7C15 * (series + 1) + 0xD1B54A32D192ED03 * (slc + 1)
         + 0x8CB92BA72F3D8DD7 * ((level << 32) | cnt)) & MASK
    return mix(x) >> 63


def okey(v: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(v, dtype=np.float64).view(np.uint64)
    return np.where((u & SIGN) != 0, ~u, u | SIGN)


def okey_inv(k: np.ndarray) -> np.ndarray:
    k = np.asarray(k, dtype=np.uint64)
    return np.where((k & SIGN) != 0, k ^ SIGN, ~k).view(np.float64)


def chunks(vals: np.ndarray, beg: int, end: int):
    """The 1,024-slot chunks the kernel's streaming skeleton delivers for [beg, end)
    (stream_segment: 16-byte aligned body, NaN padding, head/tail in slots 1022/1023)."""
    a0 = min((beg + 1) & ~1, end)
    a1 = max(end & ~1, a0)
    nunits = (a1 - a0) >> 1
    nfull, rem = divmod(nunits, CH_UNITS)
    head, tail = a0 > beg, a1 < end
    nch = nfull + (1 if (rem or head or tail) else 0)
    for ci in range(nch):
        s = np.full(1024, np.nan)
        if ci < nfull:
            s[:] = vals[a0 + 1024 * ci: a0 + 1024 * (ci + 1)]
        else:
            s[: 2 * rem] = vals[a0 + 1024 * nfull: a0 + 1024 * nfull + 2 * rem]
            if head:
                s[1022] = vals[beg]
            if tail:
                s[1023] = vals[a1]
        yield s


_POS = np.arange(1024)
_BLOCK1 = (_POS % 128) >= 64  # slot u*128 + 2*lane + h belongs to block lane >> 5
_LANE_SLOTS = [np.array([u * 128 + 2 * lane + h for u in range(8) for h in range(2)]) for lane in range(64)]
FIRST = 3  # first wave-level run level (kKllFirst)
LANE0, LANE1 = 32, 96  # coin "levels" of lane l's compactions (kKllLane0 / kKllLane1)


def build_row(vals: np.ndarray, beg: int, end: int, *, budget: int = 512, seed: int = 0, series: int = 0,
              slc: int = 0, gaps: bool = False) -> np.ndarray:
    """The exported row (uint64 [HDR + budget]; unused key words 0) of segment [beg, end).
    Keys are ordered by okey() here and stored as f64 bits; -0 is folded into +0."""
    vals = np.where(vals == 0.0, 0.0, vals)  # -0 -> +0 (the sketch keeps no zero sign)
    chs = list(chunks(vals, beg, end))
    whole = len(chs) <= 1
    runs = {}  # level -> sorted uint64 keys
    cnt = [0] * LEVELS
    sum_w2 = 0
    n_pres = n_nan = 0
    kmin, kmax = None, None
    row = np.zeros(HDR + budget, dtype=np.uint64)

    def push(t: np.ndarray, h: int):
        nonlocal sum_w2
        while t.size:  # an empty run changes nothing
            assert h < LEVELS, "run level overflow"
            if h not in runs:
                runs[h] = t
                return
            a = runs.pop(h)
            off = coin(seed, series, slc, h, cnt[h])
            cnt[h] += 1
            t = np.sort(np.concatenate([a, t]))[off::2]
            sum_w2 += 4 ** h
            h += 1

    def wave_stage(lane_runs):
        """Level 2: every lane's weight-4 keys sorted together, compacted, pushed to level 3."""
        nonlocal sum_w2
        allk = np.sort(np.concatenate(lane_runs))
        if not allk.size:
            return
        off = coin(seed, series, slc, 2, cnt[2])
        cnt[2] += 1
        sum_w2 += 16
        push(allk[off::2], FIRST)

    exact0 = None
    pend = None
    for ci, s in enumerate(chs):
        nan = np.isnan(s)
        k = okey(s[~nan])
        n_pres += k.size
        if k.size:
            kmin = k.min() if kmin is None else min(kmin, k.min())
            kmax = k.max() if kmax is None else max(kmax, k.max())
        if whole and k.size <= budget:
            exact0 = np.concatenate([np.sort(okey(s[(~_BLOCK1) & ~nan])), np.sort(okey(s[_BLOCK1 & ~nan]))])
            continue
        runs0 = []
        for lane in range(64):  # level 0, per lane: its 16 slots sorted, every other kept
            kl = np.sort(okey(s[_LANE_SLOTS[lane]][~np.isnan(s[_LANE_SLOTS[lane]])]))
            off = coin(seed, series, slc, LANE0 + lane, ci)
            sum_w2 += 1 if kl.size else 0
            runs0.append(kl[off::2])
        if pend is None:
            pend = runs0
            continue
        runs1 = []
        for lane in range(64):  # level 1, per lane: merged with the pending run, compacted
            z = np.sort(np.concatenate([pend[lane], runs0[lane]]))
            off = coin(seed, series, slc, LANE1 + lane, ci >> 1)
            sum_w2 += 4 if z.size else 0
            runs1.append(z[off::2])
        pend = None
        wave_stage(runs1)
    if pend is not None:  # an odd last chunk: its level-1 run compacted alone
        runs1 = []
        for lane in range(64):
            off = coin(seed, series, slc, LANE1 + lane, len(chs) >> 1)
            sum_w2 += 4 if pend[lane].size else 0
            runs1.append(pend[lane][off::2])
        wave_stage(runs1)
    n_nan = int(np.isnan(vals[beg:end]).sum())  # real NaN samples (the chunks' padding excluded)
    if exact0 is None:
        while True:
            total = sum(r.size for r in runs.values())
            nonempty = [h for h, r in runs.items() if r.size]
            if total <= budget or not nonempty:
                break
            low = min(nonempty)
            a = runs.pop(low)
            off = coin(seed, series, slc, low, cnt[low])
            cnt[low] += 1
            sum_w2 += 4 ** low
            push(a[off::2], low + 1)
        lens = {h: r.size for h, r in runs.items() if r.size}
        keys = np.concatenate([runs[h] for h in sorted(lens)]) if lens else np.zeros(0, np.uint64)
    else:
        lens = {0: exact0.size} if exact0.size else {}
        keys = exact0
    row[HDR: HDR + keys.size] = okey_inv(keys).view(np.uint64) if keys.size else keys
    row[0] = n_pres
    row[1] = 0 if gaps else n_nan
    nanbits = np.uint64(0x7FF8000000000000)
    row[2] = okey_inv(np.uint64(kmin)).view(np.uint64) if n_pres else nanbits
    row[3] = okey_inv(np.uint64(kmax)).view(np.uint64) if n_pres else nanbits
    for h, ln in lens.items():
        row[4 + (h >> 2)] |= np.uint64(ln << (16 * (h & 3)))
    row[8] = sum_w2
    row[9] = sum(ln << h for h, ln in lens.items())
    return row


def row_keys(row: np.ndarray):
    """(okeys, level per key) of a row."""
    keys, lvl, pos = [], [], 0
    for h in range(LEVELS):
        ln = int((int(row[4 + (h >> 2)]) >> (16 * (h & 3))) & 0xFFFF)
        keys.append(okey(row[HDR + pos: HDR + pos + ln].view(np.float64)))
        lvl.append(np.full(ln, h))
        pos += ln
    return np.concatenate(keys), np.concatenate(lvl)


def np_lerp(a: float, b: float, t: float) -> float:
    d = b - a
    return b - d * (1.0 - t) if t >= 0.5 else a + d * t


def exact_rank(n: int, p_num: int, p_den: int) -> int:
    return ((n - 1) * p_num) // (100 * p_den)


def query(rows: np.ndarray, mode: int, p_num: int, p_den: int, q: float):
    """(value, count, flags) of one series from its rows (uint64 [W, HDR + budget])."""
    n = int(rows[:, 0].sum())
    nan = int(rows[:, 1].sum())
    mins = rows[:, 2].view(np.float64)
    maxs = rows[:, 3].view(np.float64)
    if nan:
        return math.nan, n, 1
    if n == 0:
        return math.nan, 0, 4
    mn, mx = float(np.nanmin(mins)), float(np.nanmax(maxs))
    wtot = int(rows[:, 9].sum())
    ks, ls = zip(*(row_keys(r) for r in rows))
    keys, lvl = np.concatenate(ks), np.concatenate(ls)
    order = np.argsort(keys, kind="stable")
    keys, w = keys[order], (np.uint64(1) << lvl[order].astype(np.uint64)).astype(object)
    cum = np.cumsum(w)

    def select(r: int) -> float:
        if r == 0:
            return mn
        if r == n - 1:
            return mx
        if wtot == 0:  # every kept key compacted away: only the exact min / max remain
            return mn if 2 * r < n else mx
        i = next(i for i, c in enumerate(cum) if c * n > r * wtot)
        return float(okey_inv(keys[i]))

    if mode == 1:  # SORTED_LOWER
        return select(exact_rank(n, p_num, p_den)), n, 0
    vidx = float(n - 1) * q
    if vidx >= n - 1:
        r0 = r1 = n - 1
        gamma = vidx + 1.0
    else:
        fl = math.floor(vidx)
        r0, r1, gamma = int(fl), int(fl) + 1, vidx - fl
    v0 = select(r0)
    v1 = v0 if r1 == r0 else select(r1)
    return np_lerp(v0, v1, gamma), n, 0


def rank_bound(rows: np.ndarray, delta: float = 0.01) -> float:
    """Normalised rank-error bound of one series' rows (krr_amd.core.sketch.kll_rank_bound)."""
    n = float(rows[:, 0].sum())
    w2 = float(sum(int(x) for x in rows[:, 8]))
    top = max((h for r in rows for h in range(LEVELS) if (int(r[4 + (h >> 2)]) >> (16 * (h & 3))) & 0xFFFF),
              default=0)
    return (2.0 * math.sqrt(2.0 * math.log(6.0 / delta) * w2) + 2.0 ** top) / n
