"""CPU restatement of the KLL sketch, format 2 (krr_amd/csrc/krr_kll.h).

Test infrastructure only: imported by tests/ (and bench.py's checks after the timed
region), never by the product; the GPU rows and answers are compared with it bit for bit.

The sketch is a build-only extension (north_star: "an optional mergeable t-digest/KLL
sketch mode"); the reference has no sketch, so there is nothing of the reference to restate
here: this module IS the specification the kernels follow (the same pairings, coins, level
steps, set-asides, final compression, fold and query rule), and the tests check its
rank-error bound against exact ranks.

A row (uint64 words) describes one series slice, or several slices folded together:
  [0] present samples   [1] NaN samples (compact layout; 0 with gaps)
  [2] min  [3] max      (f64 bits of the present keys, NaN bits when empty)
  [4] sum of w^2 over every compaction that made the row (the rank bound's variance term)
  [5] body weight = sum over kept body keys of 2^level (always == [0]: no compaction loses weight)
  [6] tail length tl = min([0], tail cap)
  [7] budget << 32 | tail cap   (rows fold only with rows of the same format)
  [8..13] body level lengths, u16 x 24 (level h at word 8 + h // 4, bits 16 (h % 4))
  [14], [15] 0
  [16, 16 + budget)                 body keys, level 0 first, each level ascending
  [16 + budget, 16 + budget + cap)  tail: the tl largest present keys, ascending (exact)
Keys are the sample values with -0 folded into +0 (the sketch keeps no zero sign); equal
values therefore have equal bits, so ties never need an order.

Body (a KLL compactor hierarchy with a DETERMINISTIC schedule).  A compaction takes an EVEN
number of equal-weight keys, sorts them and keeps every other one from a coin-chosen offset,
doubling their weight; an odd key is SET ASIDE at its level first.  So how many keys sit at
each level after every step depends only on the presence pattern of the input, never on the
coins or the values, and sum w^2 is fixed before any coin is tossed.  The stream of a slice
is cut in 1,024-slot chunks (the kernels' streaming layout: lane l holds slots u*128 + 2l + h,
u < 8, h < 2); per lane:
  level 0  every chunk: each slot pair (u*128 + 2l, +1) with both samples present is one
           compaction (coin bit u); a lone present sample is set aside at level 0;
  level 1  odd chunks: the lane's pending 8 weight-2 keys and the new ones, sorted, compacted;
  level 2  every 4th chunk, level 3 every 8th: two runs of <= 8 keys merged and compacted;
  level 4  every 8th chunk, the wave: all 64 lanes' weight-16 keys sorted and compacted into a
           run of <= 256 weight-32 keys, pushed to level 5;
  h >= 5   one run of <= 256 keys per level: a run pushed onto an occupied level is merged
           with it and compacted (the odd largest key set aside), carrying up — a binary counter.
A set-aside key waits in its level's single ODD SLOT (per lane below level 4, per wave from
level 4 on); a second one arriving there makes a two-key compaction whose kept key goes to the
next level's slot.  The last chunks are flushed by all-absent chunks up to a multiple of 8;
then, from level 0 up, while more than `budget` keys remain, a level with >= 2 keys is
compacted once (odd largest set aside) and its output joins the next level.

Tail: the min(n, cap) largest present keys, exactly.  A rank r with n - r <= tl is answered
from it exactly; other ranks from the body: the smallest kept key whose weighted count of
keys <= it exceeds r (rank 0: the exact min).

Fold (merge) of two rows: present/NaN counts add, min/max combine, tails keep the cap largest
of their union (exact: each slice kept its own cap largest), body levels are unioned and then
compacted from level 0 up exactly as the build's final step, coins keyed by the fold index.
"""
from __future__ import annotations

import math

import numpy as np

M32 = 0xFFFFFFFF
M64 = (1 << 64) - 1
HDR = 16
LEVELS = 24
RUN = 256
CH_UNITS = 512  # double2 units per streaming chunk (kUnroll x 64 lanes)
FLAG_NAN, FLAG_EMPTY = 1, 4
NANBITS = np.uint64(0x7FF8000000000000)

# coin tags (the kernels use the same constants)
T_L0, T_L1, T_L2, T_L3 = 0x100, 0x200, 0x300, 0x400  # + lane
T_LODD = 0x800      # + 4 * lane + level (0..3): per-lane odd-slot pair compactions
T_WAVE = 0x1000     # the level-4 wave compaction
T_RUN = 0x1100      # + level: run merge-compactions (levels >= 5)
T_WODD = 0x1200     # + level: wave odd-slot pair compactions (levels >= 4)
T_FINAL = 0x1300    # + level: the build's final compression
T_FOLD = 0x2000     # + level: fold compactions (idx = fold index)

_LANES = np.arange(64, dtype=np.uint64)
_POS = np.arange(1024)
# lane l's 16 slots, j = 2u + h -> chunk position u * 128 + 2l + h
LANE_SLOTS = np.array([[u * 128 + 2 * lane + h for u in range(8) for h in range(2)] for lane in range(64)])


def mix64(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def slice_base(seed: int, series: int, slc: int) -> int:
    """The 64-bit coin key of one series slice (or of one fold epoch)."""
    return mix64(seed + 0x9E3779B97F4A7C15 * (series + 1) + 0xD1B54A32D192ED03 * (slc + 1))


def fmix32(h):
    """murmur3's 32-bit finaliser (ints or uint32 numpy arrays)."""
    if isinstance(h, np.ndarray):
        h = h.astype(np.uint32)
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
        return h
    h &= M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    return h ^ (h >> 16)


def coin32(base: int, tag, idx: int):
    """32 coin bits of event (tag, idx) of a slice: tag may be a uint32 array (per lane)."""
    lo, hi = base & M32, base >> 32
    if isinstance(tag, np.ndarray):
        with np.errstate(over="ignore"):
            t = (np.uint32(hi) + tag.astype(np.uint32) * np.uint32(0x9E3779B9)
                 + np.uint32((idx * 0x85EBCA6B) & M32))
        return fmix32(np.uint32(lo) ^ fmix32(t))
    return fmix32(lo ^ fmix32((hi + tag * 0x9E3779B9 + idx * 0x85EBCA6B) & M32))


def chunks(vals: np.ndarray, beg: int, end: int):
    """The 1,024-slot chunks the kernels' streaming skeleton delivers for [beg, end)
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


def fold_zero(x: np.ndarray) -> np.ndarray:
    return np.where(x == 0.0, 0.0, x)  # -0 -> +0 (NaN stays NaN)


class _Builder:
    """One series slice through the level hierarchy (the kernel's per-wave state)."""

    def __init__(self, base: int):
        self.base = base
        self.K = np.zeros((64, 4))             # per-lane odd slots, levels 0..3
        self.Kp = np.zeros((64, 4), bool)
        self.kcnt = np.zeros((64, 4), np.int64)  # per-lane odd-pair compactions per level
        self.arrival = [None] * 64             # per-lane key arriving at the wave level 4
        self.WK = {}                           # wave odd slots, levels >= 4
        self.wcnt = {}
        self.R = {}                            # runs, levels >= 5
        self.rcnt = {}
        self.w2 = 0
        self.pend = [None, None, None, None]   # (keys (64, 8), counts (64,)) at levels 1..3

    # -- odd slots --
    def lane_odd(self, lane: int, h: int, v: float) -> None:
        while h < 4:
            if not self.Kp[lane, h]:
                self.K[lane, h], self.Kp[lane, h] = v, True
                return
            a, b = sorted((self.K[lane, h], v))
            bit = coin32(self.base, T_LODD + 4 * lane + h, int(self.kcnt[lane, h])) & 1
            self.kcnt[lane, h] += 1
            v = b if bit else a
            self.Kp[lane, h] = False
            self.w2 += 4 ** h
            h += 1
        assert self.arrival[lane] is None, "one wave-level arrival per lane per level step"
        self.arrival[lane] = v

    def wave_odd(self, h: int, v: float) -> None:
        while True:
            assert h < LEVELS, "level overflow"
            if h not in self.WK:
                self.WK[h] = v
                return
            a, b = sorted((self.WK.pop(h), v))
            c = self.wcnt.get(h, 0)
            self.wcnt[h] = c + 1
            v = b if (coin32(self.base, T_WODD + h, c) & 1) else a
            self.w2 += 4 ** h
            h += 1

    def arrivals(self) -> None:
        for lane in range(64):
            if self.arrival[lane] is not None:
                v, self.arrival[lane] = self.arrival[lane], None
                self.wave_odd(4, v)

    # -- per-lane levels --
    def lane_compact(self, z: np.ndarray, c: np.ndarray, h: int, tag: int, idx: int):
        """z (64, 16) sorted ascending, absent keys +inf at the end, c present per lane:
        set aside the odd largest, keep every other key from the coin -> (64, 8), counts."""
        for lane in np.nonzero(c & 1)[0]:
            self.lane_odd(int(lane), h, float(z[lane, c[lane] - 1]))
            z[lane, c[lane] - 1] = np.inf
        c = c - (c & 1)
        off = (coin32(self.base, tag + _LANES, idx) & np.uint32(1)).astype(np.int64)
        y = np.where(off[:, None] == 1, z[:, 1::2], z[:, 0::2])
        self.w2 += int((c >= 2).sum()) * 4 ** h
        return y, c // 2

    def level0(self, x: np.ndarray, ci: int):
        pres = ~np.isnan(x)
        bits = coin32(self.base, T_L0 + _LANES, ci).astype(np.int64)
        out = np.full((64, 8), np.inf)
        cnt = np.zeros(64, np.int64)
        a, b = x[:, 0::2], x[:, 1::2]
        both = pres[:, 0::2] & pres[:, 1::2]
        sel = ((bits[:, None] >> np.arange(8)) & 1) == 1
        lo, hi = np.fmin(a, b), np.fmax(a, b)
        out = np.where(both, np.where(sel, hi, lo), np.inf)
        cnt = both.sum(axis=1)
        self.w2 += int(both.sum())
        lone = pres[:, 0::2] ^ pres[:, 1::2]
        for lane, u in zip(*np.nonzero(lone)):  # lane-major, pair order within a lane
            self.lane_odd(int(lane), 0, float(a[lane, u] if pres[lane, 2 * u] else b[lane, u]))
        return out, cnt

    def step(self, x: np.ndarray, ci: int) -> None:
        """One chunk (x: (64, 16) keys, NaN = absent)."""
        out, c0 = self.level0(x, ci)
        self.arrivals()
        if (ci & 1) == 0:
            self.pend[1] = (out, c0)
            return
        p, cp = self.pend[1]
        z = np.sort(np.concatenate([p, out], axis=1), axis=1)
        y, cy = self.lane_compact(z, cp + c0, 1, T_L1, ci >> 1)
        self.arrivals()
        for h, tag in ((2, T_L2), (3, T_L3)):
            if ((ci >> (h - 1)) & 1) == 0:
                self.pend[h] = (y, cy)
                return
            p, cp = self.pend[h]
            z = np.sort(np.concatenate([p, y], axis=1), axis=1)
            y, cy = self.lane_compact(z, cp + cy, h, tag, ci >> h)
            self.arrivals()
        # level 4: the wave
        u = np.sort(np.concatenate([y[lane, :cy[lane]] for lane in range(64)]))
        if u.size & 1:
            self.wave_odd(4, float(u[-1]))
            u = u[:-1]
        off = coin32(self.base, T_WAVE, ci >> 3) & 1
        if u.size >= 2:
            self.w2 += 4 ** 4
        self.push(u[off::2], 5)

    def push(self, t: np.ndarray, h: int) -> None:
        while t.size:
            assert h < LEVELS, "level overflow"
            if h not in self.R:
                self.R[h] = t
                return
            u = np.sort(np.concatenate([self.R.pop(h), t]))
            if u.size & 1:
                self.wave_odd(h, float(u[-1]))
                u = u[:-1]
            c = self.rcnt.get(h, 0)
            self.rcnt[h] = c + 1
            off = coin32(self.base, T_RUN + h, c) & 1
            t = u[off::2]
            self.w2 += 4 ** h
            h += 1

    def levels(self) -> list:
        L = []
        for h in range(LEVELS):
            parts = []
            if h < 4:
                parts.append(self.K[self.Kp[:, h], h])
            if h in self.R:
                parts.append(self.R[h])
            if h in self.WK:
                parts.append(np.array([self.WK[h]]))
            L.append(np.sort(np.concatenate(parts)) if parts else np.zeros(0))
        return L


def compress(L: list, budget: int, base: int, tag: int, idx: int):
    """From level 0 up, while more than ``budget`` keys remain, compact each level holding
    >= 2 keys once (odd largest set aside) into the next level.  -> (levels, sum w^2 added)."""
    L = [np.sort(x) for x in L]
    total = sum(x.size for x in L)
    w2 = 0
    for h in range(LEVELS):
        if total <= budget:
            break
        if L[h].size < 2:
            continue
        assert h + 1 < LEVELS, "level overflow"
        u = L[h]
        keep, u = (u[-1:], u[:-1]) if u.size & 1 else (u[:0], u)
        off = coin32(base, tag + h, idx) & 1
        out = u[off::2]
        w2 += 4 ** h
        total -= u.size - out.size
        L[h] = keep
        L[h + 1] = np.sort(np.concatenate([L[h + 1], out]))
    return L, w2


def _lens_words(L) -> list:
    words = [0] * 6
    for h, x in enumerate(L):
        words[h >> 2] |= int(x.size) << (16 * (h & 3))
    return words


def _f64bits(v: float) -> np.uint64:
    return np.array([v], dtype=np.float64).view(np.uint64)[0]


def row_words(budget: int, tail: int) -> int:
    return HDR + budget + tail


def _assemble(n: int, nan: int, mn: float, mx: float, w2: int, L: list, tail_keys: np.ndarray, budget: int,
              cap: int) -> np.ndarray:
    row = np.zeros(row_words(budget, cap), dtype=np.uint64)
    body = np.concatenate(L) if L else np.zeros(0)
    assert body.size <= budget
    weight = sum(int(x.size) << h for h, x in enumerate(L))
    assert weight == n, (weight, n)
    row[0], row[1] = n, nan
    row[2] = _f64bits(mn) if n else NANBITS
    row[3] = _f64bits(mx) if n else NANBITS
    row[4], row[5], row[6] = w2, weight, tail_keys.size
    row[7] = (budget << 32) | cap
    row[8:14] = _lens_words(L)
    row[HDR: HDR + body.size] = body.astype(np.float64).view(np.uint64)
    row[HDR + budget: HDR + budget + tail_keys.size] = tail_keys.astype(np.float64).view(np.uint64)
    return row


def build_row(vals: np.ndarray, beg: int, end: int, *, budget: int = 512, tail: int = 0, seed: int = 0,
              series: int = 0, slc: int = 0, gaps: bool = False) -> np.ndarray:
    """The row (uint64 [row_words(budget, tail)]) of segment [beg, end) of ``vals``."""
    chs = list(chunks(vals, beg, end))
    nch = len(chs)
    npad = -(-nch // 8) * 8
    B = _Builder(slice_base(seed, series, slc))
    for ci in range(npad):
        s = chs[ci] if ci < nch else np.full(1024, np.nan)
        B.step(fold_zero(s[LANE_SLOTS]), ci)
    seg = fold_zero(np.asarray(vals[beg:end], dtype=np.float64))
    pres = seg[~np.isnan(seg)]
    n = int(pres.size)
    L, w2 = compress(B.levels(), budget, B.base, T_FINAL, 0)
    tl = min(n, tail)
    tail_keys = np.sort(pres)[n - tl:] if tl else np.zeros(0)
    return _assemble(n, 0 if gaps else (end - beg) - n, float(pres.min()) if n else math.nan,
                     float(pres.max()) if n else math.nan, B.w2 + w2, L, tail_keys, budget, tail)


def row_levels(row: np.ndarray) -> list:
    """Body keys per level (float64 arrays, ascending)."""
    budget = int(row[7]) >> 32
    L, pos = [], 0
    for h in range(LEVELS):
        ln = (int(row[8 + (h >> 2)]) >> (16 * (h & 3))) & 0xFFFF
        L.append(row[HDR + pos: HDR + pos + ln].view(np.float64).copy())
        pos += ln
    assert pos <= budget
    return L


def row_tail(row: np.ndarray) -> np.ndarray:
    budget, tl = int(row[7]) >> 32, int(row[6])
    return row[HDR + budget: HDR + budget + tl].view(np.float64).copy()


def _fmin(a: float, b: float) -> float:
    return b if math.isnan(a) else (a if math.isnan(b) else min(a, b))


def _fmax(a: float, b: float) -> float:
    return b if math.isnan(a) else (a if math.isnan(b) else max(a, b))


def fold(a: np.ndarray, b: np.ndarray, base: int, idx: int) -> np.ndarray:
    """Row a folded with row b (the same budget / tail cap): fold index ``idx`` keys the coins."""
    if int(a[7]) != int(b[7]):
        raise ValueError("rows of different formats (budget, tail cap) do not fold")
    budget, cap = int(a[7]) >> 32, int(a[7]) & M32
    n = int(a[0]) + int(b[0])
    nan = int(a[1]) + int(b[1])
    mn = _fmin(float(a[2:3].view(np.float64)[0]), float(b[2:3].view(np.float64)[0]))
    mx = _fmax(float(a[3:4].view(np.float64)[0]), float(b[3:4].view(np.float64)[0]))
    t = np.sort(np.concatenate([row_tail(a), row_tail(b)]))
    t = t[t.size - min(cap, n):]
    L = [np.concatenate([x, y]) for x, y in zip(row_levels(a), row_levels(b))]
    L, w2 = compress(L, budget, base, T_FOLD, idx)
    return _assemble(n, nan, mn, mx, int(a[4]) + int(b[4]) + w2, L, t, budget, cap)


def merge_rows(rows: np.ndarray, *, seed: int = 0, series: int = 0, epoch: int = 0) -> np.ndarray:
    """W rows of one series (e.g. its time slices, in time order) folded left to right into one:
    row 0, then fold index w = 1 .. W - 1, coins keyed by (seed, series, epoch)."""
    base = slice_base(seed, series, epoch)
    acc = rows[0].copy()
    for w in range(1, rows.shape[0]):
        acc = fold(acc, rows[w], base, w)
    return acc


def np_lerp(a: float, b: float, t: float) -> float:
    d = b - a
    return b - d * (1.0 - t) if t >= 0.5 else a + d * t


def exact_rank(n: int, p_num: int, p_den: int) -> int:
    return ((n - 1) * p_num) // (100 * p_den)


def query(rows: np.ndarray, mode: int, p_num: int, p_den: int, q: float, *, seed: int = 0, series: int = 0,
          epoch: int = 0):
    """(value, count, flags) of one series from its W rows (uint64 [W, row_words]): folded
    into one row (merge_rows), then answered from it."""
    rows = np.atleast_2d(rows)
    row = merge_rows(rows, seed=seed, series=series, epoch=epoch) if rows.shape[0] > 1 else rows[0]
    n, nan = int(row[0]), int(row[1])
    if nan:
        return math.nan, n, FLAG_NAN
    if n == 0:
        return math.nan, 0, FLAG_EMPTY
    mn, mx = float(row[2:3].view(np.float64)[0]), float(row[3:4].view(np.float64)[0])
    tail = row_tail(row)
    L = row_levels(row)
    keys = np.concatenate(L)
    w = np.concatenate([np.full(x.size, 1 << h, dtype=np.int64) for h, x in enumerate(L)])
    order = np.argsort(keys, kind="stable")
    keys, cum = keys[order], np.cumsum(w[order])

    def select(r: int) -> float:
        if r == 0:
            return mn
        if r == n - 1:
            return mx
        if n - r <= tail.size:
            return float(tail[tail.size - (n - r)])
        return float(keys[int(np.searchsorted(cum, r, side="right"))])  # first cum > r

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


def rank_bound(row: np.ndarray, delta: float = 0.01) -> float:
    """Normalised rank-error bound of body answers (probability >= 1 - delta): the weighted
    count of kept keys <= x is off by a sum of martingale differences bounded by the fixed
    weights of the schedule, so by Azuma-Hoeffding by more than t = sqrt(2 ln(4/delta) sum w^2)
    at x_lo or x_hi with probability <= delta; between them the answer's rank interval meets
    [r - t, r + t].  Ranks r with n - r <= tl are exact (0)."""
    n = float(row[0])
    return math.sqrt(2.0 * math.log(4.0 / delta) * float(int(row[4]))) / n if n else math.nan
