"""TEST INFRASTRUCTURE ONLY — numpy restatement of the sketch mode (config 5).

Sketch mode is a build-only extension (the reference cannot
express 30d@15s), so there is no reference output to pin it to.  This file
restates the kernels' definitions (krr_amd/csrc/krr_kernels.hip, SKETCH
section) so tests can check the GPU build bit-exactly (counts, min, max) and the
query to float64 rounding; the sketch's distance from the EXACT percentile is
measured separately against oracle/krr_oracle.c (rank error).
"""
from __future__ import annotations

import math

import numpy as np


def width(m: int, e_lo: int, octaves: int) -> int:
    return (octaves << m) + 4


def bins_of(x: np.ndarray, m: int, e_lo: int, octaves: int) -> np.ndarray:
    """Bin of every non-NaN sample: 0 negative, 1 +-0, 2 below 2^e_lo, 3.. log-linear, last = above."""
    u = np.ascontiguousarray(x, dtype=np.float64).view(np.uint64)
    mag = u & np.uint64(0x7FFFFFFFFFFFFFFF)
    nb = octaves << m
    base = np.uint64((e_lo + 1023) << m)
    idx = (mag >> np.uint64(52 - m)) - base  # wraps below range (uint64)
    low_bits = np.uint64((e_lo + 1023) << 52)
    b = np.where(idx < np.uint64(nb), idx + np.uint64(3), np.where(mag < low_bits, 2, 3 + nb)).astype(np.int64)
    b = np.where(u >> np.uint64(63) == 1, 0, b)
    b = np.where(mag == 0, 1, b)
    return b


def build(x: np.ndarray, m: int, e_lo: int, octaves: int):
    """(counts[width], vmin, vmax) of one series (NaN samples skipped)."""
    x = np.asarray(x, dtype=np.float64)
    ok = ~np.isnan(x)
    counts = np.bincount(bins_of(x[ok], m, e_lo, octaves), minlength=width(m, e_lo, octaves)).astype(np.int64)
    vmin = float(np.min(x[ok])) if ok.any() else math.nan
    vmax = float(np.max(x[ok])) if ok.any() else math.nan
    return counts, vmin, vmax


def _value(counts, b, r, before, m, e_lo, octaves, vmin, vmax, n):
    if r == 0:
        return vmin
    if r == n - 1:
        return vmax
    c = counts[b]
    f = ((r - before) + 0.5) / c
    nb = octaves << m
    if b == 1:
        return 0.0
    if b == 0:
        lo, hi = vmin, 0.0
    elif b == 2:
        lo, hi = 0.0, math.ldexp(1.0, e_lo)
    elif b == 3 + nb:
        lo, hi = math.ldexp(1.0, e_lo + octaves), vmax
    else:
        i = b - 3
        E = e_lo + (i >> m)
        j = float(i & ((1 << m) - 1))
        step = math.ldexp(1.0, E - m)
        lo = math.ldexp(1.0, E) + j * step
        hi = lo + step
    v = lo + f * (hi - lo)
    return min(max(v, vmin), vmax)


def np_lerp(a, b, t):
    d = b - a
    return b - d * (1.0 - t) if t >= 0.5 else a + d * t


def query(counts, vmin, vmax, m, e_lo, octaves, mode: str, p_num: int, p_den: int, q: float):
    """Sketch percentile of one series: mode 'sorted_lower' or 'linear'."""
    counts = np.asarray(counts, dtype=np.int64)
    n = int(counts.sum())
    if n == 0:
        return math.nan, 0
    if mode == "sorted_lower":
        r0 = r1 = ((n - 1) * p_num) // (100 * p_den)
        gamma = 0.0
    else:
        vidx = float(n - 1) * q
        if vidx >= n - 1:
            r0 = r1 = n - 1
            gamma = vidx - (-1.0)
        else:
            r0 = int(math.floor(vidx))
            r1 = r0 + 1
            gamma = vidx - math.floor(vidx)
    cum = np.cumsum(counts)
    vals = []
    for r in (r0, r1):
        b = int(np.searchsorted(cum, r, side="right"))
        before = int(cum[b - 1]) if b else 0
        vals.append(_value(counts, b, r, before, m, e_lo, octaves, vmin, vmax, n))
    if mode == "sorted_lower":
        return vals[0], n
    return np_lerp(vals[0], vals[1], gamma), n


# ---- exact refinement (krr_sketch_locate / _collect / _refine) ----------------------------

def ranks(n: int, mode: str, p_num: int, p_den: int, q: float):
    """(r0, r1, gamma): the ascending ranks SORTED_LOWER / LINEAR need (kernels' ranks_for)."""
    if mode == "sorted_lower":
        r = ((n - 1) * p_num) // (100 * p_den)
        return r, r, 0.0
    vidx = float(n - 1) * q
    if vidx >= n - 1:
        return n - 1, n - 1, vidx - (-1.0)
    fl = math.floor(vidx)
    return int(fl), int(fl) + 1, vidx - fl


def locate(counts, mode: str, p_num: int, p_den: int, q: float):
    """(n, r0, r1, before, gamma, bin_lo, bin_hi) of one merged sketch; bin_lo > bin_hi if empty."""
    counts = np.asarray(counts, dtype=np.int64)
    n = int(counts.sum())
    if n == 0:
        return 0, -1, -1, 0, 0.0, 1, 0
    r0, r1, gamma = ranks(n, mode, p_num, p_den, q)
    cum = np.cumsum(counts)
    b0 = int(np.searchsorted(cum, r0, side="right"))
    b1 = int(np.searchsorted(cum, r1, side="right"))
    before = int(cum[b0 - 1]) if b0 else 0
    return n, r0, r1, before, gamma, b0, b1


def collect(x: np.ndarray, bin_lo: int, bin_hi: int, m: int, e_lo: int, octaves: int) -> np.ndarray:
    """Present samples of x with bin in [bin_lo, bin_hi], position order."""
    x = np.asarray(x, dtype=np.float64)
    x = x[~np.isnan(x)]
    if bin_lo > bin_hi or x.size == 0:
        return x[:0]
    b = bins_of(x, m, e_lo, octaves)
    return x[(b >= bin_lo) & (b <= bin_hi)]


def refine(lst: np.ndarray, j0: int, j1: int, gamma: float, mode: str) -> float:
    """Exact result from the collected list (time order) and local ranks j0 <= j1."""
    srt = np.sort(lst, kind="stable")
    a = float(srt[j0])
    if mode == "sorted_lower":
        if a == 0.0:  # Python sorted() is stable: the zero at rank j0 by position
            neg = int(np.count_nonzero(lst < 0))
            zeros = lst[lst == 0.0]
            return float(zeros[j0 - neg])
        return a
    return np_lerp(a, float(srt[j1]), gamma)
