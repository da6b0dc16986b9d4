"""Sketch mode and time-sharded series (BASELINE config 5: 30d@15s, 172,800 samples).

A build-only extension: the reference cannot query 30d@15s (SURVEY.md §0.5 —
``timeframe_duration`` is whole minutes, ``core/abstract/strategies.py:23``) and
keeps each object's samples in one Python list (``prometheus.py:150-155``).
Here a series too long for one GPU's window is TIME-sharded: rank r holds the
r-th contiguous time slice of every series.

* Percentile (SORTED_LOWER / LINEAR): each rank builds a log-linear histogram
  sketch per series slice (``krr_sketch_build``, one HBM pass).  Bins are
  data-independent, so the W slices of a series merge exactly by adding counts:
  ONE reduce-scatter (RCCL over xGMI) leaves each rank the merged sketches of a
  contiguous block of series, which it queries (``krr_sketch_query``).  The value
  is interpolated inside the bin holding the rank (relative bin width 2^-m); the
  rank error is measured against the exact path, never assumed (bench.py).
* Exact percentiles, ONE HBM pass (``window_exact_time_sharded``, the default): every
  rank streams its slice of each series once through the window select, with the
  other slices' slots counted as unseen, and exports the window it kept (bounds,
  exact count below, keys; ``krr_window_export``).  One all-to-all (RCCL) hands each
  series' windows to its owner, which intersects them; the exact counts decide
  whether the needed ranks lie inside, and then they are selected there
  (``krr_window_merge``) — bit-identical to one select over the whole series.  A
  miss (a slice whose distribution differs from the series', e.g. a trend) regathers
  only that series' slices to its owner and selects it whole.
* Exact percentiles, two passes (``exact_time_sharded``, kept as the reference
  design and for comparison): the merged counts are exact, so they
  say exactly which bin holds each needed rank and how many samples lie below it
  (``krr_sketch_locate``).  One all-gather gives every rank those bins, each rank
  collects its samples inside them (``krr_sketch_collect``, a second HBM pass), an
  all-to-all hands them to the owner in time order, and ``krr_sketch_refine``
  selects the ranks inside the short lists: bit-identical to selecting over the
  whole series on one GPU.
* KLL-style compactor sketch (``kll_time_sharded``, ``bench.py --sketch-only --sketch-kind
  kll``): per slice one HBM pass sorts 512-slot blocks on the wave and compacts them
  level by level into at most ``budget`` weighted keys (``krr_kll_build``); the W rows of
  a series reach its owner in one all-to-all and are queried together
  (``krr_kll_query``).  Unlike the histogram its RANK error has a data-independent bound:
  ``kll_rank_bound`` (Azuma-Hoeffding over the compactions' coins as martingale
  differences; the deterministic schedule fixes the rows' sum of w^2 before any coin).
* REF_INDEX (the reference's rule, ``simple.py:36``) stays exact: all-gather the
  per-slice present counts, the rank whose slice holds global index k selects it
  (``krr_select_present``), one all-gather collects the answers.
* Memory max stays exact: all-gather (max, count) per slice and merge in time
  order with Python ``max()``'s first-maximum rule (``simple.py:29``).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Optional

import numpy as np

from krr_amd import _native


@dataclass(frozen=True)
class SketchConfig:
    """Log-linear bins: 2^mantissa_bits per octave over [2^min_exponent, 2^(min_exponent+octaves))."""
    mantissa_bits: int = 5     # relative bin width <= 1/32
    min_exponent: int = -24    # 6e-8 cores
    octaves: int = 36          # ... up to 4096 cores

    def params(self) -> _native.KrrSketchParams:
        return _native.KrrSketchParams(self.mantissa_bits, self.min_exponent, self.octaves, 0)

    @property
    def width(self) -> int:
        return (self.octaves << self.mantissa_bits) + 4


def build(ctx: _native.Context, series: _native.KrrSeries, cfg: SketchConfig, stream=None) -> dict:
    """One HBM pass: per-series sketch of this rank's slices.  Device tensors."""
    import torch

    S = series.n_segments
    dev = series._keep[0].device
    out = {
        "counts": torch.empty((S, cfg.width), dtype=torch.int32, device=dev),
        "vmin": torch.empty(S, dtype=torch.float64, device=dev),
        "vmax": torch.empty(S, dtype=torch.float64, device=dev),
        "flags": torch.empty(S, dtype=torch.int32, device=dev),
    }
    ctx.sketch_build(series, cfg.params(), out["counts"], out["vmin"], out["vmax"], out["flags"], stream)
    return out


def owner_blocks(n_series: int, world: int) -> list[tuple[int, int]]:
    """Series [0, S) in world contiguous blocks of ceil(S / world) (the last may be short)."""
    per = -(-n_series // world) if world else 0
    return [(min(r * per, n_series), min((r + 1) * per, n_series)) for r in range(world)]


def _reduce_scatter(t, op, group, world: int):
    """Rank r gets block r of the elementwise reduction of t ([world * per, ...])."""
    import torch
    import torch.distributed as dist

    per = t.shape[0] // world
    out = torch.empty((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if dist.get_backend(group) == "nccl":
        dist.reduce_scatter_tensor(out, t, op=op, group=group)
    else:  # gloo (CPU tests): same result through all_reduce
        full = t.clone()
        dist.all_reduce(full, op=op, group=group)
        r = dist.get_rank(group)
        out.copy_(full[r * per:(r + 1) * per])
    return out


def merge_time_sharded(sk: dict, group=None) -> dict:
    """Merge the per-slice sketches of all ranks: rank r receives the merged
    sketches of its owner block (owner_blocks) as counts/vmin/vmax/flags, plus
    'block' = (lo, hi).  World size 1: the input, unchanged."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return dict(sk, block=(0, sk["vmin"].numel()))
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    S = sk["vmin"].numel()
    per = -(-S // world)
    pad = per * world - S

    def padded(t, fill):
        if not pad:
            return t
        ext = torch.full((pad,) + tuple(t.shape[1:]), fill, dtype=t.dtype, device=t.device)
        return torch.cat([t, ext], dim=0)

    counts = _reduce_scatter(padded(sk["counts"], 0), dist.ReduceOp.SUM, group, world)
    # NaN (an empty slice) must not win min/max: +-inf stand-ins, mapped back after
    vmin = _reduce_scatter(padded(torch.nan_to_num(sk["vmin"], nan=float("inf")), float("inf")),
                           dist.ReduceOp.MIN, group, world)
    vmax = _reduce_scatter(padded(torch.nan_to_num(sk["vmax"], nan=float("-inf")), float("-inf")),
                           dist.ReduceOp.MAX, group, world)
    flags = _reduce_scatter(padded(sk["flags"], 0), dist.ReduceOp.MAX, group, world)
    lo, hi = owner_blocks(S, world)[rank]
    n = hi - lo
    empty = counts[:n].sum(dim=1) == 0
    vmin = torch.where(empty, torch.full_like(vmin[:n], float("nan")), vmin[:n])
    vmax = torch.where(empty, torch.full_like(vmax[:n], float("nan")), vmax[:n])
    return {"counts": counts[:n].contiguous(), "vmin": vmin.contiguous(), "vmax": vmax.contiguous(),
            "flags": flags[:n].contiguous(), "block": (lo, hi)}


def _needs_table(params) -> bool:
    """Does the percentile's index rule need a table whatever the counts (krr_amd.core.index_rule)?
    Only then do the queries below size one from their merged counts (a synchronisation)."""
    rule = getattr(params, "rule", None)
    return (rule is not None and params.mode != _native.KRR_PCT_LINEAR and not params.k_table
            and rule.needs_table(1 << 40))  # counts past 2^40 cannot be held (see _native.bind_index_table)


def query(ctx: _native.Context, merged: dict, cfg: SketchConfig, params: _native.KrrPercentileParams,
          stream=None) -> dict:
    """Percentile of every (merged) sketch.  KRR_FLAG_NAN from the build is carried over."""
    import torch

    S = merged["vmin"].numel()
    dev = merged["vmin"].device
    out = {"value": torch.empty(S, dtype=torch.float64, device=dev),
           "count": torch.empty(S, dtype=torch.int64, device=dev),
           "flags": torch.empty(S, dtype=torch.int32, device=dev)}
    max_n = int(merged["counts"].sum(dim=1).max().item()) if S and _needs_table(params) else None
    ctx.sketch_query(merged["counts"], merged["vmin"], merged["vmax"], cfg.params(), params, out["value"],
                     out["count"], out["flags"], stream, max_n=max_n)
    nan = (merged["flags"] & _native.KRR_FLAG_NAN) != 0
    if bool(nan.any()):
        out["flags"] |= merged["flags"] & _native.KRR_FLAG_NAN
        out["value"] = torch.where(nan, torch.full_like(out["value"], float("nan")), out["value"])
    return out


# ------------------------- exact refinement of merged sketches -------------------------

def locate(ctx: _native.Context, merged: dict, cfg: SketchConfig, params: _native.KrrPercentileParams,
           stream=None):
    """krr_sketch_loc of every merged sketch: int64 [S_block, LOC_WORDS]."""
    import torch

    S = merged["counts"].shape[0]
    loc = torch.empty((S, _native.LOC_WORDS), dtype=torch.int64, device=merged["counts"].device)
    if S:
        max_n = int(merged["counts"].sum(dim=1).max().item()) if _needs_table(params) else None
        ctx.sketch_locate(merged["counts"], cfg.params(), params, loc, stream, max_n=max_n)
    return loc


def _all_gather_blocks(block, S: int, group, world: int):
    """Concatenate every rank's owner block ([<= per, ...], owner_blocks order) -> [S, ...]."""
    import torch
    import torch.distributed as dist

    per = -(-S // world)
    dev = block.device
    coll = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
    pad = torch.zeros((per,) + tuple(block.shape[1:]), dtype=block.dtype, device=coll)
    pad[: block.shape[0]] = block.to(coll)
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    out = [p[: hi - lo] for p, (lo, hi) in zip(parts, owner_blocks(S, world))]
    return torch.cat(out, dim=0).to(dev)


def exchange_to_owners(values, counts, S: int, group=None):
    """values: this rank's collected samples, CSR by series (counts[S] per series, all
    S series in order).  Returns the owner block's lists of ALL ranks, concatenated
    per series in rank (= time) order: (values, offsets[n_block + 1]) — the CSR
    krr_sketch_refine reads.  World size 1: the input as CSR."""
    import torch
    import torch.distributed as dist

    dev = values.device
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        offs = torch.zeros(S + 1, dtype=torch.int64, device=dev)
        offs[1:] = torch.cumsum(counts, 0)
        return values, offs
    rank = dist.get_rank(group)
    coll = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
    blocks = owner_blocks(S, world)
    per = -(-S // world)
    cnt_pad = torch.zeros(world * per, dtype=torch.int64, device=coll)
    for r, (lo, hi) in enumerate(blocks):
        cnt_pad[r * per: r * per + (hi - lo)] = counts[lo:hi].to(coll)
    recv_cnt = torch.empty_like(cnt_pad)
    dist.all_to_all_single(recv_cnt, cnt_pad, group=group)  # [src][per] counts of my block
    send_sizes = cnt_pad.view(world, per).sum(1).tolist()
    c = recv_cnt.view(world, per)
    recv_sizes = c.sum(1).tolist()
    recv = torch.empty(int(sum(recv_sizes)), dtype=values.dtype, device=coll)
    dist.all_to_all_single(recv, values.to(coll), output_split_sizes=recv_sizes, input_split_sizes=send_sizes,
                           group=group)
    lo, hi = blocks[rank]
    nb = hi - lo
    c = c[:, :nb]
    tot = c.sum(0)
    offs = torch.zeros(nb + 1, dtype=torch.int64, device=coll)
    offs[1:] = torch.cumsum(tot, 0)
    if recv.numel() == 0:
        return recv.to(dev), offs.to(dev)
    # source-major (rank, series) pieces -> series-major, rank order inside each series
    flat = c.reshape(-1)
    src_start = torch.cumsum(flat, 0) - flat
    dst_start = (offs[:-1][None, :] + (torch.cumsum(c, 0) - c)).reshape(-1)
    piece = torch.repeat_interleave(torch.arange(flat.numel(), device=coll), flat)
    pos = torch.arange(recv.numel(), device=coll)
    dest = dst_start[piece] + (pos - src_start[piece])
    grouped = torch.empty_like(recv)
    grouped[dest] = recv
    return grouped.to(dev), offs.to(dev)


def exact_time_sharded(ctx: _native.Context, series: _native.KrrSeries, local: dict, merged: dict,
                       cfg: SketchConfig, params: _native.KrrPercentileParams, group=None, stream=None,
                       events=None) -> dict:
    """Exact SORTED_LOWER / LINEAR percentile of every time-sharded series from this
    rank's local sketches (``build``) and its owner block's merged sketches
    (``merge_time_sharded``).  Returns device tensors value/count/flags for the
    owner block (same layout as ``query``), plus 'block' and 'collected' (samples
    this rank collected).  ``events``: optional pair of HIP events recorded around
    the collect pass (its HBM time)."""
    import torch
    import torch.distributed as dist

    S = series.n_segments
    dev = series._keep[0].device
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    loc_blk = locate(ctx, merged, cfg, params, stream)
    loc = _all_gather_blocks(loc_blk, S, group, world) if world > 1 else loc_blk
    cnt = torch.empty(S, dtype=torch.int64, device=dev)
    ctx.sketch_range_count(local["counts"], cfg.params(), loc, cnt, stream)
    offs = torch.zeros(S + 1, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(cnt, 0)
    total = int(offs[-1].item())
    vals = torch.empty(max(total, 1), dtype=torch.float64, device=dev)
    if events is not None:
        events[0].record(stream)
    ctx.sketch_collect(series, cfg.params(), loc, offs, vals, None, stream)
    if events is not None:
        events[1].record(stream)
    gvals, goffs = exchange_to_owners(vals[:total], cnt, S, group)
    nb = loc_blk.shape[0]
    gv = gvals if gvals.numel() else torch.empty(1, dtype=torch.float64, device=dev)
    coll_ser = ctx.series(gv, goffs.contiguous(), 0, False)
    out = {"value": torch.empty(nb, dtype=torch.float64, device=dev),
           "count": torch.empty(nb, dtype=torch.int64, device=dev),
           "flags": torch.empty(nb, dtype=torch.int32, device=dev)}
    if nb:
        ctx.sketch_refine(coll_ser, loc_blk, out["value"], out["count"], out["flags"], stream)
    nan = (merged["flags"] & _native.KRR_FLAG_NAN) != 0
    if bool(nan.any()):
        out["flags"] |= merged["flags"] & _native.KRR_FLAG_NAN
        out["value"] = torch.where(nan, torch.full_like(out["value"], float("nan")), out["value"])
    out["block"] = merged.get("block", (0, nb))
    out["collected"] = total
    return out


# ----------------------------- exact time-sharded merges ------------------------------

def exact_rank_np(n: np.ndarray, p_num: int, p_den: int, rule=None) -> np.ndarray:
    """floor((n-1) * p_num / (100 p_den)) exactly, elementwise (n >= 1); with ``rule``
    (krr_amd.core.index_rule.IndexRule) the reference's own k(n) instead."""
    if rule is not None:
        return rule.ks(n)
    n = np.asarray(n, dtype=np.int64)
    a = n - 1
    den = 100 * int(p_den)
    if int(a.max(initial=0)) * int(p_num) < 2**63:
        return (a * int(p_num)) // den
    return np.array([(int(x) * int(p_num)) // den for x in a], dtype=np.int64)


def refindex_locate(all_n: np.ndarray, p_num: int, p_den: int, rank: int, rule=None):
    """Global REF_INDEX position from per-slice present counts all_n[world, S]
    (time order = rank order): n[S], k[S] (-1 if empty), owner[S] = the rank whose
    slice holds k (-1 if empty), and this rank's local index (-1 if not its own)."""
    all_n = np.asarray(all_n, dtype=np.int64)
    n = all_n.sum(axis=0)
    prefix = np.cumsum(all_n, axis=0) - all_n  # samples in earlier slices
    k = np.where(n > 0, exact_rank_np(np.maximum(n, 1), p_num, p_den, rule), -1)
    inside = (k[None, :] >= prefix) & (k[None, :] < prefix + all_n)
    owner = np.where(n > 0, np.argmax(inside, axis=0), -1)
    k_local = np.where(owner == rank, k - prefix[rank], -1).astype(np.int64)
    return n, k, owner, k_local


def refindex_time_sharded(ctx: _native.Context, series: _native.KrrSeries, params: _native.KrrPercentileParams,
                          group=None, stream=None) -> dict:
    """Exact REF_INDEX (the reference's X[floor((n-1) p / 100)] over the time-ordered
    concatenation of every rank's slices, simple.py:31-36).  Returns host arrays
    value/count/flags for ALL series on every rank."""
    import torch
    import torch.distributed as dist

    S = series.n_segments
    vals, offs = series._keep
    dev = vals.device
    inf = torch.full((S,), float("inf"), dtype=torch.float64, device=dev)
    lt = torch.empty(S, dtype=torch.int64, device=dev)
    le = torch.empty(S, dtype=torch.int64, device=dev)
    if series.gaps_are_nan:
        ctx.rank_of(series, inf, lt, le, stream)  # le(+inf) = present (non-NaN) samples of the slice
        local_n = le
    else:  # compact layout: every slot is a sample, NaN included (the reference indexes the list)
        local_n = (offs[1:] - offs[:-1]).contiguous()
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if world > 1:
        coll = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
        g = [torch.empty(S, dtype=torch.int64, device=coll) for _ in range(world)]
        dist.all_gather(g, local_n.to(coll), group=group)
        all_n = torch.stack(g).cpu().numpy()  # [world, S], time order = rank order
    else:
        all_n = local_n.cpu().numpy()[None, :]
    n, k, owner, k_local = refindex_locate(all_n, params.p_num, params.p_den, rank, getattr(params, "rule", None))
    mine = owner == rank
    kt = torch.from_numpy(k_local).to(dev)
    found = torch.full((S,), float("nan"), dtype=torch.float64, device=dev)
    ctx.select_present(series, kt, found, stream)
    bits = torch.where(torch.from_numpy(mine).to(dev), found.view(torch.int64),
                       torch.zeros(S, dtype=torch.int64, device=dev))
    if world > 1:
        coll = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
        gb = [torch.empty(S, dtype=torch.int64, device=coll) for _ in range(world)]
        dist.all_gather(gb, bits.to(coll), group=group)
        allb = torch.stack(gb).cpu().numpy()
        vbits = allb[np.maximum(owner, 0), np.arange(S)]
    else:
        vbits = bits.cpu().numpy()
    value = vbits.view(np.float64).copy()
    flags = np.zeros(S, dtype=np.uint32)
    value[n == 0] = np.nan
    flags[n == 0] |= _native.KRR_FLAG_EMPTY
    return {"value": value, "count": n.astype(np.int64), "flags": flags}


def max_time_sharded(local_value, local_count, local_flags, group=None) -> dict:
    """Exact memory max over time slices: Python max() keeps the FIRST maximal
    element in time order (only +-0 differ in bits), so merge in rank order taking
    strictly greater values.  Inputs: per-slice device/host tensors [S]."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    v = local_value.view(torch.int64)
    packed = torch.stack([v, local_count, local_flags.to(torch.int64)], dim=1)
    if world > 1:
        coll = packed.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
        g = [torch.empty_like(packed, device=coll) for _ in range(world)]
        dist.all_gather(g, packed.to(coll), group=group)
        parts = [x.cpu().numpy() for x in g]
    else:
        parts = [packed.cpu().numpy()]
    S = parts[0].shape[0]
    best = np.full(S, np.nan)
    count = np.zeros(S, dtype=np.int64)
    flags = np.zeros(S, dtype=np.uint32)
    for p in parts:  # time order
        val = p[:, 0].copy().view(np.float64)
        cnt = p[:, 1]
        flg = p[:, 2].astype(np.uint32)
        count += cnt
        flags |= flg & _native.KRR_FLAG_NAN
        take = (cnt > 0) & ((np.isnan(best)) | (val > best))
        best = np.where(take, val, best)
    flags[count == 0] |= _native.KRR_FLAG_EMPTY
    best[(flags & _native.KRR_FLAG_NAN) != 0] = np.nan
    return {"value": best, "count": count, "flags": flags}


# -------------------- one-pass exact time-sharded percentiles (window export) ---------------------

_SIDE = {}


def _side_stream(dev):
    import torch

    key = (threading.get_ident(), str(dev))
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


def _max_len(series) -> int:
    if series.max_segment_len > 0:
        return int(series.max_segment_len)
    offs = series._keep[1]
    return int((offs[1:] - offs[:-1]).max().item()) if series.n_segments else 0


def gather_segments(values, offs, ids):
    """Segments ``ids`` (int64 tensor, any order) of a CSR -> (values, offsets) of a
    new CSR holding them in that order (device-side index gather)."""
    import torch

    dev = values.device
    k = int(ids.numel())
    starts = offs[ids]
    lens = offs[ids + 1] - starts
    new_offs = torch.zeros(k + 1, dtype=torch.int64, device=dev)
    if k:
        new_offs[1:] = torch.cumsum(lens, 0)
    total = int(new_offs[-1].item()) if k else 0
    if total == 0:
        return torch.empty(1, dtype=values.dtype, device=dev), new_offs
    seg = torch.repeat_interleave(torch.arange(k, device=dev), lens)
    pos = torch.arange(total, device=dev) - new_offs[seg] + starts[seg]
    return values[pos], new_offs


def _parts(series):
    """A KrrSeries, or a list of (lo, hi, KrrSeries) parts holding series [lo, hi) each in
    buffers of their own (contiguous, ascending) -> the list form."""
    if isinstance(series, (list, tuple)):
        return list(series)
    return [(0, series.n_segments, series)]


def gather_segments_parts(parts, ids):
    """gather_segments over series held in parts: ``ids`` ascending global series ids."""
    import torch

    if len(parts) == 1:
        vals, offs = parts[0][2]._keep
        return gather_segments(vals, offs, ids - parts[0][0])
    vs, ls = [], []
    for lo, hi, ser in parts:
        sel = ids[(ids >= lo) & (ids < hi)]
        if sel.numel() == 0:
            continue
        v, o = gather_segments(*ser._keep, sel - lo)
        vs.append(v[: int(o[-1].item())])
        ls.append(o[1:] - o[:-1])
    dev = parts[0][2]._keep[0].device
    if not vs:
        return torch.empty(1, dtype=torch.float64, device=dev), torch.zeros(1, dtype=torch.int64, device=dev)
    lens = torch.cat(ls)
    offs = torch.zeros(lens.numel() + 1, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(lens, 0)
    vals = torch.cat(vs)
    return (vals if vals.numel() else torch.empty(1, dtype=torch.float64, device=dev)), offs


def window_exact_time_sharded(ctx: _native.Context, series: _native.KrrSeries, params: _native.KrrPercentileParams,
                              ext_slots: Optional[int] = None, group=None, stream=None, events=None,
                              key_cap: Optional[int] = None) -> dict:
    """Exact SORTED_LOWER / LINEAR percentile of every time-sharded series in ONE pass over
    this rank's slices (module docstring).  ``series``: this rank's slice of every series
    (the same series on every rank, rank order = time order).  ``ext_slots``: slots of a
    series held by the other ranks (default (world - 1) x the longest local slice); it
    only sizes the windows, results are exact whatever it is.  Returns device tensors
    value/count/flags for this rank's owner block (``owner_blocks``), plus 'block',
    'misses' (series of the block finished by regathering their slices), 'key_cap' and
    'exchanged_bytes' (what this rank sent in the all-to-all) and 'hdr' (this rank's
    exported krr_window_hdr rows, int64 [S, HDR_WORDS]).  ``events``: optional pair
    of HIP events recorded around the export pass (its HBM time).

    ``series`` may also be a list of (lo, hi, KrrSeries) parts, series [lo, hi) of the rank
    in buffers of their own: one export launch per part, consecutive launches alternating
    between ``stream`` and a second stream (one part's drain overlaps the next one's start;
    launches over a few GiB stream faster than one over a whole 138-GB allocation)."""
    import torch

    dev = _parts(series)[0][2]._keep[0].device
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    # every allocation, copy and collective below is ordered on st (the caching allocator
    # then recycles a buffer only after st has used it)
    with torch.cuda.stream(st):
        return _window_exact_body(ctx, series, params, ext_slots, group, st, events, key_cap)


def _window_exact_body(ctx, series, params, ext_slots, group, st, events, key_cap):
    import torch
    import torch.distributed as dist

    parts = _parts(series)
    S = parts[-1][1]
    dev = parts[0][2]._keep[0].device
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    Lmax = max(_max_len(ser) for _, _, ser in parts)
    if ext_slots is None:
        ext_slots = (world - 1) * Lmax
    kc = int(key_cap or _native.window_key_cap(max(Lmax, 1), ext_slots, params))
    per = -(-S // world) if S else 0
    rows = per * world
    hdr = torch.empty((max(rows, 1), _native.HDR_WORDS), dtype=torch.int64, device=dev)
    keys = torch.empty((max(rows, 1), kc), dtype=torch.int64, device=dev)
    if events is not None:
        events[0].record(st)
    side = None
    if len(parts) > 1:
        side = _side_stream(dev)
        side.wait_stream(st)
    for j, (lo, hi, ser) in enumerate(parts):
        if hi > lo:
            ctx.window_export(ser, params, ext_slots, kc, hdr[lo:hi], keys[lo:hi], side if (side and j % 2) else st)
    if side is not None:
        st.wait_stream(side)
    if events is not None:
        events[1].record(st)
    lo, hi = owner_blocks(S, world)[rank] if world > 1 else (0, S)
    nb = hi - lo
    if world > 1:
        coll = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
        hdr_r = torch.empty((rows, _native.HDR_WORDS), dtype=torch.int64, device=coll)
        keys_r = torch.empty((rows, kc), dtype=torch.int64, device=coll)
        if rows:
            dist.all_to_all_single(hdr_r, hdr[:rows].to(coll), group=group)
            dist.all_to_all_single(keys_r, keys[:rows].to(coll), group=group)
        hdr_r, keys_r = hdr_r.to(dev), keys_r.to(dev)
        stride = per
        sent = (rows - per) * (_native.HDR_WORDS + kc) * 8
    else:
        hdr_r, keys_r, stride, sent = hdr, keys, max(S, 1), 0
    out = {"value": torch.empty(max(nb, 1), dtype=torch.float64, device=dev)[:nb],
           "count": torch.empty(max(nb, 1), dtype=torch.int64, device=dev)[:nb],
           "flags": torch.empty(max(nb, 1), dtype=torch.int32, device=dev)[:nb]}
    miss = torch.zeros(1, dtype=torch.int32, device=dev)
    # a series holds at most this rank's longest slice plus the slots elsewhere (ext_slots)
    ctx.window_merge(nb, world, stride, hdr_r, keys_r, kc, params, out["value"], out["count"], out["flags"], miss,
                     st, max_n=(Lmax + ext_slots) if _needs_table(params) else None)
    nmiss = int(miss.item())
    total = nmiss
    if world > 1:
        coll = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
        t = torch.tensor([nmiss], dtype=torch.int64, device=coll)
        dist.all_reduce(t, group=group)
        total = int(t.item())
    if total:
        finish_window_misses(ctx, parts, params, out, (lo, hi), group, st)
    out.update(block=(lo, hi), misses=nmiss, key_cap=kc, exchanged_bytes=sent, hdr=hdr[:S])
    return out


def finish_window_misses(ctx: _native.Context, series: _native.KrrSeries, params: _native.KrrPercentileParams,
                         out: dict, block, group=None, stream=None) -> None:
    """The series ``krr_window_merge`` flagged KRR_FLAG_WINDOW_MISS in ``out`` (this rank's
    owner block): their slices are regathered to the owner (RCCL all-to-all) and selected
    whole with ``krr_segmented_percentile``; ``out`` is updated in place.  Collective: every
    rank calls it (with or without misses of its own)."""
    import torch
    import torch.distributed as dist

    parts = _parts(series)
    gaps = parts[0][2].gaps_are_nan
    dev = parts[0][2]._keep[0].device
    S = parts[-1][1]
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    lo, _ = block
    mine = torch.nonzero((out["flags"] & _native.KRR_FLAG_WINDOW_MISS) != 0).flatten()
    if world == 1:
        ids = mine
        if ids.numel() == 0:
            return
        sv, so = gather_segments_parts(parts, ids)
        sub = ctx.series(sv, so, 0, gaps)
        v = torch.empty(ids.numel(), dtype=torch.float64, device=dev)
        n = torch.empty(ids.numel(), dtype=torch.int64, device=dev)
        f = torch.empty(ids.numel(), dtype=torch.int32, device=dev)
        ctx.segmented_percentile(sub, params, v, n, f, stream)
        out["value"][ids], out["count"][ids], out["flags"][ids] = v, n, f
        return
    # every rank learns every owner's missed series (global ids, ascending)
    lists = [None] * world
    dist.all_gather_object(lists, (mine + lo).tolist(), group=group)
    blocks = owner_blocks(S, world)
    per_owner = [torch.tensor(sorted(x), dtype=torch.int64, device=dev) for x in lists]
    ids_all = torch.cat(per_owner) if any(len(x) for x in lists) else torch.empty(0, dtype=torch.int64, device=dev)
    if ids_all.numel() == 0:
        return
    # this rank's slices of them, grouped by owner (= ascending id)
    sv, so = gather_segments_parts(parts, ids_all)
    lens = (so[1:] - so[:-1])
    coll = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
    counts = [len(x) for x in lists]
    send_sizes = [int(lens[sum(counts[:r]):sum(counts[:r + 1])].sum().item()) for r in range(world)]
    # every rank's slice lengths of every missed series: [world, n_missed]
    all_lens = [torch.empty_like(lens, device=coll) for _ in range(world)]
    dist.all_gather(all_lens, lens.to(coll), group=group)
    rank = dist.get_rank(group)
    a, b = sum(counts[:rank]), sum(counts[:rank + 1])
    recv_lens = torch.stack([x[a:b] for x in all_lens]).to(dev)  # [src, my missed series]
    recv_sizes = [int(x) for x in recv_lens.sum(dim=1).tolist()]
    recv = torch.empty(max(sum(recv_sizes), 1), dtype=torch.float64, device=coll)
    dist.all_to_all_single(recv[:sum(recv_sizes)], sv[:int(so[-1].item())].to(coll), output_split_sizes=recv_sizes,
                           input_split_sizes=send_sizes, group=group)
    k = b - a
    if k == 0:
        return
    recv = recv.to(dev)
    # src-major pieces -> series-major, src (= time) order inside each series
    flat = recv_lens.reshape(-1)
    src_start = torch.cumsum(flat, 0) - flat
    tot = recv_lens.sum(dim=0)
    new_offs = torch.zeros(k + 1, dtype=torch.int64, device=dev)
    new_offs[1:] = torch.cumsum(tot, 0)
    dst_start = (new_offs[:-1][None, :] + (torch.cumsum(recv_lens, 0) - recv_lens)).reshape(-1)
    n_all = int(new_offs[-1].item())
    whole = torch.empty(max(n_all, 1), dtype=torch.float64, device=dev)
    if n_all:
        piece = torch.repeat_interleave(torch.arange(flat.numel(), device=dev), flat)
        pos = torch.arange(n_all, device=dev)
        whole[dst_start[piece] + (pos - src_start[piece])] = recv[:n_all]
    sub = ctx.series(whole, new_offs, 0, gaps)
    v = torch.empty(k, dtype=torch.float64, device=dev)
    n = torch.empty(k, dtype=torch.int64, device=dev)
    f = torch.empty(k, dtype=torch.int32, device=dev)
    ctx.segmented_percentile(sub, params, v, n, f, stream)
    loc = per_owner[rank] - blocks[rank][0]
    out["value"][loc], out["count"][loc], out["flags"][loc] = v, n, f


# ------------------------- KLL sketch (row format 2) -------------------------

@dataclass(frozen=True)
class KllConfig:
    """``budget`` body keys kept per row, ``tail`` exact top keys per row (a rank within
    ``tail`` of the top is answered exactly), ``seed`` drives the compaction coins, so a run
    is reproducible (and checkable against oracle/kll_ref.py)."""
    budget: int = 512
    tail: int = 0
    seed: int = 0x4B4C4C5345454431
    one_pass_tail: bool = False  # KRR_KLL_ONE_PASS_TAIL: the tail inside the build (same rows)
    tail_flags: int = 0          # further krr_kll_params.reserved bits (testing)
    # the tail pass reads only the 128-B lines whose maximum (recorded by the body build) can
    # hold a tail key (krr_kll_build_lines / krr_kll_tail_lines; same rows); False: the tail
    # pass streams the whole slice again (krr_kll_tail)
    sparse_tail: bool = True

    def params(self, slice_id: int = 0) -> _native.KrrKllParams:
        flags = self.tail_flags | (_native.KRR_KLL_ONE_PASS_TAIL if self.one_pass_tail else 0)
        return _native.KrrKllParams(self.budget, int(slice_id), self.seed & (2 ** 64 - 1), self.tail, flags)

    @property
    def row_words(self) -> int:
        return 16 + self.budget + self.tail

    @staticmethod
    def tail_for(n_total: int, percentile, mode: str = "linear") -> int:
        """The smallest tail (a multiple of 64) that answers ``percentile`` of an ``n_total``-sample
        series exactly: it must hold every rank from the asked one (and LINEAR's next) to n - 1.
        0 when that is more than a row can hold (4,096): a tail that cannot cover the asked rank
        would cost its pass for nothing, and the body answers it within its bound."""
        from fractions import Fraction

        if n_total <= 0:
            return 0
        p = Fraction(str(percentile))
        r0 = int((n_total - 1) * p / 100)  # floor: SORTED_LOWER's rank, LINEAR's lower one
        need = -(-(n_total - r0) // 64) * 64
        return int(need) if need <= 4096 else 0


def kll_build(ctx: _native.Context, series, cfg: KllConfig, slice_id: int = 0, seg_base: int = 0,
              stream=None, events=None, stats: Optional[dict] = None):
    """int64 [S, row_words] rows of this rank's slice of every series: one HBM pass for the
    body, and (tail > 0) the tail pass over the slice again (krr_kll_tail; one pass in all with
    ``cfg.one_pass_tail``).  ``series``: a KrrSeries, or (lo, hi, KrrSeries) parts in buffers
    of their own.  ``events`` (3 HIP events, optional): recorded on ``stream`` before the body
    launches, between them and the tail launches, and after.  ``stats`` (optional dict, sparse
    tail pass): gets ``lines_read`` (int32 [S] device tensor: 128-B lines the tail pass read per
    series) and ``line_words`` (uint32 words of line maxima written per series)."""
    import torch

    parts = _parts(series)
    if not parts:
        raise ValueError("kll_build needs a KrrSeries or at least one (lo, hi, KrrSeries) part")
    S = parts[-1][1]
    dev = parts[0][2]._keep[0].device
    rows = torch.empty((max(S, 1), cfg.row_words), dtype=torch.int64, device=dev)
    kp = cfg.params(slice_id)
    split = cfg.tail > 0 and not cfg.one_pass_tail
    if split:  # every body launch first, then every tail launch (timed apart)
        kp.reserved |= _native.KRR_KLL_BODY_ONLY
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    sparse = split and cfg.sparse_tail
    lines = {}
    if sparse:  # per part: its line maxima, written by the body build, read by the tail pass
        for lo, hi, ser in parts:
            if hi > lo:
                stride = ctx.kll_line_words(_max_len(ser))
                lines[lo] = (torch.empty((hi - lo) * stride, dtype=torch.int32, device=dev), stride)
    if events is not None:
        events[0].record(st)
    for lo, hi, ser in parts:
        if hi > lo:
            if sparse:
                ctx.kll_build_lines(ser, kp, rows[lo:hi], *lines[lo], seg_base=seg_base + lo, stream=st)
            else:
                ctx.kll_build(ser, kp, rows[lo:hi], seg_base=seg_base + lo, stream=st)
    if events is not None:
        events[1].record(st)
    read = torch.zeros(max(S, 1), dtype=torch.int32, device=dev) if (sparse and stats is not None) else None
    if stats is not None and sparse:
        stats["lines_read"] = read[:S]
        stats["line_words"] = {lo: lw[1] for lo, lw in lines.items()}
    if split:
        for lo, hi, ser in parts:
            if hi > lo:
                if sparse:
                    ctx.kll_tail_lines(ser, kp, rows[lo:hi], *lines[lo],
                                       lines_read=None if read is None else read[lo:hi], stream=st)
                else:
                    ctx.kll_tail(ser, kp, rows[lo:hi], stream=st)
    if events is not None:
        events[2].record(st)
    return rows[:S]


def _max_len(ser) -> int:
    """A KrrSeries' longest segment (its max_segment_len, or from its offsets)."""
    if int(ser.max_segment_len) > 0:
        return int(ser.max_segment_len)
    offs = ser._keep[1]
    return int((offs[1:] - offs[:-1]).max().item()) if offs.numel() > 1 else 0


def kll_exchange(rows, group=None):
    """The W slice rows of each series of this rank's owner block (``owner_blocks``), as
    int64 [n_block * W, row_words] series-major (one all-to-all).  World size 1: ``rows``."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return rows, 1
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    S, RW = rows.shape
    per = -(-S // world) if S else 0
    dev = rows.device
    coll = dev if dist.get_backend(group) == "nccl" else torch.device("cpu")
    send = torch.zeros((per * world, RW), dtype=torch.int64, device=dev)
    send[:S] = rows
    recv = torch.empty((per * world, RW), dtype=torch.int64, device=coll)
    if per:
        dist.all_to_all_single(recv, send.to(coll), group=group)
    lo, hi = owner_blocks(S, world)[rank]
    # recv[v * per + i] = rank v's slice of series lo + i: to series-major [i][v]
    merged = recv.to(dev).view(world, per, RW)[:, : hi - lo].transpose(0, 1).contiguous()
    return merged.view((hi - lo) * world, RW), world


def kll_merge(ctx: _native.Context, rows, rows_per_series: int, cfg: KllConfig, series_base: int = 0,
              epoch: int = 0, stream=None):
    """Fold each series' W rows (series-major, time order) into ONE row of the same format
    (krr_kll_merge; coins keyed by (seed, series_base + s, epoch, w)).  W == 1: ``rows``."""
    import torch

    W = max(int(rows_per_series), 1)
    if W == 1:
        return rows
    n = rows.shape[0] // W
    out = torch.empty((max(n, 1), cfg.row_words), dtype=torch.int64, device=rows.device)[:n]
    if n:
        ctx.kll_merge(rows, W, cfg.params(epoch), out, series_base=series_base, stream=stream)
    return out


def kll_query(ctx: _native.Context, rows, rows_per_series: int, cfg: KllConfig,
              params: _native.KrrPercentileParams, series_base: int = 0, epoch: int = 0, stream=None) -> dict:
    import torch

    n = rows.shape[0] // max(rows_per_series, 1)
    dev = rows.device
    out = {"value": torch.empty(max(n, 1), dtype=torch.float64, device=dev)[:n],
           "count": torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n],
           "flags": torch.empty(max(n, 1), dtype=torch.int32, device=dev)[:n]}
    if n:
        max_n = None
        if _needs_table(params):  # row word 0 = the row's present count (oracle/kll_ref.py)
            max_n = int(rows.view(n, max(rows_per_series, 1), -1)[:, :, 0].sum(dim=1).max().item())
        ctx.kll_query(rows, rows_per_series, cfg.params(epoch), params, out["value"], out["count"], out["flags"],
                      series_base=series_base, stream=stream, max_n=max_n)
    return out


def kll_time_sharded(ctx: _native.Context, series, cfg: KllConfig, params: _native.KrrPercentileParams,
                     group=None, stream=None, events=None, stats: Optional[dict] = None) -> dict:
    """Sketch-only percentile of every time-sharded series: build (one pass over this
    rank's slices; slice id = rank) -> all-to-all of the rows -> fold each series' rows into
    one (krr_kll_merge) -> query on the owner.  value/count/flags of this rank's owner block,
    plus 'block' and 'rows' (the owner's folded rows, one per series, for ``kll_rank_bound``).
    Everything runs on ``stream`` (or the current stream)."""
    import torch
    import torch.distributed as dist

    dev = _parts(series)[0][2]._keep[0].device
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    with torch.cuda.stream(st):
        # events (optional, 3): before the body pass, between it and the tail pass, after
        rows = kll_build(ctx, series, cfg, slice_id=rank, stream=st, events=events, stats=stats)
        S = rows.shape[0]
        lo, hi = owner_blocks(S, world)[rank] if world > 1 else (0, S)
        gathered, W = kll_exchange(rows, group)
        merged = kll_merge(ctx, gathered, W, cfg, series_base=lo, stream=st)
        out = kll_query(ctx, merged, 1, cfg, params, series_base=lo, stream=st)
    out.update(block=(lo, hi), rows=merged, rows_per_series=1)
    return out


def kll_rank_bound(rows, rows_per_series: int = 1, delta: float = 0.01) -> np.ndarray:
    """Per series (one folded row each; fold them first with ``kll_merge`` when W > 1), the
    normalised rank-error bound of BODY answers that holds with probability >= 1 - delta:
    sqrt(2 ln(4/delta) sum w^2) / n, sum w^2 from row word 4.

    Why: a compaction of weight-w keys changes the weighted count of kept keys <= x, for a
    FIXED x, by 0 or +-w, with conditional mean zero given every earlier coin — martingale
    differences.  Their bounds w are FIXED in advance: every compaction takes an even number
    of keys (an odd one is set aside), so which compactions happen, and at what weight,
    depends on the input's presence pattern only.  Azuma-Hoeffding then gives
    |error(x)| <= t = sqrt(2 ln(4/delta) sum w^2) except with probability delta/2, at
    x_lo (the largest value of true count <= r - t) and x_hi (the smallest of true count
    > r + t); on both events the answer (the smallest kept key of estimated count > r; the
    total weight is exactly n) lies in (x_lo, x_hi], so its rank interval meets [r - t, r + t]
    (DESIGN.md §8).  Ranks within the row's exact tail (n - r <= word 6) have no error.
    NaN for empty series."""
    if int(rows_per_series) != 1:
        raise ValueError("fold the rows first (kll_merge): the bound is read from one row per series")
    h = rows[:, :16].cpu().numpy().astype(np.uint64)
    n = h[:, 0].astype(np.float64)
    w2 = h[:, 4].astype(np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.sqrt(2.0 * np.log(4.0 / delta) * w2) / n


def kll_tail_covers(rows, rank: np.ndarray) -> np.ndarray:
    """Per series, whether ``rank`` (0-based ascending) is answered from the exact tail."""
    h = rows[:, :16].cpu().numpy().astype(np.int64)
    return (h[:, 0] - np.asarray(rank, dtype=np.int64)) <= h[:, 6]
