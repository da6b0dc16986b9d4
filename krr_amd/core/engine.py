"""Device engine: moves a PackedFleet to HBM, runs the SimpleStrategy kernels
through the C ABI, and returns the raw per-object results.

There is no CPU path: ``SimpleEngine`` raises NativeUnavailable when the HIP
library or a device is missing.  One krr_ctx per (thread, device) keeps the
ABI's "one ctx per thread" rule while the reference's runner calls strategies
from a thread pool (runner.py:104-106).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Optional

import numpy as np

from krr_amd import _native
from krr_amd.core.packing import PackedFleet, PackedSeries

MODE_CODES = {"ref_index": _native.KRR_PCT_REF_INDEX, "sorted_lower": _native.KRR_PCT_SORTED_LOWER,
              "linear": _native.KRR_PCT_LINEAR}


def percentile_params(percentile, mode: str) -> _native.KrrPercentileParams:
    """The kernels' percentile parameters for any ``cpu_percentile`` the reference accepts.

    The index rule k(n) (REF_INDEX, SORTED_LOWER) is the reference's int((n-1) * p / 100)
    (simple.py:36) evaluated as it evaluates it (krr_amd.core.index_rule): the kernels'
    128-bit exact floor of p_num / p_den where that provably agrees, else a table of k(n)
    that ``_native`` binds at launch time (``params.rule``, sized by the launch's longest
    segment).  q = float(p) / 100 is numpy's LINEAR rule.
    """
    from krr_amd.core.index_rule import IndexRule

    if mode not in MODE_CODES:
        raise ValueError(f"unknown percentile mode {mode!r}; expected one of {sorted(MODE_CODES)}")
    rule = IndexRule.of(percentile)
    p_num, p_den = rule.approx()
    q = float(percentile) / 100.0
    params = _native.KrrPercentileParams(MODE_CODES[mode], 0, p_num, p_den, q)
    params.rule = rule
    return params


@dataclass
class RawResults:
    """Per-object raw proposals as the kernels return them (host numpy arrays)."""
    cpu_value: np.ndarray
    cpu_count: np.ndarray
    cpu_flags: np.ndarray
    mem_value: np.ndarray
    mem_count: np.ndarray
    mem_flags: np.ndarray
    # HistoryData segments whose Decimals the float64 values do not reproduce
    # (PackedSeries.exact): krr_locate's answers ({"cpu"|"mem": (lt, eq, pos)}, int64 [S]
    # each, -1 where not located), then krr_amd.core.exact.resolve's object index -> the
    # reference's own sample object (CPU proposal / memory max before the buffer)
    locate: Optional[dict] = None
    cpu_exact: Optional[dict] = None
    mem_exact: Optional[dict] = None


class SimpleEngine:
    def __init__(self, device: int = 0):
        self.device = int(device)
        self._tls = threading.local()

    def context(self) -> _native.Context:
        ctx = getattr(self._tls, "ctx", None)
        if ctx is None:
            ctx = _native.Context(self.device)
            self._tls.ctx = ctx
        return ctx

    def _to_device(self, ps: PackedSeries):
        import torch

        dev = torch.device("cuda", self.device)
        if isinstance(ps.values, torch.Tensor) and ps.values.is_cuda:  # already in HBM (device packer)
            if ps.values.device != dev or ps.offsets.device != dev:
                # packed on another GPU: the kernels read only this ctx's HBM
                raise ValueError(f"series packed on {ps.values.device}, engine runs on {dev}: pack on the "
                                 f"engine's device (or copy the fleet there first)")
            return ps.values, ps.offsets
        host = torch.from_numpy(np.ascontiguousarray(ps.values, dtype=np.float64))
        # page-locked values (pinned_alloc) go by DMA without blocking the host; the
        # caller synchronises before the host buffer is released
        vals = host.to(dev, non_blocking=host.is_pinned())
        offs = torch.from_numpy(np.ascontiguousarray(ps.offsets, dtype=np.int64)).to(dev, non_blocking=False)
        return vals, offs

    def run_device(self, cpu_vals, cpu_offs, mem_vals, mem_offs, params: _native.KrrPercentileParams,
                   cpu_max_len: int = 0, mem_max_len: int = 0, gaps_are_nan: bool = False,
                   out: Optional[dict] = None, stream=None) -> dict:
        """All inputs already in HBM (torch tensors).  Returns the device output dict."""
        import torch

        ctx = self.context()
        S = cpu_offs.numel() - 1
        dev = cpu_vals.device
        if out is None:
            out = {
                "cpu_value": torch.empty(S, dtype=torch.float64, device=dev),
                "cpu_count": torch.empty(S, dtype=torch.int64, device=dev),
                "cpu_flags": torch.empty(S, dtype=torch.int32, device=dev),
                "mem_value": torch.empty(S, dtype=torch.float64, device=dev),
                "mem_count": torch.empty(S, dtype=torch.int64, device=dev),
                "mem_flags": torch.empty(S, dtype=torch.int32, device=dev),
            }
        cs = ctx.series(cpu_vals, cpu_offs, cpu_max_len, gaps_are_nan)
        ms = ctx.series(mem_vals, mem_offs, mem_max_len, gaps_are_nan)
        ctx.simple_run(cs, ms, params, out, stream=stream)
        return out

    def run_packed(self, fleet: PackedFleet, params: _native.KrrPercentileParams) -> RawResults:
        import torch

        if fleet.cpu.n_segments != fleet.mem.n_segments:
            raise ValueError("cpu and memory need one segment per object each")
        self.context()  # raises NativeUnavailable without the HIP library or a device
        if fleet.n_objects == 0:
            e = np.zeros(0)
            return RawResults(e, e.astype(np.int64), e.astype(np.uint32), e, e.astype(np.int64),
                              e.astype(np.uint32))
        from krr_amd.core.distributed import unpack_records

        S = fleet.n_objects
        locate = needs_locate(fleet, params)
        with torch.cuda.device(self.device):
            # the launch writes the 32-B records straight into page-locked host memory
            # (krr_simple_run_records with a mapped host buffer): one sync, no D2H copies
            rec = torch.empty((S, 4), dtype=torch.int64, pin_memory=True)
            loc = self._run_chunks(fleet, params, rec, locate=locate)
            torch.cuda.current_stream(self.device).synchronize()
        host = unpack_records(rec.numpy())
        return RawResults(host["cpu_value"], host["cpu_count"], host["cpu_flags"], host["mem_value"],
                          host["mem_count"], host["mem_flags"], loc)


    def run_packed_records(self, fleet: PackedFleet, params: _native.KrrPercentileParams):
        """The fused kernel pass over a (shard of a) fleet, returning its 32-B result
        records as an int64 [S, 4] device tensor (krr_simple_run_records: written by the
        same launch) on the current stream — what a rank sends to rank 0."""
        import torch

        if fleet.cpu.n_segments != fleet.mem.n_segments:
            raise ValueError("cpu and memory need one segment per object each")
        self.context()
        S = fleet.n_objects
        dev = torch.device("cuda", self.device)
        rec = torch.empty((S, 4), dtype=torch.int64, device=dev)
        if S == 0:
            return rec
        with torch.cuda.device(self.device):
            self._run_chunks(fleet, params, rec)
            # the host buffers may be pinned and released by the caller: finish the copies
            torch.cuda.current_stream(self.device).synchronize()
        return rec

    # a fleet of more than 2 chunks of values runs as chunks of about this many bytes
    # (both resources), each uploaded into buffers of its own and launched on its own:
    # HBM holds one chunk at a time, and big single launches stream slower
    # (profiles/r02/footprint)
    chunk_bytes = 16 << 30

    def _run_chunks(self, fleet: PackedFleet, params: _native.KrrPercentileParams, rec,
                    locate: bool = False) -> Optional[dict]:
        """Upload + fused launch per chunk of objects, records rows into ``rec`` (device or
        page-locked host), all on the current stream: a chunk's device buffers are released
        to the caching allocator after its launch is enqueued, which reuses them in stream
        order for the next chunk.  ``locate``: also krr_locate over each chunk's segments of
        exactness class >= 1 (``_locate_chunk``); returns its answers, else None."""
        import torch

        from krr_amd.core.distributed import fleet_shard_bounds, slice_fleet

        S = fleet.n_objects
        nbytes = 8 * (int(fleet.cpu.offsets[-1]) + int(fleet.mem.offsets[-1]))
        resident = isinstance(fleet.cpu.values, torch.Tensor) and fleet.cpu.values.is_cuda
        n = 1 if resident or nbytes <= 2 * self.chunk_bytes else -(-nbytes // self.chunk_bytes)
        bounds = [(0, S)] if n == 1 else [(lo, hi) for lo, hi in fleet_shard_bounds(fleet, n) if hi > lo]
        ctx = self.context()
        dev = torch.device("cuda", self.device)
        out = {k: torch.empty(S, dtype=dt, device=dev) for k, dt in
               (("cpu_value", torch.float64), ("cpu_count", torch.int64), ("cpu_flags", torch.int32),
                ("mem_value", torch.float64), ("mem_count", torch.int64), ("mem_flags", torch.int32))}
        loc = {r: tuple(np.full(S, -1, dtype=np.int64) for _ in range(3)) for r in ("cpu", "mem")} if locate else None
        for lo, hi in bounds:
            part = fleet if (lo, hi) == (0, S) else slice_fleet(fleet, lo, hi)
            cv, co = self._to_device(part.cpu)
            mv, mo = self._to_device(part.mem)
            cs = ctx.series(cv, co, max(part.cpu.max_len, 1), part.cpu.gaps_are_nan)
            ms = ctx.series(mv, mo, max(part.mem.max_len, 1), part.mem.gaps_are_nan)
            chunk_out = {k: v[lo:hi] for k, v in out.items()}
            ctx.simple_run(cs, ms, params, chunk_out, records=rec[lo:hi])
            if locate:
                self._locate_chunk(ctx, part, cs, ms, params, chunk_out, loc, lo)
        return loc

    def _locate_chunk(self, ctx, part: PackedFleet, cs, ms, params, out: dict, loc: dict, lo: int) -> None:
        """krr_locate for the chunk's class >= 1 segments that select one sample: memory
        (rank -1: the first maximal element, simple.py:29) and SORTED_LOWER CPU (rank k of
        the stable sort).  REF_INDEX needs no search (its position IS k) and LINEAR is defined
        on the float64 values.  Synchronises the stream (the ranks come from the counts)."""
        import torch

        torch.cuda.current_stream(self.device).synchronize()
        dev = torch.device("cuda", self.device)
        for name, ps, series in (("cpu", part.cpu, cs), ("mem", part.mem, ms)):
            if ps.exact is None:
                continue
            rank = locate_ranks(name, ps.exact, out[f"{name}_count"].cpu().numpy(),
                                out[f"{name}_flags"].cpu().numpy(), params)
            if rank is None:
                continue
            rank_d = torch.from_numpy(rank).to(dev)
            lt, eq, pos = (torch.full_like(rank_d, -1) for _ in range(3))
            ctx.locate(series, out[f"{name}_value"], rank_d, lt, eq, pos)
            for dst, src in zip(loc[name], (lt, eq, pos)):
                dst[lo:lo + src.numel()] = src.cpu().numpy()


def locate_ranks(name: str, exact: np.ndarray, count: np.ndarray, flags: np.ndarray, params) -> Optional[np.ndarray]:
    """krr_locate's rank per segment ("cpu" | "mem"): -1 (the first maximal sample) for memory,
    k = floor((n-1)·p/100) for SORTED_LOWER CPU, on class >= 1 segments holding >= 2 samples and
    no NaN (those answer by the NaN rules); -2 (skip) elsewhere.  None: nothing to locate."""
    if name == "cpu" and params.mode != _native.KRR_PCT_SORTED_LOWER:
        return None
    flags = np.asarray(flags).astype(np.uint32)
    ok = (np.asarray(exact) > 0) & (flags & (_native.KRR_FLAG_EMPTY | _native.KRR_FLAG_NAN) == 0) & (count >= 2)
    if not ok.any():
        return None
    rank = np.full(count.size, -2, dtype=np.int64)
    if name == "mem":
        rank[ok] = -1
    else:
        rank[ok] = index_rule_of(params).ks(np.asarray(count)[ok])
    return rank


def index_rule_of(params):
    """The IndexRule a params struct carries (percentile_params), or the exact p_num / p_den one."""
    rule = getattr(params, "rule", None)
    if rule is None:
        from fractions import Fraction

        from krr_amd.core.index_rule import IndexRule

        rule = IndexRule.of(Fraction(int(params.p_num), int(params.p_den)))
    return rule


def needs_locate(fleet: PackedFleet, params) -> bool:
    """Does a fleet hold HistoryData segments whose answer must be located (krr_locate)?"""
    return fleet.cpu.exact is not None and params.mode == _native.KRR_PCT_SORTED_LOWER or fleet.mem.exact is not None


def pinned_alloc(n: int) -> np.ndarray:
    """float64[n] in page-locked host memory (a numpy view that keeps its torch
    tensor alive): pass as ``alloc`` to the packers so the H2D copy runs by DMA."""
    import torch

    return torch.empty(max(int(n), 1), dtype=torch.float64, pin_memory=True).numpy()[: int(n)]


_default_engines: dict[int, SimpleEngine] = {}
_engines_lock = threading.Lock()


def default_engine(device: int = 0) -> SimpleEngine:
    with _engines_lock:
        eng = _default_engines.get(device)
        if eng is None:
            eng = _default_engines[device] = SimpleEngine(device)
        return eng
