"""Multi-GPU fleet sharding and result collection (one process per GPU).

Objects are independent (runner.py:110-112; simple.py:42-49 reads only its own
object), so a fleet shards into contiguous object ranges with no data-path
collective.  Each rank runs the kernels on its shard; the only exchange is the
per-object result records (32 B each) gathered to rank 0 — over RCCL/xGMI when
the process group is "nccl" (= RCCL on ROCm), over gloo in the CPU tests.

Record layout (int64[4] per object, 32 B):
  [0] cpu value bits (float64 bit pattern)   [1] mem value bits
  [2] cpu count | cpu flags << 48            [3] mem count | mem flags << 48
"""
from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np

RECORD_WORDS = 4
_COUNT_MASK = (1 << 48) - 1


def shard_bounds(samples_per_object: Sequence[int] | np.ndarray, world_size: int) -> list[tuple[int, int]]:
    """Cut objects [0, S) into world_size contiguous ranges with ~equal sample counts.

    Cuts fall on object boundaries: rank r gets the objects whose sample prefix
    starts in [r*T/W, (r+1)*T/W).  Every object lands in exactly one shard.
    """
    w = np.asarray(samples_per_object, dtype=np.int64)
    S = int(w.size)
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    if S == 0:
        return [(0, 0)] * world_size
    prefix = np.concatenate([[0], np.cumsum(w)])
    total = int(prefix[-1])
    if total == 0:  # no samples anywhere: split by object count
        cuts = [(S * r) // world_size for r in range(world_size + 1)]
    else:
        targets = [(total * r) // world_size for r in range(world_size + 1)]
        cuts = [int(np.searchsorted(prefix[:-1], t, side="left")) for t in targets]
        cuts[0], cuts[-1] = 0, S
        for r in range(1, world_size + 1):  # monotone
            cuts[r] = max(cuts[r], cuts[r - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world_size)]


def pack_records(out: dict):
    """Device tensors from SimpleEngine.run_device -> one int64 [S, 4] tensor."""
    import torch

    cv = out["cpu_value"].view(torch.int64)
    mv = out["mem_value"].view(torch.int64)
    cc = out["cpu_count"] | (out["cpu_flags"].to(torch.int64) << 48)
    mc = out["mem_count"] | (out["mem_flags"].to(torch.int64) << 48)
    return torch.stack([cv, mv, cc, mc], dim=1).contiguous()


def records_from_raw(raw, device):
    """Host RawResults -> the int64 [S, 4] records on ``device`` (pack_records' layout)."""
    import torch

    cols = {k: torch.from_numpy(np.ascontiguousarray(getattr(raw, k))) for k in ("cpu_value", "mem_value")}
    for k in ("cpu_count", "mem_count", "cpu_flags", "mem_flags"):
        cols[k] = torch.from_numpy(np.ascontiguousarray(getattr(raw, k), dtype=np.int64))
    return pack_records(cols).to(device)


def unpack_records(rec) -> dict:
    """int64 [S, 4] (tensor or array) -> host numpy arrays of the six result fields."""
    a = rec.cpu().numpy() if hasattr(rec, "cpu") else np.asarray(rec)
    a = np.ascontiguousarray(a, dtype=np.int64).reshape(-1, RECORD_WORDS)
    return {
        "cpu_value": a[:, 0].copy().view(np.float64),
        "mem_value": a[:, 1].copy().view(np.float64),
        "cpu_count": a[:, 2] & _COUNT_MASK,
        "cpu_flags": (a[:, 2] >> 48).astype(np.uint32),
        "mem_count": a[:, 3] & _COUNT_MASK,
        "mem_flags": (a[:, 3] >> 48).astype(np.uint32),
    }


def record_counts(n_local: int, device, group=None) -> list[int]:
    """Every rank's record count (one all_gather of an int64; host sync)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = torch.tensor([n_local], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    return [int(c.item()) for c in counts]


class PendingGather:
    """An in-flight ``gather_records(..., async_op=True)``: ``wait()`` makes the
    current stream wait for the collective and returns what the blocking call would."""

    def __init__(self, work, flat, counts):
        self._work, self._flat, self._counts = work, flat, counts

    def wait(self):
        self._work.wait()
        return _assemble(self._flat, self._counts)


def _assemble(flat, counts):
    """[world * width, 4] receive buffer -> the [sum n_r, 4] fleet (a view when no rank is padded)."""
    if flat is None:
        return None
    import torch

    width = flat.shape[0] // max(len(counts), 1)
    if all(c == width for c in counts):
        return flat
    return torch.cat([flat[r * width: r * width + c] for r, c in enumerate(counts)], dim=0)


def gather_records(local, dst: int = 0, group=None, counts: Optional[list] = None, async_op: bool = False,
                   copy_local: bool = True):
    """Gather every rank's [n_r, 4] records to rank `dst` (a rank of `group`),
    concatenated in rank order.

    Ranks may hold different n_r: counts are exchanged first (``record_counts``,
    one all_gather of a single int64 and a host sync — pass ``counts`` to reuse
    them when the shard sizes do not change between calls), shards are padded to
    the max, gathered in ONE collective into one contiguous [world * max, 4]
    buffer on dst, and trimmed there (no copy when no rank is padded).  Returns
    the [sum n_r, 4] tensor on dst, None elsewhere — or, with ``async_op``, a
    PendingGather whose ``wait()`` returns it.  By default ``local`` is copied
    before the collective starts, so the caller may overwrite it at once; with
    ``copy_local=False`` an unpadded shard is sent straight from ``local``, which
    the caller must then leave untouched until ``wait()`` (bench.py alternates
    two record buffers).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)  # group-local, like dst
    gdst = dist.get_global_rank(group, dst) if group is not None else dst  # torch's gather takes a global rank
    dev = local.device
    if counts is None:
        counts = record_counts(local.shape[0], dev, group)
    width = max(max(counts), 1)
    if not copy_local and local.shape[0] == width and local.is_contiguous():
        send = local
    else:
        # one copy kernel for an unpadded shard; only the padding rows are zeroed
        send = torch.empty((width, RECORD_WORDS), dtype=torch.int64, device=dev)
        if local.shape[0]:
            send[: local.shape[0]] = local
        if local.shape[0] < width:
            send[local.shape[0]:].zero_()
    flat = torch.empty((world * width, RECORD_WORDS), dtype=torch.int64, device=dev) if rank == dst else None
    bufs = [flat[r * width:(r + 1) * width] for r in range(world)] if flat is not None else None
    work = dist.gather(send, gather_list=bufs, dst=gdst, group=group, async_op=async_op)
    if async_op:
        return PendingGather(work, flat, counts)
    return _assemble(flat, counts)


# ---------------------------------------------------------------------------
# Sharded fleets (krr_amd.core.runner.BatchedRunner's multi-GPU mode)
# ---------------------------------------------------------------------------

def slice_series(ps, lo: int, hi: int):
    """Objects [lo, hi) of a PackedSeries (values are a view, offsets rebased)."""
    from krr_amd.core.packing import PackedSeries

    a, b = int(ps.offsets[lo]), int(ps.offsets[hi])
    offs = (ps.offsets[lo:hi + 1] - a).astype(np.int64)
    lens = np.diff(offs)
    exact = getattr(ps, "exact", None)
    if exact is not None:
        exact = exact[lo:hi]
    sources = getattr(ps, "sources", None)
    return PackedSeries(ps.values[a:b], offs, int(lens.max()) if lens.size else 0, ps.gaps_are_nan,
                        exact if exact is not None and exact.any() else None,
                        sources[lo:hi] if exact is not None and exact.any() else None)


def slice_fleet(fleet, lo: int, hi: int):
    from krr_amd.core.packing import PackedFleet

    return PackedFleet(slice_series(fleet.cpu, lo, hi), slice_series(fleet.mem, lo, hi))


def fleet_shard_bounds(fleet, world_size: int) -> list[tuple[int, int]]:
    """Contiguous object ranges with ~equal slots (CPU + memory) per rank."""
    w = np.diff(fleet.cpu.offsets) + np.diff(fleet.mem.offsets)
    return shard_bounds(w, world_size)


def raw_from_records(rec):
    """int64 [S, 4] records (tensor or array) -> krr_amd.core.engine.RawResults."""
    from krr_amd.core.engine import RawResults

    u = unpack_records(rec)
    return RawResults(u["cpu_value"], u["cpu_count"], u["cpu_flags"], u["mem_value"], u["mem_count"], u["mem_flags"])


def collective_device(group=None, device: Optional[int] = None):
    """Where a collective's tensors live: the rank's GPU for "nccl" (RCCL), host for gloo.

    The rank's GPU is ``device`` (default: ``local_device()``), never the calling thread's
    current device: HIP's current device is per host thread, and a worker thread (e.g.
    ``asyncio.to_thread``) starts on device 0, which would put every rank's records on
    GPU 0 and give RCCL duplicate devices."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", local_device() if device is None else int(device))
    return torch.device("cpu")


def local_device() -> int:
    """This rank's HIP device: LOCAL_RANK (modulo the visible devices, so a gloo rehearsal
    may put several ranks on one GPU)."""
    import torch

    return int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
