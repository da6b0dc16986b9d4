"""Device packer: Prometheus query_range response bodies -> CSR float64 in HBM.

The host packer (``krr_amd.core.prom_native.pack_query_range_bodies``, libkrr_host.so)
restates the reference's per-pod ``[Decimal(value) for _, value in
pod_result[0]["values"]]`` + empty-pod drop (robusta_krr/core/integrations/prometheus.py:
147-155) on the host's cores; end to end from bodies it was the limiter.
Here the raw bodies cross PCIe instead and the MI355X parses them (include/krr_amd.h
``krr_json_parse`` / ``krr_json_compact``, krr_amd/csrc/krr_json.h):

  1. bodies are gathered into page-locked staging memory by the host runtime's parallel
     copy (``krr_pack_concat``), chunk by chunk;
  2. each chunk goes to HBM on a copy stream while the previous chunk is parsed: one wave
     per body, the values array by all 64 lanes, values to a scratch slot per body;
  3. one synchronisation reads the bodies' statuses and the CSR size; the counts' prefix
     sums (bodies are in fleet order) give the segment offsets and each body's place, and
     ``krr_json_compact`` writes the CSR.

A body outside the form the device decides (KRR_JSON_HOST: escapes in keys or values,
whitespace inside a value string, other NaN/Inf spellings, > 19 significant digits, an error
status, malformed JSON; JSON whitespace between tokens is fine) is not decided here: the whole batch is then parsed by the host packer,
which returns the host's result or raises its error — the outcome is the host packer's
either way (``DevicePacked.via`` says which ran).
"""
from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from krr_amd import _native
from krr_amd.core.packing import PackedSeries
from krr_amd.core.prom_native import KRR_PACK_OK, PrometheusResponseError, load_library, pack_query_range_bodies


def default_threads() -> int:
    """Host threads when the caller gives none: the CPUs this process may run on, capped by
    OMP_NUM_THREADS when set (a GPU box leases 16 CPUs per GPU but its affinity mask shows the
    node's) — what the native pool uses for threads = 0 (krr_pack.cpp default_threads)."""
    import os

    n = len(os.sched_getaffinity(0)) or 1
    try:
        omp = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        omp = 0
    return min(n, omp) if omp > 0 else n


@dataclass
class DevicePacked:
    series: PackedSeries            # values / offsets: torch tensors in HBM (via == "device") or numpy (host)
    via: str                        # "device" | "host"
    host_bodies: int = 0            # bodies the device left to the host (KRR_JSON_HOST)
    pod_counts: Optional[object] = None  # per body: samples kept, -1 dropped (return_pod_counts)
    timestamps: Optional[object] = None


class DevicePacker:
    """One per (thread, device): owns the page-locked staging buffer and a copy stream.

    ``chunk_bytes``: bodies are staged and copied in chunks of up to this size (the first
    ones smaller, doubling from 16 MiB, so the copy engine starts early), each parsed as
    soon as it is in HBM."""

    def __init__(self, ctx: _native.Context, chunk_bytes: int = 256 << 20, threads: int = 0, strip: Optional[bool] = None):
        import os

        import torch

        self.ctx = ctx
        # per-pod bodies are staged with their sample timestamps cut to one digit
        # (krr_pack_concat_strip, krr_amd/csrc/krr_strip.h): fewer bytes over PCIe, same CSR
        self.strip = (os.environ.get("KRR_PACK_STRIP", "1") != "0") if strip is None else bool(strip)
        self.last_upload: Optional[dict] = None
        self.strip_runs_per_thread = 1  # runs per staging thread (each run = one H2D copy)
        # grouped bodies: strip pieces per staging thread and chunk (each piece is one H2D copy: 4 per
        # thread cost 6 ms of 57 on the bench fleet against 1, which still balances the strip)
        self.pieces_per_thread = 1
        self.strip_threads = 0          # grouped strip threads (0: one fewer than self.threads)
        # grouped staging: chunks stripped by a thread of their own, one chunk ahead of the copies
        self.strip_ahead = os.environ.get("KRR_STRIP_AHEAD", "1") != "0"
        self.device = torch.device("cuda", ctx.device)
        self.chunk_bytes = int(chunk_bytes)
        self.threads = int(threads)
        self._stage = None
        self._last = None  # (device bodies, staging buffer) of the last batch
        self._copy_stream = torch.cuda.Stream(device=self.device)
        # a second copy stream: the grouped pieces (~10 MB each) alternate between the two, so one
        # copy's setup overlaps the other's transfer (54 -> 57 GB/s for 10-MiB copies on the box)
        self._copy_stream2 = torch.cuda.Stream(device=self.device)
        self._lock = threading.Lock()

    def release(self) -> None:
        """Drop the page-locked staging buffer (it keeps the largest batch's size otherwise)."""
        with self._lock:
            self._stage = None
            self._last = None
            self._seg_rows = None

    def _live_layout(self):
        """(device body offsets, piece device starts, piece staging shifts) of the batch being
        uploaded, as far as it has been staged: what the host routing of the chunks staged so far
        needs (an empty piece shares its device start with the next: the last of such a run is
        kept, so the starts increase strictly)."""
        no, pd, ps = self._live
        k = min(len(pd), len(ps))
        if not k:
            return no, np.zeros(0, np.int64), np.zeros(0, np.int64)
        pdev, psh = np.concatenate(pd[:k]), np.concatenate(ps[:k])
        keep = np.concatenate([np.diff(pdev) > 0, [True]])
        return no, np.ascontiguousarray(pdev[keep]), np.ascontiguousarray(psh[keep])

    def _host_rows(self, n: int):
        """A page-locked int64 [>= n, 7] buffer for the grouped segments, kept and grown (a batch's
        earlier chunks keep the buffer they were copied into alive through their views)."""
        import torch

        buf = getattr(self, "_seg_rows", None)
        if buf is None or buf.shape[0] < n:
            buf = self._seg_rows = torch.empty((max(n, 2 * (buf.shape[0] if buf is not None else 0), 1 << 14), 7),
                                               dtype=torch.int64, pin_memory=True)
        return buf

    def _parse_streams(self, n: int = 3):
        import torch

        if getattr(self, "_pstreams", None) is None:
            self._pstreams = [torch.cuda.Stream(device=self.device) for _ in range(n)]
        return self._pstreams

    def _staging(self, nbytes: int):
        import torch

        if self._stage is None or self._stage.numel() < nbytes:
            from krr_amd.utils.numa import page_nodes

            if self._stage is not None:  # the old buffer goes back to the system first
                self._stage = self._last = None
                empty = getattr(torch._C, "_host_emptyCache", None)
                if empty is not None:
                    empty()
            self._stage = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, pin_memory=True)
            self.stage_nodes = page_nodes(self._stage.data_ptr(), self._stage.numel())
            from krr_amd.utils.numa import mapping_info

            self.stage_mapping = mapping_info(self._stage.data_ptr(), self._stage.numel())
        return self._stage

    def pack(self, per_object_bodies: Sequence[Sequence[bytes]], *, want_timestamps: bool = False,
             return_pod_counts: bool = False, stream=None) -> DevicePacked:
        """per_object_bodies[o][i] = the raw query_range body of pod i of object o, for ONE
        resource (as ``pack_query_range_bodies``).  Returns a DevicePacked whose series is
        the host packer's CSR, bit for bit, in HBM."""
        with self._lock, self._on(stream):
            return self._pack(per_object_bodies, want_timestamps, return_pod_counts, None)

    def _on(self, stream):
        """Every buffer of a call is allocated, and every launch enqueued, on ONE stream (the
        caller's ``stream`` or the device's current one): the caching allocator then never
        hands a block that is still read by an enqueued launch to another stream."""
        import torch

        return torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream(self.device))

    def _upload(self, flat, want_ts, st, launch, strip: bool = False, pieces: bool = False, extra_slots: int = 0):
        """``flat``: the bodies (bytes), or a body table (int64 buffer addresses, int64
        lengths) from ``_body_table``.  ``pieces``: stripped in pieces that may cut a large body
        (``_upload_pieces``)."""
        if isinstance(flat, tuple):
            return self._upload_table(int(flat[0].ctypes.data), flat[1], want_ts, st, launch, strip, pieces,
                                      extra_slots)
        lens = np.fromiter((len(b) for b in flat), dtype=np.int64, count=len(flat))
        ptrs = (ctypes.c_char_p * len(flat))(*flat)  # alive while the staging below runs
        return self._upload_table(ctypes.addressof(ptrs), lens, want_ts, st, launch, strip, pieces, extra_slots)

    def _upload_table(self, ptr_addr, lens, want_ts, st, launch, strip: bool = False, pieces: bool = False,
                      extra_slots: int = 0):
        """Stage ``flat`` bodies chunk by chunk (host threads), copy each chunk to HBM on the
        copy stream and call ``launch(jb, a, b, tmp_v, tmp_t, lo, hi)`` on ``st`` for bodies
        [a, b) = bytes [lo, hi) once the chunk is there.  ``strip``: the bodies' timestamps
        are cut while staging (``_upload_stripped``; lo / hi are then the chunk's device positions,
        and ``self._layout`` says where each body sits)."""
        import torch

        dev = self.device
        nb = len(lens)
        boffs = np.zeros(nb + 1, dtype=np.int64)
        np.cumsum(lens, out=boffs[1:])
        total = int(boffs[-1])
        stage = self._staging(total + 128)
        self._layout = (boffs, None)  # device offsets, staging shift (none: same offsets)
        self._live = (boffs, [], [])  # the same while the chunks stream (see _live_layout)
        self._last_stage_ptr = stage.data_ptr()
        d_bodies = torch.empty(total + 128, dtype=torch.uint8, device=dev)
        if strip and not want_ts and nb:
            if pieces:
                return self._upload_pieces(ptr_addr, lens, boffs, total, stage, d_bodies, st, launch, extra_slots)
            return self._upload_stripped(ptr_addr, lens, boffs, total, stage, d_bodies, st, launch)
        d_boffs = torch.from_numpy(boffs).to(dev)
        slots = total // 8 + 1 + int(extra_slots)
        tmp_v = torch.empty(slots, dtype=torch.float64, device=dev)
        tmp_t = torch.empty(slots, dtype=torch.float64, device=dev) if want_ts else None
        jb = self.ctx.json_bodies(d_bodies, d_boffs, total)
        host = load_library()
        cs = self._copy_stream
        cs.wait_stream(st)  # d_bodies / d_boffs were allocated on st
        a = 0
        step = min(self.chunk_bytes, 16 << 20)  # small first chunks: the DMA starts early
        while a < nb:
            b = int(np.searchsorted(boffs, boffs[a] + step, side="left"))
            step = min(2 * step, self.chunk_bytes)
            b = min(max(b, a + 1), nb)
            lo, hi = int(boffs[a]), int(boffs[b])
            rc = host.krr_pack_concat(ptr_addr + a * 8,
                                      lens[a:].ctypes.data, b - a, boffs[a:].ctypes.data,
                                      stage.data_ptr() + lo, self.threads)
            if rc != KRR_PACK_OK:
                raise PrometheusResponseError(rc, "krr_pack_concat failed")
            with torch.cuda.stream(cs):
                d_bodies[lo:hi].copy_(stage[lo:hi], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(cs)
            st.wait_event(ev)
            launch(jb, a, b, tmp_v, tmp_t, lo, hi)
            a = b
        self._last = (d_bodies, stage)
        self.last_upload = {"bytes": total, "bytes_sent": total, "bodies": nb, "bodies_stripped": 0}
        return lens, boffs, total, jb, tmp_v, tmp_t

    def _upload_stripped(self, ptr_addr, lens, boffs, total, stage, d_bodies, st, launch):
        """_upload with the timestamps cut while staging (krr_pack_concat_strip): each chunk's
        bodies are stripped by the host threads in runs, run r back to back inside its own
        unstripped extent of the staging buffer; the runs go to HBM back to back, so the device
        offsets are the prefix sums of the stripped lengths (uploaded per chunk before its
        parse).  The scratch is sized for the unstripped bytes (an upper bound).  ``launch``
        gets the chunk's DEVICE byte range; ``self._layout`` keeps the device body offsets."""
        import os

        import torch

        dev = self.device
        nb = len(lens)
        T = self.threads or default_threads()
        max_runs = max(1, self.strip_runs_per_thread * T)
        new_lens = np.empty(nb, dtype=np.int64)
        runs = np.empty(max_runs + 1, dtype=np.int64)
        n_runs = ctypes.c_int32(0)
        new_offs = torch.zeros(nb + 1, dtype=torch.int64, pin_memory=True)
        no = new_offs.numpy()
        d_boffs = torch.empty(nb + 1, dtype=torch.int64, device=dev)
        slots = total // 8 + 1
        tmp_v = torch.empty(slots, dtype=torch.float64, device=dev)
        jb = self.ctx.json_bodies(d_bodies, d_boffs, total)
        host = load_library()
        cs, cs2 = self._copy_stream, self._copy_stream2
        cs.wait_stream(st)  # d_bodies / d_boffs were allocated on st
        cs2.wait_stream(st)
        d_base, s_base = d_bodies.data_ptr(), stage.data_ptr()
        o_base, n_base = d_boffs.data_ptr(), new_offs.data_ptr()
        a = 0
        step = min(self.chunk_bytes, 16 << 20)  # small first chunks: the DMA starts early
        while a < nb:
            left = total - int(boffs[a])
            if left <= step + step // 2:  # the end: a small last chunk, whose parse is the tail
                step = max(left * 3 // 4, 16 << 20)
            b = int(np.searchsorted(boffs, boffs[a] + step, side="left"))
            # x1.5 per chunk: staging (~130 GB/s of JSON on 16 threads) stays ahead of the
            # link (~85 GB/s of JSON once stripped) while the chunks grow
            step = min(step * 3 // 2, self.chunk_bytes)
            b = min(max(b, a + 1), nb)
            lo = int(boffs[a])
            rc = host.krr_pack_concat_strip(ptr_addr + a * 8,
                                            lens[a:].ctypes.data, b - a, boffs[a:].ctypes.data,
                                            stage.data_ptr() + lo, self.threads, max_runs,
                                            new_lens[a:].ctypes.data, runs.ctypes.data, ctypes.byref(n_runs))
            if rc != KRR_PACK_OK:
                raise PrometheusResponseError(rc, "krr_pack_concat_strip failed")
            np.cumsum(new_lens[a:b], out=no[a + 1:b + 1])
            no[a + 1:b + 1] += no[a]
            # every run of the chunk, then its body offsets: one native call of async copies
            nr = n_runs.value
            b0 = a + runs[:nr]
            dst = np.empty(nr + 1, dtype=np.int64)
            src = np.empty(nr + 1, dtype=np.int64)
            nby = np.empty(nr + 1, dtype=np.int64)
            dst[:nr] = d_base + no[b0]
            src[:nr] = s_base + boffs[b0]
            nby[:nr] = no[a + runs[1:nr + 1]] - no[b0]
            dst[nr], src[nr], nby[nr] = o_base + 8 * a, n_base + 8 * a, 8 * (b - a + 1)
            # even runs (and the offsets) on one copy stream, odd runs on the other (as the
            # grouped pieces: one copy's setup overlaps the other's transfer)
            ev_idx = np.concatenate([np.arange(0, nr, 2), [nr]])
            self.ctx.copy_h2d_batch(dst[ev_idx], src[ev_idx], nby[ev_idx], stream=cs)
            if nr > 1:
                self.ctx.copy_h2d_batch(dst[1:nr:2], src[1:nr:2], nby[1:nr:2], stream=cs2)
            for c in (cs, cs2):
                with torch.cuda.stream(c):
                    ev = torch.cuda.Event()
                    ev.record(c)
                st.wait_event(ev)
            launch(jb, a, b, tmp_v, None, int(no[a]), int(no[b]))
            a = b
        self._last = (d_bodies, stage, new_offs)
        self._layout = (no.copy(), None)
        sent = int(no[nb])
        self.last_upload = {"bytes": total, "bytes_sent": sent, "bodies": nb,
                            "bodies_stripped": int((new_lens < lens).sum())}
        return lens, boffs, total, jb, tmp_v, None

    def _upload_pieces(self, ptr_addr, lens, boffs, total, stage, d_bodies, st, launch, extra_slots: int = 0):
        """_upload_stripped for a few large bodies (grouped `sum by (pod)` responses, ~100 MB each):
        each chunk is stripped by krr_pack_concat_strip_pieces, which cuts a large body at sample
        boundaries into pieces the host threads strip apart (one thread per body would bound the
        staging at ~13 GB/s); the pieces go to HBM back to back.  ``self._layout`` = (device body
        offsets, None, (piece device starts, piece staging shifts)) for the host's routing."""
        import os

        import torch

        dev = self.device
        nb = len(lens)
        T = self.strip_threads
        if not T:  # one thread fewer than the lease: the staging and pipeline threads keep a core
            T = self.threads or default_threads()
            T = T - 1 if T >= 4 else T
        max_pieces = max(2, int(self.pieces_per_thread * T))
        new_lens = np.empty(nb, dtype=np.int64)
        new_offs = torch.zeros(nb + 1, dtype=torch.int64, pin_memory=True)
        no = new_offs.numpy()
        d_boffs = torch.empty(nb + 1, dtype=torch.int64, device=dev)
        tmp_v = torch.empty(total // 8 + 1 + int(extra_slots), dtype=torch.float64, device=dev)
        jb = self.ctx.json_bodies(d_bodies, d_boffs, total)
        host = load_library()
        cs, cs2 = self._copy_stream, self._copy_stream2
        cs.wait_stream(st)  # d_bodies / d_boffs were allocated on st
        cs2.wait_stream(st)
        d_base, s_base = d_bodies.data_ptr(), stage.data_ptr()
        o_base, n_base = d_boffs.data_ptr(), new_offs.data_ptr()
        piece_dev, piece_shift = [], []
        self._live = (no, piece_dev, piece_shift)  # grown chunk by chunk: the routing reads it
        import time

        # the chunks (whole bodies): they depend on the body sizes only
        chunks = []
        a = 0
        step = min(self.chunk_bytes, 16 << 20)
        while a < nb:
            left = total - int(boffs[a])
            if left <= step + step // 2:  # the end: a small last chunk, whose search + parse is the tail
                step = max(left * 3 // 4, 16 << 20)
            b = int(np.searchsorted(boffs, boffs[a] + step, side="left"))
            step = min(step * 3 // 2, self.chunk_bytes)
            b = min(max(b, a + 1), nb)
            chunks.append((a, b))
            a = b

        def strip_chunk(a, b):
            cap = 2 * (b - a) + max_pieces
            p_start, p_out, n_p = np.empty(cap + 1, dtype=np.int64), np.empty(cap, dtype=np.int64), ctypes.c_int32(0)
            t_s = time.perf_counter()
            rc = host.krr_pack_concat_strip_pieces(ptr_addr + a * 8, lens[a:].ctypes.data, b - a,
                                                   boffs[a:].ctypes.data, stage.data_ptr() + int(boffs[a]),
                                                   T, max_pieces, new_lens[a:].ctypes.data,
                                                   p_start.ctypes.data, p_out.ctypes.data, ctypes.byref(n_p))
            return a, b, rc, p_start, p_out, n_p.value, time.perf_counter() - t_s

        # strip_ahead: a thread strips the chunks one after the other while this one enqueues each
        # stripped chunk's copies and search (on a slow host the staging thread's own work per
        # chunk, ~0.4 ms, otherwise sits between two strips with the worker pool idle)
        import queue
        import threading

        done_q: "queue.Queue" = queue.Queue()
        stop = [False]

        def producer():
            try:
                for a, b in chunks:
                    if stop[0]:
                        break
                    item = strip_chunk(a, b)
                    done_q.put(item)
                    if item[2] != KRR_PACK_OK:
                        break
            except BaseException as e:  # noqa: BLE001 — re-raised by the consumer
                done_q.put(e)
            finally:
                done_q.put(None)

        ahead = self.strip_ahead and len(chunks) > 1
        if ahead:
            prod = threading.Thread(target=producer, name="krr-strip-ahead", daemon=True)
            prod.start()
        items = iter(done_q.get, None) if ahead else (strip_chunk(a, b) for a, b in chunks)
        t_strip = 0.0
        try:
            for item in items:
                if isinstance(item, BaseException):
                    raise item
                a, b, rc, p_start, p_out, k, dt = item
                if rc != KRR_PACK_OK:
                    raise PrometheusResponseError(rc, "krr_pack_concat_strip_pieces failed")
                t_strip += dt
                np.cumsum(new_lens[a:b], out=no[a + 1:b + 1])
                no[a + 1:b + 1] += no[a]
                pd = no[a] + np.concatenate([[0], np.cumsum(p_out[:k])[:-1]]).astype(np.int64)
                piece_dev.append(pd)
                piece_shift.append(p_start[:k] - pd)
                # every piece, then the chunk's body offsets: one native call of async copies
                dst = np.empty(k + 1, dtype=np.int64)
                src = np.empty(k + 1, dtype=np.int64)
                nby = np.empty(k + 1, dtype=np.int64)
                dst[:k], src[:k], nby[:k] = d_base + pd, s_base + p_start[:k], p_out[:k]
                dst[k], src[k], nby[k] = o_base + 8 * a, n_base + 8 * a, 8 * (b - a + 1)
                # even pieces (and the offsets) on one copy stream, odd pieces on the other
                ev_idx = np.concatenate([np.arange(0, k, 2), [k]])
                self.ctx.copy_h2d_batch(dst[ev_idx], src[ev_idx], nby[ev_idx], stream=cs)
                if k > 1:
                    self.ctx.copy_h2d_batch(dst[1:k:2], src[1:k:2], nby[1:k:2], stream=cs2)
                for c in (cs, cs2):
                    with torch.cuda.stream(c):
                        ev = torch.cuda.Event()
                        ev.record(c)
                    st.wait_event(ev)
                launch(jb, a, b, tmp_v, None, int(no[a]), int(no[b]))
        finally:
            if ahead:
                stop[0] = True
                prod.join()
        self._last = (d_bodies, stage, new_offs)
        pdev = np.concatenate(piece_dev) if piece_dev else np.zeros(0, np.int64)
        psh = np.concatenate(piece_shift) if piece_shift else np.zeros(0, np.int64)
        # an empty piece shares its device start with the next: keep the last of such a group
        keep = np.concatenate([np.diff(pdev) > 0, [True]]) if pdev.size else np.zeros(0, bool)
        self._layout = (no.copy(), None, (np.ascontiguousarray(pdev[keep]), np.ascontiguousarray(psh[keep])))
        self.last_upload = {"bytes": total, "bytes_sent": int(no[nb]), "bodies": nb,
                            "bodies_stripped": int((new_lens < lens).sum()), "pieces": int(pdev.size),
                            "strip_s": round(t_strip, 5)}
        return lens, boffs, total, jb, tmp_v, None

    def pack_grouped(self, plan, bodies: Sequence[bytes], *, want_timestamps: bool = False,
                     return_pod_counts: bool = False, stream=None, label: str = "pod") -> DevicePacked:
        """``plan`` a krr_amd.core.fleet_query.FleetQueryPlan, bodies[g] the response to its
        g-th grouped query (one resource): the CSR ``plan.pack(bodies)`` builds on the host,
        bit for bit, with the bodies parsed on the device one wave per series
        (krr_json_find_series + krr_json_parse_segments) and chained and routed by pod label
        on the host (krr_pack_route_grouped)."""
        return self.pack_grouped_many([(plan, bodies)], want_timestamps=want_timestamps,
                                      return_pod_counts=return_pod_counts, stream=stream, label=label)[0]

    def pack_grouped_many(self, items, *, want_timestamps: bool = False, return_pod_counts: bool = False,
                          stream=None, label: str = "pod", hybrid: bool = False) -> list:
        """Several (plan, bodies) pairs (e.g. CPU and memory) through ONE staging / copy /
        candidate-search pipeline; one DevicePacked per pair.  ``hybrid``: the last bodies
        (about ``grouped_share`` of the bytes) are parsed by the host packer on a worker thread
        (``FleetQueryPlan.pack_group_slots``, a quarter of the threads) while the rest cross the
        link; their slots' values join the device scratch and the same gather builds the CSR.
        The share then moves toward r_host / (r_host + r_device)."""
        with self._lock, self._on(stream):
            return self._pack_grouped_multi(items, want_timestamps, return_pod_counts, None, label,
                                            self.grouped_share if hybrid else 0.0)

    grouped_share = 0.06          # the hybrid grouped parser's host share of the bytes (adapted)
    grouped_host_threads = 0      # 0: a quarter of the threads
    # a grouped chunk's values arrays parsed in 16-KiB parts, one wave each
    # (krr_json_parse_segments_split), instead of one wave per series
    grouped_split_parse = os.environ.get("KRR_GROUPED_SPLIT", "1") != "0"
    # per-chunk parse enqueue and routing on a pipeline thread (route "chunk" only)
    grouped_pipeline_thread = os.environ.get("KRR_GROUPED_PIPELINE", "1") != "0"
    # "chunk": segments to the host and routed per chunk; "end": once, after the last parse
    grouped_route = os.environ.get("KRR_GROUPED_ROUTE", "chunk")
    _EMPTY_BODY = b'{"status":"success","data":{"resultType":"matrix","result":[]}}'

    def _pack_grouped_multi(self, items, want_ts, want_counts, stream, label, host_share: float = 0.0) -> list:
        """The grouped pipeline, chunk by chunk (a chunk = whole bodies):
          strip thread:     strip the chunk's bodies in pieces into the staging buffer;
          staging thread:   enqueue the pieces' copies (two copy streams) and the search of the
                            chunk's series starts (launch stream);
          pipeline thread:  wait for the search, enqueue the chunk's parse on a parse stream (the
                            values arrays in 16-KiB parts, segment rows written into page-locked
                            host memory), and chain and route every parsed chunk's bodies on the
                            host (their groups' slots only);
        so after the last copy only the last chunk's search, parse and route remain.  Then every
        slot's values are gathered into the CSR.  grouped_route = "end" (or no pipeline thread)
        runs the parse one chunk behind on the staging thread instead, and "end" routes once."""
        import threading
        import time

        import torch

        flat: list = []
        body0 = [0]
        for plan, bodies in items:
            if len(bodies) != len(plan.groups):
                raise ValueError(f"expected {len(plan.groups)} bodies (one per group query), got {len(bodies)}")
            flat.extend(b if isinstance(b, bytes) else bytes(b) for b in bodies)  # c_char_p takes bytes only
            body0.append(len(flat))
        dev = self.device
        st = stream if stream is not None else torch.cuda.current_stream(dev)

        def host_fallback(r, n_host):
            plan, bodies = items[r]
            res = plan.pack(bodies, want_timestamps=want_ts, threads=self.threads, return_pod_counts=want_counts)
            res = res if isinstance(res, tuple) else (res,)
            rest = list(res[1:])
            ts = rest.pop(0) if want_ts else None
            pc = rest.pop(0) if want_counts else None
            return DevicePacked(res[0], "host", n_host, pc, ts)

        if not flat or all(plan.n_slots == 0 for plan, _ in items):
            return [host_fallback(r, 0) for r in range(len(items))]
        clock = [time.perf_counter()]  # phase ends (host clock; only the existing synchronisations)
        # hybrid: the last bodies go to the host packer on a worker thread, the rest to the device
        split = len(flat)
        if host_share > 0 and not want_ts and len(flat) >= 2:
            tail = np.cumsum(np.array([len(b) for b in flat[::-1]], dtype=np.int64))
            k_host = int(np.searchsorted(tail, host_share * tail[-1], side="right"))
            split = len(flat) - min(max(k_host, 1), len(flat) - 1)
        host_res: dict = {}
        host_thread = None
        T_all = self.threads or default_threads()
        t_host = max(1, int(self.grouped_host_threads or T_all // 4))
        if split < len(flat):
            from krr_amd.core.runner import _pinned_alloc_or_none

            alloc = _pinned_alloc_or_none()

            def host_part():
                t0 = time.perf_counter()
                try:
                    for r, (plan, _) in enumerate(items):
                        lo, hi = max(body0[r], split), body0[r + 1]
                        if lo < hi:
                            host_res[r] = plan.pack_group_slots(flat[lo:hi], lo - body0[r], hi - body0[r],
                                                                threads=t_host, alloc=alloc)
                except BaseException as e:  # noqa: BLE001 — handed to the caller after the join
                    host_res["error"] = e
                finally:
                    host_res["s"] = time.perf_counter() - t0

            host_thread = threading.Thread(target=host_part, name="krr-grouped-host", daemon=True)
            host_thread.start()
        host_bytes = sum(len(b) for b in flat[split:])
        dflat = flat[:split]
        total_bytes = sum(len(b) for b in dflat)
        # candidates: a series object takes >= 48 bytes (`{"metric":{"pod":"…"},"values":[[1,"1"]]}`);
        # more than that (a body of empty label sets) overflows to the host packer
        cap = max(4096, total_bytes // 48)
        cand = torch.empty(cap, dtype=torch.int64, device=dev)
        n_cand = torch.zeros(1, dtype=torch.int64, device=dev)
        if self.grouped_route not in ("chunk", "end"):
            raise ValueError(f"grouped_route must be 'chunk' or 'end', got {self.grouped_route!r}")
        per_chunk = self.grouped_route == "chunk"
        seg_parts: list = []  # "end": each chunk's segments on the device, copied once at the end
        seen = [0]  # positions below this were searched
        # the parses run on streams of their own (a chunk holds one or two bodies = a few hundred
        # series = waves, far from filling the GPU): consecutive chunks' parses overlap each other
        # and the copies, instead of queueing behind the next chunk's copy on the launch stream
        pstreams = self._parse_streams()
        snaps = torch.zeros(max(len(dflat), 1) + 1, dtype=torch.int64, pin_memory=True)
        snap_np = snaps.numpy()
        searched: list = []     # (event, snapshot slot, first body, body end) of chunks to parse
        waited = [0.0]
        enq = [0.0]             # host seconds enqueueing the parses
        parsed = [0, False]     # candidates parsed so far, overflow
        host = load_library()
        # per resource: routing outputs in the plan's group-sorted slot order (a chunk's bodies =
        # whole groups = one contiguous range of it), and per body whether its series chained
        rk = []
        for plan, _ in items:
            ns = plan.n_slots
            rk.append({"sorted": plan.group_sorted_slots(), "src": np.full(max(ns, 1), -1, dtype=np.int64),
                       "cnt": np.full(max(ns, 1), -1, dtype=np.int64),
                       "ok": np.ones(max(len(plan.groups), 1), dtype=np.int32)})

        def route(a, b, seg_rows, threads=2):
            """Chain and route bodies [a, b) of dflat with their segments (int64 [k, 7] on the host)."""
            n_seg = seg_rows.shape[0]
            dev_offs, pdev, psh = self._live_layout()
            for r, (plan, _) in enumerate(items):
                g0, g1 = max(a, body0[r]) - body0[r], min(b, body0[r + 1]) - body0[r]
                if g0 >= g1:
                    continue
                order, sgroup, blob, noffs, gstart = rk[r]["sorted"]
                i0, i1 = int(gstart[g0]), int(gstart[g1])
                b_offs = np.ascontiguousarray(dev_offs[body0[r] + g0:body0[r] + g1 + 1])
                sb = np.ascontiguousarray(sgroup[i0:i1] - g0) if i1 > i0 else np.zeros(1, np.int64)
                src = np.empty(max(i1 - i0, 1), dtype=np.int64)
                cnt = np.empty(max(i1 - i0, 1), dtype=np.int64)
                ok = np.empty(g1 - g0, dtype=np.int32)
                rc = host.krr_pack_route_grouped_pieces(
                    self._last_stage_ptr, b_offs.ctypes.data, g1 - g0, pdev.ctypes.data, psh.ctypes.data, pdev.size,
                    label.encode(), seg_rows.ctypes.data, n_seg,
                    sb.ctypes.data, blob or b"\0", noffs[i0:].ctypes.data, i1 - i0, src.ctypes.data,
                    cnt.ctypes.data, ok.ctypes.data, threads)
                if rc != KRR_PACK_OK:
                    raise PrometheusResponseError(rc, "krr_pack_route_grouped failed")
                rk[r]["src"][order[i0:i1]] = src[:i1 - i0]
                rk[r]["cnt"][order[i0:i1]] = cnt[:i1 - i0]
                rk[r]["ok"][g0:g1] = ok

        to_route: list = []     # (event, first body, body end, segment range) of parsed chunks
        route_wait = [0.0, 0.0]  # waiting for parsed chunks, routing them
        route_threads = [2]      # while staging: 2 (the staging keeps the pool)

        def route_ready(block=False):
            """Route the parsed chunks whose parse and segment copy are done (the staging thread
            does it between chunks, never waiting on the device; ``block``: all of them)."""
            while to_route and (block or to_route[0][0].query()):
                ev, a, b, rows = to_route.pop(0)
                t_w = time.perf_counter()
                ev.synchronize()
                t_r = time.perf_counter()
                route_wait[0] += t_r - t_w
                route(a, b, rows.numpy(), route_threads[0])
                route_wait[1] += time.perf_counter() - t_r

        def parse_chunk(jb, tmp_v, tmp_t):
            parse_item(jb, tmp_v, tmp_t, searched.pop(0))

        def parse_item(jb, tmp_v, tmp_t, item):
            ev, k, a, b_end = item
            t_w = time.perf_counter()
            ev.synchronize()  # that chunk's search only: later copies keep streaming
            waited[0] += time.perf_counter() - t_w
            n = int(snap_np[k])
            lo = parsed[0]
            if parsed[1] or n > cap:
                parsed[1] = True
                return
            t_e = time.perf_counter()
            ps = pstreams[k % len(pstreams)]
            ps.wait_event(ev)
            rows = self._host_rows(n)[lo:n] if per_chunk else None
            with torch.cuda.stream(ps):
                ws = None
                if n > lo and self.grouped_split_parse:
                    # the split values parse's workspace: 1 + n + 6 words per 16-KiB part, parts
                    # <= the chunk's bytes / 16 KiB + 2 per series (include/krr_amd.h)
                    no_ = self._live_layout()[0]
                    span = int(no_[b_end]) - int(no_[max(a - 1, 0)])
                    ws = torch.empty(1 + (n - lo) + 6 * (span // 16384 + 2 * (n - lo) + 8), dtype=torch.int64,
                                     device=dev)
                if n > lo:
                    starts = torch.sort(cand[lo:n]).values
                    # the chunk's bodies' device offsets are in HBM (copied with the chunk)
                    body_of = torch.searchsorted(jb._keep[1][:b_end + 1], starts, right=True) - 1
                    # per chunk: the kernel writes the segments straight into page-locked host
                    # memory (no device-to-host DMA: on the copy engines it queued behind, and
                    # slowed, the chunks' host-to-device copies)
                    if not per_chunk:
                        seg_parts.append(torch.empty((n - lo, 7), dtype=torch.int64, device=dev))
                    self.ctx.json_parse_segments(jb, starts, body_of, label, want_ts, tmp_v, tmp_t,
                                                 rows if per_chunk else seg_parts[-1], stream=ps, workspace=ws)
                if per_chunk:
                    evp = torch.cuda.Event(blocking=pipe is not None)
                    evp.record(ps)
            if per_chunk:
                to_route.append((evp, a, b_end, rows))
            parsed[0] = n
            enq[0] += time.perf_counter() - t_e

        def launch(jb, a, b, tmp_v, tmp_t, lo, hi):  # search each chunk as it lands
            last = b == len(dflat)
            end = hi if last else max(hi - 16, seen[0])
            self.ctx.json_find_series(jb, cand, n_cand, begin=seen[0], end=end, limit=hi, stream=st)
            seen[0] = end
            k = len(done)  # this chunk's snapshot slot
            with torch.cuda.stream(st):
                snaps[k:k + 1].copy_(n_cand, non_blocking=True)
                ev = torch.cuda.Event(blocking=pipe is not None)  # a waiting thread sleeps
                ev.record(st)
            done.append(k)
            if pipe is not None:  # the pipeline thread parses and routes it
                pipe["jobs"].put((jb, tmp_v, tmp_t, (ev, k, a, b)))
                return
            searched.append((ev, k, a, b))
            if len(searched) > 1:  # parse the chunk searched before this one
                parse_chunk(jb, tmp_v, tmp_t)
            route_ready()

        done: list = []
        pipe = None
        if self.grouped_pipeline_thread and per_chunk:
            # a thread of its own waits for each chunk's search, enqueues its parse and routes
            # the parsed chunks, so the staging thread only strips and enqueues copies (on the
            # staging thread these cost ~7 ms of a 52-ms batch while the pool's helpers idled)
            import queue

            pipe = {"jobs": queue.Queue(), "err": []}

            def pipeline():
                while True:
                    job = pipe["jobs"].get()
                    if job is None:
                        return
                    if pipe["err"]:
                        continue
                    try:
                        parse_item(*job)
                        route_ready()
                    except BaseException as e:  # noqa: BLE001 — re-raised by the caller after the join
                        pipe["err"].append(e)

            pipe["thread"] = threading.Thread(target=pipeline, name="krr-grouped-pipeline", daemon=True)
            pipe["thread"].start()
        threads_was = self.threads
        if host_thread is not None:  # the staging threads: the rest
            self.threads = max(1, T_all - t_host)
        try:
            # timestamps cut while staging, as for per-pod bodies: the candidate search, the series
            # parse and the host's chain walk read structure, labels and value strings only
            try:
                lens, boffs, total, jb, tmp_v, tmp_t = self._upload(dflat, want_ts, st, launch, strip=self.strip,
                                                                    pieces=True, extra_slots=host_bytes // 8 + 1)
            finally:
                if pipe is not None:
                    t_j = time.perf_counter()
                    pipe["jobs"].put(None)
                    pipe["thread"].join()
                    pipe["join_s"] = time.perf_counter() - t_j
            if pipe is not None and pipe["err"]:
                raise pipe["err"][0]
            clock.append(time.perf_counter())
            while searched:
                parse_chunk(jb, tmp_v, tmp_t)
                route_ready()
            clock.append(time.perf_counter())
            if not parsed[1]:  # the staging is over: the last chunks' routing gets every thread
                route_threads[0] = self.threads
                route_ready(block=True)
        finally:
            self.threads = threads_was
        for ps in pstreams:
            st.wait_stream(ps)
        if not per_chunk and not parsed[1]:  # every chunk's segments at once, then one route
            nc = parsed[0]
            rows = self._host_rows(nc)[:nc]
            if nc:
                with torch.cuda.stream(st):
                    rows.copy_(torch.cat(seg_parts) if len(seg_parts) > 1 else seg_parts[0])
            route(0, len(dflat), rows.numpy(), self.threads)
        t_dev = time.perf_counter() - clock[0]
        if host_thread is not None:
            host_thread.join()
        clock.append(time.perf_counter())
        err = host_res.get("error")
        if err is not None and not isinstance(err, PrometheusResponseError):
            raise err  # not a body the host packer rejects: the host part itself failed
        if parsed[1] or err is not None:  # candidates overflow / a body the host part rejects
            return [host_fallback(r, body0[r + 1] - body0[r]) for r in range(len(items))]
        if host_thread is not None:
            # share toward r_host / (r_host + r_device) (bytes per second of each side)
            r_h = host_bytes / max(host_res["s"], 1e-6)
            r_d = total_bytes / max(t_dev, 1e-6)
            self.grouped_share = min(max(0.5 * self.grouped_share + 0.5 * r_h / (r_h + r_d), 0.01), 0.5)
            self.last_grouped_hybrid = {"share": host_bytes / (host_bytes + total_bytes), "host_bodies": len(flat) - split,
                                        "host_s": round(host_res["s"], 5), "device_s": round(t_dev, 5),
                                        "host_threads": t_host, "device_threads": max(1, T_all - t_host)}
        out = []
        host_base = int(self._live_layout()[0][len(dflat)]) // 8 + 1  # scratch slots past the device bodies'
        for r, (plan, bodies) in enumerate(items):
            ns, n_obj = plan.n_slots, plan.n_objects
            n_dev_bodies = max(0, min(body0[r + 1], split) - body0[r])
            slot_src, slot_cnt = rk[r]["src"][:ns].copy(), rk[r]["cnt"][:ns].copy()
            if not rk[r]["ok"][:n_dev_bodies].all():
                out.append(host_fallback(r, int((rk[r]["ok"][:n_dev_bodies] == 0).sum())))
                continue
            if r in host_res:  # the host-parsed groups' slots: their values after the device scratch
                idx, hv, hoff, hcnt = host_res[r]
                slot_src[idx] = host_base + hoff[:-1]
                slot_cnt[idx] = hcnt
                if hv.size:
                    with torch.cuda.stream(st):
                        tmp_v[host_base:host_base + hv.size].copy_(torch.from_numpy(hv), non_blocking=True)
                host_base += hv.size
            kept = np.maximum(slot_cnt, 0)
            dst = np.zeros(ns, dtype=np.int64)
            if ns > 1:
                np.cumsum(kept[:-1], out=dst[1:])
            seg = np.bincount(plan.slot_obj, weights=kept, minlength=n_obj).astype(np.int64) if ns else \
                np.zeros(n_obj, dtype=np.int64)
            offsets = np.zeros(n_obj + 1, dtype=np.int64)
            np.cumsum(seg, out=offsets[1:])
            n_vals = int(offsets[-1])
            # the gather's three columns and the offsets in ONE page-locked buffer, one copy
            cols = torch.empty(3 * ns + n_obj + 1, dtype=torch.int64, pin_memory=True)
            cn = cols.numpy()
            cn[:ns], cn[ns:2 * ns], cn[2 * ns:3 * ns], cn[3 * ns:] = np.maximum(slot_src, 0), kept, dst, offsets
            with torch.cuda.stream(st):
                values = torch.empty(max(n_vals, 1), dtype=torch.float64, device=dev)
                ts = torch.empty(max(n_vals, 1), dtype=torch.float64, device=dev) if want_ts else None
                cols_d = cols.to(dev, non_blocking=True)
                if ns:
                    self.ctx.json_gather(cols_d[:ns], cols_d[ns:2 * ns], cols_d[2 * ns:3 * ns], tmp_v, tmp_t, values,
                                         ts, stream=st)
                offs_d = cols_d[3 * ns:]
            series = PackedSeries(values[:n_vals], offs_d, int(seg.max()) if n_obj else 0)
            out.append(DevicePacked(series, "device", 0, slot_cnt if want_counts else None,
                                    ts[:n_vals] if ts is not None else None))
        clock.append(time.perf_counter())
        # seconds per phase: staging + copies + search + the parse and route of all chunks but the
        # last ones, the last chunks' parse, their route (+ the host part's join), the gather enqueue
        self.last_grouped_phases = dict(zip(("stage_copy_search", "last_parse", "last_route", "gather"),
                                            np.diff(clock).round(5).tolist()), parse_wait=round(waited[0], 5),
                                        route_wait=round(route_wait[0], 5), route_s=round(route_wait[1], 5),
                                        parse_enqueue_s=round(enq[0], 5),
                                        pipeline_join_s=round(pipe["join_s"], 5) if pipe else None,
                                        strip=(self.last_upload or {}).get("strip_s"))
        return out

    def pack_many(self, resources: Sequence[Sequence[Sequence[bytes]]], *, want_timestamps: bool = False,
                  return_pod_counts: bool = False, stream=None) -> list:
        """Several resources' bodies (e.g. CPU and memory of one fleet) through ONE staging /
        copy / parse pipeline: one DevicePacked per resource, each as ``pack`` would give it."""
        with self._lock, self._on(stream):
            return self._pack_multi(resources, want_timestamps, return_pod_counts, None)

    def _pack(self, per_object_bodies, want_ts, want_counts, stream) -> DevicePacked:
        return self._pack_multi([per_object_bodies], want_ts, want_counts, stream)[0]

    def _pack_multi(self, resources, want_ts, want_counts, stream) -> list:
        import torch

        obj0 = [0]
        for per_object_bodies in resources:
            obj0.append(obj0[-1] + len(per_object_bodies))
        table = _body_table(resources)
        if table is not None:  # one native pass over the bodies (krr_pydec.cpp body_table)
            ptr_col, lens_col, obj_col = table[:3]
            flat = (ptr_col, lens_col)
            obj = obj_col
            body0 = np.searchsorted(obj_col, obj0, side="left").tolist()
        else:
            fl: list = []
            ob: list = []      # global object index (objects of resource r after those of r - 1)
            body0 = [0]
            for r, per_object_bodies in enumerate(resources):
                for o, bodies in enumerate(per_object_bodies):
                    for b in bodies:
                        fl.append(b if isinstance(b, bytes) else bytes(b))  # c_char_p takes bytes only
                        ob.append(obj0[r] + o)
                body0.append(len(fl))
            flat, obj = fl, ob
        n_obj, nb = obj0[-1], body0[-1]
        dev = self.device
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        if nb == 0:
            out = []
            for per_object_bodies in resources:
                offs = torch.zeros(len(per_object_bodies) + 1, dtype=torch.int64, device=dev)
                out.append(DevicePacked(PackedSeries(torch.empty(0, dtype=torch.float64, device=dev), offs, 0),
                                        "device", 0,
                                        torch.empty(0, dtype=torch.int64, device=dev) if want_counts else None,
                                        torch.empty(0, dtype=torch.float64, device=dev) if want_ts else None))
            return out
        counts = torch.empty(nb, dtype=torch.int64, device=dev)
        status = torch.empty(nb, dtype=torch.int32, device=dev)

        def launch(jb, a, b, tmp_v, tmp_t, lo, hi):
            self.ctx.json_parse(jb, a, b - a, want_ts, tmp_v, tmp_t, counts, status, stream=st)

        lens, boffs, total, jb, tmp_v, tmp_t = self._upload(flat, want_ts, st, launch, strip=self.strip)
        R = len(resources)
        with torch.cuda.stream(st):
            obj_t = torch.from_numpy(np.asarray(obj, dtype=np.int64)).to(dev, non_blocking=False)
            seg = torch.zeros(n_obj, dtype=torch.int64, device=dev).index_add_(0, obj_t, counts)
            offsets = torch.zeros(n_obj + 1, dtype=torch.int64, device=dev)
            torch.cumsum(seg, 0, out=offsets[1:])
            host_flag = (status == _native.KRR_JSON_HOST).to(torch.int64)
            per_res = [torch.stack([host_flag[body0[r]:body0[r + 1]].sum(),
                                    seg[obj0[r]:obj0[r + 1]].max() if obj0[r + 1] > obj0[r] else offsets[0]])
                       for r in range(R)]
            summary = torch.stack(per_res + [torch.stack([offsets[-1], offsets[-1]])]).cpu()  # the one sync
        n_vals = int(summary[R, 0])
        with torch.cuda.stream(st):
            out_pos = torch.cumsum(counts, 0) - counts
            values = torch.empty(max(n_vals, 1), dtype=torch.float64, device=dev)
            ts = torch.empty(max(n_vals, 1), dtype=torch.float64, device=dev) if want_ts else None
            self.ctx.json_compact(jb, tmp_v, tmp_t, counts, status, out_pos, values, ts, stream=st)
            pc = torch.where(status == _native.KRR_JSON_DROPPED, torch.full_like(counts, -1), counts) \
                if want_counts else None
        offs_h = None
        out = []
        for r in range(R):
            n_host, max_len = int(summary[r, 0]), int(summary[r, 1])
            if n_host:  # this resource's batch goes to the host packer: its result or its error
                res = pack_query_range_bodies(resources[r], want_timestamps=want_ts, threads=self.threads,
                                              return_pod_counts=want_counts)
                res = res if isinstance(res, tuple) else (res,)
                rest = list(res[1:])
                t_r = rest.pop(0) if want_ts else None
                c_r = rest.pop(0) if want_counts else None
                out.append(DevicePacked(res[0], "host", n_host, c_r, t_r))
                continue
            if offs_h is None:
                offs_h = offsets.cpu()
            lo, hi = int(offs_h[obj0[r]]), int(offs_h[obj0[r + 1]])
            o_r = offsets[obj0[r]:obj0[r + 1] + 1] - lo
            out.append(DevicePacked(PackedSeries(values[lo:hi], o_r, max_len if obj0[r + 1] > obj0[r] else 0),
                                    "device", 0, pc[body0[r]:body0[r + 1]] if want_counts else None,
                                    ts[lo:hi] if ts is not None else None))
        # the staging buffer is reused by the next call: its copies are done (the parse
        # launches waited for them before the summary synchronised)
        return out


def _body_table(resources):
    """(buffer addresses, lengths, object ids, bytes per object) int64 arrays of the bodies of
    resources[r][o][i] from the native extension (one pass, no per-body Python), or None
    (extension missing, or a body that is not bytes)."""
    from krr_amd.core.packing import _PYDEC

    if _PYDEC is None or not hasattr(_PYDEC, "body_table"):
        return None
    t = _PYDEC.body_table(resources)
    if t is None:
        return None
    return tuple(np.frombuffer(c, dtype=np.int64).copy() for c in t)


_packers: dict = {}
_packers_lock = threading.Lock()


def default_packer(device: int = 0) -> DevicePacker:
    """The process's packer for ``device``: one page-locked staging buffer and one krr_ctx of
    its own per device, whichever thread calls (calls are serialised by the packer's lock, so
    the ctx is never used by two threads at once)."""
    device = int(device.device if isinstance(device, _native.Context) else device)
    with _packers_lock:
        p = _packers.get(device)
        if p is None:
            p = _packers[device] = DevicePacker(_native.Context(device))
        return p


__all__ = ["DevicePacked", "DevicePacker", "default_packer"]
