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
import threading
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from krr_amd import _native
from krr_amd.core.packing import PackedSeries
from krr_amd.core.prom_native import KRR_PACK_OK, PrometheusResponseError, load_library, pack_query_range_bodies


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
        self.device = torch.device("cuda", ctx.device)
        self.chunk_bytes = int(chunk_bytes)
        self.threads = int(threads)
        self._stage = None
        self._last = None  # (device bodies, staging buffer) of the last batch
        self._copy_stream = torch.cuda.Stream(device=self.device)
        self._lock = threading.Lock()

    def release(self) -> None:
        """Drop the page-locked staging buffer (it keeps the largest batch's size otherwise)."""
        with self._lock:
            self._stage = None
            self._last = None

    def _parse_streams(self, n: int = 3):
        import torch

        if getattr(self, "_pstreams", None) is None:
            self._pstreams = [torch.cuda.Stream(device=self.device) for _ in range(n)]
        return self._pstreams

    def _staging(self, nbytes: int):
        import torch

        if self._stage is None or self._stage.numel() < nbytes:
            self._stage = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, pin_memory=True)
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

    def _upload(self, flat, want_ts, st, launch, strip: bool = False, pieces: bool = False):
        """``flat``: the bodies (bytes), or a body table (int64 buffer addresses, int64
        lengths) from ``_body_table``.  ``pieces``: stripped in pieces that may cut a large body
        (``_upload_pieces``)."""
        if isinstance(flat, tuple):
            return self._upload_table(int(flat[0].ctypes.data), flat[1], want_ts, st, launch, strip, pieces)
        lens = np.fromiter((len(b) for b in flat), dtype=np.int64, count=len(flat))
        ptrs = (ctypes.c_char_p * len(flat))(*flat)  # alive while the staging below runs
        return self._upload_table(ctypes.addressof(ptrs), lens, want_ts, st, launch, strip, pieces)

    def _upload_table(self, ptr_addr, lens, want_ts, st, launch, strip: bool = False, pieces: bool = False):
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
        d_bodies = torch.empty(total + 128, dtype=torch.uint8, device=dev)
        if strip and not want_ts and nb:
            if pieces:
                return self._upload_pieces(ptr_addr, lens, boffs, total, stage, d_bodies, st, launch)
            return self._upload_stripped(ptr_addr, lens, boffs, total, stage, d_bodies, st, launch)
        d_boffs = torch.from_numpy(boffs).to(dev)
        slots = total // 8 + 1
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
        T = self.threads or len(os.sched_getaffinity(0))
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
        cs = self._copy_stream
        cs.wait_stream(st)  # d_bodies / d_boffs were allocated on st
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
            self.ctx.copy_h2d_batch(dst, src, nby, stream=cs)
            with torch.cuda.stream(cs):
                ev = torch.cuda.Event()
                ev.record(cs)
            st.wait_event(ev)
            launch(jb, a, b, tmp_v, None, int(no[a]), int(no[b]))
            a = b
        self._last = (d_bodies, stage, new_offs)
        self._layout = (no.copy(), None)
        sent = int(no[nb])
        self.last_upload = {"bytes": total, "bytes_sent": sent, "bodies": nb,
                            "bodies_stripped": int((new_lens < lens).sum())}
        return lens, boffs, total, jb, tmp_v, None

    def _upload_pieces(self, ptr_addr, lens, boffs, total, stage, d_bodies, st, launch):
        """_upload_stripped for a few large bodies (grouped `sum by (pod)` responses, ~100 MB each):
        each chunk is stripped by krr_pack_concat_strip_pieces, which cuts a large body at sample
        boundaries into pieces the host threads strip apart (one thread per body would bound the
        staging at ~13 GB/s); the pieces go to HBM back to back.  ``self._layout`` = (device body
        offsets, None, (piece device starts, piece staging shifts)) for the host's routing."""
        import os

        import torch

        dev = self.device
        nb = len(lens)
        T = self.threads or len(os.sched_getaffinity(0))
        max_pieces = max(2, 2 * T)
        cap = 2 * nb + max_pieces
        new_lens = np.empty(nb, dtype=np.int64)
        p_start = np.empty(cap + 1, dtype=np.int64)
        p_out = np.empty(cap, dtype=np.int64)
        n_p = ctypes.c_int32(0)
        new_offs = torch.zeros(nb + 1, dtype=torch.int64, pin_memory=True)
        no = new_offs.numpy()
        d_boffs = torch.empty(nb + 1, dtype=torch.int64, device=dev)
        tmp_v = torch.empty(total // 8 + 1, dtype=torch.float64, device=dev)
        jb = self.ctx.json_bodies(d_bodies, d_boffs, total)
        host = load_library()
        cs = self._copy_stream
        cs.wait_stream(st)  # d_bodies / d_boffs were allocated on st
        d_base, s_base = d_bodies.data_ptr(), stage.data_ptr()
        o_base, n_base = d_boffs.data_ptr(), new_offs.data_ptr()
        piece_dev, piece_shift = [], []
        import time

        t_strip = 0.0
        a = 0
        step = min(self.chunk_bytes, 16 << 20)
        while a < nb:
            left = total - int(boffs[a])
            if left <= step + step // 2:  # the end: a small last chunk, whose search + parse is the tail
                step = max(left * 3 // 4, 16 << 20)
            b = int(np.searchsorted(boffs, boffs[a] + step, side="left"))
            step = min(step * 3 // 2, self.chunk_bytes)
            b = min(max(b, a + 1), nb)
            lo = int(boffs[a])
            t_s = time.perf_counter()
            rc = host.krr_pack_concat_strip_pieces(ptr_addr + a * 8, lens[a:].ctypes.data, b - a,
                                                   boffs[a:].ctypes.data, stage.data_ptr() + lo, self.threads,
                                                   max_pieces, new_lens[a:].ctypes.data, p_start.ctypes.data,
                                                   p_out.ctypes.data, ctypes.byref(n_p))
            if rc != KRR_PACK_OK:
                raise PrometheusResponseError(rc, "krr_pack_concat_strip_pieces failed")
            t_strip += time.perf_counter() - t_s
            np.cumsum(new_lens[a:b], out=no[a + 1:b + 1])
            no[a + 1:b + 1] += no[a]
            k = n_p.value
            pd = no[a] + np.concatenate([[0], np.cumsum(p_out[:k])[:-1]]).astype(np.int64)
            piece_dev.append(pd)
            piece_shift.append(p_start[:k] - pd)
            # every piece, then the chunk's body offsets: one native call of async copies
            dst = np.empty(k + 1, dtype=np.int64)
            src = np.empty(k + 1, dtype=np.int64)
            nby = np.empty(k + 1, dtype=np.int64)
            dst[:k], src[:k], nby[:k] = d_base + pd, s_base + p_start[:k], p_out[:k]
            dst[k], src[k], nby[k] = o_base + 8 * a, n_base + 8 * a, 8 * (b - a + 1)
            self.ctx.copy_h2d_batch(dst, src, nby, stream=cs)
            with torch.cuda.stream(cs):
                ev = torch.cuda.Event()
                ev.record(cs)
            st.wait_event(ev)
            launch(jb, a, b, tmp_v, None, int(no[a]), int(no[b]))
            a = b
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
                          stream=None, label: str = "pod") -> list:
        """Several (plan, bodies) pairs (e.g. CPU and memory) through ONE staging / copy /
        candidate-search pipeline; one DevicePacked per pair."""
        with self._lock, self._on(stream):
            return self._pack_grouped_multi(items, want_timestamps, return_pod_counts, None, label)

    def _pack_grouped_multi(self, items, want_ts, want_counts, stream, label) -> list:
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
        import time

        clock = [time.perf_counter()]  # phase ends (host clock; only the existing synchronisations)
        total_bytes = sum(len(b) for b in flat)
        cap = max(4096, total_bytes // 256)  # a series object with a few samples takes > 256 bytes
        cand = torch.empty(cap, dtype=torch.int64, device=dev)
        n_cand = torch.zeros(1, dtype=torch.int64, device=dev)
        segs = torch.empty((cap, 7), dtype=torch.int64, device=dev)
        seen = [0]  # positions below this were searched
        # per chunk: the candidate counter after its search, copied to page-locked memory, and an
        # event; the chunk's series are parsed one chunk later (its bytes are in HBM by then),
        # so the parse runs beside the next chunks' staging and copies, not after the last one
        LAG = 1  # chunks searched but not yet parsed: the host waits on the previous chunk's search
        # the parses run on streams of their own (a chunk holds one or two bodies = a few hundred
        # series = waves, far from filling the GPU): consecutive chunks' parses overlap each other
        # and the copies, instead of queueing behind the next chunk's copy on the launch stream
        pstreams = self._parse_streams()
        snaps = torch.zeros(max(len(flat), 1) + 1, dtype=torch.int64, pin_memory=True)
        snap_np = snaps.numpy()
        pend: list = []         # (event, snap index, body end) of searched, unparsed chunks
        waited = [0.0]
        parsed = [0, False]     # candidates parsed so far, overflow

        def parse_chunk(jb, tmp_v, tmp_t):
            ev, k, b_end = pend.pop(0)
            t_w = time.perf_counter()
            ev.synchronize()  # that chunk's search only: later copies keep streaming
            waited[0] += time.perf_counter() - t_w
            n = int(snap_np[k])
            lo = parsed[0]
            if parsed[1] or n > cap:
                parsed[1] = True
                return
            if n > lo:
                ps = pstreams[k % len(pstreams)]
                ps.wait_event(ev)
                with torch.cuda.stream(ps):
                    starts = torch.sort(cand[lo:n]).values
                    # the chunk's bodies' device offsets are in HBM (copied with the chunk)
                    body_of = torch.searchsorted(jb._keep[1][:b_end + 1], starts, right=True) - 1
                    self.ctx.json_parse_segments(jb, starts, body_of, label, want_ts, tmp_v, tmp_t, segs[lo:n],
                                                 stream=ps)
            parsed[0] = n

        def launch(jb, a, b, tmp_v, tmp_t, lo, hi):  # search each chunk as it lands
            last = b == len(flat)
            end = hi if last else max(hi - 16, seen[0])
            self.ctx.json_find_series(jb, cand, n_cand, begin=seen[0], end=end, limit=hi, stream=st)
            seen[0] = end
            k = len(done)  # this chunk's snapshot slot
            with torch.cuda.stream(st):
                snaps[k:k + 1].copy_(n_cand, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
            pend.append((ev, k, b))
            done.append(k)
            if len(pend) > LAG:
                parse_chunk(jb, tmp_v, tmp_t)

        done: list = []
        # timestamps cut while staging, as for per-pod bodies: the candidate search, the series
        # parse and the host's chain walk read structure, labels and value strings only
        lens, boffs, total, jb, tmp_v, tmp_t = self._upload(flat, want_ts, st, launch, strip=self.strip,
                                                            pieces=True)
        clock.append(time.perf_counter())
        while pend:
            parse_chunk(jb, tmp_v, tmp_t)
        for ps in pstreams:
            st.wait_stream(ps)
        clock.append(time.perf_counter())
        dev_offs, shift = self._layout[:2]
        pieces = self._layout[2] if len(self._layout) > 2 else None
        nc = parsed[0]
        if parsed[1]:
            return [host_fallback(r, body0[r + 1] - body0[r]) for r in range(len(items))]
        with torch.cuda.stream(st):
            segs_h = np.ascontiguousarray(segs[:nc].cpu().numpy())  # sync
        clock.append(time.perf_counter())
        host = load_library()
        stage = self._last[1]
        out = []
        for r, (plan, bodies) in enumerate(items):
            ns, n_obj, nb = plan.n_slots, plan.n_objects, body0[r + 1] - body0[r]
            slot_src = np.empty(ns, dtype=np.int64)
            slot_cnt = np.empty(ns, dtype=np.int64)
            body_ok = np.empty(max(nb, 1), dtype=np.int32)
            b_offs = np.ascontiguousarray(dev_offs[body0[r]:body0[r + 1] + 1])
            pdev, psh = pieces if pieces is not None else (np.zeros(0, np.int64), np.zeros(0, np.int64))
            rc = host.krr_pack_route_grouped_pieces(
                stage.data_ptr(), b_offs.ctypes.data, nb, pdev.ctypes.data, psh.ctypes.data, pdev.size,
                label.encode(), segs_h.ctypes.data, nc, plan.slot_group.ctypes.data, plan._names or b"\0",
                plan._name_offsets.ctypes.data, ns, slot_src.ctypes.data, slot_cnt.ctypes.data, body_ok.ctypes.data,
                self.threads)
            if rc != KRR_PACK_OK:
                raise PrometheusResponseError(rc, "krr_pack_route_grouped failed")
            if not body_ok[:nb].all():
                out.append(host_fallback(r, int((body_ok[:nb] == 0).sum())))
                continue
            kept = np.maximum(slot_cnt, 0)
            dst = np.zeros(ns, dtype=np.int64)
            if ns > 1:
                np.cumsum(kept[:-1], out=dst[1:])
            seg = np.zeros(n_obj, dtype=np.int64)
            np.add.at(seg, plan.slot_obj, kept)
            offsets = np.zeros(n_obj + 1, dtype=np.int64)
            np.cumsum(seg, out=offsets[1:])
            n_vals = int(offsets[-1])
            with torch.cuda.stream(st):
                values = torch.empty(max(n_vals, 1), dtype=torch.float64, device=dev)
                ts = torch.empty(max(n_vals, 1), dtype=torch.float64, device=dev) if want_ts else None
                if ns:
                    d = [torch.from_numpy(x).to(dev) for x in (np.maximum(slot_src, 0), kept, dst)]
                    self.ctx.json_gather(d[0], d[1], d[2], tmp_v, tmp_t, values, ts, stream=st)
                offs_d = torch.from_numpy(offsets).to(dev)
            series = PackedSeries(values[:n_vals], offs_d, int(seg.max()) if n_obj else 0)
            out.append(DevicePacked(series, "device", 0, slot_cnt if want_counts else None,
                                    ts[:n_vals] if ts is not None else None))
        clock.append(time.perf_counter())
        # seconds per phase: staging + copies + search (+ the parse of all chunks but the last),
        # the last chunk's parse, the segments to the host, chain / route / gather enqueue
        self.last_grouped_phases = dict(zip(("stage_copy_search", "last_parse", "segments_d2h", "route_gather"),
                                            np.diff(clock).round(5).tolist()), parse_wait=round(waited[0], 5),
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
