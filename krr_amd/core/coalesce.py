"""Per-object ``run()`` calls coalesced into fleet launches.

The reference's Runner calls ``strategy.run(history, object)`` once per object, each
from a default-executor thread (``asyncio.to_thread``, robusta_krr/core/runner.py:104-106),
as the object's Prometheus queries complete.  Run one by one, every call would be a
pack + H2D + launch + D2H of its own.  ``RunCoalescer`` turns the calls that overlap
into one kernel pass: the first caller becomes the leader and launches what is pending
(its own object included); calls arriving meanwhile queue up, and when the launch
returns the leader hands leadership to the oldest queued caller, whose launch takes
every call queued by then.  No timer: a lone call launches at once, and a burst
batches itself behind the launch in flight.

Each caller turns its own row of the shared raw results into its RunResult in its own
thread, so a per-object exception (a NaN memory sample raises InvalidOperation, as
``max()`` over Decimals does in the reference) reaches that caller only.  Results do
not depend on the batch: every object is an independent segment of the launch.
"""
from __future__ import annotations

import threading
from typing import Any, Callable, Optional, Sequence


class _Call:
    __slots__ = ("history", "wake", "lead", "raw", "index", "error")

    def __init__(self, history):
        self.history = history
        self.wake = threading.Event()
        self.lead = False
        self.raw = None
        self.index = -1
        self.error: Optional[BaseException] = None


class RunCoalescer:
    """``submit(history) -> (raw, index)``: raw results of a launch that covered this
    history at row ``index``.  ``run_raw(histories) -> raw`` is the fleet pass (one
    kernel launch); at most ``max_batch`` histories go into one launch."""

    def __init__(self, run_raw: Callable[[Sequence[Any]], Any], max_batch: int = 16384):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self._run_raw = run_raw
        self._max = int(max_batch)
        self._lock = threading.Lock()
        self._pending: list[_Call] = []
        self._busy = False
        self.calls = 0      # submitted histories
        self.launches = 0   # fleet passes run

    def submit(self, history):
        call = _Call(history)
        with self._lock:
            self.calls += 1
            self._pending.append(call)
            if not self._busy:
                self._busy = True
                call.lead = True
        if not call.lead:
            call.wake.wait()  # done, or promoted to leader
        if call.lead:
            self._lead(call)
        if call.error is not None:
            raise call.error
        return call.raw, call.index

    def _lead(self, me: _Call) -> None:
        with self._lock:
            batch, self._pending = self._pending[: self._max], self._pending[self._max:]
            self.launches += 1
        raw, err = None, None
        try:
            raw = self._run_raw([c.history for c in batch])
        except BaseException as e:  # every caller of this launch sees the launch's failure
            err = e
        for i, c in enumerate(batch):
            c.raw, c.index, c.error, c.lead = raw, i, err, False
        with self._lock:
            if self._pending:  # the oldest queued call leads the next launch
                nxt = self._pending[0]
                nxt.lead = True
                nxt.wake.set()
            else:
                self._busy = False
        for c in batch:
            if c is not me:
                c.wake.set()


__all__ = ["RunCoalescer"]
