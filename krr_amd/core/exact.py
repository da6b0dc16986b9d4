"""The reference's own sample object for HistoryData the float64 values do not reproduce.

The reference returns the selected SAMPLE OBJECT: ``data_[int((n-1)·p/100)]`` for the CPU
proposal (robusta_krr/strategies/simple.py:31-36; sorted first under this build's
SORTED_LOWER rule) and ``max(data_)`` for the memory peak (:24-29), multiplied by the buffer
in Decimal.  The kernels select float64 images.  For a segment whose Decimals are all what
Prometheus' shortest strings give (PackedSeries.exact None / class 0) the host rebuilds the
object from the float (prom_decimal).  For the others the GPU locates the answer and the
host returns the object at that position:

* class 1 (FAITHFUL: values equal their float's shortest repr, representations differ, e.g.
  ``Decimal('0.10')``, ``Decimal('2.00E+7')``): float order IS Decimal order with the same
  ties, so the located sample is the reference's — REF_INDEX: position k itself; memory:
  the first sample equal to the max (``max()`` keeps the first maximal one); SORTED_LOWER:
  the (k - #less)-th equal sample in position order (a stable sort's k-th element);
* class 2 (INEXACT: some sample holds more digits than a float64, so distinct values may
  share a float): float conversion is monotone, so the reference's answer is among the
  samples whose float equals the selected one (``krr_locate``'s ``eq`` of them, ranks
  [lt, lt + eq) of the sort).  One such sample: it is the answer.  Several: they are
  ordered by their own Decimal comparisons — ``max()`` over them, or ``sorted()`` and
  element ``k - lt`` — the only Decimal arithmetic left on the host, over that tie group.

LINEAR is defined on the float64 values (numpy's ``np.percentile``), so it needs nothing here.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from krr_amd import _native
from krr_amd.core.packing import EXACT_FAITHFUL, PackedFleet


def sample_at(pods: Sequence[Sequence], pos: int):
    """X[pos] of the concatenation of a segment's (non-empty) pod lists."""
    for samples in pods:
        n = len(samples)
        if pos < n:
            return samples[pos]
        pos -= n
    raise IndexError("position past the segment's samples")


def _index_k(n: int, params) -> int:
    from krr_amd.core.engine import index_rule_of

    return index_rule_of(params).k(n)


def resolve(fleet: PackedFleet, raw, params) -> None:
    """Fill ``raw.cpu_exact`` / ``raw.mem_exact`` (object index -> sample object) for the
    fleet's class >= 1 segments whose answer is one sample.  Segments whose answer is NaN by
    the NaN rules (max() / sorted() over a NaN raise for n >= 2) get no entry: the strategy's
    own rules apply to them, as for canonical segments."""
    empty_or_nan = _native.KRR_FLAG_EMPTY | _native.KRR_FLAG_NAN
    for name, ps, values, counts, flags in (("cpu", fleet.cpu, raw.cpu_value, raw.cpu_count, raw.cpu_flags),
                                            ("mem", fleet.mem, raw.mem_value, raw.mem_count, raw.mem_flags)):
        if ps.exact is None:
            continue
        if name == "cpu" and params.mode == _native.KRR_PCT_LINEAR:
            continue
        loc = (raw.locate or {}).get(name)
        out: dict = {}
        offsets = np.asarray(ps.offsets)
        for s in np.flatnonzero(ps.exact).tolist():
            f, n = int(flags[s]), int(counts[s])
            if f & _native.KRR_FLAG_EMPTY:
                continue
            pods = ps.sources[s]
            if name == "cpu" and params.mode == _native.KRR_PCT_REF_INDEX:
                out[s] = sample_at(pods, _index_k(n, params))  # data_[k], whatever it holds
                continue
            if n == 1:  # nothing compared: the one sample (NaN included)
                out[s] = sample_at(pods, 0)
                continue
            if f & empty_or_nan:
                continue
            lt, eq, pos = (int(a[s]) for a in loc)
            if pos < 0:
                raise RuntimeError(f"object {s}: the {name} answer was not located (krr_locate)")
            if ps.exact[s] == EXACT_FAITHFUL or eq == 1:
                out[s] = sample_at(pods, pos)
                continue
            # INEXACT: settle the float's tie group in the samples' own order
            seg = np.asarray(ps.values[offsets[s]:offsets[s + 1]])
            group = [sample_at(pods, i) for i in np.flatnonzero(seg == values[s]).tolist()]
            out[s] = max(group) if name == "mem" else sorted(group)[_index_k(n, params) - lt]
        setattr(raw, f"{name}_exact", out)


__all__ = ["resolve", "sample_at"]
