"""The reference's CPU index rule, k(n) = int((n - 1) * p / 100), for every p it accepts.

``SimpleStrategySettings.calculate_cpu_proposal`` (robusta_krr/strategies/simple.py:31-36)
evaluates ``int((len(data_) - 1) * self.cpu_percentile / 100)`` with whatever object the
setting holds (simple.py:17-19 accepts any value in (0, 100]):

* a ``Decimal`` (the CLI path, and any value pydantic validated): the product is ROUNDED to
  the context's 28 significant digits (``reference_context``) before the division, which is
  then exact, and ``int`` truncates.  While ``(n-1)·p`` has at most 28 significant digits the
  product is exact and k is the exact floor ``floor((n-1)·p/100)`` the kernels compute in
  128-bit integers.  Past that the rounding can carry the product up to the next multiple of
  100: ``p = 99.99999999999999999999999999`` gives k(3) = 2 where the floor is 1.  Rounding is
  monotone and multiples of 100 are representable, so k(n) is the exact floor or one more.
* the default ``int`` 99 (pydantic v1 does not validate defaults): ``(n-1)·99`` is an exact
  int and ``/ 100`` a correctly rounded float, equal to the exact floor while the quotient is
  below 2^46 (its fraction, a multiple of 0.01, stays farther than half an ulp from 1).
* anything else (a float assigned after validation, a Fraction ...): its own arithmetic.

``IndexRule`` answers which n the exact floor covers (``exact_upto``) and, beyond that, builds
the table k[n] the kernels read (``krr_percentile_params.k_table``): the literal expression
evaluated on the host for every n whose float estimate of (n-1)·p/100 lies near an integer,
the float floor elsewhere (there the exact floor and the rounded one agree, and the float is
far enough from an integer to floor correctly).
"""
from __future__ import annotations

import decimal
import math
import threading
from decimal import Decimal
from fractions import Fraction

import numpy as np

from krr_amd.core.rounding import reference_context

# the kernels' exact floor takes p = p_num / p_den with p_den <= 1e15 (include/krr_amd.h)
KERNEL_P_DEN_MAX = 10**15
_INT_EXACT_UPTO = 1 << 46


def _sig_digits(d: Decimal) -> int:
    """Significant digits of a finite Decimal's value (trailing zeros do not count)."""
    digits = d.normalize(decimal.Context(prec=max(len(d.as_tuple().digits), 1))).as_tuple().digits
    return max(len(digits), 1)


class IndexRule:
    """k(n) for one ``cpu_percentile`` object, as the reference evaluates it."""

    def __init__(self, percentile):
        if isinstance(percentile, bool):
            raise TypeError("cpu_percentile must be a number")
        self.percentile = percentile
        try:
            frac = Fraction(percentile)
        except (TypeError, ValueError, OverflowError) as e:
            raise ValueError(f"percentile must be a finite number in (0, 100], got {percentile!r}") from e
        if not (0 < frac <= 100):
            raise ValueError(f"percentile must be in (0, 100], got {percentile}")
        self.fraction = frac
        self.kernel_exact = frac.denominator <= KERNEL_P_DEN_MAX and frac.numerator <= 100 * KERNEL_P_DEN_MAX
        if isinstance(percentile, int):
            self.exact_upto = _INT_EXACT_UPTO
        elif isinstance(percentile, Fraction):
            self.exact_upto = math.inf
        elif isinstance(percentile, Decimal):
            prec = reference_context().prec
            free = prec - _sig_digits(percentile)  # digits left for n - 1 in an exact product
            self.exact_upto = 10**free if free > 0 else 1
        else:  # float and the like: the float product rounds at any n
            self.exact_upto = 1
        self._lock = threading.Lock()
        self._table = np.zeros(1, dtype=np.int64)
        self._device: dict = {}

    # ---- the rule ----------------------------------------------------------------------------
    def approx(self) -> tuple[int, int]:
        """(p_num, p_den) for the kernels: p itself when it fits, else the closest fraction with
        p_den <= 1e15 (it sizes selection buffers only; the table carries k)."""
        f = self.fraction
        if not self.kernel_exact:
            f = f.limit_denominator(KERNEL_P_DEN_MAX)
            f = min(max(f, Fraction(1, KERNEL_P_DEN_MAX)), Fraction(100))
        return f.numerator, f.denominator

    def needs_table(self, max_n: int) -> bool:
        """Do segments of up to max_n samples need the table (else the exact floor is k)?"""
        return not (self.kernel_exact and int(max_n) <= self.exact_upto)

    def literal(self, n: int) -> int:
        """The reference's expression itself (simple.py:36) for n >= 1 samples."""
        with decimal.localcontext(reference_context()):
            return int((int(n) - 1) * self.percentile / 100)

    def k(self, n: int) -> int:
        n = int(n)
        if n <= self.exact_upto:
            f = self.fraction
            return (n - 1) * f.numerator // (100 * f.denominator)
        return self.literal(n)

    def ks(self, ns) -> np.ndarray:
        """k(n) elementwise (n >= 1), int64."""
        ns = np.asarray(ns, dtype=np.int64)
        if ns.size == 0:
            return np.zeros(0, dtype=np.int64)
        top = int(ns.max())
        if top <= self.exact_upto and self.kernel_exact:
            f = self.fraction
            a = ns - 1
            if top * f.numerator < 2**63:
                return (a * f.numerator) // (100 * f.denominator)
            return np.array([(int(x) * f.numerator) // (100 * f.denominator) for x in a], dtype=np.int64)
        return self.table(top)[ns]

    # ---- the table the kernels read ------------------------------------------------------------
    def table(self, max_n: int) -> np.ndarray:
        """int64 [max_n + 1]: k(n) at index n (entry 0 unused, 0).  Grown and cached."""
        max_n = int(max_n)
        with self._lock:
            have = self._table.size - 1
            if max_n > have:
                self._table = np.concatenate([self._table, self._build(have + 1, max_n + 1)])
            return self._table[: max_n + 1]

    def _build(self, lo: int, hi: int) -> np.ndarray:
        """k(n) for n in [lo, hi): the float estimate's floor, and the literal expression where
        the estimate is within its error bound (plus the rounding's reach) of an integer."""
        n = np.arange(lo, hi, dtype=np.int64)
        x = (n - 1).astype(np.float64) * (float(self.fraction) / 100.0)
        k = np.floor(x)
        frac = x - k
        # the estimate's error is a few ulps of x, and the 28-digit rounding of the product moves
        # it by ~1e-27 x: both far inside 1e-14 x (no absolute term: floor(x) = 0 below 1 - eps)
        eps = 1e-14 * x
        near = np.flatnonzero((frac < eps) | (frac > 1.0 - eps) | (n <= 1))
        out = k.astype(np.int64)
        for i in near.tolist():
            out[i] = self.literal(int(n[i])) if n[i] >= 1 else 0
        if lo == 0:
            out[0] = 0
        return out

    def device_table(self, max_n: int, device: int):
        """The table on a HIP device (torch int64 tensor, cached per device; grown on demand)."""
        import torch

        max_n = int(max_n)
        key = int(device)
        with self._lock:
            t = self._device.get(key)
        if t is not None and t.numel() > max_n:
            return t
        # round the length up so that nearby sizes share one upload
        want = max(max_n + 1, 1024)
        want = 1 << (want - 1).bit_length()
        host = torch.from_numpy(np.ascontiguousarray(self.table(want - 1)))
        t = host.to(torch.device("cuda", key))
        with self._lock:
            self._device[key] = t
        return t

    def __repr__(self) -> str:
        return f"IndexRule({self.percentile!r}, exact_upto={self.exact_upto})"

    @classmethod
    def of(cls, percentile) -> "IndexRule":
        """The shared rule of a percentile object (its tables are built once per process)."""
        key = (type(percentile), str(percentile))
        with _RULES_LOCK:
            rule = _RULES.get(key)
            if rule is None:
                rule = _RULES[key] = cls(percentile)
                while len(_RULES) > 64:
                    _RULES.pop(next(iter(_RULES)))
            return rule


_RULES: dict = {}
_RULES_LOCK = threading.Lock()

__all__ = ["IndexRule", "KERNEL_P_DEN_MAX"]
