"""Decimal view of a float64 sample exactly as the reference sees it.

Prometheus serialises each sample with Go's ``strconv.FormatFloat(v, 'f', -1, 64)``
(shortest round-trip digits, positional notation, "NaN", "+Inf", "-Inf"), and
the reference parses that string with ``Decimal(value)``
(robusta_krr/core/integrations/prometheus.py:152).  ``prom_decimal(x)`` rebuilds
that Decimal from the float64 the kernels return, so host-side exact arithmetic
(memory buffer, rounding) sees the same digits and exponent as the reference.
Python's ``repr`` gives the same shortest round-trip digits as Go.
"""
from __future__ import annotations

import math
from decimal import Decimal


def prom_format(x: float) -> str:
    """The string Prometheus would put in a range-query result for sample x."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "+Inf" if x > 0 else "-Inf"
    return format(prom_decimal(x), "f")


def prom_decimal(x: float) -> Decimal:
    """Decimal(FormatFloat(x, 'f', -1, 64)) without going through a string."""
    if math.isnan(x):
        return Decimal("NaN")
    if math.isinf(x):
        return Decimal("Infinity") if x > 0 else Decimal("-Infinity")
    sign, digits, exp = Decimal(repr(float(x))).as_tuple()
    digits = list(digits)
    if exp > 0:  # 'f' format never uses an exponent
        digits += [0] * exp
        exp = 0
    while exp < 0 and len(digits) > 1 and digits[-1] == 0:  # shortest repr: no trailing zeros
        digits.pop()
        exp += 1
    if exp < 0 and digits == [0]:
        exp = 0
    return Decimal((sign, tuple(digits), exp))
