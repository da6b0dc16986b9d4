"""Kubernetes quantity parsing for ResourceAllocations (reference robusta_krr/utils/resource_units.py:21-26).

Only ``parse`` is on the strategy boundary (it feeds ResourceAllocations'
validator); display formatting belongs to the formatters, which are unchanged.
"""
from __future__ import annotations

from decimal import Decimal

# Suffix -> multiplier, checked in this order (binary before decimal, "m" first).
_SUFFIXES = (
    ("m", Decimal("1e-3")),
    ("Ki", Decimal(2**10)), ("Mi", Decimal(2**20)), ("Gi", Decimal(2**30)),
    ("Ti", Decimal(2**40)), ("Pi", Decimal(2**50)), ("Ei", Decimal(2**60)),
    ("k", Decimal(1e3)), ("M", Decimal(1e6)), ("G", Decimal(1e9)),
    ("T", Decimal(1e12)), ("P", Decimal(1e15)), ("E", Decimal(1e18)),
)


def parse(quantity: str) -> Decimal:
    for suffix, mult in _SUFFIXES:
        if quantity.endswith(suffix):
            return Decimal(quantity[: -len(suffix)]) * mult
    return Decimal(quantity)
