"""Exact-decimal post-processing of raw proposals (host, O(objects)).

Restates the reference's rounding and minimum clamp bit-for-bit:
  Runner.__get_resource_minimal  robusta_krr/core/runner.py:49-55
  Runner._round_value            robusta_krr/core/runner.py:57-77
  Runner._format_result          robusta_krr/core/runner.py:79-86
with Config.cpu_min_value = 5 (millicores) and memory_min_value = 10 (MB)
(robusta_krr/core/models/config.py:26-27).

All arithmetic runs in Python's default decimal context (prec=28,
ROUND_HALF_EVEN, InvalidOperation/DivisionByZero/Overflow trapped) — the
context the reference's event-loop and worker threads use.  Doing this in
float64 is wrong (ceil(2.007*1000) = 2008 in float, 2007 in Decimal), which is
why the GPU returns raw float64 samples and the rounding stays here.
"""
from __future__ import annotations

import decimal
import math
from decimal import Decimal
from typing import Optional

from krr_amd.core.abstract.strategies import ResourceRecommendation, RunResult
from krr_amd.core.models.allocations import ResourceType

DEFAULT_CPU_MIN_VALUE = 5
DEFAULT_MEMORY_MIN_VALUE = 10


def reference_context() -> decimal.Context:
    return decimal.Context(prec=28, rounding=decimal.ROUND_HALF_EVEN, Emin=-999999, Emax=999999,
                           capitals=1, clamp=0, flags=[],
                           traps=[decimal.InvalidOperation, decimal.DivisionByZero, decimal.Overflow])


def resource_minimal(resource: ResourceType, cpu_min_value: int = DEFAULT_CPU_MIN_VALUE,
                     memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE) -> Decimal:
    # Decimal(1 / 1000) is the binary float 0.001 made exact, so the CPU floor is
    # 0.005000000000000000104083408559 after the context's 28-digit rounding.
    with decimal.localcontext(reference_context()):
        if resource == ResourceType.CPU:
            return Decimal(1 / 1000) * cpu_min_value
        if resource == ResourceType.Memory:
            return Decimal(1_000_000) * memory_min_value
        return Decimal(0)


def round_value(value: Optional[Decimal], resource: ResourceType, cpu_min_value: int = DEFAULT_CPU_MIN_VALUE,
                memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE) -> Optional[Decimal]:
    if value is None:
        return None
    if value.is_nan():
        return Decimal("nan")
    with decimal.localcontext(reference_context()):
        if resource == ResourceType.CPU:
            scale = Decimal(10**3)  # 1m granularity
        elif resource == ResourceType.Memory:
            scale = 1 / Decimal(10**6)  # 1M granularity
        else:
            scale = Decimal(1)
        rounded = Decimal(math.ceil(value * scale)) / scale
        return max(rounded, resource_minimal(resource, cpu_min_value, memory_min_value))


def format_result(result: RunResult, cpu_min_value: int = DEFAULT_CPU_MIN_VALUE,
                  memory_min_value: int = DEFAULT_MEMORY_MIN_VALUE) -> RunResult:
    return {
        resource: ResourceRecommendation(
            request=round_value(rec.request, resource, cpu_min_value, memory_min_value),
            limit=round_value(rec.limit, resource, cpu_min_value, memory_min_value),
        )
        for resource, rec in result.items()
    }
