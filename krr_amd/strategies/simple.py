"""SimpleStrategy on MI355X — the reference's default strategy
(robusta_krr/strategies/simple.py:16-49) with its per-sample work moved to HIP.

  CPU    = the sample at index k = floor((n-1) * p / 100) of the pods' samples
           concatenated in pod order, UNSORTED (simple.py:31-36)       [ref_index]
  Memory = max(samples) * Decimal(1 + b / 100)                     (simple.py:24-29)
  empty  -> Decimal('NaN');  CPU limit None, memory limit = request (simple.py:42-49)

``percentile_mode`` (build extension, default "ref_index" = reference parity):
  "sorted_lower" - sorted(samples)[k], the README's stated "99th percentile";
  "linear"       - np.percentile(samples, p) (numpy 2.2 method="linear"), bit-exact.

The GPU returns the selected/maximal float64 sample; the host rebuilds its
Decimal exactly as the reference parsed it (prom_decimal) and applies the
memory buffer in the reference's decimal context.  HistoryData whose Decimals
are not Prometheus' shortest strings ('0.10', 25-digit values ...) get the
reference's own sample object at the position the GPU located
(krr_amd.core.exact).
"""
from __future__ import annotations

import decimal
import enum
import threading
from decimal import Decimal
from typing import Optional, Sequence

import numpy as np
import pydantic.v1 as pd

from krr_amd import _native
from krr_amd.core.abstract.strategies import (
    BaseStrategy,
    HistoryData,
    K8sObjectData,
    ResourceRecommendation,
    ResourceType,
    RunResult,
    StrategySettings,
)
from krr_amd.core.engine import RawResults, default_engine, percentile_params
from krr_amd.core.packing import PackedFleet, pack_histories, pack_resource
from krr_amd.core.rounding import reference_context
from krr_amd.utils.prom_decimal import prom_decimal


class PercentileMode(str, enum.Enum):
    REF_INDEX = "ref_index"
    SORTED_LOWER = "sorted_lower"
    LINEAR = "linear"


class SimpleStrategySettings(StrategySettings):
    cpu_percentile: Decimal = pd.Field(
        99, gt=0, le=100, description="The percentile to use for the CPU recommendation."
    )
    memory_buffer_percentage: Decimal = pd.Field(
        5, gt=0, description="The percentage of added buffer to the peak memory usage for memory recommendation."
    )
    percentile_mode: PercentileMode = pd.Field(
        PercentileMode.REF_INDEX,
        description="CPU percentile rule: ref_index (reference KRR 1.0.0), sorted_lower, or linear (numpy).",
    )
    device: int = pd.Field(0, ge=0, description="HIP device that runs the kernels.")

    # --- the two proposal functions, same names and signatures as the reference ---
    def calculate_memory_proposal(self, data: dict[str, list[Decimal]]) -> Decimal:
        raw = self._run_single({ResourceType.CPU: {}, ResourceType.Memory: data})
        return self.memory_from_raw(raw, 0)

    def calculate_cpu_proposal(self, data: dict[str, list[Decimal]]) -> Decimal:
        raw = self._run_single({ResourceType.CPU: data, ResourceType.Memory: {}})
        return self.cpu_from_raw(raw, 0)

    # --- batched helpers ---
    def params(self) -> _native.KrrPercentileParams:
        return percentile_params(self.cpu_percentile, PercentileMode(self.percentile_mode).value)

    def memory_buffer(self) -> Decimal:
        with decimal.localcontext(reference_context()):
            return Decimal(1 + self.memory_buffer_percentage / 100)

    def run_fleet(self, fleet: PackedFleet, device: Optional[int] = None) -> RawResults:
        params = self.params()
        raw = default_engine(self.device if device is None else device).run_packed(fleet, params)
        if fleet.cpu.exact is not None or fleet.mem.exact is not None:
            from krr_amd.core.exact import resolve

            resolve(fleet, raw, params)
        return raw

    def run_fleet_records(self, fleet: PackedFleet, device: Optional[int] = None):
        """One kernel pass over a fleet shard -> int64 [S, 4] device records (multi-GPU path)."""
        return default_engine(self.device if device is None else device).run_packed_records(fleet, self.params())

    def _run_single(self, history: HistoryData) -> RawResults:
        return self.run_fleet(pack_histories([history]))

    def cpu_from_raw(self, raw: RawResults, i: int) -> Decimal:
        flags = int(raw.cpu_flags[i])
        if flags & _native.KRR_FLAG_CAPACITY:
            raise RuntimeError(f"object {i}: CPU selection bound violated (KRR_FLAG_CAPACITY)")
        if flags & _native.KRR_FLAG_EMPTY:
            return Decimal("NaN")
        ex = getattr(raw, "cpu_exact", None)
        if ex is not None and i in ex:  # the reference's own sample object
            return ex[i]
        if flags & _native.KRR_FLAG_NAN:
            # sorted() over Decimals compares with '<'; a NaN operand signals once any
            # comparison happens, i.e. when n >= 2 (one sample is never compared).
            if PercentileMode(self.percentile_mode) is PercentileMode.SORTED_LOWER and raw.cpu_count[i] >= 2:
                raise decimal.InvalidOperation([decimal.InvalidOperation])
            return Decimal("NaN")
        return prom_decimal(float(raw.cpu_value[i]))

    def memory_from_raw(self, raw: RawResults, i: int, buffer: Optional[Decimal] = None) -> Decimal:
        flags = int(raw.mem_flags[i])
        if flags & _native.KRR_FLAG_EMPTY:
            return Decimal("NaN")
        ex = getattr(raw, "mem_exact", None)
        if ex is not None and i in ex:  # max(data_) itself, times the buffer
            if buffer is None:
                buffer = self.memory_buffer()
            with decimal.localcontext(reference_context()):
                return ex[i] * buffer
        if flags & _native.KRR_FLAG_NAN:
            # max() over Decimals compares with '>' and a NaN operand signals
            # (simple.py:29) — unless n == 1, where nothing is compared and NaN passes.
            if raw.mem_count[i] >= 2:
                raise decimal.InvalidOperation([decimal.InvalidOperation])
            return Decimal("NaN")
        if buffer is None:
            buffer = self.memory_buffer()
        with decimal.localcontext(reference_context()):
            return prom_decimal(float(raw.mem_value[i])) * buffer


_COALESCER_LOCK = threading.Lock()


class SimpleStrategy(BaseStrategy[SimpleStrategySettings]):
    __display_name__ = "simple"

    def run(self, history_data: HistoryData, object_data: K8sObjectData) -> RunResult:
        """One object (the reference's per-object call, runner.py:106).  Calls that overlap
        in time — the reference Runner issues them from its executor threads — share one
        kernel launch (krr_amd.core.coalesce.RunCoalescer); the result is this object's
        alone, as run_batch([history_data])[0] would give it."""
        raw, i = self.coalescer().submit(history_data)
        return self.result_at(raw, i)

    def coalescer(self):
        c = self.__dict__.get("_coalescer")
        if c is None:
            from krr_amd.core.coalesce import RunCoalescer

            with _COALESCER_LOCK:
                c = self.__dict__.get("_coalescer")
                if c is None:
                    c = self.__dict__["_coalescer"] = RunCoalescer(
                        lambda hs: self.settings.run_fleet(self.pack(hs)))
        return c

    def result_at(self, raw: RawResults, i: int, buffer: Optional[Decimal] = None) -> RunResult:
        st = self.settings
        cpu = st.cpu_from_raw(raw, i)
        mem = st.memory_from_raw(raw, i, buffer)
        return {
            ResourceType.CPU: ResourceRecommendation(request=cpu, limit=None),
            ResourceType.Memory: ResourceRecommendation(request=mem, limit=mem),
        }

    def run_batch(self, histories: Sequence[HistoryData],
                  objects: Optional[Sequence[K8sObjectData]] = None) -> list[RunResult]:
        """One fleet-wide kernel pass for every object (the batched-runner hook)."""
        return self.results_from_raw(self.settings.run_fleet(self.pack(histories)))

    @staticmethod
    def pack(histories: Sequence[HistoryData]) -> PackedFleet:
        return PackedFleet(pack_resource(histories, ResourceType.CPU), pack_resource(histories, ResourceType.Memory))

    def format_packed(self, fleet: PackedFleet, cpu_min_value: int, memory_min_value: int) -> list[RunResult]:
        """Kernel pass + the reference's rounding (Runner._format_result) for a packed
        fleet, the rounding done in native exact-decimal code (krr_amd.core.fast_round):
        equal to format_result(r) for r in run_batch(...), ~20x cheaper per object."""
        return self.format_raw(self.settings.run_fleet(fleet), cpu_min_value, memory_min_value)

    def format_raw(self, raw: RawResults, cpu_min_value: int, memory_min_value: int) -> list[RunResult]:
        """Rounded RunResults from raw kernel results (e.g. records gathered from every rank)."""
        from krr_amd.core.fast_round import format_simple_batch

        return format_simple_batch(raw, self.settings, cpu_min_value, memory_min_value)

    def results_from_raw(self, raw: RawResults) -> list[RunResult]:
        buffer = self.settings.memory_buffer()
        return [self.result_at(raw, i, buffer) for i in range(int(np.asarray(raw.cpu_value).size))]
