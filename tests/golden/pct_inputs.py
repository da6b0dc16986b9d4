"""Deterministic inputs of the cpu_percentile fixtures (simple_strategy_pct.json): shared by
the generator (make_golden.py, which runs the imported reference on them) and the tests
(which rebuild them here, on any box, with integer arithmetic only)."""
from __future__ import annotations

import numpy as np

# percentiles the reference accepts whose (n-1)·p needs more than the
# 28 digits of the Decimal context (or whose p_den passes 1e15), beside ordinary ones
PERCENTILES = ["99.99999999999999999999999999", "12.3456789012345678", "33.33333333333333333333333333", "1E-20",
               "99.9999999999999999", "66.66666666666666666666666667", "0.0000000000000000000000000001",
               "50.00000000000000000000000001", "99", "100"]
# sample counts of the full-run cases (one object each, split over up to three pods)
RUN_NS = [1, 2, 3, 1001, 10080, 172800, 1000003]
# counts of the index rows (k itself, via a range(n) sample list)
INDEX_NS = [1, 2, 3, 4, 7, 10, 11, 99, 100, 101, 1001, 1440, 10080, 10081, 30240, 50400, 172800, 172801,
            1000003]
INDEX_SCAN = 600  # plus every n in 1..INDEX_SCAN


def pods_of(n: int) -> list[int]:
    """Pod lengths of an n-sample object: three pods when n >= 3 (the last takes the rest)."""
    if n < 3:
        return [n]
    return [n // 3, n // 3, n - 2 * (n // 3)]


def cpu_values(n: int) -> np.ndarray:
    """n CPU samples (cores, 6 decimals) in position order: a multiplicative hash of the index,
    so the unsorted index rule picks a value that differs from its neighbours."""
    j = np.arange(n, dtype=np.int64)
    return ((j * 2654435761 + 12345) % 1000003).astype(np.float64) / 1e6


def mem_values(n: int) -> np.ndarray:
    """n memory samples (integral bytes around 1e8)."""
    j = np.arange(n, dtype=np.int64)
    return (100_000_000 + ((j * 40503 + 7) % 65521) * 997).astype(np.float64)
