"""bench.py's config-4 right-size leg on CPU: records -> rounding -> ResourceAllocations ->
ResourceScan/Result in bulk, checked inside the leg against the per-object reference path
(runner.py:49-131, result.py:33-150).  No GPU: the records are synthetic."""
import argparse

import numpy as np

import bench
from krr_amd import _native


def _records(n: int, seed: int = 3) -> np.ndarray:
    rng = np.random.default_rng(seed)
    cpu = rng.gamma(2.0, 0.17, n)                       # around the pool's 0.35-core currents
    mem = rng.uniform(0.8e8, 1.2e9, n)                  # around its 1e8-1e9 B currents
    cnt = rng.integers(1, 50_400, n).astype(np.int64)
    rec = np.empty((n, 4), dtype=np.int64)
    rec[:, 0] = cpu.view(np.int64)
    rec[:, 1] = mem.view(np.int64)
    rec[:, 2] = cnt
    rec[:, 3] = cnt
    empty = np.arange(n) % 97 == 5                      # a few empty series: NaN -> "?"
    rec[empty, 0] = np.array([np.nan]).view(np.int64)[0]
    rec[empty, 2] = np.int64(_native.KRR_FLAG_EMPTY) << 48   # count 0
    return rec


def test_right_size_leg_equals_per_object_path():
    n = 5000
    args = argparse.Namespace(percentile=99, cpu_threads=2)
    out = bench.config4_right_size(args, _records(n), [(0, 2500), (2500, n)])
    assert out["config4_right_size_equal_per_object_path"] is True
    assert out["config4_right_size_checked_objects"] >= 4096
    sev = out["config4_right_size_checked_pair_severities"]
    # the pool puts (resource, selector) pairs in every bucket the reference scores
    assert {"GOOD", "OK", "WARNING", "CRITICAL", "UNKNOWN"} <= set(sev), sev
    split = out["config4_right_size_split_s"]
    assert set(split) == {"unpack", "round", "decimal", "scan_and_score"}
    assert out["config4_scan_objects_per_s"] > 0
