"""BASELINE.json configs[0] ("config 1"): the reference's CPU-runnable workload.

100 containers x 3 pods x 7 days at a 1-minute step (10,080 samples per pod and resource),
CPU ~ Gamma(k=2, theta=0.05) cores, memory = floor(Normal(2e8, 2e7)) bytes, numpy PCG64
seed 0.  Samples are float64 and travel as the shortest-repr strings
Prometheus sends (`krr_amd.utils.prom_decimal.prom_format`), so the reference sees
`Decimal(prom_format(x))` (`robusta_krr/core/integrations/prometheus.py:152`).

Shared by `make_config1_golden.py` (which runs the reference on it, build container only)
and the tests (which regenerate the inputs and check `input_sha256` before comparing).
"""
from __future__ import annotations

import hashlib

import numpy as np

OBJECTS = 100
PODS = 3
SAMPLES = 10_080
SEED = 0


def inputs():
    """(cpu, mem): float64 arrays of shape [OBJECTS, PODS, SAMPLES], in the draw order
    object -> pod -> (cpu series, memory series)."""
    rng = np.random.default_rng(SEED)
    cpu = np.empty((OBJECTS, PODS, SAMPLES))
    mem = np.empty((OBJECTS, PODS, SAMPLES))
    for o in range(OBJECTS):
        for p in range(PODS):
            cpu[o, p] = rng.gamma(2.0, 0.05, SAMPLES)
            mem[o, p] = np.floor(rng.normal(2e8, 2e7, SAMPLES))
    return cpu, mem


def sha256(cpu: np.ndarray, mem: np.ndarray) -> str:
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(cpu, dtype="<f8").tobytes())
    h.update(np.ascontiguousarray(mem, dtype="<f8").tobytes())
    return h.hexdigest()


def pod_names(o: int) -> list[str]:
    return [f"app-{o:03d}-pod-{p}" for p in range(PODS)]
