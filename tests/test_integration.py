"""The reference-side binding (krr_amd.integration) reaches the HIP path.

Runs tests/reference_integration_check.py in a subprocess (it imports /root/reference with
the SURVEY §8(c) recipe, which aliases pydantic and stubs modules — kept out of this
process).  Skipped where /root/reference is absent (the GPU box).  The reference itself is
never copied; only its import in the build container is used as the checker.
"""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/robusta_krr/core/runner.py"

pytestmark = pytest.mark.skipif(not os.path.exists(REF), reason="reference not present (GPU box)")


def _check(*args):
    p = subprocess.run([sys.executable, os.path.join(HERE, "reference_integration_check.py"), *args],
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_reference_runner_routes_to_c_abi_without_gpu():
    """In this GPU-less container the reference's Runner, once patched, must fail with
    NativeUnavailable: it reached the C ABI instead of silently running simple.py:42-49."""
    r = _check("--engine", "native")
    assert r["raised"] == "NativeUnavailable", r
    assert r["hip_strategy"] == "krr_amd.strategies.simple.SimpleStrategy"
    assert r["settings_types"] == {"cpu_percentile": "Decimal", "memory_buffer_percentage": "Decimal"}


@pytest.mark.parametrize("path", ["cli_99_5", "default_int"])
def test_reference_runner_results_equal_reference(path):
    """With the device engine stood in for by the oracle, the patched reference Runner returns
    the reference's own ResourceAllocations, equal to its unpatched per-object path and to the
    config-1 golden strings; custom strategies keep the per-object path."""
    r = _check("--engine", "oracle", "--path", path)
    assert r["equals_reference_runner"] and r["equals_golden"], r
    assert r["result_types"] == ["robusta_krr.core.models.allocations.ResourceAllocations"]
    if path == "default_int":  # the int-default settings path survives the translation
        assert r["settings_types"] == {"cpu_percentile": "int", "memory_buffer_percentage": "int"}
    assert r["custom_strategy_not_routed"]
    # the reference's _format_result clamps 7 B to the 10 MB memory floor (runner.py:49-77)
    assert r["custom_strategy_rows"] == [["99", "10000000", "10000000"]] * 3


@pytest.mark.parametrize("path", ["cli_99_5", "default_int"])
def test_reference_runner_exact_histories(path):
    """install(Runner) with the reference's loader handing over hand-built Decimals ('0.10',
    '2.00E+7', 25-digit values, float-colliding pairs; tests/golden/simple_strategy_exact.json):
    the patched Runner returns the reference's own rounded values, equal to its unpatched run."""
    r = _check("--engine", "oracle", "--path", path, "--exact")
    assert r["equals_reference_runner"] and r["equals_golden"], r
    assert r["n_objects"] >= 30


@pytest.mark.parametrize("loader", ["bodies", "grouped"])
def test_reference_collect_result_native_loader_and_fleet_scan(loader):
    """install(Runner, loader=..., scan="fleet"): the reference's whole _collect_result against
    a fake Prometheus session.  The per-pod (or grouped) bodies go to the native packer —
    the reference's gather_data (Decimal per sample) never runs — and the Result built by
    scan_fleet out of the reference's own models equals the unpatched reference's, scan
    for scan and in score, every severity included.  The same run first takes the real
    engine through it: the device packer (loader="bodies") or the kernel call raises
    NativeUnavailable on this GPU-less host (no CPU fallback anywhere); the stand-in run
    packs with the host packer (parser="host")."""
    r = _check("--engine", "oracle", "--loader", loader, "--scan", "fleet", "--objects", "30")
    assert r["raised"] == "NativeUnavailable", r
    assert r["collect_patched"] and r["equals_reference_result"], r
    assert r["types"] == ["robusta_krr.core.models.result.ResourceScan", "robusta_krr.core.models.result.Result"]
    assert r["severities"] == ["CRITICAL", "GOOD", "OK", "UNKNOWN", "WARNING"]
    assert r["n_scans"] == 32 and r["gather_data_calls"] == 0 and r["native_packer_used"]
    assert r["same_window_and_step"]
    if loader == "bodies":  # the reference's own per-pod requests, one for one
        assert r["http_requests"]["patched"] == r["http_requests"]["reference"] == 2 * (30 * 3 + 2)
    else:  # one grouped query per (namespace, container) and resource
        assert r["http_requests"]["patched"] == 2
