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
