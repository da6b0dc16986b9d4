"""The C-ABI library builds, loads and exports every symbol include/krr_amd.h declares.

No compute calls here (no GPU in the CPU suite): only argument validation paths
that return before touching a device.
"""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "krr_amd.h")


def _declared():
    text = open(HEADER).read()
    return set(re.findall(r"^(?:int|int64_t|const char\*)\s+(krr_\w+)\(", text, flags=re.M))


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g

    g.build()
    from krr_amd import _native

    return _native.load_library()


def test_header_matches_binding_table():
    from krr_amd import _native

    assert _declared() == set(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(lib):
    from krr_amd import _native

    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = _declared() - exported
    assert not missing, f"missing exports: {missing}"
    for name in _declared():
        assert hasattr(lib, name)


def test_library_is_gfx950_code_object(lib):
    from krr_amd import _native

    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", "--string-dump=.hip_fatbin",
                          _native.LIB_PATH], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_abi_version_and_null_handling(lib):
    assert lib.krr_abi_version() == 3
    assert lib.krr_last_error(None) == b"null krr_ctx"
    assert lib.krr_segmented_percentile(None, None, None, None, None, None, None) == -1
    assert lib.krr_segmented_max(None, None, None, None, None, None) == -1
    assert lib.krr_destroy(None) == 0
    assert lib.krr_json_parse(None, None, 0, 0, 0, None, None, None, None, None) == -1
    assert lib.krr_json_compact(None, None, None, None, None, None, None, None, None, None) == -1
    assert lib.krr_json_find_series(None, None, 0, 0, 0, None, 0, None, None) == -1
    assert lib.krr_json_parse_segments(None, None, None, None, 0, None, 0, None, None, None, None) == -1
    assert lib.krr_json_gather(None, 0, None, None, None, None, None, None, None, None) == -1
    h = ctypes.c_void_p()
    assert lib.krr_create(0, None) == -1


def test_struct_layouts_match_header():
    from krr_amd import _native

    assert ctypes.sizeof(_native.KrrSeries) == 8 * 5 + 4 * 2
    assert ctypes.sizeof(_native.KrrPercentileParams) == 4 * 2 + 8 * 5
    assert ctypes.sizeof(_native.KrrSketchLoc) == 8 * 5 + 4 * 4 and _native.LOC_WORDS == 7
    assert ctypes.sizeof(_native.KrrJsonBodies) == 8 * 4


def _declared_host():
    out = set()
    for h in ("krr_pack.h", "krr_round.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        out |= set(re.findall(r"^(?:int|int64_t|void|const char\*)\s+(krr_\w+)\(", text, flags=re.M))
    return out


def test_host_headers_match_binding_table_and_exports():
    """libkrr_host.so (JSON packer + exact rounding) exports exactly what
    include/krr_pack.h and include/krr_round.h declare."""
    import __graft_entry__ as g

    g.build()
    from krr_amd.core import prom_native

    declared = _declared_host()
    assert declared == set(prom_native.EXPORTED_SYMBOLS)
    lib = prom_native.load_library()
    for name in declared:
        assert hasattr(lib, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", prom_native.LIB_PATH], capture_output=True, text=True)
    exported = {ln.split()[-1] for ln in nm.stdout.splitlines() if " T " in ln}
    assert declared <= exported
    assert {s for s in exported if s.startswith("krr_")} == declared


def test_select_plan_layout_and_null_handling(lib):
    from krr_amd import _native

    assert ctypes.sizeof(_native.KrrSelectPlanInfo) == 4 * 2 + 8 * 3 + 4 * 2
    assert lib.krr_gather_results(None, None, 0, None, 0, None, None, None) == -1
    assert lib.krr_comm_unique_id(None, None) == -1
    assert lib.krr_comm_init(None, 1, None, 0, None) == -1
    assert lib.krr_comm_init_timeout(None, 1, None, 0, 1.0, None) == -1
    assert lib.krr_comm_destroy(None, None) == -1
    assert lib.krr_synth_fill_global(None, None, None, 0, 0, 0, 0, 0, 0, 0, 0, None) == -1
    info = _native.KrrSelectPlanInfo()
    assert lib.krr_select_plan(-1, None, ctypes.byref(info)) == -1


def _plan(L, p, mode="linear"):
    from decimal import Decimal

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    return _native.select_plan(L, percentile_params(Decimal(p), mode))


@pytest.mark.parametrize("L,p,hselect,probe,bottom,fused", [
    (50400, "99", 0, 1, 0, 0),    # headline: ~507 kept keys; the start-threshold probe saves compactions
    (50400, "98", 1, 0, 0, 0),    # 2% kept, a 1,664-key buffer: window select alone, single pass fused (r02/q)
    (50400, "97", 1, 0, 0, 0),    # 1,515 kept keys (3%): the same split
    (50400, "96", 1, 0, 0, 1),    # 4% kept: window select (krr_plan.h window_select, A/B r02 ab18/ab19)
    (50400, "94", 1, 0, 0, 1),
    (50400, "50", 1, 0, 0, 1),    # mid percentile: window select
    (50400, "93", 1, 0, 0, 1),    # 4,224 keys would be needed
    (50400, "5", 1, 0, 1, 1),     # low percentiles keep the bottom side, which has no probe
    (50400, "6", 1, 0, 1, 1),
    (50400, "3", 1, 0, 1, 1),     # 1,515 bottom keys: just past the 3% kept-fraction rule of the 2,560-key cap
    (50400, "2", 1, 0, 1, 0),     # 1,012 bottom keys: the p98 split mirrored (no probe on the bottom side)
    (50400, "1", 0, 0, 1, 0),
    (100800, "97", 1, 0, 0, 1),   # 3,027 kept keys: the window beats the probe-backed 3,712-key buffer both ways
    (100800, "96", 1, 0, 0, 1),
    (20160, "97", 0, 1, 0, 0),    # config 3's longest segment: 608 kept keys, a 1,280-key buffer
    (20160, "96", 1, 0, 0, 1),    # 810 kept keys, 4%: window select
    (20160, "95", 1, 0, 0, 1),
    (10080, "95", 0, 1, 0, 0),    # a 1,152-key buffer: the single pass never loses there
    (172800, "99", 1, 0, 0, 0),   # 30d@15s p99, 1% kept: window alone (4.42 -> 4.23 ms), single pass fused
    (172800, "99.9", 0, 1, 0, 0),
])
def test_select_plan_decisions(lib, L, p, hselect, probe, bottom, fused):
    """krr_select_plan reports the path each launch takes (krr_plan.h single_pass_ok /
    window_select) — the percentile-only launch and, in fused_hselect, krr_simple_run's —
    so the big-buffer boundary, the kept-fraction rules of the window select and the
    top-side-only probe are pinned without a GPU."""
    info = _plan(L, p)
    assert (info.hselect, info.probe, info.bottom, info.fused_hselect) == (hselect, probe, bottom, fused), \
        (p, info.tkeep, info.cap_keys)
    if hselect:
        assert info.cap_keys == 0
    else:
        assert info.tkeep < info.cap_keys <= 3712 and info.lds_bytes == 1536 + 8 * info.cap_keys


def test_select_plan_ref_index_is_not_a_selection(lib):
    from decimal import Decimal

    from krr_amd import _native
    from krr_amd.core.engine import percentile_params

    with pytest.raises(_native.NativeError):
        _native.select_plan(50400, percentile_params(Decimal("99"), "ref_index"))
