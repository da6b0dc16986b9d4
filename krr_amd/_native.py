"""ctypes binding of libkrr_amd.so — the C ABI declared in include/krr_amd.h.

This is the only way the product path reaches the GPU.  There is no CPU or
eager-PyTorch fallback: if the shared library is missing, fails to load, or no
HIP device is present, every entry point raises NativeUnavailable.

PyTorch is used only as plumbing (device memory and the current HIP stream);
it is imported BEFORE the library is loaded so that libkrr_amd.so binds to the
HIP runtime torch already mapped (both carry the soname libamdhip64.so.7).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KRR_AMD_LIB", os.path.join(_HERE, "lib", "libkrr_amd.so"))

KRR_OK = 0
KRR_E_INVALID = -1
KRR_E_HIP = -2
KRR_E_CAPACITY = -3
KRR_KLL_ONE_PASS_TAIL = 1  # krr_kll_params.reserved (include/krr_amd.h)
KRR_KLL_TAIL_NO_MARGIN = 2  # testing: the tail pass's fallback stream
KRR_KLL_BODY_ONLY = 4  # the build leaves the tail to krr_kll_tail
KRR_E_UNSUPPORTED = -4
KRR_E_TIMEOUT = -5

KRR_PCT_REF_INDEX = 0
KRR_PCT_SORTED_LOWER = 1
KRR_PCT_LINEAR = 2

KRR_FLAG_NAN = 1
KRR_FLAG_CAPACITY = 2
KRR_FLAG_EMPTY = 4
KRR_FLAG_SKETCH_RANGE = 8
KRR_FLAG_WINDOW_MISS = 16

KRR_WIN_FAIL = 0x100
KRR_WIN_POINT = 0x200

# Every symbol include/krr_amd.h declares (tests/test_abi.py checks the export table).
EXPORTED_SYMBOLS = (
    "krr_abi_version",
    "krr_json_parse",
    "krr_json_compact",
    "krr_copy_h2d_batch",
    "krr_json_find_series",
    "krr_json_parse_segments",
    "krr_json_parse_segments_split",
    "krr_json_gather",
    "krr_create",
    "krr_destroy",
    "krr_last_error",
    "krr_segmented_percentile",
    "krr_segmented_max",
    "krr_simple_run",
    "krr_simple_run_records",
    "krr_simple_run_forward",
    "krr_simple_run_host",
    "krr_pack_records",
    "krr_synth_fill",
    "krr_synth_fill_window",
    "krr_synth_fill_global",
    "krr_sketch_width",
    "krr_sketch_build",
    "krr_sketch_query",
    "krr_kll_row_words",
    "krr_kll_build",
    "krr_kll_tail",
    "krr_kll_line_words",
    "krr_kll_build_lines",
    "krr_kll_tail_lines",
    "krr_kll_merge",
    "krr_kll_query",
    "krr_sketch_locate",
    "krr_sketch_range_count",
    "krr_sketch_collect",
    "krr_sketch_refine",
    "krr_rank_of",
    "krr_select_present",
    "krr_locate",
    "krr_window_key_cap",
    "krr_window_export",
    "krr_window_merge",
    "krr_select_plan",
    "krr_get_stats",
    "krr_comm_unique_id",
    "krr_comm_init",
    "krr_comm_init_timeout",
    "krr_comm_destroy",
    "krr_comm_info",
    "krr_gather_results",
)


class NativeUnavailable(RuntimeError):
    """The HIP extension (libkrr_amd.so) or a HIP device is not available."""


class NativeError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"libkrr_amd error {code}: {message}")
        self.code = code


class KrrSeries(ctypes.Structure):
    _fields_ = [
        ("values", ctypes.c_void_p),
        ("offsets", ctypes.c_void_p),
        ("n_segments", ctypes.c_int64),
        ("n_values", ctypes.c_int64),
        ("max_segment_len", ctypes.c_int64),
        ("gaps_are_nan", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class KrrPercentileParams(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("p_num", ctypes.c_int64),
        ("p_den", ctypes.c_int64),
        ("q", ctypes.c_double),
        ("k_table", ctypes.c_void_p),
        ("k_table_len", ctypes.c_int64),
    ]


def bind_index_table(params: KrrPercentileParams, max_n: Optional[int], device: int) -> KrrPercentileParams:
    """params with krr_percentile_params.k_table set when its index rule needs one for counts of
    up to max_n samples (``params.rule``: krr_amd.core.index_rule.IndexRule, attached by
    krr_amd.core.engine.percentile_params; the reference's int((n-1) * p / 100) for p whose
    product Decimal rounds).  Unchanged for LINEAR, an explicit table, or no rule."""
    rule = getattr(params, "rule", None)
    if rule is None or params.k_table or params.mode == KRR_PCT_LINEAR:
        return params
    if max_n is None:
        # unknown counts: bounded by what a device holds (2^40 float64 = 8 TiB, past any HBM);
        # the int default's float rule is exact to 2^46 and a <= 15-digit Decimal's to >= 10^13
        if not rule.needs_table(1 << 40):
            return params
        raise ValueError(f"cpu_percentile {rule.percentile!r} needs the reference's index table here: "
                         "pass the largest present count (max_n)")
    if not rule.needs_table(max_n):
        return params
    tab = rule.device_table(max_n, device)
    out = KrrPercentileParams(params.mode, params.reserved, params.p_num, params.p_den, params.q, tab.data_ptr(),
                              tab.numel())
    out.rule = rule
    out._keep = tab
    return out


class KrrSketchParams(ctypes.Structure):
    _fields_ = [
        ("mantissa_bits", ctypes.c_int32),
        ("min_exponent", ctypes.c_int32),
        ("octaves", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class KrrKllParams(ctypes.Structure):
    """include/krr_amd.h krr_kll_params: the KLL sketch (row format 2)."""
    _fields_ = [
        ("budget", ctypes.c_int32),
        ("slice", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("tail", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class KrrSketchLoc(ctypes.Structure):
    """include/krr_amd.h krr_sketch_loc (56 bytes): device arrays of it are int64
    tensors [S, LOC_WORDS] (little-endian word view; gamma as float64 bits)."""
    _fields_ = [
        ("n", ctypes.c_int64),
        ("r0", ctypes.c_int64),
        ("r1", ctypes.c_int64),
        ("before", ctypes.c_int64),
        ("gamma", ctypes.c_double),
        ("bin_lo", ctypes.c_uint32),
        ("bin_hi", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("mode", ctypes.c_int32),
    ]


LOC_WORDS = ctypes.sizeof(KrrSketchLoc) // 8


class KrrWindowHdr(ctypes.Structure):
    """include/krr_amd.h krr_window_hdr (40 bytes): device arrays of it are int64 tensors
    [S, HDR_WORDS] (lo, hi as key bits; cnt | flags << 32 in the last word)."""
    _fields_ = [
        ("lo", ctypes.c_uint64),
        ("hi", ctypes.c_uint64),
        ("below", ctypes.c_int64),
        ("n", ctypes.c_int64),
        ("cnt", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
    ]


HDR_WORDS = ctypes.sizeof(KrrWindowHdr) // 8


class KrrSelectPlanInfo(ctypes.Structure):
    """include/krr_amd.h krr_select_plan_info (40 bytes)."""
    _fields_ = [
        ("hselect", ctypes.c_int32),
        ("bottom", ctypes.c_int32),
        ("tkeep", ctypes.c_int64),
        ("cap_keys", ctypes.c_int64),
        ("lds_bytes", ctypes.c_int64),
        ("probe", ctypes.c_int32),
        ("fused_hselect", ctypes.c_int32),
    ]


class KrrJsonBodies(ctypes.Structure):
    """include/krr_amd.h krr_json_bodies."""
    _fields_ = [
        ("bodies", ctypes.c_void_p),
        ("body_offsets", ctypes.c_void_p),
        ("n_bodies", ctypes.c_int64),
        ("total_bytes", ctypes.c_int64),
    ]


KRR_JSON_OK, KRR_JSON_DROPPED, KRR_JSON_HOST = 0, 1, 2

NCCL_UNIQUE_ID_BYTES = 128

_lib = None
_lib_lock = threading.Lock()


def load_library(require_torch: bool = True) -> ctypes.CDLL:
    """Load libkrr_amd.so and declare every prototype.  Raises NativeUnavailable."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if require_torch:
            import torch  # noqa: F401  (bind to torch's HIP runtime first)
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - depends on the host
            raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
        vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
        sp, pp = ctypes.POINTER(KrrSeries), ctypes.POINTER(KrrPercentileParams)
        lib.krr_abi_version.argtypes = []
        lib.krr_abi_version.restype = ctypes.c_int
        lib.krr_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
        lib.krr_create.restype = ctypes.c_int
        lib.krr_destroy.argtypes = [vp]
        lib.krr_destroy.restype = ctypes.c_int
        lib.krr_last_error.argtypes = [vp]
        lib.krr_last_error.restype = ctypes.c_char_p
        lib.krr_segmented_percentile.argtypes = [vp, sp, pp, vp, vp, vp, vp]
        lib.krr_segmented_percentile.restype = ctypes.c_int
        lib.krr_segmented_max.argtypes = [vp, sp, vp, vp, vp, vp]
        lib.krr_segmented_max.restype = ctypes.c_int
        lib.krr_simple_run.argtypes = [vp, sp, sp, pp, vp, vp, vp, vp, vp, vp, vp]
        lib.krr_simple_run_records.argtypes = [vp, sp, sp, pp, vp, vp, vp, vp, vp, vp, vp, vp]
        lib.krr_simple_run_records.restype = ctypes.c_int
        lib.krr_simple_run_forward.argtypes = [vp, sp, sp, pp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, vp]
        lib.krr_simple_run_forward.restype = ctypes.c_int
        lib.krr_simple_run.restype = ctypes.c_int
        lib.krr_simple_run_host.argtypes = [vp, vp, vp, vp, vp, i64, i32, pp, vp, vp, vp, vp, vp, vp]
        lib.krr_simple_run_host.restype = ctypes.c_int
        lib.krr_pack_records.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp]
        lib.krr_pack_records.restype = ctypes.c_int
        lib.krr_synth_fill.argtypes = [vp, vp, vp, i64, u64, i32, i64, i32, vp]
        lib.krr_synth_fill.restype = ctypes.c_int
        lib.krr_synth_fill_window.argtypes = [vp, vp, vp, i64, u64, i32, i64, i32, i64, i64, vp]
        lib.krr_synth_fill_window.restype = ctypes.c_int
        lib.krr_synth_fill_global.argtypes = [vp, vp, vp, i64, u64, i32, i64, i32, i64, i64, i64, vp]
        lib.krr_synth_fill_global.restype = ctypes.c_int
        lib.krr_select_plan.argtypes = [i64, pp, ctypes.POINTER(KrrSelectPlanInfo)]
        lib.krr_select_plan.restype = ctypes.c_int
        lib.krr_get_stats.argtypes = [vp, ctypes.POINTER(i64)]
        lib.krr_get_stats.restype = ctypes.c_int
        lib.krr_comm_unique_id.argtypes = [vp, vp]
        lib.krr_comm_unique_id.restype = ctypes.c_int
        lib.krr_comm_init.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, ctypes.POINTER(vp)]
        lib.krr_comm_init.restype = ctypes.c_int
        lib.krr_comm_init_timeout.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_double, ctypes.POINTER(vp)]
        lib.krr_comm_init_timeout.restype = ctypes.c_int
        lib.krr_comm_destroy.argtypes = [vp, vp]
        lib.krr_comm_destroy.restype = ctypes.c_int
        lib.krr_comm_info.argtypes = [vp, vp, vp, vp]
        lib.krr_comm_info.restype = ctypes.c_int
        lib.krr_gather_results.argtypes = [vp, vp, ctypes.c_int, vp, i64, vp, vp, vp]
        lib.krr_gather_results.restype = ctypes.c_int
        skp = ctypes.POINTER(KrrSketchParams)
        lib.krr_sketch_width.argtypes = [skp]
        lib.krr_sketch_width.restype = i64
        lib.krr_sketch_build.argtypes = [vp, sp, skp, vp, vp, vp, vp, vp]
        lib.krr_sketch_build.restype = ctypes.c_int
        lib.krr_sketch_query.argtypes = [vp, i64, vp, vp, vp, skp, pp, vp, vp, vp, vp]
        lib.krr_sketch_query.restype = ctypes.c_int
        kkp = ctypes.POINTER(KrrKllParams)
        lib.krr_kll_row_words.argtypes = [kkp]
        lib.krr_kll_row_words.restype = i64
        lib.krr_kll_build.argtypes = [vp, sp, kkp, i64, vp, vp]
        lib.krr_kll_build.restype = ctypes.c_int
        lib.krr_kll_tail.argtypes = [vp, sp, kkp, vp, vp]
        lib.krr_kll_tail.restype = ctypes.c_int
        lib.krr_kll_line_words.argtypes = [i64]
        lib.krr_kll_line_words.restype = i64
        lib.krr_kll_build_lines.argtypes = [vp, sp, kkp, i64, vp, vp, i64, vp]
        lib.krr_kll_build_lines.restype = ctypes.c_int
        lib.krr_kll_tail_lines.argtypes = [vp, sp, kkp, vp, vp, i64, vp, vp]
        lib.krr_kll_tail_lines.restype = ctypes.c_int
        lib.krr_kll_merge.argtypes = [vp, i64, i32, vp, kkp, i64, vp, vp]
        lib.krr_kll_merge.restype = ctypes.c_int
        lib.krr_kll_query.argtypes = [vp, i64, i32, vp, kkp, i64, pp, vp, vp, vp, vp]
        lib.krr_kll_query.restype = ctypes.c_int
        lib.krr_rank_of.argtypes = [vp, sp, vp, vp, vp, vp]
        lib.krr_rank_of.restype = ctypes.c_int
        lib.krr_sketch_locate.argtypes = [vp, i64, vp, skp, pp, vp, vp]
        lib.krr_sketch_locate.restype = ctypes.c_int
        lib.krr_sketch_range_count.argtypes = [vp, i64, vp, skp, vp, vp, vp]
        lib.krr_sketch_range_count.restype = ctypes.c_int
        lib.krr_sketch_collect.argtypes = [vp, sp, skp, vp, vp, vp, vp, vp]
        lib.krr_sketch_collect.restype = ctypes.c_int
        lib.krr_sketch_refine.argtypes = [vp, sp, vp, vp, vp, vp, vp]
        lib.krr_sketch_refine.restype = ctypes.c_int
        lib.krr_select_present.argtypes = [vp, sp, vp, vp, vp]
        lib.krr_select_present.restype = ctypes.c_int
        lib.krr_locate.argtypes = [vp, sp, vp, vp, vp, vp, vp, vp]
        lib.krr_locate.restype = ctypes.c_int
        lib.krr_window_key_cap.argtypes = [i64, i64, pp]
        lib.krr_window_key_cap.restype = i64
        lib.krr_window_export.argtypes = [vp, sp, pp, i64, i64, vp, vp, vp]
        lib.krr_window_export.restype = ctypes.c_int
        lib.krr_window_merge.argtypes = [vp, i64, i32, i64, vp, vp, i64, pp, vp, vp, vp, vp, vp]
        lib.krr_window_merge.restype = ctypes.c_int
        jb = ctypes.POINTER(KrrJsonBodies)
        lib.krr_json_parse.argtypes = [vp, jb, i64, i64, i32, vp, vp, vp, vp, vp]
        lib.krr_json_parse.restype = ctypes.c_int
        lib.krr_json_compact.argtypes = [vp, jb, vp, vp, vp, vp, vp, vp, vp, vp]
        lib.krr_json_compact.restype = ctypes.c_int
        lib.krr_copy_h2d_batch.argtypes = [vp, i64, vp, vp, vp, vp]
        lib.krr_copy_h2d_batch.restype = ctypes.c_int
        lib.krr_json_find_series.argtypes = [vp, jb, i64, i64, i64, vp, i64, vp, vp]
        lib.krr_json_find_series.restype = ctypes.c_int
        lib.krr_json_parse_segments.argtypes = [vp, jb, vp, vp, i64, ctypes.c_char_p, i32, vp, vp, vp, vp]
        lib.krr_json_parse_segments.restype = ctypes.c_int
        lib.krr_json_parse_segments_split.argtypes = [vp, jb, vp, vp, i64, ctypes.c_char_p, i32, vp, vp, vp, vp, i64,
                                                      vp]
        lib.krr_json_parse_segments_split.restype = ctypes.c_int
        lib.krr_json_gather.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp, vp, vp]
        lib.krr_json_gather.restype = ctypes.c_int
        if lib.krr_abi_version() != 3:
            raise NativeUnavailable("libkrr_amd.so ABI version mismatch")
        _lib = lib
        return lib


class Context:
    """One krr_ctx bound to one HIP device (not shared between threads)."""

    def __init__(self, device: int = 0):
        import torch

        if not torch.cuda.is_available():
            raise NativeUnavailable("no HIP device visible: the KRR hot path runs only on MI355X (gfx950)")
        self._lib = load_library()
        self.device = int(device)
        h = ctypes.c_void_p()
        rc = self._lib.krr_create(self.device, ctypes.byref(h))
        if rc != KRR_OK:
            raise NativeError(rc, f"krr_create(device={device}) failed")
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.krr_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int) -> None:
        if rc != KRR_OK:
            msg = self._lib.krr_last_error(self._h)
            raise NativeError(rc, msg.decode() if msg else "")

    # --- helpers ---------------------------------------------------------
    @staticmethod
    def _stream(stream) -> Optional[int]:
        import torch

        if stream is None:
            stream = torch.cuda.current_stream()
        return ctypes.c_void_p(stream.cuda_stream)

    def _bound(self, params: KrrPercentileParams, *series: KrrSeries, max_n: Optional[int] = None):
        """params with the index table its rule needs for these series (or max_n samples)."""
        if getattr(params, "rule", None) is None or params.mode == KRR_PCT_LINEAR:
            return params
        if max_n is None and series:
            max_n = max(_series_max_len(s) for s in series)
        return bind_index_table(params, max_n, self.device)

    def series(self, values, offsets, max_segment_len: int = 0, gaps_are_nan: bool = False) -> KrrSeries:
        """Describe device tensors as a krr_series.  The struct keeps references to
        both tensors, so their memory cannot be freed and reused while it is alive.
        Both must live on this ctx's device: the kernels read only its HBM."""
        _check_tensor(values, "float64")
        _check_tensor(offsets, "int64")
        for t in (values, offsets):
            if t.is_cuda and t.device.index != self.device:
                raise ValueError(f"tensor on {t.device}, ctx on cuda:{self.device}")
        ser = KrrSeries(values.data_ptr(), offsets.data_ptr(), offsets.numel() - 1, values.numel(),
                        int(max_segment_len), int(bool(gaps_are_nan)), 0)
        ser._keep = (values, offsets)
        return ser

    # --- entry points -----------------------------------------------------
    def segmented_percentile(self, series: KrrSeries, params: KrrPercentileParams, out_value, out_count,
                             out_flags, stream=None) -> None:
        for t, dt in ((out_value, "float64"), (out_count, "int64"), (out_flags, "int32")):
            _check_tensor(t, dt, series.n_segments)
        params = self._bound(params, series)
        self._check(self._lib.krr_segmented_percentile(
            self._h, ctypes.byref(series), ctypes.byref(params), out_value.data_ptr(), out_count.data_ptr(),
            out_flags.data_ptr(), self._stream(stream)))

    def segmented_max(self, series: KrrSeries, out_value, out_count, out_flags, stream=None) -> None:
        for t, dt in ((out_value, "float64"), (out_count, "int64"), (out_flags, "int32")):
            _check_tensor(t, dt, series.n_segments)
        self._check(self._lib.krr_segmented_max(
            self._h, ctypes.byref(series), out_value.data_ptr(), out_count.data_ptr(), out_flags.data_ptr(),
            self._stream(stream)))

    def simple_run(self, cpu: KrrSeries, mem: KrrSeries, params: KrrPercentileParams, out: dict,
                   stream=None, records=None, forward=None) -> None:
        """out: dict with cpu_value/cpu_count/cpu_flags/mem_value/mem_count/mem_flags tensors;
        records (optional): int64 [S, 4] device (or page-locked host) tensor the same launch
        fills with the 32-B result records (krr_simple_run_records); forward (optional):
        (src, dst) tensors of equal byte size the same launch copies src -> dst
        (krr_simple_run_forward; dst may be page-locked host memory)."""
        n = cpu.n_segments
        for k, dt in (("cpu_value", "float64"), ("cpu_count", "int64"), ("cpu_flags", "int32"),
                      ("mem_value", "float64"), ("mem_count", "int64"), ("mem_flags", "int32")):
            _check_tensor(out[k], dt, n)
        if records is not None:
            _check_tensor(records, "int64", 4 * n, host_pinned_ok=True)
        fsrc = fdst = None
        fbytes = 0
        if forward is not None:
            src, dst = forward
            _check_tensor(src, "int64", host_pinned_ok=True)
            _check_tensor(dst, "int64", host_pinned_ok=True)
            fbytes = src.numel() * 8
            if dst.numel() * 8 < fbytes:
                raise ValueError(f"forward destination holds {dst.numel() * 8} bytes, need {fbytes}")
            fsrc, fdst = src.data_ptr(), dst.data_ptr()
        params = self._bound(params, cpu)
        self._check(self._lib.krr_simple_run_forward(
            self._h, ctypes.byref(cpu), ctypes.byref(mem), ctypes.byref(params),
            out["cpu_value"].data_ptr(), out["cpu_count"].data_ptr(), out["cpu_flags"].data_ptr(),
            out["mem_value"].data_ptr(), out["mem_count"].data_ptr(), out["mem_flags"].data_ptr(),
            records.data_ptr() if records is not None else None, fsrc, fdst, fbytes, self._stream(stream)))

    def pack_records(self, out: dict, records, stream=None) -> None:
        """out: the six result tensors; records: int64 [S, 4] device tensor."""
        n = out["cpu_value"].numel()
        _check_tensor(records, "int64", 4 * n)
        self._check(self._lib.krr_pack_records(
            self._h, n, out["cpu_value"].data_ptr(), out["cpu_count"].data_ptr(), out["cpu_flags"].data_ptr(),
            out["mem_value"].data_ptr(), out["mem_count"].data_ptr(), out["mem_flags"].data_ptr(),
            records.data_ptr(), self._stream(stream)))

    def synth_fill(self, values, offsets, seed: int, kind: int, pod_len: int, gaps: bool, stream=None,
                   seg_base: int = 0) -> None:
        """Synthetic series; segment s is global segment seg_base + s of the fleet."""
        _check_tensor(values, "float64")
        _check_tensor(offsets, "int64")
        self._check(self._lib.krr_synth_fill_global(
            self._h, values.data_ptr(), offsets.data_ptr(), offsets.numel() - 1, int(seed) & (2**64 - 1),
            int(kind), int(pod_len), int(bool(gaps)), int(seg_base), 0, 0, self._stream(stream)))

    def wselect_fallbacks(self) -> int:
        """Segments whose one-pass window select missed (cumulative; synchronises)."""
        v = ctypes.c_int64()
        self._check(self._lib.krr_get_stats(self._h, ctypes.byref(v)))
        return int(v.value)

    # --- multi-GPU result collection (RCCL, include/krr_amd.h krr_gather_results) ---
    def comm_unique_id(self) -> bytes:
        buf = ctypes.create_string_buffer(NCCL_UNIQUE_ID_BYTES)
        self._check(self._lib.krr_comm_unique_id(self._h, buf))
        return buf.raw

    def comm_init(self, nranks: int, unique_id: bytes, rank: int, timeout_s: float = 0.0) -> int:
        """ncclCommInitRank on this ctx's device; returns the ncclComm_t as an int.
        timeout_s > 0: bounded (krr_comm_init_timeout; NativeError KRR_E_TIMEOUT when a peer
        never arrives)."""
        if len(unique_id) != NCCL_UNIQUE_ID_BYTES:
            raise ValueError("unique_id must be 128 bytes")
        comm = ctypes.c_void_p()
        if timeout_s > 0:
            self._check(self._lib.krr_comm_init_timeout(self._h, int(nranks), ctypes.c_char_p(unique_id), int(rank),
                                                        float(timeout_s), ctypes.byref(comm)))
        else:
            self._check(self._lib.krr_comm_init(self._h, int(nranks), ctypes.c_char_p(unique_id), int(rank),
                                                ctypes.byref(comm)))
        return int(comm.value or 0)

    def comm_destroy(self, comm: int) -> None:
        self._check(self._lib.krr_comm_destroy(self._h, ctypes.c_void_p(comm)))

    def comm_info(self, comm: int) -> tuple[int, int]:
        """(ranks in the RCCL communicator, this process's rank in it)."""
        n, r = ctypes.c_int(0), ctypes.c_int(0)
        self._check(self._lib.krr_comm_info(self._h, ctypes.c_void_p(comm), ctypes.byref(n), ctypes.byref(r)))
        return int(n.value), int(r.value)

    def gather_results(self, comm: int, root: int, records, counts=None, out=None, stream=None) -> None:
        """records: int64 [n_local, 4] device tensor; on the root, out: int64 [sum(counts), 4]
        device tensor and counts: every rank's n_local (None: all equal n_local)."""
        _check_tensor(records, "int64")
        n_local = records.numel() // 4
        carr = None
        if counts is not None:
            carr = (ctypes.c_int64 * len(counts))(*[int(c) for c in counts])
        if out is not None:
            _check_tensor(out, "int64", 4 * (sum(counts) if counts is not None else n_local))
        self._check(self._lib.krr_gather_results(
            self._h, ctypes.c_void_p(comm), int(root), records.data_ptr(), n_local,
            ctypes.cast(carr, ctypes.c_void_p) if carr is not None else None,
            out.data_ptr() if out is not None else None, self._stream(stream)))


    # --- sketch mode / time-sharded helpers (config 5) ---------------------
    def sketch_width(self, sp: KrrSketchParams) -> int:
        w = int(self._lib.krr_sketch_width(ctypes.byref(sp)))
        if w < 0:
            raise ValueError("invalid sketch parameters")
        return w

    def sketch_build(self, series: KrrSeries, sp: KrrSketchParams, counts, vmin, vmax, flags, stream=None) -> None:
        """counts: int32 [S, width] (uint32 bit patterns); vmin/vmax float64 [S]; flags int32 [S]."""
        S = series.n_segments
        _check_tensor(counts, "int32", S * self.sketch_width(sp))
        _check_tensor(vmin, "float64", S)
        _check_tensor(vmax, "float64", S)
        _check_tensor(flags, "int32", S)
        self._check(self._lib.krr_sketch_build(
            self._h, ctypes.byref(series), ctypes.byref(sp), counts.data_ptr(), vmin.data_ptr(), vmax.data_ptr(),
            flags.data_ptr(), self._stream(stream)))

    def sketch_query(self, counts, vmin, vmax, sp: KrrSketchParams, params: KrrPercentileParams, out_value,
                     out_count, out_flags, stream=None, max_n: Optional[int] = None) -> None:
        """max_n: the largest merged present count (needed when the percentile's index rule
        takes a table, krr_amd.core.index_rule)."""
        S = vmin.numel()
        params = self._bound(params, max_n=max_n)
        _check_tensor(counts, "int32", S * self.sketch_width(sp))
        for t, dt in ((vmax, "float64"), (out_value, "float64"), (out_count, "int64"), (out_flags, "int32")):
            _check_tensor(t, dt, S)
        self._check(self._lib.krr_sketch_query(
            self._h, S, counts.data_ptr(), vmin.data_ptr(), vmax.data_ptr(), ctypes.byref(sp), ctypes.byref(params),
            out_value.data_ptr(), out_count.data_ptr(), out_flags.data_ptr(), self._stream(stream)))

    def sketch_locate(self, counts, sp: KrrSketchParams, params: KrrPercentileParams, out_loc,
                      stream=None, max_n: Optional[int] = None) -> None:
        """out_loc: int64 [S, LOC_WORDS] (krr_sketch_loc per series); max_n as sketch_query."""
        S = out_loc.shape[0]
        params = self._bound(params, max_n=max_n)
        _check_tensor(counts, "int32", S * self.sketch_width(sp))
        _check_tensor(out_loc, "int64", S * LOC_WORDS)
        self._check(self._lib.krr_sketch_locate(self._h, S, counts.data_ptr(), ctypes.byref(sp), ctypes.byref(params),
                                                out_loc.data_ptr(), self._stream(stream)))

    def sketch_range_count(self, counts, sp: KrrSketchParams, loc, out, stream=None) -> None:
        S = loc.shape[0]
        _check_tensor(counts, "int32", S * self.sketch_width(sp))
        _check_tensor(loc, "int64", S * LOC_WORDS)
        _check_tensor(out, "int64", S)
        self._check(self._lib.krr_sketch_range_count(self._h, S, counts.data_ptr(), ctypes.byref(sp),
                                                     loc.data_ptr(), out.data_ptr(), self._stream(stream)))

    def sketch_collect(self, series: KrrSeries, sp: KrrSketchParams, loc, out_offsets, out_values, out_count=None,
                       stream=None) -> None:
        S = series.n_segments
        _check_tensor(loc, "int64", S * LOC_WORDS)
        _check_tensor(out_offsets, "int64", S + 1)
        _check_tensor(out_values, "float64")
        if out_count is not None:
            _check_tensor(out_count, "int64", S)
        self._check(self._lib.krr_sketch_collect(
            self._h, ctypes.byref(series), ctypes.byref(sp), loc.data_ptr(), out_offsets.data_ptr(),
            out_values.data_ptr(), out_count.data_ptr() if out_count is not None else None, self._stream(stream)))

    def sketch_refine(self, collected: KrrSeries, loc, out_value, out_count, out_flags, stream=None) -> None:
        S = collected.n_segments
        _check_tensor(loc, "int64", S * LOC_WORDS)
        for t, dt in ((out_value, "float64"), (out_count, "int64"), (out_flags, "int32")):
            _check_tensor(t, dt, S)
        self._check(self._lib.krr_sketch_refine(self._h, ctypes.byref(collected), loc.data_ptr(),
                                                out_value.data_ptr(), out_count.data_ptr(), out_flags.data_ptr(),
                                                self._stream(stream)))

    def kll_row_words(self, kp: KrrKllParams) -> int:
        w = int(self._lib.krr_kll_row_words(ctypes.byref(kp)))
        if w < 0:
            raise ValueError("invalid kll parameters (budget in [256, 4096], a multiple of 64; tail in [0, 4096])")
        return w

    def kll_build(self, series: KrrSeries, kp: KrrKllParams, rows, seg_base: int = 0, stream=None) -> None:
        """rows: int64 [S, kll_row_words] (uint64 words)."""
        S = series.n_segments
        _check_tensor(rows, "int64", S * self.kll_row_words(kp))
        self._check(self._lib.krr_kll_build(self._h, ctypes.byref(series), ctypes.byref(kp), int(seg_base),
                                            rows.data_ptr(), self._stream(stream)))

    def kll_tail(self, series: KrrSeries, kp: KrrKllParams, rows, stream=None) -> None:
        """The tail pass on rows built with KRR_KLL_BODY_ONLY (krr_kll_tail)."""
        S = series.n_segments
        _check_tensor(rows, "int64", S * self.kll_row_words(kp))
        self._check(self._lib.krr_kll_tail(self._h, ctypes.byref(series), ctypes.byref(kp), rows.data_ptr(),
                                           self._stream(stream)))

    def kll_line_words(self, max_segment_len: int) -> int:
        """uint32 words per series of the line maxima (krr_kll_line_words)."""
        return int(self._lib.krr_kll_line_words(int(max_segment_len)))

    def kll_build_lines(self, series: KrrSeries, kp: KrrKllParams, rows, lines, line_stride: int, seg_base: int = 0,
                        stream=None) -> None:
        """The body-only build that also writes the line maxima: lines int32 [S * line_stride]."""
        S = series.n_segments
        _check_tensor(rows, "int64", S * self.kll_row_words(kp))
        _check_tensor(lines, "int32", S * int(line_stride))
        self._check(self._lib.krr_kll_build_lines(self._h, ctypes.byref(series), ctypes.byref(kp), int(seg_base),
                                                  rows.data_ptr(), lines.data_ptr(), int(line_stride),
                                                  self._stream(stream)))

    def kll_tail_lines(self, series: KrrSeries, kp: KrrKllParams, rows, lines, line_stride: int,
                       lines_read=None, stream=None) -> None:
        """The sparse tail pass (krr_kll_tail_lines) over rows and line maxima from kll_build_lines;
        lines_read (optional int32 [S]): the 128-B lines it read per series."""
        S = series.n_segments
        _check_tensor(rows, "int64", S * self.kll_row_words(kp))
        _check_tensor(lines, "int32", S * int(line_stride))
        if lines_read is not None:
            _check_tensor(lines_read, "int32", S)
        self._check(self._lib.krr_kll_tail_lines(self._h, ctypes.byref(series), ctypes.byref(kp), rows.data_ptr(),
                                                 lines.data_ptr(), int(line_stride),
                                                 None if lines_read is None else lines_read.data_ptr(),
                                                 self._stream(stream)))

    def kll_merge(self, rows, rows_per_series: int, kp: KrrKllParams, out_rows, series_base: int = 0,
                  stream=None) -> None:
        """rows: int64 [S * rows_per_series, kll_row_words] series-major -> out_rows [S, kll_row_words]."""
        rw = self.kll_row_words(kp)
        S = out_rows.numel() // rw
        _check_tensor(rows, "int64", S * int(rows_per_series) * rw)
        _check_tensor(out_rows, "int64", S * rw)
        self._check(self._lib.krr_kll_merge(self._h, S, int(rows_per_series), rows.data_ptr(), ctypes.byref(kp),
                                            int(series_base), out_rows.data_ptr(), self._stream(stream)))

    def kll_query(self, rows, rows_per_series: int, kp: KrrKllParams, params: KrrPercentileParams, out_value,
                  out_count, out_flags, series_base: int = 0, stream=None, max_n: Optional[int] = None) -> None:
        """rows: int64 [S * rows_per_series, kll_row_words], series-major; max_n as sketch_query."""
        S = out_value.numel()
        params = self._bound(params, max_n=max_n)
        _check_tensor(rows, "int64", S * int(rows_per_series) * self.kll_row_words(kp))
        for t, dt in ((out_value, "float64"), (out_count, "int64"), (out_flags, "int32")):
            _check_tensor(t, dt, S)
        self._check(self._lib.krr_kll_query(self._h, S, int(rows_per_series), rows.data_ptr(), ctypes.byref(kp),
                                            int(series_base), ctypes.byref(params), out_value.data_ptr(),
                                            out_count.data_ptr(), out_flags.data_ptr(), self._stream(stream)))

    def rank_of(self, series: KrrSeries, values, out_lt, out_le, stream=None) -> None:
        S = series.n_segments
        _check_tensor(values, "float64", S)
        _check_tensor(out_lt, "int64", S)
        _check_tensor(out_le, "int64", S)
        self._check(self._lib.krr_rank_of(self._h, ctypes.byref(series), values.data_ptr(), out_lt.data_ptr(),
                                          out_le.data_ptr(), self._stream(stream)))

    def select_present(self, series: KrrSeries, k, out, stream=None) -> None:
        S = series.n_segments
        _check_tensor(k, "int64", S)
        _check_tensor(out, "float64", S)
        self._check(self._lib.krr_select_present(self._h, ctypes.byref(series), k.data_ptr(), out.data_ptr(),
                                                 self._stream(stream)))

    def locate(self, series: KrrSeries, values, rank, out_lt, out_eq, out_pos, stream=None) -> None:
        """Per segment: #samples < values[s], #== values[s], and the slot offset of the
        (rank[s] - lt)-th sample equal to values[s] (rank -1: the first one; < -1: skipped)."""
        S = series.n_segments
        _check_tensor(values, "float64", S)
        for t in (rank, out_lt, out_eq, out_pos):
            _check_tensor(t, "int64", S)
        self._check(self._lib.krr_locate(self._h, ctypes.byref(series), values.data_ptr(), rank.data_ptr(),
                                         out_lt.data_ptr(), out_eq.data_ptr(), out_pos.data_ptr(),
                                         self._stream(stream)))

    # --- time-sharded exact percentiles in one pass (window export / merge) ---------
    def window_export(self, series: KrrSeries, params: KrrPercentileParams, ext_slots: int, key_cap: int, hdr,
                      keys, stream=None) -> None:
        """hdr: int64 [>= S, HDR_WORDS]; keys: int64 [>= S, key_cap] (uint64 key bit patterns)."""
        S = series.n_segments
        _check_tensor(hdr, "int64", S * HDR_WORDS)
        _check_tensor(keys, "int64", S * int(key_cap))
        self._check(self._lib.krr_window_export(self._h, ctypes.byref(series), ctypes.byref(params), int(ext_slots),
                                                int(key_cap), hdr.data_ptr(), keys.data_ptr(), self._stream(stream)))

    def window_merge(self, n_series: int, n_slices: int, slice_stride: int, hdr, keys, key_cap: int,
                     params: KrrPercentileParams, out_value, out_count, out_flags, miss_count=None,
                     stream=None, max_n: Optional[int] = None) -> None:
        """Slice j of series i: hdr[j * slice_stride + i], keys row j * slice_stride + i.
        miss_count: optional int32 [1] device tensor (zeroed, then counts the misses); max_n as
        sketch_query."""
        params = self._bound(params, max_n=max_n)
        _check_tensor(hdr, "int64", ((n_slices - 1) * slice_stride + n_series) * HDR_WORDS if n_series else 0)
        _check_tensor(keys, "int64", ((n_slices - 1) * slice_stride + n_series) * int(key_cap) if n_series else 0)
        for t, dt in ((out_value, "float64"), (out_count, "int64"), (out_flags, "int32")):
            _check_tensor(t, dt, n_series)
        if miss_count is not None:
            _check_tensor(miss_count, "int32", 1)
        self._check(self._lib.krr_window_merge(
            self._h, int(n_series), int(n_slices), int(slice_stride), hdr.data_ptr(), keys.data_ptr(), int(key_cap),
            ctypes.byref(params), out_value.data_ptr(), out_count.data_ptr(), out_flags.data_ptr(),
            miss_count.data_ptr() if miss_count is not None else None, self._stream(stream)))

    def synth_fill_window(self, values, offsets, seed: int, kind: int, pod_len: int, gaps: bool, t0: int,
                          total_len: int, stream=None, seg_base: int = 0) -> None:
        """Time window [t0, t0 + len) of series of total_len slots; segment s is global
        segment seg_base + s."""
        _check_tensor(values, "float64")
        _check_tensor(offsets, "int64")
        self._check(self._lib.krr_synth_fill_global(
            self._h, values.data_ptr(), offsets.data_ptr(), offsets.numel() - 1, int(seed) & (2**64 - 1),
            int(kind), int(pod_len), int(bool(gaps)), int(seg_base), int(t0), int(total_len), self._stream(stream)))

    # --- device packer: query_range bodies in HBM -> CSR --------------------------------
    def json_bodies(self, bodies, body_offsets, total_bytes: int) -> KrrJsonBodies:
        """bodies: uint8 device tensor (16-B aligned, >= 128 bytes past the last body);
        body_offsets: int64 device tensor [n_bodies + 1]."""
        _check_tensor(bodies, "uint8", int(total_bytes) + 128)
        _check_tensor(body_offsets, "int64")
        if bodies.data_ptr() % 16:
            raise ValueError("bodies must be 16-byte aligned")
        jb = KrrJsonBodies(bodies.data_ptr(), body_offsets.data_ptr(), body_offsets.numel() - 1, int(total_bytes))
        jb._keep = (bodies, body_offsets)
        return jb

    def json_parse(self, jb: KrrJsonBodies, first: int, n: int, want_timestamps: bool, scratch_values, scratch_ts,
                   counts, status, stream=None) -> None:
        slots = jb.total_bytes // 8 + 1
        _check_tensor(scratch_values, "float64", slots)
        if want_timestamps:
            _check_tensor(scratch_ts, "float64", slots)
        _check_tensor(counts, "int64", jb.n_bodies)
        _check_tensor(status, "int32", jb.n_bodies)
        self._check(self._lib.krr_json_parse(
            self._h, ctypes.byref(jb), int(first), int(n), int(bool(want_timestamps)), scratch_values.data_ptr(),
            scratch_ts.data_ptr() if want_timestamps else None, counts.data_ptr(), status.data_ptr(),
            self._stream(stream)))

    def json_compact(self, jb: KrrJsonBodies, scratch_values, scratch_ts, counts, status, out_pos, values,
                     timestamps=None, stream=None) -> None:
        n = jb.n_bodies
        _check_tensor(counts, "int64", n)
        _check_tensor(status, "int32", n)
        _check_tensor(out_pos, "int64", n)
        _check_tensor(values, "float64")
        if timestamps is not None:
            _check_tensor(timestamps, "float64", values.numel())
            _check_tensor(scratch_ts, "float64")
        self._check(self._lib.krr_json_compact(
            self._h, ctypes.byref(jb), scratch_values.data_ptr(),
            scratch_ts.data_ptr() if timestamps is not None else None, counts.data_ptr(), status.data_ptr(),
            out_pos.data_ptr(), values.data_ptr(), timestamps.data_ptr() if timestamps is not None else None,
            self._stream(stream)))

    def copy_h2d_batch(self, dst, src, nbytes, stream=None) -> None:
        """int64 arrays (numpy) of device destinations, host sources (page-locked) and byte
        counts: one asynchronous copy each, in order, on ``stream`` (krr_copy_h2d_batch)."""
        import numpy as np

        dst, src, nbytes = (np.ascontiguousarray(a, dtype=np.int64) for a in (dst, src, nbytes))
        n = len(nbytes)
        if len(dst) != n or len(src) != n:
            raise ValueError("copy_h2d_batch: dst / src / nbytes differ in length")
        self._check(self._lib.krr_copy_h2d_batch(self._h, n, dst.ctypes.data, src.ctypes.data, nbytes.ctypes.data,
                                                 self._stream(stream)))

    def json_find_series(self, jb: KrrJsonBodies, candidates, n_candidates, begin: int = 0, end: Optional[int] = None,
                         limit: Optional[int] = None, stream=None) -> None:
        """candidates: int64 [cap]; n_candidates: int64 [1] device counter (zeroed by the caller);
        positions [begin, end) with the bytes below ``limit`` in place (default: all)."""
        _check_tensor(candidates, "int64")
        _check_tensor(n_candidates, "int64", 1)
        end = jb.total_bytes if end is None else int(end)
        limit = jb.total_bytes if limit is None else int(limit)
        self._check(self._lib.krr_json_find_series(self._h, ctypes.byref(jb), int(begin), end, limit,
                                                   candidates.data_ptr(), candidates.numel(), n_candidates.data_ptr(),
                                                   self._stream(stream)))

    def json_parse_segments(self, jb: KrrJsonBodies, starts, body_of, label: str, want_timestamps: bool,
                            scratch_values, scratch_ts, segments, stream=None, workspace=None) -> None:
        """``workspace``: an int64 device tensor for the split values parse
        (krr_json_parse_segments_split: 1 + n + 6 per 16-KiB part), or None (one wave per series)."""
        n = starts.numel()
        _check_tensor(starts, "int64", n)
        _check_tensor(body_of, "int64", n)
        _check_tensor(segments, "int64", 7 * n, host_pinned_ok=True)  # pinned: written through the mapping
        _check_tensor(scratch_values, "float64", jb.total_bytes // 8 + 1)
        if want_timestamps:
            _check_tensor(scratch_ts, "float64", jb.total_bytes // 8 + 1)
        args = (self._h, ctypes.byref(jb), starts.data_ptr(), body_of.data_ptr(), n, label.encode(),
                int(bool(want_timestamps)), scratch_values.data_ptr(),
                scratch_ts.data_ptr() if want_timestamps else None, segments.data_ptr())
        if workspace is None:
            self._check(self._lib.krr_json_parse_segments(*args, self._stream(stream)))
            return
        _check_tensor(workspace, "int64", n + 1 + 6)
        self._check(self._lib.krr_json_parse_segments_split(*args, workspace.data_ptr(), workspace.numel(),
                                                            self._stream(stream)))

    def json_gather(self, src, count, dst, scratch_values, scratch_ts, values, timestamps=None, stream=None) -> None:
        n = src.numel()
        for t in (src, count, dst):
            _check_tensor(t, "int64", n)
        _check_tensor(scratch_values, "float64")
        _check_tensor(values, "float64")
        if timestamps is not None:
            _check_tensor(timestamps, "float64", values.numel())
            _check_tensor(scratch_ts, "float64")
        self._check(self._lib.krr_json_gather(
            self._h, n, src.data_ptr(), count.data_ptr(), dst.data_ptr(), scratch_values.data_ptr(),
            scratch_ts.data_ptr() if timestamps is not None else None, values.data_ptr(),
            timestamps.data_ptr() if timestamps is not None else None, self._stream(stream)))


def select_plan(max_segment_len: int, params: KrrPercentileParams) -> KrrSelectPlanInfo:
    """The launch plan krr_segmented_percentile / krr_simple_run choose for SORTED_LOWER /
    LINEAR (host only: no device needed).  Raises NativeError for REF_INDEX."""
    lib = load_library()
    info = KrrSelectPlanInfo()
    rule = getattr(params, "rule", None)
    if rule is not None and not params.k_table and params.mode != KRR_PCT_LINEAR and rule.needs_table(max_segment_len):
        # the plan only needs to know a table is there (its wider margins); it reads no entry
        tab = rule.table(max(int(max_segment_len), 1))
        params = KrrPercentileParams(params.mode, params.reserved, params.p_num, params.p_den, params.q,
                                     tab.ctypes.data, tab.size)
    rc = lib.krr_select_plan(int(max_segment_len), ctypes.byref(params), ctypes.byref(info))
    if rc != KRR_OK:
        raise NativeError(rc, "krr_select_plan")
    return info


def window_key_cap(max_slice_len: int, ext_slots: int, params: KrrPercentileParams) -> int:
    """Keys per exported row (krr_window_key_cap; host only)."""
    lib = load_library()
    k = int(lib.krr_window_key_cap(int(max_slice_len), int(ext_slots), ctypes.byref(params)))
    if k <= 0:
        raise NativeError(KRR_E_INVALID, "krr_window_key_cap: REF_INDEX or invalid arguments")
    return k


def _series_max_len(series: KrrSeries) -> int:
    """The longest segment's slots: max_segment_len, or from the offsets (synchronises)."""
    if series.max_segment_len > 0:
        return int(series.max_segment_len)
    offs = series._keep[1]
    if offs.numel() < 2:
        return 0
    return int((offs[1:] - offs[:-1]).max().item())


def _check_tensor(t, dtype: str, numel: Optional[int] = None, host_pinned_ok: bool = False) -> None:
    """host_pinned_ok: a page-locked host tensor is accepted too (the device writes it
    through the mapping the pinned allocation has in its address space)."""
    import torch

    want = getattr(torch, dtype)
    on_dev = isinstance(t, torch.Tensor) and (t.is_cuda or (host_pinned_ok and t.is_pinned()))
    if not on_dev or t.dtype != want or not t.is_contiguous():
        raise TypeError(f"expected a contiguous {dtype} HIP-device tensor, got "
                        f"{getattr(t, 'dtype', type(t))} on {getattr(t, 'device', '?')}")
    if numel is not None and t.numel() < numel:
        raise ValueError(f"output tensor has {t.numel()} elements, need {numel}")
