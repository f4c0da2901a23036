"""ctypes binding of librsort.so (include/rsort.h).

The library is built in-tree (``webgpu-radix-sort_amd/lib/librsort.so``) by
``__graft_entry__.build()`` or ``make -C webgpu-radix-sort_amd/csrc``.  There is no fallback:
if the HIP library is missing, importing the sort raises.
"""
from __future__ import annotations

import ctypes
import os
import re

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RSORT_LIB", os.path.join(PKG_ROOT, "lib", "librsort.so"))
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "rsort.h")

RS_OK = 0
RS_ERR_INVALID_ARG = 1
RS_ERR_NOT_POW2 = 2
RS_ERR_BIT_COUNT = 3
RS_ERR_HIP = 4
RS_ERR_OUT_OF_MEMORY = 5
RS_ERR_CAPACITY = 6
RS_ERR_DEVICE = 7

RS_FLAG_HAS_VALUES = 0x1
RS_FLAG_CHECK_ORDER = 0x2
RS_FLAG_LOCAL_SHUFFLE = 0x4
RS_FLAG_AVOID_BANK_CONFLICTS = 0x8
RS_FLAG_INTERLEAVED = 0x10

(RS_KERNEL_HISTOGRAM, RS_KERNEL_SCAN, RS_KERNEL_SCATTER, RS_KERNEL_CHECK, RS_KERNEL_BUCKET,
 RS_KERNEL_FALLBACK, RS_KERNEL_SPLIT, RS_KERNEL_PRESORTED) = range(8)
RS_KERNEL_KINDS = 8
KERNEL_NAMES = ("histogram", "scan", "scatter", "check", "bucket", "fallback", "split", "presorted")
# rs_plan_last_path
PATH_NAMES = ("none", "lsd", "hybrid", "hybrid_fallback", "in_order", "presorted")


class RadixSortError(RuntimeError):
    """A failed librsort call (status code + the library's last-error message)."""

    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


class PlanDesc(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("count", ctypes.c_uint64),
                ("bit_count", ctypes.c_uint32), ("workgroup_x", ctypes.c_uint32),
                ("workgroup_y", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("radix_bits", ctypes.c_uint32), ("usage", ctypes.c_uint32)]


class PlanDebug(ctypes.Structure):
    """rs_plan_debug (test / diagnostics only): force a plan onto one of its paths; -1 = keep."""
    _fields_ = [("rank", ctypes.c_int32), ("tile", ctypes.c_int32), ("onesweep", ctypes.c_int32),
                ("msd", ctypes.c_int32), ("keys_cfg", ctypes.c_int32), ("msd_keys_cfg", ctypes.c_int32),
                ("kbucket_wave", ctypes.c_int32), ("selftest_fail", ctypes.c_int32),
                ("split", ctypes.c_int32), ("presorted", ctypes.c_int32),
                ("xcd", ctypes.c_int32), ("high_half", ctypes.c_int32)]


# Path overrides applied to every plan the Python wrappers create (tests select kernels with
# plan_debug(); the library itself reads no environment variables).  Values: the rs_plan_debug
# field choices, with names for the common ones ("ballot" / "atomic", "small" / "large").
_DEBUG: dict = {}
_DEBUG_NAMES = {"rank": {"atomic": 0, "lds_atomic": 0, "ballot": 1},
                "tile": {"large": 0, "small": 1}}


class plan_debug:
    """Context manager: ``with plan_debug(rank="ballot", tile="small"): ...`` - every plan created
    inside it gets rs_plan_set_debug with these fields."""

    def __init__(self, **fields):
        for k in fields:
            if k not in dict(PlanDebug._fields_):
                raise ValueError(f"unknown rs_plan_debug field {k!r}")
        self.fields = fields
        self.saved = None

    def __enter__(self):
        self.saved = dict(_DEBUG)
        _DEBUG.update(self.fields)
        return self

    def __exit__(self, *exc):
        _DEBUG.clear()
        _DEBUG.update(self.saved)
        return False


def apply_debug(plan) -> None:
    """rs_plan_set_debug(plan, the active plan_debug overrides) - a no-op when none are active."""
    if not _DEBUG:
        return
    d = PlanDebug(*([-1] * len(PlanDebug._fields_)))
    for k, v in _DEBUG.items():
        if isinstance(v, str):
            v = _DEBUG_NAMES[k][v]
        setattr(d, k, int(v))
    check(load().rs_plan_set_debug(plan, ctypes.byref(d)), "rs_plan_set_debug")


RS_USAGE_SORT = 0
RS_USAGE_PARTITION = 1
RS_HIST16_WORDS = 65792


class PlanInfo(ctypes.Structure):
    _fields_ = [("passes", ctypes.c_uint32), ("digit_bits", ctypes.c_uint32 * 16),
                ("tile_keys", ctypes.c_uint32), ("grid_blocks", ctypes.c_uint32),
                ("workspace_bytes", ctypes.c_uint64), ("rank_mode", ctypes.c_uint32),
                ("lane_order_selftest", ctypes.c_int32)]


class GroupDesc(ctypes.Structure):
    _fields_ = [("capacity", ctypes.c_uint64), ("flags", ctypes.c_uint32),
                ("transport", ctypes.c_uint32), ("top_bits", ctypes.c_uint32),
                ("rounds", ctypes.c_uint32)]


class GroupTimes(ctypes.Structure):
    _fields_ = [("rounds", ctypes.c_uint32), ("hist16_ms", ctypes.c_float),
                ("partition_ms", ctypes.c_float), ("round_done_ms", ctypes.c_float * 16),
                ("region_sorted_ms", ctypes.c_float * 16), ("done_ms", ctypes.c_float),
                ("bytes_sent", ctypes.c_uint64), ("bytes_recv", ctypes.c_uint64)]


RS_TRANSPORT_RCCL = 0
RS_TRANSPORT_COPY = 1

_lib = None

_VP = ctypes.c_void_p
_SIGS = {
    "rs_last_error": (ctypes.c_char_p, []),
    "rs_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "rs_version": (ctypes.c_uint32, []),
    "rs_plan_create": (ctypes.c_int, [ctypes.POINTER(PlanDesc), ctypes.POINTER(_VP)]),
    "rs_plan_sort": (ctypes.c_int, [_VP, _VP, _VP, _VP]),
    "rs_plan_sort_n": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint64, _VP]),
    "rs_plan_sort_copy": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, _VP]),
    "rs_plan_partition": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, ctypes.c_uint64,
                                         ctypes.c_uint32, ctypes.c_uint32, _VP, _VP]),
    "rs_plan_partition_totals": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, ctypes.c_uint64,
                                                ctypes.c_uint32, ctypes.c_uint32, _VP, _VP]),
    "rs_plan_partition_records": (ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_uint64,
                                                 ctypes.c_uint32, ctypes.c_uint32, _VP, _VP]),
    "rs_plan_sort_records": (ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_uint64, _VP]),
    "rs_plan_sort_records_range": (ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32,
                                                  ctypes.c_uint32, _VP]),
    "rs_plan_hist16": (ctypes.c_int, [_VP, _VP, ctypes.c_uint64, _VP, _VP]),
    "rs_plan_sort_region": (ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_uint64, _VP, ctypes.c_uint32,
                                           ctypes.c_uint32, _VP]),
    "rs_plan_info_get": (ctypes.c_int, [_VP, ctypes.POINTER(PlanInfo)]),
    "rs_plan_set_profiling": (ctypes.c_int, [_VP, ctypes.c_int]),
    "rs_plan_set_profiling_kinds": (ctypes.c_int, [_VP, ctypes.c_uint32]),
    "rs_plan_last_path": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint32)]),
    "rs_plan_presorted_counts": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "rs_plan_last_split": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint32)]),
    "rs_plan_kernel_times": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_uint64)]),
    "rs_plan_reset_kernel_times": (ctypes.c_int, [_VP]),
    "rs_plan_device_errors": (ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_uint32)]),
    "rs_plan_check": (ctypes.c_int, [_VP]),
    "rs_plan_set_wait_limit": (ctypes.c_int, [_VP, ctypes.c_uint32]),
    "rs_plan_set_debug": (ctypes.c_int, [_VP, ctypes.POINTER(PlanDebug)]),
    "rs_plan_destroy": (None, [_VP]),
    "rs_scan_plan_create": (ctypes.c_int, [ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.POINTER(_VP)]),
    "rs_scan_plan_run": (ctypes.c_int, [_VP, _VP, _VP]),
    "rs_scan_plan_run_indirect": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint64, _VP]),
    "rs_scan_plan_dispatch_chain": (ctypes.c_uint32, [_VP, ctypes.POINTER(ctypes.c_uint32),
                                                      ctypes.c_uint32]),
    "rs_scan_plan_check": (ctypes.c_int, [_VP]),
    "rs_scan_plan_set_wait_limit": (ctypes.c_int, [_VP, ctypes.c_uint32]),
    "rs_scan_plan_destroy": (None, [_VP]),
    "rs_group_create": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                       ctypes.POINTER(GroupDesc), ctypes.POINTER(_VP)]),
    "rs_group_sort": (ctypes.c_int, [_VP, ctypes.POINTER(_VP), ctypes.POINTER(_VP),
                                     ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_VP)]),
    "rs_group_result": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.POINTER(_VP),
                                       ctypes.POINTER(_VP), ctypes.POINTER(ctypes.c_uint64)]),
    "rs_group_synchronize": (ctypes.c_int, [_VP]),
    "rs_group_set_profiling": (ctypes.c_int, [_VP, ctypes.c_int]),
    "rs_group_times_get": (ctypes.c_int, [_VP, ctypes.c_int32, ctypes.POINTER(GroupTimes)]),
    "rs_group_destroy": (None, [_VP]),
    "rs_group_plan": (ctypes.c_int, [ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.POINTER(ctypes.c_uint32),
                                     ctypes.POINTER(ctypes.c_uint32)]),
    "rs_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int32)]),
    "rs_malloc": (ctypes.c_int, [ctypes.c_int32, ctypes.c_uint64, ctypes.POINTER(_VP)]),
    "rs_free": (ctypes.c_int, [_VP]),
    "rs_memcpy_h2d": (ctypes.c_int, [_VP, _VP, ctypes.c_uint64, _VP]),
    "rs_memcpy_d2h": (ctypes.c_int, [_VP, _VP, ctypes.c_uint64, _VP]),
    "rs_memcpy_d2d": (ctypes.c_int, [_VP, _VP, ctypes.c_uint64, _VP]),
    "rs_stream_create": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(_VP)]),
    "rs_stream_destroy": (ctypes.c_int, [_VP]),
    "rs_stream_synchronize": (ctypes.c_int, [_VP]),
    "rs_event_create": (ctypes.c_int, [ctypes.POINTER(_VP)]),
    "rs_event_destroy": (ctypes.c_int, [_VP]),
    "rs_event_record": (ctypes.c_int, [_VP, _VP]),
    "rs_event_elapsed_ms": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(ctypes.c_float)]),
    "rs_fill_random_u32": (ctypes.c_int, [_VP, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_uint64, _VP]),
    "rs_fill_iota_u32": (ctypes.c_int, [_VP, ctypes.c_uint64, ctypes.c_uint32, _VP]),
    "rs_histogram": (ctypes.c_int, [_VP, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                    _VP, _VP]),
    "rs_is_sorted": (ctypes.c_int, [_VP, ctypes.c_uint64, ctypes.c_uint32, _VP, _VP]),
}


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Names of the functions declared in include/rsort.h."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rs_[a-z0-9_]+)\s*\(", src)))


def load():
    """Load librsort.so; raises (never falls back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"librsort.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status: int, what: str = "") -> None:
    if status != RS_OK:
        L = load()
        msg = L.rs_last_error().decode(errors="replace")
        raise RadixSortError(status, f"{what}: {msg}" if what else msg)
