"""Torch-tensor conveniences over the C ABI: synthetic inputs, order check, sort plans that can
be re-used with varying counts, and the single-pass stable partition used by the multi-GPU
bucket exchange.  All compute is in librsort.so."""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import check


def _stream(t, stream=None):
    import torch
    if stream is not None:
        return stream if isinstance(stream, int) else stream.cuda_stream
    return torch.cuda.current_stream(t.device).cuda_stream


def fill_random_u32(t, seed: int, start: int = 0, stream=None) -> None:
    """t[i] = rs generator(seed, start + i) (same as oracle.gen_u32)."""
    check(_lib.load().rs_fill_random_u32(t.data_ptr(), t.numel(), seed, start, _stream(t, stream)),
          "rs_fill_random_u32")


def fill_iota_u32(t, first: int = 0, stream=None) -> None:
    check(_lib.load().rs_fill_iota_u32(t.data_ptr(), t.numel(), first, _stream(t, stream)),
          "rs_fill_iota_u32")


def is_sorted(t, n: int | None = None, bit_count: int = 32, stream=None) -> bool:
    import torch
    flag = torch.empty(1, dtype=torch.int32, device=t.device)
    n = t.numel() if n is None else n
    check(_lib.load().rs_is_sorted(t.data_ptr(), n, bit_count, flag.data_ptr(), _stream(t, stream)),
          "rs_is_sorted")
    return bool(flag.item())


def histogram(t, n: int, shift: int, bits: int, out, stream=None) -> None:
    """out[d] = number of t[:n] whose digit (key >> shift) & (2^bits - 1) is d (out: 2^bits
    int32 words on t's device, overwritten)."""
    check(_lib.load().rs_histogram(t.data_ptr(), n, shift, bits, out.data_ptr(),
                                   _stream(t, stream)), "rs_histogram")


class SortPlan:
    """A sort plan with a capacity; sorts any n <= capacity (multi-GPU receive buffers)."""

    def __init__(self, device: int, capacity: int, has_values: bool, bit_count: int = 32,
                 radix_bits: int = 0, check_order: bool = False, usage: int = 0):
        """usage: _lib.RS_USAGE_SORT (every entry point) or RS_USAGE_PARTITION (hist16() and the
        partition passes only: the multi-GPU sender, no ping-pong copy)."""
        flags = (_lib.RS_FLAG_HAS_VALUES if has_values else 0) | \
                (_lib.RS_FLAG_CHECK_ORDER if check_order else 0) | _lib.RS_FLAG_LOCAL_SHUFFLE
        desc = _lib.PlanDesc(device, capacity, bit_count, 16, 16, flags, radix_bits, usage)
        p = ctypes.c_void_p()
        check(_lib.load().rs_plan_create(ctypes.byref(desc), ctypes.byref(p)), "SortPlan")
        self._plan = p
        _lib.apply_debug(p)
        self.capacity = capacity
        self.has_values = has_values

    def sort(self, keys, values=None, n: int | None = None, stream=None) -> None:
        n = keys.numel() if n is None else n
        check(_lib.load().rs_plan_sort_n(self._plan, keys.data_ptr(),
                                         None if values is None else values.data_ptr(), n,
                                         _stream(keys, stream)), "rs_plan_sort_n")

    def sort_copy(self, in_keys, in_values, out_keys, out_values=None, n: int | None = None,
                  stream=None) -> None:
        """Out-of-place stable sort in -> out (the input is only read)."""
        n = in_keys.numel() if n is None else n
        check(_lib.load().rs_plan_sort_copy(
            self._plan, in_keys.data_ptr(), None if in_values is None else in_values.data_ptr(),
            out_keys.data_ptr(), None if out_values is None else out_values.data_ptr(), n,
            _stream(in_keys, stream)), "rs_plan_sort_copy")

    def check(self) -> None:
        """Wait for the plan's last sort; raise on a device-side failure since the last check
        (rs_plan_check)."""
        check(_lib.load().rs_plan_check(self._plan), "rs_plan_check")

    def set_profiling(self, enable: bool) -> None:
        check(_lib.load().rs_plan_set_profiling(self._plan, 1 if enable else 0), "profiling")

    def last_path(self) -> str:
        """Which path the plan's last sort took (rs_plan_last_path; waits for it)."""
        v = ctypes.c_uint32()
        check(_lib.load().rs_plan_last_path(self._plan, ctypes.byref(v)), "last_path")
        return _lib.PATH_NAMES[v.value]

    def last_split(self) -> int:
        """The bucket split depth of the plan's last sort: 0, 2 or 3 (rs_plan_last_split)."""
        v = ctypes.c_uint32()
        check(_lib.load().rs_plan_last_split(self._plan, ctypes.byref(v)), "last_split")
        return int(v.value)

    def kernel_times(self) -> dict:
        """Accumulated per-kind kernel times of the plan's launches (after set_profiling)."""
        ms = (ctypes.c_double * _lib.RS_KERNEL_KINDS)()
        n = (ctypes.c_uint64 * _lib.RS_KERNEL_KINDS)()
        check(_lib.load().rs_plan_kernel_times(self._plan, ms, n), "kernel_times")
        return {name: {"ms": ms[i], "launches": n[i]} for i, name in enumerate(_lib.KERNEL_NAMES)}

    def partition(self, in_keys, in_values, out_keys, out_values, n: int, shift: int, bits: int,
                  hist=None, stream=None) -> None:
        """Stable one-digit scatter in -> out; hist (device u32[2^bits]) gets digit totals."""
        check(_lib.load().rs_plan_partition(
            self._plan, in_keys.data_ptr(), None if in_values is None else in_values.data_ptr(),
            out_keys.data_ptr(), None if out_values is None else out_values.data_ptr(), n, shift,
            bits, None if hist is None else hist.data_ptr(), _stream(in_keys, stream)),
            "rs_plan_partition")

    def partition_totals(self, in_keys, in_values, out_keys, out_values, n: int, shift: int,
                         bits: int, totals, stream=None) -> None:
        """partition() given the digit totals of the input (device u32[2^bits], e.g. from
        histogram()): one key read fewer where the one-sweep scatter applies."""
        check(_lib.load().rs_plan_partition_totals(
            self._plan, in_keys.data_ptr(), None if in_values is None else in_values.data_ptr(),
            out_keys.data_ptr(), None if out_values is None else out_values.data_ptr(), n, shift,
            bits, totals.data_ptr(), _stream(in_keys, stream)), "rs_plan_partition_totals")

    def partition_records(self, in_keys, in_values, out_records, n: int, shift: int, bits: int,
                          totals=None, stream=None) -> None:
        """Stable one-digit partition of separate arrays into (key, value) records
        (out_records: int64 tensor, record i = key | value << 32)."""
        check(_lib.load().rs_plan_partition_records(
            self._plan, in_keys.data_ptr(), in_values.data_ptr(), out_records.data_ptr(), n, shift,
            bits, None if totals is None else totals.data_ptr(), _stream(in_keys, stream)),
            "rs_plan_partition_records")

    def sort_records(self, records, keys_out, values_out, n: int | None = None,
                     stream=None, key_range=None) -> None:
        """Stable sort of n (key, value) records into separate key / value arrays.  key_range:
        (lo, hi) with every key in [lo, hi] (rs_plan_sort_records_range: a hint, checked on the
        device)."""
        n = records.numel() if n is None else n
        L = _lib.load()
        if key_range is None:
            check(L.rs_plan_sort_records(self._plan, records.data_ptr(), keys_out.data_ptr(),
                                         values_out.data_ptr(), n, _stream(records, stream)),
                  "rs_plan_sort_records")
        else:
            lo, hi = (int(x) for x in key_range)
            check(L.rs_plan_sort_records_range(self._plan, records.data_ptr(), keys_out.data_ptr(),
                                               values_out.data_ptr(), n, lo, hi,
                                               _stream(records, stream)),
                  "rs_plan_sort_records_range")

    def hist16(self, keys, n: int, out, stream=None) -> None:
        """out[0:65536] = counts of keys[:n] per 16-bit bucket key >> 16, out[65536:65792] = the
        top-byte totals (out: RS_HIST16_WORDS int32 words on the keys' device)."""
        check(_lib.load().rs_plan_hist16(self._plan, keys.data_ptr(), n, out.data_ptr(),
                                         _stream(keys, stream)), "rs_plan_hist16")

    def sort_region(self, records, keys_out, values_out, n: int, hist16, top_lo: int, top_hi: int,
                    stream=None) -> None:
        """Stable sort of n (key, value) records grouped by top byte in [top_lo, top_hi) (a
        multi-GPU receiver's region) into key / value arrays; hist16 = the region's 16-bit bucket
        counts (65536 int32, zero outside its top bytes)."""
        check(_lib.load().rs_plan_sort_region(self._plan, records.data_ptr(), keys_out.data_ptr(),
                                              values_out.data_ptr(), n, hist16.data_ptr(), top_lo,
                                              top_hi, _stream(records, stream)), "rs_plan_sort_region")

    def destroy(self) -> None:
        if getattr(self, "_plan", None):
            _lib.load().rs_plan_destroy(self._plan)
            self._plan = None

    def __del__(self):  # pragma: no cover
        try:
            self.destroy()
        except Exception:
            pass
