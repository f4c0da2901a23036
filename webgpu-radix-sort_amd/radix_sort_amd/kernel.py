"""Host-side mirror of the reference's kernel classes, over the HIP C ABI.

Reference surface (MatthieuLepers/WebGPU-Radix-Sort v1.0.7):

* README API: ``new RadixSortKernel({device, keys, values, count, check_order, bit_count,
  workgroup_size, local_shuffle, avoid_bank_conflicts})`` (README.md:72-88,129,168)
* shipped API: ``new RadixSortBufferKernel({device, data: {keys, values}, count, bitCount,
  workgroupSize, checkOrder, localShuffle, avoidBankConflicts})``
  (src/kernels/radix-sort/RadixSortBufferKernel.ts:9-32, AbstractRadixSortKernel.ts:14-19,52-57,
  AbstractKernel.ts:3-7,22-25)
* ``kernel.dispatch(pass)`` sorts ``buffers.keys`` / ``buffers.values`` in place
  (AbstractRadixSortKernel.ts:221-276); the harness reads ``kernel.buffers.keys``
  (example/tests.ts:72-74)
* ``new PrefixSumKernel({device, data, count, workgroupSize, avoidBankConflicts}).dispatch(pass)``
  (src/kernels/PrefixSumKernel.ts:24-43,147-158): in-place exclusive scan.

Both option spellings are accepted.  Errors mirror the reference: a non-power-of-two workgroup
raises (PrefixSumKernel.ts:33-35: "workgroupSize.x * workgroupSize.y must be a power of two");
bit_count must be a multiple of 4 (README.md:97, unchecked in the reference - SURVEY Q4).
``workgroup_size``, ``local_shuffle`` and ``avoid_bank_conflicts`` never change results (the
HIP kernels use their own tuned geometry, and always stage the scatter through LDS).

Buffers are device memory: torch CUDA tensors (uint32 / int32 / float32, contiguous),
:class:`DeviceBuffer` objects, or raw device pointers (int).  ``dispatch`` is asynchronous on the
given stream (default: torch's current stream for tensors, else the null stream).
"""
from __future__ import annotations

import ctypes
from typing import Any

import numpy as np

from . import _lib
from ._lib import RadixSortError, check

_SENTINEL = object()


class DeviceBuffer:
    """A device allocation owned by librsort (the reference's GPUBuffer from createBuffers,
    example/tests.ts:227-244)."""

    def __init__(self, nbytes: int, device: int = 0):
        L = _lib.load()
        p = ctypes.c_void_p()
        check(L.rs_malloc(device, nbytes, ctypes.byref(p)), "rs_malloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self.device = device

    @classmethod
    def from_numpy(cls, arr: np.ndarray, device: int = 0) -> "DeviceBuffer":
        a = np.ascontiguousarray(arr)
        b = cls(a.nbytes, device)
        b.write(a)
        return b

    def write(self, arr: np.ndarray, stream: int | None = None) -> None:
        a = np.ascontiguousarray(arr)
        if a.nbytes > self.nbytes:
            raise ValueError("array larger than buffer")
        L = _lib.load()
        check(L.rs_memcpy_h2d(self.ptr, a.ctypes.data, a.nbytes, stream), "rs_memcpy_h2d")
        check(L.rs_stream_synchronize(stream), "rs_stream_synchronize")

    def read(self, dtype=np.uint32, count: int | None = None, stream: int | None = None) -> np.ndarray:
        itemsize = np.dtype(dtype).itemsize
        n = self.nbytes // itemsize if count is None else count
        out = np.empty(n, dtype=dtype)
        check(_lib.load().rs_memcpy_d2h(out.ctypes.data, self.ptr, n * itemsize, stream),
              "rs_memcpy_d2h")
        return out

    def free(self) -> None:
        if self.ptr:
            check(_lib.load().rs_free(self.ptr), "rs_free")
            self.ptr = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.free()
        except Exception:
            pass


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch") and hasattr(x, "data_ptr")


def _buffer_info(buf, name: str):
    """-> (device pointer, capacity in u32 elements or None, device ordinal or None)."""
    if buf is None:
        return None, None, None
    if _is_torch(buf):
        import torch
        if buf.device.type != "cuda":
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG, f"{name} must be a device (cuda) tensor")
        if buf.element_size() != 4:
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG,
                                 f"{name}: elements must be 4 bytes (README.md limitations)")
        if not buf.is_contiguous():
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG, f"{name} must be contiguous")
        del torch
        return buf.data_ptr(), buf.numel(), buf.device.index
    if isinstance(buf, DeviceBuffer):
        return buf.ptr, buf.nbytes // 4, buf.device
    if isinstance(buf, int):
        return buf, None, None
    raise RadixSortError(_lib.RS_ERR_INVALID_ARG, f"unsupported {name} buffer type {type(buf)!r}")


def _device_ordinal(device, *fallbacks) -> int:
    if device is None or device is _SENTINEL:
        for f in fallbacks:
            if f is not None:
                return int(f)
        return 0
    if isinstance(device, int):
        return device
    if hasattr(device, "index"):  # torch.device
        return 0 if device.index is None else int(device.index)
    if isinstance(device, str):
        return int(device.split(":")[1]) if ":" in device else 0
    raise RadixSortError(_lib.RS_ERR_INVALID_ARG, f"unsupported device {device!r}")


def _stream_handle(stream, uses_torch: bool, device: int):
    if stream is None:
        if uses_torch:
            import torch
            return torch.cuda.current_stream(device).cuda_stream
        return None
    if isinstance(stream, int):
        return stream
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    raise RadixSortError(_lib.RS_ERR_INVALID_ARG, f"unsupported stream {stream!r}")


def _pick(opts: dict, *names, default=None):
    for n in names:
        if n in opts and opts[n] is not None:
            return opts[n]
    return default


def _workgroup(ws) -> tuple[int, int]:
    if ws is None:
        return 16, 16
    if isinstance(ws, dict):
        return int(ws.get("x", 16)), int(ws.get("y", 1 if "x" in ws else 16))
    if isinstance(ws, (tuple, list)):
        return int(ws[0]), int(ws[1]) if len(ws) > 1 else 1
    return int(ws), 1


class RadixSortKernel:
    """Drop-in for ``RadixSortKernel`` / ``RadixSortBufferKernel``: sorts ``keys`` (and
    ``values``) in place, ascending and stable by the low ``bit_count`` bits."""

    def __init__(self, options: dict | None = None, **kw: Any):
        opts = dict(options or {})
        opts.update(kw)
        data = opts.get("data") or {}
        keys = _pick(opts, "keys") if "keys" in opts else data.get("keys")
        values = _pick(opts, "values") if "values" in opts else data.get("values")
        if keys is None:
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG, "keys buffer is required")
        kptr, kcap, kdev = _buffer_info(keys, "keys")
        vptr, vcap, vdev = _buffer_info(values, "values")
        count = _pick(opts, "count")
        if count is None:
            if kcap is None:
                raise RadixSortError(_lib.RS_ERR_INVALID_ARG, "count is required with raw pointers")
            count = kcap
        count = int(count)
        for cap, name in ((kcap, "keys"), (vcap, "values")):
            if cap is not None and cap < count:
                raise RadixSortError(_lib.RS_ERR_INVALID_ARG,
                                     f"{name} buffer holds {cap} elements < count {count}")
        self.device = _device_ordinal(opts.get("device", _SENTINEL), kdev, vdev)
        self.count = count
        self.bit_count = int(_pick(opts, "bit_count", "bitCount", default=32))
        wx, wy = _workgroup(_pick(opts, "workgroup_size", "workgroupSize"))
        self.workgroup_size = {"x": wx, "y": wy}
        self.check_order = bool(_pick(opts, "check_order", "checkOrder", default=False))
        self.local_shuffle = bool(_pick(opts, "local_shuffle", "localShuffle", default=False))
        self.avoid_bank_conflicts = bool(_pick(opts, "avoid_bank_conflicts", "avoidBankConflicts",
                                               default=False))
        self.radix_bits = int(_pick(opts, "radix_bits", "radixBits", default=0))
        self.has_values = values is not None
        self.buffers = {"keys": keys}
        if values is not None:
            self.buffers["values"] = values
        self._uses_torch = _is_torch(keys)
        self._ptrs = (kptr, vptr)
        flags = ((_lib.RS_FLAG_HAS_VALUES if self.has_values else 0)
                 | (_lib.RS_FLAG_CHECK_ORDER if self.check_order else 0)
                 | (_lib.RS_FLAG_LOCAL_SHUFFLE if self.local_shuffle else 0)
                 | (_lib.RS_FLAG_AVOID_BANK_CONFLICTS if self.avoid_bank_conflicts else 0))
        desc = _lib.PlanDesc(self.device, count, self.bit_count, wx, wy, flags, self.radix_bits, 0)
        L = _lib.load()
        plan = ctypes.c_void_p()
        check(L.rs_plan_create(ctypes.byref(desc), ctypes.byref(plan)), "RadixSortKernel")
        self._plan = plan
        _lib.apply_debug(plan)

    # -- reference surface --------------------------------------------------------------------
    def dispatch(self, pass_=None) -> None:
        """Sort in place, asynchronously on ``pass_`` (a stream; None = current stream)."""
        s = _stream_handle(pass_, self._uses_torch, self.device)
        check(_lib.load().rs_plan_sort(self._plan, self._ptrs[0], self._ptrs[1], s), "dispatch")

    def destroy(self) -> None:
        if getattr(self, "_plan", None):
            _lib.load().rs_plan_destroy(self._plan)
            self._plan = None

    def __del__(self):  # pragma: no cover
        try:
            self.destroy()
        except Exception:
            pass

    # -- extras ----------------------------------------------------------------------------
    @property
    def info(self) -> dict:
        inf = _lib.PlanInfo()
        check(_lib.load().rs_plan_info_get(self._plan, ctypes.byref(inf)), "info")
        return {"passes": inf.passes, "digit_bits": list(inf.digit_bits[: inf.passes]),
                "tile_keys": inf.tile_keys, "grid_blocks": inf.grid_blocks,
                "workspace_bytes": inf.workspace_bytes,
                "rank_mode": "ballot" if inf.rank_mode == 1 else "lds_atomic",
                "lane_order_selftest": inf.lane_order_selftest}

    def device_errors(self) -> int:
        """Device error word (synchronises): 0 = ok; non-zero = a bounded wait timed out."""
        e = ctypes.c_uint32(0)
        check(_lib.load().rs_plan_device_errors(self._plan, ctypes.byref(e)), "device_errors")
        return e.value

    def check(self) -> None:
        """Wait for the last dispatch and raise :class:`RadixSortError` (status RS_ERR_DEVICE) if
        any sort on this kernel failed on the device since the last check (a timed-out
        look-back wait: that sort's output is invalid).  Reported once."""
        check(_lib.load().rs_plan_check(self._plan), "check")

    def set_profiling(self, enable: bool, kinds=None) -> None:
        """HIP events around every launch group (kinds=None) or only around the launches of the
        named kinds (e.g. ("scatter", "fallback"): the others run back to back)."""
        L = _lib.load()
        if kinds is None or not enable:
            check(L.rs_plan_set_profiling(self._plan, 1 if enable else 0), "profiling")
        else:
            mask = 0
            for k in kinds:
                mask |= 1 << _lib.KERNEL_NAMES.index(k)
            check(L.rs_plan_set_profiling_kinds(self._plan, mask), "profiling")

    def last_path(self) -> str:
        """Which path the last dispatch took (waits for it): "lsd", "hybrid", "hybrid_fallback"
        (the device chose the LSD passes), "in_order" (check_order: nothing moved) or "none"
        (rs_plan_last_path)."""
        v = ctypes.c_uint32()
        check(_lib.load().rs_plan_last_path(self._plan, ctypes.byref(v)), "last_path")
        return _lib.PATH_NAMES[v.value]

    def presorted_counts(self) -> dict:
        """The presorted path of the last dispatch (waits for it): the elements it marked and the
        elements its merge moved (rs_plan_presorted_counts); zeros when it did not take the path."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.load().rs_plan_presorted_counts(self._plan, ctypes.byref(a), ctypes.byref(b)),
              "presorted_counts")
        return {"marked": int(a.value), "moved": int(b.value)}

    def last_split(self) -> int:
        """How deep the hybrid path's last dispatch split over-full 16-bit buckets (skewed keys):
        0, 2 (by byte 1) or 3 (some sub-buckets by byte 0 too) (rs_plan_last_split)."""
        v = ctypes.c_uint32()
        check(_lib.load().rs_plan_last_split(self._plan, ctypes.byref(v)), "last_split")
        return int(v.value)

    def kernel_times(self, reset: bool = False) -> dict:
        ms = (ctypes.c_double * _lib.RS_KERNEL_KINDS)()
        n = (ctypes.c_uint64 * _lib.RS_KERNEL_KINDS)()
        L = _lib.load()
        check(L.rs_plan_kernel_times(self._plan, ms, n), "kernel_times")
        if reset:
            check(L.rs_plan_reset_kernel_times(self._plan), "reset_kernel_times")
        return {name: {"ms": ms[i], "launches": n[i]} for i, name in enumerate(_lib.KERNEL_NAMES)}


RadixSortBufferKernel = RadixSortKernel


class RadixSortTextureKernel(RadixSortKernel):
    """Drop-in for ``RadixSortTextureKernel`` (src/kernels/radix-sort/RadixSortTextureKernel.ts:
    15-35): the data is ONE array of (key, value) u32 pairs - the rg32uint texels, texel i =
    (x, y) with i = y * width + x (RadixSortReorder.ts:42-63) - sorted in place by key, values
    always carried (``hasValues`` is true, :27-29).

    ``data={"texture": t}`` (or ``texture=t``): a contiguous device tensor whose last dimension
    is 2 (``[height, width, 2]`` or ``[n, 2]``, 4-byte elements), a :class:`DeviceBuffer`, or a
    raw device pointer (then ``count`` is required).  ``count`` defaults to all texels.
    """

    def __init__(self, options: dict | None = None, **kw: Any):
        opts = dict(options or {})
        opts.update(kw)
        data = opts.get("data") or {}
        tex = _pick(opts, "texture") if "texture" in opts else data.get("texture")
        if tex is None:
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG, "texture is required")
        if _is_torch(tex) and (tex.dim() < 2 or tex.shape[-1] != 2):
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG,
                                 "texture tensor must have a last dimension of 2 (rg32uint texels)")
        tptr, tcap, tdev = _buffer_info(tex, "texture")
        texels = None if tcap is None else tcap // 2
        count = _pick(opts, "count")
        if count is None:
            if texels is None:
                raise RadixSortError(_lib.RS_ERR_INVALID_ARG, "count is required with raw pointers")
            count = texels
        count = int(count)
        if texels is not None and texels < count:
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG,
                                 f"texture holds {texels} texels < count {count}")
        self.device = _device_ordinal(opts.get("device", _SENTINEL), tdev)
        self.count = count
        self.bit_count = int(_pick(opts, "bit_count", "bitCount", default=32))
        wx, wy = _workgroup(_pick(opts, "workgroup_size", "workgroupSize"))
        self.workgroup_size = {"x": wx, "y": wy}
        self.check_order = bool(_pick(opts, "check_order", "checkOrder", default=False))
        self.local_shuffle = False
        self.avoid_bank_conflicts = bool(_pick(opts, "avoid_bank_conflicts", "avoidBankConflicts",
                                               default=False))
        self.radix_bits = int(_pick(opts, "radix_bits", "radixBits", default=0))
        self.has_values = True
        self.textures = {"read": tex}
        self.buffers = {}
        self._uses_torch = _is_torch(tex)
        self._ptrs = (tptr, None)
        flags = (_lib.RS_FLAG_INTERLEAVED
                 | (_lib.RS_FLAG_CHECK_ORDER if self.check_order else 0)
                 | (_lib.RS_FLAG_AVOID_BANK_CONFLICTS if self.avoid_bank_conflicts else 0))
        desc = _lib.PlanDesc(self.device, count, self.bit_count, wx, wy, flags, self.radix_bits, 0)
        plan = ctypes.c_void_p()
        check(_lib.load().rs_plan_create(ctypes.byref(desc), ctypes.byref(plan)),
              "RadixSortTextureKernel")
        self._plan = plan
        _lib.apply_debug(plan)


class PrefixSumKernel:
    """Drop-in for ``PrefixSumKernel``: in-place exclusive scan (mod 2^32) of data[:count]."""

    def __init__(self, options: dict | None = None, **kw: Any):
        opts = dict(options or {})
        opts.update(kw)
        data = opts.get("data")
        if data is None:
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG, "data buffer is required")
        ptr, cap, dev = _buffer_info(data, "data")
        count = _pick(opts, "count", default=cap)
        if count is None:
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG, "count is required with raw pointers")
        count = int(count)
        if cap is not None and cap < count:
            raise RadixSortError(_lib.RS_ERR_INVALID_ARG, f"data holds {cap} elements < count {count}")
        wx, wy = _workgroup(_pick(opts, "workgroup_size", "workgroupSize"))
        self.device = _device_ordinal(opts.get("device", _SENTINEL), dev)
        self.count = count
        self.workgroup_size = {"x": wx, "y": wy}
        self.avoid_bank_conflicts = bool(_pick(opts, "avoid_bank_conflicts", "avoidBankConflicts",
                                               default=False))
        self.data = data
        self._ptr = ptr
        self._uses_torch = _is_torch(data)
        plan = ctypes.c_void_p()
        flags = _lib.RS_FLAG_AVOID_BANK_CONFLICTS if self.avoid_bank_conflicts else 0
        check(_lib.load().rs_scan_plan_create(self.device, count, wx, wy, flags,
                                              ctypes.byref(plan)), "PrefixSumKernel")
        self._plan = plan

    def dispatch(self, pass_=None, dispatch_size_buffer=None, offset: int = 0) -> None:
        """In-place exclusive scan on stream ``pass_``.  With ``dispatch_size_buffer`` (device
        memory of u32 (x, y, z) triples, e.g. :meth:`get_dispatch_chain` written to the device) the
        dispatch is indirect (PrefixSumKernel.ts:147-158): the scan runs iff the triple at byte
        ``offset`` has no zero entry, decided on the device."""
        s = _stream_handle(pass_, self._uses_torch, self.device)
        if dispatch_size_buffer is None:
            check(_lib.load().rs_scan_plan_run(self._plan, self._ptr, s), "dispatch")
            return
        bptr, _, _ = _buffer_info(dispatch_size_buffer, "dispatch_size_buffer")
        check(_lib.load().rs_scan_plan_run_indirect(self._plan, self._ptr, bptr, int(offset), s),
              "dispatch")

    def get_dispatch_chain(self) -> list:
        """The reference's dispatch chain (PrefixSumKernel.getDispatchChain, :135-137):
        [x, y, 1] per pipeline, flattened."""
        L = _lib.load()
        n = L.rs_scan_plan_dispatch_chain(self._plan, None, 0)
        out = (ctypes.c_uint32 * max(n, 1))()
        L.rs_scan_plan_dispatch_chain(self._plan, out, n)
        return list(out[:n])

    getDispatchChain = get_dispatch_chain

    def check(self) -> None:
        """Wait for the last dispatch; raise RadixSortError (RS_ERR_DEVICE) if a scan since the
        last check failed on the device (a timed-out look-back wait: its output is invalid)."""
        check(_lib.load().rs_scan_plan_check(self._plan), "check")

    def destroy(self) -> None:
        if getattr(self, "_plan", None):
            _lib.load().rs_scan_plan_destroy(self._plan)
            self._plan = None

    def __del__(self):  # pragma: no cover
        try:
            self.destroy()
        except Exception:
            pass
