"""Single-process multi-GPU sort over the C ABI (``rs_group_*``, include/rsort.h).

The reference has no multi-device path; this is the build's sharded sort for
an input spread over the GPUs of one node, driven from ONE host process the way the Node addon
(the reference's host language) reaches it: ``rs_group_create`` opens one RCCL communicator per
device (``ncclCommInitAll``), ``rs_group_sort`` runs the bucket exchange (top-digit histograms
-> host bucket plan -> stable partition -> rounds of ncclSend/ncclRecv -> local sorts that
start as each round lands).  The multi-process form of the same algorithm, one process per GPU
over ``torch.distributed``, is :mod:`radix_sort_amd.distributed`.

    g = RadixSortGroup(devices=[0, 1], capacity=n, has_values=True)
    out = g.sort([k0, k1], [v0, v1])   # -> [(keys_r, values_r), ...], rank-ordered slices
"""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import check


def group_plan(hist_all, rounds: int):
    """The C bucket plan (rs_group_plan): (bounds[world + 1], cuts[world][rounds + 1]) from the
    [world][buckets] top-digit counts; a pure host function."""
    world, buckets = len(hist_all), len(hist_all[0])
    flat = (ctypes.c_uint64 * (world * buckets))(*[int(x) for row in hist_all for x in row])
    bounds = (ctypes.c_uint32 * (world + 1))()
    cuts = (ctypes.c_uint32 * (world * (rounds + 1)))()
    check(_lib.load().rs_group_plan(world, buckets, rounds, flat, bounds, cuts), "rs_group_plan")
    return list(bounds), [list(cuts[q * (rounds + 1):(q + 1) * (rounds + 1)]) for q in range(world)]


class RadixSortGroup:
    """world ranks on `devices` (a device may repeat with transport="copy": virtual ranks)."""

    def __init__(self, devices, capacity: int, has_values: bool = True, rounds: int = 4,
                 top_bits: int = 8, transport: str = "rccl"):
        if transport not in ("rccl", "copy"):
            raise ValueError("transport must be 'rccl' or 'copy'")
        self.devices = [int(d) for d in devices]
        self.world = len(self.devices)
        self.has_values = has_values
        desc = _lib.GroupDesc(capacity, _lib.RS_FLAG_HAS_VALUES if has_values else 0,
                              _lib.RS_TRANSPORT_RCCL if transport == "rccl" else _lib.RS_TRANSPORT_COPY,
                              top_bits, rounds)
        devs = (ctypes.c_int32 * self.world)(*self.devices)
        g = ctypes.c_void_p()
        check(_lib.load().rs_group_create(self.world, devs, ctypes.byref(desc), ctypes.byref(g)),
              "rs_group_create")
        self._g = g

    def sort_async(self, keys, values=None, counts=None, streams=None) -> None:
        """Enqueue the sort of the slices keys[r] (+ values[r]) (torch tensors on devices[r]);
        streams: None (ordered after / before each device's current stream) or a list."""
        import torch
        W = self.world
        if len(keys) != W or (self.has_values and (values is None or len(values) != W)):
            raise ValueError(f"need {W} key (and value) slices")
        counts = [k.numel() for k in keys] if counts is None else list(counts)
        if streams is None:
            streams = [torch.cuda.current_stream(k.device).cuda_stream for k in keys]
        kp = (ctypes.c_void_p * W)(*[k.data_ptr() for k in keys])
        vp = (ctypes.c_void_p * W)(*[v.data_ptr() for v in values]) if self.has_values else None
        cn = (ctypes.c_uint64 * W)(*counts)
        sp = (ctypes.c_void_p * W)(*[s if isinstance(s, int) else s.cuda_stream for s in streams])
        check(_lib.load().rs_group_sort(self._g, kp, vp, cn, sp), "rs_group_sort")

    def result_pointers(self, rank: int):
        """(keys_ptr, values_ptr, count) of rank's slice (group-owned device buffers)."""
        k, v, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        check(_lib.load().rs_group_result(self._g, rank, ctypes.byref(k), ctypes.byref(v),
                                          ctypes.byref(n)), "rs_group_result")
        return k.value, v.value, n.value

    def synchronize(self) -> None:
        check(_lib.load().rs_group_synchronize(self._g), "rs_group_synchronize")

    def set_profiling(self, enable: bool) -> None:
        """Timing events on every rank from the next sort on (rs_group_set_profiling)."""
        check(_lib.load().rs_group_set_profiling(self._g, 1 if enable else 0), "rs_group_set_profiling")

    def times(self, rank: int) -> dict:
        """Where rank's last sort spent its time (rs_group_times_get; waits for it): ms since the
        sort's start, and the rank's off-rank exchange bytes."""
        t = _lib.GroupTimes()
        check(_lib.load().rs_group_times_get(self._g, rank, ctypes.byref(t)), "rs_group_times_get")
        G = t.rounds
        return {"rounds": G, "hist16_ms": t.hist16_ms, "partition_ms": t.partition_ms,
                "round_done_ms": list(t.round_done_ms[:G]), "region_sorted_ms": list(t.region_sorted_ms[:G]),
                "done_ms": t.done_ms, "bytes_sent": t.bytes_sent, "bytes_recv": t.bytes_recv}

    def sort(self, keys, values=None, counts=None):
        """Sort and return [(keys_r, values_r or None)] as new int32 tensors on devices[r]
        (copied out of the group's buffers)."""
        import torch
        self.sort_async(keys, values, counts)
        self.synchronize()
        L = _lib.load()
        out = []
        for r in range(self.world):
            kp, vp, n = self.result_pointers(r)
            dev = torch.device("cuda", self.devices[r])
            ko = torch.empty(n, dtype=torch.int32, device=dev)
            vo = torch.empty(n, dtype=torch.int32, device=dev) if self.has_values else None
            s = torch.cuda.current_stream(dev).cuda_stream
            if n:
                check(L.rs_memcpy_d2d(ko.data_ptr(), kp, 4 * n, s), "rs_memcpy_d2d")
                if vo is not None:
                    check(L.rs_memcpy_d2d(vo.data_ptr(), vp, 4 * n, s), "rs_memcpy_d2d")
            out.append((ko, vo))
        for r in range(self.world):
            torch.cuda.synchronize(self.devices[r])
        return out

    def destroy(self) -> None:
        if getattr(self, "_g", None):
            _lib.load().rs_group_destroy(self._g)
            self._g = None

    def __del__(self):  # pragma: no cover
        try:
            self.destroy()
        except Exception:
            pass
