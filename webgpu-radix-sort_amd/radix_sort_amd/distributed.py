"""Multi-GPU sort: one process per GPU, one bucket exchange at the top digit.

The reference has no multi-device path; this is the build's sharding of the
same sort for inputs spread over the GPUs of one node (BASELINE config 5):

1. rank r holds a contiguous slice of the global input, cut into C chunks;
2. the top-``bits`` digit histogram of every chunk (``rs_histogram``, one read of the keys);
3. ``all_gather`` of the [C][2^bits] histograms (RCCL over xGMI; a few KB) and one copy to the
   host, where every rank computes the same bucket -> rank assignment on whole-bucket
   boundaries (equal keys never split) and every send / receive segment's size and place;
4. per chunk: a stable partition of the chunk by the top digit (one scatter pass of the radix
   sort, ``rs_plan_partition``) on the compute stream, then an asynchronous all-to-all of its
   keys and values (RCCL: every rank sends to all peers at once, using all 7 xGMI links of a
   rank) that runs while the next chunk is partitioned.  Each received segment lands directly
   at its final place: the receive buffer is ordered by (source rank, chunk), i.e. by global
   input position;
5. a local stable LSD sort of the receive buffer is rank r's part of the global stable order.

Stability: ties keep input order because each chunk's partition is stable and segments are
placed in (source rank, chunk) order, which is global input order; the local sort is stable.

The local compute is injected (`LocalOps`): the product uses :class:`HipLocalOps` (librsort);
the CPU gloo tests inject an oracle-backed implementation to exercise the orchestration.  gloo
has no list all-to-all, so there (and only there) each chunk is exchanged with
``all_to_all_single`` into a staging buffer and copied into place.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Protocol


class LocalOps(Protocol):
    def histogram(self, keys, shift: int, bits: int):
        """-> hist[2^bits] int32 tensor on the keys' device (top-digit counts of keys)."""

    def partition(self, keys, values, shift: int, bits: int, out_keys=None, out_values=None):
        """Stable partition by (key >> shift) & (2^bits - 1) -> (keys_out, values_out); written
        into out_keys / out_values when given."""

    def sort(self, keys, values, n: int) -> None:
        """Stable in-place sort of keys[:n] (and values[:n]) by the full 32-bit key."""

    def empty(self, n: int, like):
        """Uninitialised buffer of n 32-bit words on like's device."""


def bucket_owners(hist_all, world: int):
    """Whole-bucket split of the global histogram (host, identical on every rank).

    hist_all: [world][B] counts (nested lists or array).  Returns bounds[0..world] with rank q
    owning buckets [bounds[q], bounds[q+1]).  Rank q's boundary is the first bucket at which the
    running total reaches q/world of the keys, so each rank gets ~1/world of them."""
    B = len(hist_all[0])
    totals = [sum(int(h[b]) for h in hist_all) for b in range(B)]
    grand = sum(totals)
    bounds = [0] * (world + 1)
    bounds[world] = B
    cum = 0
    q = 1
    for b in range(B):
        while q < world and cum >= (grand * q + world - 1) // world:
            bounds[q] = b
            q += 1
        cum += totals[b]
    while q < world:
        bounds[q] = B
        q += 1
    return bounds


def split_sizes(hist_all, bounds, rank: int, world: int):
    """(send sizes of this rank to every peer, receive sizes from every peer)."""
    send = [sum(int(hist_all[rank][b]) for b in range(bounds[q], bounds[q + 1]))
            for q in range(world)]
    recv = [sum(int(hist_all[s][b]) for b in range(bounds[rank], bounds[rank + 1]))
            for s in range(world)]
    return send, recv


def exchange_plan(hist_chunks, bounds, rank: int, world: int):
    """Segment sizes and receive offsets for a chunked exchange.

    hist_chunks: [world][C][B] top-digit counts.  Returns (send[c][q], recv[c][s], off[c][s])
    where off[c][s] is where source s's chunk-c segment starts in this rank's receive buffer,
    ordered by (source, chunk) = global input order."""
    C = len(hist_chunks[0])
    lo, hi = bounds[rank], bounds[rank + 1]
    send = [[sum(int(x) for x in hist_chunks[rank][c][bounds[q]:bounds[q + 1]]) for q in range(world)]
            for c in range(C)]
    recv = [[sum(int(x) for x in hist_chunks[s][c][lo:hi]) for s in range(world)] for c in range(C)]
    off = [[0] * world for _ in range(C)]
    pos = 0
    for s in range(world):
        for c in range(C):
            off[c][s] = pos
            pos += recv[c][s]
    return send, recv, off


@dataclass
class ExchangeResult:
    keys: object
    values: object
    n: int
    send_sizes: list
    recv_sizes: list


def _chunk_bounds(n: int, chunks: int):
    step = -(-n // chunks) if n else 0
    return [(min(n, c * step), min(n, (c + 1) * step)) for c in range(chunks)]


def distributed_sort(keys, values, ops: LocalOps, group=None, bits: int = 8,
                     chunks: int = 4) -> ExchangeResult:
    """Sort the global array whose slice on this rank is (keys, values); returns this rank's
    slice of the global stable sorted order (rank-ordered concatenation).

    On the GPU the work runs on a side stream (ordered after the caller's current stream, and
    the caller's stream after it): the legacy default stream would serialise every partition
    with the in-flight all-to-alls and undo the overlap."""
    import torch

    if keys.is_cuda:
        caller = torch.cuda.current_stream(keys.device)
        side = _side_stream(keys.device)
        side.wait_stream(caller)
        with torch.cuda.stream(side):
            r = _distributed_sort(keys, values, ops, group, bits, chunks)
        caller.wait_stream(side)
        for t in (r.keys, r.values):
            if t is not None:
                t.record_stream(caller)
        return r
    return _distributed_sort(keys, values, ops, group, bits, chunks)


_SIDE = {}


def _side_stream(device):
    import torch
    if device not in _SIDE:
        _SIDE[device] = torch.cuda.Stream(device)
    return _SIDE[device]


def _distributed_sort(keys, values, ops, group, bits, chunks) -> ExchangeResult:
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_local = keys.numel()
    chunks = max(1, min(chunks, n_local)) if n_local else 1
    shift = 32 - bits
    cb = _chunk_bounds(n_local, chunks)
    hist = torch.stack([ops.histogram(keys[a:b], shift, bits) for a, b in cb])   # [C][2^bits]
    gathered = [torch.empty_like(hist) for _ in range(world)]
    dist.all_gather(gathered, hist, group=group)
    sk = ops.empty(n_local, keys)
    sv = None if values is None else ops.empty(n_local, values)

    def partition(c):
        a, b = cb[c]
        ops.partition(keys[a:b], None if values is None else values[a:b], shift, bits,
                      sk[a:b], None if sv is None else sv[a:b])

    if keys.is_cuda:
        # the counts travel to the host while chunk 0 is partitioned (the partition needs no
        # bucket ownership): copy, mark, enqueue the partition, then wait for the mark only
        hcpu = torch.empty((world,) + tuple(hist.shape), dtype=hist.dtype, pin_memory=True)
        hcpu.copy_(torch.stack(gathered), non_blocking=True)
        ready = torch.cuda.Event()
        ready.record()
        partition(0)
        ready.synchronize()
        hist_all = hcpu.tolist()
    else:
        hist_all = torch.stack(gathered).tolist()
        partition(0)
    bounds = bucket_owners([[sum(h[c][b] for c in range(chunks)) for b in range(1 << bits)]
                            for h in hist_all], world)
    send, recv, off = exchange_plan(hist_all, bounds, rank, world)
    n_recv = sum(sum(r) for r in recv)
    rk = ops.empty(n_recv, keys)
    rv = None if values is None else ops.empty(n_recv, values)
    list_a2a = dist.get_backend(group) != "gloo"
    works = []
    for c, (a, b) in enumerate(cb):
        if c:
            partition(c)
        for src, dst in ((sk, rk), (sv, rv)):
            if src is None:
                continue
            ins = list(src[a:b].split(send[c]))
            outs = [dst[off[c][s]:off[c][s] + recv[c][s]] for s in range(world)]
            if list_a2a:
                works.append(dist.all_to_all(outs, ins, group=group, async_op=True))
            else:
                stage = ops.empty(sum(recv[c]), dst)
                dist.all_to_all_single(stage, src[a:b], output_split_sizes=recv[c],
                                       input_split_sizes=send[c], group=group)
                for s, o in enumerate(outs):
                    o.copy_(stage[sum(recv[c][:s]):sum(recv[c][:s + 1])])
    for w in works:
        w.wait()
    ops.sort(rk, rv, n_recv)
    return ExchangeResult(rk, rv, n_recv, [sum(send[c][q] for c in range(chunks)) for q in range(world)],
                          [sum(recv[c][s] for c in range(chunks)) for s in range(world)])


class HipLocalOps:
    """librsort-backed local steps (the product path)."""

    def __init__(self, device: int, capacity: int, has_values: bool, radix_bits: int = 0):
        from .ops import SortPlan
        self.device = device
        self.has_values = has_values
        self.radix_bits = radix_bits
        self.plan = SortPlan(device, capacity, has_values, 32, radix_bits)   # the local sort
        self.part_plan = None     # partition passes (own plan: separate kernel timings)
        self.capacity = capacity

    def empty(self, n: int, like):
        import torch
        return torch.empty(n, dtype=like.dtype, device=like.device)

    def histogram(self, keys, shift: int, bits: int):
        import torch
        from .ops import histogram
        h = torch.empty(1 << bits, dtype=torch.int32, device=keys.device)
        histogram(keys, keys.numel(), shift, bits, h)
        return h

    def partition(self, keys, values, shift: int, bits: int, out_keys=None, out_values=None):
        import torch
        n = keys.numel()
        sk = torch.empty_like(keys) if out_keys is None else out_keys
        sv = None if values is None else (torch.empty_like(values) if out_values is None else out_values)
        if self.part_plan is None or self.part_plan.capacity < n:
            from .ops import SortPlan
            if self.part_plan is not None:
                self.part_plan.destroy()
            self.part_plan = SortPlan(self.device, max(n, 1), self.has_values, 32, self.radix_bits)
        self.part_plan.partition(keys, values, sk, sv, n, shift, bits, None)
        return sk, sv

    def destroy(self) -> None:
        self.plan.destroy()
        if self.part_plan is not None:
            self.part_plan.destroy()
            self.part_plan = None

    def sort(self, keys, values, n: int) -> None:
        if n > self.capacity:
            from .ops import SortPlan
            self.plan.destroy()
            self.capacity = int(n * 1.125)
            self.plan = SortPlan(self.device, self.capacity, self.has_values, 32, self.radix_bits)
        self.plan.sort(keys, values, n)
