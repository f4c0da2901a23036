"""Multi-GPU sort: one process per GPU, one bucket exchange at the top digit.

The reference has no multi-device path; this is the build's sharding of the
same sort for inputs spread over the GPUs of one node (BASELINE config 5):

1. rank r holds a contiguous slice of the global input;
2. the top-``bits`` digit histogram of the slice (``rs_histogram``, one read of the keys);
3. ``all_gather`` of the histograms (RCCL over xGMI; a few KB) and one copy to the host, where
   every rank computes the same bucket -> rank assignment on whole-bucket boundaries (equal
   keys never split), and splits every rank's buckets into G consecutive groups of about equal
   key counts (again whole buckets);
4. a stable partition of the slice by the top digit (one scatter pass of the radix sort, the
   one-sweep pass fed the step-2 counts: one key read), written as 8-byte (key, value) records
   (``rs_plan_partition_records``; keys only: ``rs_plan_partition_totals``), overlapped with the
   host's wait for the counts: every (peer, group) send segment is now one contiguous range;
5. G exchange rounds: round g is one batch of point-to-point messages (``batch_isend_irecv``;
   RCCL sends to all peers at once, over all 7 xGMI links of a rank), one message per peer with
   its group-g buckets' records.  The receiver lays round g out as [source 0's segment,
   source 1's, ...] in its group-g region, which is therefore complete once round g lands: it
   holds every key of those buckets, equal keys in (source rank, input position) order = global
   input order;
6. as soon as round g has landed, the group-g region is sorted locally (stable LSD, the same
   plan; ``rs_plan_sort_records``: records in, separate key / value arrays out), while rounds
   g+1.. are still on the wire: the local sort hides under the exchange,
   and only the last group's sort is exposed.  Groups hold increasing buckets, so the regions
   concatenated are rank r's part of the global stable order.

Stability: the partition is stable, segments are placed in source-rank order, the local sort
is stable, and a bucket never spans two groups or two ranks.

The local compute is injected (`LocalOps`): the product uses :class:`HipLocalOps` (librsort);
the CPU gloo tests inject an oracle-backed implementation.  The exchange itself
(:func:`exchange_round`: point-to-point messages batched per round, the own segment copied
locally) is ONE code path for every backend, so the gloo world-2/3 tests run exactly what RCCL
runs on the GPUs.  With values, a message is a run of 8-byte (key, value) records (the partition
writes records, the local sort reads them and writes separate arrays): one message per peer per
round instead of two.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Protocol


class LocalOps(Protocol):
    def histogram(self, keys, shift: int, bits: int):
        """-> hist[2^bits] int32 tensor on the keys' device (top-digit counts of keys)."""

    def partition(self, keys, values, shift: int, bits: int, totals):
        """Stable partition by (key >> shift) & (2^bits - 1) -> the send buffer: with values, one
        int64 (key, value) record per key (key | value << 32, the interleaved layout: one message
        per peer carries both); keys only, the int32 keys.  totals: histogram() of the same keys."""

    def sort_records(self, records, keys_out, values_out, key_range=None) -> None:
        """Stable sort of the int64 records by their 32-bit key into keys_out / values_out.
        key_range: (lo, hi), every key in [lo, hi] (the round's top-digit buckets), a hint."""

    def sort(self, keys, n: int) -> None:
        """Stable in-place sort of keys[:n] (keys only) by the full 32-bit key."""

    def sort_copy(self, keys, values, keys_out, values_out) -> None:
        """Stable out-of-place sort of (keys, values) by the 32-bit key into keys_out /
        values_out (values None: keys only); the input is only read."""

    def empty(self, n: int, like):
        """Uninitialised buffer of n elements of like's dtype on like's device."""


def _split_whole(counts, lo: int, hi: int, parts: int):
    """Cut buckets [lo, hi) into `parts` consecutive runs of whole buckets of ~equal total count.
    Returns parts + 1 bucket indices (first lo, last hi); part p = [cut[p], cut[p + 1])."""
    total = sum(int(counts[b]) for b in range(lo, hi))
    cuts = [lo]
    cum = 0
    p = 1
    for b in range(lo, hi):
        while p < parts and cum >= (total * p + parts - 1) // parts:
            cuts.append(b)
            p += 1
        cum += int(counts[b])
    while p < parts:
        cuts.append(hi)
        p += 1
    cuts.append(hi)
    return cuts


def bucket_owners(hist_all, world: int):
    """Whole-bucket split of the global histogram (host, identical on every rank).

    hist_all: [world][B] counts (nested lists or array).  Returns bounds[0..world] with rank q
    owning buckets [bounds[q], bounds[q+1]).  Rank q's boundary is the first bucket at which the
    running total reaches q/world of the keys, so each rank gets ~1/world of them."""
    B = len(hist_all[0])
    totals = [sum(int(h[b]) for h in hist_all) for b in range(B)]
    return _split_whole(totals, 0, B, world)


def bucket_groups(hist_all, bounds, groups: int):
    """Every rank's buckets cut into `groups` exchange rounds: cuts[q] = groups + 1 bucket
    indices, round g of rank q = buckets [cuts[q][g], cuts[q][g + 1]) (whole buckets, ~equal
    key counts; empty rounds are allowed)."""
    B = len(hist_all[0])
    totals = [sum(int(h[b]) for h in hist_all) for b in range(B)]
    return [_split_whole(totals, bounds[q], bounds[q + 1], groups) for q in range(len(bounds) - 1)]


def round_key_range(cuts_rank, g: int, bits: int):
    """[lo, hi] of every key in round g's buckets [cuts_rank[g], cuts_rank[g + 1]) of the
    top-`bits` digit (the hint the group sort passes to the local sort)."""
    shift = 32 - bits
    a, b = int(cuts_rank[g]), int(cuts_rank[g + 1])
    return a << shift, min((b << shift) - 1, 0xFFFFFFFF)


def split_sizes(hist_all, bounds, rank: int, world: int):
    """(send sizes of this rank to every peer, receive sizes from every peer)."""
    send = [sum(int(hist_all[rank][b]) for b in range(bounds[q], bounds[q + 1]))
            for q in range(world)]
    recv = [sum(int(hist_all[s][b]) for b in range(bounds[rank], bounds[rank + 1]))
            for s in range(world)]
    return send, recv


@dataclass
class GroupPlan:
    send: list   # send[g][q] = (begin, end) of the partitioned slice going to peer q in round g
    recv: list   # recv[g][s] = keys arriving from source s in round g
    off: list    # off[g][s] = where they land in the receive buffer
    base: list   # base[g] = start of round g's region; base[G] = total received


def group_plan(hist_all, cuts, rank: int, world: int) -> GroupPlan:
    """Send ranges, receive sizes and receive offsets of every exchange round.

    hist_all: [world][B] top-digit counts; cuts: bucket_groups().  The partitioned slice holds
    bucket b at [start[b], start[b + 1]) (start = exclusive scan of this rank's counts), so a
    round's segment to one peer is one contiguous range.  The receive buffer is round-major,
    then source-major: round g's region is complete when round g has landed."""
    mine = [int(x) for x in hist_all[rank]]
    start = [0]
    for c in mine:
        start.append(start[-1] + c)
    G = len(cuts[0]) - 1
    send = [[(start[cuts[q][g]], start[cuts[q][g + 1]]) for q in range(world)] for g in range(G)]
    recv = [[sum(int(x) for x in hist_all[s][cuts[rank][g]:cuts[rank][g + 1]]) for s in range(world)]
            for g in range(G)]
    off, base, pos = [], [], 0
    for g in range(G):
        base.append(pos)
        row = []
        for s in range(world):
            row.append(pos)
            pos += recv[g][s]
        off.append(row)
    base.append(pos)
    return GroupPlan(send, recv, off, base)


@dataclass
class ExchangeResult:
    keys: object
    values: object
    n: int
    send_sizes: list
    recv_sizes: list


def distributed_sort(keys, values, ops: LocalOps, group=None, bits: int = 8,
                     chunks: int = 4) -> ExchangeResult:
    """Sort the global array whose slice on this rank is (keys, values); returns this rank's
    slice of the global stable sorted order (rank-ordered concatenation).  `chunks` = exchange
    rounds (bucket groups per rank), each sorted while the next ones are on the wire.

    On the GPU the work runs on a side stream (ordered after the caller's current stream, and
    the caller's stream after it): the legacy default stream would serialise every local sort
    with the in-flight exchange and undo the overlap."""
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


def exchange_round(send, recv, plan: GroupPlan, g: int, rank: int, world: int, group=None):
    """Round g of the bucket exchange, the same code on every backend (gloo on CPU, RCCL on the
    GPUs): one point-to-point message per peer carrying that peer's round-g buckets (records or
    keys), received into the peer's source slot of the round-g region; the rank's own segment is
    a local copy (RCCL moves a self segment through a few channels at ~0.3 TB/s, measured).
    Both sides skip empty messages (they compute the same sizes).  -> the round's works."""
    import torch.distributed as dist
    a, b = plan.send[g][rank]
    o = plan.off[g][rank]
    if b > a and recv.data_ptr() != send.data_ptr():
        recv[o:o + (b - a)].copy_(send[a:b])
    p2p = []
    for q in range(world):
        if q == rank:
            continue
        a, b = plan.send[g][q]
        if b > a:
            p2p.append(dist.P2POp(dist.isend, send[a:b], q, group))
        m = plan.recv[g][q]
        if m:
            o = plan.off[g][q]
            p2p.append(dist.P2POp(dist.irecv, recv[o:o + m], q, group))
    return dist.batch_isend_irecv(p2p) if p2p else []


def _distributed_sort(keys, values, ops, group, bits, chunks) -> ExchangeResult:
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_local = keys.numel()
    if world == 1:
        # one rank holds the whole array: nothing to exchange, so no partition either - one
        # out-of-place sort (pass 0 reads the input, the last pass writes the result)
        out_k = ops.empty(n_local, keys)
        out_v = None if values is None else ops.empty(n_local, values)
        ops.sort_copy(keys, values, out_k, out_v)
        return ExchangeResult(out_k, out_v, n_local, [n_local], [n_local])
    G = max(1, int(chunks))
    shift = 32 - bits
    hist = ops.histogram(keys, shift, bits)                     # [2^bits]
    gathered = [torch.empty_like(hist) for _ in range(world)]
    dist.all_gather(gathered, hist, group=group)
    if keys.is_cuda:
        # the counts travel to the host while the slice is partitioned (the partition needs no
        # bucket ownership): copy, mark, enqueue the partition, then wait for the mark only
        hcpu = torch.empty((world,) + tuple(hist.shape), dtype=hist.dtype, pin_memory=True)
        hcpu.copy_(torch.stack(gathered), non_blocking=True)
        ready = torch.cuda.Event()
        ready.record()
        send = ops.partition(keys, values, shift, bits, hist)
        ready.synchronize()
        hist_all = hcpu.tolist()
    else:
        hist_all = torch.stack(gathered).tolist()
        send = ops.partition(keys, values, shift, bits, hist)
    bounds = bucket_owners(hist_all, world)
    cuts = bucket_groups(hist_all, bounds, G)
    plan = group_plan(hist_all, cuts, rank, world)
    n_recv = plan.base[G]
    # one rank: the receive layout is the partitioned slice itself (no copy)
    recv = send if world == 1 else ops.empty(n_recv, send)
    rounds = [exchange_round(send, recv, plan, g, rank, world, group) for g in range(G)]
    if values is None:
        out_k, out_v = recv, None
    else:
        out_k, out_v = ops.empty(n_recv, keys), ops.empty(n_recv, values)
    # round g's local sort waits for round g only (the stream waits, not the host); later rounds
    # keep moving meanwhile
    for g in range(G):
        for w in rounds[g]:
            w.wait()
        a, b = plan.base[g], plan.base[g + 1]
        if b > a:
            if values is None:
                ops.sort(recv[a:b], b - a)
            else:
                ops.sort_records(recv[a:b], out_k[a:b], out_v[a:b],
                                 key_range=round_key_range(cuts[rank], g, bits))
    return ExchangeResult(out_k, out_v, n_recv,
                          [sum(b - a for a, b in (plan.send[g][q] for g in range(G))) for q in range(world)],
                          [sum(plan.recv[g][s] for g in range(G)) for s in range(world)])


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

    def partition(self, keys, values, shift: int, bits: int, totals):
        import torch
        n = keys.numel()
        if self.part_plan is None or self.part_plan.capacity < n:
            from .ops import SortPlan
            if self.part_plan is not None:
                self.part_plan.destroy()
            self.part_plan = SortPlan(self.device, max(n, 1), self.has_values, 32, self.radix_bits)
        if values is None:
            sk = torch.empty_like(keys)
            self.part_plan.partition_totals(keys, None, sk, None, n, shift, bits, totals)
            return sk
        rec = torch.empty(n, dtype=torch.int64, device=keys.device)
        self.part_plan.partition_records(keys, values, rec, n, shift, bits, totals)
        return rec

    def _grow(self, n: int) -> None:
        if n > self.capacity:
            from .ops import SortPlan
            self.plan.destroy()
            self.capacity = int(n * 1.125)
            self.plan = SortPlan(self.device, self.capacity, self.has_values, 32, self.radix_bits)

    def sort(self, keys, n: int) -> None:
        self._grow(n)
        self.plan.sort(keys, None, n)

    def sort_records(self, records, keys_out, values_out, key_range=None) -> None:
        n = records.numel()
        self._grow(n)
        self.plan.sort_records(records, keys_out, values_out, n, key_range=key_range)

    def sort_copy(self, keys, values, keys_out, values_out) -> None:
        n = keys.numel()
        self._grow(n)
        self.plan.sort_copy(keys, values, keys_out, values_out, n)

    def check(self) -> None:
        """Raise if a local sort or partition failed on the device (rs_plan_check)."""
        self.plan.check()
        if self.part_plan is not None:
            self.part_plan.check()

    def destroy(self) -> None:
        self.plan.destroy()
        if self.part_plan is not None:
            self.part_plan.destroy()
            self.part_plan = None
