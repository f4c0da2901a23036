"""Multi-GPU sort: one process per GPU, one bucket exchange at the top digit.

The reference has no multi-device path; this is the build's sharding of the
same sort for inputs spread over the GPUs of one node (BASELINE config 5):

1. rank r holds a contiguous slice of the global input;
2. the top-``bits`` digit histogram of the slice (``rs_histogram``, one read of the keys);
3. ``all_gather`` of the histograms (RCCL over xGMI; a few KB) and one copy to the host, where
   every rank computes the same bucket -> rank assignment on whole-bucket boundaries (equal
   keys never split), and splits every rank's buckets into G consecutive groups of about equal
   key counts (again whole buckets);
4. a stable partition of the slice by the top digit (one scatter pass of the radix sort,
   ``rs_plan_partition_totals``: given the step-2 counts it is the one-sweep pass, one key read),
   overlapped with the host's wait for the counts: every (peer, group) send segment is now one
   contiguous range of buckets;
5. G exchange rounds, round g an asynchronous all-to-all (RCCL: each rank sends to all peers at
   once, over all 7 xGMI links of a rank) of every rank's group-g buckets, keys and values.  The
   receiver lays round g out as [source 0's segment, source 1's, ...] in its group-g region,
   which is therefore complete once round g lands: it holds every key of those buckets,
   equal keys in (source rank, input position) order = global input order;
6. as soon as round g has landed, the group-g region is sorted locally (stable LSD, the same
   plan), while rounds g+1.. are still on the wire: the local sort hides under the exchange,
   and only the last group's sort is exposed.  Groups hold increasing buckets, so the regions
   concatenated are rank r's part of the global stable order.

Stability: the partition is stable, segments are placed in source-rank order, the local sort
is stable, and a bucket never spans two groups or two ranks.

The local compute is injected (`LocalOps`): the product uses :class:`HipLocalOps` (librsort);
the CPU gloo tests inject an oracle-backed implementation to exercise the orchestration.  gloo
has no list all-to-all, so there (and only there) a round's send segments are gathered into one
staging buffer for ``all_to_all_single``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Protocol


class LocalOps(Protocol):
    def histogram(self, keys, shift: int, bits: int):
        """-> hist[2^bits] int32 tensor on the keys' device (top-digit counts of keys)."""

    def partition(self, keys, values, shift: int, bits: int, out_keys=None, out_values=None,
                  totals=None):
        """Stable partition by (key >> shift) & (2^bits - 1) -> (keys_out, values_out); written
        into out_keys / out_values when given.  totals (optional): histogram() of the same keys,
        which lets the pass skip its own digit count."""

    def sort(self, keys, values, n: int) -> None:
        """Stable in-place sort of keys[:n] (and values[:n]) by the full 32-bit key."""

    def empty(self, n: int, like):
        """Uninitialised buffer of n 32-bit words on like's device."""


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
    G = max(1, int(chunks))
    shift = 32 - bits
    hist = ops.histogram(keys, shift, bits)                     # [2^bits]
    gathered = [torch.empty_like(hist) for _ in range(world)]
    dist.all_gather(gathered, hist, group=group)
    sk = ops.empty(n_local, keys)
    sv = None if values is None else ops.empty(n_local, values)

    def partition():
        if n_local:
            ops.partition(keys, values, shift, bits, sk, sv, totals=hist)

    if keys.is_cuda:
        # the counts travel to the host while the slice is partitioned (the partition needs no
        # bucket ownership): copy, mark, enqueue the partition, then wait for the mark only
        hcpu = torch.empty((world,) + tuple(hist.shape), dtype=hist.dtype, pin_memory=True)
        hcpu.copy_(torch.stack(gathered), non_blocking=True)
        ready = torch.cuda.Event()
        ready.record()
        partition()
        ready.synchronize()
        hist_all = hcpu.tolist()
    else:
        hist_all = torch.stack(gathered).tolist()
        partition()
    bounds = bucket_owners(hist_all, world)
    cuts = bucket_groups(hist_all, bounds, G)
    plan = group_plan(hist_all, cuts, rank, world)
    n_recv = plan.base[G]
    rk = ops.empty(n_recv, keys)
    rv = None if values is None else ops.empty(n_recv, values)
    list_a2a = dist.get_backend(group) != "gloo"
    rounds = []
    for g in range(G):
        works = []
        for src, dst in ((sk, rk), (sv, rv)):
            if src is None:
                continue
            ins = [src[a:b] for a, b in plan.send[g]]
            region = dst[plan.base[g]:plan.base[g + 1]]
            if list_a2a:
                outs = [dst[plan.off[g][s]:plan.off[g][s] + plan.recv[g][s]] for s in range(world)]
                # this rank's own segment is a local device copy (RCCL moves a self segment
                # through a few channels at ~0.3 TB/s: 0.8 ms per 256 MiB, measured)
                outs[rank].copy_(ins[rank])
                if world > 1:
                    ins[rank], outs[rank] = ins[rank][:0], outs[rank][:0]
                    works.append(dist.all_to_all(outs, ins, group=group, async_op=True))
            else:
                dist.all_to_all_single(region, torch.cat(ins), output_split_sizes=plan.recv[g],
                                       input_split_sizes=[b - a for a, b in plan.send[g]],
                                       group=group)
        rounds.append(works)
    # round g's local sort waits for round g only (the stream waits, not the host); later rounds
    # keep moving on RCCL's stream meanwhile
    for g in range(G):
        for w in rounds[g]:
            w.wait()
        a, b = plan.base[g], plan.base[g + 1]
        if b > a:
            ops.sort(rk[a:b], None if rv is None else rv[a:b], b - a)
    return ExchangeResult(rk, rv, n_recv,
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

    def partition(self, keys, values, shift: int, bits: int, out_keys=None, out_values=None,
                  totals=None):
        import torch
        n = keys.numel()
        sk = torch.empty_like(keys) if out_keys is None else out_keys
        sv = None if values is None else (torch.empty_like(values) if out_values is None else out_values)
        if self.part_plan is None or self.part_plan.capacity < n:
            from .ops import SortPlan
            if self.part_plan is not None:
                self.part_plan.destroy()
            self.part_plan = SortPlan(self.device, max(n, 1), self.has_values, 32, self.radix_bits)
        if totals is not None:
            self.part_plan.partition_totals(keys, values, sk, sv, n, shift, bits, totals)
        else:
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
