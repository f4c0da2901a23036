"""Multi-GPU sort: one process per GPU, one bucket exchange at the top digit.

The reference has no multi-device path; this is the build's sharding of the
same sort for inputs spread over the GPUs of one node (BASELINE config 5):

1. rank r holds a contiguous slice of the global input;
2. a stable local partition by the top ``bits`` key bits (one scatter pass of the radix sort,
   ``rs_plan_partition``) also yields the 2^bits bucket histogram;
3. ``all_gather`` of the histograms (RCCL over xGMI; a few KB);
4. every rank computes the same bucket -> rank assignment on whole-bucket boundaries (equal keys
   never split), balancing the global counts;
5. ``all_to_all_single`` of keys, then values (RCCL all-to-all: every rank sends to all peers at
   once, which uses all 7 xGMI links of a rank concurrently);
6. the receive buffer is the rank-ordered concatenation of stable segments; a local stable
   LSD sort of it is rank r's part of the global stable order.

Stability: ties keep input order because the partition is stable, segments arrive ordered by
source rank (= global input order), and the local sort is stable.

The local compute is injected (`LocalOps`): the product uses :class:`HipLocalOps` (librsort);
the CPU gloo tests inject an oracle-backed implementation to exercise the orchestration.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Protocol


class LocalOps(Protocol):
    def partition(self, keys, values, shift: int, bits: int):
        """-> (keys_out, values_out, hist[2^bits] int32 tensor on the keys' device)."""

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


@dataclass
class ExchangeResult:
    keys: object
    values: object
    n: int
    send_sizes: list
    recv_sizes: list


def distributed_sort(keys, values, ops: LocalOps, group=None, bits: int = 8) -> ExchangeResult:
    """Sort the global array whose slice on this rank is (keys, values); returns this rank's
    slice of the global stable sorted order (rank-ordered concatenation)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_local = keys.numel()
    sk, sv, hist = ops.partition(keys, values, 32 - bits, bits)
    gathered = [torch.empty_like(hist) for _ in range(world)]
    dist.all_gather(gathered, hist, group=group)
    hist_all = torch.stack(gathered).cpu().tolist()       # world x 2^bits, a few KB
    bounds = bucket_owners(hist_all, world)
    send, recv = split_sizes(hist_all, bounds, rank, world)
    assert sum(send) == n_local
    n_recv = sum(recv)
    rk = ops.empty(n_recv, keys)
    dist.all_to_all_single(rk, sk, output_split_sizes=recv, input_split_sizes=send, group=group)
    rv = None
    if values is not None:
        rv = ops.empty(n_recv, values)
        dist.all_to_all_single(rv, sv, output_split_sizes=recv, input_split_sizes=send,
                               group=group)
    ops.sort(rk, rv, n_recv)
    return ExchangeResult(rk, rv, n_recv, send, recv)


class HipLocalOps:
    """librsort-backed local steps (the product path)."""

    def __init__(self, device: int, capacity: int, has_values: bool, radix_bits: int = 0):
        from .ops import SortPlan
        self.device = device
        self.has_values = has_values
        self.radix_bits = radix_bits
        self.plan = SortPlan(device, capacity, has_values, 32, radix_bits)
        self.capacity = capacity
        self._send = None
        self._hist = None

    def empty(self, n: int, like):
        import torch
        return torch.empty(n, dtype=like.dtype, device=like.device)

    def partition(self, keys, values, shift: int, bits: int):
        import torch
        n = keys.numel()
        if self._send is None or self._send[0].numel() < n:
            self._send = (torch.empty_like(keys), None if values is None else torch.empty_like(values))
            self._hist = torch.empty(1 << bits, dtype=torch.int32, device=keys.device)
        sk = self._send[0][:n]
        sv = None if values is None else self._send[1][:n]
        self.plan.partition(keys, values, sk, sv, n, shift, bits, self._hist)
        return sk, sv, self._hist[: 1 << bits]

    def sort(self, keys, values, n: int) -> None:
        if n > self.capacity:
            from .ops import SortPlan
            self.plan.destroy()
            self.capacity = int(n * 1.125)
            self.plan = SortPlan(self.device, self.capacity, self.has_values, 32, self.radix_bits)
        self.plan.sort(keys, values, n)
