"""Multi-GPU sort: one process per GPU, one bucket exchange at the top digit.

The reference has no multi-device path; this is the build's sharding of the
same sort for inputs spread over the GPUs of one node (BASELINE config 5).  The exchange IS the
first pass of the single-GPU hybrid sort (rsort.hip enqueue_sort_msd), split across the ranks, so
a rank moves the bytes of one single-GPU sort of its share: 4 + 16 + 16 + 16 = 52 B/key with
values (round 2 moved 76: an 8-bit histogram, the partition, and then a whole local sort of the
received records with its own histogram read and its own top-byte pass).

1. rank r holds a contiguous slice of the global input;
2. its 16-bit bucket table (``rs_plan_hist16``: one read of the keys; 65536 counts + the 256
   top-byte totals);
3. ``all_gather`` of the tables (RCCL over xGMI; 263 KB per rank); the top-byte totals go to the
   host, where every rank computes the same top byte -> rank ownership on whole-byte boundaries
   (equal keys never split) and splits every rank's bytes into G consecutive rounds of about equal
   key counts;
4. a stable partition of the slice by the top byte (the sort's pass 0, the one-sweep pass fed the
   table's top-byte totals: one read of keys + values), written as 8-byte (key, value) records
   (``rs_plan_partition_records``; keys only: ``rs_plan_partition_totals``), overlapped with the
   host's wait for the totals;
5. G exchange rounds: round g is one batch of point-to-point messages (``batch_isend_irecv``; RCCL
   sends to all peers at once, over all 7 xGMI links of a rank), one message per (source, top
   byte) chunk.  The receiver lays round g out top byte by top byte, each byte's chunks in source
   order: its group-g region is then grouped by top byte, every byte's records in global input
   order - exactly what the hybrid sort's pass 0 would have produced;
6. as soon as round g has landed, the group-g region is sorted locally
   (``rs_plan_sort_region``: the segmented next-byte pass and the in-LDS bucket sort; its 16-bit
   bucket counts are the gathered tables summed over the sources), while rounds g+1.. are still
   on the wire: only the last group's sort is exposed.  Regions hold increasing top bytes, so
   they concatenated are rank r's part of the global stable order.

Stability: the partition is stable, chunks are placed in source-rank order, the local sort is
stable, and a top byte never spans two groups or two ranks.

The local compute is injected (`LocalOps`): the product uses :class:`HipLocalOps` (librsort);
the CPU gloo tests inject an oracle-backed implementation.  The exchange itself
(:func:`exchange_round`: point-to-point messages batched per round, the own chunks copied
locally) is ONE code path for every backend, so the gloo world-2/3 tests run exactly what RCCL
runs on the GPUs.  With values, a message is a run of 8-byte (key, value) records (the partition
writes records, the local sort reads them and writes separate arrays).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Protocol


HIST16_WORDS = 65792     # 65536 bucket counts + 256 top-byte totals (RS_HIST16_WORDS)


class LocalOps(Protocol):
    def hist16(self, keys):
        """-> int32 tensor [HIST16_WORDS] on the keys' device: counts per 16-bit bucket key >> 16,
        then the 256 top-byte totals."""

    def partition(self, keys, values, shift: int, bits: int, totals):
        """Stable partition by (key >> shift) & (2^bits - 1) -> the send buffer: with values, one
        int64 (key, value) record per key (key | value << 32, the interleaved layout: one message
        carries both); keys only, the int32 keys.  totals: the digit totals of the same keys."""

    def sort_region(self, records, keys_out, values_out, hist16, top_lo: int, top_hi: int) -> None:
        """Stable sort of the int64 records (grouped by top byte in [top_lo, top_hi), ascending;
        each group in input order) by their 32-bit key into keys_out / values_out.  hist16: the
        records' counts per 16-bit bucket (65536 int32, zero outside the region's top bytes)."""

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


def split_sizes(hist_all, bounds, rank: int, world: int):
    """(send sizes of this rank to every peer, receive sizes from every peer)."""
    send = [sum(int(hist_all[rank][b]) for b in range(bounds[q], bounds[q + 1]))
            for q in range(world)]
    recv = [sum(int(hist_all[s][b]) for b in range(bounds[rank], bounds[rank + 1]))
            for s in range(world)]
    return send, recv


@dataclass
class GroupPlan:
    send: list   # send[g] = [(peer q, begin, end)]: this rank's chunks in round g, per peer by byte
    recv: list   # recv[g] = [(source s, offset, count)]: where round g's chunks from s land
    base: list   # base[g] = start of round g's region; base[G] = total received
    cuts: list   # cuts[g] = first top byte of this rank's round g; cuts[G] = end


def group_plan(hist_all, cuts, rank: int, world: int) -> GroupPlan:
    """Send chunks, receive offsets and regions of every exchange round.

    hist_all: [world][B] top-byte counts; cuts: bucket_groups().  The partitioned slice holds byte
    t at [start[t], start[t + 1]) (start = exclusive scan of this rank's counts): one chunk per
    (peer, byte).  The receive buffer is round-major, then byte, then source: round g's region is
    complete when round g has landed, grouped by top byte, each byte in global input order."""
    B = len(hist_all[0])
    mine = [int(x) for x in hist_all[rank]]
    start = [0]
    for c in mine:
        start.append(start[-1] + c)
    G = len(cuts[0]) - 1
    send = [[(q, start[t], start[t + 1]) for q in range(world)
             for t in range(cuts[q][g], cuts[q][g + 1]) if mine[t]] for g in range(G)]
    recv, base, pos = [], [], 0
    for g in range(G):
        base.append(pos)
        row = []
        for t in range(cuts[rank][g], cuts[rank][g + 1]):
            for s in range(world):
                c = int(hist_all[s][t])
                if c:
                    row.append((s, pos, c))
                pos += c
        recv.append(row)
    base.append(pos)
    assert B >= 1
    return GroupPlan(send, recv, base, list(cuts[rank]))


@dataclass
class ExchangeResult:
    keys: object
    values: object
    n: int
    send_sizes: list
    recv_sizes: list


class StepTimeline:
    """Where one multi-GPU step's time goes on this rank (GPU events; the diagnostics of the N-rank
    bench line): marks after the 16-bit table, the table all_gather and the
    partition, the moment each exchange round has landed (an event on a watch stream that waits
    for that round's messages only) and the end of each round's region sort; the off-GPU bytes
    this rank sent and received.  `exchange_only`: post the rounds with no region sorts (the
    exchange's own time E, nothing competing)."""

    def __init__(self, exchange_only: bool = False):
        self.exchange_only = exchange_only
        self.marks = []          # (name, torch.cuda.Event)
        self.bytes_sent = 0      # off-rank message bytes (own chunks are local copies)
        self.bytes_recv = 0
        self._watch = None

    def mark(self, name: str, stream=None) -> None:
        import torch
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        self.marks.append((name, ev))

    def landed(self, g: int, works, device) -> None:
        """Event when round g's messages have arrived (waits for those works only)."""
        import torch
        if self._watch is None:
            self._watch = torch.cuda.Stream(device)
        self._watch.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(self._watch):
            for w in works:
                w.wait()
            self.mark(f"landed{g}", self._watch)

    def ms(self) -> dict:
        """{mark: ms since the step's first mark} (synchronises)."""
        if not self.marks:
            return {}
        t0 = self.marks[0][1]
        t0.synchronize()
        out = {}
        for name, ev in self.marks:
            ev.synchronize()
            out[name] = t0.elapsed_time(ev)
        return out


# the per-rank record gathered to rank 0: a fixed layout of floats (all_gather of one tensor)
def timeline_record(tl: StepTimeline, rounds: int, first_key: int, last_key: int, n_recv: int,
                    kernel_ms: list, exchange_only_ms: float) -> list:
    m = tl.ms()
    row = [m.get("hist16", 0.0), m.get("gather", 0.0), m.get("partition", 0.0)]
    row += [m.get(f"landed{g}", 0.0) for g in range(rounds)]
    row += [m.get(f"sorted{g}", 0.0) for g in range(rounds)]
    row += [float(tl.bytes_sent), float(tl.bytes_recv), float(first_key), float(last_key), float(n_recv),
            float(exchange_only_ms)]
    row += [float(x) for x in kernel_ms]
    return row


def summarize_timelines(rows: list, rounds: int, kernel_names) -> dict:
    """The N-rank bench line's breakdown from every rank's timeline_record (pure: CPU-tested).
    Times are ms since each rank's step start; the step's time is its slowest rank's."""
    G = rounds
    per = []
    for r in rows:
        d = {"hist16": r[0], "gather": r[1], "partition": r[2],
             "landed": list(r[3:3 + G]), "sorted": list(r[3 + G:3 + 2 * G])}
        (d["bytes_sent"], d["bytes_recv"], d["first_key"], d["last_key"], d["n_recv"],
         d["exchange_only_ms"]) = r[3 + 2 * G:9 + 2 * G]
        d["kernel_ms"] = dict(zip(kernel_names, r[9 + 2 * G:]))
        per.append(d)

    def mx(f):
        return round(max(f(d) for d in per), 4)

    E = [d["landed"][-1] - d["partition"] for d in per]
    xg = [(d["bytes_sent"] + d["bytes_recv"]) / (e / 1e3) / 1e9 if e > 0 else 0.0 for d, e in zip(per, E)]
    eo = [d["exchange_only_ms"] for d in per]
    xo = [(d["bytes_sent"] + d["bytes_recv"]) / (e / 1e3) / 1e9 if e > 0 else 0.0 for d, e in zip(per, eo)]
    # rank edges of the global order: the last key of every non-empty rank <= the first key of the
    # next non-empty one (keys are the u32 bit patterns, gathered as floats: exact below 2^53)
    nonempty = [d for d in per if d["n_recv"] > 0]
    edges_ok = all(a["last_key"] <= b["first_key"] for a, b in zip(nonempty, nonempty[1:]))
    return {
        "ranks": len(per),
        "step_ms_max_over_ranks": mx(lambda d: d["sorted"][-1] if G else d["partition"]),
        "local_ms_max_over_ranks": {
            "hist16": mx(lambda d: d["hist16"]),
            "table_all_gather": mx(lambda d: d["gather"] - d["hist16"]),
            "partition": mx(lambda d: d["partition"] - d["gather"]),
            "after_last_round_landed": mx(lambda d: d["sorted"][-1] - d["landed"][-1]),
        },
        "exchange": {
            "rounds": G,
            "landed_ms_after_partition_max": [round(max(d["landed"][g] - d["partition"] for d in per), 4)
                                              for g in range(G)],
            "E_ms_max": round(max(E), 4),
            "xgmi_GBs_per_rank_min": round(min(xg), 1),
            "xgmi_GBs_per_rank_max": round(max(xg), 1),
            "exchange_only_ms_max": round(max(eo), 4),
            "exchange_only_xgmi_GBs_per_rank_min": round(min(xo), 1),
            "bytes_off_gpu_per_rank_max": int(max(d["bytes_sent"] + d["bytes_recv"] for d in per)),
        },
        "kernel_ms_max_over_ranks": {k: round(max(d["kernel_ms"][k] for d in per), 4) for k in kernel_names},
        "recv_keys_min_max": [int(min(d["n_recv"] for d in per)), int(max(d["n_recv"] for d in per))],
        "rank_edges_sorted": bool(edges_ok),
    }


def distributed_sort(keys, values, ops: LocalOps, group=None, bits: int = 8,
                     chunks: int = 4, timeline: StepTimeline | None = None) -> ExchangeResult:
    """Sort the global array whose slice on this rank is (keys, values); returns this rank's
    slice of the global stable sorted order (rank-ordered concatenation).  `chunks` = exchange
    rounds (bucket groups per rank), each sorted while the next ones are on the wire.
    `timeline` (GPU only): record where the step's time goes (StepTimeline).

    On the GPU the work runs on a side stream (ordered after the caller's current stream, and
    the caller's stream after it): the legacy default stream would serialise every local sort
    with the in-flight exchange and undo the overlap."""
    import torch

    if keys.is_cuda:
        caller = torch.cuda.current_stream(keys.device)
        side = _side_stream(keys.device)
        side.wait_stream(caller)
        with torch.cuda.stream(side):
            r = _distributed_sort(keys, values, ops, group, bits, chunks, timeline)
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


def _host_staged(t, group) -> bool:
    """gloo moves host memory only: device tensors on a gloo group travel through host copies
    (the GPU tests run the product's HipLocalOps at world > 1 with every rank on one GPU this
    way; RCCL sends device memory directly)."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_gather_tables(h16, world: int, group=None):
    """[world, HIST16_WORDS] = every rank's 16-bit table (all_gather; host-staged on gloo)."""
    import torch
    import torch.distributed as dist
    if _host_staged(h16, group):
        hc = h16.cpu()
        out = [torch.empty_like(hc) for _ in range(world)]
        dist.all_gather(out, hc, group=group)
        return torch.stack(out).to(h16.device)
    out = [torch.empty_like(h16) for _ in range(world)]
    dist.all_gather(out, h16, group=group)
    return torch.stack(out)


def exchange_round(send, recv, plan: GroupPlan, g: int, rank: int, world: int, group=None):
    """Round g of the bucket exchange, the same code on every backend (gloo on CPU, RCCL on the
    GPUs): one point-to-point message per (peer, top byte) chunk, received into the byte's source
    slot of the round-g region; the rank's own chunks are local copies (RCCL moves a self message
    through a few channels at ~0.3 TB/s, measured).  A pair's messages are posted in the same
    (byte) order on both sides, so they match.  Both sides skip empty chunks.  -> the round's works.

    Device tensors on a gloo group (tests: several ranks on one GPU) are staged through host
    copies and the round completes before returning (no works)."""
    import torch.distributed as dist
    mine = [(o, m) for s, o, m in plan.recv[g] if s == rank]
    own = [(a, b) for q, a, b in plan.send[g] if q == rank]
    assert len(mine) == len(own)
    if recv.data_ptr() != send.data_ptr():
        for (o, m), (a, b) in zip(mine, own):
            recv[o:o + m].copy_(send[a:b])
    if _host_staged(send, group):
        sends = [(q, send[a:b].cpu()) for q, a, b in plan.send[g] if q != rank]
        recvs = [(s, o, m, recv.new_empty(m, device="cpu")) for s, o, m in plan.recv[g] if s != rank]
        p2p = [dist.P2POp(dist.isend, t, q, group) for q, t in sends]
        p2p += [dist.P2POp(dist.irecv, t, s, group) for s, _, _, t in recvs]
        for w in (dist.batch_isend_irecv(p2p) if p2p else []):
            w.wait()
        for _, o, m, t in recvs:
            recv[o:o + m].copy_(t)
        return []
    p2p = [dist.P2POp(dist.isend, send[a:b], q, group) for q, a, b in plan.send[g] if q != rank]
    p2p += [dist.P2POp(dist.irecv, recv[o:o + m], s, group) for s, o, m in plan.recv[g] if s != rank]
    return dist.batch_isend_irecv(p2p) if p2p else []


def _distributed_sort(keys, values, ops, group, bits, chunks, timeline=None) -> ExchangeResult:
    import torch
    import torch.distributed as dist

    tl = timeline if (timeline is not None and keys.is_cuda) else None
    if tl is not None:
        tl.mark("start")

    if bits != 8:
        raise ValueError("the exchange digit is the top byte (bits=8): the sort's first MSD pass")
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
    h16 = ops.hist16(keys)                                      # [HIST16_WORDS]
    if tl is not None:
        tl.mark("hist16")
    table = all_gather_tables(h16, world, group)                # [world, HIST16_WORDS]
    if tl is not None:
        tl.mark("gather")
    tops = table[:, 65536:]
    totals = h16[65536:]
    if keys.is_cuda:
        # the top-byte totals travel to the host while the slice is partitioned (the partition
        # needs no ownership): copy, mark, enqueue the partition, then wait for the mark only
        hcpu = torch.empty(tuple(tops.shape), dtype=tops.dtype, pin_memory=True)
        hcpu.copy_(tops, non_blocking=True)
        ready = torch.cuda.Event()
        ready.record()
        send = ops.partition(keys, values, shift, bits, totals)
        if tl is not None:
            tl.mark("partition")
        ready.synchronize()
        hist_all = hcpu.tolist()
    else:
        hist_all = tops.tolist()
        send = ops.partition(keys, values, shift, bits, totals)
    bounds = bucket_owners(hist_all, world)
    cuts = bucket_groups(hist_all, bounds, G)
    plan = group_plan(hist_all, cuts, rank, world)
    n_recv = plan.base[G]
    recv = ops.empty(n_recv, send)
    rounds = [exchange_round(send, recv, plan, g, rank, world, group) for g in range(G)]
    if tl is not None:
        rec = send.element_size()
        tl.bytes_sent = rec * sum(b - a for g in range(G) for q, a, b in plan.send[g] if q != rank)
        tl.bytes_recv = rec * sum(m for g in range(G) for s, _, m in plan.recv[g] if s != rank)
        for g in range(G):
            tl.landed(g, rounds[g], keys.device)
        if tl.exchange_only:
            for g in range(G):
                for w in rounds[g]:
                    w.wait()
            send_sizes, recv_sizes = split_sizes(hist_all, bounds, rank, world)
            return ExchangeResult(recv, None, n_recv, send_sizes, recv_sizes)
    if values is None:
        out_k, out_v, tot16 = recv, None, None
    else:
        out_k, out_v = ops.empty(n_recv, keys), ops.empty(n_recv, values)
        # this rank's regions' 16-bit counts: the tables summed over the sources
        tot16 = table[:, :65536].to(torch.int64).sum(dim=0).to(torch.int32)
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
                t0, t1 = plan.cuts[g], plan.cuts[g + 1]
                reg = torch.zeros_like(tot16)
                reg[t0 << 8:t1 << 8] = tot16[t0 << 8:t1 << 8]
                ops.sort_region(recv[a:b], out_k[a:b], out_v[a:b], reg, t0, t1)
        if tl is not None:
            tl.mark(f"sorted{g}")
    send_sizes, recv_sizes = split_sizes(hist_all, bounds, rank, world)
    return ExchangeResult(out_k, out_v, n_recv, send_sizes, recv_sizes)


class HipLocalOps:
    """librsort-backed local steps (the product path)."""

    def __init__(self, device: int, capacity: int, has_values: bool, radix_bits: int = 0):
        from .ops import SortPlan
        self.device = device
        self.has_values = has_values
        self.radix_bits = radix_bits
        self.plan = SortPlan(device, capacity, has_values, 32, radix_bits)   # the local sorts
        self.part_plan = None     # the sender's table + partition (own plan, RS_USAGE_PARTITION)
        self.capacity = capacity

    def empty(self, n: int, like):
        import torch
        return torch.empty(n, dtype=like.dtype, device=like.device)

    def _part(self, n: int):
        if self.part_plan is None or self.part_plan.capacity < n:
            from . import _lib
            from .ops import SortPlan
            if self.part_plan is not None:
                self.part_plan.destroy()
            self.part_plan = SortPlan(self.device, max(n, 1 << 15), self.has_values, 32,
                                      self.radix_bits, usage=_lib.RS_USAGE_PARTITION)
        return self.part_plan

    def hist16(self, keys):
        import torch
        h = torch.empty(HIST16_WORDS, dtype=torch.int32, device=keys.device)
        self._part(keys.numel()).hist16(keys, keys.numel(), h)
        return h

    def partition(self, keys, values, shift: int, bits: int, totals):
        import torch
        n = keys.numel()
        pp = self._part(n)
        if values is None:
            sk = torch.empty_like(keys)
            pp.partition_totals(keys, None, sk, None, n, shift, bits, totals)
            return sk
        rec = torch.empty(n, dtype=torch.int64, device=keys.device)
        pp.partition_records(keys, values, rec, n, shift, bits, totals)
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

    def sort_region(self, records, keys_out, values_out, hist16, top_lo: int, top_hi: int) -> None:
        n = records.numel()
        self._grow(n)
        self.plan.sort_region(records, keys_out, values_out, n, hist16, top_lo, top_hi)

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
