"""Multi-GPU bucket exchange (radix_sort_amd/distributed.py) on CPU with gloo, world size 2.

The local steps are injected: here an oracle-backed LocalOps (test infrastructure), on the GPU
the librsort-backed HipLocalOps.  What is tested is the orchestration: histogram all_gather,
whole-bucket split, all_to_all with uneven splits, rank-ordered concatenation, global stability.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from radix_sort_amd.distributed import (bucket_groups, bucket_owners, distributed_sort, group_plan,
                                        split_sizes)


class OracleLocalOps:
    """Test-only local steps on CPU tensors (int32 views of u32 words, int64 records)."""

    def empty(self, n, like):
        return torch.empty(n, dtype=like.dtype)

    def hist16(self, keys):
        k = keys.numpy().view(np.uint32)
        h = np.bincount(k >> np.uint32(16), minlength=1 << 16).astype(np.int64)
        top = h.reshape(256, 256).sum(axis=1)
        return torch.from_numpy(np.concatenate([h, top]).astype(np.int32))

    def partition(self, keys, values, shift, bits, totals):
        k = keys.numpy().view(np.uint32)
        top = (k >> np.uint32(shift)) & np.uint32((1 << bits) - 1)
        assert (np.bincount(top, minlength=1 << bits) == totals.numpy()).all()
        perm = np.argsort(top, kind="stable")
        if values is None:
            return torch.from_numpy(k[perm].view(np.int32).copy())
        v = values.numpy().view(np.uint32)[perm]
        rec = k[perm].astype(np.uint64) | (v.astype(np.uint64) << np.uint64(32))
        return torch.from_numpy(rec.view(np.int64))

    def sort_region(self, records, keys_out, values_out, hist16, top_lo, top_hi):
        r = records.numpy().view(np.uint64)
        k = (r & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        v = (r >> np.uint64(32)).astype(np.uint32)
        # the region contract the exchange must meet: grouped by top byte in [top_lo, top_hi),
        # ascending, and the table = its 16-bit bucket counts (zero elsewhere)
        top = k >> np.uint32(24)
        assert (np.diff(top.astype(np.int64)) >= 0).all()
        assert k.size == 0 or (top_lo <= int(top[0]) and int(top[-1]) < top_hi)
        assert (np.bincount(k >> np.uint32(16), minlength=1 << 16) == hist16.numpy()).all()
        ok, ov = O.stable_sort_masked(k, v, 32)
        keys_out.numpy().view(np.uint32)[:] = ok
        values_out.numpy().view(np.uint32)[:] = ov

    def sort_copy(self, keys, values, keys_out, values_out):
        k = keys.numpy().view(np.uint32)
        v = None if values is None else values.numpy().view(np.uint32)
        ok, ov = O.stable_sort_masked(k, v, 32)
        keys_out.numpy().view(np.uint32)[:] = ok
        if values_out is not None:
            values_out.numpy().view(np.uint32)[:] = ov

    def sort(self, keys, n):
        k = keys.numpy().view(np.uint32)
        ok, _ = O.stable_sort_masked(k[:n].copy(), None, 32)
        k[:n] = ok


def _keys(kind, n, start):
    u = O.gen_u32(9, n, start=start)
    if kind == "uniform":
        return u
    if kind == "few":             # heavy duplicates: stability across ranks matters
        return u % np.uint32(7) << np.uint32(29)
    if kind == "skewed":          # everything in a handful of top-byte buckets
        return u & np.uint32(0x03FFFFFF)
    if kind == "one_bucket":      # one top-byte bucket: one rank receives everything
        return u & np.uint32(0x00FFFFFF)
    raise ValueError(kind)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_per_rank, kind, q, chunks, kv):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        k = _keys(kind, n_per_rank, rank * n_per_rank)
        v = np.arange(rank * n_per_rank, (rank + 1) * n_per_rank, dtype=np.uint32)
        r = distributed_sort(torch.from_numpy(k.view(np.int32).copy()),
                             torch.from_numpy(v.view(np.int32).copy()) if kv else None,
                             OracleLocalOps(), chunks=chunks)
        q.put((rank, r.keys[: r.n].numpy().view(np.uint32).copy(),
               r.values[: r.n].numpy().view(np.uint32).copy() if kv else None,
               r.send_sizes, r.recv_sizes))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,chunks,kv", [
    ("uniform", 2, 4, True), ("few", 2, 3, True), ("skewed", 2, 1, True), ("uniform", 3, 4, True),
    ("few", 3, 2, True), ("one_bucket", 3, 4, True), ("one_bucket", 2, 2, False),
    ("uniform", 3, 3, False), ("uniform", 1, 4, True), ("few", 1, 2, False)])
def test_gloo_bucket_exchange_is_global_stable_sort(kind, world, chunks, kv):
    """The exchange code RCCL runs (exchange_round: batched point-to-point record messages, the
    own segment copied locally), here over gloo with oracle local steps; world size 1 takes the
    no-exchange path (one out-of-place sort)."""
    n = 20_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, kind, q, chunks, kv))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=120) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    keys = np.concatenate([o[1] for o in outs])
    all_k = np.concatenate([_keys(kind, n, r * n) for r in range(world)])
    ek, ev = O.stable_sort_masked(all_k, np.arange(world * n, dtype=np.uint32), 32)
    assert (keys == ek).all()
    if kv:
        assert (np.concatenate([o[2] for o in outs]) == ev).all()
    # every rank sent exactly its input, received what others sent it
    for r in range(world):
        assert sum(outs[r][3]) == n
        for s_ in range(world):
            assert outs[r][4][s_] == outs[s_][3][r]
    if kind == "one_bucket":      # one rank holds the whole result, the others nothing
        assert sorted(len(o[1]) for o in outs) == [0] * (world - 1) + [world * n]


def test_bucket_owners_balanced_and_whole():
    hist = [[10] * 256, [10] * 256, [5] * 256, [15] * 256]
    b = bucket_owners(hist, 4)
    assert b[0] == 0 and b[-1] == 256 and b == sorted(b)
    totals = [sum(h[i] for h in hist for i in range(b[q], b[q + 1])) for q in range(4)]
    assert max(totals) - min(totals) <= 40     # one bucket of imbalance at most
    send, recv = split_sizes(hist, b, 1, 4)
    assert sum(send) == sum(hist[1])
    # degenerate: one bucket holds everything -> it goes to a single rank
    h2 = [[0] * 256 for _ in range(2)]
    h2[0][7] = 100
    h2[1][7] = 50
    b2 = bucket_owners(h2, 2)
    s0, r0 = split_sizes(h2, b2, 0, 2)
    s1, r1 = split_sizes(h2, b2, 1, 2)
    assert sum(r0) + sum(r1) == 150 and (sum(r0) == 0 or sum(r1) == 0)


def test_group_plan_rounds_are_contiguous_and_byte_major():
    # world 2, 4 buckets, 2 rounds: rank 0 owns buckets [0, 2), rank 1 [2, 4)
    h = [[1, 2, 3, 4], [4, 3, 2, 1]]
    bounds = bucket_owners(h, 2)
    assert bounds == [0, 2, 4]
    cuts = bucket_groups(h, bounds, 2)
    assert cuts == [[0, 1, 2], [2, 3, 4]]
    p = group_plan(h, cuts, 1, 2)
    # rank 1's partitioned slice: bucket 0 at [0, 4), 1 at [4, 7), 2 at [7, 9), 3 at [9, 10);
    # one chunk per (peer, bucket)
    assert p.send == [[(0, 0, 4), (1, 7, 9)], [(0, 4, 7), (1, 9, 10)]]
    # round 0 = bucket 2: source 0's 3 records, then source 1's 2; round 1 = bucket 3: 4, then 1
    assert p.recv == [[(0, 0, 3), (1, 3, 2)], [(0, 5, 4), (1, 9, 1)]]
    assert p.base == [0, 5, 10] and p.cuts == [2, 3, 4]
    # rank 0, two buckets in one round: byte-major, then source
    p0 = group_plan(h, [[0, 2], [2, 4]], 0, 2)
    assert p0.recv == [[(0, 0, 1), (1, 1, 4), (0, 5, 2), (1, 7, 3)]]
    # more rounds than buckets: empty rounds, still whole buckets in order
    c3 = bucket_groups(h, bounds, 4)
    assert all(len(c) == 5 and c == sorted(c) for c in c3)
    assert c3[0][0] == 0 and c3[0][-1] == 2 and c3[1][0] == 2 and c3[1][-1] == 4


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [1, 4])
def test_rccl_world1_hip_local_ops_round_trip(chunks):
    """The product path (HipLocalOps + RCCL calls) on one GPU: world size 1 over nccl."""
    from radix_sort_amd.distributed import HipLocalOps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        n = 3_000_017
        k = O.gen_u32(21, n)
        v = np.arange(n, dtype=np.uint32)
        kt = torch.from_numpy(k.view(np.int32)).cuda()
        vt = torch.from_numpy(v.view(np.int32)).cuda()
        ops = HipLocalOps(0, n, True)
        r = distributed_sort(kt, vt, ops, chunks=chunks)
        torch.cuda.synchronize()
        ops.check()
        ek, ev = O.stable_sort_masked(k, v, 32)
        assert r.n == n
        assert (r.keys.cpu().numpy().view(np.uint32) == ek).all()
        assert (r.values.cpu().numpy().view(np.uint32) == ev).all()
        # keys only: the exchange carries the keys themselves
        kt2 = torch.from_numpy(k.view(np.int32)).cuda()
        ops2 = HipLocalOps(0, n, False)
        r2 = distributed_sort(kt2, None, ops2, chunks=chunks)
        torch.cuda.synchronize()
        ops2.check()
        assert r2.n == n and (r2.keys.cpu().numpy().view(np.uint32) == ek).all()
    finally:
        dist.destroy_process_group()


def _gpu_worker(rank, world, port, n_per_rank, kind, q, chunks, kv):
    """One rank of the product path (HipLocalOps: rs_plan_hist16, rs_plan_partition_records,
    rs_plan_sort_region) at world > 1, every rank on cuda:0; the exchange over gloo moves the
    device buffers through host copies (RCCL would send them directly)."""
    from radix_sort_amd.distributed import HipLocalOps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        k = _keys(kind, n_per_rank, rank * n_per_rank)
        v = np.arange(rank * n_per_rank, (rank + 1) * n_per_rank, dtype=np.uint32)
        kt = torch.from_numpy(k.view(np.int32).copy()).cuda()
        vt = torch.from_numpy(v.view(np.int32).copy()).cuda() if kv else None
        ops = HipLocalOps(0, int(n_per_rank * 1.25), kv)
        for _ in range(2):          # the second sort reuses the plans and the side stream
            r = distributed_sort(kt, vt, ops, chunks=chunks)
        torch.cuda.synchronize()
        ops.check()
        q.put((rank, r.keys[: r.n].cpu().numpy().view(np.uint32).copy(),
               r.values[: r.n].cpu().numpy().view(np.uint32).copy() if kv else None,
               r.send_sizes, r.recv_sizes))
        ops.destroy()
    except BaseException as e:       # report instead of leaving the parent waiting on the queue
        q.put((rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,world,chunks,kv,n", [
    ("uniform", 2, 4, True, 16 << 20), ("few", 2, 2, True, 3_000_017),
    ("skewed", 3, 4, True, 5_000_000), ("uniform", 3, 3, False, 6_000_011),
    ("one_bucket", 2, 4, True, 4_000_000)])
def test_hip_local_ops_multi_rank_on_one_gpu(kind, world, chunks, kv, n):
    """The multi-GPU host (distributed_sort + HipLocalOps) with world > 1 on real kernels: 16-bit
    tables gathered, top-byte partition into records, per-(source, byte) chunks, region sorts of
    the received records; output = the global stable sort (oracle)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, n, kind, q, chunks, kv))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        outs = sorted([q.get(timeout=180) for _ in range(world)], key=lambda x: x[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    for o in outs:
        assert not isinstance(o[1], str), f"rank {o[0]}: {o[1]}"
    for p in procs:
        assert p.exitcode == 0
    keys = np.concatenate([o[1] for o in outs])
    all_k = np.concatenate([_keys(kind, n, r * n) for r in range(world)])
    ek, ev = O.stable_sort_masked(all_k, np.arange(world * n, dtype=np.uint32), 32)
    assert (keys == ek).all()
    if kv:
        assert (np.concatenate([o[2] for o in outs]) == ev).all()
    for r in range(world):
        assert sum(outs[r][3]) == n
        for s_ in range(world):
            assert outs[r][4][s_] == outs[s_][3][r]


@pytest.mark.gpu
def test_rs_hist16_matches_bincount():
    """The sender's 16-bit table (rs_plan_hist16): the bucket counts and the top-byte totals, on
    a sort plan and on a partition-only plan, at sizes that use one row and many rows."""
    from radix_sort_amd import _lib
    from radix_sort_amd.ops import SortPlan
    for n, usage in ((40_000, _lib.RS_USAGE_SORT), (3_000_017, _lib.RS_USAGE_PARTITION),
                     (13_000_001, _lib.RS_USAGE_SORT)):
        k = O.gen_u32(n, n)
        kt = torch.from_numpy(k.view(np.int32)).cuda()
        plan = SortPlan(0, n, True, usage=usage)
        h = torch.empty(_lib.RS_HIST16_WORDS, dtype=torch.int32, device="cuda")
        plan.hist16(kt, n, h)
        exp = np.bincount(k >> np.uint32(16), minlength=1 << 16)
        got = h.cpu().numpy()
        assert (got[:65536] == exp).all() and (got[65536:] == exp.reshape(256, 256).sum(1)).all()
        plan.destroy()


@pytest.mark.gpu
def test_rs_histogram_matches_bincount():
    from radix_sort_amd import ops
    n = 1_000_003
    k = O.gen_u32(33, n)
    kt = torch.from_numpy(k.view(np.int32)).cuda()
    for shift, bits in ((24, 8), (0, 8), (13, 5), (30, 2)):
        h = torch.empty(1 << bits, dtype=torch.int32, device="cuda")
        ops.histogram(kt[1:], n - 1, shift, bits, h)
        exp = np.bincount((k[1:] >> np.uint32(shift)) & np.uint32((1 << bits) - 1), minlength=1 << bits)
        assert (h.cpu().numpy() == exp).all(), (shift, bits)


def test_multi_gpu_breakdown_fields():
    """The N-rank bench line's multi_gpu breakdown (bench.py, distributed.summarize_timelines):
    the layout every rank gathers (timeline_record) and the fields rank 0 derives from it - the
    exchange time E and xGMI GB/s per rank, the slowest rank's local terms, rank edges."""
    from radix_sort_amd import _lib
    from radix_sort_amd.distributed import StepTimeline, summarize_timelines, timeline_record
    G = 4
    # the layout bench.py ships: the library's kernel kinds, then the sender's two terms
    names = list(_lib.KERNEL_NAMES) + ["sender_hist16", "sender_partition"]
    kinds = {"histogram": 0.3, "scan": 0.0, "scatter": 2.0, "check": 0.0, "bucket": 2.06, "fallback": 0.0,
             "split": 0.0, "presorted": 0.0, "sender_hist16": 0.3, "sender_partition": 1.05}
    assert set(names) == set(kinds), "a kernel kind was added: give it a value here"
    tl = StepTimeline()
    tl.bytes_sent, tl.bytes_recv = 7 * 10**8, 7 * 10**8
    empty = timeline_record(tl, G, 10, 20, 1000, [0.0] * len(names), 1.5)   # no GPU marks: zeros
    assert len(empty) == 3 + 2 * G + 6 + len(names)

    def row(t_off, k0, k1, n):
        return ([0.3, 0.35, 1.4] + [1.4 + 0.6 * (g + 1) + t_off for g in range(G)]
                + [2.5 + 0.6 * (g + 1) + t_off for g in range(G)]
                + [7e8, 7e8, k0, k1, n, 2.2] + [kinds[nm] for nm in names])

    s = summarize_timelines([row(0.0, 5, 100, 10), row(0.5, 100, 300, 12), row(0.0, 0, 0, 0)], G, names)
    assert s["ranks"] == 3
    assert s["exchange"]["rounds"] == G
    assert abs(s["exchange"]["E_ms_max"] - 2.9) < 1e-9             # last round landed - partition
    assert len(s["exchange"]["landed_ms_after_partition_max"]) == G
    assert s["exchange"]["xgmi_GBs_per_rank_min"] > 0 and s["exchange"]["exchange_only_ms_max"] == 2.2
    assert s["exchange"]["bytes_off_gpu_per_rank_max"] == 14 * 10**8
    assert set(s["local_ms_max_over_ranks"]) == {"hist16", "table_all_gather", "partition",
                                                 "after_last_round_landed"}
    assert s["kernel_ms_max_over_ranks"]["bucket"] == 2.06
    assert s["recv_keys_min_max"] == [0, 12]
    assert s["rank_edges_sorted"] is True                           # the empty rank is skipped
    s2 = summarize_timelines([row(0.0, 5, 150, 10), row(0.0, 100, 300, 12)], G, names)
    assert s2["rank_edges_sorted"] is False
