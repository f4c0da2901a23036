"""rs_plan_sort_region (a multi-GPU receiver's local sort) at bucket populations that pick each
large-bucket kernel: ~7K records per 16-bit bucket (256 x 34 tiles), ~12K (1024 x 17) and ~20K
(the wide kernel over every bucket).  Every region also holds an empty bucket, one-record and
two-record buckets and one bucket near the largest tile, compared word for word with the oracle's
stable sort."""
import numpy as np
import pytest
import torch

import oracle as O
from radix_sort_amd.ops import SortPlan

WIDE_CAP = 1024 * 34


def _region(mean: int, top_lo: int, ntop: int, seed: int):
    rng = np.random.default_rng(seed)
    nb = ntop * 256
    counts = rng.integers(int(mean * 0.9), int(mean * 1.1) + 1, size=nb)
    counts[3], counts[4], counts[5] = 1, 0, 2
    counts[7] = WIDE_CAP - 17            # one bucket over every population-sized tile
    counts[nb - 1] = 1                   # the region's last bucket: one record
    buckets = (top_lo << 8) + np.repeat(np.arange(nb, dtype=np.uint32), counts)
    low = rng.integers(0, 1 << 16, size=buckets.size, dtype=np.uint32)
    low[: buckets.size // 3] &= np.uint32(0x00FF)   # many duplicates: stability matters
    keys = (buckets.astype(np.uint32) << np.uint32(16)) | low
    # grouped by top byte (ascending), each top byte's records in arbitrary (input) order
    order = np.lexsort((rng.random(keys.size), keys >> np.uint32(24)))
    keys = keys[order]
    vals = rng.permutation(keys.size).astype(np.uint32)
    hist = np.zeros(65536, dtype=np.int32)
    np.add.at(hist, keys >> np.uint32(16), 1)
    return keys, vals, hist


@pytest.mark.gpu
@pytest.mark.parametrize("mean,top_lo,ntop", [(20000, 0x42, 1), (12000, 0x10, 1), (7000, 0xF0, 2)])
def test_region_large_buckets_with_tiny_ones(mean, top_lo, ntop):
    keys, vals, hist = _region(mean, top_lo, ntop, seed=mean + ntop)
    n = keys.size
    rec = keys.astype(np.uint64) | (vals.astype(np.uint64) << np.uint64(32))
    rt = torch.from_numpy(rec.view(np.int64)).cuda()
    ht = torch.from_numpy(hist).cuda()
    ok = torch.empty(n, dtype=torch.int32, device="cuda")
    ov = torch.empty(n, dtype=torch.int32, device="cuda")
    plan = SortPlan(0, max(n, 13 << 20), True)
    try:
        plan.set_profiling(True)
        plan.sort_region(rt, ok, ov, n, ht, top_lo, top_lo + ntop)
        plan.check()
        assert plan.kernel_times()["bucket"]["launches"] > 0
        assert plan.last_path() == "hybrid"
    finally:
        plan.destroy()
    ek, ev = O.stable_sort_masked(keys, vals, 32)
    assert (ok.cpu().numpy().view(np.uint32) == ek).all()
    assert (ov.cpu().numpy().view(np.uint32) == ev).all()


# ---- buckets at high addresses (round 6) --------------------------------------------------------
# Round 5's fault: load_bucket rebuilt a bucket's base address from two readfirstlane halves and the
# low half's bit 31 sign-extended over the high half - wrong only when the bucket's address has bit 31
# of its low word set, i.e. only for some placements of the records buffer.  rs_plan_debug.high_half
# places the buffers the bucket kernels read (R2, and the split's R3) at a 2^31 low address word, so
# every tile kind below meets such buckets on every run, whatever the allocator does.
SPARE = (1 << 28) + (1 << 17)   # the shift needs up to 2^31 + 8n bytes of spare plan capacity


@pytest.mark.gpu
@pytest.mark.parametrize("mean,top_lo,ntop,huge", [
    (3900, 0x21, 1, 0),        # 256 x 17 (the config-3 tile; separate arrays: load_bucket)
    (7000, 0xF0, 2, 0),        # 256 x 34
    (12000, 0x10, 1, 0),       # 1024 x 17
    (20000, 0x42, 1, 0),       # the wide kernel over every bucket
    (3900, 0x80, 1, 3),        # a bucket over the widest tile: the split (512 x 34 sub-bucket tiles)
])
def test_region_buckets_at_high_addresses(plan_debug, mean, top_lo, ntop, huge):
    keys, vals, hist = _region(mean, top_lo, ntop, seed=7 * mean + ntop + huge)
    if huge:   # bucket 9 of the region: `huge` times the widest tile, its low bits random
        extra = ((np.uint32((top_lo << 8) + 9) << np.uint32(16)) |
                 np.random.default_rng(5).integers(0, 1 << 16, huge * WIDE_CAP, dtype=np.uint32))
        keys = np.concatenate([keys, extra])
        vals = np.random.default_rng(6).permutation(keys.size).astype(np.uint32)
        order = np.argsort(keys >> np.uint32(24), kind="stable")
        keys, vals = keys[order], vals[order]
        hist = np.zeros(65536, dtype=np.int32)
        np.add.at(hist, keys >> np.uint32(16), 1)
    n = keys.size
    rec = keys.astype(np.uint64) | (vals.astype(np.uint64) << np.uint64(32))
    rt = torch.from_numpy(rec.view(np.int64)).cuda()
    ht = torch.from_numpy(hist).cuda()
    ok = torch.empty(n, dtype=torch.int32, device="cuda")
    ov = torch.empty(n, dtype=torch.int32, device="cuda")
    plan_debug(high_half=1)
    plan = SortPlan(0, 2 * n + SPARE, True)
    try:
        plan.set_profiling(True)
        plan.sort_region(rt, ok, ov, n, ht, top_lo, top_lo + ntop)
        plan.check()
        assert plan.kernel_times()["bucket"]["launches"] > 0
        assert plan.last_path() == "hybrid"
        if huge:
            assert plan.last_split() >= 2
    finally:
        plan.destroy()
    ek, ev = O.stable_sort_masked(keys, vals, 32)
    assert (ok.cpu().numpy().view(np.uint32) == ek).all()
    assert (ov.cpu().numpy().view(np.uint32) == ev).all()


@pytest.mark.gpu
def test_whole_sort_buckets_at_high_addresses(plan_debug):
    """The whole-array hybrid sort (separate arrays) with its R2 - the plan's second records buffer -
    at a 2^31 low address word."""
    n = (16 << 20) + 77
    keys = O.gen_u32_c(21, n)
    vals = np.arange(n, dtype=np.uint32)
    ek, ev = O.stable_sort_masked_c(keys, vals, 32)
    plan_debug(high_half=1)
    kt = torch.from_numpy(keys.view(np.int32).copy()).cuda()
    vt = torch.from_numpy(vals.view(np.int32).copy()).cuda()
    plan = SortPlan(0, 2 * n + SPARE, True)
    try:
        plan.sort(kt, vt, n)
        plan.check()
        assert plan.last_path() == "hybrid"
    finally:
        plan.destroy()
    assert (kt.cpu().numpy().view(np.uint32) == ek).all() and (vt.cpu().numpy().view(np.uint32) == ev).all()


# ---- a table that does not describe the region (round 6) ----------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("split", [1, 0])
def test_region_table_mismatch(plan_debug, split):
    """Counts that do not add up to n: with the bucket split (the default) no LSD fallback is enqueued
    and the plan check reports a device error; with the split off the device sorts the region with
    the LSD passes (the stable sort, as before round 6)."""
    from radix_sort_amd._lib import RS_ERR_DEVICE, RadixSortError
    keys, vals, hist = _region(3900, 0x21, 1, seed=99)
    hist[(0x21 << 8) + 11] += 5           # five records the region does not hold
    n = keys.size
    rec = keys.astype(np.uint64) | (vals.astype(np.uint64) << np.uint64(32))
    rt = torch.from_numpy(rec.view(np.int64)).cuda()
    ht = torch.from_numpy(hist).cuda()
    ok = torch.empty(n, dtype=torch.int32, device="cuda")
    ov = torch.empty(n, dtype=torch.int32, device="cuda")
    plan_debug(split=split)
    plan = SortPlan(0, max(n, 13 << 20), True)
    try:
        plan.sort_region(rt, ok, ov, n, ht, 0x21, 0x22)
        if split:
            with pytest.raises(RadixSortError) as ei:
                plan.check()
            assert ei.value.status == RS_ERR_DEVICE
            return
        plan.check()
    finally:
        plan.destroy()
    ek, ev = O.stable_sort_masked(keys, vals, 32)
    assert (ok.cpu().numpy().view(np.uint32) == ek).all()
    assert (ov.cpu().numpy().view(np.uint32) == ev).all()
