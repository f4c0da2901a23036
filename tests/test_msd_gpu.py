"""GPU: the hybrid MSD path (rsort.hip enqueue_sort_msd; rs_kernels.hpp "hybrid MSD path") —
separate key / value arrays and interleaved records (RadixSortTextureKernel, sorted in place) of
>= 12M keys: top-byte pass, 16-bit bucket histogram, segmented
next-byte pass, in-LDS bucket sort — skewed keys whose 16-bit buckets are over the tile (split, see
test_split_gpu.py; with the split off, the device-side fallback to the LSD passes).
Parity is the same contract as every other path: the stable sort of the input, bit-exact
against the oracle (values = input index, so stability is checked too)."""
import numpy as np
import pytest
import torch

import oracle as O
from radix_sort_amd import RadixSortKernel, ops
from radix_sort_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _keys(n, kind, seed):
    k = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(k, seed)
    if kind == "top0":          # one top-byte bucket: the device picks the LSD passes
        k &= 0x00FFFFFF
    elif kind == "low0":        # (top, 0) 16-bit buckets of n/256 keys: LSD on R1
        k &= -16777216
    elif kind == "dups":        # 2^20 distinct keys spread over the key space
        k.remainder_(1 << 20)
        k.mul_(4093)
    elif kind == "few_big":     # a few 16-bit buckets just over the population-sized tile
        k[:12000] = 0x12345678
        k[12000:21000] = 0x7FFF0000
    elif kind == "wide":        # 2560 populated 16-bit buckets spread over every top byte (n / 2560
        # records each: all over the population-sized tile, listed for k_bucket_sort_wide)
        u = k.long() & 0xFFFFFFFF
        k.copy_(((((u >> 16) % 2560) * 25) << 16 | (u & 0xFFFF)).to(torch.int32))
    return k


def _sort_and_check(n, kind, seed=5, copy=False, rank=None, plan_debug=None):
    if rank and plan_debug is not None:
        plan_debug(rank=rank)
    k = _keys(n, kind, seed)
    v = torch.arange(n, dtype=torch.int32, device=DEV)
    kin = k.clone()
    kern = RadixSortKernel(keys=k, values=v, count=n, bit_count=32, local_shuffle=True)
    kern.set_profiling(True)
    if copy:
        from radix_sort_amd.ops import SortPlan
        plan = SortPlan(0, n, True)
        ok_, ov_ = torch.empty_like(k), torch.empty_like(v)
        plan.sort_copy(kin, v, ok_, ov_, n)
        torch.cuda.synchronize()
        plan.check()
        gk, gv = ok_, ov_
        path = plan.last_path()
        plan.destroy()
    else:
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        gk, gv = k, v
        path = kern.last_path()
    times = kern.kernel_times()
    times["path"] = path     # the device's choice (rs_plan_last_path)
    ek, ev = O.stable_sort_masked_c(kin.cpu().numpy().view(np.uint32), np.arange(n, dtype=np.uint32), 32)
    assert np.array_equal(gk.cpu().numpy().view(np.uint32), ek)
    assert np.array_equal(gv.cpu().numpy().view(np.uint32), ev)
    kern.destroy()
    return times


@pytest.mark.parametrize("n", [(12 << 20) + 1, 1 << 24, (1 << 25) + 12345])
def test_msd_uniform_matches_oracle(n):
    t = _sort_and_check(n, "uniform")
    assert t["bucket"]["ms"] > 0.05 and t["bucket"]["launches"] == 1   # the bucket pass ran (one timed span)


@pytest.mark.parametrize("kind", ["top0", "low0"])
def test_msd_device_fallbacks(kind, plan_debug):
    t = _sort_and_check(1 << 24, kind)
    assert t["path"] == "hybrid"            # the over-full buckets were split, no LSD pass ran
    plan_debug(split=0)
    t = _sort_and_check(1 << 24, kind)
    # the split off: the LSD fallback ran (its passes carry the time), the bucket pass gated off
    assert t["path"] == "hybrid_fallback"   # the device chose the LSD passes


@pytest.mark.parametrize("kind", ["dups", "few_big"])
def test_msd_duplicates_and_overflow_buckets(kind):
    _sort_and_check(1 << 24, kind)


@pytest.mark.parametrize("n", [(1 << 25) + 3, (1 << 26) - 5])
def test_msd_wide_buckets_match_oracle(n, plan_debug):
    """16-bit buckets of 13K-26K records (over every population-sized tile, under the wide kernel's
    34816): every populated bucket is listed and sorted by k_bucket_sort_wide (1024 threads, the
    positions through LDS, the values gathered after), bit-exact against the oracle; separate arrays,
    in place and out of place, both rank modes; and the texture layout (records in place)."""
    t = _sort_and_check(n, "wide")
    assert t["path"] == "hybrid"      # the hybrid path ran, not the LSD fallback
    _sort_and_check(n, "wide", copy=True)
    _sort_and_check(n, "wide", rank="ballot", plan_debug=plan_debug)


def test_msd_records_wide_buckets():
    t = _sort_tex_and_check((1 << 25) + 9, "wide")
    assert t["path"] == "hybrid"


def test_msd_out_of_place_and_ballot_ranking(plan_debug):
    _sort_and_check((1 << 24) + 3, "uniform", copy=True)
    _sort_and_check(1 << 24, "dups", rank="ballot", plan_debug=plan_debug)


def test_msd_path_off_by_debug(plan_debug):
    plan_debug(msd=0)
    t = _sort_and_check(1 << 24, "uniform")
    assert t["bucket"]["launches"] == 0 and t["fallback"]["launches"] == 0


def test_msd_repeated_sorts_on_one_plan():
    n = 1 << 24
    k = _keys(n, "uniform", 9)
    v = torch.arange(n, dtype=torch.int32, device=DEV)
    kern = RadixSortKernel(keys=k, values=v, count=n)
    for seed in (11, 12, 13):
        ops.fill_random_u32(k, seed)
        v.copy_(torch.arange(n, dtype=torch.int32, device=DEV))
        kin = k.clone()
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        assert ops.is_sorted(k) and torch.equal(kin[v.long()], k)
    kern.destroy()


def _sort_tex_and_check(n, kind, seed=7):
    """The texture layout (records in place: R2 is the caller's buffer)."""
    from radix_sort_amd import RadixSortTextureKernel
    k = _keys(n, kind, seed)
    rec = torch.empty((n, 2), dtype=torch.int32, device=DEV)
    rec[:, 0] = k
    rec[:, 1] = torch.arange(n, dtype=torch.int32, device=DEV)
    kern = RadixSortTextureKernel(texture=rec, count=n)
    kern.set_profiling(True)
    kern.dispatch()
    torch.cuda.synchronize()
    kern.check()
    times = kern.kernel_times()
    times["path"] = kern.last_path()
    ek, ev = O.stable_sort_masked_c(k.cpu().numpy().view(np.uint32), np.arange(n, dtype=np.uint32), 32)
    got = rec.cpu().numpy().view(np.uint32)
    assert np.array_equal(got[:, 0], ek)
    assert np.array_equal(got[:, 1], ev)
    kern.destroy()
    return times


@pytest.mark.parametrize("n", [(12 << 20) + 1, (1 << 24) + 7])
def test_msd_records_uniform_matches_oracle(n):
    t = _sort_tex_and_check(n, "uniform")
    assert t["bucket"]["ms"] > 0.05 and t["path"] == "hybrid"


@pytest.mark.parametrize("kind", ["top0", "low0", "few_big", "dups"])
def test_msd_records_fallbacks_and_overflow(kind):
    t = _sort_tex_and_check((1 << 24) + 1, kind)
    assert t["path"] == "hybrid"            # over-full buckets split: no LSD fallback


def _records_sort(keys_u32, key_range=None, profile=False):
    """SortPlan.sort_records (records in, arrays out) of (key, index) records."""
    from radix_sort_amd.ops import SortPlan
    n = keys_u32.size
    k = torch.from_numpy(keys_u32.view(np.int32)).to(DEV)
    rec = torch.empty((n, 2), dtype=torch.int32, device=DEV)
    rec[:, 0] = k
    rec[:, 1] = torch.arange(n, dtype=torch.int32, device=DEV)
    rec = rec.view(torch.int64).view(-1)
    plan = SortPlan(0, n, True)
    plan.set_profiling(True)
    ok_, ov_ = torch.empty_like(k), torch.empty_like(k)
    plan.sort_records(rec, ok_, ov_, n, key_range=key_range)
    torch.cuda.synchronize()
    plan.check()
    times = plan.kernel_times()
    times["path"] = plan.last_path()
    plan.destroy()
    ek, ev = O.stable_sort_masked_c(keys_u32, np.arange(n, dtype=np.uint32), 32)
    assert np.array_equal(ok_.cpu().numpy().view(np.uint32), ek)
    assert np.array_equal(ov_.cpu().numpy().view(np.uint32), ev)
    return times


def test_msd_records_to_arrays_full_range():
    # rs_plan_sort_records (the group sorts' records -> arrays form) takes the MSD path itself
    u = O.gen_u32(21, (1 << 24) + 3)
    t = _records_sort(u)
    assert t["bucket"]["ms"] > 0.05 and t["path"] == "hybrid"


@pytest.mark.parametrize("lo_hi", [(0x20000000, 0x27FFFFFF),      # 8 aligned top-byte buckets (27 bits)
                                   (0x1E000000, 0x25FFFFFF),      # 8 unaligned buckets (key - lo: 27 bits)
                                   (0x12345678, 0x1234F677),      # a 16-bit-wide range
                                   (0x00000000, 0xFFFFFFFF)])
def test_msd_records_key_range(lo_hi):
    lo, hi = lo_hi
    u = O.gen_u32(22, 1 << 24).astype(np.uint64)
    keys = (np.uint64(lo) + u % np.uint64(hi - lo + 1)).astype(np.uint32)
    keys[:5] = lo                      # both ends of the range present
    keys[5:9] = hi
    t = _records_sort(keys, key_range=(lo, hi))
    if hi - lo >= (1 << 24):           # populated 16-bit buckets: the MSD path ran
        assert t["bucket"]["ms"] > 0.05 and t["path"] == "hybrid"


@pytest.mark.parametrize("outside", ["below", "above"])
def test_msd_records_key_outside_range_falls_back(outside):
    lo, hi = 0x40000000, 0x47FFFFFF
    u = O.gen_u32(23, 1 << 24)
    keys = (np.uint32(lo) + (u & np.uint32(0x07FFFFFF))).astype(np.uint32)
    keys[12345] = lo - 1 if outside == "below" else hi + 1     # the hint is wrong for one key
    t = _records_sort(keys, key_range=(lo, hi))
    assert t["path"] == "hybrid_fallback"   # the 32-bit LSD passes ran


def test_msd_group_regions_use_key_range():
    # virtual ranks with one exchange round: every rank's region (>= 12M records) is sorted with
    # its buckets' key range (rs_plan_sort_records_range) - parity against the oracle
    from radix_sort_amd import RadixSortGroup
    counts = [13 << 20, (13 << 20) + 11]
    host_k = [O.gen_u32(30 + r, c) for r, c in enumerate(counts)]
    starts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    host_v = [np.arange(starts[r], starts[r + 1], dtype=np.uint32) for r in range(2)]
    g = RadixSortGroup([0, 0], capacity=max(counts), has_values=True, transport="copy", rounds=1)
    try:
        out = g.sort([torch.from_numpy(k.view(np.int32)).to(DEV) for k in host_k],
                     [torch.from_numpy(v.view(np.int32)).to(DEV) for v in host_v])
        ek, ev = O.stable_sort_masked_c(np.concatenate(host_k), np.concatenate(host_v), 32)
        assert np.array_equal(np.concatenate([o[0].cpu().numpy().view(np.uint32) for o in out]), ek)
        assert np.array_equal(np.concatenate([o[1].cpu().numpy().view(np.uint32) for o in out]), ev)
    finally:
        g.destroy()


# ---- keys only (BASELINE config2's shape): R1 = the plan's key copy, R2 = the caller's keys ----

def _sort_keys_and_check(n, kind, seed=21, copy=False, count=None):
    """Keys-only hybrid MSD path (>= 16M keys: the histogram rows live in the plan's key copy);
    `count` < n leaves the tail untouched.  Expected: the oracle's stable sort of the keys."""
    count = n if count is None else count
    k = _keys(n, kind, seed)
    kin = k.clone()
    kern = RadixSortKernel(keys=k, count=count, bit_count=32)
    kern.set_profiling(True)
    if copy:
        from radix_sort_amd.ops import SortPlan
        plan = SortPlan(0, count, False)
        out = torch.full_like(k, -1)
        plan.sort_copy(kin, None, out, None, count)
        torch.cuda.synchronize()
        plan.check()
        got = out
        path = plan.last_path()
        plan.destroy()
    else:
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        got = k
        path = kern.last_path()
    times = kern.kernel_times()
    times["path"] = path
    src = kin.cpu().numpy().view(np.uint32)
    ek, _ = O.stable_sort_masked_c(src[:count].copy(), np.arange(count, dtype=np.uint32), 32)
    g = got.cpu().numpy().view(np.uint32)
    assert np.array_equal(g[:count], ek)
    if not copy:
        assert np.array_equal(g[count:], src[count:])
    kern.destroy()
    return times


@pytest.mark.parametrize("n", [(1 << 24) + 4096, (1 << 25) + 12345, 1 << 26])
def test_msd_keys_uniform_matches_oracle(n):
    t = _sort_keys_and_check(n, "uniform")
    # the MSD path ran: two one-sweep passes and the bucket pass; the gated LSD launches are short
    assert t["bucket"]["launches"] == 1 and t["scatter"]["launches"] == 2
    assert t["path"] == "hybrid"


@pytest.mark.parametrize("kind", ["top0", "low0"])
def test_msd_keys_device_fallbacks(kind, plan_debug):
    t = _sort_keys_and_check((1 << 24) + 4096, kind)
    assert t["path"] == "hybrid"            # over-full buckets split
    plan_debug(split=0)
    t = _sort_keys_and_check((1 << 24) + 4096, kind)
    assert t["path"] == "hybrid_fallback"   # the split off: the device chose the LSD passes


@pytest.mark.parametrize("kind", ["dups", "few_big"])
def test_msd_keys_duplicates_and_overflow_buckets(kind):
    _sort_keys_and_check((1 << 24) + 4096, kind)


def test_msd_keys_out_of_place_partial_count_and_ballot(plan_debug):
    _sort_keys_and_check((1 << 24) + 4099, "uniform", copy=True)
    _sort_keys_and_check((1 << 25) + 3, "uniform", count=(1 << 24) + 5000)
    plan_debug(rank="ballot")
    _sort_keys_and_check((1 << 24) + 4096, "dups")


@pytest.mark.parametrize("n", [(12 << 20) + 9, 1 << 24])
def test_msd_keys_below_row_capacity_keeps_lsd(n):
    # the 256 histogram rows of 65536 counts and their 256 flag words do not fit the key copy
    # (n < 256 * 65537 on a 256-CU device): the histogram-path LSD sort
    t = _sort_keys_and_check(n, "uniform")
    assert t["bucket"]["launches"] == 0 and t["fallback"]["launches"] == 0


@pytest.mark.parametrize("cfg", ["0", "2"])
def test_msd_keys_pass_tile_configs(plan_debug, cfg):
    # the other pass tiles: 1024 x 16 (16K keys) and 1024 x 32 (32K keys), instead of 512 x 32
    plan_debug(msd_keys_cfg=int(cfg))
    t = _sort_keys_and_check((1 << 25) + 77, "uniform")
    assert t["scatter"]["launches"] == 2
    _sort_keys_and_check((1 << 24) + 4096, "few_big")


@pytest.mark.parametrize("n,dbg", [((1 << 27) + 5, {}),                                  # 2K-key buckets
                                   ((1 << 25) + 77, {"kbucket_wave": 0})])
def test_msd_keys_workgroup_bucket_kernel(plan_debug, n, dbg):
    # buckets over the wave kernel's 64 x 18 keys (or the wave kernel off): one workgroup per
    # bucket, in place
    plan_debug(**dbg)
    t = _sort_keys_and_check(n, "uniform")
    assert t["bucket"]["launches"] == 1 and t["scatter"]["launches"] == 2


def _chk_keys(kind, n):
    u = O.gen_u32(61, n)
    if kind == "uniform":
        return u
    if kind == "sorted":
        return np.sort(u)
    if kind == "last_pair":            # sorted but the last pair (the reference's Q1 blind spot)
        k = np.sort(u)
        k[-2], k[-1] = k[-1], k[-2]
        return k
    if kind == "reverse":
        return np.sort(u)[::-1].copy()
    if kind == "f32_nearly":           # config 4's input shape: over-full buckets, split
        import bench
        return bench.nearly_sorted_f32_bits(n, 4)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["uniform", "sorted", "last_pair", "reverse", "f32_nearly"])
def test_msd_check_order(kind):
    """check_order on the hybrid path: the input's order check rides on the 16-bit histogram read;
    an input in order gates every later launch off (the reference's early exit, CheckSort.ts:138-145)
    and comes back untouched; nearly-sorted input (a swapped last pair, config 4's f32 keys) takes
    the presorted path (test_presorted_gpu.py); otherwise the hybrid path (skewed keys: with the
    bucket split) sorts it - separate arrays, keys only, records."""
    from radix_sort_amd import RadixSortTextureKernel
    n = (1 << 25) + 3
    keys = _chk_keys(kind, n)
    vals = np.arange(n, dtype=np.uint32)
    ek, ev = O.stable_sort_masked_c(keys, vals, 32)
    kt = torch.from_numpy(keys.view(np.int32).copy()).to(DEV)
    vt = torch.from_numpy(vals.view(np.int32).copy()).to(DEV)
    kern = RadixSortKernel(keys=kt, values=vt, count=n, check_order=True)
    kern.set_profiling(True)
    kern.dispatch()
    torch.cuda.synchronize()
    kern.check()
    t = kern.kernel_times()
    path = kern.last_path()
    assert np.array_equal(kt.cpu().numpy().view(np.uint32), ek)
    assert np.array_equal(vt.cpu().numpy().view(np.uint32), ev)
    # the hybrid path's launches; the only order-check launch is the presorted path's order scan
    # (k_ns_mark, timed as "check"): no separate k_check pass
    assert t["bucket"]["launches"] >= 1 and t["check"]["launches"] == 1
    if kind in ("uniform", "reverse"):
        assert path == "hybrid"
    if kind in ("last_pair", "f32_nearly"):
        assert path == "presorted"
    if kind == "sorted":                  # everything after the read gated off
        assert path == "in_order"
    kern.destroy()
    # keys only, in place
    kt = torch.from_numpy(keys.view(np.int32).copy()).to(DEV)
    kern = RadixSortKernel(keys=kt, count=n, check_order=True)
    kern.dispatch()
    torch.cuda.synchronize()
    kern.check()
    assert np.array_equal(kt.cpu().numpy().view(np.uint32), ek), "keys only"
    kern.destroy()
    # records in place (RadixSortTextureKernel)
    rt = torch.from_numpy(np.stack([keys, vals], axis=-1).reshape(-1).view(np.int32).copy()).to(DEV).view(-1, 2)
    kern = RadixSortTextureKernel(texture=rt, count=n, check_order=True)
    kern.dispatch()
    torch.cuda.synchronize()
    kern.check()
    out = rt.cpu().numpy().view(np.uint32).reshape(-1, 2)
    assert np.array_equal(out[:, 0], ek) and np.array_equal(out[:, 1], ev), "records"
    kern.destroy()
