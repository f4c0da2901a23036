"""GPU: the hybrid path's bucket split (rs_kernels.hpp "splitting over-full buckets"): skewed keys
whose 16-bit buckets exceed the bucket tile - f32 keys in [0, 1) (random and config 4's nearly
sorted shape), every key in one 16-bit bucket, every key in one 24-bit sub-bucket, a few distinct
keys, all keys equal, half uniform + half one bucket - stay on the hybrid path (last_path() ==
"hybrid", last_split() == the levels the data needs) and are bit-exact against the oracle's stable
sort (values = input index: stability checked too), at >= 12M keys, for every layout the path
serves: separate arrays in place and out of place, keys only, records in place (texture), records
-> arrays (rs_plan_sort_records), a multi-GPU receiver's region (rs_plan_sort_region), ballot
ranking, check_order.  With the split off (rs_plan_debug.split = 0) the same inputs take the LSD
fallback, as before."""
import numpy as np
import pytest
import torch

import oracle as O
from radix_sort_amd import RadixSortKernel, RadixSortTextureKernel, ops
from radix_sort_amd.ops import SortPlan

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
N = (1 << 24) + 4099          # >= 12M: the hybrid path (keys only from 16M)

# the split levels each kind needs (level 3: sub-buckets of more than 17408 records)
LEVELS = {"f32_unit": (2, 3), "f32_nearly": (2, 3), "one_bucket": (3,), "one_sub": (3,), "few": (3,),
          "equal": (3,), "half_one_bucket": (3,)}


def _keys_u32(kind: str, n: int, seed: int = 3) -> np.ndarray:
    u = O.gen_u32(seed, n)
    if kind == "f32_unit":            # uniform f32 in [0, 1): half the keys in 128 buckets of ~n/256
        return ((u >> np.uint32(8)).astype(np.float64) * 2.0 ** -24).astype(np.float32).view(np.uint32)
    if kind == "f32_nearly":          # BASELINE config 4's shape
        import bench
        return bench.nearly_sorted_f32_bits(n, 4)
    if kind == "one_bucket":          # every key in one 16-bit bucket: 256 sub-buckets of n / 256
        return np.uint32(0x5A5A0000) | (u & np.uint32(0xFFFF))
    if kind == "one_sub":             # every key in one 24-bit sub-bucket: level 3 sorts them all
        return np.uint32(0x12345600) | (u & np.uint32(0xFF))
    if kind == "few":                 # 5 distinct keys over the whole range
        table = np.array([0x00000000, 0x7FFFFFFF, 0x80000001, 0xDEADBEEF, 0xFFFFFFFF], dtype=np.uint32)
        return table[u % np.uint32(5)]
    if kind == "equal":
        return np.full(n, 0x31415926, dtype=np.uint32)
    if kind == "half_one_bucket":     # half uniform (buckets of ~128 records), half in one bucket
        k = u.copy()
        k[::2] = np.uint32(0xC0DE0000) | (u[::2] & np.uint32(0xFFFF))
        return k
    raise ValueError(kind)


def _expect(keys: np.ndarray):
    return O.stable_sort_masked_c(keys, np.arange(keys.size, dtype=np.uint32), 32)


def _check_split(obj, kind):
    assert obj.last_path() == "hybrid"
    assert obj.last_split() in LEVELS[kind], (kind, obj.last_split())


@pytest.mark.parametrize("kind", list(LEVELS))
def test_split_arrays_in_place(kind):
    keys = _keys_u32(kind, N)
    ek, ev = _expect(keys)
    k = torch.from_numpy(keys.view(np.int32)).to(DEV)
    v = torch.arange(N, dtype=torch.int32, device=DEV)
    kern = RadixSortKernel(keys=k, values=v, count=N)
    try:
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        _check_split(kern, kind)
        assert np.array_equal(k.cpu().numpy().view(np.uint32), ek)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), ev)
    finally:
        kern.destroy()


@pytest.mark.parametrize("kind", ["f32_unit", "one_bucket", "few", "equal"])
def test_split_keys_only(kind):
    keys = _keys_u32(kind, N)
    ek, _ = _expect(keys)
    k = torch.from_numpy(keys.view(np.int32)).to(DEV)
    kern = RadixSortKernel(keys=k, count=N)
    try:
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        _check_split(kern, kind)
        assert np.array_equal(k.cpu().numpy().view(np.uint32), ek)
    finally:
        kern.destroy()


@pytest.mark.parametrize("kind", ["f32_nearly", "one_sub", "half_one_bucket"])
def test_split_records_in_place(kind):
    keys = _keys_u32(kind, N)
    ek, ev = _expect(keys)
    rec = torch.from_numpy(np.stack([keys, np.arange(N, dtype=np.uint32)], axis=-1).view(np.int32).copy()).to(DEV)
    kern = RadixSortTextureKernel(texture=rec, count=N)
    try:
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        _check_split(kern, kind)
        out = rec.cpu().numpy().view(np.uint32).reshape(-1, 2)
        assert np.array_equal(out[:, 0], ek) and np.array_equal(out[:, 1], ev)
    finally:
        kern.destroy()


@pytest.mark.parametrize("kind", ["f32_unit", "few"])
def test_split_out_of_place_and_records_to_arrays(kind):
    keys = _keys_u32(kind, N)
    ek, ev = _expect(keys)
    k = torch.from_numpy(keys.view(np.int32)).to(DEV)
    v = torch.arange(N, dtype=torch.int32, device=DEV)
    plan = SortPlan(0, N, True)
    try:
        ok_, ov_ = torch.empty_like(k), torch.empty_like(v)
        plan.sort_copy(k, v, ok_, ov_, N)
        torch.cuda.synchronize()
        plan.check()
        _check_split(plan, kind)
        assert np.array_equal(ok_.cpu().numpy().view(np.uint32), ek)
        assert np.array_equal(ov_.cpu().numpy().view(np.uint32), ev)
        assert np.array_equal(k.cpu().numpy().view(np.uint32), keys)   # the input is only read
        # records -> arrays (the group sorts' local form)
        rec = torch.stack([k, v], dim=-1).contiguous().view(torch.int64).view(-1)
        ok_.fill_(-1)
        ov_.fill_(-1)
        plan.sort_records(rec, ok_, ov_, N)
        torch.cuda.synchronize()
        plan.check()
        _check_split(plan, kind)
        assert np.array_equal(ok_.cpu().numpy().view(np.uint32), ek)
        assert np.array_equal(ov_.cpu().numpy().view(np.uint32), ev)
    finally:
        plan.destroy()


def test_split_ballot_ranking_and_repeat(plan_debug):
    plan_debug(rank="ballot")
    keys = _keys_u32("one_bucket", N, seed=8)
    ek, ev = _expect(keys)
    k = torch.from_numpy(keys.view(np.int32)).to(DEV)
    v = torch.arange(N, dtype=torch.int32, device=DEV)
    kern = RadixSortKernel(keys=k, values=v, count=N)
    try:
        for _ in range(2):   # the same plan again: tables, arrivals and tickets start clean
            k.copy_(torch.from_numpy(keys.view(np.int32)))
            v.copy_(torch.arange(N, dtype=torch.int32))
            kern.dispatch()
            torch.cuda.synchronize()
            kern.check()
            _check_split(kern, "one_bucket")
            assert np.array_equal(k.cpu().numpy().view(np.uint32), ek)
            assert np.array_equal(v.cpu().numpy().view(np.uint32), ev)
        # a uniform sort on the same plan afterwards: no split, and still right
        u = O.gen_u32(77, N)
        k.copy_(torch.from_numpy(u.view(np.int32)))
        v.copy_(torch.arange(N, dtype=torch.int32))
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        assert kern.last_path() == "hybrid" and kern.last_split() == 0
        ek2, ev2 = _expect(u)
        assert np.array_equal(k.cpu().numpy().view(np.uint32), ek2)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), ev2)
    finally:
        kern.destroy()


@pytest.mark.parametrize("kind", ["f32_nearly", "few"])
def test_split_check_order(plan_debug, kind):
    # the radix path with check_order (nearly-sorted input would take the presorted path:
    # test_presorted_gpu.py)
    plan_debug(presorted=0)
    keys = _keys_u32(kind, N)
    ek, ev = _expect(keys)
    k = torch.from_numpy(keys.view(np.int32)).to(DEV)
    v = torch.arange(N, dtype=torch.int32, device=DEV)
    kern = RadixSortKernel(keys=k, values=v, count=N, check_order=True)
    try:
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        _check_split(kern, kind)
        assert np.array_equal(k.cpu().numpy().view(np.uint32), ek)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), ev)
        # sorted now: a second dispatch finds it in order and moves nothing
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        assert kern.last_path() == "in_order" and kern.last_split() == 0
        assert np.array_equal(k.cpu().numpy().view(np.uint32), ek)
    finally:
        kern.destroy()


@pytest.mark.parametrize("kind", ["f32_unit", "one_bucket"])
def test_split_off_takes_the_fallback(plan_debug, kind):
    plan_debug(split=0)
    keys = _keys_u32(kind, N)
    ek, ev = _expect(keys)
    k = torch.from_numpy(keys.view(np.int32)).to(DEV)
    v = torch.arange(N, dtype=torch.int32, device=DEV)
    kern = RadixSortKernel(keys=k, values=v, count=N)
    try:
        kern.dispatch()
        torch.cuda.synchronize()
        kern.check()
        assert kern.last_path() == "hybrid_fallback" and kern.last_split() == 0
        assert np.array_equal(k.cpu().numpy().view(np.uint32), ek)
        assert np.array_equal(v.cpu().numpy().view(np.uint32), ev)
    finally:
        kern.destroy()


@pytest.mark.parametrize("mode", ["one_bucket", "few_top"])
def test_split_region(mode):
    """A receiver's region (records grouped by top byte, its 16-bit counts from the senders) whose
    buckets are over the tile: split inside the region form (level 2 into the plan's second
    records buffer), bit-exact."""
    n = (13 << 20) + 7
    u = O.gen_u32(41, n)
    top_lo, top_hi = 0x30, 0x34
    if mode == "one_bucket":
        keys = np.uint32(0x31AB0000) | (u & np.uint32(0xFFFF))
    else:                             # 4 top bytes, 6 distinct keys in one, uniform in the others
        keys = (np.uint32(top_lo) + (u % np.uint32(4))) << np.uint32(24) | (u >> np.uint32(8) & np.uint32(0xFFFFFF))
        sel = (keys >> np.uint32(24)) == np.uint32(0x32)
        keys[sel] = np.uint32(0x32000000) | np.uint32(0x10101) * (u[sel] % np.uint32(6))
    keys = keys.astype(np.uint32)
    order = np.argsort(keys >> np.uint32(24), kind="stable")   # grouped by top byte, input order inside
    keys = keys[order]
    vals = np.arange(n, dtype=np.uint32)
    hist = np.zeros(65536, dtype=np.int32)
    np.add.at(hist, keys >> np.uint32(16), 1)
    rec = keys.astype(np.uint64) | (vals.astype(np.uint64) << np.uint64(32))
    rt = torch.from_numpy(rec.view(np.int64)).to(DEV)
    ht = torch.from_numpy(hist).to(DEV)
    ok_ = torch.empty(n, dtype=torch.int32, device=DEV)
    ov_ = torch.empty(n, dtype=torch.int32, device=DEV)
    plan = SortPlan(0, n, True)
    try:
        plan.sort_region(rt, ok_, ov_, n, ht, top_lo, top_hi)
        plan.check()
        assert plan.last_path() == "hybrid" and plan.last_split() in (2, 3)
    finally:
        plan.destroy()
    ek, ev = O.stable_sort_masked_c(keys, vals, 32)
    assert np.array_equal(ok_.cpu().numpy().view(np.uint32), ek)
    assert np.array_equal(ov_.cpu().numpy().view(np.uint32), ev)
