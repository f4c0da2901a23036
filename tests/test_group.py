"""CPU: the single-process multi-GPU C ABI (rs_group_*, include/rsort.h) — the host bucket plan
(rs_group_plan) agrees with the torch.distributed path's (radix_sort_amd/distributed.py
bucket_owners / bucket_groups) on uniform, skewed, empty and one-bucket histograms, and
rs_group_create validates its options before touching a device.  SURVEY.md §8(b)/(e)."""
import ctypes

import numpy as np
import pytest

from radix_sort_amd import _lib
from radix_sort_amd.distributed import bucket_groups, bucket_owners
from radix_sort_amd.group import group_plan


def _hists(kind, world, buckets, rng):
    if kind == "uniform":
        return rng.integers(900, 1100, size=(world, buckets))
    if kind == "skewed":
        h = rng.integers(0, 50, size=(world, buckets))
        h[:, 3] += 100000
        return h
    if kind == "one_bucket":
        h = np.zeros((world, buckets), dtype=np.int64)
        h[:, buckets - 1] = rng.integers(1, 1 << 20, size=world)
        return h
    if kind == "empty":
        return np.zeros((world, buckets), dtype=np.int64)
    if kind == "sparse":
        h = np.zeros((world, buckets), dtype=np.int64)
        idx = rng.choice(buckets, size=max(1, buckets // 16), replace=False)
        h[:, idx] = rng.integers(1, 5000, size=(world, idx.size))
        return h
    if kind == "huge":           # counts near 2^32 per rank (64-bit arithmetic in the plan)
        return rng.integers(1 << 23, 1 << 24, size=(world, buckets))
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["uniform", "skewed", "one_bucket", "empty", "sparse", "huge"])
@pytest.mark.parametrize("world,buckets,rounds", [(1, 256, 4), (2, 256, 4), (3, 256, 1),
                                                  (8, 256, 4), (8, 16, 16), (5, 4, 3),
                                                  (64, 256, 2)])
def test_group_plan_matches_distributed_plan(kind, world, buckets, rounds):
    rng = np.random.default_rng(world * 1000 + buckets + rounds)
    h = _hists(kind, world, buckets, rng).tolist()
    bounds, cuts = group_plan(h, rounds)
    assert bounds == bucket_owners(h, world)
    assert cuts == bucket_groups(h, bounds, rounds)
    # whole buckets, every bucket owned exactly once, rounds tile each rank's range
    assert bounds[0] == 0 and bounds[-1] == buckets and bounds == sorted(bounds)
    for q in range(world):
        assert cuts[q][0] == bounds[q] and cuts[q][-1] == bounds[q + 1]
        assert cuts[q] == sorted(cuts[q])


def test_group_plan_balances_uniform_counts():
    h = [[1000] * 256 for _ in range(8)]
    bounds, _ = group_plan(h, 4)
    assert [bounds[q + 1] - bounds[q] for q in range(8)] == [32] * 8


def _create(world=1, devices=None, **kw):
    d = dict(capacity=1000, flags=_lib.RS_FLAG_HAS_VALUES, transport=_lib.RS_TRANSPORT_RCCL,
             top_bits=0, rounds=0)
    d.update(kw)
    desc = _lib.GroupDesc(**d)
    devs = devices if devices is not None else [0] * max(world, 1)
    arr = (ctypes.c_int32 * len(devs))(*devs)
    g = ctypes.c_void_p()
    st = _lib.load().rs_group_create(world, arr, ctypes.byref(desc), ctypes.byref(g))
    return st, g


@pytest.mark.parametrize("kw,msg", [
    (dict(world=0), "world"),
    (dict(world=65, devices=[0] * 65), "world"),
    (dict(top_bits=9), "top_bits"),
    (dict(rounds=17), "rounds"),
    (dict(flags=_lib.RS_FLAG_CHECK_ORDER), "flags"),
    (dict(transport=7), "transport"),
    (dict(capacity=1 << 32), "capacity"),
])
def test_group_create_rejects_bad_options(kw, msg):
    st, g = _create(**kw)
    assert st == _lib.RS_ERR_INVALID_ARG and not g.value
    assert msg in _lib.load().rs_last_error().decode()


def test_group_plan_rejects_bad_arguments():
    L = _lib.load()
    h = (ctypes.c_uint64 * 4)()
    b = (ctypes.c_uint32 * 2)()
    c = (ctypes.c_uint32 * 4)()
    assert L.rs_group_plan(0, 4, 1, h, b, c) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_group_plan(1, 4, 0, h, b, c) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_group_plan(1, 4, 1, None, b, c) == _lib.RS_ERR_INVALID_ARG
