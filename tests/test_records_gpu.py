"""GPU: the multi-GPU record path of the C ABI against the oracle.

rs_plan_partition_records (stable one-digit partition of separate arrays into 8-byte
(key, value) records) and rs_plan_sort_records (whole stable sort of records into separate
arrays), at sizes covering the single-workgroup sort, the small-tile and the large-tile one-sweep
configurations, with and without given digit totals.
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(DEV)


def _np(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n", [1, 2, 1000, 16_384, 16_385, 1_000_003, 13_000_001])
def test_sort_records_matches_oracle(n):
    from radix_sort_amd.ops import SortPlan
    keys = O.gen_u32(n + 1, n)
    keys[::3] = keys[0]                           # duplicates: stability visible
    vals = O.gen_u32(n + 2, n)
    rec = torch.from_numpy((keys.astype(np.uint64) | (vals.astype(np.uint64) << np.uint64(32)))
                           .view(np.int64)).to(DEV)
    rec_copy = rec.clone()
    ko = torch.empty(n, dtype=torch.int32, device=DEV)
    vo = torch.empty(n, dtype=torch.int32, device=DEV)
    plan = SortPlan(0, n, True)
    plan.sort_records(rec, ko, vo, n)
    plan.check()
    ek, ev = O.stable_sort_masked(keys, vals, 32)
    assert (_np(ko) == ek).all() and (_np(vo) == ev).all()
    assert torch.equal(rec, rec_copy)             # the records are only read
    plan.destroy()


@pytest.mark.parametrize("n", [5, 40_000, 2_000_001, 13_000_001])
@pytest.mark.parametrize("given_totals", [True, False])
def test_partition_records_matches_oracle(n, given_totals):
    from radix_sort_amd import ops
    from radix_sort_amd.ops import SortPlan
    keys = O.gen_u32(7 * n, n)
    vals = np.arange(n, dtype=np.uint32)
    kt, vt = _t(keys), _t(vals)
    h = torch.empty(256, dtype=torch.int32, device=DEV)
    ops.histogram(kt, n, 24, 8, h)
    out = torch.empty(n, dtype=torch.int64, device=DEV)
    plan = SortPlan(0, n, True)
    plan.partition_records(kt, vt, out, n, 24, 8, h if given_totals else None)
    plan.check()
    r = out.cpu().numpy().view(np.uint64)
    top = keys >> np.uint32(24)
    perm = np.argsort(top, kind="stable")
    assert ((r & np.uint64(0xFFFFFFFF)).astype(np.uint32) == keys[perm]).all()
    assert ((r >> np.uint64(32)).astype(np.uint32) == vals[perm]).all()
    plan.destroy()


@pytest.mark.parametrize("n", [1_000_003, 13_000_001])
def test_sorted_records_to_arrays_with_check_order(n):
    """A check_order plan sorting records that are ALREADY in order into separate arrays: the
    order check must not skip the passes (the output arrays are not the input) -
    the arrays get the records' keys and values, path "hybrid" at >= 12M keys."""
    from radix_sort_amd.ops import SortPlan
    keys = np.sort(O.gen_u32(n + 5, n))
    vals = np.arange(n, dtype=np.uint32)
    rec = torch.from_numpy((keys.astype(np.uint64) | (vals.astype(np.uint64) << np.uint64(32)))
                           .view(np.int64)).to(DEV)
    ko = torch.zeros(n, dtype=torch.int32, device=DEV)
    vo = torch.zeros(n, dtype=torch.int32, device=DEV)
    plan = SortPlan(0, n, True, check_order=True)
    plan.sort_records(rec, ko, vo, n)
    plan.check()
    assert (_np(ko) == keys).all() and (_np(vo) == vals).all()
    if n >= 12 << 20:
        assert plan.last_path() == "hybrid"
    plan.destroy()
