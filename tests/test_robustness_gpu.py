"""GPU: failure reporting and the guarded assumptions of the kernels.

* a timed-out look-back wait of the one-sweep pass is reported (RS_ERR_DEVICE) by check() and
  does not poison the plan: the next sort on the same plan is correct;
* the lane-order self-test of the LDS atomics the default ranking relies on runs at plan creation
  and a failure switches plans to the ballot ranking;
* PrefixSumKernel.dispatch(pass, dispatchSizeBuffer, offset): the indirect form
  (PrefixSumKernel.ts:147-158) and getDispatchChain (:135-137).
"""
import math

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


def test_lookback_timeout_is_reported_then_plan_recovers():
    from radix_sort_amd import RadixSortKernel, RadixSortError, _lib, ops
    n = 1 << 26
    kt = torch.empty(n, dtype=torch.int32, device=DEV)
    vt = torch.empty(n, dtype=torch.int32, device=DEV)
    k = RadixSortKernel(keys=kt, values=vt, count=n)
    L = _lib.load()
    # wait limit 0: any wait on an unpublished predecessor times out at once
    _lib.check(L.rs_plan_set_wait_limit(k._plan, 0), "wait limit")
    seen = 0
    for i in range(4):
        ops.fill_random_u32(kt, 500 + i)
        ops.fill_iota_u32(vt)
        k.dispatch()
        try:
            k.check()
        except RadixSortError as e:
            assert e.status == _lib.RS_ERR_DEVICE and "timed out" in str(e)
            seen += 1
    assert seen >= 1, "no look-back wait ever found an unpublished predecessor"
    # reported once: the next check is clean without a new failure
    k.check()
    # same plan, default limit: correct again (the device error word is cleared per sort)
    _lib.check(L.rs_plan_set_wait_limit(k._plan, 1 << 20), "wait limit")
    keys = O.gen_u32(77, n)
    kt.copy_(_t(keys))
    ops.fill_iota_u32(vt)
    k.dispatch()
    k.check()
    assert k.device_errors() == 0
    ek, ev = O.stable_sort_masked(keys, np.arange(n, dtype=np.uint32), 32)
    assert (_np(kt) == ek).all() and (_np(vt) == ev).all()


def test_pending_device_error_fails_the_next_dispatch():
    """A failure not yet reported by check() is reported by the next dispatch, which enqueues
    nothing (rs_plan_sort returns RS_ERR_DEVICE)."""
    from radix_sort_amd import RadixSortKernel, RadixSortError, _lib, ops
    n = 1 << 26
    kt = torch.empty(n, dtype=torch.int32, device=DEV)
    vt = torch.empty(n, dtype=torch.int32, device=DEV)
    k = RadixSortKernel(keys=kt, values=vt, count=n)
    L = _lib.load()
    _lib.check(L.rs_plan_set_wait_limit(k._plan, 0), "wait limit")
    failed = False
    for i in range(4):
        ops.fill_random_u32(kt, 900 + i)
        torch.cuda.synchronize()
        try:
            k.dispatch()
        except RadixSortError as e:
            assert e.status == _lib.RS_ERR_DEVICE
            failed = True
            break
    assert failed
    k.check()   # nothing pending any more


def test_lane_order_selftest_passes_and_default_ranking():
    from radix_sort_amd import RadixSortKernel
    kt = torch.zeros(1 << 20, dtype=torch.int32, device=DEV)
    info = RadixSortKernel(keys=kt, count=kt.numel()).info
    assert info["lane_order_selftest"] == 1
    assert info["rank_mode"] == "lds_atomic"


def test_selftest_failure_falls_back_to_ballot_ranking(plan_debug):
    from radix_sort_amd import RadixSortKernel
    plan_debug(selftest_fail=1)
    for n in (5_000, 1_000_003, 13_000_001):
        keys = O.gen_u32(n, n) % np.uint32(1000)          # duplicates: stability is visible
        vals = np.arange(n, dtype=np.uint32)
        kt, vt = _t(keys), _t(vals)
        k = RadixSortKernel(keys=kt, values=vt, count=n)
        info = k.info
        assert info["rank_mode"] == "ballot" and info["lane_order_selftest"] == 0
        k.dispatch()
        k.check()
        ek, ev = O.stable_sort_masked(keys, vals, 32)
        assert (_np(kt) == ek).all() and (_np(vt) == ev).all(), n


def _ref_chain(count, T):
    """PrefixSumKernel.createPassRecursive's dispatch sizes (PrefixSumKernel.ts:45-137), with
    findOptimalDispatchSize (utils.ts:8-23) at the default 65535 limit."""
    out = []

    def rec(c):
        wc = math.ceil(c / (2 * T))
        x, y = wc, 1
        if wc > 65535:
            x = int(math.floor(math.sqrt(wc)))
            y = math.ceil(wc / x)
        out.extend([x, y, 1])
        if wc > 1:
            rec(wc)
            out.extend([x, y, 1])
    rec(count)
    return out


@pytest.mark.parametrize("n,wx,wy", [(1000, 16, 16), (1 << 20, 16, 16), (100_000_000, 8, 8),
                                     (3, 1, 1)])
def test_prefix_sum_dispatch_chain_matches_reference(n, wx, wy):
    from radix_sort_amd import PrefixSumKernel
    d = torch.zeros(max(n, 1), dtype=torch.int32, device=DEV)
    k = PrefixSumKernel(data=d, count=n, workgroup_size={"x": wx, "y": wy})
    assert k.get_dispatch_chain() == _ref_chain(n, wx * wy)
    k.destroy()


def test_prefix_sum_indirect_dispatch():
    from radix_sort_amd import PrefixSumKernel
    n = 1_000_003
    data = O.gen_u32(5, n) % np.uint32(1000)
    exp = np.concatenate([[0], np.cumsum(data[:-1], dtype=np.uint64)]).astype(np.uint32)
    d = _t(data)
    k = PrefixSumKernel(data=d, count=n)
    chain = k.get_dispatch_chain()
    # the chain at byte offset 12 (after one unrelated triple), as the check-sort writes it
    buf = _t(np.array([7, 7, 7] + chain, dtype=np.uint32))
    k.dispatch(None, buf, 12)
    assert (_np(d) == exp).all()
    # zeroed x entry: the scan is skipped, on the device
    d2 = _t(data)
    zero = _t(np.array([0] + chain[1:], dtype=np.uint32))
    k2 = PrefixSumKernel(data=d2, count=n)
    k2.dispatch(None, zero, 0)
    assert (_np(d2) == data).all()


def test_prefix_sum_gated_dispatch_after_ticket_ring_wraps():
    """every launch clears the NEXT launch's ticket slot (a ring of 64).  A launch gated
    off by a zeroed indirect triple must clear it too, else after >= 64 launches the next live
    dispatch finds a stale count in its slot and scans nothing without an error."""
    from radix_sort_amd import PrefixSumKernel
    n = 200_003
    data = O.gen_u32(17, n) % np.uint32(1000)
    d = _t(data)
    k = PrefixSumKernel(data=d, count=n)
    chain = k.get_dispatch_chain()
    live = _t(np.array(chain, dtype=np.uint32))
    zero = _t(np.array([0] + chain[1:], dtype=np.uint32))
    for _ in range(70):          # wraps the 64-slot ticket ring
        k.dispatch(None, live, 0)
    k.dispatch(None, zero, 0)    # gated off on the device
    d.copy_(_t(data))
    k.dispatch(None, live, 0)    # the launch whose slot the gated one had to clear
    k.check()
    assert (_np(d) == O.prefix_sum(data, n)).all()
    k.destroy()


def test_scan_lookback_timeout_is_reported_then_plan_recovers():
    """The single-pass PrefixSumKernel: with the wait bound at 0 a look-back wait on an unpublished
    predecessor times out, check() reports it once (RS_ERR_DEVICE); with the default bound the same
    plan scans correctly again."""
    from radix_sort_amd import PrefixSumKernel, RadixSortError, _lib
    n = (1 << 26) + 5
    d = O.gen_u32(91, n) & np.uint32(0xFF)
    t = _t(d)
    k = PrefixSumKernel(data=t, count=n)
    L = _lib.load()
    _lib.check(L.rs_scan_plan_set_wait_limit(k._plan, 0), "wait limit")
    seen = 0
    for _ in range(4):
        t.copy_(_t(d))
        k.dispatch()
        try:
            k.check()
        except RadixSortError as e:
            assert e.status == _lib.RS_ERR_DEVICE and "timed out" in str(e)
            seen += 1
    assert seen >= 1, "no look-back wait ever found an unpublished predecessor"
    k.check()
    _lib.check(L.rs_scan_plan_set_wait_limit(k._plan, 1 << 20), "wait limit")
    t.copy_(_t(d))
    k.dispatch()
    k.check()
    assert (_np(t) == O.prefix_sum(d, n)).all()
    k.destroy()


@pytest.mark.parametrize("n,offset", [(1, 0), (4095, 0), (4096, 1), (4097, 3), (16383, 0), (16384, 1),
                                      (32767, 0), (32768, 1), (32769, 3), (1_000_003, 1), ((1 << 24) + 7, 0)])
def test_scan_sizes_and_unaligned_data(n, offset):
    """Tile edges of the single-pass scan (32K-element tiles), one element, and data that is not
    16-byte aligned (scalar loads / stores); the words after count are untouched."""
    from radix_sort_amd import PrefixSumKernel
    d = O.gen_u32(n + 17, n + offset + 8)
    t = _t(d)
    view = t[offset:offset + n + 8]
    k = PrefixSumKernel(data=view, count=n)
    k.dispatch()
    k.check()
    out = _np(t)
    assert (out[:offset] == d[:offset]).all()
    assert (out[offset:offset + n] == O.prefix_sum(d[offset:offset + n], n)).all()
    assert (out[offset + n:] == d[offset + n:]).all()
    k.destroy()
