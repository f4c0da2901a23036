"""GPU, large N: counts the C ABI accepts beyond BASELINE's 2^28 (README.md:100-102: N "not
bound by the implementation itself"; SURVEY §7 hard part 5, 64-bit addressing).

* 2^29 and 2^31 u32 keys + values on ONE GPU through rs_plan_sort (2^31: the single-GPU baseline
  of config 5), 2^29 keys only and as records in place - the hybrid path with the wide bucket
  kernel - verified as the stable sorted permutation of the input (sizes too large for the CPU
  oracle: sorted + a permutation with keys_out == keys_in[values_out] + equal keys in input order
  determine the stable sort uniquely);
* the largest accepted count, 2^32 - 1 keys, keys-only with check_order, and the top-byte
  histogram (k_pass_totals) at that count: every grid-stride loop near 2^32 terminates.
Each run once; together ~100 GB of HBM at peak.
"""
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.slow]
DEV = "cuda:0"


def _stable_kv_checks(keys_in, keys_out, vals_out):
    """keys_out sorted (unsigned), vals_out a permutation of 0..n-1 with keys_out ==
    keys_in[vals_out], equal keys in increasing value (= input) order."""
    from radix_sort_amd import ops
    n = keys_in.numel()
    assert ops.is_sorted(keys_out)
    seen = torch.zeros(n, dtype=torch.bool, device=DEV)
    seen[vals_out.long()] = True
    assert bool(seen.all()) and int(vals_out.min()) == 0 and int(vals_out.max()) == n - 1
    del seen
    step = 1 << 28
    for a in range(0, n, step):
        b = min(n, a + step)
        vo = vals_out[a:b].long()
        assert torch.equal(keys_in[vo], keys_out[a:b])
        # stability inside the chunk and across its left edge
        lo = max(a - 1, 0)
        k = keys_out[lo:b]
        v = vals_out[lo:b]
        eq = k[1:] == k[:-1]
        assert bool((v[1:][eq] > v[:-1][eq]).all())


def _hybrid_ran(kern) -> bool:
    """The device chose the hybrid MSD path, not its LSD fallback (rs_plan_last_path)."""
    return kern.last_path() == "hybrid"


@pytest.mark.parametrize("n", [1 << 29, 1 << 31])
def test_kv_large_single_gpu(n):
    """2^29 and 2^31 KV on one GPU (2^31: the single-GPU baseline of config 5).  Their 16-bit
    buckets hold ~8K / ~32K records, over every population-sized tile: the hybrid path sorts every
    bucket with k_bucket_sort_wide (round 2 sent both sizes to the four LSD passes)."""
    from radix_sort_amd import RadixSortKernel, ops
    kt = torch.empty(n, dtype=torch.int32, device=DEV)
    vt = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(kt, 31)
    ops.fill_iota_u32(vt)
    kin = kt.clone()
    k = RadixSortKernel(keys=kt, values=vt, count=n)
    k.set_profiling(True)
    k.dispatch()
    k.check()
    assert k.device_errors() == 0
    assert _hybrid_ran(k)
    k.destroy()
    _stable_kv_checks(kin, kt, vt)


def test_keys_only_and_records_2pow29():
    """The wide bucket kernel's other layouts at a size where it takes every bucket: keys only (in
    place) and (key, value) records in place (RadixSortTextureKernel)."""
    from radix_sort_amd import RadixSortKernel, RadixSortTextureKernel, ops
    n = 1 << 29
    kt = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(kt, 29)
    fp_in = _fingerprint(kt)
    k = RadixSortKernel(keys=kt, count=n)
    k.set_profiling(True)
    k.dispatch()
    k.check()
    assert _hybrid_ran(k)
    k.destroy()
    assert ops.is_sorted(kt, n)
    fp_out = _fingerprint(kt)
    assert torch.equal(fp_in[0], fp_out[0]) and fp_in[1:] == fp_out[1:]
    del kt
    rec = torch.empty((n, 2), dtype=torch.int32, device=DEV)
    kin = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(kin, 290)
    rec[:, 0] = kin
    rec[:, 1] = torch.arange(n, dtype=torch.int32, device=DEV)
    k = RadixSortTextureKernel(texture=rec, count=n)
    k.set_profiling(True)
    k.dispatch()
    k.check()
    assert _hybrid_ran(k)
    k.destroy()
    ko, vo = rec[:, 0].contiguous(), rec[:, 1].contiguous()
    del rec
    _stable_kv_checks(kin, ko, vo)


def _fingerprint(t):
    """Order-independent multiset fingerprint of u32 words: top-16-bit histogram, sum and sum of
    squares (mod 2^64), computed in 2^28-word chunks."""
    h = torch.zeros(1 << 16, dtype=torch.int64, device=DEV)
    s1 = torch.zeros((), dtype=torch.int64, device=DEV)
    s2 = torch.zeros((), dtype=torch.int64, device=DEV)
    step = 1 << 28
    for a in range(0, t.numel(), step):
        u = t[a:a + step].long() & 0xFFFFFFFF
        h += torch.bincount(u >> 16, minlength=1 << 16)
        s1 += u.sum()
        s2 += (u * u).sum()
    return h, int(s1), int(s2)


def test_keys_only_default_at_max_count():
    """The default route (no check_order) at the largest accepted count.  Round 2's hybrid-path
    histogram computed its per-row chunk in 32 bits, which wraps for n > 2^32 - 256: every row
    counted nothing, the plan saw all-zero buckets, picked the MSD passes and returned unsorted
    keys with RS_OK.  The chunk is 64-bit now, the plan kernel refuses a histogram that does not
    account for all n keys, and above ~2.2G keys (where some 16-bit bucket all but certainly
    exceeds the largest bucket tile) the host goes straight to the LSD passes."""
    from radix_sort_amd import RadixSortKernel, ops
    n = (1 << 32) - 1
    kt = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(kt, 33)
    fp_in = _fingerprint(kt)
    k = RadixSortKernel(keys=kt, count=n)
    k.dispatch()
    k.check()
    assert k.device_errors() == 0
    k.destroy()
    assert ops.is_sorted(kt, n)
    fp_out = _fingerprint(kt)
    assert torch.equal(fp_in[0], fp_out[0]) and fp_in[1:] == fp_out[1:]


def test_keys_only_check_order_at_max_count():
    from radix_sort_amd import RadixSortKernel, ops
    n = (1 << 32) - 1
    kt = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(kt, 32)
    # the top-byte histogram at this count (k_pass_totals' grid-stride tail near 2^32)
    h = torch.empty(256, dtype=torch.int32, device=DEV)
    ops.histogram(kt, n, 24, 8, h)
    fp_in = _fingerprint(kt)
    assert torch.equal(h.long(), fp_in[0].view(256, 256).sum(dim=1))
    k = RadixSortKernel(keys=kt, count=n, check_order=True)
    k.dispatch()
    k.check()
    k.destroy()
    assert ops.is_sorted(kt, n)
    fp_out = _fingerprint(kt)
    assert torch.equal(fp_in[0], fp_out[0]) and fp_in[1:] == fp_out[1:]
