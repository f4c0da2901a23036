"""GPU parity: the HIP sort (through the C ABI) against the oracle and the golden fixtures.

Bar: bit-exact.  Small and medium sizes compare every word with the oracle; the BASELINE
full sizes (64M keys-only, 256M KV, 256M nearly-sorted f32 + check_order) are checked through
size-independent properties: sorted by masked key, keys_out == keys_in[values_out] with
values = iota (a permutation), equal keys keep increasing values (stability), and for keys-only
an independent multiset check against torch.sort.
"""
import numpy as np
import pytest

import oracle as O
from conftest import case_arrays

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _t(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(DEV)


def _np(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint32)


def _sort(keys, vals, count=None, **opts):
    from radix_sort_amd import RadixSortKernel
    kt = _t(keys)
    vt = None if vals is None else _t(vals)
    k = RadixSortKernel(device=0, keys=kt, values=vt,
                        count=keys.size if count is None else count, **opts)
    k.dispatch()
    torch.cuda.synchronize()
    out = _np(kt), (None if vt is None else _np(vt))
    k.destroy()
    return out


def test_golden_fixtures_default_options(golden):
    manifest, arrays = golden
    for case in manifest["sort_cases"]:
        keys, vals, exp_k, exp_v = case_arrays(arrays, case)
        k, v = _sort(keys, vals, case["count"], bit_count=case["bit_count"])
        assert (k == exp_k).all(), case
        if vals is not None:
            assert (v == exp_v).all(), case


@pytest.mark.parametrize("opts", [
    dict(check_order=True),
    dict(local_shuffle=True, avoid_bank_conflicts=True),
    dict(radix_bits=2, workgroup_size={"x": 8, "y": 8}),          # the reference's 4-way pass structure
    dict(radix_bits=4, checkOrder=True, workgroupSize={"x": 32, "y": 32}),
])
def test_golden_fixtures_option_matrix(golden, opts):
    manifest, arrays = golden
    for case in manifest["sort_cases"][::3] + [c for c in manifest["sort_cases"]
                                                if c["kind"] in ("sorted", "q1", "nearly", "equal")]:
        keys, vals, exp_k, exp_v = case_arrays(arrays, case)
        k, v = _sort(keys, vals, case["count"], bit_count=case["bit_count"], **opts)
        assert (k == exp_k).all(), (case, opts)
        if vals is not None:
            assert (v == exp_v).all(), (case, opts)


def test_large_golden_sha(golden):
    import hashlib
    manifest, _ = golden
    for case in manifest["large_cases"]:
        n = case["n"]
        kt = torch.empty(n, dtype=torch.int32, device=DEV)
        from radix_sort_amd import ops, RadixSortKernel
        ops.fill_random_u32(kt, case["seed"])
        if case["kind"] == "f32":
            u = _np(kt)
            kt = _t(((u >> np.uint32(8)).astype(np.float64) * 2.0 ** -24).astype(np.float32).view(np.uint32))
        vt = None
        if case["has_values"]:
            vt = torch.empty(n, dtype=torch.int32, device=DEV)
            ops.fill_iota_u32(vt)
        k = RadixSortKernel(keys=kt, values=vt, count=n)
        k.dispatch()
        torch.cuda.synchronize()
        assert hashlib.sha256(_np(kt).tobytes()).hexdigest() == case["sha256_keys"]
        if vt is not None:
            assert hashlib.sha256(_np(vt).tobytes()).hexdigest() == case["sha256_values"]


@pytest.mark.parametrize("bits", [4, 8, 12, 16, 20, 24, 28, 32])
@pytest.mark.parametrize("radix_bits", [0, 2, 4])
def test_random_vs_oracle_bit_counts(bits, radix_bits):
    n = 300_001 if radix_bits != 2 else 70_001
    keys = O.gen_u32(bits * 31 + radix_bits, n)
    keys[::7] = keys[3]          # duplicates: stability visible through the values
    vals = np.arange(n, dtype=np.uint32)
    k, v = _sort(keys, vals, bit_count=bits, radix_bits=radix_bits)
    ek, ev = O.stable_sort_masked(keys, vals, bits)
    assert (k == ek).all() and (v == ev).all()


@pytest.mark.parametrize("n", [4095, 4096, 4097, 1 << 20, (1 << 22) + 12345, 9_000_001])
def test_sizes_keys_only_and_kv(n):
    keys = O.gen_u32(n, n)
    ek, _ = O.stable_sort_masked_c(keys, None, 32)
    k, _ = _sort(keys, None)
    assert (k == ek).all()
    vals = np.arange(n, dtype=np.uint32)
    k, v = _sort(keys, vals, check_order=(n % 2 == 1))
    ek, ev = O.stable_sort_masked_c(keys, vals, 32)
    assert (k == ek).all() and (v == ev).all()


def test_count_less_than_buffer_leaves_tail():
    n, count = 100_000, 77_777
    keys = O.gen_u32(77, n)
    vals = O.gen_u32(78, n)   # arbitrary values, not iota
    k, v = _sort(keys, vals, count=count)
    ek, ev = O.stable_sort_masked(keys, vals, 32, count)
    assert (k == ek).all() and (v == ev).all()


@pytest.mark.parametrize("kind", ["sorted", "sorted_after_first_pass", "reverse", "equal"])
def test_check_order_early_exit_paths(kind):
    n = 1 << 20
    u = O.gen_u32(5, n)
    if kind == "sorted":
        keys = np.sort(u)
    elif kind == "sorted_after_first_pass":
        # only the low 6 bits vary: sorted after pass 0, so the check before pass 1 exits
        # early with the data in the tmp buffers (exercises the tmp -> caller copy)
        keys = u & np.uint32(0x3F)
    elif kind == "reverse":
        keys = np.sort(u)[::-1].copy()
    else:
        keys = np.full(n, 12345, dtype=np.uint32)
    vals = np.arange(n, dtype=np.uint32)
    for bits in (32, 24, 8):
        k, v = _sort(keys, vals, check_order=True, bit_count=bits)
        ek, ev = O.stable_sort_masked(keys, vals, bits)
        assert (k == ek).all() and (v == ev).all(), (kind, bits)


def test_prefix_sum_kernel_golden(golden):
    from radix_sort_amd import PrefixSumKernel
    manifest, arrays = golden
    for case in manifest["scan_cases"]:
        d, exp = arrays[case["name"] + "_data"], arrays[case["name"] + "_exp"]
        t = _t(d)
        k = PrefixSumKernel(data=t, count=case["count"], workgroupSize={"x": 16, "y": 16})
        k.dispatch()
        torch.cuda.synchronize()
        assert (_np(t) == exp).all(), case["name"]


def test_prefix_sum_large_wraps():
    from radix_sort_amd import PrefixSumKernel
    n = (1 << 24) + 3
    d = O.gen_u32(11, n)          # large values: the running sum wraps mod 2^32
    t = _t(d)
    PrefixSumKernel(data=t).dispatch()
    torch.cuda.synchronize()
    assert (_np(t) == O.prefix_sum(d)).all()


def test_partition_pass_and_histogram():
    from radix_sort_amd import ops
    n = 1_000_003
    keys = O.gen_u32(3, n)
    kt, vt = _t(keys), torch.arange(n, dtype=torch.int32, device=DEV)
    ok, ov = torch.empty_like(kt), torch.empty_like(vt)
    hist = torch.empty(256, dtype=torch.int32, device=DEV)
    plan = ops.SortPlan(0, n, has_values=True)
    plan.partition(kt, vt, ok, ov, n, 24, 8, hist)
    torch.cuda.synchronize()
    top = keys >> np.uint32(24)
    perm = np.argsort(top, kind="stable")
    assert (_np(ok) == keys[perm]).all() and (_np(ov) == perm.astype(np.uint32)).all()
    assert (_np(hist) == np.bincount(top, minlength=256)).all()


@pytest.mark.parametrize("n", [1_000_003, 13_000_001])
def test_partition_given_totals(n):
    """rs_plan_partition_totals: the one-sweep partition (values, n >= 12M) fed the digit totals
    from rs_histogram, and its fallback below that size, give the stable partition."""
    from radix_sort_amd import ops
    keys = O.gen_u32(n + 5, n)
    kt, vt = _t(keys), torch.arange(n, dtype=torch.int32, device=DEV)
    ok, ov = torch.empty_like(kt), torch.empty_like(vt)
    hist = torch.empty(256, dtype=torch.int32, device=DEV)
    ops.histogram(kt, n, 24, 8, hist)
    plan = ops.SortPlan(0, n, has_values=True)
    plan.partition_totals(kt, vt, ok, ov, n, 24, 8, hist)
    torch.cuda.synchronize()
    top = keys >> np.uint32(24)
    perm = np.argsort(top, kind="stable")
    assert (_np(ok) == keys[perm]).all() and (_np(ov) == perm.astype(np.uint32)).all()
    plan.destroy()


def test_kernel_profiling_counts_launches():
    from radix_sort_amd import RadixSortKernel, ops
    n = 1 << 22
    kt = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(kt, 1)
    k = RadixSortKernel(keys=kt, count=n)
    k.set_profiling(True)
    k.dispatch()
    torch.cuda.synchronize()
    t = k.kernel_times()
    assert t["scatter"]["launches"] == k.info["passes"] == 4
    assert t["scatter"]["ms"] > 0
    assert ops.is_sorted(kt)


# ---- BASELINE full sizes (properties) ---------------------------------------------------

def _verify_kv_iota(keys_in, keys_out, vals_out, bits=32):
    n = keys_in.numel()
    vo = vals_out.long()
    assert torch.equal(torch.bincount(vo, minlength=n), torch.ones(n, dtype=torch.long, device=DEV))
    assert torch.equal(keys_in[vo], keys_out)                       # keys_out == keys_in[values]
    mask = (1 << bits) - 1
    ku = (keys_out.long() & 0xFFFFFFFF) & mask
    assert bool((ku[1:] >= ku[:-1]).all())                         # sorted
    eq = ku[1:] == ku[:-1]
    assert bool((vo[1:][eq] > vo[:-1][eq]).all())                   # stable


@pytest.mark.slow
def test_config2_64M_keys_only():
    from radix_sort_amd import RadixSortKernel, ops
    n = 1 << 26
    kt = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(kt, 2)
    ref = torch.sort(kt.long() & 0xFFFFFFFF).values
    RadixSortKernel(keys=kt, count=n, bit_count=32, workgroup_size={"x": 16, "y": 16}).dispatch()
    torch.cuda.synchronize()
    assert torch.equal(kt.long() & 0xFFFFFFFF, ref)
    del ref


@pytest.mark.slow
def test_config3_256M_kv_local_shuffle():
    from radix_sort_amd import RadixSortKernel, ops
    n = 1 << 28
    kt = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(kt, 3)
    k_in = kt.clone()
    vt = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_iota_u32(vt)
    RadixSortKernel(keys=kt, values=vt, count=n, local_shuffle=True).dispatch()
    torch.cuda.synchronize()
    _verify_kv_iota(k_in, kt, vt)


@pytest.mark.slow
def test_config4_256M_nearly_sorted_f32_check_order():
    from radix_sort_amd import RadixSortKernel, ops
    n = 1 << 28
    bits = O.nearly_sorted_f32_bits(n, 4)
    kt = _t(bits)
    k_in = kt.clone()
    vt = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_iota_u32(vt)
    kern = RadixSortKernel(keys=kt, values=vt, count=n, check_order=True)
    kern.dispatch()
    torch.cuda.synchronize()
    kern.check()
    # the presorted path: the displaced keys extracted, sorted and merged back
    assert kern.last_path() == "presorted"
    _verify_kv_iota(k_in, kt, vt)
    # fully sorted variant: early exit leaves the data untouched
    kern.dispatch()
    torch.cuda.synchronize()
    kern.check()
    assert kern.last_path() == "in_order"
    kern.destroy()
    _verify_kv_iota(k_in, kt, vt)


@pytest.mark.parametrize("rank", ["atomic", "ballot"])
@pytest.mark.parametrize("tile", ["small", "large", "large_keys1024"])
def test_rank_modes_and_tile_configs(plan_debug, golden, rank, tile):
    """Both in-wave ranking implementations and both tile configurations give the oracle's
    result (selected per plan with rs_plan_set_debug)."""
    # keys-only large tiles: 512 x 32 by default, 1024 x 16 with keys_cfg=0
    plan_debug(rank=rank, tile=tile.split("_")[0], keys_cfg=0 if tile.endswith("1024") else 1)
    for n, bits, kind in ((20_000, 32, "u32"), (300_001, 32, "few"), (1_000_003, 24, "u32"),
                          (70_001, 12, "u32")):
        keys = O.gen_u32(n + bits, n)
        if kind == "few":
            keys = keys % np.uint32(13)
        vals = np.arange(n, dtype=np.uint32)
        k, v = _sort(keys, vals, bit_count=bits, check_order=(n % 2 == 1))
        ek, ev = O.stable_sort_masked(keys, vals, bits)
        assert (k == ek).all() and (v == ev).all(), (n, bits, kind)
        k, _ = _sort(keys, None, bit_count=bits)
        assert (k == ek).all()
    manifest, arrays = golden
    for case in manifest["sort_cases"][::4]:
        keys, vals, exp_k, exp_v = case_arrays(arrays, case)
        k, v = _sort(keys, vals, case["count"], bit_count=case["bit_count"])
        assert (k == exp_k).all(), case
        if vals is not None:
            assert (v == exp_v).all(), case



@pytest.mark.parametrize("onesweep", ["1", "0"])
@pytest.mark.parametrize("tile", ["small", "large"])
def test_onesweep_and_three_kernel_paths(plan_debug, onesweep, tile):
    """The one-sweep pass (whole-array totals + decoupled look-back) and the histogram / scan /
    scatter pass give the oracle's result for every layout; no bounded wait times out."""
    from radix_sort_amd import RadixSortKernel, RadixSortTextureKernel
    plan_debug(onesweep=int(onesweep), tile=tile)
    for n, bits, kind in ((16_385, 32, "u32"), (100_003, 32, "few"), (2_500_000, 32, "u32"),
                          (5_000_001, 20, "u32"), (40_000, 8, "sorted"), (300_000, 12, "u32")):
        keys = O.gen_u32(n * 3 + bits, n)
        if kind == "few":
            keys = keys % np.uint32(5)
        elif kind == "sorted":
            keys = np.sort(keys)
        vals = O.gen_u32(n * 5 + bits, n)
        ek, ev = O.stable_sort_masked(keys, vals, bits)
        kt, vt = _t(keys), _t(vals)
        k = RadixSortKernel(keys=kt, values=vt, count=n, bit_count=bits, check_order=(n % 2 == 1))
        k.dispatch()
        assert k.device_errors() == 0
        assert (_np(kt) == ek).all() and (_np(vt) == ev).all(), (n, bits, kind)
        k.destroy()
        kt = _t(keys)
        k = RadixSortKernel(keys=kt, count=n, bit_count=bits)
        k.dispatch()
        assert k.device_errors() == 0
        assert (_np(kt) == ek).all(), (n, bits, kind, "keys only")
        k.destroy()
        rt = _t(np.stack([keys, vals], axis=-1).reshape(-1)).view(-1, 2)
        k = RadixSortTextureKernel(texture=rt, count=n, bit_count=bits)
        k.dispatch()
        assert k.device_errors() == 0
        out = _np(rt).reshape(-1, 2)
        assert (out[:, 0] == ek).all() and (out[:, 1] == ev).all(), (n, bits, kind, "aos")
        k.destroy()


@pytest.mark.parametrize("tile", ["small", "large"])
def test_onesweep_check_order_exits_and_narrow_digits(plan_debug, tile):
    """One-sweep path: check_order early exits (an exit after pass 0 or 1 leaves the data as
    (key, value) records in one of the two records buffers: k_finalize<SOA, AOS>), and 2-/4-bit
    digits.  The order checks are fused into k_pass_totals / k_onesweep here, on all three
    layouts."""
    from radix_sort_amd import RadixSortKernel, RadixSortTextureKernel
    plan_debug(onesweep=1, tile=tile)
    n = 1_500_001
    u = O.gen_u32(77, n)
    vals = O.gen_u32(78, n)
    # exits before pass 0, 1 (data in the first records buffer) and 2 (in the second one)
    for kind in ("sorted", "sorted_after_first_pass", "sorted_after_two_passes", "random"):
        keys = {"sorted": np.sort(u), "sorted_after_first_pass": u & np.uint32(0x3F),
                "sorted_after_two_passes": u & np.uint32(0xFFFF), "random": u}[kind]
        ek, ev = O.stable_sort_masked(keys, vals, 32)
        kt, vt = _t(keys), _t(vals)
        k = RadixSortKernel(keys=kt, values=vt, count=n, check_order=True)
        k.dispatch()
        assert k.device_errors() == 0
        assert (_np(kt) == ek).all() and (_np(vt) == ev).all(), kind
        k.destroy()
        # the fused checks on the other two layouts (keys only; (key, value) records, where the
        # key after a wave's last slot is word 2q of the records)
        kt = _t(keys)
        k = RadixSortKernel(keys=kt, count=n, check_order=True)
        k.dispatch()
        assert k.device_errors() == 0
        assert (_np(kt) == ek).all(), (kind, "keys only")
        k.destroy()
        rt = _t(np.stack([keys, vals], axis=-1).reshape(-1)).view(-1, 2)
        k = RadixSortTextureKernel(texture=rt, count=n, check_order=True)
        k.dispatch()
        assert k.device_errors() == 0
        out = _np(rt).reshape(-1, 2)
        assert (out[:, 0] == ek).all() and (out[:, 1] == ev).all(), (kind, "records")
        k.destroy()
    # an inversion only at the very last pair (the reference's unchecked pair, Q1), only across
    # a wave boundary inside a tile, only across a tile boundary: all must still be sorted
    for pos in (n - 2, 16384 * 3 + 1023, 16384 * 2 - 1):
        keys = np.sort(u)
        keys[pos], keys[pos + 1] = keys[pos + 1], keys[pos]
        ek, ev = O.stable_sort_masked(keys, vals, 32)
        kt, vt = _t(keys), _t(vals)
        k = RadixSortKernel(keys=kt, values=vt, count=n, check_order=True)
        k.dispatch()
        assert k.device_errors() == 0
        assert (_np(kt) == ek).all() and (_np(vt) == ev).all(), pos
        k.destroy()
    for radix_bits, bits in ((2, 12), (4, 16), (4, 32)):
        keys = u & np.uint32((1 << bits) - 1 if bits < 32 else 0xFFFFFFFF)
        ek, ev = O.stable_sort_masked(keys, vals, bits)
        kt, vt = _t(keys), _t(vals)
        k = RadixSortKernel(keys=kt, values=vt, count=n, bit_count=bits, radix_bits=radix_bits)
        k.dispatch()
        assert k.device_errors() == 0
        assert (_np(kt) == ek).all() and (_np(vt) == ev).all(), (radix_bits, bits)
        k.destroy()


def _dup_pattern(kind: str, n: int, seed: int) -> np.ndarray:
    """Duplicate-heavy key layouts that drive the run-counting ranks (rs_kernels.hpp, LDS
    counters under duplicate-heavy keys): runs of equal keys, the same digit recurring in
    separate runs of one 64-lane slot, sorted keys with repeats, few distinct keys."""
    u = O.gen_u32(seed, n)
    idx = np.arange(n, dtype=np.int64)
    if kind.startswith("runs"):
        r = int(kind[4:])
        return u[idx // r]
    if kind == "recurring":     # runs of 5 drawn from 6 values: one digit in several runs per slot
        pool = O.gen_u32(seed + 1, 6)
        return pool[(u[idx // 5] % np.uint32(6)).astype(np.int64)]
    if kind == "sorted_repeats":
        return np.sort(u[idx // 16])
    if kind == "two_values":
        return np.where(u & np.uint32(1), np.uint32(0xDEADBEEF), np.uint32(0x0000BEEF)).astype(np.uint32)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["runs2", "runs7", "runs16", "runs64", "runs100", "recurring",
                                  "sorted_repeats", "two_values"])
def test_duplicate_heavy_keys_every_layout(kind):
    """Run-counting ranks and counts give the oracle's stable order for duplicate-heavy inputs,
    on the one-sweep path, the histogram path (keys only) and the small-tile path; values are a
    permutation so stability is checked word for word."""
    from radix_sort_amd import RadixSortKernel, RadixSortTextureKernel
    for n in (3_000_017, 13_000_001):
        keys = _dup_pattern(kind, n, n + len(kind))
        vals = np.arange(n, dtype=np.uint32)
        ek, ev = O.stable_sort_masked(keys, vals, 32)
        kt, vt = _t(keys), _t(vals)
        k = RadixSortKernel(keys=kt, values=vt, count=n)
        k.dispatch()
        assert k.device_errors() == 0
        assert (_np(kt) == ek).all() and (_np(vt) == ev).all(), (kind, n)
        k.destroy()
        kt = _t(keys)
        k = RadixSortKernel(keys=kt, count=n)
        k.dispatch()
        assert (_np(kt) == ek).all(), (kind, n, "keys only")
        k.destroy()
        rt = _t(np.stack([keys, vals], axis=-1).reshape(-1)).view(-1, 2)
        k = RadixSortTextureKernel(texture=rt, count=n)
        k.dispatch()
        assert k.device_errors() == 0
        out = _np(rt).reshape(-1, 2)
        assert (out[:, 0] == ek).all() and (out[:, 1] == ev).all(), (kind, n, "aos")
        k.destroy()
