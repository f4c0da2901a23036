"""GPU: the presorted path of check_order sorts (rs_presorted.hpp; rsort.hip enqueue_presorted).
Nearly-sorted input (BASELINE config 4: sorted f32 keys with n/1000 transpositions) is sorted by
marking the displaced keys, sorting those and merging them back, instead of the radix passes; any
input the device finds unsuited goes through the hybrid radix path as before.  Either way the
result must be the stable sort, bit-exact against the oracle (values = input index, so the merge's
(key, position) order is checked too), on all three layouts: separate arrays, keys only, records
in place.  The path the device chose is read back (rs_plan_last_path)."""
import numpy as np
import pytest
import torch

import oracle as O
from radix_sort_amd import RadixSortKernel, RadixSortTextureKernel

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
N = (1 << 24) + 4099          # over the hybrid path's 12M minimum; a partial last tile


def _rng(seed):
    return np.random.default_rng(seed)


def _input(kind, n, seed=11):
    r = _rng(seed)
    if kind == "f32_nearly":                  # config 4's generator at this size
        return O.nearly_sorted_f32_bits(n, seed)
    if kind == "random":
        return O.gen_u32_c(seed, n)
    base = np.sort(O.gen_u32_c(seed, n))
    if kind == "sorted":
        return base
    if kind == "adjacent_swaps":              # one descent each
        i = r.choice(n - 1, 1000, replace=False)
        base[i], base[i + 1] = base[i + 1].copy(), base[i].copy()
        return base
    if kind == "tile_boundaries":             # inversions across the 4096-key tiles' edges
        t = np.arange(1, (n - 2) // 4096) * 4096
        base[t - 1], base[t] = base[t].copy(), base[t - 1].copy()
        base[t - 2], base[t + 1] = base[t + 1].copy(), base[t - 2].copy()
        return base
    if kind == "dups_swaps":                  # few distinct keys: the merge's ties by position
        base = np.sort(O.gen_u32_c(seed, n) % np.uint32(5000))
        a, b = r.integers(0, n, 3000), r.integers(0, n, 3000)
        for x, y in zip(a.tolist(), b.tolist()):
            base[x], base[y] = base[y], base[x]
        return base
    if kind == "far_moves":                   # elements taken out and put back far away
        sel = np.sort(r.choice(n, 400, replace=False))
        moved = base[sel]
        rest = np.delete(base, sel)
        pos = np.sort(r.integers(0, rest.size + 1, moved.size))
        return np.insert(rest, pos, r.permutation(moved))
    if kind == "rotated_blocks":              # chains: every rotated 8-key block needs rounds
        for s in r.choice(n - 16, 300, replace=False).tolist():
            base[s:s + 8] = np.roll(base[s:s + 8], 3)
        return base
    if kind == "reversed_blocks":             # 100-key runs: marked whole, may reach a tile's halo
        for s in r.choice(n - 200, 30, replace=False).tolist():
            base[s:s + 100] = base[s:s + 100][::-1].copy()
        return base
    if kind == "many_swaps":                  # n / 50 transpositions: over the extraction
        a, b = r.integers(0, n, n // 50), r.integers(0, n, n // 50)
        base[a], base[b] = base[b].copy(), base[a].copy()
        return base
    raise ValueError(kind)


# the device's choice: the presorted path for the nearly-sorted kinds, the radix path (or the
# early exit) otherwise; reversed_blocks may go either way (a marked run that reaches a halo)
EXPECT = {"f32_nearly": "presorted", "adjacent_swaps": "presorted", "tile_boundaries": "presorted",
          "dups_swaps": "presorted", "far_moves": "presorted", "rotated_blocks": "presorted",
          "reversed_blocks": None, "many_swaps": "hybrid", "random": "hybrid", "sorted": "in_order"}


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32).copy()).to(DEV)


def _np(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("kind", list(EXPECT))
def test_presorted_kinds_all_layouts(kind):
    keys = _input(kind, N)
    vals = np.arange(N, dtype=np.uint32)
    ek, ev = O.stable_sort_masked_c(keys, vals, 32)
    want = EXPECT[kind]
    # separate arrays
    kt, vt = _t(keys), _t(vals)
    kern = RadixSortKernel(keys=kt, values=vt, count=N, check_order=True)
    kern.set_profiling(True)
    kern.dispatch()
    kern.check()
    path = kern.last_path()
    times = kern.kernel_times()
    kern.destroy()
    assert np.array_equal(_np(kt), ek) and np.array_equal(_np(vt), ev), (kind, path)
    if want:
        assert path == want, (kind, path)
    assert times["presorted"]["launches"] >= 1       # enqueued on every check_order hybrid sort
    if path == "presorted":                          # no radix pass ran
        assert times["bucket"]["launches"] >= 1      # (enqueued, gated off on the device)
    # keys only
    kt = _t(keys)
    kern = RadixSortKernel(keys=kt, count=N, check_order=True)
    kern.dispatch()
    kern.check()
    p2 = kern.last_path()
    kern.destroy()
    assert np.array_equal(_np(kt), ek), (kind, "keys only", p2)
    if want:   # (keys only at this size: the LSD passes, whose early exit reports "lsd")
        assert p2 == want or (want != "presorted" and p2 == "lsd"), (kind, "keys only", p2)
    # records in place
    rt = _t(np.stack([keys, vals], axis=-1).reshape(-1)).view(-1, 2)
    kern = RadixSortTextureKernel(texture=rt, count=N, check_order=True)
    kern.dispatch()
    kern.check()
    p3 = kern.last_path()
    kern.destroy()
    out = _np(rt).reshape(-1, 2)
    assert np.array_equal(out[:, 0], ek) and np.array_equal(out[:, 1], ev), (kind, "records", p3)
    if want:
        assert p3 == want, (kind, "records", p3)


def test_presorted_off_and_second_dispatch(plan_debug):
    """rs_plan_debug.presorted = 0 keeps the radix path for nearly-sorted input; with it on, a
    second dispatch of the (now sorted) data exits early and moves nothing."""
    keys = _input("f32_nearly", N, seed=3)
    vals = np.arange(N, dtype=np.uint32)
    ek, ev = O.stable_sort_masked_c(keys, vals, 32)
    plan_debug(presorted=0)
    kt, vt = _t(keys), _t(vals)
    kern = RadixSortKernel(keys=kt, values=vt, count=N, check_order=True)
    kern.dispatch()
    kern.check()
    assert kern.last_path() == "hybrid"
    kern.destroy()
    assert np.array_equal(_np(kt), ek) and np.array_equal(_np(vt), ev)
    plan_debug(presorted=1)
    kt, vt = _t(keys), _t(vals)
    kern = RadixSortKernel(keys=kt, values=vt, count=N, check_order=True)
    kern.dispatch()
    kern.check()
    assert kern.last_path() == "presorted"
    assert np.array_equal(_np(kt), ek) and np.array_equal(_np(vt), ev)
    kern.dispatch()
    kern.check()
    assert kern.last_path() == "in_order"
    assert np.array_equal(_np(kt), ek) and np.array_equal(_np(vt), ev)
    # and unsorted data again on the same plan: the radix path
    kt.copy_(_t(O.gen_u32_c(9, N)))
    k_in = _np(kt)
    kern.dispatch()
    kern.check()
    assert kern.last_path() == "hybrid"
    assert np.array_equal(_np(kt), O.stable_sort_masked_c(k_in, None, 32)[0])
    kern.destroy()


@pytest.mark.parametrize("bits", [32, 28])
def test_presorted_on_the_lsd_path_with_bit_count(plan_debug, bits):
    """The LSD passes' check_order sorts run the presorted path too (here the hybrid path off, and
    bit_count < 32, where the order is that of the masked keys: the bits above are carried along)."""
    r = _rng(bits)
    mask = np.uint32((1 << bits) - 1 if bits < 32 else 0xFFFFFFFF)
    low = np.sort(O.gen_u32_c(5, N) & mask)
    keys = low | (r.integers(0, 1 << 32, N, dtype=np.uint64).astype(np.uint32) & ~mask)
    a, b = r.integers(0, N, N // 1000), r.integers(0, N, N // 1000)
    for x, y in zip(a.tolist(), b.tolist()):
        keys[x], keys[y] = keys[y], keys[x]
    vals = np.arange(N, dtype=np.uint32)
    ek, ev = O.stable_sort_masked_c(keys, vals, bits)
    plan_debug(msd=0)
    kt, vt = _t(keys), _t(vals)
    kern = RadixSortKernel(keys=kt, values=vt, count=N, check_order=True, bit_count=bits)
    kern.dispatch()
    kern.check()
    assert kern.last_path() == "presorted"
    kern.destroy()
    assert np.array_equal(_np(kt), ek) and np.array_equal(_np(vt), ev)


# ---- seeded randomized search (round 6) --------------------------------------------------------
# Beyond the hand-made shapes above: every case draws its size (>= the 12M-key minimum of the path),
# bit_count, duplicate ratio and a mix of perturbations (transpositions near and far, reversed and
# rotated runs of 2-300 keys) at a density from n / 10^5 to n / 50, then sorts it on all three
# layouts, compared word for word with the oracle's stable sort.  Both outcomes of the device's
# decision are exercised: low densities take the presorted path, high ones the radix path.
def _random_nearly(seed: int):
    r = _rng(1000 + seed)
    n = int(r.integers(12 << 20, 17 << 20)) | int(r.integers(0, 2))   # odd sizes too
    bits = int(r.choice([16, 28, 32]))
    mask = np.uint32((1 << bits) - 1 if bits < 32 else 0xFFFFFFFF)
    distinct = int(r.choice([n, n // 10, 1000, 3]))
    pool = np.sort(O.gen_u32_c(seed, distinct) & mask)
    keys = np.sort(pool[r.integers(0, distinct, n)])                  # sorted masked keys, duplicates
    if bits < 32:   # bits above the mask: carried along, ignored by the order (random)
        keys |= r.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32) & ~mask
    density = float(np.exp(r.uniform(np.log(1e-5), np.log(1 / 50))))
    ops = max(1, int(n * density))
    kinds = r.integers(0, 4, ops)
    for kind, at in zip(kinds.tolist(), r.integers(0, n - 301, ops).tolist()):
        ln = int(r.integers(2, 301))
        if kind == 0:                                   # transposition at distance 1..300
            b = at + ln - 1
            keys[at], keys[b] = keys[b], keys[at]
        elif kind == 1:                                 # far transposition
            b = int(r.integers(0, n))
            keys[at], keys[b] = keys[b], keys[at]
        elif kind == 2:                                 # reversed run
            keys[at:at + ln] = keys[at:at + ln][::-1].copy()
        else:                                           # rotated run
            keys[at:at + ln] = np.roll(keys[at:at + ln], int(r.integers(1, ln)))
    return n, bits, density, keys


def test_presorted_seeded_random_search():
    paths = []
    for seed in range(10):
        n, bits, density, keys = _random_nearly(seed)
        vals = np.arange(n, dtype=np.uint32)
        ek, ev = O.stable_sort_masked_c(keys, vals, bits)
        tag = (seed, n, bits, round(density * n))
        kt, vt = _t(keys), _t(vals)
        kern = RadixSortKernel(keys=kt, values=vt, count=n, check_order=True, bit_count=bits)
        kern.dispatch()
        kern.check()
        paths.append(kern.last_path())
        kern.destroy()
        assert np.array_equal(_np(kt), ek) and np.array_equal(_np(vt), ev), (tag, paths[-1])
        del kt, vt
        kt = _t(keys)
        kern = RadixSortKernel(keys=kt, count=n, check_order=True, bit_count=bits)
        kern.dispatch()
        kern.check()
        kern.destroy()
        assert np.array_equal(_np(kt), ek), (tag, "keys only")
        del kt
        rt = _t(np.stack([keys, vals], axis=-1).reshape(-1)).view(-1, 2)
        kern = RadixSortTextureKernel(texture=rt, count=n, check_order=True, bit_count=bits)
        kern.dispatch()
        kern.check()
        kern.destroy()
        out = _np(rt).reshape(-1, 2)
        assert np.array_equal(out[:, 0], ek) and np.array_equal(out[:, 1], ev), (tag, "records")
        del rt
    print("paths:", paths)
    # the search reaches both sides of the device's decision
    assert paths.count("presorted") >= 3 and len(set(paths) - {"presorted"}) >= 1, paths


@pytest.mark.parametrize("n", [15753718, (12 << 20) + 5, 14447713])
def test_presorted_at_sizes_where_the_probe_overflowed(n):
    """Sizes at which round 5's probe sampled past the array (tests/test_presorted_probe.py): the
    nearly-sorted path on all three layouts, word for word against the oracle."""
    keys = O.nearly_sorted_f32_bits(n, 5)
    vals = np.arange(n, dtype=np.uint32)
    ek, ev = O.stable_sort_masked_c(keys, vals, 32)
    kt, vt = _t(keys), _t(vals)
    kern = RadixSortKernel(keys=kt, values=vt, count=n, check_order=True)
    kern.dispatch()
    kern.check()
    assert kern.last_path() == "presorted"
    kern.destroy()
    assert np.array_equal(_np(kt), ek) and np.array_equal(_np(vt), ev)
    kt = _t(keys)
    kern = RadixSortKernel(keys=kt, count=n, check_order=True)
    kern.dispatch()
    kern.check()
    kern.destroy()
    assert np.array_equal(_np(kt), ek)
    rt = _t(np.stack([keys, vals], axis=-1).reshape(-1)).view(-1, 2)
    kern = RadixSortTextureKernel(texture=rt, count=n, check_order=True)
    kern.dispatch()
    kern.check()
    kern.destroy()
    out = _np(rt).reshape(-1, 2)
    assert np.array_equal(out[:, 0], ek) and np.array_equal(out[:, 1], ev)
