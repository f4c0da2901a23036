"""GPU parity of the interleaved (key, value) layout - RadixSortTextureKernel semantics.

Reference: src/kernels/radix-sort/RadixSortTextureKernel.ts:15-35 (always has values, :27-29),
rg32uint texel accessors RadixSortReorder.ts:42-63 / RadixSort.ts:24-48 (texel i = (i % width,
i / width)).  Same closed form as the buffer kernel: stable sort of the records by
(key & (2^bit_count - 1)); texels at index >= count untouched.  Bar: bit-exact vs the oracle.
"""
import numpy as np
import pytest

import oracle as O
from conftest import case_arrays

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _records(keys, vals):
    return np.stack([keys, vals], axis=-1).astype(np.uint32)


def _sort_tex(rec: np.ndarray, count=None, **opts) -> np.ndarray:
    from radix_sort_amd import RadixSortTextureKernel
    t = torch.from_numpy(np.ascontiguousarray(rec).view(np.int32)).to(DEV)
    k = RadixSortTextureKernel(device=0, data={"texture": t}, count=count, **opts)
    k.dispatch()
    torch.cuda.synchronize()
    out = t.cpu().numpy().view(np.uint32)
    k.destroy()
    return out


def _expect(keys, vals, bits, count=None):
    ek, ev = O.stable_sort_masked(keys, vals, bits, count)
    return _records(ek, ev)


def test_texture_golden_cases(golden):
    manifest, arrays = golden
    for case in manifest["sort_cases"]:
        keys, vals, _, _ = case_arrays(arrays, case)
        if vals is None:
            vals = np.arange(keys.size, dtype=np.uint32)
        rec = _records(keys, vals)
        out = _sort_tex(rec, case["count"], bit_count=case["bit_count"])
        assert (out == _expect(keys, vals, case["bit_count"], case["count"])).all(), case


@pytest.mark.parametrize("n", [2, 1000, 16_384, 16_385, 100_003, 1 << 20, 13_000_001])
@pytest.mark.parametrize("bits", [32, 20])
def test_texture_random_sizes(n, bits):
    keys = O.gen_u32(n + 11 * bits, n)
    vals = O.gen_u32(n + 12 * bits, n)            # arbitrary values, not iota
    out = _sort_tex(_records(keys, vals), bit_count=bits)
    assert (out == _expect(keys, vals, bits)).all(), (n, bits)


@pytest.mark.parametrize("radix_bits", [2, 4])
def test_texture_reference_pass_structure(radix_bits):
    n = 200_001
    keys = O.gen_u32(9, n) % np.uint32(1 << 16)
    vals = np.arange(n, dtype=np.uint32)
    out = _sort_tex(_records(keys, vals), bit_count=16, radix_bits=radix_bits)
    assert (out == _expect(keys, vals, 16)).all()


def test_texture_2d_shape_and_untouched_tail():
    h, w = 300, 512                                 # a [height, width] rg32uint texture
    n = h * w
    count = n - 4321
    keys = O.gen_u32(21, n)
    vals = O.gen_u32(22, n)
    rec = _records(keys, vals).reshape(h, w, 2)
    out = _sort_tex(rec, count).reshape(-1, 2)
    exp = _expect(keys, vals, 32, count)
    assert (out == exp).all()
    assert (out[count:] == _records(keys, vals)[count:]).all()


@pytest.mark.parametrize("kind", ["sorted", "sorted_after_first_pass", "reverse"])
def test_texture_check_order(kind):
    n = 1 << 20
    u = O.gen_u32(31, n)
    keys = {"sorted": np.sort(u), "sorted_after_first_pass": u & np.uint32(0x3F),
            "reverse": np.sort(u)[::-1].copy()}[kind]
    vals = np.arange(n, dtype=np.uint32)
    out = _sort_tex(_records(keys, vals), check_order=True)
    assert (out == _expect(keys, vals, 32)).all(), kind


@pytest.mark.parametrize("rank", ["atomic", "ballot"])
@pytest.mark.parametrize("tile", ["small", "large"])
def test_texture_rank_modes_and_tiles(plan_debug, rank, tile):
    plan_debug(rank=rank, tile=tile)
    for n, bits in ((40_000, 32), (1_000_003, 24), (5_000, 8)):
        keys = O.gen_u32(n + bits, n)
        vals = np.arange(n, dtype=np.uint32)
        out = _sort_tex(_records(keys, vals), bit_count=bits)
        assert (out == _expect(keys, vals, bits)).all(), (n, bits)


def test_texture_plan_rejects_separate_values():
    import ctypes
    from radix_sort_amd import _lib
    L = _lib.load()
    d = _lib.PlanDesc(0, 1000, 32, 16, 16, _lib.RS_FLAG_INTERLEAVED, 0, 0)
    plan = ctypes.c_void_p()
    assert L.rs_plan_create(ctypes.byref(d), ctypes.byref(plan)) == _lib.RS_OK
    t = torch.zeros(2000, dtype=torch.int32, device=DEV)
    v = torch.zeros(1000, dtype=torch.int32, device=DEV)
    assert L.rs_plan_sort(plan, t.data_ptr(), v.data_ptr(), None) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_plan_sort(plan, t.data_ptr() + 4, None, None) == _lib.RS_ERR_INVALID_ARG  # 8-B align
    assert L.rs_plan_sort(plan, t.data_ptr(), None, None) == _lib.RS_OK
    torch.cuda.synchronize()
    L.rs_plan_destroy(plan)


@pytest.mark.slow
def test_texture_256M_records_properties():
    """BASELINE size with the AoS layout: 2^28 (key, iota) records; sorted by key, values a
    permutation, records intact (key == input key at its value), stable."""
    from radix_sort_amd import RadixSortTextureKernel, ops
    n = 1 << 28
    rec = torch.empty((n, 2), dtype=torch.int32, device=DEV)
    keys_in = torch.empty(n, dtype=torch.int32, device=DEV)
    ops.fill_random_u32(keys_in, seed=3)
    rec[:, 0] = keys_in
    rec[:, 1] = torch.arange(n, dtype=torch.int32, device=DEV)
    k = RadixSortTextureKernel(texture=rec, count=n)
    k.dispatch()
    torch.cuda.synchronize()
    ko = rec[:, 0].contiguous()
    vo = rec[:, 1].contiguous()
    assert ops.is_sorted(ko, n)
    kl = ko.to(torch.int64) & 0xFFFFFFFF
    vl = vo.to(torch.int64)
    assert torch.equal(torch.bincount(vl, minlength=n), torch.ones(n, dtype=torch.long, device=DEV))
    assert torch.equal(keys_in[vo.long()], ko)
    same = kl[1:] == kl[:-1]
    assert bool((vl[1:][same] > vl[:-1][same]).all())
    k.destroy()
