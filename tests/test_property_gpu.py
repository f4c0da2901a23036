"""Property-test harness: the reference's randomised test matrix, seeded, plus a hypothesis
search over the option space.  Everything runs through the C ABI and is compared bit-exactly
with the oracle (oracle.stable_sort_masked / oracle.prefix_sum).

* test_reference_radix_sort_matrix ports testRadixSort (example/tests.ts:9-107): every
  workgroup size x, y in {2..256} with x*y <= 1024 (:18-25), element counts 10^exp * U(0.9, 1)
  for exp 2..7 (:27-29), a random sub-count (:30), random 32-bit keys (:33-35), values = iota,
  random checkOrder / localShuffle / avoidBankConflicts (:39-41), keys-only and keys+values.
  The reference's Math.random becomes numpy's seeded generator; 10^7-element cases run for
  every fourth workgroup size to keep the suite short.
* test_reference_prefix_sum_matrix ports test_prefix_sum (example/tests.ts:110-182): sizes
  {1..256}^2 with x*y <= 1024, data in [0, 8), random sub-count.
* test_hypothesis_option_space: n, count <= n, bit_count, radix_bits, flags, layout (keys,
  separate values, interleaved records) and key distribution drawn by hypothesis
  (derandomized, so the examples are the same every run).
"""
import numpy as np
import pytest

import oracle as O

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _t(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(DEV)


def _np(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint32)


def _workgroup_sizes(sizes):
    return [(x, y) for x in sizes for y in sizes if x * y <= 1024]


@pytest.mark.parametrize("keys_and_values", [False, True])
def test_reference_radix_sort_matrix(keys_and_values):
    from radix_sort_amd import RadixSortBufferKernel
    rng = np.random.default_rng(20250404 + keys_and_values)
    wgs = _workgroup_sizes([2, 4, 8, 16, 32, 64, 128, 256])
    cases = 0
    for wi, (wx, wy) in enumerate(wgs):
        for exp in range(2, 8):
            if exp == 7 and wi % 4:
                continue
            n = int(10 ** exp * (rng.random() * 0.1 + 0.9))
            count = int(n * rng.random() + 1)
            keys = np.ceil(rng.random(n) * (2.0 ** 32 - 1)).astype(np.uint64).astype(np.uint32)
            values = np.arange(n, dtype=np.uint32)
            check_order, local_shuffle, avoid = (bool(b) for b in rng.random(3) > 0.5)
            kt = _t(keys)
            vt = _t(values) if keys_and_values else None
            k = RadixSortBufferKernel(device=0, data={"keys": kt, "values": vt}, count=count,
                                      bitCount=32, workgroupSize={"x": wx, "y": wy},
                                      checkOrder=check_order, localShuffle=local_shuffle,
                                      avoidBankConflicts=avoid)
            k.dispatch()
            torch.cuda.synchronize()
            ek, ev = O.stable_sort_masked(keys, values, 32, count)
            ko = _np(kt)
            assert (ko == ek).all(), (n, count, wx, wy, check_order, local_shuffle, avoid)
            if keys_and_values:
                vo = _np(vt)
                assert (vo == ev).all(), (n, count, wx, wy)
                assert (ko[:count] == keys[vo[:count]]).all()       # tests.ts:94
            k.destroy()
            cases += 1
    assert cases > 200


def test_reference_prefix_sum_matrix():
    from radix_sort_amd import PrefixSumKernel
    rng = np.random.default_rng(110)
    for wi, (wx, wy) in enumerate(_workgroup_sizes([1, 2, 4, 8, 16, 32, 64, 128, 256])):
        for exp in range(2, 8):
            if exp == 7 and wi % 4:
                continue
            n = int(10 ** exp * (rng.random() * 0.1 + 0.9))
            count = int(n * rng.random() + 1)
            data = np.floor(rng.random(n) * 8).astype(np.uint32)
            t = _t(data)
            k = PrefixSumKernel(device=0, data=t, count=count, workgroupSize={"x": wx, "y": wy},
                                avoidBankConflicts=False)
            k.dispatch()
            torch.cuda.synchronize()
            assert (_np(t) == O.prefix_sum(data, count)).all(), (n, count, wx, wy)
            k.destroy()


hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

_DISTS = ("uniform", "few", "sorted", "reverse", "equal", "high_bits", "f32")


def _keys(dist: str, n: int, seed: int) -> np.ndarray:
    u = O.gen_u32(seed, n)
    if dist == "few":
        return u % np.uint32(7)
    if dist == "sorted":
        return np.sort(u)
    if dist == "reverse":
        return np.sort(u)[::-1].copy()
    if dist == "equal":
        return np.full(n, u[0] if n else 0, dtype=np.uint32)
    if dist == "high_bits":          # only bits above bit_count vary: a no-op sort
        return u & np.uint32(0xFFF00000)
    if dist == "f32":                # non-negative floats, sorted by raw bits (README.md:9)
        return ((u >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)).view(np.uint32)
    return u


@settings(max_examples=300, deadline=None, derandomize=True, database=None)
@given(n=st.one_of(st.integers(0, 70_000), st.integers(70_000, 1_500_000)),
       count_frac=st.floats(0.0, 1.0),
       bit_count=st.sampled_from([4, 8, 12, 16, 20, 24, 28, 32]),
       radix_bits=st.sampled_from([0, 2, 4, 8]),
       layout=st.sampled_from(["keys", "soa", "aos"]),
       check_order=st.booleans(), local_shuffle=st.booleans(),
       dist=st.sampled_from(_DISTS), seed=st.integers(0, 2 ** 31))
def test_hypothesis_option_space(n, count_frac, bit_count, radix_bits, layout, check_order,
                                 local_shuffle, dist, seed):
    from radix_sort_amd import RadixSortKernel, RadixSortTextureKernel
    keys = _keys(dist, n, seed)
    values = O.gen_u32(seed + 1, n)
    count = min(n, int(round(n * count_frac)))
    ek, ev = O.stable_sort_masked(keys, values, bit_count, count)
    opts = dict(count=count, bit_count=bit_count, radix_bits=radix_bits, check_order=check_order)
    if layout == "aos":
        rec = np.stack([keys, values], axis=-1) if n else np.zeros((0, 2), np.uint32)
        t = _t(rec.reshape(-1)).view(-1, 2) if n else torch.zeros((1, 2), dtype=torch.int32, device=DEV)
        k = RadixSortTextureKernel(device=0, texture=t, **opts)
        k.dispatch()
        torch.cuda.synchronize()
        out = _np(t).reshape(-1, 2)[:n]
        assert (out[:, 0] == ek).all() and (out[:, 1] == ev).all()
    else:
        kt = _t(keys) if n else torch.zeros(1, dtype=torch.int32, device=DEV)
        vt = (_t(values) if n else torch.zeros(1, dtype=torch.int32, device=DEV)) if layout == "soa" else None
        k = RadixSortKernel(device=0, keys=kt, values=vt, local_shuffle=local_shuffle, **opts)
        k.dispatch()
        torch.cuda.synchronize()
        assert (_np(kt)[:n] == ek).all()
        if vt is not None:
            assert (_np(vt)[:n] == ev).all()
    k.destroy()
