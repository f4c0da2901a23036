"""CPU: pin the oracle restatements against the golden fixtures (the reference test's own
expected-value expressions evaluated in Node, example/tests.ts:86-95,288-296)."""
import hashlib

import numpy as np
import pytest

import oracle as O
from conftest import case_arrays


def test_generator_numpy_matches_c():
    for seed in (0, 1, 2**40 + 7):
        assert (O.gen_u32(seed, 5000) == O.gen_u32_c(seed, 5000)).all()
    # counter-based: a window equals the tail of a longer stream
    assert (O.gen_u32(9, 100, start=50) == O.gen_u32(9, 150)[50:]).all()


def test_sort_restatements_match_golden(golden):
    manifest, arrays = golden
    assert len(manifest["sort_cases"]) >= 60
    for case in manifest["sort_cases"]:
        keys, vals, exp_k, exp_v = case_arrays(arrays, case)
        for fn in (O.stable_sort_masked, O.stable_sort_masked_c):
            k, v = fn(keys, vals, case["bit_count"], case["count"])
            assert (k == exp_k).all(), case["name"]
            if vals is not None:
                assert (v == exp_v).all(), case["name"]
        # the literal per-pass WGSL restatement, at several workgroup sizes / local shuffle
        for T, ls in ((4, False), (64, True), (256, False)):
            k, v = O.radix_sort_literal(keys, vals, case["bit_count"], T, ls, case["count"])
            assert (k == exp_k).all(), (case["name"], T, ls)
            if vals is not None:
                assert (v == exp_v).all(), (case["name"], T, ls)


def test_golden_values_satisfy_reference_value_check(golden):
    # example/tests.ts:94: keysResult[i] == keys[values[i]]
    manifest, arrays = golden
    for case in manifest["sort_cases"]:
        keys, vals, exp_k, exp_v = case_arrays(arrays, case)
        if vals is None:
            continue
        c = case["count"]
        assert (keys[exp_v[:c]] == exp_k[:c]).all()
        assert (exp_k[c:] == keys[c:]).all()  # words past count untouched


def test_large_cases_sha(golden):
    manifest, _ = golden
    for case in manifest["large_cases"]:
        n, seed = case["n"], case["seed"]
        u = O.gen_u32(seed, n)
        if case["kind"] == "f32":
            u = ((u >> np.uint32(8)).astype(np.float64) * 2.0 ** -24).astype(np.float32).view(np.uint32)
        vals = np.arange(n, dtype=np.uint32) if case["has_values"] else None
        k, v = O.stable_sort_masked_c(u, vals, 32)
        assert hashlib.sha256(k.tobytes()).hexdigest() == case["sha256_keys"]
        if vals is not None:
            assert hashlib.sha256(v.tobytes()).hexdigest() == case["sha256_values"]


def test_prefix_sum_restatements(golden):
    manifest, arrays = golden
    for case in manifest["scan_cases"]:
        d, exp = arrays[case["name"] + "_data"], arrays[case["name"] + "_exp"]
        assert (O.prefix_sum(d, case["count"]) == exp).all()
        for T in (1, 16, 256):
            assert (O.prefix_sum_blelloch(d, case["count"], T) == exp).all()


@pytest.mark.parametrize("bits", [4, 8, 12, 20, 28, 32])
def test_literal_vs_closed_form_random(bits):
    rng = np.random.default_rng(bits)
    for n in (1, 7, 300, 5000):
        keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        keys[rng.integers(0, n, n // 3)] = keys[0]  # duplicates
        vals = np.arange(n, dtype=np.uint32)
        a = O.radix_sort_literal(keys, vals, bits, 16, local_shuffle=True)
        b = O.stable_sort_masked(keys, vals, bits)
        assert (a[0] == b[0]).all() and (a[1] == b[1]).all()


def test_oracle_argument_errors():
    with pytest.raises(ValueError):
        O.radix_sort_literal(np.zeros(4, np.uint32), None, 32, 12)   # non pow2 (PrefixSumKernel.ts:33-35)
    with pytest.raises(ValueError):
        O.radix_sort_literal(np.zeros(4, np.uint32), None, 30, 16)   # bit_count % 4 (README.md:97)


def test_verify_stable_iota_detects_violations():
    keys = O.gen_u32(5, 1000) % np.uint32(10)
    vals = np.arange(1000, dtype=np.uint32)
    k, v = O.stable_sort_masked(keys, vals)
    assert O.verify_stable_iota(keys, k, v) == 0
    v2 = v.copy()
    i = int(np.nonzero(k[1:] == k[:-1])[0][0])
    v2[i], v2[i + 1] = v2[i + 1], v2[i]
    assert O.verify_stable_iota(keys, k, v2) != 0  # stability broken
    k2 = k.copy()
    k2[0], k2[-1] = k2[-1], k2[0]
    assert O.verify_stable_iota(keys, k2, v) != 0


def test_nearly_sorted_generator_has_interior_inversions():
    bits = O.nearly_sorted_f32_bits(100000, 4)
    inv = np.nonzero(bits[:-1] > bits[1:])[0]
    assert inv.size > 0 and (inv < bits.size - 2).any()   # never only the last pair (Q1)
