"""CPU: the presorted path's order-probe sample positions (rs_presorted.hpp k_ns_probe).

Round 5 jittered sample i inside its stride with ((hash(i) >> 8) % step).  Both operands are below
2^24, and the compiler expanded that remainder into its float-reciprocal 24-bit form: for some
(hash, step) pairs the estimated quotient came out one too large, the remainder negative, and the
24-bit mask turned it into ~2^24 - a sample position up to 16M keys past the array (a GPU memory
fault whenever that address was unmapped; the seeded search in test_presorted_gpu.py hit it at
n = 15753718).  The probe now takes the jitter as the high word of hash * step, which is in
[0, step) by construction.  These tests pin both facts: the new positions are in range for every
size, and the float expansion of the old expression does overflow at the sizes the GPU faulted on.
"""
import numpy as np
import pytest

PROBE = 16384


def new_positions(n: int) -> np.ndarray:
    step = (n - 1) // PROBE
    i = np.arange(PROBE, dtype=np.uint64)
    h = (i * np.uint64(0x9E3779B9)) & np.uint64(0xFFFFFFFF)
    jit = (h * np.uint64(step)) >> np.uint64(32)
    return i * np.uint64(step) + jit


def old_positions_as_compiled(n: int) -> np.ndarray:
    """((h >> 8) % step) through the compiler's 24-bit expansion: q = trunc(fa * rcp(fb)), one
    correction step up, remainder a - q * b masked to 24 bits."""
    step = (n - 1) // PROBE
    i = np.arange(PROBE, dtype=np.uint64)
    jit = (((i * np.uint64(0x9E3779B9)) & np.uint64(0xFFFFFFFF)) >> np.uint64(8)).astype(np.int64)
    fa = jit.astype(np.float32)
    fb = np.float32(step)
    fq = np.trunc(fa * (np.float32(1.0) / fb)).astype(np.float32)
    fr = fa.astype(np.float64) - fq.astype(np.float64) * float(fb)
    q = fq.astype(np.int64) + (np.abs(fr) >= float(fb)).astype(np.int64)
    rem = (jit - q * step) & 0xFFFFFF
    return i.astype(np.int64) * step + rem


@pytest.mark.parametrize("n", [12 << 20, (12 << 20) + 5, 12866813, 14447713, 15753718, 16394721,
                               (1 << 24) + 4099, (1 << 25) + 3, 1 << 28, (1 << 31) + 11, (1 << 32) - 1])
def test_probe_positions_in_range(n):
    p = new_positions(n)
    assert int(p.max()) + 1 <= n - 1          # every sampled pair (p, p + 1) lies in the array
    step = (n - 1) // PROBE
    assert (p // np.uint64(step) == np.arange(PROBE, dtype=np.uint64)).all()   # one per stride


def test_old_remainder_overflowed_where_the_gpu_faulted():
    p = old_positions_as_compiled(15753718)
    assert int(p.max()) >= 15753718               # past the array (the fault)
    assert int(old_positions_as_compiled(1 << 28).max()) < (1 << 28)   # why round 5's tests passed
