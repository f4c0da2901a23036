"""CPU oracle for the 4-way LSD radix sort — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker (or the timed CPU baseline).  The product package
(``webgpu-radix-sort_amd/``) never imports it; its HIP path fails loudly when the extension is
missing instead of falling back here.

Two independent restatements of the reference semantics:

* ``radix_sort_literal`` — ctypes binding of ``rs_oracle.c``'s per-2-bit-pass emulation of the
  reference's WGSL passes (RadixSort.ts:56-125, RadixSortLocalShuffle.ts:94-116,
  PrefixSum.ts:13-106 + PrefixSumKernel.ts:45-133, RadixSortReorder.ts:86-101, ping-pong at
  AbstractRadixSortKernel.ts:93-107 / RadixSortBufferKernel.ts:73-85).
* ``stable_sort_masked`` — numpy closed form: ``argsort(keys & mask, kind="stable")``.

Parity pinning: the reference ships no golden vectors; its own test oracle is the JS expression
``keys.slice(0, count).sort((a, b) => a - b)`` (example/tests.ts:86) plus the value check
``keysResult[i] == keys[values[i]]`` (example/tests.ts:94) and ``prefixSumCpu``
(example/tests.ts:288-296).  ``tests/golden/gen_golden.py`` evaluates that expression in Node
here and commits the results; ``tests/test_oracle.py`` pins both restatements to them.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "librso.so")
_lib = None

MASK64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def build() -> str:
    """Compile rs_oracle.c into oracle/build/librso.so (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.rso_gen_u32.restype = ctypes.c_uint32
        L.rso_gen_u32.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.rso_fill_u32.restype = None
        L.rso_fill_u32.argtypes = [u32p, ctypes.c_uint64, ctypes.c_uint64]
        L.rso_prefix_sum_blelloch.restype = ctypes.c_int
        L.rso_prefix_sum_blelloch.argtypes = [u32p, ctypes.c_uint64, ctypes.c_uint32]
        L.rso_prefix_sum_seq.restype = None
        L.rso_prefix_sum_seq.argtypes = [u32p, ctypes.c_uint64]
        L.rso_radix_sort_literal.restype = ctypes.c_int
        L.rso_radix_sort_literal.argtypes = [u32p, u32p, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_int]
        L.rso_stable_sort_masked.restype = ctypes.c_int
        L.rso_stable_sort_masked.argtypes = [u32p, u32p, ctypes.c_uint64, ctypes.c_uint32]
        L.rso_is_sorted_masked.restype = ctypes.c_int
        L.rso_is_sorted_masked.argtypes = [u32p, ctypes.c_uint64, ctypes.c_uint32]
        L.rso_verify_stable_iota.restype = ctypes.c_int64
        L.rso_verify_stable_iota.argtypes = [u32p, u32p, u32p, ctypes.c_uint64, ctypes.c_uint32]
        _lib = L
    return _lib


def _ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.uint32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def mask_of(bit_count: int) -> np.uint32:
    return np.uint32(0xFFFFFFFF if bit_count >= 32 else (1 << bit_count) - 1)


# ---- synthetic inputs (identical to the HIP generator rs_fill_random_u32) ----------------

def gen_u32(seed: int, n: int, start: int = 0) -> np.ndarray:
    """key[i] = low32(splitmix64_finaliser(seed * 0xD1B54A32D192ED03 + i)), numpy-vectorised."""
    with np.errstate(over="ignore"):
        i = np.arange(start, start + n, dtype=np.uint64)
        z = np.uint64((seed * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF) + i
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def gen_u32_c(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint32)
    lib().rso_fill_u32(_ptr(out), n, seed)
    return out


def nearly_sorted_f32_bits(n: int, seed: int, swaps: int | None = None) -> np.ndarray:
    """Config-4 input: f32 keys in [0,1) sorted ascending, then perturbed by n//1000 random
    transpositions (applied in sequence), returned as raw u32 bits.  The last pair is never the
    only inversion (quirk Q1): position pairs come from the seeded generator."""
    u = gen_u32(seed, n)
    keys = ((u >> np.uint32(8)).astype(np.float64) * 2.0 ** -24).astype(np.float32)
    keys.sort(kind="stable")
    bits = keys.view(np.uint32).copy()
    if swaps is None:
        swaps = max(1, n // 1000)
    r = gen_u32(seed ^ 0x5EED, 2 * swaps).astype(np.uint64)
    a = (r[0::2] % np.uint64(n)).astype(np.int64)
    b = (r[1::2] % np.uint64(n)).astype(np.int64)
    for x, y in zip(a.tolist(), b.tolist()):
        bits[x], bits[y] = bits[y], bits[x]
    return bits


# ---- sort restatements -------------------------------------------------------------------

def stable_sort_masked(keys: np.ndarray, values: np.ndarray | None, bit_count: int = 32,
                       count: int | None = None):
    """Closed form: stable ascending sort of keys[:count] & mask; words at
    index >= count untouched.  Returns new (keys, values) arrays."""
    keys = np.ascontiguousarray(keys, dtype=np.uint32).copy()
    values = None if values is None else np.ascontiguousarray(values, dtype=np.uint32).copy()
    n = keys.size if count is None else count
    perm = np.argsort(keys[:n] & mask_of(bit_count), kind="stable")
    keys[:n] = keys[:n][perm]
    if values is not None:
        values[:n] = values[:n][perm]
    return keys, values


def stable_sort_masked_c(keys, values, bit_count=32, count=None):
    keys = np.ascontiguousarray(keys, dtype=np.uint32).copy()
    values = None if values is None else np.ascontiguousarray(values, dtype=np.uint32).copy()
    n = keys.size if count is None else count
    rc = lib().rso_stable_sort_masked(_ptr(keys), _ptr(values), n, bit_count)
    if rc:
        raise ValueError(f"rso_stable_sort_masked rc={rc}")
    return keys, values


def radix_sort_literal(keys, values, bit_count=32, workgroup=256, local_shuffle=False,
                       count=None):
    """Per-pass emulation of the reference's WGSL passes (rs_oracle.c)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint32).copy()
    values = None if values is None else np.ascontiguousarray(values, dtype=np.uint32).copy()
    n = keys.size if count is None else count
    rc = lib().rso_radix_sort_literal(_ptr(keys), _ptr(values), n, bit_count, workgroup,
                                      1 if local_shuffle else 0)
    if rc:
        raise ValueError(f"rso_radix_sort_literal rc={rc}")
    return keys, values


def prefix_sum(data: np.ndarray, count: int | None = None) -> np.ndarray:
    """Exclusive scan mod 2^32 of data[:count] (example/tests.ts:288-296); tail untouched."""
    out = np.ascontiguousarray(data, dtype=np.uint32).copy()
    n = out.size if count is None else count
    if n:
        c = np.cumsum(out[:n], dtype=np.uint64) & np.uint64(0xFFFFFFFF)
        out[1:n] = c[:-1].astype(np.uint32)
        out[0] = 0
    return out


def prefix_sum_blelloch(data, count=None, workgroup=256):
    out = np.ascontiguousarray(data, dtype=np.uint32).copy()
    n = out.size if count is None else count
    rc = lib().rso_prefix_sum_blelloch(_ptr(out), n, workgroup)
    if rc:
        raise ValueError(f"rso_prefix_sum_blelloch rc={rc}")
    return out


def is_sorted_masked(keys: np.ndarray, bit_count: int = 32, count: int | None = None) -> bool:
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    n = k.size if count is None else count
    return bool(lib().rso_is_sorted_masked(_ptr(k), n, bit_count))


def verify_stable_iota(keys_in, keys_out, values_out, bit_count=32) -> int:
    """0 if (keys_out, values_out) is THE stable masked sort of keys_in with values = iota."""
    ki = np.ascontiguousarray(keys_in, dtype=np.uint32)
    ko = np.ascontiguousarray(keys_out, dtype=np.uint32)
    vo = np.ascontiguousarray(values_out, dtype=np.uint32)
    return int(lib().rso_verify_stable_iota(_ptr(ki), _ptr(ko), _ptr(vo), ki.size, bit_count))
