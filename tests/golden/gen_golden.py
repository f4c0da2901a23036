#!/usr/bin/env python3
"""Generate the committed golden fixtures for the radix-sort / prefix-sum parity tests.

The reference (MatthieuLepers/WebGPU-Radix-Sort) holds no golden vectors; its tests compare
the GPU result against a CPU expression evaluated in JS:

* sort: ``keys.slice(0, count).sort((a, b) => a - b)``  (example/tests.ts:86) and
  ``keysResult[i] == keys[values[i]]``                  (example/tests.ts:94)
* scan: ``prefixSumCpu`` (exclusive running sum)         (example/tests.ts:288-296)

This script evaluates those expressions with Node (``node_expected.js``) for every bit_count=32
case (the reference test's bitCount, example/tests.ts:32) and stores inputs + expected outputs.
Expected VALUES are the stable permutation (values = iota in), which is stricter than the
reference's index check and is derived from the numpy closed form; the script asserts that the
Node keys, the numpy closed form and the literal per-pass WGSL restatement (oracle/rs_oracle.c)
all agree before writing anything.  Cases with bit_count < 32 (the reference never tests them)
take their expected output from the restatements only and are flagged ``node_pinned = False``.

Large cases (2^20) are stored as (seed, sha256 of expected keys/values) instead of arrays.

Run from the repo root:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def node_eval(mode: str, data: np.ndarray, count: int) -> np.ndarray:
    with tempfile.TemporaryDirectory() as td:
        ip, op = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        np.ascontiguousarray(data, dtype=np.uint32).tofile(ip)
        subprocess.run(["node", os.path.join(HERE, "node_expected.js"), mode, ip, str(count), op],
                       check=True)
        return np.fromfile(op, dtype=np.uint32)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint32).tobytes()).hexdigest()


def make_keys(kind: str, n: int, seed: int) -> np.ndarray:
    u = O.gen_u32(seed, n)
    if kind == "u32":
        return u
    if kind == "f32":  # non-negative Float32 keys in [0, 1), raw bits (README.md:9)
        return ((u >> np.uint32(8)).astype(np.float64) * 2.0 ** -24).astype(np.float32).view(np.uint32)
    if kind == "f32_special":  # -0.0, +inf, NaN, denormals, negatives mixed with normals
        f = ((u >> np.uint32(8)).astype(np.float64) * 2.0 ** -24 * 100 - 20).astype(np.float32)
        specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 3.4e38],
                            dtype=np.float32)
        f[u % 7 == 0] = specials[(u[u % 7 == 0] >> np.uint32(3)) % specials.size]
        return f.view(np.uint32)
    if kind == "sorted":
        return np.sort(u)
    if kind == "reverse":
        return np.sort(u)[::-1].copy()
    if kind == "equal":
        return np.full(n, 0xDEADBEEF, dtype=np.uint32)
    if kind == "few":  # many duplicates -> stability matters
        return u % np.uint32(5)
    if kind == "nearly":
        return O.nearly_sorted_f32_bits(n, seed, swaps=max(1, n // 100))
    if kind == "q1":  # sorted except the last pair: the reference's check_order misses it (Q1)
        s = np.sort(u)
        if n >= 2:
            s[-2], s[-1] = s[-1], s[-2]
        return s
    raise ValueError(kind)


def main() -> None:
    cases = []
    arrays = {}
    cid = 0
    sizes = [1, 2, 3, 255, 256, 257, 1023, 1024, 1025, 4097, 65537]
    plan = []
    for n in sizes:
        for bits in ((4, 8, 16, 32) if n < 65537 else (32,)):
            plan.append(dict(n=n, count=n, bits=bits, kind="u32", kv=True))
        plan.append(dict(n=n, count=n, bits=32, kind="u32", kv=False))
        plan.append(dict(n=n, count=n, bits=32, kind="f32", kv=True))
    for n in (257, 4097):
        for kind in ("f32_special", "sorted", "reverse", "equal", "few", "nearly", "q1"):
            plan.append(dict(n=n, count=n, bits=32, kind=kind, kv=True))
        plan.append(dict(n=n, count=n // 3 + 1, bits=32, kind="u32", kv=True))  # count < len
        plan.append(dict(n=n, count=n - 1, bits=12, kind="few", kv=True))
    for p in plan:
        n, count, bits = p["n"], p["count"], p["bits"]
        seed = 1000 + cid
        keys = make_keys(p["kind"], n, seed)
        vals = np.arange(n, dtype=np.uint32) if p["kv"] else None
        ek, ev = O.stable_sort_masked(keys, vals, bits, count)
        lk, lv = O.radix_sort_literal(keys, vals, bits, 256, local_shuffle=bool(cid % 2), count=count)
        assert (lk == ek).all() and (vals is None or (lv == ev).all()), p
        node_pinned = bits == 32
        if node_pinned:
            nk = node_eval("sort", keys, count)
            assert (nk == ek[:count]).all(), ("node disagrees", p)
            # reference's value check (example/tests.ts:94)
            if vals is not None:
                assert (keys[ev[:count]] == ek[:count]).all()
        name = f"c{cid:03d}"
        arrays[f"{name}_keys"] = keys
        arrays[f"{name}_exp_keys"] = ek
        if vals is not None:  # input values are iota (not stored)
            arrays[f"{name}_exp_values"] = ev
        cases.append(dict(name=name, n=n, count=count, bit_count=bits, kind=p["kind"],
                          has_values=vals is not None, node_pinned=node_pinned, seed=seed))
        cid += 1

    # large cases pinned by seed + sha256 (generator: oracle.gen_u32 == rs_fill_random_u32)
    large = []
    for n, kv, kind, seed in ((1 << 20, False, "u32", 1), (1 << 20, True, "u32", 3),
                              (1 << 20, True, "f32", 4)):
        keys = make_keys(kind, n, seed)
        vals = np.arange(n, dtype=np.uint32) if kv else None
        ek, ev = O.stable_sort_masked(keys, vals, 32)
        nk = node_eval("sort", keys, n)
        assert (nk == ek).all()
        large.append(dict(n=n, kind=kind, seed=seed, has_values=kv, bit_count=32,
                          sha256_keys=sha(ek), sha256_values=sha(ev) if kv else None,
                          node_pinned=True))

    # prefix sum (PrefixSumKernel) cases: data in [0, 8) like example/tests.ts:135
    scans = []
    for i, (n, count) in enumerate(((1, 1), (2, 2), (511, 511), (512, 512), (513, 300),
                                    (100003, 100003), (262145, 200000))):
        d = (O.gen_u32(500 + i, n) & np.uint32(7)).astype(np.uint32)
        exp = O.prefix_sum(d, count)
        ne = node_eval("scan", d, count)
        assert (ne == exp[:count]).all()
        assert (O.prefix_sum_blelloch(d, count, 256) == exp).all()
        name = f"s{i:02d}"
        arrays[f"{name}_data"] = d
        arrays[f"{name}_exp"] = exp
        scans.append(dict(name=name, n=n, count=count))

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **arrays)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(dict(
            generator="tests/golden/gen_golden.py",
            node_version=subprocess.run(["node", "--version"], capture_output=True,
                                        text=True).stdout.strip(),
            key_generator="low32(splitmix64_finaliser(seed*0xD1B54A32D192ED03 + i))",
            sort_cases=cases, large_cases=large, scan_cases=scans), f, indent=1)
    print(f"wrote {len(cases)} sort cases, {len(large)} large, {len(scans)} scan cases")


if __name__ == "__main__":
    main()
