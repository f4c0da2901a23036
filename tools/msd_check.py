#!/usr/bin/env python3
"""Hybrid MSD path check + timing on the GPU (diagnostic, not a test file):
parity against the oracle at 13M-64M keys, property checks at 256M, both device fallbacks
(skewed top byte -> LSD on the input; 16-bit buckets over capacity -> LSD on R1), and the
config3 timing.  The path is the plan's own choice; each line records the one the device took
(rs_plan_last_path).  To force a path, wrap a run in ``_lib.plan_debug(msd=0)``.  Prints JSON lines."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "webgpu-radix-sort_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import torch

from radix_sort_amd import RadixSortKernel, ops

dev = torch.device("cuda", 0)


def make(n, kind, seed):
    k = torch.empty(n, dtype=torch.int32, device=dev)
    ops.fill_random_u32(k, seed)
    if kind == "top0":
        k &= 0x00FFFFFF
    elif kind == "low0":
        k &= -16777216                  # 0xFF000000: every key in a (top, 0) 16-bit bucket
    elif kind == "dups":
        k.remainder_(1 << 20)
        k.mul_(4093)                    # 2^20 distinct keys spread over the key space
    v = torch.empty(n, dtype=torch.int32, device=dev)
    ops.fill_iota_u32(v)
    return k, v


def props(kin, kout, vout):
    torch.cuda.synchronize()
    ok_sorted = ops.is_sorted(kout)
    perm = torch.equal(kin[vout.long()], kout)
    same = kout[1:] == kout[:-1]
    stable = bool(((vout[1:] > vout[:-1]) | ~same).all().item())
    return ok_sorted and perm and stable


def run(n, kind, seed, exact):
    k, v = make(n, kind, seed)
    kin = k.clone()
    kern = RadixSortKernel(keys=k, values=v, count=n, bit_count=32, local_shuffle=True)
    kern.set_profiling(True)
    kern.dispatch()
    torch.cuda.synchronize()
    kern.check()
    kt = {a: round(b["ms"], 4) for a, b in kern.kernel_times().items() if b["launches"]}
    ok = props(kin, k, v)
    if exact:
        import oracle as O
        ek, ev = O.stable_sort_masked_c(kin.cpu().numpy().view(np.uint32), np.arange(n, dtype=np.uint32), 32)
        ok = ok and np.array_equal(k.cpu().numpy().view(np.uint32), ek) and \
            np.array_equal(v.cpu().numpy().view(np.uint32), ev)
    print(json.dumps({"n": n, "kind": kind, "device_path": kern.last_path(), "ok": bool(ok),
                      "kernel_ms": kt}), flush=True)
    kern.destroy()
    return ok


def timing(n, steps=10):
    batches = [make(n, "uniform", 100 + i) for i in range(steps)]
    ks = [RadixSortKernel(keys=a, values=b, count=n, local_shuffle=True) for a, b in batches]
    wk, wv = make(n, "uniform", 99)
    RadixSortKernel(keys=wk, values=wv, count=n, local_shuffle=True).dispatch()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for kk in ks:
        kk.dispatch()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    for i, (a, b) in enumerate(batches):
        ops.fill_random_u32(a, 500 + i)
        ops.fill_iota_u32(b)
    for kk in ks:
        kk.set_profiling(True)
        kk.dispatch()
    torch.cuda.synchronize()
    kt = {}
    for kk in ks:
        for a, b in kk.kernel_times().items():
            if b["launches"]:
                e = kt.setdefault(a, [0.0, 0])
                e[0] += b["ms"] / steps
                e[1] += b["launches"] / steps
    print(json.dumps({"timing_n": n, "device_path": ks[0].last_path(),
                      "ms_per_sort": round(dt * 1e3, 4), "gkeys": round(n / dt / 1e9, 2),
                      "kernel_ms_per_sort": {a: [round(b[0], 4), b[1]] for a, b in kt.items()}}),
          flush=True)


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "check"
    if mode == "check":
        good = True
        for n, kind, exact in [((13 << 20) + 5, "uniform", True), (1 << 24, "uniform", True),
                               ((1 << 26) + 3, "uniform", True), (1 << 24, "top0", True),
                               (1 << 24, "low0", True), (1 << 24, "dups", True),
                               (1 << 28, "uniform", False), (1 << 28, "dups", False)]:
            good &= run(n, kind, 7, exact)
        sys.exit(0 if good else 1)
    timing(1 << 28)
