#!/usr/bin/env python3
"""Diagnostic: per-pass cost of the one-sweep KV sort as a function of n, with the input
re-generated right before every sort (so small sorts run with their whole working set in the
Infinity Cache).  One plan, one pair of arrays, `iters` sorts.  Run under rocprofv3 --stats for
per-kernel averages, or alone for the plan's own HIP-event kernel times.

    python tools/mall_sort_probe.py LOG2N [iters]

(the plan picks its path by size; the library reads no environment variables - force a path with
``radix_sort_amd._lib.plan_debug(tile="large", onesweep=1)`` around the plan's creation)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "webgpu-radix-sort_amd"))

import torch  # noqa: E402
from radix_sort_amd import RadixSortKernel, ops  # noqa: E402

lg = int(sys.argv[1])
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
n = 1 << lg
k = torch.empty(n, dtype=torch.int32, device="cuda")
v = torch.empty(n, dtype=torch.int32, device="cuda")
kern = RadixSortKernel(keys=k, values=v, count=n)
ops.fill_random_u32(k, 7)
ops.fill_iota_u32(v)
kern.dispatch()
torch.cuda.synchronize()
kern.set_profiling(True)
kern.kernel_times(reset=True)
t = 0.0
for i in range(iters):
    ops.fill_random_u32(k, 100 + i)
    ops.fill_iota_u32(v)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    kern.dispatch()
    e1.record()
    e1.synchronize()
    t += e0.elapsed_time(e1)
kt = kern.kernel_times()
ok = ops.is_sorted(k)
sc = kt["scatter"]
print(json.dumps({"n": n, "log2n": lg, "sorted": ok, "ms_per_sort": round(t / iters, 4),
                  "gkeys": round(n / (t / iters * 1e-3) / 1e9, 2),
                  "scatter_ms_per_launch": round(sc["ms"] / max(1, sc["launches"]), 5),
                  "scatter_GBs_16Bperkey": round(16 * n * sc["launches"] / (sc["ms"] * 1e-3) / 1e9, 1),
                  "histogram_ms_per_sort": round(kt["histogram"]["ms"] / iters, 5),
                  "device_errors": kern.device_errors()}))
