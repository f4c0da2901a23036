"""Wall time of repeated dispatches of ONE plan on the same buffers (the hipGraph replay case)
versus one-shot plans.  usage: python tools/repeat_probe.py"""
import json
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "webgpu-radix-sort_amd"))
import torch
from radix_sort_amd import RadixSortKernel, ops

for n, kv in ((100_000, False), (1 << 20, False), (1 << 20, True), (4 << 20, True), (10_000_000, False)):
    k = torch.empty(n, dtype=torch.int32, device="cuda")
    v = torch.empty(n, dtype=torch.int32, device="cuda") if kv else None
    ops.fill_random_u32(k, 1)
    kern = RadixSortKernel(keys=k, values=v, count=n)
    for _ in range(3):
        kern.dispatch()
    torch.cuda.synchronize()
    reps = 50
    t = time.perf_counter()
    for _ in range(reps):
        kern.dispatch()                       # re-sorts sorted data: same work, same launches
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    print(json.dumps({"n": n, "kv": kv, "repeat_ms": round(dt * 1e3, 4),
                      "graph": os.environ.get("RSORT_GRAPH", "1")}), flush=True)
