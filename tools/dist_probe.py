#!/usr/bin/env python3
"""Sort time vs key distribution at 2^28 keys + values (diagnostic): uniform, runs of 16 equal
keys, sorted uniform, few distinct keys.  python tools/dist_probe.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "webgpu-radix-sort_amd"))
import torch  # noqa: E402
from radix_sort_amd import RadixSortKernel, ops  # noqa: E402

n = 1 << int(os.environ.get("LOG2N", "28"))
dev = "cuda"
base = torch.empty(n, dtype=torch.int32, device=dev)
ops.fill_random_u32(base, 1)
idx = torch.arange(n, device=dev, dtype=torch.int64)
dists = {
    "uniform": lambda: base.clone(),
    "runs16": lambda: base[(idx >> 4)].clone(),
    "sorted": lambda: torch.sort(base.view(torch.int64)[: n // 2].view(torch.int32))[0].repeat(2).clone()
              if False else torch.sort((base.to(torch.int64) & 0xFFFFFFFF))[0].to(torch.int32),
    "sorted_runs16": lambda: torch.sort((base[(idx >> 4)].to(torch.int64) & 0xFFFFFFFF))[0].to(torch.int32),
    "distinct16": lambda: (base & 15),
    "runs4": lambda: base[(idx >> 2)].clone(),
    "runs64": lambda: base[(idx >> 6)].clone(),
    "runs16_shuffled_lanes": lambda: base[((idx >> 10) << 6) | (idx & 63)].clone(),
}
sel = os.environ.get("DISTS")
for name, make in dists.items():
    if sel and name not in sel.split(","):
        continue
    keys = [make() for _ in range(3)]
    kv = os.environ.get("KV", "1") != "0"
    vals = [torch.arange(n, dtype=torch.int32, device=dev) if kv else None for _ in range(3)]
    ks = [RadixSortKernel(keys=k, values=v, count=n) for k, v in zip(keys, vals)]
    w = make(); wv = torch.arange(n, dtype=torch.int32, device=dev) if kv else None
    RadixSortKernel(keys=w, values=wv, count=n).dispatch()
    for k in ks:
        k.set_profiling(True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in ks:
        k.dispatch()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / len(ks)
    kt = {}
    for k in ks:
        for a, b in k.kernel_times().items():
            kt[a] = round(kt.get(a, 0.0) + b["ms"] / len(ks), 4)
    ok = all(ops.is_sorted(k) for k in keys)
    print(json.dumps({"dist": name, "n": n, "kv": kv, "ms": round(dt * 1e3, 3), "sorted": ok, "kernel_ms": kt}), flush=True)
    del keys, vals, ks, w, wv
    torch.cuda.empty_cache()
