"""Kernel timeline of back-to-back sorts (run under rocprofv3 --kernel-trace): shows gaps
between launches.  usage: python tools/timeline_probe.py N KV REPS"""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "webgpu-radix-sort_amd"))
import torch
from radix_sort_amd import RadixSortKernel, ops

n, kv, reps = int(sys.argv[1]), sys.argv[2] == "1", int(sys.argv[3])
bs = []
for i in range(reps):
    k = torch.empty(n, dtype=torch.int32, device="cuda")
    ops.fill_random_u32(k, 100 + i)
    v = None
    if kv:
        v = torch.empty(n, dtype=torch.int32, device="cuda")
        ops.fill_iota_u32(v)
    bs.append((k, v))
ks = [RadixSortKernel(keys=k, values=v, count=n) for k, v in bs]
w = torch.empty(n, dtype=torch.int32, device="cuda"); ops.fill_random_u32(w, 7)
RadixSortKernel(keys=w, count=n).dispatch()
torch.cuda.synchronize()
t = time.perf_counter()
for kk in ks:
    kk.dispatch()
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / reps
print(f"n={n} kv={kv} wall/sort={dt*1e3:.4f} ms", flush=True)
