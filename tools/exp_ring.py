#!/usr/bin/env python3
"""Experiment (sweep build only): the hybrid path's pass 1 and bucket pass with R2 replaced by a
power-of-two ring of 2^bits records (RSORT_EXP_RING), i.e. with R2 Infinity-Cache resident.
The sort results are INVALID (the ring overwrites itself); only the kernel times matter: they
bound what an IC-blocked pass 1 + bucket pass could reach.  One subprocess per ring size.

    RSORT_LIB=exp_lib/librsort_sweep.so python tools/exp_ring.py 0 20 22 23 24 25 28
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, time
sys.path.insert(0, os.path.join(%(root)r, "webgpu-radix-sort_amd"))
import torch
from radix_sort_amd import RadixSortKernel, ops
n = 1 << 28
nb = 4
bs = []
for i in range(nb):
    k = torch.empty(n, dtype=torch.int32, device="cuda"); ops.fill_random_u32(k, 100 + i)
    v = torch.empty(n, dtype=torch.int32, device="cuda"); ops.fill_iota_u32(v)
    bs.append((k, v))
ks = [RadixSortKernel(keys=k, values=v, count=n) for k, v in bs]
for kk in ks: kk.dispatch()
torch.cuda.synchronize()
for i in range(nb): ops.fill_random_u32(bs[i][0], 500 + i)
for kk in ks: kk.set_profiling(True)
for kk in ks: kk.dispatch()
torch.cuda.synchronize()
kt = {}
for kk in ks:
    for a, b in kk.kernel_times().items():
        kt[a] = kt.get(a, 0.0) + b["ms"] / nb
print("RESULT " + json.dumps({a: round(b, 4) for a, b in kt.items()}))
'''


def main():
    for bits in sys.argv[1:] or ["0"]:
        env = dict(os.environ, RSORT_EXP_RING=bits)
        r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
        out = json.loads(line[-1][7:]) if line else {"error": r.stderr[-2000:]}
        print(json.dumps({"ring_bits": int(bits), "kernel_ms_per_sort": out}), flush=True)
        if not line:
            sys.exit(1)


if __name__ == "__main__":
    main()
