#!/usr/bin/env python3
"""Diagnostic: per-tile phase timing of the hybrid path's two k_onesweep passes (s_memtime stamps).

Needs a stamped library (tools/build_variants.sh st:-DRS_STAMPS=1 with OUTD=../lib/exp), selected
with RSORT_LIB.  n = 2^28 keys + values (BASELINE config3).  Per pass one JSON line: mean / p50 / p90
shader cycles of each phase of thread 0's tile loop - rank (incl. the wait for the tile's loads),
publish, stage (+ next ticket), look-back (prefetch issue + status rounds + barrier), scatter - and of
digit 0's look-back: cycles until its first status round returned (behind the wave's prefetch loads),
rounds, predecessors consumed, sleeps.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "webgpu-radix-sort_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from radix_sort_amd import RadixSortKernel, _lib, ops  # noqa: E402

n = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 28)
TILE = 16384
L = _lib.load()
fn = L.rs_debug_set_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p]
k = torch.empty(n, dtype=torch.int32, device="cuda")
v = torch.empty(n, dtype=torch.int32, device="cuda")
kern = RadixSortKernel(keys=k, values=v, count=n, local_shuffle=True)
nt = (n + TILE - 1) // TILE
bound = [nt, nt + 257]                      # the kernels' `ntiles` argument per pass (stamp stride)
words = (bound[0] + bound[1] * 2) * 16
st = torch.zeros(words, dtype=torch.int64, device="cuda")
for i in range(3):
    ops.fill_random_u32(k, 11 + i)
    ops.fill_iota_u32(v)
    if i == 2:
        torch.cuda.synchronize()
        _lib.check(fn(st.data_ptr()), "stamps")
    kern.dispatch()
torch.cuda.synchronize()
_lib.check(fn(None), "stamps off")
path = kern.last_path()
a = st.cpu().numpy()
names = ["rank", "publish", "stage", "lookback", "scatter"]


def stats(x):
    return {"mean": int(x.mean()), "p50": int(np.median(x)), "p90": int(np.percentile(x, 90))}


for p in range(2):
    base = p * bound[p] * 16
    s = a[base:base + bound[p] * 16].reshape(bound[p], 16).astype(np.int64)
    s = s[s[:, 0] != 0]
    d = {"pass": p, "tiles": len(s)}
    for i, nm in enumerate(names):
        d[nm] = stats(s[:, i + 1] - s[:, i])
    d["tile_total"] = stats(s[:, 5] - s[:, 0])
    lb = s[s[:, 8] != 0]                     # tiles that looked back (not a segment's first)
    if len(lb):
        d["lb_first_round_after_stage"] = stats(lb[:, 8] - lb[:, 3])
        d["lb_rounds"] = stats(lb[:, 9])
        d["lb_predecessors"] = stats(lb[:, 10])
        d["lb_sleeps"] = stats(lb[:, 11])
    wg = s[:, 7]
    order = np.lexsort((s[:, 0], wg))
    s0 = s[order, 0]
    same = wg[order][1:] == wg[order][:-1]
    cad = (s0[1:] - s0[:-1])[same]
    d["cadence"] = stats(cad) if len(cad) else {}
    d["span_cycles"] = int(s[:, 5].max() - s[:, 0].min())
    print(json.dumps(d), flush=True)
print(json.dumps({"n": n, "path": path, "sorted": ops.is_sorted(k)}))
