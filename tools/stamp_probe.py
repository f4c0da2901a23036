#!/usr/bin/env python3
"""Diagnostic: per-tile phase timing of k_onesweep from in-kernel s_memtime stamps.

Needs the stamped variant library (make -C webgpu-radix-sort_amd/csrc variants
VARIANTS="stamps:-DRS_STAMPS=1"), selected with RSORT_LIB:

    RSORT_LIB=webgpu-radix-sort_amd/lib/variants/librsort_stamps.so python tools/stamp_probe.py [log2n]

Phases (thread 0 of the workgroup, shader cycles): 0 loop top -> 1 ranked (includes the wait for
the tile's loads) -> 2 counts published, wave offsets -> 3 staged in LDS, next ticket -> 4 look-back
done -> 5 scattered.  Prints one JSON line per pass: mean / p50 / p90 cycles of each phase, the
per-tile total and the cadence between consecutive tiles of one workgroup.
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

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 28
tile = int(sys.argv[2]) if len(sys.argv) > 2 else 16384   # k_onesweep tile of the configuration
n = 1 << lg
L = _lib.load()
fn = L.rs_debug_set_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p]
k = torch.empty(n, dtype=torch.int32, device="cuda")
v = torch.empty(n, dtype=torch.int32, device="cuda")
kern = RadixSortKernel(keys=k, values=v, count=n, local_shuffle=True)
info = kern.info
passes = info["passes"]
max_tiles = (n + tile - 1) // tile
st = torch.zeros(passes * max_tiles * 16, dtype=torch.int64, device="cuda")
for i in range(3):
    ops.fill_random_u32(k, 11 + i)
    ops.fill_iota_u32(v)
    if i == 2:
        torch.cuda.synchronize()
        _lib.check(fn(st.data_ptr()), "stamps")
    kern.dispatch()
torch.cuda.synchronize()
_lib.check(fn(None), "stamps off")
a = st.cpu().numpy().reshape(passes, max_tiles, 16)
names = ["rank", "publish", "stage", "lookback", "scatter"]
for p in range(passes):
    s = a[p]
    used = s[:, 0] != 0
    s = s[used].astype(np.int64)
    nt = len(s)
    d = {"pass": p, "tiles": nt}
    for i, nm in enumerate(names):
        x = s[:, i + 1] - s[:, i]
        d[nm] = {"mean": int(x.mean()), "p50": int(np.median(x)), "p90": int(np.percentile(x, 90))}
    tot = s[:, 5] - s[:, 0]
    d["tile_total"] = {"mean": int(tot.mean()), "p50": int(np.median(tot))}
    # cadence: consecutive tiles of one workgroup
    wg = s[:, 7]
    order = np.lexsort((s[:, 0], wg))
    s0 = s[order, 0]
    same = wg[order][1:] == wg[order][:-1]
    cad = (s0[1:] - s0[:-1])[same]
    d["cadence"] = {"mean": int(cad.mean()) if len(cad) else 0,
                    "p50": int(np.median(cad)) if len(cad) else 0}
    d["span_cycles"] = int(s[:, 5].max() - s[:, 0].min())
    print(json.dumps(d), flush=True)
print(json.dumps({"n": n, "sorted": ops.is_sorted(k), "tile_keys": info["tile_keys"]}))
