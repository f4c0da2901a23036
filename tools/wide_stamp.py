#!/usr/bin/env python3
"""Diagnostic: per-bucket phase timing of k_bucket_sort_wide from in-kernel s_memtime stamps, at a
multi-GPU receiver's shape (tools/prof_driver.py `region`: 16-bit buckets of ~32K records).

Needs the stamped variant library (each stamp waits for the workgroup's memory operations and a
barrier, so phases are serialised and the total is longer than the real kernel's):

    make -C webgpu-radix-sort_amd/csrc variants VARIANTS="stamps:-DRS_STAMPS=1"
    RSORT_LIB=webgpu-radix-sort_amd/lib/variants/librsort_stamps.so python tools/wide_stamp.py

Phases (shader cycles): load (0 -> 1), pass over key bits 0-7 (1 -> 2), bits 8-15 (2 -> 3), value
exchange (3 -> 4), output stores issued and completed (4 -> 5); cadence = start to start of one
workgroup's consecutive buckets.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "webgpu-radix-sort_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from radix_sort_amd import _lib  # noqa: E402
import prof_driver  # noqa: E402


def main():
    L = _lib.load()
    fn = L.rs_debug_set_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    base = 1 << 22                   # kWideStampBase (k_onesweep's stamps below it)
    st = torch.zeros(base + 65536 * 8, dtype=torch.int64, device="cuda")
    prof_driver.region(1)            # warm-up
    torch.cuda.synchronize()
    _lib.check(fn(st.data_ptr()), "stamps")
    prof_driver.region(1)
    torch.cuda.synchronize()
    _lib.check(fn(None), "stamps off")
    a = st[base:].cpu().numpy().reshape(65536, 8)
    a = a[a[:, 0] != 0].astype(np.int64)
    names = ["load", "pass_lo", "pass_hi", "values", "store"]
    d = {"buckets": int(len(a))}
    for i, nm in enumerate(names):
        x = a[:, i + 1] - a[:, i]
        d[nm] = {"mean": int(x.mean()), "p50": int(np.median(x)), "p90": int(np.percentile(x, 90))}
    tot = a[:, 5] - a[:, 0]
    d["bucket_total"] = {"mean": int(tot.mean()), "p50": int(np.median(tot))}
    order = np.lexsort((a[:, 0], a[:, 7]))
    s0 = a[order, 0]
    same = a[order, 7][1:] == a[order, 7][:-1]
    cad = (s0[1:] - s0[:-1])[same]
    d["cadence"] = {"mean": int(cad.mean()) if len(cad) else 0, "p50": int(np.median(cad)) if len(cad) else 0}
    d["span_cycles"] = int(a[:, 5].max() - a[:, 0].min())
    print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
