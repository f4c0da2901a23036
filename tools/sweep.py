#!/usr/bin/env python3
"""Time tuning variants of librsort (lib/variants/librsort_<name>.so), one subprocess each.

    python tools/sweep.py [variant ...]      (default: every .so in lib/variants)

Prints one JSON line per (variant, workload): ms per sort, Gkeys/s, per-kernel ms.
"""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "webgpu-radix-sort_amd", "lib", "variants")

CHILD = r'''
import json, os, sys, time
sys.path.insert(0, os.path.join(%(root)r, "webgpu-radix-sort_amd"))
import torch
from radix_sort_amd import RadixSortKernel, ops
res = []
for name, n, kv, rb in %(loads)s:
    nb = 4 if n > (1 << 22) else 20
    bs = []
    for i in range(nb):
        k = torch.empty(n, dtype=torch.int32, device="cuda")
        ops.fill_random_u32(k, 100 + i)
        v = None
        if kv:
            v = torch.empty(n, dtype=torch.int32, device="cuda"); ops.fill_iota_u32(v)
        bs.append((k, v))
    wk = torch.empty(n, dtype=torch.int32, device="cuda"); ops.fill_random_u32(wk, 99)
    wv = None
    if kv:
        wv = torch.empty(n, dtype=torch.int32, device="cuda"); ops.fill_iota_u32(wv)
    RadixSortKernel(keys=wk, values=wv, count=n, radix_bits=rb).dispatch()
    ks = [RadixSortKernel(keys=k, values=v, count=n, radix_bits=rb) for k, v in bs]
    torch.cuda.synchronize()
    t = time.perf_counter()
    for kk in ks: kk.dispatch()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / nb          # wall time, profiling off
    for i in range(nb):                           # fresh unsorted inputs for the profiled run
        ops.fill_random_u32(bs[i][0], 500 + i)
    for kk in ks: kk.set_profiling(True)
    for kk in ks: kk.dispatch()
    torch.cuda.synchronize()
    kt = {}
    for kk in ks:
        for a, b in kk.kernel_times().items():
            kt[a] = kt.get(a, 0.0) + b["ms"] / nb
    ok = all(ops.is_sorted(k) for k, _ in bs)
    res.append(dict(workload=name, n=n, kv=kv, radix_bits=rb, ms=round(dt * 1e3, 4),
                    gkeys=round(n / dt / 1e9, 3), sorted=ok,
                    kernel_ms={a: round(b, 4) for a, b in kt.items()}))
    del bs, ks, wk, wv
    torch.cuda.empty_cache()
print("RESULT " + json.dumps(res))
'''

LOADS = [("config3_kv_256M", 1 << 28, True, 0), ("config2_keys_64M", 1 << 26, False, 0)]
if os.environ.get("SWEEP_SMALL"):
    LOADS = [("keys_100K", 100_000, False, 0), ("keys_1M", 1 << 20, False, 0),
             ("kv_1M", 1 << 20, True, 0), ("keys_10M", 10_000_000, False, 0),
             ("kv_16M", 1 << 24, True, 0)]

COPY = r'''
import json, time, torch
res = []
for nbytes in (1 << 31, 1 << 30):
    a = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda"); a.fill_(1)
    b = torch.empty_like(a)
    b.copy_(a); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10): b.copy_(a)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    res.append(dict(copy_bytes=nbytes, ms=round(dt * 1e3, 4), rw_GBs=round(2 * nbytes / dt / 1e9, 1)))
    a.fill_(2); torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10): a.fill_(3)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 10
    res.append(dict(fill_bytes=nbytes, ms=round(dt * 1e3, 4), w_GBs=round(nbytes / dt / 1e9, 1)))
    s = 0
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10): s = a.sum()
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 10
    res.append(dict(read_bytes=nbytes, ms=round(dt * 1e3, 4), r_GBs=round(nbytes / dt / 1e9, 1)))
print("RESULT " + json.dumps(res))
'''


def main():
    if sys.argv[1:] == ["copy"]:
        r = subprocess.run([sys.executable, "-c", COPY], capture_output=True, text=True, timeout=300)
        for line in r.stdout.splitlines():
            if line.startswith("RESULT "):
                for x in json.loads(line[7:]):
                    print(json.dumps({"variant": "torch_stream", **x}), flush=True)
        return
    names = sys.argv[1:] or sorted(os.path.basename(p)[9:-3] for p in glob.glob(os.path.join(VDIR, "librsort_*.so")))
    for spec in names:
        name, *envs = spec.split("@")
        env = dict(os.environ, RSORT_LIB=os.path.join(VDIR, f"librsort_{name}.so"))
        for e in envs:
            a, b = e.split("=", 1)
            env[a] = b
        code = CHILD % {"root": ROOT, "loads": repr(LOADS)}
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                           timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
        if r.returncode or not line:
            print(json.dumps({"variant": spec, "error": r.stderr[-2000:]}), flush=True)
            if r.returncode < 0 or r.returncode in (134, 139):
                sys.exit(r.returncode or 1)
            continue
        for x in json.loads(line[0][7:]):
            print(json.dumps({"variant": spec, **x}), flush=True)


if __name__ == "__main__":
    main()
