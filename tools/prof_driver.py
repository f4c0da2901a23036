#!/usr/bin/env python3
"""Small driver for rocprofv3: a few sorts of one BASELINE workload with the in-tree library.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python3 tools/prof_driver.py config3
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "webgpu-radix-sort_amd"))

import torch  # noqa: E402
from radix_sort_amd import RadixSortKernel, ops  # noqa: E402

WL = {"config3": (1 << 28, True, True), "config2": (1 << 26, False, False),
      "config4": (1 << 28, True, False)}   # f32 nearly sorted + check_order (bench.py's input)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "config3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    radix_bits = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    n, kv, ls = WL[name]
    k = torch.empty(n, dtype=torch.int32, device="cuda")
    v = torch.empty(n, dtype=torch.int32, device="cuda") if kv else None
    nearly = None
    if name == "config4":
        sys.path.insert(0, ROOT)
        import bench
        nearly = torch.from_numpy(bench.nearly_sorted_f32_bits(n, 4).view("int32"))
    kern = RadixSortKernel(keys=k, values=v, count=n, local_shuffle=ls, radix_bits=radix_bits,
                           check_order=nearly is not None)
    for r in range(reps):
        if nearly is not None:
            k.copy_(nearly)
        else:
            ops.fill_random_u32(k, 1000 + r)
        if kv:
            ops.fill_iota_u32(v)
        kern.dispatch()
    torch.cuda.synchronize()
    assert ops.is_sorted(k)
    print(f"prof_driver: {reps} sorts of {name} done")


if __name__ == "__main__":
    main()
