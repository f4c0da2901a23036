#!/usr/bin/env python3
"""Small driver for rocprofv3: a few sorts of one BASELINE workload with the in-tree library.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python3 tools/prof_driver.py config3

`region`: a multi-GPU receiver's local work at config 5's shape (tools/rank_model.py): 2^28 records
over 32 top bytes sorted as 4 regions by rs_plan_sort_region - 16-bit buckets of ~32K records, the
wide bucket kernel's case.
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
    if name == "region":
        return region(reps)
    if name == "prefix_sum":
        return prefix_sum(reps)
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
    # (RS_PROF_NOCHECK=1: a traffic-attribution build whose passes do not sort, rs_kernels.hpp RS_DIAG_*)
    assert os.environ.get("RS_PROF_NOCHECK") == "1" or ops.is_sorted(k)
    print(f"prof_driver: {reps} sorts of {name} done")


def prefix_sum(reps, n=1 << 28):
    """PrefixSumKernel over bench.py's prefix_sum shape (2^28 u32, values in [0, 8))."""
    from radix_sort_amd import PrefixSumKernel
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    kern = PrefixSumKernel(data=t, count=n)
    for r in range(reps):
        ops.fill_random_u32(t, 2000 + r)
        t &= 7
        kern.dispatch()
    torch.cuda.synchronize()
    kern.check()
    print(f"prof_driver: {reps} prefix sums of 2^28 u32 done")


def region(reps, n=1 << 28, span=32, rounds=4):
    from radix_sort_amd.distributed import HipLocalOps
    dev = torch.device("cuda", 0)
    lo = HipLocalOps(0, int(n * 1.25), True)
    rk = torch.empty(n, dtype=torch.int32, device=dev)
    ops.fill_random_u32(rk, 55)
    rk &= (span << 24) - 1
    rv = torch.arange(n, dtype=torch.int32, device=dev)
    rh = lo.hist16(rk)
    rec = lo.partition(rk, rv, 24, 8, rh[65536:])
    tops = rh[65536:].long().cpu().tolist()
    starts = [0]
    for c in tops:
        starts.append(starts[-1] + c)
    ok_, ov_ = torch.empty_like(rk), torch.empty_like(rv)
    per = span // rounds
    regions = []
    for g in range(rounds):
        t0, t1 = g * per, (g + 1) * per
        reg = torch.zeros(65536, dtype=torch.int32, device=dev)
        reg[t0 << 8:t1 << 8] = rh[t0 << 8:t1 << 8]
        regions.append((starts[t0], starts[t1], reg, t0, t1))
    for _ in range(reps):
        for a, b, reg, t0, t1 in regions:
            lo.sort_region(rec[a:b], ok_[a:b], ov_[a:b], reg, t0, t1)
    torch.cuda.synchronize()
    lo.check()
    assert ops.is_sorted(ok_)
    print(f"prof_driver: {reps} x {rounds} region sorts done")


if __name__ == "__main__":
    main()
