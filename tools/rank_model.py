#!/usr/bin/env python3
"""The local work of one rank of the multi-GPU sort at BASELINE config 5's shape, measured on one
GPU (the exchange itself needs an 8-GPU node): 2^28 keys + values per rank, 8 ranks, 4 rounds.

  sender:   rs_plan_hist16 of the slice (one key read), the top-byte partition into records
  receiver: 4 region sorts (rs_plan_sort_region), each 2^26 records over 8 top bytes

The receiver's regions are synthesised as what it receives: keys whose top byte lies in the
rank's 32 bytes, grouped by top byte (a stable partition of them), with their 16-bit counts.
Prints one JSON line: ms per step of every piece (HIP events, median of --reps), the rank total,
and the single-GPU sort of 2^28 for comparison.

    python tools/rank_model.py [--reps 10]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "webgpu-radix-sort_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--n", type=int, default=1 << 28)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=4)
    args = ap.parse_args()
    import torch
    from radix_sort_amd import RadixSortKernel, ops
    from radix_sort_amd.distributed import HIST16_WORDS, HipLocalOps

    n, W, G = args.n, args.world, args.rounds
    dev = torch.device("cuda", 0)
    ev = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731

    def timed(fn):
        ts = []
        for _ in range(args.reps):
            a, b = ev(), ev()
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        return ts[len(ts) // 2]

    k = torch.empty(n, dtype=torch.int32, device=dev)
    ops.fill_random_u32(k, 5)
    v = torch.empty(n, dtype=torch.int32, device=dev)
    ops.fill_iota_u32(v)
    lo = HipLocalOps(0, int(n * 1.25), True)
    res = {}
    h16 = lo.hist16(k)
    res["sender_hist16"] = timed(lambda: lo.hist16(k))
    res["sender_partition"] = timed(lambda: lo.partition(k, v, 24, 8, h16[65536:]))
    # the receiver: the rank's 256 / W top bytes, its share of the global keys (n per rank)
    span = 256 // W
    rk = torch.empty(n, dtype=torch.int32, device=dev)
    ops.fill_random_u32(rk, 55)
    rk &= (span << 24) - 1                     # top bytes [0, span)
    rv = torch.arange(n, dtype=torch.int32, device=dev)
    rh = lo.hist16(rk)
    rec = lo.partition(rk, rv, 24, 8, rh[65536:])   # grouped by top byte, as received
    tops = rh[65536:].long().cpu().tolist()
    starts = [0]
    for c in tops:
        starts.append(starts[-1] + c)
    ok_, ov_ = torch.empty_like(rk), torch.empty_like(rv)
    per = span // G
    regions = []
    for g in range(G):
        t0, t1 = g * per, (g + 1) * per
        reg = torch.zeros(65536, dtype=torch.int32, device=dev)
        reg[t0 << 8:t1 << 8] = rh[t0 << 8:t1 << 8]
        regions.append((starts[t0], starts[t1], reg, t0, t1))

    def sort_regions():
        for a, b, reg, t0, t1 in regions:
            lo.sort_region(rec[a:b], ok_[a:b], ov_[a:b], reg, t0, t1)
    res["receiver_region_sorts"] = timed(sort_regions)
    torch.cuda.synchronize()
    lo.plan.set_profiling(True)
    sort_regions()
    torch.cuda.synchronize()
    res["receiver_kernel_ms"] = {a: round(b["ms"], 4) for a, b in lo.plan.kernel_times().items() if b["launches"]}
    lo.plan.set_profiling(False)
    lo.check()
    assert ops.is_sorted(ok_)
    res["rank_total_ms"] = res["sender_hist16"] + res["sender_partition"] + res["receiver_region_sorts"]
    # the single-GPU sort of n keys + values for comparison
    sk = torch.empty(n, dtype=torch.int32, device=dev)
    sv = torch.empty(n, dtype=torch.int32, device=dev)
    kern = RadixSortKernel(keys=sk, values=sv, count=n)

    def one_gpu():
        ops.fill_random_u32(sk, 7)
        kern.dispatch()
    fill = timed(lambda: ops.fill_random_u32(sk, 7))
    res["single_gpu_sort_ms"] = timed(one_gpu) - fill
    kern.destroy()
    del sk, sv
    # the single-GPU hybrid sort at 2^29 (16-bit buckets of ~8K records: the wide bucket kernel)
    for lg in (29, 30, 31):
        m = 1 << lg
        bk = torch.empty(m, dtype=torch.int32, device=dev)
        bv = torch.empty(m, dtype=torch.int32, device=dev)
        kb = RadixSortKernel(keys=bk, values=bv, count=m)
        ops.fill_random_u32(bk, 8)
        kb.dispatch()
        ops.fill_random_u32(bk, 9)
        kb.set_profiling(True)
        kb.dispatch()
        torch.cuda.synchronize()
        res[f"single_gpu_2pow{lg}_kernel_ms"] = {a: round(b["ms"], 4) for a, b in kb.kernel_times().items()
                                                 if b["launches"]}
        kb.destroy()
        del bk, bv
    res = {a: (round(b, 4) if isinstance(b, float) else b) for a, b in res.items()}
    res.update(n_per_rank=n, world=W, rounds=G, bytes_per_key_rank=52,
               note="exchange over xGMI not included (one-GPU box)")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
