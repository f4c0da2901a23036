"""Timing of a multi-GPU rank's local sorts (the config-5 shape on one GPU): 2^28 (key, index)
records whose keys span 32 top-byte buckets (rank 0 of 8), sorted as G rounds of 8 buckets each
with rs_plan_sort_records (LSD passes; the MSD path sees sparse buckets and is gated off) and with
rs_plan_sort_records_range (the hybrid MSD path over the round's 27 range-relative bits).
Prints one JSON line per (G, mode)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "webgpu-radix-sort_amd"))
from radix_sort_amd import _lib, ops  # noqa: E402
from radix_sort_amd.ops import SortPlan  # noqa: E402

dev = torch.device("cuda", 0)
N = 1 << 28
keys = torch.empty(N, dtype=torch.int32, device=dev)
ops.fill_random_u32(keys, 5)
keys &= 0x1FFFFFFF                     # top byte in [0, 32): rank 0 of 8
for G in (1, 4):
    # the round regions: keys of round g have top byte in [8g', 8g' + 8) with 32 / G buckets each
    per = 32 // G
    top = (keys >> 24) & 0xFF
    order = torch.argsort(top // per, stable=True)
    rk = keys[order]
    counts = [int(((top // per) == g).sum()) for g in range(G)]
    rec = torch.empty((N, 2), dtype=torch.int32, device=dev)
    rec[:, 0] = rk
    rec[:, 1] = torch.arange(N, dtype=torch.int32, device=dev)
    rec = rec.view(torch.int64).view(-1)
    ok_, ov_ = torch.empty(N, dtype=torch.int32, device=dev), torch.empty(N, dtype=torch.int32, device=dev)
    for mode in ("lsd", "range"):
        with _lib.plan_debug(msd=0 if mode == "lsd" else 1):
            plan = SortPlan(0, max(counts), True)

        def step():
            a = 0
            for g in range(G):
                b = a + counts[g]
                rng = ((g * per) << 24, (((g + 1) * per) << 24) - 1) if mode == "range" else None
                plan.sort_records(rec[a:b], ok_[a:b], ov_[a:b], b - a, key_range=rng)
                a = b
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            step()
        e1.record()
        torch.cuda.synchronize()
        plan.check()
        srt = ok_.clone()
        ok = bool((srt[1:].to(torch.int64) >= srt[:-1].to(torch.int64)).all())
        print(json.dumps({"rounds": G, "mode": mode, "ms_per_rank_sort": round(e0.elapsed_time(e1) / 5, 4),
                          "sorted": ok}), flush=True)
        plan.destroy()
