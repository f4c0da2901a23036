"""Debug helper: keys-only / KV one-sweep sorts at the sizes of the GPU test, printing the device
error word and correctness per case (RSORT_* env selects the variant)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "webgpu-radix-sort_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import torch
import oracle as O
from radix_sort_amd import RadixSortKernel

for n, bits in ((16_385, 32), (100_003, 32), (2_500_000, 32), (5_000_001, 20), (40_000, 8), (300_000, 12)):
    keys = O.gen_u32(n * 3 + bits, n)
    ek, _ = O.stable_sort_masked(keys, None, bits)
    for kv in (False, True):
        kt = torch.from_numpy(keys.view(np.int32)).cuda()
        vt = torch.arange(n, dtype=torch.int32, device="cuda") if kv else None
        k = RadixSortKernel(keys=kt, values=vt, count=n, bit_count=bits)
        k.dispatch()
        err = k.device_errors()
        ok = bool((kt.cpu().numpy().view(np.uint32) == ek).all())
        print(f"n={n} bits={bits} kv={kv} info={k.info['tile_keys']},{k.info['grid_blocks']} err={err} ok={ok}", flush=True)
        k.destroy()
