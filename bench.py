#!/usr/bin/env python3
"""Headline benchmark: Gkeys/s of the MI355X-native 4-way LSD radix sort (BASELINE.json metric
"Gkeys/s sorted (32-bit keys+values) at 1/2/4/8 MI355X; % HBM roofline").

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config3]

A step = one full sort of one batch of synthetic input resident in HBM:
* N = 1: BASELINE configs[2] — 256M (2^28) uniform u32 keys + u32 values (iota),
  local_shuffle=true, bit_count 32, one RadixSortKernel.dispatch() per step.  Every step sorts a
  different pre-generated batch (sorting already-sorted data would be a different workload).
  The library takes its hybrid MSD path here: `roofline` is the scatter kernel
  (k_msd_pass, 2 launches per sort), `bucket_pass` the in-LDS bucket kernel.  `--workload
  config2` (64M keys only) takes the keys-only form of the same path (one wave per 16-bit bucket).
* N > 1 (torch.distributed.run, one process per GPU, RCCL): BASELINE configs[4] shape with
  2^28 keys+values per rank (2^31 at 8 GPUs): histogram all_gather -> stable top-byte partition
  into (key, value) records -> 4 rounds of batched RCCL point-to-point record messages over
  xGMI (bucket groups), each group sorted locally while the later rounds are in flight (the
  hybrid MSD path over the group's key range, rs_plan_sort_records_range).
  Weak scaling.

Rank 0 prints ONE JSON line.  `value` = keys sorted by all ranks / max-over-ranks wall time.
`roofline` is for the dominant kernel (the scatter pass): algorithmic bytes per launch
(n x (4 + 4) read + n x (4 + 4) write for keys+values) / its average launch duration, timed with
HIP events on the launch stream inside the timed region.  `cpu_baseline` times the reference's
CPU path (`Uint32Array.prototype.sort((a, b) => a - b)`, example/index.ts:85) in Node on a bounded
sample on this host (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "webgpu-radix-sort_amd"))

HBM_PEAK_GBS = 8000.0    # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
EXCHANGE_ROUNDS = 4      # multi-GPU: bucket groups per rank, each sorted while later rounds fly

WORKLOADS = {
    "config3": dict(n=1 << 28, values=True, local_shuffle=True, check_order=False, kind="u32",
                    seed=3, desc="256M Uint32 keys + Uint32 values, local_shuffle=true, 1xMI355X"),
    "config2": dict(n=1 << 26, values=False, local_shuffle=False, check_order=False, kind="u32",
                    seed=2, desc="64M Uint32 keys-only, bit_count=32, workgroup_size 16x16"),
    "config4": dict(n=1 << 28, values=True, local_shuffle=False, check_order=True,
                    kind="f32_nearly", seed=4,
                    desc="256M Float32 keys (nearly sorted) + Uint32 values, check_order=true"),
    # config3 with check_order=true on unsorted input (the order check rides on the hybrid path's
    # histogram read)
    "config3_check_order": dict(n=1 << 28, values=True, local_shuffle=True, check_order=True, kind="u32",
                                seed=3, desc="256M Uint32 keys + Uint32 values, check_order=true, unsorted"),
    # config3's data as one rg32uint texture of (key, value) texels (RadixSortTextureKernel)
    "config3_texture": dict(n=1 << 28, values=True, local_shuffle=False, check_order=False,
                            kind="u32", seed=3, layout="aos",
                            desc="256M (Uint32 key, Uint32 value) texels, RadixSortTextureKernel"),
    # the exported PrefixSumKernel (src/index.ts:3, PrefixSumKernel.ts:11-159) on its own
    "prefix_sum": dict(n=1 << 28, values=False, local_shuffle=False, check_order=False, kind="scan",
                       seed=6, desc="PrefixSumKernel: in-place exclusive scan of 256M u32 (single pass)"),
}


def bench_prefix_sum(args, wl, torch, json_out) -> None:
    """--workload prefix_sum: K in-place exclusive scans of pre-generated 2^28 u32 batches (small
    values: the reference test's data, example/tests.ts:135), timed wall-clock around all K and with
    HIP events around each launch; roofline at 8 B/element (one read + one write); CPU baseline: the
    reference's prefixSumCpu loop restated in numpy (example/tests.ts:288-296), 1 core, 2^26 sample."""
    import numpy as np
    from radix_sort_amd import PrefixSumKernel, ops
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    n = args.keys_per_gpu or wl["n"]
    K, W = args.steps, args.warmup
    dev = torch.device("cuda", 0)

    def make(seed):
        t = torch.empty(n, dtype=torch.int32, device=dev)
        ops.fill_random_u32(t, seed)
        t &= 7                                   # floor(random * 8), as the reference's test data
        return t
    batches = [make(wl["seed"] + i) for i in range(K)]
    warm = make(wl["seed"] + 1000)
    kw = PrefixSumKernel(data=warm, count=n)
    for _ in range(W):
        kw.dispatch()
    kernels = [PrefixSumKernel(data=b, count=n) for b in batches]
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    t0 = time.perf_counter()
    for i in range(K):
        ev[i][0].record()
        kernels[i].dispatch()
        ev[i][1].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    for k in kernels:
        k.check()
    kms = sum(a.elapsed_time(b) for a, b in ev) / K
    # the last batch against the numpy restatement of prefixSumCpu
    src = make(wl["seed"] + K - 1).cpu().numpy().view(np.uint32)
    got = batches[-1].cpu().numpy().view(np.uint32)
    if not (got == O.prefix_sum(src, n)).all():
        raise SystemExit("bench: prefix sum differs from the reference's CPU scan")
    value = n * K / elapsed / 1e9
    achieved = n * 8 / (kms / 1e3) / 1e9
    # PMC traffic of the scan kernel (tools/pmc_traffic.py prefix_sum), for this library only
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f).get("prefix_sum")
        if tj and n == tj.get("n") and tj.get("lib_sha16") == _lib_sha16():
            traffic = tj.get("scan_bytes_per_launch")
    except (OSError, ValueError):
        pass
    cpu = None
    if not args.no_cpu_baseline:
        m = 1 << 26
        d = src[:m].copy()
        t = time.perf_counter()
        O.prefix_sum(d, m)
        dt = time.perf_counter() - t
        cpu = {"value": m / dt / 1e9, "unit": "Gelements/s", "cores": 1, "kind": "port",
               "sample": f"2^26 u32, numpy cumsum restatement of prefixSumCpu (example/tests.ts:288-296), 1 thread; {dt:.3f} s"}
    out = {"metric": "Gelements/s exclusive prefix sum (u32), PrefixSumKernel; % HBM roofline",
           "value": round(value, 4), "unit": "Gelements/s", "n_gpus": 1, "steps": K, "warmup": W,
           "ms_per_step": round(elapsed / K * 1e3, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32",
           "data": "synthetic (splitmix64 counter generator, values in [0, 8))",
           "config": {"workload": "prefix_sum", "description": wl["desc"], "elements": n},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                        "kernel": "k_scan_lookback (single pass, decoupled look-back)",
                        "avg_launch_ms": round(kms, 4), "algorithmic_bytes_per_launch": n * 8,
                        "lib_sha16": _lib_sha16()},
           "cpu_baseline": cpu}
    print(json.dumps(out), file=json_out, flush=True)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _lib_sha16() -> str:
    """First 16 hex digits of the sha256 of the librsort.so this run loads."""
    import hashlib
    lib = os.environ.get("RSORT_LIB", os.path.join(ROOT, "webgpu-radix-sort_amd", "lib", "librsort.so"))
    with open(lib, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _node_sort(keys) -> dict:
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "keys.bin")
        keys.tofile(p)
        out = subprocess.run(["node", os.path.join(ROOT, "oracle", "cpu_sort_ref.js"), p],
                             capture_output=True, text=True, timeout=600, check=True)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["sorted"]
    return r


def cpu_baseline(sizes_log2, seed: int, target_log2: int = 28) -> dict:
    """Reference CPU path timed in Node on this host (kind 'reference'): the samples of
    BASELINE.md §3 / SURVEY §8(d) (2^20 mandatory, then larger ones up to ~10-30 s of CPU work),
    `value` = the rate at the largest sample, plus two clearly labelled extrapolations to the
    workload size (never measured: the comparator sort at 2^28 would take hours).  Falls back to
    the C oracle's single-threaded stable sort (kind 'port') when Node is absent."""
    import math
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    sizes_log2 = sorted(sizes_log2)
    try:
        points = []
        for lg in sizes_log2:
            r = _node_sort(O.gen_u32(seed, 1 << lg))
            points.append({"n": 1 << lg, "seconds": round(r["ms"] / 1e3, 4),
                           "gkeys_per_s": (1 << lg) / (r["ms"] / 1e3) / 1e9})
        big = points[-1]
        n_t = 1 << target_log2
        # n log n from the largest sample, and a power law fitted through all samples (the
        # comparator sort is super-linear beyond n log n here: cache misses grow with n)
        t_nlogn = big["seconds"] * (n_t * target_log2) / (big["n"] * math.log2(big["n"]))
        xs = [math.log(p["n"]) for p in points]
        ys = [math.log(p["seconds"]) for p in points]
        if len(points) > 1:
            mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
            b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
            t_pow = math.exp(my + b * (math.log(n_t) - mx))
        else:
            b, t_pow = 1.0, t_nlogn
        return {"value": big["gkeys_per_s"], "unit": "Gkeys/s", "cores": 1, "kind": "reference",
                "sample": (f"2^{sizes_log2[-1]} uniform u32 keys (keys only, as the reference's demo "
                           f"times it), Uint32Array.sort((a,b)=>a-b) in Node {r['node']} on "
                           f"'{r['cpu_model']}' ({r['cpus']} host cpus, 1 used); "
                           f"{big['seconds']:.2f} s"),
                "seconds": big["seconds"], "points": points,
                "extrapolated_to_workload": {
                    "n": n_t, "measured": False,
                    "nlogn_from_largest_sample_s": round(t_nlogn, 1),
                    "nlogn_gkeys_per_s": n_t / t_nlogn / 1e9,
                    "power_law_fit_s": round(t_pow, 1), "power_law_exponent": round(b, 3),
                    "power_law_gkeys_per_s": n_t / t_pow / 1e9,
                    "note": "EXTRAPOLATED, not measured"}}
    except (OSError, subprocess.SubprocessError, ValueError, AssertionError) as e:
        log(f"node baseline unavailable ({e!r}); timing the C oracle instead")
        lg = sizes_log2[-1]
        n = 1 << lg
        keys = O.gen_u32(seed, n)
        vals = np.arange(n, dtype=np.uint32)
        t = time.perf_counter()
        O.stable_sort_masked_c(keys, vals, 32)
        dt = time.perf_counter() - t
        return {"value": n / dt / 1e9, "unit": "Gkeys/s", "cores": 1, "kind": "port",
                "sample": f"2^{lg} u32 keys + values, oracle/rs_oracle.c stable LSD, 1 thread",
                "seconds": dt}


_NEARLY = {}


def _splitmix_u32(seed: int, n: int) -> "np.ndarray":
    """key[i] = low32(splitmix64 finaliser(seed * 0xD1B54A32D192ED03 + i)): the same counter
    generator as the device fill (rs_fill_random_u32), on the host."""
    import numpy as np
    with np.errstate(over="ignore"):
        z = np.uint64((seed * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF) + np.arange(n, dtype=np.uint64)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def nearly_sorted_f32_bits(n: int, seed: int) -> "np.ndarray":
    """BASELINE config4 input: f32 keys (u >> 8) * 2^-24 in [0, 1) sorted
    ascending, then n // 1000 seeded transpositions applied in sequence; raw u32 bits."""
    import numpy as np
    keys = ((_splitmix_u32(seed, n) >> np.uint32(8)).astype(np.float64) * 2.0 ** -24).astype(np.float32)
    keys.sort(kind="stable")
    bits = keys.view(np.uint32).copy()
    swaps = max(1, n // 1000)
    r = _splitmix_u32(seed ^ 0x5EED, 2 * swaps).astype(np.uint64)
    a = (r[0::2] % np.uint64(n)).astype(np.int64)
    b = (r[1::2] % np.uint64(n)).astype(np.int64)
    for x, y in zip(a.tolist(), b.tolist()):
        bits[x], bits[y] = bits[y], bits[x]
    return bits


def make_input(torch, ops, wl, n, seed, start, dev):
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    if wl["kind"] == "f32_nearly":
        # host generation of the nearly-sorted f32 input (untimed, ~30 s at 2^28), done once:
        # every batch is a fresh copy of the same input (a sorted batch would be a different
        # workload), so only the first seed is used
        if n not in _NEARLY:
            log(f"generating the nearly-sorted f32 input (n={n}) on the host ...")
            _NEARLY[n] = torch.from_numpy(nearly_sorted_f32_bits(n, seed).view("int32"))
        keys.copy_(_NEARLY[n])
    else:
        ops.fill_random_u32(keys, seed, start)
    vals = None
    if wl["values"]:
        vals = torch.empty(n, dtype=torch.int32, device=dev)
        ops.fill_iota_u32(vals, start)
    if wl.get("layout") == "aos":
        rec = torch.stack([keys, vals], dim=1).contiguous()   # [n, 2] texels
        return rec, None
    return keys, vals


def make_kernel(RadixSortKernel, RadixSortTextureKernel, wl, local, k, v, n, radix_bits):
    if wl.get("layout") == "aos":
        return RadixSortTextureKernel(device=local, texture=k, count=n, bit_count=32,
                                      check_order=wl["check_order"], radix_bits=radix_bits)
    return RadixSortKernel(device=local, keys=k, values=v, count=n, bit_count=32,
                           local_shuffle=wl["local_shuffle"], check_order=wl["check_order"],
                           radix_bits=radix_bits)


def verify_batch(torch, ops, wl, n, seed, batch, dev) -> None:
    """The sorted batch against its regenerated input: keys sorted (unsigned), values a
    permutation with keys_out == keys_in[values_out] (values start as iota), equal keys in input
    order.  Raises SystemExit on any mismatch."""
    kin, _ = make_input(torch, ops, wl, n, seed, 0, dev)
    if wl.get("layout") == "aos":
        kin = kin[:, 0].contiguous()
        ko, vo = batch[0][:, 0].contiguous(), batch[0][:, 1].contiguous()
    else:
        ko, vo = batch
    if not ops.is_sorted(ko):
        raise SystemExit("bench: output not sorted")
    if vo is None:
        return
    v = vo.long()
    if not torch.equal(torch.bincount(v, minlength=n), torch.ones(n, dtype=torch.long, device=dev)):
        raise SystemExit("bench: values are not a permutation")
    if not torch.equal(kin[v], ko):
        raise SystemExit("bench: keys_out != keys_in[values_out]")
    eq = ko[1:] == ko[:-1]
    if not bool((v[1:][eq] > v[:-1][eq]).all()):
        raise SystemExit("bench: equal keys out of input order (not stable)")


def launch_plan(gpus: int, env: dict, device_count: int, argv: list) -> tuple:
    """How this invocation runs `--gpus N` (decided before anything touches the GPU).

    `--share-gpu` (rehearsal only, never a measurement): every rank on GPU 0 over gloo, so one
    visible GPU is enough.

    -> ("run", None): this process is the bench (N = 1 alone, or one rank of a launcher whose
       WORLD_SIZE equals N);
       ("spawn", cmd): N > 1 without a launcher: start N rank processes under
       torch.distributed.run (one per GPU, RCCL) as a child and exit with its status;
       ("error", message): never silently measure fewer GPUs than asked for."""
    if gpus < 1:
        return "error", f"--gpus must be >= 1 (got {gpus})"
    if "--share-gpu" in argv:
        device_count = gpus if device_count >= 1 else 0
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            return "error", (f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks; "
                             "they must agree")
        if int(world) > device_count:
            return "error", f"WORLD_SIZE={world} but only {device_count} GPU(s) are visible"
        return "run", None
    if gpus == 1:
        return ("run", None) if device_count >= 1 else ("error", "no GPU visible")
    if device_count < gpus:
        return "error", f"--gpus {gpus} but only {device_count} GPU(s) are visible"
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return "spawn", cmd


def _gpus_arg(argv: list) -> int:
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    return ap.parse_known_args(argv)[0].gpus


def main() -> None:
    # `--gpus N` must measure N GPUs however it is started: a plain `python bench.py --gpus N`
    # starts N ranks itself (before any GPU call in this process); a launcher's WORLD_SIZE must
    # match N; fewer visible GPUs than N is an error, never a 1-GPU line
    import torch   # device_count() does not initialise the GPU
    what, arg = launch_plan(_gpus_arg(sys.argv[1:]), dict(os.environ), torch.cuda.device_count(),
                            sys.argv[1:])
    if what == "error":
        raise SystemExit(f"bench: {arg}")
    if what == "spawn":
        log("bench: starting " + " ".join(arg))
        raise SystemExit(subprocess.run(arg).returncode)
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="config3", choices=sorted(WORKLOADS))
    # (not "--n": torch.distributed.run, which re-reads this command line when --gpus N spawns the
    # ranks, rejects it as an ambiguous abbreviation of its own options)
    ap.add_argument("--keys-per-gpu", type=int, default=0, help="override keys per GPU (testing only)")
    ap.add_argument("--radix-bits", type=int, default=0)
    ap.add_argument("--rank", default="lds", choices=["lds", "ballot"],
                    help="in-wave ranking: lane-ordered LDS atomics (default, self-tested per device) or "
                         "the architecture-guaranteed ballot ranking (rs_plan_debug.rank = 1)")
    ap.add_argument("--plan-debug", default="",
                    help="A/B diagnostics: rs_plan_debug overrides for every plan, e.g. 'xcd=0,presorted=0'")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--distributed", action="store_true",
                    help="use the bucket-exchange path even at world size 1 (testing)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal of the N-rank path on one GPU: every rank on GPU 0, gloo moves "
                         "the exchange through host copies (the line is marked; not a measurement)")
    ap.add_argument("--cpu-log2", default="20,22,24",
                    help="CPU baseline sample sizes (log2, comma-separated; 2^20 mandatory)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per scatter launch (tools/pmc_traffic.py)")
    args = ap.parse_args()

    # stdout carries exactly one JSON line: anything native code prints there (RCCL writes a
    # version banner to stdout when a communicator is created) goes to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist
    if WORKLOADS[args.workload]["kind"] == "scan":
        if args.gpus != 1:
            raise SystemExit("bench: the prefix_sum workload runs on one GPU")
        torch.cuda.set_device(0)
        bench_prefix_sum(args, WORKLOADS[args.workload], torch, json_out)
        return
    from radix_sort_amd import RadixSortKernel, RadixSortTextureKernel, _lib, ops
    if args.rank == "ballot":   # every plan of this process ranks by ballot
        _lib.plan_debug(rank="ballot").__enter__()
    if args.plan_debug:         # e.g. xcd=0: every plan of this process (A/B runs; marked in the line)
        fields = dict(kv.split("=", 1) for kv in args.plan_debug.split(","))
        _lib.plan_debug(**{k: int(v) for k, v in fields.items()}).__enter__()
    from radix_sort_amd.distributed import (HipLocalOps, StepTimeline, distributed_sort,
                                            summarize_timelines, timeline_record)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, (world, args.gpus)   # launch_plan enforced it
    if args.share_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = world > 1 or args.distributed or args.share_gpu
    backend = "gloo" if args.share_gpu else "nccl"
    wl = dict(WORKLOADS[args.workload])
    if use_dist and wl.get("layout") == "aos":
        raise SystemExit("bench: the multi-GPU path sorts separate key/value arrays; "
                         "use config3 for --gpus > 1")
    if use_dist and "RANK" not in os.environ:     # --distributed without a launcher: world 1
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port))
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    n = args.keys_per_gpu or wl["n"]
    K, W = args.steps, args.warmup

    def barrier():
        if use_dist:
            dist.barrier()

    kernel_ms = {}
    extra = {}
    if not use_dist:
        # One pre-generated batch per timed step (HBM holds them: 2 GiB each for config3).
        per_batch = n * 4 * (2 if wl["values"] else 1)
        free, _ = torch.cuda.mem_get_info(dev)
        max_batches = max(1, int((free - 4 * per_batch) // (2 * per_batch)))  # batch + its plan's tmp
        nb = min(K, max_batches)
        if nb < K:
            log(f"note: {K} steps but room for {nb} batches; later steps re-sort batches")
        batches = [make_input(torch, ops, wl, n, wl["seed"] + 7919 * i, 0, dev) for i in range(nb)]
        wk, wv = make_input(torch, ops, wl, n, wl["seed"] + 999331, 0, dev)
        kern = make_kernel(RadixSortKernel, RadixSortTextureKernel, wl, local, wk, wv, n,
                           args.radix_bits)
        kernels = [make_kernel(RadixSortKernel, RadixSortTextureKernel, wl, local, b[0], b[1], n,
                               args.radix_bits) for b in batches]
        for w in range(W):
            if w:
                wk2, wv2 = make_input(torch, ops, wl, n, wl["seed"] + 999331 + w, 0, dev)
                wk.copy_(wk2)
                if wv is not None:
                    wv.copy_(wv2)
                del wk2, wv2
            kern.dispatch()
        torch.cuda.synchronize()
        # inside the timed region HIP events bracket only the pass launches (the roofline's kernel:
        # the scatter passes, or the LSD passes of the device's fallback); every other launch group
        # runs back to back, as it does unprofiled
        # (check_order: the presorted path's order scan too, the "check" kind: its roofline kernel)
        timed_kinds = ("scatter", "fallback") + (("check",) if wl["check_order"] else ())
        for k in kernels:
            k.set_profiling(True, kinds=timed_kinds)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            kernels[i % nb].dispatch()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        for k in kernels:
            for name, v in k.kernel_times(reset=True).items():
                acc = kernel_ms.setdefault(name, {"ms": 0.0, "launches": 0})
                acc["ms"] += v["ms"]
                acc["launches"] += v["launches"]
            k.set_profiling(False)
        # the per-kind breakdown (and which path the device took): a few more sorts of fresh
        # unsorted batches after the timed region, every launch group bracketed
        nbd = 3
        kern.set_profiling(True)
        for j in range(nbd):
            fk, fv = make_input(torch, ops, wl, n, wl["seed"] + 424242 + j, 0, dev)
            wk.copy_(fk)
            if wv is not None:
                wv.copy_(fv)
            del fk, fv
            kern.dispatch()
        torch.cuda.synchronize()
        for name, v in kern.kernel_times(reset=True).items():
            if name not in timed_kinds:
                # per-sort times of the untimed runs, scaled to K sorts (reported per step below)
                kernel_ms[name] = {"ms": v["ms"] / nbd * K, "launches": round(v["launches"] / nbd * K)}
        kern.set_profiling(False)
        extra["breakdown_from"] = (f"{nbd} profiled sorts after the timed region (the timed region "
                                   "brackets only the pass launches with HIP events)")
        # outside the timed region: no sort failed on the device (a timed-out look-back wait
        # would make its output invalid), and the last batch is a stable sorted permutation
        for k in kernels:
            k.check()
        last = (K - 1) % nb
        verify_batch(torch, ops, wl, n, wl["seed"] + 7919 * last, batches[last], dev)
        info = kernels[0].info
        device_path = kernels[last].last_path()
        split_levels = kernels[last].last_split()
        keys_per_step = n
        scatter_keys = n
        bucket_keys = n
    else:
        keys, vals = make_input(torch, ops, wl, n, wl["seed"], rank * n, dev)
        # plans and receive buffers are created during the warmup steps (the local sort plan
        # grows once if a rank receives more than 1.25 n), so the timed steps allocate nothing
        lo = HipLocalOps(local, int(n * 1.25), wl["values"], args.radix_bits)
        r = None
        for _ in range(W):
            r = distributed_sort(keys, vals, lo, chunks=EXCHANGE_ROUNDS)
        torch.cuda.synchronize()
        from radix_sort_amd import _lib
        import ctypes
        _lib.load().rs_plan_set_profiling(lo.plan._plan, 1)
        if lo.part_plan is not None:     # the sender's plan: 16-bit table + partition
            _lib.load().rs_plan_set_profiling(lo.part_plan._plan, 1)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            r = distributed_sort(keys, vals, lo, chunks=EXCHANGE_ROUNDS)
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        lo.check()      # no local sort or partition failed on the device
        device_path = lo.plan.last_path()
        split_levels = lo.plan.last_split()
        ms = (ctypes.c_double * _lib.RS_KERNEL_KINDS)()
        cnt = (ctypes.c_uint64 * _lib.RS_KERNEL_KINDS)()
        _lib.load().rs_plan_kernel_times(lo.plan._plan, ms, cnt)
        for i, name in enumerate(_lib.KERNEL_NAMES):
            kernel_ms[name] = {"ms": ms[i], "launches": int(cnt[i])}
        if lo.part_plan is not None:
            _lib.load().rs_plan_kernel_times(lo.part_plan._plan, ms, cnt)
            extra["sender_kernel_ms_per_step"] = {
                "hist16 (rs_plan_hist16: one key read)": round(ms[_lib.RS_KERNEL_HISTOGRAM] / max(K, 1), 4),
                "partition (top-byte one-sweep pass -> records)": round(ms[_lib.RS_KERNEL_SCATTER] / max(K, 1), 4)}
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if not ops.is_sorted(r.keys, r.n):
            raise SystemExit(f"bench: rank {rank} output not sorted")
        if world > 1:
            # after the timed region: where a step's time goes on every rank (one step with GPU
            # event marks, one with the exchange rounds alone), gathered to rank 0 as the line's
            # multi_gpu breakdown (E, xGMI GB/s, the slowest rank's local terms, rank edges)
            my_kernel_ms = [kernel_ms[nm]["ms"] / max(K, 1) for nm in _lib.KERNEL_NAMES]
            if lo.part_plan is not None:
                my_kernel_ms += [ms[_lib.RS_KERNEL_HISTOGRAM] / max(K, 1), ms[_lib.RS_KERNEL_SCATTER] / max(K, 1)]
            else:
                my_kernel_ms += [0.0, 0.0]
            _lib.load().rs_plan_set_profiling(lo.plan._plan, 0)
            if lo.part_plan is not None:
                _lib.load().rs_plan_set_profiling(lo.part_plan._plan, 0)
            barrier()
            tl = StepTimeline()
            r = distributed_sort(keys, vals, lo, chunks=EXCHANGE_ROUNDS, timeline=tl)
            torch.cuda.synchronize()
            barrier()
            tle = StepTimeline(exchange_only=True)
            distributed_sort(keys, vals, lo, chunks=EXCHANGE_ROUNDS, timeline=tle)
            torch.cuda.synchronize()
            me = tle.ms()
            eo_ms = me.get(f"landed{EXCHANGE_ROUNDS - 1}", 0.0) - me.get("partition", 0.0)
            lo.check()
            if not ops.is_sorted(r.keys, r.n):
                raise SystemExit(f"bench: rank {rank} output not sorted (timeline step)")
            fk = int(r.keys[0].item()) & 0xFFFFFFFF if r.n else -1
            lk = int(r.keys[r.n - 1].item()) & 0xFFFFFFFF if r.n else -1
            row = timeline_record(tl, EXCHANGE_ROUNDS, fk, lk, r.n, my_kernel_ms, eo_ms)
            mine = torch.tensor(row, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            rows = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(rows, mine)
            names = list(_lib.KERNEL_NAMES) + ["sender_hist16", "sender_partition"]
            extra["multi_gpu"] = summarize_timelines([x.cpu().tolist() for x in rows], EXCHANGE_ROUNDS, names)
            extra["multi_gpu"]["from"] = ("one step with GPU event marks after the timed region (every rank), "
                                          "one step with the exchange rounds alone; kernel_ms = the timed "
                                          "steps' per-kind launch times")
        info = {"passes": 4}
        keys_per_step = n * world
        bucket_keys = r.n
        extra["recv_keys_rank0"] = r.n
        if world == 1:
            # one rank: nothing to exchange - the slice is sorted out of place in one sort
            scatter_keys = r.n
            extra["partition"] = "none (world size 1: one out-of-place sort of the slice)"
            extra["roofline_scope"] = "the rank's whole sort"
        else:
            # the local sort runs as `chunks` group sorts per step: a pass launch handles one group
            scatter_keys = r.n / EXCHANGE_ROUNDS
            extra["partition"] = (f"16-bit tables all-gathered; the top-byte partition is the sort's pass 0; "
                                  f"whole top bytes per rank, {EXCHANGE_ROUNDS} exchange rounds of one "
                                  "message per (source, byte) chunk, each round's region sorted (next-byte "
                                  "pass + bucket sort) while the later rounds are on the wire; "
                                  "52 B/key per rank")
            extra["roofline_scope"] = ("the receiver's segmented next-byte pass (rank 0; a pass launch "
                                       f"handles one of the {EXCHANGE_ROUNDS} regions)")
            extra["group_sorts_per_step"] = EXCHANGE_ROUNDS

    value = keys_per_step * K / elapsed / 1e9
    sc = kernel_ms.get("scatter", {"ms": 0.0, "launches": 0})
    bk = kernel_ms.get("bucket", {"ms": 0.0, "launches": 0})
    fb = kernel_ms.get("fallback", {"ms": 0.0, "launches": 0})
    hist_launches = kernel_ms.get("histogram", {"launches": 0})["launches"]
    # the hybrid MSD path (separate arrays >= 12M keys): two one-sweep passes (top byte, next byte
    # within top-byte segments) and the in-LDS 16-bit bucket pass; its LSD fallbacks are enqueued
    # too and gated off on the device unless the keys are too skewed (then they carry the time)
    # the path the device chose (rs_plan_last_path: the hybrid path's gate words, read back)
    msd = device_path == "hybrid"
    extra["device_path"] = device_path
    sp = kernel_ms.get("split", {"ms": 0.0, "launches": 0})
    if split_levels:
        # skewed keys: the 16-bit buckets over the bucket tile were split (count + pass by byte 1 +
        # in-LDS sort of the 24-bit sub-buckets; level 3: count + pass by byte 0)
        extra["bucket_split"] = {"levels": split_levels, "ms_per_sort": round(sp["ms"] / max(K, 1), 4)}
    if device_path == "hybrid_fallback":
        sc = fb        # the device took the LSD fallback: its passes are the pass launches
    presorted = device_path == "presorted"
    # one-sweep path: one digit-count launch per sort instead of one per pass
    onesweep = msd or 0 < hist_launches < sc["launches"]
    bytes_per_key = 16 if wl["values"] else 8
    roof = None
    if msd:
        # the gated-off fallback launches are not pass launches: the scatter kind holds the two
        # MSD passes exactly
        extra["path"] = ("hybrid MSD: top-byte one-sweep pass, 16-bit bucket histogram, next-byte "
                         "one-sweep pass per top-byte segment, in-LDS sort of every 16-bit bucket")
        extra["bucket_pass"] = {
            "kernel": "k_bucket_sort (one workgroup per 16-bit bucket, 2 LDS passes, contiguous writes)",
            "ms_per_sort": round(bk["ms"] / max(K, 1), 4),
            "achieved_GBs": round(bucket_keys * bytes_per_key / (bk["ms"] / max(K, 1) / 1e3) / 1e9, 1),
            "frac": round(bucket_keys * bytes_per_key / (bk["ms"] / max(K, 1) / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    elif presorted:
        # check_order, nearly sorted input: no radix pass ran (their launches are gated off)
        ck = kernel_ms.get("check", {"ms": 0.0, "launches": 0})
        ps = kernel_ms.get("presorted", {"ms": 0.0, "launches": 0})
        extra["path"] = ("presorted: order scan marking the displaced keys (k_ns_mark), their extraction "
                         "and stable sort, in-place merge of the movers (k_ns_merge); the radix "
                         "launches behind it gated off")
        extra["presorted_path"] = {"order_scan_ms_per_sort": round(ck["ms"] / max(K, 1), 4),
                                   "rest_ms_per_sort": round(ps["ms"] / max(K, 1), 4)}
    elif bk["launches"]:
        extra["path"] = "LSD one-sweep passes (the hybrid MSD path's device-side fallback: skewed keys)"
    if presorted:
        # the roofline is the whole presorted path (round 6; round 5 named its order scan, a minor
        # kernel): algorithmic bytes = every key read once by the order scan (4 B) + every element
        # the merge moved read and written once (16 B with values, 8 keys only), over the path's
        # time per sort (order scan + the rest, HIP events)
        ck = kernel_ms.get("check", {"ms": 0.0, "launches": 0})
        ps = kernel_ms.get("presorted", {"ms": 0.0, "launches": 0})
        if ck["launches"]:
            counts = kernels[last].presorted_counts()
            path_ms = (ck["ms"] + ps["ms"]) / max(K, 1)
            alg = n * 4 + counts["moved"] * bytes_per_key
            achieved = alg / (path_ms / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                    "kernel": "the presorted path (order scan k_ns_mark, extraction and its sort, "
                              "k_ns_merge of the movers): 4 B per key + %d B per moved element" % bytes_per_key,
                    "avg_launch_ms": round(path_ms, 4), "algorithmic_bytes_per_launch": alg,
                    "marked": counts["marked"], "moved": counts["moved"],
                    "lib_sha16": _lib_sha16(), "traffic_lib_sha16": None}
            scan_ms = ck["ms"] / ck["launches"]
            extra["presorted_path"]["order_scan_frac"] = round(n * 4 / (scan_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
    elif sc["launches"]:
        avg_ms = sc["ms"] / sc["launches"]
        achieved = scatter_keys * bytes_per_key / (avg_ms / 1e3) / 1e9
        # PMC traffic (tools/pmc_traffic.py, separate rocprofv3 passes): used only when it was
        # measured on this very library (its sha) and the single-GPU launch shape
        traffic, traffic_lib = None, None
        lib_sha = _lib_sha16()
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f).get(args.workload)
            if tj:
                traffic_lib = tj.get("lib_sha16")
            if tj and not use_dist and traffic_lib == lib_sha:
                traffic = tj.get("scatter_bytes_per_launch")
        except (OSError, ValueError):
            pass
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": (("k_msd_pass" if (msd and wl["values"]) else "k_onesweep")
                           + " (rank + look-back + local shuffle + scatter)"
                           if onesweep else "k_scatter (rank + local shuffle + scatter)"),
                "avg_launch_ms": round(avg_ms, 4),
                "algorithmic_bytes_per_launch": scatter_keys * bytes_per_key,
                "lib_sha16": lib_sha, "traffic_lib_sha16": traffic_lib}
    passes = info["passes"]
    # algorithmic HBM bytes of one sort per GPU: every pass reads and writes keys (+values);
    # the digit counts cost one key read per pass (histogram path) or one per sort (one-sweep
    # path: k_pass_totals reads the keys once, later totals come from the scatter itself)
    hist = kernel_ms.get("histogram", {"launches": 0})["launches"]
    hist_reads = max(1, round(hist / max(K, 1))) if hist else passes
    if use_dist and hist:
        hist_reads = 1   # one totals read per group sort: each key once per step
    if presorted:
        # no radix pass: one read of the keys (the order scan); the moved records are few
        passes = 0
        hist_reads = 1
    if msd:
        # MSD pass 0, MSD pass 1, bucket pass; one read of the input for the 16-bit histogram
        # (4 B/key arrays; records are read whole: 8 B/key = two 4-byte key reads)
        passes = 3
        hist_reads = 2 if wl.get("layout") == "aos" else 1
    sort_bytes = keys_per_step / max(world, 1) * (passes * (8 + 8 * (1 if wl["values"] else 0))
                                                  + 4 * hist_reads)
    extra["digit_count_reads_per_sort"] = hist_reads
    extra["whole_sort_hbm_GBs_per_gpu"] = round(sort_bytes / (elapsed / K) / 1e9, 1)
    extra["kernel_ms_per_step"] = {k: round(v["ms"] / max(K, 1), 4) for k, v in kernel_ms.items()
                                   if not (msd and k == "fallback")}
    if msd:
        extra["fallback_ms_per_step"] = round(fb["ms"] / max(K, 1), 4)
        extra["fallback"] = "LSD fallback launches enqueued behind the MSD passes, gated off on the device"
    extra["passes"] = passes

    cpu = None
    if rank == 0 and not use_dist and not args.no_cpu_baseline:
        cpu = cpu_baseline([int(x) for x in str(args.cpu_log2).split(",")], wl["seed"],
                           (n - 1).bit_length())

    if rank == 0:
        out = {
            "metric": "Gkeys/s sorted (32-bit keys+values) at 1/2/4/8 MI355X; % HBM roofline",
            "value": round(value, 4), "unit": "Gkeys/s", "n_gpus": world, "steps": K,
            "warmup": W, "ms_per_step": round(elapsed / K * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": ("synthetic: f32 keys (u>>8)*2^-24 sorted, then n/1000 seeded transpositions "
                     "(one input, a fresh copy per step); values = iota"
                     if wl["kind"] == "f32_nearly" else
                     "synthetic (splitmix64 counter generator, uniform u32; values = iota)"),
            "config": {"workload": args.workload, "description": wl["desc"], "keys_per_gpu": n,
                       "global_keys": n * world, "bit_count": 32, "has_values": wl["values"],
                       "local_shuffle": wl["local_shuffle"], "check_order": wl["check_order"],
                       "radix_bits": args.radix_bits or 8, "ranking": args.rank,
                       "parallelism": "single GPU" if world == 1 else
                       f"{world} ranks, top-byte bucket exchange (RCCL point-to-point rounds)"},
            "rccl_ranks": dist.get_world_size() if use_dist and backend == "nccl" else 0,
            "roofline": roof, "cpu_baseline": cpu, **extra,
        }
        if args.plan_debug:
            out["plan_debug"] = args.plan_debug   # an A/B run with path overrides, not the default build
        if args.share_gpu:
            out["rehearsal"] = (f"{world} gloo ranks sharing GPU 0, exchange through host copies: "
                                "tests the N-rank code path, NOT a measurement")
        print(json.dumps(out), file=json_out, flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
