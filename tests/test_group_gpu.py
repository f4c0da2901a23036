"""GPU: the single-process multi-GPU sort through the C ABI (rs_group_*).

RCCL transport at world size 1 (the box has one GPU; ncclCommInitAll over one device), and the
peer-copy transport with device 0 listed 2-4 times: virtual ranks that run the whole multi-rank
path on one GPU — per-rank top-digit histograms, the host bucket plan, the stable partition into
records, every exchange round with uneven and empty segments, the region sorts behind the round
events — with only the wire differing from RCCL.  Checked against the oracle: the rank-ordered
concatenation equals the stable sort of the concatenated input, values = global input index
(so stability across ranks is checked too)."""
import numpy as np
import pytest
import torch

import oracle as O
from radix_sort_amd import RadixSortError, RadixSortGroup, _lib

pytestmark = pytest.mark.gpu


def _keys(kind, n, seed):
    u = O.gen_u32(seed, n)
    if kind == "uniform":
        return u
    if kind == "one_bucket":          # every key in the top bucket: one rank receives all
        return (u & np.uint32(0x00FFFFFF)) | np.uint32(0xFF000000)
    if kind == "dups":                # 64 distinct keys over 8 buckets
        return (u % np.uint32(64)) * np.uint32(0x04000001)
    if kind == "two_buckets":
        return np.where(u & np.uint32(1), u | np.uint32(0xF0000000), u & np.uint32(0x0FFFFFFF)).astype(np.uint32)
    raise ValueError(kind)


def _run(group, counts, kind, has_values, seed=11, stream=None):
    dev = torch.device("cuda", 0)
    host_k = [_keys(kind, n, seed + r) for r, n in enumerate(counts)]
    starts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    host_v = [np.arange(starts[r], starts[r + 1], dtype=np.uint32) for r in range(len(counts))]
    kt = [torch.from_numpy(k.view(np.int32)).to(dev) for k in host_k]
    vt = [torch.from_numpy(v.view(np.int32)).to(dev) for v in host_v] if has_values else None
    keep = [k.clone() for k in kt]
    if stream is not None:
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            out = group.sort(kt, vt)
    else:
        out = group.sort(kt, vt)
    for a, b in zip(kt, keep):                     # inputs are only read
        assert torch.equal(a, b)
    all_k = np.concatenate(host_k) if counts else np.zeros(0, np.uint32)
    all_v = np.concatenate(host_v) if counts else np.zeros(0, np.uint32)
    ek, ev = O.stable_sort_masked_c(all_k, all_v, 32)
    gk = np.concatenate([o[0].cpu().numpy().view(np.uint32) for o in out])
    assert gk.size == ek.size
    assert np.array_equal(gk, ek)
    if has_values:
        gv = np.concatenate([o[1].cpu().numpy().view(np.uint32) for o in out])
        assert np.array_equal(gv, ev)
    return [o[0].numel() for o in out]


@pytest.mark.parametrize("has_values", [True, False])
@pytest.mark.parametrize("n", [0, 1, 1000, 16387, 1 << 20, 13 << 20])
def test_rccl_world1(n, has_values):
    g = RadixSortGroup([0], capacity=max(n, 1), has_values=has_values, transport="rccl")
    try:
        _run(g, [n], "uniform", has_values)
    finally:
        g.destroy()


@pytest.mark.parametrize("kind", ["uniform", "one_bucket", "dups", "two_buckets"])
@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("has_values", [True, False])
def test_virtual_ranks(world, kind, has_values):
    counts = [300_000 + 777 * r for r in range(world)]
    counts[-1] = 5000 if world > 2 else counts[-1]        # ragged slices
    g = RadixSortGroup([0] * world, capacity=max(counts), has_values=has_values, transport="copy",
                       rounds=3)
    try:
        got = _run(g, counts, kind, has_values, seed=world)
        if kind == "one_bucket":      # a bucket never splits: one rank receives every key
            assert max(got) == sum(counts)
    finally:
        g.destroy()


@pytest.mark.parametrize("has_values", [True, False])
def test_virtual_ranks_one_sweep_sizes(has_values):
    # > 12M keys per rank: the partition runs the one-sweep records pass, the regions the
    # records sort; 4 rounds, the second sort reuses (and regrows) the group's buffers
    counts = [13 << 20, (12 << 20) + 5]
    g = RadixSortGroup([0, 0], capacity=max(counts), has_values=has_values, transport="copy")
    try:
        _run(g, counts, "uniform", has_values, seed=3)
        _run(g, [1 << 20, 13 << 20], "two_buckets", has_values, seed=4)
    finally:
        g.destroy()


def test_empty_rank_and_caller_stream():
    g = RadixSortGroup([0] * 3, capacity=100_000, has_values=True, transport="copy", rounds=2)
    s = torch.cuda.Stream(0)
    try:
        _run(g, [100_000, 0, 4321], "uniform", True, stream=s)
        _run(g, [0, 0, 0], "uniform", True)
    finally:
        g.destroy()


def test_capacity_and_duplicate_device_errors():
    g = RadixSortGroup([0, 0], capacity=1000, has_values=True, transport="copy")
    try:
        k = [torch.zeros(2000, dtype=torch.int32, device="cuda:0")] * 2
        with pytest.raises(RadixSortError) as e:
            g.sort_async(k, k)
        assert e.value.status == _lib.RS_ERR_CAPACITY
    finally:
        g.destroy()
    with pytest.raises(RadixSortError) as e:
        RadixSortGroup([0, 0], capacity=10, transport="rccl")
    assert "listed twice" in str(e.value)


@pytest.mark.slow
def test_config5_shape_eight_virtual_ranks():
    """BASELINE config 5's full shape on one GPU: 8 ranks x 2^28 u32 keys + values (2^31 in all,
    uniform, the splitmix counter generator over the global index), 4 exchange rounds, every rank
    a virtual rank on device 0 over the peer-copy transport - the same host plan, chunk layout,
    16-bit tables, partition passes and region sorts RCCL drives on an 8-GPU node; only the wire
    differs.  Checked by the size-independent properties (sorted within and across ranks, a top
    byte never split between ranks, values a permutation of the global indices with
    keys_out == keys_in[values_out], equal keys in input order), which determine the stable sort
    uniquely.  ~100 GB of HBM at peak."""
    from radix_sort_amd import ops
    W, n = 8, 1 << 28
    dev = torch.device("cuda", 0)
    kt, vt = [], []
    for r in range(W):
        k = torch.empty(n, dtype=torch.int32, device=dev)
        ops.fill_random_u32(k, 5, r * n)
        v = torch.empty(n, dtype=torch.int32, device=dev)
        ops.fill_iota_u32(v, r * n)
        kt.append(k)
        vt.append(v)
    g = RadixSortGroup([0] * W, capacity=n, has_values=True, transport="copy", rounds=4)
    try:
        out = g.sort(kt, vt)
    finally:
        g.destroy()
    kin = torch.cat(kt)
    del kt, vt
    sizes = [o[0].numel() for o in out]
    assert sum(sizes) == W * n
    assert max(sizes) < 1.1 * n and min(sizes) > 0.9 * n          # ~1/8 of the keys per rank
    prev_last = None
    for ko, _ in out:
        assert ops.is_sorted(ko)
        first, last = int(ko[0]) & 0xFFFFFFFF, int(ko[-1]) & 0xFFFFFFFF
        if prev_last is not None:
            assert (first >> 24) > (prev_last >> 24)               # whole top bytes per rank
        prev_last = last
    seen = torch.zeros(W * n, dtype=torch.bool, device=dev)
    for ko, vo in out:
        vi = vo.long() & 0xFFFFFFFF
        seen[vi] = True
        for a in range(0, ko.numel(), 1 << 27):
            b = min(ko.numel(), a + (1 << 27))
            assert torch.equal(kin[vi[a:b]], ko[a:b])
        eq = ko[1:] == ko[:-1]
        assert bool((vi[1:][eq] > vi[:-1][eq]).all())
        del vi
    assert bool(seen.all())


def test_group_times_explain_the_step():
    """rs_group_set_profiling / rs_group_times_get: every rank's step breakdown (16-bit table,
    partition, each round's comm-stream completion, each region's sort, done) is ordered in time,
    and the off-rank bytes match what the ranks actually exchanged (virtual ranks over copies)."""
    from radix_sort_amd import ops
    W, n, G = 3, 3 << 20, 4
    dev = torch.device("cuda", 0)
    kt, vt = [], []
    for r in range(W):
        k = torch.empty(n, dtype=torch.int32, device=dev)
        ops.fill_random_u32(k, 21, r * n)
        v = torch.empty(n, dtype=torch.int32, device=dev)
        ops.fill_iota_u32(v, r * n)
        kt.append(k)
        vt.append(v)
    g = RadixSortGroup([0] * W, capacity=n, has_values=True, transport="copy", rounds=G)
    try:
        with pytest.raises(RadixSortError):
            g.times(0)                       # no profiled sort yet
        g.set_profiling(True)
        out = g.sort(kt, vt)
        total_sent = total_recv = 0
        for r in range(W):
            t = g.times(r)
            assert t["rounds"] == G
            assert 0 < t["hist16_ms"] <= t["partition_ms"] <= t["region_sorted_ms"][0]
            assert all(a <= b for a, b in zip(t["region_sorted_ms"], t["region_sorted_ms"][1:]))
            assert t["region_sorted_ms"][-1] <= t["done_ms"]
            assert all(x >= t["partition_ms"] for x in t["round_done_ms"])
            total_sent += t["bytes_sent"]
            total_recv += t["bytes_recv"]
            # what rank r received from the others: its records minus its own keys in its top bytes
            lo_top = (int(out[r][0][0]) & 0xFFFFFFFF) >> 24
            hi_top = (int(out[r][0][-1]) & 0xFFFFFFFF) >> 24
            top = (kt[r].long() & 0xFFFFFFFF) >> 24
            own = int(((top >= lo_top) & (top <= hi_top)).sum())
            assert t["bytes_recv"] == 8 * (out[r][0].numel() - own)
        assert total_sent == total_recv > 0
        assert sum(o[0].numel() for o in out) == W * n
    finally:
        g.destroy()
