// rs_kernels.hpp — CDNA4 (gfx950) HIP kernels of the 4-way LSD radix sort.
//
// One global HBM pass sorts one digit of `w <= R` bits (R = 2: exactly the reference's 4-way
// pass; R = 8: four fused 4-way splits per HBM round trip).  Per pass, three kernels:
//
//   k_histogram  — per-workgroup digit counts over a contiguous chunk of tiles
//                  (the reference's block-sum half of radix_sort, RadixSort.ts:50-126)
//   k_scan_rows  — exclusive scan of the digit x workgroup count matrix, one row per digit,
//                  plus the per-digit totals (the PrefixSumKernel chain over the 4*WC
//                  block sums, PrefixSum.ts:13-106 / AbstractRadixSortKernel.ts:240)
//   k_scatter    — per tile: wavefront ballot ranking (stable, per digit), tile-level digit
//                  offsets, local shuffle through LDS (RadixSortLocalShuffle.ts:94-116),
//                  and a coalesced scatter of keys (+values) to their global positions
//                  (RadixSortReorder.ts:80-102)
//
// Data layout in HBM: keys / values are separate u32 arrays (structure of arrays, as the
// reference's two GPUBuffers); the count matrix is digit-major counts[d * G + g] like the
// reference's block_sums[b * WORKGROUP_COUNT + WORKGROUP_ID] (RadixSort.ts:113).
//
// Workgroup g of the histogram and scatter kernels owns the contiguous tile range
// [g*base + min(g, extra), ...) so its digit-d output for all its tiles is ONE contiguous run
// (the running per-digit base lives in a register of thread d): partial cache lines only at
// chunk edges, and the L2 of the owning XCD merges consecutive tile runs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rs {

constexpr int kBlock = 256;              // threads per workgroup: 4 waves of 64
constexpr int kWaves = kBlock / 64;

// ---- small helpers ---------------------------------------------------------------------

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Popcount of the bits of m below this lane (v_mbcnt_lo/hi).
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const uint32_t lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t u = __shfl_up(v, o, 64);
        if (lane >= (uint32_t)o) v += u;
    }
    return v;
}

// Exclusive scan of one u32 per thread over the 256-thread block.  `scratch` >= 4 u32 LDS.
// Contains two barriers; every thread of the block must call it.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t& total) {
    const uint32_t inc = wave_incl_scan(v);
    const uint32_t w = threadIdx.x >> 6;
    if (lane_id() == 63) scratch[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < (uint32_t)kWaves; ++i) {
        uint32_t s = scratch[i];
        pre += (i < w) ? s : 0u;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return pre + inc - v;
}

// check_order gate: inv[c] == 0 means check c found (or inherited) "sorted", so every kernel
// of pass >= c is skipped (replaces the reference's zeroed indirect dispatch sizes,
// CheckSort.ts:115-145).  gate == nullptr when check_order is off.
__device__ __forceinline__ bool gated_off(const uint32_t* gate, int upto) {
    if (!gate) return false;
    for (int c = 0; c <= upto; ++c)
        if (__builtin_nontemporal_load(gate + c) == 0u) return true;
    return false;
}

struct Chunk {          // tile range of one workgroup
    uint32_t first;     // first tile
    uint32_t count;     // number of tiles
};

__device__ __forceinline__ Chunk chunk_of(uint32_t g, uint32_t base, uint32_t extra) {
    Chunk c;
    c.first = g * base + (g < extra ? g : extra);
    c.count = base + (g < extra ? 1u : 0u);
    return c;
}

// ---- histogram (upsweep) -----------------------------------------------------------------
// counts[d * G + g] = number of keys of workgroup g's chunk whose digit is d.
template <int R, int TILE>
__global__ __launch_bounds__(kBlock) void k_histogram(
    const uint32_t* __restrict__ keys, uint32_t n, uint32_t shift, uint32_t mask,
    uint32_t base, uint32_t extra, uint32_t* __restrict__ counts, const uint32_t* gate, int pass) {
    constexpr int RADIX = 1 << R;
    __shared__ uint32_t hist[kWaves][RADIX];
    if (gated_off(gate, pass)) return;
    const uint32_t G = gridDim.x, g = blockIdx.x, tid = threadIdx.x, w = tid >> 6;
    for (uint32_t i = tid; i < (uint32_t)(kWaves * RADIX); i += kBlock) (&hist[0][0])[i] = 0u;
    __syncthreads();
    const Chunk ch = chunk_of(g, base, extra);
    const uint64_t lo64 = (uint64_t)ch.first * TILE;
    const uint32_t lo = (uint32_t)lo64;
    const uint64_t hi64 = lo64 + (uint64_t)ch.count * TILE;
    const uint32_t hi = (uint32_t)(hi64 < n ? hi64 : n);
    uint32_t* h = hist[w];
    const bool vec = (((uintptr_t)keys) & 15u) == 0;
    uint32_t i = lo;
    if (vec) {
        // 16-byte loads: every lane reads 4 consecutive keys; 1 KiB per wave-instruction.
        const uint32_t full_end = lo + ((hi - lo) & ~(uint32_t)(4 * kBlock - 1));
        for (; i < full_end; i += 4 * kBlock) {
            const uint4 q = *reinterpret_cast<const uint4*>(keys + i + 4 * tid);
            atomicAdd(&h[(q.x >> shift) & mask], 1u);
            atomicAdd(&h[(q.y >> shift) & mask], 1u);
            atomicAdd(&h[(q.z >> shift) & mask], 1u);
            atomicAdd(&h[(q.w >> shift) & mask], 1u);
        }
    }
    for (uint32_t j = i + tid; j < hi; j += kBlock) atomicAdd(&h[(keys[j] >> shift) & mask], 1u);
    __syncthreads();
    for (uint32_t d = tid; d < (uint32_t)RADIX; d += kBlock) {
        uint32_t s = 0;
#pragma unroll
        for (int v = 0; v < kWaves; ++v) s += hist[v][d];
        counts[(size_t)d * G + g] = s;
    }
}

// ---- digit x workgroup scan ----------------------------------------------------------------
// Block d scans row d of counts (G entries) to an exclusive prefix in place and writes the row
// total to totals[d].
__global__ __launch_bounds__(kBlock) void k_scan_rows(uint32_t* __restrict__ counts, uint32_t G,
                                                      uint32_t* __restrict__ totals,
                                                      const uint32_t* gate, int pass) {
    __shared__ uint32_t scratch[kWaves];
    if (gated_off(gate, pass)) return;
    uint32_t* row = counts + (size_t)blockIdx.x * G;
    const uint32_t per = (G + kBlock - 1) / kBlock;
    const uint32_t b0 = threadIdx.x * per;
    uint32_t s = 0;
    for (uint32_t k = 0; k < per; ++k)
        if (b0 + k < G) s += row[b0 + k];
    uint32_t tot;
    uint32_t run = block_excl_scan(s, scratch, tot);
    for (uint32_t k = 0; k < per; ++k)
        if (b0 + k < G) {
            uint32_t c = row[b0 + k];
            row[b0 + k] = run;
            run += c;
        }
    if (threadIdx.x == 0) totals[blockIdx.x] = tot;
}

// ---- rank + local shuffle + scatter (downsweep) ----------------------------------------
// Tile = 256 threads x KPT keys.  Wave w owns positions [w*64*KPT, (w+1)*64*KPT) of the tile;
// slot j of lane l is position w*64*KPT + j*64 + l (coalesced 256-B loads per slot).
template <int R, int KPT, bool HAS_VALUES, bool STAGED>
__global__ __launch_bounds__(kBlock) void k_scatter(
    const uint32_t* __restrict__ in_k, const uint32_t* __restrict__ in_v,
    uint32_t* __restrict__ out_k, uint32_t* __restrict__ out_v, uint32_t n, uint32_t shift,
    uint32_t mask, uint32_t nbits, uint32_t base, uint32_t extra,
    const uint32_t* __restrict__ counts, const uint32_t* __restrict__ totals,
    const uint32_t* gate, int pass) {
    constexpr int RADIX = 1 << R;
    constexpr int TILE = kBlock * KPT;
    constexpr int WAVE_KEYS = 64 * KPT;
    static_assert(RADIX <= kBlock, "one digit per thread");
    __shared__ uint32_t s_whist[kWaves][RADIX];     // per-wave counts -> per-wave tile offsets
    __shared__ uint32_t s_gdelta[RADIX];             // global pos - tile pos, per digit
    __shared__ uint32_t s_scratch[kWaves];
    __shared__ uint32_t s_keys[STAGED ? TILE : 1];
    __shared__ uint32_t s_vals[(STAGED && HAS_VALUES) ? TILE : 1];

    if (gated_off(gate, pass)) return;
    const uint32_t G = gridDim.x, g = blockIdx.x, tid = threadIdx.x;
    const uint32_t w = tid >> 6, lane = lane_id();

    // Running global base of digit `tid` for this workgroup:
    //   sum of totals of smaller digits + this row's exclusive prefix.
    uint32_t dtot = (tid < (uint32_t)RADIX) ? totals[tid] : 0u;
    uint32_t all;
    uint32_t run = block_excl_scan(dtot, s_scratch, all);
    if (tid < (uint32_t)RADIX) run += counts[(size_t)tid * G + g];

    const Chunk ch = chunk_of(g, base, extra);
    for (uint32_t t = 0; t < ch.count; ++t) {
        const uint32_t tile0 = (ch.first + t) * (uint32_t)TILE;
        const uint32_t wbase = tile0 + w * WAVE_KEYS;
        uint32_t k[KPT];
        uint32_t v[HAS_VALUES ? KPT : 1];
        uint32_t rank[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t p = wbase + j * 64 + lane;
            k[j] = (p < n) ? in_k[p] : 0u;
            if (HAS_VALUES) v[j] = (p < n) ? in_v[p] : 0u;
        }
        // zero this wave's counters (the previous tile's readers finished at the last barrier)
        for (uint32_t d = lane; d < (uint32_t)RADIX; d += 64) s_whist[w][d] = 0u;

        // Wavefront ballot ranking: for each slot, the lanes holding my digit (match mask),
        // my rank among them (mbcnt) and the slot count; the lowest such lane bumps the
        // wave's counter.  Slots are processed in position order, so ranks are stable.
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t p = wbase + j * 64 + lane;
            const bool valid = p < n;
            const uint32_t d = (k[j] >> shift) & mask;
            uint64_t m = __ballot(valid);
#pragma unroll
            for (int b = 0; b < R; ++b) {
                if ((uint32_t)b < nbits) {
                    const bool bit = (d >> b) & 1u;
                    const uint64_t bb = __ballot(bit);
                    m &= bit ? bb : ~bb;
                }
            }
            const uint32_t lt = mbcnt(m);
            const uint32_t prior = s_whist[w][d];
            rank[j] = prior + lt;
            if (valid && lt == 0) s_whist[w][d] = prior + (uint32_t)__popcll(m);
        }
        __syncthreads();

        // Per digit: offsets of each wave inside the tile, tile digit start, global delta.
        uint32_t c = 0, wc[kWaves];
        if (tid < (uint32_t)RADIX) {
#pragma unroll
            for (int q = 0; q < kWaves; ++q) { wc[q] = s_whist[q][tid]; c += wc[q]; }
        }
        uint32_t ttot;
        const uint32_t tstart = block_excl_scan(c, s_scratch, ttot);
        if (tid < (uint32_t)RADIX) {
            uint32_t o = tstart;
#pragma unroll
            for (int q = 0; q < kWaves; ++q) { s_whist[q][tid] = o; o += wc[q]; }
            s_gdelta[tid] = run - tstart;
            run += c;
        }
        __syncthreads();

        if (STAGED) {
            // Local shuffle: the tile, stably sorted by digit, in LDS.
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t p = wbase + j * 64 + lane;
                if (p < n) {
                    const uint32_t d = (k[j] >> shift) & mask;
                    const uint32_t s = s_whist[w][d] + rank[j];
                    if (s < (uint32_t)TILE) {
                        s_keys[s] = k[j];
                        if (HAS_VALUES) s_vals[s] = v[j];
                    }
                }
            }
            __syncthreads();
            const uint32_t nvalid = (n - tile0 < (uint32_t)TILE) ? (n - tile0) : (uint32_t)TILE;
            // Coalesced scatter: consecutive lanes write consecutive positions of a digit run.
#pragma unroll 4
            for (uint32_t i = tid; i < nvalid; i += kBlock) {
                const uint32_t key = s_keys[i];
                const uint32_t pos = s_gdelta[(key >> shift) & mask] + i;
                if (pos < n) {  // never false for a consistent histogram; keeps a bug from faulting
                    out_k[pos] = key;
                    if (HAS_VALUES) out_v[pos] = s_vals[i];
                }
            }
        } else {
            // Direct scatter from registers (no local shuffle): same positions, uncoalesced.
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t p = wbase + j * 64 + lane;
                if (p < n) {
                    const uint32_t d = (k[j] >> shift) & mask;
                    const uint32_t pos = s_gdelta[d] + s_whist[w][d] + rank[j];
                    if (pos < n) {
                        out_k[pos] = k[j];
                        if (HAS_VALUES) out_v[pos] = v[j];
                    }
                }
            }
        }
        __syncthreads();
    }
}

// ---- order check -------------------------------------------------------------------------
// inv[pass] |= 1 if any adjacent pair of keys[0..n) is out of order under `mask`.
__global__ __launch_bounds__(kBlock) void k_check(const uint32_t* __restrict__ keys, uint32_t n,
                                                  uint32_t mask, uint32_t* inv, int pass,
                                                  int gate_upto) {
    if (gate_upto >= 0 && gated_off(inv, gate_upto)) return;
    bool bad = false;
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i + 1 < n; i += stride) {
        const uint32_t a = keys[i] & mask, b = keys[i + 1] & mask;
        bad |= a > b;
    }
    if (__ballot(bad) != 0 && lane_id() == 0) atomicOr(inv + pass, 1u);
}

// After an early exit at an odd pass the sorted data sits in the tmp buffers: copy it back so
// the result is always in the caller's buffers (AbstractRadixSortKernel.ts:94-98).
template <bool HAS_VALUES>
__global__ __launch_bounds__(kBlock) void k_finalize(const uint32_t* __restrict__ tk,
                                                     const uint32_t* __restrict__ tv,
                                                     uint32_t* __restrict__ uk,
                                                     uint32_t* __restrict__ uv, uint32_t n,
                                                     const uint32_t* inv, int passes) {
    int first = -1;
    for (int c = 0; c < passes; ++c)
        if (inv[c] == 0u) { first = c; break; }
    if (first < 0 || (first & 1) == 0) return;
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        uk[i] = tk[i];
        if (HAS_VALUES) uv[i] = tv[i];
    }
}

// ---- prefix sum (PrefixSumKernel) ---------------------------------------------------------
// Three kernels, reduce-then-scan: chunk sums -> scan of chunk sums -> rescan with carry.
template <int TILE>
__global__ __launch_bounds__(kBlock) void k_chunk_sums(const uint32_t* __restrict__ data,
                                                       uint32_t n, uint32_t base, uint32_t extra,
                                                       uint32_t* __restrict__ sums) {
    __shared__ uint32_t scratch[kWaves];
    const Chunk ch = chunk_of(blockIdx.x, base, extra);
    const uint64_t lo = (uint64_t)ch.first * TILE;
    const uint64_t hi64 = lo + (uint64_t)ch.count * TILE;
    const uint32_t hi = (uint32_t)(hi64 < n ? hi64 : n);
    uint32_t s = 0;
    for (uint32_t i = (uint32_t)lo + threadIdx.x; i < hi; i += kBlock) s += data[i];
    uint32_t tot;
    block_excl_scan(s, scratch, tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <int TILE>
__global__ __launch_bounds__(kBlock) void k_chunk_rescan(uint32_t* __restrict__ data, uint32_t n,
                                                         uint32_t base, uint32_t extra,
                                                         const uint32_t* __restrict__ sums_scanned) {
    constexpr int PER = TILE / kBlock;  // consecutive elements per thread
    __shared__ uint32_t scratch[kWaves];
    const Chunk ch = chunk_of(blockIdx.x, base, extra);
    uint32_t carry = sums_scanned[blockIdx.x];
    for (uint32_t t = 0; t < ch.count; ++t) {
        const uint32_t t0 = (ch.first + t) * (uint32_t)TILE + threadIdx.x * PER;
        uint32_t x[PER];
        uint32_t s = 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            x[q] = (t0 + q < n) ? data[t0 + q] : 0u;
            s += x[q];
        }
        uint32_t tot;
        uint32_t run = carry + block_excl_scan(s, scratch, tot);
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            if (t0 + q < n) data[t0 + q] = run;
            run += x[q];
        }
        carry += tot;
    }
}

// Single-block exclusive scan of a short array (<= a few thousand) in place.
__global__ __launch_bounds__(kBlock) void k_scan_small(uint32_t* __restrict__ a, uint32_t m) {
    __shared__ uint32_t scratch[kWaves];
    const uint32_t per = (m + kBlock - 1) / kBlock;
    const uint32_t b0 = threadIdx.x * per;
    uint32_t s = 0;
    for (uint32_t k = 0; k < per; ++k)
        if (b0 + k < m) s += a[b0 + k];
    uint32_t tot;
    uint32_t run = block_excl_scan(s, scratch, tot);
    for (uint32_t k = 0; k < per; ++k)
        if (b0 + k < m) {
            uint32_t c = a[b0 + k];
            a[b0 + k] = run;
            run += c;
        }
}

// ---- synthetic inputs -----------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void k_fill_random(uint32_t* __restrict__ dst, uint64_t n,
                                                        uint64_t seed, uint64_t start) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t s = seed * 0xD1B54A32D192ED03ull + start;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        dst[i] = (uint32_t)mix64(s + i);
}

__global__ __launch_bounds__(kBlock) void k_fill_iota(uint32_t* __restrict__ dst, uint64_t n,
                                                      uint32_t first) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        dst[i] = first + (uint32_t)i;
}

__global__ __launch_bounds__(kBlock) void k_is_sorted(const uint32_t* __restrict__ keys,
                                                      uint32_t n, uint32_t mask,
                                                      uint32_t* flag) {
    bool bad = false;
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i + 1 < n; i += stride)
        bad |= (keys[i] & mask) > (keys[i + 1] & mask);
    if (__ballot(bad) != 0 && lane_id() == 0) atomicAnd(flag, 0u);
}

}  // namespace rs
