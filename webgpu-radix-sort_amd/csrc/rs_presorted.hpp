// rs_presorted.hpp — the presorted path of check_order sorts (CDNA4 / gfx950).
//
// check_order (README.md:85, AbstractRadixSortKernel.ts:249-276) exists for input that is already in
// order: the reference checks the order between its passes and skips the rest once the data is
// sorted.  Input that is NEARLY in order - sorted data with a few displaced elements, BASELINE
// config 4's "nearly sorted" f32 keys - still pays every pass there (and here, on the radix path:
// 52-80 B/key for config 4's skewed floats).  This path sorts such input in O(n) traffic instead:
//
//   1. k_ns_mark: the descents (i, i + 1: key[i] > key[i + 1] under the bit_count mask) mark both
//      their elements; the unmarked remainder is then re-checked around every marked run (the last
//      unmarked element before a run against the first after it) and both ends of any inversion
//      marked, until the remainder is in order.  Tiles of 3968 keys iterate in LDS inside a window
//      with 64 keys of context on each side (marks in the context are the neighbour's business: any
//      marking whose remainder is in order is a valid one, and a pair of remainder elements in two
//      tiles is checked by k_ns_decide).  More than 16 rounds, a tile with more than 256 descents,
//      or a tile marked whole sends the sort to the radix path.  Output: a mark bitmap, per-tile
//      mark counts and first / last remainder keys.
//   2. k_ns_decide: the decision on the device (every later launch is gated on it) and the tiles'
//      offsets into the extraction.
//   3. k_ns_extract: the marked elements, in position order, to side arrays (masked key, extraction
//      index; key, value, position); the rest of the extraction capacity padded with the largest key.
//   4. the extraction sorted stably by (masked key, extraction index): k_ns_totals (every pass's
//      digit totals) and four 8-bit one-sweep passes (k_onesweep) - equal keys keep position order.
//   5. k_ns_gather / k_ns_bounds: the sorted positions, and for every tile how many extracted
//      elements go before its first remainder element (binary search in the sorted extraction).
//   6. k_ns_save / k_ns_merge: every tile writes its remainder elements and the extracted elements
//      that fall among them, merged by (masked key, position) - the stable order - to its output
//      range, in place; the input positions another tile's output covers are saved to the plan
//      buffer first (a few hundred keys per tile boundary for config 4).
// The radix path is still enqueued behind and finds the caller's data in order (its own order
// check: every pass gated off); the hybrid path skips even its histogram read when this path has
// sorted (k_hist16_in's `skip`).  Result: the stable sort, as on the radix path.  Bytes per key
// (config 4): 4 (mark) + 16 (merge) + ~1 (save) + the extraction (~n / 250 keys, sorted).
#pragma once
#include "rs_kernels.hpp"

namespace rs {

constexpr uint32_t kNsHalo = 64;           // keys of context on each side of a tile
constexpr uint32_t kNsWin = 4096;          // a tile's window in k_ns_mark: 256 threads x 16 keys
constexpr uint32_t kNsTile = kNsWin - 2 * kNsHalo;   // keys per tile (3968: 124 bitmap words)
constexpr uint32_t kNsIter = 16;           // marking rounds per tile before giving up
constexpr uint32_t kNsBChunk = 512;        // extracted elements per LDS chunk in the merge
// control words (ctl): [1] a tile failed, [3] a tile was dense (the path is off), [4] m (marked
// total), [5] done (the path sorted: the radix path's histogram read is skipped), [8 .. 8 + 16)
// gate words, [24] the elements the merge moved (rs_plan_presorted_counts)
constexpr uint32_t kNsCtlWords = 32;
constexpr uint32_t kNsGate = 8;

// masked key of element i of a layout (KEYS / SOA: keys[i]; AOS: keys[2i])
template <int L>
__device__ __forceinline__ uint32_t ns_key(const uint32_t* keys, uint64_t i) {
    return keys[(L == LAYOUT_AOS ? 2ull : 1ull) * i];
}

// A sample of the order before any tile is read: kNsProbe adjacent pairs, one at a pseudo-random
// place in each of kNsProbe equal strides.  More than 1/16 of them descending (random input: about
// half; the count in ctl[7]) turns the path off, so that k_ns_mark's workgroups stop at once.
// Nearly sorted input (config 4: 0.2 % descents) is far below that.  A sample per thread.
constexpr uint32_t kNsProbe = 16384;
__device__ __forceinline__ bool ns_probe_off(const uint32_t* ctl) { return ctl[7] > kNsProbe / 16u; }
template <int L>
__global__ __launch_bounds__(256) void k_ns_probe(const uint32_t* __restrict__ keys, uint32_t n, uint32_t fmask,
                                                  uint32_t* ctl) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;   // (grid: kNsProbe / 256)
    const uint64_t step = (uint64_t)(n - 1) / kNsProbe;   // (n >= 12M: step >= 1)
    // (jittered inside its stride: a periodic pattern in the input must not alias the samples).
    // The jitter is the high word of hash x step - in [0, step) by construction.  Round 5 wrote
    // ((hash >> 8) % step): both operands provably below 2^24, the compiler expanded the remainder
    // into its float-reciprocal 24-bit form, whose quotient comes out one too large for some
    // operands (n = 15753718: 5 of the 16384 samples), and the negative remainder, masked to 24
    // bits, sent the sample ~2^24 keys past the array: a memory fault whenever that address was
    // unmapped (tests/test_presorted_gpu.py's seeded search found it; test_probe_sample_positions
    // pins the arithmetic).
    const uint64_t jit = ((uint64_t)(i * 0x9E3779B9u) * step) >> 32;
    const uint64_t p = (uint64_t)i * step + jit;
    uint32_t c = (ns_key<L>(keys, p) & fmask) > (ns_key<L>(keys, p + 1) & fmask) ? 1u : 0u;
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(ctl + 7, c);
}

// Persistent grid: workgroup g takes tiles g, g + grid, ... in order, with the next tile's window
// loaded into registers while this one is marked.  Thread g holds window group g (16 consecutive
// keys) in registers; the marks live in LDS as one 16-bit word per group.  A tile with more than
// kNsDense descents of its own is not nearly sorted: it turns the path off (ctl[3]) and every
// workgroup stops after its current tile (random input is read for about one tile per workgroup).
// No same-address atomics per tile: the counts go to tcnt, k_ns_decide adds them.
constexpr uint32_t kNsDense = 256;
template <int L>
__global__ __launch_bounds__(256) void k_ns_mark(const uint32_t* __restrict__ keys, uint32_t n, uint32_t fmask,
                                                 uint32_t* __restrict__ bitmap, uint32_t* __restrict__ tcnt,
                                                 uint32_t* __restrict__ tbnd, uint2* __restrict__ samp,
                                                 uint32_t* ctl) {
    constexpr uint32_t G = 16, NG = kNsWin / G, W = kNsWin, HALO = kNsHalo;
    constexpr uint32_t NWD = kNsTile / 32;
    constexpr uint32_t ESZ = L == LAYOUT_AOS ? 8u : 4u;
    static_assert(NG == 256 && NWD <= 256, "one group per thread");
    __shared__ __attribute__((aligned(16))) uint32_t s_k[W + 4];   // the window's masked keys (+ a pad group read past the end)
    __shared__ uint32_t s_mw[NG + 1];      // marks: bit j of word g = window position 16 g + j
    __shared__ uint32_t s_desc[4], s_cnt[4];
    __shared__ uint32_t s_fw[4], s_lw[4], s_stop;
    const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const uint32_t ntiles = (n + kNsTile - 1) / kNsTile;
    if (tid == 0) {
        s_mw[NG] = 0u;
        s_k[W] = 0u;
    }
    // window group `tid` of tile t into r (zeros outside the array)
    auto load = [&](uint32_t t, uint32_t (&r)[G]) {
        const int64_t w0 = (int64_t)t * kNsTile - (int64_t)HALO;
        const int64_t lo = w0 > 0 ? w0 : 0, hi = w0 + W < (int64_t)n ? w0 + W : (int64_t)n;
        const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(keys + (L == LAYOUT_AOS ? 2 : 1) * lo), (short)0, (int)((hi - lo) * ESZ), 0x00020000);
        // (tile 0: the window starts HALO keys before the array; those offsets wrap past the range)
        uint32_t off = (uint32_t)((int64_t)tid * G + (w0 - lo)) * ESZ;
        asm volatile("" : "+v"(off));
#pragma unroll
        for (uint32_t j = 0; j < G; ++j)
            r[j] = __builtin_amdgcn_raw_buffer_load_b32(rk, (int)(off + j * ESZ), 0, 0) & fmask;
    };
    if (ns_probe_off(ctl)) return;   // the probe found the input far from sorted
    uint32_t k[G], kn[G];
    uint32_t t = blockIdx.x;
    if (t < ntiles) load(t, k);
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t t0 = (uint64_t)t * kNsTile;
        const uint32_t nown = (uint32_t)((t0 + kNsTile < n ? t0 + kNsTile : (uint64_t)n) - t0);
        const int64_t w0 = (int64_t)t0 - (int64_t)HALO;
        // window index i is array position w0 + i; pairs (i, i + 1) count when both are in the array
        const int64_t pg = w0 + (int64_t)tid * G;    // this group's first position
#pragma unroll
        for (uint32_t j = 0; j < G; j += 4)
            *reinterpret_cast<uint4*>(&s_k[tid * G + j]) = make_uint4(k[j], k[j + 1], k[j + 2], k[j + 3]);
        // thread 0: the path-off flag, read now and looked at after this tile (its wait then covers
        // only this load: it is issued before the next window's)
        uint32_t stop = 0;
        if (tid == 0) stop = __hip_atomic_load(ctl + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (t + gridDim.x < ntiles) load(t + gridDim.x, kn);   // the next tile's window, in flight
        __syncthreads();
        // descents of this group's 16 pairs (pair 15: with the next group's first key)
        const uint32_t nx = s_k[tid * G + G];
        uint32_t d = 0;
#pragma unroll
        for (uint32_t j = 0; j + 1 < G; ++j) d |= (k[j] > k[j + 1] ? 1u : 0u) << j;
        d |= (tid + 1 < NG && k[G - 1] > nx ? 1u : 0u) << (G - 1);
        // pairs with both positions in [0, n)
        const int64_t jlo = -pg, jhi = (int64_t)n - 1 - pg;   // valid j: jlo <= j < jhi
        uint32_t vmask = 0xFFFFu;
        if (jlo > 0) vmask &= jlo >= (int64_t)G ? 0u : (0xFFFFu << jlo) & 0xFFFFu;
        if (jhi < (int64_t)G) vmask &= jhi <= 0 ? 0u : (1u << jhi) - 1u;
        d &= vmask;
        // the previous group's pair 15 marks this group's position 0
        const bool pd = tid > 0 && pg - 1 >= 0 && pg < (int64_t)n && s_k[tid * G - 1] > k[0];
        const uint32_t m = (d | (d << 1) | (pd ? 1u : 0u)) & 0xFFFFu;
        s_mw[tid] = m;
        // this tile's own descents (pair's first position owned)
        const int64_t olo = (int64_t)HALO - (int64_t)tid * G, ohi = olo + nown;   // owned j: olo <= j < ohi
        uint32_t omask = 0xFFFFu;
        if (olo > 0) omask &= olo >= (int64_t)G ? 0u : (0xFFFFu << olo) & 0xFFFFu;
        if (ohi < (int64_t)G) omask &= ohi <= 0 ? 0u : (1u << ohi) - 1u;
        const uint32_t own = wave_sum((uint32_t)__popc(d & omask));
        if (lane == 0) s_desc[w] = own;
        const int any = __syncthreads_or(m != 0u);
        if (s_desc[0] + s_desc[1] + s_desc[2] + s_desc[3] > kNsDense) {   // (uniform)
            if (tid == 0) __hip_atomic_store(ctl + 3, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        bool fail = false;   // (thread 0's)
        if (any) {
            // rounds: the last unmarked element before every marked run against the first after it
            for (uint32_t round = 0;; ++round) {
                const uint32_t mm = s_mw[tid], m1 = s_mw[tid + 1];
                const uint32_t ext = mm | ((m1 & 1u) << G);
                uint32_t starts = ~ext & (ext >> 1) & 0xFFFFu;   // i unmarked, i + 1 marked
                bool changed = false;
                while (starts) {
                    const uint32_t i = (uint32_t)__builtin_ctz(starts);
                    starts &= starts - 1u;
                    if (pg + i < 0) continue;              // (before the array: no predecessor)
                    uint32_t jj = W;                       // first unmarked after the run
                    const uint32_t rest = ~mm & (0xFFFFu << (i + 1u)) & 0xFFFFu;
                    if (rest) {
                        jj = tid * G + (uint32_t)__builtin_ctz(rest);
                    } else {
                        for (uint32_t q = tid + 1; q < NG; ++q) {
                            const uint32_t uq = ~s_mw[q] & 0xFFFFu;
                            if (uq) {
                                jj = q * G + (uint32_t)__builtin_ctz(uq);
                                break;
                            }
                        }
                    }
                    // the run reaches the array's end, or the window's: its successor is the next
                    // tile's first remainder element (k_ns_decide checks that pair)
                    if (jj >= W || w0 + (int64_t)jj >= (int64_t)n) continue;
                    const uint32_t ii = tid * G + i;
                    if (s_k[ii] > s_k[jj]) {
                        atomicOr(&s_mw[tid], 1u << i);
                        atomicOr(&s_mw[jj / G], 1u << (jj % G));
                        changed = true;
                    }
                }
                if (!__syncthreads_or(changed ? 1 : 0)) break;
                if (round + 1 == kNsIter) {   // not settled: give up
                    fail = true;
                    break;
                }
            }
        }
        // owned marks: bitmap word q (threads q < 124) = window groups 4 + 2q and 5 + 2q; count;
        // first / last unmarked owned position
        uint32_t cnt = 0, un = 0;
        if (tid < NWD && tid * 32u < nown) {
            const uint32_t hg = HALO / G;
            uint32_t wd = s_mw[hg + 2 * tid] | (s_mw[hg + 2 * tid + 1] << G);
            const uint32_t valid = nown - tid * 32u >= 32u ? 0xFFFFFFFFu : (1u << (nown - tid * 32u)) - 1u;
            wd &= valid;
            bitmap[(t0 >> 5) + tid] = wd;
            cnt = (uint32_t)__popc(wd);
            un = ~wd & valid;
            // the word's sample (k_ns_rank): its first unmarked position, as (masked key, position);
            // none: position ~0
            const uint32_t f = tid * 32u + (uint32_t)__builtin_ctz(un | 0x80000000u);
            samp[(t0 >> 5) + tid] = un ? make_uint2(s_k[HALO + f], (uint32_t)t0 + f) : make_uint2(0u, 0xFFFFFFFFu);
        }
        cnt = wave_sum(cnt);
        {   // the wave's first / last unmarked position: its first / last lane with one
            const uint64_t b = __ballot(un != 0u);
            const uint32_t fl = tid * 32u + (uint32_t)__builtin_ctz(un | 0x80000000u);
            const uint32_t ll = tid * 32u + 31u - (uint32_t)__builtin_clz(un | 1u);
            const uint32_t f = __shfl(fl, b ? (int)__builtin_ctzll(b) : 0, 64);
            const uint32_t l = __shfl(ll, b ? 63 - (int)__builtin_clzll(b) : 0, 64);
            if (lane == 0) {
                s_cnt[w] = cnt;
                s_fw[w] = b ? f : 0xFFFFFFFFu;
                s_lw[w] = b ? l : 0xFFFFFFFFu;
            }
        }
        __syncthreads();
        if (tid == 0) {
            tcnt[t] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
            uint32_t f = 0xFFFFFFFFu, l = 0xFFFFFFFFu;
            for (uint32_t q = 0; q < 4u; ++q) {
                if (f == 0xFFFFFFFFu) f = s_fw[q];
                if (s_lw[q] != 0xFFFFFFFFu) l = s_lw[q];
            }
            if (f == 0xFFFFFFFFu) {   // no remainder element: no boundary keys
                fail = true;
                f = l = 0u;
            }
            tbnd[2 * t] = s_k[HALO + f];
            tbnd[2 * t + 1] = s_k[HALO + l];
            if (fail) atomicOr(ctl + 1, 1u);
            s_stop = stop;
        }
        __syncthreads();   // (also: every reader of this tile's s_k / s_mw is done)
        if (s_stop) break;
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) k[j] = kn[j];
    }
}

// The path's decision: one 1024-thread workgroup per 1024 tiles writes the tiles' offsets into the
// extraction relative to their chunk (toff) and the chunk total (csum); an inversion between two
// tiles' remainders (the last remainder key of a tile against the first of the next) sets ctl[2].
// The last workgroup to finish (arrival count ctl[6]) then scans the chunk totals into coff and
// decides - on iff the probe's sample was nearly sorted (ctl[7]), no tile failed (ctl[1]), none
// was dense (ctl[3]), the remainder is in order
// across every tile boundary (ctl[2]) and 0 < marked <= cap.  On: m = ctl[4], every gate word 1,
// the extraction sort's digit totals and tickets (sub) zeroed.  Off: gate words 0 (the radix path
// runs as without this path).  A tile's offset: ns_toff().
constexpr uint32_t kNsSubWords = 4 * 256 + 32;   // the extraction sort's totals [4][256], tickets, error
__global__ __launch_bounds__(1024) void k_ns_decide(const uint32_t* __restrict__ tcnt,
                                                    const uint32_t* __restrict__ tbnd, uint32_t ntiles,
                                                    uint32_t cap, uint32_t* __restrict__ toff,
                                                    uint32_t* __restrict__ csum, uint32_t* __restrict__ coff,
                                                    uint32_t* __restrict__ sub, uint32_t* ctl) {
    __shared__ uint32_t s_scratch[16];
    __shared__ uint32_t s_last;
    const uint32_t tid = threadIdx.x;
    const uint32_t nch = gridDim.x;   // (ntiles + 1023) / 1024 <= 1024 (n < 2^32)
    bool on = !ctl[1] && !ctl[3] && !ns_probe_off(ctl);   // (uniform)
    if (on) {
        const uint32_t t = blockIdx.x * 1024u + tid;
        const uint32_t c = t < ntiles ? tcnt[t] : 0u;
        const bool bad = t + 1 < ntiles && tbnd[2 * t + 1] > tbnd[2 * t + 2];
        uint32_t tot;
        const uint32_t ex = block_excl_scan_n<16>(c, s_scratch, tot);
        if (t < ntiles) toff[t] = ex;
        const int anybad = __syncthreads_or(bad ? 1 : 0);
        if (tid == 0) {
            csum[blockIdx.x] = tot;
            if (anybad) atomicOr(ctl + 2, 1u);
            __threadfence();
            s_last = atomicAdd(ctl + 6, 1u) == nch - 1u ? 1u : 0u;
        }
        __syncthreads();
        if (!s_last) return;
        __threadfence();
        on = !__hip_atomic_load(ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (blockIdx.x != 0) {
        return;
    }
    // one workgroup from here: the last to arrive, or workgroup 0 when the path is off
    uint32_t total = 0;
    if (on) {
        const uint32_t ex = block_excl_scan_n<16>(tid < nch ? __hip_atomic_load(csum + tid, __ATOMIC_RELAXED,
                                                                                  __HIP_MEMORY_SCOPE_AGENT)
                                                            : 0u,
                                                  s_scratch, total);
        if (tid <= nch) coff[tid] = ex;
        on = total != 0u && total <= cap;   // sorted already, or too many marked
        __syncthreads();
        if (tid == 0) toff[ntiles] = total - coff[ntiles >> 10];   // ns_toff(ntiles) = m
        for (uint32_t i = tid; i < kNsSubWords; i += 1024) sub[i] = 0u;
    }
    if (tid == 0) ctl[4] = on ? total : 0u;
    if (tid < 16u) ctl[kNsGate + tid] = on ? 1u : 0u;
}

// Tile t's offset into the extraction (the marked elements of tiles before it); t == ntiles: m.
__device__ __forceinline__ uint32_t ns_toff(const uint32_t* toff, const uint32_t* coff, uint32_t t) {
    return coff[t >> 10] + toff[t];
}

// The marked elements of every tile, in position order, to the extraction: ek = masked key, ei =
// extraction index (the LSD passes sort (ek, ei) stably), sk / sv / sp = key, value, position in
// extraction order.  Past m: pads (the largest key, after every real one in a stable sort).  A
// grid-stride loop of waves, launched a wave per tile (no barrier): lane l takes bitmap words 2l and
// 2l + 1.
template <int L>
__global__ __launch_bounds__(256) void k_ns_extract(const uint32_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ vals, uint32_t n,
                                                   uint32_t fmask, uint32_t cap,
                                                   const uint32_t* __restrict__ bitmap,
                                                   const uint32_t* __restrict__ toff,
                                                   const uint32_t* __restrict__ coff, const uint32_t* ctl,
                                                   uint32_t* __restrict__ ek, uint32_t* __restrict__ ei,
                                                   uint32_t* __restrict__ sk, uint32_t* __restrict__ sv,
                                                   uint32_t* __restrict__ sp, uint32_t* __restrict__ wpre) {
    static_assert(kNsTile / 32 <= 128, "two bitmap words per lane");
    if (!ctl[kNsGate]) return;
    const uint32_t lane = lane_id(), gw = blockIdx.x * (blockDim.x / 64u) + (threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * (blockDim.x / 64u);   // waves in the grid
    const uint32_t m = ctl[4];
    // pads (grid-stride over the extraction's tail)
    for (uint64_t e = (uint64_t)m + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < cap;
         e += (uint64_t)gridDim.x * blockDim.x) {
        ek[e] = 0xFFFFFFFFu;
        ei[e] = (uint32_t)e;
    }
    const uint32_t ntiles = (n + kNsTile - 1) / kNsTile;
    for (uint32_t t = gw; t < ntiles; t += nw) {
    const uint64_t t0 = (uint64_t)t * kNsTile;
    const uint32_t nown = (uint32_t)((t0 + kNsTile < n ? t0 + kNsTile : n) - t0);
    const uint32_t nwords = (nown + 31u) / 32u;   // <= 124
    const uint32_t w0 = 2u * lane, w1 = w0 + 1u;
    uint32_t b0 = w0 < nwords ? bitmap[(t0 >> 5) + w0] : 0u;
    uint32_t b1 = w1 < nwords ? bitmap[(t0 >> 5) + w1] : 0u;
    const uint32_t c = (uint32_t)__popc(b0) + (uint32_t)__popc(b1);
    const uint32_t ex = wave_incl_scan(c) - c;   // marks of the tile before word w0
    if (w0 < nwords) wpre[(t0 >> 5) + w0] = ex;
    if (w1 < nwords) wpre[(t0 >> 5) + w1] = ex + (uint32_t)__popc(b0);
    uint32_t e = ns_toff(toff, coff, t) + ex;
    auto take = [&](uint32_t bits, uint32_t word) {
        while (bits) {
            const uint32_t b = (uint32_t)__builtin_ctz(bits);
            bits &= bits - 1u;
            const uint64_t p = t0 + word * 32u + b;
            const uint32_t key = ns_key<L>(keys, p);
            ek[e] = key & fmask;
            ei[e] = e;
            sk[e] = key;
            sv[e] = L == LAYOUT_KEYS ? 0u : (L == LAYOUT_AOS ? keys[2 * p + 1] : vals[p]);
            sp[e] = (uint32_t)p;
            ++e;
        }
    };
    take(b0, w0);
    take(b1, w1);
    }
}

// (masked key, position) order
__device__ __forceinline__ bool ns_less(uint32_t ka, uint32_t pa, uint32_t kb, uint32_t pb) {
    return ka < kb || (ka == kb && pa < pb);
}

// Every pass's digit totals of the extraction sort (sub[256 p + d], they do not depend on the
// order): the m extracted keys counted in LDS, then the cap - m pads (digit 255 of every pass).
__global__ __launch_bounds__(256) void k_ns_totals(const uint32_t* __restrict__ ek, uint32_t cap,
                                                   const uint32_t* ctl, uint32_t* __restrict__ sub) {
    __shared__ uint32_t h[4 * 256];
    if (!ctl[kNsGate]) return;
    const uint32_t m = ctl[4], tid = threadIdx.x;
    for (uint32_t i = tid; i < 4 * 256; i += 256) h[i] = 0u;
    __syncthreads();
    for (uint32_t j = blockIdx.x * 256u + tid; j < m; j += gridDim.x * 256u) {
        const uint32_t k = ek[j];
#pragma unroll
        for (uint32_t p = 0; p < 4; ++p) atomicAdd(&h[256 * p + ((k >> (8 * p)) & 255u)], 1u);
    }
    __syncthreads();
    for (uint32_t i = tid; i < 4 * 256; i += 256) {
        const uint32_t c = h[i] + (blockIdx.x == 0 && (i & 255u) == 255u ? cap - m : 0u);
        if (c) atomicAdd(&sub[i], c);
    }
}

// Threads j < m: the sorted extraction's positions, keys and values (bp, bk, bv: gathered through
// the extraction index; the sorted masked keys bm are the sorted ek itself).
__global__ __launch_bounds__(256) void k_ns_gather(const uint32_t* __restrict__ ei, const uint32_t* __restrict__ sp,
                                                   const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                                   const uint32_t* ctl, uint32_t* __restrict__ bp,
                                                   uint32_t* __restrict__ bk, uint32_t* __restrict__ bv) {
    if (!ctl[kNsGate]) return;
    const uint32_t m = ctl[4];
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < m; j += gridDim.x * 256u) {
        const uint32_t e = ei[j];
        bp[j] = sp[e];
        bk[j] = sk[e];
        bv[j] = sv[e];
    }
}

// Threads t <= ntiles: blo[t] = the extracted elements ordered before tile t's first remainder
// element - those before the last remainder element ahead of the tile (bit-scanned back; k_ns_mark
// failed the path when a tile is marked whole, so the previous tile holds one), searched in the
// sorted extraction (bm, bp); blo[0] = 0, blo[ntiles] = m.
template <int L>
__global__ __launch_bounds__(256) void k_ns_bounds(const uint32_t* __restrict__ keys, uint32_t n, uint32_t fmask,
                                                   const uint32_t* __restrict__ bitmap, uint32_t ntiles,
                                                   const uint32_t* __restrict__ bm, const uint32_t* __restrict__ bp,
                                                   const uint32_t* ctl, uint32_t* __restrict__ blo) {
    if (!ctl[kNsGate]) return;
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t > ntiles) return;
    const uint32_t m = ctl[4];
    if (t == 0) { blo[0] = 0u; return; }
    if (t == ntiles) { blo[ntiles] = m; return; }
    uint64_t q = (uint64_t)t * kNsTile - 1u;
    while ((bitmap[q >> 5] >> (q & 31u)) & 1u) --q;
    const uint32_t kq = ns_key<L>(keys, q) & fmask;
    uint32_t lo = 0, hi = m;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ns_less(bm[mid], bp[mid], kq, (uint32_t)q)) lo = mid + 1;
        else hi = mid;
    }
    blo[t] = lo;
}

// Tile t's output range [olo, ohi): the merge writes the tile's remainder elements and the
// extracted elements [blo[t], blo[t + 1]) there (the ranges of all tiles partition [0, n)).
__device__ __forceinline__ void ns_out_range(const uint32_t* toff, const uint32_t* coff, const uint32_t* blo,
                                             uint32_t t, uint32_t ntiles, uint32_t n, int64_t& olo, int64_t& ohi) {
    const int64_t t0 = (int64_t)t * kNsTile;
    const int64_t t1 = t + 1 < ntiles ? t0 + kNsTile : (int64_t)n;
    olo = t0 - (int64_t)ns_toff(toff, coff, t) + blo[t];
    ohi = t1 - (int64_t)ns_toff(toff, coff, t + 1) + blo[t + 1];
}

// The merge runs in place: a tile reads the positions of its own output range straight from the
// caller's arrays (nobody else writes them, and it writes them only after its reads); every other
// position of its input - the part another tile's output covers - is saved first, here, to the same
// position of the plan buffer tmp (records; keys only: keys).  A persistent grid, a workgroup per
// tile at a time.
template <int L>
__global__ __launch_bounds__(256) void k_ns_save(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                 uint32_t n, const uint32_t* __restrict__ toff,
                                                 const uint32_t* __restrict__ coff, const uint32_t* __restrict__ blo,
                                                 const uint32_t* ctl, uint32_t* __restrict__ tmp,
                                                 uint32_t* __restrict__ tileof) {
    if (!ctl[kNsGate]) return;
    const uint32_t tid = threadIdx.x;
    const uint32_t ntiles = (n + kNsTile - 1) / kNsTile;
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t t0 = (int64_t)t * kNsTile;
    const int64_t t1 = t + 1 < ntiles ? t0 + kNsTile : (int64_t)n;
    int64_t olo, ohi;
    ns_out_range(toff, coff, blo, t, ntiles, n, olo, ohi);
    const int64_t a1 = olo < t1 ? olo : t1;    // [t0, a1) and [b0, t1): outside the own range
    const int64_t b0 = ohi > t0 ? ohi : t0;
    auto save = [&](int64_t lo, int64_t hi) {
        for (int64_t p = lo + tid; p < hi; p += 256) {
            if (L == LAYOUT_KEYS) {
                tmp[p] = keys[p];
            } else if (L == LAYOUT_AOS) {
                reinterpret_cast<uint2*>(tmp)[p] = reinterpret_cast<const uint2*>(keys)[p];
            } else {
                reinterpret_cast<uint2*>(tmp)[p] = make_uint2(keys[p], vals[p]);
            }
        }
    };
    save(t0, a1);
    save(b0 > a1 ? b0 : a1, t1);
    for (uint32_t j = blo[t] + tid; j < blo[t + 1]; j += 256) tileof[j] = t;   // (for k_ns_rank)
    }
}

// Threads j < m: rank[j] = the remainder elements of sorted extracted element j's tile (tileof,
// from k_ns_save) ordered before it.  The remainder of a tile is in (key, position) order, so a
// binary search over the tile's word samples (k_ns_mark: the first remainder element of every
// 32-position word, as (masked key, position); a probe on a word without one moves to the next
// word with one) finds the last word whose sample is before the element; that word's own
// remainder elements are compared, and the words before it counted whole (wpre: the tile's marks
// before each word).
template <int L>
__global__ __launch_bounds__(256) void k_ns_rank(const uint32_t* __restrict__ keys, uint32_t n, uint32_t fmask,
                                                 const uint32_t* __restrict__ bitmap,
                                                 const uint32_t* __restrict__ wpre, const uint2* __restrict__ samp,
                                                 const uint32_t* __restrict__ tileof,
                                                 const uint32_t* __restrict__ bm, const uint32_t* __restrict__ bp,
                                                 const uint32_t* ctl, uint32_t* __restrict__ rank) {
    if (!ctl[kNsGate]) return;
    const uint32_t m = ctl[4];
    for (uint32_t j = blockIdx.x * 256u + threadIdx.x; j < m; j += gridDim.x * 256u) {
        const uint32_t t = tileof[j];
        const uint64_t t0 = (uint64_t)t * kNsTile;
        const uint32_t nown = (uint32_t)((t0 + kNsTile < n ? t0 + kNsTile : n) - t0);
        const uint32_t nwd = (nown + 31u) / 32u;
        const uint32_t kb = bm[j], pb = bp[j];
        const uint2* sw = samp + (t0 >> 5);
        // the number of words whose sample is before (kb, pb)
        uint32_t lo = 0, hi = nwd;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            uint32_t wq = mid;
            uint2 q = sw[mid];
            while (q.y == 0xFFFFFFFFu && ++wq < hi) q = sw[wq];   // (a word marked whole)
            if (wq >= hi) hi = mid;
            else if (ns_less(q.x, q.y, kb, pb)) lo = wq + 1;
            else hi = mid;
        }
        uint32_t r = 0;
        if (lo > 0) {
            const uint32_t wd = lo - 1;   // the last such word: holds its own sample
            const uint32_t bits = bitmap[(t0 >> 5) + wd];
            r = wd * 32u - wpre[(t0 >> 5) + wd];
            const uint64_t p0 = t0 + wd * 32u;
            const uint32_t cnt = nown - wd * 32u < 32u ? nown - wd * 32u : 32u;
            // the word's 32 keys at once (one or two cache lines), then counted
            uint32_t k[32];
#pragma unroll
            for (uint32_t i = 0; i < 32u; ++i) k[i] = i < cnt ? ns_key<L>(keys, p0 + i) : 0u;
#pragma unroll
            for (uint32_t i = 0; i < 32u; ++i)
                r += (i < cnt && !((bits >> i) & 1u) && ns_less(k[i] & fmask, (uint32_t)(p0 + i), kb, pb)) ? 1u : 0u;
        }
        rank[j] = r;
    }
}

// Tile t: its remainder elements (positions [t0, t0 + kNsTile) not in the bitmap) go to the tile's
// first output position + their remainder index + the tile's extracted elements ordered before them
// (those whose rank is at most that index); the extracted elements [blo[t], blo[t + 1]) go to the
// tile's first output position + their rank + their index in the tile's list.  Only the elements
// whose output position differs from their input position are read and written (for config 4 -
// transposed pairs - few remainder elements move at all), in place (see k_ns_save: a tile reads
// only its own output range from the caller's arrays, and writes after every thread of the
// workgroup has read).  Element e of the tile is thread e % NT's slot e / NT.
// Measured (config 4, 2^28): 0.58 ms with 0.28 GB of traffic - latency per tile (3-4 tiles in
// flight per CU), not bytes.  A wave-per-tile form that skips 64-position groups without movement
// (32 tiles in flight per CU) measured 0.91 ms: its per-slot searches cost more than the latency
// it hides (round 5, history).
#if !RS_KNOB_OPEN || !defined(RS_NS_SPEC)
#undef RS_NS_SPEC
#define RS_NS_SPEC 0       // k_ns_merge: every slot's element loaded at the top of the tile (movers or not)
#endif
#if !RS_KNOB_OPEN || !defined(RS_NS_MINB)
#undef RS_NS_MINB
#define RS_NS_MINB 1       // k_ns_merge: workgroups per CU the register budget must allow
#endif
template <int L, uint32_t NT = 512>
__global__ __launch_bounds__(NT, RS_NS_MINB) void k_ns_merge(uint32_t* keys, uint32_t* vals, uint32_t n,
                                                 const uint32_t* __restrict__ bitmap,
                                                 const uint32_t* __restrict__ toff,
                                                 const uint32_t* __restrict__ coff,
                                                 const uint32_t* __restrict__ blo,
                                                 const uint32_t* __restrict__ rank, const uint32_t* __restrict__ bk,
                                                 const uint32_t* __restrict__ bv, uint32_t* ctl,
                                                 const uint32_t* __restrict__ tmp) {
    constexpr uint32_t KPT = (kNsTile + NT - 1) / NT;
    constexpr uint32_t NWD = kNsTile / 32;
    constexpr uint32_t BC = 2 * NT;           // extracted elements per LDS chunk
    __shared__ uint32_t s_r[BC];              // a chunk of the tile's extracted elements' ranks
    __shared__ uint32_t s_w[NWD], s_wpre[NWD];   // the tile's bitmap words, marks before each word
    __shared__ uint32_t s_scratch[NT / 64];
    if (!ctl[kNsGate]) return;
    // the path has sorted once every workgroup is done (read by the radix path's histogram read,
    // a later launch: k_hist16_in's skip)
    if (blockIdx.x == 0 && threadIdx.x == 0) ctl[5] = 1u;
    const uint32_t ntiles = (n + kNsTile - 1) / kNsTile;
    // a tile's own loads - its output range, extracted-element range, bitmap word (threads 0 .. 123),
    // the first chunk's ranks and data (this thread's two) - issued one tile ahead
    struct Meta {
        int64_t olo, ohi;
        uint32_t b0, b1, wv, r0, r1, xk0, xv0, xk1, xv1;
    };
    auto fetch = [&](uint32_t t, Meta& q) {
        const uint32_t tid = threadIdx.x;
        const uint64_t t0 = (uint64_t)t * kNsTile;
        const uint32_t nown = (uint32_t)((t0 + kNsTile < n ? t0 + kNsTile : n) - t0);
        const uint32_t nwd = (nown + 31u) / 32u;
        ns_out_range(toff, coff, blo, t, ntiles, n, q.olo, q.ohi);
        q.b0 = blo[t];
        q.b1 = blo[t + 1];
        const uint32_t cn0 = q.b1 - q.b0 < BC ? q.b1 - q.b0 : BC;
        q.wv = tid < nwd ? bitmap[(t0 >> 5) + tid] : 0u;
        q.r0 = tid < cn0 ? rank[q.b0 + tid] : 0u;
        q.r1 = tid + NT < cn0 ? rank[q.b0 + tid + NT] : 0u;
        q.xk0 = q.xv0 = q.xk1 = q.xv1 = 0u;
        if (tid < cn0) {
            q.xk0 = bk[q.b0 + tid];
            if (L != LAYOUT_KEYS) q.xv0 = bv[q.b0 + tid];
        }
        if (tid + NT < cn0) {
            q.xk1 = bk[q.b0 + tid + NT];
            if (L != LAYOUT_KEYS) q.xv1 = bv[q.b0 + tid + NT];
        }
    };
    Meta cur;
    if (blockIdx.x < ntiles) fetch(blockIdx.x, cur);
    uint32_t moved = 0;   // elements this thread wrote (added to ctl[24] once, at the end)
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    // (per-slot positions recomputed each tile from an opaque copy of the thread index: hoisted out
    // of the tile loop they take a register each)
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const uint64_t t0 = (uint64_t)t * kNsTile;
    const uint32_t nown = (uint32_t)((t0 + kNsTile < n ? t0 + kNsTile : n) - t0);
    const int64_t olo = cur.olo, ohi = cur.ohi;
    const uint32_t b0 = cur.b0, b1 = cur.b1, wv = cur.wv, r0 = cur.r0, r1 = cur.r1;
    const uint32_t xk0 = cur.xk0, xv0 = cur.xv0, xk1 = cur.xk1, xv1 = cur.xv1;
    const uint32_t cn0 = b1 - b0 < BC ? b1 - b0 : BC;
    const uint32_t alo = (uint32_t)(olo - (int64_t)t0 < 0 ? 0 : (olo - (int64_t)t0 > nown ? nown : olo - (int64_t)t0));
    const uint32_t ahi = (uint32_t)(ohi - (int64_t)t0 < 0 ? 0 : (ohi - (int64_t)t0 > nown ? nown : ohi - (int64_t)t0));
    uint32_t fk[KPT], fv[KPT];
    auto read_slot = [&](uint32_t j) {   // slot j's element: own output range in place, else the save
        const uint32_t i = j * NT + tid;
        const uint64_t p = t0 + i;
        if (i >= alo && i < ahi) {
            if (L == LAYOUT_AOS) {
                const uint2 q = reinterpret_cast<const uint2*>(keys)[p];
                fk[j] = q.x;
                fv[j] = q.y;
            } else {
                fk[j] = keys[p];
                if (L == LAYOUT_SOA) fv[j] = vals[p];
            }
        } else {
            if (L == LAYOUT_KEYS) {
                fk[j] = tmp[p];
            } else {
                const uint2 q = reinterpret_cast<const uint2*>(tmp)[p];
                fk[j] = q.x;
                fv[j] = q.y;
            }
        }
    };
    if (RS_NS_SPEC) {   // every slot of the tile, in flight through the scans and searches below
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j) {
            fk[j] = 0u;
            fv[j] = 0u;
            if (j * NT + tid < nown) read_slot(j);
        }
    }
    __syncthreads();   // the previous tile's readers of the LDS arrays are done
    {
        uint32_t nmarked;
        const uint32_t pre = block_excl_scan_n<NT / 64>((uint32_t)__popc(wv), s_scratch, nmarked);
        if (tid < NWD) { s_w[tid] = wv; s_wpre[tid] = pre; }
        if (tid < cn0) s_r[tid] = r0;
        if (tid + NT < cn0) s_r[tid + NT] = r1;
    }
    __syncthreads();
    // remainder index of every slot, then the extracted elements before it, chunk by chunk
    uint32_t ao[KPT];
    uint32_t valid = 0;
#pragma unroll
    for (uint32_t j = 0; j < KPT; ++j) {
        const uint32_t i = j * NT + tid;
        const bool in = i < nown;
        const uint32_t wvi = in ? s_w[i >> 5] : 0xFFFFFFFFu;
        const bool ok = in && !((wvi >> (i & 31u)) & 1u);
        ao[j] = i - (s_wpre[i >> 5 < NWD ? i >> 5 : NWD - 1] + (uint32_t)__popc(wvi & ((1u << (i & 31u)) - 1u)));
        valid |= ok ? (1u << j) : 0u;
    }
    uint32_t bef[KPT];
#pragma unroll
    for (uint32_t j = 0; j < KPT; ++j) bef[j] = 0u;
    for (uint32_t c0 = b0; c0 < b1; c0 += BC) {
        const uint32_t cn = b1 - c0 < BC ? b1 - c0 : BC;
        if (c0 != b0) {   // (the first chunk is in LDS already)
            __syncthreads();
            for (uint32_t i = tid; i < cn; i += NT) s_r[i] = rank[c0 + i];
            __syncthreads();
        }
#pragma unroll
        for (uint32_t j = 0; j < KPT; ++j) {   // upper bound of the remainder index in the ranks
            uint32_t l = 0, h = cn;
            while (l < h) {
                const uint32_t mid = (l + h) >> 1;
                if (s_r[mid] <= ao[j]) l = mid + 1;
                else h = mid;
            }
            bef[j] += l;
        }
    }
    // the movers: read (own output range in place, the rest from tmp, where k_ns_save put them)
    const uint32_t obase = (uint32_t)olo;
    uint32_t mv = 0;
#pragma unroll
    for (uint32_t j = 0; j < KPT; ++j) {
        const uint32_t i = j * NT + tid;
        const uint32_t o = obase + ao[j] + bef[j];
        ao[j] = o;
        if (!RS_NS_SPEC) {
            fk[j] = 0u;
            fv[j] = 0u;
        }
        if (((valid >> j) & 1u) && o != (uint32_t)t0 + i) {
            mv |= 1u << j;
            if (!RS_NS_SPEC) read_slot(j);
        }
    }
    // the next tile's loads, in flight while this one writes
    if (t + gridDim.x < ntiles) fetch(t + gridDim.x, cur);
    // every load of the workgroup has landed before any thread writes (in place)
#pragma unroll
    for (uint32_t j = 0; j < KPT; ++j) asm volatile("" ::"v"(fk[j]), "v"(fv[j]));
    __syncthreads();
    auto put = [&](uint32_t o, uint32_t k, uint32_t v) {
        if (L == LAYOUT_KEYS) {
            keys[o] = k;
        } else if (L == LAYOUT_AOS) {
            reinterpret_cast<uint2*>(keys)[o] = make_uint2(k, v);
        } else {
            keys[o] = k;
            vals[o] = v;
        }
    };
#pragma unroll
    for (uint32_t j = 0; j < KPT; ++j)
        if ((mv >> j) & 1u) put(ao[j], fk[j], fv[j]);
    if (tid < cn0) put(obase + r0 + tid, xk0, xv0);
    if (tid + NT < cn0) put(obase + r1 + tid + NT, xk1, xv1);
    for (uint32_t jj = b0 + BC + tid; jj < b1; jj += NT)   // (more than one chunk)
        put(obase + rank[jj] + (jj - b0), bk[jj], L == LAYOUT_KEYS ? 0u : bv[jj]);
    moved += (uint32_t)__popc(mv) + (tid < cn0 ? 1u : 0u) + (tid + NT < cn0 ? 1u : 0u) +
             (b1 - b0 > BC + tid ? (b1 - b0 - BC - tid + NT - 1u) / NT : 0u);
    }
    moved = wave_sum(moved);
    if (lane_id() == 0 && moved) atomicAdd(ctl + 24, moved);
}

}  // namespace rs
