// rs_kernels.hpp — CDNA4 (gfx950) HIP kernels of the 4-way LSD radix sort.
//
// One global HBM pass sorts one digit of `w <= R` bits (R = 2: exactly the reference's 4-way
// pass; R = 8: four fused 4-way splits per HBM round trip).  Per pass, three kernels:
//
//   k_histogram  — per-tile digit counts, one wave per tile
//                  (the block-sum half of the reference's radix_sort, RadixSort.ts:50-126)
//   k_scan_rows  — exclusive scan of each digit's row of tile counts + digit totals
//                  (the PrefixSumKernel chain over the digit-major block sums,
//                  PrefixSum.ts:13-106, AbstractRadixSortKernel.ts:240)
//   k_scatter    — per tile: stable in-wave ranking, tile digit offsets, local shuffle through
//                  LDS (RadixSortLocalShuffle.ts:94-116), coalesced scatter of keys (+values)
//                  to their global positions (RadixSortReorder.ts:80-102)
//
// and k_sort_small: the whole sort of up to one tile in one workgroup, all passes in LDS.
//
// Data layout in HBM: keys / values are separate u32 arrays (structure of arrays, as the
// reference's two GPUBuffers); the count matrix is digit-major counts[d * ntiles + t] like the
// reference's block_sums[b * WORKGROUP_COUNT + WORKGROUP_ID] (RadixSort.ts:113).
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

// Tuning and diagnostic knobs (RS_* below): product builds fix every one at its default, whatever
// -D says, so no flag can change what librsort computes; sweep and diagnostic builds (make variants,
// tools/build_variants.sh) compile with -DRS_SWEEP=1 to vary them.
#if defined(RS_SWEEP) && RS_SWEEP
#define RS_KNOB_OPEN 1
#else
#define RS_KNOB_OPEN 0
#endif

#if !RS_KNOB_OPEN || !defined(RS_XCD_GROUP)
#undef RS_XCD_GROUP
#define RS_XCD_GROUP 1       // consecutive tiles run on one XCD in the same round (speed only)
#endif
#if !RS_KNOB_OPEN || !defined(RS_HIST_XCD)
#undef RS_HIST_XCD
#define RS_HIST_XCD 1        // k_histogram: adjacent tiles' counts written from one XCD (speed only)
#endif
#if !RS_KNOB_OPEN || !defined(RS_ONESWEEP_TRACE)
#undef RS_ONESWEEP_TRACE
#define RS_ONESWEEP_TRACE 0  // 1: printf the stuck tile when a look-back wait times out
#endif
#if !RS_KNOB_OPEN || !defined(RS_PACK_POS)
#undef RS_PACK_POS
#define RS_PACK_POS 1        // 1: staging-round kernels keep tile positions as 16-bit pairs
#endif
#if !RS_KNOB_OPEN || !defined(RS_NT_STORE)
#undef RS_NT_STORE
#define RS_NT_STORE 0        // pass output stores: 1 non-temporal, 2 write-through (sc1), 3 system scope
#endif
#if !RS_KNOB_OPEN || !defined(RS_NT_LOAD)
#undef RS_NT_LOAD
#define RS_NT_LOAD 0         // 1: pass inputs (full tiles) loaded non-temporal (read once per pass)
#endif

#if !RS_KNOB_OPEN || !defined(RS_STAGE_BATCH)
#undef RS_STAGE_BATCH
#define RS_STAGE_BATCH 1     // stage_tile: all slots' offsets read before the staging writes
#endif

#if !RS_KNOB_OPEN || !defined(RS_MSD_TAILBAR)
#undef RS_MSD_TAILBAR
#define RS_MSD_TAILBAR 0     // k_msd_pass: a barrier after the scatter (1: round 5's; 0: none - the next
                             // writers of the staging area and the digit deltas come after the next
                             // rank's barriers; 0.962 vs 0.986 ms per pass, profiles/r06/tailbar)
#endif

#if !RS_KNOB_OPEN || !defined(RS_MSD_LBLATE)
#undef RS_MSD_LBLATE
#define RS_MSD_LBLATE 0      // k_msd_pass: the look-back waves (digits, tid < 256) issue their part of the
                             // next tile's loads after their look-back, not before (a wave's re-read of
                             // a status word otherwise waits for all 16 of its tile loads: vmcnt is in order)
#endif

// Traffic attribution (sweep builds only; the output is then NOT sorted - tools/pmc_traffic.py
// with RS_PROF_NOCHECK): RS_DIAG_LB = 1 - no look-back status reads (every tile scatters as if it
// were its segment's first); RS_DIAG_SEQ = 1 - every record is written to its own input position
// (no digit runs, so no partial lines at run seams).  The pass kernels k_onesweep / k_msd_pass.
#if !RS_KNOB_OPEN || !defined(RS_DIAG_LB)
#undef RS_DIAG_LB
#define RS_DIAG_LB 0
#endif
#if !RS_KNOB_OPEN || !defined(RS_DIAG_SEQ)
#undef RS_DIAG_SEQ
#define RS_DIAG_SEQ 0
#endif

#if !RS_KNOB_OPEN || !defined(RS_OS_TAILBAR)
#undef RS_OS_TAILBAR
#define RS_OS_TAILBAR 0      // k_onesweep: a barrier after the last staging round's scatter (0: none,
                             // config2 0.650 vs 0.654 ms, profiles/r06/ostb)
#endif

#if !RS_KNOB_OPEN || !defined(RS_H16_BATCH)
#undef RS_H16_BATCH
#define RS_H16_BATCH 1       // k_hist16_in: a group's adds all issued before their crossing checks
                             // (with 3 loads per group: 0.232 vs 0.239 ms at config 3, profiles/r06/hist16)
#endif

#if !RS_KNOB_OPEN || !defined(RS_STAMPS)
#undef RS_STAMPS
#define RS_STAMPS 0          // diagnostic build: per-tile phase timestamps of k_onesweep
#endif

namespace rs {

#if RS_STAMPS
// [pass][tile][16] s_memtime stamps (thread 0 of the workgroup); slot 7 = workgroup id, slots
// 8-11 digit 0's look-back (first status round returned, rounds, predecessors consumed, sleeps).
// Set by rs_debug_set_stamps (diagnostic builds only, tools/stamp_probe.py).
__device__ unsigned long long* g_rs_stamps;
#define RS_STAMP(pass, ntiles, T, i, v)                                                        \
    do {                                                                                       \
        if (threadIdx.x == 0 && g_rs_stamps)                                                   \
            g_rs_stamps[((size_t)(pass) * (ntiles) + (T)) * 16 + (i)] = (v);                   \
    } while (0)
#else
#define RS_STAMP(pass, ntiles, T, i, v) do { } while (0)
#endif

constexpr int kBlock = 256;              // threads of the small kernels: 4 waves of 64
constexpr int kWaves = kBlock / 64;
// Pass kernels keep >= 4 waves per SIMD resident (<= 128 VGPRs) at every block size: implied
// for 1024-thread blocks, and it lets 256 / 512-thread blocks share a CU 4 / 2 ways.
constexpr int kMinWavesPerSimd = 4;
// ... except tiles of more than 32 keys per thread, which get the whole register file of one
// workgroup per CU (BLOCK / 256 waves per SIMD)
constexpr int pass_min_waves(int block, int kpt) { return kpt > 32 ? block / 256 : kMinWavesPerSimd; }

// Key/value layouts in HBM.  KEYS: keys only.  SOA: separate key and value arrays (the
// reference's RadixSortBufferKernel buffers).  AOS: one array of 8-byte (key, value) records,
// the rg32uint texels of RadixSortTextureKernel (RadixSortReorder.ts:42-63), record i at word 2i.
enum Layout { LAYOUT_KEYS = 0, LAYOUT_SOA = 1, LAYOUT_AOS = 2 };

// ---- small helpers ---------------------------------------------------------------------

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Stream accesses of the pass kernels (cache policy per RS_NT_STORE / RS_NT_LOAD).
template <class T>
__device__ __forceinline__ void st_out(T* p, T v) {
#if RS_NT_STORE == 1
    __builtin_nontemporal_store(v, p);
#elif RS_NT_STORE == 2
    // write-through (sc1) stores: agent-scope relaxed atomic stores
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#elif RS_NT_STORE == 3
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else
    *p = v;
#endif
}
template <class T>
__device__ __forceinline__ T ld_in(const T* p) {
#if RS_NT_LOAD
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

// Popcount of the bits of m below this lane (v_mbcnt_lo/hi).
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// A uniform value the compiler cannot see through: digit arithmetic recomputed from it is not
// merged with the same arithmetic of an earlier phase (keeping a slot's digit or LDS address
// alive across phases costs one register per key slot).
__device__ __forceinline__ uint32_t opaque_u(uint32_t x) {
    asm volatile("" : "+s"(x));
    return x;
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

// Exclusive scan of one u32 per thread over an NW-wave workgroup; scratch >= NW u32 of LDS.
// Contains two barriers; every thread of the workgroup must call it.
template <int NW>
__device__ __forceinline__ uint32_t block_excl_scan_n(uint32_t v, uint32_t* scratch, uint32_t& total) {
    const uint32_t inc = wave_incl_scan(v);
    const uint32_t w = threadIdx.x >> 6;
    if (lane_id() == 63) scratch[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < (uint32_t)NW; ++i) {
        uint32_t s = scratch[i];
        pre += (i < w) ? s : 0u;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return pre + inc - v;
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* scratch, uint32_t& total) {
    return block_excl_scan_n<kWaves>(v, scratch, total);
}

// check_order gate: inv[c] == 0 means check c found (or inherited) "sorted", so every kernel
// of pass >= c is skipped (replaces the reference's zeroed indirect dispatch sizes,
// CheckSort.ts:115-145).  gate == nullptr when check_order is off.
__device__ __forceinline__ bool gated_off(const uint32_t* gate, int upto) {
    if (!gate) return false;
    for (int c = 0; c <= upto; ++c)
        if (gate[c] == 0u) return true;
    return false;
}

struct Chunk {          // contiguous tile range of one workgroup (prefix-sum kernels)
    uint32_t first;     // first tile
    uint32_t count;     // number of tiles
};

__device__ __forceinline__ Chunk chunk_of(uint32_t g, uint32_t base, uint32_t extra) {
    Chunk c;
    c.first = g * base + (g < extra ? g : extra);
    c.count = base + (g < extra ? 1u : 0u);
    return c;
}

// Count d in counter row h: one atomic for the wave when every active lane has the same digit
// (a 64-way same-address conflict otherwise: sorted or few-valued keys), else one per lane.
__device__ __forceinline__ void count_uniform_or_each(uint32_t* h, uint32_t d) {
    const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
    if (__ballot(d != d0) == 0ull) {
        const uint64_t act = __ballot(true);
        if (mbcnt(act) == 0) atomicAdd(&h[d0], (uint32_t)__popcll(act));
    } else {
        atomicAdd(&h[d], 1u);
    }
}

// ---- histogram (upsweep) -----------------------------------------------------------------
// counts[d * ntiles + t] = number of keys of tile t whose digit is d.  Every wave histograms
// whole tiles on its own (wave-private LDS counters: one wave's LDS operations execute in
// order, so no barrier is needed between its atomics and its read-back), with U 16-byte loads
// per lane in flight, double-buffered across iterations.
template <int R, int TILE, int U, int KS>
__global__ __launch_bounds__(kBlock) void k_histogram(
    const uint32_t* __restrict__ keys, uint32_t n, uint32_t shift, uint32_t mask,
    uint32_t ntiles, uint32_t* __restrict__ counts, const uint32_t* gate, int pass) {
    // KS = words per key (1: key array, 2: AOS records, the key in the low word)
    constexpr int RADIX = 1 << R;
    constexpr int KPV = 4 / KS;                         // keys per 16-byte load
    constexpr int STEP = 64 * KPV * U;                  // keys per wave per iteration
    constexpr int ITERS = TILE / STEP;
    static_assert(TILE % STEP == 0, "tile must be a multiple of the wave step");
    __shared__ uint32_t hist[kWaves][RADIX];
    if (gated_off(gate, pass)) return;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t nwaves = gridDim.x * kWaves;
    uint32_t* h = hist[w];
    const bool vec = (((uintptr_t)keys) & 15u) == 0;
    auto count4 = [&](const uint4& q) {
        count_uniform_or_each(h, (q.x >> shift) & mask);
        if (KS == 1) count_uniform_or_each(h, (q.y >> shift) & mask);
        count_uniform_or_each(h, (q.z >> shift) & mask);
        if (KS == 1) count_uniform_or_each(h, (q.w >> shift) & mask);
    };
    // XCD grouping (speed only): workgroups are dealt round-robin over the 8 XCDs, so the
    // workgroups of one XCD take adjacent tile groups and a 128-B line of a digit's counts row
    // (32 tiles) is written from one L2 (from 8 XCDs it reaches memory as 8 partial writes)
    const uint32_t G = gridDim.x, g = blockIdx.x;
    const uint32_t gx = (RS_HIST_XCD && (G % 8u) == 0u) ? (g & 7u) * (G >> 3) + (g >> 3) : g;
    for (uint32_t t = gx * kWaves + w; t < ntiles; t += nwaves) {
        for (uint32_t d = lane; d < (uint32_t)RADIX; d += 64) h[d] = 0u;
        const uint32_t lo = t * (uint32_t)TILE;
        if (vec && (uint64_t)lo + TILE <= n) {
            const uint4* src = reinterpret_cast<const uint4*>(keys + (size_t)lo * KS) + lane;
            uint4 a[U], b[U];
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] = src[u * 64];
#pragma unroll 1
            for (int it = 0; it < ITERS; it += 2) {
                if (it + 1 < ITERS) {
#pragma unroll
                    for (int u = 0; u < U; ++u) b[u] = src[(it + 1) * (64 * U) + u * 64];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) count4(a[u]);
                if (it + 1 < ITERS) {
                    if (it + 2 < ITERS) {
#pragma unroll
                        for (int u = 0; u < U; ++u) a[u] = src[(it + 2) * (64 * U) + u * 64];
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) count4(b[u]);
                }
            }
        } else {
            const uint64_t hi = (uint64_t)lo + TILE < n ? (uint64_t)lo + TILE : n;
            for (uint64_t j = (uint64_t)lo + lane; j < hi; j += 64)
                atomicAdd(&h[(keys[(size_t)j * KS] >> shift) & mask], 1u);
        }
        for (uint32_t d = lane; d < (uint32_t)RADIX; d += 64) counts[(size_t)d * ntiles + t] = h[d];
    }
}

// ---- digit x tile scan ---------------------------------------------------------------------
// Block d scans row d of counts (rowlen entries) to an exclusive prefix in place and writes the
// row total to totals[d].  The row goes through LDS in segments of up to kScanSeg entries:
// coalesced loads, each thread then owns `per` CONTIGUOUS entries (thread-local scan + one block
// scan per segment), coalesced stores.  Short rows use a short segment.
constexpr int kScanSeg = 8192;
__global__ __launch_bounds__(kBlock) void k_scan_rows(uint32_t* __restrict__ counts,
                                                      uint32_t rowlen,
                                                      uint32_t* __restrict__ totals,
                                                      const uint32_t* gate, int pass) {
    __shared__ uint32_t buf[kScanSeg + kScanSeg / 32];   // +1 word per 32: conflict-free rows
    __shared__ uint32_t scratch[kWaves];
    if (gated_off(gate, pass)) return;
    uint32_t* row = counts + (size_t)blockIdx.x * rowlen;
    const uint32_t tid = threadIdx.x;
    auto at = [](uint32_t i) { return i + (i >> 5); };
    uint32_t carry = 0;
    for (uint32_t seg0 = 0; seg0 < rowlen; seg0 += kScanSeg) {
        const uint32_t len = rowlen - seg0 < (uint32_t)kScanSeg ? rowlen - seg0 : (uint32_t)kScanSeg;
        const uint32_t per = (len + kBlock - 1) / kBlock;          // <= 32
        const uint32_t seg = per * kBlock;
#pragma unroll 4
        for (uint32_t i = tid; i < seg; i += kBlock) buf[at(i)] = i < len ? row[seg0 + i] : 0u;
        __syncthreads();
        uint32_t sum = 0;
        for (uint32_t q = 0; q < per; ++q) sum += buf[at(tid * per + q)];
        uint32_t tot;
        uint32_t run = carry + block_excl_scan(sum, scratch, tot);
        for (uint32_t q = 0; q < per; ++q) {
            const uint32_t x = buf[at(tid * per + q)];
            buf[at(tid * per + q)] = run;
            run += x;
        }
        __syncthreads();
#pragma unroll 4
        for (uint32_t i = tid; i < len; i += kBlock) row[seg0 + i] = buf[at(i)];
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) totals[blockIdx.x] = carry;
}

// ---- rank + local shuffle + scatter (downsweep) ----------------------------------------
// Tile = BLOCK threads x KPT keys.  Wave w owns positions [w*64*KPT, (w+1)*64*KPT) of the
// tile; slot j of lane l is position w*64*KPT + j*64 + l (coalesced 256-B loads per slot).
//
// In-wave stable rank, two implementations (same result, tested against each other):
//  * RANK_LDS_ATOMIC: every lane does ds_add_rtn_u32(&wave_count[digit], 1).  gfx950's LDS
//    resolves one wave's same-address atomics in lane order (probed: tools/lds_order_probe.hip,
//    6.4e8 lane atomics over random / 4-address / single-address / same-bank / partial-exec
//    patterns, 0 out of order), so the returned value is the number of same-digit keys in
//    earlier slots and lower lanes: the stable rank, for ~3 VALU + 1 LDS op per 64 keys.
//  * RANK_BALLOT: match mask from R ballots (lanes sharing my digit), mbcnt for the rank in
//    the slot, the lowest lane bumps the wave counter (ds_add_rtn) and broadcasts it
//    (ds_bpermute).  Architecture-guaranteed; ~60 VALU per 64 keys.  rs_plan_debug.rank = 1.
enum RankMode { RANK_LDS_ATOMIC = 0, RANK_BALLOT = 1 };

// Per-slot 32-bit values (ranks, then tile positions) of a thread's KPT keys.  PACK keeps two
// 16-bit values per register (a position in a <= 64K-key tile), which is what lets a 32-key-per-
// thread tile hold keys, values and positions in 128 VGPRs.
template <int KPT, bool PACK>
struct Slots {
    uint32_t r[KPT];
    __device__ __forceinline__ uint32_t get(int j) const { return r[j]; }
    __device__ __forceinline__ void set(int j, uint32_t x) { r[j] = x; }
    __device__ __forceinline__ void set2(int j, uint32_t a, uint32_t b) { r[j] = a; r[j + 1] = b; }
};
template <int KPT>
struct Slots<KPT, true> {
    uint32_t r[(KPT + 1) / 2];
    __device__ __forceinline__ uint32_t get(int j) const {
        return (j & 1) ? (r[j >> 1] >> 16) : (r[j >> 1] & 0xFFFFu);
    }
    __device__ __forceinline__ void set(int j, uint32_t x) {   // x < 2^16
        r[j >> 1] = (j & 1) ? (r[j >> 1] & 0xFFFFu) | (x << 16) : (r[j >> 1] & 0xFFFF0000u) | x;
    }
    __device__ __forceinline__ void set2(int j, uint32_t a, uint32_t b) {   // j even
        r[j >> 1] = a | (b << 16);
    }
};

// Keys past n (the last tile only) load as kPadKey: every pass's digit of it is the largest, and
// it comes after every real key in input order, so the stable rank puts the pads at tile
// positions [nvalid, TILE) - after every real key - and no per-slot validity test is needed
// while ranking and staging (such tests cost a lane mask per slot, which spilled).  Only the
// published digit count (rank_tile's npad), the next-pass totals and the scatter exclude them.
constexpr uint32_t kPadKey = 0xFFFFFFFFu;

// A bucket's records (KV: 8-byte records, key then value; else keys) into slots j of lane l of the
// wave at wbase: position wbase + 64 j + l, pads (kPadKey) from cnt on.  Buffer loads bounded to the
// bucket (past cnt they return 0): no per-slot branch.  (load_tile's per-slot `if` compiles, in the
// larger bucket tiles - 256 x 34, 1024 x 17 - to a branch per slot whose load waits for itself
// before the branch joins: one memory latency per slot.)
template <int KPT, bool KV>
__device__ __forceinline__ void load_bucket(const uint32_t* src, uint32_t wbase, uint32_t cnt, uint32_t (&k)[KPT],
                                            uint32_t (&v)[KV ? KPT : 1]) {
    constexpr uint32_t ESZ = KV ? 8u : 4u;
    const uint32_t lane = lane_id();
    // (src and cnt are the workgroup's bucket: uniform, made scalar - a descriptor the compiler cannot
    // prove uniform is issued in a loop over the lanes' distinct values)
    // (readfirstlane returns int: each half goes through uint32_t, else the low half's bit 31 would
    // sign-extend over the high half)
    cnt = (uint32_t)__builtin_amdgcn_readfirstlane(cnt);
    const uint64_t sa = reinterpret_cast<uint64_t>(src);
    const uint32_t sa_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sa >> 32));
    const uint32_t sa_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sa);
    src = reinterpret_cast<const uint32_t*>(((uint64_t)sa_hi << 32) | (uint64_t)sa_lo);
    const int lim = (int)cnt - (int)(wbase + lane);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(cnt * ESZ), 0x00020000);
    uint32_t lo = (wbase + lane) * ESZ;   // (one offset register, immediate slot offsets)
    asm volatile("" : "+v"(lo));
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        uint32_t kk;
        if constexpr (KV) {
            const auto q = __builtin_amdgcn_raw_buffer_load_b64(rr, (int)(lo + j * 64 * ESZ), 0, 0);
            kk = q[0];
            v[j] = q[1];
        } else {
            kk = __builtin_amdgcn_raw_buffer_load_b32(rr, (int)(lo + j * 64 * ESZ), 0, 0);
        }
        // (the pad mask opaque: a select on the loaded word would become a branch again)
        uint32_t m = j * 64 < lim ? 0xFFFFFFFFu : 0u;
        asm volatile("" : "+v"(m));
        k[j] = (kk & m) | (kPadKey & ~m);
    }
}

template <int KPT, int L, bool CLAMP = false>
__device__ __forceinline__ void load_tile(const uint32_t* __restrict__ in_k,
                                          const uint32_t* __restrict__ in_v, uint64_t wbase,
                                          uint32_t n, bool full, uint32_t (&k)[KPT],
                                          uint32_t (&v)[L != LAYOUT_KEYS ? KPT : 1]) {
    constexpr bool HAS_VALUES = L != LAYOUT_KEYS;
    const uint32_t lane = lane_id();
    // one base address per array and constant per-slot offsets (a 32-bit index per slot would
    // have to be recomputed and widened for every slot: it may wrap)
    const size_t b = wbase + lane;
    if (L == LAYOUT_AOS) {
        const unsigned long long* rec = reinterpret_cast<const unsigned long long*>(in_k) + b;
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const unsigned long long r = (full || b + j * 64 < n) ? ld_in(rec + j * 64)
                                                                  : (unsigned long long)kPadKey;
            k[j] = (uint32_t)r;
            v[j] = (uint32_t)(r >> 32);
        }
    } else if (full) {
        const uint32_t* pk = in_k + b;
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = ld_in(pk + j * 64);
        if (HAS_VALUES) {
            const uint32_t* pv = in_v + b;
#pragma unroll
            for (int j = 0; j < KPT; ++j) v[j] = ld_in(pv + j * 64);
        }
    } else if (CLAMP) {
        // branch-free: every slot loads (index clamped to n - 1, n >= 1), pads selected after
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const size_t p = b + j * 64;
            const size_t q = p < n ? p : (size_t)n - 1;
            const uint32_t kk = in_k[q];
            k[j] = p < n ? kk : kPadKey;
            if (HAS_VALUES) v[j] = in_v[q];
        }
    } else {
        const uint32_t* pk = in_k + b;
        const uint32_t* pv = in_v + b;
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const bool ok = b + j * 64 < n;
            k[j] = ok ? pk[j * 64] : kPadKey;
            if (HAS_VALUES) v[j] = ok ? pv[j * 64] : 0u;
        }
    }
}

// Lanes of this wave whose digit equals mine (restricted to `valid`): AND over the digit bits
// of (bit set ? ballot(bit) : ~ballot(bit)).
template <int R>
__device__ __forceinline__ uint64_t match_mask(uint32_t d, uint64_t valid) {
    uint32_t mlo = (uint32_t)valid, mhi = (uint32_t)(valid >> 32);
#pragma unroll
    for (int b = 0; b < R; ++b) {
        const uint32_t x = (uint32_t)__builtin_amdgcn_sbfe((int)d, b, 1);
        const uint64_t bb = __ballot(x != 0u);
        mlo &= ~((uint32_t)bb ^ x);
        mhi &= ~((uint32_t)(bb >> 32) ^ x);
    }
    return ((uint64_t)mhi << 32) | mlo;
}

// ---- LDS counters under duplicate-heavy keys -------------------------------------------------
// Lanes of one wave instruction that add to the SAME LDS address are serialised
// (SQ_LDS_ADDR_CONFLICT): sorted input or runs of equal keys (e.g. 2^28 keys drawn from 2^24
// values, 16 equal keys in a row) put 16-64 lanes of a slot on one counter, and a pass ran up to
// 2x slower.  Equal digits of such inputs sit in neighbouring lanes.  Each wave therefore first
// counts, over its KPT slots, the lanes that start a run of equal digits (neighbour compare by
// DPP wave_shr:1), and picks for the whole tile: few runs -> one atomic per run, by its first
// lane, adding the run length (ranks = old + position in the run); otherwise one atomic per lane
// (the uniform-key path, unchanged).  Both rank a digit's lanes in lane order (stable): the LDS
// resolves one instruction's same-address atomics in lane order, so runs of one digit get their
// bases in lane order too.
#if !RS_KNOB_OPEN || !defined(RS_RUN_HEADS_MAX)
#undef RS_RUN_HEADS_MAX
#define RS_RUN_HEADS_MAX 32   // average run heads per slot at or below which a wave counts runs
#endif

// Lanes that start a run of equal d (lane 0 always does).
__device__ __forceinline__ uint64_t run_heads(uint32_t d) {
    const uint32_t dp = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d, 0x138 /* wave_shr:1 */,
                                                              0xf, 0xf, false);
    return __ballot(lane_id() == 0 || d != dp);
}

// Does this wave's tile have at most RS_RUN_HEADS_MAX run heads per slot on average?  Sampled
// on every RS_RUN_SAMPLE-th slot (the test runs on every tile of uniform keys too).
#if !RS_KNOB_OPEN || !defined(RS_RUN_SAMPLE)
#undef RS_RUN_SAMPLE
#define RS_RUN_SAMPLE 4
#endif
template <int KPT>
__device__ __forceinline__ bool few_runs(const uint32_t (&k)[KPT], uint32_t shift, uint32_t mask) {
    shift = opaque_u(shift);   // these digits are not kept for the counting loop (registers)
    uint32_t heads = 0, slots = 0;
#pragma unroll
    for (int j = 0; j < KPT; j += RS_RUN_SAMPLE) {
        heads += (uint32_t)__popcll(run_heads((k[j] >> shift) & mask));
        ++slots;
    }
    return heads <= slots * (uint32_t)RS_RUN_HEADS_MAX;
}

// Length of the run that head lane `lane` starts.
__device__ __forceinline__ uint32_t run_length(uint64_t hm, uint32_t lane) {
    const uint64_t above = lane == 63 ? 0ull : hm & (~0ull << (lane + 1));
    return (above ? (uint32_t)__builtin_ctzll(above) : 64u) - lane;
}

// Runs path, one slot: stable rank of this lane's digit d in counter row h.
__device__ __forceinline__ uint32_t rank_add_runs(uint32_t* h, uint32_t d) {
    const uint32_t lane = lane_id();
    const uint64_t hm = run_heads(d);
    uint32_t old = 0;
    if ((hm >> lane) & 1ull) old = atomicAdd(&h[d], run_length(hm, lane));
    const uint64_t le = hm & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
    const uint32_t hl = 63u - (uint32_t)__builtin_clzll(le);     // my run's first lane
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(hl << 2), (int)old) + (lane - hl);
}

// Counts every slot's digit (k >> shift) & mask in counter row h (whole-array totals).
template <int KPT>
__device__ __forceinline__ void count_slots(const uint32_t (&k)[KPT], uint32_t* h, uint32_t shift,
                                            uint32_t mask) {
    const uint32_t lane = lane_id();
    if (few_runs<KPT>(k, shift, mask)) {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t d = (k[j] >> shift) & mask;
            const uint64_t hm = run_heads(d);
            if ((hm >> lane) & 1ull) atomicAdd(&h[d], run_length(hm, lane));
        }
    } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j) atomicAdd(&h[(k[j] >> shift) & mask], 1u);
    }
}

// Stable in-wave ranks of the KPT slots (see RankMode); counters in `whist` (this wave's row).
// Every slot is ranked (pads included, see kPadKey).  PR: a slot holding pads (kPadKey: the
// bucket's tail, lanes in a row with one digit) is ranked by runs - one add per run instead of up
// to 64 returning adds to one address, which the LDS serialises.  Measured (profiles/r06/pad_runs):
// the keys-only wave bucket sort 0.183 -> 0.161 ms (its 1152-key tile holds ~128 pads: two slots);
// the KV bucket sort and the pass kernels slower (the per-slot test costs more than their pads), so
// only the wave bucket sort sets it.
template <int R, int KPT, int RANK, bool PR = false, class RK>
__device__ __forceinline__ void rank_slots(const uint32_t (&k)[KPT], RK& rank,
                                           uint32_t* whist, uint32_t shift, uint32_t mask) {
    const uint32_t lane = lane_id();
    if (RANK == RANK_LDS_ATOMIC) {
        if (few_runs<KPT>(k, shift, mask)) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t r = rank_add_runs(whist, (k[j] >> shift) & mask);
                if (j & 1) rank.set2(j - 1, rank.get(j - 1), r);
                else rank.set(j, r);
            }
        } else {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const uint32_t d = (k[j] >> shift) & mask;
                uint32_t r;
                if (PR && __ballot(k[j] == kPadKey) != 0ull) r = rank_add_runs(whist, d);
                else r = atomicAdd(&whist[d], 1u);
                if (j & 1) rank.set2(j - 1, rank.get(j - 1), r);
                else rank.set(j, r);
            }
        }
    } else {
        uint32_t info[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t d = (k[j] >> shift) & mask;
            const uint64_t m = match_mask<R>(d, ~0ull);
            const uint32_t lt = mbcnt(m);
            const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
            const uint32_t leader = lo ? (uint32_t)__builtin_ctz(lo) : 32u + (uint32_t)__builtin_ctz(hi);
            uint32_t old = 0;
            if (lt == 0) old = atomicAdd(&whist[d], (uint32_t)__popcll(m));
            info[j] = __builtin_amdgcn_ds_bpermute((int)(leader << 2), (int)old) + lt;
        }
        (void)lane;
#pragma unroll
        for (int j = 0; j < KPT; ++j) rank.set(j, info[j]);
    }
}

// ---- one tile: rank, digit offsets, local shuffle, scatter (shared by the pass kernels) -------
// Tile = BLOCK threads x KPT keys in registers (slot j of lane l of wave w = position
// w*64*KPT + j*64 + l).  `s_whist` holds per-wave digit counts, then per-wave tile offsets.

// Rank the tile's keys (stable, per wave) and return, for thread d < RADIX, the count of digit d
// in the tile without the npad pads (c) and its start in the tile (the return value).  The
// caller turns the per-wave counts into per-wave offsets (set_wave_offsets) before staging.
// Two barriers.
template <int R, int NW, int KPT, int RANK, class RK>
__device__ __forceinline__ uint32_t rank_tile(const uint32_t (&k)[KPT], RK& rank,
                                              uint32_t (*s_whist)[1 << R], uint32_t* s_scratch,
                                              uint32_t shift, uint32_t mask, uint32_t npad,
                                              uint32_t& c) {
    constexpr int RADIX = 1 << R;
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    // zero this wave's counters (the previous tile's readers finished at the last barrier)
    for (uint32_t d = lane_id(); d < (uint32_t)RADIX; d += 64) s_whist[w][d] = 0u;
    rank_slots<R, KPT, RANK>(k, rank, s_whist[w], shift, mask);
    __syncthreads();
    c = 0;
    if (tid < (uint32_t)RADIX) {
#pragma unroll
        for (int q = 0; q < NW; ++q) c += s_whist[q][tid];
        if (tid == mask) c -= npad;   // the pads' digit; they sort after every real key
    }
    uint32_t ttot;
    return block_excl_scan_n<NW>(c, s_scratch, ttot);
}

// Thread d < RADIX: per-wave counts of digit d -> per-wave offsets inside the tile.
template <int R, int NW>
__device__ __forceinline__ void set_wave_offsets(uint32_t (*s_whist)[1 << R], uint32_t tstart) {
    uint32_t o = tstart;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
        const uint32_t x = s_whist[q][threadIdx.x];
        s_whist[q][threadIdx.x] = o;
        o += x;
    }
}

// Local shuffle: the tile, stably sorted by digit, into LDS (s_kv with values, else s_keys).
// With s_ntot, also counts the next pass's digit of every key (whole-array totals; the caller
// removes the pads' count).
template <int KPT, bool HAS_VALUES, int TILE, class RK>
__device__ __forceinline__ void stage_tile(const uint32_t (&k)[KPT], const uint32_t (&v)[HAS_VALUES ? KPT : 1],
                                           const RK& rank, const uint32_t* whist_w,
                                           uint32_t* s_keys, uint2* s_kv, uint32_t shift,
                                           uint32_t mask, uint32_t* s_ntot, uint32_t nshift,
                                           uint32_t nmask) {
    shift = opaque_u(shift);
    if constexpr (RS_STAGE_BATCH && HAS_VALUES) {
        // every slot's wave offset read first (KPT LDS reads in flight), then the KPT writes: the
        // read -> write dependency of one slot no longer serialises the LDS latency slot by slot
        // (records only: keys only measured 1.5 % slower, profiles/r05/ab_hist16 config2)
        uint32_t s[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) s[j] = whist_w[(k[j] >> shift) & mask] + rank.get(j);
#pragma unroll
        for (int j = 0; j < KPT; ++j)
            if (s[j] < (uint32_t)TILE)   // always; keeps a bug from writing past the staging area
                s_kv[s[j]] = make_uint2(k[j], v[j]);
    } else {
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t s = whist_w[(k[j] >> shift) & mask] + rank.get(j);
            if (s < (uint32_t)TILE) {   // always; keeps a bug from writing past the staging area
                if (HAS_VALUES) s_kv[s] = make_uint2(k[j], v[j]);
                else s_keys[s] = k[j];
            }
        }
    }
    if (s_ntot) count_slots<KPT>(k, s_ntot, nshift, nmask);
}

// Staging round of a tile larger than the LDS staging area: the keys whose tile position
// (pos, from set_positions) lies in [lo, lo + STAGE) go to LDS slot pos - lo.
template <int KPT, bool HAS_VALUES, int STAGE, class RK>
__device__ __forceinline__ void stage_round(const uint32_t (&k)[KPT], const uint32_t (&v)[HAS_VALUES ? KPT : 1],
                                            const RK& pos, uint32_t* s_keys, uint2* s_kv,
                                            uint32_t lo) {
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t s = pos.get(j) - lo;
        if (s < (uint32_t)STAGE) {
            if (HAS_VALUES) s_kv[s] = make_uint2(k[j], v[j]);
            else s_keys[s] = k[j];
        }
    }
}

// Ranks -> tile positions in place (per-wave offsets in whist_w); with s_ntot, also counts the
// next pass's digit of every key (the caller removes the pads' count).
template <int KPT, class RK>
__device__ __forceinline__ void set_positions(const uint32_t (&k)[KPT], RK& rank,
                                              const uint32_t* whist_w, uint32_t shift, uint32_t mask,
                                              uint32_t* s_ntot, uint32_t nshift, uint32_t nmask) {
    static_assert(KPT % 2 == 0, "slot pairs");
    shift = opaque_u(shift);
#pragma unroll
    for (int j = 0; j < KPT; j += 2)
        rank.set2(j, whist_w[(k[j] >> shift) & mask] + rank.get(j),
                  whist_w[(k[j + 1] >> shift) & mask] + rank.get(j + 1));
    if (s_ntot) count_slots<KPT>(k, s_ntot, nshift, nmask);
}

// Coalesced scatter of the staged tile: consecutive lanes write consecutive positions of a digit
// run (global position = s_gdelta[digit] + position in the tile).  LO: output layout.
// The staged keys are tile positions [pbase, pbase + nvalid).
template <int BLOCK, bool HAS_VALUES, int LO>
__device__ __forceinline__ void scatter_tile(const uint32_t* s_keys, const uint2* s_kv,
                                             const uint32_t* s_gdelta, uint32_t* __restrict__ out_k,
                                             uint32_t* __restrict__ out_v, uint32_t n,
                                             uint32_t nvalid, uint32_t tile0, uint32_t shift,
                                             uint32_t mask, uint32_t pbase = 0,
                                             uint32_t pmask = 0xFFFFFFFFu) {
    // pmask: output positions taken modulo a power-of-two ring (the IC-resident R2 ring of the
    // hybrid path's fused tail); all ones otherwise
#pragma unroll 4
    for (uint32_t i = threadIdx.x; i < nvalid; i += BLOCK) {
        uint32_t key, val = 0;
        if (HAS_VALUES) {
            const uint2 kv = s_kv[i];
            key = kv.x;
            val = kv.y;
        } else {
            key = s_keys[i];
        }
        const uint32_t pos = RS_DIAG_SEQ ? tile0 + pbase + i : s_gdelta[(key >> shift) & mask] + pbase + i;
        if (pos < n) {  // never false for consistent offsets; keeps a bug from faulting
            const uint32_t q = pos & pmask;
            if (LO == LAYOUT_AOS) {
                st_out(reinterpret_cast<unsigned long long*>(out_k) + q,
                       (unsigned long long)key | ((unsigned long long)val << 32));
            } else {
                st_out(out_k + q, key);
                if (HAS_VALUES) st_out(out_v + q, val);
            }
        }
    }
}

// Workgroup g owns tiles g, g+G, g+2G, ... (per-tile counts, so any ownership works).
// XCD grouping (speed only, never correctness): workgroups are dealt round-robin over the 8
// XCDs, so workgroup g sits on XCD g % 8 as slot g / 8.  Round r gives XCD x the tiles
// (8r + x) * (G/8) + slot: the workgroups of one XCD scatter ADJACENT tiles at the same time,
// so each digit's writes from one XCD form one contiguous stream.
template <int R, int BLOCK, int KPT, int L, int RANK>
__global__ __launch_bounds__(BLOCK, pass_min_waves(BLOCK, KPT)) void k_scatter(
    const uint32_t* __restrict__ in_k, const uint32_t* __restrict__ in_v,
    uint32_t* __restrict__ out_k, uint32_t* __restrict__ out_v, uint32_t n, uint32_t shift,
    uint32_t mask, uint32_t ntiles, const uint32_t* __restrict__ counts,
    const uint32_t* __restrict__ totals, const uint32_t* gate, int pass) {
    constexpr bool HAS_VALUES = L != LAYOUT_KEYS;
    constexpr int RADIX = 1 << R;
    constexpr int NW = BLOCK / 64;
    constexpr int TILE = BLOCK * KPT;
    constexpr int WAVE_KEYS = 64 * KPT;
    static_assert(RADIX <= BLOCK, "one digit per thread");
    __shared__ uint32_t s_whist[NW][RADIX];          // per-wave counts -> per-wave tile offsets
    __shared__ uint32_t s_gdelta[RADIX];             // global pos - tile pos, per digit
    __shared__ uint32_t s_scratch[NW];
    __shared__ uint32_t s_keys[HAS_VALUES ? 1 : TILE];
    __shared__ uint2 s_kv[HAS_VALUES ? TILE : 1];    // (key, value) staged as one 64-bit word

    if (gated_off(gate, pass)) return;
    const uint32_t G = gridDim.x, g = blockIdx.x, tid = threadIdx.x;
    const uint32_t w = tid >> 6;

    // Global base of digit `tid`: sum of the totals of smaller digits; the tile's row prefix
    // is added per tile.
    uint32_t dtot = (tid < (uint32_t)RADIX) ? totals[tid] : 0u;
    uint32_t all;
    const uint32_t dbase = block_excl_scan_n<NW>(dtot, s_scratch, all);
    const bool xg = RS_XCD_GROUP && (G % 8u) == 0u;
    const uint32_t first = xg ? (g & 7u) * (G >> 3) + (g >> 3) : g;
    const uint32_t count = first < ntiles ? (ntiles - first + G - 1) / G : 0u;
    uint32_t k[KPT];
    uint32_t v[HAS_VALUES ? KPT : 1];
    if (count) {
        const uint32_t tile0 = first * (uint32_t)TILE;
        load_tile<KPT, L>(in_k, in_v, (uint64_t)tile0 + w * WAVE_KEYS, n,
                                   (uint64_t)tile0 + TILE <= n, k, v);
    }
    for (uint32_t t = 0; t < count; ++t) {
        const uint32_t tidx = first + t * G;
        const uint32_t tile0 = tidx * (uint32_t)TILE;
        const bool full = (uint64_t)tile0 + TILE <= n;
        uint32_t run = 0;
        if (tid < (uint32_t)RADIX) run = dbase + counts[(size_t)tid * ntiles + tidx];
        Slots<KPT, false> rank;
        uint32_t c;
        const uint32_t tstart = rank_tile<R, NW, KPT, RANK>(k, rank, s_whist, s_scratch, shift,
                                                            mask, full ? 0u : tile0 + TILE - n, c);
        if (tid < (uint32_t)RADIX) {
            set_wave_offsets<R, NW>(s_whist, tstart);
            s_gdelta[tid] = run - tstart;
        }
        __syncthreads();
        stage_tile<KPT, HAS_VALUES, TILE>(k, v, rank, s_whist[w], s_keys, s_kv, shift, mask,
                                          nullptr, 0u, 0u);
        __syncthreads();
        // Prefetch the next tile into the (now free) key/value registers; its latency hides
        // under this tile's scatter.
        if (t + 1 < count) {
            const uint32_t nt0 = tile0 + G * TILE;
            load_tile<KPT, L>(in_k, in_v, (uint64_t)nt0 + w * WAVE_KEYS, n, (uint64_t)nt0 + TILE <= n, k, v);
        }
        scatter_tile<BLOCK, HAS_VALUES, L>(s_keys, s_kv, s_gdelta, out_k, out_v, n,
                                           full ? (uint32_t)TILE : n - tile0, tile0, shift, mask);
        __syncthreads();
    }
}

// Digit widths of the passes of one sort (pass p uses bits [sum(width[<p]), +width[p])).
struct PassList {
    uint32_t count;
    uint32_t width[16];
};

// ---- whole-array digit totals of every pass, from one read of the keys --------------------
// The digit histogram of pass p over the whole array does not depend on the order earlier
// passes left the keys in, so the unsorted input gives every pass's totals at once.
// out[off(p) + d], off(p) = sum of 2^width[<p] (<= kTotalsMax entries), zeroed by the caller.
// Wave-private LDS counters; one global atomic per non-zero counter per workgroup.  KS = words
// per key (2 for AOS records).
// chk (may be null, check_order): the order check of pass 0's input fused into this read of it,
// *chk |= 1 if any adjacent pair is out of order under fmask (k_check's job, one read fewer).
constexpr int kTotalsMax = 1024;
#if !RS_KNOB_OPEN || !defined(RS_TOT_BLOCK)
#undef RS_TOT_BLOCK
#define RS_TOT_BLOCK 256     // k_pass_totals threads per workgroup
#endif
#if !RS_KNOB_OPEN || !defined(RS_TOT_PER_CU)
#undef RS_TOT_PER_CU
#define RS_TOT_PER_CU 8      // k_pass_totals workgroups per CU
#endif
#if !RS_KNOB_OPEN || !defined(RS_TOT_U)
#undef RS_TOT_U
#define RS_TOT_U 1           // k_pass_totals 16-byte loads per lane issued together
#endif
// only (bit p): count pass p's digit (its slot of out stays as it is otherwise).
template <int KS, int BLOCK = RS_TOT_BLOCK>
__global__ __launch_bounds__(BLOCK) void k_pass_totals(const uint32_t* __restrict__ keys,
                                                       uint32_t n, PassList pl, uint32_t shift0,
                                                       uint32_t* __restrict__ out,
                                                       uint32_t* chk = nullptr,
                                                       uint32_t fmask = 0xFFFFFFFFu,
                                                       uint32_t only = 0xFFFFu,
                                                       const uint32_t* gate = nullptr) {
    // pass p's digit starts at bit shift0 + sum(width[<p]) (shift0 = 0 for a sort)
    constexpr int NWT = BLOCK / 64;
    __shared__ uint32_t hist[NWT][kTotalsMax];
    if (gate && gated_off(gate, 0)) return;
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    uint32_t total = 0;
    for (uint32_t p = 0; p < pl.count; ++p) total += 1u << pl.width[p];
    for (uint32_t i = tid; i < (uint32_t)(NWT * kTotalsMax); i += BLOCK) (&hist[0][0])[i] = 0u;
    __syncthreads();
    uint32_t* h = hist[w];
    auto count_key = [&](uint32_t key) {
        uint32_t off = 0, shift = shift0;
        for (uint32_t p = 0; p < pl.count; ++p) {
            const uint32_t wd = pl.width[p];
            if ((only >> p) & 1u) atomicAdd(&h[off + ((key >> shift) & ((1u << wd) - 1u))], 1u);
            off += 1u << wd;
            shift += wd;
        }
    };
    constexpr uint32_t KPV = 4 / KS;               // keys per 16-byte load
    const uint32_t nv = n / KPV;
    const uint4* k4 = reinterpret_cast<const uint4*>(keys);
    const bool vec = (((uintptr_t)keys) & 15u) == 0;
    const uint32_t stride = gridDim.x * BLOCK;
    uint32_t i0 = 0;
    bool bad = false;
    auto inv = [&](uint32_t a, uint32_t b) { bad |= (a & fmask) > (b & fmask); };
    // vector i's keys, and (check) its last key against its successor: the first key of vector
    // i + 1, held by the next lane when the whole wave runs this iteration (DPP wave_shl:1),
    // else loaded; none after key n - 1
    auto vec4 = [&](uint32_t i, const uint4& q) {
        count_key(q.x);
        if (KS == 1) count_key(q.y);
        count_key(q.z);
        if (KS == 1) count_key(q.w);
        if (chk) {
            const uint32_t nl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.x, 0x130 /* wave_shl:1 */,
                                                                      0xf, 0xf, false);
            uint32_t nx = nl;
            if (!(__ballot(true) == ~0ull && lane_id() != 63)) {
                const uint32_t j = KPV * (i + 1);
                nx = j < n ? keys[(size_t)j * KS] : 0xFFFFFFFFu;
            }
            if (KS == 1) {
                inv(q.x, q.y);
                inv(q.y, q.z);
                inv(q.z, q.w);
                inv(q.w, nx);
            } else {
                inv(q.x, q.z);
                inv(q.z, nx);
            }
        }
    };
    if (vec) {
        // kTotU 16-byte loads per lane in flight, then their counts
        constexpr int kTotU = RS_TOT_U;
        uint32_t i = blockIdx.x * BLOCK + tid;
        for (; (uint64_t)i + (kTotU - 1) * (uint64_t)stride < nv; i += kTotU * stride) {
            uint4 q[kTotU];
#pragma unroll
            for (int u = 0; u < kTotU; ++u) q[u] = k4[i + u * stride];
#pragma unroll
            for (int u = 0; u < kTotU; ++u) vec4(i + u * stride, q[u]);
        }
        for (; i < nv; i += stride) vec4(i, k4[i]);
        i0 = KPV * nv;
    }
    // 64-bit index: with n close to 2^32, i + stride would wrap (stride divides 2^32)
    for (uint64_t i = (uint64_t)i0 + blockIdx.x * BLOCK + tid; i < n; i += stride) {
        const uint32_t key = keys[i * KS];
        count_key(key);
        if (chk && i + 1 < n) inv(key, keys[(i + 1) * KS]);
    }
    if (chk && __ballot(bad) != 0ull && lane_id() == 0) atomicOr(chk, 1u);
    __syncthreads();
    for (uint32_t i = tid; i < total; i += BLOCK) {
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < NWT; ++q) c += hist[q][i];
        if (c) atomicAdd(&out[i], c);
    }
}

// ---- one launch per pass: rank + scatter with decoupled look-back ----------------------
// Tiles are taken in order from a ticket counter (so every tile's predecessors are finished or
// held by running workgroups: no residency assumption, no deadlock).  Per tile and digit d the
// tile publishes status[T][d] = (AGGREGATE, its count of d) right after ranking, walks back
// over its predecessors summing aggregates until it meets an INCLUSIVE prefix, and publishes
// (INCLUSIVE, digit base + count of d in tiles <= T).  The digit bases (exclusive scan of the
// whole-array totals from k_pass_totals) replace the per-pass histogram + row scan: one read
// and one write of the keys (+values) per pass instead of two reads and one write.
// A status word is one 64-bit value ((epoch << 2 | flag) << 32 | count), stored and loaded as
// agent-scope relaxed atomics: flag and payload travel together, so no fence or counter is
// needed.  `epoch` is new for every launch, so words left by earlier launches read as "not
// published" and the region never needs clearing (the host clears it when the epoch wraps).
// Waits are bounded: a timeout sets err[0] (never a hang).
constexpr uint32_t kStAggregate = 1u, kStInclusive = 2u;
#if !RS_KNOB_OPEN || !defined(RS_LOOKBACK)
#undef RS_LOOKBACK
#define RS_LOOKBACK 4
#endif
// k_onesweep issues the next tile's loads after staging, before the look-back, in every wave.
// Measured and dropped (profiles/r03_prefetch_placement_ab.json, profiles/r04/quick1, profiles/r05/
// ab_vmwait; the code is in the history): the loads after the look-back (slower), the next ticket
// taken at the top of the tile, the loads issued slot by slot while staging with the ticket held a
// tile ahead (RS_AHEAD, within noise), and explicit vmcnt waits so that the next tile's rank runs
// while this tile's stores drain (0.5 % slower).
constexpr int kLookback = RS_LOOKBACK;   // predecessors read per look-back step
#if !RS_KNOB_OPEN || !defined(RS_LB_FIRST)
#undef RS_LB_FIRST
#define RS_LB_FIRST RS_LOOKBACK   // k_msd_pass: predecessors read by the first look-back step
#endif

__device__ __forceinline__ unsigned long long st_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_store(unsigned long long* p, uint32_t tag, uint32_t v) {
    __hip_atomic_store(p, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Any adjacent pair of this wave's slot-ordered keys out of order under fmask?  Slot j lane l is
// position j*64 + l: its successor is lane l+1 (DPP wave_shl:1), or lane 0 of slot j+1, or, after
// the last slot, `after`.  Pads (kPadKey) mask to the maximum and never form an inversion.
template <int KPT>
__device__ __forceinline__ bool wave_inversion(const uint32_t (&k)[KPT], uint32_t after,
                                               uint32_t fmask) {
    const bool last = lane_id() == 63;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)k[j], 0x130 /* wave_shl:1 */,
                                                                  0xf, 0xf, false);
        const uint32_t s0 = (j + 1 < KPT) ? (uint32_t)__builtin_amdgcn_readfirstlane(k[j + 1 < KPT ? j + 1 : j])
                                          : after;
        bad |= (k[j] & fmask) > ((last ? s0 : nx) & fmask);
    }
    return __ballot(bad) != 0ull;
}

// SR > 1: the tile is SR times the LDS staging area (32K-key tiles from 1024 threads x 32 keys
// with values, staged and scattered in two rounds of 16K positions).  Longer digit runs per tile
// mean fewer 128-B lines shared by two tiles' runs; such a line reaches memory as two partial
// writes, and those cost as much as a third more than whole lines (tools/line_probe.hip).
// SEG (the hybrid MSD path's second pass, see k_msd_plan): the input is cut into segments (the
// top-byte buckets of the first MSD pass); tiles never straddle a segment, a segment's last tile
// may be partial, and every segment has its own digit bases (base16[(seg << 8) | d]) and its own
// look-back chain (its first tile publishes an inclusive prefix at once).  segtab = [257] first
// tile of every segment (+ the total), [256] segment starts, [256] segment ends; the tile count is
// segtab[256] (ntiles is only its bound).
// SEG = 2 (the split of over-full buckets, k_split_count): the segments are listed buckets, their
// table in global memory (split_tab: [0] segment count, then first tiles [smax + 1], starts [smax],
// ends [smax]; ntiles = smax) and their digit bases absolute (base16[(seg << 8) | d]).
// KB (the hybrid MSD path's first pass over a known key range): every real key is replaced by
// key - kbase as it is loaded, so the digits and the output are of the range-relative keys.
template <int R, int BLOCK, int KPT, int L, int RANK, int LO = L, int SR = 1, int SEG = 0, bool KB = false>
__global__ __launch_bounds__(BLOCK, pass_min_waves(BLOCK, KPT)) void k_onesweep(
    const uint32_t* __restrict__ in_k, const uint32_t* __restrict__ in_v,
    uint32_t* __restrict__ out_k, uint32_t* __restrict__ out_v, uint32_t n, uint32_t shift,
    uint32_t mask, uint32_t ntiles, const uint32_t* __restrict__ dtot,
    unsigned long long* status, uint32_t* ticket, uint32_t* err, uint32_t* __restrict__ ntot,
    uint32_t nshift, uint32_t nmask, uint32_t epoch, const uint32_t* gate, int pass,
    uint32_t* chk, uint32_t fmask, uint32_t spin_max, uint32_t* host_err,
    const uint32_t* __restrict__ segtab = nullptr, const uint32_t* __restrict__ base16 = nullptr,
    uint32_t kbase = 0, uint32_t pmask = 0xFFFFFFFFu) {
    // ntot (may be null): whole-array totals of the NEXT pass's digit (key >> nshift) & nmask,
    // counted here from the keys this workgroup stages, so only pass 0 needs k_pass_totals.
    // chk (may be null, check_order, pass > 0): the order check of this pass's input, fused:
    // chk[pass] |= 1 if any adjacent pair is out of order under fmask (k_check's job, without
    // reading the keys again); this pass then gates on the checks of the passes before it only.
    // L / LO: input / output layout (SOA <-> AOS alternate on the separate-values path).
    constexpr bool HAS_VALUES = L != LAYOUT_KEYS;
    static_assert((L == LAYOUT_KEYS) == (LO == LAYOUT_KEYS), "values in and out");
    constexpr int RADIX = 1 << R;
    constexpr int NW = BLOCK / 64;
    constexpr int TILE = BLOCK * KPT;
    constexpr int STAGE = TILE / SR;
    constexpr int WAVE_KEYS = 64 * KPT;
    static_assert(RADIX <= BLOCK, "one digit per thread");
    static_assert(SR == 1 || TILE <= 65536, "packed 16-bit tile positions");
    __shared__ uint32_t s_whist[NW][RADIX];
    __shared__ uint32_t s_gdelta[RADIX];
    __shared__ uint32_t s_dbase[RADIX];
    __shared__ uint32_t s_scratch[NW];
    __shared__ uint32_t s_next;
    __shared__ uint32_t s_ntot[256];
    __shared__ uint32_t s_keys[HAS_VALUES ? 1 : STAGE];
    __shared__ uint2 s_kv[HAS_VALUES ? STAGE : 1];
    __shared__ uint32_t s_inv;
    constexpr bool SG = SEG != 0;
    static_assert(!SG || (SR == 1 && RADIX == 256), "segmented pass: one staging round, 8-bit digits");
    __shared__ uint32_t s_seg[SEG == 1 ? 769 : 1];

    if (gated_off(gate, chk ? pass - 1 : pass)) return;
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    for (uint32_t d = tid; d < 256u; d += BLOCK) s_ntot[d] = 0u;
    if (SEG == 1)
        for (uint32_t i = tid; i < 769u; i += BLOCK) s_seg[i] = segtab[i];
    // SEG = 2: the split table (global): count, first tiles, starts, ends
    const uint32_t nseg2 = SEG == 2 ? segtab[0] : 0u;
    const uint32_t* first2 = segtab + 1;
    const uint32_t* start2 = segtab + 2 + ntiles;
    const uint32_t* end2 = segtab + 2 + 2 * ntiles;
    if (tid == 0) s_inv = 0u;
    {   // first output position of every digit
        const uint32_t c = (!SG && tid < (uint32_t)RADIX && tid <= mask) ? dtot[tid] : 0u;
        uint32_t all;
        const uint32_t ex = block_excl_scan_n<NW>(c, s_scratch, all);
        if (tid < (uint32_t)RADIX) s_dbase[tid] = ex;
        if (tid == 0) s_next = atomicAdd(ticket, 1u);
        __syncthreads();
    }
    uint32_t T = s_next;
    // SEG: the tile count the plan kernel wrote
    const uint32_t nt = SEG == 1 ? s_seg[SEG == 1 ? 256 : 0] : (SEG == 2 ? first2[nseg2] : ntiles);
    // first record and end of tile t (and, SEG, its segment and the segment's first tile)
    auto geom = [&](uint32_t t, uint32_t& t0, uint32_t& tend, uint32_t& seg, uint32_t& first) {
        if (SEG == 2) {
            uint32_t lo = 0, hi = nseg2;                 // first2[lo] <= t < first2[hi]
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (first2[mid] <= t) lo = mid;
                else hi = mid;
            }
            seg = lo;
            first = first2[lo];
            // (clamped to n: see k_split_count)
            const uint32_t e = end2[lo] < n ? end2[lo] : n;
            const uint32_t t0r = start2[lo] + (t - first) * (uint32_t)TILE;
            t0 = t0r < e ? t0r : e;
            tend = e - t0 < (uint32_t)TILE ? e : t0 + (uint32_t)TILE;
        } else if (SG) {
            uint32_t lo = 0, hi = 256;                   // s_seg[lo] <= t < s_seg[hi]
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_seg[mid] <= t) lo = mid;
                else hi = mid;
            }
            seg = lo;
            first = s_seg[lo];
            t0 = s_seg[257 + lo] + (t - first) * (uint32_t)TILE;
            const uint32_t e = s_seg[513 + lo];
            tend = e - t0 < (uint32_t)TILE ? e : t0 + (uint32_t)TILE;
        } else {
            seg = 0;
            first = 0;
            t0 = t * (uint32_t)TILE;
            tend = (uint64_t)t0 + TILE <= n ? t0 + (uint32_t)TILE : n;
        }
    };
    uint32_t k[KPT];
    uint32_t v[HAS_VALUES ? KPT : 1];
    // SR > 1: no per-slot load branches (they spilled).  Records come from a plan-owned buffer
    // padded to whole tiles: whole-tile loads, and the slots past n are set to kPadKey once the
    // tile has arrived.  Arrays (the caller's) load with clamped indices.
    auto load_at = [&](uint32_t t0, uint32_t bound) {
        if (SR > 1 && L == LAYOUT_AOS)
            load_tile<KPT, L>(in_k, in_v, (uint64_t)t0 + w * WAVE_KEYS, bound, true, k, v);
        else
            load_tile<KPT, L, (SR > 1)>(in_k, in_v, (uint64_t)t0 + w * WAVE_KEYS, bound, (uint64_t)t0 + TILE <= bound, k, v);
    };
    // chk: the key after this wave's slots (next wave or next tile) is loaded with the tile, so
    // that no load is issued behind the scatter's stores (a wave's vector-memory operations
    // complete in issue order: waiting for such a load would wait for every store before it)
    uint32_t bkey_nx = kPadKey;
    auto load = [&](uint32_t t) {
        uint32_t t0, tend, sg, fi;
        geom(t, t0, tend, sg, fi);
        load_at(t0, SG ? tend : n);
        if (chk) {
            const uint64_t q = (uint64_t)t0 + (w + 1) * (uint32_t)WAVE_KEYS;
            bkey_nx = q < n ? in_k[q * (L == LAYOUT_AOS ? 2u : 1u)] : kPadKey;
        }
    };
    if (T < nt) load(T);
    while (T < nt) {
        RS_STAMP(pass, ntiles, T, 0, __builtin_amdgcn_s_memtime());
        RS_STAMP(pass, ntiles, T, 7, blockIdx.x);
        uint32_t tile0, tend, seg, seg_first;
        geom(T, tile0, tend, seg, seg_first);
        const bool full = tend - tile0 == (uint32_t)TILE;
        const uint32_t nvalid = tend - tile0;
        const bool first_tile = T == seg_first;   // publishes an inclusive prefix at once
        if (SEG == 1 && tid < (uint32_t)RADIX) s_dbase[tid] = s_seg[257 + seg] + base16[(seg << 8) | tid];
        if (SEG == 2 && tid < (uint32_t)RADIX) s_dbase[tid] = base16[(seg << 8) | tid];
        if (SR > 1 && L == LAYOUT_AOS && !full) {
            const uint64_t wb = (uint64_t)tile0 + w * WAVE_KEYS + lane_id();
#pragma unroll
            for (int j = 0; j < KPT; ++j)
                if (wb + j * 64 >= n) k[j] = kPadKey;
        }
        if (KB) {   // range-relative keys (the pads past nvalid stay kPadKey)
            const uint32_t wb = w * WAVE_KEYS + lane_id();
#pragma unroll
            for (int j = 0; j < KPT; ++j)
                if (wb + j * 64 < nvalid) k[j] -= kbase;
        }
        const uint32_t npad = (uint32_t)TILE - nvalid;
        const uint32_t bkey = bkey_nx;   // the key after this wave's slots (chk)
        Slots<KPT, RS_PACK_POS && (SR > 1)> rank;
        uint32_t c;
        const uint32_t tstart = rank_tile<R, NW, KPT, RANK>(k, rank, s_whist, s_scratch, shift,
                                                            mask, npad, c);
        RS_STAMP(pass, ntiles, T, 1, __builtin_amdgcn_s_memtime());
        if (chk && wave_inversion<KPT>(k, bkey, fmask) && lane_id() == 0) s_inv = 1u;
        // Publish this tile's counts first, then do everything that needs only tile-local
        // offsets (staging, next ticket, next-tile prefetch) before walking back: the
        // predecessors get that long to publish their inclusive prefixes, and the prefetch is
        // in flight while we wait.
        unsigned long long* st = status + (size_t)T * RADIX + tid;
        if (tid < (uint32_t)RADIX) {
            if (first_tile) st_store(st, (epoch << 2) | kStInclusive, s_dbase[tid] + c);
            else st_store(st, (epoch << 2) | kStAggregate, c);
            set_wave_offsets<R, NW>(s_whist, tstart);
        }
        __syncthreads();
        RS_STAMP(pass, ntiles, T, 2, __builtin_amdgcn_s_memtime());
        if (SR == 1) {
            stage_tile<KPT, HAS_VALUES, TILE>(k, v, rank, s_whist[w], s_keys, s_kv, shift, mask,
                                              ntot ? s_ntot : nullptr, nshift, nmask);
        } else {
            set_positions<KPT>(k, rank, s_whist[w], shift, mask, ntot ? s_ntot : nullptr, nshift,
                               nmask);
            stage_round<KPT, HAS_VALUES, STAGE>(k, v, rank, s_keys, s_kv, 0u);
        }
        if (tid == 0) {
            s_next = atomicAdd(ticket, 1u);
            if (ntot && npad) atomicSub(&s_ntot[nmask], npad);   // the pads' next digit
        }
        __syncthreads();
        const uint32_t Tn = s_next;
        RS_STAMP(pass, ntiles, T, 3, __builtin_amdgcn_s_memtime());
        // the next tile's loads: they hide under the look-back and this scatter
        if (SR == 1 && Tn < nt) load(Tn);
        if (tid < (uint32_t)RADIX) {
            uint32_t excl = s_dbase[tid];
            if (!first_tile && !RS_DIAG_LB) {
                // windowed look-back: kLookback predecessors loaded at once, consumed in order
                // (aggregates summed) up to the first inclusive prefix; a not-yet-published
                // word stops the window and is re-read next round
                excl = 0;
                uint32_t j = T - 1;                  // next predecessor to consume
                uint32_t spins = 0;
#if RS_STAMPS
                uint32_t st_rounds = 0;
#endif
                for (;;) {
                    unsigned long long sv[kLookback];
#pragma unroll
                    for (int i = 0; i < kLookback; ++i)
                        sv[i] = (j >= (uint32_t)i) ? st_load(status + (size_t)(j - i) * RADIX + tid) : 0ull;
                    uint32_t used = 0;
                    bool done = false;
#if RS_STAMPS
                    if (st_rounds++ == 0) {
                        // the first round's status words have returned (behind the wave's
                        // prefetch loads: one in-order vmcnt)
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        RS_STAMP(pass, ntiles, T, 8, __builtin_amdgcn_s_memtime());
                    }
#endif
#pragma unroll
                    for (int i = 0; i < kLookback; ++i) {
                        if (done || used != (uint32_t)i) break;
                        const uint32_t f = (uint32_t)(sv[i] >> 32);
                        if ((f >> 2) != epoch || j < (uint32_t)i) break;   // not yet published
                        excl += (uint32_t)sv[i];
                        ++used;
                        done = (f & 3u) == kStInclusive;
                    }
                    if (done) break;
                    j -= used;
                    if (used == 0u) {
                        // bounded: spin_max sleeps (~ms by default) per wait, and once any wait
                        // timed out every other wait gives up at its next check, so a bug can
                        // never hang the device.  The error reaches the host through the
                        // host-mapped word (rs_plan_check / the next rs_plan_sort report it);
                        // the device word is cleared at every sort.
                        ++spins;
                        if (spins > spin_max ||
                            ((spins & 255u) == 0u &&
                             __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
#if RS_ONESWEEP_TRACE
                            if (spins > spin_max)
                                printf("lookback timeout: pass %d tile %u/%u digit %u waiting on %u word %llx epoch %u\n",
                                       pass, T, ntiles, tid, j, sv[0], epoch);
#endif
                            atomicOr(err, 1u);
                            if (host_err)
                                __hip_atomic_fetch_or(host_err, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_SYSTEM);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                st_store(st, (epoch << 2) | kStInclusive, excl + c);
#if RS_STAMPS
                RS_STAMP(pass, ntiles, T, 9, st_rounds);
                RS_STAMP(pass, ntiles, T, 10, T - 1 - j);
                RS_STAMP(pass, ntiles, T, 11, spins);
#endif
            }
            s_gdelta[tid] = excl - tstart;
        }
        __syncthreads();
        RS_STAMP(pass, ntiles, T, 4, __builtin_amdgcn_s_memtime());
#pragma unroll
        for (int h = 0; h < SR; ++h) {
            if (h > 0) {   // the previous round's scatter has read the staging area
                stage_round<KPT, HAS_VALUES, STAGE>(k, v, rank, s_keys, s_kv, h * (uint32_t)STAGE);
                __syncthreads();
                if (h == SR - 1 && Tn < nt) load(Tn);   // registers free: prefetch
            }
            const uint32_t lo = h * (uint32_t)STAGE;
            if (lo < nvalid)
                scatter_tile<BLOCK, HAS_VALUES, LO>(s_keys, s_kv, s_gdelta, out_k, out_v, n,
                                                    nvalid - lo < (uint32_t)STAGE ? nvalid - lo : (uint32_t)STAGE,
                                                    tile0, shift, mask, lo, pmask);
            // (after the last round: no barrier unless RS_OS_TAILBAR - as in k_msd_pass, the next
            // writers of the staging area, the deltas and the counters come after the next tile's
            // rank barriers, and the next-pass totals are complete before this tile's scatter)
            if (h + 1 < SR || RS_OS_TAILBAR) __syncthreads();
        }
        RS_STAMP(pass, ntiles, T, 5, __builtin_amdgcn_s_memtime());
        T = Tn;
    }
    if (ntot) {
        for (uint32_t d = tid; d <= nmask; d += BLOCK)
            if (s_ntot[d]) atomicAdd(&ntot[d], s_ntot[d]);
    }
    if (chk && tid == 0 && s_inv) atomicOr(chk + pass, 1u);
}

// ---- the hybrid path's MSD passes with values: k_msd_pass -------------------------------------
// k_onesweep's algorithm (rank, publish, local shuffle, decoupled look-back, scatter of 16K-record
// tiles by an 8-bit digit; SEG = 1: inside every top-byte segment) specialised for the two MSD
// passes of a sort with values (BASELINE config 3's hot path: 2 of its ~3.1 ms), so that a tile's
// memory traffic is in flight throughout instead of in two separate phases:
//  * the look-back's first status words are read BEFORE the next tile's loads are issued (a wave's
//    vector-memory operations complete in issue order: read after them, the words waited for the
//    whole 128 KB prefetch, so the scatter's stores could only start once the next tile had
//    arrived); the scatter's stores of this tile now overlap the next tile's loads;
//  * the next tile's loads are branch-free (buffer loads whose range is the tile's valid records:
//    the lanes past it read 0 and become pads at the next rank) and the scatter is a fixed 16 stores
//    per thread (lanes past the tile's end repeat the tile's last record), so every path through
//    the loop has the same memory operations in flight and the compiler's waits count exactly:
//    the next tile's rank waits for its own loads only, while this tile's stores drain;
//  * the next tile's ticket is requested at the top of the tile and read after staging (its value,
//    used at once, would wait for every earlier store of the wave).
// Measured against k_onesweep on config3: the same time (the pass is bound by its scattered write
// pattern: tools/run_probe.hip copies 2^28 records in that pattern in 1.07 ms, the pass takes 0.99;
// profiles/r05/ab_lean_xcd).  XCD-grouped tile claims (adjacent tiles on one XCD, so that the line
// two tiles' runs share is completed in one L2) cut the probe from 1.07 to 0.89 ms but made the
// pass 4 % slower (the look-back chain then runs across the XCDs' claim rounds;
// profiles/r05/ab_xcd_hw); they are in the history (8b24fac), not here.
// No order check, no next-pass totals, no staging rounds (k_onesweep keeps those for the LSD passes).
// L: input layout (SOA arrays: pass 0 of separate arrays; AOS records: R1, or a texture), LO: output
// layout (AOS: R1 / R2 records; SOA: arrays).  KB: range-relative keys (key - kbase) as in k_onesweep.
//
// XC (round 6): XCD-local tile streams.  A line where two consecutive tiles' runs of one digit meet
// is written partly by each tile; when the two tiles run on different XCDs the line reaches memory
// as two partial writes from two L2s (the pass's 1.085x traffic and most of its time over a linear
// copy: tools/run_probe.hip).  With XC every XCD claims the tiles of its own contiguous tile range
// from its own ticket counter, and no look-back chain crosses two ranges, so consecutive tiles -
// and the lines they share - are (almost always) written through one L2 and the chains never wait
// on another XCD's claims (round 5's XCD-grouped claims over one global chain did, and lost 4 %):
//   SEG = 1: the ranges are runs of whole top-byte segments (every segment has its own chain
//            already), cut at the segment boundary nearest to each eighth of the tiles;
//   SEG = 0: the input is cut into 8 chunks at k_hist16_in row boundaries (rows [x hrows / 8,
//            (x + 1) hrows / 8) for XCD x), each chunk a segment with its own chain, whose digit-d
//            output starts at the digit's start + cbase[row][d] (k_hist16_reduce: the keys of digit d
//            in the rows before) - the per-chunk bases the histogram read gives for free.
// A workgroup whose range is exhausted takes tiles from the next XCDs' counters (balance; claims of
// one counter stay in tile order, so every look-back still waits only on tiles claimed earlier by
// running workgroups).  The XCD is read from HW_REG_XCC_ID: placement only, never correctness.
// Measured on config 3 (profiles/r06/xcd_claims/): pass 0 1.003 vs 0.993 ms, pass 1 1.045 vs 0.993 -
// slower, like round 5's grouped claims, so the product keeps one counter per pass (rs_plan_debug.xcd
// = 0); the seam lines are not what bounds the real pass (its per-tile phases are).
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}

template <int L, int LO, int SEG, bool KB = false, int RANK = RANK_LDS_ATOMIC, bool XC = false>
__global__ __launch_bounds__(1024, 4) void k_msd_pass(
    const uint32_t* __restrict__ in_k, const uint32_t* __restrict__ in_v,
    uint32_t* __restrict__ out_k, uint32_t* __restrict__ out_v, uint32_t n, uint32_t shift,
    uint32_t ntiles, const uint32_t* __restrict__ dtot, unsigned long long* status,
    uint32_t* ticket, uint32_t* err, uint32_t epoch, const uint32_t* gate, int gate_pass,
    uint32_t spin_max, uint32_t* host_err, const uint32_t* __restrict__ segtab,
    const uint32_t* __restrict__ base16, uint32_t kbase,
    const uint32_t* __restrict__ cbase = nullptr, uint32_t hrows = 0) {
    // XC: ticket = 8 counters (one per XCD); SEG = 0 also cbase (k_hist16_reduce's [row][top byte]
    // chunk starts) and hrows (k_hist16_in's grid: its chunk formula cuts the input here too)
    static_assert(L != LAYOUT_KEYS && LO != LAYOUT_KEYS, "with values");
    static_assert(SEG == 0 || SEG == 1, "the two MSD passes");
    constexpr int BLOCK = 1024, KPT = 16, R = 8, RADIX = 256, NW = BLOCK / 64;
    constexpr int TILE = BLOCK * KPT, WAVE_KEYS = 64 * KPT;
    constexpr uint32_t mask = RADIX - 1;
    constexpr uint32_t ESZ = L == LAYOUT_AOS ? 8u : 4u;   // bytes per input element (record / key)
    __shared__ uint32_t s_whist[NW][RADIX];
    __shared__ uint32_t s_gdelta[RADIX];
    __shared__ uint32_t s_dbase[RADIX];
    __shared__ uint32_t s_scratch[NW];
    __shared__ uint32_t s_next;
    __shared__ uint2 s_kv[TILE];
    __shared__ uint32_t s_seg[SEG == 1 ? 769 : 1];
    __shared__ uint32_t s_xf[XC ? 9 : 1];                  // XC: XCD x's tiles [s_xf[x], s_xf[x + 1])
    __shared__ uint32_t s_xs[XC && SEG == 0 ? 9 : 1];      // XC, SEG = 0: chunk x's first record
    __shared__ uint32_t s_xr[XC && SEG == 0 ? 9 : 1];      // ... and first histogram row

    if (gated_off(gate, gate_pass)) return;
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    if (SEG == 1)
        for (uint32_t i = tid; i < 769u; i += BLOCK) s_seg[i] = segtab[i];
    if (XC && SEG == 0 && tid <= 8u) {
        // chunk x: k_hist16_in rows [x hrows / 8, (x + 1) hrows / 8), row r = records [r chunk, (r + 1) chunk)
        const uint64_t chunk = (((uint64_t)n + hrows - 1) / hrows + 3u) & ~3ull;
        auto start = [&](uint32_t x) -> uint32_t {
            const uint64_t s = (uint64_t)(x * hrows / 8u) * chunk;
            return s < n ? (uint32_t)s : n;
        };
        uint32_t f = 0;
        for (uint32_t x = 0; x < tid; ++x) f += (start(x + 1) - start(x) + TILE - 1) / (uint32_t)TILE;
        s_xf[tid] = f;
        s_xs[tid] = start(tid);
        s_xr[tid] = tid * hrows / 8u;
    }
    uint32_t dglob = 0;   // XC, SEG = 0, thread d < 256: digit d's first output position
    {   // first output position of every digit (SEG = 0; SEG = 1 per segment, below)
        const uint32_t c = (SEG == 0 && tid < (uint32_t)RADIX) ? dtot[tid] : 0u;
        uint32_t all;
        const uint32_t ex = block_excl_scan_n<NW>(c, s_scratch, all);
        if (tid < (uint32_t)RADIX) s_dbase[tid] = ex;
        dglob = ex;
        if (XC && SEG == 1 && tid <= 8u) {
            // (s_seg is visible: the scan's barriers) XCD x's range starts at the first segment whose
            // first tile is at or after x/8 of the tiles
            const uint32_t ntt = s_seg[256];
            const uint32_t target = (uint32_t)((uint64_t)tid * ntt / 8u);
            uint32_t lo = 0, hi = 256;   // the first s with s_seg[s] >= target (s_seg[256] = ntt >= target)
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_seg[mid] >= target) hi = mid;
                else lo = mid + 1;
            }
            s_xf[tid] = tid == 8u ? ntt : s_seg[lo];
        }
        if (!XC && tid == 0) s_next = atomicAdd(ticket, 1u);
        __syncthreads();
    }
    // XC claims (thread 0): own XCD's counter first, then the next XCDs' in turn once exhausted;
    // nt when every counter is
    const uint32_t xid = XC ? xcc_id() : 0u;
    uint32_t xcur = 0;
    const uint32_t nt = XC ? s_xf[8] : (SEG == 1 ? s_seg[SEG == 1 ? 256 : 0] : ntiles);
    auto claim = [&]() -> uint32_t {
        // a lane-varying address as far as the compiler knows: its atomic optimizer would turn a
        // uniform-address add into a wave-aggregated one whose result is broadcast at once
        uint32_t z = 0;
        asm volatile("" : "+v"(z));
        if constexpr (XC) {
            for (; xcur < 8u; ++xcur) {
                const uint32_t x = (xid + xcur) & 7u;
                const uint32_t lo = s_xf[x], hi = s_xf[x + 1];
                if (lo < hi) {
                    const uint32_t t = atomicAdd(ticket + x + z, 1u);
                    if (t < hi - lo) return lo + t;
                }
            }
            return nt;
        } else {
            return atomicAdd(ticket + z, 1u);
        }
    };
    if (XC) {
        if (tid == 0) s_next = claim();
        __syncthreads();
    }
    uint32_t T = s_next;
    auto geom = [&](uint32_t t, uint32_t& t0, uint32_t& tend, uint32_t& seg, uint32_t& first) {
        if (XC && SEG == 0) {
            uint32_t x = 0;   // s_xf[x] <= t < s_xf[x + 1] (empty chunks skipped)
#pragma unroll
            for (int i = 1; i < 8; ++i) x += s_xf[i] <= t ? 1u : 0u;
            seg = x;
            first = s_xf[x];
            t0 = s_xs[x] + (t - first) * (uint32_t)TILE;
            const uint32_t e = s_xs[x + 1];
            tend = e - t0 < (uint32_t)TILE ? e : t0 + (uint32_t)TILE;
        } else if (SEG == 1) {
            uint32_t lo = 0, hi = 256;                   // s_seg[lo] <= t < s_seg[hi]
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_seg[mid] <= t) lo = mid;
                else hi = mid;
            }
            seg = lo;
            first = s_seg[lo];
            t0 = s_seg[257 + lo] + (t - first) * (uint32_t)TILE;
            const uint32_t e = s_seg[513 + lo];
            tend = e - t0 < (uint32_t)TILE ? e : t0 + (uint32_t)TILE;
        } else {
            seg = 0;
            first = 0;
            t0 = t * (uint32_t)TILE;
            tend = (uint64_t)t0 + TILE <= n ? t0 + (uint32_t)TILE : n;
        }
    };
    // Tile t's loads into k / v: buffer loads over [t0, tend) only (no branch; lanes past the end
    // read 0), t >= nt: none (range 0).  The 64-bit base is rebased to the tile (32-bit offsets).
    uint32_t k[KPT], v[KPT];
    uint32_t nb16 = 0;   // SEG = 1, thread d < 256: base16 of digit d in the loaded tile's segment
    const uint32_t lofs = (w * (uint32_t)WAVE_KEYS + lane) * ESZ;   // this lane's slot 0, bytes
    auto load = [&](uint32_t t) {
        uint32_t t0 = 0, tend = 0, sg = 0, fi;
        if (t < nt) geom(t, t0, tend, sg, fi);
        const uint32_t nbytes = (tend - t0) * ESZ;
        // one offset register with immediate slot offsets (left to itself the compiler hoists the
        // 16 per-slot offsets out of the tile loop: 16 registers)
        uint32_t lo = lofs;
        asm volatile("" : "+v"(lo));
        if constexpr (L == LAYOUT_AOS) {
            const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(in_k + 2ull * t0), (short)0, (int)nbytes, 0x00020000);
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b64(rr, (int)(lo + j * 64 * 8), 0, 0);
                k[j] = q[0];
                v[j] = q[1];
            }
        } else {
            const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(in_k + t0), (short)0, (int)nbytes, 0x00020000);
            const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(in_v + t0), (short)0, (int)nbytes, 0x00020000);
#pragma unroll
            for (int j = 0; j < KPT; ++j) k[j] = __builtin_amdgcn_raw_buffer_load_b32(rk, (int)(lo + j * 256), 0, 0);
#pragma unroll
            for (int j = 0; j < KPT; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b32(rv, (int)(lo + j * 256), 0, 0);
        }
        // (loaded with the tile: read at the top of a tile it would wait for every store before it)
        if (SEG == 1) nb16 = base16[(sg << 8) | (tid & 255u)];
        if (XC && SEG == 0) nb16 = t < nt ? cbase[(size_t)s_xr[sg] * 256u + (tid & 255u)] : 0u;
    };
    load(T);
    // the first tile's registers used (waited for) here, so that the loop top's state - which the
    // compiler merges over the loop's entry and its back edge - has only the back edge's operations
    // pending: the next tile's loads, then this tile's stores.  Its waits for the loads then let the
    // stores after them drain (an explicit s_waitcnt is dropped by the compiler's own wait pass)
#pragma unroll
    for (int j = 0; j < KPT; ++j) asm volatile("" ::"v"(k[j]), "v"(v[j]));
    if (SEG == 1 || XC) asm volatile("" ::"v"(nb16));
    uint32_t Tq = 0;   // thread 0: the next tile's ticket, requested at the top of this tile
    while (T < nt) {
        RS_STAMP(gate_pass, ntiles, T, 0, __builtin_amdgcn_s_memtime());
        RS_STAMP(gate_pass, ntiles, T, 7, blockIdx.x);
        if (tid == 0) Tq = claim();
        uint32_t tile0, tend, seg, seg_first;
        geom(T, tile0, tend, seg, seg_first);
        const uint32_t nvalid = tend - tile0;
        const bool first_tile = T == seg_first;   // publishes an inclusive prefix at once
        if (SEG == 1 && tid < (uint32_t)RADIX) s_dbase[tid] = s_seg[257 + seg] + nb16;
        if (XC && SEG == 0 && tid < (uint32_t)RADIX) s_dbase[tid] = dglob + nb16;
        {   // slots past the tile's end become pads (kPadKey: after every real key); KB: relative keys
            const uint32_t wb = w * (uint32_t)WAVE_KEYS + lane;
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                const bool ok = wb + j * 64u < nvalid;
                k[j] = ok ? (KB ? k[j] - kbase : k[j]) : kPadKey;
            }
        }
        Slots<KPT, false> rank;
        uint32_t c;
        const uint32_t tstart = rank_tile<R, NW, KPT, RANK>(k, rank, s_whist, s_scratch, shift, mask,
                                                            (uint32_t)TILE - nvalid, c);
        RS_STAMP(gate_pass, ntiles, T, 1, __builtin_amdgcn_s_memtime());
        unsigned long long* st = status + (size_t)T * RADIX + tid;
        if (tid < (uint32_t)RADIX) {
            if (first_tile) st_store(st, (epoch << 2) | kStInclusive, s_dbase[tid] + c);
            else st_store(st, (epoch << 2) | kStAggregate, c);
            set_wave_offsets<R, NW>(s_whist, tstart);
        }
        __syncthreads();
        RS_STAMP(gate_pass, ntiles, T, 2, __builtin_amdgcn_s_memtime());
        stage_tile<KPT, true, TILE>(k, v, rank, s_whist[w], nullptr, s_kv, shift, mask, nullptr, 0u, 0u);
        if (tid == 0) s_next = Tq;
        __syncthreads();
        RS_STAMP(gate_pass, ntiles, T, 3, __builtin_amdgcn_s_memtime());
        const uint32_t Tn = s_next;
        // the look-back's first status words, then the next tile's loads behind them
        const bool lb = tid < (uint32_t)RADIX && !first_tile && !RS_DIAG_LB;
        // (the first round may read a wider window, RS_LB_FIRST: it is issued before the tile loads)
        constexpr int KW = RS_LB_FIRST > kLookback ? RS_LB_FIRST : kLookback;
        unsigned long long sv[KW];
        if (lb) {
#pragma unroll
            for (int i = 0; i < KW; ++i)
                sv[i] = (i < RS_LB_FIRST && T - 1 >= (uint32_t)i) ? st_load(status + (size_t)(T - 1 - i) * RADIX + tid) : 0ull;
        }
        if (!RS_MSD_LBLATE || tid >= (uint32_t)RADIX) load(Tn);
        if (tid < (uint32_t)RADIX) {
            uint32_t excl = s_dbase[tid];
            if (lb) {
                excl = 0;
                uint32_t j = T - 1;                  // next predecessor to consume
                uint32_t spins = 0;
#if RS_STAMPS
                uint32_t st_rounds = 0;
#endif
                int nwin = RS_LB_FIRST;   // this round's window
                for (;;) {
#if RS_STAMPS
                    if (st_rounds++ == 0) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        RS_STAMP(gate_pass, ntiles, T, 8, __builtin_amdgcn_s_memtime());
                    }
#endif
                    uint32_t used = 0;
                    bool done = false;
#pragma unroll
                    for (int i = 0; i < KW; ++i) {
                        if (i >= nwin || done || used != (uint32_t)i) break;
                        const uint32_t f = (uint32_t)(sv[i] >> 32);
                        if ((f >> 2) != epoch || j < (uint32_t)i) break;   // not yet published
                        excl += (uint32_t)sv[i];
                        ++used;
                        done = (f & 3u) == kStInclusive;
                    }
                    if (done) break;
                    j -= used;
                    if (used == 0u) {   // bounded wait (k_onesweep's)
                        ++spins;
                        if (spins > spin_max ||
                            ((spins & 255u) == 0u &&
                             __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                            atomicOr(err, 1u);
                            if (host_err)
                                __hip_atomic_fetch_or(host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    nwin = kLookback;
#pragma unroll
                    for (int i = 0; i < kLookback; ++i)
                        sv[i] = (j >= (uint32_t)i) ? st_load(status + (size_t)(j - i) * RADIX + tid) : 0ull;
                }
                st_store(st, (epoch << 2) | kStInclusive, excl + c);
#if RS_STAMPS
                RS_STAMP(gate_pass, ntiles, T, 9, st_rounds);
                RS_STAMP(gate_pass, ntiles, T, 10, T - 1 - j);
                RS_STAMP(gate_pass, ntiles, T, 11, spins);
#endif
            }
            s_gdelta[tid] = excl - tstart;
        }
        if (RS_MSD_LBLATE && tid < (uint32_t)RADIX) load(Tn);
        __syncthreads();
        RS_STAMP(gate_pass, ntiles, T, 4, __builtin_amdgcn_s_memtime());
        // the scatter: a fixed KPT stores per thread (staged positions past the tile's end repeat the
        // last record: the same value to the same address), while the next tile's loads arrive
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t i0 = (uint32_t)j * BLOCK + tid;
            const uint32_t i = i0 < nvalid ? i0 : nvalid - 1u;
            const uint2 kv = s_kv[i];
            uint32_t pos = RS_DIAG_SEQ ? tile0 + i : s_gdelta[(kv.x >> shift) & mask] + i;
            pos = pos < n ? pos : n - 1u;   // never clamps for consistent offsets (no fault on a bug)
            if constexpr (LO == LAYOUT_AOS) {
                reinterpret_cast<uint2*>(out_k)[pos] = kv;   // (KB: the range-relative key)
            } else {
                out_k[pos] = kv.x;
                out_v[pos] = kv.y;
            }
        }
        if (RS_MSD_TAILBAR) __syncthreads();
        RS_STAMP(gate_pass, ntiles, T, 5, __builtin_amdgcn_s_memtime());
        T = Tn;
    }
}

// ---- one MSD pass over a static split: no look-back, no tickets -----------------------------
// The hybrid path reads a 16-bit histogram of the input before its passes (k_hist16_in: one row per
// contiguous input chunk), so the output start of every digit of every work unit is known before
// the pass begins - the reduce-then-scan form of the pass, with the reduce done by that read:
//   SEG = 0 (the top-byte pass): unit u = input chunk u (k_hist16_in's chunk of row u: the same
//           formula, the same grid); digit d of unit u starts at segment d's start + cbase[u][d];
//   SEG = 1 (the next-byte pass): unit u = top-byte segment u of R1; digit d of it starts at
//           the segment's start + base16[u << 8 | d] (k_hist16_reduce).
// A workgroup takes its unit's tiles in order and keeps each digit's running output position in
// LDS, so a tile's scatter waits for nothing but its own ranking.  (k_onesweep's decoupled look-back
// waits on status words whose loads queue behind the workgroup's own 128 KB tile prefetch in the
// CU's memory pipeline.)  Rank, local shuffle and scatter are k_onesweep's (the same helpers), so the
// output is the same stable partition.  KB: range-relative keys as in k_onesweep.
template <int BLOCK, int KPT, int L, int RANK, int LO, int SEG, bool KB = false>
__global__ __launch_bounds__(BLOCK, pass_min_waves(BLOCK, KPT)) void k_static_pass(
    const uint32_t* __restrict__ in_k, const uint32_t* __restrict__ in_v,
    uint32_t* __restrict__ out_k, uint32_t* __restrict__ out_v, uint32_t n, uint32_t shift,
    const uint32_t* gate, const uint32_t* __restrict__ segtab,
    const uint32_t* __restrict__ base16, const uint32_t* __restrict__ cbase, uint32_t kbase) {
    constexpr bool HAS_VALUES = L != LAYOUT_KEYS;
    static_assert((L == LAYOUT_KEYS) == (LO == LAYOUT_KEYS), "values in and out");
    constexpr int R = 8, RADIX = 256;
    constexpr int NW = BLOCK / 64;
    constexpr int TILE = BLOCK * KPT;
    constexpr int WAVE_KEYS = 64 * KPT;
    constexpr uint32_t mask = 255u;
    __shared__ uint32_t s_whist[NW][RADIX];
    __shared__ uint32_t s_gdelta[RADIX];
    __shared__ uint32_t s_scratch[NW];
    __shared__ uint32_t s_keys[HAS_VALUES ? 1 : TILE];
    __shared__ uint2 s_kv[HAS_VALUES ? TILE : 1];
    if (gated_off(gate, 0)) return;
    const uint32_t u = blockIdx.x, tid = threadIdx.x, w = tid >> 6;
    uint64_t lo, hi;
    if (SEG) {
        lo = segtab[257 + u];
        hi = segtab[513 + u];
    } else {   // k_hist16_in's chunk of row u
        const uint64_t chunk = (((uint64_t)n + gridDim.x - 1) / gridDim.x + 3u) & ~3ull;
        lo = (uint64_t)u * chunk < n ? (uint64_t)u * chunk : n;
        hi = lo + chunk < n ? lo + chunk : n;
    }
    if (lo >= hi) return;
    // running output position of digit `tid` (thread tid < 256 owns it for the whole unit)
    uint32_t run = 0;
    if (tid < (uint32_t)RADIX)
        run = SEG ? segtab[257 + u] + base16[(u << 8) | tid] : segtab[257 + tid] + cbase[(size_t)u * 256u + tid];
    uint32_t k[KPT];
    uint32_t v[HAS_VALUES ? KPT : 1];
    auto load = [&](uint64_t t0) {
        load_tile<KPT, L>(in_k, in_v, t0 + w * WAVE_KEYS, (uint32_t)hi, t0 + TILE <= hi, k, v);
    };
    load(lo);
    for (uint64_t t0 = lo; t0 < hi; t0 += TILE) {
        const uint32_t nvalid = (uint32_t)(hi - t0 < (uint64_t)TILE ? hi - t0 : (uint64_t)TILE);
        if (KB) {   // range-relative keys (the pads past nvalid stay kPadKey)
            const uint32_t wb = w * WAVE_KEYS + lane_id();
#pragma unroll
            for (int j = 0; j < KPT; ++j)
                if (wb + j * 64 < nvalid) k[j] -= kbase;
        }
        Slots<KPT, false> rank;
        uint32_t c;
        const uint32_t tstart = rank_tile<R, NW, KPT, RANK>(k, rank, s_whist, s_scratch, shift, mask,
                                                            (uint32_t)TILE - nvalid, c);
        if (tid < (uint32_t)RADIX) {
            set_wave_offsets<R, NW>(s_whist, tstart);
            s_gdelta[tid] = run - tstart;
            run += c;
        }
        __syncthreads();
        stage_tile<KPT, HAS_VALUES, TILE>(k, v, rank, s_whist[w], s_keys, s_kv, shift, mask, nullptr, 0u, 0u);
        __syncthreads();
        // the next tile's loads into the (now free) registers: in flight during this scatter
        if (t0 + TILE < hi) load(t0 + TILE);
        scatter_tile<BLOCK, HAS_VALUES, LO>(s_keys, s_kv, s_gdelta, out_k, out_v, n, nvalid,
                                            (uint32_t)t0, shift, mask);
        __syncthreads();
    }
}

// ---- whole sort of a small array in one workgroup ------------------------------------------
// n <= BLOCK*KPT: keys (+values) stay in registers between passes; every pass ranks, stages the
// tile sorted by its digit in LDS, and reloads the registers from LDS.  One launch, one HBM read
// and one HBM write for the whole sort.
template <int BLOCK, int KPT, int L, int RANK>
__global__ __launch_bounds__(BLOCK) void k_sort_small(uint32_t* __restrict__ keys,
                                                      uint32_t* __restrict__ values, uint32_t n,
                                                      PassList passes) {
    constexpr bool HAS_VALUES = L != LAYOUT_KEYS;
    constexpr int R = 8, RADIX = 256;
    constexpr int NW = BLOCK / 64;
    constexpr int TILE = BLOCK * KPT;
    constexpr int WAVE_KEYS = 64 * KPT;
    __shared__ uint32_t s_whist[NW][RADIX];
    __shared__ uint32_t s_scratch[NW];
    __shared__ uint32_t s_keys[HAS_VALUES ? 1 : TILE];
    __shared__ uint2 s_kv[HAS_VALUES ? TILE : 1];
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t wbase = w * WAVE_KEYS;
    uint32_t k[KPT];
    uint32_t v[HAS_VALUES ? KPT : 1];
    load_tile<KPT, L>(keys, values, wbase, n, false, k, v);
    uint32_t shift = 0;
    for (uint32_t p = 0; p < passes.count; ++p) {
        const uint32_t mask = (1u << passes.width[p]) - 1u;
        for (uint32_t d = lane; d < (uint32_t)RADIX; d += 64) s_whist[w][d] = 0u;
        Slots<KPT, false> rank;
        rank_slots<R, KPT, RANK>(k, rank, s_whist[w], shift, mask);   // pads included (kPadKey)
        __syncthreads();
        uint32_t c = 0, wc[NW];
        if (tid < (uint32_t)RADIX) {
#pragma unroll
            for (int q = 0; q < NW; ++q) { wc[q] = s_whist[q][tid]; c += wc[q]; }
        }
        uint32_t ttot;
        const uint32_t tstart = block_excl_scan_n<NW>(c, s_scratch, ttot);
        if (tid < (uint32_t)RADIX) {
            uint32_t o = tstart;
#pragma unroll
            for (int q = 0; q < NW; ++q) { s_whist[q][tid] = o; o += wc[q]; }
        }
        __syncthreads();
        // every key, pads too: they stay at positions [n, TILE) in every pass
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t s = s_whist[w][(k[j] >> shift) & mask] + rank.get(j);
            if (HAS_VALUES) s_kv[s] = make_uint2(k[j], v[j]);
            else s_keys[s] = k[j];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t p2 = wbase + j * 64 + lane;
            if (HAS_VALUES) {
                const uint2 kv = s_kv[p2];
                k[j] = kv.x;
                v[j] = kv.y;
            } else {
                k[j] = s_keys[p2];
            }
        }
        shift += passes.width[p];
        // the next pass writes s_whist / s_kv only after two more barriers
    }
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
        const uint32_t p2 = wbase + j * 64 + lane;
        if (p2 < n) {
            if (L == LAYOUT_AOS) {
                reinterpret_cast<uint2*>(keys)[p2] = make_uint2(k[j], v[j]);
            } else {
                keys[p2] = k[j];
                if (HAS_VALUES) values[p2] = v[j];
            }
        }
    }
}

// ---- hybrid MSD path (uniformly spread keys; rsort.hip enqueue_sort_msd) --------------------
// 1. k_hist16_in counts hist16[key >> 16] over the input (one row per workgroup), k_hist16_reduce
//    adds the rows and the top-byte totals (the digit totals of pass 0);
// 2. k_msd_plan scans hist16 into base16 (the first output position of every 16-bit bucket), lays
//    out the segmented tiles of pass 2, and picks the path on the device: MSD when every 16-bit
//    bucket fits the bucket tile and no top-byte bucket holds more than max_top keys, else the
//    four LSD passes (enqueued behind, gated the other way) sort the input;
// 3. MSD pass 0 (k_onesweep, top byte) writes the input partitioned by its top byte (R1, records);
// 4. MSD pass 1 (k_onesweep SEG, next byte within every top-byte segment) writes records R2 in
//    16-bit bucket order;
// 5. k_bucket_sort: one workgroup per 16-bit bucket sorts it by its low 16 bits in LDS and writes
//    it as one contiguous run of the output.  Every step is stable, so the result is the stable
//    sort of the input.  Gate words: g[0..15] MSD chosen, g[16..31] LSD on the input
//    (each word repeated: gated_off reads 0..pass).
constexpr uint32_t kGateMsd = 0, kGateLsd = 16;

__device__ __forceinline__ void set_gate(uint32_t* g, uint32_t v) {
    if (threadIdx.x < 16u) g[threadIdx.x] = v;
}

// hist16[key >> 16] of keys[0..n) (L = LAYOUT_AOS: the keys of n 8-byte records), one 1024-thread
// workgroup per CU over a contiguous chunk.  All 65536 buckets live in LDS as the 16-bit halves of
// 32768 words (128 KB, one ds_add per key).  A half never wraps: every add returns the old word, and
// the add that takes a half from below kHalfT to kHalfT or more (exactly one add per crossing) takes
// kHalfT back off the half and logs the bucket in LDS (s_ev); at the end each logged bucket gets
// kHalfT added to its count.  The adds in flight between a crossing and its take-back are far fewer
// than the 2^15 headroom above kHalfT (16 waves x a few loads x at most 256 per add).  Uniform keys
// never cross (2^28 keys over 256 chunks: ~16 per bucket and chunk), so the loop is one returning
// ds_add per key and the next loads are issued before the current ones are counted.  (Up to round 4
// each thread folded its 32 words into 64 registers and cleared them every 60K keys: the folds cost
// as many LDS operations as the counting, and the 64 registers left one group of loads in flight.)
// The workgroup's 65536 counts go to rows[blockIdx.x] as the packed halves plus the crossing log
// (kRowEv; k_hist16_reduce / k_hist16_sum add the rows and the logged kHalfT's).
// Range form (the multi-GPU group sorts): the buckets are of key - kbase >> shift, and a key
// outside [kbase, kbase + range] sets the workgroup's flag word (rows[gridDim.x * 65536 + block];
// k_msd_plan then picks the LSD passes over the whole 32-bit keys).  Records load 8 bytes per lane
// (a receive region is only 8-byte aligned), arrays 16.
// AOS_WIDE (records 16-byte aligned): two records per 16-byte load instead of one per 8-byte load.
// FULL (kbase = 0, the whole 32-bit range, shift = 16): the bucket is key >> 16 and its counter
// half bit 16, so a key costs ~4 VALU + 1 LDS atomic.
// CHECK (check_order on the hybrid path, FULL only): the same read also (a) checks the input's
// order - *inv |= 1 if any adjacent pair is out of order (every pair, the reference's quirks Q1/Q2
// fixed; CheckSort.ts:102-113) - and (b, CHECK = 2) counts the low byte of every key into
// b0rows[block][256] (the LSD fallback's pass-0 totals: k_hist16_reduce adds them, so the fallback
// needs no read of its own; CHECK = 1 when the sort has no fallback, see SplitWs).
constexpr uint32_t kHalfT = 1u << 15;   // a 16-bit LDS half is brought back under this
constexpr uint32_t kEvMax = 4096;       // crossings logged per workgroup: chunk / kHalfT at most, so any
                                        // chunk of up to 2^27 keys (n < 2^32 over >= 32 workgroups)
constexpr uint32_t kRowEv = 32768;      // a row (65536 words): 32768 packed count pairs, then the
                                        // crossing log (count, buckets)
template <int L, bool AOS_WIDE = false, bool FULL = false, int CHECK = 0>
__global__ __launch_bounds__(1024) void k_hist16_in(const uint32_t* __restrict__ keys, uint32_t n,
                                                     uint32_t* __restrict__ rows, uint32_t kbase,
                                                     uint32_t range, uint32_t shift,
                                                     uint32_t* __restrict__ z0, uint32_t* __restrict__ z1,
                                                     uint32_t* inv = nullptr, uint32_t* __restrict__ b0rows = nullptr,
                                                     uint32_t* __restrict__ z2 = nullptr,
                                                     const uint32_t* skip = nullptr) {
    // z2 (may be null): the bucket split's huge-bucket count (SplitWs::huge[0])
    // skip (may be null): *skip != 0 - the presorted path has sorted the data (rs_presorted.hpp):
    // nothing is read, the order check stays "in order"
    static_assert(!CHECK || FULL, "the order check rides on whole-range histograms only");
    constexpr bool B0 = CHECK == 2;   // the byte-0 counts too (the LSD fallback's pass-0 totals)
    // z0, z1: the reduction's overflow-bucket count and oversize flag (k_hist16_reduce adds to them)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *z0 = 0u;
        *z1 = 0u;
        if (z2) *z2 = 0u;
    }
    if (skip && *skip) return;
    constexpr uint32_t B = 1024, W = 32768, PER = W / B;
    constexpr bool NARROW = L == LAYOUT_AOS && !AOS_WIDE;
    constexpr uint32_t KPL = NARROW ? 1u : (L == LAYOUT_AOS ? 2u : 4u);   // keys per load
    // loads per thread per group; two groups in flight (the next one issued before this one is counted)
#if !RS_KNOB_OPEN || !defined(RS_H16_FLY)
#undef RS_H16_FLY
#define RS_H16_FLY 3
#endif
    constexpr uint32_t FLY = CHECK ? 3 : RS_H16_FLY;
    using Vec = typename std::conditional<NARROW, uint2, uint4>::type;
    __shared__ __attribute__((aligned(16))) uint32_t h[W];
    __shared__ uint32_t s_b0[B0 ? 256 : 1];
    __shared__ uint32_t s_ev[kEvMax];
    __shared__ uint32_t s_nev;
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) h[tid + B * i] = 0u;
    if (B0 && tid < 256u) s_b0[tid] = 0u;
    if (tid == 0) s_nev = 0u;
    constexpr uint32_t KS = L == LAYOUT_AOS ? 2u : 1u;   // words per key
    bool inverted = false;
    auto inv2 = [&](uint32_t a, uint32_t b) { inverted |= a > b; };
    // 64-bit: n + gridDim.x - 1 wraps in 32 bits for n > 2^32 - gridDim.x (chunk would be 0 and
    // every row would count nothing)
    const uint64_t chunk = (((uint64_t)n + gridDim.x - 1) / gridDim.x + 3u) & ~3ull;
    const uint64_t lo = (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = lo + chunk < n ? lo + chunk : (lo < n ? n : lo);
    const uint64_t nv = (hi - lo) / KPL;                          // whole vectors
    const Vec* v4 = reinterpret_cast<const Vec*>(keys + (L == LAYOUT_AOS ? 2 : 1) * lo);
    bool bad = false;
    // c added to bucket b's half; a crossing of kHalfT is taken back and logged (see above)
    auto take_back = [&](uint32_t b, uint32_t old, uint32_t c) {
        const uint32_t sh = (b & 1u) << 4;
        const uint32_t o = (old >> sh) & 0xFFFFu;
        if (o < kHalfT && o + c >= kHalfT) {
            atomicSub(&h[b >> 1], kHalfT << sh);
            const uint32_t e = atomicAdd(&s_nev, 1u);
            if (e < kEvMax) s_ev[e] = b;
        }
    };
    auto add16 = [&](uint32_t b, uint32_t c) {
        take_back(b, atomicAdd(&h[b >> 1], c << ((b & 1u) << 4)), c);
    };
    // m buckets + 1 each: every add issued before the first is checked (one LDS round trip, not m)
    auto add16n = [&](const uint32_t (&bs)[4], int m) {
        uint32_t old[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < m) old[j] = atomicAdd(&h[bs[j] >> 1], 1u << ((bs[j] & 1u) << 4));
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < m) take_back(bs[j], old[j], 1u);
    };
    // FULL, one load's keys (1, 2 or 4): sorted or duplicate-heavy input puts a whole wave's keys in
    // one 16-bit bucket (and, check_order, one low byte: config 4's small floats have few mantissa
    // bits, so a whole chunk has low byte 0), and 64 lanes adding to one LDS address serialise
    // (config 4: the slowest chunks' workgroups set the kernel at 1.0 ms instead of 0.3), so lanes
    // whose keys share a counter are grouped by counter, one add per group: up to two groups per
    // wave (a sorted run, or a run crossing one counter edge, with a few displaced keys); random keys
    // almost never share a counter within one load, and cost one ballot per counter array here
    auto grouped = [&](uint32_t c, bool uni, uint32_t m, auto&& add) {
        uint64_t left = __ballot(uni);
        bool done = false;
        for (int r = 0; r < 2 && left; ++r) {
            const int lead = __builtin_ctzll(left);
            const uint32_t cl = __builtin_amdgcn_readlane(c, lead);
            const bool mine = uni && c == cl;
            const uint64_t grp = __ballot(mine);
            if (mine && mbcnt(grp) == 0) add(cl, m * (uint32_t)__popcll(grp));
            done |= mine;
            left &= ~grp;
        }
        if (!done && uni) add(c, m);
        return done || uni;
    };
    // (ok: the lane's vector lies in the chunk; only the adds are predicated on it, so that the
    // loaded registers are used - waited for - on every path)
    auto count_load = [&](const uint32_t (&ks)[4], int m, bool ok) {
        const uint32_t b = ks[0] >> 16;
        bool uni = ok;
        for (int j = 1; j < m; ++j) uni &= (ks[j] >> 16) == b;
        if (!grouped(b, uni, (uint32_t)m, add16) && ok) {
            const uint32_t bs[4] = {ks[0] >> 16, ks[1] >> 16, ks[2] >> 16, ks[3] >> 16};
            add16n(bs, m);
        }
        if constexpr (B0) {
            const uint32_t d = ks[0] & 255u;
            bool uni0 = ok;
            for (int j = 1; j < m; ++j) uni0 &= (ks[j] & 255u) == d;
            auto add0 = [&](uint32_t x, uint32_t c) { atomicAdd(&s_b0[x], c); };
            if (!grouped(d, uni0, (uint32_t)m, add0) && ok)
                for (int j = 0; j < m; ++j) add0(ks[j] & 255u, 1u);
        }
    };
    auto count = [&](uint32_t key, bool ok) {
        if constexpr (FULL) {
            const uint32_t b = key >> 16;
            if (ok) add16(b, 1u);
            if constexpr (B0) if (ok) atomicAdd(&s_b0[key & 255u], 1u);
        } else {
            const uint32_t rk = key - kbase;
            bad |= ok && rk > range;
            const uint32_t b = (rk >> shift) & 0xFFFFu;
            if (ok) add16(b, 1u);
        }
    };
    // branch-free loads (a vector past nv loads vector nv - 1 and is not counted): with a branch per
    // load the compiler waited for every load in flight before each one, and before counting
    auto load_group = [&](uint64_t g0, Vec (&q)[FLY]) {
#pragma unroll
        for (uint32_t u = 0; u < FLY; ++u) {
            const uint64_t i = g0 + (uint64_t)u * B + tid;
            q[u] = v4[i < nv ? i : nv - 1];
        }
    };
    auto count_group = [&](uint64_t g0, const Vec (&q)[FLY]) {
        if constexpr (FULL && !NARROW && !CHECK && RS_H16_BATCH) {
            // (whole-range counts, no order check) a group in which no lane holds a load whose keys
            // share one bucket - random keys: every group - issues all of its adds first and checks
            // the returned halves for a crossing after: the adds' LDS round trips overlap instead
            // of one per load (per-load grouping below otherwise)
            constexpr int M = L == LAYOUT_AOS ? 2 : 4;
            bool uni_any = false;
#pragma unroll
            for (uint32_t u = 0; u < FLY; ++u) {
                const uint32_t ks[4] = {q[u].x, L == LAYOUT_AOS ? q[u].z : q[u].y, q[u].z, q[u].w};
                bool uni = true;
#pragma unroll
                for (int j = 1; j < M; ++j) uni &= (ks[j] >> 16) == (ks[0] >> 16);
                uni_any |= uni && g0 + (uint64_t)u * B + tid < nv;
            }
            if (__ballot(uni_any) == 0ull) {
                uint32_t old[FLY * M];
#pragma unroll
                for (uint32_t u = 0; u < FLY; ++u) {
                    const uint32_t ks[4] = {q[u].x, L == LAYOUT_AOS ? q[u].z : q[u].y, q[u].z, q[u].w};
                    const bool ok = g0 + (uint64_t)u * B + tid < nv;
#pragma unroll
                    for (int j = 0; j < M; ++j) {
                        const uint32_t b = ks[j] >> 16;
                        old[u * M + j] = ok ? atomicAdd(&h[b >> 1], 1u << ((b & 1u) << 4)) : 0u;
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < FLY; ++u) {
                    const uint32_t ks[4] = {q[u].x, L == LAYOUT_AOS ? q[u].z : q[u].y, q[u].z, q[u].w};
                    const bool ok = g0 + (uint64_t)u * B + tid < nv;
#pragma unroll
                    for (int j = 0; j < M; ++j)
                        if (ok) take_back(ks[j] >> 16, old[u * M + j], 1u);
                }
                return;
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < FLY; ++u) {
            const uint64_t i = g0 + (uint64_t)u * B + tid;
            uint32_t nxt = 0;
            if constexpr (CHECK) {
                // the first key of vector i + 1: the next lane's (DPP wave_shl:1, in uniform
                // control flow), or loaded where that lane has none (lane 63, the chunk's last
                // vector: then the key after the vectors, which may be the next chunk's)
                nxt = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q[u].x, 0x130, 0xf, 0xf, false);
                if (i < nv && (lane_id() == 63 || i + 1 >= nv)) {
                    const uint64_t j = lo + KPL * (i + 1);
                    nxt = j < n ? keys[KS * j] : 0xFFFFFFFFu;
                }
            }
            const bool ok = i < nv;
            if constexpr (FULL) {
                if constexpr (NARROW) { const uint32_t ks[4] = {q[u].x, 0u, 0u, 0u}; count_load(ks, 1, ok); }
                else if constexpr (L == LAYOUT_AOS) { const uint32_t ks[4] = {q[u].x, q[u].z, 0u, 0u}; count_load(ks, 2, ok); }
                else { const uint32_t ks[4] = {q[u].x, q[u].y, q[u].z, q[u].w}; count_load(ks, 4, ok); }
            }
            else if constexpr (NARROW) { count(q[u].x, ok); }
            else {   // the range form: every key's bucket, then the adds issued together
                constexpr int m = L == LAYOUT_AOS ? 2 : 4;
                const uint32_t ks[4] = {q[u].x, L == LAYOUT_AOS ? q[u].z : q[u].y, q[u].z, q[u].w};
                uint32_t bs[4];
#pragma unroll
                for (int j = 0; j < m; ++j) {
                    const uint32_t rk = ks[j] - kbase;
                    bad |= ok && rk > range;
                    bs[j] = (rk >> shift) & 0xFFFFu;
                }
                if (ok) add16n(bs, m);
            }
            if constexpr (CHECK) {
                if (ok) {
                    if constexpr (NARROW) { inv2(q[u].x, nxt); }
                    else if constexpr (L == LAYOUT_AOS) { inv2(q[u].x, q[u].z); inv2(q[u].z, nxt); }
                    else { inv2(q[u].x, q[u].y); inv2(q[u].y, q[u].z); inv2(q[u].z, q[u].w); inv2(q[u].w, nxt); }
                }
            }
        }
    };
    __syncthreads();
    constexpr uint64_t GS = (uint64_t)FLY * B;   // vectors per group
    if (nv) {
        // two groups per iteration, so that the registers of the group in flight are named statically;
        // the next group is loaded unconditionally (past the end: vector nv - 1 again, uncounted), so
        // that every path into the counting has the same loads outstanding (the compiler's wait for
        // the group being counted is otherwise the one of the path with fewer loads: all of them)
        // (the loop's only exit is its uniform test at the end, for the same reason)
        Vec qa[FLY], qb[FLY];
        load_group(0, qa);
        uint64_t g = 0;
        for (; g + 2 * GS < nv; g += 2 * GS) {   // a group follows the pair
            load_group(g + GS, qb);
            count_group(g, qa);
            load_group(g + 2 * GS, qa);
            count_group(g + GS, qb);
        }
        load_group(g + GS, qb);                  // the last one or two groups
        count_group(g, qa);
        count_group(g + GS, qb);
    }
    // the last (hi - lo) % KPL keys of the chunk
    const uint64_t rest = lo + nv * KPL;
    if (rest + tid < hi) {
        const uint32_t key = keys[KS * (rest + tid)];
        count(key, true);
        if (CHECK && rest + tid + 1 < n) inv2(key, keys[KS * (rest + tid + 1)]);
    }
    __syncthreads();
    if constexpr (CHECK) {
        if (__ballot(inverted) != 0ull && lane_id() == 0) atomicOr(inv, 1u);
        if (B0 && tid < 256u) b0rows[(size_t)blockIdx.x * 256u + tid] = s_b0[tid];
    }
    // the row as counted: the packed halves (half the bytes of 32-bit counts to write here and to read
    // in the reduction), then the logged crossings (kRowEv: their count, then the buckets, each worth
    // kHalfT more; the reduction adds them)
    uint32_t* row = rows + (size_t)blockIdx.x * 65536u;
#pragma unroll
    for (uint32_t i = 0; i < PER / 4; ++i)
        reinterpret_cast<uint4*>(row)[tid + B * i] = reinterpret_cast<const uint4*>(h)[tid + B * i];
    const uint32_t nev = s_nev;   // uniform (read after the barrier above)
    if (nev > kEvMax) bad = true;   // (never: the hosts launch chunks of <= 2^27 keys) -> flagged
    const uint32_t ne = nev < kEvMax ? nev : kEvMax;
    if (tid == 0) row[kRowEv] = ne;
    for (uint32_t e = tid; e < ne; e += B) row[kRowEv + 1u + e] = s_ev[e];
    const int any_bad = __syncthreads_or(bad ? 1 : 0);
    if (tid == 0) rows[(size_t)gridDim.x * 65536u + blockIdx.x] = any_bad ? 1u : 0u;
}

// hist16 = the sum of nrows rows of 65536 counts; top_tot[t] = the sum of hist16[t << 8 ..] (the
// top-byte digit totals).  One workgroup per top byte: 64 columns of 4 buckets x 16 row groups
// (nrows <= 1024).
// Workgroup t also lays out its top byte's 256 buckets (the plan work that needs every bucket):
// base16[b] = the bucket's start inside its top-byte segment (consumers add the segment start,
// segtab[257 + (b >> 8)]), buckets over `small` appended to over[1..] (over[0] counts them, up to
// kOverMax stored), *big |= a bucket over `cap`.
// cbase (may be null): cbase[r * 256 + t] = the keys with top byte t in the chunks of the rows
// before row r (an exclusive scan over the rows of each top byte's row sums): where chunk r's
// top-byte-t keys start inside segment t.  The static first MSD pass (k_static_pass) takes its
// per-digit output bases from it, so it needs no look-back.
constexpr uint32_t kOverMax = 65536;   // every bucket can be listed (no overflow to the fallback)
constexpr uint32_t kMaxRows = 1024;
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// PACKED: k_hist16_in's rows (packed halves + crossing log, kRowEv); else rows of 65536 32-bit counts
// (a multi-GPU region's table, k_region_rows).
template <bool PACKED>
__global__ __launch_bounds__(1024) void k_hist16_reduce(const uint32_t* __restrict__ rows, uint32_t nrows,
                                                         uint32_t* __restrict__ hist16,
                                                         uint32_t* __restrict__ top_tot,
                                                         uint32_t* __restrict__ range_bad,
                                                         uint32_t* __restrict__ base16, uint32_t small,
                                                         uint32_t cap, uint32_t* __restrict__ over,
                                                         uint32_t* __restrict__ big,
                                                         uint32_t* __restrict__ zero = nullptr, uint32_t nzero = 0,
                                                         const uint32_t* __restrict__ b0rows = nullptr,
                                                         uint32_t* __restrict__ cbase = nullptr,
                                                         uint32_t* __restrict__ huge = nullptr, uint32_t hmax = 0,
                                                         const uint32_t* skip = nullptr) {
    // huge (may be null): buckets over `cap` are listed in huge[1..] (huge[0] counts them, up to hmax
    // stored; zeroed with over[0]) for the bucket split instead of flagging *big
    // zero[0..nzero): the sort's pass totals, tile tickets and device error word (no memset launch);
    // with b0rows (check_order): zero[0..256) = pass 0's byte-0 totals, the rows' sums
    // skip (may be null): *skip != 0 - the presorted path sorted the data and k_hist16_in wrote no
    // rows: only the zeroing (k_msd_plan then gates every launch off on the order check)
    const bool skipped = skip && *skip;
    if (blockIdx.x == gridDim.x - 1) {
        for (uint32_t i = threadIdx.x; i < nzero; i += blockDim.x) zero[i] = 0u;
        if (b0rows && !skipped && threadIdx.x < 256u) {   // the same thread zeroed zero[threadIdx.x] above
            uint32_t c = 0;
            for (uint32_t r = 0; r < nrows; ++r) c += b0rows[(size_t)r * 256u + threadIdx.x];
            zero[threadIdx.x] = c;
        }
    }
    if (skipped) return;
    __shared__ uint4 s_part[16][64];
    __shared__ uint32_t s_rowsum[kMaxRows];
    __shared__ uint32_t s_scan[16];
    const uint32_t tid = threadIdx.x, c = tid & 63u, g = tid >> 6;
    if (blockIdx.x == 0) {   // any key outside the range (the rows' flag words)
        const int bad = __syncthreads_or(tid < nrows && rows[(size_t)nrows * 65536u + tid] != 0u);
        if (tid == 0) *range_bad = bad ? 1u : 0u;
    }
    // lane c: buckets 4c .. 4c + 3 of this top byte (PACKED: two packed words)
    const uint4* r4 = reinterpret_cast<const uint4*>(rows) + (size_t)blockIdx.x * 64u + c;
    const uint2* r2 = reinterpret_cast<const uint2*>(rows) + (size_t)blockIdx.x * 64u + c;
    constexpr size_t RS = PACKED ? 65536 / 2 : 65536 / 4;    // row stride in 8- / 16-byte words
    auto ld = [&](uint32_t row) -> uint4 {
        if constexpr (PACKED) {
            const uint2 x = r2[row * RS];
            return make_uint4(x.x & 0xFFFFu, x.x >> 16, x.y & 0xFFFFu, x.y >> 16);
        } else {
            return r4[row * RS];
        }
    };
    __shared__ uint32_t s_extra[PACKED ? 256 : 1];
    uint4 a = make_uint4(0u, 0u, 0u, 0u);
    auto add = [](uint4& x, const uint4 y) { x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w; };
    // wave g holds one row's 256 buckets of this top byte at a time: their sum is the row's
    // (chunk's) count of the top byte
    auto rowsum = [&](uint32_t row, const uint4 q) {
        if (cbase) {
            const uint32_t s = wave_sum(q.x + q.y + q.z + q.w);
            if (c == 0) s_rowsum[row] = s;
        }
    };
    uint32_t r = g;
    for (; r + 48u < nrows; r += 64u) {
        const uint4 q0 = ld(r), q1 = ld(r + 16u), q2 = ld(r + 32u), q3 = ld(r + 48u);
        add(a, q0); add(a, q1); add(a, q2); add(a, q3);
        rowsum(r, q0); rowsum(r + 16u, q1); rowsum(r + 32u, q2); rowsum(r + 48u, q3);
    }
    for (; r < nrows; r += 16u) {
        const uint4 q = ld(r);
        add(a, q);
        rowsum(r, q);
    }
    s_part[g][c] = a;
    if constexpr (PACKED) {
        // the rows' logged crossings of this top byte: kHalfT more each (uniform keys: none)
        if (tid < 256u) s_extra[tid] = 0u;
        __syncthreads();
        if (tid < nrows) {
            const uint32_t* ev = rows + (size_t)tid * 65536u + kRowEv;
            const uint32_t ne = ev[0];
            for (uint32_t e = 0; e < ne; ++e) {
                const uint32_t b = ev[1u + e];
                if ((b >> 8) == blockIdx.x) {
                    atomicAdd(&s_extra[b & 255u], kHalfT);
                    if (cbase) s_rowsum[tid] += kHalfT;
                }
            }
        }
    }
    __syncthreads();
    if (cbase) {   // exclusive scan of the row sums (uniform branch: every thread takes part)
        uint32_t tot;
        const uint32_t ex = block_excl_scan_n<16>(tid < nrows ? s_rowsum[tid] : 0u, s_scan, tot);
        if (tid < nrows) cbase[(size_t)tid * 256u + blockIdx.x] = ex;
    }
    if (tid < 64u) {
        uint4 t = s_part[0][tid];
#pragma unroll
        for (int j = 1; j < 16; ++j) add(t, s_part[j][tid]);
        if constexpr (PACKED)
            add(t, make_uint4(s_extra[4u * tid], s_extra[4u * tid + 1u], s_extra[4u * tid + 2u], s_extra[4u * tid + 3u]));
        reinterpret_cast<uint4*>(hist16)[blockIdx.x * 64u + tid] = t;
        const uint32_t s4 = t.x + t.y + t.z + t.w;
        const uint32_t inc = wave_incl_scan(s4);
        const uint32_t ex = inc - s4;
        reinterpret_cast<uint4*>(base16)[blockIdx.x * 64u + tid] =
            make_uint4(ex, ex + t.x, ex + t.x + t.y, ex + t.x + t.y + t.z);
        if (tid == 63) top_tot[blockIdx.x] = inc;
        const uint32_t mx = max(max(t.x, t.y), max(t.z, t.w));
        if (mx > cap && !huge) atomicOr(big, 1u);
        if (mx > small) {
            const uint32_t c4[4] = {t.x, t.y, t.z, t.w};
            for (uint32_t j = 0; j < 4u; ++j) {
                const uint32_t b = blockIdx.x * 256u + tid * 4u + j;
                if (huge && c4[j] > cap) {   // split by the bucket split (k_msd_plan's level 2)
                    const uint32_t slot = atomicAdd(&huge[0], 1u);
                    if (slot < hmax) huge[1 + slot] = b;
                    else atomicOr(big, 1u);
                } else if (c4[j] > small) {
                    const uint32_t slot = atomicAdd(&over[0], 1u);
                    if (slot < kOverMax) over[1 + slot] = b;
                }
            }
        }
    }
}

// out[0..65536) = the sum of nrows rows of 65536 counts (k_hist16_in's rows), out[65536 + t] = the
// sum of out[t << 8 ..]: the multi-GPU sender's table (rs_plan_hist16).  Workgroup t: top byte t.
__global__ __launch_bounds__(256) void k_hist16_sum(const uint32_t* __restrict__ rows, uint32_t nrows,
                                                    uint32_t* __restrict__ out) {
    __shared__ uint32_t s_scratch[kWaves];
    const uint32_t b = blockIdx.x * 256u + threadIdx.x;
    uint32_t c = 0;
    // the packed halves (independent loads, unrolled), then the logged crossings of the rows that
    // have any (k_hist16_in; uniform keys: none)
#pragma unroll 8
    for (uint32_t r = 0; r < nrows; ++r)
        c += (rows[(size_t)r * 65536u + (b >> 1)] >> ((b & 1u) << 4)) & 0xFFFFu;
    for (uint32_t r0 = 0; r0 < nrows; r0 += 256u) {
        const uint32_t r = r0 + threadIdx.x;
        const bool any = __syncthreads_or(r < nrows && rows[(size_t)r * 65536u + kRowEv] != 0u);
        if (!any) continue;   // (uniform)
        for (uint32_t q = r0; q < nrows && q < r0 + 256u; ++q) {
            const uint32_t* ev = rows + (size_t)q * 65536u + kRowEv;
            const uint32_t ne = ev[0];
            for (uint32_t e = 0; e < ne; ++e) c += ev[1u + e] == b ? kHalfT : 0u;
        }
    }
    out[b] = c;
    uint32_t tot;
    block_excl_scan(c, s_scratch, tot);
    if (threadIdx.x == 0) out[65536u + blockIdx.x] = tot;
}

// A multi-GPU receiver's region (rs_plan_sort_region): its 16-bit bucket counts arrive from the
// senders' tables, so instead of k_hist16_in's rows there is one row, copied here, with a clear
// range flag word; also clears the overflow count and the oversize flag (k_hist16_in's job).
__global__ __launch_bounds__(256) void k_region_rows(const uint32_t* __restrict__ hist, uint32_t* __restrict__ row,
                                                     uint32_t* z0, uint32_t* z1, uint32_t* z2 = nullptr) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    row[i] = hist[i];
    if (i == 0) {
        row[65536] = 0u;
        *z0 = 0u;
        *z1 = 0u;
        if (z2) *z2 = 0u;
    }
}

// One workgroup, after k_hist16_reduce: the segmented tile table of MSD pass 1 (segment = top
// byte: [257] first tile + total, [256] start, [256] end; the starts are what the bucket bases of
// k_hist16_reduce are relative to) and the path: MSD iff every 16-bit bucket fits the bucket tile
// (*big == 0), at most kOverMax buckets need the large tile, every top-byte bucket holds at most
// max_top keys and no key lies outside the range; else the LSD passes on the input.  over[0] is
// clamped to the stored entries.
// The histogram must account for every one of the n keys (a counting bug would otherwise send the
// data through passes with wrong digit bases and return garbage): a mismatch picks the LSD passes.
// The second MSD pass runs over a static split (k_static_pass: one workgroup per top-byte segment,
// no look-back) when the segments are balanced - none over the mean by more than 1/16 plus a tile
// - else with the look-back (k_onesweep SEG): gates g[32..47] / g[48..63], each ANDed with the MSD
// choice.  The populated buckets must lie in the top bytes [top_lo, top_hi) (a region's
// table; counts outside them would never be sorted): otherwise the LSD passes run.
constexpr uint32_t kGateSegStatic = 32, kGateSegLookback = 48;

// The bucket split's workspace (see "splitting over-full buckets" below); huge == null: no split
// (a bucket over the cap then sends the sort to the LSD fallback).
struct SplitWs {
    uint32_t* gate2 = nullptr;       // [16] level 2 runs (k_msd_plan)
    uint32_t* gate3 = nullptr;       // [16] level 3 runs (set by level 2's counting)
    uint32_t* huge = nullptr;        // [1 + smax2] count, then the buckets over the cap (k_hist16_reduce)
    uint32_t* tab2 = nullptr;        // level 2's split table (its segments: the huge buckets)
    uint32_t* rows2 = nullptr;       // [smax2][256] byte-1 counts -> absolute sub-bucket starts
    uint32_t* arrive2 = nullptr;     // [smax2 + 1]
    uint32_t smax2 = 0;
    uint32_t* tab3 = nullptr;        // level 3's (its segments: the sub-buckets over kSub8Cap)
    uint32_t* rows3 = nullptr;
    uint32_t* arrive3 = nullptr;
    uint32_t smax3 = 0;
    uint32_t tmax = 0;               // tiles one level may have (the plan's look-back status words)
    const uint32_t* hist16 = nullptr;
    const uint32_t* base16 = nullptr;
    uint32_t* err = nullptr;         // the sort's device error word ...
    uint32_t* host_err = nullptr;    // ... and the host-mapped one (bit 2: counts did not add up)
    uint32_t strict = 0;             // no LSD fallback is enqueued: a failed plan check is an error
    uint32_t n = 0;                  // the sort's record count: every table position is clamped to it
    uint32_t* mid = nullptr;         // [1 + midmax] count, then the sub-buckets for the large tile
    uint32_t midmax = 0;
    uint32_t* chunks = nullptr;      // [1 + 2 chunkmax] count, then (start, count) of the runs of
    uint32_t chunkmax = 0;           // consecutive small sub-buckets sorted together
};

__device__ __forceinline__ void split_fail(const SplitWs& sw) {
    atomicOr(sw.err, 4u);
    if (sw.host_err) __hip_atomic_fetch_or(sw.host_err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr uint32_t kSplitTile = 16384;          // k_onesweep's tile (tiles never straddle a segment)

// Lays out one split level's table from its segments (segment i: `cnt` records from `start`, both
// from seg_range): tiles per segment scanned into first tiles, rows and arrivals zeroed.  One
// workgroup of BLOCK threads; nseg <= smax.  More than tmax tiles (never, by the plan's sizing):
// an error and an empty level.  Returns the level's segment count.
template <int BLOCK, class F>
__device__ uint32_t split_layout(uint32_t nseg, uint32_t smax, uint32_t* tab, uint32_t* rows, uint32_t* arrive,
                                 const SplitWs& sw, F&& seg_range) {
    constexpr int NW = BLOCK / 64;
    __shared__ uint32_t s_scr[NW];
    const uint32_t tid = threadIdx.x;
    // contiguous chunks of segments per thread: local tile sums, one block scan, then the firsts
    const uint32_t per = (nseg + BLOCK - 1) / BLOCK;
    const uint32_t a = tid * per < nseg ? tid * per : nseg;
    const uint32_t b = a + per < nseg ? a + per : nseg;
    uint32_t sum = 0;
    for (uint32_t i = a; i < b; ++i) {
        uint32_t st, c;
        seg_range(i, st, c);
        sum += (c + kSplitTile - 1) / kSplitTile;
    }
    uint32_t tot;
    uint32_t run = block_excl_scan_n<NW>(sum, s_scr, tot);
    if (tot > sw.tmax) {
        if (tid == 0) {
            tab[0] = 0u;
            tab[1] = 0u;
            split_fail(sw);
        }
        return 0u;
    }
    for (uint32_t i = a; i < b; ++i) {
        uint32_t st, c;
        seg_range(i, st, c);
        tab[1 + i] = run;
        tab[2 + smax + i] = st;
        tab[2 + 2 * smax + i] = st + c;
        run += (c + kSplitTile - 1) / kSplitTile;
    }
    if (tid == 0) {
        tab[0] = nseg;
        tab[1 + nseg] = tot;
        arrive[smax] = 0u;
    }
    for (uint32_t i = tid; i < nseg; i += BLOCK) arrive[i] = 0u;
    for (uint32_t i = tid; i < nseg * 256u; i += BLOCK) rows[i] = 0u;
    return nseg;
}

// sw.huge != null: also the bucket split's level 2 - the huge buckets' table from the list
// k_hist16_reduce made, its rows zeroed, gate2 set when there is any, gate3 cleared (level 2's
// counting sets it).  sw.strict (whole-range sorts with the split: no LSD fallback enqueued): a
// failed check - a histogram that does not add up to n - is a device error instead.
template <int TILE>
__global__ __launch_bounds__(256) void k_msd_plan(const uint32_t* __restrict__ top_tot,
                                                  uint32_t* __restrict__ segtab, uint32_t max_top,
                                                  uint32_t* over, const uint32_t* big, uint32_t* gates,
                                                  const uint32_t* __restrict__ range_bad, uint32_t n,
                                                  const uint32_t* inv = nullptr, uint32_t top_lo = 0,
                                                  uint32_t top_hi = 256, SplitWs sw = SplitWs{}) {
    constexpr int NW = 4;
    __shared__ uint32_t s_scratch[NW];
    __shared__ uint32_t s_sstart[256];
    const uint32_t tid = threadIdx.x;
    const uint32_t cnt = top_tot[tid];
    const int any_big = __syncthreads_or((cnt > max_top || (cnt != 0u && (tid < top_lo || tid >= top_hi))) ? 1 : 0);
    const uint32_t seg_cap = n / 256u + n / 4096u + (uint32_t)TILE;
    const int unbalanced = __syncthreads_or(cnt > seg_cap ? 1 : 0);
    const uint32_t tiles = (cnt + TILE - 1) / TILE;
    uint32_t ttot;
    const uint32_t tbase = block_excl_scan_n<NW>(tiles, s_scratch, ttot);
    uint32_t stot;
    const uint32_t sbase = block_excl_scan_n<NW>(cnt, s_scratch, stot);
    segtab[tid] = tbase;
    segtab[257 + tid] = sbase;
    segtab[513 + tid] = sbase + cnt;
    s_sstart[tid] = sbase;
    if (tid == 0) segtab[256] = ttot;
    const uint32_t nover = over[0];
    const uint32_t nhuge = sw.huge ? sw.huge[0] : 0u;
    __syncthreads();   // every thread has read over[0]
    if (tid == 0) over[0] = nover < kOverMax ? nover : kOverMax;
    const uint32_t ok = (any_big || *big || nover > kOverMax || *range_bad || stot != n || nhuge > sw.smax2)
                            ? 0u : 1u;
    // check_order: an input already in order needs neither path (the reference's early exit,
    // CheckSort.ts:138-145: every later dispatch zeroed)
    const uint32_t run = (inv && *inv == 0u) ? 0u : 1u;
    set_gate(gates + kGateMsd, ok & run);
    set_gate(gates + kGateLsd, (1u - ok) & run);
    set_gate(gates + kGateSegStatic, ok & run & (unbalanced ? 0u : 1u));
    set_gate(gates + kGateSegLookback, ok & run & (unbalanced ? 1u : 0u));
    if (sw.strict && run && !ok && tid == 0) split_fail(sw);
    if (sw.huge) {
        set_gate(sw.gate3, 0u);
        if (tid == 0) {
            sw.tab3[0] = 0u;
            sw.mid[0] = 0u;
            sw.chunks[0] = 0u;
        }
        uint32_t n2 = 0;
        if (ok & run & (nhuge ? 1u : 0u))   // uniform
            n2 = split_layout<256>(nhuge, sw.smax2, sw.tab2, sw.rows2, sw.arrive2, sw,
                                   [&](uint32_t i, uint32_t& st, uint32_t& c) {
                                       const uint32_t b = sw.huge[1 + i];
                                       st = s_sstart[b >> 8] + sw.base16[b];
                                       c = sw.hist16[b];
                                   });
        set_gate(sw.gate2, n2 ? 1u : 0u);
    }
}

// ---- splitting over-full buckets (skewed keys on the hybrid path) ---------------------------
// A 16-bit bucket over kBucketCap records (f32 keys in [0, 1): half of them share 128 buckets of
// ~1M records; few distinct keys; one populated bucket) is split instead of sending the whole sort
// to the LSD passes.  Level 2: k_split_count counts byte 1 of the huge buckets' records (per bucket:
// the workgroups whose tile ranges meet it add their counts to its row, the last one turns the row
// into absolute sub-bucket starts), a segmented one-sweep pass (k_onesweep SEG = 2) partitions them
// by byte 1 from R2 into a free records buffer R3, and k_bucket_sort8 sorts every 24-bit sub-bucket
// by byte 0 in LDS into the output.  A sub-bucket over kSub8Cap records goes to level 3: the same
// count and segmented pass by byte 0, R3 -> output (its keys then differ in no other bit).  Every
// step is stable, so the result is the stable sort.  Bytes per record of a huge bucket after MSD
// passes 0 and 1: count 8 + pass 16 + bucket sort 16 (level 3: + 8 + 16).  (Round 4 also tried
// level 2 as an in-LDS sort of every 16K-record tile plus a sub-bucket sort that gathered its
// pieces from the tiles: no count and no look-back, but the gather's dependent table reads made the
// sub-bucket sort 3.5 ms for config 4 - DESIGN.md section 12.)
//
// Split table (per level): [0] segment count, [1 .. smax + 1] first tile of every segment (+ the
// total), [smax + 2 ..] segment starts, [2 smax + 2 ..] segment ends (positions in the records
// buffers).  rows: [smax][256] digit counts, turned into absolute bases in place.  arrive: [smax]
// per-segment tile arrivals + [1] segments done (zeroed by the level's layout).
constexpr uint32_t kSub8Small = 256u * 17u;     // k_bucket_sort8's small tile (4352 records)
constexpr uint32_t kSub8Cap = 1024u * 17u;      // its large tile (17408): larger sub-buckets -> level 3
__device__ __forceinline__ uint32_t split_seg_of(const uint32_t* first, uint32_t nseg, uint32_t t) {
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (first[mid] <= t) lo = mid;
        else hi = mid;
    }
    return lo;
}

// One split level's digit counts and bases (see above).  KS = words per record in `rec` (2:
// (key, value) records, 1: keys); digit = (key >> shift) & 255.  LEVEL 2 (tab = sw.tab2 ...) also
// lists and lays out level 3; LEVEL 3 (tab = sw.tab3 ...) only counts.  A list overflow or a count
// that does not add up is an error (bit 2): never a silent wrong order.
// Workgroup g takes the contiguous tiles [g per, (g + 1) per) of the level (a grid-stride split
// made every tile pay a binary search, an arrival round trip and an unhidden load: 1.5 ms for 2^28
// records): the next tile's keys are loaded while this one is counted, the counts of a segment
// accumulate in LDS over the workgroup's tiles of it, and the workgroup adds them to the segment's
// row once, when its range leaves the segment; the segment's arrivals are then the workgroups whose
// ranges meet it, and the last of them scans the row.
template <int KS, int LEVEL>
__global__ __launch_bounds__(1024, 8) void k_split_count(const uint32_t* __restrict__ rec, SplitWs sw,
                                                      uint32_t shift) {
    constexpr uint32_t B = 1024, NW = B / 64;
    constexpr uint32_t HALF = kSplitTile / 2;   // a table tile is counted in two halves: 8 keys per
    constexpr int KPT = HALF / B;               // thread + 8 in flight fit 64 VGPRs (two workgroups per CU)
    __shared__ uint32_t s_h[NW][256];
    __shared__ uint32_t s_scr[NW];
    __shared__ uint32_t s_flag;
    __shared__ uint32_t s_c[LEVEL == 2 ? 256 : 1];
    __shared__ uint32_t s_cs[LEVEL == 2 ? 256 : 1], s_cn[LEVEL == 2 ? 256 : 1], s_md[LEVEL == 2 ? 256 : 1];
    __shared__ uint32_t s_nl[4];
    const uint32_t* gate = LEVEL == 2 ? sw.gate2 : sw.gate3;
    if (gated_off(gate, 0)) return;
    uint32_t* tab = LEVEL == 2 ? sw.tab2 : sw.tab3;
    uint32_t* rows = LEVEL == 2 ? sw.rows2 : sw.rows3;
    uint32_t* arrive = LEVEL == 2 ? sw.arrive2 : sw.arrive3;
    const uint32_t smax = LEVEL == 2 ? sw.smax2 : sw.smax3;
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t nseg = tab[0];
    const uint32_t* first = tab + 1;
    const uint32_t* start = tab + 2 + smax;
    const uint32_t* end = tab + 2 + 2 * smax;
    const uint32_t ntiles = first[nseg];
    const uint32_t per = (ntiles + gridDim.x - 1) / gridDim.x;
    const uint32_t t_lo = blockIdx.x * per;
    const uint32_t t_hi = t_lo + per < ntiles ? t_lo + per : ntiles;
    if (t_lo >= t_hi) return;
    for (uint32_t d = lane; d < 256u; d += 64) s_h[w][d] = 0u;   // this wave's row (own writes only)
    // tile t of segment sg: records [t0, te) (positions clamped to n: a table is only ever wrong
    // after a counting fault, which is reported; the reads stay inside the buffers regardless)
    auto geom = [&](uint32_t t, uint32_t sg, uint32_t& t0, uint32_t& te) {
        const uint32_t e = end[sg] < sw.n ? end[sg] : sw.n;
        const uint32_t t0r = start[sg] + (t - first[sg]) * kSplitTile;
        t0 = t0r < e ? t0r : e;
        te = e - t0 < kSplitTile ? e : t0 + kSplitTile;
    };
    // wave w counts records [t0 + w * 512, +512): slot j of lane l = + j * 64 + l; the pads past
    // the half's end load as kPadKey (digit 255) and are taken off at the flush
    auto load = [&](uint32_t t0, uint32_t te, uint32_t (&k)[KPT]) {
        const uint64_t wb = (uint64_t)t0 + w * (64u * KPT) + lane;
#pragma unroll
        for (int j = 0; j < KPT; ++j) k[j] = wb + j * 64 < te ? rec[(wb + j * 64) * KS] : kPadKey;
    };
    // half u of the range: tile u / 2, records [t0 + (u & 1) HALF, ...) of it
    auto half = [&](uint32_t u, uint32_t sgu, uint32_t& h0, uint32_t& he) {
        uint32_t t0, te;
        geom(u >> 1, sgu, t0, te);
        const uint32_t a = (u & 1u) ? (te - t0 > HALF ? t0 + HALF : te) : t0;
        h0 = a;
        he = te - a < HALF ? te : a + HALF;
    };
    uint32_t sg = split_seg_of(first, nseg, t_lo);
    uint32_t h0, he;
    half(2 * t_lo, sg, h0, he);
    uint32_t k[KPT];
    load(h0, he, k);
    uint32_t pads = 0;   // pads counted as digit 255 of segment sg so far
    for (uint32_t u = 2 * t_lo; u < 2 * t_hi; ++u) {
        pads += HALF - (he - h0);
        // the next half's segment and keys (in flight while this half is counted)
        const uint32_t un = u + 1;
        const bool more = un < 2 * t_hi;
        const uint32_t tn = un >> 1;
        const uint32_t sgn = (more && (un & 1u) == 0u && first[sg + 1] <= tn) ? sg + 1 : sg;   // >= 1 tile each
        uint32_t kn[KPT], h0n = 0, hen = 0;
        if (more) {
            half(un, sgn, h0n, hen);
            load(h0n, hen, kn);
        }
        count_slots<KPT>(k, s_h[w], shift, 255u);
        if (!more || sgn != sg) {
            // this workgroup's last tile of segment sg: its counts to the row, then its arrival
            __syncthreads();
            if (tid < 256u) {
                uint32_t c = 0;
#pragma unroll
                for (uint32_t q = 0; q < NW; ++q) {
                    c += s_h[q][tid];
                    s_h[q][tid] = 0u;
                }
                if (tid == 255u) c -= pads;
                if (c) atomicAdd(&rows[(size_t)sg * 256u + tid], c);
            }
            pads = 0;
            // the adds have completed (vmcnt covers atomics) before the arrival (release)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // arrivals expected: the workgroups whose tile ranges meet the segment
                const uint32_t g0 = first[sg] / per, g1 = (first[sg + 1] - 1u) / per;
                s_flag = atomicAdd(&arrive[sg], 1u) + 1u == g1 - g0 + 1u ? 1u : 0u;
            }
            __syncthreads();
            if (s_flag) {
                // the segment's last workgroup: the row -> absolute digit bases
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                uint32_t c = 0, tot = 0;
                if (tid < 256u)
                    c = __hip_atomic_load(&rows[(size_t)sg * 256u + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t ex = block_excl_scan_n<NW>(c, s_scr, tot);
                if (tid == 0 && tot != end[sg] - start[sg]) split_fail(sw);
                if (tid < 256u) rows[(size_t)sg * 256u + tid] = start[sg] + ex;
                if constexpr (LEVEL == 2) {
                    if (tid < 256u && c > kSub8Cap) {   // a sub-bucket over the bucket tile: level 3's
                        const uint32_t slot = atomicAdd(&sw.tab3[0], 1u);
                        if (slot < sw.smax3) {
                            sw.tab3[2 + sw.smax3 + slot] = start[sg] + ex;   // its start and count
                            sw.tab3[2 + 2 * sw.smax3 + slot] = c;             // (the layout makes it an end)
                        } else {
                            split_fail(sw);
                        }
                    }
                    // the bucket sort's work list: runs of consecutive sub-buckets of at most
                    // kSub8Small records together (one 16-bit LDS sort each: as many items as the
                    // bucket pass has for uniform keys, where one item per sub-bucket made 163840
                    // mostly small ones for config 4), the larger ones alone (mid list)
                    // (one thread lays the runs out in LDS, two atomics claim their list slots,
                    // every thread writes its entry: a list atomic per run made this 2x slower)
                    if (tid < 256u) s_c[tid] = c;
                    __syncthreads();
                    if (tid == 0) {
                        uint32_t cst = start[sg], acc = 0, nch = 0, nmid = 0;
                        for (uint32_t dd = 0; dd < 256u; ++dd) {
                            const uint32_t cd = s_c[dd];
                            if (cd > kSub8Small) {
                                if (acc) { s_cs[nch] = cst; s_cn[nch++] = acc; }
                                if (cd <= kSub8Cap) s_md[nmid++] = dd;
                                cst += acc + cd;
                                acc = 0;
                            } else if (acc + cd > kSub8Small) {
                                s_cs[nch] = cst;
                                s_cn[nch++] = acc;
                                cst += acc;
                                acc = cd;
                            } else {
                                acc += cd;
                            }
                        }
                        if (acc) { s_cs[nch] = cst; s_cn[nch++] = acc; }
                        s_nl[0] = nch;
                        s_nl[1] = nmid;
                        s_nl[2] = nch ? atomicAdd(&sw.chunks[0], nch) : 0u;
                        s_nl[3] = nmid ? atomicAdd(&sw.mid[0], nmid) : 0u;
                    }
                    __syncthreads();
                    if (tid < s_nl[0]) {
                        const uint32_t slot = s_nl[2] + tid;
                        if (slot < sw.chunkmax) {
                            sw.chunks[1 + 2 * slot] = s_cs[tid];
                            sw.chunks[2 + 2 * slot] = s_cn[tid];
                        } else {
                            split_fail(sw);
                        }
                    }
                    if (tid < s_nl[1]) {
                        const uint32_t slot = s_nl[3] + tid;
                        if (slot < sw.midmax) sw.mid[1 + slot] = (sg << 8) | s_md[tid];
                        else split_fail(sw);
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                    if (tid == 0) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        s_flag = atomicAdd(&arrive[smax], 1u) + 1u == nseg ? 2u : 0u;
                    }
                    __syncthreads();
                    if (s_flag == 2u) {
                        // the last segment done: lay out level 3 from its list
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                        const uint32_t n3r = __hip_atomic_load(&sw.tab3[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint32_t n3 = n3r < sw.smax3 ? n3r : sw.smax3;
                        const uint32_t got = split_layout<B>(n3, sw.smax3, sw.tab3, sw.rows3, sw.arrive3, sw,
                                                             [&](uint32_t i, uint32_t& st, uint32_t& cn) {
                                                                 st = __hip_atomic_load(&sw.tab3[2 + sw.smax3 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                                                 cn = __hip_atomic_load(&sw.tab3[2 + 2 * sw.smax3 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                                             });
                        if (tid < 16u) sw.gate3[tid] = got ? 1u : 0u;
                    }
                }
            }
            __syncthreads();   // s_flag is reused; the rows were zeroed before this barrier
        }
        if (more) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) k[j] = kn[j];
            sg = sgn;
            h0 = h0n;
            he = hen;
        }
    }
}

// The level-2 sub-buckets, sorted in LDS and written to the output at their positions.  LISTED =
// false: the work list's runs of consecutive sub-buckets of one huge bucket (at most BLOCK x KPT
// records; their keys share the top 16 bits), sorted stably by the low 16 bits in two 8-bit LDS
// passes, one run per workgroup (grid-stride beyond the grid); LISTED = true: the sub-buckets of
// more than kSub8Small records (up to kSub8Cap; their keys share the top 24 bits), by byte 0 in one
// pass, on a small grid.  LO: the output layout (the caller's arrays, records, or keys); the input
// is records (keys, LO = KEYS).  PACK: ranks as 16-bit pairs.
template <int BLOCK, int KPT, int RANK, int LO, int MW = 1, bool PACK = false, bool LISTED = false>
__global__ __launch_bounds__(BLOCK, MW) void k_bucket_sort8(const uint32_t* rec, SplitWs sw,
                                                            uint32_t* out_k, uint32_t* __restrict__ out_v) {
    constexpr int NW = BLOCK / 64, TILE = BLOCK * KPT, WAVE_KEYS = 64 * KPT;
    constexpr bool KV = LO != LAYOUT_KEYS;
    constexpr int LI = KV ? LAYOUT_AOS : LAYOUT_KEYS;
    static_assert(BLOCK >= 256, "one digit per thread in the scan");
    __shared__ uint32_t s_whist[NW][256];
    __shared__ uint32_t s_scratch[NW];
    __shared__ uint2 s_kv[KV ? TILE : 1];
    __shared__ uint32_t s_k[KV ? 1 : TILE];
    if (gated_off(sw.gate2, 0)) return;
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t wbase = w * WAVE_KEYS;
    const uint32_t* end = sw.tab2 + 2 + 2 * sw.smax2;
    const uint32_t nitems = LISTED ? (sw.mid[0] < sw.midmax ? sw.mid[0] : sw.midmax)
                                   : (sw.chunks[0] < sw.chunkmax ? sw.chunks[0] : sw.chunkmax);
    for (uint32_t ii = blockIdx.x; ii < nitems; ii += gridDim.x) {
        uint32_t base, cnt;
        if (LISTED) {
            const uint32_t it = sw.mid[1 + ii];
            const uint32_t sg = it >> 8, d = it & 255u;
            base = sw.rows2[it];
            const uint32_t nxt = d == 255u ? end[sg] : sw.rows2[it + 1];
            cnt = nxt - base;
        } else {
            base = sw.chunks[1 + 2 * ii];
            cnt = sw.chunks[2 + 2 * ii];
        }
        if (cnt == 0u || cnt > (uint32_t)TILE) continue;        // (never: the lists' bounds)
        if ((uint64_t)base + cnt > sw.n) continue;              // (never: a counting fault, reported)
        uint32_t k[KPT], v[KV ? KPT : 1];
        // (branch-free, load_bucket; 256 x 17 records: load_tile, whose code there has no per-slot wait)
        if constexpr (!KV || KPT > 24) load_bucket<KPT, KV>(rec + (KV ? 2ull : 1ull) * base, wbase, cnt, k, v);
        else load_tile<KPT, LI>(rec + (KV ? 2ull : 1ull) * base, nullptr, wbase, cnt, false, k, v);
        if (cnt > 1u) {
            for (uint32_t p = 0, shift = 0; p < (LISTED ? 1u : 2u); ++p, shift += 8u) {
                Slots<KPT, PACK> rank;
                uint32_t c;   // pads: kPadKey, digit 255, after every real key
                const uint32_t tstart = rank_tile<8, NW, KPT, RANK>(k, rank, s_whist, s_scratch, shift, 255u, 0u, c);
                if (tid < 256u) set_wave_offsets<8, NW>(s_whist, tstart);
                __syncthreads();
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t q = s_whist[w][(k[j] >> shift) & 255u] + rank.get(j);
                    if constexpr (KV) s_kv[q] = make_uint2(k[j], v[j]);
                    else s_k[q] = k[j];
                }
                __syncthreads();
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    if constexpr (KV) {
                        const uint2 kv = s_kv[wbase + j * 64 + lane];
                        k[j] = kv.x;
                        v[j] = kv.y;
                    } else {
                        k[j] = s_k[wbase + j * 64 + lane];
                    }
                }
                __syncthreads();
            }
        }
        const size_t o0 = (size_t)base + wbase + lane;
        const int lim = (int)cnt - (int)(wbase + lane);
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            if (j * 64 < lim) {
                if constexpr (LO == LAYOUT_AOS) (reinterpret_cast<uint2*>(out_k) + o0)[j * 64] = make_uint2(k[j], v[j]);
                else if constexpr (LO == LAYOUT_KEYS) (out_k + o0)[j * 64] = k[j];
                else { (out_k + o0)[j * 64] = k[j]; (out_v + o0)[j * 64] = v[j]; }
            }
        }
    }
}

// In-LDS sort of the 16-bit buckets: a workgroup takes a bucket's records (R2, contiguous, at most
// BLOCK * KPT), sorts them stably by their low 16 bits in two 8-bit LDS passes and writes them to
// the output as one contiguous run (whole 128-B lines but at the two ends).  Workgroup i takes
// buckets i, i + grid, ... (the bucket-sized launch: one bucket per workgroup; a persistent grid
// that loads the next bucket while sorting the current one measured slower: 2 instead of 3
// workgroups per CU).  Occupancy is what bounds this kernel: MW = 3 waves per SIMD (<= 168 VGPRs)
// with a 4352-record tile (LDS for 3 workgroups per CU) runs it at 0.82 ms for 2^28 records, against
// 1.07 ms at 2 waves per SIMD.
// Two launches share the buckets: a tile sized to the bucket population (about 1.15x the mean
// bucket) takes every bucket of at most BLOCK * KPT records (min_cnt = 0), and a 16K-record tile
// takes the rest (min_cnt = the first launch's tile); k_msd_plan gates the path off when a
// bucket exceeds the large tile.
// LO: output layout (LAYOUT_SOA: the caller's two arrays; LAYOUT_AOS: records - the texture
// layout, sorted in place: R2 is then the caller's buffer itself, and every workgroup has read its
// whole bucket before it writes the same range; LAYOUT_KEYS: keys only, in place as well - `rec`
// is then a key array, R2 the caller's keys).
// PF = 1: the next bucket's keys are loaded before the current bucket is sorted (a persistent grid;
// keys only, where a bucket is a few KB and a workgroup's load latency is not hidden otherwise).
#if !RS_KNOB_OPEN || !defined(RS_BUCKET_PACK)
#undef RS_BUCKET_PACK
#define RS_BUCKET_PACK 0     // 1: k_bucket_sort keeps its ranks as 16-bit pairs (VGPRs)
#endif
#if !RS_KNOB_OPEN || !defined(RS_BUCKET_MW)
#undef RS_BUCKET_MW
#define RS_BUCKET_MW 3       // k_bucket_sort tiles of <= 18 records per thread: workgroups per CU
#endif
template <int BLOCK, int KPT, int RANK, int LO = LAYOUT_SOA, int MW = 1, int PF = 0>
__global__ __launch_bounds__(BLOCK, MW) void k_bucket_sort(const uint32_t* rec,
                                                       const uint32_t* __restrict__ hist16,
                                                       const uint32_t* __restrict__ base16,
                                                       uint32_t* out_k,
                                                       uint32_t* __restrict__ out_v,
                                                       const uint32_t* gate, uint32_t* err,
                                                       uint32_t min_cnt,
                                                       const uint32_t* __restrict__ over = nullptr,
                                                       uint32_t kbase = 0,
                                                       const uint32_t* __restrict__ sstart = nullptr,
                                                       uint32_t rmask = 0xFFFFFFFFu,
                                                       uint32_t b_lo = 0, uint32_t b_cnt = 65536) {
    // unlisted (over == null): buckets [b_lo, b_lo + b_cnt) (a multi-GPU region's top bytes)
    constexpr int R = 8, RADIX = 256;
    // bucket b's first record in rec: its top-byte segment's start + its base inside the segment
    // (modulo the ring of rmask + 1 records, sweep experiments), and in the output
    auto bstart = [&](uint32_t b) { return sstart[b >> 8] + base16[b]; };
    auto rstart = [&](uint32_t b) { return bstart(b) & rmask; };
    constexpr int NW = BLOCK / 64;
    constexpr int TILE = BLOCK * KPT;
    constexpr int WAVE_KEYS = 64 * KPT;
    constexpr bool KV = LO != LAYOUT_KEYS;
    constexpr int LI = KV ? LAYOUT_AOS : LAYOUT_KEYS;   // R2: records, or keys
    static_assert(BLOCK >= RADIX, "one digit per thread in the scan");
    __shared__ uint32_t s_whist[NW][RADIX];
    __shared__ uint32_t s_scratch[NW];
    __shared__ uint2 s_kv[KV ? TILE : 1];
    __shared__ uint32_t s_k[KV ? 1 : TILE];
    if (gated_off(gate, 0)) return;
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t wbase = w * WAVE_KEYS;
    // workgroup i takes buckets (listed buckets with `over`) i, i + grid, ...
    const uint32_t nb = over ? over[0] : b_cnt;
    auto bucket_of = [&](uint32_t it) { return over ? over[1 + it] : b_lo + it; };
    auto next_valid = [&](uint32_t it, uint32_t& cnt) {
        for (; it < nb; it += gridDim.x) {
            cnt = hist16[bucket_of(it)];
            if (cnt == 0u || cnt <= min_cnt) continue;   // empty, or the smaller tile's launch took it
            if (cnt > (uint32_t)TILE) continue;           // the next launch's (listed: the wide kernel's,
            break;                                        // which flags any bucket over its own tile)
        }
        return it;
    };
    uint32_t cnt = 0;
    uint32_t it = next_valid(blockIdx.x, cnt);
    if (it >= nb) return;
    uint32_t k[KPT], v[KV ? KPT : 1];
    uint32_t k2[PF ? KPT : 1], v2[PF && KV ? KPT : 1];
    // branch-free loads (load_bucket) but for the 256 x (<= 24) tiles writing records (texture
    // layout), whose load_tile code has no per-slot wait: measured at config 3, separate arrays
    // 0.845 -> 0.770 ms per bucket pass with load_bucket, records 0.851 -> 0.879
    // (profiles/r05/ab_bucket_buf/)
    constexpr bool BUF = LO != LAYOUT_AOS || KPT > 24 || BLOCK > 256;
    auto load = [&](const uint32_t* src, uint32_t c, uint32_t (&kk)[KPT], uint32_t (&vv)[KV ? KPT : 1]) {
        if constexpr (BUF) load_bucket<KPT, KV>(src, wbase, c, kk, vv);
        else load_tile<KPT, LI>(src, nullptr, wbase, c, false, kk, vv);
    };
    load(rec + (KV ? 2ull : 1ull) * rstart(bucket_of(it)), cnt, k, v);
    while (true) {
        const uint32_t b = bucket_of(it);
        const uint32_t base = bstart(b);
        uint32_t ncnt = 0;
        const uint32_t nit = next_valid(it + gridDim.x, ncnt);
        if constexpr (PF != 0) {
            if (nit < nb)
                load(rec + (KV ? 2ull : 1ull) * rstart(bucket_of(nit)), ncnt, k2, v2);
        }
        if (cnt > 1u) {
            for (uint32_t p = 0, shift = 0; p < 2u; ++p, shift += 8u) {
                const uint32_t mask = 255u;
                Slots<KPT, RS_BUCKET_PACK != 0> rank;
                uint32_t c;   // pads included (kPadKey: digit 255, after every real key)
                const uint32_t tstart = rank_tile<R, NW, KPT, RANK>(k, rank, s_whist, s_scratch, shift, mask, 0u, c);
                if (tid < (uint32_t)RADIX) set_wave_offsets<R, NW>(s_whist, tstart);
                __syncthreads();
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    const uint32_t q = s_whist[w][(k[j] >> shift) & mask] + rank.get(j);
                    if constexpr (KV) s_kv[q] = make_uint2(k[j], v[j]);
                    else s_k[q] = k[j];
                }
                __syncthreads();
#pragma unroll
                for (int j = 0; j < KPT; ++j) {
                    if constexpr (KV) {
                        const uint2 kv = s_kv[wbase + j * 64 + lane];
                        k[j] = kv.x;
                        v[j] = kv.y;
                    } else {
                        k[j] = s_k[wbase + j * 64 + lane];
                    }
                }
                __syncthreads();
            }
        }
        // slot j of lane l of wave w holds sorted position w * WAVE_KEYS + j * 64 + l; one base
        // address per output array and constant per-slot offsets (per-slot addresses spilled)
        {
            const size_t o0 = (size_t)base + wbase + lane;
            const int lim = (int)cnt - (int)(wbase + lane);
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                if (j * 64 < lim) {
                    if constexpr (LO == LAYOUT_AOS) {
                        (reinterpret_cast<uint2*>(out_k) + o0)[j * 64] = make_uint2(k[j] + kbase, v[j]);
                    } else if constexpr (LO == LAYOUT_KEYS) {
                        (out_k + o0)[j * 64] = k[j] + kbase;
                    } else {
                        (out_k + o0)[j * 64] = k[j] + kbase;
                        (out_v + o0)[j * 64] = v[j];
                    }
                }
            }
        }
        if (nit >= nb) break;
        it = nit;
        cnt = ncnt;
        __syncthreads();   // s_whist / s_kv are reused
        if constexpr (PF != 0) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                k[j] = k2[j];
                if constexpr (KV) v[j] = v2[j];
            }
        } else {
            load(rec + (KV ? 2ull : 1ull) * rstart(bucket_of(it)), cnt, k, v);
        }
    }
}

// Wide buckets: up to 1024 x KPT records (KPT = 34: 34816, the 16-bit buckets of up to 2^31 uniform
// keys, ~32K records each) sorted by one 1024-thread workgroup with 4 bytes of LDS per record, where
// k_bucket_sort stages 8-byte records (16K at most).  The records stay in registers; what moves
// through LDS is w = (low 16 bits of the key) << 16 | p, p = the record's position in the bucket
// (< 65536), in two stable 8-bit passes (key bits 0-7, then 8-15); the values follow in one exchange
// (s[p] = value, then value = s[w & 0xFFFF]).  The key is rebuilt from the bucket number and w:
// (b << bshift) | (w >> 16), bshift = the bucket's low bit (16; the range form: vbits - 16, where
// the bits w >> 16 shares with b << bshift agree).  Keys only: the keys themselves move (no p).
// Pads (positions >= cnt) are w = kPadKey: digit 255 in both passes, after every real key.
// One bucket per workgroup: a grid of 65536 (every bucket over min_cnt), or listed buckets (`over`).
// BLOCK x KPT per workgroup, MW waves per SIMD (the occupancy the register budget must allow:
// 1024 x 34 = one workgroup per CU, 512 x 34 two, 512 x 18 three).  VREG: the values ride in
// registers through the sort (else the bucket's records are read again, from L2 / Infinity Cache,
// for the value exchange).
#if !RS_KNOB_OPEN || !defined(RS_WIDE_GATHER)
#undef RS_WIDE_GATHER
#define RS_WIDE_GATHER 0   // sweep: 1 = values gathered from the records (see below)
#endif
template <int BLOCK, int KPT, int RANK, int LO, int MW = 4, bool VREG = false>
__global__ __launch_bounds__(BLOCK, MW) void k_bucket_sort_wide(const uint32_t* rec,
                                                              const uint32_t* __restrict__ hist16,
                                                              const uint32_t* __restrict__ base16,
                                                              uint32_t* out_k, uint32_t* __restrict__ out_v,
                                                              const uint32_t* gate, uint32_t* err,
                                                              uint32_t min_cnt,
                                                              const uint32_t* __restrict__ over,
                                                              uint32_t kbase,
                                                              const uint32_t* __restrict__ sstart,
                                                              uint32_t rmask, uint32_t bshift,
                                                              uint32_t b_lo = 0, uint32_t b_cnt = 65536) {
    // unlisted (over == null): buckets [b_lo, b_lo + b_cnt), e.g. a multi-GPU region's top bytes
    // (a persistent grid loading the next bucket while sorting one was measured slower: the
    // prefetch registers spill at one workgroup per CU, profiles/r03_bucket_prefetch_ab.json)
    constexpr int NW = BLOCK / 64, RADIX = 256;
    constexpr int TILE = BLOCK * KPT;
    constexpr int WAVE_KEYS = 64 * KPT;
    constexpr bool KV = LO != LAYOUT_KEYS;
    constexpr bool VR = KV && VREG;
    static_assert(TILE <= 65536, "16-bit record positions");
    static_assert(BLOCK >= RADIX, "one digit per thread in the scan");
    __shared__ uint32_t s_whist[NW][RADIX];
    __shared__ uint32_t s_scratch[NW];
    __shared__ uint32_t s_w[TILE];
    if (gated_off(gate, 0)) return;
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t wbase = w * WAVE_KEYS;
    const uint32_t nb = over ? over[0] : b_cnt;
    auto bucket_of = [&](uint32_t it) { return over ? over[1 + it] : b_lo + it; };
    // the next bucket at or after `it` (stride gridDim.x) this launch sorts.  A one-record bucket
    // is sorted too: the output is not R2 (with values), so every record must be written.
    auto next_valid = [&](uint32_t it, uint32_t& cnt) {
        for (; it < nb; it += gridDim.x) {
            cnt = hist16[bucket_of(it)];
            if (cnt == 0u || cnt <= min_cnt) continue;   // empty, or the smaller tile's launch took it
            if (cnt > (uint32_t)TILE) {   // unlisted: a huge bucket (the split's); listed: never
                if (over && tid == 0) atomicOr(err, 8u);
                continue;
            }
            break;
        }
        return it;
    };
    auto src_of = [&](uint32_t b) { return rec + (KV ? 2ull : 1ull) * ((sstart[b >> 8] + base16[b]) & rmask); };
    // w = (low 16 bits of the key) << 16 | position (KV), or the key (keys only); pads kPadKey
    // Branch-free buffer loads over the bucket's records (lanes past cnt read 0): a load under a
    // per-slot branch waits for itself before the branch joins, one memory latency per slot.
    constexpr uint32_t ESZ = KV ? 8u : 4u;
    auto bucket_rsrc = [](const uint32_t* src, uint32_t cnt) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(cnt * ESZ), 0x00020000);
    };
    auto load_words = [&](const uint32_t* src, uint32_t cnt, uint32_t (&xx)[KPT], uint32_t (&vv)[VR ? KPT : 1]) {
        const int lim = (int)cnt - (int)(wbase + lane);
        const __amdgpu_buffer_rsrc_t rr = bucket_rsrc(src, cnt);
        uint32_t lo = (wbase + lane) * ESZ;   // (one offset register, immediate slot offsets)
        asm volatile("" : "+v"(lo));
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t kw = __builtin_amdgcn_raw_buffer_load_b32(rr, (int)(lo + j * 64 * ESZ), 0, 0);
            if (VR) vv[VR ? j : 0] = __builtin_amdgcn_raw_buffer_load_b32(rr, (int)(lo + j * 64 * ESZ + 4), 0, 0);
            // (the pad mask opaque: a select on the loaded word becomes a branch with the load sunk
            // into it, and the wait with it)
            uint32_t m = j * 64 < lim ? 0xFFFFFFFFu : 0u;
            asm volatile("" : "+v"(m));
            const uint32_t wd = KV ? ((kw & 0xFFFFu) << 16) | (wbase + (uint32_t)j * 64u + lane) : kw;
            xx[j] = (wd & m) | (kPadKey & ~m);
        }
    };
    uint32_t cnt = 0;
    uint32_t it = next_valid(blockIdx.x, cnt);
    if (it >= nb) return;
    uint32_t x[KPT];
    uint32_t v[VR ? KPT : 1];
    load_words(src_of(bucket_of(it)), cnt, x, v);
    while (true) {
        const uint32_t b = bucket_of(it);
        const uint32_t base = sstart[b >> 8] + base16[b];
        const uint32_t* src = rec + (KV ? 2ull : 1ull) * (base & rmask);
        // KV: the key's low 16 bits sit in w's high half; keys only: the key itself
        constexpr uint32_t S0 = KV ? 16u : 0u;
#pragma unroll 1
        for (uint32_t shift = S0; shift < S0 + 16u; shift += 8u) {
            Slots<KPT, true> rank;
            uint32_t c;
            const uint32_t tstart = rank_tile<8, NW, KPT, RANK>(x, rank, s_whist, s_scratch, shift, 255u, 0u, c);
            if (tid < (uint32_t)RADIX) set_wave_offsets<8, NW>(s_whist, tstart);
            __syncthreads();
            const uint32_t sh = opaque_u(shift);
#pragma unroll
            for (int j = 0; j < KPT; ++j) s_w[s_whist[w][(x[j] >> sh) & 255u] + rank.get(j)] = x[j];
            __syncthreads();
#pragma unroll
            for (int j = 0; j < KPT; ++j) x[j] = s_w[wbase + (uint32_t)j * 64u + lane];
            __syncthreads();
        }
        // the values to their sorted positions: the bucket's records are read again (this
        // workgroup read them moments ago: Infinity Cache / L2) into LDS by position, then each
        // sorted slot gathers its value by the position in w (holding the values in registers
        // through the sort spilled).  GATHER (separate output arrays: R2 is not the output): each
        // sorted slot reads its value straight from the record instead (no LDS round).
        constexpr bool GATHER = RS_WIDE_GATHER && KV && !VR && LO == LAYOUT_SOA;
        if (KV && !GATHER) {
            // (unconditional: a slot past cnt writes the 0 its load returned to an unused position)
            const __amdgpu_buffer_rsrc_t rr = bucket_rsrc(src, cnt);
            uint32_t lo = (wbase + lane) * ESZ + 4u;
            asm volatile("" : "+v"(lo));
            uint32_t* sw = s_w + wbase + lane;
#pragma unroll
            for (int j = 0; j < KPT; ++j)
                sw[j * 64] = VR ? v[VR ? j : 0] : __builtin_amdgcn_raw_buffer_load_b32(rr, (int)(lo + j * 64 * ESZ), 0, 0);
            __syncthreads();
        }
        const uint32_t hi = b << bshift;
        // one base address per output array, constant per-slot offsets (per-slot 64-bit addresses
        // spilled); slot j is real iff j * 64 < lim (pads sort last)
        {
            const size_t o0 = (size_t)base + wbase + lane;
            const int lim = (int)cnt - (int)(wbase + lane);
            uint2* oa = reinterpret_cast<uint2*>(out_k) + o0;
            uint32_t* ok = out_k + o0;
            uint32_t* ov = KV && LO != LAYOUT_AOS ? out_v + o0 : nullptr;
#pragma unroll
            for (int j = 0; j < KPT; ++j) {
                if (j * 64 < lim) {
                    const uint32_t key = (KV ? (hi | (x[j] >> 16)) : x[j]) + kbase;
                    const uint32_t val = GATHER ? reinterpret_cast<const uint2*>(src)[x[j] & 0xFFFFu].y
                                         : KV ? s_w[x[j] & 0xFFFFu] : 0u;
                    if constexpr (LO == LAYOUT_AOS) {
                        oa[j * 64] = make_uint2(key, val);
                    } else {
                        ok[j * 64] = key;
                        if constexpr (KV) ov[j * 64] = val;
                    }
                }
            }
        }
        __syncthreads();   // s_whist / s_w are reused by the next bucket
        it = next_valid(it + gridDim.x, cnt);
        if (it >= nb) break;
        load_words(src_of(bucket_of(it)), cnt, x, v);
    }
}

// Keys-only bucket pass with one WAVE per 16-bit bucket (buckets of at most 64 * KPT keys, sorted in
// place): at ~1K keys per bucket (64M keys) a workgroup per bucket spends its time in barriers and
// load latency, so here every wave sorts its own bucket in wave-private LDS (counters + staging)
// with no workgroup barrier at all - one wave's LDS operations execute in order - and a CU holds
// ~28 buckets in flight.  Two stable 8-bit passes (low byte, then the next), pads (kPadKey) after
// every real key.  Buckets of more than 64 * KPT keys are listed by k_msd_plan for the large-tile
// launch; empty and one-key buckets are skipped.
#if !RS_KNOB_OPEN || !defined(RS_KWAVE_PF)
#undef RS_KWAVE_PF
#define RS_KWAVE_PF 0     // sweep: 1 = persistent waves that load their next bucket while sorting one
#endif
#if !RS_KNOB_OPEN || !defined(RS_KWAVE_PACK)
#undef RS_KWAVE_PACK
#define RS_KWAVE_PACK 0   // sweep: 1 = ranks as 16-bit pairs (fewer VGPRs: more waves per SIMD)
#endif
template <int KPT, int RANK, int WPB, int MW = 1>
__global__ __launch_bounds__(64 * WPB, MW) void k_bucket_sort_keys_wave(uint32_t* keys,
                                                                 const uint32_t* __restrict__ hist16,
                                                                 const uint32_t* __restrict__ base16,
                                                                 const uint32_t* gate,
                                                                 const uint32_t* __restrict__ sstart) {
    constexpr uint32_t CAP = 64u * KPT;
    __shared__ uint32_t s_h[WPB][256];
    __shared__ uint32_t s_k[WPB][CAP];
    if (gated_off(gate, 0)) return;
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    uint32_t* h = s_h[w];
    uint32_t* sk = s_k[w];
    auto wave_sync = [] { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); };
    const uint32_t stride = gridDim.x * WPB;
    // the next bucket at or after b this wave sorts (2 or more keys, within the wave tile)
    auto next_bucket = [&](uint32_t b, uint32_t& cnt) {
        for (; b < 65536u; b += stride) {
            cnt = hist16[b];
            if (cnt > 1u && cnt <= CAP) break;
        }
        return b;
    };
    auto load = [&](uint32_t b, uint32_t cnt, uint32_t (&k)[KPT]) {
        const uint32_t* src = keys + sstart[b >> 8] + base16[b];
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t q = (uint32_t)j * 64u + lane;
            k[j] = q < cnt ? src[q] : kPadKey;
        }
    };
    uint32_t cnt = 0;
    uint32_t b = next_bucket(blockIdx.x * WPB + w, cnt);
    uint32_t k[KPT];
    if (b < 65536u) load(b, cnt, k);
    while (b < 65536u) {
        uint32_t* src = keys + sstart[b >> 8] + base16[b];
        // RS_KWAVE_PF: the next bucket's keys in flight while this one is sorted
        uint32_t ncnt = 0, nb = 65536u;
        uint32_t kn[RS_KWAVE_PF ? KPT : 1];
        if (RS_KWAVE_PF) {
            nb = next_bucket(b + stride, ncnt);
            if (nb < 65536u) load(nb, ncnt, reinterpret_cast<uint32_t(&)[KPT]>(kn));
        }
#pragma unroll 1
        for (uint32_t shift = 0; shift < 16u; shift += 8u) {
#pragma unroll
            for (int i = 0; i < 4; ++i) h[lane * 4 + i] = 0u;
            wave_sync();
            Slots<KPT, RS_KWAVE_PACK != 0> rank;
            rank_slots<8, KPT, RANK, true>(k, rank, h, shift, 255u);   // (its ~128 pads by runs)
            wave_sync();
            // exclusive scan of the 256 counters: lane l owns digits 4l .. 4l + 3
            const uint4 c = *reinterpret_cast<const uint4*>(h + lane * 4);
            const uint32_t sum = c.x + c.y + c.z + c.w;
            const uint32_t ex = wave_incl_scan(sum) - sum;
            *reinterpret_cast<uint4*>(h + lane * 4) = make_uint4(ex, ex + c.x, ex + c.x + c.y, ex + c.x + c.y + c.z);
            wave_sync();
#pragma unroll
            for (int j = 0; j < KPT; ++j) sk[h[(k[j] >> shift) & 255u] + rank.get(j)] = k[j];
            wave_sync();
#pragma unroll
            for (int j = 0; j < KPT; ++j) k[j] = sk[(uint32_t)j * 64u + lane];
            wave_sync();
        }
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t q = (uint32_t)j * 64u + lane;
            if (q < cnt) src[q] = k[j];
        }
        if (RS_KWAVE_PF) {
#pragma unroll
            for (int j = 0; j < KPT; ++j) k[j] = kn[RS_KWAVE_PF ? j : 0];
            b = nb;
            cnt = ncnt;
        } else {
            b = next_bucket(b + stride, cnt);
            if (b < 65536u) load(b, cnt, k);
        }
    }
}

// ---- order check -------------------------------------------------------------------------
// inv[pass] |= 1 if any adjacent pair of keys[0..n) is out of order under `mask`.  Key i is
// word i * kstride (2 for AOS records).
__global__ __launch_bounds__(kBlock) void k_check(const uint32_t* __restrict__ keys, uint32_t n,
                                                  uint32_t kstride, uint32_t mask, uint32_t* inv,
                                                  int pass, int gate_upto) {
    if (gate_upto >= 0 && gated_off(inv, gate_upto)) return;
    bool bad = false;
    const uint32_t stride = gridDim.x * kBlock;
    // 64-bit index (n may be close to 2^32; the stride divides 2^32)
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i + 1 < n; i += stride) {
        const uint32_t a = keys[i * kstride] & mask, b = keys[(i + 1) * kstride] & mask;
        bad |= a > b;
    }
    if (__ballot(bad) != 0 && lane_id() == 0) atomicOr(inv + pass, 1u);
}

// After an early exit at an odd pass the sorted data sits in the tmp buffers: copy it back so
// the result is always in the caller's buffers (AbstractRadixSortKernel.ts:94-98).
// With a second records buffer (tk_even, one-sweep separate-values path) the data found sorted
// before an even pass > 0 sits there; otherwise even exits are already in the caller's buffers.
template <int L, int LT = L>
__global__ __launch_bounds__(kBlock) void k_finalize(const uint32_t* __restrict__ tk,
                                                     const uint32_t* __restrict__ tv,
                                                     uint32_t* __restrict__ uk,
                                                     uint32_t* __restrict__ uv, uint32_t n,
                                                     const uint32_t* inv, int passes,
                                                     const uint32_t* __restrict__ tk_even) {
    int first = -1;
    for (int c = 0; c < passes; ++c)
        if (inv[c] == 0u) { first = c; break; }
    if (first <= 0) return;
    if ((first & 1) == 0) {
        if (!tk_even) return;
        tk = tk_even;
    }
    const uint32_t stride = gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        if (L == LAYOUT_AOS) {
            reinterpret_cast<uint2*>(uk)[i] = reinterpret_cast<const uint2*>(tk)[i];
        } else if (LT == LAYOUT_AOS) {       // records in tmp -> the caller's two arrays
            const uint2 r = reinterpret_cast<const uint2*>(tk)[i];
            uk[i] = r.x;
            uv[i] = r.y;
        } else {
            uk[i] = tk[i];
            if (L == LAYOUT_SOA) uv[i] = tv[i];
        }
    }
}

// (key, value) records -> two arrays (small sorts from records; the records' last pass writes the
// arrays itself on larger ones).
__global__ __launch_bounds__(kBlock) void k_split_records(const uint2* __restrict__ rec,
                                                          uint32_t* __restrict__ k,
                                                          uint32_t* __restrict__ v, uint64_t n) {
    const uint32_t stride = gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const uint2 r = rec[i];
        k[i] = r.x;
        v[i] = r.y;
    }
}

// ---- prefix sum (PrefixSumKernel) ---------------------------------------------------------
// Three kernels, reduce-then-scan: chunk sums -> scan of chunk sums -> rescan with carry.
// ind (may be null): the caller's indirect dispatch triple (x, y, z workgroups,
// PrefixSumKernel.ts:147-158); a zero entry skips the scan, as a zeroed indirect dispatch does.
__device__ __forceinline__ bool indirect_off(const uint32_t* ind) {
    return ind && (ind[0] == 0u || ind[1] == 0u || ind[2] == 0u);
}

template <int TILE>
__global__ __launch_bounds__(kBlock) void k_chunk_sums(const uint32_t* __restrict__ data,
                                                       uint32_t n, uint32_t base, uint32_t extra,
                                                       uint32_t* __restrict__ sums,
                                                       const uint32_t* ind) {
    __shared__ uint32_t scratch[kWaves];
    if (indirect_off(ind)) return;
    const Chunk ch = chunk_of(blockIdx.x, base, extra);
    const uint64_t lo = (uint64_t)ch.first * TILE;
    const uint64_t hi64 = lo + (uint64_t)ch.count * TILE;
    const uint64_t hi = hi64 < n ? hi64 : n;
    uint32_t s = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += kBlock) s += data[i];
    uint32_t tot;
    block_excl_scan(s, scratch, tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <int TILE>
__global__ __launch_bounds__(kBlock) void k_chunk_rescan(uint32_t* __restrict__ data, uint32_t n,
                                                         uint32_t base, uint32_t extra,
                                                         const uint32_t* __restrict__ sums_scanned,
                                                         const uint32_t* ind) {
    constexpr int PER = TILE / kBlock;  // consecutive elements per thread
    __shared__ uint32_t scratch[kWaves];
    if (indirect_off(ind)) return;
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
__global__ __launch_bounds__(kBlock) void k_scan_small(uint32_t* __restrict__ a, uint32_t m,
                                                      const uint32_t* ind) {
    __shared__ uint32_t scratch[kWaves];
    if (indirect_off(ind)) return;
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

// Single-pass exclusive scan (the PrefixSumKernel export, PrefixSumKernel.ts:11-159): one read and
// one write of the data (8 B/element; the reduce-then-scan above reads it twice, 12 B/element).
// Tiles of BLOCK x EPT elements come from a ticket counter in order; each wave scans its 64 x EPT
// elements (striped: coalesced 16-byte loads, see below) with wave scans, the workgroup scans the
// wave totals, publishes the tile's aggregate, and looks back for its prefix: status words as
// k_onesweep's (((epoch << 2 | flag) << 32) | value, agent-scope relaxed 64-bit atomics, so flag
// and value travel together; the epoch tags this launch's words, so the region is never cleared),
// every wave reading 64 predecessors per round.  Waits are bounded like k_onesweep's (err[0] on a
// timeout).  PF: the next tile's ticket is taken and its loads issued before the look-back.
// History (round 4, 2^28 u32): 256 x 16 tiles, one look-back wave, per-thread contiguous elements
// 1.04 ms; 1024 x 16 tiles + PF 0.78 ms; + every wave looking back 0.78 ms (so the look-back walk
// was not the limit); the per-thread contiguous layout touched every line with four load
// instructions at 64-B lane strides - the striped layout reads each line once: 0.59 ms; 1024 x 32
// (one workgroup per CU, 128 KB of next tile in flight) 0.453 ms = 0.59 of peak (x 8: 1.33 ms,
// 512 x 16: 1.49 ms).  A wave's loads return in order, so the look-back's status words, read after
// the 128 KB of next-tile loads, waited for all of them and the stores never overlapped the loads:
// LB_FIRST reads the first round's words before those loads (0.440 ms = 0.63; profiles/r04/
// scan_lbfirst_ab).  Taking the ticket after the prefetched tile during the look-back instead of
// before it (off the critical path) ran 7.5x slower: tiles held two ahead stall their successors'
// look-backs.
// tickets: a ring of kScanTickets counters; launch e uses tickets[e % ring] and clears the next
// launch's.  VEC: the data is 16-byte aligned (16-byte loads / stores; else 4-byte ones).
#if !RS_KNOB_OPEN || !defined(RS_SCAN_LB_FIRST)
#undef RS_SCAN_LB_FIRST
#define RS_SCAN_LB_FIRST 1   // the look-back's first status words read before the next tile's loads
#endif
constexpr uint32_t kScanTickets = 64;
template <int BLOCK, int EPT, bool VEC, bool PF = true>
__global__ __launch_bounds__(BLOCK) void k_scan_lookback(uint32_t* __restrict__ data, uint32_t n,
                                                         unsigned long long* status, uint32_t* tickets,
                                                         uint32_t epoch, uint32_t* err, uint32_t spin_max,
                                                         const uint32_t* ind) {
    static_assert(EPT % 4 == 0, "whole 16-byte vectors per thread");
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t TILE = (uint32_t)BLOCK * EPT;
    __shared__ uint32_t s_wave[NW];
    __shared__ uint32_t s_t, s_prefix;
    __shared__ uint2 s_lb[NW];   // per wave of a look-back round: (sum, found | unpublished << 1)
    __shared__ uint32_t s_abort;
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    // the next launch's ticket is cleared first, also by a launch that the indirect dispatch gates
    // off: otherwise that slot would keep the count of the launch kScanTickets earlier and the next
    // live launch's first tickets would all be past the last tile (nothing scanned, no error)
    if (blockIdx.x == 0 && tid == 0) tickets[(epoch + 1) % kScanTickets] = 0u;
    if (indirect_off(ind)) return;
    uint32_t* ticket = tickets + epoch % kScanTickets;
    const uint32_t ntiles = (uint32_t)(((uint64_t)n + TILE - 1) / TILE);
    // striped layout (coalesced: each load instruction of a wave reads 1 KB contiguous): wave w's
    // EPT x 64 elements are EPT / 4 chunks of 256, lane l holding elements 4l .. 4l + 3 of each
    // (the first version gave each thread EPT contiguous elements - 64-B lane strides, every line
    // touched by 4 instructions - and ran at 2.7 TB/s)
    constexpr int NV = EPT / 4;
    auto elem0 = [&](uint32_t T, int j) {   // first element of this thread's vector j
        return (uint64_t)T * TILE + (uint64_t)w * (64u * EPT) + (uint64_t)j * 256u + lane * 4u;
    };
    auto load = [&](uint32_t T, uint32_t (&x)[EPT]) {
        if (VEC && (uint64_t)T * TILE + TILE <= n) {
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const uint4 q = *reinterpret_cast<const uint4*>(data + elem0(T, j));
                x[4 * j] = q.x; x[4 * j + 1] = q.y; x[4 * j + 2] = q.z; x[4 * j + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const uint64_t e = elem0(T, j);
#pragma unroll
                for (int c = 0; c < 4; ++c) x[4 * j + c] = e + c < n ? data[e + c] : 0u;
            }
        }
    };
    if (tid == 0) s_t = atomicAdd(ticket, 1u);
    __syncthreads();
    // uniform values (tiles, sums read back from LDS) are moved to scalar registers: the 32 + 32
    // elements in flight leave no vector registers to spare
    auto uni = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
    uint32_t T = uni(s_t), Tn = 0;
    __syncthreads();   // every thread has read s_t before thread 0 takes the next ticket into it
    uint32_t x[EPT];
    if (T < ntiles) load(T, x);
    // one look-back round over the status words sv (wave w lane l: predecessor j0 - 64w - l):
    // 1 = the prefix is complete, 2 = aborted (timeout), 0 = go on from the updated j0
    auto lb_word = [&](int64_t j0) -> unsigned long long {
        const int64_t me = j0 - (int64_t)(w * 64u + lane);
        return me >= 0 ? st_load(status + me) : (((unsigned long long)((epoch << 2) | kStInclusive)) << 32);
    };
    auto lb_round = [&](unsigned long long sv, uint32_t& prefix, int64_t& j0, uint32_t& spins) -> int {
        const uint32_t f = (uint32_t)(sv >> 32);
        const bool pub = (f >> 2) == epoch;
        const bool incl = pub && (f & 3u) == kStInclusive;
        const uint64_t unpub = __ballot(!pub), inclm = __ballot(incl);
        const uint32_t stop = inclm ? (uint32_t)__builtin_ctzll(inclm) : 64u;
        const uint64_t before = stop >= 64u ? ~0ull : ((2ull << stop) - 1ull);
        const bool bad = (unpub & before) != 0ull;
        const uint32_t wsum = wave_sum(lane <= stop && pub ? (uint32_t)sv : 0u);
        if (lane == 0) s_lb[w] = make_uint2(wsum, (stop < 64u ? 1u : 0u) | (bad ? 2u : 0u));
        __syncthreads();
        // waves in order: aggregates add up until the first inclusive prefix; an unpublished word
        // stops the round (the waves before it are consumed)
        uint32_t acc = 0, used = 0, state = 0;   // state 1 done, 2 wait
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const uint2 e = s_lb[i];
            if (state == 0) {
                if (e.y & 2u) {
                    state = 2;
                } else {
                    acc += e.x;
                    if (e.y & 1u) state = 1;
                    else ++used;
                }
            }
        }
        // a wait: bounded like k_onesweep's; thread 0 decides for the workgroup (the abort must be
        // uniform: every thread passes the same barriers)
        if (state == 2 && tid == 0) {
            const uint32_t sp = spins + 1u;
            s_abort = (sp > spin_max ||
                       ((sp & 255u) == 0u && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
                          ? 1u : 0u;
        }
        __syncthreads();   // s_lb is rewritten next round; s_abort is read
        acc = uni(acc);
        used = uni(used);
        state = uni(state);
        prefix += acc;
        if (state == 1) return 1;
        j0 -= (int64_t)used * 64;
        if (state == 2) {
            ++spins;
            if (s_abort) {
                if (tid == 0) atomicOr(err, 1u);
                return 2;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        return 0;
    };
    // the look-back of tile T (every wave at once: NW x 64 predecessors per round - the nearest
    // inclusive prefix is about as far back as there are tiles in flight); sv0: its first round's
    // words when LB_FIRST read them before the next tile's loads
    auto lookback = [&](unsigned long long sv0, uint32_t agg) {
        if (T != 0) {
            uint32_t prefix = 0, spins = 0;
            int64_t j0 = (int64_t)T - 1;
            int r = RS_SCAN_LB_FIRST ? lb_round(sv0, prefix, j0, spins) : 0;
            while (r == 0) r = lb_round(lb_word(j0), prefix, j0, spins);
            if (tid == 0) {
                st_store(status + T, (epoch << 2) | kStInclusive, prefix + agg);
                s_prefix = prefix;
            }
        } else if (tid == 0) {
            s_prefix = 0u;
        }
    };
    while (T < ntiles) {
        const bool full = (uint64_t)T * TILE + TILE <= n;
        // the wave's exclusive scan, chunk by chunk (x becomes the exclusive prefix inside the wave)
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const uint32_t a0 = x[4 * j], a1 = x[4 * j + 1], a2 = x[4 * j + 2], a3 = x[4 * j + 3];
            const uint32_t sum = a0 + a1 + a2 + a3;
            const uint32_t inc = wave_incl_scan(sum);
            const uint32_t pre = carry + inc - sum;
            x[4 * j] = pre;
            x[4 * j + 1] = pre + a0;
            x[4 * j + 2] = pre + a0 + a1;
            x[4 * j + 3] = pre + a0 + a1 + a2;
            carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        }
        // workgroup exclusive scan of the wave totals
        if (lane == 0) s_wave[w] = carry;
        if (tid == 0) s_t = atomicAdd(ticket, 1u);   // the next tile (read after the barrier)
        __syncthreads();
        uint32_t wpre = 0, agg = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const uint32_t sv = s_wave[i];
            wpre += (i < (int)w) ? sv : 0u;
            agg += sv;
        }
        agg = uni(agg);
        const uint32_t texcl = uni(wpre);   // uniform in the wave
        Tn = uni(s_t);
        // publish the aggregate at once (wave 0); then (LB_FIRST) the look-back's first status words
        // and the next tile's loads: a wave's loads return in order, so status words read after the
        // 128 KB of next-tile loads wait for all of them
        if (w == 0 && lane == 0)
            st_store(status + T, (epoch << 2) | (T == 0 ? kStInclusive : kStAggregate), agg);
        const unsigned long long sv0 = (RS_SCAN_LB_FIRST && T != 0) ? lb_word((int64_t)T - 1) : 0ull;
        uint32_t y[PF ? EPT : 1];
        if (PF && VEC) {
            // without a branch, so that the wait for sv0 counts only these loads (after a join it
            // would wait for all of them): a vector whose first element is past the end reads the
            // first vector instead and drops it; one that straddles the end reads within the
            // 16-byte block of its first element (data is 16-byte aligned) and drops the rest
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const uint64_t e = elem0(Tn, j);
                const uint4 q = *reinterpret_cast<const uint4*>(data + (e < n ? e : 0));
                y[4 * j] = e < n ? q.x : 0u;
                y[4 * j + 1] = e + 1 < n ? q.y : 0u;
                y[4 * j + 2] = e + 2 < n ? q.z : 0u;
                y[4 * j + 3] = e + 3 < n ? q.w : 0u;
            }
        } else if (PF && Tn < ntiles) {
            load(Tn, reinterpret_cast<uint32_t(&)[EPT]>(y));
        }
        lookback(sv0, agg);
        __syncthreads();
        const uint32_t add = uni(s_prefix + texcl);
        if (VEC && full) {
#pragma unroll
            for (int j = 0; j < NV; ++j)
                *reinterpret_cast<uint4*>(data + elem0(T, j)) =
                    make_uint4(x[4 * j] + add, x[4 * j + 1] + add, x[4 * j + 2] + add, x[4 * j + 3] + add);
        } else {
#pragma unroll
            for (int j = 0; j < NV; ++j) {
                const uint64_t e = elem0(T, j);
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    if (e + c < n) data[e + c] = x[4 * j + c] + add;
            }
        }
        if (PF) {
#pragma unroll
            for (int j = 0; j < EPT; ++j) x[j] = y[PF ? j : 0];
        } else if (Tn < ntiles) {
            load(Tn, x);
        }
        T = Tn;
        // s_wave / s_t / s_prefix are rewritten next tile only after its first barrier (s_t: by
        // thread 0, which passed this tile's second barrier after every thread read it)
    }
}

// ---- self-test of the lane-ordered LDS atomics that RANK_LDS_ATOMIC relies on ----------------
// gfx950 resolves one wave instruction's same-address ds_add_rtn_u32 in lane order (probed, not
// an ISA guarantee).  Every wave here repeatedly adds per-lane amounts (1, as the per-key ranks
// do, or 1-4, as the per-run ranks do) to 1-256 LDS addresses, some lanes inactive, with the same
// atomicAdd the ranking uses, and checks that each lane got the sum of the amounts of the active
// lower lanes with the same address.  *bad |= 1 on any mismatch.  Run once per device at the
// first plan creation (rsort.hip); a failure switches plans to RANK_BALLOT.
__device__ __forceinline__ uint32_t st_hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(kBlock) void k_lane_order_selftest(uint32_t iters, uint32_t* bad) {
    __shared__ uint32_t cnt[kWaves][256];
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t* c = cnt[w];
    bool fail = false;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t seed = st_hash((blockIdx.x * kWaves + w) * 0x9E3779B9u + it * 0x85EBCA6Bu);
        const uint32_t naddr = 1u << (st_hash(seed) % 9u);          // 1 .. 256 addresses
        const bool some_off = (st_hash(seed ^ 0xABCDu) & 3u) != 0u;  // 3/4: ~1/8 lanes inactive
        auto lane_info = [&](uint32_t l, uint32_t& addr, uint32_t& amt) -> bool {
            const uint32_t h = st_hash(seed + l * 0x27D4EB2Fu);
            addr = h % naddr;
            amt = (it & 1u) ? 1u + ((h >> 12) & 3u) : 1u;
            return !some_off || ((h >> 20) & 7u) != 0u;
        };
        for (uint32_t d = lane; d < 256u; d += 64) c[d] = 0u;
        uint32_t my_addr, my_amt;
        const bool act = lane_info(lane, my_addr, my_amt);
        if (act) {
            const uint32_t got = atomicAdd(&c[my_addr], my_amt);
            uint32_t expect = 0;
            for (uint32_t l = 0; l < lane; ++l) {
                uint32_t a, m;
                if (lane_info(l, a, m) && a == my_addr) expect += m;
            }
            fail |= got != expect;
        }
    }
    if (__ballot(fail) != 0ull && lane == 0) atomicOr(bad, 1u);
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
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i + 1 < n; i += stride)
        bad |= (keys[i] & mask) > (keys[i + 1] & mask);
    if (__ballot(bad) != 0 && lane_id() == 0) atomicAnd(flag, 0u);
}

}  // namespace rs
