/*
 * rs_oracle.c — CPU restatement of the reference's 4-way LSD radix sort.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product path (webgpu-radix-sort_amd/) never links or calls it.
 *
 * What it restates (paths relative to the reference root, MatthieuLepers/WebGPU-Radix-Sort
 * v1.0.7, mounted read-only at /root/reference during the build):
 *
 *   rso_radix_sort_literal   — the per-2-bit-pass structure of AbstractRadixSortKernel
 *                              (src/kernels/radix-sort/AbstractRadixSortKernel.ts:93-107,229-247),
 *                              ping-pong keys<->tmp (RadixSortBufferKernel.ts:73-85), per-workgroup
 *                              4-digit exclusive rank + digit-major block sums
 *                              (src/shaders/RadixSort.ts:56-125), optional in-place local shuffle
 *                              (src/shaders/optimizations/RadixSortLocalShuffle.ts:94-116),
 *                              Blelloch scan of the 4*WC block sums (rso_prefix_sum_blelloch) and the
 *                              reorder scatter (src/shaders/RadixSortReorder.ts:86-101).
 *   rso_prefix_sum_blelloch  — PrefixSumKernel recursion (src/kernels/PrefixSumKernel.ts:45-133):
 *                              reduce_downsweep per 2T items (src/shaders/PrefixSum.ts:13-79),
 *                              recurse on the block sums, add_block_sums (PrefixSum.ts:81-106).
 *   rso_stable_sort_masked   — the closed form of the above: a stable ascending
 *                              sort of (key & mask(bit_count)), values carried along.
 *   rso_is_sorted_masked     — the order check of src/shaders/CheckSort.ts:102-113, with the
 *                              reference quirks Q1 (last pair skipped) and Q2 (unmasked compare)
 *                              fixed: every adjacent pair, masked keys.
 *   rso_gen_u32              — the counter-based synthetic key generator shared with the HIP
 *                              library (splitmix64 finaliser of seed*C + index), so the CPU and GPU
 *                              regenerate identical inputs.
 *
 * Parity pinning: the reference holds no golden vectors.  Its test oracle is
 * `keys.slice(0,count).sort((a,b)=>a-b)` plus `keys[values[i]] == keysResult[i]`
 * (example/tests.ts:86-95) and `prefixSumCpu` (example/tests.ts:288-296).  tests/golden/ holds
 * fixtures whose expected keys were produced by that exact JS expression run in Node here
 * (tests/golden/gen_golden.py); the restatement below is checked against them.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define RSO_API __attribute__((visibility("default")))

/* ---- synthetic inputs ------------------------------------------------------------------ */

static inline uint64_t rso_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

RSO_API uint32_t rso_gen_u32(uint64_t seed, uint64_t i) {
    return (uint32_t)rso_mix64(seed * 0xD1B54A32D192ED03ull + i);
}

RSO_API void rso_fill_u32(uint32_t* dst, uint64_t n, uint64_t seed) {
    for (uint64_t i = 0; i < n; ++i) dst[i] = rso_gen_u32(seed, i);
}

/* ---- Blelloch prefix sum (PrefixSum.ts + PrefixSumKernel.ts recursion) ------------------ */

/* One reduce_downsweep workgroup over items[base .. base+2T) (PrefixSum.ts:13-79).
 * Returns the block total (blockSums[WORKGROUP_ID], PrefixSum.ts:46-51). */
static uint32_t rso_reduce_downsweep(uint32_t* items, uint64_t base, uint64_t count,
                                     uint32_t T, uint32_t* temp) {
    const uint32_t ITEMS = 2u * T;
    for (uint32_t k = 0; k < ITEMS; ++k)                       /* PrefixSum.ts:29-31 */
        temp[k] = (base + k < count) ? items[base + k] : 0u;
    uint32_t offset = 1;
    for (uint32_t d = ITEMS >> 1; d > 0; d >>= 1) {            /* up-sweep, PrefixSum.ts:36-44 */
        for (uint32_t tid = 0; tid < d; ++tid) {
            uint32_t ai = offset * (2u * tid + 1u) - 1u;
            uint32_t bi = offset * (2u * tid + 2u) - 1u;
            temp[bi] += temp[ai];
        }
        offset *= 2u;
    }
    uint32_t total = temp[ITEMS - 1];                          /* PrefixSum.ts:46-51 */
    temp[ITEMS - 1] = 0;
    for (uint32_t d = 1; d < ITEMS; d *= 2u) {                 /* down-sweep, PrefixSum.ts:54-66 */
        offset >>= 1;
        for (uint32_t tid = 0; tid < d; ++tid) {
            uint32_t ai = offset * (2u * tid + 1u) - 1u;
            uint32_t bi = offset * (2u * tid + 2u) - 1u;
            uint32_t t = temp[ai];
            temp[ai] = temp[bi];
            temp[bi] += t;
        }
    }
    for (uint32_t k = 0; k < ITEMS; ++k)                       /* PrefixSum.ts:69-78 */
        if (base + k < count) items[base + k] = temp[k];
    return total;
}

/* In-place exclusive scan of data[0..count) with workgroup size T (power of two), following
 * the recursion of PrefixSumKernel.createPassRecursive (PrefixSumKernel.ts:45-133). */
RSO_API int rso_prefix_sum_blelloch(uint32_t* data, uint64_t count, uint32_t T) {
    if (T == 0 || (T & (T - 1))) return -1;                   /* PrefixSumKernel.ts:33-35 */
    if (count == 0) return 0;
    const uint64_t ITEMS = 2ull * T;
    const uint64_t wgc = (count + ITEMS - 1) / ITEMS;          /* PrefixSumKernel.ts:47 */
    uint32_t* temp = (uint32_t*)malloc(sizeof(uint32_t) * ITEMS);
    uint32_t* block_sums = (uint32_t*)malloc(sizeof(uint32_t) * wgc);
    if (!temp || !block_sums) { free(temp); free(block_sums); return -2; }
    for (uint64_t wg = 0; wg < wgc; ++wg)
        block_sums[wg] = rso_reduce_downsweep(data, wg * ITEMS, count, T, temp);
    free(temp);
    if (wgc > 1) {                                             /* PrefixSumKernel.ts:111-132 */
        int rc = rso_prefix_sum_blelloch(block_sums, wgc, T);
        if (rc) { free(block_sums); return rc; }
        for (uint64_t i = 0; i < count; ++i)                   /* add_block_sums, PrefixSum.ts:81-106 */
            data[i] += block_sums[i / ITEMS];
    }
    free(block_sums);
    return 0;
}

/* Plain sequential exclusive scan (example/tests.ts:288-296, prefixSumCpu). */
RSO_API void rso_prefix_sum_seq(uint32_t* data, uint64_t count) {
    uint32_t sum = 0;
    for (uint64_t i = 0; i < count; ++i) { uint32_t v = data[i]; data[i] = sum; sum += v; }
}

/* ---- literal per-pass radix sort ------------------------------------------------------- */

/* One 2-bit pass: in -> out.  T threads per workgroup, WC = ceil(count/T) workgroups
 * (AbstractKernel.ts:41-47).  local_shuffle reorders `in` in place first, exactly like
 * RadixSortLocalShuffle.ts:94-116 (so `in` is modified, as in the reference). */
static int rso_radix_pass(uint32_t* in_k, uint32_t* in_v, uint32_t* out_k, uint32_t* out_v,
                          uint64_t count, uint32_t bit, uint32_t T, int local_shuffle,
                          uint32_t* local_prefix, uint32_t* block_sums, uint32_t* tmp_k,
                          uint32_t* tmp_v) {
    const uint64_t WC = (count + T - 1) / T;
    for (uint64_t wg = 0; wg < WC; ++wg) {
        const uint64_t WID = wg * T;
        const uint64_t last = (count - WID < T ? count - WID : T);   /* LAST_THREAD+1, RadixSort.ts:71-74 */
        uint32_t cnt[4] = {0, 0, 0, 0};
        /* Hillis-Steele exclusive scan of (digit==b) over the active threads == running count
         * (RadixSort.ts:81-108); block_sums digit-major (RadixSort.ts:110-114). */
        for (uint64_t t = 0; t < last; ++t) {
            uint32_t d = (in_k[WID + t] >> bit) & 3u;               /* RadixSort.ts:61-62 */
            local_prefix[WID + t] = cnt[d]++;
        }
        for (uint32_t b = 0; b < 4; ++b) block_sums[b * WC + wg] = cnt[b];
        if (local_shuffle) {
            /* s_prefix_sum_scan = exclusive scan of the block's digit totals
             * (RadixSortLocalShuffle.ts:94-106); in-place shuffle (:108-116). */
            uint32_t scan[4], s = 0;
            for (uint32_t b = 0; b < 4; ++b) { scan[b] = s; s += cnt[b]; }
            for (uint64_t t = 0; t < last; ++t) {
                uint32_t k = in_k[WID + t];
                uint32_t d = (k >> bit) & 3u;
                uint32_t np = local_prefix[WID + t] + scan[d];
                tmp_k[np] = k;
                if (in_v) tmp_v[np] = in_v[WID + t];
            }
            for (uint64_t t = 0; t < last; ++t) {
                in_k[WID + t] = tmp_k[t];
                if (in_v) in_v[WID + t] = tmp_v[t];
                /* local_prefix_sums[WID+new_pos] = prefix_sum: recompute the rank of the
                 * shuffled element (same value, since the shuffle is a stable digit split). */
            }
            uint32_t c2[4] = {0, 0, 0, 0};
            for (uint64_t t = 0; t < last; ++t)
                local_prefix[WID + t] = c2[(in_k[WID + t] >> bit) & 3u]++;
        }
    }
    int rc = rso_prefix_sum_blelloch(block_sums, 4 * WC, T);   /* AbstractRadixSortKernel.ts:240 */
    if (rc) return rc;
    for (uint64_t gid = 0; gid < count; ++gid) {               /* RadixSortReorder.ts:86-101 */
        uint64_t wg = gid / T;
        uint32_t k = in_k[gid];
        uint32_t d = (k >> bit) & 3u;
        uint64_t pos = (uint64_t)block_sums[d * WC + wg] + local_prefix[gid];
        out_k[pos] = k;
        if (in_v) out_v[pos] = in_v[gid];
    }
    return 0;
}

/* Sort keys[0..count) (and values, if non-null) in place by their low bit_count bits, as
 * RadixSortBufferKernel.dispatch does without check_order.  Returns 0, or <0 on invalid
 * arguments (T not a power of two: PrefixSumKernel.ts:33-35; bit_count not a multiple of 4:
 * README.md:97, quirk Q4 rejected). */
RSO_API int rso_radix_sort_literal(uint32_t* keys, uint32_t* values, uint64_t count,
                                   uint32_t bit_count, uint32_t T, int local_shuffle) {
    if (T == 0 || (T & (T - 1))) return -1;
    if (bit_count == 0 || bit_count > 32 || (bit_count % 4)) return -3;
    if (count == 0) return 0;
    const uint64_t WC = (count + T - 1) / T;
    uint32_t* tmp_keys = (uint32_t*)malloc(4 * count);
    uint32_t* tmp_vals = values ? (uint32_t*)malloc(4 * count) : NULL;
    uint32_t* local_prefix = (uint32_t*)malloc(4 * count);
    uint32_t* block_sums = (uint32_t*)malloc(4 * 4 * WC);
    uint32_t* sk = (uint32_t*)malloc(4 * (size_t)T);
    uint32_t* sv = (uint32_t*)malloc(4 * (size_t)T);
    int rc = 0;
    if (!tmp_keys || (values && !tmp_vals) || !local_prefix || !block_sums || !sk || !sv) rc = -2;
    for (uint32_t bit = 0; rc == 0 && bit < bit_count; bit += 2) {
        int even = (bit % 4) == 0;                             /* AbstractRadixSortKernel.ts:95-98 */
        uint32_t* ik = even ? keys : tmp_keys;
        uint32_t* iv = even ? values : tmp_vals;
        uint32_t* ok = even ? tmp_keys : keys;
        uint32_t* ov = even ? tmp_vals : values;
        rc = rso_radix_pass(ik, iv, ok, ov, count, bit, T, local_shuffle, local_prefix,
                            block_sums, sk, sv);
    }
    free(tmp_keys); free(tmp_vals); free(local_prefix); free(block_sums); free(sk); free(sv);
    return rc;
}

/* ---- closed form ------------------------------------------------------------------------ */

static inline uint32_t rso_mask(uint32_t bit_count) {
    return bit_count >= 32 ? 0xFFFFFFFFu : ((1u << bit_count) - 1u);
}

/* Stable ascending sort by (key & mask): an LSD counting sort over 8-bit digits of the masked
 * key, which is stable by construction.  Independent of the pass structure above. */
RSO_API int rso_stable_sort_masked(uint32_t* keys, uint32_t* values, uint64_t count,
                                   uint32_t bit_count) {
    if (bit_count == 0 || bit_count > 32) return -3;
    if (count <= 1) return 0;
    const uint32_t mask = rso_mask(bit_count);
    uint32_t* tk = (uint32_t*)malloc(4 * count);
    uint32_t* tv = values ? (uint32_t*)malloc(4 * count) : NULL;
    if (!tk || (values && !tv)) { free(tk); free(tv); return -2; }
    uint32_t *ik = keys, *iv = values, *ok = tk, *ov = tv;
    for (uint32_t shift = 0; shift < bit_count; shift += 8) {
        uint64_t hist[257];
        memset(hist, 0, sizeof(hist));
        for (uint64_t i = 0; i < count; ++i) hist[(((ik[i] & mask) >> shift) & 255u) + 1]++;
        for (int d = 0; d < 256; ++d) hist[d + 1] += hist[d];
        for (uint64_t i = 0; i < count; ++i) {
            uint64_t p = hist[((ik[i] & mask) >> shift) & 255u]++;
            ok[p] = ik[i];
            if (iv) ov[p] = iv[i];
        }
        uint32_t* t;
        t = ik; ik = ok; ok = t;
        t = iv; iv = ov; ov = t;
    }
    if (ik != keys) {
        memcpy(keys, ik, 4 * count);
        if (values) memcpy(values, iv, 4 * count);
    }
    free(tk); free(tv);
    return 0;
}

/* 1 if keys[0..count) is non-decreasing in (key & mask), checking every adjacent pair
 * (CheckSort.ts:102-113 with quirks Q1/Q2 fixed). */
RSO_API int rso_is_sorted_masked(const uint32_t* keys, uint64_t count, uint32_t bit_count) {
    const uint32_t mask = rso_mask(bit_count);
    for (uint64_t i = 1; i < count; ++i)
        if ((keys[i - 1] & mask) > (keys[i] & mask)) return 0;
    return 1;
}

/* Stable-sort-with-values validity check used on large outputs: keys sorted (masked), the
 * values a permutation given values_in = iota, keys_out[i] == keys_in[values_out[i]], and
 * equal masked keys carry increasing values (stability).  Returns 0 on success, else the
 * 1-based index of the first violation (or -1 on allocation failure). */
RSO_API int64_t rso_verify_stable_iota(const uint32_t* keys_in, const uint32_t* keys_out,
                                       const uint32_t* values_out, uint64_t count,
                                       uint32_t bit_count) {
    const uint32_t mask = rso_mask(bit_count);
    uint8_t* seen = (uint8_t*)calloc(count ? count : 1, 1);
    if (!seen) return -1;
    int64_t bad = 0;
    for (uint64_t i = 0; i < count && !bad; ++i) {
        uint32_t v = values_out[i];
        if (v >= count || seen[v]) { bad = (int64_t)i + 1; break; }
        seen[v] = 1;
        if (keys_out[i] != keys_in[v]) { bad = (int64_t)i + 1; break; }
        if (i) {
            uint32_t a = keys_out[i - 1] & mask, b = keys_out[i] & mask;
            if (a > b || (a == b && values_out[i - 1] > v)) { bad = (int64_t)i + 1; break; }
        }
    }
    free(seen);
    return bad;
}
