/*
 * rsort.h — C ABI of the MI355X-native 4-way LSD radix sort (librsort.so).
 *
 * This is the drop-in boundary for the reference's hot path,
 *   new RadixSortKernel({device, keys, values, count, bit_count, workgroup_size,
 *                        check_order, local_shuffle, avoid_bank_conflicts}).dispatch(pass)
 * (README.md:72-88; shipped as RadixSortBufferKernel, src/kernels/radix-sort/
 * RadixSortBufferKernel.ts:9-32, AbstractRadixSortKernel.ts:14-19,221-227) and for the
 * exported PrefixSumKernel (src/kernels/PrefixSumKernel.ts:24-43,147-158).
 *
 * Plain C: pointers, sizes and status codes only; no exceptions cross it.  Device pointers are
 * HIP device allocations (from rs_malloc, hipMalloc or torch); `stream` is a hipStream_t passed
 * as void* (NULL = the default stream).  All sort/scan calls are asynchronous on `stream`, like
 * the reference's dispatch(), which only encodes work (AbstractRadixSortKernel.ts:221-247).
 *
 * The matching host bindings (Node N-API addon, Python ctypes) are in INTEGRATION.md.
 */
#ifndef RSORT_H
#define RSORT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSORT_VERSION_MAJOR 0
#define RSORT_VERSION_MINOR 6

typedef enum rs_status {
    RS_OK = 0,
    RS_ERR_INVALID_ARG = 1,   /* null pointer, count too large, bad bit range ... */
    RS_ERR_NOT_POW2 = 2,      /* workgroup_x*workgroup_y not a power of two
                                 (PrefixSumKernel.ts:33-35) */
    RS_ERR_BIT_COUNT = 3,     /* bit_count not a multiple of 4 in [4, 32] (README.md:97;
                                 the reference leaves this unchecked) */
    RS_ERR_HIP = 4,           /* a HIP runtime call failed (message in rs_last_error) */
    RS_ERR_OUT_OF_MEMORY = 5,
    RS_ERR_CAPACITY = 6,      /* count exceeds the plan's capacity */
    RS_ERR_DEVICE = 7         /* a device-side failure of an EARLIER sort on this plan: a bounded
                                 inter-workgroup wait of the one-sweep pass timed out, so that
                                 sort's output is invalid (reported once, by rs_plan_check or by
                                 the next rs_plan_sort / rs_plan_sort_n on the plan, which then
                                 enqueues nothing).  The reference's dispatch never produces
                                 output silently wrong (AbstractRadixSortKernel.ts:221-247). */
} rs_status;

/* rs_plan_desc.flags — the reference's boolean options. */
#define RS_FLAG_HAS_VALUES           0x1u  /* data.values present (RadixSortBufferKernel.ts:25-28) */
#define RS_FLAG_CHECK_ORDER          0x2u  /* check_order (AbstractRadixSortKernel.ts:249-276) */
#define RS_FLAG_LOCAL_SHUFFLE        0x4u  /* local_shuffle (RadixSortBufferKernel.ts:38-44) */
#define RS_FLAG_AVOID_BANK_CONFLICTS 0x8u  /* avoid_bank_conflicts (PrefixSumKernel.ts:37-40) */
#define RS_FLAG_INTERLEAVED          0x10u /* RadixSortTextureKernel layout: `keys` points to count
                                              8-byte (key, value) records (the rg32uint texels,
                                              RadixSortTextureKernel.ts:15-35, RadixSortReorder.ts:
                                              42-63), sorted in place; `values` must be NULL.
                                              Implies values (RadixSortTextureKernel.ts:27-29). */

/* Options of one sort plan (one RadixSortKernel instance). */
typedef struct rs_plan_desc {
    int32_t  device;        /* HIP device ordinal                           (options.device) */
    uint64_t count;         /* elements to sort, < 2^32                     (options.count) */
    uint32_t bit_count;     /* sort by the low bit_count bits; 0 -> 32     (options.bit_count) */
    uint32_t workgroup_x;   /* 0 -> 16; x*y must be a power of two <= 1024 (options.workgroup_size) */
    uint32_t workgroup_y;   /* 0 -> 16 */
    uint32_t flags;         /* RS_FLAG_* */
    uint32_t radix_bits;    /* digit bits per HBM pass: 0 = auto (fused: 8-bit digits, four
                               4-way splits per pass); 2 = one 4-way split per pass, the
                               reference's pass structure (bit_count/2 passes); 4 or 8 */
    uint32_t usage;         /* RS_USAGE_SORT (0): every entry point; RS_USAGE_PARTITION: only
                               rs_plan_hist16 and the rs_plan_partition* passes (the multi-GPU
                               sender side) - no ping-pong copy is allocated */
} rs_plan_desc;

#define RS_USAGE_SORT      0u
#define RS_USAGE_PARTITION 1u

typedef struct rs_plan rs_plan;

/* Per-plan facts (for benches / INTEGRATION tooling). */
typedef struct rs_plan_info {
    uint32_t passes;            /* global HBM passes per sort (even) */
    uint32_t digit_bits[16];    /* digit width of each pass */
    uint32_t tile_keys;         /* keys per tile of the rank/scatter kernel */
    uint32_t grid_blocks;       /* workgroups of the histogram / scatter kernels */
    uint64_t workspace_bytes;   /* device bytes owned by the plan */
    uint32_t rank_mode;         /* in-wave stable ranking: 0 = lane-ordered LDS atomics (one
                                   ds_add_rtn_u32 per key), 1 = ballot-match ranking */
    int32_t  lane_order_selftest;  /* the device's LDS-atomic lane-order self-test (run once per
                                   device at the first plan creation): 1 passed, 0 failed (plans
                                   then use rank_mode 1), -1 could not run */
} rs_plan_info;

/* Kernel kinds reported by rs_plan_kernel_times(). */
enum {
    RS_KERNEL_HISTOGRAM = 0,    /* per-block digit histogram          (RadixSort.ts:50-126) */
    RS_KERNEL_SCAN = 1,         /* digit x block exclusive scan       (PrefixSum.ts:13-106) */
    RS_KERNEL_SCATTER = 2,      /* rank + local shuffle + scatter     (RadixSortReorder.ts:80-102,
                                                                       RadixSortLocalShuffle.ts) */
    RS_KERNEL_CHECK = 3,        /* order check                        (CheckSort.ts:70-145) */
    RS_KERNEL_BUCKET = 4,       /* hybrid MSD path: in-LDS sort of every 16-bit bucket */
    RS_KERNEL_FALLBACK = 5,     /* hybrid MSD path: the LSD passes it enqueues as its fallback
                                   (gated off on the device unless it is taken) */
    RS_KERNEL_SPLIT = 6,        /* hybrid MSD path: the bucket split of over-full 16-bit buckets
                                   (skewed keys; one span per sort, gated off for spread keys) */
    RS_KERNEL_PRESORTED = 7,    /* hybrid MSD path with check_order: the nearly-sorted path (mark
                                   the displaced keys, sort them, merge; one span per sort, gated
                                   off on the device when the input is not nearly sorted) */
    RS_KERNEL_KINDS = 8
};

/* ---- errors / versions ------------------------------------------------------------------ */
const char* rs_last_error(void);               /* thread-local message of the last failure */
const char* rs_status_string(rs_status s);
uint32_t    rs_version(void);                  /* (major << 16) | minor */

/* ---- sort plans (RadixSortKernel) ------------------------------------------------------- */
/* Validate options, allocate the workspace (tmp keys/values, block histograms) on `device`. */
rs_status rs_plan_create(const rs_plan_desc* desc, rs_plan** out);
/* Sort keys[0..count) (and values[0..count) when RS_FLAG_HAS_VALUES; records[0..count) when
 * RS_FLAG_INTERLEAVED) in place, ascending and stable by (key & (2^bit_count - 1)); elements
 * at index >= count are untouched.  Float32 keys sort by raw bit pattern (README.md:9).
 * Asynchronous on `stream`. */
rs_status rs_plan_sort(rs_plan* plan, void* keys, void* values, void* stream);
/* Same, for n <= the plan's count (multi-GPU receive buffers vary per call). */
rs_status rs_plan_sort_n(rs_plan* plan, void* keys, void* values, uint64_t n, void* stream);
/* Out-of-place sort: in_keys[0..n) (+ in_values) are only read; the stable sorted result is
 * written to out_keys[0..n) (+ out_values).  A plan with separate arrays or keys only, without
 * check_order; n <= capacity.  Pass 0 reads the input, the last pass writes the output: the same
 * HBM traffic as rs_plan_sort, no copy (the multi-GPU sorts at world size 1 use it). */
rs_status rs_plan_sort_copy(rs_plan* plan, const void* in_keys, const void* in_values,
                            void* out_keys, void* out_values, uint64_t n, void* stream);
/* One stable scatter pass by digit (key >> shift) & (2^bits - 1), bits <= 8, out of place:
 * in[0..n) -> out[0..n).  Writes the 2^bits digit totals (u32) to d_hist (device, may be
 * NULL).  The bucket-exchange partition step of the multi-GPU sort. */
rs_status rs_plan_partition(rs_plan* plan, const void* in_keys, const void* in_values,
                            void* out_keys, void* out_values, uint64_t n, uint32_t shift,
                            uint32_t bits, void* d_hist, void* stream);
/* rs_plan_partition given the digit totals of in[0..n) (device, 2^bits u32, e.g. from
 * rs_histogram): where the one-sweep scatter wins (values, n >= 12M) the pass then reads the keys
 * once instead of twice (no per-tile histogram, decoupled look-back); otherwise the same as
 * rs_plan_partition.  Multi-GPU partition step (the histogram is exchanged anyway). */
rs_status rs_plan_partition_totals(rs_plan* plan, const void* in_keys, const void* in_values,
                                   void* out_keys, void* out_values, uint64_t n, uint32_t shift,
                                   uint32_t bits, const void* d_totals, void* stream);
/* Multi-GPU record path.  rs_plan_partition_records: the stable partition of separate key / value
 * arrays in[0..n) by the digit (key >> shift) & (2^bits - 1), bits <= 8, written as n 8-byte
 * (key, value) records (one message per peer carries keys and values together); d_totals = the
 * digit totals of the input (rs_histogram) or NULL (counted here).  rs_plan_sort_records: the
 * whole stable sort of n records (the received buckets) into separate arrays keys_out /
 * values_out; records[] is only read.  Both need a plan with RS_FLAG_HAS_VALUES and capacity >= n;
 * check_order does not apply. */
rs_status rs_plan_partition_records(rs_plan* plan, const void* in_keys, const void* in_values,
                                    void* out_records, uint64_t n, uint32_t shift, uint32_t bits,
                                    const void* d_totals, void* stream);
rs_status rs_plan_sort_records(rs_plan* plan, const void* records, void* keys_out,
                               void* values_out, uint64_t n, void* stream);
/* rs_plan_sort_records with a hint: every key lies in [key_lo, key_hi] (a group sort's received
 * top-digit buckets).  The sort may then work on the range-relative bits key - key_lo only (the
 * hybrid MSD path over a rank's buckets); a key outside the range is detected on the device and
 * the 32-bit passes run instead, so the result is always the stable sort.  key_lo <= key_hi. */
rs_status rs_plan_sort_records_range(rs_plan* plan, const void* records, void* keys_out,
                                     void* values_out, uint64_t n, uint32_t key_lo, uint32_t key_hi,
                                     void* stream);
/* Multi-GPU bucket path (52 B/key per rank: the single-GPU hybrid sort's bytes, split across the
 * exchange).  Sender: rs_plan_hist16 counts keys[0..n) (4-byte keys; records with
 * RS_FLAG_INTERLEAVED) per 16-bit bucket key >> 16 in one read: d_hist16[0..65536) = the bucket
 * counts, d_hist16[65536..65792) = the top-byte totals (their sums; what rs_plan_partition_records
 * takes as d_totals).  The senders' tables are all-gathered: every receiver then knows the layout of
 * what it will receive.  Receiver: rs_plan_sort_region sorts n records whose keys all have a top
 * byte in [top_lo, top_hi) and that arrive grouped by top byte in increasing order (each group in
 * global input order: the stable partition's output, source ranks in order) into separate arrays;
 * d_hist16 (device, 65536 u32) = the region's count per 16-bit bucket, 0 outside
 * [top_lo << 8, top_hi << 8).  The top-byte pass is the senders' partition, so the region takes
 * only the next-byte pass (per top-byte segment) and the in-LDS bucket sort; a bucket larger than
 * the largest bucket tile is split on the device (the bucket split).  A table that does not describe
 * the records (counts that do not add up to n, counts outside [top_lo, top_hi)) is reported as
 * RS_ERR_DEVICE by rs_plan_check / the next call; with the split off (rs_plan_debug.split = 0) the
 * device sorts such a region with the LSD passes instead.  records[] is only read. */
#define RS_HIST16_WORDS 65792u
rs_status rs_plan_hist16(rs_plan* plan, const void* keys, uint64_t n, void* d_hist16, void* stream);
rs_status rs_plan_sort_region(rs_plan* plan, const void* records, void* keys_out, void* values_out,
                              uint64_t n, const void* d_hist16, uint32_t top_lo, uint32_t top_hi,
                              void* stream);
rs_status rs_plan_info_get(const rs_plan* plan, rs_plan_info* info);
/* Which path the plan's last sort took (waits for it): the hybrid MSD path's choice is made on
 * the device (k_msd_plan's gate words), so this reads it back.  Diagnostics and tests; the result
 * never depends on it. */
enum {
    RS_PATH_NONE = 0,             /* no sort yet */
    RS_PATH_LSD = 1,              /* the LSD passes directly (small n, keys-only < 16M, radix_bits != 8 ...) */
    RS_PATH_HYBRID = 2,           /* hybrid MSD: top-byte pass, next-byte pass, in-LDS bucket sort */
    RS_PATH_HYBRID_FALLBACK = 3,  /* the hybrid path's LSD fallback (a key outside a range hint, or
                                     a bucket over the tile with the bucket split off) */
    RS_PATH_IN_ORDER = 4,         /* check_order found the input sorted: nothing moved */
    RS_PATH_PRESORTED = 5         /* check_order found the input nearly sorted: its displaced keys
                                     were extracted, sorted and merged back (no radix pass) */
};
rs_status rs_plan_last_path(rs_plan* plan, uint32_t* path);
/* The presorted path of the plan's last sort (waits for it): *marked = the elements its order scan
 * marked and extracted, *moved = the elements its merge wrote (each read and written once); both 0
 * when that sort did not take the path (0.6). */
rs_status rs_plan_presorted_counts(rs_plan* plan, uint64_t* marked, uint64_t* moved);
/* How deep the hybrid path's last sort split over-full 16-bit buckets (skewed keys, e.g. f32 in
 * [0, 1) or few distinct keys): 0 not at all, 2 by byte 1 (24-bit sub-buckets sorted in LDS), 3 some
 * sub-buckets by byte 0 as well.  Waits for the sort.  Diagnostics: the result never depends on it. */
rs_status rs_plan_last_split(rs_plan* plan, uint32_t* levels);
/* Kernel timing: when enabled, every launch of the plan is bracketed by HIP events on the
 * launch stream and per-kind durations are accumulated (read after synchronising). */
rs_status rs_plan_set_profiling(rs_plan* plan, int enable);
/* Events around the launches of the kinds in kind_mask only (bit k = RS_KERNEL_k; 0 disables):
 * a timed run brackets just the kernel it reports, the other launch groups run back to back. */
rs_status rs_plan_set_profiling_kinds(rs_plan* plan, uint32_t kind_mask);
rs_status rs_plan_kernel_times(rs_plan* plan, double ms[RS_KERNEL_KINDS],
                               uint64_t launches[RS_KERNEL_KINDS]);
rs_status rs_plan_reset_kernel_times(rs_plan* plan);
/* Device-side error word of the plan (synchronises the device): 0 = ok; bit 0 = a bounded
 * inter-workgroup wait of the one-sweep scatter timed out (that sort's result is invalid). */
rs_status rs_plan_device_errors(rs_plan* plan, uint32_t* errors);
/* Wait for the plan's last enqueued sort and report any device-side failure since the last
 * report: RS_OK, or RS_ERR_DEVICE (cleared by the report).  The façades call it at their
 * synchronising points (mapAsync / Python check()). */
rs_status rs_plan_check(rs_plan* plan);
/* Bound of every inter-workgroup wait of the one-sweep pass, in s_sleep(1) periods (default
 * 2^20, ~ms).  0 makes any wait on a not-yet-published predecessor time out at once: the
 * failure path's test (rs_plan_check must then report it). */
rs_status rs_plan_set_wait_limit(rs_plan* plan, uint32_t sleeps);
/* Test / diagnostics only: force the plan onto one of the paths it would otherwise pick by size
 * (so parity tests can cover every kernel).  Never changes a result, only which kernels run.  The
 * library reads no environment variables: a caller's environment cannot change the path.  Each
 * field: -1 = keep the plan's own choice.  Call before the plan's first sort (it only selects
 * among the resources rs_plan_create allocated; a path whose workspace is absent stays off). */
typedef struct rs_plan_debug {
    int32_t rank;           /* 0 lane-ordered LDS-atomic ranking, 1 ballot-match ranking */
    int32_t tile;           /* 0 large tiles (16K keys), 1 small tiles (4K keys) at every size */
    int32_t onesweep;       /* 0 histogram / scan / scatter passes, 1 one-sweep passes */
    int32_t msd;            /* 0 the hybrid MSD path off (LSD passes only), 1 on where it applies */
    int32_t keys_cfg;       /* keys-only LSD tiles: 0 1024 x 16, 1 512 x 32 */
    int32_t msd_keys_cfg;   /* keys-only hybrid pass tiles: 0 1024 x 16, 1 512 x 32, 2 1024 x 32 */
    int32_t kbucket_wave;   /* keys-only bucket pass: 0 a workgroup per bucket, 1 a wave per bucket */
    int32_t selftest_fail;  /* 1: treat the lane-order self-test as failed (ballot ranking,
                               rs_plan_info.lane_order_selftest = 0) */
    int32_t split;          /* hybrid path, 16-bit buckets over the bucket tile (skewed keys): 1 split
                               them (default), 0 take the LSD fallback for the whole sort */
    int32_t presorted;      /* hybrid path with check_order: 1 the nearly-sorted path where the
                               device finds it applies (default), 0 never (the radix passes) */
    int32_t xcd;            /* hybrid MSD passes with values: XCD-local tile streams on 1 both passes,
                               2 pass 0 only, 3 pass 1 only; 0 one global tile counter (the default;
                               added in 0.6) */
    int32_t high_half;      /* test hook: 1 the hybrid path's bucket kernels read records buffers
                               placed at an address whose low 32 bits are >= 2^31 (needs spare plan
                               capacity: n + 2^28 records; RS_ERR_CAPACITY otherwise) (0.6) */
} rs_plan_debug;
rs_status rs_plan_set_debug(rs_plan* plan, const rs_plan_debug* debug);
void      rs_plan_destroy(rs_plan* plan);     /* frees the workspace (reference quirk Q9) */

/* ---- prefix sum (PrefixSumKernel) ------------------------------------------------------- */
typedef struct rs_scan_plan rs_scan_plan;
/* workgroup_x*workgroup_y must be a power of two (PrefixSumKernel.ts:33-35). */
rs_status rs_scan_plan_create(int32_t device, uint64_t count, uint32_t workgroup_x,
                              uint32_t workgroup_y, uint32_t flags, rs_scan_plan** out);
/* In-place exclusive scan (mod 2^32) of data[0..count); data[count..] untouched. */
rs_status rs_scan_plan_run(rs_scan_plan* plan, void* data, void* stream);
/* The scan is one pass (one read and one write of the data: tiles in order, each adding its
 * predecessors' sums found by a bounded look-back).  rs_scan_plan_check waits for the plan's last
 * scan and returns RS_ERR_DEVICE (once) if a look-back wait of a scan since the last check timed
 * out (that scan's output is invalid); rs_scan_plan_set_wait_limit bounds the waits (s_sleep
 * periods, default 2^20; 0: any wait on an unpublished predecessor times out - tests). */
rs_status rs_scan_plan_check(rs_scan_plan* plan);
rs_status rs_scan_plan_set_wait_limit(rs_scan_plan* plan, uint32_t sleeps);
/* PrefixSumKernel.dispatch(pass, dispatchSizeBuffer, offset) (PrefixSumKernel.ts:147-158): the
 * scan as above, gated on the device: dispatch_size_buffer (device memory) holds u32 (x, y, z)
 * workgroup triples from byte `offset`, one per pipeline of rs_scan_plan_dispatch_chain; the scan
 * runs iff the first triple has no zero entry (the reference's check-sort zeroes the chain to
 * skip work).  The HIP scan is one fused chain, so later triples are not read: it runs whole or
 * not at all.  Nothing is read on the host. */
rs_status rs_scan_plan_run_indirect(rs_scan_plan* plan, void* data, const void* dispatch_size_buffer,
                                    uint64_t offset, void* stream);
/* The reference's dispatch chain for this plan (PrefixSumKernel.getDispatchChain,
 * PrefixSumKernel.ts:135-137): (x, y, 1) per pipeline, written to out[0..max_words); returns the
 * number of words of the whole chain. */
uint32_t  rs_scan_plan_dispatch_chain(const rs_scan_plan* plan, uint32_t* out, uint32_t max_words);
void      rs_scan_plan_destroy(rs_scan_plan* plan);

/* ---- multi-GPU group sort (one process, several devices) ------------
 * The reference has no multi-device path; this is the sharded form of the same sort for an
 * input spread over the GPUs of one node (BASELINE config 5), callable from a single host
 * process (the Node addon, a C/C++ host) the way ncclCommInitAll + ncclGroupStart/End drive
 * several devices from one thread.  Rank r's input is keys[r][0..counts[r]) (+ values[r]) on
 * devices[r]; after rs_group_sort, rank r holds slice r of the global stable ascending order by
 * the 32-bit key (rank-ordered concatenation = the sorted whole).  The exchange is the first
 * MSD pass of the single-GPU hybrid sort split across the ranks (52 B/key per rank with values):
 * rs_plan_hist16 per rank (16-bit bucket table + top-byte totals, one key read) -> tables to the
 * host -> whole-top-byte ownership (~1/world of the keys per rank, equal keys never split) and
 * `rounds` groups of top bytes per rank -> stable partition by the top byte (records with values;
 * the hybrid sort's pass 0) -> `rounds` exchange rounds, one message per (source, top byte) chunk,
 * laid out round-major, then top byte, then source -> each round's region sorted by
 * rs_plan_sort_region (next-byte pass + in-LDS bucket sort) as soon as it has landed, while later
 * rounds are on the wire.  Keys only: the same exchange, each region sorted by rs_plan_sort_n. */
typedef struct rs_group rs_group;

#define RS_TRANSPORT_RCCL 0u   /* ncclCommInitAll + ncclGroupStart / ncclSend / ncclRecv (xGMI) */
#define RS_TRANSPORT_COPY 1u   /* peer copies (hipMemcpyPeerAsync, DMA over xGMI); the only one
                                  that accepts a device listed twice (virtual ranks on one GPU) */

typedef struct rs_group_desc {
    uint64_t capacity;      /* largest counts[r] a sort may pass (partition workspace); receive
                               buffers and local sort plans grow on demand */
    uint32_t flags;         /* RS_FLAG_HAS_VALUES or 0 (keys only); nothing else */
    uint32_t transport;     /* RS_TRANSPORT_* */
    uint32_t top_bits;      /* exchange digit width: 8 or 0 (-> 8, the top byte) */
    uint32_t rounds;        /* exchange rounds (bucket groups per rank), 1..16; 0 -> 4 */
} rs_group_desc;

/* Create the communicators / streams / plans for `world` ranks on devices[0..world). */
rs_status rs_group_create(int32_t world, const int32_t* devices, const rs_group_desc* desc,
                          rs_group** out);
/* Sort.  keys[r] / values[r] (values NULL without RS_FLAG_HAS_VALUES) are device pointers on
 * devices[r], only read.  streams: NULL, or world hipStream_t (as void*): the group's work is
 * ordered after each caller stream and each caller stream after the group's work.  Blocks the
 * host until the bucket counts are known (the exchange sizes, as ncclAllToAllv's host size
 * arrays); the exchange and the local sorts stay asynchronous. */
rs_status rs_group_sort(rs_group* g, void* const* keys, void* const* values,
                        const uint64_t* counts, void* const* streams);
/* Rank r's slice of the last sort: group-owned device buffers (valid until the next sort or
 * destroy), *count keys.  Read them after rs_group_synchronize or on a stream passed to the
 * sort.  values is NULL for a keys-only group. */
rs_status rs_group_result(const rs_group* g, int32_t rank, void** keys, void** values,
                          uint64_t* count);
/* Wait for the last sort on every rank; RS_ERR_DEVICE if any of its kernels failed on the
 * device (rs_plan_check of every rank's plans). */
rs_status rs_group_synchronize(rs_group* g);
/* Per-rank timing of the group sorts (diagnostics; what an N-GPU run needs to explain itself:
 * where the step's time goes, the exchange time and its xGMI rate).  rs_group_set_profiling(g, 1)
 * records timing events on every rank's streams from the next rs_group_sort on (a few per round);
 * rs_group_times_get waits for the last sort and reads rank r's: ms since the sort's start on the
 * rank's sort stream.  round_done_ms[j]: the rank's comm stream finished round j (RCCL: its sends
 * and receives of round j; peer copies: the copies it sent).  bytes_*: the rank's off-rank
 * exchange bytes (its own chunks are device copies). */
typedef struct rs_group_times {
    uint32_t rounds;              /* rounds of the last sort (0: world size 1, nothing exchanged) */
    float    hist16_ms;           /* the 16-bit table read */
    float    partition_ms;        /* the top-byte partition (the sort's first MSD pass) */
    float    round_done_ms[16];
    float    region_sorted_ms[16];/* region j's local sort done */
    float    done_ms;             /* the rank's whole sort */
    uint64_t bytes_sent;
    uint64_t bytes_recv;
} rs_group_times;
rs_status rs_group_set_profiling(rs_group* g, int enable);
rs_status rs_group_times_get(rs_group* g, int32_t rank, rs_group_times* out);
void      rs_group_destroy(rs_group* g);
/* The host-side bucket plan, a pure function (identical on every rank; no device needed):
 * hist_all[r * buckets + b] = rank r's count of bucket b.  Writes bounds[0..world] (rank q owns
 * buckets [bounds[q], bounds[q+1])) and cuts[q * (rounds + 1) + i], i <= rounds (round i of rank
 * q = buckets [cuts[.. + i], cuts[.. + i + 1])), whole buckets of ~equal global key counts. */
rs_status rs_group_plan(int32_t world, uint32_t buckets, uint32_t rounds, const uint64_t* hist_all,
                        uint32_t* bounds, uint32_t* cuts);

/* ---- device memory / streams (the reference's createBuffers / queue analogue) ---------- */
rs_status rs_device_count(int32_t* n);
rs_status rs_malloc(int32_t device, uint64_t bytes, void** ptr);
rs_status rs_free(void* ptr);
rs_status rs_memcpy_h2d(void* dst, const void* src, uint64_t bytes, void* stream);
rs_status rs_memcpy_d2h(void* dst, const void* src, uint64_t bytes, void* stream);
rs_status rs_memcpy_d2d(void* dst, const void* src, uint64_t bytes, void* stream);
rs_status rs_stream_create(int32_t device, void** stream);
rs_status rs_stream_destroy(void* stream);
rs_status rs_stream_synchronize(void* stream);

/* ---- timestamps (the reference's timestamp QuerySet, example/tests.ts:247-285; the demo
 * times kernel.dispatch between beginningOfPass / endOfPass writes, example/index.ts:124-146) */
rs_status rs_event_create(void** event);
rs_status rs_event_destroy(void* event);
rs_status rs_event_record(void* event, void* stream);
/* Milliseconds between two recorded events; waits for `end` to complete. */
rs_status rs_event_elapsed_ms(void* start, void* end, float* ms);

/* ---- synthetic inputs (bench / tests) --------------------------------------------------- */
/* dst[i] = low32(splitmix64_finaliser(seed * 0xD1B54A32D192ED03 + start + i)), i < n. */
rs_status rs_fill_random_u32(void* dst, uint64_t n, uint64_t seed, uint64_t start, void* stream);
/* dst[i] = first + i (u32 wrap), i < n. */
rs_status rs_fill_iota_u32(void* dst, uint64_t n, uint32_t first, void* stream);
/* d_hist[d] = #{i < n : ((keys[i] >> shift) & (2^bits - 1)) == d}, 1 <= bits <= 8 (device u32,
 * 2^bits words, overwritten).  The multi-GPU sort's bucket counts before the exchange. */
rs_status rs_histogram(const void* keys, uint64_t n, uint32_t shift, uint32_t bits, void* d_hist,
                       void* stream);
/* Device-side order check of keys[0..n) by (key & mask): writes 1 (sorted) or 0 to *d_flag
 * (device u32).  Checks every adjacent pair. */
rs_status rs_is_sorted(const void* keys, uint64_t n, uint32_t bit_count, void* d_flag,
                       void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RSORT_H */
