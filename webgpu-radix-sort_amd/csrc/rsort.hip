// rsort.hip — C ABI (include/rsort.h) over the gfx950 radix-sort kernels (rs_kernels.hpp).
//
// Mirrors the reference's host classes:
//   rs_plan_create  ~ new RadixSortBufferKernel(opts)   (RadixSortBufferKernel.ts:21-32:
//                     option defaults AbstractRadixSortKernel.ts:52-57, resources :50-71)
//   rs_plan_sort    ~ kernel.dispatch(pass)             (AbstractRadixSortKernel.ts:221-276)
//   rs_scan_plan_*  ~ new PrefixSumKernel(opts).dispatch (PrefixSumKernel.ts:24-43,147-158)
// Every call returns an rs_status; the message of the last failure is kept per thread.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <type_traits>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include <dlfcn.h>

#include "../../include/rsort.h"
#include "rs_internal.h"
#include "rs_kernels.hpp"
#include "rs_presorted.hpp"

#define RS_EXPORT extern "C" __attribute__((visibility("default")))

// Tuning knobs.  The product library reads no environment variables: the per-plan path choices
// the parity tests use to cover every kernel are set through rs_plan_set_debug.  The sweep build
// (`make variants`, tools/sweep.py: -DRS_SWEEP=1) adds the process-wide experiment knobs (RSORT_*
// environment variables) and the alternative kernel instantiations they select; a product build
// compiles neither.
#if !RS_KNOB_OPEN || !defined(RS_P0_SR2)
#undef RS_P0_SR2
#define RS_P0_SR2 0   // experiment: MSD pass 0 over 32K-record tiles in two staging rounds
#endif
#ifndef RS_SWEEP
#define RS_SWEEP 0
#endif
#if RS_SWEEP
static double sweep_knob(const char* name, double dflt) {
    const char* e = getenv(name);
    return e ? atof(e) : dflt;
}
#define RS_KNOB(name, dflt) sweep_knob(name, dflt)
#else
#define RS_KNOB(name, dflt) (dflt)
#endif

namespace {

thread_local std::string g_err;

rs_status fail(rs_status s, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return s;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(e_ == hipErrorOutOfMemory ? RS_ERR_OUT_OF_MEMORY : RS_ERR_HIP, \
                        "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,      \
                        __LINE__);                                                     \
    } while (0)

// Tuned geometry (sweeps in tools/sweep.py).  Two scatter configurations:
//   large: 1024 threads x 16 keys = 16384-key tiles, 145 KiB LDS, one workgroup per CU
//   small:  256 threads x 16 keys =  4096-key tiles,  37 KiB LDS, four workgroups per CU
// and a single-workgroup sort for n <= kTinyMax.
#if !RS_KNOB_OPEN || !defined(RS_SMALL_MAX)
#undef RS_SMALL_MAX
#define RS_SMALL_MAX (12u << 20)  // n below this uses the small-tile configuration
#endif
#if !RS_KNOB_OPEN || !defined(RS_HIST_U)
#undef RS_HIST_U
#define RS_HIST_U 4               // 16-byte loads per lane per histogram iteration (x2 in flight)
#endif
struct TileCfg {
    int block, kpt, tile;
    uint32_t max_grid;
};
constexpr TileCfg kLarge{1024, 16, 16384, 512};
// Words after the digit totals: [16] tile tickets (one per k_onesweep launch slot), [16] error words,
// then [2][8] the hybrid MSD passes' per-XCD tile counters (k_msd_pass XC) and 16 spare
constexpr uint32_t kTicketWords = 64;
constexpr uint32_t kXcdTickets = 32;
#if !RS_KNOB_OPEN || !defined(RS_MSD_LEAN)
#undef RS_MSD_LEAN
#define RS_MSD_LEAN 1    // the MSD passes with values on k_msd_pass (0: k_onesweep)
#endif
constexpr TileCfg kSmall{256, 16, 4096, 1024};
// keys-only at >= 12M keys: the same 16K-key tile from 512 threads x 32 keys (75 KiB LDS), so
// two workgroups share a CU and one's waits (look-back, barriers) overlap the other's work
#if !RS_KNOB_OPEN || !defined(RS_KEYS_BLOCK)
#undef RS_KEYS_BLOCK
#define RS_KEYS_BLOCK 512
#endif
#if !RS_KNOB_OPEN || !defined(RS_KEYS_KPT)
#undef RS_KEYS_KPT
#define RS_KEYS_KPT 32
#endif
constexpr TileCfg kLargeKeys{RS_KEYS_BLOCK, RS_KEYS_KPT, RS_KEYS_BLOCK * RS_KEYS_KPT, 512};
#if RS_SWEEP
// one-sweep passes that read a plan-owned records buffer (padded to whole tiles): 24K-record
// tiles (1024 threads x 24 records, positions packed 16-bit) staged through LDS in two rounds of
// 12K; longer digit runs per tile than 16K tiles (fewer lines shared by two tiles' runs)
constexpr TileCfg kHuge{1024, 24, 24576, 512};
// one-sweep KV tile configurations with two or more workgroups per CU (RSORT_KV_CFG): one
// workgroup's rank / look-back / staging phases overlap another's loads and stores
//   1: 512 threads x 16 = 8K-record tiles (~75 KiB LDS, 2 per CU)
//   2: 512 threads x 32 = 16K-record tiles staged in two rounds of 8K (2 per CU)
//   3: 256 threads x 32 = 8K-record tiles staged in two rounds of 4K (4 per CU)
//   4: 512 threads x 24 = 12K-record tiles staged in two rounds of 6K (2 per CU)
constexpr TileCfg kKv512x16{512, 16, 8192, 1024};
constexpr TileCfg kKv512x32{512, 32, 16384, 1024};
constexpr TileCfg kKv256x32{256, 32, 8192, 2048};
constexpr TileCfg kKv512x24{512, 24, 12288, 1024};
#endif
constexpr uint32_t kMinOnesweepTile = 8192;   // finest one-sweep tile (status words per plan)
constexpr uint64_t kRecPad = 49152;           // records buffers: whole tiles of every config
constexpr uint32_t kTinyMax = 1024 * 16;
// Hybrid MSD path (enqueue_sort_msd): used for key/value arrays and records of kMsdMin ... kMsdMax
// keys when no 16-bit bucket exceeds kBucketCap records (decided on the device); buckets are sorted
// in LDS by k_bucket_sort (tiles sized to the population) or, the largest, k_bucket_sort_wide.
#if !RS_KNOB_OPEN || !defined(RS_MSD_DEFAULT)
#undef RS_MSD_DEFAULT
#define RS_MSD_DEFAULT 1
#endif
constexpr uint64_t kMsdMin = 12ull << 20;
constexpr int kWideKpt = 34;                            // k_bucket_sort_wide: 1024 x 34 records
constexpr uint32_t kBucketCap = 1024u * kWideKpt;       // the largest 16-bit bucket the path sorts
// a uniform population's largest bucket (mean + ~5 sigma) still fits kBucketCap up to here (2^31
// keys: mean 32768, sigma 181); above it the device would always pick the LSD fallback
constexpr uint64_t kMsdMax = 65536ull * 33800;
constexpr uint64_t kMsdWords = 65536ull * 2 + 1024 + 64 + 1024 + 1 + rs::kOverMax +   // hist16, base16,
                                 256ull * rs::kMaxRows;             // segtab, gates, mtot, over, cbase
// The bucket split (rs_kernels.hpp, "splitting over-full buckets"): level 2 takes the 16-bit buckets
// over kBucketCap records, level 3 the 24-bit sub-buckets over kSub8Cap - at most n / (cap + 1) of
// each.  Words: gates [32], huge list [1 + smax2], per level a table [3 smax + 2], arrivals
// [smax + 1] and rows [256 smax].
inline uint32_t split_smax2(uint64_t cap) { return (uint32_t)(cap / (kBucketCap + 1ull) + 1); }
inline uint32_t split_smax3(uint64_t cap) { return (uint32_t)(cap / (rs::kSub8Cap + 1ull) + 1); }
// level 2's tiles (each huge bucket's records in 16K-record tiles: at most one partial per bucket)
inline uint32_t split_midmax(uint64_t cap) { return (uint32_t)(cap / (rs::kSub8Small + 1ull) + 1); }
// runs of small sub-buckets: two consecutive runs of one bucket hold more than kSub8Small records,
// unless a larger sub-bucket (at most cap / (kSub8Small + 1) of them) or the bucket's end is between
inline uint32_t split_chunkmax(uint64_t cap) {
    return (uint32_t)(3 * cap / (rs::kSub8Small + 1ull) + split_smax2(cap) + 1);
}
inline uint64_t split_words(uint64_t cap) {
    const uint64_t s2 = split_smax2(cap), s3 = split_smax3(cap);
    return 32ull + 1 + s2 + (3ull * s2 + 2) + (s2 + 1ull) + 256ull * s2 + (3ull * s3 + 2) + (s3 + 1ull) + 256ull * s3 +
           1ull + split_midmax(cap) +          // + the sub-buckets for the large tile
           1ull + 2ull * split_chunkmax(cap);  // + the runs of small sub-buckets
}
constexpr uint32_t kHistGrid = 2048;
constexpr int kCheckGrid = 2048;

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Every launch group of a sort is a named roctx range on the host (rocprofv3 --marker-trace
// attributes the kernels it encloses to histogram / MSD pass 0 / pass 1 / bucket / fallback / LSD
// pass without relying on template names; SURVEY.md §5 "Tracing").  roctx is bound lazily with
// dlopen: librsort.so has no link-time dependency on rocprofiler-sdk, and without it the ranges
// are no-ops.
struct Roctx {
    using Push = int (*)(const char*);
    using Pop = int (*)();
    Push push = nullptr;
    Pop pop = nullptr;
    Roctx() {
        void* h = dlopen("librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
        if (!h) h = dlopen("librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_LOCAL);
        if (h) {
            push = reinterpret_cast<Push>(dlsym(h, "roctxRangePushA"));
            pop = reinterpret_cast<Pop>(dlsym(h, "roctxRangePop"));
            if (!push || !pop) push = nullptr, pop = nullptr;
        }
    }
    static const Roctx& get() {
        static const Roctx r;
        return r;
    }
};
struct RoctxRange {
    bool on;
    explicit RoctxRange(const char* name) : on(Roctx::get().push != nullptr) {
        if (on) Roctx::get().push(name);
    }
    ~RoctxRange() {
        if (on) Roctx::get().pop();
    }
};

struct KernelTimer {
    bool enabled = false;
    uint32_t mask = ~0u;     // kinds bracketed by events (rs_plan_set_profiling_kinds)
    struct Rec { int kind; hipEvent_t a, b; };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    double ms[RS_KERNEL_KINDS] = {};
    uint64_t launches[RS_KERNEL_KINDS] = {};

    hipEvent_t get() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
    // Records events around `launch` when enabled; always a roctx range named `label`.
    template <class F>
    void run(int kind, hipStream_t s, F&& launch, const char* label = nullptr) {
        static const char* const names[RS_KERNEL_KINDS] = {"rsort.histogram", "rsort.scan", "rsort.scatter",
                                                           "rsort.check", "rsort.bucket", "rsort.fallback",
                                                           "rsort.split", "rsort.presorted"};
        RoctxRange range(label ? label : names[kind]);
        if (!enabled || !((mask >> kind) & 1u)) { launch(); return; }
        Rec r{kind, get(), get()};
        (void)hipEventRecord(r.a, s);
        launch();
        (void)hipEventRecord(r.b, s);
        pending.push_back(r);
    }
    void drain() {
        for (auto& r : pending) {
            (void)hipEventSynchronize(r.b);
            float t = 0.f;
            if (hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) ms[r.kind] += t;
            launches[r.kind] += 1;
            pool.push_back(r.a);
            pool.push_back(r.b);
        }
        pending.clear();
    }
    ~KernelTimer() {
        for (auto& r : pending) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

}  // namespace

rs_status rs_internal_fail(rs_status s, const char* msg) { return fail(s, "%s", msg); }

struct rs_plan {
    rs_plan_desc desc{};
    uint32_t bit_count = 32;
    uint32_t radix_bits = 8;
    bool has_values = false, check_order = false, local_shuffle = false;
    int layout = rs::LAYOUT_KEYS;          // rs::Layout of the caller's data
    int rank_mode = rs::RANK_LDS_ATOMIC;   // rs_plan_debug.rank = 1: the ballot-match ranking
    int tile_mode = -1;                    // rs_plan_debug.tile: -1 by size, 0 large tiles, 1 small tiles
    uint32_t usage = RS_USAGE_SORT;        // RS_USAGE_PARTITION: hist16 + partition passes only
    uint64_t rows_words = 0;               // words of tmp_k available to k_hist16_in's rows
    uint32_t passes = 0;
    uint32_t widths[16] = {};
    uint64_t capacity = 0;
    uint32_t* tmp_k = nullptr;
    uint32_t* tmp_v = nullptr;
    uint32_t* counts = nullptr;    // [256][ntiles] digit-major tile counts
    uint32_t* totals = nullptr;    // [256]
    uint32_t* flags = nullptr;     // [16] check_order results
    // one-sweep path (k_pass_totals + k_onesweep)
    int onesweep_mode = -1;                // -1 auto (use_onesweep), 0 off, 1 on (rs_plan_debug.onesweep)
    bool aos_tmp = true;                   // one-sweep KV: records as the ping-pong copy (sweep: RSORT_AOS_TMP)
    uint32_t* tmp2 = nullptr;              // one-sweep KV: second records buffer (sweep: RSORT_RECS2=0: none)
    bool keys_cfg = true;                  // keys-only 512x32 tiles (rs_plan_debug.keys_cfg = 0: 1024x16)
    int kv_cfg = 0;                        // one-sweep KV tile configuration (sweep: RSORT_KV_CFG)
    int huge_tiles = 0;                    // one-sweep KV: 24K-record tiles (sweep: RSORT_HUGE=1: every
                                           // pass; 2: the records -> arrays pass only)
    bool fused_check = true;               // one-sweep check_order: passes > 0 check their input
                                           // in k_onesweep (sweep: RSORT_FUSED_CHECK=0: k_check)
    unsigned long long* status = nullptr;  // [max_tiles][256] look-back status words
    uint64_t status_words = 0;
    uint32_t* ptot = nullptr;      // [kTotalsMax] whole-array digit totals of every pass
    uint32_t ptot_off[16] = {};    // offset of pass i's totals in ptot
    uint32_t* tickets = nullptr;   // = ptot + kTotalsMax: [16] per-pass tile tickets, [16] error
    uint32_t epoch = 0;            // tag of the last k_onesweep launch's status words
    uint32_t spin_max = 1u << 20;  // look-back wait bound in sleeps (rs_plan_set_wait_limit; tests force 0)
    int msd_mode = RS_MSD_DEFAULT;   // hybrid MSD path for values (rs_plan_debug.msd = 0/1)
    // keys-only form of the hybrid MSD path, read per plan (tests switch them):
    int msd_keys_cfg = 1;            // pass tiles (rs_plan_debug.msd_keys_cfg): 0 1024x16, 1 512x32, 2 1024x32
                                     // (32K-key tiles for pass 0 only: no faster, r03_keys_pass0_tiles_ab)
    bool kbucket_wave = true;        // one wave per 16-bit bucket (rs_plan_debug.kbucket_wave = 0: workgroups)
    bool kbucket_pf = false;         // workgroup kernel on a persistent prefetching grid (sweep: RSORT_KBUCKET_PF=1)
    bool high_half = false;          // test hook (rs_plan_debug.high_half): R2 / R3 at a 2^31 low address word
    int xcd_claims = 0;              // hybrid MSD passes with values: XCD-local tile streams (k_msd_pass XC;
                                     // rs_plan_debug.xcd: 0 none (default: XC measured slower, 1.00 / 1.04
                                     // vs 0.99 ms per pass), 1 both passes, 2 pass 0 only, 3 pass 1 only)
    bool static_passes = false;      // hybrid MSD passes over static splits (sweep only, RSORT_STATIC=1: measured
                                     // slower than the look-back passes)
    uint32_t* msd = nullptr;         // its workspace: hist16 | base16 | segtab | gates | mtot
    uint32_t* split = nullptr;       // the bucket split's workspace (rs::SplitWs; split_words())
    uint32_t smax2 = 0, smax3 = 0;   // its level-2 / level-3 segment capacities
    bool split_on = true;            // split over-full buckets (rs_plan_debug.split = 0: the LSD fallback)
    bool last_hybrid = false;        // the last sort enqueued the hybrid path (rs_plan_last_path)
    bool last_split = false;         // ... with the bucket split's launches (rs_plan_last_split)
    uint32_t* ns = nullptr;          // the presorted path's workspace (check_order plans of the hybrid
    uint32_t ns_cap = 0;             // path; ns_words()): its extraction capacity
    bool ns_on = true;               // the presorted path where it applies (rs_plan_debug.presorted = 0: off)
    bool last_ns = false;            // the last sort enqueued the presorted path (rs_plan_last_path)
    bool path_none = false;          // the last sort moved nothing (n <= 1): rs_plan_last_path NONE
    int scatter_kind = RS_KERNEL_SCATTER;   // timer kind of the pass launches being enqueued
    uint32_t* host_err = nullptr;  // host-mapped error word: set by a timed-out look-back wait,
    uint32_t* host_err_dev = nullptr;   // read + cleared by rs_plan_check / the next rs_plan_sort
    hipEvent_t done = nullptr;     // recorded after every sort (rs_plan_check waits for it)
    bool done_recorded = false;
    int selftest = -1;             // lane-order self-test of this device: 1 passed, 0 failed
    uint32_t cus = 256;
    uint64_t workspace = 0;
    KernelTimer timer;
};

struct rs_scan_plan {
    int device = 0;
    uint64_t count = 0;
    uint32_t threads = 256;       // workgroup_x * workgroup_y (reference dispatch-chain shape)
    uint32_t* sums = nullptr;     // [kScanMaxGrid] (reduce-then-scan form, sweep builds)
    // single-pass form (k_scan_lookback): status word per tile, ticket ring, device error word
    unsigned long long* status = nullptr;
    uint64_t status_words = 0;
    uint32_t* tickets = nullptr;  // [kScanTickets] tickets, then [1] error word
    uint32_t epoch = 0;
    uint32_t grid = 0;
    uint32_t spin_max = 1u << 20;
    hipEvent_t done = nullptr;    // recorded after every run (rs_scan_plan_check waits for it)
};

namespace {

uint32_t pick_R(uint32_t w) { return w <= 2 ? 2 : (w <= 4 ? 4 : 8); }

uint32_t full_mask(uint32_t bits) { return bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u); }

bool use_small_tiles(const rs_plan* p, uint64_t n) {
    if (p->tile_mode >= 0) return p->tile_mode == 1;
    return n < RS_SMALL_MAX;
}

template <int R, int TILE>
void launch_histogram(int L, const uint32_t* in, uint32_t n, uint32_t shift, uint32_t mask,
                      uint32_t ntiles, uint32_t* counts, const uint32_t* gate, int pass,
                      hipStream_t s) {
    const uint32_t grid = std::min<uint32_t>((ntiles + rs::kWaves - 1) / rs::kWaves, kHistGrid);
    if (L == rs::LAYOUT_AOS)
        hipLaunchKernelGGL((rs::k_histogram<R, TILE, RS_HIST_U, 2>), dim3(grid), dim3(rs::kBlock), 0, s,
                           in, n, shift, mask, ntiles, counts, gate, pass);
    else
        hipLaunchKernelGGL((rs::k_histogram<R, TILE, RS_HIST_U, 1>), dim3(grid), dim3(rs::kBlock), 0, s,
                           in, n, shift, mask, ntiles, counts, gate, pass);
}

template <int R, int BLOCK, int KPT, int L, int RANK>
void launch_scatter_t(const uint32_t* ik, const uint32_t* iv, uint32_t* ok, uint32_t* ov,
                      uint32_t n, uint32_t shift, uint32_t mask, uint32_t ntiles, uint32_t grid,
                      const uint32_t* counts, const uint32_t* totals, const uint32_t* gate,
                      int pass, hipStream_t s) {
    hipLaunchKernelGGL((rs::k_scatter<R, BLOCK, KPT, L, RANK>), dim3(grid), dim3(BLOCK), 0, s,
                       ik, iv, ok, ov, n, shift, mask, ntiles, counts, totals, gate, pass);
}

template <int R, int BLOCK, int KPT, int L>
void launch_scatter_l(int rank_mode, const uint32_t* ik, const uint32_t* iv, uint32_t* ok,
                      uint32_t* ov, uint32_t n, uint32_t shift, uint32_t mask, uint32_t ntiles,
                      uint32_t grid, const uint32_t* counts, const uint32_t* totals,
                      const uint32_t* gate, int pass, hipStream_t s) {
    if (rank_mode == rs::RANK_BALLOT)
        launch_scatter_t<R, BLOCK, KPT, L, rs::RANK_BALLOT>(ik, iv, ok, ov, n, shift, mask, ntiles, grid, counts, totals, gate, pass, s);
    else
        launch_scatter_t<R, BLOCK, KPT, L, rs::RANK_LDS_ATOMIC>(ik, iv, ok, ov, n, shift, mask, ntiles, grid, counts, totals, gate, pass, s);
}

template <int R, int BLOCK, int KPT>
void launch_scatter(int L, int rank_mode, const uint32_t* ik, const uint32_t* iv, uint32_t* ok,
                    uint32_t* ov, uint32_t n, uint32_t shift, uint32_t mask, uint32_t ntiles,
                    uint32_t grid, const uint32_t* counts, const uint32_t* totals,
                    const uint32_t* gate, int pass, hipStream_t s) {
    if (L == rs::LAYOUT_AOS)
        launch_scatter_l<R, BLOCK, KPT, rs::LAYOUT_AOS>(rank_mode, ik, iv, ok, ov, n, shift, mask, ntiles, grid, counts, totals, gate, pass, s);
    else if (L == rs::LAYOUT_SOA)
        launch_scatter_l<R, BLOCK, KPT, rs::LAYOUT_SOA>(rank_mode, ik, iv, ok, ov, n, shift, mask, ntiles, grid, counts, totals, gate, pass, s);
    else
        launch_scatter_l<R, BLOCK, KPT, rs::LAYOUT_KEYS>(rank_mode, ik, iv, ok, ov, n, shift, mask, ntiles, grid, counts, totals, gate, pass, s);
}

template <class F>
uint32_t resident_per_cu(F kernel, int block) {
    int api = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, kernel, block, 0) != hipSuccess || api < 1)
        api = 1;
    return (uint32_t)api;
}

template <int R, int BLOCK, int KPT, int L, int RANK, int LO, int SR>
void launch_onesweep_t(rs_plan* p, const uint32_t* ik, const uint32_t* iv, uint32_t* ok,
                       uint32_t* ov, uint32_t n, uint32_t shift, uint32_t mask, uint32_t ntiles,
                       const uint32_t* gate, int pass, hipStream_t s) {
    auto kern = rs::k_onesweep<R, BLOCK, KPT, L, RANK, LO, SR>;
    static const uint32_t per_cu = resident_per_cu(kern, BLOCK);   // per instantiation
    // sweep: RSORT_OS_GRID caps the persistent grid (tiles come from tickets, so any grid >= 1 is
    // correct)
    const uint32_t cap = (uint32_t)RS_KNOB("RSORT_OS_GRID", 0);
    uint32_t grid = std::min<uint32_t>(ntiles, p->cus * per_cu);
    if (cap > 0 && cap < grid) grid = cap;
    const bool last = (uint32_t)pass + 1 >= p->passes;
    uint32_t* ntot = last ? nullptr : p->ptot + p->ptot_off[pass + 1];
    const uint32_t nshift = last ? 0u : shift + p->widths[pass];
    const uint32_t nmask = last ? 0u : (1u << p->widths[pass + 1]) - 1u;
    // check_order: passes > 0 check their own input (k_check runs before pass 0 only)
    uint32_t* chk = (p->check_order && gate && pass > 0 && p->fused_check) ? p->flags : nullptr;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), 0, s, ik, iv, ok, ov, n, shift, mask, ntiles,
                       p->ptot + p->ptot_off[pass], p->status, p->tickets + pass,
                       p->tickets + 16, ntot, nshift, nmask, p->epoch, gate, pass, chk,
                       full_mask(p->bit_count), p->spin_max, p->host_err_dev,
                       (const uint32_t*)nullptr, (const uint32_t*)nullptr, 0u, 0xFFFFFFFFu);
}

template <int R, int BLOCK, int KPT, int L, int LO, int SR>
void launch_onesweep_l(rs_plan* p, const uint32_t* ik, const uint32_t* iv, uint32_t* ok,
                       uint32_t* ov, uint32_t n, uint32_t shift, uint32_t mask, uint32_t ntiles,
                       const uint32_t* gate, int pass, hipStream_t s) {
    if (p->rank_mode == rs::RANK_BALLOT)
        launch_onesweep_t<R, BLOCK, KPT, L, rs::RANK_BALLOT, LO, SR>(p, ik, iv, ok, ov, n, shift, mask, ntiles, gate, pass, s);
    else
        launch_onesweep_t<R, BLOCK, KPT, L, rs::RANK_LDS_ATOMIC, LO, SR>(p, ik, iv, ok, ov, n, shift, mask, ntiles, gate, pass, s);
}

// A new tag for the look-back status words of the next k_onesweep launch.
rs_status next_epoch(rs_plan* p, hipStream_t s) {
    if (++p->epoch >= (1u << 30)) {   // tag space exhausted: clear the words, restart tags
        HIP_TRY(hipMemsetAsync(p->status, 0, 8ull * p->status_words, s));
        p->epoch = 1;
    }
    return RS_OK;
}

// One pass of the hybrid MSD path (16K-record tiles, 8-bit digit at `shift`): SEG = 0 the
// top-byte pass over the whole input, SEG = 1 the next-byte pass inside every top-byte segment.
// BLOCK x KPT = 16K keys (kLarge; keys only: kLargeKeys, two workgroups per CU).
template <int L, int LO, int SEG, bool KB = false, int BLOCK = kLarge.block, int KPT = kLarge.kpt, int SR = 1>
void launch_msd_pass(rs_plan* p, const uint32_t* ik, const uint32_t* iv, uint32_t* ok, uint32_t* ov,
                     uint32_t n, uint32_t shift, uint32_t ntiles, const uint32_t* dtot, uint32_t* ticket,
                     const uint32_t* gate, const uint32_t* segtab, const uint32_t* base16,
                     hipStream_t s, uint32_t kbase = 0, uint32_t pmask = 0xFFFFFFFFu,
                     const uint32_t* cbase = nullptr, uint32_t hrows = 0) {
    // cbase / hrows (SEG = 0): the histogram rows' chunk starts, for XCD-local claims (k_msd_pass XC)
    static_assert(BLOCK * KPT == kLarge.tile || BLOCK * KPT == 2 * kLarge.tile, "k_msd_plan tile sizes");
    static_assert(SR == 1 || SEG == 0, "staging rounds: the top-byte pass only");
    auto go = [&](auto kern) {
        static const uint32_t per_cu = resident_per_cu(kern, BLOCK);
        const uint32_t grid = std::min<uint32_t>(ntiles, p->cus * per_cu);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), 0, s, ik, iv, ok, ov, n, shift, 255u,
                           ntiles, dtot, p->status, ticket, p->tickets + 16, nullptr, 0u, 0u, p->epoch,
                           gate, SEG, nullptr, 0xFFFFFFFFu, p->spin_max, p->host_err_dev, segtab, base16, kbase,
                           pmask);
    };
    constexpr bool LEAN = RS_MSD_LEAN && SEG <= 1 && SR == 1 && L != rs::LAYOUT_KEYS && BLOCK == kLarge.block &&
                          KPT == kLarge.kpt;
    if constexpr (LEAN) {
        if (pmask == 0xFFFFFFFFu) {   // (the ring experiment keeps k_onesweep)
            // XCD-local claims (rs_plan_debug.xcd): 8 counters per pass after the per-pass tickets
            const bool xc = (p->xcd_claims == 1 || p->xcd_claims == (SEG == 0 ? 2 : 3)) && (SEG == 1 || (cbase && hrows));
            auto lean = [&](auto kern) {
                static const uint32_t per_cu = resident_per_cu(kern, BLOCK);
                // (XC, SEG = 0: up to one partial tile per chunk on top)
                const uint32_t bound = xc && SEG == 0 ? ntiles + 8u : ntiles;
                const uint32_t grid = std::min<uint32_t>(bound, p->cus * per_cu);
                hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), 0, s, ik, iv, ok, ov, n, shift, bound, dtot,
                                   p->status, xc ? p->tickets + kXcdTickets + 8 * SEG : ticket, p->tickets + 16,
                                   p->epoch, gate, SEG, p->spin_max, p->host_err_dev, segtab, base16, kbase, cbase,
                                   hrows);
            };
            if (xc) {
                if (p->rank_mode == rs::RANK_BALLOT) lean(rs::k_msd_pass<L, LO, SEG, KB, rs::RANK_BALLOT, true>);
                else lean(rs::k_msd_pass<L, LO, SEG, KB, rs::RANK_LDS_ATOMIC, true>);
            } else {
                if (p->rank_mode == rs::RANK_BALLOT) lean(rs::k_msd_pass<L, LO, SEG, KB, rs::RANK_BALLOT>);
                else lean(rs::k_msd_pass<L, LO, SEG, KB, rs::RANK_LDS_ATOMIC>);
            }
            return;
        }
    }
    if (p->rank_mode == rs::RANK_BALLOT)
        go(rs::k_onesweep<8, BLOCK, KPT, L, rs::RANK_BALLOT, LO, SR, SEG, KB>);
    else
        go(rs::k_onesweep<8, BLOCK, KPT, L, rs::RANK_LDS_ATOMIC, LO, SR, SEG, KB>);
}

// The hybrid path's passes over a static split (k_static_pass; 16K-record tiles, one 1024-thread
// workgroup per unit).  Pass 0: one workgroup per k_hist16_in row (input chunk), input arrays or
// records -> R1 records; pass 1: one workgroup per top-byte segment, R1 -> R2 records.
#if RS_SWEEP
void launch_static_pass0(rs_plan* p, const uint32_t* ik, const uint32_t* iv, bool in_aos, bool kb, uint32_t* r1,
                         uint32_t n, uint32_t shift, uint32_t rows, const uint32_t* gate, const uint32_t* segtab,
                         const uint32_t* cbase, uint32_t kbase, hipStream_t s) {
    constexpr int A = rs::LAYOUT_AOS, S = rs::LAYOUT_SOA, B = kLarge.block, K = kLarge.kpt;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(rows), dim3(B), 0, s, ik, iv, r1, (uint32_t*)nullptr, n, shift, gate, segtab,
                           (const uint32_t*)nullptr, cbase, kbase);
    };
    const bool ballot = p->rank_mode == rs::RANK_BALLOT;
    constexpr int RA = rs::RANK_LDS_ATOMIC, RB = rs::RANK_BALLOT;
    if (in_aos) {
        if (kb) ballot ? go(rs::k_static_pass<B, K, A, RB, A, 0, true>) : go(rs::k_static_pass<B, K, A, RA, A, 0, true>);
        else ballot ? go(rs::k_static_pass<B, K, A, RB, A, 0>) : go(rs::k_static_pass<B, K, A, RA, A, 0>);
    } else {
        if (kb) ballot ? go(rs::k_static_pass<B, K, S, RB, A, 0, true>) : go(rs::k_static_pass<B, K, S, RA, A, 0, true>);
        else ballot ? go(rs::k_static_pass<B, K, S, RB, A, 0>) : go(rs::k_static_pass<B, K, S, RA, A, 0>);
    }
}

void launch_static_pass1(rs_plan* p, const uint32_t* r1, uint32_t* r2, uint32_t n, uint32_t shift,
                         const uint32_t* gate, const uint32_t* segtab, const uint32_t* base16, hipStream_t s) {
    constexpr int A = rs::LAYOUT_AOS, B = kLarge.block, K = kLarge.kpt;
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(256), dim3(B), 0, s, r1, (const uint32_t*)nullptr, r2, (uint32_t*)nullptr, n,
                           shift, gate, segtab, base16, (const uint32_t*)nullptr, 0u);
    };
    if (p->rank_mode == rs::RANK_BALLOT) go(rs::k_static_pass<B, K, A, rs::RANK_BALLOT, A, 1>);
    else go(rs::k_static_pass<B, K, A, rs::RANK_LDS_ATOMIC, A, 1>);
}
#endif

// Layout pair of one pass: input layout | output layout << 4 (they differ only on the one-sweep
// separate-values path, which stages its ping-pong copy as (key, value) records).
constexpr int layout_pair(int in, int out) { return in | (out << 4); }

// One stable digit pass in -> out (histogram, scan, scatter) with tile configuration C.
// KEYS_ONLY instantiates the keys-only kernels alone (configurations used only without values).
template <int R, int BLOCK, int KPT, bool KEYS_ONLY = false, int SR = 1>
rs_status run_pass_cfg(rs_plan* p, const uint32_t* ik, const uint32_t* iv, uint32_t* ok,
                       uint32_t* ov, uint32_t n, uint32_t shift, uint32_t w, int LL,
                       const uint32_t* gate, int pass, uint32_t max_grid, bool onesweep,
                       hipStream_t s) {
    constexpr int TILE = BLOCK * KPT;
    const uint32_t mask = (1u << w) - 1u;
    const uint32_t ntiles = (uint32_t)(((uint64_t)n + TILE - 1) / TILE);
    const uint32_t grid = std::min<uint32_t>(ntiles, max_grid);
    const int L = LL & 15;
    if (onesweep) {
        // the look-back status words of every tile of this launch must exist (never index past them)
        if ((uint64_t)ntiles * 256u > p->status_words)
            return fail(RS_ERR_INVALID_ARG, "internal: %u one-sweep tiles exceed the plan's %llu status words",
                        ntiles, (unsigned long long)p->status_words);
        if (rs_status st = next_epoch(p, s)) return st;
        constexpr int K = rs::LAYOUT_KEYS, S = rs::LAYOUT_SOA, A = rs::LAYOUT_AOS;
        p->timer.run(p->scatter_kind, s, [&] {
            if constexpr (KEYS_ONLY) {
                launch_onesweep_l<R, BLOCK, KPT, K, K, SR>(p, ik, iv, ok, ov, n, shift, mask, ntiles, gate, pass, s);
            } else {
                switch (LL) {
                    case layout_pair(A, A): launch_onesweep_l<R, BLOCK, KPT, A, A, SR>(p, ik, iv, ok, ov, n, shift, mask, ntiles, gate, pass, s); break;
                    case layout_pair(S, S): launch_onesweep_l<R, BLOCK, KPT, S, S, SR>(p, ik, iv, ok, ov, n, shift, mask, ntiles, gate, pass, s); break;
                    case layout_pair(S, A): launch_onesweep_l<R, BLOCK, KPT, S, A, SR>(p, ik, iv, ok, ov, n, shift, mask, ntiles, gate, pass, s); break;
                    case layout_pair(A, S): launch_onesweep_l<R, BLOCK, KPT, A, S, SR>(p, ik, iv, ok, ov, n, shift, mask, ntiles, gate, pass, s); break;
                    default: launch_onesweep_l<R, BLOCK, KPT, K, K, SR>(p, ik, iv, ok, ov, n, shift, mask, ntiles, gate, pass, s);
                }
            }
        }, p->scatter_kind == RS_KERNEL_FALLBACK ? "rsort.lsd.pass (fallback)" : "rsort.lsd.pass");
        HIP_TRY(hipGetLastError());
        return RS_OK;
    }
    if constexpr (SR != 1) {
        return fail(RS_ERR_INVALID_ARG, "staging rounds are one-sweep only");
    } else {
        // the gated LSD fallback of the hybrid MSD path (and the presorted path's sort of its
        // extraction) times all its launches as one kind
        const bool fb = p->scatter_kind != RS_KERNEL_SCATTER;
        const int fk = p->scatter_kind;
        p->timer.run(fb ? fk : RS_KERNEL_HISTOGRAM, s, [&] {
            launch_histogram<R, TILE>(L, ik, n, shift, mask, ntiles, p->counts, gate, pass, s);
        });
        HIP_TRY(hipGetLastError());
        p->timer.run(fb ? fk : RS_KERNEL_SCAN, s, [&] {
            hipLaunchKernelGGL(rs::k_scan_rows, dim3(1u << R), dim3(rs::kBlock), 0, s, p->counts,
                               ntiles, p->totals, gate, pass);
        });
        HIP_TRY(hipGetLastError());
        // The scatter always stages the tile through LDS (the local shuffle,
        // RadixSortLocalShuffle.ts:94-116): it is what makes the writes coalesced.
        p->timer.run(fb ? fk : RS_KERNEL_SCATTER, s, [&] {
            if constexpr (KEYS_ONLY)
                launch_scatter_l<R, BLOCK, KPT, rs::LAYOUT_KEYS>(p->rank_mode, ik, iv, ok, ov, n, shift, mask,
                                                                 ntiles, grid, p->counts, p->totals, gate, pass, s);
            else
                launch_scatter<R, BLOCK, KPT>(L, p->rank_mode, ik, iv, ok, ov, n, shift, mask, ntiles,
                                              grid, p->counts, p->totals, gate, pass, s);
        });
        HIP_TRY(hipGetLastError());
        return RS_OK;
    }
}

rs_status run_pass(rs_plan* p, const uint32_t* ik, const uint32_t* iv, uint32_t* ok,
                   uint32_t* ov, uint32_t n, uint32_t shift, uint32_t w, int LL,
                   const uint32_t* gate, int pass, hipStream_t s, bool onesweep = false) {
    const uint32_t R = pick_R(w);
    if (use_small_tiles(p, n)) {
        if (R == 2) return run_pass_cfg<2, kSmall.block, kSmall.kpt>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kSmall.max_grid, onesweep, s);
        if (R == 4) return run_pass_cfg<4, kSmall.block, kSmall.kpt>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kSmall.max_grid, onesweep, s);
        return run_pass_cfg<8, kSmall.block, kSmall.kpt>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kSmall.max_grid, onesweep, s);
    }
#if RS_SWEEP
    // sweep only: 24K-record tiles with values (records only from a plan-owned buffer padded to
    // whole kHuge tiles: the kernel loads whole record tiles without per-slot bounds, see
    // k_onesweep's SR > 1), and the KV tile configurations with several workgroups per CU
    const int Lin = LL & 15;
    if (R == 8 && onesweep && p->huge_tiles &&
        (p->huge_tiles == 1 || LL == layout_pair(rs::LAYOUT_AOS, rs::LAYOUT_SOA)) &&
        (Lin == rs::LAYOUT_SOA ||
         (Lin == rs::LAYOUT_AOS && (ik == p->tmp_k || (p->tmp2 && ik == p->tmp2)))))
        return run_pass_cfg<8, kHuge.block, kHuge.kpt, false, 2>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kHuge.max_grid, onesweep, s);
    // staging rounds (SR > 1) load whole record tiles: separate arrays (clamped loads) or
    // records from a plan-owned buffer padded to whole tiles
    const bool whole_ok = Lin == rs::LAYOUT_SOA ||
        (Lin == rs::LAYOUT_AOS && (ik == p->tmp_k || (p->tmp2 && ik == p->tmp2)));
    if (R == 8 && onesweep && Lin != rs::LAYOUT_KEYS && p->kv_cfg > 0) {
        switch (p->kv_cfg) {
            case 1: return run_pass_cfg<8, kKv512x16.block, kKv512x16.kpt>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kKv512x16.max_grid, onesweep, s);
            case 2: if (whole_ok) return run_pass_cfg<8, kKv512x32.block, kKv512x32.kpt, false, 2>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kKv512x32.max_grid, onesweep, s); break;
            case 3: if (whole_ok) return run_pass_cfg<8, kKv256x32.block, kKv256x32.kpt, false, 2>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kKv256x32.max_grid, onesweep, s); break;
            case 4: if (whole_ok) return run_pass_cfg<8, kKv512x24.block, kKv512x24.kpt, false, 2>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kKv512x24.max_grid, onesweep, s); break;
            default: break;
        }
        return run_pass_cfg<8, kKv512x16.block, kKv512x16.kpt>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kKv512x16.max_grid, onesweep, s);
    }
#endif
    if (R == 8 && LL == layout_pair(rs::LAYOUT_KEYS, rs::LAYOUT_KEYS) && p->keys_cfg)
        return run_pass_cfg<8, kLargeKeys.block, kLargeKeys.kpt, true>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kLargeKeys.max_grid, onesweep, s);
    if (R == 2) return run_pass_cfg<2, kLarge.block, kLarge.kpt>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kLarge.max_grid, onesweep, s);
    if (R == 4) return run_pass_cfg<4, kLarge.block, kLarge.kpt>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kLarge.max_grid, onesweep, s);
    return run_pass_cfg<8, kLarge.block, kLarge.kpt>(p, ik, iv, ok, ov, n, shift, w, LL, gate, pass, kLarge.max_grid, onesweep, s);
}

// Whole sort of n <= kTinyMax in one workgroup (k_sort_small).
rs_status run_tiny(rs_plan* p, uint32_t* k, uint32_t* v, uint32_t n, hipStream_t s) {
    rs::PassList pl{};
    pl.count = p->passes;
    for (uint32_t i = 0; i < p->passes; ++i) pl.width[i] = p->widths[i];
    const bool ballot = p->rank_mode == rs::RANK_BALLOT;
    p->timer.run(RS_KERNEL_SCATTER, s, [&] {
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(1), dim3(1024), 0, s, k, v, n, pl); };
        constexpr int A = rs::RANK_LDS_ATOMIC, B = rs::RANK_BALLOT;
        switch (p->layout) {
            case rs::LAYOUT_AOS:
                ballot ? go(rs::k_sort_small<1024, 16, rs::LAYOUT_AOS, B>) : go(rs::k_sort_small<1024, 16, rs::LAYOUT_AOS, A>);
                break;
            case rs::LAYOUT_SOA:
                ballot ? go(rs::k_sort_small<1024, 16, rs::LAYOUT_SOA, B>) : go(rs::k_sort_small<1024, 16, rs::LAYOUT_SOA, A>);
                break;
            default:
                ballot ? go(rs::k_sort_small<1024, 16, rs::LAYOUT_KEYS, B>) : go(rs::k_sort_small<1024, 16, rs::LAYOUT_KEYS, A>);
        }
    });
    HIP_TRY(hipGetLastError());
    return RS_OK;
}

// One-sweep (k_pass_totals + k_onesweep) or histogram/scan/scatter for this sort.  Measured on
// MI355X: one-sweep wins with values on large-tile sizes (256M KV: -14 %), loses
// keys-only (a keys-only tile is processed so fast that the look-back wait shows: +10 % at 64M)
// and on small tiles (thousands of tiles in flight at once make long look-back chains).
bool use_onesweep(const rs_plan* p, uint64_t n) {
    if (p->onesweep_mode >= 0) return p->onesweep_mode == 1;
    return p->layout != rs::LAYOUT_KEYS && !use_small_tiles(p, n);
}

// Words of tmp_k per k_hist16_in row: 65536 counts and a flag word; with check_order also the
// row's 256 byte-0 counts (the LSD fallback's pass-0 totals).
uint64_t hist_row_words(const rs_plan* p) { return 65537ull + (p->check_order ? 256ull : 0ull); }

// The hybrid MSD path applies (the device still falls back to the LSD passes for skewed keys).
bool use_msd(const rs_plan* p, uint64_t n) {
    if (!p->msd || p->msd_mode == 0 || p->bit_count != 32 || p->radix_bits != 8 ||
        use_small_tiles(p, n) || n < kMsdMin)
        return false;
    // above kMsdMax keys some 16-bit bucket is all but certain to exceed kBucketCap (and above
    // 65536 * kBucketCap one must, pigeonhole): the device would pick the fallback, so the
    // histogram read would be wasted
    if (n > kMsdMax) return false;
    // keys only: R1 = tmp_k (n words, which first holds the histogram rows), R2 = the caller's keys;
    // the one-sweep passes of this path are its own (the keys-only LSD sort keeps the histogram path)
    if (p->layout == rs::LAYOUT_KEYS)
        return p->onesweep_mode != 0 && (uint64_t)p->cus * hist_row_words(p) <= n;   // rows + their flag words
    const bool bufs = (p->layout == rs::LAYOUT_AOS || (p->layout == rs::LAYOUT_SOA && p->tmp2 && p->aos_tmp)) &&
                      (uint64_t)p->cus * hist_row_words(p) <= 2ull * n;   // the histogram rows fit in tmp_k
    return bufs && use_onesweep(p, n) && p->kv_cfg == 0 && !p->huge_tiles;
}

// Lane-order self-test of the device's LDS atomics (k_lane_order_selftest), once per device
// per process: 1 passed, 0 failed (plans then rank with RANK_BALLOT), -1 could not run.
// rs_plan_set_debug(selftest_fail = 1) simulates a failure (tests).
int lane_order_selftest(int dev) {
    static std::mutex mu;
    static std::map<int, int> done;
    std::lock_guard<std::mutex> lock(mu);
    auto it = done.find(dev);
    if (it != done.end()) return it->second;
    int result = -1;
    uint32_t* bad = nullptr;
    hipStream_t s = nullptr;
    if (hipMalloc((void**)&bad, 4) == hipSuccess &&
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
        hipMemsetAsync(bad, 0, 4, s) == hipSuccess) {
        hipLaunchKernelGGL(rs::k_lane_order_selftest, dim3(256), dim3(rs::kBlock), 0, s, 256u, bad);
        uint32_t h = 1;
        if (hipGetLastError() == hipSuccess &&
            hipMemcpyAsync(&h, bad, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
            hipStreamSynchronize(s) == hipSuccess)
            result = h == 0 ? 1 : 0;
    }
    if (s) (void)hipStreamDestroy(s);
    if (bad) (void)hipFree(bad);
    if (result >= 0) done[dev] = result;
    return result;
}

// A previous sort on this plan hit a device-side failure (look-back wait timeout): report it
// once and clear it.
rs_status take_device_error(rs_plan* p, const char* what) {
    if (!p->host_err) return RS_OK;
    const uint32_t e = __atomic_exchange_n(p->host_err, 0u, __ATOMIC_ACQ_REL);
    if (e == 0u) return RS_OK;
    // bit 0: a look-back wait of a one-sweep pass timed out; bit 2: the hybrid path's counts did
    // not add up (the bucket split's digit counts, or the histogram against n)
    return fail(RS_ERR_DEVICE,
                "%s: an earlier sort on this plan failed on the device (error word 0x%x: %s); that "
                "sort's output is invalid", what, e,
                (e & 4u) ? (e & 1u) ? "a look-back wait timed out and the hybrid path's counts did not add up"
                                    : "the hybrid path's counts did not add up"
                         : "a look-back wait of the one-sweep pass timed out");
}

// Sort entry points need the full workspace (a RS_USAGE_PARTITION plan has no ping-pong copy).
rs_status need_sort_plan(const rs_plan* p, const char* what) {
    if (p->usage == RS_USAGE_SORT) return RS_OK;
    return fail(RS_ERR_INVALID_ARG, "%s: a RS_USAGE_PARTITION plan only runs rs_plan_hist16 and rs_plan_partition*",
                what);
}

}  // namespace

// ============================================================================================
RS_EXPORT const char* rs_last_error(void) { return g_err.c_str(); }

RS_EXPORT const char* rs_status_string(rs_status s) {
    switch (s) {
        case RS_OK: return "ok";
        case RS_ERR_INVALID_ARG: return "invalid argument";
        case RS_ERR_NOT_POW2: return "workgroup size not a power of two";
        case RS_ERR_BIT_COUNT: return "bit_count must be a multiple of 4 in [4, 32]";
        case RS_ERR_HIP: return "HIP runtime error";
        case RS_ERR_OUT_OF_MEMORY: return "out of device memory";
        case RS_ERR_CAPACITY: return "count exceeds plan capacity";
        case RS_ERR_DEVICE: return "device-side failure (a sort's result is invalid)";
    }
    return "unknown status";
}

RS_EXPORT uint32_t rs_version(void) { return (RSORT_VERSION_MAJOR << 16) | RSORT_VERSION_MINOR; }

// The presorted path's workspace (rs_presorted.hpp): control words, per-tile counts / boundary keys /
// offsets / bounds, the chunk sums, the extraction sort's totals, the mark bitmap with its per-word
// mark prefix and samples, and twelve arrays of the extraction capacity (masked key and extraction
// index twice - the ping-pong of its sort - then key, value, position; the sorted positions, keys
// and values; ranks and tiles).  Sized for min(capacity, kMsdMax) keys: the hybrid path never sorts more.
struct NsWs {
    uint32_t *ctl, *tcnt, *tbnd, *toff, *blo, *csum, *coff, *sub, *bitmap, *wpre, *samp, *ek, *ei, *ek2, *ei2, *sk,
        *sv, *sp, *bp, *bk, *bv, *rank, *tileof;
};
uint64_t ns_keys(uint64_t capacity) { return std::min<uint64_t>(capacity, kMsdMax); }
// extraction capacity for n keys: n / 128 (config 4's n / 1000 transpositions mark ~n / 500), at
// least 64K, in whole 16K-key tiles of its sort
uint32_t ns_cap_for(uint64_t n) {
    return (uint32_t)std::max<uint64_t>(65536u, (n / 128u + 16383u) / 16384u * 16384u);
}
NsWs ns_layout(uint32_t* q, uint64_t capacity) {
    const uint64_t nt = (ns_keys(capacity) + rs::kNsTile - 1) / rs::kNsTile;
    const uint64_t cap = ns_cap_for(ns_keys(capacity));
    NsWs w;
    w.ctl = q;
    q += rs::kNsCtlWords;
    w.tcnt = q;
    q += nt;
    w.tbnd = q;
    q += 2 * nt;
    w.toff = q;
    q += nt + 1;
    w.blo = q;
    q += nt + 1;
    w.csum = q;                       // per 1024 tiles (k_ns_decide_a / _b)
    q += nt / 1024 + 1;
    w.coff = q;
    q += nt / 1024 + 2;
    w.sub = q;                        // the extraction sort's digit totals, tickets, error word
    q += rs::kNsSubWords;
    w.bitmap = q;
    q += nt * (rs::kNsTile / 32);
    w.wpre = q;                       // per bitmap word: the tile's marks before it
    q += nt * (rs::kNsTile / 32);
    w.samp = q;                       // per bitmap word: (key, position) sample (k_ns_mark, k_ns_rank)
    q += 2 * nt * (rs::kNsTile / 32);
    uint32_t** arr[12] = {&w.ek, &w.ei, &w.ek2, &w.ei2, &w.sk, &w.sv, &w.sp, &w.bp, &w.bk, &w.bv, &w.rank, &w.tileof};
    for (uint32_t** a : arr) {
        *a = q;
        q += cap;
    }
    return w;
}
uint64_t ns_words(uint64_t capacity) {
    return (uint64_t)(ns_layout(nullptr, capacity).tileof - (uint32_t*)nullptr) + ns_cap_for(ns_keys(capacity));
}

RS_EXPORT rs_status rs_plan_create(const rs_plan_desc* desc, rs_plan** out) {
    if (!desc || !out) return fail(RS_ERR_INVALID_ARG, "rs_plan_create: null argument");
    *out = nullptr;
    rs_plan_desc d = *desc;
    if (d.bit_count == 0) d.bit_count = 32;                      // AbstractRadixSortKernel.ts:54
    if (d.workgroup_x == 0) d.workgroup_x = 16;                  // AbstractKernel.ts:22-25
    if (d.workgroup_y == 0) d.workgroup_y = 16;
    const uint64_t T = (uint64_t)d.workgroup_x * d.workgroup_y;
    if (T == 0 || (T & (T - 1)) || T > 1024)
        return fail(RS_ERR_NOT_POW2,
                    "workgroupSize.x * workgroupSize.y must be a power of two <= 1024. (current: %llu)",
                    (unsigned long long)T);
    if (d.bit_count % 4 || d.bit_count > 32)
        return fail(RS_ERR_BIT_COUNT, "bit_count must be a multiple of 4 in [4, 32] (got %u)",
                    d.bit_count);
    if (d.count > 0xFFFFFFFFull)
        return fail(RS_ERR_INVALID_ARG, "count must be < 2^32 (got %llu)",
                    (unsigned long long)d.count);
    uint32_t rb = d.radix_bits ? d.radix_bits : 8;
    if (rb != 2 && rb != 4 && rb != 8)
        return fail(RS_ERR_INVALID_ARG, "radix_bits must be 0, 2, 4 or 8 (got %u)", d.radix_bits);
    if (d.flags & ~(uint32_t)0x1F) return fail(RS_ERR_INVALID_ARG, "unknown flag bits 0x%x", d.flags);
    if (d.usage != RS_USAGE_SORT && d.usage != RS_USAGE_PARTITION)
        return fail(RS_ERR_INVALID_ARG, "usage must be RS_USAGE_SORT or RS_USAGE_PARTITION (got %u)", d.usage);

    rs_plan* p = new (std::nothrow) rs_plan();
    if (!p) return fail(RS_ERR_OUT_OF_MEMORY, "host allocation failed");
    p->desc = d;
    p->bit_count = d.bit_count;
    p->radix_bits = rb;
    p->has_values = d.flags & (RS_FLAG_HAS_VALUES | RS_FLAG_INTERLEAVED);
    p->layout = (d.flags & RS_FLAG_INTERLEAVED) ? rs::LAYOUT_AOS
              : (p->has_values ? rs::LAYOUT_SOA : rs::LAYOUT_KEYS);
    p->usage = d.usage;
    p->check_order = d.flags & RS_FLAG_CHECK_ORDER;
    p->local_shuffle = d.flags & RS_FLAG_LOCAL_SHUFFLE;
    // path choices: by size; the parity tests switch them with rs_plan_set_debug
    bool recs2 = true;
#if RS_SWEEP
    p->aos_tmp = RS_KNOB("RSORT_AOS_TMP", 1) != 0;
    recs2 = RS_KNOB("RSORT_RECS2", 1) != 0;
    p->huge_tiles = (int)RS_KNOB("RSORT_HUGE", 0);
    p->kv_cfg = (int)RS_KNOB("RSORT_KV_CFG", 0);
    p->fused_check = RS_KNOB("RSORT_FUSED_CHECK", 1) != 0;
    p->kbucket_pf = RS_KNOB("RSORT_KBUCKET_PF", 0) == 1;
    p->static_passes = RS_KNOB("RSORT_STATIC", 0) != 0;
#endif
    // Even number of passes so the result lands in the caller's buffers, like the reference's
    // bit_count/2 passes with ping-pong on bit % 4 (AbstractRadixSortKernel.ts:93-107).
    uint32_t P = (d.bit_count + rb - 1) / rb;
    P += P & 1u;
    p->passes = P;
    for (uint32_t i = 0, off = 0; i < P; ++i) {
        p->widths[i] = d.bit_count / P + (i < d.bit_count % P ? 1 : 0);
        p->ptot_off[i] = off;
        off += 1u << p->widths[i];
    }
    p->capacity = d.count;

    DeviceGuard guard(d.device);
    auto cleanup = [&](rs_status s) { rs_plan_destroy(p); return s; };
    // stable ranking: lane-ordered LDS atomics where the device passes the self-test, else the
    // architecture-guaranteed ballot ranking (rs_plan_set_debug overrides)
    p->selftest = lane_order_selftest(d.device);
    p->rank_mode = p->selftest == 1 ? rs::RANK_LDS_ATOMIC : rs::RANK_BALLOT;
    auto alloc = [&](uint32_t** ptr, uint64_t bytes) -> hipError_t {
        if (bytes == 0) bytes = 4;
        p->workspace += bytes;
        return hipMalloc((void**)ptr, bytes);
    };
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d.device) == hipSuccess && prop.multiProcessorCount > 0)
            p->cus = (uint32_t)prop.multiProcessorCount;
    }
    // look-back status words: one per (tile, digit) of the finest tile configuration in use
    // (the hybrid path's segmented pass: up to one partial tile per top-byte segment on top of
    // the 16K-key tiles, which dominates below ~4M keys)
    // (and the bucket split's passes: one partial tile per segment on top, see split_smax3)
    const uint64_t max_tiles = std::max<uint64_t>(
        (d.count + kLarge.tile - 1) / kLarge.tile + 1 + std::max<uint64_t>(256, split_smax3(d.count)),
        std::max<uint64_t>((d.count + kMinOnesweepTile - 1) / kMinOnesweepTile,
                           (std::min<uint64_t>(d.count, RS_SMALL_MAX) + kSmall.tile - 1) / kSmall.tile));
    // sized whatever rs_plan_debug.onesweep says: the records / partition entry points and the hybrid
    // path's passes are one-sweep passes on every plan
    p->status_words = max_tiles * 256;
    hipError_t e;
    // with values the tmp copy is ONE 8n-byte buffer: (key, value) records for the one-sweep
    // path, or tmp_k / tmp_v halves (tmp_v = tmp_k + count) for the histogram path
    // records buffers are padded to whole kHuge tiles (k_onesweep with staging rounds reads
    // whole tiles)
    const uint64_t padded = (d.count + kRecPad - 1) / kRecPad * kRecPad;
    // tmp_k: the ping-pong copy, which also holds k_hist16_in's rows (one per CU: 65536 counts, and
    // a flag word each) before the passes use it; a partition plan keeps just the rows
    const bool sorts = d.usage == RS_USAGE_SORT;
    const uint64_t rows_bytes = 4ull * p->cus * 65537ull;
    const uint64_t tmpk_bytes = !sorts ? rows_bytes : (p->layout == rs::LAYOUT_KEYS ? 4 * d.count : 8 * padded);
    p->rows_words = tmpk_bytes / 4;
    if ((e = alloc(&p->tmp_k, tmpk_bytes)) != hipSuccess ||
        (sorts && p->layout == rs::LAYOUT_SOA && p->onesweep_mode != 0 && p->aos_tmp && recs2 &&
         d.count > kTinyMax && (e = alloc(&p->tmp2, 8 * padded)) != hipSuccess) ||
        (e = alloc(&p->counts, 4ull * 256 * std::max<uint64_t>(1, (d.count + kSmall.tile - 1) / kSmall.tile))) != hipSuccess ||
        (e = alloc(&p->totals, 4ull * 256)) != hipSuccess ||
        (e = alloc(&p->flags, 4ull * 16)) != hipSuccess ||
        (e = alloc(&p->ptot, 4ull * (rs::kTotalsMax + kTicketWords))) != hipSuccess ||
        (e = alloc((uint32_t**)&p->status, 8ull * p->status_words)) != hipSuccess)
        return cleanup(fail(e == hipErrorOutOfMemory ? RS_ERR_OUT_OF_MEMORY : RS_ERR_HIP,
                            "rs_plan_create: hipMalloc failed: %s", hipGetErrorString(e)));
    if (sorts && p->msd_mode != 0 && d.count > kTinyMax &&
        (p->layout == rs::LAYOUT_AOS || p->layout == rs::LAYOUT_KEYS ||
         (p->layout == rs::LAYOUT_SOA && p->tmp2)) &&
        (e = alloc(&p->msd, 4ull * kMsdWords)) != hipSuccess)
        return cleanup(fail(e == hipErrorOutOfMemory ? RS_ERR_OUT_OF_MEMORY : RS_ERR_HIP,
                            "rs_plan_create: hipMalloc failed: %s", hipGetErrorString(e)));
    if (p->msd) {
        p->smax2 = split_smax2(d.count);
        p->smax3 = split_smax3(d.count);
        if ((e = alloc(&p->split, 4ull * split_words(d.count))) != hipSuccess)
            return cleanup(fail(e == hipErrorOutOfMemory ? RS_ERR_OUT_OF_MEMORY : RS_ERR_HIP,
                                "rs_plan_create: hipMalloc failed: %s", hipGetErrorString(e)));
    }
    // check_order (sorts of >= kMsdMin keys): the presorted path's workspace
    if (sorts && p->check_order && d.count >= kMsdMin &&
        (e = alloc(&p->ns, 4ull * ns_words(d.count))) != hipSuccess)
        return cleanup(fail(e == hipErrorOutOfMemory ? RS_ERR_OUT_OF_MEMORY : RS_ERR_HIP,
                            "rs_plan_create: hipMalloc failed: %s", hipGetErrorString(e)));
    p->tickets = p->ptot + rs::kTotalsMax;   // [16] tickets, [16] error word

    if ((e = hipHostMalloc((void**)&p->host_err, 4, hipHostMallocMapped)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&p->host_err_dev, p->host_err, 0)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&p->done, hipEventDisableTiming)) != hipSuccess)
        return cleanup(fail(RS_ERR_HIP, "rs_plan_create: host error word: %s", hipGetErrorString(e)));
    *p->host_err = 0u;
    if (p->layout == rs::LAYOUT_SOA && sorts) p->tmp_v = p->tmp_k + d.count;
    if ((e = hipMemset(p->ptot, 0, 4ull * (rs::kTotalsMax + kTicketWords))) != hipSuccess ||
        (e = hipMemset(p->status, 0, 8ull * p->status_words)) != hipSuccess)
        return cleanup(fail(RS_ERR_HIP, "rs_plan_create: hipMemset failed: %s", hipGetErrorString(e)));
    *out = p;
    return RS_OK;
}

RS_EXPORT void rs_plan_destroy(rs_plan* p) {
    if (!p) return;
    DeviceGuard guard(p->desc.device);
    p->timer.drain();
    (void)hipFree(p->tmp_k);
    (void)hipFree(p->tmp2);
    (void)hipFree(p->counts);
    (void)hipFree(p->totals);
    (void)hipFree(p->flags);
    (void)hipFree(p->ptot);
    (void)hipFree(p->status);
    (void)hipFree(p->msd);
    (void)hipFree(p->split);
    (void)hipFree(p->ns);
    if (p->host_err) (void)hipHostFree(p->host_err);
    if (p->done) (void)hipEventDestroy(p->done);
    delete p;
}

// Enqueue every launch of one sort (n > kTinyMax) on stream s.
// The four LSD passes of a separate-arrays sort gated on `gate` (the hybrid MSD path's fallback):
// src (arrays, or records) -> records -> records -> records -> uk / uv, through the plan's two records
// buffers; pass 0's totals must be in ptot, later passes count theirs.
static rs_status enqueue_lsd_gated(rs_plan* p, const uint32_t* sk, const uint32_t* sv, bool in_aos,
                                   uint32_t* uk, uint32_t* uv, uint32_t n, const uint32_t* gate,
                                   hipStream_t s) {
    constexpr int A = rs::LAYOUT_AOS, S = rs::LAYOUT_SOA;
    uint32_t* ra = p->tmp_k;
    uint32_t* rb = p->tmp2;
    struct Step { const uint32_t* ik; const uint32_t* iv; uint32_t* ok; uint32_t* ov; int LL; };
    const Step steps[4] = {{sk, sv, ra, nullptr, layout_pair(in_aos ? A : S, A)},
                           {ra, nullptr, rb, nullptr, layout_pair(A, A)},
                           {rb, nullptr, ra, nullptr, layout_pair(A, A)},
                           {ra, nullptr, uk, uv, layout_pair(A, S)}};
    p->scatter_kind = RS_KERNEL_FALLBACK;
    uint32_t shift = 0;
    rs_status st = RS_OK;
    for (uint32_t i = 0; i < 4 && st == RS_OK; ++i, shift += 8)
        st = run_pass(p, steps[i].ik, steps[i].iv, steps[i].ok, steps[i].ov, n, shift, 8, steps[i].LL,
                      gate, (int)i, s, /*onesweep=*/true);
    p->scatter_kind = RS_KERNEL_SCATTER;
    return st;
}

// The bucket split's launches (rs_kernels.hpp, "splitting over-full buckets"; each exits at once
// unless its gate is set): level 2's counts, its pass R2 -> R3 by byte 1, the sub-buckets' sort
// R3 -> output (two tiles), level 3's counts and its pass R3 -> output by byte 0.  R2 / R3: records
// (keys only: keys); output: the caller's arrays, records (out_aos) or keys.
static rs_status enqueue_split(rs_plan* p, const rs::SplitWs& sw, bool keys, bool out_aos, uint32_t* r2,
                               uint32_t* r3, uint32_t* uk, uint32_t* uv, uint32_t n32, hipStream_t s) {
    constexpr int A = rs::LAYOUT_AOS, S = rs::LAYOUT_SOA, K = rs::LAYOUT_KEYS;
    // the passes' tiles must be the split tables' (kSplitTile): keys only, the 512 x 32 tiles
    static_assert(kLarge.tile == (int)rs::kSplitTile, "split passes: 16K-record tiles");
    constexpr bool keys512 = kLargeKeys.tile == (int)rs::kSplitTile;
    constexpr int KB_ = keys512 ? kLargeKeys.block : kLarge.block, KK = keys512 ? kLargeKeys.kpt : kLarge.kpt;
    const bool ballot = p->rank_mode == rs::RANK_BALLOT;
    constexpr int A0 = rs::RANK_LDS_ATOMIC, B0 = rs::RANK_BALLOT;
    const uint32_t cgrid = 2u * p->cus;
    auto count = [&](const uint32_t* rec, uint32_t shift, bool level3) {
        RoctxRange r(level3 ? "rsort.msd.split3_count" : "rsort.msd.split2_count");
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(cgrid), dim3(1024), 0, s, rec, sw, shift); };
        if (keys) level3 ? go(rs::k_split_count<1, 3>) : go(rs::k_split_count<1, 2>);
        else level3 ? go(rs::k_split_count<2, 3>) : go(rs::k_split_count<2, 2>);
    };
    rs_status st = RS_OK;
    // one timed span (RS_KERNEL_SPLIT) for the split's launches, each also a roctx range
    p->timer.run(RS_KERNEL_SPLIT, s, [&] {
        count(r2, 8u, false);
        st = next_epoch(p, s);
        if (st != RS_OK) return;
        {
            RoctxRange r("rsort.msd.split2_pass");
            if (keys)
                launch_msd_pass<K, K, 2, false, KB_, KK>(p, r2, nullptr, r3, nullptr, n32, 8u, sw.smax2, nullptr,
                                                         p->tickets + 6, sw.gate2, sw.tab2, sw.rows2, s);
            else
                launch_msd_pass<A, A, 2>(p, r2, nullptr, r3, nullptr, n32, 8u, sw.smax2, nullptr, p->tickets + 6,
                                         sw.gate2, sw.tab2, sw.rows2, s);
        }
        {
            RoctxRange r("rsort.msd.split2_bucket");
            auto go = [&](auto lo) {
                constexpr int LO = decltype(lo)::value;
                // one sub-bucket per workgroup (65536 of them: 256 huge buckets; more are taken
                // grid-stride), so the hardware overlaps the workgroups' load latencies
                // (a grid-stride over at most 24 workgroups per CU: gated off - no over-full bucket, the
                // usual case - 65536 workgroups cost 16 us of dispatch, this grid ~4)
                auto small = [&](auto kern) {
                    const uint32_t grid = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(65536u, 256ull * sw.smax2),
                                                                       24ull * p->cus);
                    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, (const uint32_t*)r3, sw, uk, uv);
                };
                auto large = [&](auto kern) {   // the sub-buckets the first launch listed
                    static const uint32_t per_cu = resident_per_cu(kern, 512);
                    hipLaunchKernelGGL(kern, dim3(p->cus * per_cu), dim3(512), 0, s, (const uint32_t*)r3, sw, uk, uv);
                };
                // 4352-record tiles at 3 workgroups per CU (<= 168 VGPRs); 512 x 34 = 17408 at one
                // (two waves per SIMD: <= 256 VGPRs)
                ballot ? small(rs::k_bucket_sort8<256, 17, B0, LO, 3>) : small(rs::k_bucket_sort8<256, 17, A0, LO, 3>);
                ballot ? large(rs::k_bucket_sort8<512, 34, B0, LO, 2, false, true>)
                       : large(rs::k_bucket_sort8<512, 34, A0, LO, 2, false, true>);
            };
            if (keys) go(std::integral_constant<int, K>{});
            else if (out_aos) go(std::integral_constant<int, A>{});
            else go(std::integral_constant<int, S>{});
        }
        count(r3, 0u, true);
        st = next_epoch(p, s);
        if (st != RS_OK) return;
        RoctxRange r("rsort.msd.split3_pass");
        if (keys)
            launch_msd_pass<K, K, 2, false, KB_, KK>(p, r3, nullptr, uk, nullptr, n32, 0u, sw.smax3, nullptr,
                                                     p->tickets + 7, sw.gate3, sw.tab3, sw.rows3, s);
        else if (out_aos)
            launch_msd_pass<A, A, 2>(p, r3, nullptr, uk, nullptr, n32, 0u, sw.smax3, nullptr, p->tickets + 7,
                                     sw.gate3, sw.tab3, sw.rows3, s);
        else
            launch_msd_pass<A, S, 2>(p, r3, nullptr, uk, uv, n32, 0u, sw.smax3, nullptr, p->tickets + 7,
                                     sw.gate3, sw.tab3, sw.rows3, s);
    }, "rsort.msd.split");
    if (st != RS_OK) return st;
    HIP_TRY(hipGetLastError());
    return RS_OK;
}

// The presorted path (rs_presorted.hpp) of a check_order sort, in place on the caller's data (uk /
// uv: arrays, keys, or records in uk): mark -> decide -> extract -> the extraction's sort (its four
// 8-bit digit totals from one read, then four one-sweep passes) -> gather -> bounds -> save ->
// rank -> merge in place: 13 launches.  Every launch after k_ns_decide exits at once unless the device found the input nearly
// sorted; k_ns_merge then flags the data sorted (ctl[5]) and the radix path enqueued behind finds
// it in order (the hybrid path's histogram read is skipped outright: k_hist16_in's `skip`).
#if !RS_KNOB_OPEN || !defined(RS_NS_MERGE_NT)
#undef RS_NS_MERGE_NT
#define RS_NS_MERGE_NT 512   // k_ns_merge threads per workgroup (one tile each)
#endif
constexpr uint32_t kNsMergeNT = RS_NS_MERGE_NT;
static rs_status enqueue_presorted(rs_plan* p, uint32_t* uk, uint32_t* uv, uint32_t n, hipStream_t s) {
    constexpr int K = rs::LAYOUT_KEYS, S = rs::LAYOUT_SOA, A = rs::LAYOUT_AOS;
    const NsWs w = ns_layout(p->ns, p->capacity);
    const uint32_t cap = ns_cap_for(n);
    if (n > ns_keys(p->capacity) || cap > ns_cap_for(ns_keys(p->capacity)))
        return fail(RS_ERR_INVALID_ARG, "internal: %u keys exceed the presorted workspace", n);
    const uint32_t ntiles = (n + rs::kNsTile - 1) / rs::kNsTile;
    const uint32_t fm = full_mask(p->bit_count);
    const int L = p->layout;
    const uint32_t* gate = w.ctl + rs::kNsGate;
    // the extraction sort: 16K-key tiles (cap is a whole number of them; 4K-key tiles measured
    // slower: 27 vs 20 us per pass at config 4's 2M), one look-back status word per (tile, digit)
    const uint32_t stiles = cap / (uint32_t)kLarge.tile;
    if ((uint64_t)stiles * 256u > p->status_words)
        return fail(RS_ERR_INVALID_ARG, "internal: %u extraction tiles exceed the plan's status words", stiles);
    p->last_ns = true;
    HIP_TRY(hipMemsetAsync(w.ctl, 0, 4 * rs::kNsCtlWords, s));
    // persistent grids: as many workgroups as are resident, tiles taken in order
    auto resident = [&](auto kern, uint32_t units, uint32_t block) {
        static const uint32_t per_cu = resident_per_cu(kern, (int)block);
        return std::max(1u, std::min<uint32_t>(units, p->cus * per_cu));
    };
    // the order scan (k_ns_mark) is timed as the order check it is (RS_KERNEL_CHECK), the rest of the
    // path as RS_KERNEL_PRESORTED
    p->timer.run(RS_KERNEL_CHECK, s, [&] {
        auto probe = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(rs::kNsProbe / 256u), dim3(256), 0, s, (const uint32_t*)uk, n, fm, w.ctl);
        };
        L == A ? probe(rs::k_ns_probe<A>) : probe(rs::k_ns_probe<S>);
        auto mark = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(resident(kern, ntiles, 256)), dim3(256), 0, s, (const uint32_t*)uk, n, fm,
                               w.bitmap, w.tcnt, w.tbnd, reinterpret_cast<uint2*>(w.samp), w.ctl);
        };
        L == A ? mark(rs::k_ns_mark<A>) : mark(rs::k_ns_mark<S>);   // (keys only reads as SOA)
    }, "rsort.presorted.mark");
    HIP_TRY(hipGetLastError());
    p->timer.run(RS_KERNEL_PRESORTED, s, [&] {
        hipLaunchKernelGGL(rs::k_ns_decide, dim3((ntiles + 1023u) / 1024u), dim3(1024), 0, s, (const uint32_t*)w.tcnt,
                           (const uint32_t*)w.tbnd, ntiles, cap, w.toff, w.csum, w.coff, w.sub, w.ctl);
        auto extract = [&](auto kern) {
            // (a wave per tile: a persistent grid measured slower, 75 vs 63 us at config 4)
            hipLaunchKernelGGL(kern, dim3((ntiles + 3u) / 4u), dim3(256), 0, s,
                               (const uint32_t*)uk, (const uint32_t*)uv, n, fm,
                               cap, (const uint32_t*)w.bitmap, (const uint32_t*)w.toff, (const uint32_t*)w.coff,
                               (const uint32_t*)w.ctl, w.ek, w.ei, w.sk, w.sv, w.sp, w.wpre);
        };
        L == A ? extract(rs::k_ns_extract<A>) : L == S ? extract(rs::k_ns_extract<S>) : extract(rs::k_ns_extract<K>);
        // the extraction (masked key, extraction index) sorted stably, ek / ei -> ek2 / ei2 -> ... ->
        // ek / ei: every pass's digit totals from one read (they do not depend on the order), then
        // the passes (16K-key tiles, decoupled look-back)
        hipLaunchKernelGGL(rs::k_ns_totals, dim3(std::min<uint32_t>(cap / 2048u, p->cus)), dim3(256), 0, s,
                           (const uint32_t*)w.ek, cap, (const uint32_t*)w.ctl, w.sub);
    }, "rsort.presorted.extract");
    HIP_TRY(hipGetLastError());
    const bool ballot = p->rank_mode == rs::RANK_BALLOT;
    for (uint32_t i = 0; i < 4; ++i) {
        if (rs_status st = next_epoch(p, s)) return st;
        const bool odd = i & 1u;
        p->timer.run(RS_KERNEL_PRESORTED, s, [&] {
            auto go = [&](auto kern) {
                hipLaunchKernelGGL(kern, dim3(resident(kern, stiles, kLarge.block)), dim3(kLarge.block), 0, s,
                                   (const uint32_t*)(odd ? w.ek2 : w.ek), (const uint32_t*)(odd ? w.ei2 : w.ei),
                                   odd ? w.ek : w.ek2, odd ? w.ei : w.ei2, cap, 8u * i, 255u, stiles,
                                   (const uint32_t*)(w.sub + 256u * i), p->status, w.sub + 1024u + i,
                                   w.sub + 1024u + 16u, (uint32_t*)nullptr, 0u, 0u, p->epoch, gate, (int)i,
                                   (uint32_t*)nullptr, 0xFFFFFFFFu, p->spin_max, p->host_err_dev,
                                   (const uint32_t*)nullptr, (const uint32_t*)nullptr, 0u, 0xFFFFFFFFu);
            };
            constexpr int B = kLarge.block, KP = kLarge.kpt;
            ballot ? go(rs::k_onesweep<8, B, KP, S, rs::RANK_BALLOT>) : go(rs::k_onesweep<8, B, KP, S, rs::RANK_LDS_ATOMIC>);
        }, "rsort.presorted.sort");
        HIP_TRY(hipGetLastError());
    }
    p->timer.run(RS_KERNEL_PRESORTED, s, [&] {
        hipLaunchKernelGGL(rs::k_ns_gather, dim3(std::min<uint32_t>(cap / 256u, 4u * p->cus)), dim3(256), 0, s,
                           (const uint32_t*)w.ei, (const uint32_t*)w.sp, (const uint32_t*)w.sk, (const uint32_t*)w.sv,
                           (const uint32_t*)w.ctl, w.bp, w.bk, w.bv);
        auto bounds = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((ntiles + 1u + 255u) / 256u), dim3(256), 0, s, (const uint32_t*)uk, n, fm,
                               (const uint32_t*)w.bitmap, ntiles, (const uint32_t*)w.ek, (const uint32_t*)w.bp,
                               (const uint32_t*)w.ctl, w.blo);
        };
        L == A ? bounds(rs::k_ns_bounds<A>) : bounds(rs::k_ns_bounds<S>);
        auto save = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(resident(kern, ntiles, 256)), dim3(256), 0, s, (const uint32_t*)uk,
                               (const uint32_t*)uv, n, (const uint32_t*)w.toff, (const uint32_t*)w.coff,
                               (const uint32_t*)w.blo,
                               (const uint32_t*)w.ctl, p->tmp_k, w.tileof);
        };
        L == A ? save(rs::k_ns_save<A>) : L == S ? save(rs::k_ns_save<S>) : save(rs::k_ns_save<K>);
        auto rank = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(cap / 256u), dim3(256), 0, s, (const uint32_t*)uk, n, fm,
                               (const uint32_t*)w.bitmap, (const uint32_t*)w.wpre,
                               reinterpret_cast<const uint2*>(w.samp), (const uint32_t*)w.tileof,
                               (const uint32_t*)w.ek, (const uint32_t*)w.bp, (const uint32_t*)w.ctl, w.rank);
        };
        L == A ? rank(rs::k_ns_rank<A>) : rank(rs::k_ns_rank<S>);
        auto merge = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(resident(kern, ntiles, kNsMergeNT)), dim3(kNsMergeNT), 0, s, uk, uv, n,
                               (const uint32_t*)w.bitmap, (const uint32_t*)w.toff, (const uint32_t*)w.coff,
                               (const uint32_t*)w.blo, (const uint32_t*)w.rank, (const uint32_t*)w.bk,
                               (const uint32_t*)w.bv, w.ctl, (const uint32_t*)p->tmp_k);
        };
        L == A ? merge(rs::k_ns_merge<A, kNsMergeNT>) : L == S ? merge(rs::k_ns_merge<S, kNsMergeNT>)
               : merge(rs::k_ns_merge<K, kNsMergeNT>);
    }, "rsort.presorted.merge");
    HIP_TRY(hipGetLastError());
    return RS_OK;
}

// The hybrid MSD path (rs_kernels.hpp, "hybrid MSD path"): the 16-bit bucket histogram of the
// input and the device's choice first, then top-byte pass -> segmented next-byte pass -> in-LDS
// bucket sort; the LSD passes on the input enqueued behind, gated the other way (skewed keys).
// Input (sk, sv): arrays, or records (in_aos: the texture layout in place, or a group sort's
// received region).  Output (uk, uv): arrays, or records in place (out_aos).  R1 = records in
// tmp_k (which holds the histogram rows before that); R2 = records in tmp2, or the caller's
// buffer itself when the records are sorted in place (the input is consumed by pass 0).
// Keys known to lie in [kbase, kbase + 2^vbits) (a group sort's received buckets) are sorted by
// their vbits range-relative bits: digits of key - kbase at vbits - 8 and vbits - 16 (a key
// outside the range sends the device to the 32-bit LSD passes).
// Region form (region_hist != null; rs_plan_sort_region, records -> arrays): the input records are
// already grouped by top byte (the senders' partition was pass 0) and region_hist holds their 16-bit
// bucket counts (nbuckets of them populated): no histogram read, no pass 0; R1 = the input, R2 =
// records in tmp_k.
static rs_status enqueue_sort_msd(rs_plan* p, const uint32_t* sk, const uint32_t* sv, bool in_aos,
                                  uint32_t* uk, uint32_t* uv, bool out_aos, uint64_t n, hipStream_t s,
                                  uint32_t kbase = 0, uint32_t vbits = 32,
                                  const uint32_t* region_hist = nullptr, uint32_t top_lo = 0, uint32_t top_hi = 256) {
    // the populated 16-bit buckets: all, or a region's top bytes
    const uint32_t b_lo = top_lo << 8, b_cnt = (top_hi - top_lo) << 8, nbuckets = b_cnt;
    constexpr int A = rs::LAYOUT_AOS, S = rs::LAYOUT_SOA, K = rs::LAYOUT_KEYS;
    const bool keys = p->layout == rs::LAYOUT_KEYS;   // keys only: R1 = tmp_k, R2 = the caller's keys
    const bool region = region_hist != nullptr;
    const uint32_t n32 = (uint32_t)n;
    const uint32_t range = vbits >= 32 ? 0xFFFFFFFFu : (1u << vbits) - 1u;
    uint32_t* r1 = region ? const_cast<uint32_t*>(sk) : p->tmp_k;   // region: only read
    uint32_t* r2 = region ? p->tmp_k : ((out_aos || keys) ? uk : p->tmp2);
    uint32_t* hist16 = p->msd;
    uint32_t* base16 = hist16 + 65536;
    uint32_t* segtab = base16 + 65536;
    uint32_t* gates = segtab + 1024;
    uint32_t* mtot = gates + 64;
    uint32_t* over = mtot + 1024;
    uint32_t* cbase = over + 1 + rs::kOverMax;   // [row][top byte]: chunk starts inside the segments
    uint32_t* top_tot = mtot + 768;
    uint32_t* big = mtot + 1;          // a 16-bit bucket over the large bucket tile
    uint32_t* sstart = segtab + 257;   // top-byte segment starts (bucket bases are relative to them)
    // the bucket split of over-full 16-bit buckets (whole-range sorts and regions; the key-range form
    // keeps the LSD fallback): level 2 writes into a records buffer that is free by then (R1, or a
    // region's tmp2).  Sorts with the split then enqueue no LSD fallback at all (strict: the device's
    // checks can only fail on a counting fault - or, for a region, a table that does not describe
    // its records - reported as a device error; round 6: the region's five gated-off fallback
    // launches cost 0.031 ms per region, 0.124 of a rank's 4.0 ms at config 5's shape).
    bool split = p->split && p->split_on && (region ? p->tmp2 != nullptr : (kbase == 0u && vbits == 32u));
#if RS_SWEEP
    if (RS_KNOB("RSORT_EXP_RING", 0) > 0) split = false;
#endif
    const bool strict = split;
    p->last_split = split;
    uint32_t* r3 = region ? p->tmp2 : r1;
    if (p->high_half) {
        // test hook (rs_plan_debug.high_half): the records buffers the bucket kernels read (R2, and the
        // split's R3) start where the low 32 bits of the address are 2^31, so that the buckets' base
        // addresses have bit 31 of their low word set (round 5's sign-extension fault in load_bucket);
        // the plan's spare capacity holds the shift
        const uint64_t rbytes = 8ull * ((p->capacity + kRecPad - 1) / kRecPad * kRecPad);
        auto high = [&](uint32_t*& buf) -> bool {
            if (buf != p->tmp_k && buf != p->tmp2) return true;   // the caller's buffer: left alone
            const uint64_t a = (uint64_t)(uintptr_t)buf & 0xFFFFFFFFull, need = 8ull * (n + kRecPad);
            // already wholly in the upper half of a 4 GiB window: no shift; else up to 2^31 + need bytes
            const uint64_t o = (a >= 0x80000000ull && a + need <= 0x100000000ull) ? 0ull
                             : (0x80000000ull - a) & 0xFFFFFFFFull;   // (a multiple of 4)
            if (o + need > rbytes) return false;
            buf += o / 4u;
            return true;
        };
        const bool r3_own = r3 != r1;   // (whole sorts: R3 is R1, shifted with it below only if separate)
        if (!high(r2) || (r3_own && !high(r3)))
            return fail(RS_ERR_CAPACITY, "rs_plan_debug.high_half: the plan's capacity (%llu) leaves no room to "
                        "shift %llu records to a 2^31 address", (unsigned long long)p->capacity, (unsigned long long)n);
    }
    rs::SplitWs sw{};
    if (split) {
        uint32_t* q = p->split;
        sw.gate2 = q;
        sw.gate3 = q + 16;
        q += 32;
        sw.huge = q;
        q += 1 + p->smax2;
        sw.tab2 = q;
        q += 3ull * p->smax2 + 2;
        sw.arrive2 = q;
        q += p->smax2 + 1ull;
        sw.rows2 = q;
        q += 256ull * p->smax2;
        sw.tab3 = q;
        q += 3ull * p->smax3 + 2;
        sw.arrive3 = q;
        q += p->smax3 + 1ull;
        sw.rows3 = q;
        q += 256ull * p->smax3;
        sw.mid = q;
        sw.midmax = split_midmax(p->capacity);
        q += 1ull + sw.midmax;
        sw.chunks = q;
        sw.chunkmax = split_chunkmax(p->capacity);
        sw.smax2 = p->smax2;
        sw.smax3 = p->smax3;
        sw.tmax = (uint32_t)std::min<uint64_t>(p->status_words / 256u, 0xFFFFFFFFu);
        sw.hist16 = hist16;
        sw.base16 = base16;
        sw.err = p->tickets + 16;
        sw.host_err = p->host_err_dev;
        sw.strict = strict ? 1u : 0u;
        sw.n = n32;
    }
    // keys only, pass tile configuration (rs_plan_debug.msd_keys_cfg): 0 = 1024 x 16, 1 = 512 x 32 (two
    // workgroups per CU), 2 = 1024 x 32 (32K-key tiles: 512-B digit runs, as long as a 16K-record tile's)
    const int keys_cfg = p->msd_keys_cfg;
    const uint32_t tile = (keys && keys_cfg == 2) ? 2u * kLarge.tile : (uint32_t)kLarge.tile;
    const uint32_t ntiles = (uint32_t)((n + tile - 1) / tile);
    // the segmented pass has up to ntiles + 256 tiles; each needs its look-back status words
    if ((uint64_t)(ntiles + 257) * 256u > p->status_words)
        return fail(RS_ERR_INVALID_ARG, "internal: %u segmented tiles exceed the plan's %llu status words",
                    ntiles + 257, (unsigned long long)p->status_words);
    p->last_hybrid = true;
    p->last_ns = false;
    // the pass totals, tickets and error word are zeroed by k_hist16_reduce (nothing reads them before)
    // 16-bit buckets: a tile sized to the mean bucket + 4 sigma of a uniform population takes
    // every bucket that fits it (at 2^28 keys: 4352 records, ~2 buckets over it), the large tile
    // the listed rest
    const double mean = (double)n / std::max(1u, nbuckets);
    const double slack = RS_KNOB("RSORT_BUCKET_SLACK", 1.0);
    const uint32_t want = (uint32_t)(mean * slack + 4.0 * std::sqrt(mean));
    constexpr uint32_t bb = 256;
    // (KV 256 x 34 = 8704 records: 2^29 keys, two workgroups per CU)
    static const uint32_t kpts[] = {4, 8, 12, 17, 18, 24, 34};
    static const uint32_t kpts_keys[] = {4, 5, 9, 17, 24, 0, 0};   // 64M keys: 1280-key tiles
    uint32_t small_cap = 0, small_kpt = 0;
    for (uint32_t kpt : keys ? kpts_keys : kpts)
        if (kpt && !small_cap && want <= bb * kpt) { small_cap = bb * kpt; small_kpt = kpt; }
    // keys only, buckets of up to ~1K keys (<= ~80M keys): one wave per bucket
    // (k_bucket_sort_keys_wave, 64 x wave_kpt keys; rs_plan_debug.kbucket_wave = 0 keeps the workgroup kernel)
    const bool wave_ok = p->kbucket_wave;
    uint32_t wave_kpt = 0;
    if (keys && wave_ok) {
        for (uint32_t kpt : {10u, 18u})
            if (!wave_kpt && want <= 64u * kpt) wave_kpt = kpt;
        if (wave_kpt) small_cap = 64u * wave_kpt;
    }
    // with values, buckets of up to 17408 records (2^30 keys): 1024 x 17 records, 8-byte staging,
    // one workgroup per CU (8-byte staging measured 1.7x faster than the wide kernel's 4-byte
    // positions + value exchange at 2^29: 1.67 vs 2.87 ms, profiles/r03_wide_modes.jsonl)
    const bool big_tile = !keys && !small_cap && want <= 1024u * 17u;
    if (big_tile) small_cap = 1024u * 17u;
    // buckets too large for every workgroup tile (~2^31 keys): the wide kernel takes every bucket,
    // one workgroup each, and nothing is listed
    const bool wide_all = small_cap == 0;
    if (wide_all) small_cap = kBucketCap;
    // one histogram row per CU in tmp_k (R1 is written only after the rows are added)
    uint32_t* range_bad = mtot;
    // sweep: RSORT_HIST16_DIV = one row per `div` CUs (fewer rows to write and add)
    const uint32_t hdiv = std::max(1u, (uint32_t)RS_KNOB("RSORT_HIST16_DIV", 1));
    const uint32_t hrows = region ? 1u : std::max(1u, p->cus / hdiv);
    // check_order (whole-range sorts; the region form never checks): the input's order check rides
    // on the histogram read (p->flags[0]); the byte-0 rows follow the histogram rows and flags
    // check_order rides on the histogram read only for in-place sorts: a sorted input then needs
    // nothing moved, which is right only when the output IS the input (records -> arrays and
    // out-of-place sorts always run their passes)
    const bool in_place = sk == uk && in_aos == out_aos && (in_aos || sv == uv);
    const bool chk = p->check_order && !region && kbase == 0u && vbits == 32u && in_place;
    // static work splits (k_static_pass, no look-back) for the passes with values: pass 0 over the
    // histogram's input chunks, pass 1 over the top-byte segments when they are balanced (the
    // device picks; else the look-back pass).  Keys only keeps the look-back passes (two 512-thread
    // workgroups per CU).
    const bool static_p0 = !region && !keys && p->static_passes && hrows <= rs::kMaxRows;
    const bool static_p1 = !keys && p->static_passes;
    // XCD-local claims of MSD pass 0 (k_msd_pass XC): its chunks' digit bases from the histogram rows
    // (k_hist16_reduce's cbase); the keys-only passes (k_onesweep) keep one counter
    const uint32_t* xc_cbase = (!region && !keys && (p->xcd_claims == 1 || p->xcd_claims == 2) && hrows <= rs::kMaxRows) ? cbase : nullptr;
    // (the fallback's byte-0 totals: only where a fallback is enqueued)
    uint32_t* b0rows = (chk && !strict) ? p->tmp_k + (size_t)hrows * 65537u : nullptr;
    if (!region && (uint64_t)n / hrows >= (uint64_t)rs::kEvMax * rs::kHalfT)   // k_hist16_in's crossing log
        return fail(RS_ERR_CAPACITY, "%llu keys over %u histogram rows (at most 2^27 keys per row)",
                    (unsigned long long)n, hrows);
    if (chk) HIP_TRY(hipMemsetAsync(p->flags, 0, 16 * 4, s));
    // check_order: the presorted path first (nearly-sorted input is sorted there; the histogram
    // read is then skipped and finds nothing to do)
    const uint32_t* ns_skip = nullptr;
    if (chk && p->ns && p->ns_on && n <= ns_keys(p->capacity)) {   // (the LSD caller's pre-check: an
        // input over the workspace skips the optional path instead of failing the sort)
        if (rs_status st = enqueue_presorted(p, uk, uv, n32, s)) return st;
        ns_skip = p->ns + 5;
    }
    p->timer.run(RS_KERNEL_HISTOGRAM, s, [&] {
        if (region) {   // the senders counted: one row, their table
            hipLaunchKernelGGL(rs::k_region_rows, dim3(256), dim3(256), 0, s, region_hist, p->tmp_k, over, big,
                               sw.huge);
            hipLaunchKernelGGL(rs::k_hist16_reduce<false>, dim3(256), dim3(1024), 0, s, (const uint32_t*)p->tmp_k,
                               1u, hist16, top_tot, range_bad, base16, small_cap, kBucketCap, over, big,
                               p->ptot, (uint32_t)(rs::kTotalsMax + kTicketWords), (const uint32_t*)nullptr,
                               (uint32_t*)nullptr, sw.huge, p->smax2);
            return;
        }
        // 16-byte aligned records: two per load (sweep: RSORT_HIST16_NARROW=1 keeps one per 8-byte load)
        const bool narrow = RS_KNOB("RSORT_HIST16_NARROW", 0) == 1;
        // the whole 32-bit range: the specialised counting (sweep: RSORT_HIST16_GENERIC=1 keeps the generic one)
        const bool generic = RS_KNOB("RSORT_HIST16_GENERIC", 0) == 1;
        const bool full = !generic && kbase == 0u && vbits == 32u;
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(hrows), dim3(1024), 0, s, sk, n32, p->tmp_k, kbase, range, vbits - 16,
                               over, big, chk ? p->flags : (uint32_t*)nullptr, b0rows, sw.huge, ns_skip);
        };
        if (chk && b0rows) {   // check_order: the order check and the fallback's byte-0 totals ride along
            if (in_aos && !narrow && ((uintptr_t)sk & 15u) == 0) go(rs::k_hist16_in<A, true, true, 2>);
            else if (in_aos) go(rs::k_hist16_in<A, false, true, 2>);
            else go(rs::k_hist16_in<S, false, true, 2>);
        } else if (chk) {      // the order check only (no fallback enqueued)
            if (in_aos && !narrow && ((uintptr_t)sk & 15u) == 0) go(rs::k_hist16_in<A, true, true, 1>);
            else if (in_aos) go(rs::k_hist16_in<A, false, true, 1>);
            else go(rs::k_hist16_in<S, false, true, 1>);
        } else if (in_aos && !narrow && ((uintptr_t)sk & 15u) == 0) {
            full ? go(rs::k_hist16_in<A, true, true>) : go(rs::k_hist16_in<A, true>);
        } else if (in_aos) {
            full ? go(rs::k_hist16_in<A, false, true>) : go(rs::k_hist16_in<A>);
        } else {
            full ? go(rs::k_hist16_in<S, false, true>) : go(rs::k_hist16_in<S>);
        }
        // the reduction also lays out every top byte's buckets (bases inside the segment, the
        // overflow list, the oversize flag): the plan kernel is left with the 256 segments
        hipLaunchKernelGGL(rs::k_hist16_reduce<true>, dim3(256), dim3(1024), 0, s, (const uint32_t*)p->tmp_k,
                           hrows, hist16, top_tot, range_bad, base16, small_cap, kBucketCap, over, big,
                           p->ptot, (uint32_t)(rs::kTotalsMax + kTicketWords), (const uint32_t*)b0rows,
                           (static_p0 || xc_cbase) ? cbase : (uint32_t*)nullptr, sw.huge, p->smax2, ns_skip);
    }, region ? "rsort.msd.region_table" : "rsort.msd.hist16");
    HIP_TRY(hipGetLastError());
    p->timer.run(RS_KERNEL_SCAN, s, [&] {
        auto plan = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, s, (const uint32_t*)top_tot, segtab, 0xFFFFFFFFu, over,
                               (const uint32_t*)big, gates, (const uint32_t*)range_bad, n32,
                               chk ? (const uint32_t*)p->flags : (const uint32_t*)nullptr, top_lo, top_hi, sw);
        };
        if (tile == 2u * kLarge.tile) plan(rs::k_msd_plan<2 * kLarge.tile>);
        else plan(rs::k_msd_plan<kLarge.tile>);
    }, "rsort.msd.plan");
    HIP_TRY(hipGetLastError());
    // (the fallback's launches on a low-priority side stream forked here, so that their gated-off
    // launches overlap the MSD passes, measured slower: the scatter passes lost 5-25 % beside
    // them, profiles/r03_side_stream_nogo/)
    hipStream_t fs = s;
    const uint32_t* g_msd = gates + rs::kGateMsd;
    // R2 replaced by a power-of-two ring (sweep experiment RSORT_EXP_RING = log2 records; the
    // results are then invalid: timing of an Infinity-Cache-resident R2 only)
    uint32_t* ring = nullptr;
    uint32_t rmask = 0xFFFFFFFFu;
#if RS_SWEEP
    if (const int rb = (int)RS_KNOB("RSORT_EXP_RING", 0); rb > 0 && !keys && !out_aos) {
        static uint32_t* buf = nullptr;
        if (!buf) HIP_TRY(hipMalloc((void**)&buf, 8ull * ((1ull << rb) + 65536)));
        ring = buf;
        rmask = (1u << rb) - 1u;
    }
#endif
    // MSD pass 0: input -> R1 records, partitioned by the top byte (region form: done by the senders)
    if (rs_status st = next_epoch(p, s)) return st;
    const bool keys_wide = keys_cfg == 0;
    if (!region) p->timer.run(RS_KERNEL_SCATTER, s, [&] {
        if (keys && keys_wide)
            launch_msd_pass<K, K, 0>(p, sk, nullptr, r1, nullptr, n32, vbits - 8, ntiles, top_tot, p->tickets + 4,
                                     g_msd, nullptr, nullptr, s);
        else if (keys && keys_cfg == 2)
            launch_msd_pass<K, K, 0, false, 1024, 32>(p, sk, nullptr, r1, nullptr, n32, vbits - 8, ntiles, top_tot,
                                                      p->tickets + 4, g_msd, nullptr, nullptr, s);
        else if (keys)
            launch_msd_pass<K, K, 0, false, kLargeKeys.block, kLargeKeys.kpt>(
                p, sk, nullptr, r1, nullptr, n32, vbits - 8, ntiles, top_tot, p->tickets + 4, g_msd, nullptr,
                nullptr, s);
#if RS_SWEEP
        else if (static_p0)
            launch_static_pass0(p, sk, sv, in_aos, kbase != 0u, r1, n32, vbits - 8, hrows, g_msd, segtab, cbase, kbase, s);
#endif
        else if (in_aos && kbase)
            launch_msd_pass<A, A, 0, true>(p, sk, nullptr, r1, nullptr, n32, vbits - 8, ntiles, top_tot,
                                           p->tickets + 4, g_msd, nullptr, nullptr, s, kbase, 0xFFFFFFFFu, xc_cbase,
                                           hrows);
        else if (in_aos)
            launch_msd_pass<A, A, 0>(p, sk, nullptr, r1, nullptr, n32, vbits - 8, ntiles, top_tot,
                                     p->tickets + 4, g_msd, nullptr, nullptr, s, 0u, 0xFFFFFFFFu, xc_cbase, hrows);
        else if (kbase)
            launch_msd_pass<S, A, 0, true>(p, sk, sv, r1, nullptr, n32, vbits - 8, ntiles, top_tot,
                                           p->tickets + 4, g_msd, nullptr, nullptr, s, kbase, 0xFFFFFFFFu, xc_cbase,
                                           hrows);
#if RS_P0_SR2
        else   // 32K-record tiles staged in two rounds: 128-record digit runs (tools/run_probe.hip)
            launch_msd_pass<S, A, 0, false, kLarge.block, 2 * kLarge.kpt, 2>(
                p, sk, sv, r1, nullptr, n32, vbits - 8, (uint32_t)((n + 2 * kLarge.tile - 1) / (2 * kLarge.tile)),
                top_tot, p->tickets + 4, g_msd, nullptr, nullptr, s);
#else
        else
            launch_msd_pass<S, A, 0>(p, sk, sv, r1, nullptr, n32, vbits - 8, ntiles, top_tot, p->tickets + 4,
                                     g_msd, nullptr, nullptr, s, 0u, 0xFFFFFFFFu, xc_cbase, hrows);
#endif
    }, "rsort.msd.pass0");
    HIP_TRY(hipGetLastError());
    // MSD pass 1: R1 -> R2 records, by the next byte inside every top-byte segment
    if (rs_status st = next_epoch(p, s)) return st;
    p->timer.run(RS_KERNEL_SCATTER, s, [&] {
        if (keys && keys_wide)
            launch_msd_pass<K, K, 1>(p, r1, nullptr, r2, nullptr, n32, vbits - 16, ntiles + 257, nullptr,
                                     p->tickets + 5, g_msd, segtab, base16, s);
        else if (keys && keys_cfg == 2)
            launch_msd_pass<K, K, 1, false, 1024, 32>(p, r1, nullptr, r2, nullptr, n32, vbits - 16, ntiles + 257,
                                                      nullptr, p->tickets + 5, g_msd, segtab, base16, s);
        else if (keys)
            launch_msd_pass<K, K, 1, false, kLargeKeys.block, kLargeKeys.kpt>(
                p, r1, nullptr, r2, nullptr, n32, vbits - 16, ntiles + 257, nullptr, p->tickets + 5, g_msd,
                segtab, base16, s);
        else {
            // the static split when the device found the segments balanced, else the look-back pass
            // (each launch exits at once unless its gate is set)
#if RS_SWEEP
            if (static_p1 && !ring)
                launch_static_pass1(p, r1, r2, n32, vbits - 16, gates + rs::kGateSegStatic, segtab, base16, s);
#endif
            launch_msd_pass<A, A, 1>(p, r1, nullptr, ring ? ring : r2, nullptr, n32, vbits - 16, ntiles + 257, nullptr,
                                     p->tickets + 5, (static_p1 && !ring) ? gates + rs::kGateSegLookback : g_msd,
                                     segtab, base16, s, 0u, rmask);
        }
    }, "rsort.msd.pass1");
    HIP_TRY(hipGetLastError());
    const bool ballot = p->rank_mode == rs::RANK_BALLOT;
    constexpr int A0 = rs::RANK_LDS_ATOMIC, B0 = rs::RANK_BALLOT;
    p->timer.run(RS_KERNEL_BUCKET, s, [&] {
        auto small = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(b_cnt), dim3(bb), 0, s, ring ? ring : r2, hist16, base16, uk, uv, g_msd,
                               p->tickets + 16, 0u, (const uint32_t*)nullptr, kbase, (const uint32_t*)sstart, rmask,
                               b_lo, b_cnt);
        };
        auto big = [&](auto kern) {   // the 1024 x 17 tile (big_tile), one bucket per workgroup
            hipLaunchKernelGGL(kern, dim3(b_cnt), dim3(1024), 0, s, ring ? ring : r2, hist16, base16, uk, uv, g_msd,
                               p->tickets + 16, 0u, (const uint32_t*)nullptr, kbase, (const uint32_t*)sstart, rmask,
                               b_lo, b_cnt);
        };

#if RS_SWEEP
        // sweep only, keys only: a persistent grid whose workgroups load their next bucket while
        // sorting one (measured slower, 0.265 vs 0.245 ms)
        auto small_pf = [&](auto kern) {
            static const uint32_t per_cu = resident_per_cu(kern, bb);
            const uint32_t mult = std::max(1u, (uint32_t)RS_KNOB("RSORT_KBUCKET_GRID", 1));
            const uint32_t grid = std::min<uint32_t>(65536u, p->cus * per_cu * mult);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(bb), 0, s, r2, hist16, base16, uk, uv, g_msd,
                               p->tickets + 16, 0u, (const uint32_t*)nullptr, kbase, (const uint32_t*)sstart,
                               0xFFFFFFFFu, 0u, 65536u);
        };
#endif
        // the wide kernel: every bucket (wide_all), or the listed buckets over the population-sized
        // tile on a small persistent grid (sweep: RSORT_OVER_GRID workgroups)
        const uint32_t over_grid = std::max(1u, (uint32_t)RS_KNOB("RSORT_OVER_GRID", 256));
        // the listed buckets of at most 1024 x 8 records (at 2^28 uniform keys: the ~2 buckets just
        // over the primary tile) go to a 1024 x 8 tile first: one such bucket alone on the wide
        // kernel's 1024 x 34 slots took 0.034 ms, the length of the whole launch (profiles/r06/
        // xcd_claims); the wide kernel then takes the listed rest (min_cnt = 8192)
        const bool listed8 = !wide_all && small_cap < 8192u;
        auto listed = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(over_grid), dim3(1024), 0, s, ring ? ring : r2, hist16, base16, uk, uv,
                               g_msd, p->tickets + 16, small_cap, (const uint32_t*)over, kbase,
                               (const uint32_t*)sstart, rmask, b_lo, b_cnt);
        };
        auto large = [&](auto kern, uint32_t block) {
            hipLaunchKernelGGL(kern, dim3(wide_all ? b_cnt : over_grid), dim3(block), 0, s, ring ? ring : r2,
                               hist16, base16, uk, uv, g_msd, p->tickets + 16,
                               wide_all ? 0u : (listed8 ? 8192u : small_cap),
                               wide_all ? (const uint32_t*)nullptr : (const uint32_t*)over, kbase,
                               (const uint32_t*)sstart, rmask, vbits - 16, b_lo, b_cnt);
        };
        auto both = [&](auto lo) {
            constexpr int LO = decltype(lo)::value;
#define RS_BK(KP) case KP: ballot ? small(rs::k_bucket_sort<bb, KP, B0, LO, (KP <= 18 ? RS_BUCKET_MW : (KP == 34 ? 2 : 1))>) : small(rs::k_bucket_sort<bb, KP, A0, LO, (KP <= 18 ? RS_BUCKET_MW : (KP == 34 ? 2 : 1))>); break;
            if constexpr (LO == K) {
                bool wave_done = false;
#if RS_SWEEP
                // sweep only: 2 or 8 waves (buckets) per workgroup (RSORT_KWAVE_WPB), or more waves
                // per SIMD forced through the VGPR budget (RSORT_KWAVE_MW: spilled and was slower)
                const int wpb = (int)RS_KNOB("RSORT_KWAVE_WPB", 4), mw = (int)RS_KNOB("RSORT_KWAVE_MW", 1);
                if (wave_kpt == 18 && !ballot && (wpb == 2 || wpb == 8 || mw >= 5)) {
                    auto wave = [&](auto kern, int w) {
                        hipLaunchKernelGGL(kern, dim3(65536 / w), dim3(64 * w), 0, s, uk, (const uint32_t*)hist16,
                                           (const uint32_t*)base16, g_msd, (const uint32_t*)sstart);
                    };
                    if (wpb == 2) wave(rs::k_bucket_sort_keys_wave<18, A0, 2>, 2);
                    else if (wpb == 8) wave(rs::k_bucket_sort_keys_wave<18, A0, 8>, 8);
                    else if (mw == 7) wave(rs::k_bucket_sort_keys_wave<18, A0, 4, 7>, 4);
                    else if (mw == 6) wave(rs::k_bucket_sort_keys_wave<18, A0, 4, 6>, 4);
                    else wave(rs::k_bucket_sort_keys_wave<18, A0, 4, 5>, 4);
                    small_kpt = 0;
                    wave_done = true;
                }
#endif
                if (wave_kpt && !wave_done) {
                    constexpr int WPB = 4;
                    auto wave = [&](auto kern) {
                        // one bucket per wave; RS_KWAVE_PF (sweep): persistent waves, two resident
                        // grids' worth of workgroups
                        uint32_t grid = 65536 / WPB;
                        if (RS_KWAVE_PF) {
                            static const uint32_t per_cu = resident_per_cu(kern, 64 * WPB);
                            grid = std::min<uint32_t>(grid, 2u * per_cu * p->cus);
                        }
                        hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WPB), 0, s, uk, (const uint32_t*)hist16,
                                           (const uint32_t*)base16, g_msd, (const uint32_t*)sstart);
                    };
                    if (wave_kpt == 10)
                        ballot ? wave(rs::k_bucket_sort_keys_wave<10, B0, WPB>) : wave(rs::k_bucket_sort_keys_wave<10, A0, WPB>);
                    else
                        ballot ? wave(rs::k_bucket_sort_keys_wave<18, B0, WPB>) : wave(rs::k_bucket_sort_keys_wave<18, A0, WPB>);
                    small_kpt = 0;   // no workgroup-per-bucket launch
                }
#if RS_SWEEP
#define RS_BKP(KP) case KP: ballot ? small_pf(rs::k_bucket_sort<bb, KP, B0, LO, 4, 1>) : small_pf(rs::k_bucket_sort<bb, KP, A0, LO, 4, 1>); break;
                if (p->kbucket_pf) {
                    switch (small_kpt) {
                        RS_BKP(4) RS_BKP(5) RS_BKP(9) RS_BKP(17) RS_BKP(24)
                        default: break;
                    }
                    small_kpt = 0;
                }
#undef RS_BKP
#endif
                switch (small_kpt) {
                    RS_BK(4) RS_BK(5) RS_BK(9) RS_BK(17) RS_BK(24)
                    default: break;
                }
            } else {
                switch (small_kpt) {
                    RS_BK(4) RS_BK(8) RS_BK(12) RS_BK(17) RS_BK(18) RS_BK(24) RS_BK(34)
                    default: break;   // every bucket goes to the listed large-tile launch
                }
            }
#undef RS_BK
            // the listed buckets (none for uniform keys below ~2^29): the largest wide tile; every
            // bucket (wide_all): the smallest wide tile that holds the population's buckets (512 x 18:
            // three workgroups per CU, 512 x 34: two, 1024 x 34: one)
            if (big_tile)
                ballot ? big(rs::k_bucket_sort<1024, 17, B0, LO, 4>) : big(rs::k_bucket_sort<1024, 17, A0, LO, 4>);
            if (listed8)
                ballot ? listed(rs::k_bucket_sort<1024, 8, B0, LO, 1>) : listed(rs::k_bucket_sort<1024, 8, A0, LO, 1>);
            // the listed buckets over the primary tile (none for uniform keys), or every bucket
            // (wide_all); keys only: the smallest wide tile that holds the population's buckets
            // (512 x 18: three workgroups per CU, 512 x 34: two, 1024 x 34: one)
            if (wide_all && LO == K && want <= 512u * 18u)
                ballot ? large(rs::k_bucket_sort_wide<512, 18, B0, LO, 6>, 512) : large(rs::k_bucket_sort_wide<512, 18, A0, LO, 6>, 512);
            else if (wide_all && LO == K && want <= 512u * 34u)
                ballot ? large(rs::k_bucket_sort_wide<512, 34, B0, LO, 4>, 512) : large(rs::k_bucket_sort_wide<512, 34, A0, LO, 4>, 512);
            else
                ballot ? large(rs::k_bucket_sort_wide<1024, kWideKpt, B0, LO>, 1024)
                       : large(rs::k_bucket_sort_wide<1024, kWideKpt, A0, LO>, 1024);
        };
        if (keys) both(std::integral_constant<int, K>{});
        else if (out_aos) both(std::integral_constant<int, A>{});
        else both(std::integral_constant<int, S>{});
    }, "rsort.msd.bucket");
    HIP_TRY(hipGetLastError());
    if (split)
        if (rs_status st = enqueue_split(p, sw, keys, out_aos, r2, r3, uk, uv, n32, s)) return st;
    if (strict) return RS_OK;
    // the fallback (gated off on the device unless taken): pass 0's byte-0 totals, then the four
    // LSD passes on the input
    const uint32_t* g_lsd = gates + rs::kGateLsd;
    uint32_t* t0 = p->ptot + p->ptot_off[0];
    rs::PassList pl{};
    pl.count = 1;
    pl.width[0] = 8;
    const uint32_t tgrid = (uint32_t)std::min<uint64_t>((uint64_t)RS_TOT_PER_CU * p->cus,
                                                        (n + 4ull * RS_TOT_BLOCK - 1) / (4ull * RS_TOT_BLOCK));
    // (check_order: the totals came with the histogram read, see chk above)
    if (!chk) p->timer.run(RS_KERNEL_FALLBACK, fs, [&] {
        if (in_aos)
            hipLaunchKernelGGL(rs::k_pass_totals<2>, dim3(tgrid), dim3(RS_TOT_BLOCK), 0, fs, sk, n32, pl, 0u, t0,
                               (uint32_t*)nullptr, 0xFFFFFFFFu, 0x1u, g_lsd);
        else
            hipLaunchKernelGGL(rs::k_pass_totals<1>, dim3(tgrid), dim3(RS_TOT_BLOCK), 0, fs, sk, n32, pl, 0u, t0,
                               (uint32_t*)nullptr, 0xFFFFFFFFu, 0x1u, g_lsd);
    }, "rsort.msd.fallback_totals");
    HIP_TRY(hipGetLastError());
    rs_status st = RS_OK;
    if (keys) {
        // keys only: four one-sweep passes input -> tmp_k -> uk -> tmp_k -> uk (5 gated launches;
        // the keys-only LSD sort's histogram path would be 12)
        p->scatter_kind = RS_KERNEL_FALLBACK;
        for (uint32_t i = 0; i < 4 && st == RS_OK; ++i)
            st = run_pass(p, i == 0 ? sk : ((i & 1) ? p->tmp_k : uk), nullptr, (i & 1) ? uk : p->tmp_k, nullptr,
                          n32, 8 * i, 8, layout_pair(K, K), g_lsd, (int)i, fs, /*onesweep=*/true);
        p->scatter_kind = RS_KERNEL_SCATTER;
    } else if (!out_aos) {
        st = enqueue_lsd_gated(p, sk, sv, in_aos, uk, uv, n32, g_lsd, fs);
    } else {
        // records in place: uk -> tmp_k -> uk -> tmp_k -> uk
        p->scatter_kind = RS_KERNEL_FALLBACK;
        for (uint32_t i = 0; i < 4 && st == RS_OK; ++i)
            st = run_pass(p, (i & 1) ? p->tmp_k : uk, nullptr, (i & 1) ? uk : p->tmp_k, nullptr, n32, 8 * i, 8,
                          layout_pair(A, A), g_lsd, (int)i, fs, /*onesweep=*/true);
        p->scatter_kind = RS_KERNEL_SCATTER;
    }
    return st;
}

// in_k0 / in_v0 (optional): pass 0 reads them instead of uk / uv (out-of-place sort; the
// caller's input is only read, the result lands in uk / uv; check_order not supported).
static rs_status enqueue_sort(rs_plan* p, uint32_t* uk, uint32_t* uv, uint64_t n, hipStream_t s,
                              const uint32_t* in_k0 = nullptr, const uint32_t* in_v0 = nullptr) {
    p->last_ns = false;
    if (use_msd(p, n)) {
        const bool aos = p->layout == rs::LAYOUT_AOS;
        return enqueue_sort_msd(p, in_k0 ? in_k0 : uk, aos ? nullptr : (in_k0 ? in_v0 : uv), aos, uk, uv, aos, n, s);
    }
    const int L = p->layout;
    const uint32_t n32 = (uint32_t)n;
    const uint32_t* gate = p->check_order ? p->flags : nullptr;
    if (p->check_order) HIP_TRY(hipMemsetAsync(p->flags, 0, 16 * 4, s));
    // check_order in place: the presorted path first (nearly-sorted input is sorted there, and the
    // order check before pass 0 then gates every pass off)
    if (p->check_order && !in_k0 && p->ns && p->ns_on && n >= kMsdMin && n <= ns_keys(p->capacity))
        if (rs_status st = enqueue_presorted(p, uk, uv, (uint32_t)n, s)) return st;
    const bool onesweep = use_onesweep(p, n);
    if (onesweep) {
        // totals, tickets and the device error word (a timeout never outlives its sort)
        HIP_TRY(hipMemsetAsync(p->ptot, 0, 4ull * (rs::kTotalsMax + kTicketWords), s));
        // pass 0's digit totals from one read of the input; every later pass's totals are
        // counted by the pass before it (k_onesweep's ntot)
        rs::PassList pl{};
        pl.count = 1;
        pl.width[0] = p->widths[0];
        const uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)RS_TOT_PER_CU * p->cus,
                                                           (n + 4ull * RS_TOT_BLOCK - 1) / (4ull * RS_TOT_BLOCK));
        // check_order: the check of pass 0's input rides on this read (every later pass's check
        // on that pass's k_onesweep), so no k_check launch at all
        uint32_t* chk0 = (p->check_order && p->fused_check) ? p->flags : nullptr;
        const uint32_t fm = full_mask(p->bit_count);
        const uint32_t* src = in_k0 ? in_k0 : uk;
        p->timer.run(RS_KERNEL_HISTOGRAM, s, [&] {
            if (L == rs::LAYOUT_AOS)
                hipLaunchKernelGGL(rs::k_pass_totals<2>, dim3(grid), dim3(RS_TOT_BLOCK), 0, s, src, n32, pl, 0u, p->ptot, chk0, fm);
            else
                hipLaunchKernelGGL(rs::k_pass_totals<1>, dim3(grid), dim3(RS_TOT_BLOCK), 0, s, src, n32, pl, 0u, p->ptot, chk0, fm);
        });
        HIP_TRY(hipGetLastError());
    }
    const uint32_t fmask = full_mask(p->bit_count);
    // one-sweep with separate values: the ping-pong copy is (key, value) records - every
    // even pass writes 8-byte records (twice the bytes per digit run of two 4-byte arrays,
    // measured faster) and every odd pass reads them back into the caller's arrays
    const bool recs = onesweep && L == rs::LAYOUT_SOA && p->aos_tmp;
    // with a second records buffer only the last pass writes the caller's two arrays:
    // U -> R1, R1 -> R2, R2 -> R1, ..., R1 -> U (every other pass writes 8-byte records)
    uint32_t* r2 = recs ? p->tmp2 : nullptr;
    constexpr int A = rs::LAYOUT_AOS;
    uint32_t shift = 0;
    for (uint32_t i = 0; i < p->passes; ++i) {
        const bool even = (i % 2) == 0;
        const uint32_t* ik = even ? uk : p->tmp_k;
        const uint32_t* iv = even ? uv : (recs ? nullptr : p->tmp_v);
        uint32_t* ok = even ? p->tmp_k : uk;
        uint32_t* ov = even ? (recs ? nullptr : p->tmp_v) : uv;
        int in_layout = (recs && !even) ? A : L;
        int LL = recs ? (even ? layout_pair(L, A) : layout_pair(A, L)) : layout_pair(L, L);
        if (i == 0 && in_k0) {
            ik = in_k0;
            if (iv) iv = in_v0;
        }
        if (r2 && i > 0 && i + 1 < p->passes) {
            ik = even ? r2 : p->tmp_k;
            ok = even ? p->tmp_k : r2;
            iv = nullptr;
            ov = nullptr;
            in_layout = A;
            LL = layout_pair(A, A);
        }
        if (p->check_order && !(onesweep && p->fused_check)) {
            // Order check before every pass (the reference checks every second 2-bit pass,
            // AbstractRadixSortKernel.ts:257-261); all pairs, masked keys (Q1/Q2 fixed).
            const uint32_t grid = (uint32_t)std::min<uint64_t>(kCheckGrid, (n + rs::kBlock - 1) / rs::kBlock);
            p->timer.run(RS_KERNEL_CHECK, s, [&] {
                hipLaunchKernelGGL(rs::k_check, dim3(grid), dim3(rs::kBlock), 0, s, ik, n32,
                                   in_layout == A ? 2u : 1u, fmask, p->flags, (int)i, (int)i - 1);
            });
            HIP_TRY(hipGetLastError());
        }
        rs_status st = run_pass(p, ik, iv, ok, ov, n32, shift, p->widths[i], LL, gate, (int)i, s,
                                onesweep);
        if (st != RS_OK) return st;
        shift += p->widths[i];
    }
    if (p->check_order) {
        const uint32_t grid = (uint32_t)std::min<uint64_t>(kCheckGrid, (n + rs::kBlock - 1) / rs::kBlock);
        auto fin = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(grid), dim3(rs::kBlock), 0, s, p->tmp_k, p->tmp_v, uk, uv,
                               n32, p->flags, (int)p->passes, (const uint32_t*)r2);
        };
        if (L == rs::LAYOUT_AOS) fin(rs::k_finalize<rs::LAYOUT_AOS>);
        else if (recs) fin(rs::k_finalize<rs::LAYOUT_SOA, rs::LAYOUT_AOS>);
        else if (L == rs::LAYOUT_SOA) fin(rs::k_finalize<rs::LAYOUT_SOA>);
        else fin(rs::k_finalize<rs::LAYOUT_KEYS>);
        HIP_TRY(hipGetLastError());
    }
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_sort_n(rs_plan* p, void* keys, void* values, uint64_t n,
                                   void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_sort: null plan");
    if (n > p->capacity)
        return fail(RS_ERR_CAPACITY, "count %llu exceeds plan capacity %llu",
                    (unsigned long long)n, (unsigned long long)p->capacity);
    if (rs_status st = need_sort_plan(p, "rs_plan_sort")) return st;
    if (n <= 1) {   // nothing to move: no path taken
        p->last_hybrid = false;
        p->path_none = true;
        return RS_OK;
    }
    if (!keys) return fail(RS_ERR_INVALID_ARG, "rs_plan_sort: keys is null");
    const int L = p->layout;
    if (L == rs::LAYOUT_SOA && !values)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_sort: plan has values but values is null");
    if (L == rs::LAYOUT_AOS && values)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_sort: interleaved plan takes (key, value) records in keys; values must be null");
    if (((uintptr_t)keys & 3) || (values && ((uintptr_t)values & 3)))
        return fail(RS_ERR_INVALID_ARG, "keys/values must be 4-byte aligned (README.md limitations)");
    if (L == rs::LAYOUT_AOS && ((uintptr_t)keys & 7))
        return fail(RS_ERR_INVALID_ARG, "interleaved records must be 8-byte aligned");
    DeviceGuard guard(p->desc.device);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t n32 = (uint32_t)n;
    uint32_t* uk = (uint32_t*)keys;
    uint32_t* uv = L == rs::LAYOUT_SOA ? (uint32_t*)values : nullptr;
    if (rs_status st = take_device_error(p, "rs_plan_sort")) return st;
    p->last_hybrid = false;
    const rs_status st = n <= kTinyMax ? run_tiny(p, uk, uv, n32, s)   // one launch; check_order moot
                                       : enqueue_sort(p, uk, uv, n, s);
    if (st != RS_OK) return st;
    HIP_TRY(hipEventRecord(p->done, s));
    p->done_recorded = true;
    p->path_none = false;
    return RS_OK;
}

// Out-of-place sort (rsort.h; the multi-GPU paths at world size 1): in[0..n) is only read, the
// sorted result is written to out[0..n): pass 0 reads the input, the last pass writes the output.
RS_EXPORT rs_status rs_plan_sort_copy(rs_plan* p, const void* in_k, const void* in_v, void* out_k,
                                      void* out_v, uint64_t n, void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_copy: null plan");
    if (n > p->capacity)
        return fail(RS_ERR_CAPACITY, "count %llu exceeds plan capacity %llu",
                    (unsigned long long)n, (unsigned long long)p->capacity);
    if (rs_status st = need_sort_plan(p, "rs_plan_sort_copy")) return st;
    if (p->layout == rs::LAYOUT_AOS || p->check_order)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_copy: needs a plan with separate arrays (not interleaved) and no check_order");
    const bool kv = p->layout == rs::LAYOUT_SOA;
    if (n == 0) {
        p->last_hybrid = false;
        p->path_none = true;
        return RS_OK;
    }
    if (!in_k || !out_k || (kv && (!in_v || !out_v)))
        return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_copy: null buffer");
    if (((uintptr_t)in_k | (uintptr_t)out_k | (kv ? ((uintptr_t)in_v | (uintptr_t)out_v) : 0)) & 3)
        return fail(RS_ERR_INVALID_ARG, "keys/values must be 4-byte aligned");
    if (rs_status st = take_device_error(p, "rs_plan_sort_copy")) return st;
    p->last_hybrid = false;
    DeviceGuard guard(p->desc.device);
    hipStream_t s = (hipStream_t)stream;
    uint32_t* uk = (uint32_t*)out_k;
    uint32_t* uv = kv ? (uint32_t*)out_v : nullptr;
    rs_status st;
    if (n <= kTinyMax) {
        HIP_TRY(hipMemcpyAsync(uk, in_k, 4 * n, hipMemcpyDeviceToDevice, s));
        if (kv) HIP_TRY(hipMemcpyAsync(uv, in_v, 4 * n, hipMemcpyDeviceToDevice, s));
        st = n > 1 ? run_tiny(p, uk, uv, (uint32_t)n, s) : RS_OK;
    } else {
        st = enqueue_sort(p, uk, uv, n, s, (const uint32_t*)in_k, kv ? (const uint32_t*)in_v : nullptr);
    }
    if (st != RS_OK) return st;
    HIP_TRY(hipEventRecord(p->done, s));
    p->done_recorded = true;
    p->path_none = false;
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_last_path(rs_plan* p, uint32_t* path) {
    if (!p || !path) return fail(RS_ERR_INVALID_ARG, "rs_plan_last_path: null argument");
    DeviceGuard guard(p->desc.device);
    *path = RS_PATH_NONE;
    if (!p->done_recorded || p->path_none) return RS_OK;
    HIP_TRY(hipEventSynchronize(p->done));
    if (p->last_ns) {   // the presorted path's done word (ctl[5])
        uint32_t done = 0u;
        HIP_TRY(hipMemcpy(&done, p->ns + 5, 4, hipMemcpyDeviceToHost));
        if (done) {
            *path = RS_PATH_PRESORTED;
            return RS_OK;
        }
    }
    if (!p->last_hybrid) {
        *path = RS_PATH_LSD;
        return RS_OK;
    }
    // the plan kernel's gate words (first word of each gate block)
    const uint32_t* gates = p->msd + 65536 * 2 + 1024;
    uint32_t g[2] = {0u, 0u};
    HIP_TRY(hipMemcpy(&g[0], gates + rs::kGateMsd, 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&g[1], gates + rs::kGateLsd, 4, hipMemcpyDeviceToHost));
    *path = g[0] ? RS_PATH_HYBRID : g[1] ? RS_PATH_HYBRID_FALLBACK : RS_PATH_IN_ORDER;
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_last_split(rs_plan* p, uint32_t* levels) {
    if (!p || !levels) return fail(RS_ERR_INVALID_ARG, "rs_plan_last_split: null argument");
    DeviceGuard guard(p->desc.device);
    *levels = 0;
    if (!p->done_recorded || p->path_none || !p->last_hybrid || !p->last_split) return RS_OK;
    HIP_TRY(hipEventSynchronize(p->done));
    uint32_t g[2] = {0u, 0u};   // gate2, gate3 (first words): SplitWs layout in enqueue_sort_msd
    HIP_TRY(hipMemcpy(&g[0], p->split, 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&g[1], p->split + 16, 4, hipMemcpyDeviceToHost));
    *levels = g[1] ? 3u : g[0] ? 2u : 0u;
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_check(rs_plan* p) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_check: null plan");
    DeviceGuard guard(p->desc.device);
    if (p->done_recorded) HIP_TRY(hipEventSynchronize(p->done));
    return take_device_error(p, "rs_plan_check");
}

RS_EXPORT rs_status rs_plan_sort(rs_plan* p, void* keys, void* values, void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_sort: null plan");
    return rs_plan_sort_n(p, keys, values, p->capacity, stream);
}

static rs_status onesweep_digit_pass(rs_plan* p, const uint32_t* ik, const uint32_t* iv,
                                     uint32_t* ok, uint32_t* ov, uint64_t n, uint32_t shift,
                                     uint32_t bits, int LL, const void* d_totals, hipStream_t s);

RS_EXPORT rs_status rs_plan_partition(rs_plan* p, const void* in_keys, const void* in_values,
                                      void* out_keys, void* out_values, uint64_t n,
                                      uint32_t shift, uint32_t bits, void* d_hist, void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_partition: null plan");
    if (n > p->capacity)
        return fail(RS_ERR_CAPACITY, "count %llu exceeds plan capacity %llu",
                    (unsigned long long)n, (unsigned long long)p->capacity);
    if (bits == 0 || bits > 8 || shift + bits > 32)
        return fail(RS_ERR_INVALID_ARG, "partition digit must satisfy 1 <= bits <= 8, shift+bits <= 32");
    const int L = p->layout == rs::LAYOUT_AOS ? (int)rs::LAYOUT_AOS
                : (p->has_values && in_values && out_values ? (int)rs::LAYOUT_SOA : (int)rs::LAYOUT_KEYS);
    if (n && (!in_keys || !out_keys)) return fail(RS_ERR_INVALID_ARG, "rs_plan_partition: null keys");
    DeviceGuard guard(p->desc.device);
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        if (d_hist) HIP_TRY(hipMemsetAsync(d_hist, 0, 4u << bits, s));
        return RS_OK;
    }
    rs_status st = run_pass(p, (const uint32_t*)in_keys, (const uint32_t*)in_values,
                            (uint32_t*)out_keys, (uint32_t*)out_values, (uint32_t)n, shift, bits,
                            layout_pair(L, L), nullptr, 0, s);
    if (st != RS_OK) return st;
    if (d_hist) HIP_TRY(hipMemcpyAsync(d_hist, p->totals, 4u << bits, hipMemcpyDeviceToDevice, s));
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_partition_totals(rs_plan* p, const void* in_keys, const void* in_values,
                                             void* out_keys, void* out_values, uint64_t n,
                                             uint32_t shift, uint32_t bits, const void* d_totals,
                                             void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_partition_totals: null plan");
    if (!d_totals) return fail(RS_ERR_INVALID_ARG, "rs_plan_partition_totals: null totals");
    const bool soa = p->layout == rs::LAYOUT_SOA && in_values && out_values;
    // the one-sweep pass where it wins (with values, large tiles); elsewhere the
    // histogram / scan / scatter pass, which counts for itself
    if (n > p->capacity || bits == 0 || bits > 8 || shift + bits > 32 || n == 0 ||
        !(soa || p->layout == rs::LAYOUT_AOS) || !use_onesweep(p, n))
        return rs_plan_partition(p, in_keys, in_values, out_keys, out_values, n, shift, bits,
                                 nullptr, stream);
    if (!in_keys || !out_keys) return fail(RS_ERR_INVALID_ARG, "rs_plan_partition_totals: null keys");
    if (rs_status st = take_device_error(p, "rs_plan_partition_totals")) return st;
    DeviceGuard guard(p->desc.device);
    const int L = p->layout;
    return onesweep_digit_pass(p, (const uint32_t*)in_keys, (const uint32_t*)in_values,
                               (uint32_t*)out_keys, (uint32_t*)out_values, n, shift, bits,
                               layout_pair(L, L), d_totals, (hipStream_t)stream);
}

// One stable one-sweep pass in -> out by the digit (key >> shift) & (2^bits - 1), run as the
// plan's last pass (no next-pass totals): digit totals copied from d_totals, or counted here
// (one read of the keys) when d_totals is null.  LL = layout_pair(in, out).
static rs_status onesweep_digit_pass(rs_plan* p, const uint32_t* ik, const uint32_t* iv,
                                     uint32_t* ok, uint32_t* ov, uint64_t n, uint32_t shift,
                                     uint32_t bits, int LL, const void* d_totals, hipStream_t s) {
    const int pass = (int)p->passes - 1;
    uint32_t* slot = p->ptot + p->ptot_off[pass];   // 2^bits words fit: kTotalsMax >= off + 256
    HIP_TRY(hipMemsetAsync(p->tickets + pass, 0, 4, s));
    HIP_TRY(hipMemsetAsync(p->tickets + 16, 0, 4, s));
    if (d_totals) {
        HIP_TRY(hipMemcpyAsync(slot, d_totals, 4u << bits, hipMemcpyDeviceToDevice, s));
    } else {
        HIP_TRY(hipMemsetAsync(slot, 0, 4u << bits, s));
        rs::PassList pl{};
        pl.count = 1;
        pl.width[0] = bits;
        const uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)RS_TOT_PER_CU * p->cus,
                                                           (n + 4ull * RS_TOT_BLOCK - 1) / (4ull * RS_TOT_BLOCK));
        if ((LL & 15) == rs::LAYOUT_AOS)
            hipLaunchKernelGGL(rs::k_pass_totals<2>, dim3(grid), dim3(RS_TOT_BLOCK), 0, s, ik, (uint32_t)n, pl, shift, slot);
        else
            hipLaunchKernelGGL(rs::k_pass_totals<1>, dim3(grid), dim3(RS_TOT_BLOCK), 0, s, ik, (uint32_t)n, pl, shift, slot);
        HIP_TRY(hipGetLastError());
    }
    return run_pass(p, ik, iv, ok, ov, (uint32_t)n, shift, bits, LL, nullptr, pass, s, /*onesweep=*/true);
}

RS_EXPORT rs_status rs_plan_partition_records(rs_plan* p, const void* in_keys, const void* in_values,
                                              void* out_records, uint64_t n, uint32_t shift,
                                              uint32_t bits, const void* d_totals, void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_partition_records: null plan");
    if (p->layout != rs::LAYOUT_SOA)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_partition_records: needs a plan with separate values (RS_FLAG_HAS_VALUES)");
    if (n > p->capacity)
        return fail(RS_ERR_CAPACITY, "count %llu exceeds plan capacity %llu",
                    (unsigned long long)n, (unsigned long long)p->capacity);
    if (bits == 0 || bits > 8 || shift + bits > 32)
        return fail(RS_ERR_INVALID_ARG, "partition digit must satisfy 1 <= bits <= 8, shift+bits <= 32");
    if (n == 0) return RS_OK;
    if (!in_keys || !in_values || !out_records)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_partition_records: null buffer");
    if ((uintptr_t)out_records & 7) return fail(RS_ERR_INVALID_ARG, "records must be 8-byte aligned");
    if (rs_status st = take_device_error(p, "rs_plan_partition_records")) return st;
    DeviceGuard guard(p->desc.device);
    return onesweep_digit_pass(p, (const uint32_t*)in_keys, (const uint32_t*)in_values,
                               (uint32_t*)out_records, nullptr, n, shift, bits,
                               layout_pair(rs::LAYOUT_SOA, rs::LAYOUT_AOS), d_totals, (hipStream_t)stream);
}

// Whole sort of n (key, value) records into two arrays: pass 0 reads the records, the last pass
// writes the arrays; the passes between go through the plan's records buffers (R1 <-> R2), or
// alternate with the output arrays when there is no second records buffer.  One-sweep passes at
// every size (tiles of the size's configuration).
static rs_status enqueue_sort_records(rs_plan* p, const uint32_t* rec, uint32_t* uk, uint32_t* uv,
                                      uint64_t n, hipStream_t s) {
    const uint32_t n32 = (uint32_t)n;
    HIP_TRY(hipMemsetAsync(p->ptot, 0, 4ull * (rs::kTotalsMax + kTicketWords), s));
    {
        rs::PassList pl{};
        pl.count = 1;
        pl.width[0] = p->widths[0];
        const uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)RS_TOT_PER_CU * p->cus,
                                                           (n + 4ull * RS_TOT_BLOCK - 1) / (4ull * RS_TOT_BLOCK));
        p->timer.run(RS_KERNEL_HISTOGRAM, s, [&] {
            hipLaunchKernelGGL(rs::k_pass_totals<2>, dim3(grid), dim3(RS_TOT_BLOCK), 0, s, rec, n32, pl, 0u, p->ptot);
        });
        HIP_TRY(hipGetLastError());
    }
    constexpr int A = rs::LAYOUT_AOS, S = rs::LAYOUT_SOA;
    uint32_t* r1 = p->tmp_k;
    uint32_t* r2 = p->tmp2;
    uint32_t shift = 0;
    for (uint32_t i = 0; i < p->passes; ++i) {
        const bool last = i + 1 == p->passes, odd = (i & 1u) != 0;
        const uint32_t* ik;
        const uint32_t* iv = nullptr;
        uint32_t* ok;
        uint32_t* ov = nullptr;
        int LL;
        if (r2) {            // rec -> R1 -> R2 -> R1 ... -> arrays
            ik = i == 0 ? rec : (odd ? r1 : r2);
            if (last) { ok = uk; ov = uv; LL = layout_pair(A, S); }
            else { ok = odd ? r2 : r1; LL = layout_pair(A, A); }
        } else {             // rec -> R1 -> arrays -> R1 -> arrays
            if (i == 0) { ik = rec; ok = r1; LL = layout_pair(A, A); }
            else if (odd) { ik = r1; ok = uk; ov = uv; LL = layout_pair(A, S); }
            else { ik = uk; iv = uv; ok = r1; LL = layout_pair(S, A); }
        }
        rs_status st = run_pass(p, ik, iv, ok, ov, n32, shift, p->widths[i], LL, nullptr, (int)i, s,
                                /*onesweep=*/true);
        if (st != RS_OK) return st;
        shift += p->widths[i];
    }
    return RS_OK;
}

static rs_status sort_records_impl(rs_plan* p, const void* records, void* keys_out, void* values_out,
                                   uint64_t n, uint32_t key_lo, uint32_t key_hi, void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_records: null plan");
    if (rs_status st = need_sort_plan(p, "rs_plan_sort_records")) return st;
    if (p->layout != rs::LAYOUT_SOA)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_records: needs a plan with separate values (RS_FLAG_HAS_VALUES)");
    if (n > p->capacity)
        return fail(RS_ERR_CAPACITY, "count %llu exceeds plan capacity %llu",
                    (unsigned long long)n, (unsigned long long)p->capacity);
    if (n == 0) {
        p->last_hybrid = false;
        p->path_none = true;
        return RS_OK;
    }
    if (!records || !keys_out || !values_out)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_records: null buffer");
    if (((uintptr_t)records & 7) || ((uintptr_t)keys_out & 3) || ((uintptr_t)values_out & 3))
        return fail(RS_ERR_INVALID_ARG, "records must be 8-byte and arrays 4-byte aligned");
    if (rs_status st = take_device_error(p, "rs_plan_sort_records")) return st;
    p->last_hybrid = false;
    DeviceGuard guard(p->desc.device);
    hipStream_t s = (hipStream_t)stream;
    uint32_t* uk = (uint32_t*)keys_out;
    uint32_t* uv = (uint32_t*)values_out;
    rs_status st;
    if (n <= kTinyMax) {
        hipLaunchKernelGGL(rs::k_split_records, dim3((uint32_t)((n + rs::kBlock - 1) / rs::kBlock)),
                           dim3(rs::kBlock), 0, s, (const uint2*)records, uk, uv, n);
        HIP_TRY(hipGetLastError());
        st = n > 1 ? run_tiny(p, uk, uv, (uint32_t)n, s) : RS_OK;
    } else if (use_msd(p, n) && key_lo <= key_hi && key_hi - key_lo >= 0xFFFFu) {
        // the hybrid MSD path over the range-relative bits of the keys
        const uint32_t range = key_hi - key_lo;
        const uint32_t vbits = 32u - (uint32_t)__builtin_clz(range);
        st = enqueue_sort_msd(p, (const uint32_t*)records, nullptr, true, uk, uv, false, n, s, key_lo, vbits);
    } else {
        st = enqueue_sort_records(p, (const uint32_t*)records, uk, uv, n, s);
    }
    if (st != RS_OK) return st;
    HIP_TRY(hipEventRecord(p->done, s));
    p->done_recorded = true;
    p->path_none = false;
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_sort_records(rs_plan* p, const void* records, void* keys_out,
                                         void* values_out, uint64_t n, void* stream) {
    return sort_records_impl(p, records, keys_out, values_out, n, 0u, 0xFFFFFFFFu, stream);
}

RS_EXPORT rs_status rs_plan_sort_records_range(rs_plan* p, const void* records, void* keys_out,
                                               void* values_out, uint64_t n, uint32_t key_lo,
                                               uint32_t key_hi, void* stream) {
    if (key_lo > key_hi) return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_records_range: key_lo > key_hi");
    return sort_records_impl(p, records, keys_out, values_out, n, key_lo, key_hi, stream);
}

RS_EXPORT rs_status rs_plan_hist16(rs_plan* p, const void* keys, uint64_t n, void* d_hist16, void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_hist16: null plan");
    if (!d_hist16 || (n && !keys)) return fail(RS_ERR_INVALID_ARG, "rs_plan_hist16: null pointer");
    if (n > p->capacity)
        return fail(RS_ERR_CAPACITY, "count %llu exceeds plan capacity %llu",
                    (unsigned long long)n, (unsigned long long)p->capacity);
    const bool aos = p->layout == rs::LAYOUT_AOS;
    if (((uintptr_t)keys & 3) || (aos && ((uintptr_t)keys & 7)))
        return fail(RS_ERR_INVALID_ARG, "rs_plan_hist16: keys must be 4-byte (records 8-byte) aligned");
    DeviceGuard guard(p->desc.device);
    hipStream_t s = (hipStream_t)stream;
    // one row per CU where tmp_k holds them (k_hist16_in: 65536 counts per row, then a flag word
    // per row); k_hist16_sum adds the rows and the top-byte totals
    const uint32_t hrows = (uint32_t)std::min<uint64_t>(p->cus, p->rows_words / 65537ull);
    if (hrows == 0)
        return fail(RS_ERR_CAPACITY, "rs_plan_hist16: the plan's workspace holds no histogram row (a keys-only "
                    "sort plan needs capacity >= 65537; plans with values and RS_USAGE_PARTITION plans always hold one)");
    if (n / hrows >= (uint64_t)rs::kEvMax * rs::kHalfT)
        return fail(RS_ERR_CAPACITY, "rs_plan_hist16: %llu keys over %u histogram rows (at most 2^27 keys per row)",
                    (unsigned long long)n, hrows);
    p->timer.run(RS_KERNEL_HISTOGRAM, s, [&] {
        // z0 / z1 (the MSD path's overflow words) point into the rows' flag area: unused here
        uint32_t* z = p->tmp_k + (size_t)hrows * 65536u;
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(hrows), dim3(1024), 0, s, (const uint32_t*)keys, (uint32_t)n, p->tmp_k, 0u,
                               0xFFFFFFFFu, 16u, z, z, (uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                               (const uint32_t*)nullptr);
        };
        if (aos && ((uintptr_t)keys & 15u) == 0) go(rs::k_hist16_in<rs::LAYOUT_AOS, true, true>);
        else if (aos) go(rs::k_hist16_in<rs::LAYOUT_AOS, false, true>);
        else go(rs::k_hist16_in<rs::LAYOUT_SOA, false, true>);
        hipLaunchKernelGGL(rs::k_hist16_sum, dim3(256), dim3(256), 0, s, (const uint32_t*)p->tmp_k, hrows,
                           (uint32_t*)d_hist16);
    });
    HIP_TRY(hipGetLastError());
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_sort_region(rs_plan* p, const void* records, void* keys_out, void* values_out,
                                        uint64_t n, const void* d_hist16, uint32_t top_lo, uint32_t top_hi,
                                        void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_region: null plan");
    if (rs_status st = need_sort_plan(p, "rs_plan_sort_region")) return st;
    if (p->layout != rs::LAYOUT_SOA)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_region: needs a plan with separate values (RS_FLAG_HAS_VALUES)");
    if (n > p->capacity)
        return fail(RS_ERR_CAPACITY, "count %llu exceeds plan capacity %llu",
                    (unsigned long long)n, (unsigned long long)p->capacity);
    if (top_lo >= top_hi || top_hi > 256)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_region: need top_lo < top_hi <= 256 (got %u, %u)", top_lo, top_hi);
    if (n == 0) {
        p->last_hybrid = false;
        p->path_none = true;
        return RS_OK;
    }
    if (!records || !keys_out || !values_out || !d_hist16)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_sort_region: null buffer");
    if (((uintptr_t)records & 7) || ((uintptr_t)keys_out & 3) || ((uintptr_t)values_out & 3) || ((uintptr_t)d_hist16 & 3))
        return fail(RS_ERR_INVALID_ARG, "records must be 8-byte and arrays 4-byte aligned");
    if (rs_status st = take_device_error(p, "rs_plan_sort_region")) return st;
    p->last_hybrid = false;
    DeviceGuard guard(p->desc.device);
    hipStream_t s = (hipStream_t)stream;
    uint32_t* uk = (uint32_t*)keys_out;
    uint32_t* uv = (uint32_t*)values_out;
    rs_status st;
    if (n <= kTinyMax) {
        hipLaunchKernelGGL(rs::k_split_records, dim3((uint32_t)((n + rs::kBlock - 1) / rs::kBlock)),
                           dim3(rs::kBlock), 0, s, (const uint2*)records, uk, uv, n);
        HIP_TRY(hipGetLastError());
        st = n > 1 ? run_tiny(p, uk, uv, (uint32_t)n, s) : RS_OK;
    } else if (p->msd && p->tmp2 && p->msd_mode != 0 && p->radix_bits == 8 && p->bit_count == 32 &&
               !p->check_order && n <= kMsdMax) {
        // the senders' partition was pass 0: the segmented next-byte pass and the bucket pass
        st = enqueue_sort_msd(p, (const uint32_t*)records, nullptr, true, uk, uv, false, n, s, 0u, 32u,
                              (const uint32_t*)d_hist16, top_lo, top_hi);
    } else {
        st = enqueue_sort_records(p, (const uint32_t*)records, uk, uv, n, s);
    }
    if (st != RS_OK) return st;
    HIP_TRY(hipEventRecord(p->done, s));
    p->done_recorded = true;
    p->path_none = false;
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_device_errors(rs_plan* p, uint32_t* errors) {
    if (!p || !errors) return fail(RS_ERR_INVALID_ARG, "rs_plan_device_errors: null argument");
    DeviceGuard guard(p->desc.device);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(errors, p->tickets + 16, 4, hipMemcpyDeviceToHost));
    *errors |= p->host_err ? __atomic_load_n(p->host_err, __ATOMIC_ACQUIRE) : 0u;
    return RS_OK;
}

#if RS_STAMPS
// Diagnostic builds only (not in rsort.h): device buffer for k_onesweep's phase stamps.
RS_EXPORT rs_status rs_debug_set_stamps(void* dev_ptr) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(rs::g_rs_stamps), &dev_ptr, sizeof(dev_ptr)));
    return RS_OK;
}
#endif

RS_EXPORT rs_status rs_plan_info_get(const rs_plan* p, rs_plan_info* info) {
    if (!p || !info) return fail(RS_ERR_INVALID_ARG, "rs_plan_info_get: null argument");
    memset(info, 0, sizeof(*info));
    info->passes = p->passes;
    for (uint32_t i = 0; i < p->passes && i < 16; ++i) info->digit_bits[i] = p->widths[i];
    const TileCfg& c = use_small_tiles(p, p->capacity) ? kSmall : kLarge;
    info->tile_keys = p->capacity <= kTinyMax ? kTinyMax : (uint32_t)c.tile;
    info->grid_blocks = p->capacity <= kTinyMax ? 1u
        : (uint32_t)std::min<uint64_t>((p->capacity + c.tile - 1) / c.tile, c.max_grid);
    info->workspace_bytes = p->workspace;
    info->rank_mode = (uint32_t)p->rank_mode;
    info->lane_order_selftest = p->selftest;
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_set_wait_limit(rs_plan* p, uint32_t sleeps) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_plan_set_wait_limit: null plan");
    p->spin_max = sleeps;
    return RS_OK;
}

// The presorted path's counts of the plan's last sort (waits for it): marked = the elements the
// order scan marked and the path extracted, moved = the elements its merge wrote (each read and
// written once: 16 B with values); both 0 when the last sort did not take the path.
RS_EXPORT rs_status rs_plan_presorted_counts(rs_plan* p, uint64_t* marked, uint64_t* moved) {
    if (!p || !marked || !moved) return fail(RS_ERR_INVALID_ARG, "rs_plan_presorted_counts: null argument");
    *marked = 0;
    *moved = 0;
    if (!p->last_ns || !p->ns) return RS_OK;
    DeviceGuard guard(p->desc.device);
    if (p->done_recorded) HIP_TRY(hipEventSynchronize(p->done));
    const NsWs w = ns_layout(p->ns, p->capacity);
    uint32_t ctl[rs::kNsCtlWords];
    HIP_TRY(hipMemcpy(ctl, w.ctl, sizeof(ctl), hipMemcpyDeviceToHost));
    if (ctl[rs::kNsGate]) {   // the path was on
        *marked = ctl[4];
        *moved = ctl[24];
    }
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_set_debug(rs_plan* p, const rs_plan_debug* d) {
    if (!p || !d) return fail(RS_ERR_INVALID_ARG, "rs_plan_set_debug: null argument");
    auto tri = [](int32_t v, int hi) { return v >= -1 && v <= hi; };
    if (!tri(d->rank, 1) || !tri(d->tile, 1) || !tri(d->onesweep, 1) || !tri(d->msd, 1) ||
        !tri(d->keys_cfg, 1) || !tri(d->msd_keys_cfg, 2) || !tri(d->kbucket_wave, 1) ||
        !tri(d->selftest_fail, 1) || !tri(d->split, 1) || !tri(d->presorted, 1) || !tri(d->xcd, 3) ||
        !tri(d->high_half, 1))
        return fail(RS_ERR_INVALID_ARG, "rs_plan_set_debug: every field must be -1 or a listed choice");
    if (d->selftest_fail == 1) {
        p->selftest = 0;
        p->rank_mode = rs::RANK_BALLOT;
    }
    if (d->rank >= 0) p->rank_mode = d->rank == 1 ? rs::RANK_BALLOT : rs::RANK_LDS_ATOMIC;
    if (d->tile >= 0) p->tile_mode = d->tile;
    if (d->onesweep >= 0) p->onesweep_mode = d->onesweep;
    if (d->msd >= 0) p->msd_mode = d->msd;
    if (d->keys_cfg >= 0) p->keys_cfg = d->keys_cfg == 1;
    if (d->msd_keys_cfg >= 0) p->msd_keys_cfg = d->msd_keys_cfg;
    if (d->kbucket_wave >= 0) p->kbucket_wave = d->kbucket_wave == 1;
    if (d->split >= 0) p->split_on = d->split == 1;
    if (d->presorted >= 0) p->ns_on = d->presorted == 1;
    if (d->xcd >= 0) p->xcd_claims = d->xcd;
    if (d->high_half >= 0) p->high_half = d->high_half == 1;
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_set_profiling(rs_plan* p, int enable) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "null plan");
    p->timer.enabled = enable != 0;
    p->timer.mask = ~0u;
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_set_profiling_kinds(rs_plan* p, uint32_t kind_mask) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "null plan");
    if (kind_mask >> RS_KERNEL_KINDS)
        return fail(RS_ERR_INVALID_ARG, "rs_plan_set_profiling_kinds: mask 0x%x has bits beyond the %d kinds",
                    kind_mask, RS_KERNEL_KINDS);
    p->timer.enabled = kind_mask != 0;
    p->timer.mask = kind_mask;
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_kernel_times(rs_plan* p, double ms[RS_KERNEL_KINDS],
                                         uint64_t launches[RS_KERNEL_KINDS]) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "null plan");
    DeviceGuard guard(p->desc.device);
    p->timer.drain();
    for (int k = 0; k < RS_KERNEL_KINDS; ++k) {
        if (ms) ms[k] = p->timer.ms[k];
        if (launches) launches[k] = p->timer.launches[k];
    }
    return RS_OK;
}

RS_EXPORT rs_status rs_plan_reset_kernel_times(rs_plan* p) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "null plan");
    DeviceGuard guard(p->desc.device);
    p->timer.drain();
    for (int k = 0; k < RS_KERNEL_KINDS; ++k) { p->timer.ms[k] = 0; p->timer.launches[k] = 0; }
    return RS_OK;
}

// ---- prefix sum ----------------------------------------------------------------------------
namespace {
constexpr int kScanTile = 4096;
constexpr uint32_t kScanMaxGrid = 1024;
// single-pass scan (k_scan_lookback): 1024 threads x 32 elements = 32K-element tiles, one workgroup
// per CU, the next tile's 128 KB in flight across the look-back and the stores (profiles/r04/scan*)
#if !RS_KNOB_OPEN || !defined(RS_SCAN_BLOCK)
#undef RS_SCAN_BLOCK
#define RS_SCAN_BLOCK 1024
#endif
#if !RS_KNOB_OPEN || !defined(RS_SCAN_EPT)
#undef RS_SCAN_EPT
#define RS_SCAN_EPT 32   // 32K-element tiles, one workgroup per CU (0.453 vs 0.591 ms at 16, 1.33 at 8)
#endif
#if !RS_KNOB_OPEN || !defined(RS_SCAN_PF)
#undef RS_SCAN_PF
#define RS_SCAN_PF 1
#endif
constexpr int kScanBlock = RS_SCAN_BLOCK, kScanEpt = RS_SCAN_EPT;
constexpr uint32_t kScanLbTile = kScanBlock * kScanEpt;
struct Geometry { uint32_t grid, base, extra; };
Geometry geometry(uint64_t n, uint32_t tile, uint32_t max_grid) {
    const uint64_t tiles = (n + tile - 1) / tile;
    Geometry g;
    g.grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(tiles, 1), max_grid);
    g.base = (uint32_t)(tiles / g.grid);
    g.extra = (uint32_t)(tiles % g.grid);
    return g;
}
}

RS_EXPORT rs_status rs_scan_plan_create(int32_t device, uint64_t count, uint32_t wx, uint32_t wy,
                                        uint32_t flags, rs_scan_plan** out) {
    if (!out) return fail(RS_ERR_INVALID_ARG, "rs_scan_plan_create: null out");
    *out = nullptr;
    if (wx == 0) wx = 16;
    if (wy == 0) wy = 16;
    const uint64_t T = (uint64_t)wx * wy;
    if ((T & (T - 1)) || T > 1024)
        return fail(RS_ERR_NOT_POW2,
                    "workgroupSize.x * workgroupSize.y must be a power of two. (current: %llu)",
                    (unsigned long long)T);
    if (count > 0xFFFFFFFFull) return fail(RS_ERR_INVALID_ARG, "count must be < 2^32");
    if (flags & ~(uint32_t)RS_FLAG_AVOID_BANK_CONFLICTS)
        return fail(RS_ERR_INVALID_ARG, "unknown flag bits 0x%x", flags);
    rs_scan_plan* p = new (std::nothrow) rs_scan_plan();
    if (!p) return fail(RS_ERR_OUT_OF_MEMORY, "host allocation failed");
    p->device = device;
    p->count = count;
    p->threads = (uint32_t)T;
    DeviceGuard guard(device);
    p->status_words = std::max<uint64_t>(1, (count + kScanLbTile - 1) / kScanLbTile);
    int cus = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            cus = prop.multiProcessorCount;
    }
    p->grid = (uint32_t)cus;   // resident workgroups per CU: scan_run (occupancy of the instantiation)
    hipError_t e = hipMalloc((void**)&p->sums, 4ull * kScanMaxGrid);
    if (e == hipSuccess) e = hipMalloc((void**)&p->status, 8ull * p->status_words);
    if (e == hipSuccess) e = hipMalloc((void**)&p->tickets, 4ull * (rs::kScanTickets + 1));
    if (e == hipSuccess) e = hipMemset(p->status, 0, 8ull * p->status_words);
    if (e == hipSuccess) e = hipMemset(p->tickets, 0, 4ull * (rs::kScanTickets + 1));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->done, hipEventDisableTiming);
    if (e != hipSuccess) {
        rs_scan_plan_destroy(p);
        return fail(RS_ERR_OUT_OF_MEMORY, "rs_scan_plan_create: %s", hipGetErrorString(e));
    }
    *out = p;
    return RS_OK;
}

static rs_status scan_run(rs_scan_plan* p, void* data, const uint32_t* ind, hipStream_t s) {
    const uint64_t n = p->count;
    if (RS_KNOB("RSORT_SCAN_3K", 0) == 0) {
        // single pass: a new tag for this launch's status words (cleared when the tags wrap)
        if (++p->epoch >= (1u << 30)) {
            HIP_TRY(hipMemsetAsync(p->status, 0, 8ull * p->status_words, s));
            HIP_TRY(hipMemsetAsync(p->tickets, 0, 4ull * rs::kScanTickets, s));
            p->epoch = 1;
        }
        const bool vec = ((uintptr_t)data & 15u) == 0;
        auto go = [&](auto kern) {
            // the resident workgroups of the device (tiles come from tickets in order)
            static const uint32_t per_cu = resident_per_cu(kern, kScanBlock);
            const uint32_t grid = (uint32_t)std::min<uint64_t>(p->status_words, (uint64_t)per_cu * p->grid);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(kScanBlock), 0, s, (uint32_t*)data, (uint32_t)n,
                               p->status, p->tickets, p->epoch, p->tickets + rs::kScanTickets, p->spin_max, ind);
        };
        if (vec) go(rs::k_scan_lookback<kScanBlock, kScanEpt, true, RS_SCAN_PF != 0>);
        else go(rs::k_scan_lookback<kScanBlock, kScanEpt, false, RS_SCAN_PF != 0>);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(p->done, s));
        return RS_OK;
    }
    const Geometry geo = geometry(n, kScanTile, kScanMaxGrid);
    hipLaunchKernelGGL(rs::k_chunk_sums<kScanTile>, dim3(geo.grid), dim3(rs::kBlock), 0, s,
                       (const uint32_t*)data, (uint32_t)n, geo.base, geo.extra, p->sums, ind);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(rs::k_scan_small, dim3(1), dim3(rs::kBlock), 0, s, p->sums, geo.grid, ind);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(rs::k_chunk_rescan<kScanTile>, dim3(geo.grid), dim3(rs::kBlock), 0, s,
                       (uint32_t*)data, (uint32_t)n, geo.base, geo.extra, (const uint32_t*)p->sums,
                       ind);
    HIP_TRY(hipGetLastError());
    return RS_OK;
}

RS_EXPORT rs_status rs_scan_plan_run(rs_scan_plan* p, void* data, void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_scan_plan_run: null plan");
    if (p->count == 0) return RS_OK;
    if (!data) return fail(RS_ERR_INVALID_ARG, "rs_scan_plan_run: null data");
    DeviceGuard guard(p->device);
    return scan_run(p, data, nullptr, (hipStream_t)stream);
}

RS_EXPORT rs_status rs_scan_plan_run_indirect(rs_scan_plan* p, void* data,
                                              const void* dispatch_size_buffer, uint64_t offset,
                                              void* stream) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_scan_plan_run_indirect: null plan");
    if (!dispatch_size_buffer)
        return fail(RS_ERR_INVALID_ARG, "rs_scan_plan_run_indirect: null dispatch size buffer");
    if (offset % 4)
        return fail(RS_ERR_INVALID_ARG, "rs_scan_plan_run_indirect: offset %llu is not a multiple of 4",
                    (unsigned long long)offset);
    if (p->count == 0) return RS_OK;
    if (!data) return fail(RS_ERR_INVALID_ARG, "rs_scan_plan_run_indirect: null data");
    DeviceGuard guard(p->device);
    return scan_run(p, data, (const uint32_t*)((const char*)dispatch_size_buffer + offset),
                    (hipStream_t)stream);
}

RS_EXPORT uint32_t rs_scan_plan_dispatch_chain(const rs_scan_plan* p, uint32_t* out,
                                               uint32_t max_words) {
    // the reference's chain for T = workgroup_x * workgroup_y threads, 2T items per workgroup:
    // scan(count) [+ chain(workgroups) + add_block_sums] (PrefixSumKernel.ts:45-137), one
    // (x, y, 1) triple per pipeline; findOptimalDispatchSize folds x > 65535 (the default
    // maxComputeWorkgroupsPerDimension) into x = floor(sqrt(wc)), y = ceil(wc / x) (utils.ts:8-23)
    if (!p) return 0;
    std::vector<uint32_t> chain;
    const uint64_t T = p->threads;
    std::function<void(uint64_t)> rec = [&](uint64_t count) {
        const uint64_t wc = (count + 2 * T - 1) / (2 * T);
        uint64_t x = wc, y = 1;
        if (wc > 65535) {
            x = (uint64_t)std::floor(std::sqrt((double)wc));
            y = (wc + x - 1) / x;
        }
        chain.insert(chain.end(), {(uint32_t)x, (uint32_t)y, 1u});
        if (wc > 1) {
            rec(wc);
            chain.insert(chain.end(), {(uint32_t)x, (uint32_t)y, 1u});
        }
    };
    rec(std::max<uint64_t>(p->count, 1));
    for (uint32_t i = 0; i < max_words && i < chain.size(); ++i) out[i] = chain[i];
    return (uint32_t)chain.size();
}

RS_EXPORT rs_status rs_scan_plan_check(rs_scan_plan* p) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_scan_plan_check: null plan");
    DeviceGuard guard(p->device);
    if (!p->tickets || !p->done) return RS_OK;
    HIP_TRY(hipEventSynchronize(p->done));
    uint32_t e = 0;
    HIP_TRY(hipMemcpy(&e, p->tickets + rs::kScanTickets, 4, hipMemcpyDeviceToHost));
    if (!e) return RS_OK;
    HIP_TRY(hipMemset(p->tickets + rs::kScanTickets, 0, 4));
    return fail(RS_ERR_DEVICE, "rs_scan_plan_check: a look-back wait of an earlier scan on this plan timed out; "
                "that scan's output is invalid");
}

RS_EXPORT rs_status rs_scan_plan_set_wait_limit(rs_scan_plan* p, uint32_t sleeps) {
    if (!p) return fail(RS_ERR_INVALID_ARG, "rs_scan_plan_set_wait_limit: null plan");
    p->spin_max = sleeps;
    return RS_OK;
}

RS_EXPORT void rs_scan_plan_destroy(rs_scan_plan* p) {
    if (!p) return;
    DeviceGuard guard(p->device);
    if (p->done) (void)hipEventDestroy(p->done);
    (void)hipFree(p->sums);
    (void)hipFree(p->status);
    (void)hipFree(p->tickets);
    delete p;
}

// ---- memory / streams ----------------------------------------------------------------------
RS_EXPORT rs_status rs_device_count(int32_t* n) {
    if (!n) return fail(RS_ERR_INVALID_ARG, "null");
    int c = 0;
    HIP_TRY(hipGetDeviceCount(&c));
    *n = c;
    return RS_OK;
}

RS_EXPORT rs_status rs_malloc(int32_t device, uint64_t bytes, void** ptr) {
    if (!ptr) return fail(RS_ERR_INVALID_ARG, "null");
    DeviceGuard guard(device);
    HIP_TRY(hipMalloc(ptr, bytes ? bytes : 4));
    return RS_OK;
}

RS_EXPORT rs_status rs_free(void* ptr) {
    HIP_TRY(hipFree(ptr));
    return RS_OK;
}

RS_EXPORT rs_status rs_memcpy_h2d(void* dst, const void* src, uint64_t bytes, void* stream) {
    if (bytes == 0) return RS_OK;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return RS_OK;
}

RS_EXPORT rs_status rs_memcpy_d2h(void* dst, const void* src, uint64_t bytes, void* stream) {
    if (bytes == 0) return RS_OK;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return RS_OK;
}

RS_EXPORT rs_status rs_memcpy_d2d(void* dst, const void* src, uint64_t bytes, void* stream) {
    if (bytes == 0) return RS_OK;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return RS_OK;
}

RS_EXPORT rs_status rs_stream_create(int32_t device, void** stream) {
    if (!stream) return fail(RS_ERR_INVALID_ARG, "null");
    DeviceGuard guard(device);
    hipStream_t s;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = (void*)s;
    return RS_OK;
}

RS_EXPORT rs_status rs_stream_destroy(void* stream) {
    HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return RS_OK;
}

RS_EXPORT rs_status rs_stream_synchronize(void* stream) {
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    return RS_OK;
}

RS_EXPORT rs_status rs_event_create(void** event) {
    if (!event) return fail(RS_ERR_INVALID_ARG, "rs_event_create: null");
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    *event = (void*)e;
    return RS_OK;
}

RS_EXPORT rs_status rs_event_destroy(void* event) {
    if (event) HIP_TRY(hipEventDestroy((hipEvent_t)event));
    return RS_OK;
}

RS_EXPORT rs_status rs_event_record(void* event, void* stream) {
    if (!event) return fail(RS_ERR_INVALID_ARG, "rs_event_record: null event");
    HIP_TRY(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
    return RS_OK;
}

RS_EXPORT rs_status rs_event_elapsed_ms(void* start, void* end, float* ms) {
    if (!start || !end || !ms) return fail(RS_ERR_INVALID_ARG, "rs_event_elapsed_ms: null");
    HIP_TRY(hipEventSynchronize((hipEvent_t)end));
    HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end));
    return RS_OK;
}

RS_EXPORT rs_status rs_fill_random_u32(void* dst, uint64_t n, uint64_t seed, uint64_t start,
                                       void* stream) {
    if (n == 0) return RS_OK;
    if (!dst) return fail(RS_ERR_INVALID_ARG, "null");
    const uint32_t grid = (uint32_t)std::min<uint64_t>(8192, (n + rs::kBlock - 1) / rs::kBlock);
    hipLaunchKernelGGL(rs::k_fill_random, dim3(grid), dim3(rs::kBlock), 0, (hipStream_t)stream,
                       (uint32_t*)dst, n, seed, start);
    HIP_TRY(hipGetLastError());
    return RS_OK;
}

RS_EXPORT rs_status rs_fill_iota_u32(void* dst, uint64_t n, uint32_t first, void* stream) {
    if (n == 0) return RS_OK;
    if (!dst) return fail(RS_ERR_INVALID_ARG, "null");
    const uint32_t grid = (uint32_t)std::min<uint64_t>(8192, (n + rs::kBlock - 1) / rs::kBlock);
    hipLaunchKernelGGL(rs::k_fill_iota, dim3(grid), dim3(rs::kBlock), 0, (hipStream_t)stream,
                       (uint32_t*)dst, n, first);
    HIP_TRY(hipGetLastError());
    return RS_OK;
}

RS_EXPORT rs_status rs_histogram(const void* keys, uint64_t n, uint32_t shift, uint32_t bits,
                                 void* d_hist, void* stream) {
    if (bits == 0 || bits > 8 || shift + bits > 32)
        return fail(RS_ERR_INVALID_ARG, "rs_histogram: need 1 <= bits <= 8 and shift + bits <= 32");
    if (!d_hist || (n && !keys)) return fail(RS_ERR_INVALID_ARG, "rs_histogram: null pointer");
    if (n > 0xFFFFFFFFull) return fail(RS_ERR_INVALID_ARG, "rs_histogram: n must be < 2^32");
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemsetAsync(d_hist, 0, 4u << bits, s));
    if (n == 0) return RS_OK;
    rs::PassList pl{};
    pl.count = 1;
    pl.width[0] = bits;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(2048, (n + 4ull * rs::kBlock - 1) / (4ull * rs::kBlock));
    hipLaunchKernelGGL((rs::k_pass_totals<1, rs::kBlock>), dim3(grid), dim3(rs::kBlock), 0, s, (const uint32_t*)keys,
                       (uint32_t)n, pl, shift, (uint32_t*)d_hist);
    HIP_TRY(hipGetLastError());
    return RS_OK;
}

RS_EXPORT rs_status rs_is_sorted(const void* keys, uint64_t n, uint32_t bit_count, void* d_flag,
                                 void* stream) {
    if (!d_flag) return fail(RS_ERR_INVALID_ARG, "null flag");
    if (n > 0xFFFFFFFFull) return fail(RS_ERR_INVALID_ARG, "n must be < 2^32");
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)d_flag, 1, 1, s));
    if (n < 2) return RS_OK;
    if (!keys) return fail(RS_ERR_INVALID_ARG, "null keys");
    const uint32_t grid = (uint32_t)std::min<uint64_t>(kCheckGrid, (n + rs::kBlock - 1) / rs::kBlock);
    hipLaunchKernelGGL(rs::k_is_sorted, dim3(grid), dim3(rs::kBlock), 0, s, (const uint32_t*)keys,
                       (uint32_t)n, full_mask(bit_count ? bit_count : 32), (uint32_t*)d_flag);
    HIP_TRY(hipGetLastError());
    return RS_OK;
}
