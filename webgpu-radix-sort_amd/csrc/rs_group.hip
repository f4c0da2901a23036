// rs_group.hip — multi-GPU group sort over the C ABI (include/rsort.h, rs_group_*).
//
// One host process drives `world` devices (rs_group_create / rs_group_sort;
// §8(e): the bucket exchange).  Host code only: every kernel is a librsort plan call
// (rsort.hip); the exchange is RCCL point-to-point (ncclCommInitAll + ncclGroupStart /
// ncclSend / ncclRecv, the single-process multi-device pattern) or peer DMA copies.
//
// The exchange is the first pass of the single-GPU hybrid sort split across the ranks, so a rank
// moves the bytes of one single-GPU sort of its share (52 B/key with values):
//   1. rs_plan_hist16: the 16-bit bucket table of keys[r] (one key read, 4 B/key) -> pinned host
//   2. the stable partition of keys[r] / values[r] by the top byte into the send buffer (records
//      with values), fed the table's top-byte totals (16 B/key) = the hybrid sort's pass 0
//   3. host: every rank's table; whole-top-byte ownership (~1/world of the keys per rank, equal keys
//      never split) and `rounds` groups of top bytes per rank (rs_group_plan); every receiver's
//      layout: round-major, then top byte, then source rank (so each top-byte segment of a round's
//      region holds that byte's records in global input order), and its region tables (the 16-bit
//      counts summed over the sources), uploaded to the receiver
//   4. `rounds` exchange rounds on the comm stream: one message per (source, top byte) chunk, the
//      own chunks device copies
//   5. the sort stream waits for round g only, then sorts region g with rs_plan_sort_region (the
//      segmented next-byte pass + the in-LDS bucket sort, 32 B/key; records in, separate arrays
//      out) while later rounds move.  Keys only: the same exchange, rs_plan_sort_n per region.
// At world size 1 nothing is exchanged: the slice is sorted straight from the input into the
// output (rs_plan_sort_copy), no partition pass.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "rs_internal.h"

#define RS_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

rs_status gfail(rs_status s, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    return rs_internal_fail(s, buf);
}

#define G_HIP(expr)                                                                      \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return gfail(e_ == hipErrorOutOfMemory ? RS_ERR_OUT_OF_MEMORY : RS_ERR_HIP,  \
                         "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,       \
                         __LINE__);                                                      \
    } while (0)

#define G_NCCL(expr)                                                                     \
    do {                                                                                 \
        ncclResult_t r_ = (expr);                                                        \
        if (r_ != ncclSuccess)                                                           \
            return gfail(RS_ERR_HIP, "%s: %s (%s:%d)", #expr, ncclGetErrorString(r_),     \
                         __FILE__, __LINE__);                                            \
    } while (0)

#define G_TRY(expr)                                                                      \
    do {                                                                                 \
        rs_status s_ = (expr);                                                           \
        if (s_ != RS_OK) return s_;                                                      \
    } while (0)

constexpr int kMaxWorld = 64;
constexpr uint32_t kMaxRounds = 16;

struct Dev {
    int prev = -1;
    explicit Dev(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (d != prev) (void)hipSetDevice(d);
    }
    ~Dev() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Cut buckets [lo, hi) into `parts` consecutive runs of whole buckets of ~equal total count:
// cut p is the first bucket at which the running total reaches ceil(p * total / parts)
// (radix_sort_amd/distributed.py _split_whole, the same arithmetic).
void split_whole(const uint64_t* counts, uint32_t lo, uint32_t hi, uint32_t parts, uint32_t* cuts) {
    uint64_t total = 0;
    for (uint32_t b = lo; b < hi; ++b) total += counts[b];
    uint32_t k = 0, p = 1;
    cuts[k++] = lo;
    uint64_t cum = 0;
    for (uint32_t b = lo; b < hi; ++b) {
        while (p < parts && cum >= (total * p + parts - 1) / parts) {
            cuts[k++] = b;
            ++p;
        }
        cum += counts[b];
    }
    while (p < parts) {
        cuts[k++] = hi;
        ++p;
    }
    cuts[k] = hi;
}

struct Rank {
    int device = 0;
    hipStream_t sort_s = nullptr, comm_s = nullptr;
    hipEvent_t ev_in = nullptr, ev_part = nullptr, ev_hist = nullptr, ev_done = nullptr;
    hipEvent_t ev_round[kMaxRounds] = {};
    ncclComm_t comm = nullptr;
    rs_plan* part = nullptr;        // 16-bit table + partition pass (RS_USAGE_PARTITION, capacity =
                                    // desc.capacity)
    rs_plan* local = nullptr;       // local sorts (grows with the received regions)
    uint64_t local_cap = 0;
    uint32_t* hist = nullptr;       // device [RS_HIST16_WORDS]: the slice's 16-bit table + top totals
    uint32_t* hist_host = nullptr;  // pinned copy
    uint32_t* reg = nullptr;        // device [rounds][65536]: this rank's region tables
    uint32_t* reg_host = nullptr;   // pinned staging of them
    void* send = nullptr;           // partitioned slice (records or keys)
    uint64_t send_cap = 0;          // bytes
    void* recv = nullptr;           // received regions: round-major, then top byte, then source
    uint64_t recv_cap = 0;
    uint32_t* out_k = nullptr;      // result with values: separate arrays
    uint32_t* out_v = nullptr;
    uint64_t out_k_cap = 0, out_v_cap = 0;   // bytes
    // result of the last sort
    void* res_k = nullptr;
    void* res_v = nullptr;
    uint64_t res_n = 0;
    // rs_group_set_profiling: timing events of the last sort (start, hist16, partition, per round
    // the comm stream's completion and the region sort's, done) and its off-rank exchange bytes
    hipEvent_t t_start = nullptr, t_hist = nullptr, t_part = nullptr, t_done = nullptr;
    hipEvent_t t_round[kMaxRounds] = {}, t_sorted[kMaxRounds] = {};
    uint32_t t_rounds = 0;
    bool t_valid = false;
    uint64_t bytes_sent = 0, bytes_recv = 0;
};

rs_status grow(void** ptr, uint64_t* cap, uint64_t need) {
    if (need <= *cap && *ptr) return RS_OK;
    if (*ptr) G_HIP(hipFree(*ptr));
    *ptr = nullptr;
    *cap = 0;
    const uint64_t bytes = std::max<uint64_t>(need + need / 8, 64);
    G_HIP(hipMalloc(ptr, bytes));
    *cap = bytes;
    return RS_OK;
}

}  // namespace

struct rs_group {
    int world = 0;
    rs_group_desc desc{};
    bool kv = false;
    bool profiling = false;
    std::vector<Rank> r;
    std::vector<uint64_t> hist_all;   // [world][buckets]
    std::vector<uint32_t> bounds, cuts;
};

RS_EXPORT rs_status rs_group_plan(int32_t world, uint32_t buckets, uint32_t rounds,
                                  const uint64_t* hist_all, uint32_t* bounds, uint32_t* cuts) {
    if (world < 1 || world > kMaxWorld || buckets == 0 || rounds == 0 || !hist_all || !bounds || !cuts)
        return gfail(RS_ERR_INVALID_ARG, "rs_group_plan: need 1 <= world <= %d, buckets >= 1, rounds >= 1 and non-null arrays", kMaxWorld);
    std::vector<uint64_t> totals(buckets, 0);
    for (int q = 0; q < world; ++q)
        for (uint32_t b = 0; b < buckets; ++b) totals[b] += hist_all[(uint64_t)q * buckets + b];
    split_whole(totals.data(), 0, buckets, (uint32_t)world, bounds);
    for (int q = 0; q < world; ++q)
        split_whole(totals.data(), bounds[q], bounds[q + 1], rounds, cuts + (uint64_t)q * (rounds + 1));
    return RS_OK;
}

RS_EXPORT void rs_group_destroy(rs_group* g) {
    if (!g) return;
    for (auto& k : g->r) {
        Dev dev(k.device);
        if (k.sort_s) (void)hipStreamSynchronize(k.sort_s);
        if (k.comm_s) (void)hipStreamSynchronize(k.comm_s);
    }
    for (auto& k : g->r) {
        Dev dev(k.device);
        if (k.comm) (void)ncclCommDestroy(k.comm);
        if (k.part) rs_plan_destroy(k.part);
        if (k.local) rs_plan_destroy(k.local);
        (void)hipFree(k.hist);
        if (k.hist_host) (void)hipHostFree(k.hist_host);
        (void)hipFree(k.reg);
        if (k.reg_host) (void)hipHostFree(k.reg_host);
        (void)hipFree(k.send);
        (void)hipFree(k.recv);
        (void)hipFree(k.out_k);
        (void)hipFree(k.out_v);
        for (hipEvent_t e : {k.ev_in, k.ev_part, k.ev_hist, k.ev_done})
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : k.ev_round)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : {k.t_start, k.t_hist, k.t_part, k.t_done})
            if (e) (void)hipEventDestroy(e);
        for (uint32_t j = 0; j < kMaxRounds; ++j) {
            if (k.t_round[j]) (void)hipEventDestroy(k.t_round[j]);
            if (k.t_sorted[j]) (void)hipEventDestroy(k.t_sorted[j]);
        }
        if (k.sort_s) (void)hipStreamDestroy(k.sort_s);
        if (k.comm_s) (void)hipStreamDestroy(k.comm_s);
    }
    delete g;
}

static rs_status group_create(int32_t world, const int32_t* devices, const rs_group_desc* desc,
                              rs_group* g) {
    int ndev = 0;
    G_HIP(hipGetDeviceCount(&ndev));
    for (int i = 0; i < world; ++i) {
        if (devices[i] < 0 || devices[i] >= ndev)
            return gfail(RS_ERR_INVALID_ARG, "rs_group_create: device %d out of range (%d devices)", devices[i], ndev);
        if (desc->transport == RS_TRANSPORT_RCCL)
            for (int j = 0; j < i; ++j)
                if (devices[j] == devices[i])
                    return gfail(RS_ERR_INVALID_ARG, "rs_group_create: device %d listed twice; RCCL needs one rank per device (RS_TRANSPORT_COPY allows virtual ranks)", devices[i]);
    }
    g->r.resize(world);
    for (int i = 0; i < world; ++i) {
        Rank& k = g->r[i];
        k.device = devices[i];
        Dev dev(k.device);
        G_HIP(hipStreamCreateWithFlags(&k.sort_s, hipStreamNonBlocking));
        G_HIP(hipStreamCreateWithFlags(&k.comm_s, hipStreamNonBlocking));
        for (hipEvent_t* e : {&k.ev_in, &k.ev_part, &k.ev_hist, &k.ev_done})
            G_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
        for (uint32_t j = 0; j < g->desc.rounds; ++j)
            G_HIP(hipEventCreateWithFlags(&k.ev_round[j], hipEventDisableTiming));
        if (world > 1) {
            G_HIP(hipMalloc((void**)&k.hist, 4ull * RS_HIST16_WORDS));
            G_HIP(hipHostMalloc((void**)&k.hist_host, 4ull * RS_HIST16_WORDS, hipHostMallocDefault));
            if (g->kv) {
                G_HIP(hipMalloc((void**)&k.reg, 4ull * 65536 * g->desc.rounds));
                G_HIP(hipHostMalloc((void**)&k.reg_host, 4ull * 65536 * g->desc.rounds, hipHostMallocDefault));
            }
            // the sender's plan: its 16-bit table and the partition pass only (no ping-pong copy;
            // rs_plan_hist16 needs room for one histogram row: capacity >= 32768)
            rs_plan_desc pd{};
            pd.device = k.device;
            pd.count = std::max<uint64_t>(g->desc.capacity, 32768);
            pd.bit_count = 32;
            pd.flags = g->kv ? RS_FLAG_HAS_VALUES : 0u;
            pd.usage = RS_USAGE_PARTITION;
            G_TRY(rs_plan_create(&pd, &k.part));
        }
        if (desc->transport == RS_TRANSPORT_COPY)
            for (int j = 0; j < world; ++j)
                if (devices[j] != k.device) {
                    hipError_t e = hipDeviceEnablePeerAccess(devices[j], 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                        (void)hipGetLastError();   // copies still work, staged by the runtime
                }
    }
    if (desc->transport == RS_TRANSPORT_RCCL) {
        std::vector<ncclComm_t> comms(world);
        std::vector<int> devs(devices, devices + world);
        G_NCCL(ncclCommInitAll(comms.data(), world, devs.data()));
        for (int i = 0; i < world; ++i) g->r[i].comm = comms[i];
    }
    return RS_OK;
}

RS_EXPORT rs_status rs_group_create(int32_t world, const int32_t* devices, const rs_group_desc* desc,
                                    rs_group** out) {
    if (!out || !devices || !desc) return gfail(RS_ERR_INVALID_ARG, "rs_group_create: null argument");
    *out = nullptr;
    if (world < 1 || world > kMaxWorld)
        return gfail(RS_ERR_INVALID_ARG, "rs_group_create: world must be in [1, %d] (got %d)", kMaxWorld, world);
    rs_group_desc d = *desc;
    if (d.top_bits == 0) d.top_bits = 8;
    if (d.rounds == 0) d.rounds = 4;
    if (d.top_bits != 8)
        return gfail(RS_ERR_INVALID_ARG, "rs_group_create: top_bits must be 8 or 0 (got %u): the exchange digit is the top "
                     "byte, the sort's first MSD pass", d.top_bits);
    if (d.rounds > kMaxRounds) return gfail(RS_ERR_INVALID_ARG, "rs_group_create: rounds must be in [1, %u] (got %u)", kMaxRounds, d.rounds);
    if (d.flags & ~RS_FLAG_HAS_VALUES) return gfail(RS_ERR_INVALID_ARG, "rs_group_create: flags may only hold RS_FLAG_HAS_VALUES (got 0x%x)", d.flags);
    if (d.transport != RS_TRANSPORT_RCCL && d.transport != RS_TRANSPORT_COPY)
        return gfail(RS_ERR_INVALID_ARG, "rs_group_create: unknown transport %u", d.transport);
    if (d.capacity > 0xFFFFFFFFull) return gfail(RS_ERR_INVALID_ARG, "rs_group_create: capacity must be < 2^32");
    rs_group* g = new (std::nothrow) rs_group();
    if (!g) return gfail(RS_ERR_OUT_OF_MEMORY, "host allocation failed");
    g->world = world;
    g->desc = d;
    g->kv = (d.flags & RS_FLAG_HAS_VALUES) != 0;
    rs_status st = group_create(world, devices, &d, g);
    if (st != RS_OK) {
        rs_group_destroy(g);
        return st;
    }
    *out = g;
    return RS_OK;
}

// Local sort plan of rank k with capacity >= n (recreated larger when needed; the previous sort
// on the rank is complete, rs_group_sort synchronises first).
static rs_status ensure_local(rs_group* g, Rank& k, uint64_t n) {
    if (k.local && k.local_cap >= n) return RS_OK;
    if (k.local) rs_plan_destroy(k.local);
    k.local = nullptr;
    rs_plan_desc pd{};
    pd.device = k.device;
    pd.count = std::min<uint64_t>(std::max<uint64_t>(n + n / 8, 1), 0xFFFFFFFFull);
    pd.bit_count = 32;
    pd.flags = g->kv ? RS_FLAG_HAS_VALUES : 0u;
    G_TRY(rs_plan_create(&pd, &k.local));
    k.local_cap = pd.count;
    return RS_OK;
}

static rs_status group_sort_world1(rs_group* g, void* const* keys, void* const* values, uint64_t n) {
    Rank& k = g->r[0];
    Dev dev(k.device);
    G_TRY(ensure_local(g, k, n));
    if (g->kv) {
        G_TRY(grow((void**)&k.out_k, &k.out_k_cap, 4 * n));
        G_TRY(grow((void**)&k.out_v, &k.out_v_cap, 4 * n));
        G_TRY(rs_plan_sort_copy(k.local, keys[0], values[0], k.out_k, k.out_v, n, k.sort_s));
        k.res_k = k.out_k;
        k.res_v = k.out_v;
    } else {
        G_TRY(grow(&k.recv, &k.recv_cap, 4 * n));
        G_TRY(rs_plan_sort_copy(k.local, keys[0], nullptr, k.recv, nullptr, n, k.sort_s));
        k.res_k = k.recv;
        k.res_v = nullptr;
    }
    k.res_n = n;
    return RS_OK;
}

RS_EXPORT rs_status rs_group_sort(rs_group* g, void* const* keys, void* const* values,
                                  const uint64_t* counts, void* const* streams) {
    if (!g || !keys || !counts) return gfail(RS_ERR_INVALID_ARG, "rs_group_sort: null argument");
    if (g->kv && !values) return gfail(RS_ERR_INVALID_ARG, "rs_group_sort: group has values but values is null");
    const int W = g->world;
    const uint32_t bits = g->desc.top_bits, B = 1u << bits, G = g->desc.rounds;
    const uint32_t shift = 32 - bits;
    const uint64_t esz = g->kv ? 8 : 4;   // bytes per exchanged element (record or key)
    for (int i = 0; i < W; ++i) {
        if (counts[i] > g->desc.capacity)
            return gfail(RS_ERR_CAPACITY, "rs_group_sort: counts[%d] = %llu exceeds the group capacity %llu", i,
                         (unsigned long long)counts[i], (unsigned long long)g->desc.capacity);
        if (counts[i] && (!keys[i] || (g->kv && !values[i])))
            return gfail(RS_ERR_INVALID_ARG, "rs_group_sort: rank %d has a null buffer", i);
    }
    // the previous sort on every rank is complete (its buffers may be regrown below), and a
    // device-side failure of it is reported now rather than lost
    G_TRY(rs_group_synchronize(g));
    for (int i = 0; i < W; ++i) {
        Rank& k = g->r[i];
        Dev dev(k.device);
        if (streams && streams[i]) {
            G_HIP(hipEventRecord(k.ev_in, (hipStream_t)streams[i]));
            G_HIP(hipStreamWaitEvent(k.sort_s, k.ev_in, 0));
        }
    }
    const bool prof = g->profiling;
    auto mark = [&](Rank& k, hipEvent_t e, hipStream_t s) -> rs_status {
        if (prof) G_HIP(hipEventRecord(e, s));
        return RS_OK;
    };
    for (int i = 0; i < W; ++i) {
        Rank& k = g->r[i];
        Dev dev(k.device);
        k.t_valid = false;   // set once t_done is recorded: a sort that fails partway has no timing
        k.t_rounds = W == 1 ? 0u : G;
        k.bytes_sent = k.bytes_recv = 0;
        G_TRY(mark(k, k.t_start, k.sort_s));
    }
    if (W == 1) {
        G_TRY(group_sort_world1(g, keys, values, counts[0]));
    } else {
        // 1-2: the 16-bit table, its copy to the host, then the partition (fed the top totals)
        for (int i = 0; i < W; ++i) {
            Rank& k = g->r[i];
            Dev dev(k.device);
            const uint64_t n = counts[i];
            G_TRY(grow(&k.send, &k.send_cap, esz * n));
            G_TRY(rs_plan_hist16(k.part, keys[i], n, k.hist, k.sort_s));
            G_HIP(hipMemcpyAsync(k.hist_host, k.hist, 4ull * RS_HIST16_WORDS, hipMemcpyDeviceToHost, k.sort_s));
            G_HIP(hipEventRecord(k.ev_hist, k.sort_s));
            G_TRY(mark(k, k.t_hist, k.sort_s));
            if (n) {
                if (g->kv)
                    G_TRY(rs_plan_partition_records(k.part, keys[i], values[i], k.send, n, shift, bits, k.hist + 65536,
                                                    k.sort_s));
                else
                    G_TRY(rs_plan_partition_totals(k.part, keys[i], nullptr, k.send, nullptr, n, shift, bits,
                                                   k.hist + 65536, k.sort_s));
            }
            G_HIP(hipEventRecord(k.ev_part, k.sort_s));
            G_TRY(mark(k, k.t_part, k.sort_s));
        }
        // 3: the bucket plan (host, from every rank's top-byte totals)
        g->hist_all.assign((size_t)W * B, 0);
        for (int i = 0; i < W; ++i) {
            Dev dev(g->r[i].device);
            G_HIP(hipEventSynchronize(g->r[i].ev_hist));
            for (uint32_t b = 0; b < B; ++b) g->hist_all[(size_t)i * B + b] = g->r[i].hist_host[65536 + b];
        }
        g->bounds.assign(W + 1, 0);
        g->cuts.assign((size_t)W * (G + 1), 0);
        G_TRY(rs_group_plan(W, B, G, g->hist_all.data(), g->bounds.data(), g->cuts.data()));
        auto cut = [&](int q, uint32_t j) { return g->cuts[(size_t)q * (G + 1) + j]; };
        auto cnt = [&](int src, uint32_t t) { return g->hist_all[(size_t)src * B + t]; };
        // start[src][t]: top byte t's offset in rank src's partitioned slice
        std::vector<uint64_t> start((size_t)W * (B + 1), 0);
        for (int i = 0; i < W; ++i)
            for (uint32_t b = 0; b < B; ++b)
                start[(size_t)i * (B + 1) + b + 1] = start[(size_t)i * (B + 1) + b] + cnt(i, b);
        // receive layout: top byte t from source s lands at off[t * W + s] of its owner's buffer
        // (round-major, then top byte, then source); region j of rank q = [base[q][j], base[q][j+1])
        std::vector<uint64_t> off((size_t)B * W, 0), base((size_t)W * (G + 1), 0);
        for (int q = 0; q < W; ++q) {
            uint64_t pos = 0;
            for (uint32_t j = 0; j < G; ++j) {
                base[(size_t)q * (G + 1) + j] = pos;
                for (uint32_t t = cut(q, j); t < cut(q, j + 1); ++t)
                    for (int src = 0; src < W; ++src) {
                        off[(size_t)t * W + src] = pos;
                        pos += cnt(src, t);
                    }
            }
            base[(size_t)q * (G + 1) + G] = pos;
            if (pos > 0xFFFFFFFFull)
                return gfail(RS_ERR_CAPACITY, "rs_group_sort: rank %d would receive %llu keys (>= 2^32)", q, (unsigned long long)pos);
        }
        for (int q = 0; q < W; ++q) {
            Rank& k = g->r[q];
            Dev dev(k.device);
            const uint64_t n_recv = base[(size_t)q * (G + 1) + G];
            uint64_t biggest = 0;
            for (uint32_t j = 0; j < G; ++j)
                biggest = std::max(biggest, base[(size_t)q * (G + 1) + j + 1] - base[(size_t)q * (G + 1) + j]);
            G_TRY(grow(&k.recv, &k.recv_cap, esz * n_recv));
            if (g->kv) {
                G_TRY(grow((void**)&k.out_k, &k.out_k_cap, 4 * n_recv));
                G_TRY(grow((void**)&k.out_v, &k.out_v_cap, 4 * n_recv));
                // the region tables: round j's 16-bit counts summed over the sources, zero outside
                // its top bytes; uploaded on the sort stream (ordered before the region sorts)
                for (uint32_t j = 0; j < G; ++j) {
                    uint32_t* t16 = k.reg_host + (size_t)j * 65536;
                    memset(t16, 0, 4 * 65536);
                    for (uint32_t b = cut(q, j) << 8; b < (cut(q, j + 1) << 8); ++b) {
                        uint64_t c = 0;
                        for (int src = 0; src < W; ++src) c += g->r[src].hist_host[b];
                        t16[b] = (uint32_t)c;
                    }
                }
                G_HIP(hipMemcpyAsync(k.reg, k.reg_host, 4ull * 65536 * G, hipMemcpyHostToDevice, k.sort_s));
            }
            G_TRY(ensure_local(g, k, biggest));
            G_HIP(hipStreamWaitEvent(k.comm_s, k.ev_part, 0));
            // off-rank exchange bytes: what q sends to every other rank and receives from them
            for (uint32_t j = 0; j < G; ++j)
                for (int o = 0; o < W; ++o) {
                    if (o == q) continue;
                    for (uint32_t t = cut(o, j); t < cut(o, j + 1); ++t) k.bytes_sent += esz * cnt(q, t);
                    for (uint32_t t = cut(q, j); t < cut(q, j + 1); ++t) k.bytes_recv += esz * cnt(o, t);
                }
        }
        // 4: exchange rounds, one message per (source, top byte) chunk
        const bool rccl = g->desc.transport == RS_TRANSPORT_RCCL;
        for (uint32_t j = 0; j < G; ++j) {
            // every send / receive of round j; inside an RCCL group a failure must not return
            // before ncclGroupEnd (the group depth is per thread: the next round would nest in
            // the open group), so the calls run in a lambda and the group is always closed
            auto post = [&]() -> rs_status {
                for (int src = 0; src < W; ++src) {
                    Rank& k = g->r[src];
                    Dev dev(k.device);
                    for (int dst = 0; dst < W; ++dst)
                        for (uint32_t t = cut(dst, j); t < cut(dst, j + 1); ++t) {
                            const uint64_t m = cnt(src, t);
                            if (!m) continue;
                            char* from = (char*)k.send + esz * start[(size_t)src * (B + 1) + t];
                            char* to = (char*)g->r[dst].recv + esz * off[(size_t)t * W + src];
                            if (dst == src || !rccl) {
                                if (g->r[dst].device == k.device)
                                    G_HIP(hipMemcpyAsync(to, from, esz * m, hipMemcpyDeviceToDevice, k.comm_s));
                                else
                                    G_HIP(hipMemcpyPeerAsync(to, g->r[dst].device, from, k.device, esz * m, k.comm_s));
                            } else {
                                G_NCCL(ncclSend(from, m, g->kv ? ncclUint64 : ncclUint32, dst, k.comm, k.comm_s));
                            }
                        }
                    if (rccl)   // what src receives from every peer, in the peer's send order (t ascending)
                        for (int s = 0; s < W; ++s) {
                            if (s == src) continue;
                            for (uint32_t t = cut(src, j); t < cut(src, j + 1); ++t) {
                                const uint64_t m = cnt(s, t);
                                if (!m) continue;
                                char* to = (char*)k.recv + esz * off[(size_t)t * W + s];
                                G_NCCL(ncclRecv(to, m, g->kv ? ncclUint64 : ncclUint32, s, k.comm, k.comm_s));
                            }
                        }
                }
                return RS_OK;
            };
            if (rccl) G_NCCL(ncclGroupStart());
            const rs_status posted = post();
            if (rccl) {
                const ncclResult_t ended = ncclGroupEnd();
                G_TRY(posted);
                if (ended != ncclSuccess)
                    return gfail(RS_ERR_HIP, "ncclGroupEnd: %s (%s:%d)", ncclGetErrorString(ended), __FILE__, __LINE__);
            }
            G_TRY(posted);
            for (int src = 0; src < W; ++src) {
                Dev dev(g->r[src].device);
                G_HIP(hipEventRecord(g->r[src].ev_round[j], g->r[src].comm_s));
                G_TRY(mark(g->r[src], g->r[src].t_round[j], g->r[src].comm_s));
            }
        }
        // 5: region j sorted once round j has landed (RCCL: the receiver's own comm stream;
        // copies: every sender's), later rounds still on the wire
        for (int q = 0; q < W; ++q) {
            Rank& k = g->r[q];
            Dev dev(k.device);
            for (uint32_t j = 0; j < G; ++j) {
                if (rccl) {
                    G_HIP(hipStreamWaitEvent(k.sort_s, k.ev_round[j], 0));
                } else {
                    for (int s = 0; s < W; ++s) G_HIP(hipStreamWaitEvent(k.sort_s, g->r[s].ev_round[j], 0));
                }
                const uint64_t a = base[(size_t)q * (G + 1) + j], b = base[(size_t)q * (G + 1) + j + 1];
                if (b > a) {
                    if (g->kv)
                        G_TRY(rs_plan_sort_region(k.local, (char*)k.recv + 8 * a, k.out_k + a, k.out_v + a, b - a,
                                                  k.reg + (size_t)j * 65536, cut(q, j), cut(q, j + 1), k.sort_s));
                    else
                        G_TRY(rs_plan_sort_n(k.local, (uint32_t*)k.recv + a, nullptr, b - a, k.sort_s));
                }
                G_TRY(mark(k, k.t_sorted[j], k.sort_s));
            }
            k.res_k = g->kv ? (void*)k.out_k : k.recv;
            k.res_v = g->kv ? (void*)k.out_v : nullptr;
            k.res_n = base[(size_t)q * (G + 1) + G];
        }
    }
    for (int i = 0; i < W; ++i) {
        Rank& k = g->r[i];
        Dev dev(k.device);
        G_TRY(mark(k, k.t_done, k.sort_s));
        k.t_valid = prof;
        G_HIP(hipEventRecord(k.ev_done, k.sort_s));
        if (streams && streams[i]) G_HIP(hipStreamWaitEvent((hipStream_t)streams[i], k.ev_done, 0));
    }
    return RS_OK;
}

RS_EXPORT rs_status rs_group_result(const rs_group* g, int32_t rank, void** keys, void** values,
                                    uint64_t* count) {
    if (!g || rank < 0 || rank >= g->world)
        return gfail(RS_ERR_INVALID_ARG, "rs_group_result: null group or rank out of range");
    const Rank& k = g->r[rank];
    if (keys) *keys = k.res_k;
    if (values) *values = k.res_v;
    if (count) *count = k.res_n;
    return RS_OK;
}

RS_EXPORT rs_status rs_group_set_profiling(rs_group* g, int enable) {
    if (!g) return gfail(RS_ERR_INVALID_ARG, "rs_group_set_profiling: null group");
    if (enable)
        for (auto& k : g->r) {
            Dev dev(k.device);
            for (hipEvent_t* e : {&k.t_start, &k.t_hist, &k.t_part, &k.t_done})
                if (!*e) G_HIP(hipEventCreate(e));
            for (uint32_t j = 0; j < g->desc.rounds; ++j) {
                if (!k.t_round[j]) G_HIP(hipEventCreate(&k.t_round[j]));
                if (!k.t_sorted[j]) G_HIP(hipEventCreate(&k.t_sorted[j]));
            }
        }
    g->profiling = enable != 0;
    return RS_OK;
}

RS_EXPORT rs_status rs_group_times_get(rs_group* g, int32_t rank, rs_group_times* out) {
    if (!g || !out || rank < 0 || rank >= g->world)
        return gfail(RS_ERR_INVALID_ARG, "rs_group_times_get: null argument or rank out of range");
    memset(out, 0, sizeof(*out));
    Rank& k = g->r[rank];
    if (!k.t_valid) return gfail(RS_ERR_INVALID_ARG, "rs_group_times_get: the last sort ran without rs_group_set_profiling");
    Dev dev(k.device);
    G_HIP(hipEventSynchronize(k.t_done));
    for (uint32_t j = 0; j < k.t_rounds; ++j) G_HIP(hipEventSynchronize(k.t_round[j]));
    auto since = [&](hipEvent_t e, float* ms) -> rs_status {
        G_HIP(hipEventElapsedTime(ms, k.t_start, e));
        return RS_OK;
    };
    out->rounds = k.t_rounds;
    if (k.t_rounds) {
        G_TRY(since(k.t_hist, &out->hist16_ms));
        G_TRY(since(k.t_part, &out->partition_ms));
        for (uint32_t j = 0; j < k.t_rounds; ++j) {
            G_TRY(since(k.t_round[j], &out->round_done_ms[j]));
            G_TRY(since(k.t_sorted[j], &out->region_sorted_ms[j]));
        }
    }
    G_TRY(since(k.t_done, &out->done_ms));
    out->bytes_sent = k.bytes_sent;
    out->bytes_recv = k.bytes_recv;
    return RS_OK;
}

RS_EXPORT rs_status rs_group_synchronize(rs_group* g) {
    if (!g) return gfail(RS_ERR_INVALID_ARG, "rs_group_synchronize: null group");
    for (auto& k : g->r) {
        Dev dev(k.device);
        G_HIP(hipStreamSynchronize(k.sort_s));
        G_HIP(hipStreamSynchronize(k.comm_s));
    }
    rs_status first = RS_OK;
    for (auto& k : g->r)
        for (rs_plan* p : {k.part, k.local})
            if (p) {
                rs_status s = rs_plan_check(p);
                if (s != RS_OK && first == RS_OK) first = s;
            }
    return first;
}
