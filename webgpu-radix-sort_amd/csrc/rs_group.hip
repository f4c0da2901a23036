// rs_group.hip — multi-GPU group sort over the C ABI (include/rsort.h, rs_group_*).
//
// One host process drives `world` devices (rs_group_create / rs_group_sort;
// §8(e): the bucket exchange).  Host code only: every kernel is a librsort plan call
// (rsort.hip); the exchange is RCCL point-to-point (ncclCommInitAll + ncclGroupStart /
// ncclSend / ncclRecv, the single-process multi-device pattern) or peer DMA copies.
//
// Per rank r (devices[r]), one sort:
//   1. rs_histogram of the top digit of keys[r]            (sort stream; one key read)
//   2. stable partition by the top digit into the send buffer (records with values), fed the
//      step-1 counts (rs_plan_partition_records / _totals: one read of keys + values)
//   3. the counts to the host (pinned copy, overlapped with 2), then the bucket plan on the host
//      (rs_group_plan, identical to radix_sort_amd/distributed.py's bucket_owners/bucket_groups)
//   4. `rounds` exchange rounds on the comm stream: round g sends rank q its round-g buckets (one
//      contiguous range of the partitioned slice) and receives every source's round-g segment
//      into [base_g + off_s, ...): source-major, so the region is the bucket range's keys in
//      global input order; the own segment is a device copy
//   5. the sort stream waits for round g only, then sorts region g (rs_plan_sort_records: records
//      in, separate arrays out; keys only: rs_plan_sort_n in place) while later rounds move.
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
    rs_plan* part = nullptr;        // partition pass (capacity = desc.capacity)
    rs_plan* local = nullptr;       // local sorts (grows with the received regions)
    uint64_t local_cap = 0;
    uint32_t* hist = nullptr;       // device [buckets]
    uint32_t* hist_host = nullptr;  // pinned [buckets]
    void* send = nullptr;           // partitioned slice (records or keys)
    uint64_t send_cap = 0;          // bytes
    void* recv = nullptr;           // received regions, round-major then source-major
    uint64_t recv_cap = 0;
    uint32_t* out_k = nullptr;      // result with values: separate arrays
    uint32_t* out_v = nullptr;
    uint64_t out_k_cap = 0, out_v_cap = 0;   // bytes
    // result of the last sort
    void* res_k = nullptr;
    void* res_v = nullptr;
    uint64_t res_n = 0;
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
        (void)hipFree(k.send);
        (void)hipFree(k.recv);
        (void)hipFree(k.out_k);
        (void)hipFree(k.out_v);
        for (hipEvent_t e : {k.ev_in, k.ev_part, k.ev_hist, k.ev_done})
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : k.ev_round)
            if (e) (void)hipEventDestroy(e);
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
    const uint32_t buckets = 1u << g->desc.top_bits;
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
        G_HIP(hipMalloc((void**)&k.hist, 4ull * buckets));
        G_HIP(hipHostMalloc((void**)&k.hist_host, 4ull * buckets, hipHostMallocDefault));
        if (world > 1) {
            rs_plan_desc pd{};
            pd.device = k.device;
            pd.count = std::max<uint64_t>(g->desc.capacity, 1);
            pd.bit_count = 32;
            pd.flags = g->kv ? RS_FLAG_HAS_VALUES : 0u;
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
    if (d.top_bits > 8) return gfail(RS_ERR_INVALID_ARG, "rs_group_create: top_bits must be in [1, 8] (got %u)", d.top_bits);
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
    if (W == 1) {
        G_TRY(group_sort_world1(g, keys, values, counts[0]));
    } else {
        // 1-2: top-digit counts, their copy to the host, then the partition (fed the counts)
        for (int i = 0; i < W; ++i) {
            Rank& k = g->r[i];
            Dev dev(k.device);
            const uint64_t n = counts[i];
            G_TRY(grow(&k.send, &k.send_cap, esz * n));
            G_TRY(rs_histogram(keys[i], n, shift, bits, k.hist, k.sort_s));
            G_HIP(hipMemcpyAsync(k.hist_host, k.hist, 4ull * B, hipMemcpyDeviceToHost, k.sort_s));
            G_HIP(hipEventRecord(k.ev_hist, k.sort_s));
            if (n) {
                if (g->kv)
                    G_TRY(rs_plan_partition_records(k.part, keys[i], values[i], k.send, n, shift, bits, k.hist, k.sort_s));
                else
                    G_TRY(rs_plan_partition_totals(k.part, keys[i], nullptr, k.send, nullptr, n, shift, bits, k.hist, k.sort_s));
            }
            G_HIP(hipEventRecord(k.ev_part, k.sort_s));
        }
        // 3: the bucket plan (host, from every rank's counts)
        g->hist_all.assign((size_t)W * B, 0);
        for (int i = 0; i < W; ++i) {
            Dev dev(g->r[i].device);
            G_HIP(hipEventSynchronize(g->r[i].ev_hist));
            for (uint32_t b = 0; b < B; ++b) g->hist_all[(size_t)i * B + b] = g->r[i].hist_host[b];
        }
        g->bounds.assign(W + 1, 0);
        g->cuts.assign((size_t)W * (G + 1), 0);
        G_TRY(rs_group_plan(W, B, G, g->hist_all.data(), g->bounds.data(), g->cuts.data()));
        auto cut = [&](int q, uint32_t j) { return g->cuts[(size_t)q * (G + 1) + j]; };
        // start[r][b]: bucket b's offset in rank r's partitioned slice
        std::vector<uint64_t> start((size_t)W * (B + 1), 0);
        for (int i = 0; i < W; ++i)
            for (uint32_t b = 0; b < B; ++b)
                start[(size_t)i * (B + 1) + b + 1] = start[(size_t)i * (B + 1) + b] + g->hist_all[(size_t)i * B + b];
        auto seg = [&](int src, uint32_t b0, uint32_t b1) {   // [begin, end) in src's slice
            return std::make_pair(start[(size_t)src * (B + 1) + b0], start[(size_t)src * (B + 1) + b1]);
        };
        // receive layout of rank q: off[q][g][s], region bases base[q][g]
        std::vector<uint64_t> off((size_t)W * G * W), base((size_t)W * (G + 1));
        for (int q = 0; q < W; ++q) {
            uint64_t pos = 0;
            for (uint32_t j = 0; j < G; ++j) {
                base[(size_t)q * (G + 1) + j] = pos;
                for (int s = 0; s < W; ++s) {
                    off[((size_t)q * G + j) * W + s] = pos;
                    auto r = seg(s, cut(q, j), cut(q, j + 1));
                    pos += r.second - r.first;
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
            }
            G_TRY(ensure_local(g, k, biggest));
            G_HIP(hipStreamWaitEvent(k.comm_s, k.ev_part, 0));
        }
        // 4: exchange rounds
        const bool rccl = g->desc.transport == RS_TRANSPORT_RCCL;
        for (uint32_t j = 0; j < G; ++j) {
            // every send / receive of round j; inside an RCCL group a failure must not return
            // before ncclGroupEnd (the group depth is per thread: the next round would nest in
            // the open group), so the calls run in a lambda and the group is always closed
            auto post = [&]() -> rs_status {
                for (int src = 0; src < W; ++src) {
                    Rank& k = g->r[src];
                    Dev dev(k.device);
                    for (int dst = 0; dst < W; ++dst) {
                        auto r = seg(src, cut(dst, j), cut(dst, j + 1));
                        const uint64_t m = r.second - r.first;
                        char* from = (char*)k.send + esz * r.first;
                        char* to = (char*)g->r[dst].recv + esz * off[((size_t)dst * G + j) * W + src];
                        if (dst == src || !rccl) {
                            if (!m) continue;
                            if (g->r[dst].device == k.device)
                                G_HIP(hipMemcpyAsync(to, from, esz * m, hipMemcpyDeviceToDevice, k.comm_s));
                            else
                                G_HIP(hipMemcpyPeerAsync(to, g->r[dst].device, from, k.device, esz * m, k.comm_s));
                        } else if (m) {
                            G_NCCL(ncclSend(from, m, g->kv ? ncclUint64 : ncclUint32, dst, k.comm, k.comm_s));
                        }
                    }
                    if (rccl)
                        for (int s = 0; s < W; ++s) {
                            if (s == src) continue;
                            auto r = seg(s, cut(src, j), cut(src, j + 1));
                            const uint64_t m = r.second - r.first;
                            if (!m) continue;
                            char* to = (char*)k.recv + esz * off[((size_t)src * G + j) * W + s];
                            G_NCCL(ncclRecv(to, m, g->kv ? ncclUint64 : ncclUint32, s, k.comm, k.comm_s));
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
            }
        }
        // 5: region g sorted once round g has landed (RCCL: the receiver's own comm stream;
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
                if (b <= a) continue;
                // every key of round j lies in its buckets' range: the local sort may work on the
                // range-relative bits (the hybrid MSD path over this rank's buckets)
                const uint32_t ca = g->cuts[(size_t)q * (G + 1) + j], cb = g->cuts[(size_t)q * (G + 1) + j + 1];
                const uint32_t klo = ca << (32 - bits);
                const uint32_t khi = cb >= B ? 0xFFFFFFFFu : (cb << (32 - bits)) - 1u;
                if (g->kv)
                    G_TRY(rs_plan_sort_records_range(k.local, (char*)k.recv + 8 * a, k.out_k + a, k.out_v + a, b - a,
                                                     klo, khi, k.sort_s));
                else
                    G_TRY(rs_plan_sort_n(k.local, (uint32_t*)k.recv + a, nullptr, b - a, k.sort_s));
            }
            k.res_k = g->kv ? (void*)k.out_k : k.recv;
            k.res_v = g->kv ? (void*)k.out_v : nullptr;
            k.res_n = base[(size_t)q * (G + 1) + G];
        }
    }
    for (int i = 0; i < W; ++i) {
        Rank& k = g->r[i];
        Dev dev(k.device);
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
