// Host-side AddressSanitizer / UBSan driver (SURVEY.md §5 "sanitizers"): exercises every C-ABI
// entry point of a librsort built with host-only sanitizers (make -C webgpu-radix-sort_amd/csrc
// asan: `-Xarch_host -fsanitize=address,undefined`; device code is not instrumented), so plan
// creation, the launch/schedule code, the multi-GPU group planner and its buffer management run
// under ASan on a GPU box.  Every result is checked on the host (sorted, a stable permutation).
// Exit status 0 = all checks passed and the sanitizers reported nothing.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#include "../include/rsort.h"

static int g_fail = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);              \
            fprintf(stderr, "\n");                     \
            ++g_fail;                                  \
        }                                              \
    } while (0)
#define OK(call) CHECK((call) == RS_OK, "%s -> %s", #call, rs_last_error())

static uint32_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)(z ^ (z >> 31));
}

// keys sorted ascending; values[i] = original index, stable (equal keys keep index order)
static bool verify(const std::vector<uint32_t>& in, const std::vector<uint32_t>& k,
                   const std::vector<uint32_t>* v, size_t n) {
    for (size_t i = 0; i + 1 < n; ++i)
        if (k[i] > k[i + 1]) return false;
    if (v) {
        for (size_t i = 0; i < n; ++i) {
            if ((*v)[i] >= n || in[(*v)[i]] != k[i]) return false;
            if (i + 1 < n && k[i] == k[i + 1] && (*v)[i] >= (*v)[i + 1]) return false;
        }
    }
    return true;
}

static void sort_case(size_t n, bool kv, uint32_t flags_extra, uint32_t key_mask) {
    std::vector<uint32_t> hk(n), hv(n);
    for (size_t i = 0; i < n; ++i) { hk[i] = mix(i * 7 + n) & key_mask; hv[i] = (uint32_t)i; }
    void *dk = nullptr, *dv = nullptr;
    OK(rs_malloc(0, 4 * n, &dk));
    OK(rs_malloc(0, 4 * n, &dv));
    OK(rs_memcpy_h2d(dk, hk.data(), 4 * n, nullptr));
    OK(rs_memcpy_h2d(dv, hv.data(), 4 * n, nullptr));
    rs_plan_desc d{};
    d.device = 0;
    d.count = n;
    d.flags = (kv ? RS_FLAG_HAS_VALUES : 0u) | flags_extra;
    rs_plan* p = nullptr;
    OK(rs_plan_create(&d, &p));
    if (p) {
        uint32_t path = 99;
        OK(rs_plan_last_path(p, &path));
        CHECK(path == RS_PATH_NONE, "last_path before any sort: %u", path);
        // events around the pass launches only (the bench's timed region)
        OK(rs_plan_set_profiling_kinds(p, (1u << RS_KERNEL_SCATTER) | (1u << RS_KERNEL_FALLBACK)));
        CHECK(rs_plan_set_profiling_kinds(p, 1u << RS_KERNEL_KINDS) == RS_ERR_INVALID_ARG, "bad kind mask accepted");
        OK(rs_plan_sort(p, dk, kv ? dv : nullptr, nullptr));
        OK(rs_plan_check(p));
        OK(rs_plan_last_path(p, &path));
        // (a count of 0 or 1 enqueues nothing: no sort to report)
        CHECK(n < 2 ? path == RS_PATH_NONE : (path >= RS_PATH_LSD && path <= RS_PATH_IN_ORDER),
              "last_path after a sort of %zu: %u", n, path);
        uint32_t levels = 99;
        OK(rs_plan_last_split(p, &levels));
        CHECK(levels == 0 || levels == 2 || levels == 3, "last_split: %u", levels);
        CHECK(rs_plan_last_split(p, nullptr) == RS_ERR_INVALID_ARG, "null levels accepted");
        double ms[RS_KERNEL_KINDS];
        uint64_t launches[RS_KERNEL_KINDS];
        OK(rs_plan_kernel_times(p, ms, launches));
        CHECK(launches[RS_KERNEL_HISTOGRAM] == 0 && launches[RS_KERNEL_BUCKET] == 0,
              "only the pass kinds are bracketed");
        OK(rs_plan_set_profiling(p, 0));
        std::vector<uint32_t> ok(n), ov(n);
        OK(rs_memcpy_d2h(ok.data(), dk, 4 * n, nullptr));
        OK(rs_memcpy_d2h(ov.data(), dv, 4 * n, nullptr));
        CHECK(verify(hk, ok, kv ? &ov : nullptr, n), "sort n=%zu kv=%d flags=%x", n, kv, flags_extra);
        rs_plan_info info;
        OK(rs_plan_info_get(p, &info));
        // a 1-key sort after a real one reports no path (nothing moved)
        if (n >= 2) {
            OK(rs_plan_sort_n(p, dk, kv ? dv : nullptr, 1, nullptr));
            OK(rs_plan_last_path(p, &path));
            CHECK(path == RS_PATH_NONE, "last_path after a 1-key sort: %u", path);
        }
        // the test-only path overrides: a bad field is refused, a valid set sorts the same
        rs_plan_debug dbg;
        memset(&dbg, 0xFF, sizeof(dbg));   // every field -1: keep
        dbg.tile = 3;
        CHECK(rs_plan_set_debug(p, &dbg) == RS_ERR_INVALID_ARG, "bad debug field accepted");
        CHECK(rs_plan_set_debug(p, nullptr) == RS_ERR_INVALID_ARG, "null debug accepted");
        dbg.tile = -1;
        dbg.split = 2;
        CHECK(rs_plan_set_debug(p, &dbg) == RS_ERR_INVALID_ARG, "bad split field accepted");
        dbg.split = 0;
        dbg.rank = 1;
        dbg.msd = 0;
        OK(rs_plan_set_debug(p, &dbg));
        OK(rs_memcpy_h2d(dk, hk.data(), 4 * n, nullptr));
        OK(rs_memcpy_h2d(dv, hv.data(), 4 * n, nullptr));
        OK(rs_plan_sort(p, dk, kv ? dv : nullptr, nullptr));
        OK(rs_plan_check(p));
        OK(rs_memcpy_d2h(ok.data(), dk, 4 * n, nullptr));
        OK(rs_memcpy_d2h(ov.data(), dv, 4 * n, nullptr));
        CHECK(verify(hk, ok, kv ? &ov : nullptr, n), "debug sort n=%zu kv=%d flags=%x", n, kv, flags_extra);
        rs_plan_destroy(p);
    }
    OK(rs_free(dk));
    OK(rs_free(dv));
}

static void copy_and_records(size_t n) {
    std::vector<uint32_t> hk(n), hv(n);
    for (size_t i = 0; i < n; ++i) { hk[i] = mix(i ^ 0x5555); hv[i] = (uint32_t)i; }
    void *ik, *iv, *ok, *ov, *rec;
    OK(rs_malloc(0, 4 * n, &ik));
    OK(rs_malloc(0, 4 * n, &iv));
    OK(rs_malloc(0, 4 * n, &ok));
    OK(rs_malloc(0, 4 * n, &ov));
    OK(rs_malloc(0, 8 * n, &rec));
    OK(rs_memcpy_h2d(ik, hk.data(), 4 * n, nullptr));
    OK(rs_memcpy_h2d(iv, hv.data(), 4 * n, nullptr));
    rs_plan_desc d{};
    d.count = n;
    d.flags = RS_FLAG_HAS_VALUES;
    rs_plan* p = nullptr;
    OK(rs_plan_create(&d, &p));
    std::vector<uint32_t> gk(n), gv(n);
    if (p) {
        OK(rs_plan_sort_copy(p, ik, iv, ok, ov, n, nullptr));
        OK(rs_plan_check(p));
        OK(rs_memcpy_d2h(gk.data(), ok, 4 * n, nullptr));
        OK(rs_memcpy_d2h(gv.data(), ov, 4 * n, nullptr));
        CHECK(verify(hk, gk, &gv, n), "sort_copy n=%zu", n);
        OK(rs_plan_partition_records(p, ik, iv, rec, n, 24, 8, nullptr, nullptr));
        OK(rs_plan_sort_records(p, rec, ok, ov, n, nullptr));
        OK(rs_plan_check(p));
        OK(rs_memcpy_d2h(gk.data(), ok, 4 * n, nullptr));
        OK(rs_memcpy_d2h(gv.data(), ov, 4 * n, nullptr));
        CHECK(verify(hk, gk, &gv, n), "partition+sort_records n=%zu", n);
        rs_plan_destroy(p);
    }
    // records already in order, through a check_order plan: the arrays are still written
    d.flags = RS_FLAG_HAS_VALUES | RS_FLAG_CHECK_ORDER;
    p = nullptr;
    OK(rs_plan_create(&d, &p));
    if (p) {
        std::vector<uint32_t> sk(hk), sr(2 * n);
        std::sort(sk.begin(), sk.end());
        for (size_t i = 0; i < n; ++i) { sr[2 * i] = sk[i]; sr[2 * i + 1] = (uint32_t)i; }
        OK(rs_memcpy_h2d(rec, sr.data(), 8 * n, nullptr));
        std::vector<uint32_t> zero(n, 0u);
        OK(rs_memcpy_h2d(ok, zero.data(), 4 * n, nullptr));
        OK(rs_plan_sort_records(p, rec, ok, ov, n, nullptr));
        OK(rs_plan_check(p));
        OK(rs_memcpy_d2h(gk.data(), ok, 4 * n, nullptr));
        OK(rs_memcpy_d2h(gv.data(), ov, 4 * n, nullptr));
        CHECK(verify(sk, gk, &gv, n), "sorted records -> arrays with check_order n=%zu", n);
        rs_plan_destroy(p);
    }
    for (void* q : {ik, iv, ok, ov, rec}) OK(rs_free(q));
}

// records -> arrays with a key-range hint (the group sorts' form; hybrid MSD path over the range),
// a wrong hint (one key outside: the device falls back), and the texture layout in place
static void range_and_texture(size_t n) {
    const uint32_t lo = 0x30000000u, hi = 0x37FFFFFFu;
    std::vector<uint32_t> hk(n), hr(2 * n);
    for (size_t i = 0; i < n; ++i) {
        hk[i] = lo + (mix(i + 77) & (hi - lo));
        hr[2 * i] = hk[i];
        hr[2 * i + 1] = (uint32_t)i;
    }
    void *rec, *ok, *ov;
    OK(rs_malloc(0, 8 * n, &rec));
    OK(rs_malloc(0, 4 * n, &ok));
    OK(rs_malloc(0, 4 * n, &ov));
    rs_plan_desc d{};
    d.count = n;
    d.flags = RS_FLAG_HAS_VALUES;
    rs_plan* p = nullptr;
    OK(rs_plan_create(&d, &p));
    std::vector<uint32_t> gk(n), gv(n);
    for (int wrong = 0; wrong < 2 && p; ++wrong) {
        if (wrong) { hk[n / 2] = hi + 1; hr[2 * (n / 2)] = hi + 1; }
        OK(rs_memcpy_h2d(rec, hr.data(), 8 * n, nullptr));
        OK(rs_plan_sort_records_range(p, rec, ok, ov, n, lo, hi, nullptr));
        OK(rs_plan_check(p));
        OK(rs_memcpy_d2h(gk.data(), ok, 4 * n, nullptr));
        OK(rs_memcpy_d2h(gv.data(), ov, 4 * n, nullptr));
        CHECK(verify(hk, gk, &gv, n), "sort_records_range n=%zu wrong_hint=%d", n, wrong);
    }
    if (p) rs_plan_destroy(p);
    d.flags = RS_FLAG_INTERLEAVED;
    p = nullptr;
    OK(rs_plan_create(&d, &p));
    if (p) {
        OK(rs_memcpy_h2d(rec, hr.data(), 8 * n, nullptr));
        OK(rs_plan_sort(p, rec, nullptr, nullptr));
        OK(rs_plan_check(p));
        std::vector<uint32_t> out(2 * n);
        OK(rs_memcpy_d2h(out.data(), rec, 8 * n, nullptr));
        for (size_t i = 0; i < n; ++i) { gk[i] = out[2 * i]; gv[i] = out[2 * i + 1]; }
        CHECK(verify(hk, gk, &gv, n), "texture n=%zu", n);
        rs_plan_destroy(p);
    }
    for (void* q : {rec, ok, ov}) OK(rs_free(q));
}

// the multi-GPU bucket path's entry points on one device: the sender's 16-bit table (a
// partition-usage plan), its partition fed the table's top-byte totals, and region sorts of the
// partitioned records (all 8 populated top bytes, then top bytes [2, 5) with their own table)
static void hist16_and_region(size_t n) {
    std::vector<uint32_t> hk(n), hv(n);
    for (size_t i = 0; i < n; ++i) { hk[i] = mix(i + 4242) & 0x07FFFFFFu; hv[i] = (uint32_t)i; }
    std::vector<uint32_t> ref(RS_HIST16_WORDS, 0);
    for (uint32_t k : hk) { ++ref[k >> 16]; ++ref[65536 + (k >> 24)]; }
    void *dk, *dv, *dh, *dr, *rec, *ok, *ov;
    OK(rs_malloc(0, 4 * n, &dk));
    OK(rs_malloc(0, 4 * n, &dv));
    OK(rs_malloc(0, 4ull * RS_HIST16_WORDS, &dh));
    OK(rs_malloc(0, 4ull * 65536, &dr));
    OK(rs_malloc(0, 8 * n, &rec));
    OK(rs_malloc(0, 4 * n, &ok));
    OK(rs_malloc(0, 4 * n, &ov));
    OK(rs_memcpy_h2d(dk, hk.data(), 4 * n, nullptr));
    OK(rs_memcpy_h2d(dv, hv.data(), 4 * n, nullptr));
    rs_plan_desc d{};
    d.count = n;
    d.flags = RS_FLAG_HAS_VALUES;
    d.usage = RS_USAGE_PARTITION;
    rs_plan *part = nullptr, *sp = nullptr;
    OK(rs_plan_create(&d, &part));
    d.usage = RS_USAGE_SORT;
    OK(rs_plan_create(&d, &sp));
    if (part && sp) {
        CHECK(rs_plan_sort(part, dk, dv, nullptr) == RS_ERR_INVALID_ARG, "sort on a partition plan refused");
        OK(rs_plan_hist16(part, dk, n, dh, nullptr));
        std::vector<uint32_t> got(RS_HIST16_WORDS);
        OK(rs_memcpy_d2h(got.data(), dh, 4ull * RS_HIST16_WORDS, nullptr));
        CHECK(got == ref, "rs_plan_hist16 n=%zu", n);
        OK(rs_plan_partition_records(part, dk, dv, rec, n, 24, 8, (const uint32_t*)dh + 65536, nullptr));
        OK(rs_plan_sort_region(sp, rec, ok, ov, n, dh, 0, 8, nullptr));
        OK(rs_plan_check(sp));
        std::vector<uint32_t> gk(n), gv(n);
        OK(rs_memcpy_d2h(gk.data(), ok, 4 * n, nullptr));
        OK(rs_memcpy_d2h(gv.data(), ov, 4 * n, nullptr));
        CHECK(verify(hk, gk, &gv, n), "sort_region [0, 8) n=%zu", n);
        // top bytes [2, 5): the records of those bytes, their table, zero elsewhere
        size_t a = 0, m = 0;
        for (uint32_t t = 0; t < 2; ++t) a += ref[65536 + t];
        for (uint32_t t = 2; t < 5; ++t) m += ref[65536 + t];
        std::vector<uint32_t> reg(65536, 0), sk, sv;
        for (uint32_t b = 2u << 8; b < (5u << 8); ++b) reg[b] = ref[b];
        for (size_t i = 0; i < n; ++i)
            if ((hk[i] >> 24) >= 2 && (hk[i] >> 24) < 5) { sk.push_back(hk[i]); sv.push_back((uint32_t)i); }
        OK(rs_memcpy_h2d(dr, reg.data(), 4ull * 65536, nullptr));
        OK(rs_plan_sort_region(sp, (const uint64_t*)rec + a, ok, ov, m, dr, 2, 5, nullptr));
        OK(rs_plan_check(sp));
        gk.assign(m, 0);
        gv.assign(m, 0);
        OK(rs_memcpy_d2h(gk.data(), ok, 4 * m, nullptr));
        OK(rs_memcpy_d2h(gv.data(), ov, 4 * m, nullptr));
        bool good = m == sk.size();
        for (size_t i = 0; good && i < m; ++i) good = hk[gv[i]] == gk[i] && (i == 0 || gk[i - 1] < gk[i] || (gk[i - 1] == gk[i] && gv[i - 1] < gv[i]));
        CHECK(good, "sort_region [2, 5) m=%zu", m);
    }
    if (part) rs_plan_destroy(part);
    if (sp) rs_plan_destroy(sp);
    for (void* q : {dk, dv, dh, dr, rec, ok, ov}) OK(rs_free(q));
}

static void scan_case(size_t n) {
    std::vector<uint32_t> h(n), out(n);
    for (size_t i = 0; i < n; ++i) h[i] = mix(i) & 0xFF;
    void* dd;
    OK(rs_malloc(0, 4 * n, &dd));
    OK(rs_memcpy_h2d(dd, h.data(), 4 * n, nullptr));
    rs_scan_plan* s = nullptr;
    OK(rs_scan_plan_create(0, n, 16, 16, 0, &s));
    if (s) {
        OK(rs_scan_plan_run(s, dd, nullptr));
        OK(rs_memcpy_d2h(out.data(), dd, 4 * n, nullptr));
        uint32_t acc = 0;
        bool good = true;
        for (size_t i = 0; i < n; ++i) { good &= out[i] == acc; acc += h[i]; }
        CHECK(good, "scan n=%zu", n);
        uint32_t chain[64];
        CHECK(rs_scan_plan_dispatch_chain(s, chain, 64) > 0, "dispatch chain");
        rs_scan_plan_destroy(s);
    }
    OK(rs_free(dd));
}

static void group_case(int world, uint32_t transport, bool kv, size_t n_per) {
    std::vector<int32_t> devs(world, 0);
    rs_group_desc gd{};
    gd.capacity = n_per;
    gd.flags = kv ? RS_FLAG_HAS_VALUES : 0u;
    gd.transport = transport;
    gd.rounds = 3;
    rs_group* g = nullptr;
    OK(rs_group_create(world, devs.data(), &gd, &g));
    if (!g) return;
    std::vector<void*> k(world), v(world);
    std::vector<uint64_t> cnt(world);
    std::vector<uint32_t> all, allv;
    for (int r = 0; r < world; ++r) {
        cnt[r] = n_per - (size_t)r * 1000;
        std::vector<uint32_t> hk(cnt[r]), hv(cnt[r]);
        for (size_t i = 0; i < cnt[r]; ++i) {
            hk[i] = mix(all.size() + 99) & 0xFF00FFFFu;
            hv[i] = (uint32_t)all.size();
            all.push_back(hk[i]);
        }
        OK(rs_malloc(0, 4 * cnt[r], &k[r]));
        OK(rs_malloc(0, 4 * cnt[r], &v[r]));
        OK(rs_memcpy_h2d(k[r], hk.data(), 4 * cnt[r], nullptr));
        OK(rs_memcpy_h2d(v[r], hv.data(), 4 * cnt[r], nullptr));
    }
    OK(rs_group_sort(g, k.data(), kv ? v.data() : nullptr, cnt.data(), nullptr));
    OK(rs_group_synchronize(g));
    std::vector<uint32_t> gk, gv;
    for (int r = 0; r < world; ++r) {
        void *rk, *rv;
        uint64_t m;
        OK(rs_group_result(g, r, &rk, &rv, &m));
        std::vector<uint32_t> a(m), b(m);
        if (m) OK(rs_memcpy_d2h(a.data(), rk, 4 * m, nullptr));
        if (m && kv) OK(rs_memcpy_d2h(b.data(), rv, 4 * m, nullptr));
        gk.insert(gk.end(), a.begin(), a.end());
        gv.insert(gv.end(), b.begin(), b.end());
    }
    CHECK(gk.size() == all.size(), "group sizes");
    if (gk.size() == all.size())
        CHECK(verify(all, gk, kv ? &gv : nullptr, all.size()), "group world=%d transport=%u kv=%d", world,
              transport, kv);
    rs_group_destroy(g);
    for (int r = 0; r < world; ++r) { OK(rs_free(k[r])); OK(rs_free(v[r])); }
}

static void error_paths() {
    rs_plan_desc d{};
    d.count = 10;
    d.workgroup_x = 3;
    rs_plan* p = nullptr;
    CHECK(rs_plan_create(&d, &p) == RS_ERR_NOT_POW2 && !p, "non-pow2 workgroup");
    d.workgroup_x = 16;
    d.bit_count = 6;
    CHECK(rs_plan_create(&d, &p) == RS_ERR_BIT_COUNT, "bit_count 6");
    CHECK(rs_plan_sort(nullptr, nullptr, nullptr, nullptr) == RS_ERR_INVALID_ARG, "null plan");
    rs_group_desc gd{};
    gd.top_bits = 9;
    int32_t dev = 0;
    rs_group* g = nullptr;
    CHECK(rs_group_create(1, &dev, &gd, &g) == RS_ERR_INVALID_ARG && !g, "top_bits 9");
    CHECK(strlen(rs_last_error()) > 0, "error message");
    uint64_t h[8] = {1, 2, 3, 4, 5, 6, 7, 8};
    uint32_t bounds[3], cuts[6];
    OK(rs_group_plan(2, 4, 2, h, bounds, cuts));
    CHECK(bounds[0] == 0 && bounds[2] == 4, "plan bounds");
}

int main() {
    error_paths();
    for (size_t n : {1ul, 2ul, 1000ul, 16385ul, 300000ul, 5000000ul, 13000000ul}) {
        sort_case(n, true, 0, ~0u);
        sort_case(n, false, 0, ~0u);
    }
    sort_case(17000000, false, 0, ~0u);                            // keys-only hybrid MSD path
    sort_case(20000, true, RS_FLAG_CHECK_ORDER, 0xFFu);          // duplicate-heavy + check_order
    sort_case(13000000, true, RS_FLAG_CHECK_ORDER | RS_FLAG_LOCAL_SHUFFLE, ~0u);
    copy_and_records(70000);
    copy_and_records(13000000);
    range_and_texture(13000001);
    hist16_and_region(3000000);
    hist16_and_region(20000003);
    scan_case(1000);
    scan_case(3000017);
    group_case(1, RS_TRANSPORT_RCCL, true, 200000);
    group_case(3, RS_TRANSPORT_COPY, true, 300000);
    group_case(2, RS_TRANSPORT_COPY, false, 13000000);
    group_case(4, RS_TRANSPORT_COPY, true, 13000000);             // region sorts on the hybrid path
    printf("asan driver: %d failure(s)\n", g_fail);
    return g_fail ? 1 : 0;
}
