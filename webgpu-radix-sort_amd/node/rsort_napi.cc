// rsort_napi.cc — Node N-API binding of librsort (include/rsort.h).
//
// The thin FFI layer between the reference's host language (JavaScript/TypeScript, Node) and the
// gfx950 HIP kernels.  Device pointers and HIP streams cross as BigInt; plans cross as externals
// with a finalizer (the reference never frees its GPU resources).  Every failed
// call throws Error(rs_last_error()).  No compute happens here.
#define NAPI_VERSION 8
#include <node_api.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rsort.h"

namespace {

#define NAPI_CALL(env, call)                                              \
    do {                                                                  \
        if ((call) != napi_ok) {                                          \
            napi_throw_error((env), nullptr, "N-API call failed: " #call); \
            return nullptr;                                               \
        }                                                                 \
    } while (0)

napi_value throw_status(napi_env env, rs_status st, const char* what) {
    std::string msg = std::string(what) + ": " + rs_last_error();
    napi_throw_error(env, rs_status_string(st), msg.c_str());
    return nullptr;
}

#define RS_CALL(env, call, what)                               \
    do {                                                       \
        rs_status st_ = (call);                                \
        if (st_ != RS_OK) return throw_status((env), st_, what); \
    } while (0)

// A non-negative integer: BigInt (must fit u64 exactly: negative or wider BigInts are rejected),
// a Number (integral, >= 0, < 2^53), or null/undefined (0).
bool get_u64(napi_env env, napi_value v, uint64_t* out) {
    napi_valuetype t;
    if (napi_typeof(env, v, &t) != napi_ok) return false;
    if (t == napi_null || t == napi_undefined) { *out = 0; return true; }
    if (t == napi_bigint) {
        bool lossless = false;
        return napi_get_value_bigint_uint64(env, v, out, &lossless) == napi_ok && lossless;
    }
    if (t == napi_number) {
        double d = 0;
        if (napi_get_value_double(env, v, &d) != napi_ok || !(d >= 0) || d >= 9007199254740992.0 ||
            d != (double)(uint64_t)d)
            return false;
        *out = (uint64_t)d;
        return true;
    }
    return false;
}

bool get_u32_prop(napi_env env, napi_value obj, const char* key, uint32_t* out, uint32_t dflt) {
    bool has = false;
    *out = dflt;
    if (napi_has_named_property(env, obj, key, &has) != napi_ok) return false;
    if (!has) return true;
    napi_value v;
    if (napi_get_named_property(env, obj, key, &v) != napi_ok) return false;
    uint64_t x = 0;
    if (!get_u64(env, v, &x) || x > 0xFFFFFFFFull) return false;   // no silent truncation
    *out = (uint32_t)x;
    return true;
}

napi_value bigint(napi_env env, uint64_t x) {
    napi_value r;
    napi_create_bigint_uint64(env, x, &r);
    return r;
}

template <int N>
bool args(napi_env env, napi_callback_info info, napi_value (&argv)[N], size_t* argc_out = nullptr) {
    size_t argc = N;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok) return false;
    for (size_t i = argc; i < (size_t)N; ++i) napi_get_undefined(env, &argv[i]);
    if (argc_out) *argc_out = argc;
    return true;
}

void* ptr_of(napi_env env, napi_value v, bool* ok) {
    uint64_t x = 0;
    *ok = get_u64(env, v, &x);
    return (void*)(uintptr_t)x;
}

// Pointer / stream arguments: every one must convert, else TypeError (a bad argument never
// silently becomes NULL).
#define PTR_ARG(env, var, value, what)                                   \
    void* var;                                                           \
    do {                                                                 \
        bool ok_;                                                        \
        var = ptr_of((env), (value), &ok_);                              \
        if (!ok_) {                                                      \
            napi_throw_type_error((env), nullptr, what);                 \
            return nullptr;                                              \
        }                                                                \
    } while (0)

// ---- plans as externals ------------------------------------------------------------------
struct PlanBox { rs_plan* plan; };
struct ScanBox { rs_scan_plan* plan; };

void plan_finalize(napi_env, void* data, void*) {
    auto* b = static_cast<PlanBox*>(data);
    if (b->plan) rs_plan_destroy(b->plan);
    delete b;
}
void scan_finalize(napi_env, void* data, void*) {
    auto* b = static_cast<ScanBox*>(data);
    if (b->plan) rs_scan_plan_destroy(b->plan);
    delete b;
}

template <class Box>
Box* box_of(napi_env env, napi_value v) {
    void* p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, nullptr, "expected a plan handle");
        return nullptr;
    }
    return static_cast<Box*>(p);
}

// ---- functions ---------------------------------------------------------------------------
napi_value DeviceCount(napi_env env, napi_callback_info) {
    int32_t n = 0;
    RS_CALL(env, rs_device_count(&n), "deviceCount");
    napi_value r;
    napi_create_int32(env, n, &r);
    return r;
}

napi_value Version(napi_env env, napi_callback_info) {
    napi_value r;
    napi_create_uint32(env, rs_version(), &r);
    return r;
}

// malloc(device, bytes) -> BigInt
napi_value Malloc(napi_env env, napi_callback_info info) {
    napi_value a[2];
    if (!args(env, info, a)) return nullptr;
    uint64_t dev = 0, bytes = 0;
    if (!get_u64(env, a[0], &dev) || !get_u64(env, a[1], &bytes))
        return napi_throw_type_error(env, nullptr, "malloc(device, bytes)"), nullptr;
    void* p = nullptr;
    RS_CALL(env, rs_malloc((int32_t)dev, bytes, &p), "malloc");
    return bigint(env, (uint64_t)(uintptr_t)p);
}

napi_value Free(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    PTR_ARG(env, p, a[0], "free(ptr)");
    RS_CALL(env, rs_free(p), "free");
    return nullptr;
}

// h2d(ptr, typedArray|ArrayBuffer) / d2h(typedArray|ArrayBuffer, ptr): synchronous copies
bool host_span(napi_env env, napi_value v, void** data, size_t* bytes) {
    bool is_ta = false, is_ab = false;
    napi_is_typedarray(env, v, &is_ta);
    if (is_ta) {
        napi_typedarray_type t;
        size_t len = 0, off = 0;
        napi_value ab;
        if (napi_get_typedarray_info(env, v, &t, &len, data, &ab, &off) != napi_ok) return false;
        size_t el = 1;
        switch (t) {
            case napi_int16_array: case napi_uint16_array: el = 2; break;
            case napi_int32_array: case napi_uint32_array: case napi_float32_array: el = 4; break;
            case napi_float64_array: case napi_bigint64_array: case napi_biguint64_array: el = 8; break;
            default: el = 1;
        }
        *bytes = len * el;
        return true;
    }
    napi_is_arraybuffer(env, v, &is_ab);
    if (is_ab) return napi_get_arraybuffer_info(env, v, data, bytes) == napi_ok;
    return false;
}

napi_value H2D(napi_env env, napi_callback_info info) {
    napi_value a[3];
    if (!args(env, info, a)) return nullptr;
    PTR_ARG(env, dst, a[0], "h2d(ptr, typedArray, stream)");
    void* src = nullptr;
    size_t bytes = 0;
    if (!host_span(env, a[1], &src, &bytes))
        return napi_throw_type_error(env, nullptr, "h2d(ptr, typedArray)"), nullptr;
    PTR_ARG(env, stream, a[2], "h2d: bad stream");
    RS_CALL(env, rs_memcpy_h2d(dst, src, bytes, stream), "h2d");
    RS_CALL(env, rs_stream_synchronize(stream), "h2d");
    return nullptr;
}

napi_value D2H(napi_env env, napi_callback_info info) {
    napi_value a[3];
    if (!args(env, info, a)) return nullptr;
    void* dst = nullptr;
    size_t bytes = 0;
    if (!host_span(env, a[0], &dst, &bytes))
        return napi_throw_type_error(env, nullptr, "d2h(typedArray, ptr)"), nullptr;
    PTR_ARG(env, src, a[1], "d2h(typedArray, ptr, stream): bad ptr");
    PTR_ARG(env, stream, a[2], "d2h: bad stream");
    RS_CALL(env, rs_memcpy_d2h(dst, src, bytes, stream), "d2h");
    return nullptr;
}

napi_value D2D(napi_env env, napi_callback_info info) {
    napi_value a[4];
    if (!args(env, info, a)) return nullptr;
    PTR_ARG(env, dst, a[0], "d2d(dst, src, bytes, stream): bad dst");
    PTR_ARG(env, src, a[1], "d2d(dst, src, bytes, stream): bad src");
    uint64_t bytes = 0;
    if (!get_u64(env, a[2], &bytes)) return napi_throw_type_error(env, nullptr, "d2d: bad bytes"), nullptr;
    PTR_ARG(env, stream, a[3], "d2d: bad stream");
    RS_CALL(env, rs_memcpy_d2d(dst, src, bytes, stream), "d2d");
    return nullptr;
}

napi_value StreamCreate(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    uint64_t dev = 0;
    if (!get_u64(env, a[0], &dev) || dev > 0x7FFFFFFF)
        return napi_throw_type_error(env, nullptr, "streamCreate(device)"), nullptr;
    void* s = nullptr;
    RS_CALL(env, rs_stream_create((int32_t)dev, &s), "streamCreate");
    return bigint(env, (uint64_t)(uintptr_t)s);
}

napi_value StreamDestroy(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    PTR_ARG(env, s, a[0], "streamDestroy(stream)");
    RS_CALL(env, rs_stream_destroy(s), "streamDestroy");
    return nullptr;
}

napi_value StreamSynchronize(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    PTR_ARG(env, s, a[0], "streamSynchronize(stream)");
    RS_CALL(env, rs_stream_synchronize(s), "streamSynchronize");
    return nullptr;
}

// Timestamp events: eventCreate() -> bigint, eventRecord(ev, stream), eventElapsed(a, b) -> ms,
// eventDestroy(ev).  Back the WebGPU-shaped timestamp QuerySet of index.js.
napi_value EventCreate(napi_env env, napi_callback_info info) {
    (void)info;
    void* e = nullptr;
    RS_CALL(env, rs_event_create(&e), "eventCreate");
    return bigint(env, (uint64_t)(uintptr_t)e);
}

napi_value EventRecord(napi_env env, napi_callback_info info) {
    napi_value a[2];
    if (!args(env, info, a)) return nullptr;
    PTR_ARG(env, e, a[0], "eventRecord(event, stream): bad event");
    PTR_ARG(env, s, a[1], "eventRecord: bad stream");
    RS_CALL(env, rs_event_record(e, s), "eventRecord");
    return nullptr;
}

napi_value EventElapsed(napi_env env, napi_callback_info info) {
    napi_value a[2];
    if (!args(env, info, a)) return nullptr;
    PTR_ARG(env, e0, a[0], "eventElapsed(a, b): bad event");
    PTR_ARG(env, e1, a[1], "eventElapsed(a, b): bad event");
    float ms = 0.f;
    RS_CALL(env, rs_event_elapsed_ms(e0, e1, &ms), "eventElapsed");
    napi_value r;
    napi_create_double(env, (double)ms, &r);
    return r;
}

napi_value EventDestroy(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    PTR_ARG(env, e, a[0], "eventDestroy(event)");
    RS_CALL(env, rs_event_destroy(e), "eventDestroy");
    return nullptr;
}

// planCreate({device, count, bitCount, workgroupX, workgroupY, flags, radixBits}) -> external
napi_value PlanCreate(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    rs_plan_desc d;
    memset(&d, 0, sizeof(d));
    uint32_t dev = 0, countlo = 0;
    (void)countlo;
    napi_value cnt;
    bool has = false;
    napi_has_named_property(env, a[0], "count", &has);
    uint64_t count = 0;
    if (has) {
        napi_get_named_property(env, a[0], "count", &cnt);
        if (!get_u64(env, cnt, &count)) return napi_throw_type_error(env, nullptr, "count"), nullptr;
    }
    if (!get_u32_prop(env, a[0], "device", &dev, 0) ||
        !get_u32_prop(env, a[0], "bitCount", &d.bit_count, 32) ||
        !get_u32_prop(env, a[0], "workgroupX", &d.workgroup_x, 16) ||
        !get_u32_prop(env, a[0], "workgroupY", &d.workgroup_y, 16) ||
        !get_u32_prop(env, a[0], "flags", &d.flags, 0) ||
        !get_u32_prop(env, a[0], "radixBits", &d.radix_bits, 0))
        return napi_throw_type_error(env, nullptr, "planCreate: bad option"), nullptr;
    d.device = (int32_t)dev;
    d.count = count;
    rs_plan* p = nullptr;
    RS_CALL(env, rs_plan_create(&d, &p), "RadixSortKernel");
    napi_value ext;
    auto* box = new PlanBox{p};
    if (napi_create_external(env, box, plan_finalize, nullptr, &ext) != napi_ok) {
        plan_finalize(env, box, nullptr);
        return napi_throw_error(env, nullptr, "external"), nullptr;
    }
    return ext;
}

// planSort(plan, keysPtr, valuesPtr|null, stream|null [, n])
napi_value PlanSort(napi_env env, napi_callback_info info) {
    napi_value a[5];
    size_t argc = 0;
    if (!args(env, info, a, &argc)) return nullptr;
    PlanBox* b = box_of<PlanBox>(env, a[0]);
    if (!b) return nullptr;
    if (!b->plan) return napi_throw_error(env, nullptr, "plan destroyed"), nullptr;
    PTR_ARG(env, k, a[1], "planSort(plan, keys, values, stream[, n]): bad keys");
    PTR_ARG(env, v, a[2], "planSort: bad values");
    PTR_ARG(env, s, a[3], "planSort: bad stream");
    if (argc >= 5) {
        uint64_t n = 0;
        if (!get_u64(env, a[4], &n)) return napi_throw_type_error(env, nullptr, "n"), nullptr;
        RS_CALL(env, rs_plan_sort_n(b->plan, k, v, n, s), "dispatch");
    } else {
        RS_CALL(env, rs_plan_sort(b->plan, k, v, s), "dispatch");
    }
    return nullptr;
}

napi_value PlanDestroy(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    PlanBox* b = box_of<PlanBox>(env, a[0]);
    if (!b) return nullptr;
    if (b->plan) rs_plan_destroy(b->plan);
    b->plan = nullptr;
    return nullptr;
}

napi_value PlanInfo(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    PlanBox* b = box_of<PlanBox>(env, a[0]);
    if (!b || !b->plan) return napi_throw_error(env, nullptr, "plan destroyed"), nullptr;
    rs_plan_info inf;
    RS_CALL(env, rs_plan_info_get(b->plan, &inf), "info");
    napi_value o, x, arr;
    napi_create_object(env, &o);
    napi_create_uint32(env, inf.passes, &x); napi_set_named_property(env, o, "passes", x);
    napi_create_uint32(env, inf.tile_keys, &x); napi_set_named_property(env, o, "tileKeys", x);
    napi_create_uint32(env, inf.grid_blocks, &x); napi_set_named_property(env, o, "gridBlocks", x);
    napi_create_double(env, (double)inf.workspace_bytes, &x); napi_set_named_property(env, o, "workspaceBytes", x);
    napi_create_string_utf8(env, inf.rank_mode == 1 ? "ballot" : "lds_atomic", NAPI_AUTO_LENGTH, &x);
    napi_set_named_property(env, o, "rankMode", x);
    napi_create_int32(env, inf.lane_order_selftest, &x); napi_set_named_property(env, o, "laneOrderSelftest", x);
    napi_create_array_with_length(env, inf.passes, &arr);
    for (uint32_t i = 0; i < inf.passes && i < 16; ++i) {
        napi_create_uint32(env, inf.digit_bits[i], &x);
        napi_set_element(env, arr, i, x);
    }
    napi_set_named_property(env, o, "digitBits", arr);
    return o;
}

// scanPlanCreate(device, count, wx, wy, flags) -> external
napi_value ScanPlanCreate(napi_env env, napi_callback_info info) {
    napi_value a[5];
    if (!args(env, info, a)) return nullptr;
    uint64_t dev = 0, count = 0, wx = 16, wy = 16, flags = 0;
    if (!get_u64(env, a[0], &dev) || !get_u64(env, a[1], &count) || !get_u64(env, a[2], &wx) ||
        !get_u64(env, a[3], &wy) || !get_u64(env, a[4], &flags))
        return napi_throw_type_error(env, nullptr, "scanPlanCreate(device, count, wx, wy, flags)"), nullptr;
    rs_scan_plan* p = nullptr;
    RS_CALL(env, rs_scan_plan_create((int32_t)dev, count, (uint32_t)wx, (uint32_t)wy, (uint32_t)flags, &p),
            "PrefixSumKernel");
    napi_value ext;
    auto* box = new ScanBox{p};
    if (napi_create_external(env, box, scan_finalize, nullptr, &ext) != napi_ok) {
        scan_finalize(env, box, nullptr);
        return napi_throw_error(env, nullptr, "external"), nullptr;
    }
    return ext;
}

napi_value ScanPlanRun(napi_env env, napi_callback_info info) {
    napi_value a[3];
    if (!args(env, info, a)) return nullptr;
    ScanBox* b = box_of<ScanBox>(env, a[0]);
    if (!b || !b->plan) return napi_throw_error(env, nullptr, "plan destroyed"), nullptr;
    PTR_ARG(env, d, a[1], "scanPlanRun(plan, data, stream): bad data");
    PTR_ARG(env, s, a[2], "scanPlanRun: bad stream");
    RS_CALL(env, rs_scan_plan_run(b->plan, d, s), "dispatch");
    return nullptr;
}

// scanPlanRunIndirect(plan, data, dispatchSizeBuffer, offsetBytes, stream)
napi_value ScanPlanRunIndirect(napi_env env, napi_callback_info info) {
    napi_value a[5];
    if (!args(env, info, a)) return nullptr;
    ScanBox* b = box_of<ScanBox>(env, a[0]);
    if (!b || !b->plan) return napi_throw_error(env, nullptr, "plan destroyed"), nullptr;
    PTR_ARG(env, d, a[1], "scanPlanRunIndirect: bad data");
    PTR_ARG(env, buf, a[2], "scanPlanRunIndirect: bad dispatch size buffer");
    uint64_t off = 0;
    if (!get_u64(env, a[3], &off)) return napi_throw_type_error(env, nullptr, "scanPlanRunIndirect: bad offset"), nullptr;
    PTR_ARG(env, s, a[4], "scanPlanRunIndirect: bad stream");
    RS_CALL(env, rs_scan_plan_run_indirect(b->plan, d, buf, off, s), "dispatch");
    return nullptr;
}

// scanPlanDispatchChain(plan) -> number[] (PrefixSumKernel.getDispatchChain)
napi_value ScanPlanDispatchChain(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    ScanBox* b = box_of<ScanBox>(env, a[0]);
    if (!b || !b->plan) return napi_throw_error(env, nullptr, "plan destroyed"), nullptr;
    const uint32_t n = rs_scan_plan_dispatch_chain(b->plan, nullptr, 0);
    std::string buf(4 * (size_t)n, '\0');
    uint32_t* w = reinterpret_cast<uint32_t*>(&buf[0]);
    rs_scan_plan_dispatch_chain(b->plan, w, n);
    napi_value arr, x;
    napi_create_array_with_length(env, n, &arr);
    for (uint32_t i = 0; i < n; ++i) {
        napi_create_uint32(env, w[i], &x);
        napi_set_element(env, arr, i, x);
    }
    return arr;
}

// planCheck(plan): waits for the plan's last sort; throws on a device-side failure since the
// last check (rs_plan_check)
napi_value PlanCheck(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    PlanBox* b = box_of<PlanBox>(env, a[0]);
    if (!b || !b->plan) return napi_throw_error(env, nullptr, "plan destroyed"), nullptr;
    RS_CALL(env, rs_plan_check(b->plan), "check");
    return nullptr;
}

// planLastPath(plan): the path the plan's last sort took ("none", "lsd", "hybrid",
// "hybrid_fallback", "in_order", "presorted"; rs_plan_last_path, waits for it)
napi_value PlanLastPath(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    PlanBox* b = box_of<PlanBox>(env, a[0]);
    if (!b || !b->plan) return napi_throw_error(env, nullptr, "plan destroyed"), nullptr;
    uint32_t path = 0;
    RS_CALL(env, rs_plan_last_path(b->plan, &path), "lastPath");
    static const char* const names[] = {"none", "lsd", "hybrid", "hybrid_fallback", "in_order", "presorted"};
    napi_value v;
    napi_create_string_utf8(env, path < sizeof(names) / sizeof(names[0]) ? names[path] : "unknown", NAPI_AUTO_LENGTH, &v);
    return v;
}

// planLastSplit(plan): 0, 2 or 3 - how deep the last hybrid sort split over-full 16-bit buckets
// (rs_plan_last_split)
napi_value PlanLastSplit(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    PlanBox* b = box_of<PlanBox>(env, a[0]);
    if (!b || !b->plan) return napi_throw_error(env, nullptr, "plan destroyed"), nullptr;
    uint32_t levels = 0;
    RS_CALL(env, rs_plan_last_split(b->plan, &levels), "lastSplit");
    napi_value v;
    napi_create_uint32(env, levels, &v);
    return v;
}

napi_value ScanPlanCheck(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    void* p = nullptr;
    if (napi_get_value_external(env, a[0], &p) != napi_ok || !p)
        return napi_throw_type_error(env, nullptr, "expected a scan plan handle"), nullptr;
    auto* b = static_cast<ScanBox*>(p);
    if (b->plan) RS_CALL(env, rs_scan_plan_check(b->plan), "PrefixSumKernel.check");
    return nullptr;
}

napi_value ScanPlanDestroy(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    ScanBox* b = box_of<ScanBox>(env, a[0]);
    if (!b) return nullptr;
    if (b->plan) rs_scan_plan_destroy(b->plan);
    b->plan = nullptr;
    return nullptr;
}

// ---- multi-GPU group (rs_group_*) ----------------------------------------------------------
struct GroupBox { rs_group* group; };

void group_finalize(napi_env, void* data, void*) {
    auto* b = static_cast<GroupBox*>(data);
    if (b->group) rs_group_destroy(b->group);
    delete b;
}

// Array of pointers / counts (BigInt or Number each); null/undefined -> empty (ok stays true).
bool u64_array(napi_env env, napi_value v, std::vector<uint64_t>* out, bool* present) {
    napi_valuetype t;
    out->clear();
    *present = false;
    if (napi_typeof(env, v, &t) != napi_ok) return false;
    if (t == napi_null || t == napi_undefined) return true;
    bool isarr = false;
    if (napi_is_array(env, v, &isarr) != napi_ok || !isarr) return false;
    uint32_t len = 0;
    napi_get_array_length(env, v, &len);
    for (uint32_t i = 0; i < len; ++i) {
        napi_value e;
        uint64_t x = 0;
        if (napi_get_element(env, v, i, &e) != napi_ok || !get_u64(env, e, &x)) return false;
        out->push_back(x);
    }
    *present = true;
    return true;
}

// groupCreate([devices], {capacity, hasValues, transport: 'rccl'|'copy', topBits, rounds})
napi_value GroupCreate(napi_env env, napi_callback_info info) {
    napi_value a[2];
    if (!args(env, info, a)) return nullptr;
    std::vector<uint64_t> devs;
    bool present = false;
    if (!u64_array(env, a[0], &devs, &present) || devs.empty())
        return napi_throw_type_error(env, nullptr, "groupCreate: devices must be a non-empty array"), nullptr;
    std::vector<int32_t> d32;
    for (uint64_t d : devs) {
        if (d > 0x7FFFFFFF) return napi_throw_type_error(env, nullptr, "groupCreate: bad device"), nullptr;
        d32.push_back((int32_t)d);
    }
    rs_group_desc d;
    memset(&d, 0, sizeof(d));
    uint32_t has_values = 1;
    bool has = false;
    napi_has_named_property(env, a[1], "capacity", &has);
    if (has) {
        napi_value c;
        napi_get_named_property(env, a[1], "capacity", &c);
        if (!get_u64(env, c, &d.capacity)) return napi_throw_type_error(env, nullptr, "capacity"), nullptr;
    }
    napi_has_named_property(env, a[1], "hasValues", &has);
    if (has) {
        napi_value hv;
        bool bv = true;
        napi_get_named_property(env, a[1], "hasValues", &hv);
        if (napi_get_value_bool(env, hv, &bv) != napi_ok)
            return napi_throw_type_error(env, nullptr, "hasValues must be a boolean"), nullptr;
        has_values = bv ? 1u : 0u;
    }
    napi_has_named_property(env, a[1], "transport", &has);
    if (has) {
        napi_value tv;
        char buf[16] = {0};
        size_t len = 0;
        napi_get_named_property(env, a[1], "transport", &tv);
        if (napi_get_value_string_utf8(env, tv, buf, sizeof(buf), &len) != napi_ok)
            return napi_throw_type_error(env, nullptr, "transport must be 'rccl' or 'copy'"), nullptr;
        if (strcmp(buf, "rccl") == 0) d.transport = RS_TRANSPORT_RCCL;
        else if (strcmp(buf, "copy") == 0) d.transport = RS_TRANSPORT_COPY;
        else return napi_throw_type_error(env, nullptr, "transport must be 'rccl' or 'copy'"), nullptr;
    }
    if (!get_u32_prop(env, a[1], "topBits", &d.top_bits, 0) ||
        !get_u32_prop(env, a[1], "rounds", &d.rounds, 0))
        return napi_throw_type_error(env, nullptr, "groupCreate: bad option"), nullptr;
    d.flags = has_values ? RS_FLAG_HAS_VALUES : 0u;
    rs_group* g = nullptr;
    RS_CALL(env, rs_group_create((int32_t)d32.size(), d32.data(), &d, &g), "RadixSortGroup");
    napi_value ext;
    auto* box = new GroupBox{g};
    if (napi_create_external(env, box, group_finalize, nullptr, &ext) != napi_ok) {
        group_finalize(env, box, nullptr);
        return napi_throw_error(env, nullptr, "external"), nullptr;
    }
    return ext;
}

GroupBox* group_of(napi_env env, napi_value v) {
    void* p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, nullptr, "expected a group handle");
        return nullptr;
    }
    auto* b = static_cast<GroupBox*>(p);
    if (!b->group) {
        napi_throw_error(env, nullptr, "group destroyed");
        return nullptr;
    }
    return b;
}

// groupSort(group, [keysPtr], [valuesPtr]|null, [count], [stream]|null)
napi_value GroupSort(napi_env env, napi_callback_info info) {
    napi_value a[5];
    if (!args(env, info, a)) return nullptr;
    GroupBox* b = group_of(env, a[0]);
    if (!b) return nullptr;
    std::vector<uint64_t> k, v, n, s;
    bool hk, hv, hn, hs;
    if (!u64_array(env, a[1], &k, &hk) || !u64_array(env, a[2], &v, &hv) ||
        !u64_array(env, a[3], &n, &hn) || !u64_array(env, a[4], &s, &hs) || !hk || !hn ||
        n.size() != k.size() || (hv && v.size() != k.size()) || (hs && s.size() != k.size()))
        return napi_throw_type_error(env, nullptr, "groupSort(group, keys[], values[]|null, counts[], streams[]|null): bad arrays"), nullptr;
    std::vector<void*> kp(k.size()), vp(v.size()), sp(s.size());
    for (size_t i = 0; i < k.size(); ++i) kp[i] = (void*)(uintptr_t)k[i];
    for (size_t i = 0; i < v.size(); ++i) vp[i] = (void*)(uintptr_t)v[i];
    for (size_t i = 0; i < s.size(); ++i) sp[i] = (void*)(uintptr_t)s[i];
    RS_CALL(env, rs_group_sort(b->group, kp.data(), hv ? vp.data() : nullptr, n.data(),
                               hs ? sp.data() : nullptr), "RadixSortGroup.sort");
    return nullptr;
}

// groupResult(group, rank) -> {keys: BigInt, values: BigInt|null, count: Number}
napi_value GroupResult(napi_env env, napi_callback_info info) {
    napi_value a[2];
    if (!args(env, info, a)) return nullptr;
    GroupBox* b = group_of(env, a[0]);
    if (!b) return nullptr;
    uint64_t rank = 0;
    if (!get_u64(env, a[1], &rank) || rank > 0x7FFFFFFF)
        return napi_throw_type_error(env, nullptr, "groupResult: bad rank"), nullptr;
    void* kp = nullptr;
    void* vp = nullptr;
    uint64_t n = 0;
    RS_CALL(env, rs_group_result(b->group, (int32_t)rank, &kp, &vp, &n), "groupResult");
    napi_value o, x;
    napi_create_object(env, &o);
    napi_set_named_property(env, o, "keys", bigint(env, (uint64_t)(uintptr_t)kp));
    if (vp) x = bigint(env, (uint64_t)(uintptr_t)vp);
    else napi_get_null(env, &x);
    napi_set_named_property(env, o, "values", x);
    napi_create_double(env, (double)n, &x);
    napi_set_named_property(env, o, "count", x);
    return o;
}

napi_value GroupSynchronize(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    GroupBox* b = group_of(env, a[0]);
    if (!b) return nullptr;
    RS_CALL(env, rs_group_synchronize(b->group), "RadixSortGroup.synchronize");
    return nullptr;
}

napi_value GroupSetProfiling(napi_env env, napi_callback_info info) {
    napi_value a[2];
    if (!args(env, info, a)) return nullptr;
    GroupBox* b = group_of(env, a[0]);
    if (!b) return nullptr;
    bool on = false;
    napi_get_value_bool(env, a[1], &on);
    RS_CALL(env, rs_group_set_profiling(b->group, on ? 1 : 0), "RadixSortGroup.setProfiling");
    return nullptr;
}

// rs_group_times_get -> {rounds, hist16Ms, partitionMs, roundDoneMs[], regionSortedMs[], doneMs,
// bytesSent, bytesRecv}
napi_value GroupTimes(napi_env env, napi_callback_info info) {
    napi_value a[2];
    if (!args(env, info, a)) return nullptr;
    GroupBox* b = group_of(env, a[0]);
    if (!b) return nullptr;
    uint64_t rank = 0;
    if (!get_u64(env, a[1], &rank) || rank > 0x7FFFFFFF)
        return napi_throw_type_error(env, nullptr, "groupTimes: bad rank"), nullptr;
    rs_group_times t;
    RS_CALL(env, rs_group_times_get(b->group, (int32_t)rank, &t), "RadixSortGroup.times");
    napi_value o, x, arr;
    napi_create_object(env, &o);
    auto num = [&](const char* k, double v) { napi_create_double(env, v, &x); napi_set_named_property(env, o, k, x); };
    num("rounds", t.rounds);
    num("hist16Ms", t.hist16_ms);
    num("partitionMs", t.partition_ms);
    num("doneMs", t.done_ms);
    num("bytesSent", (double)t.bytes_sent);
    num("bytesRecv", (double)t.bytes_recv);
    for (int which = 0; which < 2; ++which) {
        napi_create_array_with_length(env, t.rounds, &arr);
        for (uint32_t j = 0; j < t.rounds; ++j) {
            napi_create_double(env, which ? t.region_sorted_ms[j] : t.round_done_ms[j], &x);
            napi_set_element(env, arr, j, x);
        }
        napi_set_named_property(env, o, which ? "regionSortedMs" : "roundDoneMs", arr);
    }
    return o;
}

napi_value GroupDestroy(napi_env env, napi_callback_info info) {
    napi_value a[1];
    if (!args(env, info, a)) return nullptr;
    void* p = nullptr;
    if (napi_get_value_external(env, a[0], &p) != napi_ok || !p)
        return napi_throw_type_error(env, nullptr, "expected a group handle"), nullptr;
    auto* b = static_cast<GroupBox*>(p);
    if (b->group) rs_group_destroy(b->group);
    b->group = nullptr;
    return nullptr;
}

napi_value Define(napi_env env, napi_value exports, const char* name, napi_callback cb) {
    napi_value fn;
    napi_create_function(env, name, NAPI_AUTO_LENGTH, cb, nullptr, &fn);
    napi_set_named_property(env, exports, name, fn);
    return exports;
}

napi_value Init(napi_env env, napi_value exports) {
    Define(env, exports, "version", Version);
    Define(env, exports, "deviceCount", DeviceCount);
    Define(env, exports, "malloc", Malloc);
    Define(env, exports, "free", Free);
    Define(env, exports, "h2d", H2D);
    Define(env, exports, "d2h", D2H);
    Define(env, exports, "d2d", D2D);
    Define(env, exports, "streamCreate", StreamCreate);
    Define(env, exports, "streamDestroy", StreamDestroy);
    Define(env, exports, "streamSynchronize", StreamSynchronize);
    Define(env, exports, "eventCreate", EventCreate);
    Define(env, exports, "eventRecord", EventRecord);
    Define(env, exports, "eventElapsed", EventElapsed);
    Define(env, exports, "eventDestroy", EventDestroy);
    Define(env, exports, "planCreate", PlanCreate);
    Define(env, exports, "planSort", PlanSort);
    Define(env, exports, "planDestroy", PlanDestroy);
    Define(env, exports, "planInfo", PlanInfo);
    Define(env, exports, "scanPlanCreate", ScanPlanCreate);
    Define(env, exports, "scanPlanRun", ScanPlanRun);
    Define(env, exports, "scanPlanRunIndirect", ScanPlanRunIndirect);
    Define(env, exports, "scanPlanDispatchChain", ScanPlanDispatchChain);
    Define(env, exports, "planCheck", PlanCheck);
    Define(env, exports, "planLastPath", PlanLastPath);
    Define(env, exports, "planLastSplit", PlanLastSplit);
    Define(env, exports, "scanPlanDestroy", ScanPlanDestroy);
    Define(env, exports, "groupCreate", GroupCreate);
    Define(env, exports, "groupSort", GroupSort);
    Define(env, exports, "groupResult", GroupResult);
    Define(env, exports, "groupSynchronize", GroupSynchronize);
    Define(env, exports, "groupDestroy", GroupDestroy);
    Define(env, exports, "groupSetProfiling", GroupSetProfiling);
    Define(env, exports, "groupTimes", GroupTimes);
    Define(env, exports, "scanPlanCheck", ScanPlanCheck);
    napi_value v;
    napi_create_uint32(env, RS_FLAG_HAS_VALUES, &v); napi_set_named_property(env, exports, "FLAG_HAS_VALUES", v);
    napi_create_uint32(env, RS_FLAG_CHECK_ORDER, &v); napi_set_named_property(env, exports, "FLAG_CHECK_ORDER", v);
    napi_create_uint32(env, RS_FLAG_LOCAL_SHUFFLE, &v); napi_set_named_property(env, exports, "FLAG_LOCAL_SHUFFLE", v);
    napi_create_uint32(env, RS_FLAG_AVOID_BANK_CONFLICTS, &v); napi_set_named_property(env, exports, "FLAG_AVOID_BANK_CONFLICTS", v);
    napi_create_uint32(env, RS_FLAG_INTERLEAVED, &v); napi_set_named_property(env, exports, "FLAG_INTERLEAVED", v);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
