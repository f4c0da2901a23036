// Round 6 diagnostic (not product code): what bounds the 16-bit bucket histogram read (k_hist16_in)?
// 2^28 uniform u32 keys, one 1024-thread workgroup per CU over a contiguous chunk, 65536 buckets
// (key >> 16) counted in LDS, one row of counts written per workgroup.  Variants (timing; only the
// product-like ones count correctly, which is checked against a host histogram of a 2^20 prefix):
//   read     : the loads only (keys summed)
//   ret16    : returning ds_add on 16-bit halves (the product's atomic; its crossing check elided)
//   noret16  : non-returning ds_add on 16-bit halves (no overflow handling: wrong past 65535 per half)
//   half32   : two workgroups per chunk, each counting the keys of one half of the buckets in 32768
//              32-bit counters (non-returning, never overflows): the chunk is read twice
//   fold16   : non-returning ds_add on 16-bit halves, and every 65535 keys per workgroup the halves
//              are folded into per-thread 32-bit registers (correct for any input)
//   hipcc -O3 --offload-arch=gfx950 -o tools/hist_probe tools/hist_probe.hip && tools/hist_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint32_t B = 1024, W = 32768, FLY = 6;

__global__ void fill(uint32_t* k, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x1234567ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        k[i] = (uint32_t)(z ^ (z >> 31));
    }
}

template <int MODE>
__global__ __launch_bounds__(1024) void hist(const uint32_t* __restrict__ keys, uint64_t n, uint32_t* __restrict__ rows,
                                             uint32_t* sink) {
    __shared__ uint32_t h[W];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < W; i += B) h[i] = 0u;
    __syncthreads();
    const uint32_t parts = MODE == 3 ? 2u : 1u;
    const uint32_t unit = blockIdx.x / parts, half = blockIdx.x % parts;
    const uint32_t units = gridDim.x / parts;
    const uint64_t chunk = ((n + units - 1) / units + 3) & ~3ull;
    const uint64_t lo = unit * chunk, hi = lo + chunk < n ? lo + chunk : n;
    const uint64_t nv = (hi - lo) / 4;
    const uint4* v4 = reinterpret_cast<const uint4*>(keys + lo);
    uint32_t acc = 0;
    uint32_t fold[64];
    if (MODE == 4)
#pragma unroll
        for (int i = 0; i < 64; ++i) fold[i] = 0;
    uint32_t since = 0;
    auto add = [&](uint32_t k) {
        const uint32_t b = k >> 16;
        if (MODE == 1) acc ^= atomicAdd(&h[b >> 1], 1u << ((b & 1u) << 4));
        else if (MODE == 2 || MODE == 4) __hip_atomic_fetch_add(&h[b >> 1], 1u << ((b & 1u) << 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else if (MODE == 3) { if ((b >> 15) == half) __hip_atomic_fetch_add(&h[b & 32767u], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
        else acc += k;
    };
    for (uint64_t g = 0; g < nv; g += (uint64_t)FLY * B) {
        uint4 q[FLY];
#pragma unroll
        for (uint32_t u = 0; u < FLY; ++u) {
            const uint64_t i = g + u * B + tid;
            q[u] = v4[i < nv ? i : nv - 1];
        }
#pragma unroll
        for (uint32_t u = 0; u < FLY; ++u) {
            if (g + u * B + tid < nv) { add(q[u].x); add(q[u].y); add(q[u].z); add(q[u].w); }
        }
        if (MODE == 4) {
            since += FLY * B * 4;
            if (since + FLY * B * 4 > 65535u) {   // (uniform) fold before any half can wrap
                __syncthreads();
#pragma unroll
                for (int i = 0; i < 32; ++i) {
                    const uint32_t x = h[tid * 32 + i];
                    fold[2 * i] += x & 0xFFFFu;
                    fold[2 * i + 1] += x >> 16;
                    h[tid * 32 + i] = 0u;
                }
                __syncthreads();
                since = 0;
            }
        }
    }
    __syncthreads();
    if (MODE == 0) { if (acc == 0x12345u) sink[0] = acc; return; }
    if (MODE == 1 && acc == 0xFFFFFFFFu) sink[1] = acc;
    uint32_t* row = rows + (size_t)unit * 65536u;
    if (MODE == 3) {
        for (uint32_t i = tid; i < W; i += B) row[half * 32768u + i] = h[i];
    } else if (MODE == 4) {
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const uint32_t x = h[tid * 32 + i];
            row[2 * (tid * 32 + i)] = fold[2 * i] + (x & 0xFFFFu);
            row[2 * (tid * 32 + i) + 1] = fold[2 * i + 1] + (x >> 16);
        }
    } else {
        for (uint32_t i = tid; i < W; i += B) { const uint32_t x = h[i]; row[2 * i] = x & 0xFFFFu; row[2 * i + 1] = x >> 16; }
    }
}

int main() {
    const uint64_t n = 1ull << 28;
    int cus = 256;
    { hipDeviceProp_t prop; if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount; }
    uint32_t *k = nullptr, *rows = nullptr, *sink = nullptr;
    CK(hipMalloc(&k, 4 * n));
    CK(hipMalloc(&rows, 4ull * 65536 * cus));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, k, n);
    CK(hipDeviceSynchronize());
    // reference: the total over all rows of a correct variant must equal a host histogram
    std::vector<uint32_t> hk(n);
    CK(hipMemcpy(hk.data(), k, 4 * n, hipMemcpyDeviceToHost));
    std::vector<uint32_t> ref(65536, 0);
    for (uint64_t i = 0; i < n; ++i) ref[hk[i] >> 16]++;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"read", "ret16", "noret16", "half32", "fold16"};
    for (int round = 0; round < 2; ++round)
    for (int m = 0; m < 5; ++m) {
        const int grid = m == 3 ? 2 * cus : cus;
        float sum = 0.f;
        const int reps = 20;
        for (int r = -3; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            switch (m) {
                case 0: hipLaunchKernelGGL(hist<0>, dim3(grid), dim3(B), 0, 0, k, n, rows, sink); break;
                case 1: hipLaunchKernelGGL(hist<1>, dim3(grid), dim3(B), 0, 0, k, n, rows, sink); break;
                case 2: hipLaunchKernelGGL(hist<2>, dim3(grid), dim3(B), 0, 0, k, n, rows, sink); break;
                case 3: hipLaunchKernelGGL(hist<3>, dim3(grid), dim3(B), 0, 0, k, n, rows, sink); break;
                case 4: hipLaunchKernelGGL(hist<4>, dim3(grid), dim3(B), 0, 0, k, n, rows, sink); break;
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) sum += ms;
        }
        int ok = -1;
        if (m == 3 || m == 4) {   // exact variants: the rows must add up to the host histogram
            std::vector<uint32_t> hr(65536ull * cus);
            CK(hipMemcpy(hr.data(), rows, 4ull * 65536 * cus, hipMemcpyDeviceToHost));
            ok = 1;
            for (uint32_t b = 0; b < 65536 && ok; ++b) {
                uint64_t s = 0;
                for (int r = 0; r < cus; ++r) s += hr[(size_t)r * 65536 + b];
                if (s != ref[b]) ok = 0;
            }
        }
        printf("{\"probe\": \"hist_probe\", \"round\": %d, \"variant\": \"%s\", \"avg_ms\": %.4f, \"read_GBs\": %.1f, \"exact\": %d}\n",
               round, names[m], sum / reps, 4.0 * n / (sum / reps * 1e-3) / 1e9, ok);
        fflush(stdout);
    }
    return 0;
}
