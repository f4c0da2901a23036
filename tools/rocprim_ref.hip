// Known-good reference on the same hardware (guide §5.4 rule 10): hipCUB/rocPRIM
// DeviceRadixSort on the BASELINE shapes.  Diagnostic only; not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -o tools/rocprim_ref tools/rocprim_ref.hip
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void fill(uint32_t* k, uint32_t* v, size_t n, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = seed * 0xD1B54A32D192ED03ull + i + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        k[i] = (uint32_t)(z ^ (z >> 31));
        if (v) v[i] = (uint32_t)i;
    }
}

int run(size_t n, bool kv) {
    uint32_t *k, *v = nullptr, *k2, *v2 = nullptr;
    CK(hipMalloc(&k, n * 4)); CK(hipMalloc(&k2, n * 4));
    if (kv) { CK(hipMalloc(&v, n * 4)); CK(hipMalloc(&v2, n * 4)); }
    size_t tmp = 0;
    if (kv) CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, k, k2, v, v2, (int)n));
    else CK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, k, k2, (int)n));
    void* t; CK(hipMalloc(&t, tmp));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e30f, sum = 0; int reps = 5;
    for (int r = 0; r < reps + 1; ++r) {
        fill<<<4096, 256>>>(k, v, n, 3 + r);
        CK(hipEventRecord(a));
        if (kv) CK(hipcub::DeviceRadixSort::SortPairs(t, tmp, k, k2, v, v2, (int)n));
        else CK(hipcub::DeviceRadixSort::SortKeys(t, tmp, k, k2, (int)n));
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (r) { best = ms < best ? ms : best; sum += ms; }
    }
    std::vector<uint32_t> h(1 << 20);
    CK(hipMemcpy(h.data(), k2, h.size() * 4, hipMemcpyDeviceToHost));
    bool ok = true; for (size_t i = 1; i < h.size(); ++i) ok &= h[i - 1] <= h[i];
    printf("{\"impl\": \"hipcub::DeviceRadixSort\", \"n\": %zu, \"kv\": %s, \"ms_best\": %.4f, \"ms_avg\": %.4f, \"gkeys_best\": %.3f, \"sorted_prefix\": %s}\n",
           n, kv ? "true" : "false", best, sum / reps, n / (best * 1e-3) / 1e9, ok ? "true" : "false");
    hipFree(k); hipFree(k2); hipFree(v); hipFree(v2); hipFree(t);
    return 0;
}

int main() {
    if (run(size_t(1) << 28, true)) return 1;
    if (run(size_t(1) << 26, false)) return 1;
    if (run(size_t(1) << 20, false)) return 1;
    if (run(size_t(1) << 20, true)) return 1;
    if (run(100000, false)) return 1;
    if (run(10000000, false)) return 1;
    if (run(size_t(1) << 24, true)) return 1;
    return 0;
}
