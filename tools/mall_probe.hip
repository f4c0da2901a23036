// Infinity Cache (MALL) probe (diagnostic): ping-pong copy A->B->A over a working set of S
// bytes (both buffers), many iterations; reports effective read+write GB/s vs S.  Also a
// read-only re-read of S bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void cp(const uint4* __restrict__ a, uint4* __restrict__ b, uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) b[i] = a[i];
}
__global__ __launch_bounds__(256) void rd(const uint4* __restrict__ a, uint64_t n4, uint32_t* o) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) {
        uint4 q = a[i]; acc += q.x ^ q.y ^ q.z ^ q.w;
    }
    if (acc == 0x1234567u) o[0] = acc;
}

int main() {
    uint4 *a, *b; uint32_t* o;
    const uint64_t maxb = 1ull << 31;
    hipMalloc(&a, maxb); hipMalloc(&b, maxb); hipMalloc(&o, 4);
    hipMemset(a, 1, maxb); hipMemset(b, 2, maxb);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (uint64_t mb : {8ull, 16ull, 32ull, 64ull, 96ull, 128ull, 192ull, 256ull, 512ull, 2048ull}) {
        const uint64_t bytes = mb << 20, n4 = bytes / 16;
        const int iters = (int)(8192 / mb) + 4;
        cp<<<4096, 256>>>(a, b, n4); cp<<<4096, 256>>>(b, a, n4);
        hipEventRecord(e0);
        for (int i = 0; i < iters; ++i) { cp<<<4096, 256>>>(a, b, n4); cp<<<4096, 256>>>(b, a, n4); }
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double cpbw = 2.0 * 2 * bytes * iters / (ms * 1e-3) / 1e9;
        rd<<<4096, 256>>>(a, n4, o);
        hipEventRecord(e0);
        for (int i = 0; i < 2 * iters; ++i) rd<<<4096, 256>>>(a, n4, o);
        hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        const double rdbw = 1.0 * bytes * 2 * iters / (ms * 1e-3) / 1e9;
        printf("{\"buffer_MiB\": %llu, \"pingpong_copy_rw_GBs\": %.1f, \"reread_GBs\": %.1f}\n",
               (unsigned long long)mb, cpbw, rdbw);
    }
    return 0;
}
