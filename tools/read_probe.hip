// Streaming-read ceiling (diagnostic): sum 2 GiB with 16-byte loads, U loads in flight per
// lane, various grid sizes; also the same read right after a 2 GiB write of the same buffer.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int U>
__global__ __launch_bounds__(256) void rd(const uint4* __restrict__ p, uint64_t n4, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += stride) {
        uint4 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = (i + u * 256 < n4) ? p[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += q[u].x ^ q[u].y ^ q[u].z ^ q[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void wr(uint4* p, uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256)
        p[i] = make_uint4(i, i, i, i);
}

template <int U>
float t_rd(const uint4* p, uint64_t n4, uint32_t* o, int grid, bool after_write, uint4* w) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    float tot = 0;
    for (int r = 0; r < 6; ++r) {
        if (after_write) wr<<<4096, 256>>>(w, n4);
        hipEventRecord(a);
        rd<U><<<grid, 256>>>(p, n4, o);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (r) tot += ms;
    }
    return tot / 5;
}

int main() {
    const uint64_t bytes = 1ull << 31, n4 = bytes / 16;
    uint4 *p, *q; uint32_t* o;
    hipMalloc(&p, bytes); hipMalloc(&q, bytes); hipMalloc(&o, 4);
    hipMemset(p, 1, bytes); hipMemset(q, 1, bytes);
    for (int grid : {1024, 2048, 4096, 8192}) {
        float a4 = t_rd<4>(p, n4, o, grid, false, q), a8 = t_rd<8>(p, n4, o, grid, false, q);
        float w4 = t_rd<4>(p, n4, o, grid, true, p);   // read right after writing the same buffer
        float x4 = t_rd<4>(p, n4, o, grid, true, q);   // read after writing another buffer
        printf("{\"grid\": %d, \"read_U4_GBs\": %.1f, \"read_U8_GBs\": %.1f, \"read_after_write_same_GBs\": %.1f, \"read_after_write_other_GBs\": %.1f}\n",
               grid, bytes / (a4 * 1e-3) / 1e9, bytes / (a8 * 1e-3) / 1e9, bytes / (w4 * 1e-3) / 1e9, bytes / (x4 * 1e-3) / 1e9);
    }
    return 0;
}
