// Infinity Cache (MALL) probe (diagnostic).
//  1. ping-pong copy A->B->A over a working set of S bytes (both buffers), many iterations;
//     effective read+write GB/s vs S; and a read-only re-read of S bytes.
//  2. grouped pipeline: a 2 GiB input is processed in groups of G bytes; per group
//     in[g] -> S1 -> S2 -> S1 -> out[g] (4 copies, the middle two on scratch buffers reused by
//     every group).  This is the byte pattern of an MSD split followed by a three-pass LSD per
//     bucket group with the group's ping-pong buffers resident in the Infinity Cache.  Reported
//     against the same 4 copies done over the whole 2 GiB (every pass through HBM).
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
    uint4 *a, *b, *in, *out; uint32_t* o;
    const uint64_t maxb = 1ull << 31;
    hipMalloc(&a, maxb); hipMalloc(&b, maxb); hipMalloc(&o, 4);
    hipMalloc(&in, maxb); hipMalloc(&out, maxb);
    hipMemset(a, 1, maxb); hipMemset(b, 2, maxb); hipMemset(in, 3, maxb); hipMemset(out, 4, maxb);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float ms;
    for (uint64_t mb : {8ull, 16ull, 32ull, 64ull, 96ull, 128ull, 192ull, 256ull, 512ull, 2048ull}) {
        const uint64_t bytes = mb << 20, n4 = bytes / 16;
        const int iters = (int)(8192 / mb) + 4;
        cp<<<4096, 256>>>(a, b, n4); cp<<<4096, 256>>>(b, a, n4);
        hipEventRecord(e0);
        for (int i = 0; i < iters; ++i) { cp<<<4096, 256>>>(a, b, n4); cp<<<4096, 256>>>(b, a, n4); }
        hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        const double cpbw = 2.0 * 2 * bytes * iters / (ms * 1e-3) / 1e9;
        rd<<<4096, 256>>>(a, n4, o);
        hipEventRecord(e0);
        for (int i = 0; i < 2 * iters; ++i) rd<<<4096, 256>>>(a, n4, o);
        hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        const double rdbw = 1.0 * bytes * 2 * iters / (ms * 1e-3) / 1e9;
        printf("{\"buffer_MiB\": %llu, \"pingpong_copy_rw_GBs\": %.1f, \"reread_GBs\": %.1f}\n",
               (unsigned long long)mb, cpbw, rdbw);
        fflush(stdout);
    }
    // grouped pipeline
    const uint64_t total4 = maxb / 16;
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        for (int i = 0; i < 3; ++i) {
            cp<<<8192, 256>>>(in, a, total4); cp<<<8192, 256>>>(a, b, total4);
            cp<<<8192, 256>>>(b, a, total4); cp<<<8192, 256>>>(a, out, total4);
        }
        hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("{\"pipeline\": \"whole\", \"group_MiB\": 2048, \"ms_per_4_copies\": %.4f, \"hbm_equiv_GBs\": %.1f}\n",
               ms / 3, 4.0 * 2 * maxb / (ms / 3 * 1e-3) / 1e9);
        for (uint64_t gmb : {8ull, 16ull, 32ull, 48ull, 64ull, 96ull, 128ull}) {
            const uint64_t g4 = (gmb << 20) / 16;
            const uint64_t groups = total4 / g4;
            const int grid = (int)(g4 / 256 < 4096 ? g4 / 256 : 4096);
            hipEventRecord(e0);
            for (int i = 0; i < 3; ++i)
                for (uint64_t g = 0; g < groups; ++g) {
                    cp<<<grid, 256>>>(in + g * g4, a, g4); cp<<<grid, 256>>>(a, b, g4);
                    cp<<<grid, 256>>>(b, a, g4); cp<<<grid, 256>>>(a, out + g * g4, g4);
                }
            hipEventRecord(e1); hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            printf("{\"pipeline\": \"grouped\", \"group_MiB\": %llu, \"ms_per_4_copies\": %.4f, \"hbm_equiv_GBs\": %.1f}\n",
                   (unsigned long long)gmb, ms / 3, 4.0 * 2 * maxb / (ms / 3 * 1e-3) / 1e9);
            fflush(stdout);
        }
    }
    return 0;
}
