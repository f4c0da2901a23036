// Ceiling probe for the radix scatter's write pattern (diagnostic, not product code):
// copy 2 GiB src -> dst where the source is consumed linearly in runs of L bytes and run i goes
// to bucket r = (i * 167) % B at that bucket's next free slot (B append streams, like a B-way
// radix scatter with perfectly regular runs).  Reports read+write GB/s versus L and B.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int L4>  // run length in u32
__global__ __launch_bounds__(256) void scatter_runs(const uint32_t* __restrict__ src,
                                                   uint32_t* __restrict__ dst, uint64_t nruns,
                                                   uint32_t buckets, uint64_t bucket_len) {
    const uint64_t lanes = (uint64_t)gridDim.x * 256;
    for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < nruns * L4; e += lanes) {
        const uint64_t i = e / L4, o = e % L4;
        const uint64_t r = (i * 167) % buckets, k = i / buckets;
        dst[r * bucket_len + k * L4 + o] = src[e];
    }
}

template <int L4>
float run(const uint32_t* s, uint32_t* d, uint64_t n, uint32_t buckets) {
    const uint64_t nruns = n / L4;
    const uint64_t blen = n / buckets;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    scatter_runs<L4><<<4096, 256>>>(s, d, nruns, buckets, blen);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) scatter_runs<L4><<<4096, 256>>>(s, d, nruns, buckets, blen);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const uint64_t n = 1ull << 29;  // 2 GiB of u32
    uint32_t *s, *d;
    if (hipMalloc(&s, n * 4) != hipSuccess || hipMalloc(&d, n * 4) != hipSuccess) return 1;
    hipMemset(s, 1, n * 4); hipMemset(d, 0, n * 4);
    for (uint32_t B : {256u, 64u, 1024u}) {
        float t[8];
        t[0] = run<16>(s, d, n, B);    // 64 B
        t[1] = run<32>(s, d, n, B);    // 128 B
        t[2] = run<64>(s, d, n, B);    // 256 B
        t[3] = run<128>(s, d, n, B);   // 512 B
        t[4] = run<256>(s, d, n, B);   // 1 KiB
        t[5] = run<1024>(s, d, n, B);  // 4 KiB
        const int Ls[6] = {64, 128, 256, 512, 1024, 4096};
        for (int i = 0; i < 6; ++i)
            printf("{\"buckets\": %u, \"run_bytes\": %d, \"ms\": %.4f, \"rw_GBs\": %.1f}\n", B, Ls[i], t[i],
                   2.0 * n * 4 / (t[i] * 1e-3) / 1e9);
    }
    // linear copy reference
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) hipMemcpyAsync(d, s, n * 4, hipMemcpyDeviceToDevice);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("{\"memcpy_d2d_ms\": %.4f, \"rw_GBs\": %.1f}\n", ms / 5, 2.0 * n * 4 / (ms / 5 * 1e-3) / 1e9);
    return 0;
}
