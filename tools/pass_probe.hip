// Run-length probe on the real pass kernel, round 5 (diagnostic, not product code).  Times the
// hybrid path's MSD pass 0 kernel (k_onesweep, 16K-record tiles: caller arrays -> records) over 2^28
// uniform keys + values at digit widths 8 / 7 / 6 bits (a digit run of a tile is 16384 / 2^w
// records: 64 / 128 / 256), so that the cost of the run length is measured on the kernel itself
// rather than on a copy (tools/run_probe.hip).  Each launch is checked to have placed every record
// (a permutation check of the keys' sum and the values' xor over the output).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I webgpu-radix-sort_amd/csrc -o tools/pass_probe tools/pass_probe.hip
#include "rs_kernels.hpp"
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void hist_bits(const uint32_t* k, size_t n, uint32_t shift, uint32_t mask, uint32_t* h) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        atomicAdd(&h[(k[i] >> shift) & mask], 1u);
}
__global__ void sum_out(const uint2* r, size_t n, unsigned long long* acc) {
    unsigned long long s = 0, x = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        s += r[i].x;
        x ^= (unsigned long long)r[i].y * 0x9E3779B97F4A7C15ull;
    }
    atomicAdd(&acc[0], s);
    atomicXor(&acc[1], x);
}

int main() {
    const size_t n = 1ull << 28;
    constexpr int BLOCK = 1024, KPT = 16, TILE = BLOCK * KPT;
    const uint32_t ntiles = (uint32_t)(n / TILE);
    int cus = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
    }
    uint32_t *k = nullptr, *v = nullptr, *h = nullptr, *tk = nullptr, *err = nullptr;
    uint2* out = nullptr;
    unsigned long long *status = nullptr, *acc = nullptr;
    CK(hipMalloc(&k, 4 * n));
    CK(hipMalloc(&v, 4 * n));
    CK(hipMalloc(&out, 8 * n));
    CK(hipMalloc(&h, 4 * 1024));
    CK(hipMalloc(&tk, 64));
    CK(hipMalloc(&err, 64));
    CK(hipMalloc(&acc, 16));
    CK(hipMalloc(&status, 8ull * ntiles * 512));
    CK(hipMemset(status, 0, 8ull * ntiles * 512));
    CK(hipMemset(err, 0, 64));
    hipLaunchKernelGGL(rs::k_fill_random, dim3(4096), dim3(256), 0, 0, k, (uint64_t)n, 12345ull, 0ull);
    hipLaunchKernelGGL(rs::k_fill_iota, dim3(4096), dim3(256), 0, 0, v, (uint64_t)n, 0u);
    CK(hipDeviceSynchronize());
    // expected checksums
    std::vector<uint32_t> hk(n), hv(n);
    CK(hipMemcpy(hk.data(), k, 4 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hv.data(), v, 4 * n, hipMemcpyDeviceToHost));
    unsigned long long es = 0, ex = 0;
    for (size_t i = 0; i < n; ++i) { es += hk[i]; ex ^= (unsigned long long)hv[i] * 0x9E3779B97F4A7C15ull; }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto kern = rs::k_onesweep<8, BLOCK, KPT, rs::LAYOUT_SOA, rs::RANK_LDS_ATOMIC, rs::LAYOUT_AOS, 1, 0, false>;
    uint32_t epoch = 0;
    const int widths[] = {8, 7, 6, 8, 7};
    for (int w : widths) {
        const uint32_t shift = 32 - w, mask = (1u << w) - 1u;
        CK(hipMemset(h, 0, 4 * 1024));
        hipLaunchKernelGGL(hist_bits, dim3(4096), dim3(256), 0, 0, k, n, shift, mask, h);
        const int reps = 10;
        float sum = 0.f, best = 1e30f;
        bool ok = true;
        for (int r = -2; r < reps; ++r) {
            ++epoch;
            CK(hipMemset(tk, 0, 64));
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(kern, dim3(std::min<uint32_t>(ntiles, cus)), dim3(BLOCK), 0, 0, k, v, (uint32_t*)out,
                               (uint32_t*)nullptr, (uint32_t)n, shift, mask, ntiles, (const uint32_t*)h, status, tk,
                               err, (uint32_t*)nullptr, 0u, 0u, epoch, (const uint32_t*)nullptr, 0, (uint32_t*)nullptr,
                               0xFFFFFFFFu, 1u << 20, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                               (const uint32_t*)nullptr, 0u, 0xFFFFFFFFu);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) { sum += ms; best = ms < best ? ms : best; }
            if (r == reps - 1) {
                CK(hipMemset(acc, 0, 16));
                hipLaunchKernelGGL(sum_out, dim3(4096), dim3(256), 0, 0, (const uint2*)out, n, acc);
                unsigned long long a[2];
                uint32_t e = 0;
                CK(hipMemcpy(a, acc, 16, hipMemcpyDeviceToHost));
                CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
                ok = a[0] == es && a[1] == ex && e == 0;
            }
        }
        const float avg = sum / reps;
        printf("{\"probe\": \"pass_probe\", \"digit_bits\": %d, \"run_records\": %u, \"avg_ms\": %.4f, \"best_ms\": %.4f, "
               "\"frac_of_8TBs\": %.4f, \"checksum_ok\": %s}\n",
               w, (uint32_t)(TILE >> w), avg, best, 16.0 * n / (avg * 1e-3) / 8e12, ok ? "true" : "false");
        fflush(stdout);
    }
    return 0;
}
