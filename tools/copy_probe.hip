// HBM ceiling probe (diagnostic, not product code): what a streaming copy of one MSD pass's bytes
// (2^28 8-byte records: 2 GiB read + 2 GiB written) achieves on this MI355X, in the shapes the
// pass kernels use.  Prints one JSON line per variant: ms and (read + written bytes) / time.
//   hipcc -O3 --offload-arch=gfx950 -o tools/copy_probe tools/copy_probe.hip && tools/copy_probe
//
//   f4_256      16-B loads/stores, 256-thread blocks, grid-stride (8 blocks per CU)
//   f4_1024x1   16-B, 1024-thread blocks, one per CU (k_onesweep's occupancy), 4 loads in flight
//   rec_tile    k_onesweep's load shape: 16K-record tiles of 8-byte records, 1024 threads x 16
//               slots (one 8-byte load per slot, 512 B per wave-instruction), the next tile's loads
//               issued before this tile's stores, one workgroup per CU, tiles from a ticket counter
//   read_f4     16-B loads only (sum), 256-thread blocks
//   write_f4    16-B stores only, 256-thread blocks
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void f4_256(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) out[i] = in[i];
}

__global__ __launch_bounds__(1024) void f4_1024x1(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n4) {
    const size_t stride = (size_t)gridDim.x * 1024;
    size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        const uint4 a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
        out[i] = a; out[i + stride] = b; out[i + 2 * stride] = c; out[i + 3 * stride] = d;
    }
    for (; i < n4; i += stride) out[i] = in[i];
}

__global__ __launch_bounds__(1024) void rec_tile(const uint2* __restrict__ in, uint2* __restrict__ out,
                                                 uint32_t ntiles, uint32_t* ticket) {
    constexpr int KPT = 16, TILE = 1024 * KPT;
    __shared__ uint32_t s_t;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
    __syncthreads();
    uint32_t T = s_t;
    uint2 r[KPT];
    auto load = [&](uint32_t t) {
        const uint2* p = in + (size_t)t * TILE + w * 64 * KPT + lane;
#pragma unroll
        for (int j = 0; j < KPT; ++j) r[j] = p[j * 64];
    };
    if (T < ntiles) load(T);
    while (T < ntiles) {
        __syncthreads();
        if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint32_t Tn = s_t;
        uint2 q[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) q[j] = r[j];
        if (Tn < ntiles) load(Tn);
        uint2* o = out + (size_t)T * TILE + w * 64 * KPT + lane;
#pragma unroll
        for (int j = 0; j < KPT; ++j) o[j * 64] = q[j];
        T = Tn;
    }
}

__global__ __launch_bounds__(256) void read_f4(const uint4* __restrict__ in, uint32_t* out, size_t n4) {
    uint32_t s = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const uint4 q = in[i];
        s ^= q.x ^ q.y ^ q.z ^ q.w;
    }
    if (s == 0x12345678u) out[0] = s;
}

__global__ __launch_bounds__(256) void write_f4(uint4* __restrict__ out, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        out[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

int main() {
    const size_t recs = 1ull << 28, bytes = recs * 8, n4 = bytes / 16;
    int cus = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
    }
    void *a = nullptr, *b = nullptr;
    uint32_t* tk = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc((void**)&tk, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t ntiles = (uint32_t)(recs / 16384);
    for (int v = 0; v < 8; ++v) {
        const char* name = "";
        double moved = 2.0 * bytes;
        const int reps = 10;
        float best = 1e30f, sum = 0.f;
        for (int r = -2; r < reps; ++r) {
            CK(hipMemset(tk, 0, 64));
            CK(hipEventRecord(e0, 0));
            switch (v) {
                case 0: name = "f4_256_g8"; hipLaunchKernelGGL(f4_256, dim3(cus * 8), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n4); break;
                case 1: name = "f4_256_g32"; hipLaunchKernelGGL(f4_256, dim3(cus * 32), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n4); break;
                case 2: name = "f4_1024x1"; hipLaunchKernelGGL(f4_1024x1, dim3(cus), dim3(1024), 0, 0, (const uint4*)a, (uint4*)b, n4); break;
                case 3: name = "f4_1024x2"; hipLaunchKernelGGL(f4_1024x1, dim3(cus * 2), dim3(1024), 0, 0, (const uint4*)a, (uint4*)b, n4); break;
                case 4: name = "rec_tile"; hipLaunchKernelGGL(rec_tile, dim3(cus), dim3(1024), 0, 0, (const uint2*)a, (uint2*)b, ntiles, tk); break;
                case 5: name = "read_f4"; moved = bytes; hipLaunchKernelGGL(read_f4, dim3(cus * 8), dim3(256), 0, 0, (const uint4*)a, tk, n4); break;
                case 6: name = "write_f4"; moved = bytes; hipLaunchKernelGGL(write_f4, dim3(cus * 8), dim3(256), 0, 0, (uint4*)b, n4); break;
                case 7: name = "hipMemcpyD2D"; CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0)); break;
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) { sum += ms; if (ms < best) best = ms; }
        }
        const float avg = sum / reps;
        printf("{\"variant\": \"%s\", \"bytes_moved\": %.0f, \"avg_ms\": %.4f, \"best_ms\": %.4f, \"avg_GBs\": %.1f, \"best_GBs\": %.1f}\n",
               name, moved, avg, best, moved / (avg * 1e-3) / 1e9, moved / (best * 1e-3) / 1e9);
    }
    return 0;
}
