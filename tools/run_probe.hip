// Write-pattern probe, round 5 (diagnostic, not product code).  k_onesweep's memory shape (16K-record
// tiles of 8-byte records from a ticket counter, one 1024-thread workgroup per CU, the next tile's
// loads issued before this tile's stores) with the stores laid out as the MSD pass lays them out:
// staged record i of tile T belongs to run d = i' / R (i' = (i + off) mod 16K), and the runs of one
// digit are adjacent in tile order: run (d, T) starts at d * ntiles * R + T * R + sh(d).
// Store instruction k of a wave writes staged records [64k, 64k + 64) (k_onesweep's scatter order).
//   sh = 0        every run starts on a 128-B line (no partial line at run ends)
//   sh = 7d & 15  runs start mid-line: the line at each run boundary is written by two tiles
//   off = 0       (R = 64) each run is one store instruction; off = 37: each run is split over two
//                 store instructions (two waves) at a point that is not a line boundary, as a run
//                 of the real pass is wherever it straddles a 64-record group of the staging order
// Prints one JSON line per variant (ms per 2^28-record pass, read + written bytes / time).
//   hipcc -O3 --offload-arch=gfx950 -o tools/run_probe tools/run_probe.hip && tools/run_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int KPT = 16, TILE = 1024 * KPT;

// xcd: tiles are claimed per XCD (HW_REG_XCC_ID) in groups of 32 consecutive tiles, group g of every
// round of 256 going to XCD g: adjacent tiles (whose runs share the boundary lines) are then written
// by the same L2 at about the same time, except at every 32nd tile
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}
__global__ __launch_bounds__(1024) void run_tile(const uint2* __restrict__ in, uint2* __restrict__ out,
                                                 uint32_t ntiles, uint32_t* ticket, uint32_t R,
                                                 uint32_t shifted, uint32_t off, uint32_t linear, uint32_t xcd) {
    __shared__ uint32_t s_t;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t x = xcd == 1 ? xcc_id() : (xcd == 2 ? (blockIdx.x & 7u) : 0u);   // 2: the blockIdx % 8 guess
    auto claim = [&]() -> uint32_t {
        if (!xcd) return atomicAdd(ticket, 1u);
        const uint32_t c = atomicAdd(ticket + 1 + x, 1u);
        const uint32_t t = (c / 32u) * 256u + x * 32u + (c % 32u);
        return t < ntiles ? t : 0xFFFFFFFFu;
    };
    if (threadIdx.x == 0) s_t = claim();
    __syncthreads();
    uint32_t T = s_t;
    uint2 r[KPT];
    auto load = [&](uint32_t t) {
        const uint2* p = in + (size_t)t * TILE + w * 64 * KPT + lane;
#pragma unroll
        for (int j = 0; j < KPT; ++j) r[j] = p[j * 64];
    };
    if (T < ntiles) load(T);
    const size_t per_digit = (size_t)ntiles * R;
    while (T < ntiles) {
        __syncthreads();
        if (threadIdx.x == 0) s_t = claim();
        __syncthreads();
        const uint32_t Tn = s_t;
        uint2 q[KPT];
#pragma unroll
        for (int j = 0; j < KPT; ++j) q[j] = r[j];
        if (Tn < ntiles) load(Tn);
#pragma unroll
        for (int j = 0; j < KPT; ++j) {
            const uint32_t i = j * 1024u + threadIdx.x;          // staged index (scatter order)
            size_t pos;
            if (linear) {
                pos = (size_t)T * TILE + i;
            } else {
                const uint32_t ip = (i + off) & (TILE - 1u);
                const uint32_t d = ip / R, o = ip % R;
                pos = d * per_digit + (size_t)T * R + o + (shifted ? ((d * 7u) & 15u) : 0u);
            }
            out[pos] = q[j];
        }
        T = Tn;
    }
}

__global__ void placement(uint32_t* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

int main() {
    const size_t recs = 1ull << 28, bytes = recs * 8;
    int cus = 256;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
    }
    void *a = nullptr, *b = nullptr;
    uint32_t* tk = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes + 4096));
    CK(hipMalloc((void**)&tk, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes + 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint32_t ntiles = (uint32_t)(recs / TILE);
    {   // where a grid of `cus` 1024-thread workgroups lands: XCC_ID of every block vs blockIdx % 8
        uint32_t* pl = nullptr;
        CK(hipMalloc((void**)&pl, 4 * cus));
        hipLaunchKernelGGL(placement, dim3(cus), dim3(1024), 0, 0, pl);
        CK(hipDeviceSynchronize());
        uint32_t h[1024];
        CK(hipMemcpy(h, pl, 4 * cus, hipMemcpyDeviceToHost));
        int match = 0, per[8] = {0};
        for (int i = 0; i < cus; ++i) { match += (h[i] & 7u) == (uint32_t)(i & 7); per[h[i] & 7u]++; }
        printf("{\"probe\": \"placement\", \"blocks\": %d, \"xcc_eq_blockidx_mod8\": %d, \"per_xcc\": [%d,%d,%d,%d,%d,%d,%d,%d], \"first16\": [", cus, match,
               per[0], per[1], per[2], per[3], per[4], per[5], per[6], per[7]);
        for (int i = 0; i < 16; ++i) printf("%u%s", h[i], i < 15 ? "," : "]}\n");
        CK(hipFree(pl));
    }
    struct V { const char* name; uint32_t R, shifted, off, linear, xcd; };
    const V vs[] = {
        {"linear", 64, 0, 0, 1, 0},
        {"aligned_R64", 64, 0, 0, 0, 0},
        {"shifted_R64", 64, 1, 0, 0, 0},
        {"shifted_R64_split", 64, 1, 37, 0, 0},
        {"shifted_R128", 128, 1, 0, 0, 0},
        {"linear_xcd", 64, 0, 0, 1, 1},
        {"aligned_R64_xcd", 64, 0, 0, 0, 1},
        {"shifted_R64_xcd", 64, 1, 0, 0, 1},
        {"shifted_R64_split_xcd", 64, 1, 37, 0, 1},
        {"shifted_R128_xcd", 128, 1, 0, 0, 1},
        {"shifted_R32_split_xcd", 32, 1, 37, 0, 1},
        {"shifted_R64_xcdguess", 64, 1, 0, 0, 2},
        {"linear_xcdguess", 64, 0, 0, 1, 2},
    };
    for (int pass = 0; pass < 2; ++pass) {
        for (const V& v : vs) {
            const int reps = 10;
            float best = 1e30f, sum = 0.f;
            for (int r = -2; r < reps; ++r) {
                CK(hipMemset(tk, 0, 64));
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(run_tile, dim3(cus), dim3(1024), 0, 0, (const uint2*)a, (uint2*)b, ntiles, tk,
                                   v.R, v.shifted, v.off, v.linear, v.xcd);
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0.f;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 0) { sum += ms; if (ms < best) best = ms; }
            }
            const float avg = sum / reps;
            printf("{\"probe\": \"run_probe\", \"round\": %d, \"variant\": \"%s\", \"avg_ms\": %.4f, \"best_ms\": %.4f, \"avg_GBs\": %.1f}\n",
                   pass, v.name, avg, best, 2.0 * bytes / (avg * 1e-3) / 1e9);
            fflush(stdout);
        }
    }
    return 0;
}
