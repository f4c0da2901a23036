// Write-pattern probe, round 2 (diagnostic, not product code).  Same run layout as
// tools/line_probe.hip: 2^28 8-byte records copied tile by tile (16K records per tile), record i
// of tile t goes to run (t, d = i / 64) of 64 records, digit d's runs of consecutive tiles adjacent.
// Questions:
//   A. does a partial 128-B line cost when the data stays in the Infinity Cache (MALL)?  Groups of
//      `group` records are copied back and forth 4 times (4 "passes") between two buffers of the
//      group's size before the next group; aligned vs shifted runs, whole array vs 16-64 MiB groups
//   B. what does a tail carry cost when every line is written whole: runs write their head line
//      completed with the previous tile's tail records, read from a RING of whole 128-B carry slots
//      (every slot written whole by one store instruction, 16 lanes, unused lanes garbage), so the
//      carry traffic stays on die; no synchronisation (timing only)
//   C. write-through (sc1) stores for shifted runs
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/line_probe2 tools/line_probe2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"

constexpr uint32_t kTile = 16384;

// MODE 0 aligned runs, 1 shifted runs, 2 shifted + ring carry (whole lines), 3 shifted, sc1 stores
template <int MODE>
__global__ __launch_bounds__(1024) void copy_runs(const uint2* __restrict__ src, uint2* __restrict__ dst,
                                                  uint32_t ntiles, uint2* __restrict__ ring,
                                                  uint32_t ring_tiles) {
    const uint32_t G = gridDim.x, b = blockIdx.x;
    for (uint32_t t = b; t < ntiles; t += G) {
        uint2 r[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) r[j] = src[(size_t)t * kTile + j * 1024 + threadIdx.x];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = j * 1024 + threadIdx.x, d = i / 64, o = i % 64;
            if (MODE == 2) {
                const uint32_t sh = (d * 7u) & 15u;
                const size_t L0 = ((size_t)d * ntiles + t) * 64;     // head line (aligned)
                const uint32_t lane = threadIdx.x & 63u;
                const int src_lane = (int)lane - (int)sh;
                const uint32_t x = __builtin_amdgcn_ds_bpermute((src_lane & 63) << 2, (int)r[j].x);
                const uint32_t y = __builtin_amdgcn_ds_bpermute((src_lane & 63) << 2, (int)r[j].y);
                uint2 val = make_uint2(x, y);
                const uint32_t pslot = ((t + ring_tiles - 1) % ring_tiles) * 256 + d;
                if (lane < 16) {                       // head line: previous tile's carry slot
                    const uint2 cv = ring[(size_t)pslot * 16 + lane];
                    if (src_lane < 0) val = cv;
                }
                dst[L0 + lane] = val;                  // 4 whole lines
                // this tile's carry slot: the last 16 records of the run, one whole line
                const uint32_t tl = (lane + sh) & 63u;  // lanes 48..63 of the shifted view
                const uint32_t cx = __builtin_amdgcn_ds_bpermute((int)((tl) << 2), (int)r[j].x);
                const uint32_t cy = __builtin_amdgcn_ds_bpermute((int)((tl) << 2), (int)r[j].y);
                if (lane >= 48)
                    ring[((size_t)(t % ring_tiles) * 256 + d) * 16 + (lane - 48)] = make_uint2(cx, cy);
                continue;
            }
            const size_t pos = ((size_t)d * ntiles + t) * 64 + o + (MODE == 0 ? 0u : ((d * 7u) & 15u));
            if (MODE == 3) {
                __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst + pos),
                                   (unsigned long long)r[j].x | ((unsigned long long)r[j].y << 32),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                dst[pos] = r[j];
            }
        }
    }
}

template <int MODE>
float run_whole(uint2* a, uint2* bb, uint32_t ntiles, uint2* ring, uint32_t ring_tiles) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    copy_runs<MODE><<<256, 1024>>>(a, bb, ntiles, ring, ring_tiles);
    hipEventRecord(e0);
    for (int r = 0; r < 4; ++r) {   // 4 "passes" ping-pong
        copy_runs<MODE><<<256, 1024>>>((r & 1) ? bb : a, (r & 1) ? a : bb, ntiles, ring, ring_tiles);
    }
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

// groups of gtiles tiles: 4 passes inside the group's two buffers (the group regions of a and b)
template <int MODE>
float run_grouped(uint2* a, uint2* bb, uint32_t ntiles, uint32_t gtiles, uint2* ring, uint32_t ring_tiles) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (uint32_t g0 = 0; g0 < ntiles; g0 += gtiles) {
        uint2* ga = a + (size_t)g0 * kTile;
        uint2* gb = bb + (size_t)g0 * kTile;
        for (int r = 0; r < 4; ++r)
            copy_runs<MODE><<<256, 1024>>>((r & 1) ? gb : ga, (r & 1) ? ga : gb, gtiles, ring, ring_tiles);
    }
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    const uint32_t ntiles = 16384;
    const size_t n = (size_t)ntiles * kTile;   // 2^28 records, 2 GiB
    uint2 *a, *b, *ring;
    if (hipMalloc(&a, n * 8 + 4096) != hipSuccess || hipMalloc(&b, n * 8 + 4096) != hipSuccess) return 1;
    if (hipMalloc(&ring, (size_t)ntiles * 256 * 128) != hipSuccess) return 1;
    hipMemset(a, 1, n * 8);
    hipMemset(b, 0, n * 8);
    const char* names[4] = {"aligned", "shifted", "shifted_ring_carry", "shifted_sc1"};
    auto line = [&](const char* what, int mode, uint32_t gtiles, uint32_t ring_tiles, float ms) {
        printf("{\"probe\": \"line_probe2\", \"what\": \"%s\", \"mode\": \"%s\", \"group_MiB\": %u, \"ring_tiles\": %u, \"ms_4_passes\": %.4f, \"ms_per_pass\": %.4f, \"rw_GBs\": %.1f}\n",
               what, names[mode], (unsigned)((size_t)gtiles * kTile * 8 >> 20), ring_tiles, ms, ms / 4,
               4 * 2.0 * n * 8 / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    for (int rep = 0; rep < 2; ++rep) {
        line("whole", 0, ntiles, 0, run_whole<0>(a, b, ntiles, ring, 1));
        line("whole", 1, ntiles, 0, run_whole<1>(a, b, ntiles, ring, 1));
        line("whole", 3, ntiles, 0, run_whole<3>(a, b, ntiles, ring, 1));
        for (uint32_t rt : {512u, 1024u, 16384u})
            line("whole", 2, ntiles, rt, run_whole<2>(a, b, ntiles, ring, rt));
        for (uint32_t gt : {512u, 1024u}) {          // 64 / 128 MiB per buffer (128 KiB tiles)
            line("grouped", 0, gt, 0, run_grouped<0>(a, b, ntiles, gt, ring, 1));
            line("grouped", 1, gt, 0, run_grouped<1>(a, b, ntiles, gt, ring, 1));
            line("grouped", 2, gt, 512, run_grouped<2>(a, b, ntiles, gt, ring, 512));
        }
    }
    return 0;
}
