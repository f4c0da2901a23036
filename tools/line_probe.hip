// Write-pattern probe (diagnostic, not product code): what do partial 128-B lines cost the radix
// scatter?  Copies 2^28 8-byte records tile by tile (16K records per tile, one tile per
// workgroup iteration) into 256 digit regions; record i of tile t goes to run (t, d = i / 64),
// i.e. every (tile, digit) run is exactly 64 records = 512 B, and digit d's runs of consecutive
// tiles are adjacent, as in a real pass over uniform keys.
//   mode 0: linear copy (pos = input pos)
//   mode 1: runs start on 128-B lines (every write is a whole line)
//   mode 2: digit d's region shifted by (7d mod 16) records: every run touches 5 lines, the two
//           end lines shared with the neighbouring tiles' runs (written by other workgroups)
//   mode 3: as 2, but tiles dealt so that the workgroups of one XCD (dispatch round-robin over
//           the 8 XCDs) copy ADJACENT tiles at the same time: shared end lines meet in one L2
//   mode 4: as 1 with mode 3's tile order
//   mode 5: as 2, but every store instruction covers whole aligned lines: a wave writes its run
//           through a line-aligned 80-slot window (two stores, lanes outside the run masked),
//           so a run's two end lines are still shared with the neighbouring tiles' runs
//   mode 6: as 2, but every line of the output is written whole, once: a run writes its head
//           line completed with the previous tile's tail records (read from a side buffer of
//           16-record slots) and its body lines, and leaves its own tail records in its side slot
//           (the traffic of a tail-carrying scatter, without its synchronisation)
//   mode 7: as 3, but the shift is a multiple of 4 records: runs start on 32-B sectors, not on
//           128-B lines (is the cost per partial line or per partial 32-B sector?)
//   mode 8: as 1, but the last 4 records of every run are not written: each run's last line is
//           partial and nobody else writes it (does a partial line cost without a second writer?)
//   mode 9: as 0 shifted by 8 records: every 4th line is written half by one wave, half by the
//           next wave of the same workgroup (does a line split inside a workgroup cost?)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/line_probe tools/line_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"

template <int MODE, int RL = 64>
__global__ __launch_bounds__(1024) void copy_runs(const uint2* __restrict__ src,
                                                  uint2* __restrict__ dst, uint32_t ntiles,
                                                  uint2* __restrict__ side) {
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t first = (MODE >= 3 && MODE <= 7) ? (b & 7u) * (G >> 3) + (b >> 3) : b;
    for (uint32_t t = first; t < ntiles; t += G) {
        uint2 r[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) r[j] = src[(size_t)t * 16384 + j * 1024 + threadIdx.x];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t i = j * 1024 + threadIdx.x, d = i / RL, o = i % RL;
            size_t pos;
            if (MODE == 6) {
                const uint32_t sh = (d * 7u) & 15u;
                const size_t L0 = ((size_t)d * ntiles + t) * 64;     // head line (aligned)
                const uint32_t lane = threadIdx.x & 63u;
                const int src_lane = (int)lane - (int)sh;
                const uint32_t x = __builtin_amdgcn_ds_bpermute((src_lane & 63) << 2, (int)r[j].x);
                const uint32_t y = __builtin_amdgcn_ds_bpermute((src_lane & 63) << 2, (int)r[j].y);
                uint2 val = make_uint2(x, y);
                if (src_lane < 0 && t > 0) val = side[((size_t)(t - 1) * 256 + d) * 16 + lane];
                dst[L0 + lane] = val;                                 // 4 whole lines
                if (o >= 64u - sh) side[((size_t)t * 256 + d) * 16 + (o - (64u - sh))] = r[j];
                continue;
            }
            if (MODE == 5) {
                const uint32_t sh = (d * 7u) & 15u;              // run start within its line
                const size_t P = ((size_t)d * ntiles + t) * 64 + sh;
                const uint32_t lane = threadIdx.x & 63u;
                // window slot q = lane (first store) or 64 + lane (second) holds run offset q - sh
                for (int h = 0; h < 2; ++h) {
                    const int q = h * 64 + (int)lane;
                    const int src_lane = q - (int)sh;
                    const uint32_t x = __builtin_amdgcn_ds_bpermute((src_lane & 63) << 2, (int)r[j].x);
                    const uint32_t y = __builtin_amdgcn_ds_bpermute((src_lane & 63) << 2, (int)r[j].y);
                    if (src_lane >= 0 && src_lane < 64) dst[P - sh + q] = make_uint2(x, y);
                }
                continue;
            }
            if (MODE == 0) pos = (size_t)t * 16384 + i;
            else if (MODE == 9) pos = (size_t)t * 16384 + i + 8;   // linear, lines split between waves
            else pos = ((size_t)d * ntiles + t) * RL + o + ((MODE == 2 || MODE == 3) ? ((d * 7u) & 15u)
                                                            : MODE == 7 ? ((d * 7u) & 12u) : 0u);
            if (MODE == 8 && o >= (uint32_t)RL - 4u) continue;   // last line 12/16 written, by one writer
            dst[pos] = r[j];
        }
    }
}

static uint2* g_side = nullptr;
template <int MODE, int RL = 64>
float run(const uint2* s, uint2* d, uint32_t ntiles, int grid) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    copy_runs<MODE, RL><<<grid, 1024>>>(s, d, ntiles, g_side);
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r) copy_runs<MODE, RL><<<grid, 1024>>>(s, d, ntiles, g_side);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 10;
}

int main(int argc, char** argv) {
    const uint32_t ntiles = 16384;
    const size_t n = (size_t)ntiles * 16384;   // 2^28 records, 2 GiB
    uint2 *s, *d;
    if (hipMalloc(&s, n * 8) != hipSuccess || hipMalloc(&d, n * 8 + 4096) != hipSuccess) return 1;
    hipMemset(s, 1, n * 8);
    hipMemset(d, 0, n * 8 + 4096);
    if (hipMalloc(&g_side, (size_t)ntiles * 256 * 128) != hipSuccess) return 1;
    if (argc > 1 && strcmp(argv[1], "runs") == 0) {
        // run length series (digit width go/no-go: 11-bit digits leave ~8-record runs per 16K tile)
        for (int rep = 0; rep < 2; ++rep) {
            const float t[8] = {run<1, 8>(s, d, ntiles, 256), run<2, 8>(s, d, ntiles, 256),
                                run<1, 16>(s, d, ntiles, 256), run<2, 16>(s, d, ntiles, 256),
                                run<1, 32>(s, d, ntiles, 256), run<2, 32>(s, d, ntiles, 256),
                                run<1, 64>(s, d, ntiles, 256), run<2, 64>(s, d, ntiles, 256)};
            const int rl[8] = {8, 8, 16, 16, 32, 32, 64, 64};
            for (int m = 0; m < 8; ++m)
                printf("{\"probe\": \"line_probe\", \"mode\": \"%s\", \"run_records\": %d, \"grid\": 256, \"ms\": %.4f, \"rw_GBs\": %.1f}\n",
                       (m & 1) ? "runs_shifted" : "runs_line_aligned", rl[m], t[m], 2.0 * n * 8 / (t[m] * 1e-3) / 1e9);
        }
        return 0;
    }
    for (int grid : {256, 512, 1024}) {
        const float t0 = run<0>(s, d, ntiles, grid);
        const float t1 = run<1>(s, d, ntiles, grid);
        const float t2 = run<2>(s, d, ntiles, grid);
        const float t3 = run<3>(s, d, ntiles, grid);
        const float t4 = run<4>(s, d, ntiles, grid);
        const float t5 = run<5>(s, d, ntiles, grid);
        const float t6 = run<6>(s, d, ntiles, grid);
        const float t7 = run<7>(s, d, ntiles, grid);
        const float t8 = run<8>(s, d, ntiles, grid);
        const float t9 = run<9>(s, d, ntiles, grid);
        const char* names[10] = {"linear", "runs_line_aligned", "runs_shifted",
                                 "runs_shifted_xcd_adjacent", "runs_line_aligned_xcd_adjacent",
                                 "runs_shifted_aligned_stores", "runs_shifted_tail_carry",
                                 "runs_sector_aligned", "runs_aligned_last_line_partial_one_writer",
                                 "linear_shifted_lines_split_between_waves"};
        const float ts[10] = {t0, t1, t2, t3, t4, t5, t6, t7, t8, t9};
        for (int m = 0; m < 10; ++m)
            printf("{\"probe\": \"line_probe\", \"mode\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"rw_GBs\": %.1f}\n",
                   names[m], grid, ts[m], 2.0 * n * 8 / (ts[m] * 1e-3) / 1e9);
    }
    for (int grid : {256, 1024}) {
        const float a1 = run<1, 128>(s, d, ntiles, grid), a2 = run<2, 128>(s, d, ntiles, grid);
        const float b1 = run<1, 256>(s, d, ntiles, grid), b2 = run<2, 256>(s, d, ntiles, grid);
        const float c1 = run<1, 32>(s, d, ntiles, grid), c2 = run<2, 32>(s, d, ntiles, grid);
        const int rl[6] = {128, 128, 256, 256, 32, 32};
        const float ts[6] = {a1, a2, b1, b2, c1, c2};
        for (int m = 0; m < 6; ++m)
            printf("{\"probe\": \"line_probe\", \"mode\": \"%s\", \"run_records\": %d, \"grid\": %d, \"ms\": %.4f, \"rw_GBs\": %.1f}\n",
                   (m & 1) ? "runs_shifted" : "runs_line_aligned", rl[m], grid, ts[m],
                   2.0 * n * 8 / (ts[m] * 1e-3) / 1e9);
    }
    return 0;
}
