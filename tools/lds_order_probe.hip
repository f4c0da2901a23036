// Probe: does ds_add_rtn_u32 from one wave return values in lane order for lanes that hit the
// same LDS address?  If so, old == (# lower lanes with the same address) for zeroed counters,
// which is exactly the stable in-wave rank a radix sort needs.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ uint32_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; return (uint32_t)(z ^ (z >> 31));
}

template <int MODE>
__global__ __launch_bounds__(256) void probe(uint64_t* bad, uint64_t* total, int trials, uint32_t seed) {
    __shared__ uint32_t cnt[4][1024];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint64_t nb = 0, nt = 0;
    for (int t = 0; t < trials; ++t) {
        for (int i = lane; i < 1024; i += 64) cnt[w][i] = 0;
        uint32_t r = mix(((uint64_t)seed << 40) ^ ((uint64_t)blockIdx.x << 20) ^ ((uint64_t)t << 8) ^ (w << 6) ^ 0);
        uint32_t rl = mix(((uint64_t)r << 7) ^ lane);
        uint32_t d;
        if (MODE == 0) d = rl & 255;                  // random 8-bit digit
        else if (MODE == 1) d = rl & 3;               // 4 addresses
        else if (MODE == 2) d = 0;                    // all lanes one address
        else if (MODE == 3) d = (rl & 7) * 32;        // same bank, 8 addresses
        else d = (r & 1) ? (rl & 15) : (rl & 255) * 4 % 1024;  // mixed
        bool active = (MODE == 4) ? ((rl >> 12) & 3) != 0 : true;   // partial exec mask
        uint64_t act = __ballot(active);
        uint32_t old = 0;
        if (active) old = atomicAdd(&cnt[w][d], 1u);
        // expected: active lanes below me with the same d
        uint32_t exp = 0;
        for (int l = 0; l < 64; ++l) {
            uint32_t dl = __shfl(d, l);
            if (l < lane && dl == d && ((act >> l) & 1)) ++exp;
        }
        if (active) { nt++; if (old != exp) nb++; }
    }
    atomicAdd((unsigned long long*)bad, (unsigned long long)nb);
    atomicAdd((unsigned long long*)total, (unsigned long long)nt);
}

int main() {
    uint64_t *d; hipMalloc(&d, 16);
    const char* names[] = {"random8", "four_addr", "one_addr", "same_bank", "mixed_partial_exec"};
    for (int mode = 0; mode < 5; ++mode) {
        hipMemset(d, 0, 16);
        for (int rep = 0; rep < 4; ++rep) {
            switch (mode) {
                case 0: probe<0><<<2048, 256>>>(d, d + 1, 64, rep); break;
                case 1: probe<1><<<2048, 256>>>(d, d + 1, 64, rep); break;
                case 2: probe<2><<<2048, 256>>>(d, d + 1, 64, rep); break;
                case 3: probe<3><<<2048, 256>>>(d, d + 1, 64, rep); break;
                default: probe<4><<<2048, 256>>>(d, d + 1, 64, rep); break;
            }
        }
        uint64_t h[2]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("{\"mode\": \"%s\", \"lane_atomics\": %llu, \"out_of_lane_order\": %llu}\n", names[mode],
               (unsigned long long)h[1], (unsigned long long)h[0]);
    }
    return 0;
}
