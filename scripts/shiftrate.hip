// Issue-rate probe for the MQ decoder's bit window: a variable 64-bit shift
// (v_lshlrev_b64 / v_lshrrev_b64) against v_alignbit_b32 and a plain 32-bit
// shift.  8 independent chains per lane, 4096 workgroups of 256 lanes;
// prints ns per chain step (wave instruction slot) for each op.
//   hipcc --offload-arch=gfx950 -O3 -o shiftrate scripts/shiftrate.hip && ./shiftrate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed, int iters) {
    uint64_t w[8];
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        w[i] = ((uint64_t)(seed ^ (threadIdx.x * 8 + i)) << 32) | (seed + i);
        v[i] = seed * 7u + threadIdx.x + i;
    }
    const uint32_t n = (seed >> 3) & 15u;  // a runtime shift count, as the renormalisation's
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (MODE == 0) w[i] = (w[i] << n) ^ (uint64_t)it;           // 64-bit shift
            else if constexpr (MODE == 1) v[i] = __builtin_amdgcn_alignbit(v[i], v[(i + 1) & 7], 32 - n) ^ it;
            else v[i] = (v[i] << n) ^ (uint32_t)it;                              // 32-bit shift
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += (uint32_t)w[i] ^ (uint32_t)(w[i] >> 32) ^ v[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
static double run(uint32_t *d, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k<MODE><<<4096, 256>>>(d, 0x5a5a5a5au, iters);
    hipEventRecord(a);
    k<MODE><<<4096, 256>>>(d, 0x5a5a5a5au, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    // wave-steps per SIMD: 4096 * 4 waves * iters * 8 chains over 1024 SIMDs
    const double steps = 4096.0 * 4 * iters * 8 / 1024.0;
    return ms * 1e6 / steps;
}

int main() {
    uint32_t *d;
    hipMalloc(&d, 4096 * 256 * 4);
    const int iters = 2000;
    printf("ns per wave-step per SIMD (each step = op + xor):\n");
    printf("  64-bit shift  %.3f\n", run<0>(d, iters));
    printf("  alignbit      %.3f\n", run<1>(d, iters));
    printf("  32-bit shift  %.3f\n", run<2>(d, iters));
    hipFree(d);
    return 0;
}
