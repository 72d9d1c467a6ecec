// Throughput probe: wave-instructions per SIMD-cycle of the integer ops the
// 9/7 lifting uses (v_mad_i64_i32 + v_alignbit vs 24-bit split).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE>
__global__ void k(int32_t *out, int32_t seed, int iters) {
    int32_t a0 = threadIdx.x + seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 11, a5 = a0 + 13, a6 = a0 - 1, a7 = a0 ^ 5;
    for (int i = 0; i < iters; ++i) {
#define STEP(a) \
        if (MODE == 0) a = (int32_t)(((int64_t)a * 12994 + 4096) >> 13) + i; \
        else if (MODE == 1) { int32_t h = a >> 13, l = a & 0x1fff; a = h * 12994 + (int32_t)(((uint32_t)l * 12994u + 4096u) >> 13) + i; } \
        else a = a + (a >> 1) + i;
        STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

int main() {
    int32_t *o; hipMalloc(&o, 1 << 26);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 4096, blocks = 256 * 8 * 4, threads = 256;  // 8 waves/SIMD
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (mode == 0) k<0><<<blocks, threads>>>(o, 1, iters);
            if (mode == 1) k<1><<<blocks, threads>>>(o, 1, iters);
            if (mode == 2) k<2><<<blocks, threads>>>(o, 1, iters);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            double steps = (double)blocks * threads / 64 * iters * 8;  // wave-steps
            if (rep) printf("mode %d: %.3f ms, %.3f ns per wave-step per SIMD (x1024 SIMDs)\n", mode, ms, ms * 1e6 / steps * 1024);
        }
    }
    return 0;
}
