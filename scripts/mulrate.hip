// Issue-rate probe for the 9/7 lifting multiply: fixmul13 as one 64-bit
// v_mad_i64_i32 (+ alignbit) against the 24-bit decomposition (5 full-rate
// ops), and a plain 32-bit add chain for scale.  8 independent chains per
// lane, 4096 workgroups of 256 lanes; prints ns per wave instruction slot.
//   hipcc --offload-arch=gfx950 -O3 -o mulrate scripts/mulrate.hip && ./mulrate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ int32_t fm64(int32_t a, int32_t b) {
    return (int32_t)(((int64_t)a * (int64_t)b + 4096) >> 13);
}
__device__ __forceinline__ int32_t fm24(int32_t a, int32_t b) {
    const uint32_t lo = (((uint32_t)a & 0x1fffu) * (uint32_t)b + 4096u) >> 13;
    return (int32_t)((uint32_t)(a >> 13) * (uint32_t)b + lo);
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
// the 16-bit split through the packed dot products: (s*c + 4096) >> 13 =
// 8 (s_hi c) + ((s_lo c + 4096) >> 13), exact mod 2^32 for 0 <= c < 2^15
__device__ __forceinline__ int32_t fmdot(int32_t a, int32_t b) {
    const uint32_t X = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), u16x2{(unsigned short)b, 0}, 4096u, false);
    const int32_t Y = __builtin_amdgcn_sdot2(__builtin_bit_cast(i16x2, a), i16x2{0, (short)b}, 0, false);
    return (int32_t)(((uint32_t)Y << 3) + (X >> 13));
}

// the lift held in doubles: s c / 2^13 + 1/2 is exact (|s| < 2^31, c < 2^15),
// so floor() of it is fixmul13; values stay integers in f64 registers
__device__ __forceinline__ double lift_f64(double t, double s, double c13) {
    return t - __builtin_floor(__builtin_fma(s, c13, 0.5));
}

// one 24-bit multiply-add (v_mad_i32_i24): exact while |s| < 2^23 and
// |s c| + 4096 < 2^31 -- the bounded-magnitude lift
__device__ __forceinline__ int32_t fm24s(int32_t a, int32_t b) { return (__mul24(a, b) + 4096) >> 13; }
// a plain 32-bit multiply (v_mul_lo_u32), exact while |s c| + 4096 < 2^31
__device__ __forceinline__ int32_t fm32(int32_t a, int32_t b) { return (a * b + 4096) >> 13; }

template <int MODE>
__global__ __launch_bounds__(256) void kd(int32_t *out, int32_t seed, int iters) {
    constexpr double c13 = 12994.0 / 8192.0;
    double x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = (double)(seed + threadIdx.x * 8 + i);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (MODE == 4) x[i] = lift_f64(x[i], x[i] + 77.0, c13);
            else {  // int32 storage, converted around the f64 multiply
                const int32_t xi = (int32_t)x[i];
                x[i] = (double)(xi - (int32_t)__builtin_floor(__builtin_fma((double)(xi + 77), c13, 0.5)));
            }
        }
    }
    int32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += (int32_t)x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
__global__ __launch_bounds__(256) void k(int32_t *out, int32_t seed, int iters) {
    constexpr int32_t c = 12994;  // a lifting constant (compile-time, as in dwt.hip)
    int32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = seed + threadIdx.x * 8 + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (MODE == 0) x[i] = x[i] - fm64(x[i] + 77, c);
            else if constexpr (MODE == 1) x[i] = x[i] - fm24(x[i] + 77, c);
            else if constexpr (MODE == 3) x[i] = x[i] - fmdot(x[i] + 77, c);
            else if constexpr (MODE == 5) x[i] = x[i] - fm24s(x[i] + 77, c);
            else if constexpr (MODE == 6) x[i] = x[i] - fm32(x[i] + 77, c);
            else x[i] = (x[i] + 77) ^ (x[i] >> 3);
        }
    }
    int32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    const int nb = 4096, iters = 2048;
    int32_t *out;
    if (hipMalloc(&out, nb * 256 * 4) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[7] = {"v_mad_i64_i32 fixmul13", "24-bit fixmul13", "add/xor/shift chain", "dot2 fixmul13",
                            "f64 lift (fma + floor)", "one mad_i32_i24 (bounded)", "one mul_lo_u32 (bounded)"};
    for (int mode = 0; mode < 7; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0, 0);
            if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(nb), dim3(256), 0, 0, out, rep, iters);
            else if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(nb), dim3(256), 0, 0, out, rep, iters);
            else if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(nb), dim3(256), 0, 0, out, rep, iters);
            else if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(nb), dim3(256), 0, 0, out, rep, iters);
            else if (mode == 4) hipLaunchKernelGGL(kd<4>, dim3(nb), dim3(256), 0, 0, out, rep, iters);
            else if (mode == 5) hipLaunchKernelGGL(k<5>, dim3(nb), dim3(256), 0, 0, out, rep, iters);
            else hipLaunchKernelGGL(k<6>, dim3(nb), dim3(256), 0, 0, out, rep, iters);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            // lane-steps: nb * 256 lanes * iters * 8 chains; per SIMD (1024 SIMDs, 64 lanes / wave)
            const double wave_steps = (double)nb * 4 * iters * 8;
            int32_t h[4];
            hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
            if (rep) printf("%-26s %.3f ms  %.3f ns per wave-step per SIMD  (check %d %d)\n", names[mode], ms,
                            ms * 1e6 / (wave_steps / 1024), h[0], h[3]);
        }
    }
    return 0;
}
