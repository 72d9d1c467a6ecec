// Latency calibration probes for the serial T1 lanes (not product code).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_valu_chain(uint32_t *out, uint32_t n, uint32_t seed) {
    uint32_t x = seed + threadIdx.x;
    for (uint32_t i = 0; i < n; ++i) {
        x = x * 2654435761u + 12345u;
        x ^= x >> 13;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_lds_chain(uint32_t *out, uint32_t n, uint32_t seed) {
    __shared__ uint32_t t[1024];
    for (uint32_t k = threadIdx.x; k < 1024; k += blockDim.x) t[k] = (k * 7 + 3) & 1023;
    __syncthreads();
    uint32_t x = seed & 1023;
    for (uint32_t i = 0; i < n; ++i) x = t[x];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_lds_rw_chain(uint32_t *out, uint32_t n, uint32_t seed) {
    __shared__ uint32_t t[64 * 33];
    uint32_t *m = t + threadIdx.x * 33;
    for (uint32_t k = 0; k < 32; ++k) m[k] = k;
    uint32_t x = seed & 31;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t v = m[x];
        m[x] = v + 1;
        x = (v * 5 + 1) & 31;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_branchy(uint32_t *out, uint32_t n, uint32_t seed) {
    uint32_t x = seed + threadIdx.x * 77, a = 0, b = 0;
    for (uint32_t i = 0; i < n; ++i) {
        x = x * 1103515245u + 12345u;
        if (x & 0x10000) { a += x >> 3; } else { b ^= x; }
        if ((x & 0x300000) == 0) { a = a * 3 + b; }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b;
}

__global__ void k_gload_chain(const uint32_t *tab, uint32_t *out, uint32_t n) {
    uint32_t x = threadIdx.x;
    for (uint32_t i = 0; i < n; ++i) x = tab[x];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

extern "C" int probe(int which, uint32_t *out, const uint32_t *tab, uint32_t n, int blocks, int threads, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (which) {
        case 0: hipLaunchKernelGGL(k_valu_chain, dim3(blocks), dim3(threads), 0, s, out, n, 1u); break;
        case 1: hipLaunchKernelGGL(k_lds_chain, dim3(blocks), dim3(threads), 0, s, out, n, 1u); break;
        case 2: hipLaunchKernelGGL(k_lds_rw_chain, dim3(blocks), dim3(threads), 0, s, out, n, 1u); break;
        case 3: hipLaunchKernelGGL(k_branchy, dim3(blocks), dim3(threads), 0, s, out, n, 1u); break;
        case 4: hipLaunchKernelGGL(k_gload_chain, dim3(blocks), dim3(threads), 0, s, tab, out, n); break;
    }
    return (int)hipGetLastError();
}
