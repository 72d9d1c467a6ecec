// Read-pattern probe: HBM read rate of window tilings over three 7680x4320
// int32 planes (the 8K level-0 DWT input), loads only (sum kept live).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int W = 7680, H = 4320, NC = 3;

// wave reads ROWS rows x (64 lanes x VB bytes), WPG waves per workgroup side by
// side (XW = 64*VB/4 columns per wave), workgroups tile the planes row-major.
template <int VB, int ROWS, int WPG, int HX = 0, int HY = 0>
__global__ __launch_bounds__(64 * WPG) void k_win(const int32_t *__restrict__ in, int32_t *out) {
    constexpr int XW = 64 * VB / 4 - 2 * HX;  // window step (columns)
    constexpr int YS = ROWS - 2 * HY;        // window step (rows)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wx = W / (XW * WPG);
    const int b = blockIdx.x;
    const int comp = b / (wx * (H / YS)), rem = b % (wx * (H / YS));
    const int ty = rem / wx, tx = rem % wx;
    const int x = min((tx * WPG + wave) * XW + lane * (VB / 4), W - VB / 4);
    const int y0 = min(ty * YS, H - ROWS);
    const int32_t *p = in + (size_t)comp * W * H + (size_t)y0 * W + x;
    int32_t acc = 0;
    if constexpr (VB == 16) {
        int4 v[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) v[r] = *(const int4 *)(p + (size_t)r * W);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc += v[r].x ^ v[r].y ^ v[r].z ^ v[r].w;
    } else if constexpr (VB == 8) {
        int2 v[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) v[r] = *(const int2 *)(p + (size_t)r * W);
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc += v[r].x ^ v[r].y;
    }
    if (acc == 0x7123457) out[threadIdx.x] = acc;
}

// same tiling through buffer loads (row offset in an SGPR, lane offset in a VGPR)
template <int ROWS, int HX, int HY>
__global__ __launch_bounds__(256) void k_buf(const int32_t *__restrict__ in, int32_t *out) {
    constexpr int XW = 128 - 2 * HX, YS = ROWS - 2 * HY, WPG = 4;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wx = W / (XW * WPG);
    const int b = blockIdx.x;
    const int comp = b / (wx * (H / YS)), rem = b % (wx * (H / YS));
    const int ty = rem / wx, tx = rem % wx;
    const int x = min((tx * WPG + wave) * XW + lane * 2, W - 2);
    const int y0 = min(ty * YS, H - ROWS);
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + (size_t)comp * W * H), 0, W * H * 4, 0x00020000);
    int32_t acc = 0;
    int32_t lo[ROWS], hi[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, x * 4, (y0 + r) * W * 4, 0);
        lo[r] = v[0]; hi[r] = v[1];
    }
#pragma unroll
    for (int r = 0; r < ROWS; ++r) acc += lo[r] ^ hi[r];
    if (acc == 0x7123457) out[threadIdx.x] = acc;
}

template <int ROWS, int HX, int HY>
void runb(const int32_t *in, int32_t *out, hipEvent_t e0, hipEvent_t e1, const char *name, int dirty = 0) {
    constexpr int XW = 128 - 2 * HX, YS = ROWS - 2 * HY;
    const int blocks = NC * (W / (XW * 4)) * (H / YS);
    float best = 1e9;
    for (int it = 0; it < 5; ++it) {
        if (dirty == 1) (void)hipMemsetAsync((void *)in, it, (size_t)NC * W * H * 4);  // predecessor writes the input
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_buf<ROWS, HX, HY>), dim3(blocks), dim3(256), 0, 0, in, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    printf("%-28s rows %2d halo %d,%d dirty %d: %7.1f us  %.2f TB/s\n", name, ROWS, HX, HY, dirty, best * 1e3,
           (double)NC * W * H * 4 / (best * 1e-3) / 1e12);
}

__global__ void k_lin(const int4 *__restrict__ in, int32_t *out, size_t n) {
    int32_t acc = 0;
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        int4 v = in[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x7123457) out[threadIdx.x] = acc;
}

template <int VB, int ROWS, int WPG, int HX = 0, int HY = 0>
void run(const int32_t *in, int32_t *out, hipEvent_t e0, hipEvent_t e1, const char *name) {
    constexpr int XW = 64 * VB / 4 - 2 * HX, YS = ROWS - 2 * HY;
    const int blocks = NC * (W / (XW * WPG)) * (H / YS);
    float best = 1e9;
    for (int it = 0; it < 5; ++it) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_win<VB, ROWS, WPG, HX, HY>), dim3(blocks), dim3(64 * WPG), 0, 0, in, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    printf("%-28s VB %2d rows %2d waves/WG %d halo %d,%d: %7.1f us  %.2f TB/s\n", name, VB, ROWS, WPG, HX, HY, best * 1e3,
           (double)NC * W * H * 4 / (best * 1e-3) / 1e12);
}

int main() {
    int32_t *in, *out;
    const size_t bytes = (size_t)NC * W * H * 4;
    if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&out, 4096) != hipSuccess) return 1;
    (void)hipMemset(in, 1, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int it = 0; it < 3; ++it) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_lin, dim3(256 * 32), dim3(256), 0, 0, (const int4 *)in, out, bytes / 16);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (it == 2) printf("linear int4 grid-stride      : %7.1f us  %.2f TB/s\n", ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    }
    run<8, 32, 4>(in, out, e0, e1, "dwt-like 128col");
    run<8, 32, 4, 4, 0>(in, out, e0, e1, "128col halo x");
    run<8, 32, 4, 0, 4>(in, out, e0, e1, "128col halo y");
    run<8, 32, 4, 4, 4>(in, out, e0, e1, "128col halo xy");
    run<8, 40, 4, 4, 4>(in, out, e0, e1, "128col halo xy");
    run<16, 32, 4, 4, 4>(in, out, e0, e1, "256col halo xy");
    run<16, 24, 4, 4, 4>(in, out, e0, e1, "256col halo xy");
    run<8, 32, 4, 2, 2>(in, out, e0, e1, "128col halo xy 5/3");
    runb<32, 0, 0>(in, out, e0, e1, "buffer 128col");
    runb<32, 4, 4>(in, out, e0, e1, "buffer 128col halo");
    runb<32, 4, 4>(in, out, e0, e1, "buffer 128col halo", 1);
    runb<32, 0, 0>(in, out, e0, e1, "buffer 128col", 1);
    return 0;
}
