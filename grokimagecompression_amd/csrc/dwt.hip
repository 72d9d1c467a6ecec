// dwt.hip -- 5/3 and 9/7 DWT levels for gfx950, register-resident lifting.
//
// One wavefront owns a window of 128 columns x R rows of one resolution of
// one tile-component.  Lane l holds the column pair (2l, 2l+1) of every
// window row in VGPRs: the low-pass sample in .x and the high-pass sample in
// .y (the window origin is shifted by the resolution's parity `cas`, so the
// pairing is the same for every job).  Hence
//   * vertical lifting is straight-line register arithmetic down each column
//     (no LDS, no barriers),
//   * horizontal lifting needs only the neighbouring lane's value, moved with
//     one DPP wave shift (v_mov_b32_dpp wave_shl:1 / wave_shr:1) per step,
//   * loads are one 8-byte access per lane per row (512 B per wave
//     instruction) and stores are one dword per lane per sub-band row.
// The window carries a lifting halo (2 samples for 5/3, 4 for 9/7) on each
// side, filled by whole-sample symmetric extension at the resolution edges.
// Lifting the symmetrically extended signal gives exactly the reference's
// per-step index clamping (dwt53.cpp:109-115 GROK_S_/D_ macros, dwt97.cpp,
// dwt.cpp:1392-1537 "2c * neighbour" edge terms): every step is symmetric in
// its two neighbours, so the extension stays symmetric step after step.
//
// Forward (WaveletForward.h:40-160): vertical lifting, then horizontal, then
// the four sub-bands are written in the Mallat layout (dwt_utils.cpp:84-127),
// LL to a separate buffer (next level's input).  Inverse (dwt.cpp:724-858,
// :1544-1738): the sub-bands are read back interleaved, horizontal lifting,
// then vertical, then the reconstructed resolution is stored.
//
// A launch covers one decomposition level of every tile-component (job table
// in HBM, grid.y = job), so a frame's DWT is numres-1 launches.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grk_device.h"
#include <stdlib.h>

namespace grkgpu {

constexpr int DWT_WIN = 128;   // window columns per wavefront (64 lanes x 2)
constexpr int DWT_WAVES = 4;   // wavefronts (independent windows) per workgroup

template <bool IRREV, int TH_>
struct DwtGeo {
    static constexpr int HALO = IRREV ? 4 : 2;
    static constexpr int CW = DWT_WIN - 2 * HALO;  // core columns per window
    static constexpr int TH = TH_;                 // core rows per window
    static constexpr int R = TH + 2 * HALO;        // window rows
};

__device__ __forceinline__ int32_t fixmul13(int32_t a, int32_t b) {
    return (int32_t)(((int64_t)a * (int64_t)b + 4096) >> 13);
}

// lane l receives lane l+1's value (wave_shl:1) / lane l-1's (wave_shr:1)
__device__ __forceinline__ int32_t from_next(int32_t v) { return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xf, 0xf, false); }
__device__ __forceinline__ int32_t from_prev(int32_t v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false); }

// Whole-sample symmetric extension of index p into [0, n).  Exact for every
// position that can reach a kept sample (|p - edge| <= halo); positions
// further out only need a valid address.
__device__ __forceinline__ int mirror_idx(int p, int n) {
    if (n > 4) {
        p = p < 0 ? -p : p;
        p = p >= n ? 2 * (n - 1) - p : p;
    } else {
        for (int i = 0; i < 8 && (p < 0 || p >= n); ++i) p = p < 0 ? -p : 2 * (n - 1) - p;
    }
    return p < 0 ? 0 : (p >= n ? n - 1 : p);
}

// buffer resources: 32-bit offsets (row offset in an SGPR, lane offset in a
// VGPR); an offset past num_records drops a store, which is how lanes
// outside the resolution are masked without branching.
using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr int OOB = 0x7ffffff0;
__device__ __forceinline__ rsrc_t mkbuf(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ int32_t ld32(rsrc_t r, int voff, int soff) {
    return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}
__device__ __forceinline__ void st32(int32_t v, rsrc_t r, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, r, voff, soff, 0);
}

// ---------------------------------------------------------------------------
// 1-D lifting kernels on register arrays.  Interleaved position k: even = low
// pass, odd = high pass.  Positions near the array ends come out wrong (the
// halo); the callers only keep the core.
// ---------------------------------------------------------------------------
template <int OP> __device__ __forceinline__ int32_t lift(int32_t t, int32_t l, int32_t r) {
    if constexpr (OP == 0) return t - ((l + r) >> 1);                 // 5/3 fwd, high
    else if constexpr (OP == 1) return t + ((l + r + 2) >> 2);        // 5/3 fwd, low
    else if constexpr (OP == 2) return t - fixmul13(l + r, 12994);    // 9/7 fwd 1 (high)
    else if constexpr (OP == 3) return t - fixmul13(l + r, 434);      // 9/7 fwd 2 (low)
    else if constexpr (OP == 4) return t + fixmul13(l + r, 7233);     // 9/7 fwd 3 (high)
    else if constexpr (OP == 5) return t + fixmul13(l + r, 3633);     // 9/7 fwd 4 (low)
    else if constexpr (OP == 6) return t - ((l + r + 2) >> 2);        // 5/3 inv, low
    else if constexpr (OP == 7) return t + ((l + r) >> 1);            // 5/3 inv, high
    else {                                                            // 9/7 inv (float, no FMA)
        constexpr float c = OP == 8 ? -0.443506852f : OP == 9 ? -0.882911075f : OP == 10 ? 0.052980118f : 1.586134342f;
        return __float_as_int(__fadd_rn(__int_as_float(t), __fmul_rn(__fadd_rn(__int_as_float(l), __int_as_float(r)), c)));
    }
}

// vertical step over rows [lo, hi) of parity PAR (0 low, 1 high)
template <int OP, int PAR, int R>
__device__ __forceinline__ void vstep(int32_t (&v)[R]) {
#pragma unroll
    for (int k = PAR == 0 ? 2 : 1; k + 1 < R; k += 2) v[k] = lift<OP>(v[k], v[k - 1], v[k + 1]);
}

// ---------------------------------------------------------------------------
// forward level
// ---------------------------------------------------------------------------

template <bool IRREV, int TH>
__global__ __launch_bounds__(64 * DWT_WAVES) void k_dwt_fwd(const DwtJob *__restrict__ jobs) {
    using G = DwtGeo<IRREV, TH>;
    constexpr int R = G::R;
    const DwtJob J = jobs[blockIdx.y];
    const int tile = blockIdx.x * DWT_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (tile >= J.ntiles) return;
    const int lane = threadIdx.x & 63;
    const int tx = tile % J.tiles_x, ty = tile / J.tiles_x;
    const int rw = J.rw, rh = J.rh, casx = J.casx, casy = J.casy;
    const int xw = tx * G::CW - casx - G::HALO;  // window column origin (parity of casx)
    const int yw = ty * G::TH - casy - G::HALO;
    const int gx0 = xw + 2 * lane, gx1 = gx0 + 1;

    int32_t lo[R], hi[R];  // column 2l (low pass) and 2l+1 (high pass)
    {
        const rsrc_t in = mkbuf(J.in, J.in_bytes);
        const int st = (int)J.in_stride * 4;
        const bool vec = (casx | (J.in_stride & 1)) == 0 && xw >= 0 && xw + DWT_WIN <= rw;  // wave-uniform
        if (vec) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const auto p = __builtin_amdgcn_raw_buffer_load_b64(in, gx0 * 4, mirror_idx(yw + r, rh) * st, 0);
                lo[r] = (int32_t)p[0]; hi[r] = (int32_t)p[1];
            }
        } else {
            const int o0 = mirror_idx(gx0, rw) * 4, o1 = mirror_idx(gx1, rw) * 4;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int so = mirror_idx(yw + r, rh) * st;
                lo[r] = ld32(in, o0, so); hi[r] = ld32(in, o1, so);
            }
        }
    }
    // vertical (position = window row; even rows are low pass)
    if (rh > 1) {
        if constexpr (!IRREV) {
            vstep<0, 1>(lo); vstep<0, 1>(hi);
            vstep<1, 0>(lo); vstep<1, 0>(hi);
        } else {
            vstep<2, 1>(lo); vstep<2, 1>(hi);
            vstep<3, 0>(lo); vstep<3, 0>(hi);
            vstep<4, 1>(lo); vstep<4, 1>(hi);
            vstep<5, 0>(lo); vstep<5, 0>(hi);
        }
    } else if (!IRREV && casy) {  // single row, odd origin: S0 <<= 1 (dwt53.cpp:161)
#pragma unroll
        for (int r = 0; r < R; ++r) { lo[r] = (int32_t)((uint32_t)lo[r] << 1); hi[r] = (int32_t)((uint32_t)hi[r] << 1); }
    }
    // horizontal on the core rows, then store
    const int corel = G::HALO / 2, coreh = corel + G::CW / 2;
    const bool lane_core = lane >= corel && lane < coreh;
    const bool okx0 = lane_core && gx0 >= 0 && gx0 < rw, okx1 = lane_core && gx1 >= 0 && gx1 < rw;
    const int vl = okx0 ? ((gx0 - casx) >> 1) * 4 : OOB;                  // low-pass column -> L bands
    const int vh = okx1 ? (J.snx + ((gx1 - 1 + casx) >> 1)) * 4 : OOB;     // high-pass column -> H bands
    const rsrc_t outb = mkbuf(J.out, J.out_bytes), bandb = mkbuf(J.bands, J.bands_bytes);
    const int ost = (int)J.out_stride * 4, bst = (int)J.bands_stride * 4;
#pragma unroll
    for (int r = G::HALO; r < G::HALO + G::TH; ++r) {
        int32_t L = lo[r], H = hi[r];
        if (IRREV && rh > 1) {
            const int32_t k = (r & 1) ? 5039 : 6659;  // vertical scale: high rows K/2, low rows 1/K
            L = fixmul13(L, k); H = fixmul13(H, k);
        }
        if (rw > 1) {
            if constexpr (!IRREV) {
                H = lift<0>(H, L, from_next(L));
                L = lift<1>(L, from_prev(H), H);
            } else {
                H = lift<2>(H, L, from_next(L));
                L = lift<3>(L, from_prev(H), H);
                H = lift<4>(H, L, from_next(L));
                L = lift<5>(L, from_prev(H), H);
                H = fixmul13(H, 5039);
                L = fixmul13(L, 6659);
            }
        } else if (!IRREV && casx) {
            L = (int32_t)((uint32_t)L << 1);
            H = (int32_t)((uint32_t)H << 1);
        }
        const int gy = yw + r;
        if (gy < 0 || gy >= rh) continue;
        if ((r & 1) == 0) {  // low row -> LL | HL
            const int iy = (gy - casy) >> 1;
            st32(L, outb, vl, iy * ost);
            st32(H, bandb, vh, iy * bst);
        } else {             // high row -> LH | HH
            const int so = (J.sny + ((gy - 1 + casy) >> 1)) * bst;
            st32(L, bandb, vl, so);
            st32(H, bandb, vh, so);
        }
    }
}

// ---------------------------------------------------------------------------
// inverse level
// ---------------------------------------------------------------------------
template <bool IRREV, int TH>
__global__ __launch_bounds__(64 * DWT_WAVES) void k_dwt_inv(const DwtJob *__restrict__ jobs) {
    using G = DwtGeo<IRREV, TH>;
    constexpr int R = G::R;
    const DwtJob J = jobs[blockIdx.y];
    const int tile = blockIdx.x * DWT_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (tile >= J.ntiles) return;
    const int lane = threadIdx.x & 63;
    const int tx = tile % J.tiles_x, ty = tile / J.tiles_x;
    const int rw = J.rw, rh = J.rh, casx = J.casx, casy = J.casy;
    const int xw = tx * G::CW - casx - G::HALO;
    const int yw = ty * G::TH - casy - G::HALO;
    const int gx0 = xw + 2 * lane, gx1 = gx0 + 1;

    int32_t lo[R], hi[R];
    {
        // mirroring keeps parity: column 2l is always a low-pass column, 2l+1
        // high-pass; even window rows are low-pass rows
        const int ix0 = ((mirror_idx(gx0, rw) - casx) >> 1) * 4;
        const int ix1 = (J.snx + ((mirror_idx(gx1, rw) - 1 + casx) >> 1)) * 4;
        const rsrc_t llb = mkbuf(J.in, J.in_bytes), cb = mkbuf(J.coef, J.coef_bytes);
        const int lst = (int)J.in_stride * 4, cst = (int)J.coef_stride * 4;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int my = mirror_idx(yw + r, rh);
            if ((r & 1) == 0) {
                const int iy = (my - casy) >> 1;
                lo[r] = ld32(llb, ix0, iy * lst);
                hi[r] = ld32(cb, ix1, iy * cst);
            } else {
                const int so = (J.sny + ((my - 1 + casy) >> 1)) * cst;
                lo[r] = ld32(cb, ix0, so);
                hi[r] = ld32(cb, ix1, so);
            }
        }
    }
    // horizontal on every window row (the vertical pass needs the halo rows)
    if (rw > 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            int32_t L = lo[r], H = hi[r];
            if constexpr (!IRREV) {
                L = lift<6>(L, from_prev(H), H);
                H = lift<7>(H, L, from_next(L));
            } else {
                L = __float_as_int(__fmul_rn(__int_as_float(L), 1.230174105f));
                H = __float_as_int(__fmul_rn(__int_as_float(H), 1.625732422f));
                L = lift<8>(L, from_prev(H), H);
                H = lift<9>(H, L, from_next(L));
                L = lift<10>(L, from_prev(H), H);
                H = lift<11>(H, L, from_next(L));
            }
            lo[r] = L; hi[r] = H;
        }
    } else if (!IRREV && casx) {  // single column, odd origin: S0 /= 2 (dwt.cpp:341)
#pragma unroll
        for (int r = 0; r < R; ++r) { lo[r] /= 2; hi[r] /= 2; }
    }
    // vertical
    if (rh > 1) {
        if constexpr (!IRREV) {
            vstep<6, 0>(lo); vstep<6, 0>(hi);
            vstep<7, 1>(lo); vstep<7, 1>(hi);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const float s = (r & 1) ? 1.625732422f : 1.230174105f;
                lo[r] = __float_as_int(__fmul_rn(__int_as_float(lo[r]), s));
                hi[r] = __float_as_int(__fmul_rn(__int_as_float(hi[r]), s));
            }
            vstep<8, 0>(lo); vstep<8, 0>(hi);
            vstep<9, 1>(lo); vstep<9, 1>(hi);
            vstep<10, 0>(lo); vstep<10, 0>(hi);
            vstep<11, 1>(lo); vstep<11, 1>(hi);
        }
    } else if (!IRREV && casy) {
#pragma unroll
        for (int r = 0; r < R; ++r) { lo[r] /= 2; hi[r] /= 2; }
    }
    const int corel = G::HALO / 2, coreh = corel + G::CW / 2;
    if (lane < corel || lane >= coreh) return;
    const bool okx0 = gx0 >= 0 && gx0 < rw, okx1 = gx1 >= 0 && gx1 < rw;
    const rsrc_t ob = mkbuf(J.out, J.out_bytes);
    const int ost = (int)J.out_stride * 4;
    const bool vec = (casx | (J.out_stride & 1)) == 0 && xw >= 0 && xw + DWT_WIN <= rw;  // wave-uniform
    const int v0 = okx0 ? gx0 * 4 : OOB, v1 = okx1 ? gx1 * 4 : OOB;
#pragma unroll
    for (int r = G::HALO; r < G::HALO + G::TH; ++r) {
        const int gy = yw + r;
        if (gy < 0 || gy >= rh) continue;
        if (vec) {
            const __attribute__((ext_vector_type(2))) uint32_t p = {(uint32_t)lo[r], (uint32_t)hi[r]};
            __builtin_amdgcn_raw_buffer_store_b64(p, ob, v0, gy * ost, 0);
        } else {
            st32(lo[r], ob, v0, gy * ost);
            st32(hi[r], ob, v1, gy * ost);
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Rows per window: tall windows for big levels (less halo re-read), short
// ones for small levels (more wavefronts, shorter per-wave chains).
// GRKGPU_DWT_TH overrides the big-level choice (8/16/24/32).
static int dwt_th_big(int irrev) {
    static int th = [] {
        const char *e = getenv("GRKGPU_DWT_TH");
        int v = e ? atoi(e) : 0;
        return (v == 8 || v == 16 || v == 24 || v == 32) ? v : 0;
    }();
    return th ? th : (irrev ? 24 : 32);
}

int dwt_pick_th(int irrev, uint64_t level_samples) {
    return level_samples >= (1u << 22) ? dwt_th_big(irrev) : 8;
}

void dwt_job_tiles(int irrev, int th, int rw, int rh, int casx, int casy, int32_t *tiles_x, int32_t *ntiles) {
    const int cw = irrev ? DwtGeo<true, 8>::CW : DwtGeo<false, 8>::CW;
    const int tx = (rw + casx + cw - 1) / cw, ty = (rh + casy + th - 1) / th;
    *tiles_x = tx;
    *ntiles = tx * ty;
}

template <int TH>
static void launch_th(const DwtJob *jobs, dim3 grid, dim3 block, int irrev, int inverse, hipStream_t s) {
    if (!inverse) {
        if (irrev) hipLaunchKernelGGL((k_dwt_fwd<true, TH>), grid, block, 0, s, jobs);
        else hipLaunchKernelGGL((k_dwt_fwd<false, TH>), grid, block, 0, s, jobs);
    } else {
        if (irrev) hipLaunchKernelGGL((k_dwt_inv<true, TH>), grid, block, 0, s, jobs);
        else hipLaunchKernelGGL((k_dwt_inv<false, TH>), grid, block, 0, s, jobs);
    }
}

hipError_t launch_dwt_jobs(const DwtJob *jobs_dev, uint32_t njobs, uint32_t max_tiles, int th, int irrev,
                           int inverse, hipStream_t s) {
    if (!njobs || !max_tiles) return hipSuccess;
    dim3 grid((max_tiles + DWT_WAVES - 1) / DWT_WAVES, njobs), block(64 * DWT_WAVES);
    switch (th) {
        case 8: launch_th<8>(jobs_dev, grid, block, irrev, inverse, s); break;
        case 16: launch_th<16>(jobs_dev, grid, block, irrev, inverse, s); break;
        case 24: launch_th<24>(jobs_dev, grid, block, irrev, inverse, s); break;
        case 32: launch_th<32>(jobs_dev, grid, block, irrev, inverse, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace grkgpu
