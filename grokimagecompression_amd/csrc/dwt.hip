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

#include <algorithm>
#include <type_traits>

#include "grk_device.h"

namespace grkgpu {

constexpr int DWT_WIN = 128;   // window columns per wavefront (64 lanes x 2)
constexpr int DWT_WAVES = 4;   // wavefronts (independent windows) per workgroup

template <bool IRREV, int TH_, int WIN = DWT_WIN>
struct DwtGeo {
    static constexpr int HALO = IRREV ? 4 : 2;
    static constexpr int CW = WIN - 2 * HALO;      // core columns per window
    static constexpr int TH = TH_;                 // core rows per window
    static constexpr int R = TH + 2 * HALO;        // window rows
};

// One v_mad_i64_i32 + v_alignbit.  The 64-bit multiply issues at about a
// quarter of the 32-bit rate, and the forward 9/7 levels are VALU-issue-bound
// (DESIGN.md §3), but the exact split into two 24-bit multiplies
// (ah b + ((al b + 4096) >> 13), scripts/mulrate.hip) costs more: the 24-bit
// multiplies issue at half rate (8K frame: 252 vs 216 us).
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
template <int AUX = 0>
__device__ __forceinline__ void st32(int32_t v, rsrc_t r, int voff, int soff) {
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, r, voff, soff, AUX);
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

// The forward 9/7 lifting held in f64 registers: every value is an integer
// below 2^31 in magnitude, s c / 2^13 + 1/2 (s = l + r, c < 2^14) is exact in
// a double, so floor(fma(s, c / 8192, 1/2)) is fixmul13(s, c) bit for bit,
// and a subtracted step t - floor(.) is the reference's int32 difference (no
// wrap below 2^31).  An f64 FMA + floor issue at the full VALU rate where
// v_mad_i64_i32 issues at about a quarter (scripts/mulrate.hip).
__device__ __forceinline__ double fixd(double s, double c13) { return __builtin_floor(__builtin_fma(s, c13, 0.5)); }
template <int OP> __device__ __forceinline__ double liftd(double t, double l, double r) {
    if constexpr (OP == 2) return t - fixd(l + r, 12994.0 / 8192.0);
    else if constexpr (OP == 3) return t - fixd(l + r, 434.0 / 8192.0);
    else if constexpr (OP == 4) return t + fixd(l + r, 7233.0 / 8192.0);
    else return t + fixd(l + r, 3633.0 / 8192.0);
}
__device__ __forceinline__ double from_next(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)from_next((int32_t)(uint32_t)b), hi = (uint32_t)from_next((int32_t)(uint32_t)(b >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double from_prev(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)from_prev((int32_t)(uint32_t)b), hi = (uint32_t)from_prev((int32_t)(uint32_t)(b >> 32));
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// value-type dispatch for the forward 9/7 (int32: v_mad_i64_i32, double: f64)
template <int OP> __device__ __forceinline__ int32_t liftv(int32_t t, int32_t l, int32_t r) { return lift<OP>(t, l, r); }
template <int OP> __device__ __forceinline__ double liftv(double t, double l, double r) { return liftd<OP>(t, l, r); }
__device__ __forceinline__ int32_t scalev(int32_t v, int32_t k) { return fixmul13(v, k); }
__device__ __forceinline__ double scalev(double v, int32_t k) { return fixd(v, (double)k / 8192.0); }
__device__ __forceinline__ int32_t to_i32(int32_t v) { return v; }
__device__ __forceinline__ int32_t to_i32(double v) { return (int32_t)v; }

// vertical lifting step S (0-based) over the window rows of parity PAR (0
// low, 1 high).  The rows a window keeps are [H, R - H), H = the number of
// steps (the halo), so step S only needs rows [S + 1, R - 1 - S): the rows
// further out feed nothing that is kept.
template <int OP, int PAR, int S, int R, typename T>
__device__ __forceinline__ void vstep(T (&v)[R]) {
    constexpr int K0 = ((S + 1) & 1) == PAR ? S + 1 : S + 2;
#pragma unroll
    for (int k = K0; k + 1 + S < R; k += 2) v[k] = liftv<OP>(v[k], v[k - 1], v[k + 1]);
}

// Linear workgroup id -> position in an order where each XCD (workgroups are
// dealt round-robin to the 8 XCDs by linear id) owns one contiguous run.
__device__ __forceinline__ int xcd_remap(int L, int total) {
    const int q = total >> 3, r = total & 7, x = L & 7, k = L >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// Workgroup wg of a pair kernel (row-major over ntx x nty) -> (tx, ty) in
// groups of G columns walked top to bottom (G = 0: row-major): a workgroup's
// vertical neighbour then runs G workgroups later on the same XCD, while the
// rows both read are still in its L2.
__device__ __forceinline__ void group_order(int wg, int ntx, int nty, int G, int &tx, int &ty) {
    if (G <= 0 || G >= ntx) { tx = wg % ntx; ty = wg / ntx; return; }
    const int full = ntx / G, per = G * nty, g = wg / per;
    if (g < full) {
        const int rem = wg - g * per;
        ty = rem / G; tx = g * G + rem % G;
    } else {
        const int rem = wg - full * per, gw = ntx - full * G;
        ty = rem / gw; tx = full * G + rem % gw;
    }
}

// Window of this wavefront.  The launch is a 2-D grid (x: workgroups of one
// job, y: job); `lay` bit 0 remaps the linear workgroup id so that each XCD
// (workgroups are dealt round-robin to the 8 XCDs) receives a contiguous run
// of workgroups -- neighbouring windows, whose halo rows and columns overlap,
// then share one L2; bit 1 stacks the 4 wavefronts of a workgroup vertically
// (same column window, 4 consecutive row windows) instead of horizontally;
// bit 2 orders the workgroups job-minor, so the same window of every job
// (the components of a tile, which the fused level 0 reads from the same
// image planes) is processed at the same time on the same XCD.
// Returns false for a wavefront past the job's windows.
__device__ __forceinline__ bool dwt_window(const DwtJob *__restrict__ jobs, int lay, int th, DwtJob &J, int &tx,
                                           int &ty) {
    const int gx = gridDim.x;
    int L = blockIdx.y * gx + blockIdx.x;
    if (lay & 1) L = xcd_remap(L, gx * gridDim.y);
    int wg, job;
    if (lay & 4) { job = L % (int)gridDim.y; wg = L / (int)gridDim.y; }  // job-minor: same window of every job adjacent
    else { wg = L % gx; job = L / gx; }
    J = jobs[job];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (lay & 2) {
        tx = wg % J.tiles_x;
        ty = (wg / J.tiles_x) * DWT_WAVES + w;
    } else {
        const int tile = wg * DWT_WAVES + w;
        tx = tile % J.tiles_x;
        ty = tile / J.tiles_x;
    }
    const bool ok = ty < J.win_ny;
    tx += J.win_x0;
    ty += J.win_y0;
    return ok;
}

// ---------------------------------------------------------------------------
// forward level
// ---------------------------------------------------------------------------

// Image samples of type S as the fused level 0 reads them: a column pair
// (2 adjacent samples, one load: 8 / 4 / 2 bytes) or one sample, widened to
// int32 (unsigned types zero-, signed types sign-extended).
template <typename S> struct Smp;
template <> struct Smp<int32_t> {
    static constexpr int B = 4;
    static __device__ __forceinline__ void pair(rsrc_t r, int vo, int so, int32_t &a, int32_t &b) {
        const auto p = __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0);
        a = (int32_t)p[0]; b = (int32_t)p[1];
    }
    static __device__ __forceinline__ int32_t one(rsrc_t r, int vo, int so) { return ld32(r, vo, so); }
};
template <> struct Smp<uint16_t> {
    static constexpr int B = 2;
    static __device__ __forceinline__ void pair(rsrc_t r, int vo, int so, int32_t &a, int32_t &b) {
        const uint32_t p = __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0);
        a = (int32_t)(p & 0xffffu); b = (int32_t)(p >> 16);
    }
    static __device__ __forceinline__ int32_t one(rsrc_t r, int vo, int so) {
        return (int32_t)(uint16_t)__builtin_amdgcn_raw_buffer_load_b16(r, vo, so, 0);
    }
};
template <> struct Smp<uint8_t> {
    static constexpr int B = 1;
    static __device__ __forceinline__ void pair(rsrc_t r, int vo, int so, int32_t &a, int32_t &b) {
        const uint32_t p = (uint16_t)__builtin_amdgcn_raw_buffer_load_b16(r, vo, so, 0);
        a = (int32_t)(p & 0xffu); b = (int32_t)(p >> 8);
    }
    static __device__ __forceinline__ int32_t one(rsrc_t r, int vo, int so) {
        return (int32_t)(uint8_t)__builtin_amdgcn_raw_buffer_load_b8(r, vo, so, 0);
    }
};

// Window rows of a fused level 0 for a component outside an MCT triple: the
// DC shift (TileProcessor.cpp:1449-1471; 9/7: then << 11) applied as the
// image plane is read.  (MCT triples take k_dwt_fwd_mct3.)
template <bool IRREV, int R, typename S>
__device__ __forceinline__ void fused_load(const DwtJob &J, int32_t (&lo)[R], int32_t (&hi)[R], int xw, int yw,
                                           int gx0, int gx1) {
    const int rw = J.rw, rh = J.rh;
    const int st = (int)J.src_stride * Smp<S>::B;
    const rsrc_t p0 = mkbuf(J.src[0], J.src_bytes);
    const bool vec = J.src_vec && J.casx == 0 && xw >= 0 && xw + DWT_WIN <= rw;  // wave-uniform
    const bool rows_in = yw >= 0 && yw + R <= rh;
    const int o0 = mirror_idx(gx0, rw) * Smp<S>::B, o1 = mirror_idx(gx1, rw) * Smp<S>::B;
    const int32_t sh = J.shift[0];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int so = (rows_in ? yw + r : mirror_idx(yw + r, rh)) * st;
        int32_t a0, a1;
        if (vec) {
            Smp<S>::pair(p0, gx0 * Smp<S>::B, so, a0, a1);
        } else {
            a0 = Smp<S>::one(p0, o0, so); a1 = Smp<S>::one(p0, o1, so);
        }
        lo[r] = IRREV ? (int32_t)((uint32_t)(a0 - sh) << 11) : a0 - sh;
        hi[r] = IRREV ? (int32_t)((uint32_t)(a1 - sh) << 11) : a1 - sh;
    }
}

// Vertical lifting of a window (position = window row; even rows are low pass).
template <bool IRREV, int R, typename T = int32_t>
__device__ __forceinline__ void fwd_vertical(T (&lo)[R], T (&hi)[R], int rh, int casy) {
    if (rh > 1) {
        if constexpr (!IRREV) {
            vstep<0, 1, 0>(lo); vstep<0, 1, 0>(hi);
            vstep<1, 0, 1>(lo); vstep<1, 0, 1>(hi);
        } else {
            vstep<2, 1, 0>(lo); vstep<2, 1, 0>(hi);
            vstep<3, 0, 1>(lo); vstep<3, 0, 1>(hi);
            vstep<4, 1, 2>(lo); vstep<4, 1, 2>(hi);
            vstep<5, 0, 3>(lo); vstep<5, 0, 3>(hi);
        }
    } else if constexpr (!IRREV) {
        if (casy) {  // single row, odd origin: S0 <<= 1 (dwt53.cpp:161)
#pragma unroll
            for (int r = 0; r < R; ++r) { lo[r] = (int32_t)((uint32_t)lo[r] << 1); hi[r] = (int32_t)((uint32_t)hi[r] << 1); }
        }
    }
}

// Horizontal lifting of the window's core rows, then the stores into the
// LL buffer and the Mallat bands.
template <bool IRREV, int TH, int WIN = DWT_WIN, typename T = int32_t>
__device__ __forceinline__ void fwd_horizontal_store(const DwtJob &J, T (&lo)[DwtGeo<IRREV, TH>::R],
                                                     T (&hi)[DwtGeo<IRREV, TH>::R], int ty, int yw, int gx0,
                                                     int lane) {
    using G = DwtGeo<IRREV, TH, WIN>;
    const int rw = J.rw, rh = J.rh, casx = J.casx, casy = J.casy;
    const int gx1 = gx0 + 1;
    const int corel = G::HALO / 2, coreh = corel + G::CW / 2;
    const bool lane_core = lane >= corel && lane < coreh;
    const bool okx0 = lane_core && gx0 >= 0 && gx0 < rw, okx1 = lane_core && gx1 >= 0 && gx1 < rw;
    const int vl = okx0 ? ((gx0 - casx) >> 1) * 4 : OOB;                  // low-pass column -> L bands
    const int vh = okx1 ? (J.snx + ((gx1 - 1 + casx) >> 1)) * 4 : OOB;     // high-pass column -> H bands
    const rsrc_t outb = mkbuf(J.out, J.out_bytes), bandb = mkbuf(J.bands, J.bands_bytes);
    const int ost = (int)J.out_stride * 4, bst = (int)J.bands_stride * 4;
    // Output rows: window row r (even: low pass) of gy = yw + r goes to row
    // lbase + r/2 of the L bands (LL | HL), odd r to row hbase + (r-1)/2 of the
    // H bands (LH | HH); both bases are scalars (ty * TH, HALO even).
    const int lbase = ty * (G::TH / 2) - casy - G::HALO / 2;
    const int hbase = J.sny + ty * (G::TH / 2) - G::HALO / 2;
    const int ylo = yw + G::HALO, yhi = ylo + G::TH;  // core rows [ylo, yhi)
    const bool rows_all = ylo >= 0 && yhi <= rh;      // wave-uniform: no per-row checks
#pragma unroll
    for (int r = G::HALO; r < G::HALO + G::TH; ++r) {
        T L = lo[r], H = hi[r];
        if (IRREV && rh > 1) {
            const int32_t k = (r & 1) ? 5039 : 6659;  // vertical scale: high rows K/2, low rows 1/K
            L = scalev(L, k); H = scalev(H, k);
        }
        if (rw > 1) {
            if constexpr (!IRREV) {
                H = lift<0>(H, L, from_next(L));
                L = lift<1>(L, from_prev(H), H);
            } else {
                H = liftv<2>(H, L, from_next(L));
                L = liftv<3>(L, from_prev(H), H);
                H = liftv<4>(H, L, from_next(L));
                L = liftv<5>(L, from_prev(H), H);
                H = scalev(H, 5039);
                L = scalev(L, 6659);
            }
        } else if constexpr (!IRREV) {
            if (casx) {
                L = (int32_t)((uint32_t)L << 1);
                H = (int32_t)((uint32_t)H << 1);
            }
        }
        if (!rows_all) {
            const int gy = yw + r;
            if (gy < 0 || gy >= rh) continue;
        }
        if ((r & 1) == 0) {  // low row -> LL | HL
            const int iy = lbase + r / 2;
            st32(to_i32(L), outb, vl, iy * ost);
            st32(to_i32(H), bandb, vh, iy * bst);
        } else {             // high row -> LH | HH
            const int so = (hbase + (r - 1) / 2) * bst;
            st32(to_i32(L), bandb, vl, so);
            st32(to_i32(H), bandb, vh, so);
        }
    }
}

// FUSED: 0 = reads `in`; 1 = DC shift (+ MCT for a component of an MCT
// triple) fused into the loads (fused_load: 3 planes per MCT component).
template <bool IRREV, int TH, int FUSED = 0, typename S = int32_t, typename T = int32_t>
__global__ __launch_bounds__(64 * DWT_WAVES) void k_dwt_fwd(const DwtJob *__restrict__ jobs, int lay) {
    using G = DwtGeo<IRREV, TH>;
    constexpr int R = G::R;
    DwtJob J;
    int tx, ty;
    if (!dwt_window(jobs, lay, TH, J, tx, ty)) return;
    const int lane = threadIdx.x & 63;
    const int rw = J.rw, rh = J.rh, casx = J.casx, casy = J.casy;
    const int xw = tx * G::CW - casx - G::HALO;  // window column origin (parity of casx)
    const int yw = ty * G::TH - casy - G::HALO;
    const int gx0 = xw + 2 * lane, gx1 = gx0 + 1;

    T lo[R], hi[R];  // column 2l (low pass) and 2l+1 (high pass)
    if constexpr (FUSED == 1) {
        static_assert(sizeof(T) == 4, "fused loads: int32 lifting");
        fused_load<IRREV, R, S>(J, lo, hi, xw, yw, gx0, gx1);
    } else {
        const rsrc_t in = mkbuf(J.in, J.in_bytes);
        const int st = (int)J.in_stride * 4;
        const bool vec = (casx | (J.in_stride & 1)) == 0 && xw >= 0 && xw + DWT_WIN <= rw;  // wave-uniform
        const bool rows_in = yw >= 0 && yw + R <= rh;  // no row mirroring: offsets are base + r * stride
        if (vec && rows_in) {
            const int base = yw * st;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const auto p = __builtin_amdgcn_raw_buffer_load_b64(in, gx0 * 4, base + r * st, 0);
                lo[r] = (T)(int32_t)p[0]; hi[r] = (T)(int32_t)p[1];
            }
        } else if (vec) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const auto p = __builtin_amdgcn_raw_buffer_load_b64(in, gx0 * 4, mirror_idx(yw + r, rh) * st, 0);
                lo[r] = (T)(int32_t)p[0]; hi[r] = (T)(int32_t)p[1];
            }
        } else {
            const int o0 = mirror_idx(gx0, rw) * 4, o1 = mirror_idx(gx1, rw) * 4;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int so = mirror_idx(yw + r, rh) * st;
                lo[r] = (T)ld32(in, o0, so); hi[r] = (T)ld32(in, o1, so);
            }
        }
    }
    fwd_vertical<IRREV, R, T>(lo, hi, rh, casy);
    fwd_horizontal_store<IRREV, TH, DWT_WIN, T>(J, lo, hi, ty, yw, gx0, lane);
}

// Forward level 0 of an MCT component triple in ONE wavefront per window:
// the three image planes are read once (8-byte loads), the DC shift + RCT /
// ICT forms all three components in registers, and each component
// is lifted and stored in turn.  jobs = component triples (blockIdx.y).
template <bool IRREV, int TH, typename S = int32_t>
__global__ __launch_bounds__(64 * DWT_WAVES) void k_dwt_fwd_mct3(const DwtJob *__restrict__ jobs, int lay) {
    using G = DwtGeo<IRREV, TH>;
    constexpr int R = G::R;
    const int gx = gridDim.x;
    int L = blockIdx.y * gx + blockIdx.x;
    if (lay & 1) L = xcd_remap(L, gx * gridDim.y);
    const int wg = L % gx, trip = L / gx;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const DwtJob &J0 = jobs[trip * 3];
    const int tile = wg * DWT_WAVES + w;
    const int tx = tile % J0.tiles_x, ty = tile / J0.tiles_x;
    const int rw = J0.rw, rh = J0.rh, casx = J0.casx, casy = J0.casy;
    if (ty >= (rh + casy + TH - 1) / TH) return;
    const int lane = threadIdx.x & 63;
    const int xw = tx * G::CW - casx - G::HALO;
    const int yw = ty * G::TH - casy - G::HALO;
    const int gx0 = xw + 2 * lane, gx1 = gx0 + 1;
    int32_t a0[R], a1[R], b0[R], b1[R], c0[R], c1[R];
    {
        constexpr int B = Smp<S>::B;
        const int st = (int)J0.src_stride * B;
        const rsrc_t p0 = mkbuf(J0.src[0], J0.src_bytes), p1 = mkbuf(J0.src[1], J0.src_bytes),
                     p2 = mkbuf(J0.src[2], J0.src_bytes);
        const bool vec = J0.src_vec && casx == 0 && xw >= 0 && xw + DWT_WIN <= rw;  // wave-uniform
        const bool rows_in = yw >= 0 && yw + R <= rh;
        if (vec) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int so = (rows_in ? yw + r : mirror_idx(yw + r, rh)) * st;
                Smp<S>::pair(p0, gx0 * B, so, a0[r], a1[r]);
                Smp<S>::pair(p1, gx0 * B, so, b0[r], b1[r]);
                Smp<S>::pair(p2, gx0 * B, so, c0[r], c1[r]);
            }
        } else {
            const int o0 = mirror_idx(gx0, rw) * B, o1 = mirror_idx(gx1, rw) * B;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int so = mirror_idx(yw + r, rh) * st;
                a0[r] = Smp<S>::one(p0, o0, so); a1[r] = Smp<S>::one(p0, o1, so);
                b0[r] = Smp<S>::one(p1, o0, so); b1[r] = Smp<S>::one(p1, o1, so);
                c0[r] = Smp<S>::one(p2, o0, so); c1[r] = Smp<S>::one(p2, o1, so);
            }
        }
    }
    // DC shift + forward MCT in place: a = component 0, b = 1, c = 2
    const int32_t s0 = J0.shift[0], s1 = J0.shift[1], s2 = J0.shift[2];
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int32_t rr = (h ? a1[r] : a0[r]) - s0, gg = (h ? b1[r] : b0[r]) - s1, bb = (h ? c1[r] : c0[r]) - s2;
            int32_t y, u, v;
            if constexpr (!IRREV) {
                y = (rr + (gg * 2) + bb) >> 2; u = bb - gg; v = rr - gg;
            } else {
                y = ict_term(rr, 2449) + ict_term(gg, 4809) + ict_term(bb, 934);
                u = -ict_term(rr, 1382) - ict_term(gg, 2714) + ict_term(bb, 4096);
                v = ict_term(rr, 4096) - ict_term(gg, 3430) - ict_term(bb, 666);
            }
            if (h) { a1[r] = y; b1[r] = u; c1[r] = v; } else { a0[r] = y; b0[r] = u; c0[r] = v; }
        }
        if (IRREV) __builtin_amdgcn_sched_barrier(0);
    }
    // scheduling fences between the components keep the live set at the
    // three windows (6 R registers) instead of interleaved lifting chains
    __builtin_amdgcn_sched_barrier(0);
    fwd_vertical<IRREV, R>(a0, a1, rh, casy);
    fwd_horizontal_store<IRREV, TH>(jobs[trip * 3 + 0], a0, a1, ty, yw, gx0, lane);
    __builtin_amdgcn_sched_barrier(0);
    fwd_vertical<IRREV, R>(b0, b1, rh, casy);
    fwd_horizontal_store<IRREV, TH>(jobs[trip * 3 + 1], b0, b1, ty, yw, gx0, lane);
    __builtin_amdgcn_sched_barrier(0);
    fwd_vertical<IRREV, R>(c0, c1, rh, casy);
    fwd_horizontal_store<IRREV, TH>(jobs[trip * 3 + 2], c0, c1, ty, yw, gx0, lane);
}

// ---------------------------------------------------------------------------
// inverse level
// ---------------------------------------------------------------------------
// Inverse lifting of a window (dwt.cpp:724-858 5/3, :1544-1738 9/7):
// horizontal on every window row (the vertical pass needs the halo rows),
// then vertical.
template <bool IRREV, int R>
__device__ __forceinline__ void inv_lift(int32_t (&lo)[R], int32_t (&hi)[R], int rw, int rh, int casx, int casy) {
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
    if (rh > 1) {
        if constexpr (!IRREV) {
            vstep<6, 0, 0>(lo); vstep<6, 0, 0>(hi);
            vstep<7, 1, 1>(lo); vstep<7, 1, 1>(hi);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const float s = (r & 1) ? 1.625732422f : 1.230174105f;
                lo[r] = __float_as_int(__fmul_rn(__int_as_float(lo[r]), s));
                hi[r] = __float_as_int(__fmul_rn(__int_as_float(hi[r]), s));
            }
            vstep<8, 0, 0>(lo); vstep<8, 0, 0>(hi);
            vstep<9, 1, 1>(lo); vstep<9, 1, 1>(hi);
            vstep<10, 0, 2>(lo); vstep<10, 0, 2>(hi);
            vstep<11, 1, 3>(lo); vstep<11, 1, 3>(hi);
        }
    } else if (!IRREV && casy) {
#pragma unroll
        for (int r = 0; r < R; ++r) { lo[r] /= 2; hi[r] /= 2; }
    }
}

template <bool IRREV, int TH>
__global__ __launch_bounds__(64 * DWT_WAVES) void k_dwt_inv(const DwtJob *__restrict__ jobs, int lay) {
    using G = DwtGeo<IRREV, TH>;
    constexpr int R = G::R;
    DwtJob J;
    int tx, ty;
    if (!dwt_window(jobs, lay, TH, J, tx, ty)) return;
    const int lane = threadIdx.x & 63;
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
        if (yw >= 0 && yw + R <= rh) {  // no row mirroring: scalar row bases (see k_dwt_fwd)
            const int lbase = ty * (G::TH / 2) - casy - G::HALO / 2;
            const int hbase = J.sny + ty * (G::TH / 2) - G::HALO / 2;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if ((r & 1) == 0) {
                    const int iy = lbase + r / 2;
                    lo[r] = ld32(llb, ix0, iy * lst);
                    hi[r] = ld32(cb, ix1, iy * cst);
                } else {
                    const int so = (hbase + (r - 1) / 2) * cst;
                    lo[r] = ld32(cb, ix0, so);
                    hi[r] = ld32(cb, ix1, so);
                }
            }
        } else {
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
    }
    inv_lift<IRREV, R>(lo, hi, rw, rh, casx, casy);
    const int corel = G::HALO / 2, coreh = corel + G::CW / 2;
    if (lane < corel || lane >= coreh) return;
    const bool okx0 = gx0 >= 0 && gx0 < rw, okx1 = gx1 >= 0 && gx1 < rw;
    const rsrc_t ob = mkbuf(J.out, J.out_bytes);
    const int ost = (int)J.out_stride * 4;
    const bool vec = (casx | (J.out_stride & 1)) == 0 && xw >= 0 && xw + DWT_WIN <= rw;  // wave-uniform
    const int v0 = okx0 ? gx0 * 4 : OOB, v1 = okx1 ? gx1 * 4 : OOB;
    const bool rows_all = yw + G::HALO >= 0 && yw + G::HALO + G::TH <= rh;  // wave-uniform
#pragma unroll
    for (int r = G::HALO; r < G::HALO + G::TH; ++r) {
        const int gy = yw + r;
        if (!rows_all && (gy < 0 || gy >= rh)) continue;
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
// Forward levels 0 and 1 in one launch (9/7).  Level 1 reads level 0's LL
// band, which the separate launches write to HBM and read back (2 x 4 B per
// LL sample, a quarter of level 0's bytes); here a workgroup computes the LL
// samples its level-1 window needs into LDS and lifts level 1 from there, so
// LL0 never leaves the chip.
//   * Level-1 window (LL0 coordinates): W1 = 120 columns x R1 = 12 NY rows,
//     core CW1 = 112 x TH1 = R1 - 8, origin (xw1, yw1) as in k_dwt_fwd.
//   * Level-0 stage: the LL0 samples of that window (extended coordinates,
//     left / top edges included) come from 2 x NY level-0 windows of 128
//     columns x (24 + 8) rows (60 x 12 LL0 samples each), NY / 2 per
//     wavefront.  Their LL samples go to LDS; their HL / LH / HH samples go to
//     HBM for the level-0 pairs this workgroup owns (those under its level-1
//     core; the first / last workgroup of a row or column also owns the pairs
//     before / after it), so every band sample is written once.
//   * Level-1 stage: each wavefront lifts TH1 / 4 core rows (+ 2 x 4 halo) of
//     the window from LDS, with whole-sample symmetric extension of LL0
//     applied to the LDS indices (the level-0 stage computed every real LL0
//     sample the mirrored window reaches), then stores as k_dwt_fwd.
// Level-0 windows overlap (halo re-reads hit in L2) and the LL0 halo of the
// level-1 windows is computed twice; in exchange 8 B per LL0 sample of HBM
// traffic and one launch disappear.  (A variant walking 4 consecutive
// 16-row windows per wavefront with the overlap rows carried in registers,
// measured 189 us against 182 for NY = 4; non-temporal
// band stores 203 us.)
// ---------------------------------------------------------------------------
constexpr int F01_TH0 = 24;  // level-0 window rows
template <bool IRREV, int NY>
struct F01Geo {
    static constexpr int H = IRREV ? 4 : 2;
    static constexpr int PW = (DWT_WIN - 2 * H) / 2;  // LL0 columns per level-0 window
    static constexpr int W1 = 2 * PW;                 // level-1 window columns
    static constexpr int CW1 = W1 - 2 * H;
    static constexpr int R1 = NY * F01_TH0 / 2;       // level-1 window rows
    static constexpr int TH1 = R1 - 2 * H;
    static constexpr int THW = TH1 / 4;               // level-1 core rows per wavefront
    static_assert(THW * 4 == TH1 && THW % 2 == 0, "level-1 rows split into even per-wavefront windows");
};

// ny: level-0 row windows per workgroup (2 / 4 / 6)
int dwt01_tiles(int irrev, int ny, int rw1, int rh1, int casx1, int casy1, int *tiles_x) {
    if (!irrev) return 0;  // 9/7 only
    const int cw = F01Geo<true, 4>::CW1;
    const int th = ny == 2 ? F01Geo<true, 2>::TH1 : ny == 6 ? F01Geo<true, 6>::TH1 : F01Geo<true, 4>::TH1;
    *tiles_x = (rw1 + casx1 + cw - 1) / cw;
    return *tiles_x * ((rh1 + casy1 + th - 1) / th);
}

template <bool IRREV, int NY, typename T = int32_t>
__global__ __launch_bounds__(64 * DWT_WAVES) void k_dwt_fwd01(const DwtJob *__restrict__ jobs0,
                                                             const DwtJob *__restrict__ jobs1, int lay) {
    using F = F01Geo<IRREV, NY>;
    using G0 = DwtGeo<IRREV, F01_TH0>;
    constexpr int H = F::H, R0 = G0::R;
    __shared__ int32_t ll[F::R1][F::W1];
    const int gx = gridDim.x;
    int L = blockIdx.y * gx + blockIdx.x;
    if (lay & 1) L = xcd_remap(L, gx * gridDim.y);
    const int job = L / gx, wg = L % gx;
    const DwtJob &J0 = jobs0[job];
    const DwtJob &J1 = jobs1[job];
    const int rw1 = J1.rw, rh1 = J1.rh, casx1 = J1.casx, casy1 = J1.casy;
    const int ntx = (rw1 + casx1 + F::CW1 - 1) / F::CW1, nty = (rh1 + casy1 + F::TH1 - 1) / F::TH1;
    if (wg >= ntx * nty) return;  // uniform over the workgroup
    int tx1, ty1;
    group_order(wg, ntx, nty, lay >> 8, tx1, ty1);
    const int xw1 = tx1 * F::CW1 - casx1 - H, yw1 = ty1 * F::TH1 - casy1 - H;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // level-0 pairs (LL0 coordinates) whose bands this workgroup stores
    const int P0 = tx1 == 0 ? INT32_MIN : xw1 + H, P1 = tx1 == ntx - 1 ? INT32_MAX : xw1 + H + F::CW1;
    const int Q0 = ty1 == 0 ? INT32_MIN : yw1 + H, Q1 = ty1 == nty - 1 ? INT32_MAX : yw1 + H + F::TH1;

    // ---- level 0: 2 column windows x NY row windows ----
    {
        const int rw = J0.rw, rh = J0.rh, casx = J0.casx, casy = J0.casy;
        const int k = w & 1;
        const int xw = 2 * (xw1 + F::PW * k) + casx - H;
        const int gx0 = xw + 2 * lane, gx1 = gx0 + 1;
        const rsrc_t in = mkbuf(J0.in, J0.in_bytes);
        const int st = (int)J0.in_stride * 4;
        const bool vec = (casx | (J0.in_stride & 1)) == 0 && xw >= 0 && xw + DWT_WIN <= rw;  // wave-uniform
        const int o0 = mirror_idx(gx0, rw) * 4, o1 = mirror_idx(gx1, rw) * 4;
        const int corel = H / 2, coreh = corel + F::PW;
        const bool lane_core = lane >= corel && lane < coreh;
        const int pc = (gx0 - casx) >> 1;  // this lane's pair column (LL0 coordinates)
        const bool own_c = lane_core && pc >= P0 && pc < P1;
        const bool okx0 = own_c && gx0 >= 0 && gx0 < rw, okx1 = own_c && gx1 >= 0 && gx1 < rw;
        const int vl = okx0 ? pc * 4 : OOB;
        const int vh = okx1 ? (J0.snx + pc + casx) * 4 : OOB;
        const rsrc_t bandb = mkbuf(J0.bands, J0.bands_bytes);
        const int bst = (int)J0.bands_stride * 4;
        const int lcol = lane_core ? pc - xw1 : 0;  // LDS column of this lane's LL sample
        for (int jy = w >> 1; jy < NY; jy += DWT_WAVES / 2) {
            const int yw = 2 * (yw1 + (F01_TH0 / 2) * jy) + casy - H;
            T lo[R0], hi[R0];
            const bool rows_in = yw >= 0 && yw + R0 <= rh;  // wave-uniform
            if (vec && rows_in) {
                const int base = yw * st;
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const auto p = __builtin_amdgcn_raw_buffer_load_b64(in, gx0 * 4, base + r * st, 0);
                    lo[r] = (T)(int32_t)p[0]; hi[r] = (T)(int32_t)p[1];
                }
            } else {
#pragma unroll
                for (int r = 0; r < R0; ++r) {
                    const int so = mirror_idx(yw + r, rh) * st;
                    lo[r] = (T)ld32(in, o0, so); hi[r] = (T)ld32(in, o1, so);
                }
            }
            fwd_vertical<IRREV, R0, T>(lo, hi, rh, casy);
            const int prow0 = yw1 + (F01_TH0 / 2) * jy;  // pair row of window row H
#pragma unroll
            for (int r = H; r < H + F01_TH0; ++r) {
                T Lv = lo[r], Hv = hi[r];
                if constexpr (IRREV) {
                    const int32_t kk = (r & 1) ? 5039 : 6659;  // vertical scale: high rows K/2, low rows 1/K
                    Lv = scalev(Lv, kk); Hv = scalev(Hv, kk);
                    Hv = liftv<2>(Hv, Lv, from_next(Lv));
                    Lv = liftv<3>(Lv, from_prev(Hv), Hv);
                    Hv = liftv<4>(Hv, Lv, from_next(Lv));
                    Lv = liftv<5>(Lv, from_prev(Hv), Hv);
                    Hv = scalev(Hv, 5039);
                    Lv = scalev(Lv, 6659);
                } else {
                    Hv = lift<0>(Hv, Lv, from_next(Lv));
                    Lv = lift<1>(Lv, from_prev(Hv), Hv);
                }
                const int prow = prow0 + ((r - H) >> 1);
                const int gy = yw + r;
                const bool rok = prow >= Q0 && prow < Q1 && gy >= 0 && gy < rh;  // wave-uniform
                if ((r & 1) == 0) {
                    if (lane_core) ll[prow - yw1][lcol] = to_i32(Lv);
                    if (rok) st32(to_i32(Hv), bandb, vh, prow * bst);  // HL
                } else if (rok) {
                    const int so = (J0.sny + prow + casy) * bst;  // LH | HH row (pair row + casy)
                    st32(to_i32(Lv), bandb, vl, so);
                    st32(to_i32(Hv), bandb, vh, so);
                }
            }
        }
    }
    __syncthreads();
    // ---- level 1 from LDS: wavefront w lifts core rows [w THW, (w + 1) THW) ----
    {
        constexpr int RW = F::THW + 2 * H;
        const int yw = yw1 + F::THW * w;
        const int gx0 = xw1 + 2 * lane;
        const int c0 = min(max(mirror_idx(gx0, rw1) - xw1, 0), F::W1 - 1);
        const int c1 = min(max(mirror_idx(gx0 + 1, rw1) - xw1, 0), F::W1 - 1);
        T lo[RW], hi[RW];
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int rr = min(max(mirror_idx(yw + r, rh1) - yw1, 0), F::R1 - 1);
            lo[r] = (T)ll[rr][c0];
            hi[r] = (T)ll[rr][c1];
        }
        fwd_vertical<IRREV, RW, T>(lo, hi, rh1, casy1);
        fwd_horizontal_store<IRREV, F::THW, F::W1, T>(J1, lo, hi, ty1 * 4 + w, yw, gx0, lane);
    }
}

// ---------------------------------------------------------------------------
// Forward levels l and l + 1 streamed down column strips (k_dwt_fwd_pair;
// 5/3 and 9/7).  k_dwt_fwd01 lifts independent windows: every window
// re-reads and re-lifts 2 x 4 halo rows, and every workgroup re-computes the
// LL halo of its level-(l+1) window -- the 8K frame's pair reads 1.49x its
// input.  Here a workgroup owns a strip of CW1 level-(l+1) columns x S1 rows
// and walks it top to bottom:
//   * NW0 level-l waves, side by side (128 columns each, PW = 60 / 62 LL
//     columns of core), stream down the strip in chunks of C0 = 8 rows.
//     The vertical lifting is carried from chunk to chunk: the last P = NS + 2
//     rows of a chunk, partially lifted, stay in registers and head the next
//     chunk's array, so no row is loaded or lifted twice (vlift_stream).  The
//     next chunk's rows are loaded before the barrier that ends a chunk.
//   * A chunk's finished rows are lifted horizontally; their HL / LH / HH
//     samples go to the Mallat bands in HBM, the LL row into an LDS ring of
//     RING rows x LW columns.
//   * NW1 level-(l+1) waves stream the LL rows out of the ring in chunks of
//     C1 = 8 rows the same way (LL whole-sample symmetric extension applied
//     to the ring's row / column indices), then store LL_{l+1} and the level's
//     bands as k_dwt_fwd does.
//   * One workgroup barrier per level-l chunk; a level-(l+1) chunk runs in
//     the first iteration after the level-l chunk holding its last LL row.
// A segment re-reads only the rows above and below it that its two lifting
// halos need (~2 x 12 rows per segment of 2 S1), and a strip the 2 x 4 LL
// columns of the level-(l+1) halo plus the level-l halo at its sides: the 8K
// frame's 9/7 pair reads 435 MB for 398 MB of input (k_dwt_fwd01: 593 MB).
// Measured (profiles/r05/dwt_pair_ab.txt): the 5/3 pairs beat one launch per
// level (8K: levels 1 + 2 in 54 us against 47 + 16, 3 + 4 in 11 against
// 9 + 7), so they are the 5/3 default; the 9/7 pair (198 us) does not beat
// k_dwt_fwd01 (185 us) -- its 64-bit fixed-point lifting chains stay
// latency-bound at the ~3 resident waves per SIMD the strips leave -- and
// runs only on request (grkgpu_dwt_options.pair_kernel = 2).
// ---------------------------------------------------------------------------
template <bool IRREV, int NW0_, int C0_ = 8, int C1_ = 8>
struct PairGeo {
    static constexpr int NS = IRREV ? 4 : 2;           // lifting steps: halo rows / columns per side
    static constexpr int P = NS + 2;                   // rows carried from one chunk to the next
    static constexpr int PW = (DWT_WIN - 2 * NS) / 2;  // LL columns per level-l wave (60 / 62)
    static constexpr int NW0 = NW0_;                   // level-l waves
    static constexpr int LW = NW0 * PW;                // LL columns a workgroup computes
    static constexpr int CW = DWT_WIN - 2 * NS;        // core columns of a level-(l+1) window
    static constexpr int CW1 = LW - 2 * NS;            // level-(l+1) core columns per workgroup
    static constexpr int NW1 = (CW1 + CW - 1) / CW;    // level-(l+1) waves
    static constexpr int WAVES = NW0 + NW1;
    static constexpr int C0 = C0_, C1 = C1_;           // rows per chunk (level l, level l + 1)
    static constexpr int RING = 32;                    // LL rows held in LDS
};

// Vertical lifting step S over rows k >= K0 of parity K0 (see vstep).
template <int OP, int K0, int S, int R, typename T>
__device__ __forceinline__ void vstep_at(T (&v)[R]) {
#pragma unroll
    for (int k = K0; k + 1 + S < R; k += 2) v[k] = liftv<OP>(v[k], v[k - 1], v[k + 1]);
}

// Streaming vertical lifting of an array of R = P + C rows whose even rows
// are low pass.  FIRST: fresh rows, the steps start at the array's top (its
// first NS rows come out inexact).  Otherwise rows [0, P) are the previous
// array's rows [C, C + P) as it left them: its last two rows raw, the two
// before with the first one / two steps, the two before those final.  Step S
// then resumes at row P - 1 - S.  Either way rows [2, 2 + C) come out final
// and the array's last P rows are left in the state the next chunk expects
// (every step S stops at k + 1 + S < R).
template <bool IRREV, bool FIRST, int R, typename T>
__device__ __forceinline__ void vlift_stream(T (&lo)[R], T (&hi)[R]) {
    if constexpr (!IRREV) {
        vstep_at<0, FIRST ? 1 : 3, 0>(lo); vstep_at<0, FIRST ? 1 : 3, 0>(hi);
        vstep_at<1, 2, 1>(lo); vstep_at<1, 2, 1>(hi);
    } else {
        vstep_at<2, FIRST ? 1 : 5, 0>(lo); vstep_at<2, FIRST ? 1 : 5, 0>(hi);
        vstep_at<3, FIRST ? 2 : 4, 1>(lo); vstep_at<3, FIRST ? 2 : 4, 1>(hi);
        vstep_at<4, 3, 2>(lo); vstep_at<4, 3, 2>(hi);
        vstep_at<5, FIRST ? 4 : 2, 3>(lo); vstep_at<5, FIRST ? 4 : 2, 3>(hi);
    }
}

// Horizontal lifting of one vertically lifted row (9/7: after the vertical
// scale, K/2 for a high row, 1/K for a low one).  rw, rh > 1.
template <bool IRREV, typename T>
__device__ __forceinline__ void hlift_row(T &L, T &H, bool high) {
    if constexpr (IRREV) {
        const int32_t k = high ? 5039 : 6659;
        L = scalev(L, k); H = scalev(H, k);
        H = liftv<2>(H, L, from_next(L));
        L = liftv<3>(L, from_prev(H), H);
        H = liftv<4>(H, L, from_next(L));
        L = liftv<5>(L, from_prev(H), H);
        H = scalev(H, 5039);
        L = scalev(L, 6659);
    } else {
        H = lift<0>(H, L, from_next(L));
        L = lift<1>(L, from_prev(H), H);
    }
}

// Workgroup barrier ordering LDS only: outstanding global loads (the next
// chunk's rows) stay in flight across it.
__device__ __forceinline__ void lds_barrier() { __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// mirror_idx for n >= 2 without the small-n loop: exact within one
// reflection, any valid index beyond (rows no kept sample depends on)
__device__ __forceinline__ int mirror1(int p, int n) {
    p = p < 0 ? -p : p;
    p = p >= n ? 2 * (n - 1) - p : p;
    return p < 0 ? 0 : p;
}

// byte offsets of rows t .. t + N - 1 of a resolution of rh rows (mirrored
// at its edges); wave-uniform
template <int N>
__device__ __forceinline__ void row_offsets(int t, int rh, int st, int (&so)[N]) {
    if (t >= 0 && t + N <= rh) {
#pragma unroll
        for (int r = 0; r < N; ++r) so[r] = (t + r) * st;
    } else {
#pragma unroll
        for (int r = 0; r < N; ++r) so[r] = mirror1(t + r, rh) * st;
    }
}

// strip geometry shared by the kernel and the host
struct PairStrip {
    int xs1, ys1, ye1, t1, nC1, e0, t0, nC0, Q0, Q1, P0, P1;
};
template <bool IRREV, int NW0, int C0X>
__device__ __forceinline__ bool pair_strip(const DwtJob &J0, const DwtJob &J1, int S1, int wg, PairStrip &g, int &tx,
                                           int &ntx) {
    using G = PairGeo<IRREV, NW0, (C0X & 255), ((C0X >> 12) & 15)>;
    constexpr int NS = G::NS;
    const int rw1 = J1.rw, rh1 = J1.rh, casx1 = J1.casx, casy1 = J1.casy;
    ntx = (rw1 + casx1 + G::CW1 - 1) / G::CW1;
    const int nty = (rh1 + casy1 + S1 - 1) / S1;
    if (wg >= ntx * nty) return false;
    tx = wg % ntx;
    const int ty = wg / ntx;
    g.xs1 = tx * G::CW1 - casx1;
    g.ys1 = ty * S1 - casy1;
    g.ye1 = min(g.ys1 + S1, rh1);
    g.t1 = g.ys1 - NS;                                        // level-(l+1) stream: first row
    g.nC1 = (g.ye1 - g.t1 - 2 + G::C1 - 1) / G::C1;           // chunks until row ye1 - 1 is final
    const int lo1 = max(0, g.t1), hi1 = min(rh1, g.ye1 + NS);  // LL rows it needs exactly
    const int casy0 = J0.casy;
    g.Q0 = ty == 0 ? INT32_MIN : g.ys1;                       // level-l band pair rows owned
    g.Q1 = ty == nty - 1 ? INT32_MAX : g.ys1 + S1;
    g.P0 = tx == 0 ? INT32_MIN : g.xs1;                       // ... and pair columns
    g.P1 = tx == ntx - 1 ? INT32_MAX : g.xs1 + G::CW1;
    const int first = ty == 0 ? min(lo1, -casy0) : lo1;      // first pair row to compute
    const int plast = (J0.rh - 1 - casy0) >> 1;
    const int pmax = ty == nty - 1 ? max(hi1 - 1, plast) : hi1 - 1;
    g.t0 = 2 * first + casy0 - NS;                           // level-l stream: first row
    g.e0 = first - (NS - 2) / 2;                             // pair row of its first emitted row
    g.nC0 = (pmax + 1 - g.e0 + G::C0 / 2 - 1) / (G::C0 / 2);
    return true;
}

// level-l waves of k_dwt_fwd_pair (VEC: 8-byte column-pair loads)
template <bool IRREV, int NW0, int C0X, bool VEC, typename T>
__device__ __forceinline__ void pair_level0(const DwtJob &J0, const PairStrip &g,
                                            int32_t (*ll)[PairGeo<IRREV, NW0>::LW + 1], int k, int lane) {
    using G = PairGeo<IRREV, NW0, (C0X & 255), ((C0X >> 12) & 15)>;
    constexpr int NS = G::NS, P = G::P, C0 = G::C0, RING = G::RING;
    const int rw0 = J0.rw, rh0 = J0.rh, casx0 = J0.casx, casy0 = J0.casy;
    const int xw = 2 * (g.xs1 - NS + G::PW * k) + casx0 - NS;  // window column origin
    const int gx0 = xw + 2 * lane, gx1 = gx0 + 1;
    const rsrc_t in = mkbuf(J0.in, J0.in_bytes);
    const int st = (int)J0.in_stride * 4;
    const int o0 = VEC ? gx0 * 4 : mirror_idx(gx0, rw0) * 4, o1 = mirror_idx(gx1, rw0) * 4;
    const bool lane_core = lane >= NS / 2 && lane < NS / 2 + G::PW;
    const int pc = (gx0 - casx0) >> 1;  // this lane's pair column (LL coordinates)
    const bool own_c = lane_core && pc >= g.P0 && pc < g.P1;
    const bool okx0 = own_c && gx0 >= 0 && gx0 < rw0, okx1 = own_c && gx1 >= 0 && gx1 < rw0;
    const int vl = okx0 ? pc * 4 : OOB;
    const int vh = okx1 ? (J0.snx + pc + casx0) * 4 : OOB;
    const rsrc_t bandb = mkbuf(J0.bands, J0.bands_bytes);
    const int bst = (int)J0.bands_stride * 4;
    // LDS column of this lane's LL sample; the halo lanes write a spare column
    const int lcol = lane_core ? pc - (g.xs1 - NS) : G::LW;
    auto ldrows = [&](int t, T *a, T *b, auto n) {
        constexpr int N = decltype(n)::value;
        int so[N];
        row_offsets<N>(t, rh0, st, so);
#pragma unroll
        for (int r = 0; r < N; ++r) {
            if constexpr (VEC) {
                const auto p = __builtin_amdgcn_raw_buffer_load_b64(in, o0, so[r], 0);
                a[r] = (T)(int32_t)p[0]; b[r] = (T)(int32_t)p[1];
            } else {
                a[r] = (T)ld32(in, o0, so[r]); b[r] = (T)ld32(in, o1, so[r]);
            }
        }
    };
    T lo[P + C0], hi[P + C0];
    ldrows(g.t0, lo, hi, std::integral_constant<int, P + C0>{});
    for (int c = 0; c <= g.nC0; ++c) {
        if (c < g.nC0) {
            const bool more = c + 1 < g.nC0;  // wave-uniform
            if (c == 0) vlift_stream<IRREV, true>(lo, hi);
            else vlift_stream<IRREV, false>(lo, hi);
            const int tb = g.t0 + c * C0;
            const int pb = (tb + 2 - casy0) >> 1;  // pair row of the chunk's first emitted row
#pragma unroll
            for (int i = 2; i < 2 + C0; ++i) {
                T Lv = lo[i], Hv = hi[i];
                hlift_row<IRREV>(Lv, Hv, i & 1);
                const int t = tb + i;
                const int p = pb + (i - 2) / 2;
                // rows this workgroup does not own: stores dropped through an
                // out-of-range lane offset (no branch)
                const bool rok = p >= g.Q0 && p < g.Q1 && t >= 0 && t < rh0;  // wave-uniform
                const int rl = rok ? vl : OOB, rh = rok ? vh : OOB;
                if ((i & 1) == 0) {
                    ll[(p - g.e0) & (RING - 1)][lcol] = to_i32(Lv);
                    st32(to_i32(Hv), bandb, rh, p * bst);  // HL
                } else {
                    const int so = (J0.sny + p + casy0) * bst;  // LH | HH
                    st32(to_i32(Lv), bandb, rl, so);
                    st32(to_i32(Hv), bandb, rh, so);
                }
            }
#pragma unroll
            for (int r = 0; r < P; ++r) { lo[r] = lo[r + C0]; hi[r] = hi[r + C0]; }
            // the next chunk's rows, in flight across the barrier
            if (more) ldrows(g.t0 + P + (c + 1) * C0, lo + P, hi + P, std::integral_constant<int, C0>{});
        }
        lds_barrier();
    }
}

// level-(l+1) waves of k_dwt_fwd_pair
template <bool IRREV, int NW0, int C0X, typename T>
__device__ __forceinline__ void pair_level1(const DwtJob &J1, const PairStrip &g,
                                            int32_t (*ll)[PairGeo<IRREV, NW0>::LW + 1], int a, int lane) {
    using G = PairGeo<IRREV, NW0, (C0X & 255), ((C0X >> 12) & 15)>;
    constexpr int NS = G::NS, P = G::P, C1 = G::C1, RING = G::RING, LW = G::LW;
    const int rw1 = J1.rw, rh1 = J1.rh, casx1 = J1.casx, casy1 = J1.casy;
    const int base = g.xs1 - NS;  // LL column of LDS column 0
    const int oa = a == 0 ? 0 : max(0, min(a * G::CW, LW - DWT_WIN));
    const int gx0 = base + oa + 2 * lane, gx1 = gx0 + 1;
    const int c0 = min(max(mirror_idx(gx0, rw1) - base, 0), LW - 1);
    const int c1 = min(max(mirror_idx(gx1, rw1) - base, 0), LW - 1);
    const bool lane_core = lane >= NS / 2 && lane < NS / 2 + G::CW / 2;
    const int ox0 = g.xs1 + a * G::CW, ox1 = g.xs1 + min((a + 1) * G::CW, G::CW1);  // columns this wave stores
    const bool own0 = lane_core && gx0 >= ox0 && gx0 < ox1 && gx0 >= 0 && gx0 < rw1;
    const bool own1 = lane_core && gx1 >= ox0 && gx1 < ox1 && gx1 >= 0 && gx1 < rw1;
    const int vl = own0 ? ((gx0 - casx1) >> 1) * 4 : OOB;
    const int vh = own1 ? (J1.snx + ((gx1 - 1 + casx1) >> 1)) * 4 : OOB;
    const rsrc_t outb = mkbuf(J1.out, J1.out_bytes), bandb = mkbuf(J1.bands, J1.bands_bytes);
    const int ost = (int)J1.out_stride * 4, bst = (int)J1.bands_stride * 4;
    auto ldsrows = [&](int t, T *x, T *y, auto n) {
        constexpr int N = decltype(n)::value;
        int rr[N];
        if (t >= 0 && t + N <= rh1) {
#pragma unroll
            for (int r = 0; r < N; ++r) rr[r] = (t + r - g.e0) & (RING - 1);
        } else {
#pragma unroll
            for (int r = 0; r < N; ++r) rr[r] = (mirror1(t + r, rh1) - g.e0) & (RING - 1);
        }
#pragma unroll
        for (int r = 0; r < N; ++r) { x[r] = (T)ll[rr[r]][c0]; y[r] = (T)ll[rr[r]][c1]; }
    };
    T lo[P + C1], hi[P + C1];
    int j = 0;
    const int hi1 = min(rh1, g.ye1 + NS);
    for (int c = 0; c <= g.nC0; ++c) {
        for (; j < g.nC1; ++j) {
            // ready once the level-l chunk holding its last exact LL row is in the ring
            const int mj = min(hi1, g.t1 + P + (j + 1) * C1) - 1;
            if ((mj - g.e0) / (G::C0 / 2) + 1 > c) break;
            if (j == 0) {
                ldsrows(g.t1, lo, hi, std::integral_constant<int, P + C1>{});
                vlift_stream<IRREV, true>(lo, hi);
            } else {
                ldsrows(g.t1 + P + j * C1, lo + P, hi + P, std::integral_constant<int, C1>{});
                vlift_stream<IRREV, false>(lo, hi);
            }
            const int tb = g.t1 + j * C1;
#pragma unroll
            for (int i = 2; i < 2 + C1; ++i) {
                T Lv = lo[i], Hv = hi[i];
                hlift_row<IRREV>(Lv, Hv, i & 1);
                const int t = tb + i;
                const bool rok = t >= g.ys1 && t < g.ye1 && t >= 0;  // wave-uniform
                const int rl = rok ? vl : OOB, rh = rok ? vh : OOB;
                if ((i & 1) == 0) {  // low row -> LL | HL
                    const int iy = (t - casy1) >> 1;
                    st32(to_i32(Lv), outb, rl, iy * ost);
                    st32(to_i32(Hv), bandb, rh, iy * bst);
                } else {             // high row -> LH | HH
                    const int so = (J1.sny + ((t - 1 + casy1) >> 1)) * bst;
                    st32(to_i32(Lv), bandb, rl, so);
                    st32(to_i32(Hv), bandb, rh, so);
                }
            }
#pragma unroll
            for (int r = 0; r < P; ++r) { lo[r] = lo[r + C1]; hi[r] = hi[r + C1]; }
        }
        lds_barrier();
    }
}

template <bool IRREV, int NW0, int C0X, typename T = int32_t>
__global__ __launch_bounds__((64 * PairGeo<IRREV, NW0>::WAVES)) __attribute__((amdgpu_waves_per_eu((C0X >> 16) & 15))) void k_dwt_fwd_pair(const DwtJob *__restrict__ jobs0,
                                                                                   const DwtJob *__restrict__ jobs1,
                                                                                   int S1, int lay) {
    using G = PairGeo<IRREV, NW0, (C0X & 255), ((C0X >> 12) & 15)>;
    __shared__ int32_t ll[G::RING][G::LW + 1];  // + a spare column for the halo lanes' writes
    const int gx = gridDim.x;
    int L = blockIdx.y * gx + blockIdx.x;
    if (lay & 1) L = xcd_remap(L, gx * gridDim.y);
    const int job = L / gx, wg = L % gx;
    const DwtJob &J0 = jobs0[job];
    const DwtJob &J1 = jobs1[job];
    PairStrip g;
    int tx, ntx;
    if (!pair_strip<IRREV, NW0, C0X>(J0, J1, S1, wg, g, tx, ntx)) return;  // uniform over the workgroup
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w < NW0) {
        const int xw = 2 * (g.xs1 - G::NS + G::PW * w) + J0.casx - G::NS;
        const bool vec = (J0.casx | (J0.in_stride & 1)) == 0 && xw >= 0 && xw + DWT_WIN <= J0.rw;  // wave-uniform
        if (vec) pair_level0<IRREV, NW0, C0X, true, T>(J0, g, ll, w, lane);
        else pair_level0<IRREV, NW0, C0X, false, T>(J0, g, ll, w, lane);
    } else {
        pair_level1<IRREV, NW0, C0X, T>(J1, g, ll, w - NW0, lane);
    }
}

// Host geometry of k_dwt_fwd_pair: level-(l+1) core columns per workgroup for
// nw0 level-l waves (3 or 4), and workgroups per job for S1 rows per segment.
int dwt_pair_cw1(int irrev, int nw0) {
    if (irrev) return nw0 == 3 ? PairGeo<true, 3>::CW1 : PairGeo<true, 4>::CW1;
    return nw0 == 3 ? PairGeo<false, 3>::CW1 : PairGeo<false, 4>::CW1;
}
int dwt_pair_wgs(int irrev, int nw0, int s1, int rw1, int rh1, int casx1, int casy1) {
    const int cw1 = dwt_pair_cw1(irrev, nw0);
    return ((rw1 + casx1 + cw1 - 1) / cw1) * ((rh1 + casy1 + s1 - 1) / s1);
}

hipError_t launch_dwt_fwd_pair(const DwtJob *jobs0, const DwtJob *jobs1, uint32_t njobs, uint32_t max_wgs, int irrev,
                               int nw0, int s1, hipStream_t s) {
    if (!njobs || !max_wgs || s1 < 2 || (s1 & 1)) return hipErrorInvalidValue;
    const int lay = 1;  // XCD-contiguous runs: a strip's horizontal neighbours share an L2
    const dim3 g(max_wgs, njobs);
#define GRK_PAIR(IR, NW, C)                                                                          \
    hipLaunchKernelGGL((k_dwt_fwd_pair<IR, NW, C>), g, dim3(64 * PairGeo<IR, NW>::WAVES), 0, s, jobs0, jobs1, s1, lay)
    // chunk geometry C0 | C1 << 12 | waves per SIMD << 16: 8-row chunks at
    // both levels, 6 wavefronts per SIMD (75 VGPRs) -- measured best against
    // 16-row chunks (4 or 3 per SIMD), 4-row chunks (8 per SIMD) and the next
    // chunk's rows held in registers during the lifting (profiles/r05/dwt_pair_ab.txt)
    if (irrev) { if (nw0 == 3) GRK_PAIR(true, 3, 0x68008); else GRK_PAIR(true, 4, 0x68008); }
    else { if (nw0 == 3) GRK_PAIR(false, 3, 0x68008); else GRK_PAIR(false, 4, 0x68008); }
#undef GRK_PAIR
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The two largest inverse levels in one launch (the mirror of k_dwt_fwd01).
// Separately, the first writes the LL band of the second (the resolution
// below the full one) to HBM and the second reads it back: 8 B per LL sample,
// 20 % of the pair's bytes.  Here a workgroup owns an output core of
// 2 NPX x 2 NPY samples of the larger resolution R_b:
//   * stage A reconstructs the R_a samples (R_a = the LL band of R_b) that
//     core's synthesis windows read -- NPX + H pairs wide plus one column of
//     parity slack, i.e. one window of CW columns, NA windows of THA rows --
//     from R_a's LL band and bands in HBM (k_dwt_inv's windows), into LDS;
//   * stage B runs k_dwt_inv's windows over the core (2 x NB windows of CW x
//     THB), their low-pass samples read from LDS (whole-sample symmetric
//     extension applied to the LDS indices; stage A covered every real sample
//     a mirrored index reaches), their high-pass bands from HBM, and stores
//     the owned samples of R_b.
// R_a's halo rows / columns are reconstructed by two workgroups (~1.1x of
// stage A's lifting); the launch boundary and the LL round trip go away.
// ---------------------------------------------------------------------------

template <bool IRREV, int NA_ = 2>
struct I01Geo {
    static constexpr int H = IRREV ? 4 : 2;
    static constexpr int CW = DWT_WIN - 2 * H;            // window core columns (120 / 124)
    static constexpr int NA = NA_, THA = 48 / NA_;        // stage A: NA windows of THA rows
    static constexpr int TR = NA * THA;                   // LDS tile rows (R_a)
    static constexpr int NPX = CW - H - 2;                // owned R_b pairs per row (114 / 120)
    static constexpr int NPY = TR - H - 2;                // owned R_b pair rows (42 / 44)
    static constexpr int THB = 22;                        // stage B window rows
    static constexpr int NB = (2 * NPY + THB - 1) / THB;  // stage B row windows (4)
    static constexpr int NBX = (2 * NPX + CW - 1) / CW;   // stage B column windows (2)
};

int dwt_inv01_tiles(int irrev, int rw_b, int rh_b, int casx_b, int casy_b) {
    const int cx = irrev ? 2 * I01Geo<true>::NPX : 2 * I01Geo<false>::NPX;
    const int cy = irrev ? 2 * I01Geo<true>::NPY : 2 * I01Geo<false>::NPY;
    return ((rw_b + casx_b + cx - 1) / cx) * ((rh_b + casy_b + cy - 1) / cy);
}

template <bool IRREV, int NA, int WPE = 1>
__global__ __launch_bounds__(64 * DWT_WAVES) __attribute__((amdgpu_waves_per_eu(WPE))) void k_dwt_inv01(const DwtJob *__restrict__ jobsA,
                                                             const DwtJob *__restrict__ jobsB, int lay) {
    using G = I01Geo<IRREV, NA>;
    constexpr int H = G::H, CW = G::CW;
    __shared__ int32_t tile[G::TR][CW];
    const int gx = gridDim.x;
    int L = blockIdx.y * gx + blockIdx.x;
    if (lay & 1) L = xcd_remap(L, gx * gridDim.y);
    const int job = L / gx, wg = L % gx;
    const DwtJob &JA = jobsA[job];
    const DwtJob &JB = jobsB[job];
    const int rwb = JB.rw, rhb = JB.rh, casxb = JB.casx, casyb = JB.casy;
    const int ntx = (rwb + casxb + 2 * G::NPX - 1) / (2 * G::NPX), nty = (rhb + casyb + 2 * G::NPY - 1) / (2 * G::NPY);
    if (wg >= ntx * nty) return;  // uniform over the workgroup
    int tx, ty;
    group_order(wg, ntx, nty, lay >> 8, tx, ty);
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // owned core of R_b: [bx0, bx0 + 2 NPX) x [by0, by0 + 2 NPY), bx0 = casx_b (mod 2)
    const int bx0 = tx * 2 * G::NPX - casxb, by0 = ty * 2 * G::NPY - casyb;
    // R_a samples stage B reads: pairs [m - H/2, m + NPX + H/2); the tile's
    // origin takes R_a's parity (k_dwt_inv's window alignment), one sample of slack
    const int mx = (bx0 - casxb) >> 1, my = (by0 - casyb) >> 1;
    const int ax0 = mx - H / 2, ay0 = my - H / 2;
    const int axA = ax0 - ((ax0 - JA.casx) & 1), ayA = ay0 - ((ay0 - JA.casy) & 1);

    // ---- stage A: R_a tile [axA, axA + CW) x [ayA, ayA + TR) into LDS ----
    for (int k = w; k < G::NA; k += DWT_WAVES) {
        constexpr int R = G::THA + 2 * H;
        const int rw = JA.rw, rh = JA.rh, casx = JA.casx, casy = JA.casy;
        const int xw = axA - H, yw = ayA + k * G::THA - H;
        const int gx0 = xw + 2 * lane, gx1 = gx0 + 1;
        const int ix0 = ((mirror_idx(gx0, rw) - casx) >> 1) * 4;
        const int ix1 = (JA.snx + ((mirror_idx(gx1, rw) - 1 + casx) >> 1)) * 4;
        const rsrc_t llb = mkbuf(JA.in, JA.in_bytes), cb = mkbuf(JA.coef, JA.coef_bytes);
        const int lst = (int)JA.in_stride * 4, cst = (int)JA.coef_stride * 4;
        int32_t lo[R], hi[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int my2 = mirror_idx(yw + r, rh);
            if ((r & 1) == 0) {
                const int iy = (my2 - casy) >> 1;
                lo[r] = ld32(llb, ix0, iy * lst);
                hi[r] = ld32(cb, ix1, iy * cst);
            } else {
                const int so = (JA.sny + ((my2 - 1 + casy) >> 1)) * cst;
                lo[r] = ld32(cb, ix0, so);
                hi[r] = ld32(cb, ix1, so);
            }
        }
        inv_lift<IRREV, R>(lo, hi, rw, rh, casx, casy);
        if (lane >= H / 2 && lane < H / 2 + CW / 2) {
            const int c = gx0 - axA;  // in [0, CW - 1)
#pragma unroll
            for (int r = H; r < H + G::THA; ++r) {
                tile[k * G::THA + r - H][c] = lo[r];
                tile[k * G::THA + r - H][c + 1] = hi[r];
            }
        }
    }
    __syncthreads();
    // ---- stage B: R_b windows over the owned core, low-pass from LDS ----
    for (int k = w; k < G::NBX * G::NB; k += DWT_WAVES) {
        constexpr int R = G::THB + 2 * H;
        const int kx = k % G::NBX, ky = k / G::NBX;
        const int xw = bx0 + kx * CW - H, yw = by0 + ky * G::THB - H;
        const int gx0 = xw + 2 * lane, gx1 = gx0 + 1;
        const int ta = min(max(((mirror_idx(gx0, rwb) - casxb) >> 1) - axA, 0), CW - 1);  // LDS column
        const int ix1 = (JB.snx + ((mirror_idx(gx1, rwb) - 1 + casxb) >> 1)) * 4;
        const int ixl = ((mirror_idx(gx0, rwb) - casxb) >> 1) * 4;  // LH column
        const rsrc_t cb = mkbuf(JB.coef, JB.coef_bytes);
        const int cst = (int)JB.coef_stride * 4;
        int32_t lo[R], hi[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int my2 = mirror_idx(yw + r, rhb);
            if ((r & 1) == 0) {
                const int iy = (my2 - casyb) >> 1;
                lo[r] = tile[min(max(iy - ayA, 0), G::TR - 1)][ta];
                hi[r] = ld32(cb, ix1, iy * cst);
            } else {
                const int so = (JB.sny + ((my2 - 1 + casyb) >> 1)) * cst;
                lo[r] = ld32(cb, ixl, so);
                hi[r] = ld32(cb, ix1, so);
            }
        }
        inv_lift<IRREV, R>(lo, hi, rwb, rhb, casxb, casyb);
        const int cx1 = bx0 + 2 * G::NPX, cy1 = by0 + 2 * G::NPY;  // owned core end
        const bool lane_core = lane >= H / 2 && lane < H / 2 + CW / 2;
        const bool okx0 = lane_core && gx0 >= 0 && gx0 < rwb && gx0 < cx1;
        const bool okx1 = lane_core && gx1 >= 0 && gx1 < rwb && gx1 < cx1;
        const rsrc_t ob = mkbuf(JB.out, JB.out_bytes);
        const int ost = (int)JB.out_stride * 4;
        const int v0 = okx0 ? gx0 * 4 : OOB, v1 = okx1 ? gx1 * 4 : OOB;
        // pair stores: even origin, width and stride put both samples of a
        // pair on the same side of every bound (wave-uniform)
        const bool vec = (casxb | (rwb & 1) | (JB.out_stride & 1)) == 0;
#pragma unroll
        for (int r = H; r < H + G::THB; ++r) {
            const int gy = yw + r;
            if (gy < 0 || gy >= rhb || gy >= cy1) continue;  // wave-uniform
            if (vec) {
                const __attribute__((ext_vector_type(2))) uint32_t pv = {(uint32_t)lo[r], (uint32_t)hi[r]};
                __builtin_amdgcn_raw_buffer_store_b64(pv, ob, v0, gy * ost, 0);
            } else {
                st32(lo[r], ob, v0, gy * ost);
                st32(hi[r], ob, v1, gy * ost);
            }
        }
    }
}

// na: stage-A row windows per workgroup (2 of 24 rows, 4 of 12)
hipError_t launch_dwt_inv01(const DwtJob *jobsA, const DwtJob *jobsB, uint32_t njobs, uint32_t max_tiles, int irrev,
                            int na, hipStream_t s) {
    if (!njobs || !max_tiles) return hipErrorInvalidValue;
    const dim3 g(max_tiles, njobs), b(64 * DWT_WAVES);
    const int lay = 1 | (dwt_options().pair_group << 8);  // XCD-contiguous runs, column groups
    if (na == 4) {
        if (irrev) hipLaunchKernelGGL((k_dwt_inv01<true, 4>), g, b, 0, s, jobsA, jobsB, lay);
        else hipLaunchKernelGGL((k_dwt_inv01<false, 4>), g, b, 0, s, jobsA, jobsB, lay);
    } else {
        // 9/7 held to 80 VGPRs: 6 wavefronts per SIMD instead of 5 (36 B of
        // spills): 183.6-184.7 -> 179.5-182.3 us on the 8K frame, three
        // alternating rounds (profiles/r05/dwt_occupancy_ab.txt); the 5/3 pair
        // at 128 VGPRs (4 instead of 3) and the 5/3 DC shift + RCT level 0 at 5
        // per SIMD (96 VGPRs, spilled) gained nothing / lost 45 %
        if (irrev) hipLaunchKernelGGL((k_dwt_inv01<true, 2, 6>), g, b, 0, s, jobsA, jobsB, lay);
        else hipLaunchKernelGGL((k_dwt_inv01<false, 2>), g, b, 0, s, jobsA, jobsB, lay);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Rows per window: tall windows for big levels (less halo re-read: 32 rows
// for 5/3, 24 for 9/7 at >= 2^23 samples), short ones for small levels (more
// wavefronts, shorter per-wave chains).
int dwt_pick_th(int irrev, uint64_t level_samples, int, int) {
    if (level_samples >= ((uint64_t)1 << 23)) return irrev ? 24 : 32;
    if (level_samples >= ((uint64_t)1 << 21) && dwt_options().mid_th) return dwt_options().mid_th;
    return 8;
}

void dwt_job_tiles(int irrev, int code, DwtJob &j) {
    const int th = code & 0xff;
    const int cw = irrev ? DwtGeo<true, 8>::CW : DwtGeo<false, 8>::CW;
    // window (tx, ty) holds the core [tx cw - casx, +cw) x [ty th - casy, +th)
    int x0 = 0, y0 = 0, x1 = j.rw, y1 = j.rh;
    if (j.reg_x1 > 0) {
        x0 = std::max(0, j.reg_x0); y0 = std::max(0, j.reg_y0);
        x1 = std::min(j.rw, j.reg_x1); y1 = std::min(j.rh, j.reg_y1);
        if (x1 <= x0 || y1 <= y0) x0 = y0 = 0, x1 = y1 = 1;  // empty: one window, harmless
    }
    j.win_x0 = (x0 + j.casx) / cw;
    j.win_y0 = (y0 + j.casy) / th;
    const int tx = (x1 - 1 + j.casx) / cw - j.win_x0 + 1;
    const int ny = (y1 - 1 + j.casy) / th - j.win_y0 + 1;
    j.win_ny = ny;
    j.tiles_x = tx;
    j.ntiles = tx * ((ny + DWT_WAVES - 1) / DWT_WAVES * DWT_WAVES);  // whole workgroups (see dwt_window)
}

// Workgroup order: each XCD gets a contiguous run of windows (dwt_window bit 0).
constexpr int kDwtLay = 1;

template <int TH>
static void launch_th(const DwtJob *jobs, dim3 grid, dim3 block, int irrev, int inverse, int fused, int fmt,
                      hipStream_t s) {
    const int lay = kDwtLay;
    if (fused == 3) {  // forward level 0, MCT triples: one wavefront = the 3 components of one window
        const dim3 g3(grid.x, grid.y / 3);
#define GRK_M3(S)                                                                         \
    if (irrev) hipLaunchKernelGGL((k_dwt_fwd_mct3<true, TH, S>), g3, block, 0, s, jobs, lay); \
    else hipLaunchKernelGGL((k_dwt_fwd_mct3<false, TH, S>), g3, block, 0, s, jobs, lay)
        if (fmt == SMP_U16) { GRK_M3(uint16_t); } else if (fmt == SMP_U8) { GRK_M3(uint8_t); } else { GRK_M3(int32_t); }
#undef GRK_M3
        return;
    }
    if (fused == 1) {  // forward level 0 with the DC shift in the loads
#define GRK_F1(S)                                                                            \
    if (irrev) hipLaunchKernelGGL((k_dwt_fwd<true, TH, 1, S>), grid, block, 0, s, jobs, lay); \
    else hipLaunchKernelGGL((k_dwt_fwd<false, TH, 1, S>), grid, block, 0, s, jobs, lay)
        if (fmt == SMP_U16) { GRK_F1(uint16_t); } else if (fmt == SMP_U8) { GRK_F1(uint8_t); } else { GRK_F1(int32_t); }
#undef GRK_F1
        return;
    }
    if (!inverse) {
        if (irrev && dwt_options().f64_lift)
            hipLaunchKernelGGL((k_dwt_fwd<true, TH, 0, int32_t, double>), grid, block, 0, s, jobs, lay);
        else if (irrev) hipLaunchKernelGGL((k_dwt_fwd<true, TH>), grid, block, 0, s, jobs, lay);
        else hipLaunchKernelGGL((k_dwt_fwd<false, TH>), grid, block, 0, s, jobs, lay);
    } else {
        if (irrev) hipLaunchKernelGGL((k_dwt_inv<true, TH>), grid, block, 0, s, jobs, lay);
        else hipLaunchKernelGGL((k_dwt_inv<false, TH>), grid, block, 0, s, jobs, lay);
    }
}

// Forward levels 0 + 1 of a 9/7 plan in one launch (k_dwt_fwd01); jobs1[i]
// is level 1 of the tile-component of jobs0[i].
hipError_t launch_dwt_fwd01(const DwtJob *jobs0, const DwtJob *jobs1, uint32_t njobs, uint32_t max_tiles, int irrev,
                            int ny, hipStream_t s) {
    if (!njobs || !max_tiles || !irrev) return hipErrorInvalidValue;
    const int lay = kDwtLay | (dwt_options().pair_group << 8);
    const dim3 g(max_tiles, njobs), b(64 * DWT_WAVES);
    switch (ny) {
        case 2: hipLaunchKernelGGL((k_dwt_fwd01<true, 2>), g, b, 0, s, jobs0, jobs1, lay); break;
        case 6: hipLaunchKernelGGL((k_dwt_fwd01<true, 6>), g, b, 0, s, jobs0, jobs1, lay); break;
        default:
            if (dwt_options().f64_lift) hipLaunchKernelGGL((k_dwt_fwd01<true, 4, double>), g, b, 0, s, jobs0, jobs1, lay);
            else hipLaunchKernelGGL((k_dwt_fwd01<true, 4>), g, b, 0, s, jobs0, jobs1, lay);
            break;
    }
    return hipGetLastError();
}

hipError_t launch_dwt_jobs(const DwtJob *jobs_dev, uint32_t njobs, uint32_t max_tiles, int code, int irrev,
                           int inverse, hipStream_t s) {
    if (!njobs || !max_tiles) return hipSuccess;
    dim3 grid((max_tiles + DWT_WAVES - 1) / DWT_WAVES, njobs), block(64 * DWT_WAVES);
    const int fused = inverse ? 0 : (code & DWT_FUSED_MCT3) ? 3 : (code & DWT_FUSED) ? 1 : 0;
    const int fmt = (code >> DWT_FMT_SHIFT) & 7;  // image sample format of a fused level 0
    switch (code & 0xff) {
        case 8: launch_th<8>(jobs_dev, grid, block, irrev, inverse, fused, fmt, s); break;
        case 16: launch_th<16>(jobs_dev, grid, block, irrev, inverse, fused, fmt, s); break;
        case 24: launch_th<24>(jobs_dev, grid, block, irrev, inverse, fused, fmt, s); break;
        case 32: launch_th<32>(jobs_dev, grid, block, irrev, inverse, fused, fmt, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace grkgpu
