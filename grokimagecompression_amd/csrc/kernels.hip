// kernels.hip -- CDNA4 (gfx950) kernels for the JPEG 2000 hot path.
//
//   * pointwise: DC level shift + RCT/ICT (forward), inverse RCT/ICT + DC
//     shift + clamp (TileProcessor.cpp:1449-1518 / 1303-1432, mct/mct.cpp)
//   * DWT: see dwt.hip
//   * T1: EBCOT encode / decode, one lane per code-block (t1_lane.h).
//   * gather: compacts per-code-block MQ output into one contiguous buffer.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "grk_device.h"
#include "t1_flat.h"
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

namespace grkgpu {

__constant__ uint32_t c_mq_tab[47] = GRK_MQ_TABLE_INIT;

// ---------------------------------------------------------------------------
// pointwise
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t fix_mul13(int32_t a, int32_t b) {
    int64_t t = (int64_t)a * (int64_t)b + 4096;
    return (int32_t)(t >> 13);
}

// NT: non-temporal stores (the output is streamed to HBM instead of lingering
// dirty in the caches for the next kernel to evict).
template <bool NT>
__device__ __forceinline__ void put(int32_t *p, int32_t v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// src: image planes of samples S (row stride sstride), dst: tile-component
// buffers (row stride tw).  One thread per sample of the tile.
template <bool NT, typename S>
__global__ void k_dcshift_mct_fwd(SrcPlanes src, uint32_t sstride, PlanePtrs dst, uint32_t tw, uint32_t th,
                                  uint32_t ncomp, ShiftArr shift, int32_t mct, int32_t irrev) {
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y = blockIdx.y;
    if (x >= tw || y >= th) return;
    size_t si = (size_t)y * sstride + x, di = (size_t)y * tw + x;
    auto smp = [&](uint32_t c) { return (int32_t)((const S *)src.p[c])[si]; };
    uint32_t c0 = 0;
    if (mct && ncomp >= 3) {
        int32_t r = smp(0) - shift.v[0], g = smp(1) - shift.v[1], b = smp(2) - shift.v[2];
        int32_t o0, o1, o2;
        if (!irrev) {
            o0 = (r + (g * 2) + b) >> 2;
            o1 = b - g;
            o2 = r - g;
        } else {
            o0 = ict_term(r, 2449) + ict_term(g, 4809) + ict_term(b, 934);
            o1 = -ict_term(r, 1382) - ict_term(g, 2714) + ict_term(b, 4096);
            o2 = ict_term(r, 4096) - ict_term(g, 3430) - ict_term(b, 666);
        }
        put<NT>(&dst.p[0][di], o0); put<NT>(&dst.p[1][di], o1); put<NT>(&dst.p[2][di], o2);
        c0 = 3;
    }
    for (uint32_t c = c0; c < ncomp; ++c) {
        int32_t v = smp(c) - shift.v[c];
        put<NT>(&dst.p[c][di], irrev ? (int32_t)((uint32_t)v << 11) : v);
    }
}

// DC shift + custom array-based MCT (Part 2): TileProcessor.cpp:1449-1471
// then mct::encode_custom (mct.cpp:429-475) -- (x - shift) << 11, then per
// output component j the int32 sum over k of int_fix_mul(C[j][k], x_k), C the
// encoding matrix in 13-bit fixed point, in the reference's order.
template <typename S>
__global__ void k_dcshift_mct_custom(SrcPlanes src, uint32_t sstride, PlanePtrs dst, uint32_t tw, uint32_t th,
                                     uint32_t ncomp, ShiftArr shift, MctMatrix m) {
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y = blockIdx.y;
    if (x >= tw || y >= th) return;
    size_t si = (size_t)y * sstride + x, di = (size_t)y * tw + x;
    int32_t v[GRK_MAX_COMPS];
    for (uint32_t c = 0; c < ncomp; ++c)
        v[c] = (int32_t)((uint32_t)((int32_t)((const S *)src.p[c])[si] - shift.v[c]) << 11);
    for (uint32_t j = 0; j < ncomp; ++j) {
        uint32_t acc = 0;
        for (uint32_t k = 0; k < ncomp; ++k)
            acc += (uint32_t)(int32_t)(((int64_t)m.c[j * ncomp + k] * (int64_t)v[k] + 4096) >> 13);
        put<true>(&dst.p[j][di], (int32_t)acc);
    }
}

// Inverse MCT + DC shift + clamp, tile buffers -> image planes.
__global__ void k_mct_inv_dcshift(PlanePtrs src, uint32_t sstride, uint32_t tw, uint32_t th, PlanePtrs dst,
                                  uint32_t dstride, uint32_t ncomp, ShiftArr shift, ShiftArr minv, ShiftArr maxv,
                                  int32_t mct, int32_t irrev) {
    uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t y = blockIdx.y;
    if (x >= tw || y >= th) return;
    size_t si = (size_t)y * sstride + x, di = (size_t)y * dstride + x;
    uint32_t c0 = 0;
    if (mct && ncomp >= 3) {
        int32_t o[3];
        if (!(irrev & 1)) {
            int32_t yv = src.p[0][si], u = src.p[1][si], v = src.p[2][si];
            int32_t g = yv - ((u + v) >> 2);
            o[0] = v + g; o[1] = g; o[2] = u + g;
        } else {
            float yv = __int_as_float(src.p[0][si]), u = __int_as_float(src.p[1][si]), v = __int_as_float(src.p[2][si]);
            // mct::decode_irrev (mct.cpp:352-408): separate mul/add, no FMA
            float r = __fadd_rn(yv, __fmul_rn(v, 1.402f));
            float g = __fsub_rn(__fsub_rn(yv, __fmul_rn(u, 0.34413f)), __fmul_rn(v, 0.71414f));
            float b = __fadd_rn(yv, __fmul_rn(u, 1.772f));
            o[0] = (int32_t)rintf(r); o[1] = (int32_t)rintf(g); o[2] = (int32_t)rintf(b);
        }
        for (int c = 0; c < 3; ++c) {
            int32_t v = o[c] + shift.v[c];
            dst.p[c][di] = v < minv.v[c] ? minv.v[c] : (v > maxv.v[c] ? maxv.v[c] : v);
        }
        c0 = 3;
    }
    for (uint32_t c = c0; c < ncomp; ++c) {
        int32_t v = src.p[c][si];
        if ((irrev >> c) & 1) v = (int32_t)rintf(__int_as_float(v));
        v += shift.v[c];
        dst.p[c][di] = v < minv.v[c] ? minv.v[c] : (v > maxv.v[c] ? maxv.v[c] : v);
    }
}

// ---------------------------------------------------------------------------
// T1 (t1_lane.h).  Encode = prep (wave per block: quantise, sign rows, numbps,
// magnitude bit-planes via ballots) + lane coder (one lane per block).
// Decode = lane decoder (one lane per block, write-only bit-plane rows) +
// rebuild (workgroup per block: values + post-decode scaling, coalesced).
// ---------------------------------------------------------------------------
// Lane-interleaved rows (t1_lane.h) through buffer instructions: the group's
// region is one buffer resource (wave-uniform, SGPRs) and a row access is a
// 32-bit lane offset, so the decoder keeps one offset VGPR per row index
// instead of a 64-bit pointer per state array.
struct LRef {
    __amdgpu_buffer_rsrc_t r;
    uint32_t so, vo;
    __device__ operator uint64_t() const {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0);
        return (uint64_t)v[0] | ((uint64_t)v[1] << 32);
    }
    __device__ const LRef &operator=(uint64_t v) const {
        const __attribute__((ext_vector_type(2))) uint32_t p = {(uint32_t)v, (uint32_t)(v >> 32)};
        __builtin_amdgcn_raw_buffer_store_b64(p, r, vo, so, 0);
        return *this;
    }
};
// so: the field's byte offset (scalar); vo: the lane's byte offset + rows
struct LRow {
    __amdgpu_buffer_rsrc_t r;
    uint32_t so, vo;
    __device__ LRef operator[](uint32_t y) const { return LRef{r, so, vo + y * 512u}; }
    __device__ LRow operator+(uint32_t n) const { return LRow{r, so, vo + n * 512u}; }
};
// the buffer resource of one 64-block group of lane-interleaved rows
__device__ __forceinline__ __amdgpu_buffer_rsrc_t group_rsrc(void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
}
template <int LANES>
__device__ __forceinline__ void t1_tables_init(uint8_t *zc, uint8_t *sc, uint32_t *mq) {
    for (uint32_t k = threadIdx.x; k < 2048; k += LANES) zc[k] = zc_lut_entry(k >> 9, k & 511);
    for (uint32_t k = threadIdx.x; k < 256; k += LANES) sc[k] = sc_lut_entry(k);
    for (uint32_t k = threadIdx.x; k < 47; k += LANES) mq[k] = c_mq_tab[k];
    __syncthreads();
}

// One wavefront per block, lane = row.  Workgroup b runs on XCD b % 8 (the
// dispatcher deals workgroups round-robin), so the 64 blocks of group g are
// given to workgroups of one XCD, back to back: their row words, 8 bytes per
// lane at a 512-byte stride (the group layout, t1_lane.h EncScratch), meet as
// whole lines in that XCD's L2.
__global__ __launch_bounds__(64) void k_t1_prep(const EncBlock *__restrict__ blocks, uint32_t n, uint32_t maxdepth,
                                                const int32_t *__restrict__ coef, uint8_t *__restrict__ scr,
                                                EncResult *__restrict__ res) {
    const uint32_t wg = blockIdx.x, k = wg >> 3;
    const uint32_t i = (((k >> 6) << 3) | (wg & 7)) * 64 + (k & 63), x = threadIdx.x;
    if (i >= n) return;
    const EncBlock b = blocks[i];
    const int32_t *src = coef + b.coef_off;
    uint32_t m[64];
    uint64_t negrow = 0;
    uint32_t orv = 0;
#pragma unroll
    for (int y = 0; y < 64; ++y) {
        uint32_t mv = 0, ng = 0;
        if ((uint32_t)y < b.h && x < b.w) mv = quant_mag(src[(size_t)y * b.stride + x], b.qmfbid, b.inv_step, &ng);
        m[y] = mv;
        orv |= mv;
        uint64_t bal = __ballot(ng);
        if (x == (uint32_t)y) negrow = bal;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) orv |= __shfl_xor(orv, off);
    uint32_t numbps = 0;
    if (orv) {
        uint32_t t = 32u - (uint32_t)__clz(orv);
        numbps = t <= 6 ? 0 : t - 6;
    }
    const EncScratch E = enc_scratch(scr, n, maxdepth);
    uint64_t *G = E.group(i >> 6) + (i & 63);  // row R of this block: G[R * 64]
    G[(T1E_NEG + x + 1) * 64] = x < b.h ? negrow : 0;
    if (x == 0) G[T1E_NEG * 64] = 0;
    if (x == 63) G[(T1E_NEG + 65) * 64] = 0;
    const uint32_t nd = numbps < maxdepth ? numbps : maxdepth;  // numbps > maxdepth: refused (res.pad)
    uint64_t acc = 0;  // significance before plane p = OR of the planes above
    for (uint32_t d = 0; d < nd; ++d) {
        const uint32_t p = numbps - 1 - d;
        uint64_t mine = 0;
#pragma unroll
        for (int y = 0; y < 64; ++y) {
            uint64_t bal = __ballot((m[y] >> (p + 6)) & 1u);
            if (x == (uint32_t)y) mine = bal;
        }
        if (x < b.h) {
            G[(t1e_depth_row(d) + T1E_BITS + x) * 64] = mine;
            G[(t1e_depth_row(d) + T1E_ABOVE + x) * 64] = acc;
        }
        acc |= mine;
    }
    if (x == 0) {
        res[i].numbps = numbps;
        res[i].pad = 0;
    }
}

// Context modelling, one lane per (block, bit-plane): lanes are laid out
// depth-major (depth = numbps-1-p) so a wavefront holds the same depth of the
// 64 blocks of a group -- similar statistics, little divergence -- and, with
// the group-interleaved rows of t1_lane.h EncScratch, every row access of the
// wavefront is one 512-byte run.  Per-block rows (round 4) had each lane read
// its own 8-byte rows from 64 different lines, evicted between stripes: 3.3-3.7
// GB read per 8K 9/7 frame; interleaved 1.2-1.3 GB (profiles/r05/
// t1_model_interleave.txt), the post-SPP / visited rows moved from the symbol
// slots into the group rows with them.
__device__ __forceinline__ uint64_t sym_block_off(const uint64_t *sym_off, uint32_t i, uint32_t *cap) {
    if (!sym_off) {
        *cap = 32;
        return (uint64_t)i * 32 * sym_slot_bytes(64, 64);
    }
    return sym_off[i];
}

template <bool COND>
__global__ __launch_bounds__(64) void k_t1_model(
    const EncBlock *__restrict__ blocks, uint32_t n, uint32_t maxdepth, uint8_t *__restrict__ scr,
    uint8_t *__restrict__ sym, const uint64_t *__restrict__ sym_off, EncResult *__restrict__ res, uint32_t cblksty) {
    __shared__ uint8_t s_sc[256];
    __shared__ uint32_t s_ring[32 * 64];  // SymOut: 32 words per lane, word j at (j % 32) * 64 + lane
    for (uint32_t k = threadIdx.x; k < 256; k += 64) s_sc[k] = sc_lut_entry(k);
    __syncthreads();
    // wavefront = (group, depth): lane = the group's block
    const uint32_t n64 = t1_scratch_records(n), w0 = blockIdx.x * 64;
    const uint32_t g0 = w0 % n64, d = w0 / n64, i = g0 + threadIdx.x;
    if (d >= maxdepth || i >= n) return;
    const uint32_t numbps = res[i].numbps;
    if (d >= numbps) return;
    const EncBlock b = blocks[i];
    const uint32_t slot = sym_slot_bytes(b.w, b.h);
    uint32_t cap = 0;
    const uint64_t off = sym_block_off(sym_off, i, &cap);
    if (sym_off) cap = (uint32_t)((sym_off[i + 1] - off) / slot);
    if (numbps > cap) {
        if (d == 0) res[i].pad = 1;  // numbps above the band's bound: reported by the host
        return;
    }
    const uint32_t p = numbps - 1 - d;
    const EncScratch E = enc_scratch(scr, n, maxdepth);
    const __amdgpu_buffer_rsrc_t gr = group_rsrc(E.group(g0 >> 6), 64 * E.rec_rows * 8);
    const uint32_t lo = threadIdx.x * 8, dr = t1e_depth_row(d);
    const LRow bits{gr, (dr + T1E_BITS) * 512, lo}, above{gr, (dr + T1E_ABOVE) * 512, lo};
    const LRow ref{gr, (d ? dr - T1E_DEPTH_ROWS + T1E_ABOVE : 0) * 512, lo}, negr{gr, T1E_NEG * 512, lo};
    const LRow tmp{gr, (dr + T1E_POST) * 512, lo};
    uint8_t *base = sym + off + (uint64_t)p * slot;
    t1_model_plane<LRow, LRow, COND>(b.w, b.h, b.orient, bits, above, ref, d > 0, negr, tmp, s_sc, (uint32_t *)base,
                   E.cnt + (size_t)i * 128 + p * 4, cblksty, t1_pass_raw(cblksty, (int32_t)p, 0, numbps),
                   s_ring + threadIdx.x);
}

constexpr uint32_t MQ_CX_STRIDE = 21;  // LDS words per lane for the MQ encoder's context words

// MQ coding, one lane per block (lane j codes block perm[j], or j).  WAVES
// wavefronts per workgroup share the state table and the read-ahead slack
// (CXS: context words per lane).
template <int LANES, int MINW = 1, bool LAZY = false, int WAVES = 1, uint32_t CXS = MQ_CX_STRIDE>
__global__ __launch_bounds__(LANES * WAVES, MINW) void k_t1_mq(const EncBlock *__restrict__ blocks, uint32_t n,
                                                 const uint32_t *__restrict__ cnt, const uint8_t *__restrict__ sym,
                                                 const uint64_t *__restrict__ sym_off, uint8_t *__restrict__ out,
                                                 EncResult *__restrict__ res, const uint32_t *__restrict__ perm,
                                                 uint32_t cblksty, uint32_t bpw) {
    __shared__ uint32_t s_mq[48];
    // 19 context words per lane at an odd stride (no bank conflicts).  The
    // read-ahead of the symbol after a pass's last one may index up to 31
    // (its value is never used): the next lane's slots, or for the last lane
    // the tail slack, keep it inside the array.
    __shared__ uint32_t s_cx[WAVES * LANES * CXS + 32];
    for (uint32_t k = threadIdx.x; k < 47; k += LANES * WAVES) s_mq[k] = c_mq_tab[k];
    __syncthreads();
    const uint32_t lane = threadIdx.x % LANES;
    if (lane >= bpw) return;  // bpw blocks per wavefront (t1_blocks_per_wave)
    const uint32_t j = (blockIdx.x * WAVES + threadIdx.x / LANES) * bpw + lane;
    if (j >= n) return;
    const uint32_t i = perm ? perm[j] : j;
    const EncBlock b = blocks[i];
    EncResult &r = res[i];
    if (r.pad) return;
    uint32_t cap;
    const uint64_t off = sym_block_off(sym_off, i, &cap);
    uint32_t len;
    uint32_t np = t1_mq_block<LAZY>(r.numbps, (const uint32_t *)(sym + off), sym_slot_bytes(b.w, b.h) / 4, cnt + (size_t)i * 128, s_mq,
                              s_cx + threadIdx.x * CXS, (uint32_t *)(out + b.out_off), r.rate, &len, cblksty);
    r.numpasses = np;
    r.len = len;
    uint32_t nsym = 0;
    const uint32_t *c = cnt + (size_t)i * 128;
    for (uint32_t q = 0; q < r.numbps && q < 32; ++q) nsym += c[q * 4] + c[q * 4 + 1] + c[q * 4 + 2];
    r.nsym = nsym;
}

// Work order for k_t1_mq (the decoder's host-side order, on the device: the
// encoder's work per block is only known after k_t1_model).  A counting sort
// of the blocks by their symbol count, heaviest first, in MQ_ORDER_BUCKETS
// log-spaced buckets (8 per octave): per block its bucket, a histogram with
// vector atomics, an exclusive scan in one workgroup, then a scatter.  The
// order inside a bucket follows the atomics (it varies from run to run);
// every block's output is its own, so the codestream does not.
constexpr uint32_t MQ_ORDER_BUCKETS = 256;
__device__ __forceinline__ uint32_t mq_work_bucket(const uint32_t *c, uint32_t numbps) {
    uint32_t w = 0;
    for (uint32_t q = 0; q < numbps && q < 32; ++q) w += c[q * 4] + c[q * 4 + 1] + c[q * 4 + 2];
    w += 1;
    const uint32_t o = 31u - (uint32_t)__builtin_clz(w);            // octave
    const uint32_t f = o >= 3 ? (w >> (o - 3)) & 7u : (w << (3 - o)) & 7u;  // 3 bits below the top one
    return (MQ_ORDER_BUCKETS - 1) - min((o << 3) | f, MQ_ORDER_BUCKETS - 1);  // heaviest first
}
__global__ __launch_bounds__(256) void k_mq_order_hist(const uint32_t *__restrict__ cnt,
                                                      const EncResult *__restrict__ res, uint32_t n,
                                                      uint32_t *__restrict__ key, uint32_t *__restrict__ hist) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = mq_work_bucket(cnt + (size_t)i * 128, res[i].numbps);
    key[i] = k;
    atomicAdd(&hist[k], 1u);
}
__global__ __launch_bounds__(MQ_ORDER_BUCKETS) void k_mq_order_scan(uint32_t *__restrict__ hist) {
    __shared__ uint32_t s[MQ_ORDER_BUCKETS];
    const uint32_t t = threadIdx.x;
    s[t] = hist[t];
    __syncthreads();
    for (uint32_t d = 1; d < MQ_ORDER_BUCKETS; d <<= 1) {  // inclusive Hillis-Steele scan
        const uint32_t v = t >= d ? s[t - d] : 0u;
        __syncthreads();
        s[t] += v;
        __syncthreads();
    }
    hist[t] = s[t] - hist[t];  // exclusive: the bucket's first slot
}
__global__ __launch_bounds__(256) void k_mq_order_scatter(const uint32_t *__restrict__ key, uint32_t n,
                                                         uint32_t *__restrict__ next, uint32_t *__restrict__ perm) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    perm[atomicAdd(&next[key[i]], 1u)] = i;
}

// Per-pass distortion sums (the nmsedec of t1_enc_sigpass / refpass /
// clnpass, t1.cpp:197-338, 443-555, 639-782 with t1_getnmsedec_sig/_ref
// :155-166): one wavefront per block, lane = column.  A sample contributes
// to the plane of its most significant bit (significance: to the SPP when
// the modelling kernel found it significant during that plane's SPP, else
// to the cleanup pass) and to every lower plane's refinement pass.  The
// SPP membership comes from the post-SPP significance rows k_t1_model left
// behind each plane's symbol stream.
__global__ __launch_bounds__(64) void k_t1_dist(const EncBlock *__restrict__ blocks, uint32_t n, uint32_t maxdepth,
                                                const int32_t *__restrict__ coef, const uint8_t *__restrict__ scr,
                                                EncResult *__restrict__ res, NmseLut lutv) {
    __shared__ NmseLut lut;
    {
        const int16_t *src = &lutv.sig[0];
        int16_t *dst = &lut.sig[0];
        for (uint32_t k = threadIdx.x; k < 512; k += 64) dst[k] = src[k];
    }
    __syncthreads();
    const uint32_t i = blockIdx.x, x = threadIdx.x;
    const EncBlock b = blocks[i];
    EncResult &r = res[i];
    const uint32_t numbps = r.numbps;
    if (numbps == 0 || r.pad) return;
    const int32_t *src = coef + b.coef_off;
    uint32_t m[64];
#pragma unroll
    for (int y = 0; y < 64; ++y) {
        uint32_t ng;
        m[y] = ((uint32_t)y < b.h && x < b.w) ? quant_mag(src[(size_t)y * b.stride + x], b.qmfbid, b.inv_step, &ng) : 0;
    }
    const EncScratch E = enc_scratch(const_cast<uint8_t *>(scr), n, maxdepth);
    const uint64_t *G = E.group(i >> 6) + (i & 63);
    for (int32_t p = (int32_t)numbps - 1; p >= 0; --p) {
        // the block's post-SPP significance rows of plane p (row y at post[y * 64])
        const uint64_t *post = G + (size_t)(t1e_depth_row(numbps - 1 - (uint32_t)p) + T1E_POST) * 64;
        int32_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
        for (int y = 0; y < 64; ++y) {
            const uint32_t mag = (uint32_t)y < b.h ? m[y] : 0u;  // no break: m stays in registers
            const uint32_t win = p > 0 ? (mag >> p) & 127u : mag & 127u;
            if ((mag >> (p + 6)) == 1u) {
                const int32_t v = p > 0 ? lut.sig[win] : lut.sig0[win];
                if ((post[(size_t)y * 64] >> x) & 1u) a0 += v; else a2 += v;
            } else if (mag >> (p + 7)) {
                a1 += p > 0 ? lut.ref[win] : lut.ref0[win];
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            a0 += __shfl_xor(a0, o);
            a1 += __shfl_xor(a1, o);
            a2 += __shfl_xor(a2, o);
        }
        if (x == 0) {
            if (p == (int32_t)numbps - 1) {
                r.nmsedec[0] = a2;
            } else {
                const uint32_t base = 1 + 3 * (numbps - 2 - (uint32_t)p);
                r.nmsedec[base] = a0;
                r.nmsedec[base + 1] = a1;
                r.nmsedec[base + 2] = a2;
            }
        }
    }
}

// T1 decoder (t1_flat.h t1_decode_v5).  Pass 1, lane per block: remove the MQ
// byte stuffing into a plain bit stream + carry events (region of block i at
// ubuf + i * fixed_words words, or at blocks[i].pad * 16 bytes when
// fixed_words == 0: header {nwords, ncarry}, words, carries).  Pass 2, lane
// per block: the pass / stripe / column walk over the unstuffed stream.
__device__ __forceinline__ size_t ub_region(const DecBlock &b, uint32_t i, uint32_t fixed_words) {
    return fixed_words ? (size_t)i * fixed_words : (size_t)b.pad * 4;
}

// unstuff one segment (len bytes at data + data_off) into region: header
// {nwords, ncarry}, words, carries
__device__ __forceinline__ void unstuff_segment(const uint8_t *__restrict__ data, uint64_t data_off, uint32_t len,
                                                uint32_t *__restrict__ region) {
    uint32_t *words = region + 4, *carries = words + unstuff_word_cap(len);
    const uintptr_t pa = (uintptr_t)(data + data_off);
    const uint4 *src = (const uint4 *)(pa & ~(uintptr_t)15);
    const uint32_t skip = (uint32_t)(pa & 15), end = skip + len;
    const uint32_t nch = (end + 15) >> 4;
    Unstuff u;
    uint32_t nw = 0, nc = 0;
    uint4 nxt = nch ? src[0] : uint4{0, 0, 0, 0};
    for (uint32_t ch = 0; ch < nch; ++ch) {
        const uint4 cur = nxt;
        if (ch + 1 < nch) nxt = src[ch + 1];
        const uint32_t wv4[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t pos = ch * 16 + j;
            if (pos < skip || pos >= end) continue;
            uint32_t wv, cv;
            if (u.push((wv4[j >> 2] >> (8 * (j & 3))) & 0xffu, &wv, &cv)) words[nw++] = wv;
            if (cv != 0xffffffffu) carries[nc++] = cv;
        }
    }
    words[nw++] = u.tail();
    do { words[nw++] = 0xffffffffu; } while (nw & 3);
    for (int k = 0; k < 8; ++k) words[nw++] = 0xffffffffu;
    carries[nc] = 0xffffffffu;
    region[0] = nw;
    region[1] = nc;
}

// segs / seg_first (codestream decode): block i's segments are
// segs[seg_first[i] .. seg_first[i+1]); null: one segment per block at
// blocks[i].data_off (the stage entry point)
__global__ __launch_bounds__(64) void k_t1_unstuff(const DecBlock *__restrict__ blocks, uint32_t n,
                                                   const uint8_t *__restrict__ data, uint32_t *__restrict__ ubuf,
                                                   uint32_t fixed_words, const DecSeg *__restrict__ segs,
                                                   const uint32_t *__restrict__ seg_first) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const DecBlock b = blocks[i];
    if (b.len == 0 || b.numpasses == 0 || b.numbps == 0 || b.numbps > T1_MAX_DEC_BPS) return;
    if (segs) {
        for (uint32_t q = seg_first[i]; q < seg_first[i + 1]; ++q) {
            const DecSeg sg = segs[q];
            unstuff_segment(data, sg.data_off, sg.len, ubuf + (size_t)sg.ub_off * 4);
        }
        return;
    }
    unstuff_segment(data, b.data_off, b.len, ubuf + ub_region(b, i, fixed_words));
}

// The same pre-pass with one wavefront per code-block segment: 64 bytes per
// step, one per lane.  A byte's bit count (7 after a 0xFF, else 8) and its
// bit position in the output stream come from a wave prefix sum, its bits are
// ORed into the step's words in LDS (a byte may straddle two words), the
// completed words leave as one coalesced store, the partial last one stays
// for the next step; a marker (0xFF then > 0x8F) ends the stream at the first
// lane holding one, and carry events are compacted by ballot in stream
// order.  Output identical to unstuff_segment's.  The lane-per-block pass runs
// 64 blocks' serial byte loops per wavefront -- ~390 wavefronts for a whole
// 8K frame, a long dependent chain per lane: the shorter chain for a call
// alone on the GPU, the fewer instructions for a batch (launch_t1_decode).
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane, uint32_t *tot) {
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        x += lane >= (uint32_t)d ? y : 0u;
    }
    *tot = __shfl(x, 63, 64);
    return x - v;
}

__device__ void unstuff_segment_wave(const uint8_t *__restrict__ data, uint64_t data_off, uint32_t len,
                                     uint32_t *__restrict__ region, uint32_t *wbuf, uint32_t lane) {
    uint32_t *words = region + 4, *carries = words + unstuff_word_cap(len);
    uint32_t bitpos = 0, nc = 0;  // bits emitted, carry events written
    bool pff_in = false;          // the byte before this step's first one is 0xFF
    if (lane < 20) wbuf[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (uint32_t base = 0; base < len; base += 64) {
        const uint32_t j = base + lane;
        const bool inb = j < len;
        const uint32_t b = inb ? (uint32_t)data[data_off + j] : 0u;
        const uint32_t prev = __shfl_up(b, 1, 64);
        const bool pff = lane ? prev == 0xffu : pff_in;
        const uint64_t mk = __ballot(inb && pff && b > 0x8fu);  // markers: the stream ends at the first
        const uint32_t first = mk ? (uint32_t)__builtin_ctzll(mk) : 64u;
        const bool valid = inb && lane < first;
        const uint32_t nb = valid ? (pff ? 7u : 8u) : 0u;
        uint32_t tot;
        const uint32_t o = bitpos + wave_excl_scan(nb, lane, &tot);
        // carry event: a stuffed byte's top bit (see Unstuff)
        const bool ev = valid && pff && (b & 0x80u);
        const uint64_t em = __ballot(ev);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
        if (ev) carries[nc + rank] = o - 1 + 17;
        nc += (uint32_t)__builtin_popcountll(em);
        // the byte's bits at stream bits [o, o + nb), MSB first; word index relative to this step's first
        if (nb) {
            const uint32_t v = b & (pff ? 0x7fu : 0xffu);
            const uint32_t k = (o >> 5) - (bitpos >> 5), p = o & 31u, e = p + nb;
            if (e <= 32) {
                atomicOr(&wbuf[k], v << (32 - e));
            } else {
                atomicOr(&wbuf[k], v >> (e - 32));
                atomicOr(&wbuf[k + 1], v << (64 - e));
            }
        }
        // one wavefront's LDS operations complete in order; the fence keeps the
        // compiler from moving the reads above the ORs (no workgroup barrier:
        // the other wavefronts of the workgroup work on other blocks)
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t end = bitpos + tot, done = (end >> 5) - (bitpos >> 5);  // completed words
        uint32_t w = lane < 20 ? wbuf[lane] : 0u;
        if (lane < done) words[(bitpos >> 5) + lane] = w;
        // the partial word moves to slot 0, the rest is cleared
        const uint32_t carry_w = __shfl(w, (int)done, 64);
        if (lane < 20) wbuf[lane] = lane == 0 ? carry_w : 0u;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        bitpos = end;
        pff_in = __shfl(b, 63, 64) == 0xffu;
        if (mk) break;
    }
    // tail (Unstuff::tail): the pending bits, then 1-bits; a word of 1-bits
    // when none is pending; then 1-bit words to a multiple of 4 and 8 more
    const uint32_t nw0 = bitpos >> 5, pend = bitpos & 31u;
    const uint32_t w0 = __shfl(lane < 20 ? wbuf[lane] : 0u, 0, 64);
    const uint32_t tailw = pend ? (w0 | ((1u << (32 - pend)) - 1u)) : 0xffffffffu;
    uint32_t nw = nw0 + 1;
    nw += (4 - (nw & 3)) & 3;
    if ((nw - nw0 - 1) == 0) nw += 4;  // the serial pass writes at least one 1-bit word after the tail
    nw += 8;
    for (uint32_t q = lane; nw0 + q < nw; q += 64) words[nw0 + q] = q == 0 ? tailw : 0xffffffffu;
    if (lane == 0) {
        carries[nc] = 0xffffffffu;
        region[0] = nw;
        region[1] = nc;
    }
}

__global__ __launch_bounds__(256) void k_t1_unstuff_w(const DecBlock *__restrict__ blocks, uint32_t n,
                                                     const uint8_t *__restrict__ data, uint32_t *__restrict__ ubuf,
                                                     uint32_t fixed_words, const DecSeg *__restrict__ segs,
                                                     const uint32_t *__restrict__ seg_first) {
    __shared__ uint32_t s_w[4][20];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 4 + wv;
    if (i >= n) return;
    const DecBlock b = blocks[i];
    if (b.len == 0 || b.numpasses == 0 || b.numbps == 0 || b.numbps > T1_MAX_DEC_BPS) return;
    if (segs) {
        for (uint32_t q = seg_first[i]; q < seg_first[i + 1]; ++q) {
            const DecSeg sg = segs[q];
            unstuff_segment_wave(data, sg.data_off, sg.len, ubuf + (size_t)sg.ub_off * 4, s_w[wv], lane);
        }
        return;
    }
    unstuff_segment_wave(data, b.data_off, b.len, ubuf + ub_region(b, i, fixed_words), s_w[wv], lane);
}

struct LState {
    LRow sig, neg, vis, ref;
};

// Decoder workgroups: DEC_WAVES wavefronts share one copy of the LUTs in LDS,
// and the kernel is held to 128 VGPRs (a few spills at pass boundaries), so 4
// wavefronts fit per SIMD by both registers and LDS (38 KB per workgroup: the
// LUTs, 19 context words per lane -- odd, so the lanes spread over the banks --
// and the bit readers' word rings).  Against one wavefront per workgroup at 144
// VGPRs (3 per SIMD): 8K batch 3264-3280 -> 3507-3508 Mpixels/s, lone decode
// T1 31.7-31.9 -> 30.9-31.3 ms (profiles/r05/t1_dec_wg_ab.txt).  (Round 3's
// 128-VGPR build with single-wavefront workgroups had measured no gain: LDS
// then still held it near 3 per SIMD.)
constexpr int DEC_WAVES = 4;
constexpr uint32_t DEC_CX_STRIDE = 19;

template <int LANES, bool LAZY, int WAVES, int WPE>
__global__ __launch_bounds__(LANES * WAVES) __attribute__((amdgpu_waves_per_eu(WPE))) void k_t1_decode_ub(const DecBlock *__restrict__ blocks, uint32_t n,
                                                        const uint32_t *__restrict__ ubuf, uint32_t fixed_words,
                                                        T1Scratch *__restrict__ scr, const DecSeg *__restrict__ segs,
                                                        const uint32_t *__restrict__ seg_first, uint32_t sty,
                                                        const uint8_t *__restrict__ roi, uint32_t bpw) {
    __shared__ uint8_t s_zc[2048];
    __shared__ uint8_t s_sc[256];
    __shared__ uint32_t s_mq[MQ_DEC_WORDS + 2];  // decoder successor table (t1_lane.h mq_dec_table_entry)
    __shared__ uint32_t s_cx[WAVES * LANES * DEC_CX_STRIDE];
    __shared__ uint32_t s_ring[WAVES * LANES * FB_RING];  // bit readers' word rings (t1_flat.h FlatBits), slot stride 64
    static_assert(LANES == 64, "the word rings interleave 64 lanes");
    for (uint32_t k = threadIdx.x; k < 2048; k += LANES * WAVES) s_zc[k] = zc_lut_entry(k >> 9, k & 511);
    for (uint32_t k = threadIdx.x; k < 256; k += LANES * WAVES) s_sc[k] = sc_win_entry(k);
    for (uint32_t k = threadIdx.x; k < MQ_DEC_WORDS; k += LANES * WAVES) s_mq[k] = mq_dec_table_entry(c_mq_tab, k);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane >= bpw) return;  // bpw blocks per wavefront (t1_blocks_per_wave)
    const uint32_t gw = blockIdx.x * WAVES + wv;  // the wavefront's index in the grid
    const uint32_t i = gw * bpw + lane;
    if (i >= n) return;
    const DecBlock b = blocks[i];
    if (b.len == 0 || b.numpasses == 0 || b.numbps == 0 || b.numbps > T1_MAX_DEC_BPS) return;
    const DecTables T{s_zc + b.orient * 512, s_sc, s_mq};
    // lane-interleaved state and bit-plane rows of this block (t1_lane.h T1Group)
    // bpw is a power of two <= 64, so the wavefront's blocks share one group:
    // the group (and the buffer resource) stays wave-uniform, in SGPRs
    const uint32_t grp = __builtin_amdgcn_readfirstlane((gw * bpw) >> 6);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        t1_group_base(scr, grp, sizeof(T1Scratch)), 0, (int)(64 * sizeof(T1Scratch)), 0x00020000);
    const uint32_t lo = (i & 63) * 8;
    LState st{LRow{gr, T1R_SIG * 512, lo}, LRow{gr, T1R_NEG * 512, lo}, LRow{gr, T1R_VIS * 512, lo},
              LRow{gr, T1R_REF * 512, lo}};
    const LRow pa{gr, T1R_PA * 512, lo}, pb{gr, T1R_PB * 512, lo};
    uint32_t *const ring = s_ring + wv * (LANES * FB_RING) + lane;
    uint32_t *cxw = s_cx + threadIdx.x * DEC_CX_STRIDE;
    if (segs) {
        const uint32_t q0 = seg_first[i], nseg = seg_first[i + 1] - q0;
        const DecSeg s0 = segs[q0];
        const uint32_t *region = ubuf + (size_t)s0.ub_off * 4;
        for (uint32_t y = 0; y < b.h + 2; ++y) { st.sig[y] = 0; st.neg[y] = 0; st.vis[y] = 0; st.ref[y] = 0; }
        mq_reset_words_dec(cxw, T.mq);
        BitDecT<LAZY> d;
        d.set_ring(ring, 6);
        d.init(region + 4, region[0], region + 4 + unstuff_word_cap(s0.len));
        SegCursor cur{segs + q0, ubuf, nseg, 0, s0.npasses};
        t1_decode_passes(d, b.numpasses, b.numbps, b.w, b.h, st, T, cxw, pa, pb, sty, cur, roi ? roi[i] : 0u);
        return;
    }
    const uint32_t *region = ubuf + ub_region(b, i, fixed_words);
    t1_decode_v5(region + 4, region[0], region + 4 + unstuff_word_cap(b.len), b.numpasses, b.numbps, b.w, b.h, st, T,
                 cxw, pa, pb, ring, 6);
}

// Rebuild of the decoded values from the lane-interleaved bit-plane rows:
// one workgroup of 4 wavefronts per (64-block group, RB_ROWS rows).  For
// each row, lane l of every wavefront stages its block's plane words of that
// row into LDS (wavefront w takes the planes q = w mod 4; one 512-byte run
// per plane); then wavefront w takes blocks b = w mod 4, and lane x forms
// coefficient (y, x) from the LDS words (broadcast reads; the block's
// parameters by readlane) and the row is stored coalesced.  Then
// T1Part1::postDecode scaling (5/3: v/2, 9/7: float(v) * step).  roi (null:
// none): per-block ROI up-shift -- T1Part1::post_decode (T1Part1.cpp:230-250)
// shifts magnitudes >= 2^roishift down by roishift (and zeroes the block for
// a shift >= 31) before the scaling.
constexpr uint32_t RB_ROWS = 8;
__global__ __launch_bounds__(256) void k_t1_rebuild(const DecBlock *__restrict__ blocks, uint32_t n,
                                                    const T1Scratch *__restrict__ scr, int32_t *__restrict__ tiles,
                                                    const uint8_t *__restrict__ roi) {
    __shared__ uint64_t s_sig[32][64];  // [plane][block]
    __shared__ uint64_t s_ref[32][64];
    __shared__ uint64_t s_neg[64];
    const uint32_t g = blockIdx.x, l = threadIdx.x & 63;
    const int32_t w = (int32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t y0 = blockIdx.y * RB_ROWS;
    const uint64_t *gb = t1_group_base(const_cast<T1Scratch *>(scr), g, sizeof(T1Scratch));
    const uint32_t nb = n - g * 64 < 64 ? n - g * 64 : 64;
    // this lane's block (lane l < nb)
    DecBlock mb{};
    DecodedPlanes dp{-1, 0, 32};
    uint32_t rs = 0;
    if (l < nb) {
        mb = blocks[g * 64 + l];
        dp = decoded_planes(mb.len && mb.numbps <= T1_MAX_DEC_BPS ? mb.numpasses : 0, mb.numbps);
        rs = roi ? roi[g * 64 + l] : 0u;
    }
    // packed per-block parameters for the readlane broadcasts
    const uint32_t pk = (uint32_t)(dp.top & 0xff) | ((uint32_t)dp.low & 0xff) << 8 | ((uint32_t)dp.qlow & 0xff) << 16 |
                        (rs & 0xff) << 24;
    const uint32_t wh = mb.w | mb.h << 8 | (mb.irrev ? 1u << 16 : 0u);
    const uint64_t *pa = gb + (size_t)T1R_PA * 64 + l, *pb = gb + (size_t)T1R_PB * 64 + l;
    const uint64_t *ng = gb + (size_t)T1R_NEG * 64 + l;
    for (uint32_t y = y0; y < y0 + RB_ROWS; ++y) {
        if (y < mb.h && dp.top >= 0) {
            for (int32_t q = dp.low + ((w - dp.low) & 3); q <= dp.top; q += 4)
                s_sig[q][l] = pa[(size_t)((uint32_t)q * 64 + y) * 64];
            for (int32_t q = dp.qlow + ((w - dp.qlow) & 3); q < dp.top; q += 4)
                s_ref[q][l] = pb[(size_t)((uint32_t)q * 64 + y) * 64];
            if (w == 0) s_neg[l] = ng[(size_t)(y + 1) * 64];
        }
        __syncthreads();
        for (uint32_t b = (uint32_t)w; b < nb; b += 4) {
            const uint32_t bwh = __builtin_amdgcn_readlane(wh, b);
            const uint32_t bh = (bwh >> 8) & 0xff, bw = bwh & 0xff;
            if (y >= bh) continue;  // uniform
            const uint32_t bpk = __builtin_amdgcn_readlane(pk, b);
            const int32_t top = (int8_t)(bpk & 0xff), low = (int32_t)((bpk >> 8) & 0xff);
            const int32_t qlow = (int32_t)((bpk >> 16) & 0xff);
            const uint32_t brs = bpk >> 24;
            int32_t v = 0;
            if (top >= 0) {
                uint32_t cs = 0;  // bit (q - low): significant after plane q
                for (int32_t q = top; q >= low; --q) cs = (cs << 1) | (uint32_t)((s_sig[q][b] >> l) & 1u);
                if (cs) {
                    const int32_t p = low + 31 - (int32_t)__clz(cs);
                    const int32_t ql = p < qlow ? p : qlow;
                    uint32_t cr = 0;  // bit (q - ql): refinement bit at plane q, q in [ql, p)
                    for (int32_t q = p - 1; q >= ql; --q) cr = (cr << 1) | (uint32_t)((s_ref[q][b] >> l) & 1u);
                    const uint32_t bits = (1u << (p - ql)) | cr;
                    int32_t mag = (int32_t)((bits << (ql + 1)) | (1u << ql));
                    if (brs) mag = brs >= 31 ? 0 : (mag >= (1 << brs) ? mag >> brs : mag);
                    v = ((s_neg[b] >> l) & 1u) ? -mag : mag;
                }
            }
            const float step = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mb.step), b));
            const int32_t o = (bwh >> 16) ? __float_as_int(__fmul_rn((float)v, step)) : v / 2;
            const uint32_t off_lo = __builtin_amdgcn_readlane((uint32_t)mb.dst_off, b);
            const uint32_t off_hi = __builtin_amdgcn_readlane((uint32_t)(mb.dst_off >> 32), b);
            const uint32_t stride = __builtin_amdgcn_readlane(mb.dstride, b);
            if (l < bw) tiles[(((uint64_t)off_hi << 32) | off_lo) + (size_t)y * stride + l] = o;
        }
        __syncthreads();
    }
}

// Codestream assembly: copy each run (header bytes from the host-written blob,
// or a code-block's MQ bytes from the T1 slab) to its final offset.
__global__ void k_gather(const uint8_t *__restrict__ hdr, const uint8_t *__restrict__ slab,
                         const GatherItem *__restrict__ items, uint32_t n, uint8_t *__restrict__ dst) {
    uint32_t i = blockIdx.x;
    if (i >= n) return;
    GatherItem it = items[i];
    const uint8_t *src = (it.pad ? slab : hdr) + it.src;
    for (uint32_t k = threadIdx.x; k < it.len; k += blockDim.x) dst[it.dst + k] = src[k];
}

// ---------------------------------------------------------------------------
// launchers (host side, used by codec.cpp)
// ---------------------------------------------------------------------------
hipError_t launch_dcshift_mct_fwd(const SrcPlanes &src, int32_t fmt, uint32_t sstride, const PlanePtrs &dst,
                                  uint32_t tw, uint32_t th, uint32_t ncomp, const ShiftArr &shift, int32_t mct,
                                  int32_t irrev, hipStream_t s) {
    dim3 grid((tw + 255) / 256, th);
    // Non-temporal output stores: with plain stores the 8 B/sample this pass
    // writes sit dirty in L2 / MALL and are written back while the first DWT
    // level runs, which then reads at ~4 TB/s instead of ~6
    // (scripts/probe/read_pattern.hip "dirty 1").  Measured on the 8K frame:
    // MCT 0.137 -> 0.150 ms, 9/7 DWT 0.255 -> 0.239.
#define GRK_DCS(S) hipLaunchKernelGGL((k_dcshift_mct_fwd<true, S>), grid, dim3(256), 0, s, src, sstride, dst, tw, th, \
                                      ncomp, shift, mct, irrev)
    switch (fmt) {
        case SMP_I32: GRK_DCS(int32_t); break;
        case SMP_U8: GRK_DCS(uint8_t); break;
        case SMP_I8: GRK_DCS(int8_t); break;
        case SMP_U16: GRK_DCS(uint16_t); break;
        case SMP_I16: GRK_DCS(int16_t); break;
        default: return hipErrorInvalidValue;
    }
#undef GRK_DCS
    return hipGetLastError();
}

hipError_t launch_dcshift_mct_custom(const SrcPlanes &src, int32_t fmt, uint32_t sstride, const PlanePtrs &dst,
                                     uint32_t tw, uint32_t th, uint32_t ncomp, const ShiftArr &shift,
                                     const MctMatrix &m, hipStream_t s) {
    if (ncomp > GRK_MAX_COMPS) return hipErrorInvalidValue;
    dim3 grid((tw + 255) / 256, th);
#define GRK_DCC(S) hipLaunchKernelGGL((k_dcshift_mct_custom<S>), grid, dim3(256), 0, s, src, sstride, dst, tw, th, ncomp, \
                                      shift, m)
    switch (fmt) {
        case SMP_I32: GRK_DCC(int32_t); break;
        case SMP_U8: GRK_DCC(uint8_t); break;
        case SMP_I8: GRK_DCC(int8_t); break;
        case SMP_U16: GRK_DCC(uint16_t); break;
        case SMP_I16: GRK_DCC(int16_t); break;
        default: return hipErrorInvalidValue;
    }
#undef GRK_DCC
    return hipGetLastError();
}

hipError_t launch_mct_inv_dcshift(const PlanePtrs &src, uint32_t sstride, uint32_t tw, uint32_t th,
                                  const PlanePtrs &dst, uint32_t dstride, uint32_t ncomp, const ShiftArr &shift,
                                  const ShiftArr &mn, const ShiftArr &mx, int32_t mct, int32_t irrev, hipStream_t s) {
    dim3 grid((tw + 255) / 256, th);
    hipLaunchKernelGGL(k_mct_inv_dcshift, grid, dim3(256), 0, s, src, sstride, tw, th, dst, dstride, ncomp, shift, mn,
                       mx, mct, irrev);
    return hipGetLastError();
}

// MQ encoder: 64 blocks (lanes) per wavefront.  The coder is a serial chain
// per block, so throughput = resident blocks / block time: 64 lanes per
// wavefront keep 4x more blocks resident per wave slot than 16.
constexpr int MQ_LANES = 64;
constexpr int MQ_WAVES = 4;  // wavefronts per MQ-coder workgroup
// T1 decoder: 64 blocks (lanes) per wavefront, same reasoning (8K frame batch,
// 12 frames in flight: 2.0-2.2 vs 1.25 Gpix/s with 16; a lone frame decodes
// ~10% faster with 16).
constexpr int DEC_LANES = 64;

// Blocks per wavefront of the lane coders: 64 keeps the most blocks resident
// per wave slot, which is what the throughput of many frames in flight
// needs; a launch of few blocks (a small image) is bound by its longest
// block's chain instead, and the 64 blocks of a wavefront execute the union of
// their paths -- there one block per wavefront (n <= 1024: at most one
// wavefront per SIMD), then 2, 4, ... up to 64 from 4096 blocks on.
uint32_t lone_bpw(uint32_t n) {
    uint32_t b = 1;
    while (b < 64 && (uint64_t)n >= 1536ull * (2 * b)) b <<= 1;
    return b;
}

static uint32_t t1_blocks_per_wave(uint32_t n) {
    uint32_t b = 1;
    while (b < 64 && (uint64_t)n > 1024ull * b) b <<= 1;
    return n >= 4096 ? 64 : b;
}

uint32_t t1_order_words(uint32_t n) { return 2 * n + MQ_ORDER_BUCKETS; }

hipError_t launch_t1_encode(const EncBlock *blocks, uint32_t n, const int32_t *coef, void *scratch_v,
                            uint8_t *sym, const uint64_t *sym_off, uint32_t maxdepth, uint8_t *out, EncResult *res,
                            hipStream_t s, uint32_t cblksty, uint32_t bpw_req, uint32_t *order) {
    if (!n) return hipSuccess;
    uint8_t *scratch = (uint8_t *)scratch_v;
    if (maxdepth > 32) maxdepth = 32;
    if (maxdepth < 1) maxdepth = 1;
    const uint32_t groups8 = (t1_scratch_records(n) / 64 + 7) & ~7u;  // k_t1_prep's XCD deal: whole rounds of 8 groups
    hipLaunchKernelGGL(k_t1_prep, dim3(groups8 * 64), dim3(64), 0, s, blocks, n, maxdepth, coef, scratch, res);
    const uint64_t threads = (uint64_t)t1_scratch_records(n) * maxdepth;
    hipLaunchKernelGGL(k_t1_model<true>, dim3((uint32_t)(threads / 64)), dim3(64), 0, s, blocks, n, maxdepth, scratch,
                       sym, sym_off, res, cblksty);
    const uint32_t bpw = dwt_options().t1_enc_bpw ? (uint32_t)dwt_options().t1_enc_bpw
                         : bpw_req                ? bpw_req
                                                  : t1_blocks_per_wave(n);
    const uint32_t *perm = nullptr;
    const uint32_t *cnt = enc_scratch(scratch, n, maxdepth).cnt;
    if (order && dwt_options().t1_enc_sort && n > 64) {  // order: t1_order_words(n) words
        uint32_t *key = order, *permw = order + n, *hist = order + 2 * n;
        const hipError_t e = hipMemsetAsync(hist, 0, MQ_ORDER_BUCKETS * 4, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_mq_order_hist, dim3((n + 255) / 256), dim3(256), 0, s, cnt, res, n, key, hist);
        hipLaunchKernelGGL(k_mq_order_scan, dim3(1), dim3(MQ_ORDER_BUCKETS), 0, s, hist);
        hipLaunchKernelGGL(k_mq_order_scatter, dim3((n + 255) / 256), dim3(256), 0, s, key, n, hist, permw);
        perm = permw;
    }
    // Concurrent calls: MQ_WAVES wavefronts per workgroup, 19 context words
    // per lane -- LDS no longer holds the coder at 7 wavefronts per SIMD (5.7
    // KB per single-wavefront workgroup); 8 per SIMD by registers and LDS: 8K
    // batch 3519 / 3476 -> 3664 / 3577 Mpixels/s alternating (profiles/r05/
    // t1_mq_wg_ab.txt).  A call alone on the GPU or a small launch keeps one
    // wavefront per workgroup: its lanes' chains run on separate CUs instead of
    // four wavefronts sharing one CU's LDS -- the 512^2 image's coder took
    // 6.8 ms in 4-wavefront workgroups against 4.1 (profiles/r05/
    // rocprof_512_r4_r5.txt)
    const uint32_t nwv = (n + bpw - 1) / bpw, nwg = (nwv + MQ_WAVES - 1) / MQ_WAVES;
    const bool wide = !bpw_req && n > 4096;
    if (wide && (cblksty & CBLKSTY_LAZY))
        hipLaunchKernelGGL((k_t1_mq<MQ_LANES, 1, true, MQ_WAVES, 19>), dim3(nwg), dim3(MQ_LANES * MQ_WAVES), 0, s,
                           blocks, n, cnt, sym, sym_off, out, res, perm, cblksty, bpw);
    else if (wide)
        hipLaunchKernelGGL((k_t1_mq<MQ_LANES, 1, false, MQ_WAVES, 19>), dim3(nwg), dim3(MQ_LANES * MQ_WAVES), 0, s,
                           blocks, n, cnt, sym, sym_off, out, res, perm, cblksty, bpw);
    else if (cblksty & CBLKSTY_LAZY)
        hipLaunchKernelGGL((k_t1_mq<MQ_LANES, 1, true>), dim3(nwv), dim3(MQ_LANES), 0, s, blocks, n, cnt, sym, sym_off,
                           out, res, perm, cblksty, bpw);
    else
        hipLaunchKernelGGL((k_t1_mq<MQ_LANES, 1, false>), dim3(nwv), dim3(MQ_LANES), 0, s, blocks, n, cnt, sym, sym_off,
                           out, res, perm, cblksty, bpw);
    return hipGetLastError();
}

// t1_generate_luts.cpp:290-318: floor((u^2 - v^2) * 2^6 + 0.5) / 2^6 * 8192
// with t = i / 2^6, clamped at 0 (host double arithmetic, as generated)
static NmseLut make_nmse_lut() {
    NmseLut L;
    for (int i = 0; i < 128; ++i) {
        const double t = i / 64.0;
        double u = t, v = t - 1.5;
        L.sig[i] = (int16_t)std::max(0, (int)(floor((u * u - v * v) * 64.0 + 0.5) / 64.0 * 8192.0));
        L.sig0[i] = (int16_t)std::max(0, (int)(floor((u * u) * 64.0 + 0.5) / 64.0 * 8192.0));
        u = t - 1.0;
        v = (i & 64) ? t - 1.5 : t - 0.5;
        L.ref[i] = (int16_t)std::max(0, (int)(floor((u * u - v * v) * 64.0 + 0.5) / 64.0 * 8192.0));
        L.ref0[i] = (int16_t)std::max(0, (int)(floor((u * u) * 64.0 + 0.5) / 64.0 * 8192.0));
    }
    return L;
}
const NmseLut &nmse_lut() {
    static const NmseLut L = make_nmse_lut();
    return L;
}

hipError_t launch_t1_dist(const EncBlock *blocks, uint32_t n, uint32_t maxdepth, const int32_t *coef,
                          const void *scratch, EncResult *res, hipStream_t s) {
    if (!n) return hipSuccess;
    if (maxdepth > 32) maxdepth = 32;
    if (maxdepth < 1) maxdepth = 1;
    hipLaunchKernelGGL(k_t1_dist, dim3(n), dim3(64), 0, s, blocks, n, maxdepth, coef, (const uint8_t *)scratch, res,
                       nmse_lut());
    return hipGetLastError();
}

// One thread per block (grk_device.h DevPass / PassSum).  The arithmetic is
// the host's, operation for operation in IEEE double (no contraction: the
// library builds with -ffp-contract=off), so the records are bit-identical.
__global__ __launch_bounds__(256) void k_pass_records(const EncBlock *__restrict__ blocks,
                                                      const EncResult *__restrict__ res, const double *__restrict__ wfac,
                                                      const uint64_t *__restrict__ pass0, uint32_t n, uint32_t sty,
                                                      DevPass *__restrict__ out, PassSum *__restrict__ sum) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const EncResult &r = res[i];
    const EncBlock &b = blocks[i];
    PassSum ps{};
    ps.numbps = r.numbps;
    ps.numpasses = r.numpasses;
    ps.len = r.len;
    ps.nsym = r.nsym;
    const uint64_t p0 = pass0[i], cap = pass0[i + 1] - p0;
    uint32_t np = r.numpasses;
    if (r.pad) ps.bad |= 1u;
    if (np > cap || np > GRK_MAX_PASSES) { ps.bad |= 2u; np = 0; }
    if (np && r.rate[np - 1] > b.w * b.h * 4 + 64) ps.bad |= 4u;
    if (ps.bad) np = 0;
    const double f = wfac[i];
    double cum = 0.0, mn = DBL_MAX, mx = -1, m0 = -HUGE_VAL;
    uint32_t prev = 0, z0 = 0;
    double prevdd = 0.0;
    DevPass *o = out + p0;
    for (uint32_t k = 0; k < np; ++k) {
        DevPass d;
        d.rate = r.rate[k];
        d.len = d.rate - prev;
        const int32_t bp = k == 0 ? (int32_t)r.numbps - 1 : (int32_t)r.numbps - 2 - (int32_t)((k - 1) / 3);
        const int pt = k == 0 ? 2 : (int)((k - 1) % 3);
        d.term = t1_pass_term(sty, bp, pt, r.numbps) ? 1 : 0;
        d.slope = 0;
        // t1_wmsedec_at (t2.h): factor * 2^bpno, squared with nmsedec / 8192
        double w = f * (1 << bp);
        w *= w * r.nmsedec[k] / 8192.0;
        cum += w;
        d.dd = cum;
        o[k] = d;
        // block_slopes (t2.cpp)
        if (d.rate) { const double q = d.dd / d.rate; m0 = m0 < q ? q : m0; }
        else if (d.dd != 0) z0 = 1;
        const int32_t dr = k == 0 ? (int32_t)d.rate : (int32_t)(d.rate - prev);
        const double ddd = k == 0 ? d.dd : d.dd - prevdd;
        if (dr != 0) {
            const double q = ddd / dr;
            if (q < mn) mn = q;
            if (q > mx) mx = q;
        }
        prev = d.rate;
        prevdd = d.dd;
    }
    ps.z0 = z0;
    ps.smin = mn;
    ps.smax = mx;
    ps.s0max = m0;
    ps.disto = cum;
    sum[i] = ps;
}

hipError_t launch_pass_records(const EncBlock *blocks, const EncResult *res, const double *wfac, const uint64_t *pass0,
                               uint32_t n, uint32_t cblksty, DevPass *out, PassSum *sum, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_pass_records, dim3((n + 255) / 256), dim3(256), 0, s, blocks, res, wfac, pass0, n, cblksty,
                       out, sum);
    return hipGetLastError();
}

hipError_t launch_t1_decode(const DecBlock *blocks, uint32_t n, const uint8_t *data, T1Scratch *scratch,
                            int32_t *tiles, hipStream_t s, uint32_t *ubuf, uint32_t fixed_words, const DecSeg *segs,
                            const uint32_t *seg_first, uint32_t cblksty, const uint8_t *roi, uint32_t bpw_req) {
    if (!n) return hipSuccess;
    // a call alone on the GPU (bpw_req: the lone packing) or a small one
    // unstuffs a segment per wavefront: 1.37 ms -> 0.27 ms per 8K frame, lone
    // decode T1 29.0 / 29.8 -> 28.1 / 27.5 ms; under 16 frames in flight the
    // lane-per-block pass does the same work in fewer instructions, and the
    // batch is issue-bound: 3529 / 3473 vs 3473 / 3415 Mpixels/s with the
    // wavefront pass (profiles/r05/t1_unstuff_wave_ab.txt)
    if (bpw_req || n <= 4096)
        hipLaunchKernelGGL(k_t1_unstuff_w, dim3((n + 3) / 4), dim3(256), 0, s, blocks, n, data, ubuf, fixed_words, segs,
                           seg_first);
    else
        hipLaunchKernelGGL(k_t1_unstuff, dim3((n + 63) / 64), dim3(64), 0, s, blocks, n, data, ubuf, fixed_words, segs,
                           seg_first);
    const uint32_t bpw = dwt_options().t1_dec_bpw ? (uint32_t)dwt_options().t1_dec_bpw
                         : bpw_req                ? bpw_req
                                                  : t1_blocks_per_wave(n);
    // DEC_WAVES wavefronts per workgroup share the LUTs (roi only for BYPASS:
    // the ROI shift only moves BYPASS pass boundaries)
    const uint32_t nw = (n + bpw - 1) / bpw, nwg = (nw + DEC_WAVES - 1) / DEC_WAVES;
    // A launch of few blocks does not fill the GPU, so occupancy buys nothing
    // and the 128-VGPR cap's spills sit on each lane's chain: single-wavefront
    // workgroups at the uncapped 144 VGPRs -- the 512^2 image (70 blocks)
    // decodes in 9.1-9.4 ms of T1 against 16.8-18.4 (profiles/r05/
    // t1_lone_variants.txt); the 4K frame (6,321 blocks, more than 4,096)
    // and the lone 8K frame were the same either way
    if (n <= 4096) {
        if (cblksty & CBLKSTY_LAZY)
            hipLaunchKernelGGL((k_t1_decode_ub<DEC_LANES, true, 1, 1>), dim3(nw), dim3(DEC_LANES), 0, s, blocks, n,
                               (const uint32_t *)ubuf, fixed_words, scratch, segs, seg_first, cblksty, roi, bpw);
        else
            hipLaunchKernelGGL((k_t1_decode_ub<DEC_LANES, false, 1, 1>), dim3(nw), dim3(DEC_LANES), 0, s, blocks, n,
                               (const uint32_t *)ubuf, fixed_words, scratch, segs, seg_first, cblksty, nullptr, bpw);
    } else if (cblksty & CBLKSTY_LAZY)
        hipLaunchKernelGGL((k_t1_decode_ub<DEC_LANES, true, DEC_WAVES, DEC_WAVES>), dim3(nwg), dim3(DEC_LANES * DEC_WAVES),
                           0, s, blocks, n, (const uint32_t *)ubuf, fixed_words, scratch, segs, seg_first, cblksty, roi,
                           bpw);
    else
        hipLaunchKernelGGL((k_t1_decode_ub<DEC_LANES, false, DEC_WAVES, DEC_WAVES>), dim3(nwg),
                           dim3(DEC_LANES * DEC_WAVES), 0, s, blocks, n, (const uint32_t *)ubuf, fixed_words, scratch,
                           segs, seg_first, cblksty, nullptr, bpw);
    hipLaunchKernelGGL(k_t1_rebuild, dim3((n + 63) / 64, 64 / RB_ROWS), dim3(256), 0, s, blocks, n, scratch, tiles,
                       roi);
    return hipGetLastError();
}

hipError_t launch_gather(const uint8_t *hdr, const uint8_t *slab, const GatherItem *items, uint32_t n, uint8_t *dst,
                         hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_gather, dim3(n), dim3(256), 0, s, hdr, slab, items, n, dst);
    return hipGetLastError();
}

}  // namespace grkgpu
