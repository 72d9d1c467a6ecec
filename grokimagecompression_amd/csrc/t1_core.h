// t1_core.h -- EBCOT Tier-1 constants and context rules shared by the HIP
// kernels (t1_lane.h, t1_dec.h, t1_flat.h) and their host unit test
// (tests/cpp/test_t1_core.cpp; compiled for both sides: __host__ __device__).
//
// Semantics follow Grok v5.1.0 (src/lib/jp2/t1/t1_part1/t1.cpp, mqc_enc.cpp,
// mqc_dec_inl.h): ISO 15444-1 Annex C MQ coder + Annex D context modelling
// with Grok's pass-rate bookkeeping.  The state layout is MI355X-first: the
// significance / sign / visited / refined state of a code-block is kept as
// 64-bit ROW MASKS (bit x = column x), so a wavefront (or a lane) forms the
// 3x3 neighbourhood of a sample with shifts instead of per-sample flag words.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GRK_HD __host__ __device__ __forceinline__
#else
#define GRK_HD inline
struct uint4 { uint32_t x, y, z, w; };  // host build of the shared coder
#endif

namespace grkgpu {

// ---------------------------------------------------------------------------
// MQ probability-state machine (ISO 15444-1 Table C.2; Grok mqc_enc.cpp:69-166)
// packed per state: Qe[15:0] | NMPS[21:16] | NLPS[27:22] | SWITCH[28]
// ---------------------------------------------------------------------------
#define GRK_MQ_PACK(qe, nmps, nlps, sw) ((uint32_t)(qe) | ((uint32_t)(nmps) << 16) | ((uint32_t)(nlps) << 22) | ((uint32_t)(sw) << 28))
#define GRK_MQ_TABLE_INIT                                                                                        \
    {GRK_MQ_PACK(0x5601, 1, 1, 1),   GRK_MQ_PACK(0x3401, 2, 6, 0),   GRK_MQ_PACK(0x1801, 3, 9, 0),           \
     GRK_MQ_PACK(0x0AC1, 4, 12, 0),  GRK_MQ_PACK(0x0521, 5, 29, 0),  GRK_MQ_PACK(0x0221, 38, 33, 0),         \
     GRK_MQ_PACK(0x5601, 7, 6, 1),   GRK_MQ_PACK(0x5401, 8, 14, 0),  GRK_MQ_PACK(0x4801, 9, 14, 0),          \
     GRK_MQ_PACK(0x3801, 10, 14, 0), GRK_MQ_PACK(0x3001, 11, 17, 0), GRK_MQ_PACK(0x2401, 12, 18, 0),         \
     GRK_MQ_PACK(0x1C01, 13, 20, 0), GRK_MQ_PACK(0x1601, 29, 21, 0), GRK_MQ_PACK(0x5601, 15, 14, 1),         \
     GRK_MQ_PACK(0x5401, 16, 14, 0), GRK_MQ_PACK(0x5101, 17, 15, 0), GRK_MQ_PACK(0x4801, 18, 16, 0),         \
     GRK_MQ_PACK(0x3801, 19, 17, 0), GRK_MQ_PACK(0x3401, 20, 18, 0), GRK_MQ_PACK(0x3001, 21, 19, 0),         \
     GRK_MQ_PACK(0x2801, 22, 19, 0), GRK_MQ_PACK(0x2401, 23, 20, 0), GRK_MQ_PACK(0x2201, 24, 21, 0),         \
     GRK_MQ_PACK(0x1C01, 25, 22, 0), GRK_MQ_PACK(0x1801, 26, 23, 0), GRK_MQ_PACK(0x1601, 27, 24, 0),         \
     GRK_MQ_PACK(0x1401, 28, 25, 0), GRK_MQ_PACK(0x1201, 29, 26, 0), GRK_MQ_PACK(0x1101, 30, 27, 0),         \
     GRK_MQ_PACK(0x0AC1, 31, 28, 0), GRK_MQ_PACK(0x09C1, 32, 29, 0), GRK_MQ_PACK(0x08A1, 33, 30, 0),         \
     GRK_MQ_PACK(0x0521, 34, 31, 0), GRK_MQ_PACK(0x0441, 35, 32, 0), GRK_MQ_PACK(0x02A1, 36, 33, 0),         \
     GRK_MQ_PACK(0x0221, 37, 34, 0), GRK_MQ_PACK(0x0141, 38, 35, 0), GRK_MQ_PACK(0x0111, 39, 36, 0),         \
     GRK_MQ_PACK(0x0085, 40, 37, 0), GRK_MQ_PACK(0x0049, 41, 38, 0), GRK_MQ_PACK(0x0025, 42, 39, 0),         \
     GRK_MQ_PACK(0x0015, 43, 40, 0), GRK_MQ_PACK(0x0009, 44, 41, 0), GRK_MQ_PACK(0x0005, 45, 42, 0),         \
     GRK_MQ_PACK(0x0001, 45, 43, 0), GRK_MQ_PACK(0x5601, 46, 46, 0)}

// context numbers (t1.h:65-76)
enum { CX_ZC = 0, CX_SC = 9, CX_MAG = 14, CX_AGG = 17, CX_UNI = 18, NUM_CX = 19 };

// Zero-coding context (t1_generate_luts.cpp:63-140); orient 1 (HL) swaps h/v.
GRK_HD int zc_ctx(int h, int v, int d, uint32_t orient) {
    if (orient == 3) {
        int hv = h + v;
        if (d == 0) return hv == 0 ? 0 : (hv == 1 ? 1 : 2);
        if (d == 1) return hv == 0 ? 3 : (hv == 1 ? 4 : 5);
        if (d == 2) return hv == 0 ? 6 : 7;
        return 8;
    }
    if (orient == 1) { int t = h; h = v; v = t; }
    if (h == 0) {
        if (v == 0) return d == 0 ? 0 : (d == 1 ? 1 : 2);
        return v == 1 ? 3 : 4;
    }
    if (h == 1) return v == 0 ? (d == 0 ? 5 : 6) : 7;
    return 8;
}

// Sign-coding context + XOR bit (t1_generate_luts.cpp:142-215, Table D.3).
// sig/neg: 4-neighbour significance and sign: W, E, N, S.
GRK_HD int sc_ctx(uint32_t sw, uint32_t se, uint32_t sn, uint32_t ss, uint32_t nw_, uint32_t ne_, uint32_t nn_,
                  uint32_t ns_, uint32_t *xorbit) {
    int hc = (sw ? (nw_ ? -1 : 1) : 0) + (se ? (ne_ ? -1 : 1) : 0);
    int vc = (sn ? (nn_ ? -1 : 1) : 0) + (ss ? (ns_ ? -1 : 1) : 0);
    hc = hc > 1 ? 1 : (hc < -1 ? -1 : hc);
    vc = vc > 1 ? 1 : (vc < -1 ? -1 : vc);
    uint32_t x = (hc < 0 || (hc == 0 && vc < 0)) ? 1u : 0u;
    if (hc < 0) { hc = -hc; vc = -vc; }
    *xorbit = x;
    if (hc == 0) return CX_SC + (vc == 0 ? 0 : 1);
    return CX_SC + (vc == -1 ? 2 : (vc == 0 ? 3 : 4));
}

// int_fix_mul_t1 (T1Part1.cpp:45-56)
GRK_HD int32_t fix_mul_t1(int32_t a, int32_t b) {
    int64_t t = (int64_t)a * (int64_t)b + ((int64_t)1 << 17);
    return (int32_t)(t >> 18);
}

// preEncode quantisation of one coefficient (T1Part1.cpp:58-94): magnitude
// with the T1_NMSEDEC_FRACBITS = 6 fraction bits, sign in *neg.
GRK_HD uint32_t quant_mag(int32_t v, int32_t qmfbid, int32_t inv_step, uint32_t *neg) {
    int32_t q = (qmfbid == 1) ? (int32_t)((uint32_t)v << 6) : fix_mul_t1(v, inv_step);
    *neg = q < 0 ? 1u : 0u;
    return (uint32_t)(q < 0 ? -q : q);
}

}  // namespace grkgpu
