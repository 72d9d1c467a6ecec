// t1_core.h -- EBCOT Tier-1 block coder shared by the HIP kernels and the host
// unit tests (compiled for both sides: __host__ __device__).
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

// A context register: state index in bits [5:0], MPS in bit 6.
// mqc_resetstates (mqc_dec.cpp:207-215): UNI -> 46, AGG -> 3, ZC0 -> 4.
GRK_HD void mq_reset_ctx(uint8_t *cx) {
    for (int i = 0; i < NUM_CX; ++i) cx[i] = 0;
    cx[CX_UNI] = 46;
    cx[CX_AGG] = 3;
    cx[CX_ZC] = 4;
}

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

// Neighbourhood of sample (x, y) from row masks.  nb9: bits 0..2 = row y-1
// (x-1,x,x+1), 3..5 = row y, 6..8 = row y+1.
GRK_HD uint32_t bits3(uint64_t row, uint32_t x) {
    uint32_t left = x ? (uint32_t)(row >> (x - 1)) & 1u : 0u;
    return left | ((uint32_t)(row >> x) & 3u) << 1;
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

struct PassInfo {
    uint32_t rate;
    uint32_t len;
    uint32_t term;
};

// ---------------------------------------------------------------------------
// MQ encoder (mqc_enc.cpp).  out[-1] must exist and be 0 (bp = start - 1).
// ---------------------------------------------------------------------------
struct MqEnc {
    uint32_t a, c, ct;
    int32_t bp;
    uint8_t *buf;
};

GRK_HD void mqe_byteout(MqEnc &e) {
    uint8_t *b = e.buf;
    if (b[e.bp] == 0xff) {
        e.bp++; b[e.bp] = (uint8_t)(e.c >> 20); e.c &= 0xfffff; e.ct = 7;
    } else if ((e.c & 0x8000000) == 0) {
        e.bp++; b[e.bp] = (uint8_t)(e.c >> 19); e.c &= 0x7ffff; e.ct = 8;
    } else {
        b[e.bp]++;
        if (b[e.bp] == 0xff) {
            e.c &= 0x7ffffff;
            e.bp++; b[e.bp] = (uint8_t)(e.c >> 20); e.c &= 0xfffff; e.ct = 7;
        } else {
            e.bp++; b[e.bp] = (uint8_t)(e.c >> 19); e.c &= 0x7ffff; e.ct = 8;
        }
    }
}

GRK_HD void mqe_encode(MqEnc &e, uint8_t *cxs, const uint32_t *tab, int cx, uint32_t d) {
    uint32_t s = cxs[cx];
    uint32_t t = tab[s & 63];
    uint32_t qe = t & 0xffff;
    uint32_t mps = s >> 6;
    e.a -= qe;
    if (d == mps) {
        if ((e.a & 0x8000) == 0) {
            if (e.a < qe) e.a = qe; else e.c += qe;
            cxs[cx] = (uint8_t)(((t >> 16) & 63) | (mps << 6));
        } else {
            e.c += qe;
            return;
        }
    } else {
        if (e.a < qe) e.c += qe; else e.a = qe;
        uint32_t nm = mps ^ ((t >> 28) & 1);
        cxs[cx] = (uint8_t)(((t >> 22) & 63) | (nm << 6));
    }
    do {
        e.a <<= 1; e.c <<= 1; e.ct--;
        if (e.ct == 0) mqe_byteout(e);
    } while ((e.a & 0x8000) == 0);
}

GRK_HD void mqe_flush(MqEnc &e) {
    uint32_t tempc = e.c + e.a;
    e.c |= 0xffff;
    if (e.c >= tempc) e.c -= 0x8000;
    e.c <<= e.ct; mqe_byteout(e);
    e.c <<= e.ct; mqe_byteout(e);
    if (e.buf[e.bp] != 0xff) e.bp++;
}

// ---------------------------------------------------------------------------
// MQ decoder (mqc_dec.cpp:178-193, mqc_dec_inl.h).  Bytes at index >= len
// read as 0xFF (Grok's artificial 0xFF 0xFF end marker).
// ---------------------------------------------------------------------------
struct MqDec {
    uint32_t a, c, ct;
    uint32_t bp, len;
    const uint8_t *buf;
};

GRK_HD uint32_t mqd_byte(const MqDec &d, uint32_t i) { return i < d.len ? d.buf[i] : 0xffu; }

GRK_HD void mqd_bytein(MqDec &d) {
    uint32_t next = mqd_byte(d, d.bp + 1);
    if (mqd_byte(d, d.bp) == 0xff) {
        if (next > 0x8f) { d.c += 0xff00; d.ct = 8; }
        else { d.bp++; d.c += next << 9; d.ct = 7; }
    } else {
        d.bp++; d.c += next << 8; d.ct = 8;
    }
}

GRK_HD void mqd_init(MqDec &d, const uint8_t *buf, uint32_t len) {
    d.buf = buf; d.len = len; d.bp = 0;
    d.c = (uint32_t)((len == 0) ? 0xffu : buf[0]) << 16;
    mqd_bytein(d);
    d.c <<= 7; d.ct -= 7; d.a = 0x8000;
}

GRK_HD uint32_t mqd_decode(MqDec &d, uint8_t *cxs, const uint32_t *tab, int cx) {
    uint32_t s = cxs[cx];
    uint32_t t = tab[s & 63];
    uint32_t qe = t & 0xffff;
    uint32_t mps = s >> 6;
    uint32_t r;
    d.a -= qe;
    if (d.c < (qe << 16)) {
        if (d.a < qe) { d.a = qe; r = mps; cxs[cx] = (uint8_t)(((t >> 16) & 63) | (mps << 6)); }
        else { d.a = qe; r = mps ^ 1; cxs[cx] = (uint8_t)(((t >> 22) & 63) | ((mps ^ ((t >> 28) & 1)) << 6)); }
    } else {
        d.c -= qe << 16;
        if (d.a >= 0x8000) return mps;
        if (d.a < qe) { r = mps ^ 1; cxs[cx] = (uint8_t)(((t >> 22) & 63) | ((mps ^ ((t >> 28) & 1)) << 6)); }
        else { r = mps; cxs[cx] = (uint8_t)(((t >> 16) & 63) | (mps << 6)); }
    }
    do {
        if (d.ct == 0) mqd_bytein(d);
        d.a <<= 1; d.c <<= 1; d.ct--;
    } while (d.a < 0x8000);
    return r;
}

// ---------------------------------------------------------------------------
// Block state: row masks (bit x = column x), rows -1..h (index y+1).
// ---------------------------------------------------------------------------
struct BlockRows {
    uint64_t sig[66];
    uint64_t neg[66];
    uint64_t visit[66];
    uint64_t ref[66];
};

GRK_HD uint32_t getbit(uint64_t row, uint32_t x) { return (uint32_t)(row >> x) & 1u; }

GRK_HD int zc_of(const BlockRows &s, uint32_t x, uint32_t y, uint32_t orient) {
    uint32_t up = bits3(s.sig[y], x), mid = bits3(s.sig[y + 1], x), dn = bits3(s.sig[y + 2], x);
    int h = (int)((mid & 1) + ((mid >> 2) & 1));
    int v = (int)(((up >> 1) & 1) + ((dn >> 1) & 1));
    int d = (int)((up & 1) + ((up >> 2) & 1) + (dn & 1) + ((dn >> 2) & 1));
    return zc_ctx(h, v, d, orient);
}

GRK_HD bool any_nb(const BlockRows &s, uint32_t x, uint32_t y) {
    return ((bits3(s.sig[y], x) | (bits3(s.sig[y + 1], x) & 5u) | bits3(s.sig[y + 2], x)) != 0);
}

GRK_HD int sc_of(const BlockRows &s, uint32_t x, uint32_t y, uint32_t *xorbit) {
    uint32_t sm = bits3(s.sig[y + 1], x), nm = bits3(s.neg[y + 1], x);
    uint32_t su = bits3(s.sig[y], x), nu = bits3(s.neg[y], x);
    uint32_t sd = bits3(s.sig[y + 2], x), nd = bits3(s.neg[y + 2], x);
    return sc_ctx(sm & 1, (sm >> 2) & 1, (su >> 1) & 1, (sd >> 1) & 1, nm & 1, (nm >> 2) & 1, (nu >> 1) & 1,
                  (nd >> 1) & 1, xorbit);
}

GRK_HD int mag_of(const BlockRows &s, uint32_t x, uint32_t y) {
    if (getbit(s.ref[y + 1], x)) return CX_MAG + 2;
    return CX_MAG + (any_nb(s, x, y) ? 1 : 0);
}

GRK_HD void setbit(uint64_t &row, uint32_t x) { row |= (uint64_t)1 << x; }
GRK_HD void clrbit(uint64_t &row, uint32_t x) { row &= ~((uint64_t)1 << x); }

// ---------------------------------------------------------------------------
// Encode one code-block (w <= 64, h <= 64), cblksty 0.
// Coefficients are DWT-domain values from the tile buffer; the preEncode
// quantisation (T1Part1.cpp:58-94) is folded in.  Returns the pass count.
// ---------------------------------------------------------------------------
GRK_HD uint32_t quant_mag(int32_t v, int32_t qmfbid, int32_t inv_step, uint32_t *neg) {
    int32_t q = (qmfbid == 1) ? (int32_t)((uint32_t)v << 6) : fix_mul_t1(v, inv_step);
    *neg = q < 0 ? 1u : 0u;
    return (uint32_t)(q < 0 ? -q : q);
}

GRK_HD uint32_t t1_encode_block(const int32_t *coef, uint32_t stride, uint32_t w, uint32_t h, uint32_t orient,
                                int32_t qmfbid, int32_t inv_step, BlockRows &s, const uint32_t *tab,
                                uint8_t *out, PassInfo *passes, uint32_t *numbps_out, uint32_t *len_out) {
    uint32_t maxv = 0;
    for (uint32_t y = 0; y < h + 2; ++y) { s.sig[y] = 0; s.neg[y] = 0; s.visit[y] = 0; s.ref[y] = 0; }
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            uint32_t ng;
            uint32_t m = quant_mag(coef[(size_t)y * stride + x], qmfbid, inv_step, &ng);
            if (ng) setbit(s.neg[y + 1], x);
            maxv = m > maxv ? m : maxv;
        }
    uint32_t numbps = 0;
    if (maxv) {
        uint32_t t = 31u - (uint32_t)__builtin_clz(maxv) + 1u;
        numbps = t <= 6 ? 0 : t - 6;
    }
    *numbps_out = numbps;
    *len_out = 0;
    if (numbps == 0) return 0;

    uint8_t cxs[NUM_CX];
    mq_reset_ctx(cxs);
    MqEnc e;
    e.a = 0x8000; e.c = 0; e.ct = 12; e.bp = -1; e.buf = out;
    uint32_t passno = 0;
    int32_t bpno = (int32_t)numbps - 1;
    int passtype = 2;
#define MAGBIT(x, y) ((quant_mag(coef[(size_t)(y) * stride + (x)], qmfbid, inv_step, &ng_) >> (bpno + 6)) & 1u)
    for (; bpno >= 0; ++passno) {
        uint32_t ng_;
        if (passtype == 0) {  // significance propagation (t1.cpp:197-231, 287-338)
            for (uint32_t k = 0; k < h; k += 4)
                for (uint32_t x = 0; x < w; ++x)
                    for (uint32_t y = k; y < k + 4 && y < h; ++y) {
                        if (getbit(s.sig[y + 1] | s.visit[y + 1], x) || !any_nb(s, x, y)) continue;
                        uint32_t bit = MAGBIT(x, y);
                        mqe_encode(e, cxs, tab, CX_ZC + zc_of(s, x, y, orient), bit);
                        if (bit) {
                            uint32_t xr;
                            int cx = sc_of(s, x, y, &xr);
                            mqe_encode(e, cxs, tab, cx, getbit(s.neg[y + 1], x) ^ xr);
                            setbit(s.sig[y + 1], x);
                        }
                        setbit(s.visit[y + 1], x);
                    }
        } else if (passtype == 1) {  // magnitude refinement (t1.cpp:443-463, 498-555)
            for (uint32_t k = 0; k < h; k += 4)
                for (uint32_t x = 0; x < w; ++x)
                    for (uint32_t y = k; y < k + 4 && y < h; ++y) {
                        if (!getbit(s.sig[y + 1], x) || getbit(s.visit[y + 1], x)) continue;
                        mqe_encode(e, cxs, tab, mag_of(s, x, y), MAGBIT(x, y));
                        setbit(s.ref[y + 1], x);
                    }
        } else {  // cleanup + run-length (t1.cpp:639-699, 739-782)
            for (uint32_t k = 0; k < h; k += 4) {
                for (uint32_t x = 0; x < w; ++x) {
                    uint32_t y0 = k;
                    bool partial = false;
                    if (k + 4 <= h) {
                        uint64_t win = 0;
                        for (uint32_t yy = k; yy < k + 6; ++yy) win |= s.sig[yy];  // rows k-1..k+4
                        uint64_t vis = s.visit[k + 1] | s.visit[k + 2] | s.visit[k + 3] | s.visit[k + 4];
                        bool agg = bits3(win, x) == 0 && getbit(vis, x) == 0;
                        if (agg) {
                            uint32_t runlen = 0;
                            for (; runlen < 4; ++runlen)
                                if (MAGBIT(x, k + runlen)) break;
                            mqe_encode(e, cxs, tab, CX_AGG, runlen != 4);
                            if (runlen == 4) continue;
                            mqe_encode(e, cxs, tab, CX_UNI, runlen >> 1);
                            mqe_encode(e, cxs, tab, CX_UNI, runlen & 1);
                            y0 = k + runlen;
                            partial = true;
                        }
                    }
                    for (uint32_t y = y0; y < k + 4 && y < h; ++y) {
                        bool sign = false;
                        if (partial && y == y0) sign = true;
                        else if (!getbit(s.sig[y + 1] | s.visit[y + 1], x)) {
                            uint32_t bit = MAGBIT(x, y);
                            mqe_encode(e, cxs, tab, CX_ZC + zc_of(s, x, y, orient), bit);
                            sign = bit != 0;
                        }
                        if (sign) {
                            uint32_t xr;
                            int cx = sc_of(s, x, y, &xr);
                            mqe_encode(e, cxs, tab, cx, getbit(s.neg[y + 1], x) ^ xr);
                            setbit(s.sig[y + 1], x);
                        }
                        clrbit(s.visit[y + 1], x);
                    }
                }
            }
        }
        PassInfo &ps = passes[passno];
        if (passtype == 2 && bpno == 0) {  // last cleanup pass is terminated
            mqe_flush(e);
            ps.term = 1;
            ps.rate = (uint32_t)e.bp;
        } else {  // rate_extra_bytes (t1.cpp:1278-1288)
            ps.term = 0;
            ps.rate = (uint32_t)e.bp + 5 + (e.ct < 5 ? 1 : 0);
        }
        if (++passtype == 3) { passtype = 0; bpno--; }
    }
#undef MAGBIT
    uint32_t total = passno;
    uint32_t last = (uint32_t)e.bp;
    for (uint32_t i = total; i > 0;) {  // non-increasing rates (t1.cpp:1303-1313)
        PassInfo &ps = passes[--i];
        if (ps.rate > last) ps.rate = last; else last = ps.rate;
    }
    for (uint32_t i = 0; i < total; ++i) {  // no pass ends on 0xFF (t1.cpp:1315-1324)
        PassInfo &ps = passes[i];
        if (ps.rate > 0 && out[ps.rate - 1] == 0xFF) ps.rate--;
        ps.len = ps.rate - (i == 0 ? 0 : passes[i - 1].rate);
    }
    *len_out = (uint32_t)e.bp;
    return total;
}

// ---------------------------------------------------------------------------
// Decode one single-segment code-block (t1.cpp:1038-1130) and apply the
// post-decode scaling (T1Part1.cpp:216-330): 5/3 -> v/2, 9/7 -> float(v)*step.
// dst has row stride dstride (tile buffer); values are written as int32 bits.
// ---------------------------------------------------------------------------
template <typename Store>
GRK_HD void t1_decode_block_impl(const uint8_t *data, uint32_t len, uint32_t numpasses, uint32_t numbps,
                                 uint32_t w, uint32_t h, uint32_t orient, BlockRows &s, const uint32_t *tab,
                                 int32_t *dst, uint32_t dstride, Store store) {
    for (uint32_t y = 0; y < h + 2; ++y) { s.sig[y] = 0; s.neg[y] = 0; s.visit[y] = 0; s.ref[y] = 0; }
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) dst[(size_t)y * dstride + x] = 0;
    uint8_t cxs[NUM_CX];
    mq_reset_ctx(cxs);
    MqDec d;
    mqd_init(d, data, len);
    int32_t bpno_plus_one = (int32_t)numbps;
    int passtype = 2;
    for (uint32_t passno = 0; passno < numpasses && bpno_plus_one >= 1; ++passno) {
        const int32_t one = 1 << bpno_plus_one;
        const int32_t half = one >> 1;
        const int32_t oneplushalf = one | half;
        if (passtype == 0) {
            for (uint32_t k = 0; k < h; k += 4)
                for (uint32_t x = 0; x < w; ++x)
                    for (uint32_t y = k; y < k + 4 && y < h; ++y) {
                        if (getbit(s.sig[y + 1] | s.visit[y + 1], x) || !any_nb(s, x, y)) continue;
                        if (mqd_decode(d, cxs, tab, CX_ZC + zc_of(s, x, y, orient))) {
                            uint32_t xr;
                            int cx = sc_of(s, x, y, &xr);
                            uint32_t sg = mqd_decode(d, cxs, tab, cx) ^ xr;
                            dst[(size_t)y * dstride + x] = sg ? -oneplushalf : oneplushalf;
                            setbit(s.sig[y + 1], x);
                            if (sg) setbit(s.neg[y + 1], x);
                        }
                        setbit(s.visit[y + 1], x);
                    }
        } else if (passtype == 1) {
            for (uint32_t k = 0; k < h; k += 4)
                for (uint32_t x = 0; x < w; ++x)
                    for (uint32_t y = k; y < k + 4 && y < h; ++y) {
                        if (!getbit(s.sig[y + 1], x) || getbit(s.visit[y + 1], x)) continue;
                        uint32_t v = mqd_decode(d, cxs, tab, mag_of(s, x, y));
                        int32_t *dp = &dst[(size_t)y * dstride + x];
                        *dp += (v ^ (uint32_t)(*dp < 0)) ? half : -half;
                        setbit(s.ref[y + 1], x);
                    }
        } else {
            for (uint32_t k = 0; k < h; k += 4)
                for (uint32_t x = 0; x < w; ++x) {
                    uint32_t y0 = k;
                    bool partial = false;
                    if (k + 4 <= h) {
                        uint64_t win = 0;
                        for (uint32_t yy = k; yy < k + 6; ++yy) win |= s.sig[yy];
                        uint64_t vis = s.visit[k + 1] | s.visit[k + 2] | s.visit[k + 3] | s.visit[k + 4];
                        if (bits3(win, x) == 0 && getbit(vis, x) == 0) {
                            if (!mqd_decode(d, cxs, tab, CX_AGG)) continue;
                            uint32_t r = mqd_decode(d, cxs, tab, CX_UNI);
                            r = (r << 1) | mqd_decode(d, cxs, tab, CX_UNI);
                            y0 = k + r;
                            partial = true;
                        }
                    }
                    for (uint32_t y = y0; y < k + 4 && y < h; ++y) {
                        uint32_t code_sign = 0;
                        if (partial && y == y0) code_sign = 1;
                        else if (!getbit(s.sig[y + 1] | s.visit[y + 1], x))
                            code_sign = mqd_decode(d, cxs, tab, CX_ZC + zc_of(s, x, y, orient));
                        if (code_sign) {
                            uint32_t xr;
                            int cx = sc_of(s, x, y, &xr);
                            uint32_t sg = mqd_decode(d, cxs, tab, cx) ^ xr;
                            dst[(size_t)y * dstride + x] = sg ? -oneplushalf : oneplushalf;
                            setbit(s.sig[y + 1], x);
                            if (sg) setbit(s.neg[y + 1], x);
                        }
                        clrbit(s.visit[y + 1], x);
                    }
                }
        }
        if (++passtype == 3) { passtype = 0; bpno_plus_one--; }
    }
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) store(&dst[(size_t)y * dstride + x]);
}

struct PostDecode {
    int32_t irreversible;
    float step;
    GRK_HD void operator()(int32_t *p) const {
        int32_t v = *p;
        if (!irreversible) {
            *p = v / 2;
        } else {
            float f = (float)v * step;
            *p = __builtin_bit_cast(int32_t, f);
        }
    }
};

}  // namespace grkgpu
