// t1_dec.h -- the EBCOT Tier-1 decoder's pass / stripe / column walk: one
// lane per code-block (the decoder "v5", fed by t1_flat.h's unstuffed bit
// stream; kernels.hip k_t1_decode_ub).
//
//   * block state = 64-bit row masks in HBM, one 4-row stripe held in
//     registers (Stripe); each lane visits only the columns of a stripe that
//     hold work for the pass (bit-scan of candidate masks)
//   * per column, the 3x6 significance neighbourhood (rows k-1..k+4, columns
//     x-1..x+1) is packed into an 18-bit window P; the zero-coding context of
//     row r is the LUT entry for (P >> 3r) & 0x1FF and the sign context comes
//     from the N/W/E/S bits of P and of the matching sign window Q
//   * the symbols of a column go through ONE decode site (a small state
//     machine: ZC -> SC, AGG -> UNI -> UNI -> SC), so lanes of a wavefront
//     that sit in different rows / symbol kinds still share the MQ code
//   * outputs are write-only bit-plane rows (sigafter / refbit, t1_lane.h)
//     rebuilt into coefficients by k_t1_rebuild.
//
// Semantics: Grok v5.1.0 t1/t1_part1/t1.cpp t1_decode_cblk (:1038) with
// dec_sigpass / dec_refpass / dec_clnpass, mqc_dec_inl.h, and the mode
// switches (see t1_decode_passes).
#pragma once
#include "t1_lane.h"

// T1_WALK(event, value): a host analysis hook on the walk (pass start: 0,
// pass type; stripe start: 1, row; column start: 2, column); empty in the
// library (tests/cpp/t1_walk_sim.cpp defines it).
#ifndef T1_WALK
#define T1_WALK(ev, v)
#endif

namespace grkgpu {

// sign LUT in window order: bit0 sigN, 1 negN, 2 sigW, 3 negW, 4 sigE, 5 negE,
// 6 sigS, 7 negS  ->  context | xorbit << 7
GRK_HD uint8_t sc_win_entry(uint32_t i) {
    uint32_t xr;
    int cx = sc_ctx((i >> 2) & 1, (i >> 4) & 1, i & 1, (i >> 6) & 1, (i >> 3) & 1, (i >> 5) & 1, (i >> 1) & 1,
                    (i >> 7) & 1, &xr);
    return (uint8_t)(cx | (xr << 7));
}

// 18-bit 3x6 window of column x: bits 3i..3i+2 = row i (k-1+i), columns x-1..x+1
// (column 0: the rows' bits 0..2 moved up one, the left column zero -- one
// shift and mask of the whole window instead of a per-row shift)
GRK_HD uint32_t win18(const uint64_t *r6, uint32_t x) {
    const uint32_t s1 = x ? x - 1 : 0;
    uint32_t P = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) P |= (((uint32_t)(r6[i] >> s1)) & 7u) << (3 * i);
    return x ? P : (P << 1) & 0x36DB6u;
}

// A column's four rows as a mask in the window's row spacing: row i at bit
// 3i (SPREAD), so a row's bit position is also its window shift
constexpr uint32_t SPREAD4 = 0x249u;  // rows 0..3
GRK_HD uint32_t col4s(const uint64_t *r4, uint32_t x) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) v |= (uint32_t)((r4[i] >> x) & 1) << (3 * i);
    return v;
}

GRK_HD void setcol4s(uint64_t *r4, uint32_t x, uint32_t bits) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r4[i] |= (uint64_t)((bits >> (3 * i)) & 1) << x;
}

// self bits of the window (rows k..k+3 of column x), spread
GRK_HD uint32_t win_self4s(uint32_t P) { return (P >> 4) & SPREAD4; }

// Keep v computed at this point for every lane: stops the compiler from
// sinking its producer (an LDS read) into a branch around its one use.
GRK_HD void keep_here(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" ::"v"(v));
#else
    (void)v;
#endif
}

// true if p holds on any active lane of the wavefront (wave-uniform); the
// host build runs one block at a time
GRK_HD bool wave_any(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __ballot(p) != 0;
#else
    return p;
#endif
}

struct DecTables {
    const uint8_t *zc;   // 512 entries for this block's orientation
    const uint8_t *sc;   // 256, window order
    const uint32_t *mq;  // MQ_DEC_WORDS successor-table entries (t1_lane.h mq_dec_table_entry)
};

// significance propagation (CUP = false) or cleanup (CUP = true) of one
// column; returns true if a sample became significant.
// CUP < 0: the pass type is the runtime flag `cup` (one instantiation for
// both passes, so lanes of a wavefront in an SPP and in a cleanup pass share
// the column code and its decode site).
template <int CUP_, class D>
GRK_HD bool d3_column(D &d, uint32_t *cxw, const DecTables &T, Stripe &s, uint32_t x, uint32_t nr, bool cup_rt = false) {
    const bool CUP = CUP_ < 0 ? cup_rt : CUP_ != 0;
    T1_WALK(2, x);
    // row masks are spread (row r at bit 3r: col4s), so the current row's
    // position p = 3r is its window shift as it stands
    uint32_t P = win18(s.sig, x);
    const uint32_t vis4 = col4s(s.vis, x);
    const uint32_t rows = SPREAD4 >> (12 - 3 * nr);
    const uint32_t sig4 = win_self4s(P);
    uint32_t nz = SPREAD4;  // SPP: rows with a significant neighbour
    if (CUP_ <= 0) {
        uint32_t z = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) z |= (((P >> (3 * r)) & 0x1EF) != 0 ? 1u : 0u) << (3 * r);
        nz = CUP ? SPREAD4 : z;
    }
    uint32_t todo = nz & ~sig4 & ~vis4 & rows;
    const uint32_t todo0 = todo;
    uint32_t kind = 0, p = 0;  // kind: 0 ZC, 1 SC, 2 AGG, 3 UNI(hi), 4 UNI(lo); p = 3 x row
    // the context of the next symbol when it is not a ZC one: AGG, then UNI
    // after an aggregation 1, or the SC context read with the sign LUT -- set
    // at the transitions, so a step only selects between it and the ZC LUT's
    uint32_t cxn = CX_AGG;
    if (CUP && nr == 4 && P == 0 && vis4 == 0) {
        kind = 2;
    } else {
        if (!todo) return false;
        p = (uint32_t)__builtin_ctz(todo);
    }
    // the sign window, read at the column start by every lane: a lane's first
    // sign symbol comes at almost every decision step of a wavefront, so a
    // lazy read would be a branch entered at every step
    uint32_t Q = win18(s.neg, x), si = 0;
    // The symbol-kind transitions are selects, not branches: the 64 lanes of
    // a wavefront sit in different kinds, and every branch taken by any lane
    // costs the whole wavefront its exec-mask bookkeeping.
    for (;;) {
        const uint32_t zcx = T.zc[(P >> p) & 0x1FF];  // read for every kind (LDS, in bounds)
        keep_here(zcx);
        const uint32_t cx = kind == 0 ? zcx : cxn;
        const uint32_t bit = d.decode(cxw, T.mq, cx);
        if (kind == 2 && !bit) break;  // aggregation symbol 0: the column is done
        const bool k0 = kind == 0, k1 = kind == 1, k3 = kind == 3, k4 = kind == 4;
        // SC: the sample is significant with sign sg
        const uint32_t sg = bit ^ ((D::kLazy && d.raw) ? 0u : (si >> 7));  // a raw sign is the sign itself
        // the new significance and sign go into the windows only: the
        // column's new rows are read back from them once, after the loop
        P |= k1 ? 1u << (p + 4) : 0u;
        Q |= k1 ? sg << (p + 4) : 0u;
        // the sample below now has a significant neighbour (SPP)
        todo |= (!CUP && k1) ? (rows & ~(sig4 | vis4)) & (8u << p) : 0u;
        // UNI, UNI: the run position (row 2 bit1 + bit0); the rows after it are plain ZC
        p = k3 ? (bit ? 6u : 0u) : k4 ? p + (bit ? 3u : 0u) : p;
        todo = k4 ? rows & ~((8u << p) - 1) : todo;
        const bool advance = k1 || (k0 && !bit);
        cxn = kind == 2 ? (uint32_t)CX_UNI : cxn;  // aggregation 1: the run position in UNI
        kind = k0 ? bit : k1 ? 0u : kind == 2 ? 3u : k3 ? 4u : 1u;
        if (kind == 1 && !advance) {
            si = T.sc[(((P >> p) & 0xAA) >> 1) | ((Q >> p) & 0xAA)];
            cxn = si & 0x7fu;
        }
        todo = advance ? todo & ~((8u << p) - 1) : todo;
        if (advance && !todo) break;
        p = advance ? (uint32_t)__builtin_ctz(todo | (1u << 12)) : p;
    }
    const uint32_t newsig = win_self4s(P) & ~sig4;
    // SPP: every row of the column's candidates was visited (a ZC symbol),
    // the rows a new significant sample above made candidates included
    const uint32_t newvis = todo0 | ((newsig << 3) & rows & ~(sig4 | vis4));
    if (!CUP && newvis) setcol4s(s.vis, x, newvis);
    if (newsig) {
        setcol4s(s.sig + 1, x, newsig);
        setcol4s(s.neg + 1, x, win_self4s(Q) & newsig);
        return true;
    }
    return false;
}

// Magnitude refinement, 8 columns at a time.  The pass never changes
// significance, so the stripe's rows to refine (e) and their "a neighbour is
// significant" rows (nb: the 8-neighbourhood of t1.cpp's T1_SIGMA_NEIGHBOURS)
// are formed once per stripe with row-mask operations.  Its decisions come in
// column-major order within the stripe (column x, rows k..k+3), so a group of
// 8 columns is turned into one 32-bit word with bit 4c + i = row i of column
// c (nib4): the group's decisions are the word's set bits in order, their
// contexts bits of two more such words, and the refinement bits are gathered
// in a fourth and spread back into the rows once per group -- no per-column
// extraction of row bits.
GRK_HD uint32_t spread8(uint32_t b) {  // bit c of b -> bit 4c
    b = (b | (b << 12)) & 0x000F000Fu;
    b = (b | (b << 6)) & 0x03030303u;
    return (b | (b << 3)) & 0x11111111u;
}
GRK_HD uint32_t unspread8(uint32_t x) {  // bit 4c of x -> bit c
    x &= 0x11111111u;
    x = (x | (x >> 3)) & 0x03030303u;
    x = (x | (x >> 6)) & 0x000F000Fu;
    return (x | (x >> 12)) & 0xFFu;
}
GRK_HD uint32_t nib4(const uint64_t *r4, uint32_t sh) {
    return spread8((uint32_t)(r4[0] >> sh) & 0xFFu) | spread8((uint32_t)(r4[1] >> sh) & 0xFFu) << 1 |
           spread8((uint32_t)(r4[2] >> sh) & 0xFFu) << 2 | spread8((uint32_t)(r4[3] >> sh) & 0xFFu) << 3;
}

template <bool REG, class D>
GRK_HD void d3_mrp_stripe(D &d, uint32_t *cxw, const DecTables &T, const uint64_t *e, const uint64_t *nb,
                          const uint64_t *ref, uint64_t *bit, uint64_t mem) {
    // REG: the pass's three contexts (t1.cpp dec_refpass: 14 + (refined before
    // ? 2 : a significant neighbour)) live in registers for the stripe -- no
    // LDS round trip on the decision chain: lone 8K 9/7 decode T1 30.4 / 31.3
    // -> 29.4 / 29.2 ms, the 16-frame batch unchanged (3438 / 3514 vs 3452 /
    // 3486 Mpixels/s alternating, profiles/r05/t1_mrp_reg_ab.txt)
    uint32_t w0 = 0, w1 = 0, w2 = 0;
    if constexpr (REG) { w0 = cxw[CX_MAG]; w1 = cxw[CX_MAG + 1]; w2 = cxw[CX_MAG + 2]; }
    for (uint32_t g = 0; g < 8; ++g) {
        const uint32_t sh = 8 * g;
        if (!((mem >> sh) & 0xFFu)) continue;
        T1_WALK(2, sh);
        uint32_t E = nib4(e, sh);
        const uint32_t R = nib4(ref, sh), N = nib4(nb, sh);
        uint32_t res = 0;
        // context 14 (a first refinement without a significant neighbour) is
        // rare (~1 in 10^5 refinement decisions): a group no lane of the
        // wavefront needs it for picks between 15 and 16 on one mask bit
        if (REG && !wave_any((E & ~R & ~N) != 0)) {
            while (E) {
                const uint32_t pos = (uint32_t)__builtin_ctz(E);
                E &= E - 1;
                const bool r2 = (R >> pos) & 1;
                uint32_t wd = r2 ? w2 : w1;
                res |= d.decode_reg(wd, T.mq, CX_MAG + (r2 ? 2u : 1u)) << pos;
                w1 = r2 ? w1 : wd;
                w2 = r2 ? wd : w2;
            }
        }
        while (E) {
            const uint32_t pos = (uint32_t)__builtin_ctz(E);
            E &= E - 1;
            const uint32_t k = ((R >> pos) & 1) ? 2u : (N >> pos) & 1;
            if constexpr (REG) {
                uint32_t wd = k == 2 ? w2 : k == 1 ? w1 : w0;
                res |= d.decode_reg(wd, T.mq, CX_MAG + k) << pos;
                w0 = k == 0 ? wd : w0;
                w1 = k == 1 ? wd : w1;
                w2 = k == 2 ? wd : w2;
            } else {
                res |= d.decode(cxw, T.mq, CX_MAG + k) << pos;
            }
        }
        if (res) {
#pragma unroll
            for (int i = 0; i < 4; ++i) bit[i] |= (uint64_t)unspread8(res >> i) << sh;
        }
    }
    if constexpr (REG) { cxw[CX_MAG] = w0; cxw[CX_MAG + 1] = w1; cxw[CX_MAG + 2] = w2; }
}

// Codeword segments of a block: a single one (NoSegs) or a cursor that
// re-initialises the decoder at each segment's first pass (t1_decode_cblk's
// per-segment mqc_init_dec, t1.cpp:1066-1113).
struct NoSegs {
    template <class D> GRK_HD void at_pass(D &, uint32_t, bool) {}
};

// The pass / stripe / column walk over an MQ / raw bit source D (BitDecT,
// t1_flat.h).  Mode switches
// (cblksty): VSC -- row k+4 reads as insignificant for row k+3 (the flags
// update of t1.cpp:168-190 skips the north neighbours of a stripe's first
// row); RESET -- contexts re-initialised after every pass (t1.cpp:1104-1105);
// SEGSYM -- four uniform-context symbols end every cleanup pass (t1.cpp:873-889).
// ST / RP: the block state and the bit-plane row pointers -- plain arrays
// (BlockState, uint64_t *: host tests) or the GPU decoder's lane-interleaved
// rows (kernels.hip LState / LRow, t1_lane.h).
template <class D, class S = NoSegs, class ST = BlockState, class RP = uint64_t *, bool MRPREG = true>
GRK_HD void t1_decode_passes(D &d, uint32_t numpasses, uint32_t numbps, uint32_t w, uint32_t h, ST &st,
                             const DecTables &T, uint32_t *cxw, RP sigafter, RP refbit,
                             uint32_t sty = 0, S segs = S(), uint32_t roishift = 0) {
    // BYPASS pass types are classified against the block's bit-planes less
    // the ROI shift (t1_decode_cblk gets numbps - roishift, T1Part1.cpp:186,
    // while its bit-plane counter starts at numbps, t1.cpp:1055 / 1070-1072)
    const uint32_t rawbps = numbps - roishift;
    const uint64_t wm = w >= 64 ? ~(uint64_t)0 : (((uint64_t)1 << w) - 1);
    const bool vsc = (sty & CBLKSTY_VSC) != 0;
    int32_t bpno = (int32_t)numbps - 1;
    int passtype = 2;
    for (uint32_t passno = 0; passno < numpasses && bpno >= 0; ++passno) {
        segs.at_pass(d, passno, t1_pass_raw(sty, bpno, passtype, rawbps));
        T1_WALK(0, passtype);
        const RP sa = sigafter + (uint32_t)bpno * 64;
        const RP rb = refbit + (uint32_t)bpno * 64;
        // Each pass type loads and stores only the state rows it reads or
        // changes (SPP / CUP: sig, neg, vis; MRP: sig, vis, ref + the
        // refinement bits), so no row is live across the three branches:
        // fewer VGPRs for the lane decoder and fewer state round trips.
        for (uint32_t k = 0; k < h; k += 4) {
            const uint32_t nr = h - k < 4 ? h - k : 4;
            d.fill();  // the bit source tops up its word ring with the stripe's row loads
            T1_WALK(1, k);
            Stripe s;
#pragma unroll
            for (int i = 0; i < 6; ++i) s.sig[i] = st.sig[k + i];
            if (vsc) s.sig[5] = 0;
            // vis (visited by this plane's SPP) is reset by every cleanup
            // pass, so an SPP starts from zero and only the SPP stores it
#pragma unroll
            for (int i = 0; i < 4; ++i) s.vis[i] = passtype == 0 ? 0 : (uint64_t)st.vis[k + 1 + i];
            if (passtype == 1) {
                uint64_t e[4], nb[4], mem = 0;  // rows to refine, rows with a significant neighbour
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    s.ref[i] = st.ref[k + 1 + i];
                    s.bit[i] = 0;
                    const uint64_t sg = s.sig[i + 1];
                    e[i] = (uint32_t)i < nr ? sg & ~s.vis[i] : 0;
                    nb[i] = dil(s.sig[i]) | dil(s.sig[i + 2]) | (sg << 1) | (sg >> 1);
                    mem |= e[i];
                }
                if (mem) d3_mrp_stripe<MRPREG>(d, cxw, T, e, nb, s.ref, s.bit, mem);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    st.ref[k + 1 + i] = s.ref[i] | e[i];  // every refined sample is now "refined once"
                    if ((uint32_t)i < nr) rb[k + i] = s.bit[i];
                }
                continue;
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) s.neg[i] = st.neg[k + i];
            if (vsc) s.neg[5] = 0;
            bool chg = false;  // a sample of the stripe became significant
            if (passtype == 0) {
                uint64_t cand = spp_candidates(s, nr) & wm;
                while (cand) {
                    const uint32_t x = ctz64(cand);
                    const uint64_t done = ((uint64_t)2 << x) - 1;  // x = 63 wraps to all ones
                    const bool grew = d3_column<0>(d, cxw, T, s, x, nr);
                    cand &= ~done;
                    // a new significant sample in column x can only make
                    // column x + 1 a candidate (x - 1 is behind the scan)
                    if (grew) cand |= ((uint64_t)2 << x) & wm;
                    chg = chg || grew;
                }
            } else {
                uint64_t cand = 0;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if ((uint32_t)r < nr) cand |= ~(s.sig[r + 1] | s.vis[r]);
                cand &= wm;
                while (cand) {
                    const uint32_t x = ctz64(cand);
                    cand &= cand - 1;
                    chg = d3_column<1>(d, cxw, T, s, x, nr) || chg;
                }
            }
            // write back only what changed: sig / neg if the stripe grew, vis
            // after an SPP, and the significance-after-plane rows after the
            // cleanup pass -- or after the SPP when this plane's cleanup is
            // not decoded (truncated pass count)
            const bool wsa = passtype == 2 || passno + 2 >= numpasses;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (chg) {
                    st.sig[k + 1 + i] = s.sig[i + 1];
                    st.neg[k + 1 + i] = s.neg[i + 1];
                }
                if (passtype == 0) st.vis[k + 1 + i] = s.vis[i];
                if (wsa && (uint32_t)i < nr) sa[k + i] = s.sig[i + 1];
            }
        }
        if (passtype == 2 && (sty & CBLKSTY_SEGSYM))
            for (int q = 0; q < 4; ++q) d.decode(cxw, T.mq, CX_UNI);
        if ((sty & CBLKSTY_RESET) && !(D::kLazy && d.raw)) mq_reset_words_dec(cxw, T.mq);  // after MQ passes (t1.cpp:1104-1105)
        if (++passtype == 3) { passtype = 0; bpno--; }
    }
}

}  // namespace grkgpu
