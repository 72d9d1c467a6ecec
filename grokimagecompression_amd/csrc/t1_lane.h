// t1_lane.h -- lane-per-code-block EBCOT Tier-1 encoder (MI355X layout) and
// the block state shared with the decoder.
//
// All per-block state lives in HBM as 64-bit ROW MASKS (bit x = column x).
// The encoder is split in two kernels (kernels.hip):
//   * k_t1_model: the context modelling of one bit-plane of one block per
//     lane (t1_model_plane): significance / refinement / cleanup passes formed
//     with row-mask arithmetic, one byte per MQ symbol (context | decision)
//     into the block's symbol stream;
//   * k_t1_mq: the serial MQ coder per block (t1_mq_block) over those symbols,
//     with Grok's rate bookkeeping, pass terminations and BYPASS raw coding.
// Decoded magnitudes are never read back by the decoder (t1_dec.h): it writes
// write-only bit-plane rows (significance after each plane, refinement bits
// per plane) and a separate, fully parallel kernel rebuilds the values
// (t1_rebuild).  Same source compiles for the host (tests/cpp) and gfx950.
//
// Semantics: Grok v5.1.0 t1/t1_part1/t1.cpp (t1_encode_cblk :1182,
// t1_decode_cblk :1038), mqc_enc.cpp, mqc_dec_inl.h.
#pragma once
#include "t1_core.h"

namespace grkgpu {

// ---- LUTs (built once per workgroup into LDS; host: static arrays) ----
// zero coding: index orient*512 + 9-bit neighbourhood (NW,N,NE,W,-,E,SW,S,SE)
GRK_HD uint8_t zc_lut_entry(uint32_t orient, uint32_t nb) {
    int h = (int)(((nb >> 3) & 1) + ((nb >> 5) & 1));
    int v = (int)(((nb >> 1) & 1) + ((nb >> 7) & 1));
    int d = (int)((nb & 1) + ((nb >> 2) & 1) + ((nb >> 6) & 1) + ((nb >> 8) & 1));
    return (uint8_t)zc_ctx(h, v, d, orient);
}
// sign coding: index bit0 sigW, 1 negW, 2 sigE, 3 negE, 4 sigN, 5 negN, 6 sigS, 7 negS
// entry: context number | xorbit << 7
GRK_HD uint8_t sc_lut_entry(uint32_t i) {
    uint32_t xr;
    int cx = sc_ctx(i & 1, (i >> 2) & 1, (i >> 4) & 1, (i >> 6) & 1, (i >> 1) & 1, (i >> 3) & 1, (i >> 5) & 1,
                    (i >> 7) & 1, &xr);
    return (uint8_t)(cx | (xr << 7));
}

struct T1Tables {
    const uint8_t *zc;    // 2048
    const uint8_t *sc;    // 256
    const uint32_t *mq;   // 47
};

// 3 bits (x-1, x, x+1) of a row mask
GRK_HD uint32_t b3(uint64_t row, uint32_t x) {
    uint32_t left = x ? (uint32_t)(row >> (x - 1)) & 1u : 0u;
    return left | (((uint32_t)(row >> x) & 3u) << 1);
}

GRK_HD uint32_t nb9(uint64_t up, uint64_t mid, uint64_t dn, uint32_t x) {
    return b3(up, x) | ((b3(mid, x) & 5u) << 3) | (b3(dn, x) << 6);
}

GRK_HD uint32_t sc_index(uint64_t sup, uint64_t smid, uint64_t sdn, uint64_t nup, uint64_t nmid, uint64_t ndn,
                         uint32_t x) {
    uint32_t sm = b3(smid, x), nm = b3(nmid, x);
    uint32_t i = (sm & 1) | ((nm & 1) << 1) | (((sm >> 2) & 1) << 2) | (((nm >> 2) & 1) << 3);
    i |= (uint32_t)((sup >> x) & 1) << 4 | (uint32_t)((nup >> x) & 1) << 5;
    i |= (uint32_t)((sdn >> x) & 1) << 6 | (uint32_t)((ndn >> x) & 1) << 7;
    return i;
}

// ---- per-block HBM state (rows y = -1..h stored at index y+1) ----
struct BlockState {
    uint64_t sig[66];
    uint64_t neg[66];
    uint64_t vis[66];
    uint64_t ref[66];
};

// pass index -> (plane, type): pass 0 = cleanup of plane numbps-1, then
// (sig, ref, cln) per lower plane.
GRK_HD void pass_info(uint32_t passno, uint32_t numbps, int32_t *plane, int *type) {
    if (passno == 0) { *plane = (int32_t)numbps - 1; *type = 2; return; }
    *plane = (int32_t)numbps - 2 - (int32_t)((passno - 1) / 3);
    *type = (int)((passno - 1) % 3);
}

// explicit s_waitcnt vmcnt(0): placed where the data is known to have landed
// long ago, so the compiler does not scatter conservative waits in hot loops
GRK_HD void vm_wait_all() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
}
GRK_HD uint32_t clz32(uint32_t v) { return (uint32_t)__builtin_clz(v); }
// v_alignbit_b32: the low 32 bits of {hi, lo} >> (sh & 31)
GRK_HD uint32_t alignbit32(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (sh & 31));
#endif
}
// v_bfe_u32: w bits of v from bit (off & 31); w = 0 gives 0 (w < 32 here)
GRK_HD uint32_t bfe32(uint32_t v, uint32_t off, uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ubfe(v, off, w);
#else
    return w ? (v >> (off & 31)) & ((1u << w) - 1) : 0u;
#endif
}
GRK_HD uint32_t ctz64(uint64_t v) { return (uint32_t)__builtin_ctzll(v); }
GRK_HD uint64_t dil(uint64_t m) { return m | (m << 1) | (m >> 1); }

// code-block style bits (COD SPcod, grok.h GRK_CBLKSTY_*): the mode switches
// this coder takes (BYPASS 0x01 and HT 0x40 are rejected by the host)
constexpr uint32_t CBLKSTY_LAZY = 0x01, CBLKSTY_RESET = 0x02, CBLKSTY_TERMALL = 0x04, CBLKSTY_VSC = 0x08,
                   CBLKSTY_PTERM = 0x10, CBLKSTY_SEGSYM = 0x20;

// Pass classification of t1_encode_cblk / t1_decode_cblk: BYPASS (LAZY)
// codes the significance and refinement passes below the four most
// significant bit-planes raw (t1.cpp:1223-1225, 1070-1072), and
// t1_enc_is_term_pass (t1.cpp:1131-1151) decides which passes end a codeword
// segment.
GRK_HD bool t1_pass_raw(uint32_t sty, int32_t bpno, int passtype, uint32_t numbps) {
    return (sty & CBLKSTY_LAZY) && bpno < (int32_t)numbps - 4 && passtype < 2;
}
GRK_HD bool t1_pass_term(uint32_t sty, int32_t bpno, int passtype, uint32_t numbps) {
    if (passtype == 2 && bpno == 0) return true;
    if (sty & CBLKSTY_TERMALL) return true;
    if (sty & CBLKSTY_LAZY) {
        if (bpno == (int32_t)numbps - 4 && passtype == 2) return true;
        if (bpno < (int32_t)numbps - 4 && passtype > 0) return true;
    }
    return false;
}

// MQ context registers are 32-bit words: the packed table entry of the
// current state (Qe | NMPS<<16 | NLPS<<22 | SWITCH<<28) | MPS<<31, so one LDS
// read per symbol yields Qe; the next-state lookup is off the critical path.
// mqc_resetstates (mqc_dec.cpp:207-215): UNI -> 46, AGG -> 3, ZC0 -> 4.
GRK_HD void mq_reset_words(uint32_t *cxw, const uint32_t *tab) {
    for (int i = 0; i < NUM_CX; ++i) cxw[i] = tab[0];
    cxw[CX_UNI] = tab[46];
    cxw[CX_AGG] = tab[3];
    cxw[CX_ZC] = tab[4];
}

// The DECODER's context words (t1_flat.h BitDecT::step): one word per
// (state, MPS) pair i = 2 state + mps -- Qe[31:16] | i << 2 | MPS [0].  Qe
// sits where the decoder's A and C registers compare against it (A held
// << 16, C[31:16] = Chigh), so the decision needs no shifts of it; bits
// [8:2] are the pair's byte offset in the successor table below, and the
// decoded bit is (word ^ LPS) & 1.
GRK_HD uint32_t mq_dec_word(const uint32_t *tab47, uint32_t i) {
    const uint32_t qe = tab47[i >> 1] & 0xffffu;
    return (qe << 16) | (i << 2) | (i & 1u);
}
// The successor table the decoder reads after every decision (LDS):
// entry i (< 94) is the word of pair i's MPS successor, entry 128 + i that
// of its LPS successor (SWITCH's MPS flip folded in), so the address is
// (word & 0x1FC) | (LPS ? 512 : 0) bytes -- one op on the decision chain.
// Entries 94..97 hold the reset words (mqc_resetstates, mqc_dec.cpp:207-215:
// every context state 0 MPS 0, UNI -> 46, AGG -> 3, ZC0 -> 4).  ISO 15444-1
// Table C.2 via the encoder table (Qe | NMPS<<16 | NLPS<<22 | SWITCH<<28).
constexpr uint32_t MQ_DEC_WORDS = 128 + 94;
GRK_HD uint32_t mq_dec_table_entry(const uint32_t *tab47, uint32_t k) {
    if (k >= 128) {
        const uint32_t i = k - 128, t = tab47[i >> 1], m = i & 1u;
        return mq_dec_word(tab47, 2 * ((t >> 22) & 63u) + (m ^ ((t >> 28) & 1u)));
    }
    if (k < 94) {
        const uint32_t t = tab47[k >> 1];
        return mq_dec_word(tab47, 2 * ((t >> 16) & 63u) + (k & 1u));
    }
    switch (k) {
        case 94: return mq_dec_word(tab47, 0);
        case 95: return mq_dec_word(tab47, 2 * 46);
        case 96: return mq_dec_word(tab47, 2 * 3);
        case 97: return mq_dec_word(tab47, 2 * 4);
        default: return 0;
    }
}
// mqc_resetstates in decoder words, from the table's entries 94..97
GRK_HD void mq_reset_words_dec(uint32_t *cxw, const uint32_t *dtab) {
    for (int i = 0; i < NUM_CX; ++i) cxw[i] = dtab[94];
    cxw[CX_UNI] = dtab[95];
    cxw[CX_AGG] = dtab[96];
    cxw[CX_ZC] = dtab[97];
}

// ---------------------------------------------------------------------------
// MQ encoder (mqc_enc.cpp) with a register byte sink: only the byte at bp can
// still change (carry); everything before it is final and leaves as dwords.
// ---------------------------------------------------------------------------
struct MqEncLane {
    uint32_t a, c, ct;
    int32_t bp;        // index of `cur` (starts at -1: Grok's bp = start - 1)
    uint32_t cur;      // byte at bp (still subject to carry)
    uint32_t acc;      // committed bytes of the current dword
    uint32_t *out;     // 4-byte aligned
};

// acc's byte at pos is zero until pos is committed (acc starts at zero, is
// zeroed with every store, and mqel_step_back clears the byte it re-opens),
// so a commit is one shift-or.  The pad byte before the block (pos -1) is
// committed like any other and lands in out[-1]: the caller leaves a dword
// of headroom before `out` (codec.cpp's MQ slab: 16 bytes between blocks),
// and nothing reads it back (mqel_byte_at answers 0 for pos < 0).
GRK_HD void sink_commit(MqEncLane &e, int32_t pos, uint32_t byte) {
    const uint32_t sh = ((uint32_t)pos & 3u) * 8u;
    e.acc |= byte << sh;
    if ((pos & 3) == 3) { e.out[pos >> 2] = e.acc; e.acc = 0; }
}

GRK_HD void mqel_emit(MqEncLane &e, uint32_t byte) {  // new byte at bp + 1
    sink_commit(e, e.bp, e.cur);
    e.bp++;
    e.cur = byte & 0xFF;
}

// BYTEOUT (mqc_enc.cpp:168-199)
GRK_HD void mqel_byteout(MqEncLane &e) {
    if (e.cur == 0xff) {
        mqel_emit(e, e.c >> 20); e.c &= 0xfffff; e.ct = 7;
    } else if ((e.c & 0x8000000) == 0) {
        mqel_emit(e, e.c >> 19); e.c &= 0x7ffff; e.ct = 8;
    } else {
        e.cur++;
        if (e.cur == 0xff) {
            e.c &= 0x7ffffff;
            mqel_emit(e, e.c >> 20); e.c &= 0xfffff; e.ct = 7;
        } else {
            mqel_emit(e, e.c >> 19); e.c &= 0x7ffff; e.ct = 8;
        }
    }
}

// encode (mqc_enc.cpp:50-110); RENORME's one-bit loop becomes clz-sized
// shifts between byte boundaries (identical state sequence).
GRK_HD void mqel_encode(MqEncLane &e, uint32_t *cxw, const uint32_t *tab, uint32_t cx, uint32_t d) {
    const uint32_t w = cxw[cx];
    const uint32_t qe = w & 0xffff, mps = w >> 31;
    e.a -= qe;
    if (d == mps) {
        if (e.a & 0x8000) { e.c += qe; return; }
        if (e.a < qe) e.a = qe; else e.c += qe;
        cxw[cx] = tab[(w >> 16) & 63] | (mps << 31);
    } else {
        if (e.a < qe) e.c += qe; else e.a = qe;
        cxw[cx] = tab[(w >> 22) & 63] | ((mps ^ ((w >> 28) & 1)) << 31);
    }
    uint32_t n = clz32(e.a) - 16;
    while (n) {
        uint32_t sh = n < e.ct ? n : e.ct;
        e.a <<= sh; e.c <<= sh; e.ct -= sh; n -= sh;
        if (e.ct == 0) mqel_byteout(e);
    }
}

GRK_HD void mqel_flush(MqEncLane &e) {
    uint32_t tempc = e.c + e.a;
    e.c |= 0xffff;
    if (e.c >= tempc) e.c -= 0x8000;
    e.c <<= e.ct; mqel_byteout(e);
    e.c <<= e.ct; mqel_byteout(e);
    if (e.cur != 0xff) mqel_emit(e, 0);  // "if (*bp != 0xff) bp++"
}

// ERTERM, predictable termination (mqc_erterm_enc, mqc_enc.cpp:384-395)
GRK_HD void mqel_erterm(MqEncLane &e) {
    int32_t k = (int32_t)(11 - e.ct + 1);
    while (k > 0) {
        e.c <<= e.ct;
        e.ct = 0;
        mqel_byteout(e);
        k -= (int32_t)e.ct;
    }
    if (e.cur != 0xff) mqel_byteout(e);
}

// The byte at position pos (< bp): committed, in `acc` when it shares bp's
// dword, else in `out`.
GRK_HD uint32_t mqel_byte_at(const MqEncLane &e, int32_t pos) {
    if (pos < 0) return 0;  // the zero pad byte before the block
    if ((pos >> 2) == (e.bp >> 2)) return (e.acc >> ((pos & 3) * 8)) & 0xffu;
    return (e.out[pos >> 2] >> ((pos & 3) * 8)) & 0xffu;
}

// bp-- (the reference steps its byte pointer back in a few terminations):
// the byte there becomes `cur` again, and acc is reloaded when bp crosses
// back into the previous (already stored) dword.
GRK_HD void mqel_step_back(MqEncLane &e) {
    const int32_t nb = e.bp - 1;
    if (nb < 0) {
        e.cur = 0;
        e.acc = 0;
    } else {
        if ((nb >> 2) != (e.bp >> 2)) e.acc = e.out[nb >> 2];
        e.cur = (e.acc >> ((nb & 3) * 8)) & 0xffu;
        e.acc &= ~(0xffu << ((nb & 3) * 8));  // open again (sink_commit ORs into it)
    }
    e.bp = nb;
}

// Restart after a terminated pass (mqc_restart_init_enc, mqc_enc.cpp:366-382):
// INITENC again with bp stepped back onto the segment's last counted byte,
// which becomes the carry target again.
GRK_HD void mqel_restart(MqEncLane &e) {
    mqel_step_back(e);
    e.a = 0x8000;
    e.c = 0;
    e.ct = e.cur == 0xff ? 13u : 12u;
}

// ---- raw (BYPASS) coding, mqc_enc.cpp:264-364 ----
constexpr uint32_t BYPASS_CT_INIT = 0xDEADBEEFu;  // "no raw bit coded yet"

GRK_HD void mqel_bypass_init(MqEncLane &e) {  // mqc_bypass_init_enc: bp stays
    e.c = 0;
    e.ct = BYPASS_CT_INIT;
}

GRK_HD void mqel_bypass(MqEncLane &e, uint32_t d) {  // mqc_bypass_enc
    if (e.ct == BYPASS_CT_INIT) e.ct = 8;
    e.ct--;
    e.c += d << e.ct;
    if (e.ct == 0) {
        e.cur = e.c & 0xffu;  // *bp = c
        e.ct = e.cur == 0xff ? 7u : 8u;
        mqel_emit(e, 0);      // bp++
        e.c = 0;
    }
}

GRK_HD uint32_t mqel_bypass_extra(const MqEncLane &e, bool erterm) {  // mqc_bypass_get_extra_bytes_enc
    return (e.ct < 7 || (e.ct == 7 && (erterm || mqel_byte_at(e, e.bp - 1) != 0xff))) ? 2u : 1u;
}

GRK_HD void mqel_bypass_flush(MqEncLane &e, bool erterm) {  // mqc_bypass_flush_enc
    const uint32_t prev = mqel_byte_at(e, e.bp - 1);
    if (e.ct < 7 || (e.ct == 7 && (erterm || prev != 0xff))) {
        uint32_t bit = 0;  // fill the remaining bits with 0 1 0 1 ...
        while (e.ct > 0) {
            e.ct--;
            e.c += bit << e.ct;
            bit = 1u - bit;
        }
        e.cur = e.c & 0xffu;
        mqel_emit(e, 0);
    } else if (e.ct == 7 && prev == 0xff) {  // discard the last 0xFF
        mqel_step_back(e);
    } else if (e.ct == 8 && !erterm && prev == 0x7f && mqel_byte_at(e, e.bp - 2) == 0xff) {
        mqel_step_back(e);  // discard a terminating 0xFF 0x7F
        mqel_step_back(e);
    }
}

GRK_HD void mqel_finish(MqEncLane &e, uint32_t len) {
    if (e.bp >= 0 && (uint32_t)e.bp < len) sink_commit(e, e.bp, e.cur);
    if (len & 3) e.out[len >> 2] = e.acc;
}

// ---------------------------------------------------------------------------
// Coding passes, shared by encoder and decoder.  A 4-row stripe of the block
// state is held in registers; each lane walks only the columns that hold
// work for the pass (bit-scan over candidate masks), which keeps SIMT
// divergence between the blocks of a wavefront low.
// ---------------------------------------------------------------------------
struct Stripe {
    uint64_t sig[6], neg[6];  // rows k-1 .. k+4
    uint64_t vis[4], ref[4];  // rows k .. k+3
    uint64_t bit[4];          // encoder: magnitude bits of the plane; decoder: refinement bits out
};

GRK_HD uint64_t spp_candidates(const Stripe &s, uint32_t nr) {
    uint64_t c = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if ((uint32_t)r >= nr) break;
        uint64_t nb = dil(s.sig[r]) | dil(s.sig[r + 2]) | (s.sig[r + 1] << 1) | (s.sig[r + 1] >> 1);
        c |= nb & ~(s.sig[r + 1] | s.vis[r]);
    }
    return c;
}

struct LaneEncoder {
    static constexpr bool kDecoder = false;
    MqEncLane e;
    uint32_t *cxw;
    const uint32_t *tab;
    const uint64_t *planes, *pl;
    uint32_t *rate;
    uint32_t sty = 0;     // CBLKSTY_* mode switches
    uint32_t numbps = 0;
    bool raw = false;     // the current pass is coded raw (BYPASS)
    GRK_HD void begin_pass(int32_t bpno) { pl = planes + (uint32_t)bpno * 64; }
    GRK_HD uint64_t stripe_bits(uint32_t y, uint32_t h) const { return y < h ? pl[y] : 0; }
    GRK_HD uint32_t code(uint32_t cx, uint32_t v) { mqel_encode(e, cxw, tab, cx, v); return v; }
    GRK_HD void end_stripe(uint32_t, uint32_t, int, const Stripe &) {}
    // t1_encode_cblk's pass end (t1.cpp:1256-1298) and the next pass's start
    // (:1222-1233): a terminated pass is flushed -- ERTERM under PTERM, the
    // raw flush for a raw pass -- and the coder restarts (MQ) or re-enters
    // raw mode for the next pass; a pass that is not terminated gets the
    // rate_extra_bytes correction.  RESET re-initialises the contexts.
    GRK_HD void end_pass(uint32_t passno, int passtype, int32_t bpno) {
        const bool last = passtype == 2 && bpno == 0;
        int nt = passtype + 1;
        int32_t nb = bpno;
        if (nt == 3) { nt = 0; nb--; }
        const bool next_raw = t1_pass_raw(sty, nb, nt, numbps);
        const bool pterm = (sty & CBLKSTY_PTERM) != 0;
        if (t1_pass_term(sty, bpno, passtype, numbps)) {
            if (raw) mqel_bypass_flush(e, pterm);
            else if (pterm) mqel_erterm(e);
            else mqel_flush(e);
            rate[passno] = (uint32_t)e.bp;
            if (!last) {
                if (next_raw) mqel_bypass_init(e);
                else mqel_restart(e);
            }
        } else {
            rate[passno] = (uint32_t)e.bp + (raw ? mqel_bypass_extra(e, pterm) : 5u + (e.ct < 5 ? 1u : 0u));
        }
        if (sty & CBLKSTY_RESET) mq_reset_words(cxw, tab);
        raw = next_raw;
    }
};

// ===========================================================================
// Encoder, split form.  Because the encoder knows every magnitude up front,
// the significance state before bit-plane p is simply "magnitude >= 2^(p+1)"
// (the `above` rows), so each bit-plane's three passes can be modelled
// independently of the others and of the MQ coder:
//   t1_model_plane  one lane per (block, plane): bit-parallel row-mask
//                   modelling (64 columns per op), emits the plane's symbol
//                   stream (SPP, MRP, CUP) as bytes  ctx | decision << 5
//   t1_mq_block     one lane per block: MQ-codes the streams plane by plane,
//                   recording Grok's pass rates.
// ===========================================================================
GRK_HD uint32_t sym_stream_bytes(uint32_t w, uint32_t h) {
    // per plane: <= 1 ZC/MAG + 1 sign per sample, <= 2 extra (AGG/UNI) per
    // stripe column, 4 segmentation symbols (SEGSYM)
    return (w * h * 2 + ((h + 3) / 4) * w * 2 + 4 + 15) & ~15u;
}
GRK_HD uint32_t sym_slot_bytes(uint32_t w, uint32_t h) { return sym_stream_bytes(w, h); }

// A lane's symbol stream, 4 symbols per word.  On the GPU the 64 lanes of a
// wavefront write 64 different streams, and a word stored straight to HBM is
// a 4-byte piece of its own cache line, evicted before the line fills: the
// model kernel wrote 3.55 GB per 8K 9/7 frame for 0.76 GB of symbols
// (DESIGN.md 3).  So words go to a per-lane ring of 32 words in LDS (word j
// of lane l at ring[(j % 32) * 64], ring = lds + l: the 64 lanes hit 64
// banks; 8 KB per wavefront) and leave in whole 64-byte runs -- four 16-byte stores of one lane
// back to back -- at the stripe ends (stripe_flush, where the lanes of a
// wavefront meet), or early when a dense stripe fills the ring.  The host
// build stores words directly.
struct SymOut {
    uint32_t *out;
    uint32_t acc, n;
    uint32_t *ring = nullptr;  // device: this lane's ring (stride 64 words)
    uint32_t done = 0;         // device: words already written to out
    GRK_HD void store(uint32_t i, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
        ring[(i & 31) * 64] = v;
#else
        out[i] = v;
#endif
    }
#if defined(__HIP_DEVICE_COMPILE__)
    // words [done, done + 16) -> out, as four 16-byte stores
    __device__ void run16() {
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            u4 v;
            v.x = ring[((done + 4 * q) & 31) * 64];
            v.y = ring[((done + 4 * q + 1) & 31) * 64];
            v.z = ring[((done + 4 * q + 2) & 31) * 64];
            v.w = ring[((done + 4 * q + 3) & 31) * 64];
            *(u4 *)(out + done + 4 * q) = v;
        }
        done += 16;
    }
    __device__ void room() {  // a dense stripe: keep <= 26 words unwritten (a put adds <= 2)
        if ((n >> 2) - done >= 24) run16();
    }
#endif
    GRK_HD void put(uint32_t b) {
        acc |= b << ((n & 3) * 8);
        ++n;
        if ((n & 3) == 0) {
            store((n >> 2) - 1, acc);
            acc = 0;
#if defined(__HIP_DEVICE_COMPILE__)
            room();
#endif
        }
    }
    // cnt (<= 4) symbols at once, packed in `word` from its low byte up: at
    // most one store
    GRK_HD void put_n(uint32_t word, uint32_t cnt) {
        const uint32_t f = (n & 3) * 8;
        const uint64_t v = (uint64_t)acc | ((uint64_t)word << f);
        n += cnt;
        if (f + cnt * 8 >= 32) {
            store((n >> 2) - 1, (uint32_t)v);
            acc = (uint32_t)(v >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
            room();
#endif
        } else {
            acc = (uint32_t)v;
        }
    }
    // cnt (<= 8) symbols at once: at most two stores
    GRK_HD void put_n64(uint64_t word, uint32_t cnt) {
        const uint32_t f = (n & 3) * 8, tot = (n & 3) + cnt, i = n >> 2;
        const uint64_t lo = (uint64_t)acc | (word << f);
        const uint32_t hi = f ? (uint32_t)(word >> (64 - f)) : 0u;
        n += cnt;
        if (tot >= 4) store(i, (uint32_t)lo);
        if (tot >= 8) store(i + 1, (uint32_t)(lo >> 32));
        acc = tot >= 8 ? hi : tot >= 4 ? (uint32_t)(lo >> 32) : (uint32_t)lo;
#if defined(__HIP_DEVICE_COMPILE__)
        if (tot >= 4) room();
#endif
    }
    // the lanes of the wavefront write their complete 64-byte runs together
    GRK_HD void stripe_flush() {
#if defined(__HIP_DEVICE_COMPILE__)
        while ((n >> 2) - done >= 16) run16();
#endif
    }
    GRK_HD void flush() {
#if defined(__HIP_DEVICE_COMPILE__)
        stripe_flush();
        if (n & 3) ring[((n >> 2) & 31) * 64] = acc;
        for (uint32_t j = done; j < (n + 3) >> 2; ++j) out[j] = ring[(j & 31) * 64];
#else
        if (n & 3) out[n >> 2] = acc;
#endif
    }
};

// Bit-sliced zero-coding context (t1_generate_luts.cpp:63-140) for 64
// samples at once from the 8 neighbour significance masks (bit x = sample x).
struct Ctx4 { uint64_t c0, c1, c2, c3; };

GRK_HD Ctx4 zc_slices(uint64_t NW, uint64_t N, uint64_t NE, uint64_t W, uint64_t E, uint64_t SW, uint64_t S,
                      uint64_t SE, uint32_t orient) {
    uint64_t hA = orient == 1 ? N : W, hB = orient == 1 ? S : E;
    uint64_t vA = orient == 1 ? W : N, vB = orient == 1 ? E : S;
    const uint64_t h1 = hA ^ hB, h2 = hA & hB, hz = ~(hA | hB);
    const uint64_t v1 = vA ^ vB, v2 = vA & vB, vz = ~(vA | vB);
    const uint64_t a = NW ^ NE, b = NW & NE, c = SW ^ SE, e = SW & SE;
    const uint64_t s0 = a ^ c, cr = a & c;
    const uint64_t s1 = b ^ e ^ cr;
    const uint64_t s2 = (b & e) | ((b ^ e) & cr);
    const uint64_t dz = ~(NW | NE | SW | SE);
    const uint64_t d1 = s0 & ~s1 & ~s2;
    const uint64_t dge2 = ~dz & ~d1;
    const uint64_t dge3 = s2 | (s1 & s0);
    uint64_t x1, x2, x3, x4, x5, x6, x7, x8;
    if (orient != 3) {
        x8 = h2; x7 = h1 & ~vz; x6 = h1 & vz & ~dz; x5 = h1 & vz & dz;
        x4 = hz & v2; x3 = hz & v1; x2 = hz & vz & dge2; x1 = hz & vz & d1;
    } else {
        const uint64_t hv0 = hz & vz, hv1 = (h1 & vz) | (hz & v1), hv2 = ~hv0 & ~hv1;
        const uint64_t d2 = dge2 & ~dge3;
        x8 = dge3; x7 = d2 & ~hv0; x6 = d2 & hv0; x5 = d1 & hv2; x4 = d1 & hv1; x3 = d1 & hv0;
        x2 = dz & hv2; x1 = dz & hv1;
    }
    Ctx4 r;
    r.c0 = x1 | x3 | x5 | x7;
    r.c1 = x2 | x3 | x6 | x7;
    r.c2 = x4 | x5 | x6 | x7;
    r.c3 = x8;
    return r;
}

GRK_HD uint32_t ctx_at(const Ctx4 &c, uint32_t x) {
    return (uint32_t)((c.c0 >> x) & 1) | (uint32_t)((c.c1 >> x) & 1) << 1 | (uint32_t)((c.c2 >> x) & 1) << 2 |
           (uint32_t)((c.c3 >> x) & 1) << 3;
}

// sign symbol for sample x: W/E/N/S significance masks already aligned to x
GRK_HD uint32_t sc_symbol(const uint8_t *sc, uint64_t sW, uint64_t nW, uint64_t sE, uint64_t nE, uint64_t sN,
                          uint64_t nN, uint64_t sS, uint64_t nS, uint64_t neg, uint32_t x, bool raw = false) {
    uint32_t i = (uint32_t)((sW >> x) & 1) | (uint32_t)((nW >> x) & 1) << 1 | (uint32_t)((sE >> x) & 1) << 2 |
                 (uint32_t)((nE >> x) & 1) << 3 | (uint32_t)((sN >> x) & 1) << 4 | (uint32_t)((nN >> x) & 1) << 5 |
                 (uint32_t)((sS >> x) & 1) << 6 | (uint32_t)((nS >> x) & 1) << 7;
    uint32_t si = sc[i];
    // a raw (BYPASS) pass codes the sign itself, not its XOR with the prediction (t1.cpp:221-222)
    return (si & 0x7f) | ((((uint32_t)(neg >> x) & 1u) ^ (raw ? 0u : (si >> 7))) << 5);
}

// a: a row array (host: a pointer; device: the lane-interleaved rows of
// kernels.hip LRow)
template <class A>
GRK_HD uint64_t ldrow(const A &a, int32_t y, uint32_t h) {
    return (y >= 0 && (uint32_t)y < h) ? (uint64_t)a[y] : 0;
}

// Model bit-plane p of one block.  above = significance before plane p,
// ref = significance before plane p+1 (refined-before flags; has_ref false
// for the top plane), negr = sign rows (index y+1), tmp = 128 rows of scratch
// (post-SPP significance, then the SPP's visited rows).  Writes the plane's stream and
// cnt[0..2] = symbols of its SPP / MRP / CUP (SPP and MRP are empty for the
// top plane).  Semantics: t1.cpp:197-338 (SPP), 443-555 (MRP), 639-782 (CUP).
//
// Mode switches (cblksty): VSC -- the contexts of a stripe's last row never
// see the row below it (t1_update_flags_macro skips the north update from a
// stripe's first row, t1.cpp:168-190), i.e. row k+4 reads as insignificant
// for row k+3; SEGSYM -- the cleanup pass ends with the segmentation symbols
// 1 0 1 0 in the uniform context (mqc_segmark_enc, t1.cpp:1244-1245).
template <class R, class T, bool COND = true>
GRK_HD void t1_model_plane(uint32_t w, uint32_t h, uint32_t orient, const R &bitp, const R &above, const R &ref,
                           bool has_ref, const R &negr, const T &tmp, const uint8_t *sc, uint32_t *out, uint32_t *cnt,
                           uint32_t cblksty = 0, bool raw_spp = false, uint32_t *ring = nullptr) {
    const uint64_t wm = w >= 64 ? ~(uint64_t)0 : (((uint64_t)1 << w) - 1);
    const bool vsc = (cblksty & CBLKSTY_VSC) != 0;
    const T postS = tmp, visS = tmp + 64;
    SymOut so{out, 0, 0, ring, 0};
    // ---- significance propagation ----
    uint64_t U = 0;  // post-SPP significance of row k-1
    for (uint32_t k = 0; k < h; k += 4) {
        const uint32_t nr = h - k < 4 ? h - k : 4;
        // Rows are read only where the stripe needs them (the lanes that skip
        // a read fetch nothing): the plane's bits where a sample can become
        // significant -- a candidate, and a significant sample in or next to
        // the stripe to start the propagation -- and the sign rows where one
        // did.
        uint64_t pre[4], bit[4] = {0, 0, 0, 0}, C[4], post[4], ng[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            pre[r] = ldrow(above, (int32_t)(k + r), h);
            C[r] = (uint32_t)r < nr ? ~pre[r] & wm : 0;
            post[r] = pre[r];
        }
        const uint64_t D = vsc ? 0 : ldrow(above, (int32_t)(k + 4), h);
        if (!COND || ((C[0] | C[1] | C[2] | C[3]) && (pre[0] | pre[1] | pre[2] | pre[3] | U | D))) {
#pragma unroll
            for (int r = 0; r < 4; ++r) bit[r] = ldrow(bitp, (int32_t)(k + r), h);
        }
        // fixed point of the causal significance recurrence; the W->E chain
        // inside a row is resolved with one carry-propagating add
        for (int it = 0; it < 300; ++it) {
            uint64_t changed = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint64_t up = r == 0 ? U : post[r - 1], ne = r == 0 ? U : pre[r - 1];
                const uint64_t dnp = r == 3 ? D : post[r + 1], dn = r == 3 ? D : pre[r + 1];
                const uint64_t B = (up << 1) | up | (ne >> 1) | (pre[r] << 1) | (pre[r] >> 1) | (dnp << 1) | dn |
                                   (dn >> 1);
                const uint64_t P = C[r] & bit[r], sd = P & B;
                const uint64_t ns = (((P + sd) ^ P) | sd) & P;
                const uint64_t np = pre[r] | ns;
                changed |= np ^ post[r];
                post[r] = np;
            }
            if (!changed) break;
        }
        if (!COND || ((post[0] ^ pre[0]) | (post[1] ^ pre[1]) | (post[2] ^ pre[2]) | (post[3] ^ pre[3]))) {
#pragma unroll
            for (int i = 0; i < 6; ++i) ng[i] = negr[k + i];
            if (vsc) ng[5] = 0;
        }
        uint64_t coded[4];
        Ctx4 cz[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint64_t up = r == 0 ? U : post[r - 1], ne = r == 0 ? U : pre[r - 1];
            const uint64_t dnp = r == 3 ? D : post[r + 1], dn = r == 3 ? D : pre[r + 1];
            const uint64_t NW = up << 1, N = up, NE = ne >> 1, W = post[r] << 1, E = pre[r] >> 1, SW = dnp << 1,
                           S = dn, SE = dn >> 1;
            coded[r] = C[r] & (NW | N | NE | W | E | SW | S | SE);
            cz[r] = zc_slices(NW, N, NE, W, E, SW, S, SE, orient);
            if ((uint32_t)r < nr) { postS[k + r] = post[r]; visS[k + r] = coded[r]; }
        }
        uint64_t cols = coded[0] | coded[1] | coded[2] | coded[3];
        // a column's symbols (<= 4 ZC + 4 SC) go out as one packed word
        while (cols) {
            const uint32_t x = ctz64(cols);
            cols &= cols - 1;
            uint64_t word = 0;
            uint32_t sh = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (!((coded[r] >> x) & 1)) continue;
                const uint32_t s = (uint32_t)((post[r] >> x) & 1);
                word |= (uint64_t)(ctx_at(cz[r], x) | s << 5) << sh;
                sh += 8;
                if (s) {
                    const uint64_t up = r == 0 ? U : post[r - 1], dn = r == 3 ? D : pre[r + 1];
                    word |= (uint64_t)sc_symbol(sc, post[r] << 1, ng[r + 1] << 1, pre[r] >> 1, ng[r + 1] >> 1, up,
                                                ng[r], dn, ng[r + 2], ng[r + 1], x, raw_spp) << sh;
                    sh += 8;
                }
            }
            so.put_n64(word, sh >> 3);
        }
        U = post[3];
        so.stripe_flush();
    }
    cnt[0] = so.n;
    // ---- magnitude refinement: members = significant before this plane ----
    // The context offset of every member is fixed for the stripe (refined
    // before: 2, else a significant neighbour: 1), so it is formed as two
    // row masks up front and a column's symbols are packed into one word.
    for (uint32_t k = 0; k < h; k += 4) {
        uint64_t m[4], o0[4], o1[4], bit[4], sS[6];
#pragma unroll
        for (int r = 0; r < 4; ++r) m[r] = ldrow(above, (int32_t)(k + r), h);
        uint64_t cols = m[0] | m[1] | m[2] | m[3];
        if (COND && !cols) continue;  // no member: nothing else of the stripe is read
#pragma unroll
        for (int i = 0; i < 6; ++i) sS[i] = ldrow(postS, (int32_t)(k + i) - 1, h);
        if (vsc) sS[5] = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            o1[r] = has_ref ? ldrow(ref, (int32_t)(k + r), h) : 0;
            bit[r] = ldrow(bitp, (int32_t)(k + r), h);
            const uint64_t nb = dil(sS[r]) | dil(sS[r + 2]) | (sS[r + 1] << 1) | (sS[r + 1] >> 1);
            o0[r] = nb & ~o1[r];
        }
        while (cols) {
            const uint32_t x = ctz64(cols);
            cols &= cols - 1;
            uint32_t word = 0, sh = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t pr = (uint32_t)(m[r] >> x) & 1;
                const uint32_t sym = CX_MAG + ((uint32_t)(o0[r] >> x) & 1) + (((uint32_t)(o1[r] >> x) & 1) << 1) +
                                     (((uint32_t)(bit[r] >> x) & 1) << 5);
                word |= pr ? sym << sh : 0;
                sh += pr << 3;
            }
            so.put_n(word, sh >> 3);
        }
        so.stripe_flush();
    }
    cnt[1] = so.n - cnt[0];
    // ---- cleanup (+ run-length) ----
    U = 0;  // post-CUP significance of row k-1
    for (uint32_t k = 0; k < h; k += 4) {
        const uint32_t nr = h - k < 4 ? h - k : 4;
        uint64_t sS[4], cand[4], bit[4] = {0, 0, 0, 0}, pc[4], ng[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            sS[r] = ldrow(postS, (int32_t)(k + r), h);
            cand[r] = (uint32_t)r < nr ? ~(sS[r] | ldrow(visS, (int32_t)(k + r), h)) & wm : 0;
        }
        if (!COND || (cand[0] | cand[1] | cand[2] | cand[3])) {  // the bits of candidates, the signs of new significance
#pragma unroll
            for (int r = 0; r < 4; ++r) bit[r] = ldrow(bitp, (int32_t)(k + r), h);
            if (!COND || ((cand[0] & bit[0]) | (cand[1] & bit[1]) | (cand[2] & bit[2]) | (cand[3] & bit[3]))) {
#pragma unroll
                for (int i = 0; i < 6; ++i) ng[i] = negr[k + i];
                if (vsc) ng[5] = 0;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) pc[r] = sS[r] | (cand[r] & bit[r]);
        const uint64_t D = vsc ? 0 : ldrow(postS, (int32_t)(k + 4), h);
        uint64_t agg = 0;
        if (nr == 4) {
            agg = cand[0] & cand[1] & cand[2] & cand[3];
            agg &= ~((pc[0] | pc[1] | pc[2] | pc[3]) << 1);
            agg &= ~((sS[0] | sS[1] | sS[2] | sS[3]) >> 1);
            agg &= ~(dil(U) | dil(D));
        }
        Ctx4 cz[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint64_t up = r == 0 ? U : pc[r - 1], ne = r == 0 ? U : sS[r - 1];
            const uint64_t dnc = r == 3 ? D : pc[r + 1], dn = r == 3 ? D : sS[r + 1];
            cz[r] = zc_slices(up << 1, up, ne >> 1, pc[r] << 1, sS[r] >> 1, dnc << 1, dn, dn >> 1, orient);
        }
        uint64_t cols = cand[0] | cand[1] | cand[2] | cand[3];
        // a column's symbols go out as packed words: the aggregation / run
        // symbols (<= 3), then the rows' ZC / SC symbols (<= 8)
        while (cols) {
            const uint32_t x = ctz64(cols);
            cols &= cols - 1;
            int r0 = 0;
            bool rl = false;
            if ((agg >> x) & 1) {
                uint32_t colbits = (uint32_t)((bit[0] >> x) & 1) | (uint32_t)((bit[1] >> x) & 1) << 1 |
                                   (uint32_t)((bit[2] >> x) & 1) << 2 | (uint32_t)((bit[3] >> x) & 1) << 3;
                if (!colbits) {
                    so.put(CX_AGG);
                    continue;
                }
                const uint32_t run = (uint32_t)__builtin_ctz(colbits);
                so.put_n((CX_AGG | 1u << 5) | (CX_UNI | (run >> 1) << 5) << 8 | (CX_UNI | (run & 1) << 5) << 16, 3);
                r0 = (int)run;
                rl = true;
            }
            uint64_t word = 0;
            uint32_t sh = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (r < r0 || !((cand[r] >> x) & 1)) continue;
                const uint32_t s = (uint32_t)((bit[r] >> x) & 1);
                if (!(rl && r == r0)) {
                    word |= (uint64_t)(ctx_at(cz[r], x) | s << 5) << sh;
                    sh += 8;
                }
                if (s) {
                    const uint64_t up = r == 0 ? U : pc[r - 1], dn = r == 3 ? D : sS[r + 1];
                    word |= (uint64_t)sc_symbol(sc, pc[r] << 1, ng[r + 1] << 1, sS[r] >> 1, ng[r + 1] >> 1, up, ng[r],
                                                dn, ng[r + 2], ng[r + 1], x) << sh;
                    sh += 8;
                }
            }
            so.put_n64(word, sh >> 3);
        }
        U = pc[3];
        so.stripe_flush();
    }
    if (cblksty & CBLKSTY_SEGSYM) {
        so.put(CX_UNI | 1u << 5);
        so.put(CX_UNI);
        so.put(CX_UNI | 1u << 5);
        so.put(CX_UNI);
    }
    cnt[2] = so.n - cnt[0] - cnt[1];
    so.flush();
}

// MQ-code one block from its per-plane symbol streams (slot p at
// sym + p * slot_words); the bytes are those of mqc_enc.cpp's coder over the
// symbol order of t1.cpp:1182-1326 (tests/test_gpu_parity.py).  The loop is
// built for a lone lane: symbols are consumed in 16-byte chunks while the
// chunk two ahead is in flight (the only wait on it sits at the chunk end),
// the next symbol's context word is read from LDS before the current one is
// written back (same-context bypass), and the coding step is select-based.

// BYTEOUT without data-dependent branches (mqc_enc.cpp:168-199): the carry
// into a non-0xFF byte, then 7 or 8 bits out depending on whether the byte
// before is 0xFF.  Bit 27 of C is the carry into the previous byte unless
// that byte is 0xFF, where it is the top bit of the 8 going out; the 8-bit
// case drops it with the byte's mask (it lands in bit 8), the 7-bit case
// after a carry made the byte 0xFF clears it (mqc_enc.cpp:186), and the new
// C keeps only the sh bits below the byte either way.
GRK_HD void mqel_byteout_bf(MqEncLane &e) {
    const bool big0 = e.cur == 0xff;
    const uint32_t carry = big0 ? 0u : (e.c >> 27) & 1u;
    e.cur += carry;
    const bool big = e.cur == 0xff;
    const uint32_t cm = big0 ? e.c : e.c & 0x7ffffffu;
    const uint32_t sh = big ? 20u : 19u;
    const uint32_t byte = (cm >> sh) & 0xffu;
    e.c &= (1u << sh) - 1u;
    e.ct = 27u - sh;
    mqel_emit(e, byte);
}

// one MQ coding step with the context word already in hand; returns the
// context's new word (mqc_enc.cpp:50-110).  Select-based: the MPS/LPS and
// exchange cases share one instruction stream, the next-state table read is
// unconditional (its latency overlaps the renormalisation) and only a renorm
// that crosses a byte boundary branches.
GRK_HD uint32_t mqel_step(MqEncLane &e, const uint32_t *tab, uint32_t w, uint32_t d) {
    const uint32_t qe = w & 0xffff, mps = w >> 31;
    const uint32_t a = e.a - qe;
    const bool is_mps = d == mps;
    const bool addc = is_mps != (a < qe);
    e.c += addc ? qe : 0u;
    uint32_t na = addc ? a : qe;
    const bool keep = is_mps && (a & 0x8000);  // no renormalisation, no state change
    const uint32_t nidx = (w >> (is_mps ? 16 : 22)) & 63;
    const uint32_t nmps = mps ^ (is_mps ? 0u : (w >> 28) & 1u);
    const uint32_t tw = tab[nidx];
    uint32_t n = clz32(na) - 16;
    // renormalisation: shift to each byte boundary the n bits cross, BYTEOUT
    // there (the first one straight-line: the lanes that cross one are a few
    // of the 64 in any step, so the divergent block is kept short), then the
    // rest of the shift, shared by every lane
    if (n >= e.ct) {
        na <<= e.ct; e.c <<= e.ct; n -= e.ct;
        mqel_byteout_bf(e);
        while (n >= e.ct) {  // a second / third boundary (n <= 15): rare
            na <<= e.ct; e.c <<= e.ct; n -= e.ct;
            mqel_byteout_bf(e);
        }
    }
    na <<= n; e.c <<= n; e.ct -= n;
    e.a = na;
    return keep ? w : (tw | (nmps << 31));
}

template <bool LAZY = false>
GRK_HD uint32_t t1_mq_block(uint32_t numbps, const uint32_t *sym, uint32_t slot_words, const uint32_t *cnt,
                            const uint32_t *tab, uint32_t *cxw, uint32_t *out, uint32_t *rate, uint32_t *len_out,
                            uint32_t cblksty = 0) {
    *len_out = 0;
    if (numbps == 0) return 0;
    LaneEncoder cd;
    cd.sty = cblksty;
    cd.numbps = numbps;
    mq_reset_words(cxw, tab);
    cd.e.a = 0x8000; cd.e.c = 0; cd.e.ct = 12; cd.e.bp = -1; cd.e.cur = 0; cd.e.acc = 0; cd.e.out = out;
    cd.cxw = cxw; cd.tab = tab; cd.rate = rate;
    uint32_t passno = 0;
    for (int32_t p = (int32_t)numbps - 1; p >= 0; --p) {
        const uint32_t *c = cnt + p * 4;
        int t = (p == (int32_t)numbps - 1) ? 2 : 0;
        const uint32_t b0 = t == 2 ? 0 : c[0], b1 = t == 2 ? 0 : c[0] + c[1];
        const uint32_t total = b1 + c[2];
        uint32_t bnd = t == 0 ? b0 : t == 1 ? b1 : total;  // end of the current pass
        const uint4 *src = (const uint4 *)(sym + (size_t)p * slot_words);
        uint4 c0 = src[0], c1 = src[1];
        src += 2;
        uint32_t i = 0;
        while (t < 3 && i == bnd) {  // leading empty passes
            cd.end_pass(passno++, t, p);
            ++t;
            bnd = t == 1 ? b1 : total;
        }
        uint32_t w = cxw[c0.x & 31];
        uint4 c2 = *src++;
        // one symbol; the next symbol's context word is read before this one's
        // is written back (the LDS pipe keeps the order), bypassed if equal
#define GRK_MQ_SYMBOL()                                                   \
    {                                                                     \
        const uint32_t b = cur & 0xff;                                    \
        cur >>= 8;                                                        \
        ++i;                                                              \
        if (LAZY && cd.raw) {                                             \
            mqel_bypass(cd.e, b >> 5);                                    \
        } else {                                                          \
            const uint32_t wn = cxw[cur & 31];                            \
            const uint32_t nw = mqel_step(cd.e, tab, w, b >> 5);          \
            cxw[b & 31] = nw;                                             \
            w = (((cur ^ b) & 31) == 0) ? nw : wn;                        \
        }                                                                 \
        if (i == bnd) {                                                   \
            do {                                                          \
                cd.end_pass(passno++, t, p);                              \
                ++t;                                                      \
                bnd = t == 1 ? b1 : total;                                \
            } while (t < 3 && i == bnd);                                  \
            w = cxw[cur & 31]; /* RESET may have re-initialised it */     \
        }                                                                 \
    }
        while (total - i >= 16) {  // full chunks
#pragma unroll 1
            for (int q = 0; q < 4; ++q) {  // not unrolled: keeps the kernel's code small (I-cache)
                uint32_t cur = q == 0 ? c0.x : q == 1 ? c0.y : q == 2 ? c0.z : c0.w;
                const uint32_t nxt = q == 0 ? c0.y : q == 1 ? c0.z : q == 2 ? c0.w : c1.x;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k == 3) cur |= nxt << 8;  // read-ahead byte for the last symbol of the word
                    GRK_MQ_SYMBOL();
                }
            }
            c0 = c1; c1 = c2; c2 = *src++;
        }
        while (i < total) {  // tail: < 16 symbols, all in c0
            uint32_t cur = c0.x;
            for (int k = 0; k < 4 && i < total; ++k) {
                if (k == 3) cur |= c0.y << 8;
                GRK_MQ_SYMBOL();
            }
            c0.x = c0.y; c0.y = c0.z; c0.z = c0.w;
        }
#undef GRK_MQ_SYMBOL
    }
    const uint32_t total = passno;
    const uint32_t len = (uint32_t)cd.e.bp;
    mqel_finish(cd.e, len);
    uint32_t last = len;
    for (uint32_t i = total; i > 0;) {
        --i;
        uint32_t r = rate[i];
        if (r > last) r = last; else last = r;
        rate[i] = r;
    }
    const uint8_t *ob = (const uint8_t *)out;
    for (uint32_t i = 0; i < total; ++i)
        if (rate[i] > 0 && ob[rate[i] - 1] == 0xFF) rate[i]--;
    *len_out = len;
    return total;
}

// Which bit-planes a decode produced: sigafter rows are valid for planes
// [low, top], refinement rows for planes [qlow, top-1] (qlow = 32: none).
struct DecodedPlanes { int32_t top, low, qlow; };

GRK_HD DecodedPlanes decoded_planes(uint32_t numpasses, uint32_t numbps) {
    DecodedPlanes d{-1, 0, 32};
    if (numbps == 0 || numpasses == 0) return d;
    uint32_t maxp = 3 * numbps - 2;
    uint32_t last = (numpasses < maxp ? numpasses : maxp) - 1;
    int32_t plane; int type;
    pass_info(last, numbps, &plane, &type);
    d.top = (int32_t)numbps - 1;
    d.low = plane;
    if (last >= 2) {
        uint32_t im = last - (last - 2) % 3;  // last decoded refinement pass
        d.qlow = (int32_t)numbps - 2 - (int32_t)((im - 1) / 3);
    }
    return d;
}

// Grok's decoded value (t1->data incl. the extra half-LSB) of sample (x, y):
// significant at plane p (highest plane whose sigafter bit is set), refined at
// planes p-1..qlow:  M = (1 v_{p-1} .. v_ql)b << (ql+1) | 1 << ql, ql = min(p, qlow).
GRK_HD int32_t t1_rebuild(uint32_t x, uint32_t y, const DecodedPlanes &dp, const uint64_t *sigafter,
                          const uint64_t *refbit, uint64_t negrow) {
    int32_t p = -1;
    for (int32_t q = dp.top; q >= dp.low; --q)
        if ((sigafter[(uint32_t)q * 64 + y] >> x) & 1u) { p = q; break; }
    if (p < 0) return 0;
    uint32_t bits = 1;
    int32_t ql = p;
    for (int32_t q = p - 1; q >= dp.qlow; --q) {
        bits = (bits << 1) | (uint32_t)((refbit[(uint32_t)q * 64 + y] >> x) & 1u);
        ql = q;
    }
    int32_t m = (int32_t)((bits << (ql + 1)) | (1u << ql));
    return ((negrow >> x) & 1u) ? -m : m;
}

// Deepest block the decoder accepts: t1_decode_cblk refuses roishift + numbps
// >= 31 (t1.cpp:1055-1060); blocks deeper than this are left zero on the
// device and rejected by the host (ECORRUPT) before the launch.
constexpr uint32_t T1_MAX_DEC_BPS = 30;

// Per-block HBM scratch: state rows + two 32-plane x 64-row bit-plane sets
// (encoder: pa = magnitude bit-planes; decoder: pa = sigafter, pb = refbit).
struct T1Scratch {
    BlockState st;
    uint64_t pa[32 * 64];
    uint64_t pb[32 * 64];
    uint32_t cnt[32 * 4];  // encoder: symbols per (plane, pass type)
};

// ---- lane-interleaved scratch (encoder) ----
// The encoder's modelling kernel runs one lane per (block, bit-plane) with the
// 64 lanes of a wavefront at the same depth (numbps - 1 - plane) of the 64
// blocks of a group, so its rows are kept like the decoder's: the 64 blocks of
// a group share a region in which row R of block l is word R * 64 + l, and the
// bit-plane rows are indexed by depth, so every row access of a wavefront is
// one 512-byte run.  Per block: the sign rows (66), then per depth 256 rows:
// the plane's magnitude bits, the significance before it, and the modelling
// kernel's post-SPP significance and SPP-visited rows.  The symbol counts per
// (plane, pass) sit ahead of the groups, 128 words per block.
constexpr uint32_t T1E_NEG = 0, T1E_PL = 66, T1E_DEPTH_ROWS = 256;
constexpr uint32_t T1E_BITS = 0, T1E_ABOVE = 64, T1E_POST = 128, T1E_VIS = 192;  // inside a depth
GRK_HD constexpr uint32_t t1e_rec_rows(uint32_t maxdepth) { return T1E_PL + maxdepth * T1E_DEPTH_ROWS; }
GRK_HD constexpr uint32_t t1e_depth_row(uint32_t d) { return T1E_PL + d * T1E_DEPTH_ROWS; }
// bytes of the encoder scratch for n blocks of at most maxdepth planes
GRK_HD constexpr uint64_t t1e_scratch_bytes(uint32_t n, uint32_t maxdepth) {
    return (uint64_t)((n + 63) & ~63u) * (128 * 4 + (uint64_t)t1e_rec_rows(maxdepth) * 8);
}
struct EncScratch {
    uint32_t *cnt;    // 128 words per block
    uint64_t *rows;   // the groups
    uint32_t rec_rows;
    GRK_HD uint64_t *group(uint32_t g) const { return rows + (uint64_t)g * 64 * rec_rows; }
};
GRK_HD EncScratch enc_scratch(void *base, uint32_t n, uint32_t maxdepth) {
    const uint32_t n64 = (n + 63) & ~63u;
    return EncScratch{(uint32_t *)base, (uint64_t *)((uint8_t *)base + (uint64_t)n64 * 128 * 4), t1e_rec_rows(maxdepth)};
}

// ---- lane-interleaved scratch (decoder) ----
// The 64 blocks of a decoder wavefront (a "group") share one region of
// 64 * sizeof(T1Scratch) bytes in which row R of the T1Scratch fields of
// lane l lives at word R * 64 + l.  A row access of the wavefront is then one
// 512-byte contiguous run (4 cache lines) instead of 64 lines 35 KB apart,
// and the rows a lane writes fill whole lines together with its neighbours'.
// The last group also spans 64 records: scratch holds the block count
// rounded up to a multiple of 64 (t1_scratch_records).
// row offsets of the T1Scratch fields (in 8-byte rows)
constexpr uint32_t T1R_SIG = 0, T1R_NEG = 66, T1R_VIS = 132, T1R_REF = 198, T1R_PA = 264, T1R_PB = 264 + 2048;
GRK_HD uint64_t *t1_group_base(void *scr, uint32_t g, size_t rec_bytes) {
    return (uint64_t *)((uint8_t *)scr + (size_t)g * 64 * rec_bytes);
}
GRK_HD constexpr uint32_t t1_scratch_records(uint32_t n) { return (n + 63) & ~63u; }

// Serial restatement of the encoder prep kernel (quantise, sign rows,
// numbps, magnitude bit-planes): T1Part1::preEncode (T1Part1.cpp:58-94).
GRK_HD uint32_t t1_prep_serial(const int32_t *coef, uint32_t stride, uint32_t w, uint32_t h, int32_t qmfbid,
                               int32_t inv_step, BlockState &st, uint64_t *planes) {
    uint32_t maxv = 0;
    for (uint32_t y = 0; y < 66; ++y) st.neg[y] = 0;
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            uint32_t ng;
            uint32_t m = quant_mag(coef[(size_t)y * stride + x], qmfbid, inv_step, &ng);
            if (ng) st.neg[y + 1] |= (uint64_t)1 << x;
            maxv |= m;
        }
    uint32_t numbps = 0;
    if (maxv) {
        uint32_t t = 32u - (uint32_t)__builtin_clz(maxv);
        numbps = t <= 6 ? 0 : t - 6;
    }
    for (uint32_t p = 0; p < numbps; ++p)
        for (uint32_t y = 0; y < h; ++y) {
            uint64_t row = 0;
            for (uint32_t x = 0; x < w; ++x) {
                uint32_t ng;
                uint32_t m = quant_mag(coef[(size_t)y * stride + x], qmfbid, inv_step, &ng);
                row |= (uint64_t)((m >> (p + 6)) & 1u) << x;
            }
            planes[p * 64 + y] = row;
        }
    return numbps;
}

// above[p*64+y] = OR of magnitude planes q > p (significance before plane p)
GRK_HD void t1_prep_above(uint32_t h, uint32_t numbps, const uint64_t *planes, uint64_t *above) {
    for (uint32_t y = 0; y < h; ++y) {
        uint64_t acc = 0;
        for (int32_t p = (int32_t)numbps - 1; p >= 0; --p) {
            above[(uint32_t)p * 64 + y] = acc;
            acc |= planes[(uint32_t)p * 64 + y];
        }
    }
}

}  // namespace grkgpu
