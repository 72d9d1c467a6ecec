// t1_flat.h -- EBCOT Tier-1 decoder, v4 ("flat"): one lane per code-block,
// ONE MQ decision per loop iteration.
//
// Why: with nested pass / stripe / column loops (v3), the lanes of a
// wavefront re-converge at every loop exit, so a wavefront pays, for every
// (pass, stripe), the slowest of its blocks.  Here the whole decoder is a
// single loop whose body (1) forms the context of the pending decision,
// (2) runs the MQ decoder, (3) applies the decision and (4) moves the
// cursor to the next decision.  Lanes advance independently; a lane only
// leaves the common path for a stripe switch (row-mask load/store), a chunk
// refill of its bit stream, or the end of its block.
//
//   * The MQ byte stuffing is removed beforehand (t1_unstuff, one pass per
//     block): the decoder reads a plain bit stream, so renormalisation is
//     C = C << n | next n bits, with no per-byte branches.  Equivalence with
//     the ct / BYTEIN formulation of mqc_dec_inl.h: the comparisons only use
//     C[31:16], subtractions never borrow into it, and BYTEIN always supplies
//     a bit before it is shifted into C[31:16]; after a 0xFF byte the next
//     byte contributes its low 7 bits (its top bit is the stuffed 0), and a
//     0xFF followed by a byte > 0x8F (a marker), or the end of the segment
//     (Grok pads with 0xFF 0xFF), turns the stream into 1-bits forever.
//   * Block state = 64-bit row masks (t1_lane.h BlockState) in HBM; the
//     current 4-row stripe lives in registers.  Stripes that cannot hold
//     work for a significance / refinement pass are skipped using a 16-bit
//     "stripe has a significant sample" mask, so the significance-after-plane
//     rows (sa) are zero-filled up front and written only for visited
//     stripes.
//
// Semantics: Grok v5.1.0 t1/t1_part1/t1.cpp t1_decode_cblk (:1038),
// dec_sigpass / dec_refpass / dec_clnpass, mqc_dec_inl.h; cblksty 0.
// Outputs are those of v3 (t1_dec.h): sa / rb bit-plane rows + st.neg,
// consumed by k_t1_rebuild.
#pragma once
#include "t1_dec.h"

namespace grkgpu {

// ---------------------------------------------------------------------------
// Byte-stuffing removal.  Output: MSB-first bit stream packed in 32-bit
// words, ending with 1-bits (at least one all-ones word), plus "carry
// events".  A byte b in 0x80..0x8F after a 0xFF (it occurs: Grok's encoder
// propagates carries into stuffed bytes) contributes its low 7 bits AND adds
// its top bit at the position of the 0xFF's last bit -- an arithmetic carry
// into the code register that BYTEIN applies at the moment that bit sits at
// C[16].  The event is recorded as q = (stream index of that bit) + 17 (the
// decoder's consumed-bit count at that moment, see t1_decode_flat).
// Returns the word count; *ncarry = events written to carries[].
// ---------------------------------------------------------------------------
struct Unstuff {
    uint64_t acc = 0;
    uint32_t nacc = 0, emitted = 0;
    bool prevff = false, stop = false;
    // feed one byte; returns true if a word is ready in *out; *carry = event or ~0
    GRK_HD bool push(uint32_t b, uint32_t *out, uint32_t *carry) {
        *carry = 0xffffffffu;
        if (stop) return false;
        if (prevff && b > 0x8f) { stop = true; return false; }  // marker: 1-bits from here
        if (prevff && (b & 0x80u)) *carry = emitted - 1 + 17;
        const uint32_t nb = prevff ? 7u : 8u;
        acc = (acc << nb) | (b & (prevff ? 0x7fu : 0xffu));
        nacc += nb;
        emitted += nb;
        prevff = b == 0xff;
        if (nacc >= 32) {
            *out = (uint32_t)(acc >> (nacc - 32));
            nacc -= 32;
            return true;
        }
        return false;
    }
    // tail: fill the pending bits with 1s
    GRK_HD uint32_t tail() const {
        const uint32_t fill = 32 - nacc;
        return nacc ? (uint32_t)(((acc << fill) | ((1ull << fill) - 1)) & 0xffffffffu) : 0xffffffffu;
    }
};

// capacity (32-bit words) of the word and carry areas for a segment of len bytes
// (data words + the 1-bit tail + two all-ones chunks, rounded to chunks)
GRK_HD uint32_t unstuff_word_cap(uint32_t len) { return ((len * 8) / 32 + 1 + 1 + 8 + 3) & ~3u; }
GRK_HD uint32_t unstuff_carry_cap(uint32_t len) { return (len / 2 + 4 + 3) & ~3u; }

GRK_HD uint32_t t1_unstuff(const uint8_t *data, uint32_t len, uint32_t *words, uint32_t *carries,
                           uint32_t *ncarry) {
    Unstuff u;
    uint32_t nw = 0, nc = 0, wv, cv;
    for (uint32_t i = 0; i < len; ++i) {
        if (u.push(data[i], &wv, &cv)) words[nw++] = wv;
        if (cv != 0xffffffffu) carries[nc++] = cv;
    }
    words[nw++] = u.tail();
    do { words[nw++] = 0xffffffffu; } while (nw & 3);
    for (int i = 0; i < 8; ++i) words[nw++] = 0xffffffffu;
    carries[nc] = 0xffffffffu;  // sentinel
    *ncarry = nc;
    return nw;
}

// ---------------------------------------------------------------------------
// Bit reader over the unstuffed words: 64-bit MSB-aligned window W holding
// NB >= 32 valid bits after every refill; 4-word chunks (uint4) are fetched
// when the current one is used up (no prefetch register: the decoder's VGPR
// budget sets its occupancy).  Past the end it returns 1-bits.
// ---------------------------------------------------------------------------
struct FlatBits {
    uint64_t W;
    uint32_t NB;
    uint4 cur;
    uint32_t wi;            // next word of `cur` (0..3)
    uint32_t chunk;         // index of the chunk held in `cur`
    uint32_t nchunks;
    const uint4 *base;
};

// the stream ends with two all-ones chunks, so reads past the end clamp to
// the last chunk (no branch around the load, no select on its result)
GRK_HD uint4 fb_load(const FlatBits &b, uint32_t ci) { return b.base[ci < b.nchunks ? ci : b.nchunks - 1]; }

GRK_HD uint32_t fb_word(FlatBits &b) {
    const uint32_t v = b.wi == 0 ? b.cur.x : b.wi == 1 ? b.cur.y : b.wi == 2 ? b.cur.z : b.cur.w;
    if (++b.wi == 4) {
        b.wi = 0;
        b.cur = fb_load(b, ++b.chunk);  // no chunk prefetch: 4 VGPRs fewer (decoder occupancy)
    }
    return v;
}

// ---------------------------------------------------------------------------
// MQ decoder over the unstuffed stream (used by the nested-loop decoder v5
// in t1_dec.h and by t1_decode_flat): branch-free renormalisation.
// ---------------------------------------------------------------------------
// LAZY: the decoder may meet raw (BYPASS) segments; compiled out otherwise,
// so the common case keeps its per-symbol path branch-free.
template <bool LAZY>
struct BitDecT {
    static constexpr bool kLazy = LAZY;
    FlatBits bits;
    uint32_t A, C, consumed, cq;
    const uint32_t *cp;
    bool raw;  // the current segment is raw (BYPASS): bits straight from the stream
    // raw segment (mqc_raw_init_dec / mqc_raw_decode, mqc_dec.cpp:195-200,
    // mqc_dec_inl.h:90-112): the unstuffed stream IS the raw bit sequence --
    // 7 bits from the byte after a 0xFF, 1-bits from a marker on
    GRK_HD void init_raw(const uint32_t *words, uint32_t nwords) {
        bits.base = (const uint4 *)words;
        bits.nchunks = (nwords + 3) >> 2;
        bits.cur = fb_load(bits, 0);
        bits.chunk = 0;
        bits.wi = 0;
        const uint64_t w0 = fb_word(bits), w1 = fb_word(bits);
        bits.W = (w0 << 32) | w1;
        bits.NB = 64;
        raw = true;
    }
    GRK_HD uint32_t rawbit() {
        const uint32_t b = (uint32_t)(bits.W >> 63);
        bits.W <<= 1;
        if (--bits.NB < 32) {
            bits.W |= (uint64_t)fb_word(bits) << (32 - bits.NB);
            bits.NB += 32;
        }
        return b;
    }
    GRK_HD void init(const uint32_t *words, uint32_t nwords, const uint32_t *carries) {
        raw = false;
        bits.base = (const uint4 *)words;
        bits.nchunks = (nwords + 3) >> 2;
        bits.cur = fb_load(bits, 0);
        bits.chunk = 0;
        bits.wi = 0;
        const uint64_t w0 = fb_word(bits), w1 = fb_word(bits);
        const uint64_t v = (w0 << 32) | w1;
        C = (uint32_t)(v >> 33);  // first 31 stream bits (INITDEC: consumed 24, then 7 shifts)
        bits.W = v << 31;
        bits.NB = 33;
        A = 0x8000;
        consumed = 31;
        cq = carries[0];
        cp = carries + 1;
        if (cq < 31) { C += 1u << (16 + 31 - cq); cq = *cp++; }
    }
    GRK_HD uint32_t decode(uint32_t *cxw, const uint32_t *tab, uint32_t cx) {
        if constexpr (LAZY) {
            if (raw) return rawbit();
        }
        const uint32_t wd = cxw[cx];
        const uint32_t qe = wd & 0xffffu, mps = wd >> 31;
        uint32_t a = A - qe;
        const bool lo = (C >> 16) < qe;
        const bool lps = lo ? (a >= qe) : (a < qe);
        const bool keep = !lo && (a & 0x8000u);
        C = lo ? C : C - (qe << 16);
        a = lo ? qe : a;
        const uint32_t nidx = (wd >> (lps ? 22 : 16)) & 63u;
        const uint32_t nmps = mps ^ (lps ? (wd >> 28) & 1u : 0u);
        const uint32_t tw = tab[nidx];
        const uint32_t n = clz32(a) - 16;
        C = (C << n) | (uint32_t)((bits.W >> 1) >> (63 - n));
        bits.W <<= n;
        bits.NB -= n;
        A = a << n;
        const uint32_t c1 = consumed + n;
        if (cq < c1) { C += 1u << (16 + c1 - cq); cq = *cp++; }  // carry event (see Unstuff)
        consumed = c1;
        if (bits.NB < 32) {
            bits.W |= (uint64_t)fb_word(bits) << (32 - bits.NB);
            bits.NB += 32;
        }
        cxw[cx] = keep ? wd : (tw | (nmps << 31));  // unconditional LDS write: no branch
#ifdef T1_TRACE
        T1_TRACE(cx, mps ^ (uint32_t)lps, A, C >> 16);
#endif
        return mps ^ (uint32_t)lps;
    }
};
using BitDec = BitDecT<false>;

// One codeword segment of a code-block (grk_tcd_seg): its bytes in the data
// buffer, its passes, and where its unstuffed stream lives (16-byte units).
struct DecSeg {
    uint64_t data_off;
    uint32_t len, npasses, ub_off, pad;
};

// Segment cursor for t1_decode_passes: BitDec moves to segment j+1's stream
// at that segment's first pass (t1_decode_cblk's mqc_init_dec per segment,
// t1.cpp:1066-1081; contexts carry over unless RESET).
struct SegCursor {
    const DecSeg *seg;
    const uint32_t *ubuf;
    uint32_t nseg, cur, next;
    // raw: the segment starting here is a BYPASS (raw) one (t1.cpp:1070-1080)
    template <class D> GRK_HD void at_pass(D &d, uint32_t passno, bool raw) {
        if (passno != next || cur + 1 >= nseg) return;
        ++cur;
        const uint32_t *region = ubuf + (size_t)seg[cur].ub_off * 4;
        if (raw) d.init_raw(region + 4, region[0]);
        else d.init(region + 4, region[0], region + 4 + unstuff_word_cap(seg[cur].len));
        next += seg[cur].npasses;
    }
};

// v5: the nested pass / stripe / column walk of v3 (lanes of a wavefront stay
// converged on the pass structure) fed by the unstuffed bit stream.
template <class ST = BlockState, class RP = uint64_t *>
GRK_HD void t1_decode_v5(const uint32_t *words, uint32_t nwords, const uint32_t *carries, uint32_t numpasses,
                         uint32_t numbps, uint32_t w, uint32_t h, ST &st, const DecTables &T, uint32_t *cxw,
                         RP sa, RP rb) {
    for (uint32_t y = 0; y < h + 2; ++y) { st.sig[y] = 0; st.neg[y] = 0; st.vis[y] = 0; st.ref[y] = 0; }
    mq_reset_words(cxw, T.mq);
    BitDec d;
    d.init(words, nwords, carries);
    t1_decode_passes(d, numpasses, numbps, w, h, st, T, cxw, sa, rb);
}

// ---------------------------------------------------------------------------
// the flat decoder
// ---------------------------------------------------------------------------
enum FlatKind : uint32_t { FK_ZC = 0, FK_SC = 1, FK_MAG = 2, FK_AGG = 3, FK_UNI1 = 4, FK_UNI2 = 5 };

struct FlatStripe {
    uint64_t s[6], n[6];  // sig / neg rows k-1 .. k+4
    uint64_t v[4], f[4];  // vis / ref rows k .. k+3
    uint64_t b[4];        // refinement bits out (MRP)
};

// words / carries: t1_unstuff output (words 16-byte aligned; carries end
// with a ~0 sentinel).
GRK_HD void t1_decode_flat(const uint32_t *words, uint32_t nwords, const uint32_t *carries, uint32_t numpasses,
                           uint32_t numbps, uint32_t w, uint32_t h, BlockState &st, const DecTables &T, uint32_t *cxw,
                           uint64_t *sa, uint64_t *rb) {
    if (numpasses == 0 || numbps == 0) return;
    const uint32_t maxp = 3 * numbps - 2;
    if (numpasses > maxp) numpasses = maxp;
    for (uint32_t y = 0; y < 66; ++y) { st.sig[y] = 0; st.neg[y] = 0; st.vis[y] = 0; st.ref[y] = 0; }
    // significance-after-plane rows of skipped stripes stay zero
    {
        int32_t lowp; int ty;
        pass_info(numpasses - 1, numbps, &lowp, &ty);
        for (int32_t p = lowp; p < (int32_t)numbps; ++p)
            for (uint32_t y = 0; y < h; ++y) sa[(uint32_t)p * 64 + y] = 0;
    }
    mq_reset_words(cxw, T.mq);
    const uint64_t wmask = w >= 64 ? ~(uint64_t)0 : (((uint64_t)1 << w) - 1);
    const uint32_t nstripes = (h + 3) >> 2;

    BitDec md;
    md.init(words, nwords, carries);

    // pass / stripe / column cursor
    uint32_t ptype = 2;                 // first pass: cleanup of the top plane
    int32_t bpno = (int32_t)numbps - 1;
    uint32_t passno = 0;
    uint32_t sigstr = 0;                // stripes holding a significant sample
    uint32_t k = 0, nr = 0, si = 0;     // stripe start row, rows, stripe index
    FlatStripe S;
    uint64_t cand = 0;                  // columns of this stripe still to visit
    uint32_t x = 0, r = 0, kind = FK_ZC, todo = 0, rows = 0;
    uint32_t P = 0, Q = 0, sig4 = 0, vis4 = 0, ref4 = 0;
    bool grew = false;                  // SPP: a sample became significant in this column
    bool need_stripe = true;            // enter the first stripe of the pass
    si = 0;

    for (;;) {
        // ---------------- stripe / pass switch (rare path) ----------------
        if (need_stripe) {
            bool found = false;
            while (!found) {
                // find the next stripe of this pass that can hold work
                uint32_t pot;
                if (ptype == 2) pot = 0xffffu;
                else if (ptype == 0) pot = sigstr | (sigstr << 1) | (sigstr >> 1);
                else pot = sigstr;
                pot &= ((1u << nstripes) - 1) & ~((1u << si) - 1);
                if (!pot) {
                    // next pass
                    if (++passno >= numpasses) return;
                    if (++ptype == 3) { ptype = 0; --bpno; }
                    si = 0;
                    continue;
                }
                si = (uint32_t)__builtin_ctz(pot);
                k = si << 2;
                nr = h - k < 4 ? h - k : 4;
#pragma unroll
                for (int i = 0; i < 6; ++i) { S.s[i] = st.sig[k + i]; S.n[i] = st.neg[k + i]; }
#pragma unroll
                for (int i = 0; i < 4; ++i) { S.v[i] = st.vis[k + 1 + i]; S.f[i] = st.ref[k + 1 + i]; S.b[i] = 0; }
                Stripe tmp;
#pragma unroll
                for (int i = 0; i < 6; ++i) tmp.sig[i] = S.s[i];
#pragma unroll
                for (int i = 0; i < 4; ++i) tmp.vis[i] = S.v[i];
                if (ptype == 0) {
                    cand = spp_candidates(tmp, nr) & wmask;
                } else if (ptype == 1) {
                    cand = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if ((uint32_t)i < nr) cand |= S.s[i + 1] & ~S.v[i];
                    cand &= wmask;
                } else {
                    cand = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if ((uint32_t)i < nr) cand |= ~(S.s[i + 1] | S.v[i]);
                    cand &= wmask;
                }
                if (cand) { found = true; break; }
                // nothing to decode here: finish the stripe as the pass would
                if (ptype == 2) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) st.vis[k + 1 + i] = 0;
                }
                if (ptype != 1) {
                    uint64_t *sap = sa + (uint32_t)bpno * 64;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if ((uint32_t)i < nr) sap[k + i] = S.s[i + 1];
                } else {
                    uint64_t *rbp = rb + (uint32_t)bpno * 64;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if ((uint32_t)i < nr) rbp[k + i] = 0;
                }
                ++si;
            }
            need_stripe = false;
            // enter the first column
            x = ctz64(cand);
            goto column_entry;
        }

        {
            // ---------------- one decision ----------------
            const uint32_t nb9 = (P >> (3 * r)) & 0x1FFu;
            uint32_t cx;
            const uint32_t scw = T.sc[((nb9 & 0xAAu) >> 1) | ((Q >> (3 * r)) & 0xAAu)];
            if (kind == FK_ZC) cx = T.zc[nb9];
            else if (kind == FK_SC) cx = scw & 0x7fu;
            else if (kind == FK_MAG) cx = ((ref4 >> r) & 1u) ? CX_MAG + 2 : CX_MAG + ((nb9 & 0x1EFu) ? 1u : 0u);
            else cx = kind == FK_AGG ? (uint32_t)CX_AGG : (uint32_t)CX_UNI;

            const uint32_t d = md.decode(cxw, T.mq, cx);

            // ---------------- apply ----------------
            bool advance = true;
            if (kind == FK_ZC) {
                if (ptype == 0) S.v[r] |= (uint64_t)1 << x;
                if (d) { kind = FK_SC; advance = false; }
            } else if (kind == FK_SC) {
                const uint32_t sg = d ^ (scw >> 7);
                P |= 1u << (3 * r + 4);
                Q |= sg << (3 * r + 4);
                sig4 |= 1u << r;
                S.s[r + 1] |= (uint64_t)1 << x;
                S.n[r + 1] |= (uint64_t)sg << x;
                if (ptype == 0) {
                    grew = true;
                    vis4 |= 1u << r;
                    todo |= rows & ~(sig4 | vis4) & (2u << r);  // the sample below gains a neighbour
                }
                kind = FK_ZC;
            } else if (kind == FK_MAG) {
                S.f[r] |= (uint64_t)1 << x;
                S.b[r] |= (uint64_t)d << x;
            } else if (kind == FK_AGG) {
                if (d) { kind = FK_UNI1; advance = false; }
                else todo = 0;  // four zeros: column done
            } else if (kind == FK_UNI1) {
                r = d << 1;
                kind = FK_UNI2;
                advance = false;
            } else {
                r |= d;
                todo = rows & ~((2u << r) - 1);  // rows after the run are plain ZC
                kind = FK_SC;
                advance = false;
            }
            if (!advance) continue;
            todo &= ~((2u << r) - 1);
            if (todo) {
                r = (uint32_t)__builtin_ctz(todo);
                kind = ptype == 1 ? FK_MAG : FK_ZC;
                continue;
            }
            // ---------------- next column ----------------
            const uint64_t done = (x >= 63) ? ~(uint64_t)0 : (((uint64_t)2 << x) - 1);
            cand &= ~done;
            if (ptype == 0 && grew) {
                Stripe tmp;
#pragma unroll
                for (int i = 0; i < 6; ++i) tmp.sig[i] = S.s[i];
#pragma unroll
                for (int i = 0; i < 4; ++i) tmp.vis[i] = S.v[i];
                cand = spp_candidates(tmp, nr) & wmask & ~done;
            }
            if (!cand) {
                // ---------------- stripe end: write back ----------------
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    st.sig[k + 1 + i] = S.s[i + 1];
                    st.neg[k + 1 + i] = S.n[i + 1];
                    st.vis[k + 1 + i] = ptype == 2 ? 0 : S.v[i];
                    st.ref[k + 1 + i] = S.f[i];
                }
                if (ptype != 1) {
                    uint64_t *sap = sa + (uint32_t)bpno * 64;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if ((uint32_t)i < nr) sap[k + i] = S.s[i + 1];
                } else {
                    uint64_t *rbp = rb + (uint32_t)bpno * 64;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if ((uint32_t)i < nr) rbp[k + i] = S.b[i];
                }
                if (S.s[1] | S.s[2] | S.s[3] | S.s[4]) sigstr |= 1u << si;
                ++si;
                need_stripe = true;
                continue;
            }
            x = ctz64(cand);
        }
    column_entry:
        // ---------------- column entry ----------------
        {
            uint32_t pp = 0, qq = 0;
            const uint32_t s1 = x ? x - 1 : 0, m = x ? 7u : 3u, s2 = x ? 0u : 1u;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                pp |= ((((uint32_t)(S.s[i] >> s1)) & m) << s2) << (3 * i);
                qq |= ((((uint32_t)(S.n[i] >> s1)) & m) << s2) << (3 * i);
            }
            P = pp;
            Q = qq;
        }
        vis4 = 0;
        ref4 = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            vis4 |= (uint32_t)((S.v[i] >> x) & 1u) << i;
            ref4 |= (uint32_t)((S.f[i] >> x) & 1u) << i;
        }
        sig4 = win_self4(P);
        rows = (1u << nr) - 1;
        grew = false;
        if (ptype == 0) {
            uint32_t nz = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) nz |= (((P >> (3 * i)) & 0x1EFu) != 0 ? 1u : 0u) << i;
            todo = nz & ~sig4 & ~vis4 & rows;
            kind = FK_ZC;
        } else if (ptype == 1) {
            todo = sig4 & ~vis4 & rows;
            kind = FK_MAG;
        } else {
            todo = ~sig4 & ~vis4 & rows;
            kind = (nr == 4 && P == 0 && vis4 == 0) ? (uint32_t)FK_AGG : (uint32_t)FK_ZC;
        }
        r = kind == FK_AGG ? 0u : (uint32_t)__builtin_ctz(todo | 16u);
    }
}

}  // namespace grkgpu
