// t1_flat.h -- the T1 decoder's input side: byte-stuffing removal (the
// k_t1_unstuff pre-pass) and the MQ / raw bit decoder over the unstuffed
// stream (BitDecT), driven by t1_dec.h's pass walk (t1_decode_v5 /
// t1_decode_passes).
//
//   * The MQ byte stuffing is removed beforehand (one pass per block): the
//     decoder reads a plain bit stream, so renormalisation is
//     C = C << n | next n bits, with no per-byte branches.  Equivalence with
//     the ct / BYTEIN formulation of mqc_dec_inl.h: the comparisons only use
//     C[31:16], subtractions never borrow into it, and BYTEIN always supplies
//     a bit before it is shifted into C[31:16]; after a 0xFF byte the next
//     byte contributes its low 7 bits (its top bit is the stuffed 0), and a
//     0xFF followed by a byte > 0x8F (a marker), or the end of the segment
//     (Grok pads with 0xFF 0xFF), turns the stream into 1-bits forever.
//
// Semantics: Grok v5.1.0 t1/t1_part1/mqc_dec_inl.h (decode_macro :148,
// bytein), mqc_dec.cpp:178-193 (mqc_init_dec), t1.cpp:1038 t1_decode_cblk.
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
// decoder's consumed-bit count at that moment, see BitDecT).
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
// Bit reader over the unstuffed words: a two-word window (w0, w1) fed one
// word at a time from a per-lane ring of FB_RING words (LDS on the device:
// the 64 lanes' words of one slot sit in 64 different banks, slot stride
// 1 << rsh words).  The ring is topped up from the stream in HBM at the start
// of every stripe (fill: one or two 16-byte chunks, loaded together with the
// stripe's state rows, whose wait the decoder pays anyway); inside the stripe
// the next word comes from the ring, and only a ring that runs dry (a stripe
// coding more than ~300 bits) reaches HBM.  Fetching the stream straight from
// HBM at each 16-byte boundary stalled the whole wavefront on a memory round
// trip about every second decision step.  Past the end of the stream it
// returns 1-bits.
//
// Position: the reader keeps u = ~(pos + 63), pos = the stream index of the
// next bit not yet in C.  Then the window (w0 = word K - 1, w1 = word K,
// K = ceil(pos / 32)) starts at bit offset (-pos) & 31 = u & 31 from w1's
// start, which is alignbit's shift operand as it stands; a move by n bits
// is u -= n, crossing into the next word exactly when u and u - n differ
// above bit 4; and word K + 1 (nextw) sits in ring slot 15 - ((K + 1) % 16)
// = bits [8:5] of u -- the ring is laid out in reverse so that no position
// arithmetic is left on the per-decision path.  The two rare events, a carry
// event (below) and a dry ring, are one unsigned compare against `ulim`.
// ---------------------------------------------------------------------------
constexpr uint32_t FB_RING = 16;  // words per lane
struct FlatBits {
    uint32_t *ring;         // this lane's ring (see above)
    uint32_t rsh;           // slot stride = 1 << rsh words
    uint32_t wp;            // words put into the ring
    uint32_t chunk;         // next chunk of the stream to fetch
    uint32_t nchunks;
    const uint4 *base;
};

// the stream ends with two all-ones chunks, so reads past the end clamp to
// the last chunk (no branch around the load, no select on its result)
GRK_HD uint4 fb_load(const FlatBits &b, uint32_t ci) { return b.base[ci < b.nchunks ? ci : b.nchunks - 1]; }

// stream word j lives in ring slot 15 - j % 16
GRK_HD uint32_t &fb_slot(const FlatBits &b, uint32_t j) { return b.ring[(FB_RING - 1 - (j % FB_RING)) << b.rsh]; }

GRK_HD void fb_put(FlatBits &b, const uint4 &c) {
    fb_slot(b, b.wp + 0) = c.x;
    fb_slot(b, b.wp + 1) = c.y;
    fb_slot(b, b.wp + 2) = c.z;
    fb_slot(b, b.wp + 3) = c.w;
    b.wp += 4;
}

// top the ring up (both chunk loads issued before either is stored); never
// past FB_RING words from rp, the oldest word the reader still reads
GRK_HD void fb_fill(FlatBits &b, uint32_t rp) {
    const uint32_t held = b.wp - rp;
    if (held <= FB_RING - 8) {
        const uint4 c0 = fb_load(b, b.chunk), c1 = fb_load(b, b.chunk + 1);
        b.chunk += 2;
        fb_put(b, c0);
        fb_put(b, c1);
    } else if (held <= FB_RING - 4) {
        const uint4 c0 = fb_load(b, b.chunk++);
        fb_put(b, c0);
    }
}

GRK_HD void fb_start(FlatBits &b, const uint32_t *words, uint32_t nwords) {
    b.base = (const uint4 *)words;
    b.nchunks = (nwords + 3) >> 2;
    b.chunk = 0;
    b.wp = 0;
    fb_fill(b, 0);
}

// ---------------------------------------------------------------------------
// MQ decoder over the unstuffed stream (used by the pass walk of t1_dec.h):
// branch-free renormalisation and word advance.
// ---------------------------------------------------------------------------
// LAZY: the decoder may meet raw (BYPASS) segments; compiled out otherwise,
// so the common case keeps its per-symbol path branch-free.
template <bool LAZY>
struct BitDecT {
    static constexpr bool kLazy = LAZY;
    FlatBits bits;
    uint32_t A, C;
    uint32_t cq, cqn;  // next carry event (a stream bit index, Unstuff), the one after
    // the window {w0, w1}, the position u (see FlatBits) and nextw, word
    // K + 1, re-read from the ring at every decision -- the read needs no
    // branch, and by the next word advance it has landed
    uint32_t w0, w1, u, nextw;
    uint32_t ulim;  // u below it: a carry event is due or the ring is dry
    const uint32_t *cp;
    bool raw;  // the current segment is raw (BYPASS): bits straight from the stream
    // the lane's word ring (FlatBits), set once before the first init
    GRK_HD void set_ring(uint32_t *ring, uint32_t rsh) {
        bits.ring = ring;
        bits.rsh = rsh;
    }
    GRK_HD uint32_t next_word() const { return ~u >> 5; }  // K + 1 = (pos + 63) >> 5
    // u < ulim: pos passed the carry event cq (pos > cq: u < ~(cq + 63)), or
    // word K + 1 is not in the ring (K + 1 >= wp: u <= ~(32 wp))
    GRK_HD void set_limit() {
        const uint32_t lc = cq == 0xffffffffu ? 0u : ~(cq + 63u);
        const uint32_t ld = ~(32u * bits.wp) + 1u;
        ulim = lc > ld ? lc : ld;
    }
    // stripe start (t1_decode_passes): top the word ring up from HBM
    GRK_HD void fill() {
        fb_fill(bits, next_word());
        set_limit();
    }
    // the rare path of a move to u1: a carry event, a dry ring (a chunk
    // straight from HBM), or both; the carry is added to C after its shift
    GRK_HD void slow(const uint32_t u1) {
        const uint32_t pos1 = ~u1 - 63u;
        if (cq != 0xffffffffu && cq < pos1) {  // carry event (see Unstuff)
            C += 1u << (16 + pos1 - cq);
            next_carry();
        }
        if ((~u1 >> 5) >= bits.wp) {
            const uint4 c0 = fb_load(bits, bits.chunk++);
            fb_put(bits, c0);
        }
        set_limit();
    }
    // the window moves by n bits (n <= 16): a move past w0 takes the next
    // word (a select, no branch) and reads the one after from the ring
    GRK_HD void advance(uint32_t n) {
        const bool cross = (u & 31u) < n;  // fewer than n bits left in w0
        w0 = cross ? w1 : w0;
        w1 = cross ? nextw : w1;
        // the window moves here, before the rare branch: the old u and
        // nextw die at once and their registers carry the new ones (left to
        // itself the compiler sinks the selects past the branch and copies
        // both at every step)
        keep_here(w0);
        keep_here(w1);
        u -= n;
        if (u < ulim) slow(u);
        nextw = bits.ring[ring_slot(u) << bits.rsh];
    }
    // bits [8:5] of u, as one v_bfe_u32 (the compiler's shift-and-mask form
    // of it costs an op more on the address)
    GRK_HD static uint32_t ring_slot(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
        uint32_t r;
        asm("v_bfe_u32 %0, %1, 5, 4" : "=v"(r) : "v"(v));
        return r;
#else
        return (v >> 5) & (FB_RING - 1);
#endif
    }
    // raw segment (mqc_raw_init_dec / mqc_raw_decode, mqc_dec.cpp:195-200,
    // mqc_dec_inl.h:90-112): the unstuffed stream IS the raw bit sequence --
    // 7 bits from the byte after a 0xFF, 1-bits from a marker on
    GRK_HD void init_raw(const uint32_t *words, uint32_t nwords) {
        fb_start(bits, words, nwords);
        // pos 0: K = 0, so w1 = word 0 and w0 = (none); nextw = word 1
        w0 = 0;
        w1 = fb_slot(bits, 0);
        nextw = fb_slot(bits, 1);
        u = ~63u;
        cq = cqn = 0xffffffffu;
        set_limit();
        raw = true;
    }
    GRK_HD uint32_t rawbit() {
        const uint32_t b = alignbit32(w0, w1, u) >> 31;
        advance(1);
        return b;
    }
    GRK_HD void init(const uint32_t *words, uint32_t nwords, const uint32_t *carries) {
        raw = false;
        fb_start(bits, words, nwords);
        // pos 31 (INITDEC: consumed 24, then 7 shifts): C = the first 31
        // stream bits, K = 1 (w0 = word 0, w1 = word 1), nextw = word 2
        w0 = fb_slot(bits, 0);
        w1 = fb_slot(bits, 1);
        nextw = fb_slot(bits, 2);
        C = w0 >> 1;
        u = ~(31u + 63u);
        A = 0x80000000u;  // 0x8000 << 16
        cq = carries[0];
        cp = carries + 1;
        if (cq < 31) { C += 1u << (16 + 31 - cq); cq = *cp++; }
        cqn = cq == 0xffffffffu ? cq : *cp++;  // the sentinel ends the list: never read past it
        set_limit();
    }
    // the carry event after the one just applied: cqn was loaded one event
    // earlier, so the rare path never waits on a load
    GRK_HD void next_carry() {
        cq = cqn;
        cqn = cq == 0xffffffffu ? cq : *cp++;
    }
    GRK_HD uint32_t decode(uint32_t *cxw, const uint32_t *tab, uint32_t cx) {
        if constexpr (LAZY) {
            if (raw) return rawbit();
        }
        uint32_t wd = cxw[cx];
        const uint32_t bit = step(wd, tab);
        cxw[cx] = wd;  // unconditional LDS write: no branch
#ifdef T1_TRACE
        T1_TRACE(cx, bit, A >> 16, C >> 16);
#endif
        return bit;
    }
    // the same decision with the context word in a register (the magnitude
    // refinement keeps its three contexts in registers for a stripe: no LDS
    // round trip on its decision chain)
    GRK_HD uint32_t decode_reg(uint32_t &wd, const uint32_t *tab, uint32_t cx) {
        if constexpr (LAZY) {
            if (raw) return rawbit();
        }
        const uint32_t bit = step(wd, tab);
#ifdef T1_TRACE
        T1_TRACE(cx, bit, A >> 16, C >> 16);
#else
        (void)cx;
#endif
        return bit;
    }
    // One MQ decision with context word wd (updated in place).  A is held
    // << 16 and the context word carries Qe << 16 (mq_dec_word), so the
    // interval and the code register compare against Qe as it is loaded:
    // C < Qe << 16  <=>  C[31:16] < Qe, and the renormalisation shift is
    // clz(A) directly.  The next word comes from the successor table
    // (mq_dec_table_entry: the MPS flip already in it) at the word's own
    // byte offset, + 512 for the LPS successor.  The renormalisation shifts the next n
    // window bits into C (a bit-field extract of the 32 window bits).
    GRK_HD uint32_t step(uint32_t &wd, const uint32_t *tab) {
        const uint32_t qe = wd & 0xffff0000u;
        uint32_t a = A - qe;
        const bool lo = C < qe;
        const bool lps = lo ? (a >= qe) : (a < qe);
        const bool keep = !lo && (int32_t)a < 0;  // MPS, no renormalisation
        C = lo ? C : C - qe;
        a = lo ? qe : a;
        const uint32_t tw = *(const uint32_t *)((const char *)tab + ((wd & 0x1FCu) | (lps ? 512u : 0u)));
        const uint32_t n = clz32(a);
        const uint32_t win = alignbit32(w0, w1, u);
        C = (C << n) | bfe32(win, 32 - n, n);
        A = a << n;
        advance(n);
        // the bit as (wd ^ lps) & 1 on a materialised lps (one select and
        // one 3-input op), not the mask logic the compiler would form
        uint32_t lv = lps ? 1u : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(lv));
#endif
        const uint32_t bit = (wd ^ lv) & 1u;
        wd = keep ? wd : tw;
        return bit;
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

// v5: the nested pass / stripe / column walk (lanes of a wavefront stay
// converged on the pass structure) fed by the unstuffed bit stream.
// ring / rsh: the lane's word ring (FlatBits).
template <class ST = BlockState, class RP = uint64_t *, bool MRPREG = true>
GRK_HD void t1_decode_v5(const uint32_t *words, uint32_t nwords, const uint32_t *carries, uint32_t numpasses,
                         uint32_t numbps, uint32_t w, uint32_t h, ST &st, const DecTables &T, uint32_t *cxw,
                         RP sa, RP rb, uint32_t *ring, uint32_t rsh) {
    for (uint32_t y = 0; y < h + 2; ++y) { st.sig[y] = 0; st.neg[y] = 0; st.vis[y] = 0; st.ref[y] = 0; }
    mq_reset_words_dec(cxw, T.mq);
    BitDec d;
    d.set_ring(ring, rsh);
    d.init(words, nwords, carries);
    t1_decode_passes<BitDec, NoSegs, ST, RP, MRPREG>(d, numpasses, numbps, w, h, st, T, cxw, sa, rb);
}

}  // namespace grkgpu
