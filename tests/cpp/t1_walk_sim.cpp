// t1_walk_sim.cpp -- host analysis of the T1 decoder's SIMT efficiency (not a
// test; scripts/t1_walk_sim.py drives it).  Reads code-blocks of DWT
// coefficients, codes each with the C oracle's T1 encoder, decodes it with the
// GPU decoder's walk compiled for the host (t1_dec.h / t1_flat.h) while the
// T1_WALK / T1_TRACE hooks record every pass, stripe, column and decision,
// then replays wavefronts of 64 consecutive blocks under several loop
// structures and reports lane utilisation = decisions / (64 x wave steps):
//   nested   the decoder as built: passes, stripes, column steps and symbol
//            steps in lock step (a wave step per symbol step of the slowest
//            lane in each column step)
//   stripe   columns and symbols of a stripe flattened (a lane moves to its
//            next column inside the symbol loop)
//   pass     a lane's whole pass flattened
//   block    a lane's whole block flattened (upper bound)
// plus the column steps (one column set-up each) of the nested walk.
//
// input (stdin, binary little-endian): n, then per block: w, h, orient,
// qmfbid, inv_step (int32 each) and w*h int32 coefficients.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

struct Ev {
    uint8_t kind;   // 0 pass, 1 stripe, 2 column
    uint16_t v;
    uint32_t nsym;  // decisions after this event until the next one
};
static std::vector<Ev> *g_ev;
#define T1_WALK(e, val) (g_ev->push_back(Ev{(uint8_t)(e), (uint16_t)(val), 0}), (e) == 0 ? (g_pass = (val)) : 0)
static uint64_t g_cx[19][2];
static uint32_t g_pass;
static uint64_t g_bypass[3];
#define T1_TRACE(cx, bit, a, c) (g_ev->back().nsym++, g_cx[cx][bit]++, g_bypass[g_pass]++)

#include "../../grokimagecompression_amd/csrc/t1_flat.h"
#include "../../oracle/grk_oracle.h"

using namespace grkgpu;
static const uint32_t kTab[47] = GRK_MQ_TABLE_INIT;
static uint32_t kDecTab[MQ_DEC_WORDS];
static const bool kDecInit = [] { for (uint32_t i = 0; i < MQ_DEC_WORDS; ++i) kDecTab[i] = mq_dec_table_entry(kTab, i); return true; }();
static T1Scratch scr;

// per block: passes -> stripes -> columns -> decisions
struct Col { uint32_t n; };
struct Stripe_ { std::vector<uint32_t> cols; uint32_t lead; };  // lead: decisions before the first column (SEGSYM etc.)
struct Pass_ { uint32_t type; std::vector<Stripe_> stripes; };
struct Blk { std::vector<Pass_> passes; uint64_t total; };

int main() {
    uint32_t n;
    if (fread(&n, 4, 1, stdin) != 1) return 1;
    static uint8_t zc[2048], scw[256];
    for (uint32_t i = 0; i < 2048; ++i) zc[i] = zc_lut_entry(i >> 9, i & 511);
    for (uint32_t i = 0; i < 256; ++i) scw[i] = sc_win_entry(i);
    std::vector<Blk> blks;
    uint64_t tot_dec = 0;
    std::vector<Ev> ev;
    g_ev = &ev;
    for (uint32_t b = 0; b < n; ++b) {
        int32_t hdr[5];
        if (fread(hdr, 4, 5, stdin) != 5) return 2;
        const uint32_t w = hdr[0], h = hdr[1], orient = hdr[2];
        std::vector<int32_t> coef((size_t)w * h);
        if (fread(coef.data(), 4, coef.size(), stdin) != coef.size()) return 3;
        std::vector<uint8_t> obuf(w * h * 8 + 64, 0);
        orc_pass op[100];
        uint32_t onb = 0, olen = 0;
        const int onp = orc_t1_encode_cblk(coef.data(), w, w, h, orient, hdr[3], hdr[4], obuf.data() + 1,
                                           (uint32_t)obuf.size() - 1, op, &onb, &olen);
        Blk bk;
        bk.total = 0;
        if (onp > 0) {
            const uint32_t len = olen;
            std::vector<uint32_t> words(unstuff_word_cap(len) + 16, 0), carr(unstuff_carry_cap(len) + 4, 0);
            uint32_t *wp = (uint32_t *)(((uintptr_t)words.data() + 15) & ~(uintptr_t)15);
            uint32_t ncar = 0;
            const uint32_t nw = t1_unstuff(obuf.data() + 1, len, wp, carr.data(), &ncar);
            const DecTables DT{zc + orient * 512, scw, kDecTab};
            uint32_t cx4[32], ring[FB_RING];
            ev.clear();
            ev.push_back(Ev{9, 0, 0});
            t1_decode_v5(wp, nw, carr.data(), (uint32_t)onp, onb, w, h, scr.st, DT, cx4, scr.pa, scr.pb, ring, 0);
            for (const Ev &e : ev) {
                bk.total += e.nsym;
                if (e.kind == 0) bk.passes.push_back(Pass_{e.v, {}});
                else if (e.kind == 1) bk.passes.back().stripes.push_back(Stripe_{{}, e.nsym});
                else if (e.kind == 2) bk.passes.back().stripes.back().cols.push_back(e.nsym);
                else if (e.nsym) fprintf(stderr, "decisions before the first pass?\n");
            }
        }
        tot_dec += bk.total;
        blks.push_back(std::move(bk));
    }
    // replay wavefronts of 64 consecutive blocks
    uint64_t st_nested = 0, st_colsteps = 0, st_stripe = 0, st_pass = 0, st_block = 0, st_stripes = 0;
    // per pass type (0 SPP, 1 MRP, 2 CUP): nested symbol steps, column steps, stripe-flat and pass-flat steps
    uint64_t pt_nested[3] = {}, pt_cols[3] = {}, pt_stripe[3] = {}, pt_pass[3] = {}, pt_dec[3] = {};
    // column steps in which every lane's column took one decision (cleanup:
    // mostly aggregation-0 columns, whose set-up could be skipped)
    uint64_t pt_cols1[3] = {};
    for (auto &bk : blks)
        for (auto &ps : bk.passes)
            for (auto &sp : ps.stripes) { pt_dec[ps.type] += sp.lead; for (uint32_t c : sp.cols) pt_dec[ps.type] += c; }
    for (size_t w0 = 0; w0 < blks.size(); w0 += 64) {
        const size_t w1 = std::min(blks.size(), w0 + 64);
        size_t maxp = 0;
        uint64_t maxb = 0;
        for (size_t i = w0; i < w1; ++i) { maxp = std::max(maxp, blks[i].passes.size()); maxb = std::max(maxb, blks[i].total); }
        st_block += maxb;
        for (size_t p = 0; p < maxp; ++p) {
            size_t maxs = 0;
            uint64_t maxpass = 0;
            for (size_t i = w0; i < w1; ++i)
                if (p < blks[i].passes.size()) {
                    maxs = std::max(maxs, blks[i].passes[p].stripes.size());
                    uint64_t t = 0;
                    for (auto &s : blks[i].passes[p].stripes) { t += s.lead; for (uint32_t c : s.cols) t += c; }
                    maxpass = std::max(maxpass, t);
                }
            st_pass += maxpass;
            st_stripes += maxs;
            uint32_t ptype = 0;
            for (size_t i = w0; i < w1; ++i)
                if (p < blks[i].passes.size()) { ptype = blks[i].passes[p].type; break; }
            pt_pass[ptype] += maxpass;
            for (size_t k = 0; k < maxs; ++k) {
                size_t maxc = 0;
                uint64_t maxst = 0, maxlead = 0;
                for (size_t i = w0; i < w1; ++i) {
                    if (p >= blks[i].passes.size() || k >= blks[i].passes[p].stripes.size()) continue;
                    const Stripe_ &s = blks[i].passes[p].stripes[k];
                    maxc = std::max(maxc, s.cols.size());
                    uint64_t t = s.lead;
                    for (uint32_t c : s.cols) t += c;
                    maxst = std::max(maxst, t);
                    maxlead = std::max<uint64_t>(maxlead, s.lead);
                }
                st_stripe += maxst;
                st_colsteps += maxc;
                st_nested += maxlead;
                pt_stripe[ptype] += maxst;
                pt_cols[ptype] += maxc;
                pt_nested[ptype] += maxlead;
                for (size_t j = 0; j < maxc; ++j) {
                    uint32_t m = 0;
                    for (size_t i = w0; i < w1; ++i) {
                        if (p >= blks[i].passes.size() || k >= blks[i].passes[p].stripes.size()) continue;
                        const Stripe_ &s = blks[i].passes[p].stripes[k];
                        if (j < s.cols.size()) m = std::max(m, s.cols[j]);
                    }
                    if (m == 1) pt_cols1[ptype]++;
                    st_nested += m;
                    pt_nested[ptype] += m;
                }
            }
        }
    }
    const double d = (double)tot_dec;
    printf("{\"blocks\": %zu, \"decisions\": %llu, \"util\": {\"nested\": %.4f, \"stripe\": %.4f, \"pass\": %.4f, "
           "\"block\": %.4f}, \"wave_steps\": {\"nested_symbol\": %llu, \"nested_column\": %llu, \"stripes\": %llu, "
           "\"stripe\": %llu, \"pass\": %llu, \"block\": %llu}}\n",
           blks.size(), (unsigned long long)tot_dec, d / (64.0 * st_nested), d / (64.0 * st_stripe), d / (64.0 * st_pass),
           d / (64.0 * st_block), (unsigned long long)st_nested, (unsigned long long)st_colsteps,
           (unsigned long long)st_stripes, (unsigned long long)st_stripe, (unsigned long long)st_pass,
           (unsigned long long)st_block);
    for (int t = 0; t < 3; ++t)
        fprintf(stderr, "pass type %d: decisions %llu ideal steps %llu | nested symbol steps %llu, column steps %llu | "
                        "stripe-flat %llu | pass-flat %llu\n", t, (unsigned long long)pt_dec[t],
                (unsigned long long)(pt_dec[t] / 64), (unsigned long long)pt_nested[t], (unsigned long long)pt_cols[t],
                (unsigned long long)pt_stripe[t], (unsigned long long)pt_pass[t]);
    fprintf(stderr, "column steps with one decision on every lane: spp %llu mrp %llu cup %llu\n",
            (unsigned long long)pt_cols1[0], (unsigned long long)pt_cols1[1], (unsigned long long)pt_cols1[2]);
    fprintf(stderr, "decisions by context (bit 0 / bit 1):\n");
    for (int c = 0; c < 19; ++c)
        fprintf(stderr, "  cx %2d: %10llu %10llu\n", c, (unsigned long long)g_cx[c][0], (unsigned long long)g_cx[c][1]);
    fprintf(stderr, "decisions by pass type: spp %llu mrp %llu cup %llu\n", (unsigned long long)g_bypass[0],
            (unsigned long long)g_bypass[1], (unsigned long long)g_bypass[2]);
    return 0;
}
