// Host-side check of the T1 coders of the HIP kernels (the split encoder of
// t1_lane.h, the decoder of t1_dec.h / t1_flat.h, compiled for the host)
// against the CPU oracle, block by block (bytes, pass rates, coefficients).
// Built and run by tests/test_t1_core_host.py (no GPU needed).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include "../../grokimagecompression_amd/csrc/t1_flat.h"
#include "../../oracle/grk_oracle.h"

using namespace grkgpu;
static const uint32_t kTab[47] = GRK_MQ_TABLE_INIT;
static uint32_t kDecTab[MQ_DEC_WORDS];
static const bool kDecInit = [] { for (uint32_t i = 0; i < MQ_DEC_WORDS; ++i) kDecTab[i] = mq_dec_table_entry(kTab, i); return true; }();

static uint64_t rng = 88172645463325252ull;
static uint32_t rnd() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (uint32_t)rng; }

static T1Scratch scr;

int main(int argc, char **argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 400;
    int fails = 0;
    static uint8_t zc[2048], sc[256];
    for (uint32_t i = 0; i < 2048; ++i) zc[i] = zc_lut_entry(i >> 9, i & 511);
    for (uint32_t i = 0; i < 256; ++i) sc[i] = sc_lut_entry(i);
    static uint8_t scw[256];
    for (uint32_t i = 0; i < 256; ++i) scw[i] = sc_win_entry(i);
    for (int it = 0; it < iters; ++it) {
        uint32_t w = 1 + rnd() % 64, h = 1 + rnd() % 64;
        if (it % 3 == 0) { w = 64; h = 64; }
        uint32_t orient = rnd() % 4;
        int qmfbid = rnd() % 2;
        int32_t inv_step = 1000 + rnd() % 20000;
        uint32_t amp = 1u << (rnd() % (qmfbid ? 15 : 24));
        int kind = rnd() % 4;
        std::vector<int32_t> coef(w * h);
        for (uint32_t i = 0; i < w * h; ++i) {
            int32_t v = (int32_t)(rnd() % (2 * amp + 1)) - (int32_t)amp;
            if (kind == 1 && (rnd() % 8)) v = 0;           // sparse
            if (kind == 2) v = (int32_t)(i % w) - (int32_t)(w / 2);  // ramps
            coef[i] = v;
        }
        // oracle
        std::vector<uint8_t> obuf(w * h * 8 + 64, 0);
        orc_pass op[100];
        uint32_t onb = 0, olen = 0;
        int onp = orc_t1_encode_cblk(coef.data(), w, w, h, orient, qmfbid, inv_step, obuf.data() + 1,
                                     (uint32_t)obuf.size() - 1, op, &onb, &olen);
        // the GPU encoder's device code compiled for the host: prep, per-plane
        // context modelling (k_t1_model) + MQ coder (k_t1_mq)
        {
            uint32_t lnb = t1_prep_serial(coef.data(), w, w, h, qmfbid, inv_step, scr.st, scr.pa);
            uint32_t cx[32];
            t1_prep_above(h, lnb, scr.pa, scr.pb);
            const uint32_t slot = sym_slot_bytes(w, h);
            std::vector<uint32_t> sym((size_t)(lnb ? lnb : 1) * slot / 4 + 16, 0);
            uint64_t tmp[128];
            for (uint32_t p = 0; p < lnb; ++p) {
                uint32_t *base = sym.data() + (size_t)p * slot / 4;
                const uint64_t *ref = p + 1 < lnb ? scr.pb + (p + 1) * 64 : scr.pb;
                t1_model_plane<const uint64_t *, uint64_t *>(w, h, orient, scr.pa + p * 64, scr.pb + p * 64, ref,
                                                             p + 1 < lnb, scr.st.neg, tmp, sc, base, scr.cnt + p * 4);
            }
            // a dword of headroom before the output (the pad byte's commit)
            std::vector<uint32_t> sbuf(w * h * 2 + 64 + 1, 0);
            uint32_t *sout = sbuf.data() + 1;
            uint32_t srate[100], slen = 0;
            uint32_t snp = t1_mq_block(lnb, sym.data(), slot / 4, scr.cnt, kTab, cx, sout, srate, &slen);
            bool sok = lnb == onb && (int)snp == onp && slen == olen && memcmp(sout, obuf.data() + 1, olen) == 0;
            for (int p = 0; sok && p < onp; ++p) sok = srate[p] == op[p].rate;
            if (!sok) {
                printf("ENC MISMATCH it=%d w=%u h=%u orient=%u q=%d np %u/%d nb %u/%u len %u/%u\n", it, w, h, orient,
                       qmfbid, snp, onp, lnb, onb, slen, olen);
                fails++;
                continue;
            }
        }
        if (onp == 0) continue;
        // decode round trip: all passes, and a truncated prefix
        for (int trunc = 0; trunc < 2; ++trunc) {
            uint32_t np = trunc ? (uint32_t)(1 + rnd() % onp) : (uint32_t)onp;
            uint32_t len = op[np - 1].rate;
            std::vector<uint8_t> data(obuf.begin() + 1, obuf.begin() + 1 + len);
            data.push_back(0); data.push_back(0);
            std::vector<int32_t> od(w * h);
            orc_t1_decode_cblk(data.data(), len, np, onb, w, h, orient, od.data());
            DecodedPlanes dp = decoded_planes(np, onb);
            // the GPU decoder (k_t1_unstuff + k_t1_decode_ub, decoder v5) from an
            // arbitrarily aligned copy, then the rebuild (k_t1_rebuild)
            std::vector<uint8_t> pad(len + 160, 0);
            uint8_t *lp = pad.data() + 16 + (it & 7);
            memcpy(lp, obuf.data() + 1, len);
            const DecTables DT{zc + orient * 512, scw, kDecTab};
            uint32_t cx4[32];
            std::vector<uint32_t> words(unstuff_word_cap(len) + 8, 0), carr(unstuff_carry_cap(len), 0);
            uint32_t *wp = (uint32_t *)(((uintptr_t)words.data() + 15) & ~(uintptr_t)15);
            uint32_t ncar = 0;
            uint32_t nw = t1_unstuff(lp, len, wp, carr.data(), &ncar);
            std::fill(scr.pa, scr.pa + 32 * 64, ~0ull);
            std::fill(scr.pb, scr.pb + 32 * 64, ~0ull);
            for (int i = 0; i < 66; ++i) { scr.st.sig[i] = scr.st.neg[i] = scr.st.vis[i] = scr.st.ref[i] = ~0ull; }
            uint32_t ring[FB_RING];
            t1_decode_v5(wp, nw, carr.data(), np, onb, w, h, scr.st, DT, cx4, scr.pa, scr.pb, ring, 0);
            std::vector<int32_t> v5(w * h);
            for (uint32_t y = 0; y < h; ++y)
                for (uint32_t x = 0; x < w; ++x) v5[y * w + x] = t1_rebuild(x, y, dp, scr.pa, scr.pb, scr.st.neg[y + 1]);
            if (od != v5) {
                printf("DEC MISMATCH it=%d w=%u h=%u np=%u nb=%u orient=%u\n", it, w, h, np, onb, orient);
                fails++;
            }
        }
    }
    printf("%s: %d failures / %d blocks\n", fails ? "FAIL" : "OK", fails, iters);
    return fails ? 1 : 0;
}
