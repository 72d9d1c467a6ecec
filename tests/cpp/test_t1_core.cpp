// Host-side check of the T1 block coder used by the HIP kernels
// (grokimagecompression_amd/csrc/t1_core.h) against the CPU oracle.
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

static uint64_t rng = 88172645463325252ull;
static uint32_t rnd() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (uint32_t)rng; }

static T1Scratch scr;

int main(int argc, char **argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 400;
    int fails = 0;
    static uint8_t zc[2048], sc[256];
    for (uint32_t i = 0; i < 2048; ++i) zc[i] = zc_lut_entry(i >> 9, i & 511);
    for (uint32_t i = 0; i < 256; ++i) sc[i] = sc_lut_entry(i);
    const T1Tables T{zc, sc, kTab};
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
        std::vector<uint8_t> obuf(w * h * 8 + 64, 0), gbuf(w * h * 8 + 64, 0);
        orc_pass op[100];
        uint32_t onb = 0, olen = 0;
        int onp = orc_t1_encode_cblk(coef.data(), w, w, h, orient, qmfbid, inv_step, obuf.data() + 1,
                                     (uint32_t)obuf.size() - 1, op, &onb, &olen);
        // device code compiled for the host
        BlockRows rows;
        PassInfo gp[100];
        uint32_t gnb = 0, glen = 0;
        uint32_t gnp = t1_encode_block(coef.data(), w, w, h, orient, qmfbid, inv_step, rows, kTab, gbuf.data() + 1,
                                       gp, &gnb, &glen);
        bool ok = (int)gnp == onp && gnb == onb && glen == olen && memcmp(obuf.data(), gbuf.data(), olen + 1) == 0;
        for (int p = 0; ok && p < onp; ++p) ok = gp[p].rate == op[p].rate && gp[p].len == op[p].len && gp[p].term == op[p].term;
        if (!ok) {
            printf("ENC MISMATCH it=%d w=%u h=%u orient=%u q=%d np %u/%d nb %u/%u len %u/%u\n", it, w, h, orient, qmfbid,
                   gnp, onp, gnb, onb, glen, olen);
            fails++;
            continue;
        }
        // lane coder v2 (t1_lane.h): prep + encode must give the same bytes and rates
        {
            uint32_t lnb = t1_prep_serial(coef.data(), w, w, h, qmfbid, inv_step, scr.st, scr.pa);
            std::vector<uint32_t> lout(w * h * 2 + 64, 0);
            uint32_t lrate[100], llen = 0;
            uint32_t cx[32];
            uint32_t lnp = t1_encode_lane(w, h, lnb, scr.pa, scr.st, T, orient, cx, lout.data(), lrate, &llen);
            bool lok = (int)lnp == onp && lnb == onb && llen == olen && memcmp(lout.data(), obuf.data() + 1, olen) == 0;
            for (int p = 0; lok && p < onp; ++p) lok = lrate[p] == op[p].rate;
            // split encoder: per-plane modelling + MQ
            t1_prep_above(h, lnb, scr.pa, scr.pb);
            const uint32_t slot = sym_slot_bytes(w, h), sb = sym_stream_bytes(w, h);
            std::vector<uint32_t> sym((size_t)(lnb ? lnb : 1) * slot / 4 + 16, 0);
            for (uint32_t p = 0; p < lnb; ++p) {
                uint32_t *base = sym.data() + (size_t)p * slot / 4;
                t1_model_plane(w, h, orient, scr.pa + p * 64, scr.pb + p * 64, p + 1 < lnb ? scr.pb + (p + 1) * 64 : nullptr,
                               scr.st.neg, (uint64_t *)(base + sb / 4), sc, base, scr.cnt + p * 4);
            }
            std::vector<uint32_t> sout(w * h * 2 + 64, 0);
            uint32_t srate[100], slen = 0;
            uint32_t snp = t1_mq_block(lnb, sym.data(), slot / 4, scr.cnt, kTab, cx, sout.data(), srate, &slen);
            bool sok = (int)snp == onp && slen == olen && memcmp(sout.data(), obuf.data() + 1, olen) == 0;
            for (int p = 0; sok && p < onp; ++p) sok = srate[p] == op[p].rate;
            if (!sok) {
                printf("SPLIT ENC MISMATCH it=%d w=%u h=%u orient=%u q=%d np %u/%d len %u/%u\n", it, w, h, orient, qmfbid,
                       snp, onp, slen, olen);
                fails++;
            }
            if (!lok) {
                printf("LANE ENC MISMATCH it=%d w=%u h=%u orient=%u q=%d np %u/%d nb %u/%u len %u/%u\n", it, w, h,
                       orient, qmfbid, lnp, onp, lnb, onb, llen, olen);
                fails++;
            }
        }
        if (onp == 0) continue;
        // decode round trip: all passes, and a truncated prefix
        for (int trunc = 0; trunc < 2; ++trunc) {
            uint32_t np = trunc ? (uint32_t)(1 + rnd() % onp) : (uint32_t)onp;
            uint32_t len = op[np - 1].rate;
            std::vector<uint8_t> data(gbuf.begin() + 1, gbuf.begin() + 1 + len);
            data.push_back(0); data.push_back(0);
            std::vector<int32_t> od(w * h), gd(w * h);
            orc_t1_decode_cblk(data.data(), len, np, onb, w, h, orient, od.data());
            struct Id { void operator()(int32_t *) const {} };
            t1_decode_block_impl(data.data(), len, np, onb, w, h, orient, rows, kTab, gd.data(), w, Id());
            if (od != gd) {
                printf("DEC MISMATCH it=%d w=%u h=%u np=%u\n", it, w, h, np);
                fails++;
            }
            // lane decoder v2 + rebuild, from an arbitrarily aligned copy
            std::vector<uint8_t> pad(len + 160, 0);
            uint8_t *lp = pad.data() + 16 + (it & 7);
            memcpy(lp, gbuf.data() + 1, len);
            uint32_t cx[20];
            t1_decode_lane(lp, len, np, onb, w, h, orient, scr.st, T, cx, scr.pa, scr.pb);
            DecodedPlanes dp = decoded_planes(np, onb);
            std::vector<int32_t> ld(w * h);
            for (uint32_t y = 0; y < h; ++y)
                for (uint32_t x = 0; x < w; ++x) ld[y * w + x] = t1_rebuild(x, y, dp, scr.pa, scr.pb, scr.st.neg[y + 1]);
            if (od != ld) {
                printf("LANE DEC MISMATCH it=%d w=%u h=%u np=%u nb=%u\n", it, w, h, np, onb);
                fails++;
            }
            // decoder v3 (t1_dec.h)
            {
                const DecTables DT{zc + orient * 512, scw, kTab};
                uint32_t cx3[32];
                std::fill(scr.pa, scr.pa + 32 * 64, ~0ull);
                std::fill(scr.pb, scr.pb + 32 * 64, ~0ull);
                t1_decode_v3(lp, len, np, onb, w, h, scr.st, DT, cx3, scr.pa, scr.pb);
                std::vector<int32_t> vd(w * h);
                for (uint32_t y = 0; y < h; ++y)
                    for (uint32_t x = 0; x < w; ++x) vd[y * w + x] = t1_rebuild(x, y, dp, scr.pa, scr.pb, scr.st.neg[y + 1]);
                if (od != vd) {
                    printf("V3 DEC MISMATCH it=%d w=%u h=%u np=%u nb=%u orient=%u\n", it, w, h, np, onb, orient);
                    fails++;
                }
            }
            // decoder v4 (t1_flat.h): unstuffed bit stream, one decision per step
            {
                const DecTables DT{zc + orient * 512, scw, kTab};
                uint32_t cx4[32];
                std::vector<uint32_t> words(unstuff_word_cap(len) + 8, 0), carr(unstuff_carry_cap(len), 0);
                uint32_t *wp = (uint32_t *)(((uintptr_t)words.data() + 15) & ~(uintptr_t)15);
                uint32_t ncar = 0;
                uint32_t nw = t1_unstuff(lp, len, wp, carr.data(), &ncar);
                std::fill(scr.pa, scr.pa + 32 * 64, ~0ull);
                std::fill(scr.pb, scr.pb + 32 * 64, ~0ull);
                for (int i = 0; i < 66; ++i) { scr.st.sig[i] = scr.st.neg[i] = scr.st.vis[i] = scr.st.ref[i] = ~0ull; }
                t1_decode_flat(wp, nw, carr.data(), np, onb, w, h, scr.st, DT, cx4, scr.pa, scr.pb);
                std::vector<int32_t> fd(w * h);
                for (uint32_t y = 0; y < h; ++y)
                    for (uint32_t x = 0; x < w; ++x) fd[y * w + x] = t1_rebuild(x, y, dp, scr.pa, scr.pb, scr.st.neg[y + 1]);
                // v5: v3's walk over the same unstuffed stream
                {
                    std::fill(scr.pa, scr.pa + 32 * 64, ~0ull);
                    std::fill(scr.pb, scr.pb + 32 * 64, ~0ull);
                    t1_decode_v5(wp, nw, carr.data(), np, onb, w, h, scr.st, DT, cx4, scr.pa, scr.pb);
                    std::vector<int32_t> v5(w * h);
                    for (uint32_t y = 0; y < h; ++y)
                        for (uint32_t x = 0; x < w; ++x) v5[y * w + x] = t1_rebuild(x, y, dp, scr.pa, scr.pb, scr.st.neg[y + 1]);
                    if (od != v5) {
                        printf("V5 DEC MISMATCH it=%d w=%u h=%u np=%u nb=%u orient=%u\n", it, w, h, np, onb, orient);
                        fails++;
                    }
                }
                if (od != fd) {
                    int bad = 0;
                    for (uint32_t i = 0; i < w * h; ++i) bad += od[i] != fd[i];
                    printf("V4 DEC MISMATCH it=%d w=%u h=%u np=%u nb=%u orient=%u bad=%d\n", it, w, h, np, onb, orient, bad);
                    fails++;
                }
            }
        }
    }
    printf("%s: %d failures / %d blocks\n", fails ? "FAIL" : "OK", fails, iters);
    return fails ? 1 : 0;
}
