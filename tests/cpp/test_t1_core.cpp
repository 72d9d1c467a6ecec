// Host-side check of the T1 block coder used by the HIP kernels
// (grokimagecompression_amd/csrc/t1_core.h) against the CPU oracle.
// Built and run by tests/test_t1_core_host.py (no GPU needed).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "../../grokimagecompression_amd/csrc/t1_core.h"
#include "../../oracle/grk_oracle.h"

using namespace grkgpu;
static const uint32_t kTab[47] = GRK_MQ_TABLE_INIT;

static uint64_t rng = 88172645463325252ull;
static uint32_t rnd() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return (uint32_t)rng; }

int main(int argc, char **argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 400;
    int fails = 0;
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
        }
    }
    printf("%s: %d failures / %d blocks\n", fails ? "FAIL" : "OK", fails, iters);
    return fails ? 1 : 0;
}
