// codestream.cpp -- host geometry, quantisation parameters, Tier-2 packets and
// headers for the MI355X JPEG 2000 path (see codestream.h).
#include "codestream.h"

#include <math.h>

#include <algorithm>

namespace grkgpu {

// ---------------------------------------------------------------------------
// quantisation parameters -- param_qcd::generate (codestream/HTParams.cpp:164)
// ---------------------------------------------------------------------------
namespace {
// BIBO gains (HTParams.cpp:105-149) and sqrt energy gains (HTParams.cpp:49-84)
const float kBibo53L[34] = {1.0000e+00f, 1.5000e+00f, 1.6250e+00f, 1.6875e+00f, 1.6963e+00f, 1.7067e+00f,
    1.7116e+00f, 1.7129e+00f, 1.7141e+00f, 1.7145e+00f, 1.7151e+00f, 1.7152e+00f, 1.7155e+00f, 1.7155e+00f,
    1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f,
    1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f,
    1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f};
const float kBibo53H[34] = {2.0000e+00f, 2.5000e+00f, 2.7500e+00f, 2.8047e+00f, 2.8198e+00f, 2.8410e+00f,
    2.8558e+00f, 2.8601e+00f, 2.8628e+00f, 2.8656e+00f, 2.8662e+00f, 2.8667e+00f, 2.8669e+00f, 2.8670e+00f,
    2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f,
    2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f,
    2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f};
const float kGain97L[34] = {1.0000e+00f, 1.4021e+00f, 2.0304e+00f, 2.9012e+00f, 4.1153e+00f, 5.8245e+00f,
    8.2388e+00f, 1.1652e+01f, 1.6479e+01f, 2.3304e+01f, 3.2957e+01f, 4.6609e+01f, 6.5915e+01f, 9.3217e+01f,
    1.3183e+02f, 1.8643e+02f, 2.6366e+02f, 3.7287e+02f, 5.2732e+02f, 7.4574e+02f, 1.0546e+03f, 1.4915e+03f,
    2.1093e+03f, 2.9830e+03f, 4.2185e+03f, 5.9659e+03f, 8.4371e+03f, 1.1932e+04f, 1.6874e+04f, 2.3864e+04f,
    3.3748e+04f, 4.7727e+04f, 6.7496e+04f, 9.5454e+04f};
const float kGain97H[34] = {1.4425e+00f, 1.9669e+00f, 2.8839e+00f, 4.1475e+00f, 5.8946e+00f, 8.3472e+00f,
    1.1809e+01f, 1.6701e+01f, 2.3620e+01f, 3.3403e+01f, 4.7240e+01f, 6.6807e+01f, 9.4479e+01f, 1.3361e+02f,
    1.8896e+02f, 2.6723e+02f, 3.7792e+02f, 5.3446e+02f, 7.5583e+02f, 1.0689e+03f, 1.5117e+03f, 2.1378e+03f,
    3.0233e+03f, 4.2756e+03f, 6.0467e+03f, 8.5513e+03f, 1.2093e+04f, 1.7103e+04f, 2.4187e+04f, 3.4205e+04f,
    4.8373e+04f, 6.8410e+04f, 9.6747e+04f, 1.3682e+05f};

int rev_bits(float g) { return (int)std::ceil(std::log((double)g) / M_LN2); }

StepSize irrev_step(float delta) {
    StepSize s;
    while (delta < 1.0f) { s.expn++; delta *= 2.0f; }
    uint32_t m = (uint32_t)std::round(delta * (float)(1 << 11)) - (1 << 11);
    s.mant = m < (1u << 11) ? m : 0x7FFu;
    return s;
}
}  // namespace

void generate_qcd(CodingParams &cp) {
    const uint32_t nd = cp.numres - 1;
    uint32_t s = 0;
    if (!cp.irrev) {
        // set_rev_quant (HTParams.cpp:187-207); the RCT bit is never added
        // because j2k_setup_encoder calls generate() before tcp->mct is set
        // (j2k.cpp:1839 vs :1861).
        const int B = (int)cp.prec[0];
        float l = kBibo53L[nd];
        cp.ss[s++] = {(uint32_t)(B + rev_bits(l * l * 1.1f)), 0};
        for (int d = (int)nd - 1; d >= 0; --d) {
            float bl = kBibo53L[d + 1], bh = kBibo53H[d];
            uint32_t e = (uint32_t)(B + rev_bits(bh * bl * 1.1f));
            cp.ss[s++] = {e, 0};
            cp.ss[s++] = {e, 0};
            cp.ss[s++] = {(uint32_t)(B + rev_bits(bh * bh * 1.1f)), 0};
        }
    } else {
        // set_irrev_quant (HTParams.cpp:210-253), base_delta = 2^-(prec+sgnd)
        const float base = 1.0f / (float)(1u << (cp.prec[0] + (uint32_t)cp.sgnd[0]));
        float gl = kGain97L[nd];
        cp.ss[s++] = irrev_step(base / (gl * gl));
        for (int d = (int)nd - 1; d >= 0; --d) {
            float l = kGain97L[d + 1], h = kGain97H[d];
            StepSize t = irrev_step(base / (l * h));
            cp.ss[s++] = t;
            cp.ss[s++] = t;
            cp.ss[s++] = irrev_step(base / (h * h));
        }
    }
    cp.nsteps = s;
    sync_comps(cp);
}

void comp_style_from_cod(CodingParams &cp, uint32_t k) {
    CompParams &c = cp.comp[k];
    c.numres = cp.numres; c.cblkw = cp.cblkw; c.cblkh = cp.cblkh; c.cblksty = cp.cblksty; c.irrev = cp.irrev;
    c.csty = cp.csty & CSTY_PRT;
    memcpy(c.prcw, cp.prcw, sizeof(c.prcw));
    memcpy(c.prch, cp.prch, sizeof(c.prch));
}

void comp_quant_from_qcd(CodingParams &cp, uint32_t k) {
    CompParams &c = cp.comp[k];
    c.qntsty = cp.qntsty; c.numgbits = cp.numgbits; c.nsteps = cp.nsteps;
    memcpy(c.ss, cp.ss, sizeof(c.ss));
}

void sync_comps(CodingParams &cp) {
    for (uint32_t k = 0; k < 16; ++k) {
        comp_style_from_cod(cp, k);
        comp_quant_from_qcd(cp, k);
    }
}

// ---------------------------------------------------------------------------
// geometry (TileComponent.cpp:165-507, Quantizer.cpp:65-104, Tier1.cpp:49-62)
// ---------------------------------------------------------------------------
Rect tile_rect(const CodingParams &cp, uint32_t tileno) {
    uint32_t p = tileno % cp.tw, q = tileno / cp.tw;
    uint32_t x0 = cp.tx0 + p * cp.tdx, y0 = cp.ty0 + q * cp.tdy;
    Rect r;
    r.x0 = std::max(x0, cp.image.x0);
    r.y0 = std::max(y0, cp.image.y0);
    r.x1 = (uint32_t)std::min<uint64_t>((uint64_t)x0 + cp.tdx, cp.image.x1);
    r.y1 = (uint32_t)std::min<uint64_t>((uint64_t)y0 + cp.tdy, cp.image.y1);
    return r;
}

void TagTree::init(uint32_t nh, uint32_t nv) {
    uint32_t nplh[40], nplv[40], lv = 0, n, total = 0;
    nplh[0] = nh; nplv[0] = nv;
    do {
        n = nplh[lv] * nplv[lv];
        nplh[lv + 1] = (nplh[lv] + 1) / 2;
        nplv[lv + 1] = (nplv[lv] + 1) / 2;
        total += n;
        ++lv;
    } while (n > 1);
    nodes.assign(total ? total : 1, Node{INT64_MAX, 0, -1, 0});
    uint32_t base = 0, pbase = nh * nv;
    for (uint32_t l = 0; l + 1 < lv; ++l) {
        for (uint32_t j = 0; j < nplv[l]; ++j)
            for (uint32_t i = 0; i < nplh[l]; ++i)
                nodes[base + j * nplh[l] + i].parent = (int32_t)(pbase + (j >> 1) * nplh[l + 1] + (i >> 1));
        base = pbase;
        pbase += nplh[l + 1] * nplv[l + 1];
    }
    nodes.back().parent = -1;
}

void TagTree::reset() {
    for (auto &n : nodes) { n.value = INT64_MAX; n.low = 0; n.known = 0; }
}

void TagTree::setvalue(uint32_t leaf, int64_t v) {
    int32_t n = (int32_t)leaf;
    while (n >= 0 && nodes[n].value > v) { nodes[n].value = v; n = nodes[n].parent; }
}

Rect comp_rect(const Rect &r, uint32_t dx, uint32_t dy) {
    return {ceildiv(r.x0, dx), ceildiv(r.y0, dy), ceildiv(r.x1, dx), ceildiv(r.y1, dy)};
}

void build_tilecomp(TileComp &tc, const Rect &tile_r, const CodingParams &cp, uint32_t compno, bool encoder) {
    const CompParams &cc = cp.comp[compno];  // the component's COD / COC and QCD / QCC
    // the tile-component on the component's subsampled grid (TileComponent.cpp:193-196)
    const Rect tr = comp_rect(tile_r, cp.dx[compno], cp.dy[compno]);
    tc.r = tr;
    tc.numres = cc.numres;
    tc.irrev = cc.irrev;
    tc.res.assign(cc.numres, Resolution());
    for (uint32_t resno = 0; resno < cc.numres; ++resno) {
        Resolution &res = tc.res[resno];
        const uint32_t lev = cc.numres - 1 - resno;
        res.r = {ceildivpow2(tr.x0, lev), ceildivpow2(tr.y0, lev), ceildivpow2(tr.x1, lev), ceildivpow2(tr.y1, lev)};
        const uint32_t pdx = cc.prcw[resno], pdy = cc.prch[resno];  // log2 precinct size (COD SPcod I_i)
        uint32_t tpx0 = (res.r.x0 >> pdx) << pdx, tpy0 = (res.r.y0 >> pdy) << pdy;
        uint32_t bpx1 = ceildivpow2(res.r.x1, pdx) << pdx, bpy1 = ceildivpow2(res.r.y1, pdy) << pdy;
        res.pw = (res.r.x0 == res.r.x1) ? 0 : ((bpx1 - tpx0) >> pdx);
        res.ph = (res.r.y0 == res.r.y1) ? 0 : ((bpy1 - tpy0) >> pdy);
        uint32_t tlcbgx, tlcbgy, cbgw, cbgh;
        if (resno == 0) { tlcbgx = tpx0; tlcbgy = tpy0; cbgw = pdx; cbgh = pdy; res.numbands = 1; }
        else { tlcbgx = ceildivpow2(tpx0, 1); tlcbgy = ceildivpow2(tpy0, 1); cbgw = pdx - 1; cbgh = pdy - 1; res.numbands = 3; }
        const uint32_t cbw = std::min(cc.cblkw, cbgw), cbh = std::min(cc.cblkh, cbgh);
        for (uint32_t bandno = 0; bandno < res.numbands; ++bandno) {
            Band &b = res.bands[bandno];
            if (resno == 0) {
                b.bandno = 0;
                b.r = {ceildivpow2(tr.x0, lev), ceildivpow2(tr.y0, lev), ceildivpow2(tr.x1, lev), ceildivpow2(tr.y1, lev)};
            } else {
                b.bandno = bandno + 1;
                uint64_t x0b = b.bandno & 1, y0b = b.bandno >> 1, d = (uint64_t)1 << (lev + 1);
                b.r.x0 = (uint32_t)(((uint64_t)tr.x0 - (x0b << lev) + d - 1) >> (lev + 1));
                b.r.y0 = (uint32_t)(((uint64_t)tr.y0 - (y0b << lev) + d - 1) >> (lev + 1));
                b.r.x1 = (uint32_t)(((uint64_t)tr.x1 - (x0b << lev) + d - 1) >> (lev + 1));
                b.r.y1 = (uint32_t)(((uint64_t)tr.y1 - (y0b << lev) + d - 1) >> (lev + 1));
            }
            // Quantizer::setBandStepSizeAndBps (Quantizer.cpp:65-104)
            uint32_t gain = cc.irrev ? 0 : (b.bandno == 0 ? 0 : (b.bandno < 3 ? 1 : 2));
            uint32_t numbps = cp.prec[compno] + gain;
            uint32_t off = resno == 0 ? 0 : 3 * resno - 2;
            const StepSize &st = cc.ss[off + bandno];
            b.stepsize = (float)((1.0 + st.mant / 2048.0) * std::pow(2.0, (int32_t)(numbps - st.expn))) *
                         (encoder ? 1.0f : 0.5f);
            b.numbps = cp.roishift[compno] + st.expn + cc.numgbits - 1;  // + ROI (Quantizer.cpp:90-93)
            b.inv_step = (uint32_t)((8192.0 / b.stepsize) + 0.5f);
            uint32_t np = res.pw * res.ph;
            b.precs.assign(np, Precinct());
            for (uint32_t precno = 0; precno < np; ++precno) {
                Precinct &pr = b.precs[precno];
                uint32_t cbgx0 = tlcbgx + (precno % res.pw) * (1u << cbgw);
                uint32_t cbgy0 = tlcbgy + (precno / res.pw) * (1u << cbgh);
                pr.r = {std::max(cbgx0, b.r.x0), std::max(cbgy0, b.r.y0), std::min(cbgx0 + (1u << cbgw), b.r.x1),
                        std::min(cbgy0 + (1u << cbgh), b.r.y1)};
                if (pr.r.x1 <= pr.r.x0 || pr.r.y1 <= pr.r.y0) { pr.cw = pr.ch = 0; continue; }
                uint32_t tlx = (pr.r.x0 >> cbw) << cbw, tly = (pr.r.y0 >> cbh) << cbh;
                uint32_t brx = ceildivpow2(pr.r.x1, cbw) << cbw, bry = ceildivpow2(pr.r.y1, cbh) << cbh;
                pr.cw = (brx - tlx) >> cbw;
                pr.ch = (bry - tly) >> cbh;
                pr.cblks.assign(pr.cw * pr.ch, Cblk());
                for (uint32_t cb = 0; cb < pr.cw * pr.ch; ++cb) {
                    Cblk &c = pr.cblks[cb];
                    uint32_t cx0 = tlx + (cb % pr.cw) * (1u << cbw), cy0 = tly + (cb / pr.cw) * (1u << cbh);
                    c.r = {std::max(cx0, pr.r.x0), std::max(cy0, pr.r.y0), std::min(cx0 + (1u << cbw), pr.r.x1),
                           std::min(cy0 + (1u << cbh), pr.r.y1)};
                    c.bx = c.r.x0 - b.r.x0;
                    c.by = c.r.y0 - b.r.y0;
                    if (b.bandno & 1) c.bx += tc.res[resno - 1].r.w();
                    if (b.bandno & 2) c.by += tc.res[resno - 1].r.h();
                }
                pr.incl.init(pr.cw, pr.ch);
                pr.imsb.init(pr.cw, pr.ch);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// headers (codestream/j2k.cpp marker writers :3117-5540)
// ---------------------------------------------------------------------------
void write_poc(ByteBuf &cs, const CodingParams &cp) {
    const uint32_t n = cp.numpocs, room = cp.numcomps <= 256 ? 1 : 2;
    cs.put16(0xFF5F); cs.put16(2 + (5 + 2 * room) * n);  // Lpoc = getPocSize - 2 (j2k.cpp:4208-4216)
    for (uint32_t i = 0; i < n; ++i) {
        const PocSpec &q = cp.pocs[i];
        cs.put8(q.resno0);
        if (room == 2) cs.put16(q.compno0); else cs.put8(q.compno0);
        cs.put16(q.layno1);
        cs.put8(q.resno1);
        if (room == 2) cs.put16(q.compno1); else cs.put8(q.compno1);
        cs.put8(q.prg);
    }
}

void write_main_header(ByteBuf &cs, const CodingParams &cp, size_t *tlm_at, uint32_t total_tile_parts) {
    const uint32_t nc = cp.numcomps, nd = cp.numres - 1, nb = 3 * nd + 1;
    const bool prt = (cp.csty & CSTY_PRT) != 0;
    cs.put16(0xFF4F);  // SOC
    cs.put16(0xFF51); cs.put16(38 + 3 * nc); cs.put16(cp.rsiz);  // SIZ
    cs.put32(cp.image.x1); cs.put32(cp.image.y1); cs.put32(cp.image.x0); cs.put32(cp.image.y0);
    cs.put32(cp.tdx); cs.put32(cp.tdy); cs.put32(cp.tx0); cs.put32(cp.ty0);
    cs.put16(nc);
    for (uint32_t k = 0; k < nc; ++k) {
        cs.put8((cp.prec[k] - 1) + ((uint32_t)cp.sgnd[k] << 7));
        cs.put8(cp.dx[k]);
        cs.put8(cp.dy[k]);
    }
    // COD (j2k_write_cod + j2k_write_SPCod_SPCoc, j2k.cpp:3723-3770, 6905-6950)
    cs.put16(0xFF52); cs.put16(12 + (prt ? cp.numres : 0));
    cs.put8(cp.csty); cs.put8(cp.prog); cs.put16(cp.numlayers); cs.put8((uint32_t)cp.mct);
    cs.put8(nd); cs.put8(cp.cblkw - 2); cs.put8(cp.cblkh - 2); cs.put8(cp.cblksty); cs.put8(cp.irrev ? 0 : 1);
    if (prt)
        for (uint32_t r = 0; r < cp.numres; ++r) cs.put8(cp.prcw[r] + (cp.prch[r] << 4));
    cs.put16(0xFF5C); cs.put16(3 + nb * (cp.irrev ? 2 : 1));  // QCD
    cs.put8((cp.numgbits << 5) | (cp.irrev ? 2u : 0u));
    for (uint32_t i = 0; i < nb; ++i) {
        if (cp.irrev) cs.put16((cp.ss[i].expn << 11) | cp.ss[i].mant);
        else cs.put8(cp.ss[i].expn << 3);
    }
    if (tlm_at) *tlm_at = 0;
    if (cp.rsiz == RSIZ_CINEMA_2K || cp.rsiz == RSIZ_CINEMA_4K) {
        // TLM (j2k_write_tlm, j2k.cpp:5027-5063): Ztlm 0, Stlm 0x50 (8-bit
        // tile index, 32-bit lengths); records patched once every tile-part is
        // written (j2k_write_updated_tlm, :2555-2577)
        cs.put16(0xFF55); cs.put16(4 + 5 * total_tile_parts); cs.put8(0); cs.put8(0x50);
        if (tlm_at) *tlm_at = cs.size();
        for (uint32_t i = 0; i < 5 * total_tile_parts; ++i) cs.put8(0);
        if (cp.rsiz == RSIZ_CINEMA_4K) write_poc(cs, cp);  // main-header POC (j2k.cpp:2353-2356)
    }
    // RGN per ROI component (j2k_write_regions / j2k_write_rgn, j2k.cpp:5482-5531, 5687-5706):
    // Crgn (1 or 2 bytes), Srgn 0, SPrgn = roishift
    for (uint32_t k = 0; k < cp.numcomps; ++k) {
        if (!cp.roishift[k]) continue;
        const uint32_t room = cp.numcomps <= 256 ? 1 : 2;
        cs.put16(0xFF5E); cs.put16(4 + room);
        if (room == 2) cs.put16(k); else cs.put8(k);
        cs.put8(0); cs.put8(cp.roishift[k]);
    }
    static const char kCom[] = "Created by Grok     version 5.1.0";  // j2k.cpp:1798
    cs.put16(0xFF64); cs.put16(4 + (uint32_t)strlen(kCom)); cs.put16(1);
    cs.putn((const uint8_t *)kCom, strlen(kCom));
    if ((cp.rsiz & (RSIZ_PART2 | RSIZ_EXT_MCT)) == (RSIZ_PART2 | RSIZ_EXT_MCT)) write_mct_group(cs, cp);
}

// The Part-2 array-based MCT marker group (j2k_write_mct_data_group,
// j2k.cpp:5615-5652, with the records j2k_setup_mct_encoding makes,
// :2580-2741): CBD (component bit depths), an MCT record holding the
// decoding matrix (index 1, decorrelation array, float elements), one
// holding the DC shifts (index 2, offset array, float), an MCC collection
// (index 3, irreversible, array 1 + offsets 2, components in order) and MCO
// naming it.  Floats big-endian, as grk_write_float writes them.
static void put_float(ByteBuf &cs, float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    cs.put32(u);
}
void write_mct_group(ByteBuf &cs, const CodingParams &cp) {
    const uint32_t n = cp.numcomps;
    cs.put16(0xFF78); cs.put16(4 + n); cs.put16(n);  // CBD (j2k_write_cbd, :6476-6510)
    for (uint32_t k = 0; k < n; ++k) cs.put8(((uint32_t)cp.sgnd[k] << 7) | (cp.prec[k] - 1));
    enum { ARRAY_DECORRELATION = 1, ARRAY_OFFSET = 2, ELEM_FLOAT = 2 };
    auto mct_head = [&](uint32_t index, uint32_t array, uint32_t nbytes) {  // j2k_write_mct_record (:5779-5822)
        cs.put16(0xFF74); cs.put16(8 + nbytes);
        cs.put16(0);                                                   // Zmct
        cs.put16((index & 0xff) | (array << 8) | (ELEM_FLOAT << 10));  // Imct
        cs.put16(0);                                                   // Ymct
    };
    mct_head(1, ARRAY_DECORRELATION, 4 * n * n);
    for (uint32_t i = 0; i < n * n; ++i) put_float(cs, cp.mct_decoding[i]);
    mct_head(2, ARRAY_OFFSET, 4 * n);
    for (uint32_t k = 0; k < n; ++k) put_float(cs, (float)cp.shift[k]);
    // MCC (j2k_write_mcc_record, :5961-6070): one collection, 1- or 2-byte component indices
    const uint32_t cb = n > 255 ? 2 : 1, mask = n > 255 ? 0x8000 : 0;
    cs.put16(0xFF75); cs.put16(17 + 2 * n * cb);
    cs.put16(0); cs.put8(3); cs.put16(0); cs.put16(1); cs.put8(1);
    for (int side = 0; side < 2; ++side) {
        cs.put16(n | mask);
        for (uint32_t k = 0; k < n; ++k) { if (cb == 2) cs.put16(k); else cs.put8(k); }
    }
    const uint32_t tmcc = (0u << 16) | (2u << 8) | 1u;  // irreversible, offsets = record 2, matrix = record 1
    cs.put8(tmcc >> 16); cs.put8((tmcc >> 8) & 0xff); cs.put8(tmcc & 0xff);
    cs.put16(0xFF77); cs.put16(4); cs.put8(1); cs.put8(3);  // MCO (j2k_write_mco, :6298-6333)
}

// matrix_inversion_f (mct/invert.cpp:78-286), restated: an LU decomposition
// with row pivoting on the largest |value| of each column (in float, a
// separate multiply and subtract per update), then one forward / back
// substitution per unit vector.  false for a singular matrix.
bool mct_invert(const float *src_in, float *dst, uint32_t n) {
    std::vector<float> a(src_in, src_in + (size_t)n * n);
    std::vector<uint32_t> perm(n);
    for (uint32_t i = 0; i < n; ++i) perm[i] = i;
    for (uint32_t k = 0; k + 1 < n; ++k) {
        float p = 0.0f;
        uint32_t k2 = 0;
        for (uint32_t i = k; i < n; ++i) {
            const float v = a[(size_t)i * n + k];
            const float m = v > 0 ? v : -v;
            if (m > p) { p = m; k2 = i; }
        }
        if (p == 0.0f) return false;
        if (k2 != k) {
            std::swap(perm[k], perm[k2]);
            for (uint32_t j = 0; j < n; ++j) std::swap(a[(size_t)k * n + j], a[(size_t)k2 * n + j]);
        }
        const float d = a[(size_t)k * n + k];
        for (uint32_t i = k + 1; i < n; ++i) {
            const float f = a[(size_t)i * n + k] / d;
            a[(size_t)i * n + k] = f;
            for (uint32_t j = k + 1; j < n; ++j) {
                const float prod = f * a[(size_t)k * n + j];
                a[(size_t)i * n + j] = a[(size_t)i * n + j] - prod;
            }
        }
    }
    std::vector<float> y(n), x(n), e(n);
    for (uint32_t col = 0; col < n; ++col) {
        for (uint32_t i = 0; i < n; ++i) e[i] = i == col ? 1.0f : 0.0f;
        for (uint32_t i = 0; i < n; ++i) {  // L y = P e (unit lower triangle)
            float sum = 0.0f;
            for (uint32_t j = 0; j < i; ++j) { const float t = a[(size_t)i * n + j] * y[j]; sum = sum + t; }
            y[i] = e[perm[i]] - sum;
        }
        for (int32_t k = (int32_t)n - 1; k >= 0; --k) {  // U x = y
            float sum = 0.0f;
            for (uint32_t j = (uint32_t)k + 1; j < n; ++j) { const float t = a[(size_t)k * n + j] * x[j]; sum = sum + t; }
            x[k] = (y[k] - sum) / a[(size_t)k * n + k];
        }
        for (uint32_t i = 0; i < n; ++i) dst[(size_t)i * n + col] = x[i];
    }
    return true;
}

// ---------------------------------------------------------------------------
// packet header bit writer (codestream/BitIO.cpp)
// ---------------------------------------------------------------------------
namespace {
struct BitReader {
    const uint8_t *p;
    size_t n, off = 0;
    uint32_t buf = 0, ct = 0;
    uint32_t fails = 0;  // reads that ran out of bytes (BitIO::bytein returning false, BitIO.cpp:95-104)
    BitReader(const uint8_t *pp, size_t nn) : p(pp), n(nn) {}
    // past the end the reader keeps its state (ct stays 0): every later read
    // fails too, and a failed read leaves the bits it got at the top of the
    // value, zeros below (BitIO::read, BitIO.cpp:143-160)
    bool bytein() {
        if (off >= n) { ++fails; return false; }
        ct = (buf == 0xff) ? 7 : 8;
        buf = p[off++];
        return true;
    }
    uint32_t bit() { if (ct == 0 && !bytein()) return 0; ct--; return (buf >> ct) & 1; }
    uint32_t read(uint32_t k) { uint32_t v = 0; for (uint32_t i = 0; i < k; ++i) v = (v << 1) | bit(); return v; }
    bool align() { if (buf == 0xff && !bytein()) return false; ct = 0; return true; }  // BitIO::inalign
    uint32_t numpasses() {
        if (!read(1)) return 1;
        if (!read(1)) return 2;
        uint32_t v = read(2);
        if (v != 3) return v + 3;
        v = read(5);
        if (v != 31) return v + 6;
        return read(7) + 37;
    }
    uint32_t comma() { uint32_t k = 0, f = fails; while (bit() && fails == f) ++k; return k; }
    // TagTree::decodeValue (TagTree.cpp:295-321)
    int64_t tagtree(TagTree &t, uint32_t leaf, int64_t threshold) {
        int32_t stk[64], sp = 0, node = (int32_t)leaf;
        while (t.nodes[node].parent >= 0) { stk[sp++] = node; node = t.nodes[node].parent; }
        int64_t low = 0;
        for (;;) {
            TagTree::Node &nd = t.nodes[node];
            if (low > nd.low) nd.low = low; else low = nd.low;
            while (low < threshold && low < nd.value) {
                const uint32_t f = fails;
                const uint32_t b = bit();
                if (fails != f) return INT64_MAX;
                if (b) nd.value = low; else ++low;
            }
            nd.low = low;
            if (sp == 0) break;
            node = stk[--sp];
        }
        return t.nodes[node].value;
    }
};
}  // namespace

int64_t decode_packet(TileComp &tc, uint32_t resno, uint32_t precno, uint32_t layno, const uint8_t *p, size_t n,
                      uint64_t base_off, uint32_t csty, uint32_t *packno, bool skip_data, uint32_t cblksty,
                      PackedHdr *hdr) {
    // passes per codeword segment (T2::init_seg, T2.cpp:821-850): 1 when every
    // pass is terminated; BYPASS: 10 for the first, then 2 (raw) and 1 (MQ)
    // alternately; else 109 (a longer block is cut there, T2.cpp:566-577)
    auto seg_max = [cblksty](const Cblk &c) -> uint32_t {
        if (cblksty & 0x04) return 1;
        if (cblksty & 0x01) {
            if (c.segs.empty()) return 10;
            const uint32_t pm = c.segs.back().maxpasses;
            return (pm == 1 || pm == 10) ? 2 : 1;
        }
        return 109;
    };
    const bool single = !(cblksty & 0x05);
    Resolution &res = tc.res[resno];
    if (layno == 0) {
        for (uint32_t bandno = 0; bandno < res.numbands; ++bandno) {
            Band &b = res.bands[bandno];
            if (b.empty() || precno >= b.precs.size()) continue;
            Precinct &pr = b.precs[precno];
            if (pr.cblks.empty()) continue;
            pr.incl.reset(); pr.imsb.reset();
            for (auto &c : pr.cblks) { c.included = false; c.numpasses = 0; c.segs.clear(); c.seglen = 0; }
        }
    }
    size_t hstart = 0;
    // SOP (T2::read_packet_header, T2.cpp:346-365): a missing marker is only a
    // warning there; a packet counter that does not match is an error
    if (csty & CSTY_SOP) {
        if (n >= 6 && p[0] == 0xFF && p[1] == 0x91) {
            const uint32_t cnt = ((uint32_t)p[4] << 8) | p[5];
            if (packno) {
                if (cnt != (*packno & 0xFFFF)) return -1;
                ++*packno;
            }
            hstart = 6;
        }
    }
    // the header bits: in the packet (after the SOP), or the packed headers
    // of the tile (PPT) / tile-part (PPM) when the stream carries them there
    // (T2::read_packet_header, T2.cpp:366-392)
    const uint8_t *hp = hdr ? hdr->p + hdr->off : p + hstart;
    const size_t hn = hdr ? (hdr->off <= hdr->n ? hdr->n - hdr->off : 0) : n - hstart;
    BitReader r(hp, hn);
    struct Part { Cblk *c; uint32_t seg, passes, len; };  // one segment's share of this packet
    std::vector<Part> parts;
    if (hn && r.read(1)) {
        for (uint32_t bandno = 0; bandno < res.numbands; ++bandno) {
            Band &b = res.bands[bandno];
            if (b.empty() || precno >= b.precs.size()) continue;
            Precinct &pr = b.precs[precno];
            if (pr.cblks.empty()) continue;
            for (uint32_t cb = 0; cb < pr.cblks.size(); ++cb) {
                Cblk &c = pr.cblks[cb];
                // a read past the header's bytes fails the packet -- except a
                // segment length's, which T2.cpp:595-598 only warns about
                // (the bits read so far, zeros below, are its value)
                const uint32_t f0 = r.fails;
                uint32_t inc = c.included ? r.read(1) : (r.tagtree(pr.incl, cb, layno + 1) <= (int64_t)layno);
                if (r.fails != f0) return -1;
                if (!inc) continue;
                if (!c.included) {
                    int64_t k = r.tagtree(pr.imsb, cb, INT64_MAX);
                    if (r.fails != f0 || k < 0) return -1;
                    // more missing bit-planes than the band has: the reference
                    // warns and takes the band's count (T2.cpp:516-521)
                    c.numbps = k > (int64_t)b.numbps ? b.numbps : (uint32_t)((int64_t)b.numbps - k);
                    if (c.numbps > 16 + 33 * 5) return -1;  // T2.cpp:523-529
                    c.numlenbits = 3;
                    c.included = true;
                }
                uint32_t np = r.numpasses();
                if (r.fails != f0) return -1;
                c.numlenbits += r.comma();
                if (r.fails != f0) return -1;
                if (single && np > 109) np = 109;  // single segment: truncated (T2.cpp:566-577)
                // the packet's passes fill the open segment, then new ones
                // (T2::read_packet_header, T2.cpp:560-605)
                auto open_seg = [&]() {
                    const uint32_t m = seg_max(c);
                    c.segs.emplace_back();
                    c.segs.back().maxpasses = m;
                };
                if (c.segs.empty() || c.segs.back().numpasses == c.segs.back().maxpasses) open_seg();
                uint32_t left = np;
                while (left) {
                    const uint32_t si = (uint32_t)c.segs.size() - 1;
                    const uint32_t take = std::min(left, c.segs[si].maxpasses - c.segs[si].numpasses);
                    const uint32_t bits = c.numlenbits + (uint32_t)floorlog2((int32_t)take);
                    if (bits > 32) return -1;  // "too many bits in segment length", T2.cpp:590-593
                    const uint32_t L = r.read(bits);
                    parts.push_back({&c, si, take, L});
                    c.segs[si].numpasses += take;
                    left -= take;
                    if (left) open_seg();
                }
                c.numpasses += np;
            }
        }
    }
    if (!r.align()) return -1;
    // EPH (T2.cpp:405-418 / 640-652): skipped when present -- it ends the
    // header, wherever the header is
    size_t hoff = r.off;
    if ((csty & CSTY_EPH) && hoff + 2 <= hn && hp[hoff] == 0xFF && hp[hoff + 1] == 0x92) hoff += 2;
    size_t off = hstart;
    if (hdr) hdr->off += hoff;
    else off += hoff;
    for (auto &pt : parts) {
        // T2::read_packet_data (T2.cpp:686-698): a segment running past the
        // tile data is truncated to what is there (the decoder reads the
        // missing tail as the 0xFF fill), not an error
        if (off + pt.len > n) pt.len = (uint32_t)(n - off);
        // a layer beyond the decoded ones (T2::skip_packet_data, T2.cpp:
        // 758-819): its passes still count, its bytes are stepped over
        if (!skip_data) {
            Cblk::Seg &sg = pt.c->segs[pt.seg];
            if (pt.len) sg.chunks.push_back({base_off + off, pt.len});
            sg.len += pt.len;
            pt.c->seglen += pt.len;
        }
        off += pt.len;
    }
    return (int64_t)off;
}

// ---------------------------------------------------------------------------
// main header parsing (j2k.cpp j2k_read_siz / cod / qcd)
// ---------------------------------------------------------------------------
static uint32_t rd16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t rd32(const uint8_t *p) { return (rd16(p) << 16) | rd16(p + 2); }

// POC marker body (j2k_read_poc, j2k.cpp:4367-4440): entries are appended;
// layno1 / compno1 are clamped to the layer / component counts.
bool parse_poc(const uint8_t *p, uint32_t size, CodingParams &cp) {
    const uint32_t room = cp.numcomps <= 256 ? 1 : 2, chunk = 5 + 2 * room;
    if (!size || size % chunk) return false;
    const uint32_t n = cp.numpocs + size / chunk;
    if (n >= 32) return false;
    for (uint32_t i = cp.numpocs; i < n; ++i) {
        PocSpec &q = cp.pocs[i];
        q.resno0 = p[0];
        q.compno0 = room == 2 ? rd16(p + 1) : p[1];
        p += 1 + room;
        q.layno1 = std::min<uint32_t>(rd16(p), cp.numlayers);
        q.resno1 = p[2];
        q.compno1 = room == 2 ? rd16(p + 3) : p[3];
        p += 3 + room;
        q.prg = p[0];
        p += 1;
        q.compno1 = std::min<uint32_t>(q.compno1, cp.numcomps);
        if (q.prg > 4) return false;
    }
    cp.numpocs = n;
    return true;
}

// SPcod / SPcoc (j2k_read_SPCod_SPCoc, j2k.cpp:6978-7025): decomposition
// levels, code-block size and style, transform, precinct sizes; prt: the
// Scod / Scoc precinct flag
static bool parse_spcod(const uint8_t *p, uint32_t size, bool prt, CompParams &c, std::string &err) {
    if (size < 5) { err = "Error reading SPCod SPCoc element"; return false; }
    c.numres = p[0] + 1u; c.cblkw = p[1] + 2u; c.cblkh = p[2] + 2u; c.cblksty = p[3];
    c.irrev = p[4] == 0;
    c.csty = prt ? 1u : 0u;
    if (c.numres > 33) { err = "Number of resolutions is greater than GRK_J2K_MAXRLVLS"; return false; }
    if (p[1] > 8 || p[2] > 8 || p[1] + p[2] > 8) { err = "Error reading SPCod SPCoc element, invalid code-block size"; return false; }
    if (p[4] > 1) { err = "Invalid qmfbid"; return false; }
    if (prt) {
        if (size != 5 + c.numres) { err = "Error reading SPCod SPCoc element"; return false; }
        for (uint32_t r = 0; r < c.numres; ++r) {
            c.prcw[r] = p[5 + r] & 0xf;
            c.prch[r] = p[5 + r] >> 4;
            if (r && (!c.prcw[r] || !c.prch[r])) { err = "invalid precinct size"; return false; }
        }
    } else {
        if (size != 5) { err = "Error reading SPCod SPCoc element"; return false; }
        for (uint32_t r = 0; r < c.numres; ++r) c.prcw[r] = c.prch[r] = 15;
    }
    return true;
}

bool parse_cod(const uint8_t *p, uint32_t size, CodingParams &cp, std::string &err) {
    // j2k_read_cod (j2k.cpp:3829-3884): Scod, SGcod (progression, layers, MCT), SPcod
    if (size < 10) { err = "Error reading COD marker"; return false; }
    if (p[0] & ~7u) { err = "unknown Scod bits"; return false; }
    cp.csty = p[0];
    cp.prog = p[1]; cp.numlayers = rd16(p + 2); cp.mct = p[4];
    if (cp.mct > 1) { err = "Invalid MCT value: should be either 0 or 1"; return false; }  // j2k.cpp:3869-3872
    if (cp.numlayers == 0) { err = "Invalid number of layers in COD marker"; return false; }
    if (cp.prog > 4) { err = "Unknown progression order in COD marker"; return false; }
    CompParams c;
    if (!parse_spcod(p + 5, size - 5, (cp.csty & CSTY_PRT) != 0, c, err)) return false;
    cp.numres = c.numres; cp.cblkw = c.cblkw; cp.cblkh = c.cblkh; cp.cblksty = c.cblksty; cp.irrev = c.irrev;
    memcpy(cp.prcw, c.prcw, sizeof(cp.prcw));
    memcpy(cp.prch, c.prch, sizeof(cp.prch));
    return true;
}

int32_t parse_coc(const uint8_t *p, uint32_t size, CodingParams &cp, std::string &err) {
    const uint32_t room = cp.numcomps <= 256 ? 1 : 2;
    if (size < room + 1) { err = "Error reading COC marker"; return -1; }
    const uint32_t k = room == 2 ? rd16(p) : p[0];
    if (k >= cp.numcomps) { err = "Error reading COC marker (bad number of components)"; return -1; }
    if (p[room] & ~1u) { err = "unknown Scoc bits"; return -1; }
    CompParams c = cp.comp[k];
    if (!parse_spcod(p + room + 1, size - room - 1, (p[room] & 1) != 0, c, err)) return -1;
    CompParams &d = cp.comp[k];
    d.numres = c.numres; d.cblkw = c.cblkw; d.cblkh = c.cblkh; d.cblksty = c.cblksty; d.irrev = c.irrev;
    d.csty = c.csty;
    memcpy(d.prcw, c.prcw, sizeof(d.prcw));
    memcpy(d.prch, c.prch, sizeof(d.prch));
    return (int32_t)k;
}

// SQcd / SQcc + SPqcd / SPqcc (j2k_read_SQcd_SQcc, j2k.cpp:7047-7135): the
// style (0 none: 8-bit exponents; 2 scalar expounded: 16-bit expn / mantissa),
// guard bits, one step size per band
// Style 1 (scalar derived) carries one step size; band b >= 1 then gets
// expn0 - (b - 1) / 3 (not below 0) and mant0 (Quantizer.cpp:326-336).  The
// marker must hold exactly its step sizes (j2k_read_qcd / _qcc: bytes left
// over are an error).
static bool parse_sqcd(const uint8_t *p, uint32_t size, CompParams &c, std::string &err) {
    if (size < 1) { err = "Error reading SQcd or SQcc element"; return false; }
    const uint32_t sq = p[0] & 0x1f;
    if (sq > 2) { err = "unknown quantisation style"; return false; }
    c.numgbits = p[0] >> 5;
    const uint32_t body = size - 1;
    const uint32_t nb = sq == 0 ? body : (sq == 1 ? 1 : body / 2);
    if ((sq == 0 && body != nb) || (sq != 0 && body != 2 * nb)) { err = "Error reading QCD marker"; return false; }
    c.qntsty = sq;
    c.nsteps = std::min<uint32_t>(nb, 3 * 33 + 1);
    for (uint32_t i = 0; i < c.nsteps; ++i) {
        if (sq == 0) c.ss[i] = {(uint32_t)(p[1 + i] >> 3), 0};
        else { const uint32_t v = rd16(p + 1 + 2 * i); c.ss[i] = {v >> 11, v & 0x7ff}; }
    }
    if (sq == 1)
        for (uint32_t b = 1; b < 3 * 33 + 1; ++b) {
            const uint32_t d = (b - 1) / 3;
            c.ss[b] = {c.ss[0].expn > d ? c.ss[0].expn - d : 0, c.ss[0].mant};
        }
    return true;
}

bool check_qcd_steps(const CodingParams &cp, const bool *qcc, bool tile_qcd, const bool *tile_qcc, std::string &err) {
    // j2k.cpp:868-930: the main QCD's step sizes must cover the deepest
    // component it governs (3 L + 1), and so must a tile QCD's
    if (cp.main_qntsty == 1) return true;
    uint32_t dmax = 0;
    for (uint32_t k = 0; k < cp.numcomps; ++k)
        if (!qcc[k] && !tile_qcd && !tile_qcc[k]) dmax = std::max(dmax, cp.comp[k].numres - 1);
    if (cp.main_nsteps < 3 * dmax + 1) {
        err = "From Main QCD marker, number of step sizes is less than 3 * (tile decompositions) + 1";
        return false;
    }
    if (tile_qcd && cp.qntsty != 1) {
        dmax = 0;
        for (uint32_t k = 0; k < cp.numcomps; ++k)
            if (!tile_qcc[k]) dmax = std::max(dmax, cp.comp[k].numres - 1);
        if (cp.nsteps < 3 * dmax + 1) {
            err = "From Tile QCD marker, number of step sizes is less than 3 * (tile decompositions) + 1";
            return false;
        }
    }
    return true;
}

bool parse_qcd(const uint8_t *p, uint32_t size, CodingParams &cp, std::string &err) {
    if (size < 2) { err = "Error reading QCD marker"; return false; }  // j2k.cpp:4075
    CompParams c;
    if (!parse_sqcd(p, size, c, err)) return false;
    cp.qntsty = c.qntsty; cp.numgbits = c.numgbits; cp.nsteps = c.nsteps;
    memcpy(cp.ss, c.ss, sizeof(cp.ss));
    return true;
}

int32_t parse_qcc(const uint8_t *p, uint32_t size, CodingParams &cp, std::string &err) {
    const uint32_t room = cp.numcomps <= 256 ? 1 : 2;
    if (size < room + 1) { err = "Error reading QCC marker"; return -1; }
    const uint32_t k = room == 2 ? rd16(p) : p[0];
    if (k >= cp.numcomps) { err = "Invalid component number in QCC marker"; return -1; }
    if (!parse_sqcd(p + room, size - room, cp.comp[k], err)) return -1;
    return (int32_t)k;
}

bool parse_main_header(const uint8_t *cs, size_t len, CodingParams &cp, size_t &first_sot, std::string &err) {
    if (len < 4 || rd16(cs) != 0xFF4F) { err = "missing SOC"; return false; }
    size_t pos = 2;
    first_sot = 0;
    bool have_siz = false, have_cod = false, have_qcd = false;
    while (pos + 4 <= len) {
        uint32_t m = rd16(cs + pos);
        if (m == 0xFF90) { first_sot = pos; break; }
        uint32_t L = rd16(cs + pos + 2);
        if (pos + 2 + L > len || L < 2) { err = "truncated marker"; return false; }
        const uint8_t *p = cs + pos + 4;
        if (m == 0xFF51) {
            cp.image = {rd32(p + 10), rd32(p + 14), rd32(p + 2), rd32(p + 6)};
            cp.tdx = rd32(p + 18); cp.tdy = rd32(p + 22); cp.tx0 = rd32(p + 26); cp.ty0 = rd32(p + 30);
            cp.numcomps = rd16(p + 34);
            // read_siz checks, j2k.cpp:3380-3480: marker length vs Csiz, non-empty
            // image, tile size, tile origin at or before the image origin
            if (L < 38) { err = "Error with SIZ marker size"; return false; }
            if (cp.numcomps == 0 || cp.numcomps > 16) { err = "unsupported component count"; return false; }
            if (L != 38 + 3 * cp.numcomps) { err = "Error with SIZ marker: number of components vs marker length"; return false; }
            if (cp.image.x0 >= cp.image.x1 || cp.image.y0 >= cp.image.y1) { err = "Error with SIZ marker: negative or zero image size"; return false; }
            for (uint32_t k = 0; k < cp.numcomps; ++k) {
                cp.prec[k] = (p[36 + 3 * k] & 0x7f) + 1u;
                cp.sgnd[k] = p[36 + 3 * k] >> 7;
                if (cp.prec[k] > 16) { err = "precision above 16 bits not supported"; return false; }
                cp.dx[k] = p[37 + 3 * k];
                cp.dy[k] = p[38 + 3 * k];
                if (!cp.dx[k] || !cp.dy[k]) { err = "Invalid component subsampling dx / dy (should be between 1 and 255 according to the JPEG2000 norm)"; return false; }
            }
            if (cp.tdx == 0 || cp.tdy == 0) { err = "bad tile size"; return false; }
            if (cp.tx0 > cp.image.x0 || cp.ty0 > cp.image.y0 || (uint64_t)cp.tx0 + cp.tdx <= cp.image.x0 ||
                (uint64_t)cp.ty0 + cp.tdy <= cp.image.y0) { err = "Error with SIZ marker: illegal tile offset"; return false; }
            cp.tw = ceildiv(cp.image.x1 - cp.tx0, cp.tdx);
            cp.th = ceildiv(cp.image.y1 - cp.ty0, cp.tdy);
            have_siz = true;
        } else if (m == 0xFF52) {
            if (!parse_cod(p, L - 2, cp, err)) return false;
            // COD sets every component (j2k_copy_tile_component_parameters,
            // j2k.cpp:3889): a COC read before it is overwritten
            for (uint32_t k = 0; k < 16; ++k) cp.coc_set[k] = false;
            have_cod = true;
        } else if (m == 0xFF5C) {
            if (!parse_qcd(p, L - 2, cp, err)) return false;
            cp.main_qntsty = cp.qntsty;
            cp.main_nsteps = cp.nsteps;
            have_qcd = true;
        } else if (m == 0xFF53) {  // COC (j2k_read_coc, j2k.cpp:3991-4060)
            if (!have_siz) { err = "COC before SIZ"; return false; }
            const int32_t k = parse_coc(p, L - 2, cp, err);
            if (k < 0) return false;
            cp.coc_set[k] = true;
        } else if (m == 0xFF5D) {  // QCC (j2k_read_qcc, j2k.cpp:4160-4200)
            if (!have_siz) { err = "QCC before SIZ"; return false; }
            const int32_t k = parse_qcc(p, L - 2, cp, err);
            if (k < 0) return false;
            cp.qcc_set[k] = true;
        } else if (m == 0xFF60) {  // PPM (j2k_read_ppm, j2k.cpp:4693-4765): Zppm, then Nppm / Ippm pairs
            if (L < 3) { err = "Error reading PPM marker"; return false; }
            for (auto &q : cp.ppm)
                if (q.z == p[0]) { err = "Zppm already read"; return false; }
            cp.ppm.push_back({p[0], pos + 5, (size_t)L - 3});
        } else if (m == 0xFF5F) {
            if (!parse_poc(p, L - 2, cp)) { err = "Error reading POC marker"; return false; }
        } else if (m == 0xFF5E) {  // RGN (j2k_read_rgn, j2k.cpp:5555-5604)
            if (!have_siz) { err = "RGN before SIZ"; return false; }
            const uint32_t room = cp.numcomps <= 256 ? 1 : 2;
            if (L - 2 != 2 + room) { err = "Error reading RGN marker"; return false; }
            const uint32_t comp = room == 2 ? rd16(p) : p[0];
            if (comp >= cp.numcomps) { err = "bad component number in RGN"; return false; }
            cp.roishift[comp] = p[room + 1];  // Srgn != 0 is only a warning there
        }
        pos += 2 + L;
    }
    if (!have_siz || !have_cod || !have_qcd) { err = "incomplete main header"; return false; }
    // COD / QCD for every component without its own COC / QCC
    for (uint32_t k = 0; k < 16; ++k) {
        if (!cp.coc_set[k]) comp_style_from_cod(cp, k);
        if (!cp.qcc_set[k]) comp_quant_from_qcd(cp, k);
    }
    std::sort(cp.ppm.begin(), cp.ppm.end(), [](const PpxSeg &a, const PpxSeg &b) { return a.z < b.z; });
    // j2k_read_header stops at the first SOT; a stream that ends before it is truncated
    if (first_sot == 0) { err = "truncated main header (no SOT)"; return false; }
    // mode switches: BYPASS, RESET, TERMALL, VSC, PTERM, SEGSYM; not HT (0x40)
    if (cp.cblksty & ~0x3Fu) { err = "HT code-block style not supported"; return false; }
    if (cp.cblkw > 6 || cp.cblkh > 6) { err = "code-blocks larger than 64 not supported"; return false; }
    for (uint32_t k = 0; k < cp.numcomps; ++k) {
        if (cp.comp[k].cblksty & ~0x3Fu) { err = "HT code-block style not supported"; return false; }
        if (cp.comp[k].cblkw > 6 || cp.comp[k].cblkh > 6) { err = "code-blocks larger than 64 not supported"; return false; }
    }
    for (uint32_t k = 0; k < cp.numcomps; ++k) cp.shift[k] = cp.sgnd[k] ? 0 : (1 << (cp.prec[k] - 1));
    return true;
}

}  // namespace grkgpu
