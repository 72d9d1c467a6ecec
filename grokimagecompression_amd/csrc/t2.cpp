// t2.cpp -- host Tier-2: packet iteration (progressions, POC, tile-parts),
// packet headers, quality layers and PCRD rate control.  See t2.h.
//
// Everything here decides codestream BYTES, so it restates the reference's
// behaviour exactly, quirks included (each function cites what it follows).
// The iteration is written as plain nested loops that emit the whole packet
// order at once instead of the reference's resumable pi_next() generators; the
// order, the skip conditions and the duplicate suppression ("include" array)
// are the same.
#include "t2.h"

#include "host_pool.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>

namespace grkgpu {

namespace {

const char *prog_string(uint32_t prg) {
    static const char *s[5] = {"LRCP", "RLCP", "RPCL", "PCRL", "CPRL"};
    return prg < 5 ? s[prg] : "";
}

uint32_t ceildiv64(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }
uint32_t floordivpow2(uint32_t a, uint32_t b) { return a >> b; }

// ---------------------------------------------------------------------------
// packet iterator state (PacketIter / grk_pi_comp / grk_pi_resolution)
// ---------------------------------------------------------------------------
struct PiRes { uint32_t pdx = 0, pdy = 0, pw = 0, ph = 0; };
struct PiComp {
    uint32_t dx = 1, dy = 1, numres = 0;
    PiRes res[33];
};
struct Range {  // grk_poc fields a PacketIter walks
    uint32_t resno0 = 0, resno1 = 0, compno0 = 0, compno1 = 0, layno0 = 0, layno1 = 0, precno0 = 0, precno1 = 0;
    uint32_t tx0 = 0, ty0 = 0, tx1 = 0, ty1 = 0, prg = 0;
};
struct Pi {
    Range poc;
    std::vector<PiComp> comps;
    uint32_t tx0 = 0, ty0 = 0, tx1 = 0, ty1 = 0, dx = 0, dy = 0;
    bool tp_on = false;
    uint32_t step_p = 0, step_c = 0, step_r = 0, step_l = 0;
    std::vector<uint8_t> *include = nullptr;
};

// grk_get_all_encoding_parameters (PacketIter.cpp:762-870): tile extent,
// per (component, resolution) precinct exponents and counts, the smallest
// precinct step on the reference grid, the largest precinct count / resolution
// count.
struct TileGeom {
    uint32_t tx0, tx1, ty0, ty1, dx_min, dy_min, max_prec, max_res;
    std::vector<PiComp> comps;
};

TileGeom tile_geom(const CodingParams &cp, const Tile &tile) {
    TileGeom g;
    g.tx0 = tile.r.x0; g.tx1 = tile.r.x1; g.ty0 = tile.r.y0; g.ty1 = tile.r.y1;
    g.max_prec = 0; g.max_res = 0;
    g.dx_min = g.dy_min = 0x7fffffff;
    g.comps.resize(cp.numcomps);
    for (uint32_t k = 0; k < cp.numcomps; ++k) {
        PiComp &c = g.comps[k];
        const CompParams &cc = cp.comp[k];  // the component's COD / COC
        c.numres = cc.numres;
        c.dx = cp.dx[k];
        c.dy = cp.dy[k];
        g.max_res = std::max(g.max_res, cc.numres);
        for (uint32_t r = 0; r < cc.numres; ++r) {
            const uint32_t level = cc.numres - 1 - r;
            c.res[r].pdx = cc.prcw[r];
            c.res[r].pdy = cc.prch[r];
            const uint64_t dx = (uint64_t)c.dx << (cc.prcw[r] + level), dy = (uint64_t)c.dy << (cc.prch[r] + level);
            if (dx < UINT_MAX) g.dx_min = std::min<uint32_t>(g.dx_min, (uint32_t)dx);
            if (dy < UINT_MAX) g.dy_min = std::min<uint32_t>(g.dy_min, (uint32_t)dy);
            if (tile.comps.empty()) continue;
            const Resolution &res = tile.comps[k].res[r];
            c.res[r].pw = res.pw;
            c.res[r].ph = res.ph;
            g.max_prec = std::max(g.max_prec, res.pw * res.ph);
        }
    }
    return g;
}

void setup_pi(Pi &pi, const TileGeom &g, const CodingParams &cp, std::vector<uint8_t> *include) {
    pi.comps = g.comps;
    pi.tx0 = g.tx0; pi.tx1 = g.tx1; pi.ty0 = g.ty0; pi.ty1 = g.ty1;
    pi.dx = g.dx_min; pi.dy = g.dy_min;
    pi.step_p = 1;
    pi.step_c = g.max_prec;
    pi.step_r = cp.numcomps * pi.step_c;
    pi.step_l = g.max_res * pi.step_r;
    pi.include = include;
}

// update_pi_dxy_for_comp / update_pi_dxy (PacketIter.cpp:220-250)
void dxy_for_comp(Pi &pi, const PiComp &c) {
    for (uint32_t r = 0; r < c.numres; ++r) {
        const uint64_t dx = (uint64_t)c.dx << (c.res[r].pdx + c.numres - 1 - r);
        const uint64_t dy = (uint64_t)c.dy << (c.res[r].pdy + c.numres - 1 - r);
        if (dx < UINT_MAX) pi.dx = !pi.dx ? (uint32_t)dx : std::min<uint32_t>(pi.dx, (uint32_t)dx);
        if (dy < UINT_MAX) pi.dy = !pi.dy ? (uint32_t)dy : std::min<uint32_t>(pi.dy, (uint32_t)dy);
    }
}
void dxy_all(Pi &pi) {
    pi.dx = pi.dy = 0;
    for (auto &c : pi.comps) dxy_for_comp(pi, c);
}

bool take(Pi &pi, uint32_t l, uint32_t r, uint32_t c, uint32_t p, std::vector<PacketId> &out) {
    const size_t idx = (size_t)l * pi.step_l + (size_t)r * pi.step_r + (size_t)c * pi.step_c + (size_t)p * pi.step_p;
    if (idx >= pi.include->size()) pi.include->resize(idx + 1, 0);
    if ((*pi.include)[idx]) return false;
    (*pi.include)[idx] = 1;
    out.push_back({l, r, c, p});
    return true;
}

// pi_next_lrcp / pi_next_rlcp (PacketIter.cpp:252-348)
void walk_lrcp(Pi &pi, bool rl, std::vector<PacketId> &out) {
    Range &q = pi.poc;
    auto body = [&](uint32_t l, uint32_t r) {
        for (uint32_t c = q.compno0; c < q.compno1; ++c) {
            const PiComp &comp = pi.comps[c];
            if (r >= comp.numres) continue;
            const PiRes &res = comp.res[r];
            if (!pi.tp_on) q.precno1 = res.pw * res.ph;
            for (uint32_t p = q.precno0; p < q.precno1; ++p) {
                if (p >= res.pw * res.ph) continue;
                take(pi, l, r, c, p, out);
            }
        }
    };
    if (!rl) {
        for (uint32_t l = q.layno0; l < q.layno1; ++l)
            for (uint32_t r = q.resno0; r < q.resno1; ++r) body(l, r);
    } else {
        for (uint32_t r = q.resno0; r < q.resno1; ++r)
            for (uint32_t l = q.layno0; l < q.layno1; ++l) body(l, r);
    }
}

// The position-driven progressions (RPCL / PCRL / CPRL, PacketIter.cpp:350-657):
// precinct index of (x, y) in resolution r of component c, or -1 when (x, y)
// is not a precinct origin there.  Returns -2 for the reference's "Precinct
// index invalid" abort (CPRL only).
int64_t prec_at(const Pi &pi, const PiComp &comp, uint32_t r, uint32_t x, uint32_t y, bool check) {
    const PiRes &res = comp.res[r];
    const uint32_t levelno = comp.numres - 1 - r;
    if (levelno >= 33) return -1;
    const uint32_t trx0 = ceildiv64(pi.tx0, (uint64_t)comp.dx << levelno);
    const uint32_t try0 = ceildiv64(pi.ty0, (uint64_t)comp.dy << levelno);
    const uint32_t trx1 = ceildiv64(pi.tx1, (uint64_t)comp.dx << levelno);
    const uint32_t try1 = ceildiv64(pi.ty1, (uint64_t)comp.dy << levelno);
    const uint32_t rpx = res.pdx + levelno, rpy = res.pdy + levelno;
    if (!(((uint64_t)y % ((uint64_t)comp.dy << rpy) == 0) ||
          ((y == pi.ty0) && (((uint64_t)try0 << levelno) % ((uint64_t)1 << rpy)))))
        return -1;
    if (!(((uint64_t)x % ((uint64_t)comp.dx << rpx) == 0) ||
          ((x == pi.tx0) && (((uint64_t)trx0 << levelno) % ((uint64_t)1 << rpx)))))
        return -1;
    if (res.pw == 0 || res.ph == 0) return -1;
    if (trx0 == trx1 || try0 == try1) return -1;
    const uint32_t ax = floordivpow2(ceildiv64(x, (uint64_t)comp.dx << levelno), res.pdx), bx = floordivpow2(trx0, res.pdx);
    const uint32_t ay = floordivpow2(ceildiv64(y, (uint64_t)comp.dy << levelno), res.pdy), by = floordivpow2(try0, res.pdy);
    if (check && (bx > ax || by > ay)) return -2;
    const uint32_t precno = (ax - bx) + (ay - by) * res.pw;
    if (precno >= res.pw * res.ph) return -1;
    return precno;
}

void walk_positional(Pi &pi, std::vector<PacketId> &out) {
    Range &q = pi.poc;
    auto set_extent = [&]() {
        if (!pi.tp_on) { q.ty0 = pi.ty0; q.tx0 = pi.tx0; q.ty1 = pi.ty1; q.tx1 = pi.tx1; }
    };
    auto layers = [&](uint32_t r, uint32_t c, uint32_t p) {
        for (uint32_t l = q.layno0; l < q.layno1; ++l) take(pi, l, r, c, p, out);
    };
    if (q.prg == PROG_RPCL) {
        dxy_all(pi);
        set_extent();
        for (uint32_t r = q.resno0; r < q.resno1; ++r)
            for (uint32_t y = q.ty0; y < q.ty1; y += pi.dy - (y % pi.dy))
                for (uint32_t x = q.tx0; x < q.tx1; x += pi.dx - (x % pi.dx))
                    for (uint32_t c = q.compno0; c < q.compno1; ++c) {
                        const PiComp &comp = pi.comps[c];
                        if (r >= comp.numres) continue;
                        const int64_t p = prec_at(pi, comp, r, x, y, false);
                        if (p >= 0) layers(r, c, (uint32_t)p);
                    }
    } else if (q.prg == PROG_PCRL) {
        dxy_all(pi);
        set_extent();
        for (uint32_t y = q.ty0; y < q.ty1; y += pi.dy - (y % pi.dy))
            for (uint32_t x = q.tx0; x < q.tx1; x += pi.dx - (x % pi.dx))
                for (uint32_t c = q.compno0; c < q.compno1; ++c) {
                    const PiComp &comp = pi.comps[c];
                    for (uint32_t r = q.resno0; r < std::min(q.resno1, comp.numres); ++r) {
                        const int64_t p = prec_at(pi, comp, r, x, y, false);
                        if (p >= 0) layers(r, c, (uint32_t)p);
                    }
                }
    } else {  // CPRL
        for (uint32_t c = q.compno0; c < q.compno1; ++c) {
            const PiComp &comp = pi.comps[c];
            pi.dx = pi.dy = 0;
            dxy_for_comp(pi, comp);
            set_extent();
            for (uint32_t y = q.ty0; y < q.ty1; y += pi.dy - (y % pi.dy))
                for (uint32_t x = q.tx0; x < q.tx1; x += pi.dx - (x % pi.dx))
                    for (uint32_t r = q.resno0; r < std::min(q.resno1, comp.numres); ++r) {
                        const int64_t p = prec_at(pi, comp, r, x, y, true);
                        if (p == -2) return;  // "Precinct index invalid": pi_next returns false
                        if (p >= 0) layers(r, c, (uint32_t)p);
                    }
        }
    }
}

void walk(Pi &pi, std::vector<PacketId> &out) {
    switch (pi.poc.prg) {
        case PROG_LRCP: walk_lrcp(pi, false, out); break;
        case PROG_RLCP: walk_lrcp(pi, true, out); break;
        case PROG_RPCL: case PROG_PCRL: case PROG_CPRL: walk_positional(pi, out); break;
        default: break;
    }
}

// pi_update_encode_poc_and_final / pi_update_encode_not_poc (PacketIter.cpp:925-1033)
void update_encode_pocs(const CodingParams &cp, std::vector<EncPoc> &pocs, const TileGeom &g, bool poc) {
    if (poc) {
        for (size_t i = 0; i < pocs.size(); ++i) {
            EncPoc &p = pocs[i];
            p.compS = p.compno0; p.compE = p.compno1;
            p.resS = p.resno0; p.resE = p.resno1;
            p.layE = p.layno1;
            p.prg = p.prg1;
            p.prcS = 0;
            // the reference's quirk: later entries start at layE when their
            // layer end grows, else at 0 (PacketIter.cpp:978-980)
            p.layS = i == 0 ? 0 : (p.layE > pocs[i - 1].layE ? p.layE : 0);
            p.prcE = g.max_prec;
            p.txS = g.tx0; p.txE = g.tx1; p.tyS = g.ty0; p.tyE = g.ty1;
            p.dx = g.dx_min; p.dy = g.dy_min;
        }
    } else {
        for (auto &p : pocs) {
            p.compS = 0; p.compE = cp.numcomps;
            p.resS = 0; p.resE = g.max_res;
            p.layS = 0; p.layE = cp.numlayers;
            p.prg = cp.prog;
            p.prcS = 0; p.prcE = g.max_prec;
            p.txS = g.tx0; p.txE = g.tx1; p.tyS = g.ty0; p.tyE = g.ty1;
            p.dx = g.dx_min; p.dy = g.dy_min;
        }
    }
}

// The tile-part position T2 works with is TileProcessor::tp_pos, copied from
// the coding parameters when the tile processor is created
// (TileProcessor.cpp:1627-1638, j2k_setup_header_writing j2k.cpp:2328-2333)
// -- BEFORE j2k_calculate_tp sets m_tp_pos (j2k_init_info, the first header
// procedure).  So packets are divided among tile-parts by the FIRST
// progression letter only, whatever -u names; e.g. "-u R" with LRCP writes
// the whole tile into each of its numres tile-parts.  The tile-part COUNT does
// use the real position (j2k_get_num_tp).  Restated as is.
constexpr uint32_t kStaleTpPos = 0;

bool is_cinema(const CodingParams &cp) { return cp.rsiz == RSIZ_CINEMA_2K || cp.rsiz == RSIZ_CINEMA_4K; }

// pi_check_next_level (PacketIter.cpp:1101-1180)
bool check_next_level(int32_t pos, const EncPoc &t, const char *prog) {
    if (pos < 0) return false;
    switch (prog[pos]) {
        case 'R': return t.res_t == t.resE ? check_next_level(pos - 1, t, prog) : true;
        case 'C': return t.comp_t == t.compE ? check_next_level(pos - 1, t, prog) : true;
        case 'L': return t.lay_t == t.layE ? check_next_level(pos - 1, t, prog) : true;
        case 'P':
            if (t.prg == PROG_LRCP || t.prg == PROG_RLCP)
                return t.prc_t == t.prcE ? check_next_level(pos - 1, t, prog) : true;
            if (t.tx0_t == t.txE) return t.ty0_t == t.tyE ? check_next_level(pos - 1, t, prog) : true;
            return true;
    }
    return false;
}

// pi_init_encode (PacketIter.cpp:1532-1799): the range of pi for tile-part
// tpnum of POC pino; the tile-part odometer state lives in `t`.
void init_encode(Pi &pi, const CodingParams &cp, EncPoc &t, uint32_t tpnum, uint32_t tppos, bool final_pass) {
    const char *prog = prog_string(t.prg);
    Range &q = pi.poc;
    q.prg = t.prg;
    const bool split = cp.tp_on && ((!is_cinema(cp) && final_pass) || is_cinema(cp));
    if (!split) {
        q.resno0 = t.resS; q.resno1 = t.resE;
        q.compno0 = t.compS; q.compno1 = t.compE;
        q.layno0 = t.layS; q.layno1 = t.layE;
        q.precno0 = t.prcS; q.precno1 = t.prcE;
        q.tx0 = t.txS; q.ty0 = t.tyS; q.tx1 = t.txE; q.ty1 = t.tyE;
        return;
    }
    const bool lr = t.prg == PROG_LRCP || t.prg == PROG_RLCP;
    for (uint32_t i = tppos + 1; i < 4; i++) {
        switch (prog[i]) {
            case 'R': q.resno0 = t.resS; q.resno1 = t.resE; break;
            case 'C': q.compno0 = t.compS; q.compno1 = t.compE; break;
            case 'L': q.layno0 = t.layS; q.layno1 = t.layE; break;
            case 'P':
                if (lr) { q.precno0 = t.prcS; q.precno1 = t.prcE; }
                else { q.tx0 = t.txS; q.ty0 = t.tyS; q.tx1 = t.txE; q.ty1 = t.tyE; }
                break;
        }
    }
    if (tpnum == 0) {
        for (int32_t i = (int32_t)tppos; i >= 0; i--) {
            switch (prog[i]) {
                case 'C': t.comp_t = t.compS; q.compno0 = t.comp_t; q.compno1 = t.comp_t + 1; t.comp_t += 1; break;
                case 'R': t.res_t = t.resS; q.resno0 = t.res_t; q.resno1 = t.res_t + 1; t.res_t += 1; break;
                case 'L': t.lay_t = t.layS; q.layno0 = t.lay_t; q.layno1 = t.lay_t + 1; t.lay_t += 1; break;
                case 'P':
                    if (lr) {
                        t.prc_t = t.prcS; q.precno0 = t.prc_t; q.precno1 = t.prc_t + 1; t.prc_t += 1;
                    } else {
                        t.tx0_t = t.txS; t.ty0_t = t.tyS;
                        q.tx0 = t.tx0_t; q.tx1 = t.tx0_t + t.dx - (t.tx0_t % t.dx);
                        q.ty0 = t.ty0_t; q.ty1 = t.ty0_t + t.dy - (t.ty0_t % t.dy);
                        t.tx0_t = q.tx1; t.ty0_t = q.ty1;
                    }
                    break;
            }
        }
        return;
    }
    uint32_t incr_top = 1, resetX = 0;
    for (int32_t i = (int32_t)tppos; i >= 0; i--) {
        switch (prog[i]) {
            case 'C': q.compno0 = t.comp_t - 1; q.compno1 = t.comp_t; break;
            case 'R': q.resno0 = t.res_t - 1; q.resno1 = t.res_t; break;
            case 'L': q.layno0 = t.lay_t - 1; q.layno1 = t.lay_t; break;
            case 'P':
                if (lr) { q.precno0 = t.prc_t - 1; q.precno1 = t.prc_t; }
                else {
                    q.tx0 = t.tx0_t - t.dx - (t.tx0_t % t.dx); q.tx1 = t.tx0_t;
                    q.ty0 = t.ty0_t - t.dy - (t.ty0_t % t.dy); q.ty1 = t.ty0_t;
                }
                break;
        }
        if (incr_top != 1) continue;
        switch (prog[i]) {
            case 'R':
                if (t.res_t == t.resE) {
                    if (check_next_level(i - 1, t, prog)) {
                        t.res_t = t.resS; q.resno0 = t.res_t; q.resno1 = t.res_t + 1; t.res_t += 1; incr_top = 1;
                    } else incr_top = 0;
                } else {
                    q.resno0 = t.res_t; q.resno1 = t.res_t + 1; t.res_t += 1; incr_top = 0;
                }
                break;
            case 'C':
                if (t.comp_t == t.compE) {
                    if (check_next_level(i - 1, t, prog)) {
                        t.comp_t = t.compS; q.compno0 = t.comp_t; q.compno1 = t.comp_t + 1; t.comp_t += 1; incr_top = 1;
                    } else incr_top = 0;
                } else {
                    q.compno0 = t.comp_t; q.compno1 = t.comp_t + 1; t.comp_t += 1; incr_top = 0;
                }
                break;
            case 'L':
                if (t.lay_t == t.layE) {
                    if (check_next_level(i - 1, t, prog)) {
                        t.lay_t = t.layS; q.layno0 = t.lay_t; q.layno1 = t.lay_t + 1; t.lay_t += 1; incr_top = 1;
                    } else incr_top = 0;
                } else {
                    q.layno0 = t.lay_t; q.layno1 = t.lay_t + 1; t.lay_t += 1; incr_top = 0;
                }
                break;
            case 'P':
                if (lr) {
                    if (t.prc_t == t.prcE) {
                        if (check_next_level(i - 1, t, prog)) {
                            t.prc_t = t.prcS; q.precno0 = t.prc_t; q.precno1 = t.prc_t + 1; t.prc_t += 1; incr_top = 1;
                        } else incr_top = 0;
                    } else {
                        q.precno0 = t.prc_t; q.precno1 = t.prc_t + 1; t.prc_t += 1; incr_top = 0;
                    }
                } else {
                    if (t.tx0_t >= t.txE) {
                        if (t.ty0_t >= t.tyE) {
                            if (check_next_level(i - 1, t, prog)) {
                                t.ty0_t = t.tyS; q.ty0 = t.ty0_t; q.ty1 = t.ty0_t + t.dy - (t.ty0_t % t.dy);
                                t.ty0_t = q.ty1; incr_top = 1; resetX = 1;
                            } else {
                                incr_top = 0; resetX = 0;
                            }
                        } else {
                            q.ty0 = t.ty0_t; q.ty1 = t.ty0_t + t.dy - (t.ty0_t % t.dy);
                            t.ty0_t = q.ty1; incr_top = 0; resetX = 1;
                        }
                        if (resetX == 1) {
                            t.tx0_t = t.txS; q.tx0 = t.tx0_t; q.tx1 = t.tx0_t + t.dx - (t.tx0_t % t.dx);
                            t.tx0_t = q.tx1;
                        }
                    } else {
                        q.tx0 = t.tx0_t; q.tx1 = t.tx0_t + t.dx - (t.tx0_t % t.dx);
                        t.tx0_t = q.tx1; incr_top = 0;
                    }
                }
                break;
        }
    }
}

// pi_initialise_encode (PacketIter.cpp:1357-1530): fresh iterators (one per
// POC entry, sharing one include array), ranges from the POC entries when
// the tile has them and (cinema or final pass), else the whole tile.  Only
// the first iterator carries tp_on (the others are calloc'ed zero there).
void initialise_encode(const CodingParams &cp, TileEnc &te, bool final_pass, std::vector<Pi> &pis,
                       std::vector<uint8_t> &include, TileGeom &g) {
    g = tile_geom(cp, *te.tile);
    pis.assign(te.pocs.size(), Pi());
    include.assign((size_t)cp.numlayers * g.max_res * cp.numcomps * std::max<uint32_t>(g.max_prec, 1), 0);
    for (auto &pi : pis) setup_pi(pi, g, cp, &include);
    pis[0].tp_on = cp.tp_on;
    update_encode_pocs(cp, te.pocs, g, cp.numpocs && (is_cinema(cp) || final_pass));
}

}  // namespace

// ---------------------------------------------------------------------------
// decoder packet order: T2::decode_packets over pi_create_decode
// (PacketIter.cpp:1187-1355, pi_update_decode_poc / _not_poc :1035-1099)
// ---------------------------------------------------------------------------
void decode_packet_order(const CodingParams &cp, const Tile &tile, std::vector<PacketId> &out) {
    const TileGeom g = tile_geom(cp, tile);
    std::vector<uint8_t> include((size_t)(cp.numlayers + 1) * g.max_res * cp.numcomps * std::max<uint32_t>(g.max_prec, 1), 0);
    const uint32_t n = num_poc_entries(cp);
    out.clear();
    for (uint32_t pino = 0; pino < n; ++pino) {
        Pi pi;
        setup_pi(pi, g, cp, &include);
        Range &q = pi.poc;
        if (cp.numpocs) {
            const PocSpec &p = cp.pocs[pino];
            q.prg = p.prg;
            q.resno0 = p.resno0; q.compno0 = p.compno0; q.layno0 = 0; q.precno0 = 0;
            q.resno1 = p.resno1; q.compno1 = p.compno1;
            q.layno1 = std::min(p.layno1, cp.numlayers);
            q.precno1 = g.max_prec;
        } else {
            q.prg = cp.prog;
            q.resno0 = 0; q.compno0 = 0; q.layno0 = 0; q.precno0 = 0;
            q.resno1 = g.max_res; q.compno1 = cp.numcomps; q.layno1 = cp.numlayers; q.precno1 = g.max_prec;
        }
        // a POC range past the components the tile has: no packets there
        q.compno1 = std::min(q.compno1, cp.numcomps);
        walk(pi, out);
    }
}

// ---------------------------------------------------------------------------
// encoder: tile-part plan
// ---------------------------------------------------------------------------
void init_enc_pocs(const CodingParams &cp, TileEnc &te) {
    te.pocs.assign(num_poc_entries(cp), EncPoc());
    for (uint32_t i = 0; i < cp.numpocs; ++i) {
        EncPoc &p = te.pocs[i];
        const PocSpec &s = cp.pocs[i];
        p.resno0 = s.resno0; p.compno0 = s.compno0; p.layno1 = s.layno1;
        p.resno1 = s.resno1; p.compno1 = s.compno1; p.prg1 = s.prg;
    }
}

std::vector<uint32_t> tile_part_counts(CodingParams &cp, const Tile &tile) {
    // pi_update_encoding_parameters then j2k_get_num_tp per POC entry
    TileEnc te;
    init_enc_pocs(cp, te);
    const TileGeom g = tile_geom(cp, tile);
    update_encode_pocs(cp, te.pocs, g, cp.numpocs != 0);
    std::vector<uint32_t> counts;
    const char *prog = prog_string(cp.prog);
    for (auto &p : te.pocs) {
        uint32_t tpnum = 1;
        if (cp.tp_on) {
            for (uint32_t i = 0; i < 4; ++i) {
                switch (prog[i]) {
                    case 'C': tpnum *= p.compE; break;
                    case 'R': tpnum *= p.resE; break;
                    case 'P': tpnum *= p.prcE; break;
                    case 'L': tpnum *= p.layE; break;
                }
                if (cp.tp_flag == prog[i]) {
                    cp.tp_pos = i;
                    break;
                }
            }
        }
        counts.push_back(tpnum);
    }
    return counts;
}

void encode_packet_order(const CodingParams &cp, TileEnc &te, uint32_t pino, uint32_t tp_num,
                         std::vector<PacketId> &out) {
    std::vector<Pi> pis;
    std::vector<uint8_t> include;
    TileGeom g;
    initialise_encode(cp, te, true, pis, include, g);
    init_encode(pis[pino], cp, te.pocs[pino], tp_num, kStaleTpPos, true);
    out.clear();
    walk(pis[pino], out);
}

// ---------------------------------------------------------------------------
// packet writer / simulator (T2::encode_packet T2.cpp:859-1060,
// T2::encode_packet_simulate :1300-1506)
// ---------------------------------------------------------------------------
namespace {

// Bit counter with the simulator's buffer bound: BitIO(0, length) fails once
// a byte would land past `length` (BitIO.cpp:71-85); every such failure makes
// the packet "not fit", so counting the header bytes and comparing at the end
// is equivalent.
struct BitCount {
    uint64_t bytes = 0;
    uint32_t buf = 0, ct = 8;
    void byteout() { ++bytes; ct = (buf == 0xff) ? 7 : 8; buf = 0; }
    void putbit(uint32_t b) { if (ct == 0) byteout(); ct--; buf |= (b & 1) << ct; }
    // the n low bits of v, MSB first: putbit() per bit, a byte's free bits at a time
    void write(uint32_t v, uint32_t n) {
        while (n) {
            if (ct == 0) byteout();
            const uint32_t k = n < ct ? n : ct;
            n -= k;
            ct -= k;
            buf |= ((v >> n) & ((1u << k) - 1)) << ct;
        }
    }
    void flush() { byteout(); if (ct == 7) byteout(); }
    void numpasses(uint32_t n) {
        if (n == 1) write(0, 1);
        else if (n == 2) write(2, 2);
        else if (n <= 5) write(0xc | (n - 3), 4);
        else if (n <= 36) write(0x1e0 | (n - 6), 9);
        else write(0xff80 | (n - 37), 16);
    }
    void comma(int32_t n) { while (--n >= 0) write(1, 1); write(0, 1); }
    void tagtree(TagTree &t, uint32_t leaf, int64_t threshold) {
        int32_t stk[64], sp = 0, node = (int32_t)leaf;
        while (t.nodes[node].parent >= 0) { stk[sp++] = node; node = t.nodes[node].parent; }
        int64_t low = 0;
        for (;;) {
            TagTree::Node &n = t.nodes[node];
            if (low > n.low) n.low = low; else low = n.low;
            while (low < threshold) {
                if (low >= n.value) {
                    if (!n.known) { write(1, 1); n.known = 1; }
                    break;
                }
                write(0, 1);
                ++low;
            }
            n.low = low;
            if (sp == 0) break;
            node = stk[--sp];
        }
    }
};

// Packet header body shared by the writer and the simulator: inclusion,
// missing MSBs, pass counts, length indicators.
template <class W>
void packet_header(const CodingParams &cp, TileEnc &te, Resolution &res, uint32_t precno, uint32_t layno, W &w) {
    std::vector<EncCblkState> &cs = *te.cblk;
    std::vector<EncLayer> &lay = *te.layers;
    const EncPass *passes = te.passes;
    const uint32_t L = cp.numlayers;
    if (layno == 0) {
        for (uint32_t bandno = 0; bandno < res.numbands; ++bandno) {
            Band &b = res.bands[bandno];
            if (b.empty() || precno >= b.precs.size()) continue;
            Precinct &pr = b.precs[precno];
            if (pr.cblks.empty()) continue;
            pr.incl.reset();
            pr.imsb.reset();
            for (uint32_t cb = 0; cb < pr.cblks.size(); ++cb) {
                EncCblkState &s = cs[pr.cblks[cb].gidx];
                s.incl_cur = 0;
                if (b.numbps >= s.numbps) pr.imsb.setvalue(cb, (int64_t)b.numbps - (int64_t)s.numbps);
            }
        }
    }
    w.write(1, 1);  // Grok always signals a non-empty packet (T2.cpp:924-927)
    for (uint32_t bandno = 0; bandno < res.numbands; ++bandno) {
        Band &b = res.bands[bandno];
        if (b.empty() || precno >= b.precs.size()) continue;
        Precinct &pr = b.precs[precno];
        if (pr.cblks.empty()) continue;
        for (uint32_t cb = 0; cb < pr.cblks.size(); ++cb) {
            const EncCblkState &s = cs[pr.cblks[cb].gidx];
            if (!s.incl_cur && lay[(size_t)pr.cblks[cb].gidx * L + layno].numpasses) pr.incl.setvalue(cb, layno);
        }
        for (uint32_t cb = 0; cb < pr.cblks.size(); ++cb) {
            EncCblkState &s = cs[pr.cblks[cb].gidx];
            const EncLayer &ly = lay[(size_t)pr.cblks[cb].gidx * L + layno];
            if (!s.incl_cur) w.tagtree(pr.incl, cb, layno + 1);
            else w.write(ly.numpasses != 0, 1);
            if (!ly.numpasses) continue;
            if (!s.incl_cur) {
                s.numlenbits = 3;
                w.tagtree(pr.imsb, cb, INT64_MAX);
            }
            w.numpasses(ly.numpasses);
            const uint32_t nb = s.incl_cur + ly.numpasses;
            int32_t increment = 0;
            uint32_t nump = 0, len = 0;
            for (uint32_t pn = s.incl_cur; pn < nb; ++pn) {
                const EncPass &ps = passes[s.pass0 + pn];
                ++nump;
                len += ps.len;
                if (ps.term || pn == nb - 1) {
                    increment = std::max<int32_t>(increment, floorlog2((int32_t)len) + 1 -
                                                                 ((int32_t)s.numlenbits + floorlog2((int32_t)nump)));
                    len = 0;
                    nump = 0;
                }
            }
            w.comma(increment);
            s.numlenbits += (uint32_t)increment;
            for (uint32_t pn = s.incl_cur; pn < nb; ++pn) {
                const EncPass &ps = passes[s.pass0 + pn];
                ++nump;
                len += ps.len;
                if (ps.term || pn == nb - 1) {
                    w.write(len, s.numlenbits + (uint32_t)floorlog2((int32_t)nump));
                    len = 0;
                    nump = 0;
                }
            }
        }
    }
    w.flush();
}

}  // namespace

bool write_packet(const CodingParams &cp, TileEnc &te, const PacketId &pk, ByteBuf &hdr, std::vector<PlanItem> &plan) {
    Resolution &res = te.tile->comps[pk.compno].res[pk.resno];
    const size_t hstart = hdr.size();
    if (cp.csty & CSTY_SOP) {
        const uint32_t n = te.packno % 0x10000;
        hdr.put8(0xFF); hdr.put8(0x91); hdr.put8(0); hdr.put8(4); hdr.put8(n >> 8); hdr.put8(n & 0xff);
    }
    {
        BitWriter w(hdr);
        packet_header(cp, te, res, pk.precno, pk.layno, w);
    }
    if (cp.csty & CSTY_EPH) { hdr.put8(0xFF); hdr.put8(0x92); }
    plan.push_back({hstart, (uint32_t)(hdr.size() - hstart), 0});
    const uint32_t L = cp.numlayers;
    for (uint32_t bandno = 0; bandno < res.numbands; ++bandno) {
        Band &b = res.bands[bandno];
        if (b.empty() || pk.precno >= b.precs.size()) continue;
        Precinct &pr = b.precs[pk.precno];
        for (auto &c : pr.cblks) {
            EncCblkState &s = (*te.cblk)[c.gidx];
            const EncLayer &ly = (*te.layers)[(size_t)c.gidx * L + pk.layno];
            if (!ly.numpasses) continue;
            if (ly.len) plan.push_back({s.dev_off + ly.data_off, ly.len, 1});
            s.incl_cur += ly.numpasses;
        }
    }
    ++te.packno;
    return true;
}

namespace {

// T2::encode_packet_simulate (T2.cpp:1300-1506): bytes of one packet, or
// false when it does not fit in `length`.  Unsigned wrap-around of `length`
// (SOP / EPH subtractions) is the reference's.
bool simulate_packet(const CodingParams &cp, TileEnc &te, const PacketId &pk, uint64_t length, uint64_t *bytes) {
    Resolution &res = te.tile->comps[pk.compno].res[pk.resno];
    uint64_t written = 0;
    if (cp.csty & CSTY_SOP) { length -= 6; written += 6; }
    BitCount w;
    packet_header(cp, te, res, pk.precno, pk.layno, w);
    if (w.bytes > length) return false;
    written += w.bytes;
    length -= w.bytes;
    if (cp.csty & CSTY_EPH) { length -= 2; written += 2; }
    const uint32_t L = cp.numlayers;
    for (uint32_t bandno = 0; bandno < res.numbands; ++bandno) {
        Band &b = res.bands[bandno];
        if (b.empty() || pk.precno >= b.precs.size()) continue;
        Precinct &pr = b.precs[pk.precno];
        for (auto &c : pr.cblks) {
            EncCblkState &s = (*te.cblk)[c.gidx];
            const EncLayer &ly = (*te.layers)[(size_t)c.gidx * L + pk.layno];
            if (!ly.numpasses) continue;
            if (ly.len > length) return false;
            s.incl_cur += ly.numpasses;
            written += ly.len;
            length -= ly.len;
        }
    }
    *bytes = written;
    return true;
}

// Rate-control probes, evaluated incrementally with the results of a full
// evaluation.  A bisection step forms the layer at a threshold
// (make_layer_simple / makelayer_feasible) and simulates the tile's packets
// (simulate_tile):
//  * a block's pass count at threshold t follows from comparisons of t with
//    pass slopes, each monotone in t; the comparisons a block made at its last
//    evaluation keep their outcomes on an interval of t (two bounds per
//    block), so a probe inside that interval leaves the block's layer record
//    as it is and skips the block;
//  * a packet's header depends only on its precinct's earlier packets (tag
//    trees, inclusion and length-indicator state of the precinct's
//    code-blocks), and a precinct's packets come in increasing layer order, so
//    each precinct's packets are simulated on their own (in parallel), and
//    only the precincts holding a block whose layer record changed since the
//    last probe are simulated again; the packet order for a layer count is
//    built once.
// the current rate allocation's RateStats (one allocation per thread at a time)
struct RateTrace {
    bool on = true;
    double hull = 0, form = 0, sim = 0;
    uint32_t probes = 0, skipped = 0;
    uint64_t redo = 0, precs = 0;
};
thread_local RateTrace g_rt;
double t2_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct RateProbe {
    // per block, in te.blist order
    std::vector<uint32_t> gidx;        // its record index (te.blist[i]->gidx, without the pointer chase)
    std::vector<uint32_t> prec;        // precinct id
    struct BoundD { double lo, hi; };  // simple: largest slope compared false, smallest compared true
    struct BoundU { uint32_t lo, hi; };  // feasible: the slope it stopped at, smallest slope it passed
    std::vector<BoundD> bd;            // (a block's two bounds on one cache line)
    std::vector<BoundU> bu;
    std::vector<uint32_t> redo;        // per probe: scratch kept across probes
    std::vector<uint8_t> changed;
    std::vector<int64_t> dlen;
    std::vector<uint32_t> ub_old;
    std::vector<uint8_t> valid;        // bounds hold for the current layer records
    // blocks a probe still has to check: a block whose bounds hold over the
    // whole remaining bisection interval [lower, upper] never changes again
    // in this layer's search (each probe lies in that interval, which only
    // shrinks), so prune() drops it
    std::vector<uint32_t> active;
    // code-block bytes of the layer records of layers [0, layno]: in total
    // and per component (kept up to date by form_layer); without SOP / EPH a
    // probe whose bytes exceed the budget, or a component cap, cannot fit
    // (simulate_tile's budget never wraps then), so it needs no simulation
    std::vector<uint8_t> comp;          // per block: its component
    uint64_t body_prev = 0;             // layers below layno (fixed during its search)
    std::vector<uint64_t> comp_prev;
    int64_t body = 0;                   // layer layno
    std::vector<int64_t> comp_body;
    // the first layer's packet headers, bounded from above: per block the
    // bits its records cost (tag-tree bits taken as the whole path, the rest
    // exact), summed per precinct; a packet of B bits is at most B / 7 + 2
    // bytes (bit stuffing leaves >= 7 bits in every byte, the flush adds <= 2)
    std::vector<uint8_t> lev;           // per block: its tag trees' path length
    std::vector<uint8_t> bnumbps;       // per block: its band's bit-planes
    std::vector<uint32_t> ub;           // per block: header bits bound of its layer-0 record
    std::vector<int64_t> prec_bits;     // per precinct: sum of its blocks' ub
    std::vector<uint8_t> prec_comp;     // per precinct: its component
    bool fresh = true;                 // no probe of the current layer yet: evaluate every block
    // packets of layers [0, layers) in THRESH_CALC order, grouped per precinct
    uint32_t layers = 0, nprec = 0, npoc = 0;  // npoc: POC groups per component
    bool bad = false;
    // the plan holds every precinct holding code-blocks once per layer (so
    // the simulated packets carry exactly the layer records' bytes), and
    // comp_exact: each component's groups hold only that component's packets
    bool body_exact = false, comp_exact = false;
    std::vector<PacketId> order;
    std::vector<size_t> group_end;     // end index of each (compno, poc) group
    std::vector<uint32_t> head, pos;   // packets of precinct p: order[pos[head[p] .. head[p + 1])]
    std::vector<uint64_t> hbytes, dbytes;
    std::vector<uint8_t> dirty;        // per precinct
};

// precinct ids of te.blist (a precinct = one resolution's precinct of a component)
void probe_init(const CodingParams &cp, TileEnc &te, RateProbe &rp) {
    rp.prec.clear();
    rp.comp.clear();
    rp.lev.clear();
    rp.bnumbps.clear();
    rp.prec_comp.clear();
    const size_t nbl = te.blist.size();
    rp.prec.reserve(nbl);
    rp.comp.reserve(nbl);
    rp.lev.reserve(nbl);
    rp.bnumbps.reserve(nbl);
    uint32_t base = 0;
    for (uint32_t k = 0; k < cp.numcomps; ++k) {
        TileComp &tc = te.tile->comps[k];
        for (auto &res : tc.res) {
            for (uint32_t b = 0; b < res.numbands; ++b)
                for (size_t p = 0; p < res.bands[b].precs.size(); ++p) {
                    Precinct &pr = res.bands[b].precs[p];
                    uint32_t depth = 0;  // nodes on a leaf's path to the root
                    if (!pr.incl.nodes.empty())
                        for (int32_t nd = 0; nd >= 0; nd = pr.incl.nodes[nd].parent) ++depth;
                    for (size_t n = 0; n < pr.cblks.size(); ++n) {
                        rp.prec.push_back(base + (uint32_t)p);
                        rp.comp.push_back((uint8_t)k);
                        rp.lev.push_back((uint8_t)std::min<uint32_t>(depth, 255));
                        rp.bnumbps.push_back((uint8_t)std::min<uint32_t>(res.bands[b].numbps, 255));
                    }
                }
            for (uint32_t p = 0; p < res.pw * res.ph; ++p) rp.prec_comp.push_back((uint8_t)k);
            base += res.pw * res.ph;
        }
    }
    rp.gidx.resize(te.blist.size());
    for (size_t i = 0; i < te.blist.size(); ++i) rp.gidx[i] = te.blist[i]->gidx;
    rp.ub.assign(rp.prec.size(), 0);
    rp.prec_bits.assign(base, 0);
    rp.body_prev = 0;
    rp.comp_prev.assign(cp.numcomps, 0);
    rp.body = 0;
    rp.comp_body.assign(cp.numcomps, 0);
    rp.nprec = base;
    const size_t nb = rp.prec.size();
    rp.bd.assign(nb, RateProbe::BoundD{0, 0});
    rp.bu.assign(nb, RateProbe::BoundU{0, 0});
    rp.valid.assign(nb, 0);
    rp.active.clear();
    rp.dirty.assign(rp.nprec, 1);
    rp.layers = 0;
    rp.fresh = true;
}

void probe_plan(CodingParams &cp, TileEnc &te, uint32_t max_layers, RateProbe &rp) {
    const uint32_t pocno = cp.rsiz == RSIZ_CINEMA_4K ? 2 : 1;
    const uint32_t max_comp = cp.max_comp_size > 0 ? cp.numcomps : 1;
    std::vector<Pi> pis;
    std::vector<uint8_t> include;
    TileGeom g;
    initialise_encode(cp, te, false, pis, include, g);
    rp.npoc = std::min<uint32_t>(pocno, (uint32_t)pis.size());
    rp.order.clear();
    rp.group_end.clear();
    std::vector<PacketId> part;
    for (uint32_t compno = 0; compno < max_comp; ++compno)
        for (uint32_t poc = 0; poc < rp.npoc; ++poc) {
            init_encode(pis[poc], cp, te.pocs[poc], compno, kStaleTpPos, false);
            part.clear();
            walk(pis[poc], part);
            for (const auto &pk : part)
                if (pk.layno < max_layers) rp.order.push_back(pk);
            rp.group_end.push_back(rp.order.size());
        }
    std::vector<std::vector<uint32_t>> prec_base(cp.numcomps);
    uint32_t nprec = 0;
    for (uint32_t k = 0; k < cp.numcomps; ++k) {
        const TileComp &tc = te.tile->comps[k];
        prec_base[k].resize(tc.res.size());
        for (size_t r = 0; r < tc.res.size(); ++r) {
            prec_base[k][r] = nprec;
            nprec += tc.res[r].pw * tc.res[r].ph;
        }
    }
    rp.head.assign(nprec + 1, 0);
    rp.pos.assign(rp.order.size(), 0);
    for (const auto &pk : rp.order) ++rp.head[prec_base[pk.compno][pk.resno] + pk.precno + 1];
    for (uint32_t i = 0; i < nprec; ++i) rp.head[i + 1] += rp.head[i];
    std::vector<uint32_t> fill(rp.head.begin(), rp.head.end() - 1);
    for (uint32_t i = 0; i < rp.order.size(); ++i) {
        const PacketId &pk = rp.order[i];
        rp.pos[fill[prec_base[pk.compno][pk.resno] + pk.precno]++] = i;
    }
    // a precinct whose packets are not in increasing layer order (never seen
    // from these iterators) would make the per-precinct split wrong: such a
    // tile takes the packet-by-packet route
    rp.bad = false;
    for (uint32_t p = 0; p < nprec && !rp.bad; ++p)
        for (uint32_t q = rp.head[p] + 1; q < rp.head[p + 1]; ++q)
            if (rp.order[rp.pos[q]].layno <= rp.order[rp.pos[q - 1]].layno) rp.bad = true;
    {
        std::vector<uint8_t> has(nprec, 0);
        for (uint32_t p : rp.prec) has[p] = 1;
        rp.body_exact = !rp.bad;
        for (uint32_t p = 0; p < nprec && rp.body_exact; ++p)
            if (has[p] && rp.head[p + 1] - rp.head[p] != max_layers) rp.body_exact = false;
        rp.comp_exact = rp.body_exact;
        for (size_t gi = 0, i = 0; gi < rp.group_end.size() && rp.comp_exact; ++gi)
            for (; i < rp.group_end[gi]; ++i)
                if (max_comp > 1 && rp.order[i].compno != gi / rp.npoc) { rp.comp_exact = false; break; }
    }
    rp.hbytes.assign(rp.order.size(), 0);
    rp.dbytes.assign(rp.order.size(), 0);
    rp.dirty.assign(nprec, 1);
    rp.layers = max_layers;
}

// UB_NONE: no header bound (a block above its band's bit-planes; header_bits_ub).
constexpr uint32_t UB_NONE = 1u << 24;
#ifdef GRKGPU_CHECK_HEADER_UB
std::atomic<uint64_t> g_ub_checks{0}, g_ub_viol{0};
#endif

// the packets of one precinct, in layer order: header and body bytes
void probe_precinct(CodingParams &cp, TileEnc &te, RateProbe &rp, uint32_t p) {
    const uint32_t L = cp.numlayers;
    for (uint32_t q = rp.head[p]; q < rp.head[p + 1]; ++q) {
        const PacketId &pk = rp.order[rp.pos[q]];
        Resolution &res = te.tile->comps[pk.compno].res[pk.resno];
        BitCount w;
        packet_header(cp, te, res, pk.precno, pk.layno, w);
        uint64_t d = 0;
        for (uint32_t bandno = 0; bandno < res.numbands; ++bandno) {
            Band &b = res.bands[bandno];
            if (b.empty() || pk.precno >= b.precs.size()) continue;
            for (auto &c : b.precs[pk.precno].cblks) {
                const EncLayer &ly = (*te.layers)[(size_t)c.gidx * L + pk.layno];
                if (!ly.numpasses) continue;
                (*te.cblk)[c.gidx].incl_cur += ly.numpasses;
                d += ly.len;
            }
        }
        rp.hbytes[rp.pos[q]] = w.bytes;
        rp.dbytes[rp.pos[q]] = d;
#ifdef GRKGPU_CHECK_HEADER_UB
        // the bound body_fits takes for this packet (header_bits_ub summed per precinct)
        if (rp.layers == 1 && rp.body_exact && !(cp.csty & (CSTY_SOP | CSTY_EPH)) && rp.prec_bits[p] < (int64_t)UB_NONE) {
            ++g_ub_checks;
            if ((uint64_t)w.bytes > (uint64_t)(1 + rp.prec_bits[p]) / 7 + 2) ++g_ub_viol;
        }
#endif
    }
}

// T2::encode_packets_simulate (T2.cpp:126-192): the tile's packets of layers
// [0, max_layers) in THRESH_CALC order -- per component tile-part for the 4K
// cinema profile with a per-component size cap -- against max_len bytes.
// The per-packet sizes come from the precinct simulations (RateProbe); the
// walk in packet order then applies the reference's running budget check
// (simulate_packet's subtractions, SOP / EPH wrap-around included) and the
// per-component cap.
bool simulate_tile(CodingParams &cp, TileEnc &te, uint32_t max_layers, uint64_t max_len, RateProbe &rp) {
    const uint32_t max_comp = cp.max_comp_size > 0 ? cp.numcomps : 1;
    if (rp.layers != max_layers) probe_plan(cp, te, max_layers, rp);
    if (rp.bad) {
        for (uint32_t compno = 0, gi = 0; compno < max_comp; ++compno) {
            uint64_t comp_len = 0;
            for (uint32_t poc = 0; poc < rp.npoc; ++poc, ++gi) {
                for (size_t i = gi ? rp.group_end[gi - 1] : 0; i < rp.group_end[gi]; ++i) {
                    uint64_t b = 0;
                    if (!simulate_packet(cp, te, rp.order[i], max_len, &b)) return false;
                    comp_len += b;
                    max_len -= b;
                }
                if (cp.max_comp_size && comp_len > cp.max_comp_size) return false;
            }
        }
        return true;
    }
    std::vector<uint32_t> todo;
    for (uint32_t p = 0; p < rp.nprec; ++p)
        if (rp.dirty[p] && rp.head[p + 1] > rp.head[p]) todo.push_back(p);
    std::fill(rp.dirty.begin(), rp.dirty.end(), 0);
    g_rt.precs += todo.size();
    if (todo.size() > 16) {
        host_parallel_for(todo.size(), 8, [&](size_t a, size_t b) {
            for (size_t i = a; i < b; ++i) probe_precinct(cp, te, rp, todo[i]);
        });
    } else {
        for (uint32_t p : todo) probe_precinct(cp, te, rp, p);
    }
    const bool sop = (cp.csty & CSTY_SOP) != 0, eph = (cp.csty & CSTY_EPH) != 0;
    size_t i = 0, gi = 0;
    for (uint32_t compno = 0; compno < max_comp; ++compno) {
        uint64_t comp_len = 0;
        for (uint32_t poc = 0; poc < rp.npoc; ++poc, ++gi) {
            for (; i < rp.group_end[gi]; ++i) {
                uint64_t length = max_len, written = 0;
                if (sop) { length -= 6; written += 6; }
                if (rp.hbytes[i] > length) return false;
                written += rp.hbytes[i];
                length -= rp.hbytes[i];
                if (eph) { length -= 2; written += 2; }
                if (rp.dbytes[i] > length) return false;  // the body's blocks, each checked against what is left
                written += rp.dbytes[i];
                comp_len += written;
                max_len -= written;
            }
            if (cp.max_comp_size && comp_len > cp.max_comp_size) return false;
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// layer formation (TileProcessor.cpp:281-852)
// ---------------------------------------------------------------------------
template <class F>
void for_each_block(TileEnc &te, F f) {
    for (auto &tc : te.tile->comps)
        for (auto &res : tc.res)
            for (uint32_t b = 0; b < res.numbands; ++b)
                for (auto &pr : res.bands[b].precs)
                    for (auto &c : pr.cblks) f(c);
}

// The layer record of a block from its cumulative pass count (the per-block
// body of makelayer_* / make_layer_simple); the layer's distortion is summed
// into distolayer afterwards, in block order (sum_layer).
void set_layer(TileEnc &te, uint32_t gidx, uint32_t layno, uint32_t L, uint32_t cumul) {
    EncCblkState &s = (*te.cblk)[gidx];
    EncLayer &ly = (*te.layers)[(size_t)gidx * L + layno];
    const EncPass *P = te.passes;
    ly.numpasses = cumul - s.incl_prev;
    if (!ly.numpasses) {
        ly.disto = 0;
        return;
    }
    if (s.incl_prev == 0) {
        ly.len = P[s.pass0 + cumul - 1].rate;
        ly.data_off = 0;
        ly.disto = P[s.pass0 + cumul - 1].dd;
    } else {
        ly.len = P[s.pass0 + cumul - 1].rate - P[s.pass0 + s.incl_prev - 1].rate;
        ly.data_off = P[s.pass0 + s.incl_prev - 1].rate;
        ly.disto = P[s.pass0 + cumul - 1].dd - P[s.pass0 + s.incl_prev - 1].dd;
    }
}

// tile->distolayer[layno] += layer->disto over the blocks that contribute
// passes, in the reference's block order (floating-point sum order kept)
void sum_layer(TileEnc &te, uint32_t layno, uint32_t L) {
    double d = 0;
    for (Cblk *c : te.blist) {
        const EncLayer &ly = (*te.layers)[(size_t)c->gidx * L + layno];
        if (ly.numpasses) d += ly.disto;
    }
    te.distolayer[layno] = d;
}

// per-block loops of the layer formation: independent blocks, on the host pool
template <class F>
void blocks_parallel(TileEnc &te, F f) {
    host_parallel_for(te.blist.size(), 256, [&](size_t b0, size_t b1) {
        for (size_t i = b0; i < b1; ++i) f(*te.blist[i]);
    });
}

// makelayer_final (TileProcessor.cpp:783-852)
void makelayer_final(CodingParams &cp, TileEnc &te, uint32_t layno) {
    const uint32_t L = cp.numlayers;
    blocks_parallel(te, [&](Cblk &c) {
        EncCblkState &s = (*te.cblk)[c.gidx];
        if (layno == 0) { s.incl_prev = 0; s.incl_cur = 0; s.numlenbits = 0; }
        uint32_t cumul = s.incl_prev;
        if (s.numpasses > s.incl_prev) cumul = s.numpasses;
        set_layer(te, c.gidx, layno, L, cumul);
        if ((*te.layers)[(size_t)c.gidx * L + layno].numpasses) s.incl_prev = cumul;
    });
    sum_layer(te, layno, L);
}

// make_layer_simple's per-block pass selection (TileProcessor.cpp:700-760):
// the last pass whose slope against the passes taken so far reaches the
// threshold; *lo / *hi = the largest slope that failed / smallest that passed
// (the comparisons `thresh - slope < DBL_EPSILON` keep their outcomes for
// every threshold t with !(t - *lo < DBL_EPSILON) and t - *hi < DBL_EPSILON)
uint32_t simple_cumul(const EncCblkState &s, const EncPass *P, bool slopes, double thresh, double *lo, double *hi) {
    uint32_t cumul = s.incl_prev;
    double l = -HUGE_VAL, h = HUGE_VAL;
    if (thresh == 0) return s.numpasses;
    if (slopes && cumul == 0 && !s.z0 && !(thresh - s.s0max < DBL_EPSILON)) {
        // no pass taken yet, so every slope is dd / rate from zero; the
        // largest fails, so every one does (fl(thresh - x) is monotone in x):
        // none taken, lo = their std::max fold, hi untouched
        *lo = s.s0max;
        *hi = h;
        return 0;
    }
    for (uint32_t pn = s.incl_prev; pn < s.numpasses; ++pn) {
        const EncPass &ps = P[pn];
        uint32_t dr;
        double dd;
        if (cumul == 0) { dr = ps.rate; dd = ps.dd; }
        else {
            dr = ps.rate - P[cumul - 1].rate;
            dd = ps.dd - P[cumul - 1].dd;
        }
        if (!dr) {
            if (dd != 0) cumul = pn + 1;
            continue;
        }
        const double slope = dd / dr;
        if (thresh - slope < DBL_EPSILON) {
            cumul = pn + 1;
            h = std::min(h, slope);
        } else {
            l = std::max(l, slope);
        }
    }
    *lo = l;
    *hi = h;
    return cumul;
}

// makelayer_feasible's per-block pass selection (TileProcessor.cpp:300-330):
// passes up to the first hull slope <= thresh; the outcome holds for every
// threshold t with *lo <= t < *hi
uint32_t feasible_cumul(const EncCblkState &s, const EncPass *P, uint32_t thresh, uint32_t *lo, uint32_t *hi) {
    uint32_t cumul = s.incl_prev, l = 0, h = 0x10000;
    for (uint32_t pn = s.incl_prev; pn < s.numpasses; ++pn) {
        const EncPass &ps = P[pn];
        if (ps.slope) {
            if (ps.slope <= thresh) { l = ps.slope; break; }
            cumul = pn + 1;
            h = std::min<uint32_t>(h, ps.slope);
        }
    }
    *lo = l;
    *hi = h;
    return cumul;
}

// Upper bound on the packet-header bits block i's layer-0 record costs
// (packet_header with incl_cur = 0, numlenbits = 3): the inclusion tag tree
// at threshold 1 emits at most one bit per node of the leaf's path, the
// missing-MSB tree at most its value plus one per node, the rest exactly.
uint32_t header_bits_ub(const RateProbe &rp, size_t i, const EncCblkState &s, const EncLayer &ly, const EncPass *P) {
    uint32_t bits = rp.lev[i];
    if (!ly.numpasses) return bits;
    if (rp.bnumbps[i] < s.numbps) return UB_NONE;
    bits += (rp.bnumbps[i] - s.numbps) + rp.lev[i];
    const uint32_t n = ly.numpasses;
    bits += n == 1 ? 1 : n == 2 ? 2 : n <= 5 ? 4 : n <= 36 ? 9 : 16;
    int32_t increment = 0;
    uint32_t nump = 0, len = 0;
    for (uint32_t pn = 0; pn < n; ++pn) {
        ++nump;
        len += P[pn].len;
        if (P[pn].term || pn == n - 1) {
            increment = std::max<int32_t>(increment, floorlog2((int32_t)len) + 1 - (3 + floorlog2((int32_t)nump)));
            len = 0;
            nump = 0;
        }
    }
    bits += (uint32_t)increment + 1;  // comma code
    const uint32_t numlenbits = 3 + (uint32_t)increment;
    for (uint32_t pn = 0; pn < n; ++pn) {
        ++nump;
        if (P[pn].term || pn == n - 1) {
            bits += numlenbits + (uint32_t)floorlog2((int32_t)nump);
            nump = 0;
        }
    }
    return bits;
}

// One probe or the final formation of layer `layno` at a threshold
// (make_layer_simple, TileProcessor.cpp:675-780, or makelayer_feasible,
// :281-364).  A probe re-evaluates only the blocks whose bounds exclude the
// threshold (RateProbe) and marks the precincts of blocks whose record
// changed; the final formation evaluates every block and commits
// incl_prev.  need_sum: tile->distolayer[layno] is read afterwards.
template <bool FEASIBLE, class T>
void form_layer(CodingParams &cp, TileEnc &te, uint32_t layno, T thresh, bool final, bool need_sum, RateProbe &rp) {
    const uint32_t L = cp.numlayers;
    const EncPass *P = te.passes;
    const size_t nb = te.blist.size();
    // true if the block's layer record changed; *dlen = its change of bytes
    auto eval = [&](size_t i, int64_t *dlen) -> bool {
        const uint32_t gidx = rp.gidx[i];
        EncCblkState &s = (*te.cblk)[gidx];
        uint32_t cumul;
        if constexpr (FEASIBLE) cumul = feasible_cumul(s, P + s.pass0, (uint32_t)thresh, &rp.bu[i].lo, &rp.bu[i].hi);
        else cumul = simple_cumul(s, P + s.pass0, te.slopes, (double)thresh, &rp.bd[i].lo, &rp.bd[i].hi);
        EncLayer &ly = (*te.layers)[(size_t)gidx * L + layno];
        const uint32_t old = ly.numpasses;
        const int64_t oldlen = old ? (int64_t)ly.len : 0;
        set_layer(te, gidx, layno, L, cumul);
        *dlen = (ly.numpasses ? (int64_t)ly.len : 0) - oldlen;
        if (layno == 0) rp.ub[i] = header_bits_ub(rp, i, s, ly, P + s.pass0);
        return ly.numpasses != old;
    };
    std::vector<uint32_t> &redo = rp.redo;
    redo.clear();
    // the final formation re-evaluates only the blocks whose bounds exclude
    // the threshold, as a probe does: every block was evaluated by the
    // layer's first probe and its record is exact wherever its bounds hold
    const bool full = rp.fresh || (!FEASIBLE && thresh == 0);
    if (layno == 0 && (full || final))
        for (Cblk *c : te.blist) {
            EncCblkState &s = (*te.cblk)[c->gidx];
            s.incl_prev = 0; s.incl_cur = 0; s.numlenbits = 0;
        }
    if (full) {
        redo.resize(nb);
        for (size_t i = 0; i < nb; ++i) redo[i] = (uint32_t)i;
        rp.active = redo;
    } else {
        for (uint32_t i : rp.active) {
            bool ok = rp.valid[i] != 0;
            if constexpr (FEASIBLE) ok = ok && rp.bu[i].lo <= (uint32_t)thresh && (uint32_t)thresh < rp.bu[i].hi;
            else ok = ok && ((double)thresh - rp.bd[i].hi < DBL_EPSILON) && !((double)thresh - rp.bd[i].lo < DBL_EPSILON);
            if (!ok) redo.push_back(i);
        }
    }
    std::vector<uint8_t> &changed = rp.changed;
    std::vector<int64_t> &dlen = rp.dlen;
    std::vector<uint32_t> &ub_old = rp.ub_old;  // the layer-0 header bounds before this probe's re-evaluations
    changed.resize(redo.size());
    dlen.resize(redo.size());
    if (layno == 0 && !full) {
        ub_old.resize(redo.size());
        for (size_t j = 0; j < redo.size(); ++j) ub_old[j] = rp.ub[redo[j]];
    }
    g_rt.redo += redo.size();
    // A re-evaluation walks its block's pass records, ~0.5 KB away from the
    // previous block's: fetched PF blocks ahead, its wait is off the chain
    // (the real C5 frame's evaluations: 35 -> 19 M cycles of pass walking,
    // tests/cpp/pcrd_bench.cpp on its dumped pass records).
    constexpr size_t PF = 6;
    auto prefetch = [&](size_t j) {
        const EncCblkState &sp = (*te.cblk)[rp.gidx[redo[j]]];
        const char *pp = (const char *)(P + sp.pass0);
        for (size_t o = 0; o < (size_t)sp.numpasses * sizeof(EncPass); o += 64) __builtin_prefetch(pp + o);
    };
    auto eval_range = [&](size_t a, size_t b) {
        for (size_t j = a; j < std::min(b, a + PF); ++j) prefetch(j);
        for (size_t j = a; j < b; ++j) {
            if (j + PF < b) prefetch(j + PF);
            changed[j] = eval(redo[j], &dlen[j]);
        }
    };
    if (redo.size() > 512) {  // a probe's re-evaluations (~0.2 us each) on the pool from 512
        host_parallel_for(redo.size(), 128, eval_range);
    } else {
        eval_range(0, redo.size());
    }
    const bool keep = !final && (FEASIBLE || thresh != 0);
    if (full) {  // the layer's bytes (and first-layer header bounds) from scratch
        rp.body = 0;
        std::fill(rp.comp_body.begin(), rp.comp_body.end(), 0);
        std::fill(rp.prec_bits.begin(), rp.prec_bits.end(), 0);
        for (size_t i = 0; i < nb; ++i) {
            if (layno == 0) rp.prec_bits[rp.prec[i]] += rp.ub[i];
            const EncLayer &ly = (*te.layers)[(size_t)rp.gidx[i] * L + layno];
            if (!ly.numpasses) continue;
            rp.body += ly.len;
            rp.comp_body[rp.comp[i]] += ly.len;
        }
    }
    for (size_t j = 0; j < redo.size(); ++j) {
        const uint32_t i = redo[j];
        if (changed[j]) rp.dirty[rp.prec[i]] = 1;
        if (!full) {
            rp.body += dlen[j];
            rp.comp_body[rp.comp[i]] += dlen[j];
            if (layno == 0) rp.prec_bits[rp.prec[i]] += (int64_t)rp.ub[i] - (int64_t)ub_old[j];
        }
        rp.valid[i] = keep;
    }
    rp.fresh = false;
    if (final) {
        for (Cblk *c : te.blist) {
            EncCblkState &s = (*te.cblk)[c->gidx];
            const EncLayer &ly = (*te.layers)[(size_t)c->gidx * L + layno];
            if (ly.numpasses) s.incl_prev += ly.numpasses;
        }
        // incl_prev moved: every bound is stale, and the next layer's probes
        // simulate a different layer count (a new plan)
        std::fill(rp.valid.begin(), rp.valid.end(), 0);
        rp.fresh = true;
        rp.body_prev += (uint64_t)rp.body;
        for (size_t k = 0; k < rp.comp_prev.size(); ++k) rp.comp_prev[k] += (uint64_t)rp.comp_body[k];
        rp.body = 0;
        std::fill(rp.comp_body.begin(), rp.comp_body.end(), 0);
    }
    if (need_sum || final) sum_layer(te, layno, L);
}

// The probe's code-block bytes alone exceed the budget or a component cap:
// simulate_tile would return false (without SOP / EPH its running budget
// only shrinks by what each packet writes, so it never wraps).
bool body_over(CodingParams &cp, TileEnc &te, uint32_t max_layers, uint64_t max_len, RateProbe &rp) {
    if (cp.csty & (CSTY_SOP | CSTY_EPH)) return false;
    if (rp.layers != max_layers) probe_plan(cp, te, max_layers, rp);
    if (!rp.body_exact) return false;  // the walk's packets are not the records' bytes once each
    if (rp.body_prev + (uint64_t)rp.body > max_len) return true;
    if (cp.max_comp_size && rp.comp_exact)
        for (size_t k = 0; k < rp.comp_body.size(); ++k)
            if (rp.comp_prev[k] + (uint64_t)rp.comp_body[k] > cp.max_comp_size) return true;
    return false;
}

// The probe certainly fits: a single-layer search (the first layer's
// header bounds apply), no SOP / EPH, the plan's packets exactly the
// records, and code-block bytes plus every packet's header bound within the
// budget and each component cap -- simulate_tile's running budget then
// covers every packet, so it would return true.
bool body_fits(CodingParams &cp, TileEnc &te, uint32_t max_layers, uint64_t max_len, RateProbe &rp) {
    if (max_layers != 1 || (cp.csty & (CSTY_SOP | CSTY_EPH))) return false;
    if (rp.layers != max_layers) probe_plan(cp, te, max_layers, rp);
    if (!rp.body_exact) return false;
    uint64_t hb = 0;
    std::vector<uint64_t> chb(cp.numcomps, 0);
    for (uint32_t p = 0; p < rp.nprec; ++p) {
        const uint32_t npk = rp.head[p + 1] - rp.head[p];
        if (!npk) continue;
        if (rp.prec_bits[p] >= (int64_t)UB_NONE) return false;
        const uint64_t b = (uint64_t)npk * ((uint64_t)(1 + rp.prec_bits[p]) / 7 + 2);
        hb += b;
        chb[rp.prec_comp[p]] += b;
    }
    if ((uint64_t)rp.body + hb > max_len) return false;
    if (cp.max_comp_size) {
        if (!rp.comp_exact) return false;
        for (uint32_t k = 0; k < cp.numcomps; ++k)
            if ((uint64_t)rp.comp_body[k] + chb[k] > cp.max_comp_size) return false;
    }
    return true;
}

// RateProbe::active after a probe: keep the blocks whose layer record could
// still change for some threshold of [L, U] (the bisection interval, ends in
// either order in the search; every later probe of this layer is a midpoint
// of two points of it, so lies in it).  The bound tests are monotone in the
// threshold (a rounded difference is monotone), so a block valid at both ends
// is valid in between.
void prune_simple(RateProbe &rp, double L, double U) {
    size_t k = 0;
    for (uint32_t i : rp.active) {
        const bool keep = !rp.valid[i] || !(U - rp.bd[i].hi < DBL_EPSILON) || (L - rp.bd[i].lo < DBL_EPSILON);
        if (keep) rp.active[k++] = i;
    }
    rp.active.resize(k);
}
void prune_feasible(RateProbe &rp, uint32_t L, uint32_t U) {
    size_t k = 0;
    for (uint32_t i : rp.active) {
        const bool keep = !rp.valid[i] || !(rp.bu[i].lo <= L && U < rp.bu[i].hi);
        if (keep) rp.active[k++] = i;
    }
    rp.active.resize(k);
}

bool layer_needs_rate_control(const CodingParams &cp, uint32_t layno) {
    return (cp.disto_alloc == 1 && cp.rates[layno] > 0.0) || (cp.fixed_quality == 1 && cp.distoratio[layno] > 0.0f);
}

// make_single_lossless_layer (TileProcessor.cpp:272-279)
bool single_lossless(CodingParams &cp, TileEnc &te) {
    if (cp.numlayers == 1 && !layer_needs_rate_control(cp, 0)) {
        makelayer_final(cp, te, 0);
        return true;
    }
    return false;
}

// max squared error of the tile (maxSE, used only for fixed-quality layers)
double tile_max_se(const CodingParams &cp, TileEnc &te) {
    double maxSE = 0;
    for (uint32_t k = 0; k < cp.numcomps; ++k) {
        uint64_t numpix = 0;
        TileComp &tc = te.tile->comps[k];
        for (auto &res : tc.res)
            for (uint32_t b = 0; b < res.numbands; ++b)
                for (auto &pr : res.bands[b].precs)
                    for (auto &c : pr.cblks) numpix += (uint64_t)c.r.w() * c.r.h();
        const double m = (double)(((uint64_t)1 << cp.prec[k]) - 1);
        maxSE += m * m * (double)numpix;
    }
    return maxSE;
}

// pcrd_bisect_simple (TileProcessor.cpp:508-667)
bool pcrd_simple(CodingParams &cp, TileEnc &te, uint64_t len) {
    double cumdisto[100];
    const double K = 1;
    double min_slope = DBL_MAX, max_slope = -1;
    if (single_lossless(cp, te)) return true;
    const EncPass *P = te.passes;
    const double h0 = g_rt.on ? t2_ms() : 0;
    {  // min / max over every pass of every block (order-free), per chunk then combined
        std::mutex mu;
        host_parallel_for(te.blist.size(), 512, [&](size_t b0, size_t b1) {
            double mn = DBL_MAX, mx = -1;
            for (size_t i = b0; i < b1; ++i) {
                const EncCblkState &s = (*te.cblk)[te.blist[i]->gidx];
                if (te.slopes) {  // the per-block extremes, from the pass records' producer
                    if (s.smin < mn) mn = s.smin;
                    if (s.smax > mx) mx = s.smax;
                    continue;
                }
                for (uint32_t pn = 0; pn < s.numpasses; ++pn) {
                    const EncPass &ps = P[s.pass0 + pn];
                    int32_t dr;
                    double dd;
                    if (pn == 0) { dr = (int32_t)ps.rate; dd = ps.dd; }
                    else { dr = (int32_t)(ps.rate - P[s.pass0 + pn - 1].rate); dd = ps.dd - P[s.pass0 + pn - 1].dd; }
                    if (dr == 0) continue;
                    const double r = dd / dr;
                    if (r < mn) mn = r;
                    if (r > mx) mx = r;
                }
            }
            std::lock_guard<std::mutex> lk(mu);
            if (mn < min_slope) min_slope = mn;
            if (mx > max_slope) max_slope = mx;
        });
    }
    const double maxSE = cp.fixed_quality ? tile_max_se(cp, te) : 0.0;  // only the PSNR targets read it
    RateProbe rp;
    probe_init(cp, te, rp);
    if (g_rt.on) g_rt.hull += t2_ms() - h0;
    double upper = max_slope;
    for (uint32_t layno = 0; layno < cp.numlayers; ++layno) {
        if (layer_needs_rate_control(cp, layno)) {
            double lower = min_slope;
            const uint64_t maxlen = cp.rates[layno] > 0.0f ? std::min<uint64_t>((uint64_t)ceil(cp.rates[layno]), len) : len;
            double prevthresh = -1;
            const double distotarget = te.distotile - ((K * maxSE) / pow(10.0, cp.distoratio[layno] / 10.0));
            double thresh = 0;
            for (uint32_t i = 0; i < 128; ++i) {
                thresh = (upper == -1) ? lower : (lower + upper) / 2;
                const double f0 = g_rt.on ? t2_ms() : 0;
                form_layer<false>(cp, te, layno, thresh, false, cp.fixed_quality != 0, rp);
                ++g_rt.probes;
                if (g_rt.on) g_rt.form += t2_ms() - f0;
                if (prevthresh != -1 && (fabs(prevthresh - thresh)) < 0.001) break;
                prevthresh = thresh;
                if (cp.fixed_quality) {
                    const double achieved = layno == 0 ? te.distolayer[0] : cumdisto[layno - 1] + te.distolayer[layno];
                    if (achieved < distotarget) { upper = thresh; continue; }
                    lower = thresh;
                } else {
                    const double f1 = g_rt.on ? t2_ms() : 0;
                    const bool over = body_over(cp, te, layno + 1, maxlen, rp);
                    const bool sure = !over && body_fits(cp, te, layno + 1, maxlen, rp);
                    g_rt.skipped += over || sure;
                    const bool fits = sure || (!over && simulate_tile(cp, te, layno + 1, maxlen, rp));
                    if (g_rt.on) g_rt.sim += t2_ms() - f1;
                    if (!fits) lower = thresh;
                    else upper = thresh;
                    if (upper != -1) prune_simple(rp, std::min(lower, upper), std::max(lower, upper));
                }
            }
            const double good = (upper == -1) ? thresh : upper;
            form_layer<false>(cp, te, layno, good, true, true, rp);
            cumdisto[layno] = layno == 0 ? te.distolayer[0] : cumdisto[layno - 1] + te.distolayer[layno];
            upper = lower - 1;
        } else {
            makelayer_final(cp, te, layno);
            return true;
        }
    }
    return true;
}

// RateControl::convexHull + slopeToLog (RateControl.cpp:31-175)
uint16_t slope_to_log(double slope) {
    static const double cutoff = pow(2, 64), scale = 256 / log(2), shift = 1 << 16;
    if (slope > cutoff) slope = cutoff;
    double ls = log(slope) * scale - log(cutoff) * scale + shift;
    if (ls < 1) ls = 1;
    if (ls > 0xFFFF) ls = 0xFFFF;
    return (uint16_t)ls;
}

void convex_hull(EncPass *pass, uint32_t n) {
    std::vector<double> cache(n);
    for (uint32_t p = 0; p < n; p++) {
        EncPass *cur = pass + p;
        double dd = 0, dr = 0;
        int pi = (int)p;
        EncPass *ip = pass + pi;
        while (1) {
            dr += ip->len;
            dd += pi == 0 ? ip->dd : ip->dd - (ip - 1)->dd;
            if (dd <= 0) { cur->slope = 0; break; }
            pi--;
            ip--;
            if (pi == -1) {
                cache[p] = dd / dr;
                cur->slope = slope_to_log(cache[p]);
                break;
            }
            if (ip->slope == 0) continue;
            if (dr == 0) ip->slope = 0;
            else if ((cache[pi] * dr) <= dd) ip->slope = 0;
            else {
                cache[p] = dd / dr;
                cur->slope = slope_to_log(cache[p]);
                if (cur->slope >= ip->slope) ip->slope = 0;
                break;
            }
        }
    }
}

// pcrd_bisect_feasible (TileProcessor.cpp:371-506)
bool pcrd_feasible(CodingParams &cp, TileEnc &te, uint64_t len) {
    double cumdisto[100];
    const double K = 1;
    const bool sl = single_lossless(cp, te);
    uint32_t min_slope = USHRT_MAX;
    if (!sl) {  // per-block convex hulls (independent), then the smallest slope
        const double h0 = g_rt.on ? t2_ms() : 0;
        blocks_parallel(te, [&](Cblk &c) {
            EncCblkState &s = (*te.cblk)[c.gidx];
            convex_hull(te.passes + s.pass0, s.numpasses);
        });
        for (Cblk *c : te.blist) {
            const EncCblkState &s = (*te.cblk)[c->gidx];
            const EncPass *P = te.passes + s.pass0;
            for (uint32_t pn = 0; pn < s.numpasses; ++pn)
                if (P[pn].slope && P[pn].slope < min_slope) min_slope = P[pn].slope;
        }
        if (g_rt.on) g_rt.hull += t2_ms() - h0;
    }
    if (sl) {
        makelayer_final(cp, te, 0);
        return true;
    }
    const double maxSE = cp.fixed_quality ? tile_max_se(cp, te) : 0.0;  // only the PSNR targets read it
    RateProbe rp;
    probe_init(cp, te, rp);
    uint32_t upper = USHRT_MAX;
    for (uint32_t layno = 0; layno < cp.numlayers; ++layno) {
        uint32_t lower = min_slope;
        const uint64_t maxlen = cp.rates[layno] > 0.0f ? std::min<uint64_t>((uint64_t)ceil(cp.rates[layno]), len) : len;
        uint32_t prevthresh = 0;
        if (layer_needs_rate_control(cp, layno)) {
            const double distotarget = te.distotile - ((K * maxSE) / pow(10.0, cp.distoratio[layno] / 10.0));
            for (uint32_t i = 0; i < 128; ++i) {
                const uint32_t thresh = (lower + upper) >> 1;
                if (prevthresh != 0 && prevthresh == thresh) break;
                const double f0 = g_rt.on ? t2_ms() : 0;
                form_layer<true>(cp, te, layno, (uint16_t)thresh, false, cp.fixed_quality != 0, rp);
                ++g_rt.probes;
                prevthresh = thresh;
                if (cp.fixed_quality) {
                    const double achieved = layno == 0 ? te.distolayer[0] : cumdisto[layno - 1] + te.distolayer[layno];
                    if (achieved < distotarget) { upper = thresh; continue; }
                    lower = thresh;
                } else {
                    const double f1 = g_rt.on ? t2_ms() : 0;
                    const bool over = body_over(cp, te, layno + 1, maxlen, rp);
                    const bool sure = !over && body_fits(cp, te, layno + 1, maxlen, rp);
                    g_rt.skipped += over || sure;
                    const bool fits = sure || (!over && simulate_tile(cp, te, layno + 1, maxlen, rp));
                    if (g_rt.on) {
                        const double f2 = t2_ms();
                        g_rt.form += f1 - f0;
                        g_rt.sim += f2 - f1;
                    }
                    if (!fits) lower = thresh;
                    else upper = thresh;
                    prune_feasible(rp, std::min(lower, upper), std::max(lower, upper));
                }
            }
            form_layer<true>(cp, te, layno, (uint16_t)upper, true, true, rp);
            cumdisto[layno] = layno == 0 ? te.distolayer[0] : cumdisto[layno - 1] + te.distolayer[layno];
            upper = lower - 1;
        } else {
            makelayer_final(cp, te, layno);
        }
    }
    return true;
}

}  // namespace
#ifdef GRKGPU_CHECK_HEADER_UB
uint64_t header_ub_checks() { return g_ub_checks.load(); }
uint64_t header_ub_violations() { return g_ub_viol.load(); }
#endif

void block_slopes(EncCblkState &s, const EncPass *P) {
    double mn = DBL_MAX, mx = -1, m0 = -HUGE_VAL;
    bool z0 = false;
    for (uint32_t k = 0; k < s.numpasses; ++k) {
        const EncPass &ps = P[k];
        if (ps.rate) m0 = std::max(m0, ps.dd / ps.rate);
        else if (ps.dd != 0) z0 = true;
        int32_t dr;
        double dd;
        if (k == 0) { dr = (int32_t)ps.rate; dd = ps.dd; }
        else { dr = (int32_t)(ps.rate - P[k - 1].rate); dd = ps.dd - P[k - 1].dd; }
        if (dr == 0) continue;
        const double r = dd / dr;
        if (r < mn) mn = r;
        if (r > mx) mx = r;
    }
    s.smin = mn;
    s.smax = mx;
    s.s0max = m0;
    s.z0 = z0;
}

bool rate_allocate(CodingParams &cp, TileEnc &te, uint64_t len, RateStats *st) {
    te.distolayer.assign(cp.numlayers + 1, 0.0);
    te.blist.clear();
    for_each_block(te, [&](Cblk &c) { te.blist.push_back(&c); });
    if (!(cp.disto_alloc || cp.fixed_quality)) return true;
    g_rt = RateTrace{};
    const bool ok = cp.rate_algo == 0 ? pcrd_simple(cp, te, len) : pcrd_feasible(cp, te, len);
    if (st) {
        st->probes = g_rt.probes;
        st->skipped = g_rt.skipped;
        st->evals = g_rt.redo;
        st->sims = g_rt.precs;
        st->form_ms = g_rt.form;
        st->sim_ms = g_rt.sim;
    }
    return ok;
}

// ---------------------------------------------------------------------------
// distortion (t1.cpp:912-930, dwt_utils.cpp:132-166, mct.cpp:65-79)
// ---------------------------------------------------------------------------
namespace {
// sqrt energy gains (HTParams.cpp:54-96), float as in the reference
const float kG97L[34] = {1.0000e+00f, 1.4021e+00f, 2.0304e+00f, 2.9012e+00f, 4.1153e+00f, 5.8245e+00f, 8.2388e+00f,
    1.1652e+01f, 1.6479e+01f, 2.3304e+01f, 3.2957e+01f, 4.6609e+01f, 6.5915e+01f, 9.3217e+01f, 1.3183e+02f,
    1.8643e+02f, 2.6366e+02f, 3.7287e+02f, 5.2732e+02f, 7.4574e+02f, 1.0546e+03f, 1.4915e+03f, 2.1093e+03f,
    2.9830e+03f, 4.2185e+03f, 5.9659e+03f, 8.4371e+03f, 1.1932e+04f, 1.6874e+04f, 2.3864e+04f, 3.3748e+04f,
    4.7727e+04f, 6.7496e+04f, 9.5454e+04f};
const float kG97H[34] = {1.4425e+00f, 1.9669e+00f, 2.8839e+00f, 4.1475e+00f, 5.8946e+00f, 8.3472e+00f, 1.1809e+01f,
    1.6701e+01f, 2.3620e+01f, 3.3403e+01f, 4.7240e+01f, 6.6807e+01f, 9.4479e+01f, 1.3361e+02f, 1.8896e+02f,
    2.6723e+02f, 3.7792e+02f, 5.3446e+02f, 7.5583e+02f, 1.0689e+03f, 1.5117e+03f, 2.1378e+03f, 3.0233e+03f,
    4.2756e+03f, 6.0467e+03f, 8.5513e+03f, 1.2093e+04f, 1.7103e+04f, 2.4187e+04f, 3.4205e+04f, 4.8373e+04f,
    6.8410e+04f, 9.6747e+04f, 1.3682e+05f};
const float kG53L[34] = {1.0000e+00f, 1.2247e+00f, 1.3229e+00f, 1.5411e+00f, 1.7139e+00f, 1.9605e+00f, 2.2044e+00f,
    2.5047e+00f, 2.8277e+00f, 3.2049e+00f, 3.6238e+00f, 4.1033e+00f, 4.6423e+00f, 5.2548e+00f, 5.9462e+00f,
    6.7299e+00f, 7.6159e+00f, 8.6193e+00f, 9.7544e+00f, 1.1039e+01f, 1.2493e+01f, 1.4139e+01f, 1.6001e+01f,
    1.8108e+01f, 2.0493e+01f, 2.3192e+01f, 2.6246e+01f, 2.9702e+01f, 3.3614e+01f, 3.8041e+01f, 4.3051e+01f,
    4.8721e+01f, 5.5138e+01f, 6.2399e+01f};
const float kG53H[34] = {1.0458e+00f, 1.3975e+00f, 1.4389e+00f, 1.7287e+00f, 1.8880e+00f, 2.1841e+00f, 2.4392e+00f,
    2.7830e+00f, 3.1341e+00f, 3.5576e+00f, 4.0188e+00f, 4.5532e+00f, 5.1494e+00f, 5.8301e+00f, 6.5963e+00f,
    7.4663e+00f, 8.4489e+00f, 9.5623e+00f, 1.0821e+01f, 1.2247e+01f, 1.3860e+01f, 1.5685e+01f, 1.7751e+01f,
    2.0089e+01f, 2.2735e+01f, 2.5729e+01f, 2.9117e+01f, 3.2952e+01f, 3.7292e+01f, 4.2203e+01f, 4.7761e+01f,
    5.4051e+01f, 6.1170e+01f, 6.9226e+01f};

double getnorm(uint32_t level, uint32_t orient, bool rev) {
    const float *Lg = rev ? kG53L : kG97L, *Hg = rev ? kG53H : kG97H;
    // float products, widened on return (dwt_utils.cpp:143-166)
    switch (orient) {
        case 0: return (double)(float)(Lg[level] * Lg[level]);
        case 1: case 2: return (double)(float)(Lg[level + 1] * Hg[level]);
        case 3: return (double)(float)(Hg[level] * Hg[level]);
    }
    return 0;
}
}  // namespace

double t1_wmsedec_factor(uint32_t compno, uint32_t level, uint32_t orient, uint32_t qmfbid, double stepsize,
                         const double *mct_norms, uint32_t mct_numcomps) {
    double w1 = 1;
    if (mct_norms && compno < mct_numcomps) w1 = mct_norms[compno];
    return w1 * getnorm(level, orient, qmfbid == 1) * stepsize;
}

double t1_wmsedec(int32_t nmsedec, uint32_t compno, uint32_t level, uint32_t orient, int32_t bpno, uint32_t qmfbid,
                  double stepsize, const double *mct_norms, uint32_t mct_numcomps) {
    return t1_wmsedec_at(t1_wmsedec_factor(compno, level, orient, qmfbid, stepsize, mct_norms, mct_numcomps), nmsedec,
                         bpno);
}

}  // namespace grkgpu
