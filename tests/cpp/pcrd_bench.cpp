// pcrd_bench.cpp -- host-only harness for the rate allocator (t2.cpp
// rate_allocate): a DCI 4K cinema-like tile (4096x2160, 3 components, 7
// resolutions, 32x32 code-blocks, 256^2 precincts, CPRL with the profile's two
// POC entries, tile-parts per component, per-component cap) with synthetic
// per-pass rates and distortions, rate-allocated to a byte budget.  Prints the
// time and a digest of every block's layer records, so two builds of t2.cpp
// (e.g. before / after a change) can be compared on the same inputs.
//
//   g++ -O2 -std=c++17 -I<csrc> pcrd_bench.cpp <csrc>/t2.cpp <csrc>/codestream.cpp -lpthread
//   ./a.out [algo 0|1] [budget_bytes] [seed] [layers] [reps] [slopes 0|1] [terms 0|1|2] [dump]
// terms: codeword segment ends -- 0 the last pass only, 1 every pass (TERMALL),
// 2 the BYPASS pattern (passes 10, then the raw MRP and the cleanup of every
// later plane).  dump: real pass records of a cinema frame instead of the
// synthetic ones, as a one-off hook in codec.cpp wrote them before its
// rate_allocate call (round 5; the file is not kept): f64 distotile, u64
// tile byte bound, u32 layers (1), f64 rate, u64 component cap, then per
// block in for_each_cblk order u32 numbps, u32 numpasses, f64 smin, f64 smax
// and its EncPass records.  On the -cinema4K 24 frame of bench.py it
// reproduces the codec's probes / evaluations / simulations exactly.  Built with -DGRKGPU_CHECK_HEADER_UB it also prints how many
// simulated first-layer packets were checked against the header bound of
// t2.cpp's body_fits shortcut, and how many exceeded it (must be 0).
#include <float.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <random>

#include "t2.h"

using namespace grkgpu;

int main(int argc, char **argv) {
    const uint32_t algo = argc > 1 ? (uint32_t)atoi(argv[1]) : 0;
    const double budget = argc > 2 ? atof(argv[2]) : 1.29e6;
    const uint32_t seed = argc > 3 ? (uint32_t)atoi(argv[3]) : 1;
    const uint32_t L = argc > 4 ? (uint32_t)atoi(argv[4]) : 1;
    const int reps = argc > 5 ? atoi(argv[5]) : 3;
    const bool slopes = argc > 6 && atoi(argv[6]) != 0;  // per-block slope extremes precomputed
    const int terms = argc > 7 ? atoi(argv[7]) : 0;
    FILE *dump = argc > 8 ? fopen(argv[8], "rb") : nullptr;
    double dump_disto = 0;
    uint64_t dump_bound = 0;
    if (dump) {
        uint32_t nl = 0;
        if (fread(&dump_disto, 8, 1, dump) != 1 || fread(&dump_bound, 8, 1, dump) != 1 || fread(&nl, 4, 1, dump) != 1) return 2;
    }
    CodingParams cp;
    cp.numcomps = 3;
    cp.image = {0, 0, 4096, 2160};
    for (int k = 0; k < 3; ++k) { cp.prec[k] = 12; cp.shift[k] = 2048; }
    cp.numres = 7;
    cp.cblkw = cp.cblkh = 5;
    cp.irrev = 1;
    cp.mct = 1;
    cp.tdx = 4096; cp.tdy = 2160; cp.tw = cp.th = 1;
    cp.numlayers = L;
    cp.prog = PROG_CPRL;
    cp.csty = CSTY_PRT;
    for (int r = 0; r < 7; ++r) cp.prcw[r] = cp.prch[r] = 8;
    if (dump) {  // -cinema4K 24 as codec.cpp sets it: 6 resolutions, 256^2 precincts above the lowest
        cp.numres = 6;
        cp.prcw[0] = cp.prch[0] = 15;
        cp.pocs[0] = {0, 0, 1, 5, 3, PROG_CPRL};
        cp.pocs[1] = {5, 0, 1, 6, 3, PROG_CPRL};
    }
    cp.numpocs = 2;
    cp.pocs[0] = {0, 0, 1, 6, 3, PROG_CPRL};
    cp.pocs[1] = {6, 0, 1, 7, 3, PROG_CPRL};
    cp.rsiz = RSIZ_CINEMA_4K;
    cp.tp_on = true;
    cp.tp_flag = 'C';
    cp.disto_alloc = 1;
    cp.rate_algo = algo;
    for (uint32_t l = 0; l < L; ++l) cp.rates[l] = budget * (l + 1) / L;
    cp.max_comp_size = 1041666;
    if (dump) {  // the dumped tile's rate targets (a single layer)
        if (fread(&cp.rates[0], sizeof(cp.rates[0]), 1, dump) != 1 ||
            fread(&cp.max_comp_size, sizeof(cp.max_comp_size), 1, dump) != 1) return 2;
    }
    generate_qcd(cp);

    Tile tile;
    tile.r = tile_rect(cp, 0);
    tile.comps.resize(3);
    for (uint32_t k = 0; k < 3; ++k) build_tilecomp(tile.comps[k], tile.r, cp, k, true);
    std::vector<EncCblkState> cst;
    std::vector<EncPass> passes;
    std::mt19937 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    double distotile = 0;
    for (auto &tc : tile.comps)
        for (size_t r = 0; r < tc.res.size(); ++r)
            for (uint32_t b = 0; b < tc.res[r].numbands; ++b) {
                Band &band = tc.res[r].bands[b];
                for (auto &pr : band.precs)
                    for (auto &c : pr.cblks) {
                        c.gidx = (uint32_t)cst.size();
                        EncCblkState s;
                        if (dump) {
                            if (fread(&s.numbps, 4, 1, dump) != 1 || fread(&s.numpasses, 4, 1, dump) != 1 ||
                                fread(&s.smin, 8, 1, dump) != 1 || fread(&s.smax, 8, 1, dump) != 1) return 3;
                            s.pass0 = (uint32_t)passes.size();
                            passes.resize(passes.size() + s.numpasses);
                            if (s.numpasses && fread(passes.data() + s.pass0, sizeof(EncPass), s.numpasses, dump) != s.numpasses) return 3;
                            block_slopes(s, passes.data() + s.pass0);  // the dump's smin / smax recomputed, plus the rest
                            cst.push_back(s);
                            continue;
                        }
                        const uint32_t drop = (uint32_t)(U(rng) * 4);
                        s.numbps = band.numbps > drop + 1 ? band.numbps - drop : 1;
                        s.numpasses = 3 * s.numbps - 2;
                        s.pass0 = (uint32_t)passes.size();
                        uint32_t rate = 0;
                        double dd = 0;
                        for (uint32_t k = 0; k < s.numpasses; ++k) {
                            const uint32_t plane = (k + 2) / 3;  // 0 for the first cleanup pass
                            EncPass p{};
                            const double scale = std::pow(1.9, (double)plane);
                            const uint32_t inc = U(rng) < 0.08 ? 0 : (uint32_t)(U(rng) * scale * 3.0);
                            rate += inc;
                            p.len = inc;
                            p.rate = rate;
                            dd += std::ldexp(U(rng) + 0.05, 2 * (int)(s.numbps - plane)) * (1 + r);
                            p.dd = dd;
                            p.term = k + 1 == s.numpasses || terms == 1 ||
                                     (terms == 2 && (k == 9 || (k > 9 && (k - 10) % 3 != 0)));
                            passes.push_back(p);
                        }
                        // the slope fields codec.cpp's pass-record fill stores (TileEnc::slopes)
                        block_slopes(s, passes.data() + s.pass0);
                        distotile += dd;
                        cst.push_back(s);
                    }
            }
    if (dump) {
        distotile = dump_disto;
        fclose(dump);
    }
    std::vector<EncLayer> layers((size_t)cst.size() * L);
    double best = 1e30;
    uint64_t digest = 1469598103934665603ull;
    for (int rep = 0; rep < reps; ++rep) {
        std::vector<EncCblkState> cs = cst;
        std::vector<EncPass> ps = passes;
        std::fill(layers.begin(), layers.end(), EncLayer{});
        TileEnc te;
        te.tile = &tile;
        te.cblk = &cs;
        te.passes = ps.data();
        te.layers = &layers;
        te.slopes = slopes;
        init_enc_pocs(cp, te);
        te.distotile = distotile;
        CodingParams cpt = cp;
        const auto t0 = std::chrono::steady_clock::now();
        RateStats rs;
        if (!rate_allocate(cpt, te, dump ? dump_bound : (uint64_t)(budget * 1.2), &rs)) { printf("rate_allocate failed\n"); return 1; }
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        best = std::min(best, ms);
        digest = 1469598103934665603ull;
        uint64_t tot = 0;
        for (auto &ly : layers) {
            digest = (digest ^ ly.numpasses) * 1099511628211ull;
            digest = (digest ^ ly.len) * 1099511628211ull;
            tot += ly.len;
        }
        if (rep == 0)
            printf("blocks %zu passes %zu bytes %llu probes %u (%u by bytes alone) evals %llu sims %llu form_ms %.2f "
                   "sim_ms %.2f ", cst.size(), passes.size(), (unsigned long long)tot, rs.probes, rs.skipped,
                   (unsigned long long)rs.evals, (unsigned long long)rs.sims, rs.form_ms, rs.sim_ms);
    }
    printf("digest %016llx best_ms %.3f\n", (unsigned long long)digest, best);
#ifdef GRKGPU_CHECK_HEADER_UB
    printf("header_ub checks %llu violations %llu\n", (unsigned long long)header_ub_checks(),
           (unsigned long long)header_ub_violations());
#endif
    return 0;
}
