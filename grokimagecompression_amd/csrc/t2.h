// t2.h -- host Tier-2 of the MI355X JPEG 2000 path: packet iteration in the
// five progression orders with progression-order changes (POC) and tile-part
// division, quality layers, packet headers (tag trees, comma / pass-count
// codes, length indicators, SOP / EPH), and the rate-distortion layer
// formation (PCRD bisection) that decides which coding passes go into which
// layer.  Restated from the reference's behaviour (citations per function in
// t2.cpp); it stays on the host -- the GPU supplies the
// per-pass rates and the per-pass distortion terms.
#pragma once
#include <stdint.h>

#include <math.h>
#include <vector>

#include "codestream.h"

namespace grkgpu {

enum Prog : uint32_t { PROG_LRCP = 0, PROG_RLCP = 1, PROG_RPCL = 2, PROG_PCRL = 3, PROG_CPRL = 4 };

// One packet of a tile: (layer, resolution, component, precinct).
struct PacketId {
    uint32_t layno, resno, compno, precno;
};

// Encoder per-pass record (grk_tcd_pass): cumulative rate, bytes of this
// pass, terminated flag, cumulative distortion decrease, log slope (PCRD
// "feasible" algorithm).
struct EncPass {
    uint32_t rate, len;
    double dd;
    uint16_t slope;
    uint8_t term;
};

// Encoder per-(block, layer) record (grk_tcd_layer): passes, bytes and the
// byte offset of the layer's data within the block's MQ output.
struct EncLayer {
    uint32_t numpasses, len, data_off;
    double disto;
};

// Encoder state of one code-block across rate control and Tier-2.
struct EncCblkState {
    uint32_t numbps = 0, numpasses = 0, pass0 = 0;  // passes at passes[pass0 .. pass0 + numpasses)
    uint32_t incl_prev = 0;  // num_passes_included_in_previous_layers (layer formation)
    uint32_t incl_cur = 0;   // num_passes_included_in_current_layer (packet writer)
    uint32_t numlenbits = 0;
    uint64_t dev_off = 0;    // byte offset of the block's MQ output in the device slab
    // smallest / largest pass slope dd / dr over passes with dr != 0 (the
    // simple PCRD's search range, TileProcessor.cpp:528-560), when the pass
    // records' producer filled them (TileEnc::slopes)
    double smin = 0, smax = 0;
    // with them: the largest dd / rate over passes with rate != 0 (each pass
    // against none taken, folded with std::max in pass order from -HUGE_VAL),
    // and whether a pass has rate == 0 with dd != 0 -- a threshold this
    // slope fails takes none of the block's passes (simple_cumul)
    double s0max = -HUGE_VAL;
    bool z0 = false;
};

// Per-POC encoder state (the reference's tcp->pocs[] entries: user range +
// the tile-part odometer, PacketIter.cpp:925-1033, 1532-1799).
struct EncPoc {
    uint32_t resno0 = 0, compno0 = 0, layno1 = 0, resno1 = 0, compno1 = 0, prg1 = 0;
    uint32_t compS = 0, compE = 0, resS = 0, resE = 0, layS = 0, layE = 0, prcS = 0, prcE = 0;
    uint32_t txS = 0, txE = 0, tyS = 0, tyE = 0, dx = 0, dy = 0, prg = 0;
    uint32_t comp_t = 0, res_t = 0, lay_t = 0, prc_t = 0, tx0_t = 0, ty0_t = 0;
};

// Everything Tier-2 needs about one tile while encoding.
struct TileEnc {
    Tile *tile = nullptr;
    std::vector<EncCblkState> *cblk = nullptr;  // indexed by Cblk::gidx
    EncPass *passes = nullptr;  // the pass records, block b's at passes[cblk[b].pass0 ...]
    std::vector<EncLayer> *layers = nullptr;    // [gidx * numlayers + layno]
    std::vector<EncPoc> pocs;                   // numpocs + 1 entries (at least one)
    uint32_t packno = 0;                        // SOP packet counter
    double distotile = 0;
    std::vector<double> distolayer;
    std::vector<Cblk *> blist;                  // the tile's code-blocks in for_each_block order (rate control)
    bool slopes = false;                        // EncCblkState::smin / smax hold every block's pass slopes
};

// The slope fields of s (smin / smax / s0max / z0) from its pass records P
// (codec.cpp's pass-record fill; TileEnc::slopes).
void block_slopes(EncCblkState &s, const EncPass *P);

// number of POC entries of a tile (tcp->numpocs + 1)
inline uint32_t num_poc_entries(const CodingParams &cp) { return cp.numpocs ? cp.numpocs : 1; }

// ---- decoder -------------------------------------------------------------
// Packet order of a tile for decoding (T2::decode_packets over
// pi_create_decode, PacketIter.cpp:1187-1355 + the pi_next_* walks).
void decode_packet_order(const CodingParams &cp, const Tile &tile, std::vector<PacketId> &out);

// ---- encoder -------------------------------------------------------------
// tile-part count of each POC entry of the tile (j2k_calculate_tp /
// j2k_get_num_tp, j2k.cpp:2928-3048); also fixes cp.tp_pos
std::vector<uint32_t> tile_part_counts(CodingParams &cp, const Tile &tile);
// Initialise te.pocs from the coding parameters (j2k_setup_encoder POC copy, j2k.cpp:1864-1890).
void init_enc_pocs(const CodingParams &cp, TileEnc &te);

// Packets of tile-part (pino, tp_num) in FINAL_PASS order (T2::encode_packets
// with pi_initialise_encode + pi_init_encode, T2.cpp:64-125).
void encode_packet_order(const CodingParams &cp, TileEnc &te, uint32_t pino, uint32_t tp_num,
                         std::vector<PacketId> &out);

// Write one packet (T2::encode_packet, T2.cpp:859-1060): header bytes into
// hdr (SOP / EPH included), the packet's runs (header, then code-block layer
// data from the device slab) appended to plan.  Returns false if a layer
// exceeds the available bytes.
bool write_packet(const CodingParams &cp, TileEnc &te, const PacketId &pk, ByteBuf &hdr, std::vector<PlanItem> &plan);

// Rate allocation (TileProcessor::rate_allocate_encode, TileProcessor.cpp:
// 1649-1683): forms every layer of the tile; len = the tile buffer bound.
// what the bisection did (grkgpu_stats rate_*): probes, probes decided by
// their code-block bytes alone, block evaluations, precinct simulations and
// the time forming layers / simulating packets
struct RateStats {
    uint32_t probes = 0, skipped = 0;
    uint64_t evals = 0, sims = 0;
    double form_ms = 0, sim_ms = 0;
};
bool rate_allocate(CodingParams &cp, TileEnc &te, uint64_t len, RateStats *st = nullptr);
#ifdef GRKGPU_CHECK_HEADER_UB
// checked builds (tests/cpp/pcrd_bench.cpp): every simulated first-layer
// packet of a single-layer search is compared with the header bound the
// body_fits shortcut relies on; checks made / packets above their bound
uint64_t header_ub_checks();
uint64_t header_ub_violations();
#endif

// distortion weight of a pass (t1_getwmsedec, t1.cpp:912-930)
double t1_wmsedec(int32_t nmsedec, uint32_t compno, uint32_t level, uint32_t orient, int32_t bpno, uint32_t qmfbid,
                  double stepsize, const double *mct_norms, uint32_t mct_numcomps);
// the same in two steps, the block's constant first (w1 * w2 * stepsize,
// evaluated left to right as t1.cpp:912-930 does), then per pass:
// t1_wmsedec_at(factor, nmsedec, bpno) == t1_wmsedec(...) bit for bit
double t1_wmsedec_factor(uint32_t compno, uint32_t level, uint32_t orient, uint32_t qmfbid, double stepsize,
                         const double *mct_norms, uint32_t mct_numcomps);
inline double t1_wmsedec_at(double factor, int32_t nmsedec, int32_t bpno) {
    double wmsedec = factor * (1 << bpno);
    wmsedec *= wmsedec * nmsedec / 8192.0;
    return wmsedec;
}

}  // namespace grkgpu
