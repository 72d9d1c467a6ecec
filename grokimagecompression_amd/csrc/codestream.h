// codestream.h -- host side of the MI355X JPEG 2000 path: coding parameters,
// tile/resolution/band/precinct/code-block geometry, Tier-2 packets and the
// main/tile-part headers.  These stay on the host by design (SURVEY.md 1:
// "codestream markers, T2 packets, rate control ... stay on the host"); the
// GPU owns DC shift / MCT / DWT / T1.
#pragma once
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

namespace grkgpu {

struct Rect {
    uint32_t x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    uint32_t w() const { return x1 - x0; }
    uint32_t h() const { return y1 - y0; }
    bool empty() const { return x0 >= x1 || y0 >= y1; }
};

inline uint32_t ceildivpow2(uint32_t a, uint32_t e) { return (uint32_t)(((uint64_t)a + ((uint64_t)1 << e) - 1) >> e); }
inline uint32_t ceildiv(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + b - 1) / b); }
inline int32_t floorlog2(int32_t a) { int32_t l = 0; while (a > 1) { a >>= 1; l++; } return l; }

struct StepSize { uint32_t expn = 0, mant = 0; };

// One progression-order change (grk_poc, grok.h:393-410; POC marker
// j2k.cpp:4227-4306): resolutions [resno0, resno1), components [compno0,
// compno1), layers [0, layno1), progression prg.
struct PocSpec {
    uint32_t resno0 = 0, compno0 = 0, layno1 = 0, resno1 = 0, compno1 = 0, prg = 0;
};

constexpr uint32_t CSTY_PRT = 1, CSTY_SOP = 2, CSTY_EPH = 4;  // Scod bits (j2k.h J2K_CP_CSTY_*)
constexpr uint16_t RSIZ_CINEMA_2K = 3, RSIZ_CINEMA_4K = 4;     // grok.h:160-161
constexpr uint16_t RSIZ_PART2 = 0x8000, RSIZ_EXT_MCT = 0x0100;  // GRK_PROFILE_PART2, GRK_EXTENSION_MCT

// Coding style and quantisation of one component (the reference's grk_tccp):
// COD / COC and QCD / QCC of the main header or of a tile's first tile-part
// header, resolved in the order of precedence tile COC > tile COD > main COC
// > main COD (QCC / QCD alike; j2k_read_cod / _coc / _qcd / _qcc,
// j2k.cpp:3829-4160).  The encoder writes one COD / QCD: every component
// gets the global values (sync_comps).
struct CompParams {
    uint32_t numres = 6, cblkw = 6, cblkh = 6, cblksty = 0;
    uint32_t csty = 0;  // Scoc (tccp->csty): the precinct flag
    int32_t irrev = 0;
    uint8_t prcw[33], prch[33];
    uint32_t qntsty = 0, numgbits = 2, nsteps = 0;
    StepSize ss[3 * 33 + 1];
};

// A PPM / PPT marker segment (packed packet headers): its index Zppm / Zppt
// and where its data lies in the codestream.
struct PpxSeg {
    uint32_t z;
    size_t off, len;
};

// Coding parameters as j2k_setup_encoder derives them (codestream/j2k.cpp:1609-2050)
struct CodingParams {
    uint32_t numcomps = 0;
    Rect image;
    uint32_t prec[16] = {};
    int32_t sgnd[16] = {};
    uint32_t dx[16] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};  // SIZ XRsiz / YRsiz: component subsampling
    uint32_t dy[16] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
    uint32_t numres = 6, cblkw = 6, cblkh = 6;
    int32_t irrev = 0, mct = 0;
    uint32_t tdx = 0, tdy = 0, tx0 = 0, ty0 = 0, tw = 1, th = 1;
    uint32_t numlayers = 1, prog = 0, cblksty = 0;
    StepSize ss[3 * 33 + 1];
    uint32_t numgbits = 2;  // guard bits (QCD Sqcd >> 5; the encoder writes 2, j2k.cpp:1834)
    uint32_t qntsty = 0;    // QCD Sqcd & 0x1f (0 none, 2 scalar expounded), as read; nsteps step sizes
    uint32_t nsteps = 0;
    int32_t shift[16] = {};
    // coding style (Scod): precinct partition, SOP, EPH; log2 precinct size per resolution
    uint32_t csty = 0;
    uint8_t prcw[33], prch[33];
    // progression-order changes (0 = none)
    uint32_t numpocs = 0;
    PocSpec pocs[32];
    uint16_t rsiz = 0;
    // tile-parts (grk_cparameters tp_on / tp_flag; tp_pos derived, j2k.cpp:2955-2958)
    bool tp_on = false;
    char tp_flag = 0;
    uint32_t tp_pos = 0;
    // rate control (grk_cparameters cp_disto_alloc / cp_fixed_quality /
    // rateControlAlgorithm; tcp->rates in bytes after j2k_update_rates)
    uint32_t disto_alloc = 1, fixed_quality = 0, rate_algo = 0;
    double rates[100] = {};
    double distoratio[100] = {};
    uint64_t max_cs_size = 0, max_comp_size = 0;
    uint32_t nb_tile_parts = 1;  // per tile (tcp->m_nb_tile_parts)
    // ROI up-shift per component (tccp->roishift: grk_compress -ROI, the RGN
    // marker, j2k.cpp:1997-2001 / 5482-5604): adds to every band's bit-plane
    // count, and the decoder shifts decoded magnitudes >= 2^roishift down
    uint8_t roishift[16] = {};
    // custom array-based MCT (mct == 2, Part 2; j2k.cpp:1899-1961): the
    // encoding matrix in 13-bit fixed point, its float inverse (written to
    // the codestream) and the inverse's column norms (rate-control weights)
    int32_t mct_coding[16 * 16] = {};
    float mct_decoding[16 * 16] = {};
    double mct_norms[16] = {};
    // per component (decoder: COC / QCC resolved; encoder: sync_comps)
    CompParams comp[16];
    bool coc_set[16] = {}, qcc_set[16] = {};  // main-header COC / QCC seen
    uint32_t main_qntsty = 0, main_nsteps = 0;  // the main QCD's (tcp->main_qcd_qntsty / _numStepSizes)
    std::vector<PpxSeg> ppm;                  // main-header PPM segments
    CodingParams() {
        for (int i = 0; i < 33; ++i) prcw[i] = prch[i] = 15;
    }
};

// Part-2 MCT: matrix_inversion_f restated (false: singular)
bool mct_invert(const float *src, float *dst, uint32_t n);

// COD's coding style / QCD's quantisation -> component k (the global fields)
void comp_style_from_cod(CodingParams &cp, uint32_t k);
void comp_quant_from_qcd(CodingParams &cp, uint32_t k);
// every component from the global COD / QCD values (the encoder's one COD / QCD)
void sync_comps(CodingParams &cp);
// the QCD step-size count check of j2k.cpp:868-930 over a tile's resolved
// components: qcc = main QCC seen, tile_qcd / tile_qcc = the tile's own
bool check_qcd_steps(const CodingParams &cp, const bool *qcc, bool tile_qcd, const bool *tile_qcc, std::string &err);
// COC / QCC marker segment bodies (size bytes) -> cp.comp[...]; returns the
// component or -1 when malformed
int32_t parse_coc(const uint8_t *p, uint32_t size, CodingParams &cp, std::string &err);
int32_t parse_qcc(const uint8_t *p, uint32_t size, CodingParams &cp, std::string &err);
// COD / QCD marker segment bodies -> the global fields
bool parse_cod(const uint8_t *p, uint32_t size, CodingParams &cp, std::string &err);
bool parse_qcd(const uint8_t *p, uint32_t size, CodingParams &cp, std::string &err);

// TagTree (codestream/TagTree.cpp)
struct TagTree {
    struct Node { int64_t value, low; int32_t parent; int32_t known; };
    std::vector<Node> nodes;
    void init(uint32_t nh, uint32_t nv);
    void reset();
    void setvalue(uint32_t leaf, int64_t v);
};

struct Cblk {
    Rect r;                 // band coordinates
    uint32_t bx = 0, by = 0;  // offset in the tile-component (Mallat) buffer
    uint32_t gidx = 0;      // index in the flat block table
    // T2 state
    uint32_t numbps = 0, numpasses = 0, numlenbits = 0;
    bool included = false;
    // decoder: codeword segments (grk_tcd_seg): passes, bytes and the chunks
    // (offset into the codestream, length) holding them.  One segment unless
    // the code-block style terminates passes (TERMALL: one per pass; BYPASS:
    // 10 passes, then raw / MQ segments of 2 and 1).
    struct Seg {
        uint32_t numpasses = 0, len = 0, maxpasses = 109;
        std::vector<std::pair<uint64_t, uint32_t>> chunks;
    };
    std::vector<Seg> segs;
    uint32_t seglen = 0;  // bytes over all segments
};

struct Precinct {
    Rect r;
    uint32_t cw = 0, ch = 0;
    std::vector<Cblk> cblks;
    TagTree incl, imsb;
};

struct Band {
    Rect r;
    uint32_t bandno = 0;
    float stepsize = 0.f;
    uint32_t inv_step = 0;
    uint32_t numbps = 0;
    std::vector<Precinct> precs;
    bool empty() const { return r.empty(); }
};

struct Resolution {
    Rect r;
    uint32_t pw = 0, ph = 0, numbands = 0;
    Band bands[3];
};

struct TileComp {
    Rect r;
    uint32_t numres = 0;
    int32_t irrev = 0;  // 9/7 (COD / COC transform 0)
    std::vector<Resolution> res;
    uint64_t arena_off = 0;  // element offset of this tile-component's buffers
};

struct Tile {
    uint32_t index = 0;
    Rect r;
    std::vector<TileComp> comps;
};

// geometry (TileComponent.cpp:165-507); comp_rect: a rectangle of the
// reference grid on a component's subsampled grid (ceil of each coordinate / dx, dy)
Rect comp_rect(const Rect &r, uint32_t dx, uint32_t dy);
void build_tilecomp(TileComp &tc, const Rect &tr, const CodingParams &cp, uint32_t compno, bool encoder);
Rect tile_rect(const CodingParams &cp, uint32_t tileno);
// QCD generation (HTParams.cpp:164-260)
void generate_qcd(CodingParams &cp);

// growable byte buffer
struct ByteBuf {
    std::vector<uint8_t> v;
    void put8(uint32_t x) { v.push_back((uint8_t)x); }
    void put16(uint32_t x) { put8(x >> 8); put8(x); }
    void put32(uint32_t x) { put16(x >> 16); put16(x); }
    void putn(const uint8_t *p, size_t n) { v.insert(v.end(), p, p + n); }
    void set32(size_t at, uint32_t x) {
        v[at] = (uint8_t)(x >> 24); v[at + 1] = (uint8_t)(x >> 16); v[at + 2] = (uint8_t)(x >> 8); v[at + 3] = (uint8_t)x;
    }
    size_t size() const { return v.size(); }
};
// the Part-2 MCT marker group (CBD, MCT x 2, MCC, MCO) of a custom-MCT encode
void write_mct_group(ByteBuf &cs, const CodingParams &cp);


// The codestream is assembled on the device: the host writes headers into a
// small blob and a plan of (source, length) runs; a gather kernel copies the
// runs (header bytes or code-block bytes) into their final positions.
struct PlanItem {
    uint64_t src;   // kind 0: offset in the header blob; kind 1: offset in the MQ slab
    uint32_t len;
    uint32_t kind;
};

// main header up to (not including) the first SOT: SOC SIZ COD QCD [TLM] [POC] COM
// (j2k_setup_header_writing, j2k.cpp:2330-2374).  tlm_at receives the offset
// of the TLM marker's tile-part records (0 without TLM).
// packet-header bit writer / reader (codestream/BitIO.cpp): after an 0xFF
// byte only 7 bits are used (bit stuffing)
struct BitWriter {
    ByteBuf &out;
    uint32_t buf = 0, ct = 8;
    explicit BitWriter(ByteBuf &o) : out(o) {}
    void byteout() { out.put8(buf); ct = (buf == 0xff) ? 7 : 8; buf = 0; }
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
    // TagTree::encode (TagTree.cpp:251-287)
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

void write_main_header(ByteBuf &cs, const CodingParams &cp, size_t *tlm_at = nullptr, uint32_t total_tile_parts = 0);
// POC marker (j2k_write_poc_in_memory, j2k.cpp:4227-4306)
void write_poc(ByteBuf &cs, const CodingParams &cp);
// decoder
bool parse_main_header(const uint8_t *cs, size_t len, CodingParams &cp, size_t &first_sot, std::string &err);
// POC marker segment body of `size` bytes (main or tile-part header)
bool parse_poc(const uint8_t *p, uint32_t size, CodingParams &cp);
// returns bytes consumed or -1 (T2::read_packet_header / read_packet_data,
// T2.cpp:314-725); csty: SOP / EPH markers; packno: SOP packet counter;
// skip_data: a layer beyond the decoded ones (T2::skip_packet); cblksty: the
// code-block style (segment boundaries)
// hdr: packed packet headers (PPM / PPT, j2k.cpp:4693-4990): the packet's
// header bits are read from hdr->p + hdr->off (advanced past them and the
// EPH), its SOP marker and body from p; nullptr: everything from p
struct PackedHdr {
    const uint8_t *p = nullptr;
    size_t n = 0, off = 0;
};
int64_t decode_packet(TileComp &tc, uint32_t resno, uint32_t precno, uint32_t layno, const uint8_t *p, size_t n,
                      uint64_t base_off, uint32_t csty = 0, uint32_t *packno = nullptr, bool skip_data = false,
                      uint32_t cblksty = 0, PackedHdr *hdr = nullptr);

}  // namespace grkgpu
