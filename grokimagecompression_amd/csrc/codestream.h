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

// Coding parameters as j2k_setup_encoder derives them (codestream/j2k.cpp:1609-2050)
struct CodingParams {
    uint32_t numcomps = 0;
    Rect image;
    uint32_t prec[16] = {};
    int32_t sgnd[16] = {};
    uint32_t numres = 6, cblkw = 6, cblkh = 6;
    int32_t irrev = 0, mct = 0;
    uint32_t tdx = 0, tdy = 0, tx0 = 0, ty0 = 0, tw = 1, th = 1;
    uint32_t numlayers = 1, prog = 0, cblksty = 0;
    StepSize ss[3 * 33 + 1];
    int32_t shift[16] = {};
};

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
    // decoder: segment chunks (offset into codestream, length)
    std::vector<std::pair<uint64_t, uint32_t>> chunks;
    uint32_t seglen = 0;
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
    std::vector<Resolution> res;
    uint64_t arena_off = 0;  // element offset of this tile-component's buffers
};

struct Tile {
    uint32_t index = 0;
    Rect r;
    std::vector<TileComp> comps;
};

// geometry (TileComponent.cpp:165-507)
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

// Encoder-side per-block results needed by T2.
struct BlockT2 {
    uint32_t numbps, numpasses, datalen;
    const uint32_t *rate;     // cumulative rates (numpasses)
    uint64_t dev_off;         // offset of the block's MQ bytes in the device slab
};

// The codestream is assembled on the device: the host writes headers into a
// small blob and a plan of (source, length) runs; a gather kernel copies the
// runs (header bytes or code-block bytes) into their final positions.
struct PlanItem {
    uint64_t src;   // kind 0: offset in the header blob; kind 1: offset in the MQ slab
    uint32_t len;
    uint32_t kind;
};

void write_main_header(ByteBuf &cs, const CodingParams &cp);
// one packet (T2.cpp:859-1110), layer 0 containing all passes: header bits go
// to `hdr`, the packet's runs are appended to `plan`
void encode_packet(TileComp &tc, uint32_t resno, uint32_t precno, const std::vector<BlockT2> &blk, ByteBuf &hdr,
                   std::vector<PlanItem> &plan);

// decoder
bool parse_main_header(const uint8_t *cs, size_t len, CodingParams &cp, size_t &first_sot, std::string &err);
// returns bytes consumed or -1
int64_t decode_packet(TileComp &tc, uint32_t resno, uint32_t precno, uint32_t layno, const uint8_t *p, size_t n,
                      uint64_t base_off);

}  // namespace grkgpu
