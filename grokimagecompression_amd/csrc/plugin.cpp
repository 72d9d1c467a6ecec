// libgrok_plugin.so: Grok's minpf plugin ABI on top of libgrk_mi355x.so
// (include/grk_plugin_abi.h).  Host side: grok.cpp:810-955,
// TileProcessor.cpp:994-1012, plugin_bridge.cpp:24-258.
//
// Encode: the host (grk_compress, or any grk_* user) calls
// grk_plugin_encode(params, cb) -> plugin_encode(params, internal_cb).  The
// plugin reads the input image, codes every tile-component up to and
// including Tier-1 on the GPU (grkgpu_encode_blocks), describes the result as
// a grk_plugin_tile and calls back; the host's grk_encode_with_plugin then
// skips DC shift / MCT / DWT / T1 and runs rate control + Tier-2 on the
// plugin's code-blocks.  Pass rates follow the bridge's convention: the host
// takes rate + 1, clamps it to the block length and steps back over a
// trailing 0xFF (plugin_bridge.cpp:236-255), so a pass whose final rate is R
// is handed over as R - 1.
#include "../../include/grk_plugin_abi.h"
#include "../../include/grk_mi355x.h"

#include <dirent.h>
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define PLUGIN_API __attribute__((visibility("default")))

namespace {
std::mutex g_mu;
grkgpu_ctx *g_ctx = nullptr;  // one GPU context per loaded plugin (grok's plugin manager is a global too)
bool g_verbose = false;
int32_t g_device = 0;  // grk_plugin_init_info.deviceId: -1 = every device (grok.h:1816-1821)
// The host-vs-accelerator parity harness of the reference (grok.h:1790-1808,
// plugin_get_debug_state): with GRK_PLUGIN_STATE_DEBUG the host runs its own
// Tier-1 on the coefficients the plugin hands over as image data and checks
// every block of the plugin against it (plugin_bridge.cpp:144-258: pass
// counts, bytes, rates, distortion within 1 %), warning on any difference.
// A diagnostic state, chosen when the plugin is initialised:
// GRKGPU_PLUGIN_DEBUG_STATE=<state bits> in the environment (0 / unset:
// production, GRK_PLUGIN_STATE_NO_DEBUG).  Only the DEBUG bit is offered.
uint32_t g_debug_state = GRK_PLUGIN_STATE_NO_DEBUG;

void batch_end();
int32_t exit_plugin(void) {
    batch_end();  // a batch still running when the host unloads the plugin
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx) grkgpu_destroy(g_ctx);
    g_ctx = nullptr;
    return 0;
}
// minpf object factory: Grok never calls these for the T1 plugin (Plugin.cpp:24-31)
void *create_object(minpf_object_params *) { return nullptr; }
int32_t destroy_object(void *) { return 0; }

void log(const char *msg) {
    if (g_verbose) fprintf(stderr, "[grok mi355x plugin] %s\n", msg);
}

// ---- input image: binary PGM / PPM, as grk_compress's PNMFormat reads it
// (PNMFormat.cpp:343-460: precision = bits of maxval, at least 8; 1 byte per
// sample up to 8 bits, else 2 big-endian bytes) ----
struct Pnm {
    uint32_t w = 0, h = 0, c = 0, prec = 0;
    std::vector<int32_t> planes;  // (c, h, w)
};

bool pnm_token(FILE *f, uint32_t *v) {
    int ch;
    do {
        ch = fgetc(f);
        if (ch == '#')
            while (ch != '\n' && ch != EOF) ch = fgetc(f);
    } while (ch == ' ' || ch == '\t' || ch == '\n' || ch == '\r');
    if (ch < '0' || ch > '9') return false;
    uint64_t x = 0;
    while (ch >= '0' && ch <= '9') {
        x = x * 10 + (uint32_t)(ch - '0');
        if (x > 0xffffffffu) return false;
        ch = fgetc(f);
    }
    *v = (uint32_t)x;
    return ch == ' ' || ch == '\t' || ch == '\n' || ch == '\r';
}

bool read_pnm(const char *path, Pnm &img) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    std::unique_ptr<FILE, int (*)(FILE *)> guard(f, fclose);
    char magic[2];
    if (fread(magic, 1, 2, f) != 2 || magic[0] != 'P' || (magic[1] != '5' && magic[1] != '6')) return false;
    uint32_t maxval;
    if (!pnm_token(f, &img.w) || !pnm_token(f, &img.h) || !pnm_token(f, &maxval)) return false;
    if (!img.w || !img.h || !maxval || maxval > 65535) return false;
    img.c = magic[1] == '6' ? 3 : 1;
    uint32_t prec = 1;
    while (prec < 16 && (maxval >> prec)) ++prec;
    img.prec = prec < 8 ? 8 : prec;
    const bool one = img.prec < 9;
    const uint64_t area = (uint64_t)img.w * img.h;
    img.planes.resize(area * img.c);
    std::vector<uint8_t> row((size_t)img.w * img.c * (one ? 1 : 2));
    for (uint32_t y = 0; y < img.h; ++y) {
        if (fread(row.data(), 1, row.size(), f) != row.size()) return false;
        for (uint32_t x = 0; x < img.w; ++x)
            for (uint32_t k = 0; k < img.c; ++k) {
                const size_t i = (size_t)x * img.c + k;
                const int32_t v = one ? row[i] : (int32_t)((row[2 * i] << 8) | row[2 * i + 1]);
                img.planes[(size_t)k * area + (size_t)y * img.w + x] = v;
            }
    }
    return true;
}

// grk_cparameters -> grkgpu_cparams (the subset that shapes the partition
// and the Tier-1 output; rate control and Tier-2 stay with the host)
bool map_params(const grkp_cparameters *g, uint32_t numcomps, grkgpu_cparams *p) {
    grkgpu_default_cparams(p);
    p->numresolution = g->numresolution;
    p->cblockw_init = g->cblockw_init;
    p->cblockh_init = g->cblockh_init;
    p->irreversible = g->irreversible ? 1 : 0;
    // tcp_mct 255 = "decide from the image" (grk_compress.cpp:1997-1998)
    p->tcp_mct = g->tcp_mct == 255 ? -1 : g->tcp_mct;
    if (g->tcp_mct == 2 || g->mct_data) return false;  // custom MCT
    // mode switches: the host's plugin path writes one codeword segment per
    // block (encode_synch_with_plugin never sets pass->term), so only the
    // single-segment ones travel: RESET, VSC, PTERM, SEGSYM -- not TERMALL,
    // BYPASS or HT
    if ((g->cblk_sty & ~0x3Au) || g->isHT) return false;
    if (g->subsampling_dx != 1 || g->subsampling_dy != 1) return false;
    if (g->tile_size_on) return false;  // the host hands ONE plugin tile to every tile (j2k.cpp:2059-2069)
    p->cp_tx0 = g->cp_tx0;
    p->cp_ty0 = g->cp_ty0;
    p->tcp_numlayers = g->tcp_numlayers;
    for (int i = 0; i < 100; ++i) {
        p->tcp_rates[i] = g->tcp_rates[i];
        p->tcp_distoratio[i] = g->tcp_distoratio[i];
    }
    p->cp_disto_alloc = (int32_t)g->cp_disto_alloc;
    p->cp_fixed_quality = (int32_t)g->cp_fixed_quality;
    p->rate_control_algorithm = g->rateControlAlgorithm == 255 ? 0 : (int32_t)g->rateControlAlgorithm;
    p->csty = g->csty;
    p->res_spec = g->res_spec;
    for (int i = 0; i < 33; ++i) {
        p->prcw_init[i] = g->prcw_init[i];
        p->prch_init[i] = g->prch_init[i];
    }
    p->prog_order = g->prog_order;
    p->numpocs = g->numpocs > 32 ? 32 : g->numpocs;
    for (uint32_t i = 0; i < p->numpocs; ++i)
        p->POC[i] = {g->POC[i].tile, g->POC[i].resno0, g->POC[i].compno0, g->POC[i].layno1, g->POC[i].resno1,
                     g->POC[i].compno1, g->POC[i].prg1};
    p->tp_on = g->tp_on;
    p->tp_flag = g->tp_flag;
    p->rsiz = g->rsiz;
    p->framerate = (uint32_t)g->framerate;
    p->max_cs_size = g->max_cs_size;
    p->max_comp_size = g->max_comp_size;
    p->cblk_sty = g->cblk_sty;
    if (g->roi_compno >= 0) {
        p->roi_compno = g->roi_compno;
        p->roi_shift = g->roi_shift;
    }
    (void)numcomps;
    return true;
}

// Does layer l need rate control (TileProcessor::layer_needs_rate_control,
// TileProcessor.cpp:254-260)?  The cinema profiles always do: their layer
// rate comes from the profile's size caps (j2k set_cinema_parameters).
bool layer_rc(const grkp_cparameters *g, uint32_t l) {
    if (g->rsiz == GRKGPU_PROFILE_CINEMA_2K || g->rsiz == GRKGPU_PROFILE_CINEMA_4K) return true;
    return (g->cp_disto_alloc && g->tcp_rates[l] > 0) || (g->cp_fixed_quality && g->tcp_distoratio[l] > 0);
}
bool needs_distortion(const grkp_cparameters *g) {
    for (uint32_t l = 0; l < g->tcp_numlayers && l < 100; ++l)
        if (layer_rc(g, l)) return true;
    return false;
}

// The grk_plugin_tile tree over the exported code-blocks: the host walks it
// by (component, resolution, band, precinct, code-block) index
// (plugin_bridge.cpp:150-156), so every level is an index-addressed array.
struct TileTree {
    grk_plugin_tile tile{};
    std::vector<grk_plugin_tile_component> comps;
    std::vector<grk_plugin_tile_component *> comp_ptrs;
    std::vector<std::vector<grk_plugin_resolution>> res;
    std::vector<std::vector<grk_plugin_resolution *>> res_ptrs;
    std::vector<std::unique_ptr<grk_plugin_band>> bands;
    std::vector<std::vector<grk_plugin_band *>> band_ptrs;
    std::vector<std::unique_ptr<grk_plugin_precinct>> precs;
    std::vector<std::vector<grk_plugin_precinct *>> prec_ptrs;
    std::vector<grk_plugin_code_block> blocks;
    std::vector<std::vector<grk_plugin_code_block *>> block_ptrs;
};

bool build_tree(const grkgpu_block_info *b, uint32_t n, uint32_t numcomps, uint32_t numres, TileTree &T) {
    // sizes per level from the block list (canonical order)
    std::vector<std::vector<std::vector<uint32_t>>> nprec(numcomps, std::vector<std::vector<uint32_t>>(numres, {0, 0, 0}));
    std::vector<std::vector<std::vector<std::vector<uint32_t>>>> nblk(
        numcomps, std::vector<std::vector<std::vector<uint32_t>>>(numres, std::vector<std::vector<uint32_t>>(3)));
    for (uint32_t i = 0; i < n; ++i) {
        if (b[i].tileno != 0 || b[i].compno >= numcomps || b[i].resno >= numres) return false;
        const uint32_t bi = b[i].resno == 0 ? 0 : b[i].bandno - 1;
        if (bi > 2) return false;
        auto &np = nprec[b[i].compno][b[i].resno][bi];
        np = std::max(np, b[i].precno + 1);
        auto &nb = nblk[b[i].compno][b[i].resno][bi];
        if (nb.size() < np) nb.resize(np, 0);
        nb[b[i].precno] = std::max(nb[b[i].precno], b[i].cblkno + 1);
    }
    T.blocks.assign(n, grk_plugin_code_block{});
    T.comps.assign(numcomps, grk_plugin_tile_component{});
    T.comp_ptrs.resize(numcomps);
    T.res.assign(numcomps, std::vector<grk_plugin_resolution>(numres));
    T.res_ptrs.assign(numcomps, std::vector<grk_plugin_resolution *>(numres));
    std::vector<std::vector<std::vector<grk_plugin_band *>>> bandp(numcomps, std::vector<std::vector<grk_plugin_band *>>(numres));
    std::vector<std::vector<std::vector<std::vector<grk_plugin_precinct *>>>> precp(
        numcomps, std::vector<std::vector<std::vector<grk_plugin_precinct *>>>(numres, std::vector<std::vector<grk_plugin_precinct *>>(3)));
    for (uint32_t k = 0; k < numcomps; ++k) {
        T.comp_ptrs[k] = &T.comps[k];
        T.comps[k].numResolutions = numres;
        for (uint32_t r = 0; r < numres; ++r) {
            T.res_ptrs[k][r] = &T.res[k][r];
            grk_plugin_resolution &R = T.res[k][r];
            R.level = numres - 1 - r;
            R.numBands = r == 0 ? 1 : 3;
            T.band_ptrs.emplace_back(R.numBands);
            for (uint32_t bi = 0; bi < R.numBands; ++bi) {
                T.bands.emplace_back(new grk_plugin_band());
                grk_plugin_band *B = T.bands.back().get();
                B->orient = r == 0 ? 0 : bi + 1;
                B->numPrecincts = nprec[k][r][bi];
                B->stepsize = 0.0f;  // the band's step size, from its blocks below
                T.band_ptrs.back()[bi] = B;
                T.prec_ptrs.emplace_back(B->numPrecincts);
                for (uint32_t q = 0; q < B->numPrecincts; ++q) {
                    T.precs.emplace_back(new grk_plugin_precinct());
                    grk_plugin_precinct *P = T.precs.back().get();
                    P->numBlocks = q < nblk[k][r][bi].size() ? nblk[k][r][bi][q] : 0;
                    T.block_ptrs.emplace_back(P->numBlocks, nullptr);
                    P->blocks = T.block_ptrs.back().data();
                    T.prec_ptrs.back()[q] = P;
                }
                B->precincts = T.prec_ptrs.back().data();
                precp[k][r][bi] = T.prec_ptrs.back();
            }
            R.bands = T.band_ptrs.back().data();
        }
        T.comps[k].resolutions = T.res_ptrs[k].data();
    }
    for (uint32_t i = 0; i < n; ++i) {
        const grkgpu_block_info &s = b[i];
        grk_plugin_code_block &o = T.blocks[i];
        o.x0 = s.x0; o.y0 = s.y0; o.x1 = s.x1; o.y1 = s.y1;
        o.numPix = (size_t)(s.x1 - s.x0) * (s.y1 - s.y0);
        o.compressedData = (uint8_t *)s.data;
        o.compressedDataLength = s.len;
        o.numBitPlanes = s.numbps;
        if (s.numpasses > 67) return false;
        o.numPasses = s.numpasses;
        size_t prev = 0;
        for (uint32_t k = 0; k < s.numpasses; ++k) {
            o.passes[k].distortionDecrease = s.distortion[k];
            o.passes[k].rate = s.rate[k] ? s.rate[k] - 1 : 0;  // the host adds one back
            o.passes[k].length = s.rate[k] - prev;
            prev = s.rate[k];
        }
        const uint32_t bi = s.resno == 0 ? 0 : s.bandno - 1;
        precp[s.compno][s.resno][bi][s.precno]->blocks[s.cblkno] = &o;
        T.res[s.compno][s.resno].bands[bi]->stepsize = s.stepsize;
    }
    T.tile.decode_flags = 0;
    T.tile.numComponents = numcomps;
    T.tile.tileComponents = T.comp_ptrs.data();
    return true;
}

using ImageCreate = grkp_image *(*)(uint32_t, grkp_image_cmptparm *, int32_t);
using ImageDestroy = void (*)(grkp_image *);
using CompAlloc = bool (*)(grkp_image_comp *);

bool read_file(const char *path, std::vector<uint8_t> &out) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    std::unique_ptr<FILE, int (*)(FILE *)> guard(f, fclose);
    if (fseek(f, 0, SEEK_END)) return false;
    const long n = ftell(f);
    if (n < 0 || fseek(f, 0, SEEK_SET)) return false;
    out.resize((size_t)n);
    return fread(out.data(), 1, out.size(), f) == out.size();
}

}  // namespace

extern "C" {

PLUGIN_API minpf_exit_func minpf_post_load_plugin(const char *, const minpf_platform_services *services) {
    if (!services || !services->registerObject) return nullptr;
    minpf_register_params rp;
    rp.version.major = 1;
    rp.version.minor = 0;
    rp.createFunc = create_object;
    rp.destroyFunc = destroy_object;
    if (services->registerObject(GRKGPU_PLUGIN_ID, &rp) < 0) return nullptr;
    return exit_plugin;
}

// grk_plugin_init (grok.cpp:877-890): false keeps the host on its CPU path.
PLUGIN_API bool plugin_init(grk_plugin_init_info info) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_verbose = info.verbose;
    const char *ds = getenv("GRKGPU_PLUGIN_DEBUG_STATE");
    g_debug_state = ds && *ds ? (uint32_t)strtoul(ds, nullptr, 0) & GRK_PLUGIN_STATE_DEBUG : GRK_PLUGIN_STATE_NO_DEBUG;
    g_device = info.deviceId;
    if (g_ctx) return true;
    return grkgpu_create(info.deviceId < 0 ? 0 : info.deviceId, &g_ctx) == GRKGPU_OK;
}

PLUGIN_API uint32_t plugin_get_debug_state(void) { return g_debug_state; }

}  // extern "C"

namespace {

// The coding options the plugin route cannot take (the host then encodes on
// its CPU path), or nullptr.
const char *encode_decline(const grkp_cparameters *params) {
    // A single layer without rate control is formed by the host's
    // make_single_lossless_layer BEFORE the loop that copies the plugin's
    // passes in (TileProcessor.cpp:521 vs :537, :374 vs :404), so the host
    // would write an empty layer: decline, the host encodes on its CPU path.
    if (params->tcp_numlayers <= 1 && !layer_rc(params, 0))
        return "single lossless layer: the host forms it before taking the plugin's passes; declined";
    // Fixed quality (-q) targets tile->distotile, which only the host's own
    // T1 accumulates (T1Encoder.cpp:51); with a plugin tile it stays 0 and
    // the PSNR search degenerates (TileProcessor.cpp:611-635): decline.
    if (params->cp_fixed_quality) return "fixed-quality layers need the host's own T1 distortion total; declined";
    grkgpu_cparams p;
    if (!map_params(params, 3, &p)) return "coding options outside the plugin's path";
    return nullptr;
}

// One image file through the GPU (DC shift .. T1 + distortion), then the
// host's callback with the plugin tile (grok.cpp:905-918).  outname /
// relative: what the callback receives as the output file (batch: the input's
// bare file name, relative to the output directory, grk_compress.cpp:1783-1797).
int32_t encode_file(grkgpu_ctx *ctx, grkp_cparameters *params, const char *path, const char *outname, bool relative,
                    PLUGIN_ENCODE_USER_CALLBACK cb) {
    auto create = (ImageCreate)dlsym(RTLD_DEFAULT, "grk_image_create");
    auto destroy = (ImageDestroy)dlsym(RTLD_DEFAULT, "grk_image_destroy");
    if (!create || !destroy) {
        log("host grk_image_create not found");
        return -1;
    }
    Pnm pnm;
    if (!read_pnm(path, pnm)) {
        log("input is not a binary PGM / PPM");
        return -1;
    }
    grkgpu_image_desc d{};
    d.x0 = params->image_offset_x0;
    d.y0 = params->image_offset_y0;
    d.x1 = d.x0 + pnm.w;
    d.y1 = d.y0 + pnm.h;
    d.numcomps = pnm.c;
    for (uint32_t k = 0; k < pnm.c; ++k) d.prec[k] = pnm.prec;
    grkgpu_cparams p;
    if (!map_params(params, pnm.c, &p)) {
        log("coding options outside the plugin's path");
        return -1;
    }
    std::vector<const int32_t *> planes(pnm.c);
    const size_t area = (size_t)pnm.w * pnm.h;
    for (uint32_t k = 0; k < pnm.c; ++k) planes[k] = pnm.planes.data() + k * area;
    const grkgpu_block_info *blocks = nullptr;
    uint32_t nblocks = 0;
    if (grkgpu_encode_blocks(ctx, &d, &p, planes.data(), 0, needs_distortion(params) ? 1 : 0, &blocks, &nblocks)) {
        log(grkgpu_last_error());
        return -1;
    }
    // resolutions after the profile rules (cinema may clamp them)
    uint32_t numres = params->numresolution;
    for (uint32_t i = 0; i < nblocks; ++i) numres = std::max(numres, blocks[i].resno + 1);
    TileTree T;
    if (!build_tree(blocks, nblocks, pnm.c, numres, T)) {
        log("block layout not representable as a plugin tile");
        return -1;
    }
    // the host's image (its allocator owns the component buffers, which
    // grk_start_compress moves into the codec, j2k.cpp:2141-2151)
    std::vector<grkp_image_cmptparm> cm(pnm.c);
    for (uint32_t k = 0; k < pnm.c; ++k) cm[k] = {1, 1, pnm.w, pnm.h, 0, 0, pnm.prec, 0};
    grkp_image *img = create(pnm.c, cm.data(), pnm.c >= 3 ? 2 /* sRGB */ : 3 /* gray */);
    if (!img) return -1;
    img->x0 = d.x0; img->y0 = d.y0; img->x1 = d.x1; img->y1 = d.y1;
    for (uint32_t k = 0; k < pnm.c; ++k) {
        if (!img->comps[k].data) continue;
        if (g_debug_state & GRK_PLUGIN_STATE_DEBUG) {
            // debug: the image data is the plugin's DWT output, so the host's
            // own T1 starts from the same coefficients (TileProcessor.cpp:
            // 988-1012 skips its DC shift, MCT and DWT in this state)
            if (grkgpu_encode_blocks_coefficients(ctx, 0, k, img->comps[k].data, pnm.w)) {
                log(grkgpu_last_error());
                destroy(img);
                return -1;
            }
        } else {
            memcpy(img->comps[k].data, planes[k], area * 4);
        }
    }
    plugin_encode_user_callback_info info{};
    info.input_file_name = path;
    info.outputFileNameIsRelative = relative;
    info.output_file_name = outname;
    info.encoder_parameters = params;
    info.image = img;
    info.tile = &T.tile;
    cb(&info);
    destroy(img);
    return info.error_code ? -1 : 0;
}

// ---- batch route (grk_compress / grk_decompress with -ImgDir / -OutDir,
// grk_compress.cpp:2224-2243, grk_decompress.cpp:1237-1262) ----
// The plugin walks the input directory itself: frames in flight on worker
// threads, each with its own GPU context -- frames_per_device() per device,
// over every device for deviceId -1 (grok.h:1816-1821) -- so one frame's host
// work (rate control, Tier-2, file output in the host's callback) overlaps
// the others' GPU work.  The host polls plugin_is_batch_complete and ends the
// batch with plugin_stop_batch_encode / _decode.
// Frames in flight per device: GRKGPU_PLUGIN_FRAMES (1 .. 64; the plugin ABI
// has no parameter for it), default 8 -- measured on this route itself
// (scripts/plugin_batch_sweep.py, 24 DCI 4K cinema frames through
// grk_compress's directory mode, two rounds: 4 -> 72 / 70, 8 -> 67 / 82, 16 ->
// 58 / 61 Mpixels/s; profiles/r05/plugin_batch_sweep.txt): the host's own
// per-frame work (PPM read, its rate control and Tier-2, the file write)
// bounds the route, and more frames in flight only contend for its cores.
// (The library's own frame batch runs best at 16: profiles/r03_concurrency_
// sweep.txt, profiles/r04z/c5_concurrency_sweep.txt.)
static int frames_per_device() {
    const char *e = getenv("GRKGPU_PLUGIN_FRAMES");
    const int v = e ? atoi(e) : 8;
    return v < 1 ? 1 : v > 64 ? 64 : v;
}

struct Batch {
    bool decode = false;
    std::vector<std::string> files;  // bare file names in the input directory
    std::string in_dir, out_dir;
    grkp_cparameters eparams{};
    grkp_decompress_parameters dparams{};
    PLUGIN_ENCODE_USER_CALLBACK ecb = nullptr;
    PLUGIN_DECODE_USER_CALLBACK dcb = nullptr;
    std::atomic<size_t> next{0};
    std::atomic<bool> stop{false};
    std::atomic<int> running{0};
    std::vector<std::thread> workers;
    std::vector<grkgpu_ctx *> ctxs;
};
std::mutex g_batch_mu;
std::unique_ptr<Batch> g_batch;

bool has_ext(const std::string &f, std::initializer_list<const char *> exts) {
    const size_t dot = f.rfind('.');
    if (dot == std::string::npos) return false;
    std::string e = f.substr(dot + 1);
    for (auto &ch : e) ch = (char)tolower(ch);
    for (const char *x : exts)
        if (e == x) return true;
    return false;
}

std::vector<std::string> list_dir(const char *dir, std::initializer_list<const char *> exts) {
    std::vector<std::string> out;
    DIR *d = opendir(dir);
    if (!d) return out;
    while (dirent *e = readdir(d)) {
        const std::string n = e->d_name;
        if (n != "." && n != ".." && has_ext(n, exts)) out.push_back(n);
    }
    closedir(d);
    std::sort(out.begin(), out.end());
    return out;
}

std::string join_path(const std::string &dir, const std::string &name) {
    return dir.empty() || dir.back() == '/' ? dir + name : dir + "/" + name;
}

int32_t decode_file(grkgpu_ctx *ctx, grkp_decompress_parameters *params, const char *infile, const char *outfile,
                    PLUGIN_DECODE_USER_CALLBACK cb);

// the output file of a batch decode: <output dir>/<input stem>.<extension of
// the requested format> (the host's post_decode writes parameters->outfile,
// or this name when that is empty, grk_decompress.cpp:1577-1579)
std::string decode_out_name(const Batch &b, const std::string &in) {
    static const char *ext[] = {"", "j2k", "jp2", "ppm", "pgx", "bmp", "tif", "raw", "tga", "png", "rawl", "jpg"};
    const uint32_t f = b.dparams.cod_format < 12 ? b.dparams.cod_format : 0;
    const std::string stem = in.substr(0, in.find('.'));
    return join_path(b.out_dir, stem + "." + (f ? ext[f] : "raw"));
}

void batch_worker(Batch *b, grkgpu_ctx *ctx) {
    size_t k;
    while (!b->stop.load() && (k = b->next.fetch_add(1)) < b->files.size()) {
        const std::string in = join_path(b->in_dir, b->files[k]);
        if (!b->decode) {
            grkp_cparameters p = b->eparams;  // the host may adjust them per image (tcp_mct, ...)
            snprintf(p.infile, sizeof(p.infile), "%s", in.c_str());
            if (encode_file(ctx, &p, in.c_str(), b->files[k].c_str(), true, b->ecb)) log("batch: a frame failed");
        } else {
            grkp_decompress_parameters p = b->dparams;
            p.infile[0] = p.outfile[0] = 0;  // per file: the callback's names
            p.core.infile[0] = p.core.outfile[0] = 0;
            const std::string out = decode_out_name(*b, b->files[k]);
            if (decode_file(ctx, &p, in.c_str(), out.c_str(), b->dcb)) log("batch: a codestream failed");
        }
    }
    b->running.fetch_sub(1);
}

// start the workers of a prepared batch; false if no GPU context could be made
bool batch_start(Batch *b) {
    std::vector<int> devs;
    if (g_device < 0)
        for (int d = 0; d < grkgpu_device_count(); ++d) devs.push_back(d);
    else
        devs.push_back(g_device);
    const int fpd = frames_per_device();
    for (int f = 0; f < fpd; ++f)
        for (int d : devs) {
            grkgpu_ctx *c = nullptr;
            if (grkgpu_create(d, &c) != GRKGPU_OK) continue;
            b->ctxs.push_back(c);
        }
    if (b->ctxs.empty()) return false;
    b->running = (int)b->ctxs.size();
    for (auto *c : b->ctxs) b->workers.emplace_back(batch_worker, b, c);
    return true;
}

void batch_end() {
    std::lock_guard<std::mutex> lk(g_batch_mu);
    if (!g_batch) return;
    g_batch->stop = true;
    for (auto &t : g_batch->workers) t.join();
    for (auto *c : g_batch->ctxs) grkgpu_destroy(c);
    g_batch.reset();
}

// One codestream through the GPU decoder, then the host's callback protocol.
// The decode runs first, on the GPU, so that anything the plugin cannot take
// (JP2 boxes, a window at a reduced resolution, a corrupt or unsupported
// stream) is declined with -1 before the host has been called: the host then
// decodes on its CPU path.  Then:
//   HEADER     the host reads the main header into its own grk_image;
//   (plugin)   component geometry of the decoded region + the samples, in
//              buffers of the host's allocator
//              (grk_image_single_component_data_alloc);
//   POST_T1    the host writes the output file (post_decode);
//   CLEAN      the host releases stream, codec and image.
int32_t decode_file(grkgpu_ctx *ctx, grkp_decompress_parameters *params, const char *infile, const char *outfile,
                    PLUGIN_DECODE_USER_CALLBACK cb) {
    auto comp_alloc = (CompAlloc)dlsym(RTLD_DEFAULT, "grk_image_single_component_data_alloc");
    if (!comp_alloc) {
        log("host grk_image_single_component_data_alloc not found");
        return -1;
    }
    std::vector<uint8_t> cs;
    if (!read_file(infile, cs) || cs.size() < 4 || cs[0] != 0xFF || cs[1] != 0x4F || cs[2] != 0xFF || cs[3] != 0x51) {
        log("input is not a raw J2K codestream; declined");
        return -1;
    }
    grkgpu_image_desc d{};
    if (grkgpu_read_header(cs.data(), cs.size(), &d)) {
        log(grkgpu_last_error());
        return -1;
    }
    for (uint32_t k = 0; k < d.numcomps; ++k)
        if (d.dx[k] != 1 || d.dy[k] != 1) {
            log("subsampled components; declined");
            return -1;
        }
    const uint32_t r = params->core.cp_reduce;
    grkgpu_dparams dp{r, params->core.cp_layer, params->DA_x0, params->DA_y0, params->DA_x1, params->DA_y1};
    const bool win = dp.DA_x0 || dp.DA_y0 || dp.DA_x1 || dp.DA_y1;
    // decoded region: the image or the window clipped to it (reference grid),
    // at the decoded resolution ceil(x / 2^r) (update_image_dimensions, image.cpp:207-246)
    auto cdiv = [r](uint32_t v) { return (uint32_t)(((uint64_t)v + (1ull << r) - 1) >> r); };
    uint32_t fx0 = d.x0, fy0 = d.y0, fx1 = d.x1, fy1 = d.y1;
    if (win) {
        fx0 = std::max(d.x0, dp.DA_x0); fy0 = std::max(d.y0, dp.DA_y0);
        fx1 = std::min(d.x1, dp.DA_x1); fy1 = std::min(d.y1, dp.DA_y1);
        if (fx1 <= fx0 || fy1 <= fy0) return -1;
    }
    const uint32_t x0 = cdiv(fx0), y0 = cdiv(fy0), x1 = cdiv(fx1), y1 = cdiv(fy1);
    if (x1 <= x0 || y1 <= y0) return -1;
    // the core's planes: a window's extent, or the image's ceil(size / 2^r)
    // (grk_image_comp_header_update; see grkgpu_image_desc)
    const uint32_t w = win ? x1 - x0 : cdiv(fx1 - fx0), h = win ? y1 - y0 : cdiv(fy1 - fy0), nc = d.numcomps;
    std::vector<int32_t> samples((size_t)w * h * nc);
    std::vector<int32_t *> planes(nc);
    for (uint32_t k = 0; k < nc; ++k) planes[k] = samples.data() + (size_t)k * w * h;
    if (grkgpu_decompress_ex(ctx, cs.data(), cs.size(), &dp, nullptr, planes.data(), 0)) {
        log(grkgpu_last_error());
        return -1;
    }
    PluginDecodeCallbackInfo info(infile, outfile ? outfile : "", params, GRKP_J2K_FMT, GRK_DECODE_HEADER);
    info.deviceId = params->deviceId < 0 ? 0 : (size_t)params->deviceId;
    int32_t rc = cb(&info);
    if (rc == 0 && info.image && info.image->numcomps == nc) {
        grkp_image *img = info.image;
        if (win) {  // grk_set_decode_area's image bounds: the window (TileProcessor.cpp:109-240)
            img->x0 = fx0; img->y0 = fy0; img->x1 = fx1; img->y1 = fy1;
        }
        for (uint32_t k = 0; k < nc && rc == 0; ++k) {
            grkp_image_comp &cm = img->comps[k];
            cm.x0 = win ? fx0 : x0; cm.y0 = win ? fy0 : y0; cm.w = w; cm.h = h;
            if (!comp_alloc(&cm)) rc = -1;
            else memcpy(cm.data, planes[k], (size_t)w * h * 4);
        }
        if (rc == 0) {
            info.decode_flags = GRK_DECODE_POST_T1;
            rc = cb(&info);
        }
    } else if (rc == 0) {
        rc = -1;
    }
    info.decode_flags = GRK_PLUGIN_DECODE_CLEAN;
    cb(&info);
    return rc;
}

}  // namespace

extern "C" {

// grk_plugin_encode (grok.cpp:917-935).  -1 = not handled (the host then runs
// its CPU path, grk_compress.cpp:2206-2222).
PLUGIN_API int32_t plugin_encode(grkp_cparameters *params, PLUGIN_ENCODE_USER_CALLBACK cb) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ctx || !params || !cb) return -1;
    if (const char *why = encode_decline(params)) {
        log(why);
        return -1;
    }
    return encode_file(g_ctx, params, params->infile, params->outfile, false, cb);
}

// grk_plugin_batch_encode (grok.cpp:938-955, grk_compress.cpp:2224-2243):
// every PGM / PPM of input_dir, frames in flight over the plugin's devices;
// the host's callback receives each input's bare file name as a relative
// output name and writes output_dir/<name>.<format>.  0 = the batch started
// (the host then polls plugin_is_batch_complete); -1 = not taken (options the
// plugin declines, no input, a batch already running).
PLUGIN_API int32_t plugin_batch_encode(const char *input_dir, const char *output_dir, grkp_cparameters *params,
                                       PLUGIN_ENCODE_USER_CALLBACK cb) {
    if (!input_dir || !output_dir || !params || !cb) return -1;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_ctx) return -1;
    }
    if (const char *why = encode_decline(params)) {
        log(why);
        return -1;
    }
    std::lock_guard<std::mutex> lk(g_batch_mu);
    if (g_batch) return -1;
    auto b = std::make_unique<Batch>();
    b->files = list_dir(input_dir, {"pgm", "ppm", "pnm"});
    if (b->files.empty()) return -1;
    b->in_dir = input_dir;
    b->out_dir = output_dir;
    b->eparams = *params;
    b->ecb = cb;
    if (!batch_start(b.get())) return -1;
    g_batch = std::move(b);
    return 0;
}

PLUGIN_API bool plugin_is_batch_complete(void) {
    std::lock_guard<std::mutex> lk(g_batch_mu);
    return !g_batch || g_batch->running.load() == 0;
}

// the host's stop (after completion, or on a signal): pending frames are
// dropped, frames in flight finish, the workers and their contexts go
PLUGIN_API void plugin_stop_batch_encode(void) { batch_end(); }

// grk_plugin_decode (grok.cpp:1031-1051), driven by grk_decompress's
// plugin_main (grk_decompress.cpp:1186-1319) with its decode_callback
// (:1336-1367); see decode_file.
PLUGIN_API int32_t plugin_decode(grkp_decompress_parameters *params, PLUGIN_DECODE_USER_CALLBACK cb) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ctx || !params || !cb) return -1;
    const char *infile = params->infile[0] ? params->infile : params->core.infile;
    const char *outfile = params->outfile[0] ? params->outfile : params->core.outfile;
    if (params->nb_tile_to_decode) {
        log("single-tile decode (grk_get_decoded_tile) not taken; declined");
        return -1;
    }
    return decode_file(g_ctx, params, infile, outfile, cb);
}

// grk_plugin_init_batch_decode (grok.cpp:1052-1072): remember the batch.  The
// reference host starts it (grk_plugin_batch_decode) only when this returns
// non-zero (grk_decompress.cpp:1242-1245), so success is 1 here.
PLUGIN_API int32_t plugin_init_batch_decode(const char *input_dir, const char *output_dir,
                                            grkp_decompress_parameters *params, void *cb) {
    if (!input_dir || !output_dir || !params || !cb) return 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_ctx) return 0;
    }
    std::lock_guard<std::mutex> lk(g_batch_mu);
    if (g_batch) return 0;
    auto b = std::make_unique<Batch>();
    b->decode = true;
    b->files = list_dir(input_dir, {"j2k", "j2c"});
    if (b->files.empty()) return 0;
    b->in_dir = input_dir;
    b->out_dir = output_dir;
    b->dparams = *params;
    b->dcb = (PLUGIN_DECODE_USER_CALLBACK)cb;
    g_batch = std::move(b);
    return 1;
}

// grk_plugin_batch_decode (grok.cpp:1074-1087): start the batch set up by
// plugin_init_batch_decode; 0 = started.
PLUGIN_API int32_t plugin_batch_decode(void) {
    std::lock_guard<std::mutex> lk(g_batch_mu);
    if (!g_batch || !g_batch->decode || !g_batch->workers.empty()) return -1;
    return batch_start(g_batch.get()) ? 0 : -1;
}

PLUGIN_API void plugin_stop_batch_decode(void) { batch_end(); }
PLUGIN_API void plugin_debug_mqc_next_cxd(void *, uint32_t) {}
PLUGIN_API void plugin_debug_next_cxd(void *, uint32_t) {}
PLUGIN_API void plugin_debug_mqc_next_plane(void *) {}

}  // extern "C"
