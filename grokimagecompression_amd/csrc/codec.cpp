// codec.cpp -- tile pipeline (the reference's TileProcessor, "tcd") turned into
// a HIP dispatch layer, plus the extern "C" API of include/grk_mi355x.h.
//
// Encode (TileProcessor::encode_tile, TileProcessor.cpp:951-1025):
//   H2D planes (if host) -> per tile: DC shift + MCT kernel -> per component
//   DWT levels -> ONE T1 launch over every code-block of every tile ->
//   D2H per-block results -> gather kernel packs block bytes -> D2H ->
//   host Tier-2 + headers.
// Decode (TileProcessor::decode_tile, TileProcessor.cpp:1069-1179):
//   host header + Tier-2 parse -> H2D codestream -> ONE T1 decode launch ->
//   per tile/component inverse DWT levels -> inverse MCT + DC shift.
#include <float.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/grk_mi355x.h"
#include "codestream.h"
#include "grk_device.h"
#include "host_pool.h"
#include "t2.h"

using namespace grkgpu;

static thread_local std::string g_err;
static int set_err(int code, const std::string &msg) { g_err = msg; return code; }
namespace grkgpu {
int set_error(int code, const std::string &msg) { return set_err(code, msg); }  // multi.cpp
}

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return set_err(GRKGPU_EHIP, std::string(#expr ": ") + hipGetErrorString(e_));    \
    } while (0)

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr; cap = 0;
        size_t nb = bytes + bytes / 8 + 256;
        hipError_t e = hipMalloc(&p, nb);
        if (e == hipSuccess) cap = nb;
        return e;
    }
    template <typename T> T *as() const { return (T *)p; }
    ~DevBuf() { if (p) hipFree(p); }
};

struct HostBuf {  // pinned host staging
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) hipHostFree(p);
        p = nullptr; cap = 0;
        size_t nb = bytes + bytes / 8 + 256;
        hipError_t e = hipHostMalloc(&p, nb, hipHostMallocDefault);
        if (e == hipSuccess) cap = nb;
        return e;
    }
    template <typename T> T *as() const { return (T *)p; }
    ~HostBuf() { if (p) hipHostFree(p); }
};

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct grkgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    DevBuf img, work, coef, ll, scratch, mqout, blocks, results, gather, packed, cs, sym, symoff, dwtjobs, ubuf, segs;
    HostBuf h_results, h_packed, h_gather, h_blocks, h_out, h_symoff, h_dwtjobs, h_segs;
    DevBuf dwtjobs53;  // decode: the 5/3 tile-components' job table when 9/7 ones share the call
    DevBuf t1order;    // encode: the MQ coder's work order (keys, permutation, bucket counters)
    // encode with rate control: the pass records formed on the device
    // (launch_pass_records): per block its distortion factor and record slots
    // (in), its summary and records (out)
    DevBuf pinfo, precs;
    HostBuf h_pinfo, h_psum, h_precs;
    // encode: the pass records of the last call, kept so that a frame of the
    // same size does not zero ~20 MB again before overwriting every record
    std::vector<EncPass> enc_passes;
    HostBuf h_dwtjobs53;
    hipEvent_t ev[8] = {};
    grkgpu_stats stats = {};
    // grkgpu_encode_blocks output (valid until the next call on the context)
    HostBuf h_slab;
    std::vector<grkgpu_block_info> bexp;
    struct CoefRec { uint32_t tileno, compno, w, h; uint64_t off; };  // coefficient arena of each tile-component
    std::vector<CoefRec> bexp_coef;
    std::vector<uint32_t> bexp_rate;
    std::vector<double> bexp_dist;
    // per-launch DWT timing (grkgpu_set_launch_timing): a start / end event per
    // launch of the last forward DWT, read after the call's final sync
    bool launch_timing = false;
    std::vector<hipEvent_t> lev;
    std::vector<grkgpu_launch_time> ltimes;
    std::vector<std::pair<uint32_t, uint32_t>> lidx;  // per logged launch: its start / end event in lev
    // guards h_out and out_spare against grkgpu_give_output from another thread
    std::mutex out_mu;
    // output buffers given back while h_out held a newer one (a caller keeping
    // several views alive): the next compress whose h_out was taken reuses one
    // instead of pinning a fresh buffer; at most OUT_SPARE, the largest kept
    std::vector<std::pair<void *, size_t>> out_spare;
};
static constexpr size_t OUT_SPARE = 4;

// Device check, cached per device index (hipGetDeviceProperties is slow and
// the stage entry points run it per call).  device < 0: the calling thread's
// current HIP device (the stage entry points work on the caller's device).
static int check_device(int device) {
    static std::mutex mu;
    static int ok[64] = {};  // 0 unknown, 1 gfx950, -1 unusable
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return set_err(GRKGPU_ENODEV, "no HIP device available (MI355X / gfx950 required; no CPU fallback)");
    if (device < 0 && hipGetDevice(&device) != hipSuccess) return set_err(GRKGPU_ENODEV, "hipGetDevice failed");
    if (device < 0 || device >= n) return set_err(GRKGPU_ENODEV, "device index out of range");
    std::lock_guard<std::mutex> lk(mu);
    if (device < 64 && ok[device] == 1) return GRKGPU_OK;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return set_err(GRKGPU_ENODEV, "hipGetDeviceProperties failed");
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) {
        if (device < 64) ok[device] = -1;
        return set_err(GRKGPU_ENODEV, std::string("unsupported device arch ") + prop.gcnArchName + " (gfx950 required)");
    }
    if (device < 64) ok[device] = 1;
    return GRKGPU_OK;
}

extern "C" {

const char *grkgpu_version(void) { return "grk-mi355x 0.1.0 (Grok 5.1.0 codestream-compatible)"; }
const char *grkgpu_last_error(void) { return g_err.c_str(); }

int grkgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int grkgpu_set_mct(grkgpu_cparams *p, const float *matrix, const int32_t *dc_shift, uint32_t n) {
    if (!p || !matrix || !dc_shift || !n || n > GRKGPU_MAX_COMPS) return set_err(GRKGPU_EINVAL, "custom MCT: 1..16 components");
    p->rsiz = (p->rsiz & RSIZ_PART2) ? (p->rsiz | RSIZ_EXT_MCT) : (RSIZ_PART2 | RSIZ_EXT_MCT);  // grok.cpp:612-617
    p->irreversible = 1;
    p->tcp_mct = 2;
    p->mct_ncomp = n;
    memcpy(p->mct_matrix, matrix, sizeof(float) * n * n);
    memcpy(p->mct_dc_shift, dc_shift, sizeof(int32_t) * n);
    return GRKGPU_OK;
}

// grk_set_default_encoder_parameters (grok.cpp) + grk_compress's defaults
void grkgpu_default_cparams(grkgpu_cparams *p) {
    memset(p, 0, sizeof(*p));
    p->numresolution = 6;
    p->cblockw_init = 64;
    p->cblockh_init = 64;
    p->irreversible = 0;
    p->tcp_mct = -1;
    p->prog_order = GRKGPU_LRCP;
    p->tcp_numlayers = 0;  // -> one lossless layer (disto_alloc set then, grk_compress.cpp:1579-1583)
}

int grkgpu_create(int device, grkgpu_ctx **out) {
    int rc = check_device(device);
    if (rc) return rc;
    HIPCHK(hipSetDevice(device));
    auto *c = new grkgpu_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return set_err(GRKGPU_EHIP, "hipStreamCreate failed");
    }
    c->own_stream = true;
    for (auto &e : c->ev) hipEventCreate(&e);
    *out = c;
    return GRKGPU_OK;
}

void grkgpu_destroy(grkgpu_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    for (auto &e : c->ev) if (e) hipEventDestroy(e);
    for (auto &e : c->lev) if (e) hipEventDestroy(e);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    for (auto &b : c->out_spare) hipHostFree(b.first);
    delete c;
}

int grkgpu_set_stream(grkgpu_ctx *c, void *stream) {
    if (!c) return set_err(GRKGPU_EINVAL, "null ctx");
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    c->stream = (hipStream_t)stream;
    c->own_stream = false;
    return GRKGPU_OK;
}

}  // extern "C"

namespace grkgpu {
static DwtOptions g_dwt_opts;
const DwtOptions &dwt_options() { return g_dwt_opts; }

// Codec calls in progress in this process.  A call that has the GPU to itself
// (a lone frame: grk_decompress of one image) cannot fill the chip with its
// T1 lanes packed 64 blocks to a wavefront (24,669 blocks of an 8K frame =
// 386 wavefronts for 1,024 SIMDs), so it spreads them (lone_bpw) and orders
// them by work; concurrent calls (frame batches) keep full wavefronts.
static std::atomic<int> g_active_calls{0};
struct ActiveCall {
    ActiveCall() { g_active_calls.fetch_add(1); }
    ~ActiveCall() { g_active_calls.fetch_sub(1); }
};
static bool lone_call() { return g_active_calls.load() <= 1; }
}  // namespace grkgpu

extern "C" {

void grkgpu_get_dwt_options(grkgpu_dwt_options *out) {
    if (!out) return;
    out->fuse_level0 = g_dwt_opts.fuse_level0;
    out->f01_rows = g_dwt_opts.f01_rows;
    out->f01_min_samples = g_dwt_opts.f01_min_samples;
    out->f01_small_min_samples = g_dwt_opts.f01_small_min_samples;
    out->inv01 = g_dwt_opts.inv01;
    out->pair_group = g_dwt_opts.pair_group;
    out->inv01_min_samples = g_dwt_opts.inv01_min_samples;
    out->f64_lift = g_dwt_opts.f64_lift;
    out->t1_dec_sort = g_dwt_opts.t1_dec_sort;
    out->t1_dec_bpw = g_dwt_opts.t1_dec_bpw;
    out->mid_th = g_dwt_opts.mid_th;
    out->t1_enc_bpw = g_dwt_opts.t1_enc_bpw;
    out->t1_enc_sort = g_dwt_opts.t1_enc_sort;
    out->pair_kernel = g_dwt_opts.pair_kernel;
    out->pair_rows = g_dwt_opts.pair_rows;
    out->pair_waves = g_dwt_opts.pair_waves;
    out->pair_min_samples = g_dwt_opts.pair_min_samples;
}

int grkgpu_set_dwt_options(const grkgpu_dwt_options *o) {
    if (!o) {
        g_dwt_opts = DwtOptions();
        return GRKGPU_OK;
    }
    if (o->fuse_level0 < -1 || o->fuse_level0 > 1) return set_err(GRKGPU_EINVAL, "fuse_level0 must be -1, 0 or 1");
    if (o->f01_rows != 0 && o->f01_rows != 2 && o->f01_rows != 4 && o->f01_rows != 6)
        return set_err(GRKGPU_EINVAL, "f01_rows must be 0, 2, 4 or 6");
    if (o->inv01 != 0 && o->inv01 != 2 && o->inv01 != 4) return set_err(GRKGPU_EINVAL, "inv01 must be 0, 2 or 4");
    if (o->pair_group < 0 || o->pair_group > 4096) return set_err(GRKGPU_EINVAL, "pair_group must be 0 .. 4096");
    if (o->f64_lift != 0 && o->f64_lift != 1) return set_err(GRKGPU_EINVAL, "f64_lift must be 0 or 1");
    if (o->t1_dec_sort < -1 || o->t1_dec_sort > 1) return set_err(GRKGPU_EINVAL, "t1_dec_sort must be -1, 0 or 1");
    if (o->t1_dec_bpw < 0 || o->t1_dec_bpw > 64 || (o->t1_dec_bpw & (o->t1_dec_bpw - 1)))
        return set_err(GRKGPU_EINVAL, "t1_dec_bpw must be 0 or a power of two <= 64");
    if (o->mid_th != 0 && o->mid_th != 8 && o->mid_th != 16 && o->mid_th != 24)
        return set_err(GRKGPU_EINVAL, "mid_th must be 0, 8, 16 or 24");
    if (o->t1_enc_bpw < 0 || o->t1_enc_bpw > 64 || (o->t1_enc_bpw & (o->t1_enc_bpw - 1)))
        return set_err(GRKGPU_EINVAL, "t1_enc_bpw must be 0 or a power of two <= 64");
    if (o->t1_enc_sort != 0 && o->t1_enc_sort != 1) return set_err(GRKGPU_EINVAL, "t1_enc_sort must be 0 or 1");
    if (o->pair_kernel < 0 || o->pair_kernel > 2) return set_err(GRKGPU_EINVAL, "pair_kernel must be 0, 1 or 2");
    if (o->pair_rows < 0 || o->pair_rows > 65536 || (o->pair_rows & 1))
        return set_err(GRKGPU_EINVAL, "pair_rows must be 0 or an even count <= 65536");
    if (o->pair_waves != 0 && o->pair_waves != 3 && o->pair_waves != 4)
        return set_err(GRKGPU_EINVAL, "pair_waves must be 0, 3 or 4");
    g_dwt_opts.pair_kernel = o->pair_kernel;
    g_dwt_opts.pair_rows = o->pair_rows;
    g_dwt_opts.pair_waves = o->pair_waves;
    g_dwt_opts.pair_min_samples = o->pair_min_samples;
    g_dwt_opts.t1_enc_sort = o->t1_enc_sort;
    g_dwt_opts.t1_enc_bpw = o->t1_enc_bpw;
    g_dwt_opts.f64_lift = o->f64_lift;
    g_dwt_opts.t1_dec_sort = o->t1_dec_sort;
    g_dwt_opts.t1_dec_bpw = o->t1_dec_bpw;
    g_dwt_opts.mid_th = o->mid_th;
    g_dwt_opts.inv01 = o->inv01;
    g_dwt_opts.pair_group = o->pair_group;
    g_dwt_opts.inv01_min_samples = o->inv01_min_samples;
    g_dwt_opts.fuse_level0 = o->fuse_level0;
    g_dwt_opts.f01_rows = o->f01_rows;
    g_dwt_opts.f01_min_samples = o->f01_min_samples;
    g_dwt_opts.f01_small_min_samples = o->f01_small_min_samples;
    return GRKGPU_OK;
}

int grkgpu_take_output(grkgpu_ctx *c, void **buf, size_t *cap) {
    if (!c || !buf || !cap) return set_err(GRKGPU_EINVAL, "null arg");
    std::lock_guard<std::mutex> lk(c->out_mu);
    *buf = c->h_out.p;
    *cap = c->h_out.cap;
    c->h_out.p = nullptr;
    c->h_out.cap = 0;
    return GRKGPU_OK;
}

int grkgpu_give_output(grkgpu_ctx *c, void *buf, size_t cap) {
    if (!buf) return GRKGPU_OK;
    if (!c) {
        hipHostFree(buf);
        return GRKGPU_OK;
    }
    std::lock_guard<std::mutex> lk(c->out_mu);
    if (cap > c->h_out.cap) std::swap(buf, c->h_out.p), std::swap(cap, c->h_out.cap);
    if (!buf) return GRKGPU_OK;
    if (c->out_spare.size() < OUT_SPARE) {
        c->out_spare.push_back({buf, cap});
        return GRKGPU_OK;
    }
    auto small = std::min_element(c->out_spare.begin(), c->out_spare.end(),
                                  [](const auto &a, const auto &b) { return a.second < b.second; });
    if (cap > small->second) std::swap(buf, small->first), std::swap(cap, small->second);
    hipHostFree(buf);
    return GRKGPU_OK;
}

void grkgpu_free_output(void *buf) {
    if (buf) hipHostFree(buf);
}

int grkgpu_set_launch_timing(grkgpu_ctx *c, int on) {
    if (!c) return set_err(GRKGPU_EINVAL, "null ctx");
    c->launch_timing = on != 0;
    c->ltimes.clear();
    c->lidx.clear();
    return GRKGPU_OK;
}

int grkgpu_get_launch_times(grkgpu_ctx *c, grkgpu_launch_time *out, uint32_t max, uint32_t *n) {
    if (!c || !n || (max && !out)) return set_err(GRKGPU_EINVAL, "null arg");
    *n = (uint32_t)c->ltimes.size();
    for (uint32_t i = 0; i < max && i < c->ltimes.size(); ++i) out[i] = c->ltimes[i];
    return GRKGPU_OK;
}

int grkgpu_get_stats(grkgpu_ctx *c, grkgpu_stats *out) {
    if (!c || !out) return set_err(GRKGPU_EINVAL, "null arg");
    *out = c->stats;
    return GRKGPU_OK;
}

void grkgpu_free(void *p) { free(p); }

// Per-block scratch of the T1 stage entry points (per record; the records are
// the block count rounded up to 64): encode -- the encoder's interleaved rows
// for 32 planes, then 32 symbol-stream slots; decode -- the block state, then
// the unstuffed-stream region of a segment of up to GRKGPU_T1_MAX_SEG bytes.
static uint32_t t1_stage_dec_words() { return t1_unstuff_region_words(GRKGPU_T1_MAX_SEG); }
size_t grkgpu_t1_scratch_bytes(void) {
    return std::max<size_t>(t1e_scratch_bytes(64, 32) / 64 + 32 * (size_t)sym_slot_bytes(64, 64),
                            sizeof(T1Scratch) + (size_t)t1_stage_dec_words() * 4);
}
size_t grkgpu_t1_scratch_bytes_n(uint32_t nblocks) {
    return (((size_t)nblocks + 63) & ~(size_t)63) * grkgpu_t1_scratch_bytes();
}

}  // extern "C"

// ---------------------------------------------------------------------------
// shared helpers
// ---------------------------------------------------------------------------
static bool cinema_compliant(const grkgpu_image_desc *img, uint32_t rsiz) {
    // J2KProfile::is_cinema_compliant (j2kprofile.cpp:1083-1135)
    if (img->numcomps != 3) return false;
    for (uint32_t k = 0; k < 3; ++k)
        if (img->prec[k] != 12 || img->sgnd[k]) return false;
    const uint32_t w = img->x1 - img->x0, h = img->y1 - img->y0;
    if (rsiz == GRKGPU_PROFILE_CINEMA_2K) return w <= 2048 && h <= 1080;
    return w <= 4096 && h <= 2160;
}

// J2KProfile::set_cinema_parameters (j2kprofile.cpp:941-1081)
static void set_cinema_parameters(grkgpu_cparams *p, const grkgpu_image_desc *img) {
    p->tile_size_on = 0;
    p->cp_tdx = p->cp_tdy = 1;
    p->tp_flag = 'C';
    p->tp_on = 1;
    p->cp_tx0 = p->cp_ty0 = 0;
    p->cblockw_init = p->cblockh_init = 32;
    p->irreversible = 1;
    if (p->tcp_numlayers > 1) {
        p->tcp_rates[0] = p->tcp_rates[p->tcp_numlayers - 1];
        p->tcp_numlayers = 1;
    }
    if (p->rsiz == GRKGPU_PROFILE_CINEMA_2K) {
        if (p->numresolution > 6) p->numresolution = 6;
    } else {
        if (p->numresolution < 2) p->numresolution = 1;
        else if (p->numresolution > 7) p->numresolution = 7;
    }
    p->csty |= GRKGPU_CSTY_PRT;
    p->res_spec = p->numresolution - 1;
    for (uint32_t i = 0; i < p->res_spec; i++) p->prcw_init[i] = p->prch_init[i] = 256;
    p->prog_order = GRKGPU_CPRL;
    if (p->rsiz == GRKGPU_PROFILE_CINEMA_4K) {  // initialise_4K_poc (j2kprofile.cpp:922-939)
        const uint32_t nr = p->numresolution;
        p->POC[0] = {1, 0, 0, 1, nr - 1, 3, GRKGPU_CPRL};
        p->POC[1] = {1, nr - 1, 0, 1, nr, 3, GRKGPU_CPRL};
        p->numpocs = 2;
    } else {
        p->numpocs = 0;
    }
    p->cp_disto_alloc = 1;
    const uint64_t kCs = 1302083u, kComp = 1041666u;  // GRK_CINEMA_24_CS / _COMP (grok.h:316-318)
    if (p->max_cs_size == 0 || p->max_cs_size > kCs) p->max_cs_size = kCs;
    if (p->max_comp_size == 0 || p->max_comp_size > kComp) p->max_comp_size = kComp;
    const double w = img->x1 - img->x0, h = img->y1 - img->y0;
    p->tcp_rates[0] = ((double)img->numcomps * w * h * img->prec[0]) / ((double)p->max_cs_size * 8 * 1 * 1);
}

// j2k_setup_encoder (j2k.cpp:1609-2050) with the grk_compress post-parse
// defaults (grk_compress.cpp:1579-1583 one lossless layer, :1997-1998 MCT)
// and the cinema profiles, for the options grkgpu_cparams carries.  Layer
// rates stay compression ratios here; update_rates converts them to bytes.
static int setup_params(const grkgpu_image_desc *img, const grkgpu_cparams *pin, CodingParams &cp) {
    if (!img || !pin) return set_err(GRKGPU_EINVAL, "null image/params");
    grkgpu_cparams P = *pin;  // the profiles rewrite the parameters, as the reference does
    grkgpu_cparams *p = &P;
    if (img->numcomps < 1 || img->numcomps > 16) return set_err(GRKGPU_EINVAL, "numcomps must be 1..16");
    if (img->x1 <= img->x0 || img->y1 <= img->y0) return set_err(GRKGPU_EINVAL, "empty image");
    for (uint32_t k = 0; k < img->numcomps; ++k)
        if (img->prec[k] < 1 || img->prec[k] > 16) return set_err(GRKGPU_EUNSUPPORTED, "precision must be 1..16");
    if (p->tcp_numlayers > 100) return set_err(GRKGPU_EINVAL, "at most 100 quality layers");
    // code-block mode switches (COD SPcod style, j2k.cpp j2k_setup_encoder):
    // BYPASS, RESET, TERMALL, VSC, PTERM, SEGSYM; not HT (0x40)
    if (p->cblk_sty & ~0x3Fu) return set_err(GRKGPU_EUNSUPPORTED, "HT code-block style not supported");
    cp.cblksty = p->cblk_sty;
    if (p->roi_shift) {  // j2k_setup_encoder (j2k.cpp:1997-2001)
        if (p->roi_compno < 0 || (uint32_t)p->roi_compno >= img->numcomps)
            return set_err(GRKGPU_EINVAL, "ROI component out of range");
        if (p->roi_shift > 255) return set_err(GRKGPU_EINVAL, "ROI shift must fit a byte");
        cp.roishift[p->roi_compno] = (uint8_t)p->roi_shift;
    }
    if (p->tcp_numlayers == 0) {
        p->tcp_rates[0] = 0;
        p->tcp_numlayers = 1;
        p->cp_disto_alloc = 1;
    }
    if (p->cp_disto_alloc && p->cp_fixed_quality) return set_err(GRKGPU_EINVAL, "-r and -q cannot be used together");
    {  // max codestream size vs layer rates (j2k.cpp:1663-1689)
        // component 0's plane size, divided by its subsampling once more (sic)
        const uint32_t dx0 = img->dx[0] ? img->dx[0] : 1, dy0 = img->dy[0] ? img->dy[0] : 1;
        const Rect c0 = comp_rect({img->x0, img->y0, img->x1, img->y1}, dx0, dy0);
        const double image_bytes =
            ((double)img->numcomps * c0.w() * c0.h() * img->prec[0]) / (8.0 * dx0 * dy0);
        const uint32_t L = p->tcp_numlayers;
        if (p->max_cs_size == 0) {
            if (p->tcp_rates[L - 1] > 0) p->max_cs_size = (uint64_t)floor(image_bytes / p->tcp_rates[L - 1]);
        } else {
            const double min_rate = image_bytes / (double)p->max_cs_size;
            for (uint32_t i = 0; i < L; i++)
                if (p->tcp_rates[i] < min_rate) p->tcp_rates[i] = min_rate;
        }
    }
    if (p->rsiz == GRKGPU_PROFILE_CINEMA_2K || p->rsiz == GRKGPU_PROFILE_CINEMA_4K) {
        if (cinema_compliant(img, p->rsiz)) set_cinema_parameters(p, img);
        else p->rsiz = 0;  // "Non-profile-3/4 codestream will be generated"
    } else if (p->rsiz & RSIZ_PART2) {  // j2k.cpp:1720-1731: Part 2 with the MCT extension only
        if (p->rsiz != (RSIZ_PART2 | RSIZ_EXT_MCT)) p->rsiz = 0;
    } else if (p->rsiz != 0) {
        return set_err(GRKGPU_EUNSUPPORTED, "only the 2K / 4K digital cinema profiles and Part-2 MCT are supported");
    }
    if (p->numresolution < 1 || p->numresolution > 33) return set_err(GRKGPU_EINVAL, "numresolution must be 1..33");
    auto pow2 = [](uint32_t v) { return v >= 4 && v <= 64 && (v & (v - 1)) == 0; };
    if (!pow2(p->cblockw_init) || !pow2(p->cblockh_init))
        return set_err(GRKGPU_EINVAL, "code-block dimensions must be powers of two in [4, 64]");
    cp.numcomps = img->numcomps;
    cp.image = {img->x0, img->y0, img->x1, img->y1};
    for (uint32_t k = 0; k < img->numcomps; ++k) {
        cp.prec[k] = img->prec[k];
        cp.sgnd[k] = img->sgnd[k] ? 1 : 0;
        cp.shift[k] = cp.sgnd[k] ? 0 : (1 << (cp.prec[k] - 1));
        cp.dx[k] = img->dx[k] ? img->dx[k] : 1;
        cp.dy[k] = img->dy[k] ? img->dy[k] : 1;
        if (cp.dx[k] > 255 || cp.dy[k] > 255) return set_err(GRKGPU_EINVAL, "component subsampling must be 1..255");
    }
    cp.numres = p->numresolution;
    cp.cblkw = (uint32_t)floorlog2((int32_t)p->cblockw_init);
    cp.cblkh = (uint32_t)floorlog2((int32_t)p->cblockh_init);
    cp.irrev = p->irreversible ? 1 : 0;
    cp.mct = p->tcp_mct < 0 ? (img->numcomps >= 3 ? 1 : 0) : (p->tcp_mct == 2 ? 2 : p->tcp_mct ? 1 : 0);
    if (cp.mct == 1 && img->numcomps < 3) cp.mct = 0;
    if (p->mct_ncomp) {  // grk_set_MCT's mct_data (j2k.cpp:1899-1961)
        const uint32_t n = img->numcomps;
        if (p->mct_ncomp != n) return set_err(GRKGPU_EINVAL, "custom MCT matrix size differs from the component count");
        if (!p->irreversible) return set_err(GRKGPU_EUNSUPPORTED, "a custom MCT needs the 9/7 wavelet (grk_set_MCT sets it)");
        cp.mct = 2;
        for (uint32_t i = 0; i < n * n; ++i)  // (int32)(m * 2^13), mct.cpp:452-454
            cp.mct_coding[i] = (int32_t)(p->mct_matrix[i] * (float)(1 << 13));
        float m[16 * 16];
        memcpy(m, p->mct_matrix, sizeof(float) * n * n);
        if (!mct_invert(m, cp.mct_decoding, n))
            return set_err(GRKGPU_EINVAL, "Failed to inverse encoder MCT decoding matrix");
        for (uint32_t i = 0; i < n; ++i) {  // mct::calculate_norms (mct.cpp:409-427): column norms of the inverse
            double s = 0;
            for (uint32_t j = 0; j < n; ++j) {
                const float v = cp.mct_decoding[(size_t)j * n + i];
                s += (double)(v * v);
            }
            cp.mct_norms[i] = sqrt(s);
        }
    } else if (cp.mct == 2) {
        return set_err(GRKGPU_EINVAL, "tcp_mct 2 without a custom matrix (grkgpu_set_mct)");
    }
    // "Cannot perform MCT on components with different sizes. Disabling MCT." (j2k.cpp:1963-1971)
    if (cp.mct == 1 && (cp.dx[1] != cp.dx[0] || cp.dx[2] != cp.dx[0] || cp.dy[1] != cp.dy[0] || cp.dy[2] != cp.dy[0]))
        cp.mct = 0;
    if (cp.mct == 2) {
        for (uint32_t k = 1; k < img->numcomps; ++k)
            if (cp.dx[k] != cp.dx[0] || cp.dy[k] != cp.dy[0])
                return set_err(GRKGPU_EUNSUPPORTED, "a custom MCT over components of different sizes");
        for (uint32_t k = 0; k < img->numcomps; ++k) cp.shift[k] = p->mct_dc_shift[k];  // j2k.cpp:1952-1955
    }
    if (p->tile_size_on) {
        if (!p->cp_tdx || !p->cp_tdy) return set_err(GRKGPU_EINVAL, "zero tile size");
        if (p->cp_tx0 > img->x0 || p->cp_ty0 > img->y0 || (uint64_t)p->cp_tx0 + p->cp_tdx <= img->x0 ||
            (uint64_t)p->cp_ty0 + p->cp_tdy <= img->y0)
            return set_err(GRKGPU_EINVAL, "tile origin must satisfy tx0 <= x0 < tx0 + tdx");
        cp.tdx = p->cp_tdx; cp.tdy = p->cp_tdy; cp.tx0 = p->cp_tx0; cp.ty0 = p->cp_ty0;
        cp.tw = ceildiv(img->x1 - cp.tx0, cp.tdx);
        cp.th = ceildiv(img->y1 - cp.ty0, cp.tdy);
    } else {
        cp.tx0 = p->cp_tx0; cp.ty0 = p->cp_ty0;
        if (cp.tx0 > img->x0 || cp.ty0 > img->y0) return set_err(GRKGPU_EINVAL, "tile origin after the image origin");
        cp.tdx = img->x1 - cp.tx0; cp.tdy = img->y1 - cp.ty0;
        cp.tw = cp.th = 1;
    }
    if ((uint64_t)cp.tw * cp.th > 65535) return set_err(GRKGPU_EINVAL, "too many tiles");
    // layers and rate control (j2k.cpp:1841-1857)
    cp.numlayers = p->tcp_numlayers;
    cp.disto_alloc = p->cp_disto_alloc ? 1 : 0;
    cp.fixed_quality = p->cp_fixed_quality ? 1 : 0;
    cp.rate_algo = p->rate_control_algorithm == 1 ? 1 : 0;
    for (uint32_t j = 0; j < cp.numlayers; ++j) {
        const bool prof = p->rsiz != 0;
        if (cp.fixed_quality) cp.distoratio[j] = p->tcp_distoratio[j];
        if (prof || !cp.fixed_quality) cp.rates[j] = p->tcp_rates[j];
    }
    cp.rsiz = (uint16_t)p->rsiz;
    cp.max_cs_size = p->max_cs_size;
    cp.max_comp_size = p->max_comp_size;
    // coding style, precincts (j2k.cpp:1989-2041), progression, tile-parts
    if (p->csty & ~7u) return set_err(GRKGPU_EINVAL, "unknown csty bits");
    cp.csty = p->csty;
    if (p->prog_order < 0 || p->prog_order > 4) return set_err(GRKGPU_EINVAL, "unknown progression order");
    cp.prog = (uint32_t)p->prog_order;
    if ((cp.csty & CSTY_PRT) && p->res_spec) {
        uint32_t q = 0;
        for (int32_t r = (int32_t)cp.numres - 1; r >= 0; --r, ++q) {
            uint32_t w, h;
            if (q < p->res_spec) {
                w = p->prcw_init[q];
                h = p->prch_init[q];
            } else {
                const uint32_t rs = p->res_spec;
                w = p->prcw_init[rs - 1] >> (q - (rs - 1));
                h = p->prch_init[rs - 1] >> (q - (rs - 1));
            }
            cp.prcw[r] = (uint8_t)(w < 1 ? 1 : floorlog2((int32_t)w));
            cp.prch[r] = (uint8_t)(h < 1 ? 1 : floorlog2((int32_t)h));
        }
    } else {
        cp.csty &= ~CSTY_PRT;
        for (uint32_t r = 0; r < cp.numres; ++r) cp.prcw[r] = cp.prch[r] = 15;
    }
    if (p->numpocs) {
        // POC entries of tile 1 (the reference copies tile-matching entries,
        // j2k.cpp:1866-1890); more than one tile with POCs is not supported
        if (p->numpocs > 32) return set_err(GRKGPU_EINVAL, "at most 32 progression order changes");
        if (cp.tw * cp.th != 1) return set_err(GRKGPU_EUNSUPPORTED, "progression order changes need a single tile");
        uint32_t n = 0;
        for (uint32_t i = 0; i < p->numpocs; ++i) {
            if (p->POC[i].tile != 1) continue;
            const grkgpu_poc &src = p->POC[n];  // sic: indexed by the entry count (j2k.cpp:1872-1878)
            if (src.prog < 0 || src.prog > 4) return set_err(GRKGPU_EINVAL, "unknown POC progression");
            cp.pocs[n] = {src.resno0, src.compno0, src.layno1, src.resno1, src.compno1, (uint32_t)src.prog};
            ++n;
        }
        if (!n) return set_err(GRKGPU_EINVAL, "Problem with specified progression order changes");
        cp.numpocs = n;
    }
    cp.tp_on = p->tp_on != 0;
    cp.tp_flag = (char)p->tp_flag;
    generate_qcd(cp);
    return GRKGPU_OK;
}

// ---------------------------------------------------------------------------
// DWT job tables (dwt.hip).  Every tile-component owns two LL ping-pong
// buffers (A: the largest LL, R_{numres-2}; B: the next one), with rows padded
// to 16 elements.  Forward level l writes its LL into buffer l % 2 (the last
// level straight into the Mallat buffer); inverse level r writes into
// (numres - 2 - r) % 2 (the last into the output buffer).
// ---------------------------------------------------------------------------
static uint32_t pad16(uint32_t v) { return (v + 15) & ~15u; }

struct LLGeom { uint32_t strideA = 0, rowsA = 0, strideB = 0, rowsB = 0; uint64_t elems = 0; };

static LLGeom ll_geom(const TileComp &tc) {
    LLGeom g;
    if (tc.numres >= 2) { g.strideA = pad16(tc.res[tc.numres - 2].r.w()); g.rowsA = tc.res[tc.numres - 2].r.h(); }
    if (tc.numres >= 3) { g.strideB = pad16(tc.res[tc.numres - 3].r.w()); g.rowsB = tc.res[tc.numres - 3].r.h(); }
    g.elems = ((uint64_t)g.strideA * g.rowsA + 63) / 64 * 64 + ((uint64_t)g.strideB * g.rowsB + 63) / 64 * 64;
    return g;
}

struct DwtPlan {
    std::vector<std::vector<DwtJob>> levels;  // [level][job]
    std::vector<int> th;                      // window rows per level (dwt_finalize)
    std::vector<std::pair<int32_t *, const int32_t *>> copies;  // numres == 1: dst <- src
    uint64_t copy_elems = 0;
    struct Copy2D { int32_t *dst; const int32_t *src; uint32_t dpitch, spitch, w, h; };  // elements
    std::vector<Copy2D> copies2d;  // reduced decode at resolution 0: LL band -> compact output
    bool fused0 = false;  // forward level 0 reads the image planes (DC shift + MCT fused, dwt.hip)
    bool mct3 = false;    // ... and its jobs are MCT component triples (tile-major, component-minor)
    int32_t fmt = SMP_I32;  // ... reading image samples of this format
    bool inverse = false;
    std::vector<uint32_t> f01;  // per level: workgroups per job if levels l, l+1 run fused (k_dwt_fwd01), else 0
    std::vector<uint8_t> f01ny; // ... and its level-0 row windows per workgroup (k_dwt_fwd01)
    std::vector<uint8_t> pnw;   // ... or, run by k_dwt_fwd_pair: its level-l waves per workgroup (0: k_dwt_fwd01)
    std::vector<int32_t> ps1;   // ... and its level-(l+1) rows per segment
    uint32_t i01 = 0;           // inverse: workgroups per job if the last two levels run fused (k_dwt_inv01)
    bool restricted = false;    // inverse jobs limited to output regions (window decode)
};

// inverse with numres_dec < tc.numres (reduced-resolution decode): only the
// levels up to resolution numres_dec - 1; the last writes that resolution
// compactly (stride = its width) into `work`.
// resneed (window decode, inverse): per resolution the region (absolute
// resolution coordinates) whose samples the window needs (window_need); each
// inverse level then runs only the windows over its region.
static void dwt_plan_tc(DwtPlan &P, const TileComp &tc, int32_t *work, int32_t *coef, int32_t *llbase, int irrev,
                        bool inverse, uint32_t numres_dec = 0, const std::vector<Rect> *resneed = nullptr) {
    const uint32_t stride = tc.r.w(), rows = tc.r.h();
    P.inverse = inverse;
    if (!inverse || numres_dec == 0 || numres_dec > tc.numres) numres_dec = tc.numres;
    if (inverse && numres_dec == 1 && tc.numres > 1) {
        const Rect &r0 = tc.res[0].r;
        if (r0.w() && r0.h()) P.copies2d.push_back({work, coef, r0.w(), stride, r0.w(), r0.h()});
        return;
    }
    if (tc.numres == 1) {
        if (inverse) P.copies.push_back({work, coef});
        else P.copies.push_back({coef, work});
        P.copy_elems = (uint64_t)stride * rows;
        return;
    }
    const LLGeom g = ll_geom(tc);
    int32_t *buf[2] = {llbase, llbase + ((uint64_t)g.strideA * g.rowsA + 63) / 64 * 64};
    const uint32_t bstride[2] = {g.strideA, g.strideB}, brows[2] = {g.rowsA, g.rowsB};
    const uint32_t full_bytes = (uint32_t)std::min<uint64_t>((uint64_t)stride * rows * 4, 0xffffffffu);
    const uint32_t nlev = inverse ? numres_dec : tc.numres;
    if (P.levels.size() < nlev - 1) P.levels.resize(nlev - 1);
    for (uint32_t lvl = 0; lvl + 1 < nlev; ++lvl) {
        DwtJob j{};
        const bool last = lvl + 2 == nlev;
        Rect cur, lo;
        uint32_t slot;
        if (!inverse) {
            cur = tc.res[tc.numres - 1 - lvl].r;
            lo = tc.res[tc.numres - 2 - lvl].r;
            slot = lvl & 1;
            const uint32_t pslot = (lvl - 1) & 1;
            j.in = lvl == 0 ? work : buf[pslot];
            j.in_stride = lvl == 0 ? stride : bstride[pslot];
            j.in_bytes = lvl == 0 ? full_bytes : bstride[pslot] * brows[pslot] * 4;
            j.out = last ? coef : buf[slot];
            j.out_stride = last ? stride : bstride[slot];
            j.out_bytes = last ? full_bytes : bstride[slot] * brows[slot] * 4;
            j.bands = coef;
            j.bands_stride = stride;
            j.bands_bytes = full_bytes;
        } else {
            const uint32_t r = lvl + 1;
            cur = tc.res[r].r;
            lo = tc.res[r - 1].r;
            slot = (tc.numres - 2 - r) & 1;
            const uint32_t pslot = slot ^ 1;
            j.in = r == 1 ? coef : buf[pslot];
            j.in_stride = r == 1 ? stride : bstride[pslot];
            j.in_bytes = r == 1 ? full_bytes : bstride[pslot] * brows[pslot] * 4;
            j.coef = coef;
            j.coef_stride = stride;
            j.coef_bytes = full_bytes;
            const bool compact = numres_dec < tc.numres;  // reduced: the last level's output is compact
            j.out = last ? work : buf[slot];
            j.out_stride = last ? (compact ? cur.w() : stride) : bstride[slot];
            j.out_bytes = last ? full_bytes : bstride[slot] * brows[slot] * 4;
        }
        if (!cur.w() || !cur.h()) continue;
        j.rw = (int32_t)cur.w(); j.rh = (int32_t)cur.h();
        j.casx = (int32_t)(cur.x0 & 1); j.casy = (int32_t)(cur.y0 & 1);
        j.snx = (int32_t)lo.w(); j.sny = (int32_t)lo.h();
        if (inverse && resneed && lvl + 1 < resneed->size()) {
            const Rect &n = (*resneed)[lvl + 1];  // region of the resolution this level reconstructs
            j.reg_x0 = (int32_t)n.x0 - (int32_t)cur.x0; j.reg_x1 = (int32_t)n.x1 - (int32_t)cur.x0;
            j.reg_y0 = (int32_t)n.y0 - (int32_t)cur.y0; j.reg_y1 = (int32_t)n.y1 - (int32_t)cur.y0;
            if (j.reg_x1 <= j.reg_x0 || j.reg_y1 <= j.reg_y0) j.reg_x0 = j.reg_y0 = 0, j.reg_x1 = j.reg_y1 = 1;
            P.restricted = true;
        }
        P.levels[lvl].push_back(j);
    }
}

// Forward 9/7 levels l and l + 1 fused into one launch (dwt.hip
// k_dwt_fwd01: level l + 1 lifted from level l's LL band kept in LDS) when
// every tile-component has both levels, level l is not the fused DC shift +
// MCT one, and the resolutions are big enough (>= 16 samples each way) for
// the fused windows; f01_rows = 0 keeps one launch per level.  Returns
// the workgroups per job, 0 = not fused.
static uint32_t dwt_f01_tiles(const DwtPlan &P, size_t li, int irrev, int *ny, int *nw0, int *s1) {
    const DwtOptions &o = dwt_options();
    *nw0 = 0;
    if (P.inverse || (li == 0 && P.fused0) || li + 1 >= P.levels.size() || !o.f01_rows) return 0;
    // k_dwt_fwd_pair for 5/3 (pair_kernel 1, the default) or for both (2);
    // 9/7 keeps k_dwt_fwd01's windows by default: the streamed pair moves
    // less (435 vs 593 MB read per 8K frame) but its barrier-coupled
    // strips leave the 64-bit fixed-point lifting latency-bound -- 198 us
    // against 185 (profiles/r05/dwt_pair_ab.txt)
    const bool stream = o.pair_kernel == 2 || (o.pair_kernel == 1 && !irrev);
    if (!irrev && !stream) return 0;
    const auto &l0 = P.levels[li], &l1 = P.levels[li + 1];
    if (l0.empty() || l0.size() != l1.size()) return 0;
    uint64_t samples = 0;
    for (auto &j : l0) samples += (uint64_t)j.rw * j.rh;
    for (size_t i = 0; i < l0.size(); ++i) {
        const DwtJob &a = l0[i], &b = l1[i];
        if (a.snx != b.rw || a.sny != b.rh || a.rw < 16 || a.rh < 16 || b.rw < 16 || b.rh < 16) return 0;
        if (a.out != b.in) return 0;  // level l + 1 must read level l's LL
        if (a.reg_x1 > 0 || b.reg_x1 > 0) return 0;
    }
    if (stream) {
        // k_dwt_fwd_pair: strips of CW1 level-(l+1) columns (3 or 4 level-l
        // waves, whichever wastes fewer columns at the jobs' widths), segments
        // of S1 rows sized so that the launch is about one resident wave of
        // workgroups (3 per CU: 30 KB of LDS and 6 wavefronts each)
        if (samples < o.pair_min_samples) return 0;
        uint64_t cols[2] = {0, 0};
        int maxh = 0;
        for (auto &b : l1) {
            for (int k = 0; k < 2; ++k) {
                const int cw1 = dwt_pair_cw1(irrev, 3 + k);
                cols[k] += (uint64_t)((b.rw + b.casx + cw1 - 1) / cw1) * (3 + k);
            }
            maxh = std::max(maxh, b.rh + b.casy);
        }
        *nw0 = o.pair_waves ? o.pair_waves : cols[0] < cols[1] ? 3 : 4;
        uint64_t strips = 0;
        for (auto &b : l1) {
            const int cw1 = dwt_pair_cw1(irrev, *nw0);
            strips += (uint64_t)((b.rw + b.casx + cw1 - 1) / cw1);
        }
        int rows = o.pair_rows;
        if (!rows) {
            const uint64_t target = 768;
            const uint64_t nseg = std::max<uint64_t>(1, (target + strips / 2) / std::max<uint64_t>(strips, 1));
            rows = (int)(((uint64_t)maxh + nseg - 1) / nseg);
            // whole level-(l+1) chunks of 8 rows: 9/7 streams start 2 rows
            // above the segment (8k - 2 rows), 5/3 at it (8k)
            rows = irrev ? std::max(14, (rows + 2 + 7) / 8 * 8 - 2) : std::max(8, (rows + 7) / 8 * 8);
        }
        *s1 = rows;
        uint32_t maxt = 0;
        for (auto &b : l1)
            maxt = std::max<uint32_t>(maxt, (uint32_t)dwt_pair_wgs(irrev, *nw0, rows, b.rw, b.rh, b.casx, b.casy));
        return maxt;
    }
    // k_dwt_fwd01: only where the pair still fills the chip (f01_min_samples,
    // default 2^23): the 8K frame's levels 2 + 3 fused with 4 row windows took
    // 26 us against 14 + 7 apart (378 workgroups), and with 2 row windows
    // (twice the workgroups; f01_small_min_samples, off by default) 26.4 us
    // of kernel time, the frame's DWT span 220 us against 217 apart
    if (samples >= o.f01_min_samples) *ny = o.f01_rows;
    else if (samples >= o.f01_small_min_samples) *ny = 2;
    else return 0;
    uint32_t maxt = 0;
    for (size_t i = 0; i < l0.size(); ++i) {
        const DwtJob &b = l1[i];
        int tx;
        const int n = dwt01_tiles(irrev, *ny, b.rw, b.rh, b.casx, b.casy, &tx);
        if (n <= 0) return 0;
        maxt = std::max<uint32_t>(maxt, (uint32_t)n);
    }
    return maxt;
}

// The two largest inverse levels (the last two of an inverse plan) in one
// launch (dwt.hip k_dwt_inv01: the smaller one's output kept in LDS) when
// every tile-component has both, the second reads the first's output, both
// resolutions are >= 16 samples each way and the larger level has at least
// inv01_min_samples samples.  Returns the workgroups per job, 0 = apart.
static uint32_t dwt_inv01_plan(const DwtPlan &P, int irrev) {
    const DwtOptions &o = dwt_options();
    const size_t n = P.levels.size();
    if (!P.inverse || !o.inv01 || n < 2 || P.restricted) return 0;
    const auto &la = P.levels[n - 2], &lb = P.levels[n - 1];
    if (la.empty() || la.size() != lb.size()) return 0;
    uint64_t samples = 0;
    for (auto &j : lb) samples += (uint64_t)j.rw * j.rh;
    if (samples < o.inv01_min_samples) return 0;
    uint32_t maxt = 0;
    for (size_t i = 0; i < la.size(); ++i) {
        const DwtJob &a = la[i], &b = lb[i];
        if (b.in != a.out || b.snx != a.rw || b.sny != a.rh || a.rw < 16 || a.rh < 16 || b.rw < 16 || b.rh < 16)
            return 0;
        maxt = std::max<uint32_t>(maxt, (uint32_t)dwt_inv01_tiles(irrev, b.rw, b.rh, b.casx, b.casy));
    }
    return maxt;
}

// Pick each level's window height from the level's total size; tile counts.
static void dwt_finalize(DwtPlan &P, int irrev) {
    P.i01 = dwt_inv01_plan(P, irrev);
    P.th.assign(P.levels.size(), 8);
    for (size_t l = 0; l < P.levels.size(); ++l) {
        uint64_t samples = 0;
        int minw = INT32_MAX, minh = INT32_MAX;
        for (auto &j : P.levels[l]) {
            samples += (uint64_t)j.rw * j.rh;
            minw = std::min(minw, (int)j.rw);
            minh = std::min(minh, (int)j.rh);
        }
        P.th[l] = dwt_pick_th(irrev, samples, minw, minh);
        // the fused DC shift + MCT level 0 holds the windows of three
        // components: 8-row windows (measured on the 8K frame: 5/3 162 us at
        // TH 8, 168 at 16, 194 at 32; 9/7 229 / 319 / 330)
        if (l == 0 && P.mct3) P.th[l] = 8;
        for (auto &j : P.levels[l]) dwt_job_tiles(irrev, P.th[l], j);
    }
    // Fused level pairs (k_dwt_fwd01).  A fused pair never writes its first
    // level's LL band, so the LL ping-pong is re-dealt: every level reads the
    // last LL band written and keeps its own output slot unless its launch
    // reads that slot (for a fused pair: the pair's input), in which case it
    // takes the other one -- no launch reads and writes one buffer.
    P.f01.assign(P.levels.size(), 0);
    P.f01ny.assign(P.levels.size(), 0);
    P.pnw.assign(P.levels.size(), 0);
    P.ps1.assign(P.levels.size(), 0);
    bool any = false;
    for (size_t l = 0; l + 1 < P.levels.size(); ++l) {
        int ny = 4, nw0 = 0, s1 = 0;
        if ((P.f01[l] = dwt_f01_tiles(P, l, irrev, &ny, &nw0, &s1))) {
            P.f01ny[l] = (uint8_t)ny;
            P.pnw[l] = (uint8_t)nw0;
            P.ps1[l] = s1;
            any = true;
            ++l;
        }
    }
    // the re-deal below pairs job i of every level (one tile-component)
    for (auto &l : P.levels) any = any && l.size() == P.levels[0].size();
    if (!any) {
        P.f01.assign(P.levels.size(), 0);
        return;
    }
    struct Slot { int32_t *p; uint32_t stride, bytes; };
    for (size_t i = 0; i < P.levels[0].size(); ++i) {
        Slot slot[2] = {{P.levels[0][i].out, P.levels[0][i].out_stride, P.levels[0][i].out_bytes}, {nullptr, 0, 0}};
        if (P.levels.size() > 2) slot[1] = {P.levels[1][i].out, P.levels[1][i].out_stride, P.levels[1][i].out_bytes};
        Slot prev{const_cast<int32_t *>(P.levels[0][i].in), P.levels[0][i].in_stride, P.levels[0][i].in_bytes};
        for (size_t l = 0; l < P.levels.size(); ++l) {
            DwtJob &j = P.levels[l][i];
            const bool second = l > 0 && P.f01[l - 1];
            if (!second) { j.in = prev.p; j.in_stride = prev.stride; j.in_bytes = prev.bytes; }
            if (j.out != j.bands) {  // not the last level (that one writes its LL into the Mallat buffer)
                // the plan's own slot unless the launch reads it
                const int32_t *rd = second ? P.levels[l - 1][i].in : j.in;
                if (j.out == rd) {
                    const Slot &o = slot[0].p != rd ? slot[0] : slot[1];
                    j.out = o.p; j.out_stride = o.stride; j.out_bytes = o.bytes;
                }
            }
            prev = {j.out, j.out_stride, j.out_bytes};
        }
    }
}

// Upload the job table (one H2D from pinned memory).
static hipError_t dwt_upload(DwtPlan &P, DevBuf &djobs, HostBuf &hjobs, int irrev, hipStream_t s) {
    dwt_finalize(P, irrev);
    size_t n = 0;
    for (auto &l : P.levels) n += l.size();
    if (!n) return hipSuccess;
    hipError_t e = djobs.ensure(n * sizeof(DwtJob) + 256);
    if (e == hipSuccess) e = hjobs.ensure(n * sizeof(DwtJob) + 256);
    if (e != hipSuccess) return e;
    DwtJob *h = hjobs.as<DwtJob>();
    size_t k = 0;
    for (auto &l : P.levels)
        for (auto &j : l) h[k++] = j;
    return hipMemcpyAsync(djobs.p, hjobs.p, n * sizeof(DwtJob), hipMemcpyHostToDevice, s);
}

// Run the levels (job table already uploaded by dwt_upload on the same stream).
// All levels of an uploaded plan (job table at djobs, levels back to back);
// fused 9/7 level pairs (P.f01) as one launch (8K frame: 0+1, then 2, 3, 4).
// Launch log (grkgpu_set_launch_timing): events around every level launch
// and each launch's kernel and algorithmic bytes (B_DWT's 8 B per sample of
// every level it computes).
// Per-launch device times: one event between consecutive launches of a
// level sequence (a launch's end is the next one's start), so what a launch
// is charged is the stream's time from the previous launch's end to its own
// -- an event pair around every launch added ~1.5 us of event handling to
// each (8K 9/7: 224.7 us summed vs 213.4 by rocprof, 218.6 span).
struct LaunchLog {
    std::vector<hipEvent_t> *ev;
    std::vector<grkgpu_launch_time> *rec;
    std::vector<std::pair<uint32_t, uint32_t>> *idx;
    uint32_t used = 0;  // events recorded in this call
};

static uint64_t level_bytes(const std::vector<DwtJob> &l) {
    uint64_t n = 0;
    for (auto &j : l) n += 8ull * (uint64_t)j.rw * (uint64_t)j.rh;
    return n;
}

static hipError_t log_event(LaunchLog *log, hipStream_t s, uint32_t *at) {
    while (log->ev->size() <= log->used) {
        hipEvent_t e;
        hipError_t r = hipEventCreate(&e);
        if (r != hipSuccess) return r;
        log->ev->push_back(e);
    }
    *at = log->used++;
    return hipEventRecord((*log->ev)[*at], s);
}

// chained: the previous logged launch ended right before this one (same
// level sequence, nothing else enqueued in between): its end event is this
// launch's start
static hipError_t log_begin(LaunchLog *log, hipStream_t s, const char *name, uint32_t lev0, uint32_t nlev, uint64_t bytes,
                            bool chained = false) {
    if (!log) return hipSuccess;
    grkgpu_launch_time t{};
    snprintf(t.kernel, sizeof(t.kernel), "%s", name);
    t.level0 = lev0;
    t.levels = nlev;
    t.bytes = bytes;
    uint32_t at;
    if (chained && !log->idx->empty()) {
        at = log->idx->back().second;
    } else {
        hipError_t r = log_event(log, s, &at);
        if (r != hipSuccess) return r;
    }
    log->rec->push_back(t);
    log->idx->push_back({at, at});
    return hipSuccess;
}

static hipError_t log_end(LaunchLog *log, hipStream_t s) {
    if (!log) return hipSuccess;
    return log_event(log, s, &log->idx->back().second);
}

static hipError_t dwt_run_levels(const DwtPlan &P, DwtJob *djobs, int irrev, bool inverse, hipStream_t s,
                                 LaunchLog *log = nullptr) {
    hipError_t e = hipSuccess;
    size_t k = 0;
    const char *wl = irrev ? "9/7" : "5/3";
    char name[48];
    for (size_t li = 0; li < P.levels.size(); ++li) {
        const auto &l = P.levels[li];
        if (li < P.f01.size() && P.f01[li]) {
            snprintf(name, sizeof(name), P.pnw[li] ? "k_dwt_fwd_pair<%s>" : "k_dwt_fwd01<%s>", wl);
            if ((e = log_begin(log, s, name, (uint32_t)li, 2, level_bytes(l) + level_bytes(P.levels[li + 1]), li > 0)))
                return e;
            if (P.pnw[li])
                e = launch_dwt_fwd_pair(djobs + k, djobs + k + l.size(), (uint32_t)l.size(), P.f01[li], irrev, P.pnw[li],
                                        P.ps1[li], s);
            else
                e = launch_dwt_fwd01(djobs + k, djobs + k + l.size(), (uint32_t)l.size(), P.f01[li], irrev, P.f01ny[li],
                                     s);
            if (e != hipSuccess || (e = log_end(log, s))) return e;
            k += l.size() + P.levels[li + 1].size();
            ++li;
            continue;
        }
        if (inverse && P.i01 && li + 2 == P.levels.size()) {
            snprintf(name, sizeof(name), "k_dwt_inv01<%s>", wl);
            if ((e = log_begin(log, s, name, (uint32_t)li, 2, level_bytes(l) + level_bytes(P.levels[li + 1]), li > 0)))
                return e;
            e = launch_dwt_inv01(djobs + k, djobs + k + l.size(), (uint32_t)l.size(), P.i01, irrev,
                                 dwt_options().inv01, s);
            if (e != hipSuccess || (e = log_end(log, s))) return e;
            k += l.size() + P.levels[li + 1].size();
            ++li;
            continue;
        }
        uint32_t maxt = 0;
        for (auto &j : l) maxt = std::max<uint32_t>(maxt, (uint32_t)j.ntiles);
        const bool f0 = li == 0 && P.fused0 && !inverse;
        const int code = P.th[li] | (f0 ? (P.mct3 ? DWT_FUSED_MCT3 : DWT_FUSED) | (P.fmt << DWT_FMT_SHIFT) : 0);
        snprintf(name, sizeof(name), "%s<%s,%d>", inverse ? "k_dwt_inv" : f0 && P.mct3 ? "k_dwt_fwd_mct3" : "k_dwt_fwd", wl,
                 P.th[li] & 0xff);
        if ((e = log_begin(log, s, name, (uint32_t)li, 1, level_bytes(l), li > 0))) return e;
        e = launch_dwt_jobs(djobs + k, (uint32_t)l.size(), maxt, code, irrev, inverse ? 1 : 0, s);
        if (e != hipSuccess || (e = log_end(log, s))) return e;
        k += l.size();
    }
    return hipSuccess;
}

// fill in the launch times once the stream has passed the logged launches
static void log_collect(grkgpu_ctx *c) {
    for (size_t i = 0; i < c->ltimes.size() && i < c->lidx.size(); ++i)
        if (hipEventElapsedTime(&c->ltimes[i].ms, c->lev[c->lidx[i].first], c->lev[c->lidx[i].second]) != hipSuccess)
            c->ltimes[i].ms = -1;
}

static hipError_t dwt_launch(DwtPlan &P, DevBuf &djobs, int irrev, bool inverse, hipStream_t s,
                             LaunchLog *log = nullptr) {
    for (auto &cp : P.copies) {
        hipError_t e = hipMemcpyAsync(cp.first, cp.second, P.copy_elems * 4, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
    }
    for (auto &cp : P.copies2d) {
        hipError_t e = hipMemcpy2DAsync(cp.dst, (size_t)cp.dpitch * 4, cp.src, (size_t)cp.spitch * 4, (size_t)cp.w * 4,
                                        cp.h, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
    }
    return dwt_run_levels(P, djobs.as<DwtJob>(), irrev, inverse, s, log);
}

static bool overlap(const Rect &a, const Rect &b) { return a.x0 < b.x1 && b.x0 < a.x1 && a.y0 < b.y1 && b.y0 < a.y1; }
static Rect intersect(const Rect &a, const Rect &b) {
    Rect r{std::max(a.x0, b.x0), std::max(a.y0, b.y0), std::min(a.x1, b.x1), std::min(a.y1, b.y1)};
    if (r.x1 < r.x0) r.x1 = r.x0;
    if (r.y1 < r.y0) r.y1 = r.y0;
    return r;
}

using BandNeed = std::vector<std::array<Rect, 3>>;  // [resno][band] region a window needs

// need: (window decode) only code-blocks overlapping need[resno][band].
template <typename F>
static void for_each_cblk(TileComp &tc, F f, uint32_t maxres = 0xffffffffu, const BandNeed *need = nullptr) {
    for (uint32_t resno = 0; resno < tc.numres && resno < maxres; ++resno) {
        Resolution &res = tc.res[resno];
        for (uint32_t b = 0; b < res.numbands; ++b) {
            Band &band = res.bands[b];
            for (auto &pr : band.precs)
                for (auto &c : pr.cblks)
                    if (!need || overlap(c.r, (*need)[resno][b])) f(band, c);
        }
    }
}

// Window decode: the sub-band regions whose coefficients reach the samples
// of `win` (tile-component coordinates).  Going down from the full
// resolution, a region of resolution r needs, in each of its bands and in the
// resolution r-1 below, the half-size region widened by M samples on every
// side -- more than the synthesis supports (5/3: 2 taps, 9/7: 4 taps at the
// full scale, i.e. <= 2 at the band scale), so every coefficient that
// influences the window is decoded and the window's samples come out exactly
// as in a full decode (dwt.cpp decode_tile_53 / _97 compute each output from
// its support only).
// resneed (optional): per resolution the region of its samples the window
// needs (the inverse DWT levels run only over these).
static BandNeed window_need(const TileComp &tc, const Rect &win, std::vector<Rect> *resneed = nullptr,
                            uint32_t reduce = 0) {
    constexpr uint32_t M = 4;
    BandNeed need(tc.numres);
    // win: on the component's grid at resolution numres - 1 - reduce
    Rect n = intersect(win, tc.res[tc.numres - 1 - reduce].r);
    if (resneed) resneed->assign(tc.numres, Rect{});
    for (int32_t r = (int32_t)tc.numres - 1 - (int32_t)reduce; r >= 0; --r) {
        const Resolution &res = tc.res[r];
        if (resneed) (*resneed)[r] = n;
        if (r == 0) {
            need[0][0] = intersect(n, res.bands[0].r);
            break;
        }
        const Rect half{n.x0 / 2 > M ? n.x0 / 2 - M : 0, n.y0 / 2 > M ? n.y0 / 2 - M : 0, (n.x1 + 1) / 2 + M,
                        (n.y1 + 1) / 2 + M};
        for (uint32_t b = 0; b < res.numbands; ++b) need[r][b] = intersect(half, res.bands[b].r);
        n = intersect(half, tc.res[r - 1].r);
    }
    return need;
}

// ---------------------------------------------------------------------------
// encode
// ---------------------------------------------------------------------------
// Encode tiles [tb, te) (a tile shard: j2k_encode's per-tile loop,
// j2k.cpp:2088-2111) and emit [main header][their tile-parts][EOC] per `parts`.
// export_blocks: stop after Tier-1 and hand the per-code-block results to the
// caller instead of writing a codestream (grkgpu_encode_blocks).
//
// row0 / nrows: the planes hold only image rows [row0, row0 + nrows) (a tile-
// row shard: a rank loads just the rows of its tiles); nrows = 0: all rows.
static int compress_impl(grkgpu_ctx *c, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                         const void *const *planes, int planes_on_device, int32_t fmt, const uint8_t **view,
                         size_t *outlen,
                         uint32_t tb = 0, uint32_t te = 0xffffffffu, uint32_t parts = GRKGPU_PART_ALL,
                         bool export_blocks = false, int force_dist = 0, uint32_t row0 = 0, uint32_t nrows = 0,
                         uint32_t col0 = 0, uint32_t ncols = 0) {
    if (!c || !planes) return set_err(GRKGPU_EINVAL, "null argument");
    ActiveCall active;
    CodingParams cp;
    int rc = setup_params(img, p, cp);
    if (rc) return rc;
    if (fmt < SMP_I32 || fmt > SMP_I16) return set_err(GRKGPU_EINVAL, "unknown sample format");
    for (uint32_t k = 0; fmt != SMP_I32 && k < img->numcomps; ++k) {
        const bool sg = fmt == SMP_I8 || fmt == SMP_I16;
        if ((img->sgnd[k] != 0) != sg || img->prec[k] > 8 * sample_bytes(fmt))
            return set_err(GRKGPU_EINVAL, "sample format does not hold the component's precision / signedness");
    }
    const uint32_t sb = sample_bytes(fmt);  // bytes per input sample
    {
        const uint32_t nt = cp.tw * cp.th;
        if (te > nt) te = nt;
        if (tb > te) return set_err(GRKGPU_EINVAL, "bad tile range");
    }
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    double t_start = now_ms();
    const uint32_t nc = cp.numcomps, iw = cp.image.w(), ih = cp.image.h();
    if (nrows == 0) {
        if (row0) return set_err(GRKGPU_EINVAL, "row0 without nrows");
        nrows = ih;
    }
    if ((uint64_t)row0 + nrows > ih) return set_err(GRKGPU_EINVAL, "row range outside the image");
    if (ncols == 0) {
        if (col0) return set_err(GRKGPU_EINVAL, "col0 without ncols");
        ncols = iw;
    }
    if ((uint64_t)col0 + ncols > iw) return set_err(GRKGPU_EINVAL, "column range outside the image");
    const uint32_t pw = ncols;                    // row stride of the caller's planes (samples)
    const uint64_t plane = (uint64_t)pw * nrows;  // samples per plane held by the caller
    // subsampled components (SIZ XRsiz / YRsiz): each plane on its own grid
    bool subs = false, mixed = false;  // mixed: components on different grids
    for (uint32_t k = 0; k < nc; ++k) {
        subs = subs || cp.dx[k] != 1 || cp.dy[k] != 1;
        mixed = mixed || cp.dx[k] != cp.dx[0] || cp.dy[k] != cp.dy[0];
    }
    // the rectangle each caller plane covers (the rows / columns held, on the
    // component's grid: ceil(x / dx), TileComponent.cpp:150-196 -- a tile's
    // plane holds its tile-component, as grk_write_tile's data does,
    // TileProcessor.cpp:1923-1972), its stride, and its offset in the staging
    // buffer (samples)
    Rect prect[GRKGPU_MAX_COMPS];
    uint64_t poff[GRKGPU_MAX_COMPS + 1];
    poff[0] = 0;
    const Rect held{cp.image.x0 + col0, cp.image.y0 + row0, cp.image.x0 + col0 + ncols, cp.image.y0 + row0 + nrows};
    for (uint32_t k = 0; k < nc; ++k) {
        prect[k] = comp_rect(held, cp.dx[k], cp.dy[k]);
        poff[k + 1] = poff[k] + (uint64_t)prect[k].w() * prect[k].h();
    }
    (void)subs;
    // element offset of tile-component tc's first sample in plane k
    auto plane_org = [&](uint32_t k, const TileComp &tc) {
        return (uint64_t)(tc.r.y0 - prect[k].y0) * prect[k].w() + (tc.r.x0 - prect[k].x0);
    };

    // geometry for every tile of the shard, arena offsets, block table
    const uint32_t ntiles = te - tb;
    std::vector<Tile> tiles(ntiles);
    uint64_t arena = 0, llarena = 0;
    std::vector<uint64_t> lloff(ntiles * nc);
    std::vector<EncBlock> eb;
    struct BlkInfo {  // position + distortion weights (t1_getwmsedec)
        uint32_t compno, level, orient;
        float stepsize;
        uint32_t tileno, resno, precno, cblkno;
        Rect r;
    };
    std::vector<BlkInfo> binfo;
    std::vector<uint64_t> symoff;  // per-block symbol-stream slots, sized by the band's numbps bound
    std::vector<uint32_t> pcap;    // per-block pass-record slots (3 numbps - 2 of that bound)
    uint64_t sym_total = 0;
    uint32_t maxdepth = 1;
    // tile geometry (independent per tile) on the host pool, then the block
    // table in tile order
    for (uint32_t t = 0; t < ntiles; ++t) {
        const Rect r = tile_rect(cp, tb + t);
        if (r.y0 - cp.image.y0 < row0 || r.y1 - cp.image.y0 > row0 + nrows || r.x0 - cp.image.x0 < col0 ||
            r.x1 - cp.image.x0 > col0 + ncols)
            return set_err(GRKGPU_EINVAL, "a tile of the range lies outside the rows / columns given");
    }
    host_parallel_for(ntiles, 1, [&](size_t t0, size_t t1) {
        for (size_t t = t0; t < t1; ++t) {
            Tile &tile = tiles[t];
            tile.index = tb + (uint32_t)t;
            tile.r = tile_rect(cp, tile.index);
            tile.comps.resize(nc);
            for (uint32_t k = 0; k < nc; ++k) build_tilecomp(tile.comps[k], tile.r, cp, k, true);
        }
    });
    for (uint32_t t = 0; t < ntiles; ++t) {
        Tile &tile = tiles[t];
        for (uint32_t k = 0; k < nc; ++k) {
            TileComp &tc = tile.comps[k];
            tc.arena_off = arena;
            uint64_t area = (uint64_t)tc.r.w() * tc.r.h();
            arena += (area + 63) & ~63ull;
            lloff[t * nc + k] = llarena;
            llarena += ll_geom(tc).elems;
            for_each_cblk(tc, [&](Band &band, Cblk &cb) {
                cb.gidx = (uint32_t)eb.size();
                EncBlock b;
                b.coef_off = tc.arena_off + (uint64_t)cb.by * tc.r.w() + cb.bx;
                b.out_off = 0;
                b.stride = tc.r.w();
                b.w = cb.r.w();
                b.h = cb.r.h();
                b.orient = band.bandno;
                b.qmfbid = cp.irrev ? 0 : 1;
                b.inv_step = (int32_t)band.inv_step;
                eb.push_back(b);
                uint32_t resno = 0;
                while (&tc.res[resno].bands[0] > &band || &tc.res[resno].bands[2] < &band) ++resno;
                uint32_t precno = 0, cblkno = 0;
                for (size_t q = 0; q < band.precs.size(); ++q) {
                    const auto &cv = band.precs[q].cblks;
                    if (!cv.empty() && &cb >= &cv.front() && &cb <= &cv.back()) {
                        precno = (uint32_t)q;
                        cblkno = (uint32_t)(&cb - &cv.front());
                        break;
                    }
                }
                binfo.push_back({k, tc.numres - 1 - resno, band.bandno, band.stepsize, tile.index, resno, precno,
                                 cblkno, cb.r});
                const uint32_t bound = std::min<uint32_t>(band.numbps, 32);
                pcap.push_back(bound ? 3 * bound - 2 : 0);
                symoff.push_back(sym_total);
                sym_total += (uint64_t)bound * sym_slot_bytes(b.w, b.h);
                maxdepth = std::max(maxdepth, bound);
            });
        }
    }
    const uint32_t nblk = (uint32_t)eb.size();
    uint64_t out_total = 0;
    for (auto &b : eb) {  // MQ output slab: w*h*4 bytes (+ the zero pad byte before)
        out_total += 16;
        b.out_off = out_total;
        out_total += ((uint64_t)b.w * b.h * 4 + 64 + 15) & ~15ull;
    }
    HIPCHK(c->work.ensure(arena * 4 + 256));
    HIPCHK(c->coef.ensure(arena * 4 + 256));
    HIPCHK(c->ll.ensure(llarena * 4 + 256));
    HIPCHK(c->scratch.ensure((size_t)t1e_scratch_bytes(nblk, maxdepth) + 256));
    HIPCHK(c->t1order.ensure((size_t)t1_order_words(nblk) * 4 + 256));
    HIPCHK(c->mqout.ensure(out_total + 256));
    HIPCHK(c->blocks.ensure((size_t)nblk * sizeof(EncBlock) + 256));
    HIPCHK(c->results.ensure((size_t)nblk * sizeof(EncResult) + 256));
    HIPCHK(c->h_results.ensure((size_t)nblk * sizeof(EncResult) + 256));
    HIPCHK(c->h_blocks.ensure((size_t)nblk * sizeof(EncBlock) + 256));
    symoff.push_back(sym_total);
    HIPCHK(c->sym.ensure(sym_total + 256));
    HIPCHK(c->symoff.ensure(symoff.size() * 8 + 256));
    HIPCHK(c->h_symoff.ensure(symoff.size() * 8 + 256));

    HIPCHK(hipEventRecord(c->ev[0], s));
    // input planes on the device, as the caller's samples (widened to int32
    // by the first kernel that reads them)
    SrcPlanes src{};
    if (planes_on_device) {
        for (uint32_t k = 0; k < nc; ++k) src.p[k] = planes[k];
    } else {
        HIPCHK(c->img.ensure(poff[nc] * sb + 256));
        for (uint32_t k = 0; k < nc; ++k) {
            src.p[k] = c->img.as<uint8_t>() + poff[k] * sb;
            HIPCHK(hipMemcpyAsync((void *)src.p[k], planes[k], (poff[k + 1] - poff[k]) * sb, hipMemcpyHostToDevice,
                                  s));
        }
    }
    auto src_at = [&](uint32_t k, uint64_t off) { return (const void *)((const uint8_t *)src.p[k] + off * sb); };
    HIPCHK(hipEventRecord(c->ev[1], s));
    ShiftArr sh{};
    for (uint32_t k = 0; k < nc; ++k) sh.v[k] = cp.shift[k];
    // The DC shift + RCT of a 3-component 5/3 tile is fused into its first
    // DWT level (k_dwt_fwd_mct3: one wavefront reads the three image planes
    // once and lifts the three components of its window): 162 us instead of
    // 132 (MCT pass) + 133 (level 0) on the 8K frame.  The 9/7 (ICT) triple
    // is left separate: fused 229 us vs 132 + 145, but the separate level-0
    // launch is the DWT whose roofline the bench reports.
    // grkgpu_dwt_options.fuse_level0 = 0 / 1 forces it off / on (1: also 9/7
    // and single components, DC shift in the loads).  Requires every
    // tile-component to be decomposed at least once and to span its tile.
    const int fo = dwt_options().fuse_level0;
    bool fuse = fo >= 0 ? fo != 0 : (!cp.irrev && cp.mct == 1 && nc == 3);
    for (auto &tile : tiles)
        for (uint32_t k = 0; k < nc; ++k) {
            const TileComp &tc = tile.comps[k];
            fuse = fuse && tc.numres >= 2 && tc.r.w() == tile.r.w() && tc.r.h() == tile.r.h();
        }
    if ((cp.mct && nc != 3) || cp.mct == 2) fuse = false;  // MCT over more than 3 components, custom MCT: separate pass
    if (fmt == SMP_I8 || fmt == SMP_I16) fuse = false;  // the fused loads read int32, u16 or u8 samples
    DwtPlan dplan;
    dplan.fused0 = fuse;
    dplan.mct3 = fuse && cp.mct == 1 && nc == 3;
    for (auto &tile : tiles)
        for (uint32_t k = 0; k < nc; ++k) {
            const TileComp &tc = tile.comps[k];
            const size_t before = dplan.levels.empty() ? 0 : dplan.levels[0].size();
            dwt_plan_tc(dplan, tc, c->work.as<int32_t>() + tc.arena_off, c->coef.as<int32_t>() + tc.arena_off,
                        c->ll.as<int32_t>() + lloff[(tile.index - tb) * nc + k], cp.irrev, false);
            if (!fuse || dplan.levels.empty() || dplan.levels[0].size() == before) continue;
            DwtJob &j = dplan.levels[0].back();
            const uint64_t org = plane_org(k, tc);  // fused: no subsampling, every plane alike
            const bool mct3 = cp.mct == 1 && nc >= 3 && k < 3;
            for (uint32_t i = 0; i < 3; ++i) {
                const uint32_t pk = mct3 ? i : k;
                j.src[i] = src_at(pk, org);
                j.shift[i] = cp.shift[pk];
            }
            j.src_stride = pw;
            j.src_bytes = (uint32_t)std::min<uint64_t>((plane - org) * sb, 0xffffffffu);
            j.src_fmt = fmt;
            j.mct_mode = mct3 ? (cp.irrev ? 3 : 2) : 1;
            j.comp = (int32_t)k;
            bool al = (pw & 1) == 0;
            for (uint32_t i = 0; i < 3; ++i) al = al && ((uintptr_t)j.src[i] & (2 * sb - 1)) == 0;
            j.src_vec = al ? 1 : 0;
        }
    dplan.fmt = fmt;
    HIPCHK(dwt_upload(dplan, c->dwtjobs, c->h_dwtjobs, cp.irrev, s));
    for (auto &tile : tiles) {
        if (fuse) break;
        if (mixed) {  // one launch per tile-component, each on its own grid (no MCT, j2k.cpp:1963-1971)
            for (uint32_t k = 0; k < nc; ++k) {
                const TileComp &tc = tile.comps[k];
                SrcPlanes tsrc{};
                PlanePtrs tdst{};
                ShiftArr sk{};
                tsrc.p[0] = src_at(k, plane_org(k, tc));
                tdst.p[0] = c->work.as<int32_t>() + tc.arena_off;
                sk.v[0] = sh.v[k];
                HIPCHK(launch_dcshift_mct_fwd(tsrc, fmt, prect[k].w(), tdst, tc.r.w(), tc.r.h(), 1, sk, 0, cp.irrev,
                                              s));
            }
            continue;
        }
        // every component on one grid (no subsampling, or the same dx / dy
        // for all): one launch over the tile, MCT included
        SrcPlanes tsrc{};
        PlanePtrs tdst{};
        for (uint32_t k = 0; k < nc; ++k) {
            tsrc.p[k] = src_at(k, plane_org(k, tile.comps[k]));
            tdst.p[k] = c->work.as<int32_t>() + tile.comps[k].arena_off;
        }
        const Rect &tcr = tile.comps[0].r;
        const uint32_t spw = prect[0].w();
        if (cp.mct == 2) {
            MctMatrix mm{};
            memcpy(mm.c, cp.mct_coding, sizeof(int32_t) * nc * nc);
            HIPCHK(launch_dcshift_mct_custom(tsrc, fmt, spw, tdst, tcr.w(), tcr.h(), nc, sh, mm, s));
        } else {
            HIPCHK(launch_dcshift_mct_fwd(tsrc, fmt, spw, tdst, tcr.w(), tcr.h(), nc, sh, cp.mct, cp.irrev, s));
        }
    }
    HIPCHK(hipEventRecord(c->ev[2], s));
    c->ltimes.clear();
    c->lidx.clear();
    LaunchLog llog{&c->lev, &c->ltimes, &c->lidx};
    HIPCHK(dwt_launch(dplan, c->dwtjobs, cp.irrev, false, s, c->launch_timing ? &llog : nullptr));
    HIPCHK(hipEventRecord(c->ev[3], s));
    memcpy(c->h_blocks.p, eb.data(), (size_t)nblk * sizeof(EncBlock));
    HIPCHK(hipMemcpyAsync(c->blocks.p, c->h_blocks.p, (size_t)nblk * sizeof(EncBlock), hipMemcpyHostToDevice, s));
    memcpy(c->h_symoff.p, symoff.data(), symoff.size() * 8);
    HIPCHK(hipMemcpyAsync(c->symoff.p, c->h_symoff.p, symoff.size() * 8, hipMemcpyHostToDevice, s));
    HIPCHK(launch_t1_encode(c->blocks.as<EncBlock>(), nblk, c->coef.as<int32_t>(), c->scratch.p,
                            c->sym.as<uint8_t>(), c->symoff.as<uint64_t>(), maxdepth, c->mqout.as<uint8_t>(),
                            c->results.as<EncResult>(), s, cp.cblksty, lone_call() ? lone_bpw(nblk) : 0,
                            c->t1order.as<uint32_t>()));
    // per-pass distortion only when some layer is rate-controlled
    // (TileProcessor::needs_rate_control, TileProcessor.cpp:260-266)
    bool need_rc = force_dist != 0;
    for (uint32_t l = 0; l < cp.numlayers; ++l)
        need_rc = need_rc || (cp.disto_alloc && cp.rates[l] > 0.0) || (cp.fixed_quality && cp.distoratio[l] > 0.0f);
    const double *mct_norms = nullptr;
    uint32_t mct_numcomps = 0;
    if (cp.mct == 1) {  // TileProcessor::t1_encode (TileProcessor.cpp:1535-1551), mct.cpp:65-79
        static const double kRev[3] = {1.732, .8292, .8292}, kIrrev[3] = {1.732, 1.805, 1.573};
        mct_norms = cp.irrev ? kIrrev : kRev;
        mct_numcomps = 3;
    } else {  // custom MCT: the inverse's column norms (TileProcessor.cpp:1548-1551); else none
        mct_numcomps = nc;
        if (cp.mct == 2) mct_norms = cp.mct_norms;
    }
    // With rate control the pass records are formed on the device
    // (launch_pass_records): the host fills each block's distortion factor
    // and record slots while the GPU codes, and after the coders only the
    // records and per-block summaries come back.  Without it the host forms
    // them from the coders' results (rates only: no distortion to weigh).
    const bool dev_rec = need_rc && nblk;
    uint64_t ptotal = 0;
    if (dev_rec) {
        HIPCHK(c->h_pinfo.ensure((size_t)nblk * 16 + 8 + 256));
        double *wf = c->h_pinfo.as<double>();
        uint64_t *p0 = (uint64_t *)(wf + nblk);
        for (uint32_t i = 0; i < nblk; ++i) {
            const BlkInfo &bi = binfo[i];
            wf[i] = t1_wmsedec_factor(bi.compno, bi.level, bi.orient, cp.irrev ? 0 : 1, (double)bi.stepsize, mct_norms,
                                      mct_numcomps);
            p0[i] = ptotal;
            ptotal += pcap[i];
        }
        p0[nblk] = ptotal;
        HIPCHK(c->pinfo.ensure((size_t)nblk * 16 + 8 + 256));
        HIPCHK(hipMemcpyAsync(c->pinfo.p, c->h_pinfo.p, (size_t)nblk * 16 + 8, hipMemcpyHostToDevice, s));
    }
    if (need_rc)
        HIPCHK(launch_t1_dist(c->blocks.as<EncBlock>(), nblk, maxdepth, c->coef.as<int32_t>(), c->scratch.p,
                              c->results.as<EncResult>(), s));
    HIPCHK(hipEventRecord(c->ev[4], s));
    if (dev_rec) {
        const size_t sum_bytes = ((size_t)nblk * sizeof(PassSum) + 255) & ~(size_t)255;
        HIPCHK(c->precs.ensure(sum_bytes + ptotal * sizeof(DevPass) + 256));
        HIPCHK(c->h_psum.ensure(sum_bytes + 256));
        HIPCHK(c->h_precs.ensure(ptotal * sizeof(DevPass) + 256));
        PassSum *dsum = c->precs.as<PassSum>();
        DevPass *dpass = (DevPass *)(c->precs.as<uint8_t>() + sum_bytes);
        const double *dwf = c->pinfo.as<double>();
        HIPCHK(launch_pass_records(c->blocks.as<EncBlock>(), c->results.as<EncResult>(), dwf,
                                   (const uint64_t *)(dwf + nblk), nblk, cp.cblksty, dpass, dsum, s));
        HIPCHK(hipMemcpyAsync(c->h_psum.p, dsum, (size_t)nblk * sizeof(PassSum), hipMemcpyDeviceToHost, s));
        if (ptotal)
            HIPCHK(hipMemcpyAsync(c->h_precs.p, dpass, ptotal * sizeof(DevPass), hipMemcpyDeviceToHost, s));
    } else if (nblk) {
        HIPCHK(hipMemcpy2DAsync(c->h_results.p, sizeof(EncResult), c->results.p, sizeof(EncResult),
                                ENC_RESULT_RATE_BYTES, nblk, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    const EncResult *res = c->h_results.as<EncResult>();

    // Tier-2 + headers on the host (j2k_encode :2059, j2k_post_write_tile
    // :2196, T2::encode_packets): only header BITS are produced here; the
    // code-block bytes never visit the host -- a gather kernel assembles the
    // codestream in HBM and one D2H copies it into the pinned output buffer.
    double t_t2 = now_ms();
    const uint32_t L = cp.numlayers;
    std::vector<EncCblkState> cst(nblk);
    std::vector<EncPass> &passes = c->enc_passes;  // host-formed records: [0, npass) filled below
    EncPass *precs = nullptr;                      // the records Tier-2 reads: these, or the device's
    uint64_t npass = 0;
    std::vector<EncLayer> layers((size_t)nblk * L, EncLayer{0, 0, 0, 0.0});
    std::vector<double> blk_disto(nblk, 0.0);
    std::vector<uint32_t> blen(nblk, 0);  // each block's MQ bytes
    uint64_t nsym = 0;
    if (dev_rec) {
        const PassSum *sm = c->h_psum.as<PassSum>();
        const uint64_t *p0 = (const uint64_t *)(c->h_pinfo.as<double>() + nblk);
        for (uint32_t i = 0; i < nblk; ++i) {
            const PassSum &q = sm[i];
            if (q.bad & 1u) return set_err(GRKGPU_EUNSUPPORTED, "code-block numbps exceeds its band's bound");
            if (q.bad & 2u) return set_err(GRKGPU_EUNSUPPORTED, "too many coding passes");
            if (q.bad & 4u) return set_err(GRKGPU_EUNSUPPORTED, "MQ slab overflow");
            nsym += q.nsym;
            EncCblkState &st = cst[i];
            st.numbps = q.numbps;
            st.numpasses = q.numpasses;
            st.pass0 = (uint32_t)p0[i];
            st.dev_off = eb[i].out_off;
            st.smin = q.smin;
            st.smax = q.smax;
            st.s0max = q.s0max;
            st.z0 = q.z0 != 0;
            blk_disto[i] = q.disto;
            blen[i] = q.len;
        }
        if (ptotal > 0xffffffffu) return set_err(GRKGPU_EUNSUPPORTED, "too many coding passes");
        npass = ptotal;
        precs = c->h_precs.as<EncPass>();
    } else {
        // per-block pass records: validate and lay the blocks' passes out (prefix
        // sum), then fill them on the host pool (blocks are independent)
        {
            for (uint32_t i = 0; i < nblk; ++i) {
                const EncResult &r = res[i];
                if (r.pad) return set_err(GRKGPU_EUNSUPPORTED, "code-block numbps exceeds its band's bound");
                if (r.numpasses > GRK_MAX_PASSES) return set_err(GRKGPU_EUNSUPPORTED, "too many coding passes");
                const uint32_t np = r.numpasses;
                if (np && r.rate[np - 1] > eb[i].w * eb[i].h * 4 + 64) return set_err(GRKGPU_EUNSUPPORTED, "MQ slab overflow");
                nsym += r.nsym;
                EncCblkState &st = cst[i];
                st.numbps = r.numbps;
                st.numpasses = np;
                st.pass0 = (uint32_t)npass;
                st.dev_off = eb[i].out_off;
                npass += np;
            }
            if (passes.size() < npass) passes.resize(npass);
        }
        host_parallel_for(nblk, 1024, [&](size_t b0, size_t b1) {
            for (size_t i = b0; i < b1; ++i) {
                const EncResult &r = res[i];
                const uint32_t np = r.numpasses;
                EncPass *out = passes.data() + cst[i].pass0;
                double cum = 0.0;
                const BlkInfo &bi = binfo[i];
                const double wfac = need_rc ? t1_wmsedec_factor(bi.compno, bi.level, bi.orient, cp.irrev ? 0 : 1,
                                                                (double)bi.stepsize, mct_norms, mct_numcomps)
                                            : 0.0;
                for (uint32_t k = 0; k < np; ++k) {
                    EncPass ps;
                    ps.rate = r.rate[k];
                    ps.len = r.rate[k] - (k ? r.rate[k - 1] : 0);
                    // t1_enc_is_term_pass (t1.cpp:1131-1151)
                    {
                        const int32_t bp = k == 0 ? (int32_t)r.numbps - 1 : (int32_t)r.numbps - 2 - (int32_t)((k - 1) / 3);
                        const int pt = k == 0 ? 2 : (int)((k - 1) % 3);
                        ps.term = t1_pass_term(cp.cblksty, bp, pt, r.numbps);
                    }
                    ps.slope = 0;
                    if (need_rc) {  // t1_encode_cblk's cumulative distortion (t1.cpp:1249-1254)
                        const int32_t bpno = k == 0 ? (int32_t)r.numbps - 1 : (int32_t)r.numbps - 2 - (int32_t)((k - 1) / 3);
                        cum += t1_wmsedec_at(wfac, r.nmsedec[k], bpno);
                    }
                    ps.dd = cum;
                    out[k] = ps;
                }
                // the simple PCRD's slope range over this block's passes, from
                // the records just written (pcrd_simple's own loop, TileEnc::slopes)
                block_slopes(cst[i], out);
                blk_disto[i] = cum;
            }
        });
        precs = passes.data();
        for (uint32_t i = 0; i < nblk; ++i) blen[i] = res[i].len;
    }
    const double t_passrec = now_ms() - t_t2;
    if (export_blocks) {
        // the MQ slab to pinned host memory, then one record per block
        HIPCHK(c->h_slab.ensure(out_total + 256));
        if (out_total) HIPCHK(hipMemcpyAsync(c->h_slab.p, c->mqout.p, out_total, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        c->bexp.assign(nblk, grkgpu_block_info{});
        c->bexp_rate.resize((size_t)npass + 1);
        c->bexp_dist.resize((size_t)npass + 1);
        for (size_t k = 0; k < npass; ++k) {
            c->bexp_rate[k] = precs[k].rate;
            c->bexp_dist[k] = precs[k].dd;
        }
        for (uint32_t i = 0; i < nblk; ++i) {
            grkgpu_block_info &o = c->bexp[i];
            const BlkInfo &bi = binfo[i];
            o.tileno = bi.tileno; o.compno = bi.compno; o.resno = bi.resno; o.bandno = bi.orient;
            o.precno = bi.precno; o.cblkno = bi.cblkno;
            o.x0 = bi.r.x0; o.y0 = bi.r.y0; o.x1 = bi.r.x1; o.y1 = bi.r.y1;
            o.numbps = cst[i].numbps;
            o.numpasses = cst[i].numpasses;
            o.len = blen[i];
            o.stepsize = bi.stepsize;
            o.data = c->h_slab.as<uint8_t>() + eb[i].out_off;
            o.rate = c->bexp_rate.data() + cst[i].pass0;
            o.distortion = c->bexp_dist.data() + cst[i].pass0;
        }
        c->bexp_coef.clear();
        for (auto &tile : tiles)
            for (uint32_t k = 0; k < nc; ++k)
                c->bexp_coef.push_back({tile.index, k, tile.comps[k].r.w(), tile.comps[k].r.h(), tile.comps[k].arena_off});
        grkgpu_stats &st0 = c->stats;
        memset(&st0, 0, sizeof(st0));
        hipEventElapsedTime(&st0.h2d_ms, c->ev[0], c->ev[1]);
        hipEventElapsedTime(&st0.dcshift_mct_ms, c->ev[1], c->ev[2]);
        hipEventElapsedTime(&st0.dwt_ms, c->ev[2], c->ev[3]);
        hipEventElapsedTime(&st0.t1_ms, c->ev[3], c->ev[4]);
        log_collect(c);
        st0.num_cblks = nblk;
        st0.mq_symbols = nsym;
        st0.total_ms = (float)(now_ms() - t_start);
        return GRKGPU_OK;
    }
    // tile-parts of every tile (j2k_calculate_tp, j2k.cpp:2990-3048): needed
    // for the TLM marker and the rate bookkeeping even outside the shard
    const uint32_t ntot = cp.tw * cp.th;
    std::vector<std::vector<uint32_t>> tp_counts(ntot);  // [tile][poc entry]
    uint32_t total_tile_parts = 0;
    for (uint32_t t = 0; t < ntot; ++t) {
        Tile tmp;
        const Tile *tp = nullptr;
        if (t >= tb && t < te) tp = &tiles[t - tb];
        else if (cp.tp_on) {
            tmp.index = t;
            tmp.r = tile_rect(cp, t);
            tmp.comps.resize(nc);
            for (uint32_t k = 0; k < nc; ++k) build_tilecomp(tmp.comps[k], tmp.r, cp, k, true);
            tp = &tmp;
        }
        if (tp) tp_counts[t] = tile_part_counts(cp, *tp);
        else tp_counts[t].assign(num_poc_entries(cp), 1);
        uint32_t n = 0;
        for (uint32_t v : tp_counts[t]) n += v;
        if (n > 255) return set_err(GRKGPU_EUNSUPPORTED, "more than 255 tile-parts in a tile");
        total_tile_parts += n;
    }
    ByteBuf hdr;
    hdr.v.reserve(1 << 20);
    std::vector<PlanItem> plan;
    plan.reserve(nblk + 64);
    size_t tlm_at = 0;
    ByteBuf mainhdr;
    write_main_header(mainhdr, cp, &tlm_at, total_tile_parts);
    if (parts & GRKGPU_PART_HEADER) {
        hdr.putn(mainhdr.v.data(), mainhdr.size());
        plan.push_back({0, (uint32_t)hdr.size(), 0});
    }
    // j2k_update_rates (j2k.cpp:2806-2926): layer ratios -> byte budgets per tile
    const double header_size = (double)mainhdr.size();
    const double bits_empty = 8.0 * cp.dx[0] * cp.dy[0], size_pixel = (double)nc * cp.prec[0];
    const uint32_t width = iw, height = ih;
    auto tile_rates = [&](const Rect &tr, uint32_t ntp, double *rates) {
        const double offset = (double)(cp.tp_on ? (float)((ntp - 1) * 14) : 0.0f) / L;
        const uint64_t npix = (uint64_t)tr.w() * tr.h();
        for (uint32_t k = 0; k < L; ++k) {
            rates[k] = cp.rates[k];
            if (rates[k] > 0.0f) rates[k] = (size_pixel * (double)npix) / (rates[k] * bits_empty) - offset;
        }
        rates[L] = 0;
        const double sot_adjust = ((double)npix * header_size) / ((double)width * height);
        double *r = rates;
        if (*r > 0.0) {
            *r -= sot_adjust;
            if (*r < 30.0f) *r = 30.0f;
        }
        ++r;
        const uint32_t last_res = L - 1;
        for (uint32_t k = 1; k < last_res; ++k) {
            if (*r > 0.0) {
                *r -= sot_adjust;
                if (*r < *(r - 1) + 10.0) *r = (*(r - 1)) + 20.0;
            }
            ++r;
        }
        if (*r > 0.0) {
            *r -= (sot_adjust + 2.0);
            if (*r < *(r - 1) + 10.0) *r = (*(r - 1)) + 20.0;
        }
    };
    // tile buffer bound for the rate allocator (j2k_post_write_tile :2196-2222,
    // j2k_get_specific_header_sizes :4346-4366, then SOT / POC / SOD / EOC room)
    const bool cinema = cp.rsiz == RSIZ_CINEMA_2K || cp.rsiz == RSIZ_CINEMA_4K;
    uint64_t tile_bound;
    {
        uint64_t ts = 0;
        for (uint32_t k = 0; k < nc; ++k) ts += (uint64_t)cp.tdx * cp.tdy * cp.prec[k];
        ts = (uint64_t)((double)ts * 0.1625);
        uint32_t max_tp = 0;
        for (auto &v : tp_counts) {
            uint32_t n = 0;
            for (uint32_t x : v) n += x;
            max_tp = std::max(max_tp, n);
        }
        uint64_t spec = 12ull * max_tp;
        if (!cinema) {
            const uint64_t coc = 6 + ((cp.csty & CSTY_PRT) ? 5 + cp.numres : 5);
            spec += (uint64_t)(nc - 1) * coc * 2;
        }
        spec += 4 + 9ull * num_poc_entries(cp);
        ts += spec;
        if (ts < 256ull * nc) ts = 256ull * nc;
        const uint64_t pocsz = (!cinema && cp.numpocs) ? 4 + (5 + 2 * (nc <= 256 ? 1 : 2)) * cp.numpocs : 0;
        tile_bound = ts - 12 - pocsz - 4;
    }
    std::vector<uint8_t> tlm;  // TLM records (j2k_update_tlm, j2k.cpp:6649-6660)
    // Tiles are independent in rate control and Tier-2 (their blocks, layer
    // records and packet state are disjoint): each tile's tile-parts are
    // formed on the host pool into its own header blob and plan, then
    // appended in tile order (header runs rebased onto the shared blob).
    struct TileOut {
        ByteBuf hdr;
        std::vector<PlanItem> plan;
        std::vector<uint8_t> tlm;
        double rate_ms = 0, packet_ms = 0;
        RateStats rs;
        bool ok = true;
    };
    std::vector<TileOut> touts(tiles.size());
    double t_rate = 0;  // summed over tiles (host CPU time of the rate allocation)
    host_parallel_for(tiles.size(), 1, [&](size_t t0, size_t t1) {
        for (size_t ti = t0; ti < t1; ++ti) {
            Tile &tile = tiles[ti];
            TileOut &to = touts[ti];
            TileEnc tenc;
            tenc.tile = &tile;
            tenc.cblk = &cst;
            tenc.passes = precs;
            tenc.layers = &layers;
            tenc.slopes = true;  // the pass-record fill above computed every block's slope range
            init_enc_pocs(cp, tenc);
            CodingParams cpt = cp;
            uint32_t ntp = 0;
            for (uint32_t v : tp_counts[tile.index]) ntp += v;
            tile_rates(tile.r, ntp, cpt.rates);
            tenc.distotile = 0;
            for (auto &tc : tile.comps) for_each_cblk(tc, [&](Band &, Cblk &cb) { tenc.distotile += blk_disto[cb.gidx]; });
            const double tr0 = now_ms();
            if (!rate_allocate(cpt, tenc, tile_bound, &to.rs)) { to.ok = false; continue; }
            const double tp0 = now_ms();
            to.rate_ms = tp0 - tr0;
            // The tile-parts' packets (T2::encode_packets per tile-part,
            // T2.cpp:64-125).  Tile-parts whose packets touch disjoint
            // precincts (tile-parts split by component or resolution, no POC
            // revisiting a precinct: the cinema profiles) are independent --
            // a packet header's state is its precinct's tag trees and its
            // code-blocks' inclusion records -- and are written in parallel,
            // each from its own SOP packet number; the bytes are the same.
            struct TpOut {
                uint32_t pino, tpn, packno0 = 0;
                std::vector<PacketId> order;
                ByteBuf hdr;
                std::vector<PlanItem> plan;
            };
            std::vector<TpOut> tps;
            for (uint32_t pino = 0; pino < tenc.pocs.size(); ++pino)
                for (uint32_t tpn = 0; tpn < tp_counts[tile.index][pino]; ++tpn) {
                    tps.push_back(TpOut{pino, tpn});
                    encode_packet_order(cpt, tenc, pino, tpn, tps.back().order);
                }
            bool disjoint = tps.size() > 1;
            {
                std::vector<int32_t> owner;  // precinct -> tile-part
                std::vector<std::vector<uint32_t>> pb(nc);  // first precinct index of (component, resolution)
                uint32_t np = 0;
                for (uint32_t k = 0; k < nc; ++k) {
                    pb[k].resize(tile.comps[k].numres);
                    for (uint32_t r = 0; r < tile.comps[k].numres; ++r) {
                        pb[k][r] = np;
                        np += tile.comps[k].res[r].pw * tile.comps[k].res[r].ph;
                    }
                }
                owner.assign(np, -1);
                uint32_t packno = 0;
                for (size_t j = 0; j < tps.size() && disjoint; ++j) {
                    tps[j].packno0 = packno;
                    for (auto &pk : tps[j].order) {
                        if (pk.layno >= L) continue;
                        ++packno;
                        int32_t &o = owner[pb[pk.compno][pk.resno] + pk.precno];
                        if (o >= 0 && o != (int32_t)j) { disjoint = false; break; }
                        o = (int32_t)j;
                    }
                }
            }
            auto write_tp = [&](TpOut &t, TileEnc &te) {
                for (auto &pk : t.order)
                    if (pk.layno < L) write_packet(cpt, te, pk, t.hdr, t.plan);
            };
            if (disjoint) {
                host_parallel_for(tps.size(), 1, [&](size_t j0, size_t j1) {
                    for (size_t j = j0; j < j1; ++j) {
                        TileEnc te = tenc;  // shares the tile's state; its own packet counter
                        te.packno = tps[j].packno0;
                        write_tp(tps[j], te);
                    }
                });
            } else {
                for (auto &t : tps) write_tp(t, tenc);
            }
            uint32_t tpno = 0;
            ByteBuf &th = to.hdr;
            for (auto &t : tps) {
                const size_t sot = th.size();
                th.put16(0xFF90); th.put16(10); th.put16(tile.index); th.put32(0); th.put8(tpno); th.put8(ntp);
                if (tpno == 0 && !cinema && cp.numpocs) write_poc(th, cpt);
                th.put16(0xFF93);
                to.plan.push_back({sot, (uint32_t)(th.size() - sot), 0});
                const size_t first = to.plan.size() - 1;
                const uint64_t base = th.size();
                th.putn(t.hdr.v.data(), t.hdr.size());
                for (PlanItem it : t.plan) {
                    if (it.kind == 0) it.src += base;
                    to.plan.push_back(it);
                }
                uint64_t psot = 0;
                for (size_t i = first; i < to.plan.size(); ++i) psot += to.plan[i].len;
                th.set32(sot + 6, (uint32_t)psot);  // Psot (j2k.cpp:2418-2426)
                if (cinema) {
                    to.tlm.push_back((uint8_t)tile.index);
                    for (int b = 3; b >= 0; --b) to.tlm.push_back((uint8_t)(psot >> (8 * b)));
                }
                ++tpno;
            }
            to.packet_ms = now_ms() - tp0;
        }
    });
    double t_packets = 0;
    RateStats rsum;
    for (auto &to : touts) {
        if (!to.ok) return set_err(GRKGPU_EINVAL, "rate allocation failed");
        t_rate += to.rate_ms;
        t_packets += to.packet_ms;
        rsum.probes += to.rs.probes;
        rsum.skipped += to.rs.skipped;
        rsum.evals += to.rs.evals;
        rsum.sims += to.rs.sims;
        rsum.form_ms += to.rs.form_ms;
        rsum.sim_ms += to.rs.sim_ms;
        const uint64_t base = hdr.size();
        hdr.putn(to.hdr.v.data(), to.hdr.size());
        for (PlanItem it : to.plan) {
            if (it.kind == 0) it.src += base;
            plan.push_back(it);
        }
        tlm.insert(tlm.end(), to.tlm.begin(), to.tlm.end());
    }
    if ((parts & GRKGPU_PART_HEADER) && tlm_at && tlm.size() == 5ull * total_tile_parts)
        memcpy(hdr.v.data() + tlm_at, tlm.data(), tlm.size());  // j2k_write_updated_tlm (:2555-2577)
    if (parts & GRKGPU_PART_EOC) {
        size_t eoc = hdr.size();
        hdr.put16(0xFFD9);
        plan.push_back({eoc, 2, 0});
    }
    // gather list: dst offsets = prefix sum of run lengths
    std::vector<GatherItem> gi;
    gi.reserve(plan.size());
    uint64_t total = 0;
    for (auto &pi : plan) {
        if (pi.len) gi.push_back({pi.src, total, pi.len, pi.kind});
        total += pi.len;
    }
    double t_t2_end = now_ms();
    HIPCHK(c->gather.ensure(gi.size() * sizeof(GatherItem) + hdr.size() + 512));
    HIPCHK(c->h_gather.ensure(gi.size() * sizeof(GatherItem) + hdr.size() + 512));
    HIPCHK(c->packed.ensure(total + 256));
    std::unique_lock<std::mutex> out_lk(c->out_mu);
    if (!c->h_out.p && !c->out_spare.empty()) {  // taken by a view: reuse a given-back buffer
        auto big = std::max_element(c->out_spare.begin(), c->out_spare.end(),
                                    [](const auto &a, const auto &b) { return a.second < b.second; });
        c->h_out.p = big->first;
        c->h_out.cap = big->second;
        c->out_spare.erase(big);
    }
    HIPCHK(c->h_out.ensure(total + 256));
    const size_t gbytes = gi.size() * sizeof(GatherItem);
    const size_t hoff = (gbytes + 255) & ~(size_t)255;
    memcpy(c->h_gather.p, gi.data(), gbytes);
    memcpy(c->h_gather.as<uint8_t>() + hoff, hdr.v.data(), hdr.size());
    HIPCHK(hipEventRecord(c->ev[5], s));
    HIPCHK(hipMemcpyAsync(c->gather.p, c->h_gather.p, hoff + hdr.size(), hipMemcpyHostToDevice, s));
    HIPCHK(launch_gather(c->gather.as<uint8_t>() + hoff, c->mqout.as<uint8_t>(), c->gather.as<GatherItem>(),
                         (uint32_t)gi.size(), c->packed.as<uint8_t>(), s));
    HIPCHK(hipEventRecord(c->ev[6], s));
    HIPCHK(hipMemcpyAsync(c->h_out.p, c->packed.p, total, hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(c->ev[7], s));
    HIPCHK(hipStreamSynchronize(s));
    double t_end = now_ms();
    *view = c->h_out.as<uint8_t>();
    *outlen = total;

    grkgpu_stats &st = c->stats;
    memset(&st, 0, sizeof(st));
    hipEventElapsedTime(&st.h2d_ms, c->ev[0], c->ev[1]);
    hipEventElapsedTime(&st.dcshift_mct_ms, c->ev[1], c->ev[2]);
    hipEventElapsedTime(&st.dwt_ms, c->ev[2], c->ev[3]);
    hipEventElapsedTime(&st.t1_ms, c->ev[3], c->ev[4]);
    hipEventElapsedTime(&st.gather_ms, c->ev[5], c->ev[6]);
    hipEventElapsedTime(&st.d2h_ms, c->ev[6], c->ev[7]);
    log_collect(c);
    st.host_t2_ms = (float)(t_t2_end - t_t2);
    st.total_ms = (float)(t_end - t_start);
    st.num_cblks = nblk;
    st.cs_bytes = total;
    st.mq_symbols = nsym;
    st.rate_ms = (float)t_rate;
    st.packet_ms = (float)t_packets;
    st.rate_probes = rsum.probes;
    st.rate_probes_skipped = rsum.skipped;
    st.rate_block_evals = rsum.evals;
    st.rate_precinct_sims = rsum.sims;
    st.rate_form_ms = (float)rsum.form_ms;
    st.rate_sim_ms = (float)rsum.sim_ms;
    st.passrec_ms = (float)t_passrec;
    return GRKGPU_OK;
}

extern "C" int grkgpu_compress_view(grkgpu_ctx *c, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                                    const int32_t *const *planes, int planes_on_device, const uint8_t **out,
                                    size_t *outlen) {
    if (!out || !outlen) return set_err(GRKGPU_EINVAL, "null argument");
    return compress_impl(c, img, p, (const void *const *)planes, planes_on_device, SMP_I32, out, outlen);
}

extern "C" int grkgpu_compress(grkgpu_ctx *c, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                               const int32_t *const *planes, int planes_on_device, uint8_t **out, size_t *outlen) {
    if (!out || !outlen) return set_err(GRKGPU_EINVAL, "null argument");
    const uint8_t *v = nullptr;
    size_t n = 0;
    int rc = compress_impl(c, img, p, (const void *const *)planes, planes_on_device, SMP_I32, &v, &n);
    if (rc) return rc;
    uint8_t *o = (uint8_t *)malloc(n ? n : 1);
    if (!o) return set_err(GRKGPU_EINVAL, "out of host memory");
    memcpy(o, v, n);
    *out = o;
    *outlen = n;
    return GRKGPU_OK;
}

extern "C" int grkgpu_compress_ex(grkgpu_ctx *c, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                                  const grkgpu_planes *in, uint32_t tile_begin, uint32_t tile_end, uint32_t parts,
                                  const uint8_t **out, size_t *outlen) {
    if (!in || !out || !outlen) return set_err(GRKGPU_EINVAL, "null argument");
    if (in->nrows == 0 && in->row0) return set_err(GRKGPU_EINVAL, "row0 without nrows");
    if (in->ncols == 0 && in->col0) return set_err(GRKGPU_EINVAL, "col0 without ncols");
    return compress_impl(c, img, p, in->planes, in->on_device, (int32_t)in->sample_fmt, out, outlen, tile_begin,
                         tile_end, parts, false, 0, in->row0, in->nrows, in->col0, in->ncols);
}

extern "C" int grkgpu_encode_blocks(grkgpu_ctx *c, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                                    const int32_t *const *planes, int planes_on_device, int with_distortion,
                                    const grkgpu_block_info **blocks, uint32_t *nblocks) {
    if (!blocks || !nblocks) return set_err(GRKGPU_EINVAL, "null argument");
    int rc = compress_impl(c, img, p, (const void *const *)planes, planes_on_device, SMP_I32, nullptr, nullptr, 0,
                           0xffffffffu, GRKGPU_PART_ALL, true, with_distortion);
    if (rc) return rc;
    *blocks = c->bexp.data();
    *nblocks = (uint32_t)c->bexp.size();
    return GRKGPU_OK;
}

extern "C" int grkgpu_encode_blocks_coefficients(grkgpu_ctx *c, uint32_t tileno, uint32_t compno, int32_t *dst,
                                                  uint32_t dst_stride) {
    if (!c || !dst) return set_err(GRKGPU_EINVAL, "null argument");
    for (const auto &r : c->bexp_coef) {
        if (r.tileno != tileno || r.compno != compno) continue;
        if (dst_stride < r.w) return set_err(GRKGPU_EINVAL, "dst_stride below the tile-component width");
        HIPCHK(hipSetDevice(c->device));
        HIPCHK(hipMemcpy2DAsync(dst, (size_t)dst_stride * 4, c->coef.as<int32_t>() + r.off, (size_t)r.w * 4,
                                (size_t)r.w * 4, r.h, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        return GRKGPU_OK;
    }
    return set_err(GRKGPU_EINVAL, "no such tile-component in the last grkgpu_encode_blocks call");
}

extern "C" int grkgpu_num_tiles(const grkgpu_image_desc *img, const grkgpu_cparams *p, uint32_t *ntiles) {
    if (!ntiles) return set_err(GRKGPU_EINVAL, "null argument");
    CodingParams cp;
    int rc = setup_params(img, p, cp);
    if (rc) return rc;
    *ntiles = cp.tw * cp.th;
    return GRKGPU_OK;
}

extern "C" int grkgpu_compress_tiles(grkgpu_ctx *c, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                                     const int32_t *const *planes, int planes_on_device, uint32_t tile_begin,
                                     uint32_t tile_end, uint32_t parts, uint8_t **out, size_t *outlen) {
    if (!out || !outlen) return set_err(GRKGPU_EINVAL, "null argument");
    const uint8_t *v = nullptr;
    size_t n = 0;
    int rc = compress_impl(c, img, p, (const void *const *)planes, planes_on_device, SMP_I32, &v, &n, tile_begin,
                           tile_end, parts);
    if (rc) return rc;
    uint8_t *o = (uint8_t *)malloc(n ? n : 1);
    if (!o) return set_err(GRKGPU_EINVAL, "out of host memory");
    memcpy(o, v, n);
    *out = o;
    *outlen = n;
    return GRKGPU_OK;
}

extern "C" int grkgpu_compress_tile_rows(grkgpu_ctx *c, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                                         const int32_t *const *planes, int planes_on_device, uint32_t row0,
                                         uint32_t nrows, uint32_t tile_begin, uint32_t tile_end, uint32_t parts,
                                         uint8_t **out, size_t *outlen) {
    if (!out || !outlen) return set_err(GRKGPU_EINVAL, "null argument");
    if (nrows == 0) return set_err(GRKGPU_EINVAL, "nrows must be > 0");
    const uint8_t *v = nullptr;
    size_t n = 0;
    int rc = compress_impl(c, img, p, (const void *const *)planes, planes_on_device, SMP_I32, &v, &n, tile_begin,
                           tile_end, parts, false, 0, row0, nrows);
    if (rc) return rc;
    uint8_t *o = (uint8_t *)malloc(n ? n : 1);
    if (!o) return set_err(GRKGPU_EINVAL, "out of host memory");
    memcpy(o, v, n);
    *out = o;
    *outlen = n;
    return GRKGPU_OK;
}

// ---------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------
extern "C" int grkgpu_read_header(const uint8_t *cs, size_t len, grkgpu_image_desc *img) {
    if (!cs || !img) return set_err(GRKGPU_EINVAL, "null argument");
    CodingParams cp;
    size_t sot = 0;
    std::string err;
    if (!parse_main_header(cs, len, cp, sot, err)) return set_err(GRKGPU_EUNSUPPORTED, err);
    memset(img, 0, sizeof(*img));
    img->x0 = cp.image.x0; img->y0 = cp.image.y0; img->x1 = cp.image.x1; img->y1 = cp.image.y1;
    img->numcomps = cp.numcomps;
    for (uint32_t k = 0; k < cp.numcomps; ++k) {
        img->prec[k] = cp.prec[k];
        img->sgnd[k] = cp.sgnd[k];
        img->dx[k] = cp.dx[k];
        img->dy[k] = cp.dy[k];
    }
    return GRKGPU_OK;
}

extern "C" int grkgpu_read_header_info(const uint8_t *cs, size_t len, grkgpu_header_info *hi) {
    if (!cs || !hi) return set_err(GRKGPU_EINVAL, "null argument");
    CodingParams cp;
    size_t sot = 0;
    std::string err;
    if (!parse_main_header(cs, len, cp, sot, err)) return set_err(GRKGPU_EUNSUPPORTED, err);
    memset(hi, 0, sizeof(*hi));
    // the code-block / wavelet / precinct fields are component 0's (j2k.cpp:
    // 445-467 reads tcp->tccps[0]: a main COC for component 0 shows here)
    const CompParams &c0 = cp.comp[0];
    hi->cblockw_init = 1u << c0.cblkw;
    hi->cblockh_init = 1u << c0.cblkh;
    hi->irreversible = (uint32_t)c0.irrev;
    hi->mct = (uint32_t)cp.mct;
    hi->rsiz = cp.rsiz;
    hi->numresolutions = c0.numres;
    hi->csty = cp.csty;
    hi->cblk_sty = c0.cblksty;
    for (uint32_t r = 0; r < 33; ++r) {
        hi->prcw_init[r] = 1u << c0.prcw[r];
        hi->prch_init[r] = 1u << c0.prch[r];
    }
    hi->tx0 = cp.tx0; hi->ty0 = cp.ty0; hi->tdx = cp.tdx; hi->tdy = cp.tdy; hi->tw = cp.tw; hi->th = cp.th;
    hi->numlayers = cp.numlayers;
    hi->prog = cp.prog;
    hi->numcomps = cp.numcomps;
    hi->numgbits = cp.numgbits;
    hi->qntsty = cp.qntsty;
    hi->nsteps = std::min<uint32_t>(cp.nsteps, 97);
    for (uint32_t b = 0; b < hi->nsteps; ++b) { hi->step_expn[b] = cp.ss[b].expn; hi->step_mant[b] = cp.ss[b].mant; }
    for (uint32_t k = 0; k < cp.numcomps && k < 16; ++k) hi->roishift[k] = cp.roishift[k];
    return GRKGPU_OK;
}

extern "C" int grkgpu_read_comp_info(const uint8_t *cs, size_t len, uint32_t compno, grkgpu_comp_info *ci) {
    if (!cs || !ci) return set_err(GRKGPU_EINVAL, "null argument");
    CodingParams cp;
    size_t sot = 0;
    std::string err;
    if (!parse_main_header(cs, len, cp, sot, err)) return set_err(GRKGPU_EUNSUPPORTED, err);
    if (compno >= cp.numcomps) return set_err(GRKGPU_EINVAL, "component index out of range");
    const CompParams &c = cp.comp[compno];
    memset(ci, 0, sizeof(*ci));
    ci->csty = c.csty;
    ci->numresolutions = c.numres;
    ci->cblkw = c.cblkw;
    ci->cblkh = c.cblkh;
    ci->cblk_sty = c.cblksty;
    ci->qmfbid = c.irrev ? 0 : 1;
    for (uint32_t r = 0; r < 33; ++r) { ci->prcw[r] = c.prcw[r]; ci->prch[r] = c.prch[r]; }
    ci->qntsty = c.qntsty;
    ci->numgbits = c.numgbits;
    ci->nsteps = std::min<uint32_t>(c.nsteps, 100);
    for (uint32_t b = 0; b < ci->nsteps; ++b) { ci->step_expn[b] = c.ss[b].expn; ci->step_mant[b] = c.ss[b].mant; }
    ci->roishift = cp.roishift[compno];
    return GRKGPU_OK;
}

static uint32_t rd16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t rd32(const uint8_t *p) { return (rd16(p) << 16) | rd16(p + 2); }

static uint32_t ceil_pow2(uint32_t v, uint32_t r) { return (uint32_t)(((uint64_t)v + ((1ull << r) - 1)) >> r); }


// ---------------------------------------------------------------------------
// The reference decoder's walk over the tile-parts, restated over a memory
// stream (j2k_decode_tiles, j2k.cpp:1136-1224; j2k_read_tile_header :627-978
// with j2k_read_sot :5138-5260 and j2k_read_sod :5399-5480; the marker read
// after a decoded tile in j2k_decode_tile :979-1120; the look-ahead of
// j2k_need_nb_tile_parts_correction :534-625; BufferedStream / mem_stream
// reads and seeks, util/BufferedStream.cpp, util/mem_stream.cpp).  It decides
// which tiles a decode produces, from which of their tile-parts, and which
// short or damaged streams fail:
//   * tiles are decoded as their last tile-part (TNsot) is read; a stream
//     that ends -- or reaches EOC -- before a tile is complete still decodes
//     a tile whose data has begun, from the tile-parts read;
//   * a tile the walk never reaches is not decoded: its samples stay zero
//     (the multi-tile output image is cleared first, j2k.cpp:1148-1156);
//   * a stream ending inside a tile-part header, between a tile-part and the
//     next one of the same tile, or right after an SOD (a tile with no data)
//     fails, as do headers the reference refuses (tile-part index order,
//     Psot, markers outside their place, an unknown marker);
//   * the once-per-decode look-ahead over the following SOT headers fails on
//     an SOT cut inside its 10 header bytes, wherever the walk itself stops.
// A tile-part's data length is Psot less its header, clamped to the stream
// (Psot = 0: up to the last 2 bytes); skipped tiles (outside a decode
// window) step over their tile-parts, which a memory stream does past its
// end without failing -- the next read fails instead.
// ---------------------------------------------------------------------------
struct TpMarker { uint32_t m; size_t off; uint32_t len; };
struct TileWalk {
    std::vector<std::vector<std::pair<size_t, size_t>>> parts;  // per tile: data of the tile-parts read
    std::vector<std::vector<TpMarker>> marks;                  // per tile: its tile-part header markers
    std::vector<std::vector<uint32_t>> seq;                    // per tile: codestream index of each tile-part
    std::vector<uint8_t> decoded;                              // per tile: decoded by the walk
    uint32_t ntp = 0;
};

static bool tph_marker(uint32_t m) {  // allowed in a tile-part header (j2k.cpp:87-106, J2K_DEC_STATE_TPH)
    switch (m) {
        case 0xFF52: case 0xFF53: case 0xFF5E: case 0xFF5C: case 0xFF5D: case 0xFF5F: case 0xFF58: case 0xFF61:
        case 0xFF64: case 0xFF74: case 0xFF75: case 0xFF77: return true;
        default: return false;
    }
}

// j2k_need_nb_tile_parts_correction from position q (after tile `tile`'s
// last tile-part): false = the decode fails; *fix = a later SOT of the same
// tile has TPsot == TNsot (the non-conformant streams the reference patches:
// walk_tile_parts then raises every tile-part count by one, as j2k.cpp:809-835)
static bool tp_lookahead(const uint8_t *cs, size_t len, uint64_t q, uint32_t tile, bool *fix, std::string &err) {
    *fix = false;
    for (;;) {
        if (q > len || len - q < 2) return true;  // no further marker: assumed fine
        const uint32_t m = rd16(cs + q);
        q += 2;
        if (m != 0xFF90) return true;
        if (len - q < 2) { err = "Stream too short"; return false; }
        if (rd16(cs + q) != 10) { err = "Inconsistent marker size"; return false; }
        q += 2;
        if (len - q < 8) { err = "Stream too short"; return false; }
        const uint32_t t = rd16(cs + q), tot = rd32(cs + q + 2), part = cs[q + 6], nparts = cs[q + 7];
        q += 8;
        if (t == tile) { *fix = part == nparts; return true; }
        if (tot < 14) return true;  // 0: the last tile-part; < 14: invalid -- assumed fine
        q += tot - 12;              // a seek past the end succeeds; the next read fails
    }
}

// skip[t]: tile t lies outside the decode window (m_skip_data, j2k.cpp:5262-5274)
static bool walk_tile_parts(const uint8_t *cs, size_t len, size_t sot0, uint32_t ntiles, const std::vector<uint8_t> &skip,
                            TileWalk &w, std::string &err) {
    enum : uint32_t { TPHSOT = 0x08, TPH = 0x10, NEOC = 0x40, EOC = 0x100 };
    w.parts.assign(ntiles, {});
    w.marks.assign(ntiles, {});
    w.seq.assign(ntiles, {});
    w.decoded.assign(ntiles, 0);
    w.ntp = 0;
    std::vector<int32_t> cur_tp(ntiles, -1);
    std::vector<uint32_t> nb_tp(ntiles, 0);
    std::vector<uint8_t> has_data(ntiles, 0);
    uint64_t p = sot0 + 2;  // the first SOT's code was read with the main header
    // bytes left; past the end (after a seek) the stream's unsigned count is huge
    auto left = [&]() -> uint64_t { return p <= len ? len - p : ~0ull; };
    auto read = [&](uint64_t n, uint64_t *at) -> bool {  // a short read takes what is left
        *at = p;
        if (p <= len && n <= len - p) { p += n; return true; }
        if (p < len) p = len;
        return false;
    };
    uint32_t state = TPHSOT, tcur = 0, tpl = 0, ndec = 0;
    uint32_t corr = 0;  // m_nb_tile_parts_correction: 1 once a TPsot == TNsot stream was detected
    bool ready = false, last_tp = false, checked = false, skipping = false;
    uint64_t at;
    for (uint32_t nr = 0; nr < ntiles; ++nr) {
        uint32_t marker = 0xFF90;
        if (state == EOC) marker = 0xFFD9;
        else if (state != TPHSOT) { err = "Stream too short"; return false; }
        while (!ready && marker != 0xFFD9) {
            while (marker != 0xFF93) {
                if (left() == 0) { state = NEOC; break; }
                if (!read(2, &at)) { err = "Stream too short"; return false; }
                uint32_t ms = rd16(cs + at);
                if (ms < 2) { err = "Inconsistent marker size"; return false; }
                if (state & TPH) tpl -= ms + 2;
                ms -= 2;
                const bool sot = marker == 0xFF90;
                if (sot ? !(state & TPHSOT) : (!(state & TPH) || !tph_marker(marker))) {
                    err = "Marker is not compliant with its position";
                    return false;
                }
                if (!read(ms, &at)) { err = "Stream too short"; return false; }
                if (sot) {  // j2k_read_sot
                    if (ms != 8) { err = "Error reading SOT marker"; return false; }
                    const uint32_t t = rd16(cs + at), psot = rd32(cs + at + 2), part = cs[at + 6], nparts = cs[at + 7];
                    if (t >= ntiles) { err = "Invalid tile number"; return false; }
                    tcur = t;
                    if (cur_tp[t] + 1 != (int32_t)part) { err = "Invalid tile part index"; return false; }
                    ++cur_tp[t];
                    if (psot && psot < 14 && psot != 12) { err = "Psot value is not correct"; return false; }
                    if (!psot) last_tp = true;
                    if (nb_tp[t] && part >= nb_tp[t]) { err = "Current tile part number greater than the tile-parts"; return false; }
                    if (nparts) {  // j2k.cpp:5210-5236: TNsot + the correction, as a byte
                        const uint32_t np = (nparts + corr) & 0xFF;
                        if (part >= np) { err = "In SOT marker, TPSot is not valid"; return false; }
                        nb_tp[t] = np;
                    }
                    if (nb_tp[t] && nb_tp[t] == part + 1) ready = true;
                    tpl = last_tp ? 0u : psot - 12;
                    state = TPH;
                    skipping = skip[t] != 0;
                    w.seq[t].push_back(w.ntp++);
                } else if (marker == 0xFF52 || marker == 0xFF5C || marker == 0xFF53 || marker == 0xFF5D ||
                           marker == 0xFF5E || marker == 0xFF5F || marker == 0xFF61) {
                    w.marks[tcur].push_back({marker, (size_t)at, ms});
                }
                if (skipping) {  // the rest of the tile-part stepped over
                    p += tpl;
                    marker = 0xFF93;
                } else {
                    if (!read(2, &at)) { err = "Stream too short"; return false; }
                    marker = rd16(cs + at);
                }
            }
            if (left() == 0 && state == NEOC) break;
            if (!skipping) {  // j2k_read_sod
                if (last_tp) tpl = (uint32_t)(left() - 2);
                else if (tpl >= 2) tpl -= 2;
                if (tpl && tpl > left()) tpl = (uint32_t)left();
                if (tpl) {
                    w.parts[tcur].push_back({(size_t)p, tpl});
                    has_data[tcur] = 1;
                    p += tpl;
                }
                state = TPHSOT;
                if (ready && !checked) {
                    checked = true;
                    bool fix = false;
                    if (!tp_lookahead(cs, len, p, tcur, &fix, err)) return false;
                    if (fix) {  // Issue 254 (j2k.cpp:809-835): every known tile-part count + 1, later TNsot + 1
                        ready = false;
                        corr = 1;
                        for (auto &n : nb_tp)
                            if (n) n = (n + 1) & 0xFF;
                    }
                }
                if (!ready) {
                    if (!read(2, &at)) { err = "Stream too short"; return false; }
                    marker = rd16(cs + at);
                }
            } else {
                skipping = false;
                ready = false;
                state = TPHSOT;
                if (!read(2, &at)) { err = "Stream too short"; return false; }
                marker = rd16(cs + at);
            }
        }
        if (marker == 0xFFD9 && state != EOC) { state = EOC; tcur = 0; }
        if (!ready) {  // the stream ended or reached EOC: the next tile holding data, if any
            while (tcur < ntiles && !has_data[tcur]) ++tcur;
            if (tcur == ntiles) break;
        }
        // j2k_decode_tile
        if (!has_data[tcur]) { err = "Failed to decode tile (no tile data)"; return false; }
        w.decoded[tcur] = 1;
        has_data[tcur] = 0;
        ready = false;
        ++ndec;
        if (left() == 0 && state == NEOC) break;
        if (state != EOC && read(2, &at)) {  // the marker after the tile: EOC, SOT, or the end
            const uint32_t m = rd16(cs + at);
            if (m == 0xFFD9) { tcur = 0; state = EOC; }
            else if (m != 0xFF90) {
                if (left() == 0) state = NEOC;
                else if (nr + 1 < ntiles) { err = "Stream too short, expected SOT"; return false; }
            }
        }
        if (left() == 0 && state == NEOC) break;
    }
    if (!ndec) { err = "No tiles were decoded"; return false; }
    return true;
}

// reduce > 0 (whole-image decode only): the image at resolution
// numres - 1 - reduce (grk_decompress -r, cp_reduce, grok.h:698-702): every
// packet is still parsed, code-blocks of the dropped resolutions are not
// decoded, the inverse DWT stops `reduce` levels early (TileProcessor.cpp:1165,
// TileComponent.cpp:199-204) and MCT + DC shift run on the reduced tiles; the
// image is ceil(coordinate / 2^reduce) (j2k.cpp:1464-1476).
//
// win (image coordinates; whole-image decode only): the window decode of
// grk_set_decode_area (grok.h:1587, j2k.cpp j2k_set_decode_area): only tiles
// meeting the window are parsed, only code-blocks whose coefficients reach it
// are decoded (window_need), the inverse DWT runs on those tiles and MCT +
// DC shift on the window; the output planes are the window.
//
// max_layers > 0: only the first max_layers quality layers are decoded
// (grk_decompress -l, cp_layer, grok.h:703-709; tcp->num_layers_to_decode,
// j2k.cpp:3861-3865): the packets of later layers are parsed and stepped over
// and their passes still count toward the block's pass total
// (T2::skip_packet_data, T2.cpp:758-819), so T1 runs those passes over the
// 0xFF fill past the decoded bytes, exactly as the reference does.
// host_only: stop after the host Tier-2 (tile-part walk, packet headers, the
// code-block table) -- no device call; *decoded_out (when given) receives the
// tiles decoded (grkgpu_walk_tiles)
static int decompress_impl(grkgpu_ctx *c, const uint8_t *csb, size_t len, grkgpu_image_desc *img,
                           int32_t *const *planes, int planes_on_device, uint32_t tb, uint32_t te,
                           uint32_t reduce = 0, const Rect *win = nullptr, uint32_t max_layers = 0,
                           bool host_only = false, std::vector<uint8_t> *decoded_out = nullptr) {
    if ((!c && !host_only) || !csb || (!planes && !host_only)) return set_err(GRKGPU_EINVAL, "null argument");
    ActiveCall active;
    double t_start = now_ms();
    CodingParams cp;
    size_t pos = 0;
    std::string err;
    if (!parse_main_header(csb, len, cp, pos, err)) return set_err(GRKGPU_EUNSUPPORTED, err);
    if (img) {
        int rc = grkgpu_read_header(csb, len, img);
        if (rc) return rc;
    }
    if (reduce >= cp.numres)  // j2k.cpp:6994
        return set_err(GRKGPU_EINVAL, "reduce must be smaller than the number of resolutions");
    Rect wr{};  // window, clipped to the image
    if (win) {
        wr = intersect(*win, cp.image);
        if (wr.empty()) return set_err(GRKGPU_EINVAL, "decode window outside the image");
    }
    // output image geometry: the image or the window (reference grid), at the
    // decoded resolution ceil(x / 2^reduce) (j2k_set_decode_area, j2k.cpp:1464-1476)
    const Rect full = win ? wr : cp.image;
    const uint32_t ix0 = ceil_pow2(full.x0, reduce), iy0 = ceil_pow2(full.y0, reduce);
    const uint32_t ix1 = ceil_pow2(full.x1, reduce), iy1 = ceil_pow2(full.y1, reduce);
    if (win && (ix1 <= ix0 || iy1 <= iy0)) return set_err(GRKGPU_EINVAL, "decode window empty at this resolution");
    // Without a window the planes take grk_image_comp_header_update's sizes,
    // ceil(size / 2^reduce) (image.cpp:124-155), while the tiles land from
    // ceil(x0 / 2^reduce) (TileProcessor.cpp:1729-1734): with an odd origin
    // that is one row / column more than the decoded samples, left zero.
    // A window takes update_image_dimensions' (image.cpp:207-246) exact extent.
    const uint32_t ox1 = win ? ix1 : ix0 + ceil_pow2(full.w(), reduce);
    const uint32_t oy1 = win ? iy1 : iy0 + ceil_pow2(full.h(), reduce);
    if (img && (reduce || win)) {
        img->x0 = ix0; img->y0 = iy0;
        img->x1 = ox1; img->y1 = oy1;
    }
    const uint32_t nc = cp.numcomps, ntiles = cp.tw * cp.th;
    const uint32_t iw = ox1 - ix0;
    if (te > ntiles) te = ntiles;
    if (tb > te) return set_err(GRKGPU_EINVAL, "bad tile range");
    const bool whole = tb == 0 && te == ntiles;
    if (reduce && !whole) return set_err(GRKGPU_EINVAL, "reduced decode of a tile range is not supported");
    // subsampled components: component k's output plane is the output
    // rectangle on its grid (ceil(x / dx), the nested ceilings of a reduced
    // decode commute), rows of its own width
    bool subs = false, mixed = false;  // mixed: components on different grids
    for (uint32_t k = 0; k < nc; ++k) {
        subs = subs || cp.dx[k] != 1 || cp.dy[k] != 1;
        mixed = mixed || cp.dx[k] != cp.dx[0] || cp.dy[k] != cp.dy[0];
    }
    if (subs && !whole) return set_err(GRKGPU_EUNSUPPORTED, "tile-range decode of subsampled images is not supported");
    Rect orect[GRKGPU_MAX_COMPS];
    uint64_t ooff[GRKGPU_MAX_COMPS + 1];
    ooff[0] = 0;
    bool opad = false;  // planes extending past the decoded samples (zero filled)
    for (uint32_t k = 0; k < nc; ++k) {
        orect[k] = comp_rect({ix0, iy0, ix1, iy1}, cp.dx[k], cp.dy[k]);
        if (!win) {  // ceil(ceil(size on the component grid) / 2^reduce)
            const Rect cr = comp_rect(cp.image, cp.dx[k], cp.dy[k]);
            const Rect sized{orect[k].x0, orect[k].y0, orect[k].x0 + ceil_pow2(cr.w(), reduce),
                             orect[k].y0 + ceil_pow2(cr.h(), reduce)};
            opad = opad || sized.x1 != orect[k].x1 || sized.y1 != orect[k].y1;
            orect[k] = sized;
        }
        ooff[k + 1] = ooff[k] + (uint64_t)orect[k].w() * orect[k].h();
    }
    // the window on each component's grid at the decoded resolution
    Rect cwin[GRKGPU_MAX_COMPS];
    for (uint32_t k = 0; k < nc; ++k) cwin[k] = comp_rect({ix0, iy0, ix1, iy1}, cp.dx[k], cp.dy[k]);

    // tile-parts: the reference's walk (walk_tile_parts) -- which tiles are
    // decoded, from which tile-parts, and where a short stream fails; the
    // coding-parameter markers of the tile-part headers (COD / COC / QCD / QCC
    // / RGN / POC / PPT, j2k.cpp:3829-4990) are applied to the tile's own copy
    // of the parameters below
    std::vector<uint8_t> wskip(ntiles, 0);
    if (win)
        for (uint32_t t = 0; t < ntiles; ++t)
            wskip[t] = !overlap(comp_rect(tile_rect(cp, t), 1u << reduce, 1u << reduce), {ix0, iy0, ix1, iy1});
    TileWalk walk;
    if (!walk_tile_parts(csb, len, pos, ntiles, wskip, walk, err)) return set_err(GRKGPU_ECORRUPT, err);
    const auto &tparts = walk.parts;
    const auto &tmarks = walk.marks;
    const auto &tpseq = walk.seq;
    bool missing = false;  // tiles the walk did not decode: zero in the output
    for (uint32_t t = tb; t < te; ++t) missing = missing || (!walk.decoded[t] && !wskip[t]);
    // PPM (j2k_merge_ppm, j2k.cpp:4766-4900): the main header's packed packet
    // headers, Zppm order, as Nppm / Ippm pairs -- the i-th pair holds the
    // headers of the codestream's i-th tile-part
    std::vector<uint8_t> ppm_buf;
    std::vector<std::pair<size_t, size_t>> ppm_chunk;  // (offset in ppm_buf, Nppm)
    if (!cp.ppm.empty()) {
        std::vector<uint8_t> raw;
        for (auto &q : cp.ppm) raw.insert(raw.end(), csb + q.off, csb + q.off + q.len);
        size_t o = 0;
        while (o < raw.size()) {
            if (o + 4 > raw.size()) return set_err(GRKGPU_ECORRUPT, "Not enough bytes to read Nppm");
            const uint32_t nppm = rd32(raw.data() + o);
            o += 4;
            if (o + nppm > raw.size()) return set_err(GRKGPU_ECORRUPT, "Corrupted PPM markers");
            ppm_chunk.push_back({ppm_buf.size(), nppm});
            ppm_buf.insert(ppm_buf.end(), raw.begin() + o, raw.begin() + o + nppm);
            o += nppm;
        }
    }

    // host Tier-2 over every tile of the shard; code-block segments -> DecBlock table
    const uint32_t nsh = te - tb;
    std::vector<Tile> tiles(nsh);
    uint64_t arena = 0, llarena = 0;
    std::vector<uint64_t> lloff(nsh * nc);
    std::vector<DecBlock> db;
    std::vector<DecSeg> dsegs;        // codeword segments of all blocks
    std::vector<uint8_t> droi;        // per-block ROI shift (empty: no ROI)
    std::vector<uint8_t> dsty;        // per-block code-block style (COD / COC of its tile-component)
    std::vector<uint32_t> seg_first;  // per block: first segment (+ the total at the end)
    std::vector<uint8_t> extra;  // concatenated multi-chunk segments
    bool too_deep = false;
    // Packet headers of the tiles, parsed in parallel on the host pool (each
    // tile's geometry, tag trees and code-block segments are its own); then
    // the arenas and the DecBlock table in tile order.
    std::vector<std::vector<uint8_t>> tbufs(nsh);  // tiles of several tile-parts: their data concatenated
    std::vector<std::vector<uint8_t>> tpacked(nsh);  // packed packet headers (PPM / PPT) of each tile
    std::vector<uint8_t> tpacked_on(nsh, 0);
    std::vector<size_t> ppm_from(nsh, 0);  // PPM: where each tile's packet headers start in ppm_buf
    std::vector<uint8_t> contig(nsh, 1);
    // 1: bad POC marker, 2: corrupt packet header, 3: bad tile-part COD / COC
    // / QCD / QCC / RGN / PPT, 4: tile-component parameters this decoder does
    // not take (code-block style, wavelet or MCT other than the main header's,
    // reduce >= its resolutions)
    std::vector<int> terr(nsh, 0);
    std::vector<std::array<uint8_t, 16>> troi(nsh);  // per tile: ROI shift of each component
    std::vector<std::array<uint8_t, 16>> tsty(nsh);  // per tile: code-block style of each component
    std::vector<int32_t> tmct(nsh, cp.mct);            // per tile: MCT (a tile COD may change it)
    host_parallel_for(nsh, 1, [&](size_t l0, size_t l1) {
        for (size_t lt = l0; lt < l1; ++lt) {
            const uint32_t t = tb + (uint32_t)lt;
            Tile &tile = tiles[lt];
            tile.index = t;
            tile.r = tile_rect(cp, t);
            for (uint32_t k = 0; k < 16; ++k) troi[lt][k] = cp.roishift[k];
            if (win && !overlap(comp_rect(tile.r, 1u << reduce, 1u << reduce), {ix0, iy0, ix1, iy1}))
                continue;  // left without components: skipped below
            if (!walk.decoded[t]) continue;  // never reached: its samples stay zero
            // the tile's coding parameters: the main header's, then its
            // tile-part headers' markers (precedence tile COC > tile COD >
            // main COC > main COD; QCC / QCD alike); POC entries appended
            CodingParams tcp = cp;
            {
                bool tcod = false, tqcd = false, tcoc[16] = {}, tqcc[16] = {}, ok = true;
                std::string e;
                std::vector<PpxSeg> ppt;
                for (const TpMarker &mk : tmarks[t]) {
                    const uint8_t *mp = csb + mk.off;
                    if (mk.m == 0xFF52) {  // sets every component, a COC before it included
                        ok = parse_cod(mp, mk.len, tcp, e);
                        tcod = true;
                        for (uint32_t k = 0; k < 16; ++k) tcoc[k] = false;
                    }
                    else if (mk.m == 0xFF5C) { ok = parse_qcd(mp, mk.len, tcp, e); tqcd = true; }
                    else if (mk.m == 0xFF53) { const int32_t k = parse_coc(mp, mk.len, tcp, e); ok = k >= 0; if (ok) tcoc[k] = true; }
                    else if (mk.m == 0xFF5D) { const int32_t k = parse_qcc(mp, mk.len, tcp, e); ok = k >= 0; if (ok) tqcc[k] = true; }
                    else if (mk.m == 0xFF5E) {  // RGN (j2k_read_rgn, j2k.cpp:5555-5604)
                        const uint32_t room = nc <= 256 ? 1 : 2;
                        const uint32_t k = room == 2 ? rd16(mp) : mp[0];
                        ok = mk.len == 2 + room && k < nc;
                        if (ok) tcp.roishift[k] = mp[room + 1];
                    } else if (mk.m == 0xFF5F) {
                        if (!parse_poc(mp, mk.len, tcp)) { terr[lt] = 1; break; }
                    } else if (mk.m == 0xFF61) {  // PPT (j2k_read_ppt, j2k.cpp:4901-4978): Zppt, Ippt
                        ok = mk.len >= 1;
                        if (ok) ppt.push_back({mp[0], mk.off + 1, (size_t)mk.len - 1});
                    }
                    if (!ok) break;
                }
                if (terr[lt]) continue;
                if (!ok) { terr[lt] = 3; continue; }
                for (uint32_t k = 0; k < 16; ++k) {
                    if (tcod && !tcoc[k]) comp_style_from_cod(tcp, k);
                    if (tqcd && !tqcc[k]) comp_quant_from_qcd(tcp, k);
                }
                if (!check_qcd_steps(tcp, cp.qcc_set, tqcd, tqcc, e)) { terr[lt] = 5; continue; }
                for (uint32_t k = 0; k < nc; ++k) {
                    const CompParams &cc = tcp.comp[k];
                    if ((cc.cblksty & ~0x3Fu) || reduce >= cc.numres || cc.cblkw > 6 || cc.cblkh > 6) ok = false;
                    troi[lt][k] = tcp.roishift[k];
                    tsty[lt][k] = (uint8_t)cc.cblksty;
                }
                // MCT over components of different wavelets (the reference
                // picks the transform by component 0's alone) or sizes
                if (tcp.mct && nc >= 3 && (tcp.comp[1].irrev != tcp.comp[0].irrev ||
                                           tcp.comp[2].irrev != tcp.comp[0].irrev || cp.dx[1] != cp.dx[0] ||
                                           cp.dx[2] != cp.dx[0] || cp.dy[1] != cp.dy[0] || cp.dy[2] != cp.dy[0]))
                    ok = false;
                tmct[lt] = tcp.mct;
                if (!ok) { terr[lt] = 4; continue; }
                // the tile's packed packet headers: its PPT segments in Zppt
                // order (j2k_merge_ppt), or its tile-parts' PPM chunks
                std::sort(ppt.begin(), ppt.end(), [](const PpxSeg &a, const PpxSeg &b) { return a.z < b.z; });
                for (size_t q = 1; q < ppt.size(); ++q)
                    if (ppt[q].z == ppt[q - 1].z) ok = false;  // "Zppt already read" (j2k.cpp:4958)
                std::vector<uint8_t> &ph = tpacked[lt];
                ph.clear();
                if (!ppm_chunk.empty()) {
                    // the reference reads PPM headers through one running
                    // pointer over the merged Nppm chunks (T2.cpp:366-375): a
                    // tile's headers start at its first tile-part's chunk and
                    // run on past its own chunks when the stream ended before
                    // its later tile-parts (the tile is decoded from the
                    // tile-parts read, its later packets' headers still parsed)
                    for (uint32_t q : tpseq[t])
                        if (q >= ppm_chunk.size()) ok = false;
                    if (ok && !tpseq[t].empty()) ppm_from[lt] = ppm_chunk[tpseq[t][0]].first;
                    tpacked_on[lt] = 1;
                } else if (!ppt.empty()) {
                    for (auto &q : ppt) ph.insert(ph.end(), csb + q.off, csb + q.off + q.len);
                    tpacked_on[lt] = 1;
                }
                if (!ok) { terr[lt] = 3; continue; }
            }
            tile.comps.resize(nc);
            for (uint32_t k = 0; k < nc; ++k) build_tilecomp(tile.comps[k], tile.r, tcp, k, false);
            // tile data: single tile-part -> decode in place; else concatenate
            const uint8_t *td;
            size_t tlen;
            uint64_t base;
            contig[lt] = tparts[t].size() <= 1;
            if (contig[lt]) {
                td = tparts[t].empty() ? csb : csb + tparts[t][0].first;
                tlen = tparts[t].empty() ? 0 : tparts[t][0].second;
                base = tparts[t].empty() ? 0 : tparts[t][0].first;
            } else {
                std::vector<uint8_t> &tbuf = tbufs[lt];
                for (auto &pp : tparts[t]) tbuf.insert(tbuf.end(), csb + pp.first, csb + pp.first + pp.second);
                td = tbuf.data();
                tlen = tbuf.size();
                base = 0;
            }
            // packets in the tile's progression (T2::decode_packets, T2.cpp:194-258),
            // POC entries of the main header followed by the tile's own
            std::vector<PacketId> order;
            decode_packet_order(tcp, tile, order);
            size_t off = 0;
            uint32_t packno = 0;
            PackedHdr packed = ppm_chunk.empty() ? PackedHdr{tpacked[lt].data(), tpacked[lt].size(), 0}
                                                 : PackedHdr{ppm_buf.data() + ppm_from[lt], ppm_buf.size() - ppm_from[lt], 0};
            for (const auto &pk : order) {
                // the data ends before the packets do (a truncated stream):
                // the remaining packets are empty (a zero-length header reads
                // as "no data", T2.cpp:393-400) -- unless the headers are packed
                // (PPM / PPT), which keep coming; their bodies are then empty
                if (off >= tlen && !tpacked_on[lt]) break;
                const bool skip = max_layers && pk.layno >= max_layers;
                int64_t used = decode_packet(tile.comps[pk.compno], pk.resno, pk.precno, pk.layno, td + off, tlen - off,
                                             base + off, tcp.csty, &packno, skip, tcp.comp[pk.compno].cblksty,
                                             tpacked_on[lt] ? &packed : nullptr);
                if (used < 0) { terr[lt] = 2; break; }
                off += (size_t)used;
            }
        }
    });
    for (uint32_t lt = 0; lt < nsh; ++lt) {
        if (terr[lt] == 1) return set_err(GRKGPU_ECORRUPT, "Error reading POC marker");
        if (terr[lt] == 2) return set_err(GRKGPU_ECORRUPT, "corrupt packet header");
        if (terr[lt] == 3) return set_err(GRKGPU_ECORRUPT, "corrupt tile-part header marker (COD/COC/QCD/QCC/RGN/PPT/PPM)");
        if (terr[lt] == 5)
            return set_err(GRKGPU_ECORRUPT, "QCD marker: number of step sizes is less than 3 * (tile decompositions) + 1");
        if (terr[lt] == 4)
            return set_err(GRKGPU_EUNSUPPORTED, "tile-component coding style not supported (HT code-block style, "
                                                "code-blocks above 64 x 64, MCT over components of different "
                                                "wavelets or sizes, or reduce too large)");
    }
    bool any_roi = false;
    for (uint32_t lt = 0; lt < nsh; ++lt)
        for (uint32_t k = 0; k < nc; ++k) any_roi = any_roi || troi[lt][k];
    for (uint32_t lt = 0; lt < nsh; ++lt) {
        Tile &tile = tiles[lt];
        if (tile.comps.empty()) continue;
        for (uint32_t k = 0; k < nc; ++k) {
            tile.comps[k].arena_off = arena;
            uint64_t area = (uint64_t)tile.comps[k].r.w() * tile.comps[k].r.h();
            arena += (area + 63) & ~63ull;
            lloff[lt * nc + k] = llarena;
            llarena += ll_geom(tile.comps[k]).elems;
        }
        const bool contiguous = contig[lt] != 0;
        const std::vector<uint8_t> &tilebuf = tbufs[lt];
        for (uint32_t k = 0; k < nc; ++k) {
            TileComp &tc = tile.comps[k];
            const BandNeed need = win ? window_need(tc, cwin[k], nullptr, reduce) : BandNeed();
            for_each_cblk(tc, [&](Band &band, Cblk &cb) {
                DecBlock d{};
                d.dst_off = tc.arena_off + (uint64_t)cb.by * tc.r.w() + cb.bx;
                d.dstride = tc.r.w();
                d.w = cb.r.w();
                d.h = cb.r.h();
                d.orient = band.bandno;
                d.irrev = tc.irrev;
                d.step = band.stepsize;
                dsty.push_back(tsty[lt][k]);
                // passes beyond the last bit-plane are not decoded (t1_decode_cblk
                // stops at bpno < 0, t1.cpp:1086-1090)
                d.numpasses = std::min<uint32_t>(cb.numpasses, cb.numbps ? 3 * cb.numbps - 2 : 0);
                d.numbps = cb.numbps;
                d.len = cb.seglen;
                // codeword segments (one unless TERMALL): each points at its
                // bytes in place when they are one contiguous chunk, else at
                // a copy appended after the codestream
                seg_first.push_back((uint32_t)dsegs.size());
                for (const auto &sg : cb.segs) {
                    DecSeg ds{};
                    ds.len = sg.len;
                    ds.npasses = sg.numpasses;
                    if (sg.chunks.size() == 1 && contiguous) {
                        ds.data_off = sg.chunks[0].first;
                    } else if (!sg.chunks.empty()) {
                        ds.data_off = (uint64_t)len + extra.size();  // placed after the codestream
                        for (auto &ch : sg.chunks) {
                            const uint8_t *srcp = contiguous ? csb + ch.first : tilebuf.data() + ch.first;
                            extra.insert(extra.end(), srcp, srcp + ch.second);
                        }
                    } else {
                        ds.data_off = 0;
                        ds.len = 0;
                    }
                    dsegs.push_back(ds);
                }
                d.data_off = cb.segs.empty() ? 0 : dsegs[seg_first.back()].data_off;
                if (any_roi) droi.push_back(troi[lt][k]);
                // no bytes: the block stays zero (T1Part1::decode returns before
                // t1_decode_cblk when the block has no data, T1Part1.cpp:139-140)
                if (!d.len) d.numpasses = 0;
                // t1_decode_cblk refuses bpno_plus_one = roishift + numbps >= 31
                // (t1.cpp:1055-1060; our numbps already holds the ROI shift, as
                // T1Part1.cpp:186 subtracts it before the call); the decoder's
                // scratch holds 32 planes
                if (d.numpasses && d.numbps >= 31) too_deep = true;
                db.push_back(d);
            }, tc.numres - reduce, win ? &need : nullptr);
        }
    }
    if (too_deep) return set_err(GRKGPU_ECORRUPT, "unsupported bpno_plus_one >= 31 (code-block bit-planes + ROI shift)");
    if (decoded_out) *decoded_out = walk.decoded;
    if (host_only) return GRKGPU_OK;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint32_t nblk = (uint32_t)db.size();
    seg_first.push_back((uint32_t)dsegs.size());
    bool mixed_sty = false;  // tile-components of different code-block styles: one decode launch per style
    for (uint32_t i = 1; i < nblk; ++i) mixed_sty = mixed_sty || dsty[i] != dsty[0];
    const bool lone = lone_call();
    const bool sort_work = (dwt_options().t1_dec_sort == 1 || (dwt_options().t1_dec_sort < 0 && lone)) && nblk > 64;
    if (sort_work || mixed_sty) {
        // blocks grouped by style (a launch each), and -- t1_dec_sort -- since
        // lanes of a wavefront run until its slowest block is done, blocks of
        // similar work (pass count, then coded bytes) together, heaviest first
        // (an LSD radix sort of one 48-bit key per block -- style, then
        // passes and bytes descending -- is the comparison sort's stable
        // order at a fraction of its cost: 26 K blocks, ~0.2 vs ~3 ms)
        std::vector<uint64_t> key(nblk);
        for (uint32_t i = 0; i < nblk; ++i) {
            key[i] = (uint64_t)dsty[i] << 40;
            if (sort_work)
                key[i] |= (uint64_t)(255u - std::min<uint32_t>(db[i].numpasses, 255u)) << 32 | (0xFFFFFFFFu - db[i].len);
        }
        std::vector<uint32_t> ord(nblk), tmp(nblk);
        for (uint32_t i = 0; i < nblk; ++i) ord[i] = i;
        for (int sh = 0; sh < 48; sh += 8) {
            uint32_t cnt[257] = {0};
            for (uint32_t i : ord) ++cnt[((key[i] >> sh) & 255u) + 1];
            if (*std::max_element(cnt + 1, cnt + 257) == nblk) continue;  // one digit value: order unchanged
            for (int b = 0; b < 256; ++b) cnt[b + 1] += cnt[b];
            for (uint32_t i : ord) tmp[cnt[(key[i] >> sh) & 255u]++] = i;
            ord.swap(tmp);
        }
        std::vector<DecBlock> db2(nblk);
        std::vector<DecSeg> segs2;
        segs2.reserve(dsegs.size());
        std::vector<uint32_t> first2(nblk + 1);
        std::vector<uint8_t> roi2(droi.size()), sty2(nblk);
        for (uint32_t j = 0; j < nblk; ++j) {
            const uint32_t i = ord[j];
            db2[j] = db[i];
            sty2[j] = dsty[i];
            first2[j] = (uint32_t)segs2.size();
            segs2.insert(segs2.end(), dsegs.begin() + seg_first[i], dsegs.begin() + seg_first[i + 1]);
            if (!droi.empty()) roi2[j] = droi[i];
        }
        first2[nblk] = (uint32_t)segs2.size();
        db.swap(db2);
        dsegs.swap(segs2);
        seg_first.swap(first2);
        droi.swap(roi2);
        dsty.swap(sty2);
    }
    // launch ranges: one per code-block style, each with its own scratch
    // groups (64 blocks each) so the ranges need no alignment
    struct StyRange { uint32_t b0, n, sty; uint64_t scr0; };
    std::vector<StyRange> sranges;
    uint64_t scr_records = 0;
    for (uint32_t i = 0; i < nblk;) {
        uint32_t j = i;
        while (j < nblk && dsty[j] == dsty[i]) ++j;
        sranges.push_back({i, j - i, dsty[i], scr_records});
        scr_records += t1_scratch_records(j - i);
        i = j;
    }
    double t_t2 = now_ms();
    HIPCHK(c->cs.ensure(len + extra.size() + 256));
    HIPCHK(c->coef.ensure(arena * 4 + 256));
    HIPCHK(c->work.ensure(arena * 4 + 256));
    HIPCHK(c->ll.ensure(llarena * 4 + 256));
    // the decoder's lane-interleaved groups span 64 records each (t1_lane.h)
    HIPCHK(c->scratch.ensure((size_t)scr_records * sizeof(T1Scratch) + 256));
    // per-segment unstuffed-stream regions (16-byte units)
    uint64_t uwords = 0;
    for (auto &sg : dsegs) {
        sg.ub_off = (uint32_t)(uwords / 4);
        uwords += t1_unstuff_region_words(sg.len);
    }
    if (uwords / 4 > 0xffffffffull) return set_err(GRKGPU_EUNSUPPORTED, "codestream too large for one call");
    const size_t segbytes = dsegs.size() * sizeof(DecSeg), sfbytes = seg_first.size() * 4, roibytes = droi.size();
    HIPCHK(c->segs.ensure(segbytes + sfbytes + roibytes + 256));
    HIPCHK(c->h_segs.ensure(segbytes + sfbytes + roibytes + 256));
    memcpy(c->h_segs.p, dsegs.data(), segbytes);
    memcpy((uint8_t *)c->h_segs.p + segbytes, seg_first.data(), sfbytes);
    if (roibytes) memcpy((uint8_t *)c->h_segs.p + segbytes + sfbytes, droi.data(), roibytes);
    HIPCHK(c->ubuf.ensure(uwords * 4 + 256));
    HIPCHK(c->blocks.ensure((size_t)nblk * sizeof(DecBlock) + 256));
    HIPCHK(c->h_blocks.ensure((size_t)nblk * sizeof(DecBlock) + 256));
    memcpy(c->h_blocks.p, db.data(), (size_t)nblk * sizeof(DecBlock));

    HIPCHK(hipEventRecord(c->ev[0], s));
    HIPCHK(hipMemcpyAsync(c->cs.p, csb, len, hipMemcpyHostToDevice, s));
    if (!extra.empty()) {
        HIPCHK(c->h_packed.ensure(extra.size() + 256));
        memcpy(c->h_packed.p, extra.data(), extra.size());
        HIPCHK(hipMemcpyAsync(c->cs.as<uint8_t>() + len, c->h_packed.p, extra.size(), hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipMemcpyAsync(c->blocks.p, c->h_blocks.p, (size_t)nblk * sizeof(DecBlock), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->segs.p, c->h_segs.p, segbytes + sfbytes + roibytes, hipMemcpyHostToDevice, s));
    // one plan per wavelet (COC / tile COD may mix 5/3 and 9/7 components)
    DwtPlan dplan[2];
    for (auto &tile : tiles)
        for (uint32_t k = 0; k < tile.comps.size(); ++k) {
            const TileComp &tc = tile.comps[k];
            // a window decode reconstructs, per level, only the windows over
            // the region the window's samples depend on
            std::vector<Rect> rn;
            if (win) window_need(tc, cwin[k], &rn, reduce);
            dwt_plan_tc(dplan[tc.irrev], tc, c->work.as<int32_t>() + tc.arena_off, c->coef.as<int32_t>() + tc.arena_off,
                        c->ll.as<int32_t>() + lloff[(tile.index - tb) * nc + k], tc.irrev, true, tc.numres - reduce,
                        win ? &rn : nullptr);
        }
    HIPCHK(dwt_upload(dplan[1], c->dwtjobs, c->h_dwtjobs, 1, s));
    HIPCHK(dwt_upload(dplan[0], c->dwtjobs53, c->h_dwtjobs53, 0, s));
    // window decode: the coefficients of the code-blocks left undecoded are
    // zero (they lie outside every window sample's support; zero keeps the
    // 9/7 float lifting free of stale NaNs)
    if (win && arena) HIPCHK(hipMemsetAsync(c->coef.p, 0, arena * 4, s));
    HIPCHK(hipEventRecord(c->ev[1], s));
    for (const StyRange &g : sranges)
        HIPCHK(launch_t1_decode(c->blocks.as<DecBlock>() + g.b0, g.n, c->cs.as<uint8_t>(),
                                c->scratch.as<T1Scratch>() + g.scr0, c->coef.as<int32_t>(), s, c->ubuf.as<uint32_t>(),
                                0, c->segs.as<DecSeg>(),
                                (const uint32_t *)(c->segs.as<uint8_t>() + segbytes) + g.b0, g.sty,
                                roibytes ? c->segs.as<uint8_t>() + segbytes + sfbytes + g.b0 : nullptr,
                                lone ? lone_bpw(nblk) : 0));
    HIPCHK(hipEventRecord(c->ev[2], s));
    c->ltimes.clear();
    c->lidx.clear();
    LaunchLog llog{&c->lev, &c->ltimes, &c->lidx};
    HIPCHK(dwt_launch(dplan[1], c->dwtjobs, 1, true, s, c->launch_timing ? &llog : nullptr));
    HIPCHK(dwt_launch(dplan[0], c->dwtjobs53, 0, true, s, c->launch_timing ? &llog : nullptr));
    HIPCHK(hipEventRecord(c->ev[3], s));
    PlanePtrs dst{};
    if (planes_on_device) {
        for (uint32_t k = 0; k < nc; ++k) dst.p[k] = planes[k];
    } else {
        HIPCHK(c->img.ensure(ooff[nc] * 4 + 256));
        for (uint32_t k = 0; k < nc; ++k) dst.p[k] = c->img.as<int32_t>() + ooff[k];
    }
    if (opad)
        for (uint32_t k = 0; k < nc; ++k)
            HIPCHK(hipMemsetAsync(dst.p[k], 0, (ooff[k + 1] - ooff[k]) * 4, s));
    else if (missing)  // tiles the tile-part walk never reached: zero (their regions only -- a shard's
                       // device planes hold other tiles)
        for (uint32_t t = tb; t < te; ++t) {
            if (walk.decoded[t] || wskip[t]) continue;
            for (uint32_t k = 0; k < nc; ++k) {
                const Rect cr = comp_rect(tile_rect(cp, t), cp.dx[k], cp.dy[k]);
                const Rect rr{ceil_pow2(cr.x0, reduce), ceil_pow2(cr.y0, reduce), ceil_pow2(cr.x1, reduce),
                              ceil_pow2(cr.y1, reduce)};
                const Rect o = intersect(rr, orect[k]);
                if (o.empty()) continue;
                const uint32_t ow = orect[k].w();
                HIPCHK(hipMemset2DAsync(dst.p[k] + (uint64_t)(o.y0 - orect[k].y0) * ow + (o.x0 - orect[k].x0),
                                        (size_t)ow * 4, 0, (size_t)o.w() * 4, o.h(), s));
            }
        }
    ShiftArr sh{}, mn{}, mx{};
    for (uint32_t k = 0; k < nc; ++k) {
        sh.v[k] = cp.shift[k];
        if (cp.sgnd[k]) { mn.v[k] = -(1 << (cp.prec[k] - 1)); mx.v[k] = (1 << (cp.prec[k] - 1)) - 1; }
        else { mn.v[k] = 0; mx.v[k] = (1 << cp.prec[k]) - 1; }
    }
    for (auto &tile : tiles) {
        if (tile.comps.empty()) continue;  // outside the window
        if (mixed) {  // each tile-component on its own grid, no MCT
            for (uint32_t k = 0; k < nc; ++k) {
                const TileComp &tc = tile.comps[k];
                const Rect tr = tc.res[tc.numres - 1 - reduce].r;
                const Rect out = intersect(tr, orect[k]);
                if (out.empty()) continue;
                PlanePtrs tsrc{}, tdst{};
                ShiftArr sk{}, mnk{}, mxk{};
                tsrc.p[0] = c->work.as<int32_t>() + tc.arena_off + (uint64_t)(out.y0 - tr.y0) * tr.w() + (out.x0 - tr.x0);
                tdst.p[0] = dst.p[k] + (uint64_t)(out.y0 - orect[k].y0) * orect[k].w() + (out.x0 - orect[k].x0);
                sk.v[0] = sh.v[k];
                mnk.v[0] = mn.v[k];
                mxk.v[0] = mx.v[k];
                HIPCHK(launch_mct_inv_dcshift(tsrc, tr.w(), out.w(), out.h(), tdst, orect[k].w(), 1, sk, mnk, mxk, 0,
                                              tc.irrev, s));
            }
            continue;
        }
        // every component on one grid: one launch, MCT included (orect[k]
        // is the output on that grid -- the image itself without subsampling)
        PlanePtrs tsrc{}, tdst{};
        const Rect tr = tile.comps[0].res[tile.comps[0].numres - 1 - reduce].r;  // the tile at the decoded resolution
        const Rect out = intersect(tr, orect[0]);             // its part of the output
        if (out.empty()) continue;
        const uint32_t ow = orect[0].w();
        for (uint32_t k = 0; k < nc; ++k) {
            tsrc.p[k] = c->work.as<int32_t>() + tile.comps[k].arena_off + (uint64_t)(out.y0 - tr.y0) * tr.w() +
                        (out.x0 - tr.x0);
            tdst.p[k] = dst.p[k] + (uint64_t)(out.y0 - orect[0].y0) * ow + (out.x0 - orect[0].x0);
        }
        int32_t wmask = 0;  // components holding 9/7 (float) samples
        for (uint32_t k = 0; k < nc; ++k) wmask |= tile.comps[k].irrev << k;
        HIPCHK(launch_mct_inv_dcshift(tsrc, tr.w(), out.w(), out.h(), tdst, ow, nc, sh, mn, mx,
                                      tmct[tile.index - tb], wmask, s));
    }
    HIPCHK(hipEventRecord(c->ev[4], s));
    if (!planes_on_device) {
        if (whole) {
            for (uint32_t k = 0; k < nc; ++k)
                HIPCHK(hipMemcpyAsync(planes[k], dst.p[k], (ooff[k + 1] - ooff[k]) * 4, hipMemcpyDeviceToHost, s));
        } else {  // only the shard's tiles
            for (auto &tile : tiles)
                for (uint32_t k = 0; k < nc; ++k) {
                    const uint64_t o = (uint64_t)(tile.r.y0 - cp.image.y0) * iw + (tile.r.x0 - cp.image.x0);
                    HIPCHK(hipMemcpy2DAsync(planes[k] + o, (size_t)iw * 4, dst.p[k] + o, (size_t)iw * 4,
                                            (size_t)tile.r.w() * 4, tile.r.h(), hipMemcpyDeviceToHost, s));
                }
        }
    }
    HIPCHK(hipEventRecord(c->ev[5], s));
    HIPCHK(hipStreamSynchronize(s));
    double t_end = now_ms();
    grkgpu_stats &st = c->stats;
    memset(&st, 0, sizeof(st));
    hipEventElapsedTime(&st.h2d_ms, c->ev[0], c->ev[1]);
    hipEventElapsedTime(&st.t1_ms, c->ev[1], c->ev[2]);
    hipEventElapsedTime(&st.dwt_ms, c->ev[2], c->ev[3]);
    hipEventElapsedTime(&st.dcshift_mct_ms, c->ev[3], c->ev[4]);
    hipEventElapsedTime(&st.d2h_ms, c->ev[4], c->ev[5]);
    log_collect(c);
    st.host_t2_ms = (float)(t_t2 - t_start);
    st.total_ms = (float)(t_end - t_start);
    st.num_cblks = nblk;
    st.cs_bytes = len;
    return GRKGPU_OK;
}

extern "C" int grkgpu_decompress(grkgpu_ctx *c, const uint8_t *csb, size_t len, grkgpu_image_desc *img,
                                 int32_t *const *planes, int planes_on_device) {
    return decompress_impl(c, csb, len, img, planes, planes_on_device, 0, 0xffffffffu);
}

extern "C" int grkgpu_decompress_reduced(grkgpu_ctx *c, const uint8_t *csb, size_t len, uint32_t reduce,
                                         grkgpu_image_desc *img, int32_t *const *planes, int planes_on_device) {
    return decompress_impl(c, csb, len, img, planes, planes_on_device, 0, 0xffffffffu, reduce);
}

extern "C" int grkgpu_decompress_window(grkgpu_ctx *c, const uint8_t *csb, size_t len, uint32_t x0, uint32_t y0,
                                        uint32_t x1, uint32_t y1, grkgpu_image_desc *img, int32_t *const *planes,
                                        int planes_on_device) {
    const Rect w{x0, y0, x1, y1};
    return decompress_impl(c, csb, len, img, planes, planes_on_device, 0, 0xffffffffu, 0, &w);
}

extern "C" int grkgpu_decompress_ex(grkgpu_ctx *c, const uint8_t *csb, size_t len, const grkgpu_dparams *dp,
                                    grkgpu_image_desc *img, int32_t *const *planes, int planes_on_device) {
    if (!dp) return decompress_impl(c, csb, len, img, planes, planes_on_device, 0, 0xffffffffu);
    const bool win = dp->DA_x0 || dp->DA_y0 || dp->DA_x1 || dp->DA_y1;
    const Rect w{dp->DA_x0, dp->DA_y0, dp->DA_x1, dp->DA_y1};
    if (win && (dp->DA_x1 <= dp->DA_x0 || dp->DA_y1 <= dp->DA_y0)) return set_err(GRKGPU_EINVAL, "empty decode area");
    return decompress_impl(c, csb, len, img, planes, planes_on_device, 0, 0xffffffffu, dp->cp_reduce,
                           win ? &w : nullptr, dp->cp_layer);
}

extern "C" int grkgpu_walk_tiles(const uint8_t *csb, size_t len, uint8_t *decoded, uint32_t cap, uint32_t *ntiles) {
    if (!csb || !ntiles) return set_err(GRKGPU_EINVAL, "null argument");
    grkgpu_image_desc d{};
    int rc = grkgpu_read_header(csb, len, &d);
    if (rc) return rc;
    std::vector<uint8_t> dec;
    rc = decompress_impl(nullptr, csb, len, nullptr, nullptr, 0, 0, 0xffffffffu, 0, nullptr, 0, true, &dec);
    if (rc) return rc;
    *ntiles = (uint32_t)dec.size();
    if (decoded)
        for (uint32_t t = 0; t < dec.size() && t < cap; ++t) decoded[t] = dec[t];
    return GRKGPU_OK;
}

extern "C" int grkgpu_decompress_tiles(grkgpu_ctx *c, const uint8_t *csb, size_t len, uint32_t tile_begin,
                                       uint32_t tile_end, int32_t *const *planes, int planes_on_device) {
    return decompress_impl(c, csb, len, nullptr, planes, planes_on_device, tile_begin, tile_end);
}

// ---------------------------------------------------------------------------
// stage entry points
// ---------------------------------------------------------------------------
extern "C" int grkgpu_dcshift_mct_fwd(int32_t *const *planes, uint32_t numcomps, uint32_t w, uint32_t h,
                                      uint32_t stride, const int32_t *shift, int32_t mct, int32_t irreversible,
                                      void *stream) {
    if (!planes || !shift || numcomps < 1 || numcomps > 16) return set_err(GRKGPU_EINVAL, "bad arguments");
    int rc = check_device(-1);
    if (rc) return rc;
    PlanePtrs p{};
    SrcPlanes ps{};
    ShiftArr sh{};
    for (uint32_t k = 0; k < numcomps; ++k) { p.p[k] = planes[k]; ps.p[k] = planes[k]; sh.v[k] = shift[k]; }
    HIPCHK(launch_dcshift_mct_fwd(ps, SMP_I32, stride, p, w, h, numcomps, sh, mct, irreversible, (hipStream_t)stream));
    return GRKGPU_OK;
}

extern "C" int grkgpu_mct_inv_dcshift(int32_t *const *planes, uint32_t numcomps, uint32_t w, uint32_t h,
                                      uint32_t stride, const uint32_t *prec, const int32_t *sgnd, int32_t mct,
                                      int32_t irreversible, void *stream) {
    if (!planes || !prec || !sgnd || numcomps < 1 || numcomps > 16 || stride < w)
        return set_err(GRKGPU_EINVAL, "bad arguments (stride must be >= w)");
    int rc = check_device(-1);
    if (rc) return rc;
    PlanePtrs p{};
    ShiftArr sh{}, mn{}, mx{};
    for (uint32_t k = 0; k < numcomps; ++k) {
        p.p[k] = planes[k];
        sh.v[k] = sgnd[k] ? 0 : (1 << (prec[k] - 1));
        if (sgnd[k]) { mn.v[k] = -(1 << (prec[k] - 1)); mx.v[k] = (1 << (prec[k] - 1)) - 1; }
        else { mn.v[k] = 0; mx.v[k] = (1 << prec[k]) - 1; }
    }
    HIPCHK(launch_mct_inv_dcshift(p, stride, w, h, p, stride, numcomps, sh, mn, mx, mct, irreversible ? 0xFFFF : 0,
                                  (hipStream_t)stream));
    return GRKGPU_OK;
}

static void dwt_stage_geom(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t numres, int32_t irrev,
                           bool inverse, TileComp &tc) {
    CodingParams cp;
    cp.numcomps = 1;
    cp.image = {x0, y0, x1, y1};
    cp.prec[0] = 8;
    cp.numres = numres;
    cp.irrev = irrev;
    generate_qcd(cp);
    build_tilecomp(tc, cp.image, cp, 0, !inverse);
}

// scratch layout: [temporary copy of buf | LL ping-pong | job table]
extern "C" size_t grkgpu_dwt_scratch_bytes(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t numres) {
    if (x1 <= x0 || y1 <= y0 || numres < 1 || numres > 33) return 0;
    TileComp tc;
    dwt_stage_geom(x0, y0, x1, y1, numres, 0, false, tc);
    const uint64_t area = ((uint64_t)(x1 - x0) * (y1 - y0) + 63) / 64 * 64;
    return (size_t)(area + ll_geom(tc).elems) * 4 + 64 * sizeof(DwtJob) + 512;
}

static int dwt_common(int32_t *buf, int32_t *scratch, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                      uint32_t numres, int32_t irrev, void *stream, bool inverse) {
    if (!buf || !scratch || x1 <= x0 || y1 <= y0 || numres < 1 || numres > 33)
        return set_err(GRKGPU_EINVAL, "bad arguments");
    int rc = check_device(-1);
    if (rc) return rc;
    TileComp tc;
    dwt_stage_geom(x0, y0, x1, y1, numres, irrev, inverse, tc);
    const uint64_t area = ((uint64_t)(x1 - x0) * (y1 - y0) + 63) / 64 * 64;
    int32_t *tmp = scratch, *ll = scratch + area;
    DwtJob *djobs = (DwtJob *)(((uintptr_t)(ll + ll_geom(tc).elems) + 255) & ~(uintptr_t)255);
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(tmp, buf, (uint64_t)(x1 - x0) * (y1 - y0) * 4, hipMemcpyDeviceToDevice, s));
    DwtPlan P;
    if (!inverse) dwt_plan_tc(P, tc, tmp, buf, ll, irrev, false);
    else dwt_plan_tc(P, tc, buf, tmp, ll, irrev, true);
    dwt_finalize(P, irrev);
    std::vector<DwtJob> flat;
    for (auto &l : P.levels) flat.insert(flat.end(), l.begin(), l.end());
    if (!flat.empty()) {
        HIPCHK(hipMemcpyAsync(djobs, flat.data(), flat.size() * sizeof(DwtJob), hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    for (auto &cpy : P.copies) HIPCHK(hipMemcpyAsync(cpy.first, cpy.second, P.copy_elems * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(dwt_run_levels(P, djobs, irrev, inverse, s));
    return GRKGPU_OK;
}

extern "C" int grkgpu_dwt_fwd(int32_t *buf, int32_t *scratch, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                              uint32_t numres, int32_t irreversible, void *stream) {
    return dwt_common(buf, scratch, x0, y0, x1, y1, numres, irreversible, stream, false);
}

extern "C" int grkgpu_dwt_inv(int32_t *buf, int32_t *scratch, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                              uint32_t numres, int32_t irreversible, void *stream) {
    return dwt_common(buf, scratch, x0, y0, x1, y1, numres, irreversible, stream, true);
}

static_assert(sizeof(grkgpu_enc_block) == sizeof(EncBlock), "EncBlock ABI");
// the device's pass records are read in place as the host's (launch_pass_records)
static_assert(sizeof(DevPass) == sizeof(EncPass) && offsetof(DevPass, dd) == offsetof(EncPass, dd) &&
                  offsetof(DevPass, slope) == offsetof(EncPass, slope) && offsetof(DevPass, term) == offsetof(EncPass, term),
              "DevPass layout");
static_assert(sizeof(grkgpu_enc_result) == sizeof(EncResult), "EncResult ABI");
static_assert(sizeof(grkgpu_dec_block) == sizeof(DecBlock), "DecBlock ABI");

extern "C" int grkgpu_t1_encode_blocks(const grkgpu_enc_block *blocks, uint32_t nblocks, const int32_t *coef,
                                       void *scratch, uint8_t *out, grkgpu_enc_result *results, int with_distortion,
                                       void *stream) {
    if (!blocks || !coef || !scratch || !out || !results) return set_err(GRKGPU_EINVAL, "null argument");
    int rc = check_device(-1);
    if (rc) return rc;
    // scratch layout: the encoder's rows for nblocks (rounded up to 64) blocks
    // of 32 planes, then 32 fixed symbol slots per block
    uint8_t *sym = (uint8_t *)scratch + t1e_scratch_bytes(nblocks, 32);
    HIPCHK(launch_t1_encode((const EncBlock *)blocks, nblocks, coef, scratch, sym, nullptr, 32, out,
                            (EncResult *)results, (hipStream_t)stream));
    if (with_distortion)
        HIPCHK(launch_t1_dist((const EncBlock *)blocks, nblocks, 32, coef, scratch, (EncResult *)results,
                              (hipStream_t)stream));
    return GRKGPU_OK;
}

extern "C" int grkgpu_t1_decode_blocks(const grkgpu_dec_block *blocks, uint32_t nblocks, const uint8_t *data,
                                       void *scratch, int32_t *dst, void *stream) {
    if (!blocks || !data || !scratch || !dst) return set_err(GRKGPU_EINVAL, "null argument");
    int rc = check_device(-1);
    if (rc) return rc;
    // scratch layout: nblocks rounded up to a multiple of 64 T1Scratch
    // records (the decoder's lane-interleaved groups), then one fixed-size
    // unstuffed-stream region per block
    uint32_t *ubuf = (uint32_t *)((uint8_t *)scratch + (size_t)t1_scratch_records(nblocks) * sizeof(T1Scratch));
    HIPCHK(launch_t1_decode((const DecBlock *)blocks, nblocks, data, (T1Scratch *)scratch, dst, (hipStream_t)stream,
                            ubuf, t1_stage_dec_words()));
    return GRKGPU_OK;
}
