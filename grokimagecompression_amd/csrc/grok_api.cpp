// libgrok.so: Grok's public grk_* C API (include/grk_api.h) over the MI355X
// path (grk_mi355x.h).  A drop-in for the reference's libgrok under
// grk_compress / grk_decompress; host code only.
//
// Reference behaviour followed (file:line of /root/reference/src/lib/jp2):
//   grok.cpp:152-170 initialize, :342-347 / :518-544 default parameters,
//   :381-466 decode calls, :470-592 compress calls, :620-800 streams and
//   images; BufferedStream.cpp (mem / file streams); codestream/j2k.cpp
//   j2k_read_header (image from SIZ), j2k_set_decode_area (window clip and
//   image bounds), j2k_decode (cp_reduce / cp_layer).
#include "../../include/grk_api.h"
#include "../../include/grk_mi355x.h"

#include <stdarg.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <string>
#include <vector>

#define GRK_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

// ---- messages ----
struct Handler {
    grk_msg_callback cb = nullptr;
    void *user = nullptr;
};
Handler g_info, g_warn, g_err;

void emit(const Handler &h, const char *fmt, ...) {
    if (!h.cb) return;
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf) - 1, fmt, ap);
    va_end(ap);
    strcat(buf, "\n");
    h.cb(buf, h.user);
}
#define GRK_ERROR(...) emit(g_err, __VA_ARGS__)

// ---- GPU contexts: a pool per device ----
// A grkgpu_ctx (its stream, arenas and pinned result buffer) serves one call
// at a time.  The reference allows one codec per caller thread
// (SURVEY 8(b1)), so each grk_encode / grk_decode leases a context from its
// device's pool for the whole call -- the GPU work and the copy of the result
// out of the context's buffer -- and returns it; concurrent codecs get
// different contexts, and a context is created only when all are leased.
std::mutex g_mu;
std::vector<std::vector<grkgpu_ctx *>> g_free;  // [device] idle contexts
std::vector<grkgpu_ctx *> g_all;                // every live context (grk_deinitialize)
std::vector<grkgpu_ctx *> g_retired;            // leased when grk_deinitialize ran: destroyed on return

struct Lease {
    grkgpu_ctx *ctx = nullptr;
    int device = 0;
    explicit Lease(int dev) : device(dev < 0 ? 0 : dev) {
        {
            std::lock_guard<std::mutex> lk(g_mu);
            if ((size_t)device >= g_free.size()) g_free.resize(device + 1);
            if (!g_free[device].empty()) {
                ctx = g_free[device].back();
                g_free[device].pop_back();
                return;
            }
        }
        grkgpu_ctx *c = nullptr;
        if (grkgpu_create(device, &c) != GRKGPU_OK) {
            GRK_ERROR("MI355X context on device %d: %s", device, grkgpu_last_error());
            return;
        }
        std::lock_guard<std::mutex> lk(g_mu);
        g_all.push_back(c);
        ctx = c;
    }
    ~Lease() {
        if (!ctx) return;
        std::lock_guard<std::mutex> lk(g_mu);
        auto r = std::find(g_retired.begin(), g_retired.end(), ctx);
        if (r != g_retired.end()) {  // grk_deinitialize ran during this call
            g_retired.erase(r);
            grkgpu_destroy(ctx);
            return;
        }
        if ((size_t)device >= g_free.size()) g_free.resize(device + 1);
        g_free[device].push_back(ctx);
    }
    Lease(const Lease &) = delete;
    Lease &operator=(const Lease &) = delete;
};

// ---- streams (BufferedStream semantics for the calls the codec makes:
// sequential read to the end, sequential write) ----
struct MemBuf {
    uint8_t *buf = nullptr;
    size_t len = 0, off = 0, high = 0;
    bool owns = false;
    void *map = nullptr;  // mapped file (munmap on free)
};

size_t mem_read(void *dst, size_t n, void *u) {
    MemBuf *m = (MemBuf *)u;
    const size_t k = std::min(n, m->len - std::min(m->off, m->len));
    if (!k) return (size_t)-1;  // end of stream (BufferedStream's convention)
    memcpy(dst, m->buf + m->off, k);
    m->off += k;
    return k;
}
size_t mem_write(void *src, size_t n, void *u) {
    MemBuf *m = (MemBuf *)u;
    if (m->off + n > m->len) return (size_t)-1;
    memcpy(m->buf + m->off, src, n);
    m->off += n;
    m->high = std::max(m->high, m->off);
    return n;
}
bool mem_seek(uint64_t pos, void *u) {
    MemBuf *m = (MemBuf *)u;
    if (pos > m->len) return false;
    m->off = (size_t)pos;
    return true;
}
void mem_free(void *u) {
    MemBuf *m = (MemBuf *)u;
    if (m->map) munmap(m->map, m->len);
    else if (m->owns) delete[] m->buf;
    delete m;
}
size_t file_read(void *dst, size_t n, void *u) {
    const size_t k = fread(dst, 1, n, (FILE *)u);
    return k ? k : (size_t)-1;
}
size_t file_write(void *src, size_t n, void *u) { return fwrite(src, 1, n, (FILE *)u); }
bool file_seek(uint64_t pos, void *u) { return fseeko((FILE *)u, (off_t)pos, SEEK_SET) == 0; }
void file_free(void *u) { fclose((FILE *)u); }

struct Stream {
    bool input = true;
    size_t buffer_size = 0;
    grk_stream_read_fn read = nullptr;
    grk_stream_zero_copy_read_fn zc_read = nullptr;
    grk_stream_write_fn write = nullptr;
    grk_stream_seek_fn seek = nullptr;
    void *user = nullptr;
    grk_stream_free_user_data_fn free_user = nullptr;
    uint64_t user_len = 0;
    MemBuf *mem = nullptr;  // set for memory / mapped streams

    bool read_all(std::vector<uint8_t> &out) {
        if (mem) {  // the whole buffer, no copy through callbacks
            out.assign(mem->buf + std::min(mem->off, mem->len), mem->buf + mem->len);
            mem->off = mem->len;
            return true;
        }
        if (!read) return false;
        out.clear();
        std::vector<uint8_t> chunk(std::max<size_t>(buffer_size, 1 << 20));
        for (;;) {
            const size_t k = read(chunk.data(), chunk.size(), user);
            if (k == (size_t)-1 || k == 0) break;
            out.insert(out.end(), chunk.data(), chunk.data() + k);
        }
        return true;
    }
    bool write_all(const uint8_t *p, size_t n) {
        if (!write) return false;
        while (n) {
            const size_t k = write((void *)p, n, user);
            if (k == (size_t)-1 || k == 0) return false;
            p += k;
            n -= k;
        }
        return true;
    }
};

// ---- codecs ----
struct Codec {
    bool decompressor = false;
    Stream *stream = nullptr;
    // compress
    grk_cparameters cparams{};
    grk_image *image = nullptr;
    bool setup = false;
    std::vector<uint8_t> mct;  // grk_set_MCT's matrix + DC shifts, taken out of the parameters at setup
    // decompress
    grk_dparameters dparams{};
    std::vector<uint8_t> cs;
    bool have_header = false;
    grkgpu_image_desc desc{};
    grkgpu_header_info hinfo{};
    std::vector<grkgpu_comp_info> cinfo;  // per component (main COD / COC, QCD / QCC)
    bool window = false;
    uint32_t win[4] = {0, 0, 0, 0};
    // tile streaming, encode (grk_write_tile): next tile expected, parts written
    uint32_t next_tile = 0;
    bool header_written = false, eoc_written = false;
    // tile streaming, decode (grk_read_tile_header / grk_decode_tile_data)
    std::vector<uint32_t> tile_order;  // tiles in codestream order (first tile-part), meeting the decode area
    bool tile_order_ready = false;
    size_t tile_pos = 0;
    int64_t cur_tile = -1;
    std::vector<int32_t> reduced;  // reduced-resolution decode of the whole image (cp_reduce > 0), decoded once
    grkgpu_image_desc reduced_desc{};
    bool decoded = false;  // grk_decode has read every tile-part (what grk_get_cstr_index reports)
};

uint32_t cdivpow2(uint32_t v, uint32_t r) { return (uint32_t)(((uint64_t)v + (1ull << r) - 1) >> r); }
uint32_t cdiv(uint32_t v, uint32_t d) { return (uint32_t)(((uint64_t)v + d - 1) / d); }
// a component's origin and size for an image / area [x0, x1) x [y0, y1) of
// the reference grid, on its dx / dy grid at resolution reduce r
// (j2k_read_header / j2k_set_decode_area: ceil(ceil(x / dx) / 2^r))
void comp_geom(grk_image_comp &cp, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t r) {
    const uint32_t dx = cp.dx ? cp.dx : 1, dy = cp.dy ? cp.dy : 1;
    cp.x0 = cdivpow2(cdiv(x0, dx), r);
    cp.y0 = cdivpow2(cdiv(y0, dy), r);
    cp.w = cdivpow2(cdiv(x1, dx), r) - cp.x0;
    cp.h = cdivpow2(cdiv(y1, dy), r) - cp.y0;
}

struct TileRect { uint32_t x0, y0, x1, y1; };
// tile t of the grid (j2k tile geometry: tile (p, q) spans tx0 + p tdx .. clipped to the image)
TileRect tile_rect(uint32_t t, uint32_t tw, uint32_t tx0, uint32_t ty0, uint32_t tdx, uint32_t tdy,
                   const grkgpu_image_desc &d) {
    const uint32_t p = t % tw, q = t / tw;
    return {std::max(d.x0, tx0 + p * tdx), std::max(d.y0, ty0 + q * tdy),
            (uint32_t)std::min<uint64_t>(d.x1, (uint64_t)tx0 + (uint64_t)(p + 1) * tdx),
            (uint32_t)std::min<uint64_t>(d.y1, (uint64_t)ty0 + (uint64_t)(q + 1) * tdy)};
}

// The matrix size of each live grk_set_MCT allocation (the ABI's mct_data is
// a bare pointer): map_cparams refuses an image whose component count differs
// from the one grk_set_MCT was given, instead of reading past the allocation.
// grk_setup_encoder takes the matrix out and frees the allocation, as
// j2k_setup_encoder does (j2k.cpp:1899-1956 copy, :2052-2055 free), and erases
// the entry, so a reused address never matches a stale size.  A pointer the
// caller filled in directly (not from grk_set_MCT) is read as numcomps x
// numcomps floats + numcomps DC shifts, as the reference reads it, and stays
// the caller's.
static std::mutex g_mct_mu;
static std::unordered_map<const void *, uint32_t> g_mct_n;

// grk_cparameters -> grkgpu_cparams (j2k_setup_encoder's reading of them,
// codestream/j2k.cpp:1609-2050); false for options outside grk_mi355x.h
bool map_cparams(const grk_cparameters *g, uint32_t numcomps, grkgpu_cparams *p) {
    grkgpu_default_cparams(p);
    if (g->cblk_sty & ~0x3Fu) { GRK_ERROR("code-block style 0x%x: HT is not supported", g->cblk_sty); return false; }
    if (g->isHT) { GRK_ERROR("HTJ2K is not supported"); return false; }
    if (g->mct_data) {  // grk_set_MCT: numcomps x numcomps matrix, then numcomps DC shifts (j2k.cpp:1899-1956)
        if (numcomps > GRKGPU_MAX_COMPS) return false;
        {
            std::lock_guard<std::mutex> lk(g_mct_mu);
            const auto it = g_mct_n.find(g->mct_data);
            if (it != g_mct_n.end() && it->second != numcomps) {
                GRK_ERROR("custom MCT matrix (grk_set_MCT) of %u components for an image of %u", it->second, numcomps);
                return false;
            }
        }
        p->mct_ncomp = numcomps;
        memcpy(p->mct_matrix, g->mct_data, sizeof(float) * numcomps * numcomps);
        memcpy(p->mct_dc_shift, (const uint8_t *)g->mct_data + sizeof(float) * numcomps * numcomps,
               sizeof(int32_t) * numcomps);
    }
    // subsampling_dx / _dy are the CLI image readers' (PNMFormat.cpp:397-417);
    // the library takes each component's dx / dy from the image
    p->numresolution = g->numresolution;
    p->cblockw_init = g->cblockw_init;
    p->cblockh_init = g->cblockh_init;
    p->irreversible = g->irreversible ? 1 : 0;
    p->tcp_mct = g->tcp_mct == 255 ? -1 : g->tcp_mct == 2 ? 2 : (g->tcp_mct && numcomps >= 3 ? 1 : 0);
    p->tile_size_on = g->tile_size_on ? 1 : 0;
    p->cp_tdx = g->cp_tdx;
    p->cp_tdy = g->cp_tdy;
    p->cp_tx0 = g->cp_tx0;
    p->cp_ty0 = g->cp_ty0;
    p->tcp_numlayers = g->tcp_numlayers;
    for (int i = 0; i < 100; ++i) {
        p->tcp_rates[i] = g->tcp_rates[i];
        p->tcp_distoratio[i] = g->tcp_distoratio[i];
    }
    p->cp_disto_alloc = (int32_t)g->cp_disto_alloc;
    p->cp_fixed_quality = (int32_t)g->cp_fixed_quality;
    // TileProcessor::rate_allocate_encode (TileProcessor.cpp:1661-1677): 0 bisect, anything else feasible
    p->rate_control_algorithm = g->rateControlAlgorithm == 0 ? 0 : 1;
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
    p->framerate = g->framerate > 0 ? (uint32_t)g->framerate : 0;
    p->max_cs_size = g->max_cs_size;
    p->max_comp_size = g->max_comp_size;
    p->cblk_sty = g->cblk_sty;
    if (g->roi_compno >= 0) {
        p->roi_compno = g->roi_compno;
        p->roi_shift = g->roi_shift;
    }
    return true;
}

bool image_desc(const grk_image *img, grkgpu_image_desc *d) {
    if (!img || !img->comps || img->numcomps == 0 || img->numcomps > GRKGPU_MAX_COMPS) {
        GRK_ERROR("image: 1..%d components required", GRKGPU_MAX_COMPS);
        return false;
    }
    memset(d, 0, sizeof(*d));
    d->x0 = img->x0; d->y0 = img->y0; d->x1 = img->x1; d->y1 = img->y1;
    d->numcomps = img->numcomps;
    for (uint32_t k = 0; k < img->numcomps; ++k) {
        const grk_image_comp &c = img->comps[k];
        if (!c.dx || !c.dy || c.dx > 255 || c.dy > 255) { GRK_ERROR("component %u: dx / dy must be 1..255", k); return false; }
        // the component's plane: the image on its subsampled grid (TileComponent.cpp:150-163)
        const uint32_t cw = cdiv(img->x1, c.dx) - cdiv(img->x0, c.dx), ch = cdiv(img->y1, c.dy) - cdiv(img->y0, c.dy);
        if (c.w != cw || c.h != ch) {
            GRK_ERROR("component %u size differs from the image's on its grid", k);
            return false;
        }
        d->dx[k] = c.dx;
        d->dy[k] = c.dy;
        if (!c.data) { GRK_ERROR("component %u has no data", k); return false; }
        d->prec[k] = c.prec;
        d->sgnd[k] = (int32_t)c.sgnd;
    }
    return true;
}

}  // namespace

// ---------------------------------------------------------------------------
// library
// ---------------------------------------------------------------------------
GRK_EXPORT const char *grk_version(void) { return "5.1.0"; }

GRK_EXPORT bool grk_initialize(const char *, uint32_t) { return false; }  // "plugin loaded" (grok.cpp:152-160): none

GRK_EXPORT void grk_deinitialize(void) {
    // idle contexts go now; a context leased by a grk_encode / grk_decode
    // still running on another thread is destroyed when that call returns it
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto *c : g_all) {
        bool idle = false;
        for (auto &f : g_free) idle = idle || std::find(f.begin(), f.end(), c) != f.end();
        if (idle) grkgpu_destroy(c);
        else g_retired.push_back(c);
    }
    g_all.clear();
    g_free.clear();
    grkgpu_multi_release();  // the multi-device calls' pooled contexts
}

// The device workers of a call: grk_cparameters.deviceId for an encode
// (-1 = all devices, grok.h:565, grk_compress.cpp:423-426); a decode's
// grk_dparameters carry no device (grok.h:693-738; grk_decompress -G reaches
// only a plugin, grk_decompress.cpp:1227-1230), so it runs on device 0
// unless GRKGPU_DEVICES lists its workers.  Several workers shard the tiles
// (grkgpu_compress_multi / grkgpu_decompress_multi).
static bool device_set(int device, grkgpu_device_set *ds) {
    if (device < -1) device = 0;
    if (grkgpu_device_set_for(device, ds) != GRKGPU_OK) {
        GRK_ERROR("%s", grkgpu_last_error());
        return false;
    }
    return true;
}
static int decode_device() { return getenv("GRKGPU_DEVICES") ? -1 : 0; }

// ---------------------------------------------------------------------------
// images (image.cpp grk_image_create / grok.cpp:760-797)
// ---------------------------------------------------------------------------
GRK_EXPORT void grk_image_single_component_data_free(grk_image_comp *comp) {
    if (!comp || !comp->data || !comp->owns_data) return;
    free(comp->data);
    comp->data = nullptr;
    comp->owns_data = false;
}

GRK_EXPORT bool grk_image_single_component_data_alloc(grk_image_comp *comp) {
    if (!comp) return false;
    const size_t n = (size_t)comp->w * comp->h * sizeof(int32_t);
    void *p = nullptr;
    if (posix_memalign(&p, 64, n ? n : 64)) return false;
    grk_image_single_component_data_free(comp);
    comp->data = (int32_t *)p;
    comp->owns_data = true;
    return true;
}

GRK_EXPORT void grk_image_all_components_data_free(grk_image *image) {
    if (!image || !image->comps) return;
    for (uint32_t k = 0; k < image->numcomps; ++k) grk_image_single_component_data_free(image->comps + k);
}

GRK_EXPORT grk_image *grk_image_create(uint32_t numcmpts, grk_image_cmptparm *cmptparms, GRK_COLOR_SPACE clrspc) {
    if (!numcmpts || !cmptparms) return nullptr;
    grk_image *img = (grk_image *)calloc(1, sizeof(grk_image));
    if (!img) return nullptr;
    img->color_space = clrspc;
    img->numcomps = numcmpts;
    img->comps = (grk_image_comp *)calloc(numcmpts, sizeof(grk_image_comp));
    if (!img->comps) { free(img); return nullptr; }
    for (uint32_t k = 0; k < numcmpts; ++k) {
        grk_image_comp &c = img->comps[k];
        const grk_image_cmptparm &p = cmptparms[k];
        c.dx = p.dx; c.dy = p.dy; c.w = p.w; c.h = p.h; c.x0 = p.x0; c.y0 = p.y0;
        c.prec = p.prec; c.sgnd = p.sgnd;
        if (!grk_image_single_component_data_alloc(&c)) {
            grk_image_all_components_data_free(img);
            free(img->comps);
            free(img);
            return nullptr;
        }
        memset(c.data, 0, (size_t)c.w * c.h * 4);
    }
    return img;
}

GRK_EXPORT void grk_image_destroy(grk_image *image) {
    if (!image) return;
    grk_image_all_components_data_free(image);
    free(image->comps);
    free(image->icc_profile_buf);
    free(image->iptc_buf);
    free(image->xmp_buf);
    free(image);
}

GRK_EXPORT uint8_t *grk_buffer_new(size_t len) { return new uint8_t[len]; }
GRK_EXPORT void grk_buffer_delete(uint8_t *buffer) { delete[] buffer; }

// ---------------------------------------------------------------------------
// streams
// ---------------------------------------------------------------------------
GRK_EXPORT grk_stream *grk_stream_create(size_t buffer_size, bool is_input) {
    Stream *s = new Stream();
    s->input = is_input;
    s->buffer_size = buffer_size;
    return (grk_stream *)s;
}

GRK_EXPORT void grk_stream_destroy(grk_stream *stream) {
    Stream *s = (Stream *)stream;
    if (!s) return;
    if (s->free_user && s->user) s->free_user(s->user);
    delete s;
}

GRK_EXPORT void grk_stream_set_read_function(grk_stream *stream, grk_stream_read_fn fn) {
    if (stream && ((Stream *)stream)->input) ((Stream *)stream)->read = fn;
}
GRK_EXPORT void grk_stream_set_zero_copy_read_function(grk_stream *stream, grk_stream_zero_copy_read_fn fn) {
    if (stream && ((Stream *)stream)->input) ((Stream *)stream)->zc_read = fn;
}
GRK_EXPORT void grk_stream_set_write_function(grk_stream *stream, grk_stream_write_fn fn) {
    if (stream && !((Stream *)stream)->input) ((Stream *)stream)->write = fn;
}
GRK_EXPORT void grk_stream_set_seek_function(grk_stream *stream, grk_stream_seek_fn fn) {
    if (stream) ((Stream *)stream)->seek = fn;
}
GRK_EXPORT void grk_stream_set_user_data(grk_stream *stream, void *data, grk_stream_free_user_data_fn fn) {
    if (!stream) return;
    ((Stream *)stream)->user = data;
    ((Stream *)stream)->free_user = fn;
}
GRK_EXPORT void grk_stream_set_user_data_length(grk_stream *stream, uint64_t len) {
    if (stream) ((Stream *)stream)->user_len = len;
}

GRK_EXPORT grk_stream *grk_stream_create_mem_stream(uint8_t *buf, size_t len, bool owns, bool is_read) {
    if (!buf || !len) return nullptr;
    Stream *s = (Stream *)grk_stream_create(len, is_read);
    MemBuf *m = new MemBuf();
    m->buf = buf;
    m->len = len;
    m->owns = owns;
    s->mem = m;
    s->user = m;
    s->free_user = mem_free;
    s->user_len = len;
    if (is_read) s->read = mem_read;
    else s->write = mem_write;
    s->seek = mem_seek;
    return (grk_stream *)s;
}

GRK_EXPORT size_t grk_stream_get_write_mem_stream_length(grk_stream *stream) {
    Stream *s = (Stream *)stream;
    return s && s->mem && !s->input ? s->mem->high : 0;
}

GRK_EXPORT grk_stream *grk_stream_create_file_stream(const char *fname, size_t buffer_size, bool is_read) {
    if (!fname) return nullptr;
    FILE *f = fopen(fname, is_read ? "rb" : "wb");
    if (!f) return nullptr;
    Stream *s = (Stream *)grk_stream_create(buffer_size, is_read);
    s->user = f;
    s->free_user = file_free;
    if (is_read) {
        s->read = file_read;
        struct stat st;
        if (fstat(fileno(f), &st) == 0) s->user_len = (uint64_t)st.st_size;
    } else {
        s->write = file_write;
    }
    s->seek = file_seek;
    return (grk_stream *)s;
}

GRK_EXPORT grk_stream *grk_stream_create_mapped_file_read_stream(const char *fname) {
    if (!fname) return nullptr;
    const int fd = open(fname, O_RDONLY);
    if (fd < 0) return nullptr;
    struct stat st;
    if (fstat(fd, &st) || st.st_size <= 0) { close(fd); return nullptr; }
    void *p = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return nullptr;
    Stream *s = (Stream *)grk_stream_create((size_t)st.st_size, true);
    MemBuf *m = new MemBuf();
    m->buf = (uint8_t *)p;
    m->len = (size_t)st.st_size;
    m->map = p;
    s->mem = m;
    s->user = m;
    s->free_user = mem_free;
    s->read = mem_read;
    s->seek = mem_seek;
    s->user_len = m->len;
    return (grk_stream *)s;
}

// ---------------------------------------------------------------------------
// messages
// ---------------------------------------------------------------------------
GRK_EXPORT bool grk_set_info_handler(grk_msg_callback cb, void *u) { g_info = {cb, u}; return true; }
GRK_EXPORT bool grk_set_warning_handler(grk_msg_callback cb, void *u) { g_warn = {cb, u}; return true; }
GRK_EXPORT bool grk_set_error_handler(grk_msg_callback cb, void *u) { g_err = {cb, u}; return true; }

// ---------------------------------------------------------------------------
// decompression
// ---------------------------------------------------------------------------
GRK_EXPORT grk_codec *grk_create_decompress(GRK_CODEC_FORMAT format, grk_stream *stream) {
    if (format != GRK_CODEC_J2K) { GRK_ERROR("only raw J2K codestreams are supported (no JP2)"); return nullptr; }
    if (!stream) return nullptr;
    Codec *c = new Codec();
    c->decompressor = true;
    c->stream = (Stream *)stream;
    grk_set_default_decoder_parameters(&c->dparams);
    return (grk_codec *)c;
}

GRK_EXPORT void grk_destroy_codec(grk_codec *codec) { delete (Codec *)codec; }

GRK_EXPORT void grk_set_default_decoder_parameters(grk_dparameters *p) {
    if (p) memset(p, 0, sizeof(*p));
}

// The tile-streaming caches (grk_read_tile_header's tile sequence, clipped to
// the decode area; grk_decode_tile_data's reduced-resolution image) follow
// the decode area and parameters: dropped whenever either is set again.
static void reset_tile_caches(Codec *c) {
    c->tile_order.clear();
    c->tile_order_ready = false;
    c->tile_pos = 0;
    c->reduced.clear();
}

GRK_EXPORT bool grk_setup_decoder(grk_codec *codec, grk_dparameters *p) {
    Codec *c = (Codec *)codec;
    if (!c || !p) return false;
    if (!c->decompressor) { GRK_ERROR("Codec provided to grk_setup_decoder is not a decompressor handler."); return false; }
    c->dparams = *p;
    reset_tile_caches(c);  // reduce / layers may have changed
    return true;
}

// j2k_read_header: the image from SIZ (grid coordinates, one component per
// SIZ entry, no sample buffers yet) + the main header's coding parameters
GRK_EXPORT bool grk_read_header(grk_codec *codec, grk_header_info *hi, grk_image **image) {
    Codec *c = (Codec *)codec;
    if (!c || !c->decompressor || !image) return false;
    if (!c->have_header) {
        if (!c->stream->read_all(c->cs) || c->cs.empty()) { GRK_ERROR("empty stream"); return false; }
        if (grkgpu_read_header(c->cs.data(), c->cs.size(), &c->desc) ||
            grkgpu_read_header_info(c->cs.data(), c->cs.size(), &c->hinfo)) {
            GRK_ERROR("%s", grkgpu_last_error());
            return false;
        }
        c->cinfo.assign(c->desc.numcomps, grkgpu_comp_info{});
        for (uint32_t k = 0; k < c->desc.numcomps; ++k)
            if (grkgpu_read_comp_info(c->cs.data(), c->cs.size(), k, &c->cinfo[k])) {
                GRK_ERROR("%s", grkgpu_last_error());
                return false;
            }
        c->have_header = true;
    }
    if (c->dparams.cp_reduce >= c->hinfo.numresolutions) {  // j2k.cpp:6994
        GRK_ERROR("Error decoding component: the number of resolutions to remove is higher than the number of "
                  "resolutions of this component");
        return false;
    }
    const grkgpu_image_desc &d = c->desc;
    grk_image *img = (grk_image *)calloc(1, sizeof(grk_image));
    img->comps = (grk_image_comp *)calloc(d.numcomps, sizeof(grk_image_comp));
    img->numcomps = d.numcomps;
    img->x0 = d.x0; img->y0 = d.y0; img->x1 = d.x1; img->y1 = d.y1;
    img->color_space = GRK_CLRSPC_UNKNOWN;  // a raw codestream carries none (JP2 colr box)
    const uint32_t r = c->dparams.cp_reduce;
    for (uint32_t k = 0; k < d.numcomps; ++k) {
        grk_image_comp &cp = img->comps[k];
        cp.dx = d.dx[k];
        cp.dy = d.dy[k];
        cp.prec = d.prec[k];
        cp.sgnd = (uint32_t)d.sgnd[k];
        // grk_image_comp_header_update (image.cpp:124-155): the origin on the
        // component grid, the size at the decoded resolution
        cp.x0 = cdiv(d.x0, cp.dx);
        cp.y0 = cdiv(d.y0, cp.dy);
        cp.w = cdivpow2(cdiv(d.x1, cp.dx) - cp.x0, r);
        cp.h = cdivpow2(cdiv(d.y1, cp.dy) - cp.y0, r);
    }
    *image = img;
    if (hi) {
        memset(hi, 0, sizeof(*hi));
        const grkgpu_header_info &h = c->hinfo;
        hi->cblockw_init = h.cblockw_init;
        hi->cblockh_init = h.cblockh_init;
        hi->irreversible = h.irreversible != 0;
        hi->mct = h.mct;
        hi->rsiz = (uint16_t)h.rsiz;
        hi->numresolutions = h.numresolutions;
        hi->csty = (uint8_t)c->cinfo[0].csty;  // tccps[0]->csty: the precinct flag (j2k.cpp:461)
        hi->cblk_sty = (uint8_t)h.cblk_sty;
        for (int i = 0; i < 33; ++i) { hi->prcw_init[i] = h.prcw_init[i]; hi->prch_init[i] = h.prch_init[i]; }
        hi->cp_tx0 = h.tx0; hi->cp_ty0 = h.ty0; hi->cp_tdx = h.tdx; hi->cp_tdy = h.tdy;
        hi->cp_tw = h.tw; hi->cp_th = h.th;
        hi->tcp_numlayers = h.numlayers;
    }
    return true;
}

// j2k_set_decode_area: all zero = the whole image; else the area clipped to
// the image becomes the image (and component) bounds
GRK_EXPORT bool grk_set_decode_area(grk_codec *codec, grk_image *image, uint32_t x0, uint32_t y0, uint32_t x1,
                                    uint32_t y1) {
    Codec *c = (Codec *)codec;
    if (!c || !c->decompressor || !c->have_header || !image) return false;
    reset_tile_caches(c);  // the tile sequence is clipped to the area
    if (!x0 && !y0 && !x1 && !y1) {
        c->window = false;
        return true;
    }
    const grkgpu_image_desc &d = c->desc;
    if (x0 >= d.x1 || y0 >= d.y1 || x1 <= d.x0 || y1 <= d.y0 || x1 <= x0 || y1 <= y0) {
        GRK_ERROR("decode area (%u,%u,%u,%u) outside the image", x0, y0, x1, y1);
        return false;
    }
    c->window = true;
    c->win[0] = std::max(x0, d.x0); c->win[1] = std::max(y0, d.y0);
    c->win[2] = std::min(x1, d.x1); c->win[3] = std::min(y1, d.y1);
    image->x0 = c->win[0]; image->y0 = c->win[1]; image->x1 = c->win[2]; image->y1 = c->win[3];
    // update_image_dimensions (image.cpp:207-246): the component origin on its
    // grid at full resolution, its size at the decoded one
    const uint32_t r = c->dparams.cp_reduce;
    for (uint32_t k = 0; k < image->numcomps; ++k) {
        grk_image_comp &cp = image->comps[k];
        comp_geom(cp, c->win[0], c->win[1], c->win[2], c->win[3], r);
        cp.x0 = cdiv(c->win[0], cp.dx ? cp.dx : 1);
        cp.y0 = cdiv(c->win[1], cp.dy ? cp.dy : 1);
    }
    return true;
}

GRK_EXPORT bool grk_decode(grk_codec *codec, grk_plugin_tile *, grk_image *image) {
    Codec *c = (Codec *)codec;
    if (!c || !c->decompressor || !c->have_header || !image || image->numcomps != c->desc.numcomps) return false;
    grkgpu_device_set ds;
    if (!device_set(decode_device(), &ds)) return false;
    std::vector<int32_t *> planes(image->numcomps);
    // The planes take the extent the decode writes under the current settings
    // (cp_reduce and the decode area may have changed since grk_read_header /
    // grk_set_decode_area filled the image in): grk_image_comp_header_update
    // (image.cpp:124-155) without an area, update_image_dimensions
    // (image.cpp:207-246) with one -- the decoder's own output geometry, so
    // a stale w / h can never make it write past a plane.
    const uint32_t r = c->dparams.cp_reduce;
    if (r >= c->hinfo.numresolutions) {
        GRK_ERROR("Error decoding component: the number of resolutions to remove is higher than the number of "
                  "resolutions of this component");
        return false;
    }
    const grkgpu_image_desc &d = c->desc;
    for (uint32_t k = 0; k < image->numcomps; ++k) {
        grk_image_comp &cp = image->comps[k];
        cp.dx = d.dx[k];
        cp.dy = d.dy[k];
        if (c->window) {
            comp_geom(cp, c->win[0], c->win[1], c->win[2], c->win[3], r);
            cp.x0 = cdiv(c->win[0], cp.dx);
            cp.y0 = cdiv(c->win[1], cp.dy);
        } else {
            cp.x0 = cdiv(d.x0, cp.dx);
            cp.y0 = cdiv(d.y0, cp.dy);
            cp.w = cdivpow2(cdiv(d.x1, cp.dx) - cp.x0, r);
            cp.h = cdivpow2(cdiv(d.y1, cp.dy) - cp.y0, r);
        }
        if (!grk_image_single_component_data_alloc(&cp)) return false;
        planes[k] = cp.data;
    }
    grkgpu_dparams dp{c->dparams.cp_reduce, c->dparams.cp_layer, 0, 0, 0, 0};
    if (c->window) { dp.DA_x0 = c->win[0]; dp.DA_y0 = c->win[1]; dp.DA_x1 = c->win[2]; dp.DA_y1 = c->win[3]; }
    if (ds.n > 1 && !c->window && !dp.cp_reduce && !dp.cp_layer) {  // tile shards over the device workers
        if (grkgpu_decompress_multi(&ds, c->cs.data(), c->cs.size(), nullptr, planes.data())) {
            GRK_ERROR("%s", grkgpu_last_error());
            return false;
        }
    } else {
        Lease lease(ds.dev[0]);
        if (!lease.ctx) return false;
        if (grkgpu_decompress_ex(lease.ctx, c->cs.data(), c->cs.size(), &dp, nullptr, planes.data(), 0)) {
            GRK_ERROR("%s", grkgpu_last_error());
            return false;
        }
    }
    for (uint32_t k = 0; k < image->numcomps; ++k)
        image->comps[k].resno_decoded = c->hinfo.numresolutions - 1 - c->dparams.cp_reduce;
    c->decoded = true;
    return true;
}

// one tile (j2k_get_tile): the tile's rectangle decoded as a window
GRK_EXPORT bool grk_get_decoded_tile(grk_codec *codec, grk_image *image, uint16_t tile_index) {
    Codec *c = (Codec *)codec;
    if (!c || !c->decompressor || !c->have_header || !image) return false;
    const grkgpu_header_info &h = c->hinfo;
    if (tile_index >= h.tw * h.th) { GRK_ERROR("tile index %u out of range", tile_index); return false; }
    const grkgpu_image_desc &d = c->desc;
    const uint32_t p = tile_index % h.tw, q = tile_index / h.tw;
    const uint32_t x0 = std::max(d.x0, h.tx0 + p * h.tdx), y0 = std::max(d.y0, h.ty0 + q * h.tdy);
    const uint32_t x1 = std::min(d.x1, h.tx0 + (p + 1) * h.tdx), y1 = std::min(d.y1, h.ty0 + (q + 1) * h.tdy);
    return grk_set_decode_area(codec, image, x0, y0, x1, y1) && grk_decode(codec, nullptr, image);
}

GRK_EXPORT bool grk_end_decompress(grk_codec *codec) { return codec && ((Codec *)codec)->decompressor; }

// Tile order of the codestream: the tile of each first tile-part, in stream
// order (j2k_read_tile_header reads SOT after SOT, j2k.cpp:627-960), from the
// first SOT after the main header, following Psot (0: to the end).
static std::vector<uint32_t> stream_tile_order(const std::vector<uint8_t> &cs, uint32_t ntiles) {
    std::vector<uint32_t> order;
    std::vector<uint8_t> seen(ntiles, 0);
    auto rd16 = [&](size_t p) { return (uint32_t)cs[p] << 8 | cs[p + 1]; };
    size_t pos = 2;  // after SOC
    while (pos + 4 <= cs.size() && rd16(pos) != 0xFF90) pos += 2 + rd16(pos + 2);
    while (pos + 12 <= cs.size() && rd16(pos) == 0xFF90) {
        const uint32_t isot = rd16(pos + 4);
        const uint32_t psot = rd16(pos + 6) << 16 | rd16(pos + 8);
        if (isot < ntiles && !seen[isot]) {
            seen[isot] = 1;
            order.push_back(isot);
        }
        if (!psot) break;
        pos += psot;
    }
    return order;
}

// the decoded rectangle of tile t: its extent at the decoded resolution
// (TileComponent.cpp:560-582 reduced_image_dim), clipped to the decode area
// when `clip` -- the area only selects tiles: the reference still sizes and
// fills the whole reduced tile (get_tile_size(true) with a decode area set
// reports the full tile, tests/golden/tiles.json)
static TileRect tile_decoded_rect(const Codec *c, uint32_t t, bool clip) {
    const grkgpu_header_info &h = c->hinfo;
    const TileRect tr = tile_rect(t, h.tw, h.tx0, h.ty0, h.tdx, h.tdy, c->desc);
    const uint32_t r = c->dparams.cp_reduce;
    TileRect o{cdivpow2(tr.x0, r), cdivpow2(tr.y0, r), cdivpow2(tr.x1, r), cdivpow2(tr.y1, r)};
    if (clip && c->window) {
        o.x0 = std::max(o.x0, c->win[0]); o.y0 = std::max(o.y0, c->win[1]);
        o.x1 = std::min(o.x1, c->win[2]); o.y1 = std::min(o.y1, c->win[3]);
        if (o.x1 < o.x0) o.x1 = o.x0;
        if (o.y1 < o.y0) o.y1 = o.y0;
    }
    return o;
}

// rectangle o (reference grid, decoded resolution) on component k's grid:
// ceil(x / dx) (the nested ceilings of a reduced decode commute)
static TileRect comp_tile_rect(const Codec *c, const TileRect &o, uint32_t k) {
    const uint32_t dx = c->desc.dx[k] ? c->desc.dx[k] : 1, dy = c->desc.dy[k] ? c->desc.dy[k] : 1;
    return {cdiv(o.x0, dx), cdiv(o.y0, dy), cdiv(o.x1, dx), cdiv(o.y1, dy)};
}

// get_tile_size(true) (TileProcessor.cpp:1435-1447): every component's
// tile-component at the decoded resolution, at its sample width
static uint64_t tile_data_bytes(const Codec *c, const TileRect &o) {
    uint64_t n = 0;
    for (uint32_t k = 0; k < c->desc.numcomps; ++k) {
        const TileRect r = comp_tile_rect(c, o, k);
        n += (uint64_t)((c->desc.prec[k] + 7) >> 3) * (r.x1 - r.x0) * (r.y1 - r.y0);
    }
    return n;
}

// grk_read_tile_header (grok.cpp:408-423, j2k.cpp:627-960): the next tile of
// the codestream (tiles that miss the decode area are stepped over), its
// rectangle, component count and the bytes grk_decode_tile_data writes
// (TileProcessor::get_tile_size(true), TileProcessor.cpp:1435-1447);
// *go_on = false once the codestream has no tile left.
GRK_EXPORT bool grk_read_tile_header(grk_codec *codec, uint16_t *tile_index, uint64_t *data_size, uint32_t *x0,
                                     uint32_t *y0, uint32_t *x1, uint32_t *y1, uint32_t *nb_comps, bool *go_on) {
    Codec *c = (Codec *)codec;
    if (!c || !c->decompressor || !c->have_header || !tile_index || !data_size) return false;
    const grkgpu_header_info &h = c->hinfo;
    if (!c->tile_order_ready) {
        for (uint32_t t : stream_tile_order(c->cs, h.tw * h.th)) {
            const TileRect o = tile_decoded_rect(c, t, true);
            if (o.x1 > o.x0 && o.y1 > o.y0) c->tile_order.push_back(t);
        }
        c->tile_order_ready = true;
        c->tile_pos = 0;
    }
    if (c->tile_pos >= c->tile_order.size()) {
        if (go_on) *go_on = false;
        c->cur_tile = -1;
        return true;
    }
    const uint32_t t = c->tile_order[c->tile_pos++];
    const TileRect tr = tile_rect(t, h.tw, h.tx0, h.ty0, h.tdx, h.tdy, c->desc);
    c->cur_tile = t;
    *tile_index = (uint16_t)t;
    *data_size = tile_data_bytes(c, tile_decoded_rect(c, t, false));
    if (x0) *x0 = tr.x0;
    if (y0) *y0 = tr.y0;
    if (x1) *x1 = tr.x1;
    if (y1) *y1 = tr.y1;
    if (nb_comps) *nb_comps = c->desc.numcomps;
    if (go_on) *go_on = true;
    return true;
}

// grk_decode_tile_data (grok.cpp:425-440, j2k.cpp:979-1060): the tile read
// by grk_read_tile_header, decoded into data as TileProcessor::update_tile_data
// lays it out (TileProcessor.cpp:1201-1258): planar components, 1 or 2 bytes
// per sample by precision (signed: the value, unsigned: masked).  At full
// resolution the tile is a window decode of its rectangle (only its
// code-blocks); at a reduced resolution the image is decoded once and each
// tile cropped from it.  With a decode area set, the whole tile is decoded:
// the reference's samples there are not the tile's (most code-blocks come out
// as zero coefficients -- a reference defect, DESIGN.md "Tile streaming"), so
// parity is pinned on the reference's decode without an area, which equals
// its grk_get_decoded_tile.
GRK_EXPORT bool grk_decode_tile_data(grk_codec *codec, uint16_t tile_index, uint8_t *data, uint64_t data_size) {
    Codec *c = (Codec *)codec;
    if (!c || !c->decompressor || !data || c->cur_tile != (int64_t)tile_index) return false;
    const TileRect o = tile_decoded_rect(c, tile_index, false);
    const uint64_t need = tile_data_bytes(c, o);
    if (need > data_size) return false;
    const uint32_t nc = c->desc.numcomps;
    // per component: its samples of the tile (tile-component rectangle ct[k])
    // read from a plane whose first row / column is (px0[k], py0[k]), stride pst[k]
    TileRect ct[GRKGPU_MAX_COMPS];
    for (uint32_t k = 0; k < nc; ++k) ct[k] = comp_tile_rect(c, o, k);
    std::vector<int32_t> buf;
    const int32_t *pl[GRKGPU_MAX_COMPS];
    uint32_t pst[GRKGPU_MAX_COMPS], px0[GRKGPU_MAX_COMPS], py0[GRKGPU_MAX_COMPS];
    {
        Lease lease(0);
        if (!lease.ctx) return false;
        if (c->dparams.cp_reduce == 0) {  // the tile as a decode window: plane k = its tile-component
            uint64_t tot = 0;
            for (uint32_t k = 0; k < nc; ++k) tot += (uint64_t)(ct[k].x1 - ct[k].x0) * (ct[k].y1 - ct[k].y0);
            buf.resize(tot);
            std::vector<int32_t *> planes(nc);
            uint64_t off = 0;
            for (uint32_t k = 0; k < nc; ++k) {
                planes[k] = buf.data() + off;
                pl[k] = planes[k];
                pst[k] = ct[k].x1 - ct[k].x0;
                px0[k] = ct[k].x0;
                py0[k] = ct[k].y0;
                off += (uint64_t)pst[k] * (ct[k].y1 - ct[k].y0);
            }
            grkgpu_dparams dp{0, c->dparams.cp_layer, o.x0, o.y0, o.x1, o.y1};
            if (grkgpu_decompress_ex(lease.ctx, c->cs.data(), c->cs.size(), &dp, nullptr, planes.data(), 0)) {
                GRK_ERROR("%s", grkgpu_last_error());
                return false;
            }
        } else {  // the whole reduced image once, then each tile cut out of it
            const uint32_t r = c->dparams.cp_reduce;
            const grkgpu_image_desc &dd = c->desc;
            uint64_t roff[GRKGPU_MAX_COMPS + 1];
            roff[0] = 0;
            uint32_t rw[GRKGPU_MAX_COMPS];
            for (uint32_t k = 0; k < nc; ++k) {  // grk_image_comp_header_update's plane sizes
                const uint32_t dx = dd.dx[k] ? dd.dx[k] : 1, dy = dd.dy[k] ? dd.dy[k] : 1;
                rw[k] = cdivpow2(cdiv(dd.x1, dx) - cdiv(dd.x0, dx), r);
                const uint32_t rh = cdivpow2(cdiv(dd.y1, dy) - cdiv(dd.y0, dy), r);
                roff[k + 1] = roff[k] + (uint64_t)rw[k] * rh;
            }
            if (c->reduced.empty()) {
                grkgpu_image_desc d{};
                grkgpu_dparams dp{r, c->dparams.cp_layer, 0, 0, 0, 0};
                c->reduced.resize(roff[nc]);
                std::vector<int32_t *> planes(nc);
                for (uint32_t k = 0; k < nc; ++k) planes[k] = c->reduced.data() + roff[k];
                if (grkgpu_decompress_ex(lease.ctx, c->cs.data(), c->cs.size(), &dp, &d, planes.data(), 0)) {
                    GRK_ERROR("%s", grkgpu_last_error());
                    c->reduced.clear();
                    return false;
                }
                c->reduced_desc = d;
            }
            const grkgpu_image_desc &d = c->reduced_desc;  // the reduced image (reference grid)
            for (uint32_t k = 0; k < nc; ++k) {
                const TileRect org = comp_tile_rect(c, {d.x0, d.y0, d.x1, d.y1}, k);
                pl[k] = c->reduced.data() + roff[k];
                pst[k] = rw[k];
                px0[k] = org.x0;
                py0[k] = org.y0;
            }
        }
    }
    uint8_t *dst = data;
    for (uint32_t k = 0; k < nc; ++k) {
        const uint32_t sz = (c->desc.prec[k] + 7) >> 3;
        const bool sg = c->desc.sgnd[k] != 0;
        const uint32_t w = ct[k].x1 - ct[k].x0, h = ct[k].y1 - ct[k].y0;
        const int32_t *p = pl[k] + (uint64_t)(ct[k].y0 - py0[k]) * pst[k] + (ct[k].x0 - px0[k]);
        for (uint32_t y = 0; y < h; ++y, p += pst[k])
            for (uint32_t x = 0; x < w; ++x) {
                const int32_t v = p[x];
                if (sz == 1) *dst++ = (uint8_t)(sg ? (int8_t)v : (int8_t)(v & 0xff));
                else {
                    const uint16_t u = (uint16_t)(sg ? (int16_t)v : (int16_t)(v & 0xffff));
                    memcpy(dst, &u, 2);
                    dst += 2;
                }
            }
    }
    return true;
}

// ---------------------------------------------------------------------------
// compression
// ---------------------------------------------------------------------------
GRK_EXPORT grk_codec *grk_create_compress(GRK_CODEC_FORMAT format, grk_stream *stream) {
    if (format != GRK_CODEC_J2K) { GRK_ERROR("only raw J2K codestreams are supported (no JP2)"); return nullptr; }
    if (!stream) return nullptr;
    Codec *c = new Codec();
    c->stream = (Stream *)stream;
    return (grk_codec *)c;
}

GRK_EXPORT void grk_set_default_encoder_parameters(grk_cparameters *p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->numresolution = 6;       // GRK_COMP_PARAM_DEFAULT_NUMRESOLUTION
    p->cblockw_init = 64;       // GRK_COMP_PARAM_DEFAULT_CBLOCKW / H
    p->cblockh_init = 64;
    p->prog_order = 0;          // GRK_LRCP
    p->roi_compno = -1;
    p->subsampling_dx = 1;
    p->subsampling_dy = 1;
    p->numThreads = (uint32_t)std::max<long>(1, sysconf(_SC_NPROCESSORS_ONLN));
    p->deviceId = 0;
    p->repeats = 1;
}

GRK_EXPORT bool grk_setup_encoder(grk_codec *codec, grk_cparameters *p, grk_image *image) {
    Codec *c = (Codec *)codec;
    if (!c || c->decompressor || !p || !image) return false;
    grkgpu_cparams tmp;
    if (!map_cparams(p, image->numcomps, &tmp)) return false;
    c->cparams = *p;
    if (p->mct_data) {  // the codec's own copy from here on (j2k.cpp:1899-1956, 2052-2055)
        const size_t n = image->numcomps, bytes = n * n * sizeof(float) + n * sizeof(int32_t);
        c->mct.assign((const uint8_t *)p->mct_data, (const uint8_t *)p->mct_data + bytes);
        c->cparams.mct_data = c->mct.data();
        std::lock_guard<std::mutex> lk(g_mct_mu);
        if (g_mct_n.erase(p->mct_data)) {
            free(p->mct_data);
            p->mct_data = nullptr;
        }
    }
    c->image = image;
    c->setup = true;
    return true;
}

GRK_EXPORT bool grk_start_compress(grk_codec *codec, grk_image *image) {
    Codec *c = (Codec *)codec;
    if (!c || c->decompressor || !c->setup) return false;
    if (image) c->image = image;
    return c->image != nullptr;
}

GRK_EXPORT bool grk_encode_with_plugin(grk_codec *codec, grk_plugin_tile *tile) {
    Codec *c = (Codec *)codec;
    if (!c || c->decompressor || !c->setup || !c->image) return false;
    if (tile) { GRK_ERROR("plugin tiles are not taken by this library"); return false; }
    grkgpu_image_desc d;
    grkgpu_cparams p;
    if (!image_desc(c->image, &d) || !map_cparams(&c->cparams, d.numcomps, &p)) return false;
    grkgpu_device_set ds;
    if (!device_set(c->cparams.deviceId, &ds)) return false;
    std::vector<const int32_t *> planes(d.numcomps);
    for (uint32_t k = 0; k < d.numcomps; ++k) planes[k] = c->image->comps[k].data;
    if (ds.n > 1) {  // deviceId -1: the tiles sharded over the device workers
        grkgpu_planes pl{};
        for (uint32_t k = 0; k < d.numcomps; ++k) pl.planes[k] = planes[k];
        pl.sample_fmt = GRKGPU_SAMPLE_I32;
        uint8_t *mo = nullptr;
        size_t ml = 0;
        if (grkgpu_compress_multi(&ds, &d, &p, &pl, &mo, &ml)) {
            GRK_ERROR("%s", grkgpu_last_error());
            return false;
        }
        const bool ok = c->stream->write_all(mo, ml);
        grkgpu_free(mo);
        if (!ok) { GRK_ERROR("stream write failed"); return false; }
        return true;
    }
    Lease lease(ds.dev[0]);  // held until the codestream is written out of the context's buffer
    grkgpu_ctx *ctx = lease.ctx;
    if (!ctx) return false;
    const uint8_t *out = nullptr;
    size_t len = 0;
    if (grkgpu_compress_view(ctx, &d, &p, planes.data(), 0, &out, &len)) {
        GRK_ERROR("%s", grkgpu_last_error());
        return false;
    }
    if (!c->stream->write_all(out, len)) { GRK_ERROR("stream write failed"); return false; }
    return true;
}

GRK_EXPORT bool grk_encode(grk_codec *codec) { return grk_encode_with_plugin(codec, nullptr); }

// grk_end_compress: after tile streaming, the EOC (j2k_end_encoding,
// j2k.cpp:2234-2247; a single-tile stream was finished by its write_tile)
GRK_EXPORT bool grk_end_compress(grk_codec *codec) {
    Codec *c = (Codec *)codec;
    if (!c || c->decompressor) return false;
    if (c->header_written && !c->eoc_written) {
        const uint8_t eoc[2] = {0xFF, 0xD9};
        if (!c->stream->write_all(eoc, 2)) { GRK_ERROR("stream write failed"); return false; }
        c->eoc_written = true;
    }
    return true;
}

// grk_write_tile (grok.cpp:631-645, j2k.cpp:2763-2795): tile tile_index's
// samples -- planar components, tile width x height each, 1 or 2 bytes per
// sample by precision (TileProcessor::copy_image_data_to_tile,
// TileProcessor.cpp:1923-1972) -- encoded on the GPU and its tile-parts
// written to the stream; tiles in order 0 .. n-1.  The main header goes out
// with the first tile (it is the same for every tile), the EOC at
// grk_end_compress; a single-tile image is coded whole by its one
// write_tile (its TLM, for the cinema profiles, needs the tile-part lengths).
GRK_EXPORT bool grk_write_tile(grk_codec *codec, uint16_t tile_index, uint8_t *data, uint64_t data_size) {
    Codec *c = (Codec *)codec;
    if (!c || c->decompressor || !c->setup || !c->image || !data) return false;
    grk_image *img = c->image;
    grkgpu_image_desc d{};
    if (!img->comps || !img->numcomps || img->numcomps > GRKGPU_MAX_COMPS) return false;
    d.x0 = img->x0; d.y0 = img->y0; d.x1 = img->x1; d.y1 = img->y1;
    d.numcomps = img->numcomps;
    for (uint32_t k = 0; k < img->numcomps; ++k) {
        d.prec[k] = img->comps[k].prec;
        d.sgnd[k] = (int32_t)img->comps[k].sgnd;
        d.dx[k] = img->comps[k].dx ? img->comps[k].dx : 1;
        d.dy[k] = img->comps[k].dy ? img->comps[k].dy : 1;
    }
    grkgpu_cparams p;
    if (!map_cparams(&c->cparams, d.numcomps, &p)) return false;
    uint32_t ntiles = 0;
    if (grkgpu_num_tiles(&d, &p, &ntiles)) { GRK_ERROR("%s", grkgpu_last_error()); return false; }
    if (tile_index != c->next_tile || tile_index >= ntiles) {
        GRK_ERROR("tiles must be written in order: expected tile %u, got %u", c->next_tile, tile_index);
        return false;
    }
    // one sample width and signedness for all components (what grkgpu_planes carries)
    const uint32_t sz = (d.prec[0] + 7) >> 3;
    for (uint32_t k = 1; k < d.numcomps; ++k)
        if (((d.prec[k] + 7) >> 3) != sz || d.sgnd[k] != d.sgnd[0]) {
            GRK_ERROR("components of different sample sizes are not supported by grk_write_tile");
            return false;
        }
    if (sz > 2) { GRK_ERROR("precision above 16 bits"); return false; }
    const uint32_t tdx = p.tile_size_on ? p.cp_tdx : d.x1 - p.cp_tx0, tdy = p.tile_size_on ? p.cp_tdy : d.y1 - p.cp_ty0;
    const uint32_t tw = (uint32_t)(((uint64_t)d.x1 - p.cp_tx0 + tdx - 1) / tdx);
    const TileRect tr = tile_rect(tile_index, tw, p.cp_tx0, p.cp_ty0, tdx, tdy, d);
    // the tile's data: each component's tile-component (the tile on its grid,
    // ceil(x / dx)), one after the other (TileProcessor::copy_image_data_to_tile,
    // TileProcessor.cpp:1923-1972; get_tile_size(false))
    uint64_t off[GRKGPU_MAX_COMPS + 1];
    off[0] = 0;
    for (uint32_t k = 0; k < d.numcomps; ++k) {
        const uint64_t w = cdiv(tr.x1, d.dx[k]) - cdiv(tr.x0, d.dx[k]), h = cdiv(tr.y1, d.dy[k]) - cdiv(tr.y0, d.dy[k]);
        off[k + 1] = off[k] + w * h * sz;
    }
    if (off[d.numcomps] != data_size) {
        GRK_ERROR("Size mismatch between tile data and sent data.");
        return false;
    }
    grkgpu_planes pl{};
    for (uint32_t k = 0; k < d.numcomps; ++k) pl.planes[k] = data + off[k];
    pl.sample_fmt = sz == 1 ? (d.sgnd[0] ? GRKGPU_SAMPLE_I8 : GRKGPU_SAMPLE_U8)
                            : (d.sgnd[0] ? GRKGPU_SAMPLE_I16 : GRKGPU_SAMPLE_U16);
    pl.on_device = 0;
    pl.row0 = tr.y0 - d.y0;
    pl.nrows = tr.y1 - tr.y0;
    pl.col0 = tr.x0 - d.x0;
    pl.ncols = tr.x1 - tr.x0;
    Lease lease(c->cparams.deviceId);
    if (!lease.ctx) return false;
    const uint8_t *out = nullptr;
    size_t len = 0;
    if (ntiles == 1) {
        if (grkgpu_compress_ex(lease.ctx, &d, &p, &pl, 0, 1, GRKGPU_PART_ALL, &out, &len)) {
            GRK_ERROR("%s", grkgpu_last_error());
            return false;
        }
        c->header_written = c->eoc_written = true;
    } else {
        if (!c->header_written) {
            grkgpu_planes none{};
            none.on_device = 1;  // no samples are read for the header alone
            if (grkgpu_compress_ex(lease.ctx, &d, &p, &none, 0, 0, GRKGPU_PART_HEADER, &out, &len)) {
                GRK_ERROR("%s", grkgpu_last_error());
                return false;
            }
            if (!c->stream->write_all(out, len)) { GRK_ERROR("stream write failed"); return false; }
            c->header_written = true;
        }
        if (grkgpu_compress_ex(lease.ctx, &d, &p, &pl, tile_index, tile_index + 1u, GRKGPU_PART_TILES, &out, &len)) {
            GRK_ERROR("%s", grkgpu_last_error());
            return false;
        }
    }
    if (!c->stream->write_all(out, len)) { GRK_ERROR("stream write failed"); return false; }
    ++c->next_tile;
    return true;
}

// grk_set_MCT (grok.cpp:606-630): Part-2 MCT extension in rsiz, 9/7,
// tcp_mct = 2, mct_data = the n x n encoding matrix followed by n DC shifts
// (owned by the parameters, as there)
GRK_EXPORT bool grk_set_MCT(grk_cparameters *parameters, float *matrix, int32_t *dc_shift, uint32_t n) {
    if (!parameters || !matrix || !dc_shift) return false;
    const size_t msize = (size_t)n * n * sizeof(float), ssize = (size_t)n * sizeof(int32_t);
    if ((parameters->rsiz & 0x8000) != 0) parameters->rsiz |= 0x0100;
    else parameters->rsiz = 0x8000 | 0x0100;
    parameters->irreversible = true;
    parameters->tcp_mct = 2;
    parameters->mct_data = malloc(msize + ssize);
    if (!parameters->mct_data) return false;
    {
        std::lock_guard<std::mutex> lk(g_mct_mu);
        g_mct_n[parameters->mct_data] = n;
    }
    memcpy(parameters->mct_data, matrix, msize);
    memcpy((uint8_t *)parameters->mct_data + msize, dc_shift, ssize);
    return true;
}

// ---------------------------------------------------------------------------
// codestream information
// ---------------------------------------------------------------------------
GRK_EXPORT void grk_dump_codec(grk_codec *codec, int32_t, FILE *out) {
    Codec *c = (Codec *)codec;
    if (!c || !out || !c->have_header) return;
    const grkgpu_header_info &h = c->hinfo;
    const grkgpu_image_desc &d = c->desc;
    fprintf(out, "Image info {\n\t x0=%u, y0=%u\n\t x1=%u, y1=%u\n\t numcomps=%u\n", d.x0, d.y0, d.x1, d.y1, d.numcomps);
    for (uint32_t k = 0; k < d.numcomps; ++k) fprintf(out, "\t component %u: prec=%u sgnd=%d\n", k, d.prec[k], d.sgnd[k]);
    fprintf(out, "}\nCodestream info from main header: {\n\t tx0=%u, ty0=%u\n\t tdx=%u, tdy=%u\n\t tw=%u, th=%u\n",
            h.tx0, h.ty0, h.tdx, h.tdy, h.tw, h.th);
    fprintf(out, "\t numlayers=%u progression=%u numresolutions=%u cblk=%ux%u csty=%u cblksty=%u qmfbid=%u mct=%u\n}\n",
            h.numlayers, h.prog, h.numresolutions, h.cblockw_init, h.cblockh_init, h.csty, h.cblk_sty,
            h.irreversible ? 0 : 1, h.mct);
}
// grk_get_cstr_info (grok.cpp:673-679 -> j2k_get_cstr_info,
// j2k_dump.cpp:326-400): the main header's tile grid and the default coding /
// quantisation parameters of every component (COD / QCD, or the component's
// main-header COC / QCC).  tile_info stays null ("not filled from the
// main header").  Kept as the reference does it: compno is not set (0), and
// prcw / prch are copied with numresolutions BYTES (memcpy, :366-369), so
// only the first numresolutions / 4 entries arrive.
GRK_EXPORT grk_codestream_info_v2 *grk_get_cstr_info(grk_codec *codec) {
    Codec *c = (Codec *)codec;
    if (!c || !c->decompressor || !c->have_header) return nullptr;
    const grkgpu_header_info &h = c->hinfo;
    auto *ci = (grk_codestream_info_v2 *)calloc(1, sizeof(grk_codestream_info_v2));
    if (!ci) return nullptr;
    ci->nbcomps = h.numcomps;
    ci->tx0 = h.tx0; ci->ty0 = h.ty0; ci->tdx = h.tdx; ci->tdy = h.tdy; ci->tw = h.tw; ci->th = h.th;
    grk_tile_info_v2 &t = ci->m_default_tile_info;
    t.csty = h.csty;
    t.prg = (int32_t)h.prog;
    t.numlayers = h.numlayers;
    t.mct = h.mct;
    t.tccp_info = (grk_tccp_info *)calloc(h.numcomps ? h.numcomps : 1, sizeof(grk_tccp_info));
    if (!t.tccp_info) { free(ci); return nullptr; }
    for (uint32_t k = 0; k < h.numcomps; ++k) {
        const grkgpu_comp_info &cc = c->cinfo[k];
        grk_tccp_info &q = t.tccp_info[k];
        q.csty = (uint8_t)cc.csty;  // tccp->csty = Scod / Scoc & J2K_CCP_CSTY_PRT (j2k.cpp:3875)
        q.numresolutions = cc.numresolutions;
        q.cblkw = cc.cblkw;
        q.cblkh = cc.cblkh;
        q.cblk_sty = (uint8_t)cc.cblk_sty;
        q.qmfbid = cc.qmfbid;
        if (q.numresolutions < GRKP_MAXRLVLS) {  // tccp->prcw / prch: log2 sizes, numresolutions BYTES
            uint32_t prcw[GRKP_MAXRLVLS], prch[GRKP_MAXRLVLS];
            for (uint32_t r = 0; r < GRKP_MAXRLVLS; ++r) { prcw[r] = cc.prcw[r]; prch[r] = cc.prch[r]; }
            memcpy(q.prch, prch, q.numresolutions);
            memcpy(q.prcw, prcw, q.numresolutions);
        }
        q.qntsty = (uint8_t)cc.qntsty;
        q.numgbits = (uint8_t)cc.numgbits;
        const uint32_t nb = cc.qntsty == 1 ? 1 : cc.numresolutions * 3 - 2;
        if (nb < GRK_J2K_MAXBANDS)
            for (uint32_t b = 0; b < nb; ++b) {
                q.stepsizes_mant[b] = b < cc.nsteps ? cc.step_mant[b] : 0;
                q.stepsizes_expn[b] = b < cc.nsteps ? cc.step_expn[b] : 0;
            }
        q.roishift = cc.roishift;
    }
    return ci;
}
GRK_EXPORT void grk_destroy_cstr_info(grk_codestream_info_v2 **p) {
    if (!p || !*p) return;
    free((*p)->m_default_tile_info.tccp_info);
    free(*p);
    *p = nullptr;
}
// grk_get_cstr_index (grok.cpp:694 -> j2k_get_cstr_index, j2k_dump.cpp:
// 402-517): what the reference's decoder records while reading -- every
// main-header marker (type, position, length incl. the marker code:
// j2k.cpp:304-311, SOC 3150-3161), the first SOT's position
// (main_head_end, :341-344), and per tile its tile-part markers (SOT, the
// header markers, SOD with length 0: :739-749, 5443-5448) and tile-part
// positions (SOT, SOD, SOT + Psot: :5276-5360, 5426-5441, 6696-6704).
// codestream_size is only set when encoding (j2k_write_epc) and stays 0.
// The copy is the reference's too: tileno and the current_* fields are not
// copied (0), and since grk_malloc(0) is null, a tile without markers or
// without a TNsot count makes the whole call return null -- as it does after
// grk_read_header alone, before any tile-part is read.
static void *malloc_nz(size_t n) { return n ? malloc(n) : nullptr; }
GRK_EXPORT void grk_destroy_cstr_index(grk_codestream_index **p) {
    if (!p || !*p) return;
    grk_codestream_index *ix = *p;
    for (uint32_t t = 0; ix->tile_index && t < ix->nb_of_tiles; ++t) {
        free(ix->tile_index[t].marker);
        free(ix->tile_index[t].tp_index);
        free(ix->tile_index[t].packet_index);
    }
    free(ix->tile_index);
    free(ix->marker);
    free(ix);
    *p = nullptr;
}
GRK_EXPORT grk_codestream_index *grk_get_cstr_index(grk_codec *codec) {
    Codec *c = (Codec *)codec;
    if (!c || !c->decompressor || !c->have_header || !c->decoded) return nullptr;
    const std::vector<uint8_t> &cs = c->cs;
    const size_t len = cs.size();
    auto rd16 = [&](size_t q) { return q + 2 <= len ? (uint32_t)cs[q] << 8 | cs[q + 1] : 0u; };
    std::vector<grk_marker_info> mh{{0xFF4F, 0, 2}};
    size_t pos = 2;
    while (pos + 4 <= len && rd16(pos) != 0xFF90) {
        const uint32_t L = rd16(pos + 2);
        mh.push_back({(uint16_t)rd16(pos), (uint64_t)pos, L + 2});
        pos += 2 + L;
    }
    const size_t main_end = pos;
    const uint32_t nt = c->hinfo.tw * c->hinfo.th;
    std::vector<std::vector<grk_marker_info>> tm(nt);
    std::vector<std::vector<grk_tp_index>> tp(nt);
    std::vector<uint32_t> nb_tps(nt, 0);
    // the decoder's tile-part counts (tcp m_nb_tile_parts) and the TPsot ==
    // TNsot correction (j2k.cpp:809-835, read_sot :5202-5236): checked once,
    // after the first tile whose last counted tile-part was read; from then on
    // every known count and every later TNsot is one higher.  A SOT read_sot
    // refuses ends the walk before it is recorded.
    std::vector<uint32_t> nbp(nt, 0);
    uint32_t corr = 0;
    bool checked = false;
    while (pos + 12 <= len && rd16(pos) == 0xFF90) {
        const uint32_t isot = rd16(pos + 4), psot = rd16(pos + 6) << 16 | rd16(pos + 8);
        const uint32_t tpsot = cs[pos + 10], tnsot = cs[pos + 11];
        if (isot >= nt) break;
        if (nbp[isot] && tpsot >= nbp[isot]) break;
        if (tnsot) {
            const uint32_t np = (tnsot + corr) & 0xFF;
            if (tpsot >= np) break;
            nbp[isot] = np;
            nb_tps[isot] = np;
            tp[isot].resize(np, grk_tp_index{});  // grk_realloc to the count (j2k.cpp:5281-5310)
        } else if (tp[isot].size() < tpsot + 1) {
            tp[isot].resize(tpsot + 1, grk_tp_index{});
        }
        const bool ready = nbp[isot] && nbp[isot] == tpsot + 1;
        const size_t sot = pos;
        tm[isot].push_back({0xFF90, (uint64_t)sot, 12});
        tp[isot][tpsot].start_pos = sot;
        pos += 12;
        while (pos + 4 <= len && rd16(pos) != 0xFF93) {
            const uint32_t L = rd16(pos + 2);
            tm[isot].push_back({(uint16_t)rd16(pos), (uint64_t)pos, L + 2});
            pos += 2 + L;
        }
        tm[isot].push_back({0xFF93, (uint64_t)pos, 0});
        const size_t end = psot ? std::min<size_t>(sot + psot, len) : (len >= 2 ? len - 2 : len);
        tp[isot][tpsot].end_header = pos;
        tp[isot][tpsot].end_pos = end;
        if (!psot || end <= pos) break;
        pos = end;
        if (ready && !checked) {  // j2k_need_nb_tile_parts_correction (j2k.cpp:527-625): the tile's next SOT
            checked = true;
            size_t q = pos;
            while (q + 12 <= len && rd16(q) == 0xFF90 && rd16(q + 2) == 10) {
                const uint32_t t2 = rd16(q + 4), tot = rd16(q + 6) << 16 | rd16(q + 8);
                if (t2 == isot) {
                    if (cs[q + 10] == cs[q + 11]) {
                        corr = 1;
                        for (auto &n : nbp)
                            if (n) n = (n + 1) & 0xFF;
                    }
                    break;
                }
                if (tot < 14) break;
                q += tot;
            }
        }
    }
    for (uint32_t t = 0; t < nt; ++t)
        if (tm[t].empty() || !nb_tps[t]) return nullptr;  // grk_malloc(0) (j2k_dump.cpp:449-465, 481-498)
    auto *ix = (grk_codestream_index *)calloc(1, sizeof(grk_codestream_index));
    if (!ix) return nullptr;
    ix->main_head_start = 0;
    ix->main_head_end = main_end;
    ix->codestream_size = 0;
    ix->marknum = (uint32_t)mh.size();
    ix->marker = (grk_marker_info *)malloc_nz(mh.size() * sizeof(grk_marker_info));
    ix->nb_of_tiles = nt;
    ix->tile_index = (grk_tile_index *)calloc(nt, sizeof(grk_tile_index));
    if (!ix->marker || !ix->tile_index) { grk_destroy_cstr_index(&ix); return nullptr; }
    memcpy(ix->marker, mh.data(), mh.size() * sizeof(grk_marker_info));
    for (uint32_t t = 0; t < nt; ++t) {
        grk_tile_index &ti = ix->tile_index[t];
        ti.marknum = (uint32_t)tm[t].size();
        ti.marker = (grk_marker_info *)malloc_nz(tm[t].size() * sizeof(grk_marker_info));
        ti.nb_tps = nb_tps[t];
        ti.tp_index = (grk_tp_index *)calloc(nb_tps[t], sizeof(grk_tp_index));
        if (!ti.marker || !ti.tp_index) { grk_destroy_cstr_index(&ix); return nullptr; }
        memcpy(ti.marker, tm[t].data(), tm[t].size() * sizeof(grk_marker_info));
        memcpy(ti.tp_index, tp[t].data(), std::min<size_t>(nb_tps[t], tp[t].size()) * sizeof(grk_tp_index));
    }
    return ix;
}

// ---------------------------------------------------------------------------
// plugin management: this library is the accelerated path, no plugin loads
// (grok.cpp:834-1100 return conventions: false / -1 / no-op)
// ---------------------------------------------------------------------------
GRK_EXPORT bool grk_plugin_load(grk_plugin_load_info) { return false; }
GRK_EXPORT void grk_plugin_cleanup(void) {}
GRK_EXPORT bool grk_plugin_init(grk_plugin_init_info) { return false; }
GRK_EXPORT uint32_t grk_plugin_get_debug_state(void) { return GRK_PLUGIN_STATE_NO_DEBUG; }
GRK_EXPORT int32_t grk_plugin_encode(grk_cparameters *, GRK_PLUGIN_ENCODE_USER_CALLBACK) { return -1; }
GRK_EXPORT int32_t grk_plugin_batch_encode(const char *, const char *, grk_cparameters *,
                                           GRK_PLUGIN_ENCODE_USER_CALLBACK) {
    return -1;
}
GRK_EXPORT bool grk_plugin_is_batch_complete(void) { return true; }
GRK_EXPORT void grk_plugin_stop_batch_encode(void) {}
GRK_EXPORT int32_t grk_plugin_decode(grk_decompress_parameters *, grk_plugin_decode_callback) { return -1; }
GRK_EXPORT int32_t grk_plugin_init_batch_decode(const char *, const char *, grk_decompress_parameters *,
                                                grk_plugin_decode_callback) {
    return -1;
}
GRK_EXPORT int32_t grk_plugin_batch_decode(void) { return -1; }
GRK_EXPORT void grk_plugin_stop_batch_decode(void) {}
