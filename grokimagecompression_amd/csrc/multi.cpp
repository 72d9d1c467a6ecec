// multi.cpp -- one call, several devices: the tile shard of SURVEY 8(e) behind
// the C ABI.
//
// The reference's callers ask for "all devices" with deviceId = -1
// (grk_cparameters.deviceId, grok.h:565; grk_compress -G, "A value of -1
// will specify all devices", grk_compress.cpp:423-426).  Tiles are
// independent through DC shift, MCT, DWT, T1 and T2 (the reference's tile
// loop, j2k.cpp:2088-2111), and a codestream is [main header][tile-parts in
// tile order][EOC] (j2k.cpp:2376-2435), so one call here:
//   * encode: splits the tiles into contiguous ranges, one per worker; each
//     worker (a host thread with a context on its device) uploads only the
//     image rows of its tiles and encodes them (grkgpu_compress_ex with a row
//     window) -- worker 0 also writes the main header, the last the EOC; the
//     pieces are concatenated in worker order = tile order and the TLM
//     records, which no single worker could write, are filled in from the
//     tile-parts (j2k_write_updated_tlm, j2k.cpp:2555-2577);
//   * decode: every worker decodes its tile range into the caller's host
//     planes (grkgpu_decompress_tiles; the ranges write disjoint tiles).
// No collective and no device-to-device copy: the only exchange is the host
// concatenation.  Contexts are pooled per device across calls.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/grk_mi355x.h"

namespace grkgpu {
int set_error(int code, const std::string &msg);  // codec.cpp: the calling thread's grkgpu_last_error
}
using grkgpu::set_error;

namespace {

std::mutex g_mu;
std::vector<std::vector<grkgpu_ctx *>> g_idle;  // [device] contexts between multi-device calls

grkgpu_ctx *lease(int device, std::string &err) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if ((size_t)device < g_idle.size() && !g_idle[device].empty()) {
            grkgpu_ctx *c = g_idle[device].back();
            g_idle[device].pop_back();
            return c;
        }
    }
    grkgpu_ctx *c = nullptr;
    if (grkgpu_create(device, &c) != GRKGPU_OK) {
        err = std::string("device ") + std::to_string(device) + ": " + grkgpu_last_error();
        return nullptr;
    }
    return c;
}

void give_back(int device, grkgpu_ctx *c) {
    std::lock_guard<std::mutex> lk(g_mu);
    if ((size_t)device >= g_idle.size()) g_idle.resize(device + 1);
    g_idle[device].push_back(c);
}

// contiguous, balanced tile range of worker w of n (the first workers take
// the remainder; shard.py tile_range)
void tile_range(uint32_t ntiles, uint32_t w, uint32_t n, uint32_t &b, uint32_t &e) {
    const uint32_t base = ntiles / n, extra = ntiles % n;
    b = w * base + std::min(w, extra);
    e = b + base + (w < extra ? 1 : 0);
}

uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] << 8 | p[1]; }
uint32_t rd32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// j2k_write_updated_tlm (j2k.cpp:2555-2577) over an assembled codestream:
// every TLM record (Ttlm of Stlm's ST bytes, Ptlm of 2 or 4 bytes,
// j2k.cpp:5027-5063) from the tile-parts' own SOT headers, in codestream
// order, filled across the main header's TLM markers in their order.  A
// stream without TLM is left alone; records that do not match the tile-parts
// one to one are an error, never a silently stale TLM.
bool patch_tlm(std::vector<uint8_t> &cs, std::string &err) {
    if (cs.size() < 4 || rd16(cs.data()) != 0xFF4F) return true;
    struct Tlm { size_t pos; uint32_t st, sp, n; };
    std::vector<Tlm> tlms;
    size_t pos = 2;
    while (pos + 4 <= cs.size()) {
        const uint32_t m = rd16(&cs[pos]), L = rd16(&cs[pos + 2]);
        if (m == 0xFF90) break;
        if (L < 2 || pos + 2 + L > cs.size()) { err = "TLM patch: bad main-header marker"; return false; }
        if (m == 0xFF55) {
            if (L < 4) { err = "TLM patch: short TLM marker"; return false; }
            const uint32_t stlm = cs[pos + 5], st = (stlm >> 4) & 3, sp = (stlm >> 6) & 1 ? 4 : 2;
            if (st == 3) { err = "TLM patch: invalid Stlm"; return false; }
            tlms.push_back({pos, st, sp, (L - 4) / (st + sp)});
        }
        pos += 2 + L;
    }
    if (tlms.empty()) return true;
    std::vector<std::pair<uint32_t, uint32_t>> recs;  // (Isot, Psot) per tile-part
    while (pos + 12 <= cs.size() && rd16(&cs[pos]) == 0xFF90) {
        const uint32_t isot = rd16(&cs[pos + 4]), psot = rd32(&cs[pos + 6]);
        if (!psot || pos + psot > cs.size()) { err = "TLM patch: tile-part without a length (Psot = 0) or past the end"; return false; }
        recs.push_back({isot, psot});
        pos += psot;
    }
    size_t total = 0;
    for (auto &t : tlms) total += t.n;
    if (total != recs.size()) {
        err = "TLM patch: " + std::to_string(total) + " TLM records for " + std::to_string(recs.size()) + " tile-parts";
        return false;
    }
    size_t k = 0;
    for (auto &t : tlms) {
        uint8_t *q = &cs[t.pos + 6];
        for (uint32_t i = 0; i < t.n; ++i, ++k) {
            const uint32_t isot = recs[k].first, psot = recs[k].second;
            if ((t.st == 1 && isot > 0xFF) || (t.sp == 2 && psot > 0xFFFF)) {
                err = "TLM patch: a record does not fit its field width";
                return false;
            }
            for (uint32_t b = 0; b < t.st; ++b) *q++ = (uint8_t)(isot >> (8 * (t.st - 1 - b)));
            for (uint32_t b = 0; b < t.sp; ++b) *q++ = (uint8_t)(psot >> (8 * (t.sp - 1 - b)));
        }
    }
    return true;
}

bool subsampled(const grkgpu_image_desc *img) {
    for (uint32_t k = 0; k < img->numcomps && k < GRKGPU_MAX_COMPS; ++k)
        if ((img->dx[k] && img->dx[k] != 1) || (img->dy[k] && img->dy[k] != 1)) return true;
    return false;
}

uint32_t smp_bytes(uint32_t fmt) {
    return fmt == GRKGPU_SAMPLE_I32 ? 4 : (fmt == GRKGPU_SAMPLE_U8 || fmt == GRKGPU_SAMPLE_I8) ? 1 : 2;
}

// run f(worker) on one thread per worker; the first failing worker's error
template <typename F>
int run_workers(uint32_t n, F f) {
    std::vector<std::string> errs(n);
    std::vector<int> rcs(n, GRKGPU_OK);
    std::vector<std::thread> th;
    th.reserve(n);
    for (uint32_t w = 0; w < n; ++w) th.emplace_back([&, w] { rcs[w] = f(w, errs[w]); });
    for (auto &t : th) t.join();
    for (uint32_t w = 0; w < n; ++w)
        if (rcs[w] != GRKGPU_OK) return set_error(rcs[w], "worker " + std::to_string(w) + ": " + errs[w]);
    return GRKGPU_OK;
}

}  // namespace

extern "C" int grkgpu_device_set_for(int device, grkgpu_device_set *out) {
    if (!out) return set_error(GRKGPU_EINVAL, "null argument");
    memset(out, 0, sizeof(*out));
    const int have = grkgpu_device_count();
    if (device >= 0) {
        out->n = 1;
        out->dev[0] = device;
        return GRKGPU_OK;
    }
    if (device != -1) return set_error(GRKGPU_EINVAL, "device must be >= 0, or -1 for all devices");
    if (const char *e = getenv("GRKGPU_DEVICES")) {  // the workers: "d0,d1,..." (a device may repeat) or "all"
        if (strcmp(e, "all") != 0) {
            const char *p = e;
            while (*p) {
                char *end = nullptr;
                const long d = strtol(p, &end, 10);
                if (end == p || d < 0 || (have > 0 && d >= have) || out->n >= GRKGPU_MAX_DEVICES)
                    return set_error(GRKGPU_EINVAL, std::string("GRKGPU_DEVICES: bad device list '") + e + "'");
                out->dev[out->n++] = (int32_t)d;
                p = *end == ',' ? end + 1 : end;
                if (*end && *end != ',') return set_error(GRKGPU_EINVAL, std::string("GRKGPU_DEVICES: bad device list '") + e + "'");
            }
            if (out->n) return GRKGPU_OK;
        }
    }
    if (have <= 0) return set_error(GRKGPU_ENODEV, "no HIP device available (MI355X / gfx950 required; no CPU fallback)");
    out->n = (uint32_t)std::min(have, GRKGPU_MAX_DEVICES);
    for (uint32_t k = 0; k < out->n; ++k) out->dev[k] = (int32_t)k;
    return GRKGPU_OK;
}

extern "C" int grkgpu_compress_multi(const grkgpu_device_set *devs, const grkgpu_image_desc *img,
                                     const grkgpu_cparams *p, const grkgpu_planes *planes, uint8_t **out,
                                     size_t *outlen) {
    if (!devs || !img || !p || !planes || !out || !outlen || !devs->n || devs->n > GRKGPU_MAX_DEVICES)
        return set_error(GRKGPU_EINVAL, "null argument or empty device set");
    uint32_t ntiles = 0;
    int rc = grkgpu_num_tiles(img, p, &ntiles);
    if (rc) return rc;
    const bool whole = !planes->row0 && !planes->nrows && !planes->col0 && !planes->ncols;
    uint32_t n = std::min<uint32_t>(devs->n, ntiles);
    // one worker: one tile, planes on a device (another device cannot read
    // them), a partial window of the image, or subsampled components (the
    // tile-range encode takes none: DESIGN.md 1)
    if (planes->on_device || !whole || subsampled(img)) n = 1;
    std::vector<std::vector<uint8_t>> piece(n);
    const uint32_t w = img->x1 - img->x0, h = img->y1 - img->y0;
    // tile grid (j2k.cpp:1938-1962): tiles of cp_tdx x cp_tdy from (cp_tx0, cp_ty0), or one tile
    const uint32_t tdy = p->tile_size_on ? p->cp_tdy : h, ty0 = p->tile_size_on ? p->cp_ty0 : img->y0;
    const uint32_t tdx = p->tile_size_on ? p->cp_tdx : w, tx0 = p->tile_size_on ? p->cp_tx0 : img->x0;
    const uint32_t tw = tdx ? (img->x1 - tx0 + tdx - 1) / tdx : 1;
    rc = run_workers(n, [&](uint32_t k, std::string &err) -> int {
        uint32_t b = 0, e = ntiles;
        if (n > 1) tile_range(ntiles, k, n, b, e);
        const uint32_t parts = GRKGPU_PART_TILES | (k == 0 ? GRKGPU_PART_HEADER : 0) | (k == n - 1 ? GRKGPU_PART_EOC : 0);
        grkgpu_planes pl = *planes;
        if (n > 1) {  // only the image rows of tiles [b, e)
            const uint32_t q0 = b / tw, q1 = (e - 1) / tw;
            const uint32_t r0 = std::max(img->y0, ty0 + q0 * tdy) - img->y0;
            const uint32_t r1 = std::min(img->y1, ty0 + (q1 + 1) * tdy) - img->y0;
            const size_t skip = (size_t)r0 * w * smp_bytes(planes->sample_fmt);
            for (uint32_t c = 0; c < img->numcomps; ++c) pl.planes[c] = (const uint8_t *)planes->planes[c] + skip;
            pl.row0 = r0;
            pl.nrows = r1 - r0;
        }
        const int dev = devs->dev[k];
        grkgpu_ctx *ctx = lease(dev, err);
        if (!ctx) return GRKGPU_ENODEV;
        const uint8_t *o = nullptr;
        size_t len = 0;
        int r = n > 1 ? grkgpu_compress_ex(ctx, img, p, &pl, b, e, parts, &o, &len)
                      : grkgpu_compress_ex(ctx, img, p, &pl, 0, 0xffffffffu, GRKGPU_PART_ALL, &o, &len);
        if (r == GRKGPU_OK) piece[k].assign(o, o + len);  // out of the context's buffer before it goes back
        else err = grkgpu_last_error();
        give_back(dev, ctx);
        return r;
    });
    if (rc) return rc;
    std::vector<uint8_t> cs;
    size_t total = 0;
    for (auto &x : piece) total += x.size();
    cs.reserve(total);
    for (auto &x : piece) cs.insert(cs.end(), x.begin(), x.end());
    std::string err;
    if (n > 1 && !patch_tlm(cs, err)) return set_error(GRKGPU_EINVAL, err);
    uint8_t *o = (uint8_t *)malloc(cs.size() ? cs.size() : 1);
    if (!o) return set_error(GRKGPU_EINVAL, "out of host memory");
    if (!cs.empty()) memcpy(o, cs.data(), cs.size());
    *out = o;
    *outlen = cs.size();
    return GRKGPU_OK;
}

extern "C" int grkgpu_decompress_multi(const grkgpu_device_set *devs, const uint8_t *cs, size_t len,
                                       grkgpu_image_desc *img, int32_t *const *planes) {
    if (!devs || !cs || !planes || !devs->n || devs->n > GRKGPU_MAX_DEVICES)
        return set_error(GRKGPU_EINVAL, "null argument or empty device set");
    grkgpu_image_desc d;
    int rc = grkgpu_read_header(cs, len, &d);
    if (rc) return rc;
    grkgpu_header_info hi;
    rc = grkgpu_read_header_info(cs, len, &hi);
    if (rc) return rc;
    const uint32_t ntiles = hi.tw * hi.th;
    uint32_t n = std::min<uint32_t>(devs->n, ntiles ? ntiles : 1);
    if (subsampled(&d)) n = 1;  // the tile-range decode takes no subsampled components
    rc = run_workers(n, [&](uint32_t k, std::string &err) -> int {
        const int dev = devs->dev[k];
        grkgpu_ctx *ctx = lease(dev, err);
        if (!ctx) return GRKGPU_ENODEV;
        int r;
        if (n == 1) {
            r = grkgpu_decompress(ctx, cs, len, nullptr, planes, 0);
        } else {
            uint32_t b, e;
            tile_range(ntiles, k, n, b, e);
            r = grkgpu_decompress_tiles(ctx, cs, len, b, e, planes, 0);
        }
        if (r != GRKGPU_OK) err = grkgpu_last_error();
        give_back(dev, ctx);
        return r;
    });
    if (rc) return rc;
    if (img) *img = d;
    return GRKGPU_OK;
}

extern "C" int grkgpu_patch_tlm(uint8_t *cs, size_t len) {
    if (!cs) return set_error(GRKGPU_EINVAL, "null argument");
    std::vector<uint8_t> v(cs, cs + len);
    std::string err;
    if (!patch_tlm(v, err)) return set_error(GRKGPU_EINVAL, err);
    memcpy(cs, v.data(), len);
    return GRKGPU_OK;
}

extern "C" void grkgpu_multi_release(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto &v : g_idle) {
        for (auto *c : v) grkgpu_destroy(c);
        v.clear();
    }
}
