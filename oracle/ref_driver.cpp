// oracle/ref_driver.cpp -- fixture / baseline driver over the REFERENCE grk_*
// C API (oracle/_ref/libgrok.so, built from /root/reference by oracle/ref.mk).
//
// Test infrastructure only: it regenerates tests/golden/ (oracle/make_golden.py)
// and times the reference CPU path for bench.py's cpu_baseline leg.  The
// product never runs it.
//
// It does what grk_compress / grk_decompress do for the options the fixtures
// use, minus the image-file layer: the image arrives as raw int32 planes.
//   encode: grk_set_default_encoder_parameters, then the CLI mapping of
//           src/bin/jp2/grk_compress.cpp (-I :1107, -n :999, -b :1027-1042,
//           -d :1069, -t :994, -T :1480, -Y :1383, -r :812-846, -q :848-880,
//           -p :1050, -c :1003-1023, -M :1132, -S/-E :1101-1105, -u :1516,
//           -P :1077-1098, -cinema2K/4K :537-561 + :1146-1163), the
//           post-parse defaults (:1579-1583 lossless layer, :1997-1998 MCT,
//           :2015 rate-control algorithm), image geometry as PNMFormat sets it
//           (PNMFormat.cpp:399-417), then grk_create_compress ->
//           grk_setup_encoder -> grk_start_compress -> grk_encode ->
//           grk_end_compress into a memory stream (grk_compress.cpp:2090-2130).
//   decode: grk_create_decompress -> grk_setup_decoder (cp_reduce / cp_layer)
//           -> grk_read_header -> grk_set_decode_area -> grk_decode ->
//           grk_end_decompress (grk_decompress.cpp:1427-1530).
//
// usage:
//   ref_driver enc IN.i32 OUT.j2k W H C BITS SGND [options]
//   ref_driver dec IN.j2k OUT.i32 [-r reduce] [-l layers] [-d x0,y0,x1,y1]
//   ref_driver bench IN.i32 W H C BITS SGND THREADS REPS [options]   (enc+dec timing)
//   ref_driver plugin PLUGIN_DIR IN.i32 OUT.j2k W H C BITS [options]
//       the reference host driving OUR accelerator plugin (libgrok_plugin.so in
//       PLUGIN_DIR) exactly as grk_compress's plugin_main does
//       (grk_compress.cpp:2163-2305 + plugin_compress_callback :1770-2161):
//       grk_initialize(plugin_dir) -> grk_plugin_init -> grk_plugin_encode(
//       params, cb); cb runs grk_setup_encoder -> grk_start_compress ->
//       grk_encode_with_plugin(tile) -> grk_end_compress.  The input goes
//       through a PGM / PPM file, the format the plugin reads.  Exit 0 iff
//       the plugin handled the image; 3 if it declined (host CPU fallback).
//   ref_driver plugin-dec PLUGIN_DIR IN.j2k OUT.i32 [-r reduce] [-l layers] [-d x0,y0,x1,y1]
//       grk_decompress's plugin_main (grk_decompress.cpp:1186-1319):
//       grk_plugin_decode(params, decode_callback) with decode_callback /
//       pre_decode / post_decode restated (:1336-1557) -- post_decode writes
//       the planes as dec does.  Exit 0 iff the plugin decoded; 3 if declined.
//   ref_driver plugin-batch PLUGIN_DIR IN_DIR OUT_DIR [options]
//       grk_compress's plugin_main in batch mode (-ImgDir / -OutDir,
//       grk_compress.cpp:2196-2243): grk_plugin_batch_encode(in, out, params,
//       cb), then poll grk_plugin_is_batch_complete every 100 ms and
//       grk_plugin_stop_batch_encode; cb (plugin_compress_callback's relative
//       output naming, :1783-1797) writes OUT_DIR/<name>.j2k.  Exit 0 iff
//       every frame was written; 3 if the plugin declined the batch.
//   ref_driver plugin-batch-dec PLUGIN_DIR IN_DIR OUT_DIR
//       grk_decompress's plugin_main in batch mode (grk_decompress.cpp:
//       1237-1262): grk_plugin_init_batch_decode, grk_plugin_batch_decode,
//       the completion poll and grk_plugin_stop_batch_decode; the decode
//       callback writes each image (raw int32 planes) to the output name the
//       plugin gives.
//   ref_driver mt IN.i32 EXPECT.j2k W H C BITS SGND THREADS REPS [options]
//       THREADS caller threads, each with its own codecs (one codec per
//       caller thread), encode + decode REPS times concurrently;
//       exit 0 iff every encode equals EXPECT.j2k and every decode equals the
//       first decode (lossless: the input).
//   ref_driver index IN.j2k   (grk_get_cstr_index after grk_read_header and after grk_decode)
//   ref_driver info IN.j2k
//       grk_read_header, then grk_get_cstr_info printed field by field (the
//       grk_dump path, grk_dump.cpp:494-500) and grk_destroy_cstr_info.
// IN.i32 / OUT.i32: planar int32 little-endian (c, h, w).  dec prints
// "x0 y0 x1 y1 numcomps prec sgnd" of the decoded image on stdout.
#include <grok.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <unistd.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

static void err_cb(const char *msg, void *) { fprintf(stderr, "[grk error] %s", msg); }
// warnings of the host: in the plugin debug state every difference between
// the host's own T1 and the plugin's blocks is one (plugin_bridge.cpp:155-251)
static int g_warnings = 0;
static void warn_cb(const char *msg, void *) {
    ++g_warnings;
    fprintf(stderr, "[grk warning] %s", msg);
}

static std::vector<uint8_t> read_file(const char *p) {
    std::vector<uint8_t> v;
    FILE *f = fopen(p, "rb");
    if (!f) { perror(p); exit(2); }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    v.resize((size_t)n);
    if (n && fread(v.data(), 1, (size_t)n, f) != (size_t)n) { perror(p); exit(2); }
    fclose(f);
    return v;
}

static void write_file(const char *p, const void *d, size_t n) {
    FILE *f = fopen(p, "wb");
    if (!f || fwrite(d, 1, n, f) != n) { perror(p); exit(2); }
    fclose(f);
}

static GRK_PROG_ORDER prog(const char *s) {
    if (!strncmp(s, "LRCP", 4)) return GRK_LRCP;
    if (!strncmp(s, "RLCP", 4)) return GRK_RLCP;
    if (!strncmp(s, "RPCL", 4)) return GRK_RPCL;
    if (!strncmp(s, "PCRL", 4)) return GRK_PCRL;
    if (!strncmp(s, "CPRL", 4)) return GRK_CPRL;
    return GRK_PROG_UNKNOWN;
}

// -sub dx,dy/dx,dy/...: per-component subsampling of the grk_image the
// driver builds (grk_image_cmptparm dx / dy; the CLI's -s sets one factor for
// all components, grk_compress.cpp:1060, PNMFormat.cpp:397-417)
static std::vector<std::pair<uint32_t, uint32_t>> g_sub;
// -mct m00,m01,...:s0,s1,...: a custom MCT through grk_set_MCT (grok.cpp:606),
// row-major n x n encoding matrix and n DC shifts
static std::vector<float> g_mct;
static std::vector<int32_t> g_mct_shift;

// grk_compress option subset -> parameters (citations in the header)
static bool parse_enc_opts(grk_cparameters *p, int argc, char **argv) {
    grk_set_default_encoder_parameters(p);
    p->tcp_mct = 255;
    p->rateControlAlgorithm = 255;
    uint32_t cinema = 0, fps = 0;
    for (int i = 0; i < argc; ++i) {
        std::string a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : "";
        if (a == "-I") { p->irreversible = true; continue; }
        if (a == "-S") { p->csty |= 0x02; continue; }
        if (a == "-E") { p->csty |= 0x04; continue; }
        ++i;
        if (a == "-n") p->numresolution = (uint32_t)atoi(v);
        else if (a == "-b") { if (sscanf(v, "%u,%u", &p->cblockw_init, &p->cblockh_init) != 2) return false; }
        else if (a == "-d") { if (sscanf(v, "%u,%u", &p->image_offset_x0, &p->image_offset_y0) != 2) return false; }
        else if (a == "-t") { if (sscanf(v, "%u,%u", &p->cp_tdx, &p->cp_tdy) != 2) return false; p->tile_size_on = true; }
        else if (a == "-T") { if (sscanf(v, "%u,%u", &p->cp_tx0, &p->cp_ty0) != 2) return false; }
        else if (a == "-Y") p->tcp_mct = (uint8_t)atoi(v);
        else if (a == "-p") p->prog_order = prog(v);
        else if (a == "-mct") {
            g_mct.clear();
            g_mct_shift.clear();
            const char *s = v;
            while (*s && *s != ':') {
                g_mct.push_back(strtof(s, (char **)&s));
                if (*s == ',') s++;
            }
            if (*s == ':') s++;
            while (*s) {
                g_mct_shift.push_back((int32_t)strtol(s, (char **)&s, 10));
                if (*s == ',') s++;
                else break;
            }
        }
        else if (a == "-sub") {
            g_sub.clear();
            const char *s = v;
            uint32_t dx, dy;
            while (sscanf(s, "%u,%u", &dx, &dy) == 2) {
                g_sub.push_back({dx, dy});
                while (*s && *s != '/') s++;
                if (!*s) break;
                s++;
            }
        }
        else if (a == "-M") p->cblk_sty = (uint8_t)(atoi(v) & 0x7f);
        else if (a == "-u") { p->tp_flag = (uint8_t)v[0]; p->tp_on = 1; }
        else if (a == "-G") p->deviceId = atoi(v);  // grk_compress.cpp:720-721 (-1: all devices)
        else if (a == "-A") p->rateControlAlgorithm = (uint32_t)atoi(v);
        else if (a == "-R") {  // grk_compress.cpp:1470-1476
            if (sscanf(v, "c=%d,U=%u", &p->roi_compno, &p->roi_shift) != 2) return false;
        }
        else if (a == "-r" || a == "-q") {
            double *dst = a == "-r" ? p->tcp_rates : p->tcp_distoratio;
            p->tcp_numlayers = 0;
            const char *s = v;
            while (sscanf(s, "%lf", &dst[p->tcp_numlayers]) == 1) {
                p->tcp_numlayers++;
                while (*s && *s != ',') s++;
                if (!*s) break;
                s++;
            }
            if (a == "-r") {
                p->cp_disto_alloc = 1;
                for (uint32_t k = 0; k < p->tcp_numlayers; ++k)
                    if (p->tcp_rates[k] == 1) p->tcp_rates[k] = 0;
            } else {
                p->cp_fixed_quality = 1;
            }
        } else if (a == "-c") {
            const char *s = v;
            uint32_t rs = 0;
            char sep;
            int ret;
            do {
                sep = 0;
                ret = sscanf(s, "[%u,%u]%c", &p->prcw_init[rs], &p->prch_init[rs], &sep);
                if (!(ret == 2 && sep == 0) && !(ret == 3 && sep == ',')) return false;
                p->csty |= 0x01;
                rs++;
                s = strpbrk(s, "]") + 2;
            } while (sep == ',');
            p->res_spec = rs;
        } else if (a == "-P") {
            const char *s = v;
            uint32_t n = 0;
            grk_poc *P = p->POC;
            while (sscanf(s, "T%u=%u,%u,%u,%u,%u,%4s", &P[n].tile, &P[n].resno0, &P[n].compno0, &P[n].layno1,
                          &P[n].resno1, &P[n].compno1, P[n].progorder) == 7) {
                P[n].prg1 = prog(P[n].progorder);
                n++;
                while (*s && *s != '/') s++;
                if (!*s) break;
                s++;
            }
            p->numpocs = n;
        } else if (a == "-cinema2K" || a == "-cinema4K") {
            cinema = a == "-cinema2K" ? GRK_PROFILE_CINEMA_2K : GRK_PROFILE_CINEMA_4K;
            fps = (uint32_t)atoi(v);
        } else {
            fprintf(stderr, "unknown option %s\n", a.c_str());
            return false;
        }
    }
    if (cinema) {  // checkCinema (grk_compress.cpp:537-561)
        p->rsiz = (uint16_t)cinema;
        p->framerate = (int)fps;
        p->max_comp_size = fps == 48 ? GRK_CINEMA_48_COMP : GRK_CINEMA_24_COMP;
        p->max_cs_size = fps == 48 ? GRK_CINEMA_48_CS : GRK_CINEMA_24_CS;
    }
    if (p->tcp_numlayers == 0) {  // grk_compress.cpp:1579-1583
        p->tcp_rates[0] = 0;
        p->tcp_numlayers = 1;
        p->cp_disto_alloc = 1;
    }
    if (!g_mct.empty()) {
        const uint32_t n = (uint32_t)g_mct_shift.size();
        if (n * n != g_mct.size()) { fprintf(stderr, "-mct: n*n matrix entries and n shifts\n"); return false; }
        if (!grk_set_MCT(p, g_mct.data(), g_mct_shift.data(), n)) return false;
    }
    return true;
}

static uint32_t cdivu(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// component k's plane size for a w x h image at the parameters' offset
static void comp_size(const grk_cparameters *p, uint32_t w, uint32_t h, uint32_t k, uint32_t *cw, uint32_t *ch) {
    const uint32_t dx = k < g_sub.size() ? g_sub[k].first : 1, dy = k < g_sub.size() ? g_sub[k].second : 1;
    const uint32_t x0 = p->image_offset_x0, y0 = p->image_offset_y0;
    *cw = cdivu(x0 + w, dx) - cdivu(x0, dx);
    *ch = cdivu(y0 + h, dy) - cdivu(y0, dy);
}

static grk_image *make_image(const int32_t *planes, uint32_t w, uint32_t h, uint32_t c, uint32_t bits, uint32_t sgnd,
                             const grk_cparameters *p) {
    std::vector<grk_image_cmptparm> cm(c);
    memset(cm.data(), 0, c * sizeof(grk_image_cmptparm));
    for (uint32_t k = 0; k < c; ++k) {
        cm[k].prec = bits;
        cm[k].sgnd = sgnd;
        cm[k].dx = k < g_sub.size() ? g_sub[k].first : 1;
        cm[k].dy = k < g_sub.size() ? g_sub[k].second : 1;
        comp_size(p, w, h, k, &cm[k].w, &cm[k].h);
        cm[k].x0 = cdivu(p->image_offset_x0, cm[k].dx);
        cm[k].y0 = cdivu(p->image_offset_y0, cm[k].dy);
    }
    grk_image *img = grk_image_create(c, cm.data(), c >= 3 ? GRK_CLRSPC_SRGB : GRK_CLRSPC_GRAY);
    if (!img) return nullptr;
    img->x0 = p->image_offset_x0;
    img->y0 = p->image_offset_y0;
    img->x1 = p->image_offset_x0 + w;
    img->y1 = p->image_offset_y0 + h;
    size_t off = 0;
    for (uint32_t k = 0; k < c; ++k) {
        const size_t n = (size_t)cm[k].w * cm[k].h;
        memcpy(img->comps[k].data, planes + off, n * 4);
        off += n;
    }
    return img;
}

// returns the codestream length, 0 on failure
static size_t encode(grk_cparameters *p, const int32_t *planes, uint32_t w, uint32_t h, uint32_t c, uint32_t bits,
                     uint32_t sgnd, std::vector<uint8_t> &out) {
    grk_image *img = make_image(planes, w, h, c, bits, sgnd, p);
    if (!img) return 0;
    if (p->tcp_mct == 255) p->tcp_mct = c >= 3 ? 1 : 0;       // grk_compress.cpp:1997-1998
    if (p->rateControlAlgorithm == 255) p->rateControlAlgorithm = 0;  // :2015
    const size_t cap = (size_t)w * h * c * ((bits + 7) / 8) * 3 / 2 + (1 << 20);
    uint8_t *buf = new uint8_t[cap];
    grk_stream *st = grk_stream_create_mem_stream(buf, cap, false, false);
    grk_codec *codec = grk_create_compress(GRK_CODEC_J2K, st);
    grk_set_error_handler(err_cb, nullptr);
    bool ok = codec && grk_setup_encoder(codec, p, img) && grk_start_compress(codec, img) && grk_encode(codec) &&
              grk_end_compress(codec);
    size_t n = ok ? grk_stream_get_write_mem_stream_length(st) : 0;
    if (ok) out.assign(buf, buf + n);
    if (codec) grk_destroy_codec(codec);
    grk_stream_destroy(st);
    grk_image_destroy(img);
    delete[] buf;
    return n;
}

static grk_image *decode(const uint8_t *cs, size_t len, uint32_t reduce, uint32_t layers, const uint32_t *area,
                         grk_codec **codec_out, grk_stream **st_out) {
    grk_stream *st = grk_stream_create_mem_stream((uint8_t *)cs, len, false, true);
    grk_codec *codec = grk_create_decompress(GRK_CODEC_J2K, st);
    grk_set_error_handler(err_cb, nullptr);
    grk_dparameters dp;
    grk_set_default_decoder_parameters(&dp);
    dp.cp_reduce = reduce;
    dp.cp_layer = layers;
    grk_header_info hi;
    memset(&hi, 0, sizeof(hi));
    grk_image *img = nullptr;
    bool ok = codec && grk_setup_decoder(codec, &dp) && grk_read_header(codec, &hi, &img);
    if (ok) ok = grk_set_decode_area(codec, img, area[0], area[1], area[2], area[3]);
    if (ok) ok = grk_decode(codec, nullptr, img) && grk_end_decompress(codec);
    *codec_out = codec;
    *st_out = st;
    return ok ? img : nullptr;
}

// ---- plugin mode ----
static bool g_cb_ok = false;
static std::vector<uint8_t> g_cb_out;

static bool plugin_cb(grk_plugin_encode_user_callback_info *info) {
    grk_cparameters *p = info->encoder_parameters;
    grk_image *img = info->image;
    g_cb_ok = false;
    if (!img) return false;
    if (p->tcp_mct == 255) p->tcp_mct = img->numcomps >= 3 ? 1 : 0;        // grk_compress.cpp:1997-1998
    if (p->rateControlAlgorithm == 255) p->rateControlAlgorithm = 0;        // :2015-2017
    const size_t cap = (size_t)(img->x1 - img->x0) * (img->y1 - img->y0) * img->numcomps * 3 + (1 << 20);
    uint8_t *buf = new uint8_t[cap];
    grk_stream *st = grk_stream_create_mem_stream(buf, cap, false, false);
    grk_codec *codec = grk_create_compress(GRK_CODEC_J2K, st);
    grk_set_error_handler(err_cb, nullptr);
    grk_set_warning_handler(warn_cb, nullptr);
    bool ok = codec && grk_setup_encoder(codec, p, img) && grk_start_compress(codec, img) &&
              grk_encode_with_plugin(codec, info->tile) && grk_end_compress(codec);
    if (ok) g_cb_out.assign(buf, buf + grk_stream_get_write_mem_stream_length(st));
    if (codec) grk_destroy_codec(codec);
    grk_stream_destroy(st);
    delete[] buf;
    g_cb_ok = ok;
    return ok;
}

static bool write_pnm(const char *path, const int32_t *planes, uint32_t w, uint32_t h, uint32_t c, uint32_t bits) {
    if ((c != 1 && c != 3) || bits < 8 || bits > 16) return false;
    FILE *f = fopen(path, "wb");
    if (!f) return false;
    fprintf(f, "P%c\n%u %u\n%u\n", c == 1 ? '5' : '6', w, h, (1u << bits) - 1);
    const bool one = bits <= 8;
    std::vector<uint8_t> row((size_t)w * c * (one ? 1 : 2));
    for (uint32_t y = 0; y < h; ++y) {
        for (uint32_t x = 0; x < w; ++x)
            for (uint32_t k = 0; k < c; ++k) {
                const uint32_t v = (uint32_t)planes[(size_t)k * w * h + (size_t)y * w + x];
                const size_t i = (size_t)x * c + k;
                if (one) row[i] = (uint8_t)v;
                else { row[2 * i] = (uint8_t)(v >> 8); row[2 * i + 1] = (uint8_t)v; }
            }
        fwrite(row.data(), 1, row.size(), f);
    }
    return fclose(f) == 0;
}

static int plugin_mode(int argc, char **argv) {
    if (argc < 9) return 2;
    const char *dir = argv[2];
    const uint32_t w = (uint32_t)atoi(argv[5]), h = (uint32_t)atoi(argv[6]), c = (uint32_t)atoi(argv[7]);
    const uint32_t bits = (uint32_t)atoi(argv[8]);
    std::vector<uint8_t> in = read_file(argv[3]);
    if (in.size() != (size_t)w * h * c * 4) { fprintf(stderr, "input size mismatch\n"); return 2; }
    const std::string pnm = std::string(argv[4]) + (c == 1 ? ".pgm" : ".ppm");
    if (!write_pnm(pnm.c_str(), (const int32_t *)in.data(), w, h, c, bits)) { fprintf(stderr, "pnm\n"); return 2; }
    if (!grk_initialize(dir, 0)) { fprintf(stderr, "plugin not loaded from %s\n", dir); return 4; }
    grk_plugin_init_info ii;
    ii.deviceId = 0;
    ii.verbose = getenv("GRKGPU_PLUGIN_VERBOSE") != nullptr;
    if (!grk_plugin_init(ii)) { fprintf(stderr, "grk_plugin_init failed\n"); return 4; }
    grk_cparameters p;
    if (!parse_enc_opts(&p, argc - 9, argv + 9)) return 2;
    snprintf(p.infile, sizeof(p.infile), "%s", pnm.c_str());
    snprintf(p.outfile, sizeof(p.outfile), "%s", argv[4]);
    p.decod_format = GRK_PXM_FMT;
    p.cod_format = GRK_J2K_FMT;
    const int32_t rc = grk_plugin_encode(&p, plugin_cb);
    remove(pnm.c_str());
    if (rc != 0) { fprintf(stderr, "plugin declined (rc %d)\n", rc); grk_deinitialize(); return 3; }
    if (!g_cb_ok) { fprintf(stderr, "host encode with plugin tile failed\n"); grk_deinitialize(); return 1; }
    write_file(argv[4], g_cb_out.data(), g_cb_out.size());
    printf("debug_state=%u host_warnings=%d\n", grk_plugin_get_debug_state(), g_warnings);
    grk_deinitialize();
    return 0;
}

// ---- batch encode: callbacks come from the plugin's worker threads ----
static std::atomic<int> g_batch_written{0}, g_batch_failed{0};
static std::string g_batch_out;

static bool plugin_batch_cb(grk_plugin_encode_user_callback_info *info) {
    // plugin_compress_callback (grk_compress.cpp:1783-1797): a relative output
    // name is the part of the file name before its first '.' (get_file_name,
    // common.cpp:245-248), placed in the output directory
    std::string name = info->output_file_name ? info->output_file_name : "";
    const std::string stem = name.substr(0, name.find('.'));
    const std::string out = g_batch_out + "/" + stem + ".j2k";
    grk_cparameters *p = info->encoder_parameters;
    grk_image *img = info->image;
    if (!img) { g_batch_failed++; return false; }
    if (p->tcp_mct == 255) p->tcp_mct = img->numcomps >= 3 ? 1 : 0;        // grk_compress.cpp:1997-1998
    if (p->rateControlAlgorithm == 255) p->rateControlAlgorithm = 0;        // :2015-2017
    const size_t cap = (size_t)(img->x1 - img->x0) * (img->y1 - img->y0) * img->numcomps * 3 + (1 << 20);
    std::vector<uint8_t> buf(cap);
    grk_stream *st = grk_stream_create_mem_stream(buf.data(), cap, false, false);
    grk_codec *codec = grk_create_compress(GRK_CODEC_J2K, st);
    bool ok = codec && grk_setup_encoder(codec, p, img) && grk_start_compress(codec, img) &&
              grk_encode_with_plugin(codec, info->tile) && grk_end_compress(codec);
    if (ok) {
        write_file(out.c_str(), buf.data(), grk_stream_get_write_mem_stream_length(st));
        g_batch_written++;
    } else {
        g_batch_failed++;
    }
    if (codec) grk_destroy_codec(codec);
    grk_stream_destroy(st);
    return ok;
}

static int plugin_batch_mode(int argc, char **argv) {
    if (argc < 5) return 2;
    grk_set_error_handler(err_cb, nullptr);
    grk_set_warning_handler(warn_cb, nullptr);
    if (!grk_initialize(argv[2], 0)) { fprintf(stderr, "plugin not loaded from %s\n", argv[2]); return 4; }
    grk_plugin_init_info ii;
    ii.deviceId = -1;  // "-1 = all devices" (grk_compress -G, grok.h:1816-1821)
    ii.verbose = getenv("GRKGPU_PLUGIN_VERBOSE") != nullptr;
    if (!grk_plugin_init(ii)) { fprintf(stderr, "grk_plugin_init failed\n"); return 4; }
    grk_cparameters p;
    if (!parse_enc_opts(&p, argc - 5, argv + 5)) return 2;
    p.decod_format = GRK_PXM_FMT;
    p.cod_format = GRK_J2K_FMT;
    g_batch_out = argv[4];
    int32_t rc = grk_plugin_batch_encode(argv[3], argv[4], &p, plugin_batch_cb);
    if (rc == 0) {  // started: wait for completion in 100 ms slices (grk_compress.cpp:2229-2241)
        for (uint32_t i = 0; i < 6000; ++i) {
            usleep(100 * 1000);
            if (grk_plugin_is_batch_complete()) break;
        }
        grk_plugin_stop_batch_encode();
    }
    grk_deinitialize();
    if (rc != 0) { fprintf(stderr, "plugin declined the batch\n"); return 3; }
    printf("written=%d failed=%d\n", g_batch_written.load(), g_batch_failed.load());
    return g_batch_failed ? 1 : 0;
}

// ---- plugin decode mode: grk_decompress's decode_callback (grk_decompress.cpp:1336-1557) ----
static std::string g_dec_out;

static int dec_pre(grk_plugin_decode_callback_info *info) {
    grk_decompress_parameters *p = info->decoder_parameters;
    const char *infile = info->input_file_name ? info->input_file_name : p->infile;
    int failed = 0;
    if (!info->l_stream) info->l_stream = grk_stream_create_mapped_file_read_stream(infile);
    if (!info->l_stream) return 1;
    if (!info->l_codec) {
        info->l_codec = grk_create_decompress(GRK_CODEC_J2K, info->l_stream);
        grk_set_error_handler(err_cb, nullptr);
        if (!grk_setup_decoder(info->l_codec, &p->core)) failed = 1;
    }
    if (!failed && (info->decode_flags & GRK_DECODE_HEADER)) {
        if (!grk_read_header(info->l_codec, &info->header_info, &info->image)) failed = 1;
        else if (info->init_decoders_func) return info->init_decoders_func(&info->header_info, info->image);
    }
    if (!failed && info->decode_flags != GRK_DECODE_HEADER) {
        if (info->tile) info->tile->decode_flags = info->decode_flags;
        if (!grk_set_decode_area(info->l_codec, info->image, p->DA_x0, p->DA_y0, p->DA_x1, p->DA_y1) ||
            !grk_decode(info->l_codec, info->tile, info->image) || !grk_end_decompress(info->l_codec))
            failed = 1;
    }
    grk_stream_destroy(info->l_stream);
    info->l_stream = nullptr;
    grk_destroy_codec(info->l_codec);
    info->l_codec = nullptr;
    if (failed && info->image) {
        grk_image_destroy(info->image);
        info->image = nullptr;
    }
    return failed;
}

static int dec_post(grk_plugin_decode_callback_info *info) {
    grk_image *img = info->image;
    if (!img) return 1;
    std::vector<int32_t> out;
    for (uint32_t k = 0; k < img->numcomps; ++k) {
        const grk_image_comp &cm = img->comps[k];
        if (!cm.data) return 1;
        out.insert(out.end(), cm.data, cm.data + (size_t)cm.w * cm.h);
    }
    // post_decode's output name (grk_decompress.cpp:1577-1579): the
    // parameters' outfile, else the one the plugin gives (batch)
    const char *dst = info->decoder_parameters->outfile[0] ? g_dec_out.c_str() : info->output_file_name;
    if (!dst) return 1;
    write_file(dst, out.data(), out.size() * 4);
    printf("%u %u %u %u %u %u %u %u %u\n", img->x0, img->y0, img->x1, img->y1, img->numcomps, img->comps[0].prec,
           img->comps[0].sgnd, img->comps[0].w, img->comps[0].h);
    return 0;
}

static int32_t dec_callback(grk_plugin_decode_callback_info *info) {
    int rc = -1;
    if (info->decode_flags & GRK_DECODE_T1) info->init_decoders_func = nullptr;
    if (info->decode_flags & GRK_PLUGIN_DECODE_CLEAN) {
        if (info->l_stream) grk_stream_destroy(info->l_stream);
        info->l_stream = nullptr;
        if (info->l_codec) grk_destroy_codec(info->l_codec);
        info->l_codec = nullptr;
        if (info->image && !info->plugin_owns_image) {
            grk_image_destroy(info->image);
            info->image = nullptr;
        }
        rc = 0;
    }
    if (info->decode_flags & (GRK_DECODE_HEADER | GRK_DECODE_T1 | GRK_DECODE_T2)) {
        rc = dec_pre(info);
        if (rc) return rc;
    }
    if (info->decode_flags & GRK_DECODE_POST_T1) rc = dec_post(info);
    return rc;
}

static int plugin_batch_dec_mode(int argc, char **argv) {
    if (argc < 5) return 2;
    grk_decompress_parameters p;
    memset(&p, 0, sizeof(p));
    grk_set_default_decoder_parameters(&p.core);
    p.decod_format = GRK_J2K_FMT;
    p.cod_format = GRK_RAWL_FMT;
    if (!grk_initialize(argv[2], 0)) { fprintf(stderr, "plugin not loaded from %s\n", argv[2]); return 4; }
    grk_plugin_init_info ii;
    ii.deviceId = -1;
    ii.verbose = getenv("GRKGPU_PLUGIN_VERBOSE") != nullptr;
    if (!grk_plugin_init(ii)) { fprintf(stderr, "grk_plugin_init failed\n"); return 4; }
    // grk_decompress.cpp:1242-1262, as written there: the batch is started
    // only if the init returns non-zero, and waited for if that start returns 0
    int32_t success = grk_plugin_init_batch_decode(argv[3], argv[4], &p, dec_callback);
    if (success) success = grk_plugin_batch_decode();
    if (success == 0) {
        for (uint32_t i = 0; i < 6000; ++i) {
            usleep(100 * 1000);
            if (grk_plugin_is_batch_complete()) break;
        }
        grk_plugin_stop_batch_decode();
    }
    grk_deinitialize();
    return success == 0 ? 0 : 3;
}

static int plugin_dec_mode(int argc, char **argv) {
    if (argc < 5) return 2;
    grk_decompress_parameters p;
    memset(&p, 0, sizeof(p));
    grk_set_default_decoder_parameters(&p.core);
    for (int i = 5; i + 1 < argc; i += 2) {
        std::string a = argv[i];
        if (a == "-r") p.core.cp_reduce = (uint32_t)atoi(argv[i + 1]);
        else if (a == "-l") p.core.cp_layer = (uint32_t)atoi(argv[i + 1]);
        else if (a == "-d") {
            if (sscanf(argv[i + 1], "%u,%u,%u,%u", &p.DA_x0, &p.DA_y0, &p.DA_x1, &p.DA_y1) != 4) return 2;
        } else return 2;
    }
    snprintf(p.infile, sizeof(p.infile), "%s", argv[3]);
    snprintf(p.outfile, sizeof(p.outfile), "%s", argv[4]);
    p.decod_format = GRK_J2K_FMT;
    p.cod_format = GRK_RAWL_FMT;
    g_dec_out = argv[4];
    if (!grk_initialize(argv[2], 0)) { fprintf(stderr, "plugin not loaded from %s\n", argv[2]); return 4; }
    grk_plugin_init_info ii;
    ii.deviceId = 0;
    ii.verbose = getenv("GRKGPU_PLUGIN_VERBOSE") != nullptr;
    if (!grk_plugin_init(ii)) { fprintf(stderr, "grk_plugin_init failed\n"); return 4; }
    const int32_t rc = grk_plugin_decode(&p, dec_callback);
    grk_deinitialize();
    if (rc == -1) { fprintf(stderr, "plugin declined\n"); return 3; }
    return rc ? 1 : 0;
}

// ---- concurrent codecs (thread-safety of the library) ----
static int mt_mode(int argc, char **argv) {
    if (argc < 11) return 2;
    const uint32_t w = (uint32_t)atoi(argv[4]), h = (uint32_t)atoi(argv[5]), c = (uint32_t)atoi(argv[6]);
    const uint32_t bits = (uint32_t)atoi(argv[7]), sgnd = (uint32_t)atoi(argv[8]);
    const uint32_t threads = (uint32_t)atoi(argv[9]), reps = (uint32_t)atoi(argv[10]);
    std::vector<uint8_t> in = read_file(argv[2]);
    const std::vector<uint8_t> expect = read_file(argv[3]);
    if (in.size() != (size_t)w * h * c * 4) { fprintf(stderr, "input size mismatch\n"); return 2; }
    grk_initialize(nullptr, 0);
    std::vector<int32_t> first;
    {  // reference decode of the expected stream, single-threaded
        grk_codec *codec;
        grk_stream *st;
        const uint32_t area[4] = {0, 0, 0, 0};
        grk_image *img = decode(expect.data(), expect.size(), 0, 0, area, &codec, &st);
        if (!img) { fprintf(stderr, "decode failed\n"); return 1; }
        for (uint32_t k = 0; k < img->numcomps; ++k)
            first.insert(first.end(), img->comps[k].data, img->comps[k].data + (size_t)img->comps[k].w * img->comps[k].h);
        grk_destroy_codec(codec);
        grk_stream_destroy(st);
    }
    std::atomic<int> bad{0};
    std::vector<std::thread> pool;
    for (uint32_t t = 0; t < threads; ++t)
        pool.emplace_back([&]() {
            for (uint32_t r = 0; r < reps; ++r) {
                grk_cparameters p;
                std::vector<uint8_t> cs;
                if (!parse_enc_opts(&p, argc - 11, argv + 11) ||
                    !encode(&p, (const int32_t *)in.data(), w, h, c, bits, sgnd, cs) || cs != expect) {
                    bad++;
                    continue;
                }
                grk_codec *codec;
                grk_stream *st;
                const uint32_t area[4] = {0, 0, 0, 0};
                grk_image *img = decode(cs.data(), cs.size(), 0, 0, area, &codec, &st);
                if (!img) { bad++; continue; }
                size_t off = 0;
                for (uint32_t k = 0; k < img->numcomps; ++k) {
                    const size_t n = (size_t)img->comps[k].w * img->comps[k].h;
                    if (off + n > first.size() || memcmp(img->comps[k].data, first.data() + off, n * 4)) bad++;
                    off += n;
                }
                grk_destroy_codec(codec);
                grk_stream_destroy(st);
            }
        });
    for (auto &th : pool) th.join();
    grk_deinitialize();
    if (bad) fprintf(stderr, "%d mismatching results\n", bad.load());
    return bad ? 1 : 0;
}

int main(int argc, char **argv) {
    if (argc < 4 && !(argc == 3 && (std::string(argv[1]) == "info" || std::string(argv[1]) == "index"))) {
        fprintf(stderr, "usage: see oracle/ref_driver.cpp\n");
        return 2;
    }
    const std::string mode = argv[1];
    if (mode == "plugin") return plugin_mode(argc, argv);
    if (mode == "plugin-dec") return plugin_dec_mode(argc, argv);
    if (mode == "mt") return mt_mode(argc, argv);
    if (mode == "plugin-batch") return plugin_batch_mode(argc, argv);
    if (mode == "plugin-batch-dec") return plugin_batch_dec_mode(argc, argv);
    if (mode == "enc" || mode == "bench") {
        const bool bench = mode == "bench";
        const int need = bench ? 10 : 9;
        if (argc < need) return 2;
        int ai = bench ? 3 : 4;
        const uint32_t w = (uint32_t)atoi(argv[ai]), h = (uint32_t)atoi(argv[ai + 1]), c = (uint32_t)atoi(argv[ai + 2]);
        const uint32_t bits = (uint32_t)atoi(argv[ai + 3]), sgnd = (uint32_t)atoi(argv[ai + 4]);
        uint32_t threads = 0, reps = 1;
        ai += 5;
        if (bench) { threads = (uint32_t)atoi(argv[ai]); reps = (uint32_t)atoi(argv[ai + 1]); ai += 2; }
        std::vector<uint8_t> in = read_file(argv[2]);
        {
            grk_cparameters p0;  // the offset and -sub decide the plane sizes
            if (!parse_enc_opts(&p0, argc - ai, argv + ai)) return 2;
            size_t need = 0;
            for (uint32_t k = 0; k < c; ++k) {
                uint32_t cw, ch;
                comp_size(&p0, w, h, k, &cw, &ch);
                need += (size_t)cw * ch * 4;
            }
            if (in.size() != need) { fprintf(stderr, "input size mismatch\n"); return 2; }
        }
        grk_initialize(nullptr, threads);  // returns "plugin loaded": none is, CPU path
        std::vector<uint8_t> cs;
        double t_enc = 0, t_dec = 0;
        for (uint32_t r = 0; r < reps; ++r) {
            grk_cparameters p;
            if (!parse_enc_opts(&p, argc - ai, argv + ai)) return 2;
            auto t0 = std::chrono::steady_clock::now();
            if (!encode(&p, (const int32_t *)in.data(), w, h, c, bits, sgnd, cs)) { fprintf(stderr, "encode failed\n"); return 1; }
            auto t1 = std::chrono::steady_clock::now();
            t_enc += std::chrono::duration<double, std::milli>(t1 - t0).count();
            if (bench) {
                grk_codec *codec;
                grk_stream *st;
                const uint32_t area[4] = {0, 0, 0, 0};
                auto t2 = std::chrono::steady_clock::now();
                grk_image *img = decode(cs.data(), cs.size(), 0, 0, area, &codec, &st);
                auto t3 = std::chrono::steady_clock::now();
                if (!img) { fprintf(stderr, "decode failed\n"); return 1; }
                t_dec += std::chrono::duration<double, std::milli>(t3 - t2).count();
                grk_destroy_codec(codec);
                grk_stream_destroy(st);
            }
        }
        if (bench) {
            printf("{\"enc_ms\": %.3f, \"dec_ms\": %.3f, \"reps\": %u, \"threads\": %u, \"bytes\": %zu}\n", t_enc / reps,
                   t_dec / reps, reps, threads, cs.size());
        } else {
            write_file(argv[3], cs.data(), cs.size());
        }
        grk_deinitialize();
        return 0;
    }
    if (mode == "info") {  // grk_dump-style: grk_read_header, then grk_get_cstr_info (grk_dump.cpp:494-500)
        std::vector<uint8_t> cs = read_file(argv[2]);
        grk_initialize(nullptr, 0);
        grk_stream *st = grk_stream_create_mem_stream(cs.data(), cs.size(), false, true);
        grk_codec *codec = grk_create_decompress(GRK_CODEC_J2K, st);
        grk_set_error_handler(err_cb, nullptr);
        grk_dparameters dp;
        grk_set_default_decoder_parameters(&dp);
        grk_header_info hi;
        memset(&hi, 0, sizeof(hi));
        grk_image *img = nullptr;
        if (!(codec && grk_setup_decoder(codec, &dp) && grk_read_header(codec, &hi, &img))) return 1;
        grk_codestream_info_v2 *ci = grk_get_cstr_info(codec);
        if (!ci) { fprintf(stderr, "no cstr info\n"); return 1; }
        printf("grid %u %u %u %u %u %u comps %u tile_info %d\n", ci->tx0, ci->ty0, ci->tdx, ci->tdy, ci->tw, ci->th,
               ci->nbcomps, ci->tile_info != nullptr);
        const grk_tile_info_v2 &t = ci->m_default_tile_info;
        printf("default tileno %u csty %u prg %d layers %u mct %u\n", t.tileno, t.csty, (int)t.prg, t.numlayers, t.mct);
        for (uint32_t k = 0; k < ci->nbcomps; ++k) {
            const grk_tccp_info &q = t.tccp_info[k];
            printf("comp %u compno %u csty %u res %u cblk %u %u sty %u qmfbid %u qntsty %u gbits %u roi %u\n", k,
                   q.compno, q.csty, q.numresolutions, q.cblkw, q.cblkh, q.cblk_sty, q.qmfbid, q.qntsty, q.numgbits,
                   q.roishift);
            printf(" steps");
            for (uint32_t b = 0; b < GRK_J2K_MAXBANDS; ++b) printf(" %u/%u", q.stepsizes_expn[b], q.stepsizes_mant[b]);
            printf("\n prc");
            for (uint32_t r = 0; r < GRK_J2K_MAXRLVLS; ++r) printf(" %ux%u", q.prcw[r], q.prch[r]);
            printf("\n");
        }
        grk_destroy_cstr_info(&ci);
        printf("destroyed %d\n", ci == nullptr);
        grk_destroy_codec(codec);
        grk_stream_destroy(st);
        grk_deinitialize();
        return 0;
    }
    if (mode == "index") {  // grk_get_cstr_index after grk_read_header, then after a full grk_decode
        std::vector<uint8_t> cs = read_file(argv[2]);
        grk_initialize(nullptr, 0);
        grk_stream *st = grk_stream_create_mem_stream(cs.data(), cs.size(), false, true);
        grk_codec *codec = grk_create_decompress(GRK_CODEC_J2K, st);
        grk_set_error_handler(err_cb, nullptr);
        grk_dparameters dp;
        grk_set_default_decoder_parameters(&dp);
        grk_header_info hi;
        memset(&hi, 0, sizeof(hi));
        grk_image *img = nullptr;
        if (!(codec && grk_setup_decoder(codec, &dp) && grk_read_header(codec, &hi, &img))) return 1;
        auto dump = [](grk_codestream_index *ix, const char *when) {
            if (!ix) { printf("%s none\n", when); return; }
            printf("%s main %llu %llu size %llu marknum %u\n", when, (unsigned long long)ix->main_head_start,
                   (unsigned long long)ix->main_head_end, (unsigned long long)ix->codestream_size, ix->marknum);
            for (uint32_t i = 0; i < ix->marknum && ix->marker; ++i)
                printf(" m %04x %llu %u\n", ix->marker[i].type, (unsigned long long)ix->marker[i].pos, ix->marker[i].len);
            printf(" tiles %u %d\n", ix->nb_of_tiles, ix->tile_index != nullptr);
            for (uint32_t t = 0; ix->tile_index && t < ix->nb_of_tiles; ++t) {
                const grk_tile_index &ti = ix->tile_index[t];
                printf(" tile %u tileno %u marknum %u nb_tps %u nb_packet %u\n", t, ti.tileno, ti.marknum, ti.nb_tps,
                       ti.nb_packet);
                for (uint32_t i = 0; i < ti.marknum && ti.marker; ++i)
                    printf("  m %04x %llu %u\n", ti.marker[i].type, (unsigned long long)ti.marker[i].pos, ti.marker[i].len);
                for (uint32_t i = 0; i < ti.nb_tps && ti.tp_index; ++i)
                    printf("  tp %llu %llu %llu\n", (unsigned long long)ti.tp_index[i].start_pos,
                           (unsigned long long)ti.tp_index[i].end_header, (unsigned long long)ti.tp_index[i].end_pos);
            }
        };
        grk_codestream_index *ix = grk_get_cstr_index(codec);
        dump(ix, "header");
        grk_destroy_cstr_index(&ix);
        if (!(grk_decode(codec, nullptr, img) && grk_end_decompress(codec))) return 1;
        ix = grk_get_cstr_index(codec);
        dump(ix, "decoded");
        grk_destroy_cstr_index(&ix);
        printf("destroyed %d\n", ix == nullptr);
        grk_destroy_codec(codec);
        grk_stream_destroy(st);
        grk_deinitialize();
        return 0;
    }
    if (mode == "dec") {
        uint32_t reduce = 0, layers = 0, area[4] = {0, 0, 0, 0};
        for (int i = 4; i + 1 < argc; i += 2) {
            std::string a = argv[i];
            if (a == "-r") reduce = (uint32_t)atoi(argv[i + 1]);
            else if (a == "-l") layers = (uint32_t)atoi(argv[i + 1]);
            else if (a == "-d") {
                if (sscanf(argv[i + 1], "%u,%u,%u,%u", &area[0], &area[1], &area[2], &area[3]) != 4) return 2;
            } else return 2;
        }
        std::vector<uint8_t> cs = read_file(argv[2]);
        grk_initialize(nullptr, 0);
        grk_codec *codec;
        grk_stream *st;
        grk_image *img = decode(cs.data(), cs.size(), reduce, layers, area, &codec, &st);
        if (!img) { fprintf(stderr, "decode failed\n"); return 1; }
        std::vector<int32_t> out;
        for (uint32_t k = 0; k < img->numcomps; ++k) {
            const grk_image_comp &cm = img->comps[k];
            out.insert(out.end(), cm.data, cm.data + (size_t)cm.w * cm.h);
        }
        write_file(argv[3], out.data(), out.size() * 4);
        printf("%u %u %u %u %u %u %u %u %u\n", img->x0, img->y0, img->x1, img->y1, img->numcomps, img->comps[0].prec,
               img->comps[0].sgnd, img->comps[0].w, img->comps[0].h);
        printf("comps");  // each component's plane (subsampled ones differ)
        for (uint32_t k = 0; k < img->numcomps; ++k)
            printf(" %u %u %u %u", img->comps[k].w, img->comps[k].h, img->comps[k].dx, img->comps[k].dy);
        printf("\n");
        grk_destroy_codec(codec);
        grk_stream_destroy(st);
        grk_deinitialize();
        return 0;
    }
    return 2;
}
