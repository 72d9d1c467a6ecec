// oracle/tile_driver.cpp -- the reference's tile-streaming test programs,
// restated as one driver over the grk_* C API (test infrastructure only).
// Built twice by oracle/ref.mk: against the REFERENCE libgrok (oracle/_ref/
// tile_driver) and against OUR libgrok.so (oracle/_ref/tile_driver_mi355x);
// tests/test_gpu_grk_api.py runs both with the same arguments and compares
// their outputs byte for byte.
//
//   tile_driver enc NUMCOMPS W H TW TH PREC IRREV OUT.j2k
//       what tests/test_tile_encoder.cpp does (ctest tte0..5,
//       tests/CMakeLists.txt:92-97): an image of NUMCOMPS unsigned PREC-bit
//       components, tiles TW x TH, one fixed-quality layer at 20 dB
//       (cp_fixed_quality, tcp_distoratio[0] = 20), 6 resolutions, LRCP;
//       grk_start_compress, then grk_write_tile for every tile in order with
//       the byte ramp data[i] = (uint8_t)i (test_tile_encoder.cpp:158),
//       grk_end_compress, into a file stream.
//       Optional SUB after IRREV: 420 / 422 -- components 1.. on a 2 x 2 /
//       2 x 1 grid (SIZ XRsiz / YRsiz); each tile's data is then every
//       component's tile-component, one after the other
//       (TileProcessor::copy_image_data_to_tile).
//   tile_driver dec X0 Y0 X1 Y1 IN.j2k OUT.bin
//       what tests/test_tile_decoder.cpp does (ttd0..2): grk_read_header,
//       grk_set_decode_area, then grk_read_tile_header / grk_decode_tile_data
//       until the codestream has no tile left (X1 = Y1 = 0: no decode area
//       is set); OUT.bin receives, per tile,
//       its index, rectangle, component count, data size and data.
//   tile_driver rta IN.j2k OUT.bin
//       what tests/j2k_random_tile_access.cpp does (rta1..5): grk_get_decoded_tile
//       for the first, the last and two middle tiles, in that order, each on
//       a fresh decompressor; OUT.bin receives each tile's samples.
#include <grok.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

static void err_cb(const char *msg, void *) { fprintf(stderr, "[grk error] %s", msg); }

static void put(FILE *f, uint64_t v) { fwrite(&v, 8, 1, f); }

static int enc_mode(int argc, char **argv) {
    if (argc < 10) return 2;
    const uint32_t nc = (uint32_t)atoi(argv[2]), w = (uint32_t)atoi(argv[3]), h = (uint32_t)atoi(argv[4]);
    const uint32_t tw = (uint32_t)atoi(argv[5]), th = (uint32_t)atoi(argv[6]), prec = (uint32_t)atoi(argv[7]);
    const bool irrev = atoi(argv[8]) != 0;
    const int sub = argc > 10 ? atoi(argv[10]) : 0;
    const char *outp = argc > 10 ? argv[9] : argv[9];
    const uint32_t sdx = sub == 420 || sub == 422 ? 2 : 1, sdy = sub == 420 ? 2 : 1;
    grk_initialize(nullptr, 0);
    grk_cparameters p;
    grk_set_default_encoder_parameters(&p);
    p.tcp_numlayers = 1;
    p.cp_fixed_quality = 1;
    p.tcp_distoratio[0] = 20;
    p.cp_tx0 = p.cp_ty0 = 0;
    p.tile_size_on = true;
    p.cp_tdx = tw;
    p.cp_tdy = th;
    p.irreversible = irrev;
    p.numresolution = 6;
    p.prog_order = GRK_LRCP;
    std::vector<grk_image_cmptparm> cm(nc);
    memset(cm.data(), 0, nc * sizeof(grk_image_cmptparm));
    for (uint32_t k = 0; k < nc; ++k) {
        cm[k].dx = k ? sdx : 1;
        cm[k].dy = k ? sdy : 1;
        cm[k].w = (w + cm[k].dx - 1) / cm[k].dx;
        cm[k].h = (h + cm[k].dy - 1) / cm[k].dy;
        cm[k].prec = prec;
    }
    grk_stream *st = grk_stream_create_file_stream(outp, 1024 * 1024, false);
    grk_codec *codec = st ? grk_create_compress(GRK_CODEC_J2K, st) : nullptr;
    grk_set_error_handler(err_cb, nullptr);
    grk_image *img = grk_image_create(nc, cm.data(), GRK_CLRSPC_SRGB);
    if (img) {  // the image area (test_tile_encoder.cpp:280-284)
        img->x0 = img->y0 = 0;
        img->x1 = w;
        img->y1 = h;
        img->color_space = GRK_CLRSPC_SRGB;
    }
    int rc = 0;
    if (!codec || !img || !grk_setup_encoder(codec, &p, img) || !grk_start_compress(codec, img)) rc = 1;
    // every tile carries the same ramp (the reference test sizes it for a full tile)
    uint64_t tile_bytes = 0;
    for (uint32_t k = 0; k < nc; ++k)
        tile_bytes += (uint64_t)((tw + cm[k].dx - 1) / cm[k].dx) * ((th + cm[k].dy - 1) / cm[k].dy) * (prec / 8);
    std::vector<uint8_t> data(tile_bytes);
    for (uint64_t i = 0; i < tile_bytes; ++i) data[i] = (uint8_t)i;
    const uint32_t ntiles = (w / tw) * (h / th);
    for (uint32_t t = 0; rc == 0 && t < ntiles; ++t)
        if (!grk_write_tile(codec, (uint16_t)t, data.data(), tile_bytes)) rc = 1;
    if (rc == 0 && !grk_end_compress(codec)) rc = 1;
    if (st) grk_stream_destroy(st);
    if (codec) grk_destroy_codec(codec);
    if (img) grk_image_destroy(img);
    grk_deinitialize();
    return rc;
}

static grk_codec *open_dec(const char *path, grk_stream **st, grk_image **img) {
    *st = grk_stream_create_file_stream(path, 1024 * 1024, true);
    if (!*st) return nullptr;
    grk_codec *codec = grk_create_decompress(GRK_CODEC_J2K, *st);
    grk_set_error_handler(err_cb, nullptr);
    grk_dparameters dp;
    grk_set_default_decoder_parameters(&dp);
    if (!codec || !grk_setup_decoder(codec, &dp) || !grk_read_header(codec, nullptr, img)) return nullptr;
    return codec;
}

static int dec_mode(int argc, char **argv) {
    if (argc < 8) return 2;
    const uint32_t x0 = (uint32_t)atoi(argv[2]), y0 = (uint32_t)atoi(argv[3]), x1 = (uint32_t)atoi(argv[4]),
                   y1 = (uint32_t)atoi(argv[5]);
    grk_initialize(nullptr, 0);
    grk_stream *st = nullptr;
    grk_image *img = nullptr;
    grk_codec *codec = open_dec(argv[6], &st, &img);
    FILE *out = fopen(argv[7], "wb");
    // X1 = Y1 = 0: no grk_set_decode_area call (the whole image)
    const bool area = x1 || y1;
    int rc = codec && out && (!area || grk_set_decode_area(codec, img, x0, y0, x1, y1)) ? 0 : 1;
    bool go_on = true;
    std::vector<uint8_t> data;
    while (rc == 0 && go_on) {
        uint16_t t = 0;
        uint64_t size = 0;
        uint32_t tx0, ty0, tx1, ty1, ncomp;
        if (!grk_read_tile_header(codec, &t, &size, &tx0, &ty0, &tx1, &ty1, &ncomp, &go_on)) { rc = 1; break; }
        if (!go_on) break;
        data.assign(size, 0);
        if (!grk_decode_tile_data(codec, t, data.data(), size)) { rc = 1; break; }
        put(out, t); put(out, tx0); put(out, ty0); put(out, tx1); put(out, ty1); put(out, ncomp); put(out, size);
        fwrite(data.data(), 1, size, out);
    }
    if (out) fclose(out);
    if (codec) grk_destroy_codec(codec);
    if (st) grk_stream_destroy(st);
    if (img) grk_image_destroy(img);
    grk_deinitialize();
    return rc;
}

static int rta_mode(int argc, char **argv) {
    if (argc < 4) return 2;
    grk_initialize(nullptr, 0);
    FILE *out = fopen(argv[3], "wb");
    if (!out) return 1;
    int rc = 0;
    uint32_t ntiles = 0;
    {
        grk_stream *st = nullptr;
        grk_image *img = nullptr;
        grk_header_info hi;
        memset(&hi, 0, sizeof(hi));
        st = grk_stream_create_file_stream(argv[2], 1024 * 1024, true);
        grk_codec *codec = st ? grk_create_decompress(GRK_CODEC_J2K, st) : nullptr;
        grk_dparameters dp;
        grk_set_default_decoder_parameters(&dp);
        if (codec && grk_setup_decoder(codec, &dp) && grk_read_header(codec, &hi, &img)) ntiles = hi.cp_tw * hi.cp_th;
        if (codec) grk_destroy_codec(codec);
        if (st) grk_stream_destroy(st);
        if (img) grk_image_destroy(img);
    }
    if (!ntiles) rc = 1;
    const uint32_t pick[4] = {0, ntiles - 1, ntiles / 2, ntiles / 3};
    for (uint32_t i = 0; rc == 0 && i < 4; ++i) {
        grk_stream *st = nullptr;
        grk_image *img = nullptr;
        grk_codec *codec = open_dec(argv[2], &st, &img);
        if (!codec || !grk_get_decoded_tile(codec, img, (uint16_t)pick[i])) rc = 1;
        for (uint32_t k = 0; rc == 0 && k < img->numcomps; ++k) {
            const grk_image_comp &cm = img->comps[k];
            put(out, pick[i]); put(out, cm.x0); put(out, cm.y0); put(out, cm.w); put(out, cm.h);
            if (cm.data) fwrite(cm.data, 4, (size_t)cm.w * cm.h, out);
        }
        if (codec) grk_destroy_codec(codec);
        if (st) grk_stream_destroy(st);
        if (img) grk_image_destroy(img);
    }
    fclose(out);
    grk_deinitialize();
    return rc;
}

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    const std::string mode = argv[1];
    if (mode == "enc") return enc_mode(argc, argv);
    if (mode == "dec") return dec_mode(argc, argv);
    if (mode == "rta") return rta_mode(argc, argv);
    return 2;
}
