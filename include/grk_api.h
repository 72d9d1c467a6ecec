/* grk_api.h -- Grok's public C API (grok.h, Grok v5.1.0) as exported by
 * grokimagecompression_amd/lib/libgrok.so, the drop-in replacement of the
 * reference's libgrok for grk_compress / grk_decompress and any other grk_*
 * user (north_star: "keeping the grk_/opj_ C API so it drops
 * in under grk_compress/grk_decompress").
 *
 * Same function names, argument meaning, return conventions and structure
 * layouts as the reference (the structures are the re-declarations of
 * grk_plugin_abi.h, checked field by field against the reference's headers by
 * oracle/abi/).  Behind it: the MI355X path of grk_mi355x.h (DC shift, MCT,
 * DWT, T1 and the codestream assembly on the GPU; rate control, Tier-2 and
 * markers on the host).
 *
 * Scope (what a call outside it does: returns false / nullptr after an error
 * message through the grk_set_error_handler callback):
 *   - raw J2K codestreams (GRK_CODEC_J2K); JP2 boxes are not written / read;
 *   - components with dx = dy = 1, up to 16 bits, at most 16 components;
 *   - coding options of grk_mi355x.h: any tiling, 5/3 or 9/7, RCT / ICT,
 *     code-block sizes, precincts, the five progressions, POC, SOP / EPH,
 *     tile-parts, quality layers with -r / -q rate control (both PCRD
 *     algorithms), the cinema 2K / 4K profiles, the code-block mode switches
 *     (cblk_sty BYPASS / RESET / TERMALL / VSC / PTERM / SEGSYM) and ROI
 *     (roi_compno / roi_shift); not HTJ2K (isHT) or custom MCT (grk_set_MCT);
 *   - encode tile by tile: grk_write_tile (tiles in order, as the reference's
 *     test_tile_encoder);
 *   - decode: whole image, cp_reduce, cp_layer, grk_set_decode_area windows,
 *     single tiles (grk_get_decoded_tile) and tile-by-tile streaming
 *     (grk_read_tile_header / grk_decode_tile_data); the main header's
 *     codestream info (grk_get_cstr_info, after grk_read_header); the
 *     codestream index (grk_get_cstr_index: marker / tile-part positions) is
 *     not provided (nullptr);
 *   - the plugin entry points report "no plugin" (this library IS the
 *     accelerated path).
 */
#ifndef GRK_API_H
#define GRK_API_H

#include <stdio.h>

#include "grk_plugin_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef grkp_poc grk_poc;
typedef grkp_raw_cparameters grk_raw_cparameters;
typedef grkp_cparameters grk_cparameters;
typedef grkp_image_comp grk_image_comp;
typedef grkp_image grk_image;
typedef grkp_image_cmptparm grk_image_cmptparm;
typedef grkp_header_info grk_header_info;
typedef grkp_dparameters grk_dparameters;
typedef grkp_decompress_parameters grk_decompress_parameters;
typedef void *grk_codec;   /* grok.h:797 */
typedef void *grk_stream;  /* grok.h:836 */

/* Codestream index (grok.h:950-1214, filled by j2k_get_cstr_index,
 * j2k_dump.cpp:402-517): marker and tile-part positions recorded while
 * decoding; layouts checked by oracle/abi/. */
typedef struct grk_packet_info {     /* grok.h:953-962 */
    uint64_t start_pos, end_ph_pos, end_pos;
    double disto;
} grk_packet_info;
typedef struct grk_marker_info {     /* grok.h:967-974 */
    uint16_t type;
    uint64_t pos;
    uint32_t len;
} grk_marker_info;
typedef struct grk_tp_index {        /* grok.h:1161-1168 */
    uint64_t start_pos, end_header, end_pos;
} grk_tp_index;
typedef struct grk_tile_index {      /* grok.h:1173-1194 */
    uint16_t tileno;
    uint32_t nb_tps, current_nb_tps, current_tpsno;
    grk_tp_index *tp_index;
    uint32_t marknum;
    grk_marker_info *marker;
    uint32_t maxmarknum;
    uint32_t nb_packet;
    grk_packet_info *packet_index;
} grk_tile_index;
typedef struct grk_codestream_index { /* grok.h:1199-1214 */
    uint64_t main_head_start, main_head_end, codestream_size;
    uint32_t marknum;
    grk_marker_info *marker;
    uint32_t maxmarknum;
    uint32_t nb_of_tiles;
    grk_tile_index *tile_index;
} grk_codestream_index;

/* Codestream info of the main header (grok.h:1080-1156, filled by
 * j2k_get_cstr_info, j2k_dump.cpp:326-400); layouts checked by oracle/abi/. */
#define GRK_J2K_MAXBANDS (3 * GRKP_MAXRLVLS - 2)
typedef struct grk_tccp_info {      /* grok.h:1083-1113 */
    uint32_t compno;
    uint8_t csty;
    uint32_t numresolutions, cblkw, cblkh;
    uint8_t cblk_sty, qmfbid, qntsty;
    uint32_t stepsizes_mant[GRK_J2K_MAXBANDS];
    uint32_t stepsizes_expn[GRK_J2K_MAXBANDS];
    uint8_t numgbits;
    uint32_t roishift;
    uint32_t prcw[GRKP_MAXRLVLS];
    uint32_t prch[GRKP_MAXRLVLS];
} grk_tccp_info;
typedef struct grk_tile_info_v2 {   /* grok.h:1118-1132 */
    uint16_t tileno;
    uint32_t csty;
    int32_t prg;                    /* GRK_PROG_ORDER */
    uint32_t numlayers, mct;
    grk_tccp_info *tccp_info;
} grk_tile_info_v2;
typedef struct grk_codestream_info_v2 { /* grok.h:1137-1156 */
    uint32_t tx0, ty0, tdx, tdy, tw, th, nbcomps;
    grk_tile_info_v2 m_default_tile_info;
    grk_tile_info_v2 *tile_info;
} grk_codestream_info_v2;

typedef enum { GRK_CODEC_UNKNOWN = -1, GRK_CODEC_J2K = 0, GRK_CODEC_JP2 = 2 } GRK_CODEC_FORMAT; /* grok.h:365-368 */
typedef enum {                                                                           /* grok.h:348-359 */
    GRK_CLRSPC_UNKNOWN = 0, GRK_CLRSPC_UNSPECIFIED = 1, GRK_CLRSPC_SRGB = 2, GRK_CLRSPC_GRAY = 3,
    GRK_CLRSPC_SYCC = 4, GRK_CLRSPC_EYCC = 5, GRK_CLRSPC_CMYK = 6, GRK_CLRSPC_DEFAULT_CIE = 7,
    GRK_CLRSPC_CUSTOM_CIE = 8, GRK_CLRSPC_ICC = 9
} GRK_COLOR_SPACE;

typedef void (*grk_msg_callback)(const char *msg, void *client_data);                    /* grok.h:379 */
typedef size_t (*grk_stream_read_fn)(void *p_buffer, size_t nb_bytes, void *p_user_data); /* grok.h:808-831 */
typedef size_t (*grk_stream_zero_copy_read_fn)(void **p_buffer, size_t nb_bytes, void *p_user_data);
typedef size_t (*grk_stream_write_fn)(void *p_buffer, size_t nb_bytes, void *p_user_data);
typedef bool (*grk_stream_seek_fn)(uint64_t nb_bytes, void *p_user_data);
typedef void (*grk_stream_free_user_data_fn)(void *p_user_data);

typedef struct { const char *plugin_path; } grk_plugin_load_info; /* grok.h:1797-1799 */
typedef struct grk_plugin_encode_user_callback_info grk_plugin_encode_user_callback_info;
typedef bool (*GRK_PLUGIN_ENCODE_USER_CALLBACK)(grk_plugin_encode_user_callback_info *info);
typedef struct grk_plugin_decode_callback_info grk_plugin_decode_callback_info;
typedef int32_t (*grk_plugin_decode_callback)(grk_plugin_decode_callback_info *info);

/* library (grok.h:1280-1288) */
const char *grk_version(void);
bool grk_initialize(const char *plugin_path, uint32_t numthreads);
void grk_deinitialize(void);

/* images (grok.h:1297-1321) */
grk_image *grk_image_create(uint32_t numcmpts, grk_image_cmptparm *cmptparms, GRK_COLOR_SPACE clrspc);
void grk_image_destroy(grk_image *image);
void grk_image_all_components_data_free(grk_image *image);
void grk_image_single_component_data_free(grk_image_comp *comp);
bool grk_image_single_component_data_alloc(grk_image_comp *comp);
uint8_t *grk_buffer_new(size_t len);
void grk_buffer_delete(uint8_t *buffer);

/* streams (grok.h:1336-1430) */
grk_stream *grk_stream_create(size_t buffer_size, bool is_input);
void grk_stream_destroy(grk_stream *stream);
void grk_stream_set_read_function(grk_stream *stream, grk_stream_read_fn fn);
void grk_stream_set_zero_copy_read_function(grk_stream *stream, grk_stream_zero_copy_read_fn fn);
void grk_stream_set_write_function(grk_stream *stream, grk_stream_write_fn fn);
void grk_stream_set_seek_function(grk_stream *stream, grk_stream_seek_fn fn);
void grk_stream_set_user_data(grk_stream *stream, void *data, grk_stream_free_user_data_fn fn);
void grk_stream_set_user_data_length(grk_stream *stream, uint64_t data_length);
grk_stream *grk_stream_create_file_stream(const char *fname, size_t buffer_size, bool is_read_stream);
grk_stream *grk_stream_create_mem_stream(uint8_t *buf, size_t buffer_len, bool owns_buffer, bool is_read_stream);
size_t grk_stream_get_write_mem_stream_length(grk_stream *stream);
grk_stream *grk_stream_create_mapped_file_read_stream(const char *fname);

/* messages (grok.h:1437-1450) */
bool grk_set_info_handler(grk_msg_callback cb, void *user_data);
bool grk_set_warning_handler(grk_msg_callback cb, void *user_data);
bool grk_set_error_handler(grk_msg_callback cb, void *user_data);

/* decompression (grok.h:1468-1595) */
grk_codec *grk_create_decompress(GRK_CODEC_FORMAT format, grk_stream *stream);
void grk_destroy_codec(grk_codec *codec);
bool grk_end_decompress(grk_codec *codec);
void grk_set_default_decoder_parameters(grk_dparameters *parameters);
bool grk_setup_decoder(grk_codec *codec, grk_dparameters *parameters);
bool grk_read_header(grk_codec *codec, grk_header_info *header_info, grk_image **image);
bool grk_set_decode_area(grk_codec *codec, grk_image *image, uint32_t start_x, uint32_t start_y, uint32_t end_x,
                         uint32_t end_y);
bool grk_decode(grk_codec *codec, grk_plugin_tile *tile, grk_image *image);
bool grk_get_decoded_tile(grk_codec *codec, grk_image *image, uint16_t tile_index);
bool grk_read_tile_header(grk_codec *codec, uint16_t *tile_index, uint64_t *data_size, uint32_t *tile_x0,
                          uint32_t *tile_y0, uint32_t *tile_x1, uint32_t *tile_y1, uint32_t *nb_comps,
                          bool *should_go_on);
bool grk_decode_tile_data(grk_codec *codec, uint16_t tile_index, uint8_t *data, uint64_t data_size);

/* compression (grok.h:1640-1714) */
grk_codec *grk_create_compress(GRK_CODEC_FORMAT format, grk_stream *stream);
void grk_set_default_encoder_parameters(grk_cparameters *parameters);
bool grk_setup_encoder(grk_codec *codec, grk_cparameters *parameters, grk_image *image);
bool grk_start_compress(grk_codec *codec, grk_image *image);
bool grk_end_compress(grk_codec *codec);
bool grk_encode(grk_codec *codec);
bool grk_encode_with_plugin(grk_codec *codec, grk_plugin_tile *tile);
bool grk_write_tile(grk_codec *codec, uint16_t tile_index, uint8_t *data, uint64_t data_size);
bool grk_set_MCT(grk_cparameters *parameters, float *encoding_matrix, int32_t *dc_shift, uint32_t nb_comp);

/* codestream information (grok.h:1720-1760) */
void grk_dump_codec(grk_codec *codec, int32_t info_flag, FILE *output_stream);
grk_codestream_info_v2 *grk_get_cstr_info(grk_codec *codec);
void grk_destroy_cstr_info(grk_codestream_info_v2 **cstr_info);
grk_codestream_index *grk_get_cstr_index(grk_codec *codec);
void grk_destroy_cstr_index(grk_codestream_index **cstr_index);

/* plugin management (grok.h:1797-1891): no external plugin under this library */
bool grk_plugin_load(grk_plugin_load_info info);
void grk_plugin_cleanup(void);
bool grk_plugin_init(grk_plugin_init_info init_info);
uint32_t grk_plugin_get_debug_state(void);
int32_t grk_plugin_encode(grk_cparameters *encode_parameters, GRK_PLUGIN_ENCODE_USER_CALLBACK callback);
int32_t grk_plugin_batch_encode(const char *input_dir, const char *output_dir, grk_cparameters *encode_parameters,
                                GRK_PLUGIN_ENCODE_USER_CALLBACK callback);
bool grk_plugin_is_batch_complete(void);
void grk_plugin_stop_batch_encode(void);
int32_t grk_plugin_decode(grk_decompress_parameters *decode_parameters, grk_plugin_decode_callback callback);
int32_t grk_plugin_init_batch_decode(const char *input_dir, const char *output_dir,
                                     grk_decompress_parameters *decode_parameters,
                                     grk_plugin_decode_callback callback);
int32_t grk_plugin_batch_decode(void);
void grk_plugin_stop_batch_decode(void);

#ifdef __cplusplus
}
#endif
#endif
