/* grk_plugin_abi.h -- Grok's accelerator plugin ABI (minpf), as exported by
 * libgrok_plugin.so (grokimagecompression_amd/lib/), SURVEY.md §8(b2).
 *
 * Grok's host (`grk_plugin_load`, grok.cpp:834-861) dlopens
 * <plugin_path>/libgrok_plugin.so, calls minpf_post_load_plugin (which must
 * register one object, version {1, 0}; minpf_plugin.h:37-57, stub
 * src/lib/jp2_plugin/Plugin.cpp:32-50) and then dlsyms the plugin_* functions
 * by name (grok.cpp:810-823; typedefs plugin_interface.h:46-130).
 *
 * This plugin runs the tile hot path on the MI355X (grk_mi355x.h):
 *   plugin_init    -> grkgpu_create(deviceId): true iff a gfx950 context is up
 *   plugin_encode  -> loads the input image (PGM / PPM, the formats
 *                     grk_compress's PNMFormat reads), runs DC shift + MCT +
 *                     DWT + T1 (+ per-pass distortion) on the GPU, fills a
 *                     grk_plugin_tile and hands it to the host's callback,
 *                     whose grk_encode_with_plugin skips those stages and runs
 *                     rate control + Tier-2 on the plugin's code-blocks
 *                     (TileProcessor.cpp:994-1012, plugin_bridge.cpp:144-258).
 *   plugin_decode  -> the whole decode (host Tier-2 of this library + T1 +
 *                     inverse DWT + inverse MCT / DC shift on the GPU), with
 *                     grk_decompress's -r / -l / -d; the host reads the header
 *                     into its own image (callback, GRK_DECODE_HEADER), the
 *                     plugin fills the samples, the host writes the output
 *                     (GRK_DECODE_POST_T1) and releases (GRK_PLUGIN_DECODE_CLEAN)
 *                     -- grk_decompress.cpp:1336-1367.  The host's own T2 hand-
 *                     off (plugin_bridge.cpp:24-87) takes single-segment blocks
 *                     only, so the plugin keeps Tier-2.
 *   batch / debug  -> "not handled" (-1 / no-ops), as the reference's stub.
 *
 * The structures that cross this boundary are re-declared here with the
 * reference's layout (grok.h, Grok v5.1.0), field for field.
 */
#ifndef GRK_PLUGIN_ABI_H
#define GRK_PLUGIN_ABI_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
#include <string>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* minpf_plugin.h:22-57 */
struct minpf_platform_services;
typedef struct minpf_object_params {
    const char *id;
    const struct minpf_platform_services *platformServices;
} minpf_object_params;
typedef struct minpf_plugin_api_version {
    int32_t major;
    int32_t minor;
} minpf_plugin_api_version;
typedef void *(*minpf_create_func)(minpf_object_params *);
typedef int32_t (*minpf_destroy_func)(void *);
typedef struct minpf_register_params {
    minpf_plugin_api_version version;
    minpf_create_func createFunc;
    minpf_destroy_func destroyFunc;
} minpf_register_params;
typedef int32_t (*minpf_register_func)(const char *nodeType, const minpf_register_params *params);
typedef int32_t (*minpf_invoke_service_func)(const char *serviceName, void *serviceParams);
typedef struct minpf_platform_services {
    minpf_plugin_api_version version;
    minpf_register_func registerObject;
    minpf_invoke_service_func invokeService;
} minpf_platform_services;
typedef int32_t (*minpf_exit_func)(void);

/* ---- grok.h types that cross the plugin boundary ---- */
#define GRKP_PATH_LEN 4096          /* GRK_PATH_LEN, grok.h:114 */
#define GRKP_MAXRLVLS 33            /* GRK_J2K_MAXRLVLS, grok.h:117 */
#define GRKP_NUM_COMMENTS 256       /* GRK_NUM_COMMENTS_SUPPORTED, grok.h:370 */

typedef struct grkp_poc {           /* grk_poc, grok.h:393-410 */
    uint32_t resno0, compno0;
    uint32_t layno1, resno1, compno1;
    uint32_t layno0, precno0, precno1;
    int32_t prg1, prg;
    char progorder[5];
    uint32_t tile;
    uint32_t tx0, tx1, ty0, ty1;
    uint32_t layS, resS, compS, prcS;
    uint32_t layE, resE, compE, prcE;
    uint32_t txS, txE, tyS, tyE, dx, dy;
    uint32_t lay_t, res_t, comp_t, prc_t, tx0_t, ty0_t;
} grkp_poc;

typedef struct grkp_raw_cparameters { /* grk_raw_cparameters, grok.h:427-442 */
    uint32_t width, height;
    uint16_t numcomps;
    uint32_t prec;
    bool sgnd;
    void *comps;
} grkp_raw_cparameters;

typedef struct grkp_cparameters {   /* grk_cparameters, grok.h:447-570 */
    bool tile_size_on;
    uint32_t cp_tx0, cp_ty0, cp_tdx, cp_tdy;
    uint32_t cp_disto_alloc, cp_fixed_quality;
    char *cp_comment[GRKP_NUM_COMMENTS];
    uint16_t cp_comment_len[GRKP_NUM_COMMENTS];
    bool cp_is_binary_comment[GRKP_NUM_COMMENTS];
    size_t cp_num_comments;
    uint8_t csty;
    int32_t prog_order;
    grkp_poc POC[32];
    uint32_t numpocs;
    uint32_t tcp_numlayers;
    double tcp_rates[100];
    double tcp_distoratio[100];
    uint32_t numresolution;
    uint32_t cblockw_init, cblockh_init;
    uint8_t cblk_sty;
    bool isHT;
    bool irreversible;
    int32_t roi_compno;
    uint32_t roi_shift;
    uint32_t res_spec;
    uint32_t prcw_init[GRKP_MAXRLVLS];
    uint32_t prch_init[GRKP_MAXRLVLS];
    char infile[GRKP_PATH_LEN];
    char outfile[GRKP_PATH_LEN];
    uint32_t image_offset_x0, image_offset_y0;
    uint32_t subsampling_dx, subsampling_dy;
    int32_t decod_format, cod_format;
    grkp_raw_cparameters raw_cp;
    uint32_t max_comp_size;
    uint8_t tp_on, tp_flag, tcp_mct;
    void *mct_data;
    uint64_t max_cs_size;
    uint16_t rsiz;
    int framerate;
    bool write_capture_resolution_from_file;
    double capture_resolution_from_file[2];
    bool write_capture_resolution;
    double capture_resolution[2];
    bool write_display_resolution;
    double display_resolution[2];
    uint32_t rateControlAlgorithm;
    uint32_t numThreads;
    int32_t deviceId;
    uint32_t duration;
    uint32_t kernelBuildOptions;
    uint32_t repeats;
    bool verbose;
} grkp_cparameters;

typedef struct grkp_image_comp {    /* grk_image_comp, grok.h:851-891 */
    uint32_t dx, dy, w, h, x0, y0, prec, sgnd, resno_decoded;
    int32_t *data;
    bool owns_data;
    uint16_t alpha;
} grkp_image_comp;

typedef struct grkp_image {         /* grk_image, grok.h:896-922 */
    uint32_t x0, y0, x1, y1, numcomps;
    int32_t color_space;
    grkp_image_comp *comps;
    uint8_t *icc_profile_buf;
    uint32_t icc_profile_len;
    double capture_resolution[2];
    double display_resolution[2];
    uint8_t *iptc_buf;
    size_t iptc_len;
    uint8_t *xmp_buf;
    size_t xmp_len;
} grkp_image;

typedef struct grkp_image_cmptparm { /* grk_image_cmptparm, grok.h:927-942 */
    uint32_t dx, dy, w, h, x0, y0, prec, sgnd;
} grkp_image_cmptparm;

/* grok.h:1223-1278 */
typedef struct grk_plugin_pass {
    double distortionDecrease; /* distortion decrease up to and including this pass */
    size_t rate;               /* rate up to and including this pass */
    size_t length;             /* stream length for this pass */
} grk_plugin_pass;

typedef struct grk_plugin_code_block {
    uint32_t x0, y0, x1, y1;
    unsigned int *contextStream;
    size_t numPix;
    uint8_t *compressedData;
    size_t compressedDataLength;
    size_t numBitPlanes;
    size_t numPasses;
    grk_plugin_pass passes[67];
    unsigned int sortedIndex;
} grk_plugin_code_block;

typedef struct grk_plugin_precinct {
    size_t numBlocks;
    grk_plugin_code_block **blocks;
} grk_plugin_precinct;

typedef struct grk_plugin_band {
    size_t orient;
    size_t numPrecincts;
    grk_plugin_precinct **precincts;
    float stepsize;
} grk_plugin_band;

typedef struct grk_plugin_resolution {
    size_t level;
    size_t numBands;
    grk_plugin_band **bands;
} grk_plugin_resolution;

typedef struct grk_plugin_tile_component {
    size_t numResolutions;
    grk_plugin_resolution **resolutions;
} grk_plugin_tile_component;

#define GRK_DECODE_HEADER (1 << 0)
#define GRK_DECODE_T2 (1 << 1)
#define GRK_DECODE_T1 (1 << 2)
#define GRK_DECODE_POST_T1 (1 << 3)
#define GRK_PLUGIN_DECODE_CLEAN (1 << 4)

typedef struct grk_plugin_tile {
    uint32_t decode_flags;
    size_t numComponents;
    grk_plugin_tile_component **tileComponents;
} grk_plugin_tile;

/* grok.h:1816-1819 */
typedef struct grk_plugin_init_info {
    int32_t deviceId;
    bool verbose;
} grk_plugin_init_info;

#define GRK_PLUGIN_STATE_NO_DEBUG 0x0 /* grok.h:1791 */
#define GRK_PLUGIN_STATE_DEBUG 0x1 /* grok.h:1806: the host recomputes T1 and compares */
#define GRK_PLUGIN_STATE_PRE_TR1 0x2
#define GRK_PLUGIN_STATE_DWT_QUANTIZATION 0x4
#define GRK_PLUGIN_STATE_MCT_ONLY 0x8

/* plugin_interface.h:56-67 (what the host's internal callback receives) */
typedef struct plugin_encode_user_callback_info {
    const char *input_file_name;
    bool outputFileNameIsRelative;
    const char *output_file_name;
    grkp_cparameters *encoder_parameters;
    grkp_image *image;
    grk_plugin_tile *tile;
    int32_t error_code;
} plugin_encode_user_callback_info;
typedef void (*PLUGIN_ENCODE_USER_CALLBACK)(plugin_encode_user_callback_info *info);

/* ---- decode side ---- */
enum { GRKP_UNK_FMT = 0, GRKP_J2K_FMT = 1, GRKP_JP2_FMT = 2 }; /* GRK_SUPPORTED_FILE_FMT, grok.h:98-111 */

typedef struct grkp_jp2_color {     /* grk_jp2_color, grok.h:612-618 */
    uint8_t *icc_profile_buf;
    uint32_t icc_profile_len;
    void *jp2_cdef;
    void *jp2_pclr;
    uint8_t jp2_has_colour_specification_box;
} grkp_jp2_color;

typedef struct grkp_header_info {   /* grk_header_info, grok.h:620-689 */
    uint32_t cblockw_init, cblockh_init;
    bool irreversible;
    uint32_t mct;
    uint16_t rsiz;
    uint32_t numresolutions;
    uint8_t csty, cblk_sty;
    uint32_t prcw_init[GRKP_MAXRLVLS];
    uint32_t prch_init[GRKP_MAXRLVLS];
    uint32_t cp_tx0, cp_ty0, cp_tdx, cp_tdy, cp_tw, cp_th;
    uint32_t tcp_numlayers;
    uint32_t enumcs;
    grkp_jp2_color color;
    uint8_t *xml_data;
    size_t xml_data_len;
    size_t num_comments;
    char *comment[GRKP_NUM_COMMENTS];
    uint16_t comment_len[GRKP_NUM_COMMENTS];
    bool isBinaryComment[GRKP_NUM_COMMENTS];
    bool has_capture_resolution;
    double capture_resolution[2];
    bool has_display_resolution;
    double display_resolution[2];
} grkp_header_info;

typedef struct grkp_dparameters {   /* grk_dparameters, grok.h:694-735 */
    uint32_t cp_reduce;             /* grk_decompress -r */
    uint32_t cp_layer;              /* grk_decompress -l (0 = all) */
    char infile[GRKP_PATH_LEN];
    char outfile[GRKP_PATH_LEN];
    int32_t decod_format, cod_format;
    uint32_t DA_x0, DA_x1, DA_y0, DA_y1;
    bool m_verbose;
    uint16_t tile_index;
    uint32_t nb_tile_to_decode;
    uint32_t flags;
} grkp_dparameters;

typedef struct grkp_precision {     /* grk_precision, grok.h:741-744 */
    uint32_t prec;
    int32_t mode;
} grkp_precision;

typedef struct grkp_decompress_parameters { /* grk_decompress_parameters, grok.h:748-795 */
    grkp_dparameters core;
    char infile[GRKP_PATH_LEN];
    char outfile[GRKP_PATH_LEN];
    int32_t decod_format;
    uint32_t cod_format;
    char indexfilename[GRKP_PATH_LEN];
    uint32_t DA_x0, DA_x1, DA_y0, DA_y1; /* grk_decompress -d x0,y0,x1,y1 */
    bool m_verbose;
    uint16_t tile_index;
    uint32_t nb_tile_to_decode;
    grkp_precision *precision;
    uint32_t nb_precision;
    bool force_rgb, upsample, split_pnm, serialize_xml;
    uint32_t compression;
    int32_t compressionLevel;
    int32_t deviceId;
    uint32_t duration, kernelBuildOptions, repeats;
    bool verbose;
    uint32_t numThreads;
} grkp_decompress_parameters;

typedef int (*GRKP_INIT_DECODERS)(grkp_header_info *header_info, grkp_image *image); /* GROK_INIT_DECODERS, grok.h:1854 */

#ifdef __cplusplus
/* plugin_interface.h:86-118: what the plugin hands the host's internal decode
 * callback (a C++ object: std::string members, built by the plugin). */
struct PluginDecodeCallbackInfo {
    PluginDecodeCallbackInfo(std::string input, std::string output, grkp_decompress_parameters *params,
                             int32_t format, uint32_t flags)
        : deviceId(0), init_decoders_func(nullptr), inputFile(input), outputFile(output), decod_format(format),
          cod_format(GRKP_UNK_FMT), l_stream(nullptr), l_codec(nullptr), decoder_parameters(params), header_info(),
          image(nullptr), plugin_owns_image(false), tile(nullptr), error_code(0), decode_flags(flags) {}
    size_t deviceId;
    GRKP_INIT_DECODERS init_decoders_func;
    std::string inputFile;
    std::string outputFile;
    int32_t decod_format;
    int32_t cod_format;
    void *l_stream;
    void *l_codec;
    grkp_decompress_parameters *decoder_parameters;
    grkp_header_info header_info;
    grkp_image *image;
    bool plugin_owns_image;
    grk_plugin_tile *tile;
    int32_t error_code;
    uint32_t decode_flags;
};
typedef int32_t (*PLUGIN_DECODE_USER_CALLBACK)(PluginDecodeCallbackInfo *info);
#endif

/* Object id registered with the host (the reference stub uses "SamplePlugin",
 * Plugin.cpp:17). */
#define GRKGPU_PLUGIN_ID "GrokMI355X"

minpf_exit_func minpf_post_load_plugin(const char *pluginPath, const minpf_platform_services *services);
bool plugin_init(grk_plugin_init_info info);
uint32_t plugin_get_debug_state(void);
int32_t plugin_encode(grkp_cparameters *encode_parameters, PLUGIN_ENCODE_USER_CALLBACK user_callback);
int32_t plugin_batch_encode(const char *input_dir, const char *output_dir, grkp_cparameters *encode_parameters,
                            PLUGIN_ENCODE_USER_CALLBACK user_callback);
bool plugin_is_batch_complete(void);
void plugin_stop_batch_encode(void);
#ifdef __cplusplus
int32_t plugin_decode(grkp_decompress_parameters *decode_parameters, PLUGIN_DECODE_USER_CALLBACK user_callback);
#else
int32_t plugin_decode(grkp_decompress_parameters *decode_parameters, void *user_callback);
#endif
int32_t plugin_init_batch_decode(const char *input_dir, const char *output_dir,
                                 grkp_decompress_parameters *decode_parameters, void *user_callback);
int32_t plugin_batch_decode(void);
void plugin_stop_batch_decode(void);
/* debug hooks (plugin_interface.h:44-45; the stub's name for the first is
 * plugin_debug_next_cxd, Plugin.cpp:121 -- both names are exported) */
void plugin_debug_mqc_next_cxd(void *mqc, uint32_t d);
void plugin_debug_next_cxd(void *mqc, uint32_t d);
void plugin_debug_mqc_next_plane(void *mqc);

#ifdef __cplusplus
}
#endif
#endif
