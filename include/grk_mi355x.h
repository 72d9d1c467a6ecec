/*
 * grk_mi355x.h -- C ABI of the MI355X-native JPEG 2000 hot path
 * (libgrk_mi355x.so).  Plain C types only: no HIP/torch types cross this
 * boundary (streams are passed as void*).
 *
 * What each entry point replaces in the reference (Grok v5.1.0; paths under
 * /root/reference/src/lib/jp2/):
 *
 *   grkgpu_compress        grk_compress's in-library path  grk_setup_encoder +
 *                          grk_start_compress + grk_encode + grk_end_compress
 *                          (grok.h:1660-1748, grok.cpp:545-600 ->
 *                          codestream/j2k.cpp:1609 j2k_setup_encoder,
 *                          :2059 j2k_encode) for the default coding options
 *                          (1 layer, LRCP, 2^15 precincts, cblksty 0).
 *   grkgpu_decompress      grk_read_header + grk_decode (grok.h:1571-1600,
 *                          grok.cpp:381 -> j2k.cpp:1136 j2k_decode_tiles).
 *   grkgpu_read_header     grk_read_header (grok.h:1571, j2k.cpp:406).
 *   (stage entry points below = the tile hot path inside
 *                          TileProcessor::encode_tile (TileProcessor.cpp:
 *                          994-1012: dc_level_shift_encode :1449, mct_encode
 *                          :1473, dwt_encode :1520, t1_encode :1535) and
 *                          decode_tile (:1127-1176).)
 *   grkgpu_dwt_fwd/_inv    Wavelet::encode / Wavelet::decode
 *                          (transform/Wavelet.cpp:35-56, WaveletForward.h:40,
 *                          dwt.cpp:1208 decode_53, :2154 decode_97).
 *   grkgpu_dcshift_mct_fwd mct::encode_rev / encode_irrev + DC shift
 *                          (mct/mct.cpp:85, :195; TileProcessor.cpp:1449).
 *   grkgpu_mct_inv_dcshift mct::decode_rev / decode_irrev + DC shift + clamp
 *                          (mct/mct.cpp:143, :352; TileProcessor.cpp:1377).
 *   grkgpu_t1_encode_blocks  Tier1::encodeCodeblocks -> T1Encoder::encode ->
 *                          T1Part1::preEncode/encode (t1/Tier1.cpp:24,
 *                          T1Encoder.cpp:40-85, t1_part1/T1Part1.cpp:58-127,
 *                          t1.cpp:1182 t1_encode_cblk).
 *   grkgpu_t1_decode_blocks  Tier1::decodeCodeblocks -> T1Part1::decode +
 *                          postDecode (t1/Tier1.cpp:177, T1Decoder.cpp:43,
 *                          T1Part1.cpp:129-330, t1.cpp:1038 t1_decode_cblk).
 *
 * Error behaviour mirrors the reference: functions return 0 on success and a
 * negative code on failure (the reference returns bool false / nullptr and
 * logs through its error handler); grkgpu_last_error() returns the message.
 * Every function fails loudly (GRKGPU_ENODEV) when no gfx950 device is
 * usable -- there is no CPU fallback.
 */
#ifndef GRK_MI355X_H
#define GRK_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GRKGPU_MAX_COMPS 16

enum {
    GRKGPU_OK = 0,
    GRKGPU_EINVAL = -1,
    GRKGPU_ENODEV = -2,
    GRKGPU_EHIP = -3,
    GRKGPU_EUNSUPPORTED = -4,
    GRKGPU_ECORRUPT = -5
};

/* grk_image subset (grok.h:851-918): planar components.  [x0, x1) x [y0, y1)
 * is the image on the reference grid; component k is subsampled by dx[k],
 * dy[k] (SIZ XRsiz / YRsiz; 0 reads as 1), so its plane covers
 * [ceil(x0 / dx), ceil(x1 / dx)) x [ceil(y0 / dy), ceil(y1 / dy)) -- rows of
 * that width, planes[k] holding only component k (grk_image_comp w, h,
 * TileComponent.cpp:150-163).  A reduced / window decode reports the reduced
 * / window rectangle here, and component planes follow the same rule, except
 * that a reduced decode of the whole image sizes its planes as the reference
 * does (grk_image_comp_header_update, image.cpp:124-155): ceil(size / 2^r),
 * with x1 = x0 + that -- one more row / column than the decoded samples when
 * the origin is not a multiple of 2^r, left zero. */
typedef struct {
    uint32_t x0, y0, x1, y1;
    uint32_t numcomps;
    uint32_t prec[GRKGPU_MAX_COMPS];
    int32_t sgnd[GRKGPU_MAX_COMPS];
    uint32_t dx[GRKGPU_MAX_COMPS], dy[GRKGPU_MAX_COMPS];
} grkgpu_image_desc;

/* One progression-order change (grk_poc, grok.h:393-410; grk_compress -P
 * "T<tile>=resno0,compno0,layno1,resno1,compno1,PROG"). */
typedef struct {
    uint32_t tile;                       /* 1-based tile index the entry applies to */
    uint32_t resno0, compno0, layno1, resno1, compno1;
    int32_t prog;                        /* GRKGPU_LRCP .. GRKGPU_CPRL */
} grkgpu_poc;

enum { GRKGPU_LRCP = 0, GRKGPU_RLCP = 1, GRKGPU_RPCL = 2, GRKGPU_PCRL = 3, GRKGPU_CPRL = 4 };
#define GRKGPU_CSTY_PRT 0x01 /* user precinct sizes (grk_compress -c) */
#define GRKGPU_CSTY_SOP 0x02 /* SOP marker before each packet (-SOP) */
#define GRKGPU_CSTY_EPH 0x04 /* EPH marker after each packet header (-EPH) */
#define GRKGPU_PROFILE_CINEMA_2K 0x0003 /* grok.h:160 */
#define GRKGPU_PROFILE_CINEMA_4K 0x0004 /* grok.h:161 */

/* grk_cparameters subset (grok.h:447-570); field meaning as there */
typedef struct {
    uint32_t numresolution;                /* default 6 */
    uint32_t cblockw_init, cblockh_init;   /* default 64, 64 (powers of 2, <= 64) */
    int32_t irreversible;                  /* 0: 5/3, 1: 9/7 (-I) */
    int32_t tcp_mct;                       /* -1: auto (RGB->YCC iff >= 3 comps), 0, 1; 2: the custom
                                              matrix below (grkgpu_set_mct) */
    int32_t tile_size_on;
    uint32_t cp_tdx, cp_tdy, cp_tx0, cp_ty0;
    /* quality layers and rate control (grk_compress -r / -q / -A) */
    uint32_t tcp_numlayers;                /* 0: one lossless layer */
    double tcp_rates[100];                 /* per layer compression ratio, decreasing; 0 = lossless */
    double tcp_distoratio[100];            /* per layer PSNR (fixed quality) */
    int32_t cp_disto_alloc, cp_fixed_quality;
    int32_t rate_control_algorithm;        /* 0: bisect all passes, 1: feasible truncation points */
    /* coding style, precincts, progression (-c, -SOP, -EPH, -p, -P, -u) */
    uint32_t csty;                         /* GRKGPU_CSTY_* */
    uint32_t res_spec;                     /* precinct sizes given, highest resolution first */
    uint32_t prcw_init[33], prch_init[33];
    int32_t prog_order;                    /* GRKGPU_LRCP .. */
    uint32_t numpocs;
    grkgpu_poc POC[32];
    int32_t tp_on;                         /* tile-parts: one per change of tp_flag's dimension */
    int32_t tp_flag;                       /* 'R', 'L', 'C' */
    /* profiles (-cinema2K / -cinema4K fps): rsiz + the size caps */
    uint32_t rsiz;
    uint32_t framerate;
    uint64_t max_cs_size, max_comp_size;
    /* code-block style (-M): 0x01 BYPASS (lazy), 0x02 RESET, 0x04 TERMALL
     * (restart), 0x08 VSC, 0x10 PTERM (ERTERM), 0x20 SEGSYM */
    uint32_t cblk_sty;
    /* ROI up-shift (-ROI c=compno,U=shift; the RGN marker): roi_shift 0 = none */
    int32_t roi_compno;
    uint32_t roi_shift;
    uint32_t pad_;
    /* custom (Part 2 array-based) MCT, grk_set_MCT's mct_data: mct_ncomp x
     * mct_ncomp encoding matrix (row-major) and per-component DC shifts;
     * mct_ncomp 0 = none */
    uint32_t mct_ncomp;
    float mct_matrix[GRKGPU_MAX_COMPS * GRKGPU_MAX_COMPS];
    int32_t mct_dc_shift[GRKGPU_MAX_COMPS];
} grkgpu_cparams;

typedef struct grkgpu_ctx grkgpu_ctx;

/* Per-stage timings of the last call (device time from HIP events, ms). */
typedef struct {
    float h2d_ms, dcshift_mct_ms, dwt_ms, t1_ms, gather_ms, d2h_ms, host_t2_ms, total_ms;
    uint64_t num_cblks, cs_bytes;
    uint64_t mq_symbols;  /* MQ symbols coded (encode) */
    float rate_ms;        /* host rate allocation (PCRD) time (summed over tiles) */
    float packet_ms;      /* host packet / tile-part writing time (summed over tiles) */
    /* the PCRD bisection, summed over tiles: probes (thresholds tried), those
     * decided by their code-block bytes alone (no packet simulation), block
     * evaluations, precinct simulations, and the time forming layers /
     * simulating packets (part of rate_ms) */
    uint32_t rate_probes, rate_probes_skipped;
    uint64_t rate_block_evals, rate_precinct_sims;
    float rate_form_ms, rate_sim_ms;
    float passrec_ms;     /* host: per-pass rate / distortion records from the T1 results (part of host_t2_ms) */
    uint32_t pad_;
} grkgpu_stats;

/* One kernel launch of the last call's forward DWT, timed with HIP events on
 * the context's stream (grkgpu_set_launch_timing): kernel name, first level
 * and level count it computes, device time, and its algorithmic bytes
 * (8 B -- an int32 read and written -- per sample of every level it
 * computes: SURVEY.md 8(d)'s B_DWT split per launch). */
typedef struct {
    char kernel[48];
    uint32_t level0, levels;
    float ms;
    uint32_t pad;
    uint64_t bytes;
} grkgpu_launch_time;

const char *grkgpu_version(void);
const char *grkgpu_last_error(void);
int grkgpu_device_count(void);

int grkgpu_create(int device, grkgpu_ctx **out);
void grkgpu_destroy(grkgpu_ctx *ctx);
/* Order all work of ctx after/with this HIP stream (hipStream_t as void*). */
int grkgpu_set_stream(grkgpu_ctx *ctx, void *stream);
int grkgpu_get_stats(grkgpu_ctx *ctx, grkgpu_stats *out);
/* Time every DWT launch of later compress (forward) and decompress (inverse)
 * calls (off by default: two events per launch), and read the launches of the
 * last call: *n = their count, the first min(max, *n) are copied to out. */
int grkgpu_set_launch_timing(grkgpu_ctx *ctx, int on);

/* DWT plan options, process-wide (later calls; not while other threads are
 * inside a call).  The defaults are the plans measured fastest on the MI355X
 * (DESIGN.md 3); the others stay selectable so the parity suite can check
 * every kernel the library carries.
 *   fuse_level0      -1 (default): the DC shift + RCT of a 3-component 5/3
 *                    tile runs inside DWT level 0 (k_dwt_fwd_mct3); 0: never
 *                    (separate k_dcshift_mct_fwd pass); 1: always (also 9/7
 *                    and single components: DC shift in level 0's loads).
 *   f01_rows         9/7 levels 0 + 1 in one launch (k_dwt_fwd01) with 2 / 4
 *                    (default) / 6 level-0 row windows per workgroup; 0: one
 *                    launch per level.
 *   f01_min_samples  fuse a level pair only from this many level-l samples
 *                    (default 2^23; 0: every qualifying pair).
 *   f01_small_min_samples  fuse smaller pairs too, from this many samples,
 *                    with 2 row windows per workgroup (default all ones:
 *                    never -- the 8K frame's levels 2 + 3 fused this way
 *                    took 26 us of kernel time against 14 + 7 apart).
 *   inv01            2 (default) / 4: the two largest inverse levels in one
 *                    launch (k_dwt_inv01, with 2 / 4 row windows for the
 *                    smaller level per workgroup) when the larger has at
 *                    least inv01_min_samples samples (default 2^23; 0: any
 *                    size); 0: one launch per level.
 *   pair_group       workgroup order of the fused level pairs (k_dwt_fwd01,
 *                    k_dwt_inv01): 0 (default) row-major; G > 0: groups of G
 *                    workgroup columns, each walked top to bottom.
 *   f64_lift         forward 9/7 lifting arithmetic (fused pair and per-level
 *                    kernel, not the fused DC-shift loads): 0 the
 *                    64-bit integer multiply (v_mad_i64_i32), 1 f64 FMA +
 *                    floor (bit-identical results).
 *   t1_dec_sort      T1 decode: 1 (default) = code-blocks handed to the
 *                    lanes in decreasing order of expected work (passes,
 *                    bytes), so a wavefront's lanes finish close together;
 *                    0 = stream order; -1 = only for a call that is the only
 *                    one in progress in the process.  Same output.
 *   t1_dec_bpw       T1 decode: code-blocks per wavefront (1, 2, 4 .. 64);
 *                    0 (default) = a lone call spreads its blocks to give
 *                    every SIMD 1.5 wavefronts, concurrent calls pack 64 (from
 *                    4096 blocks).
 *   mid_th           window rows (8, 16, 24) of the per-level DWT kernels for
 *                    a level of 2^21 .. 2^23 samples; 0 (default) = 8.
 *   t1_enc_bpw       T1 encode (MQ coder): code-blocks per wavefront, as
 *                    t1_dec_bpw.
 *   t1_enc_sort      T1 encode: 1 = the MQ coder's lanes take the code-blocks
 *                    in decreasing order of their symbol count (a counting
 *                    sort on the device after the modelling kernel); 0
 *                    (default, measured as fast) = block order.  Same
 *                    codestream.
 *   pair_kernel      fused forward level pairs: k_dwt_fwd_pair (workgroups
 *                    stream column strips top to bottom, the vertical lifting
 *                    carried in registers, the LL rows through an LDS ring)
 *                    for pairs of at least pair_min_samples level-l samples
 *                    (default 2^20) -- 1 (default): 5/3 pairs, 9/7 pairs by
 *                    k_dwt_fwd01's windows (f01_rows); 2: both wavelets
 *                    streamed; 0: no 5/3 pairs, 9/7 by k_dwt_fwd01.
 *                    f01_rows = 0 turns every fused pair off.
 *   pair_rows        k_dwt_fwd_pair: level-(l+1) rows per segment (even); 0
 *                    (default) = sized for one resident wave of workgroups.
 *   pair_waves       k_dwt_fwd_pair: level-l wavefronts per workgroup, 3 or 4;
 *                    0 (default) = whichever wastes fewer columns. */
typedef struct {
    int32_t fuse_level0;
    int32_t f01_rows;
    uint64_t f01_min_samples;
    uint64_t f01_small_min_samples;
    int32_t inv01;
    int32_t pair_group;
    uint64_t inv01_min_samples;
    int32_t f64_lift;
    int32_t t1_dec_sort;
    int32_t t1_dec_bpw;
    int32_t mid_th;
    int32_t t1_enc_bpw;
    int32_t t1_enc_sort;
    int32_t pair_kernel;
    int32_t pair_rows;
    int32_t pair_waves;
    uint64_t pair_min_samples;
} grkgpu_dwt_options;
void grkgpu_get_dwt_options(grkgpu_dwt_options *out);  /* current values */
int grkgpu_set_dwt_options(const grkgpu_dwt_options *opts);  /* NULL: the defaults */
int grkgpu_get_launch_times(grkgpu_ctx *ctx, grkgpu_launch_time *out, uint32_t max, uint32_t *n);
void grkgpu_default_cparams(grkgpu_cparams *p);
/* grk_set_MCT (grok.cpp:606-630): a custom array-based MCT -- rsiz gains the
 * Part-2 MCT extension (0x8000 | 0x0100), 9/7, tcp_mct = 2, the n x n
 * encoding matrix (row-major, applied in 13-bit fixed point,
 * mct.cpp:429-475) and the per-component DC shifts.  The codestream then
 * carries its inverse (float, j2k.cpp:1932) in CBD / MCT / MCC / MCO marker
 * segments (j2k.cpp:5615-6333). */
int grkgpu_set_mct(grkgpu_cparams *p, const float *matrix, const int32_t *dc_shift, uint32_t n);

/* Whole-codestream encode.  planes[c] = (y1-y0)*(x1-x0) int32 samples, on
 * the device when planes_on_device != 0, else host memory.  The .j2k
 * codestream is returned in *out (free with grkgpu_free). */
int grkgpu_compress(grkgpu_ctx *ctx, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                    const int32_t *const *planes, int planes_on_device, uint8_t **out, size_t *outlen);

/* Same, zero-copy: *out points into the context's pinned output buffer and
 * stays valid until the next call on ctx (like the reference's memory stream). */
int grkgpu_compress_view(grkgpu_ctx *ctx, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                         const int32_t *const *planes, int planes_on_device, const uint8_t **out, size_t *outlen);

/* Output-buffer hand-off for views that must outlive later calls: take the
 * context's pinned output buffer (holding the last compress's codestream) out
 * of the context -- its next compress allocates a buffer of its own -- and
 * give a taken buffer back when done with it (the context keeps the larger of
 * it and its current buffer and frees the other; with ctx = NULL, or after
 * grkgpu_destroy, use grkgpu_free_output).  *buf = NULL if the context holds
 * no buffer. */
int grkgpu_take_output(grkgpu_ctx *ctx, void **buf, size_t *cap);
int grkgpu_give_output(grkgpu_ctx *ctx, void *buf, size_t cap);
void grkgpu_free_output(void *buf);

/* Tile shards (multi-GPU): tiles are independent through the
 * whole path, and a codestream is [main header][tile-parts in tile order]
 * [EOC] (j2k.cpp:2088-2111, 2376-2435), so each GPU encodes a contiguous
 * tile range and the host concatenates.  grkgpu_compress_tiles encodes tiles
 * [tile_begin, tile_end) and emits the parts selected by `parts`;
 * grkgpu_compress == grkgpu_compress_tiles(0, n, GRKGPU_PART_ALL). */
#define GRKGPU_PART_HEADER 1u
#define GRKGPU_PART_TILES 0u
#define GRKGPU_PART_EOC 2u
#define GRKGPU_PART_ALL 3u
int grkgpu_num_tiles(const grkgpu_image_desc *img, const grkgpu_cparams *p, uint32_t *ntiles);
int grkgpu_compress_tiles(grkgpu_ctx *ctx, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                          const int32_t *const *planes, int planes_on_device, uint32_t tile_begin,
                          uint32_t tile_end, uint32_t parts, uint8_t **out, size_t *outlen);

/* Multi-device calls: one call shards the tiles over several devices
 *  -- what the reference's callers ask for with
 * deviceId = -1 (grk_cparameters.deviceId, grok.h:565; grk_compress -G "A
 * value of -1 will specify all devices", grk_compress.cpp:423-426; the
 * decompress parameters and the plugin init info carry the same field,
 * grok.h:789, 1817).  A device set lists the workers: one host thread and
 * one context (pooled per device across calls) each; a device may appear
 * more than once.
 *   grkgpu_device_set_for: device >= 0 -> {device}; device = -1 -> the
 *     environment's GRKGPU_DEVICES ("0,1,2,3", "0,0", or "all"), else every
 *     visible device.
 *   grkgpu_compress_multi: the whole codestream.  Worker k encodes the k-th
 *     contiguous tile range from just the image rows of its tiles (host
 *     planes; worker 0 also writes the main header, the last one the EOC);
 *     the pieces are concatenated in tile order and the TLM records filled in
 *     from the tile-parts (j2k_write_updated_tlm, j2k.cpp:2555-2577).  Bytes
 *     identical to grkgpu_compress.  One worker does it all when the image
 *     has one tile, the planes are on a device, hold a window of the image,
 *     or a component is subsampled.  *out: free with grkgpu_free.
 *   grkgpu_decompress_multi: whole-image decode into host planes, each worker
 *     decoding its tile range (grkgpu_decompress_tiles).
 *   grkgpu_multi_release: destroy the pooled contexts. */
#define GRKGPU_MAX_DEVICES 64
typedef struct {
    uint32_t n;
    int32_t dev[GRKGPU_MAX_DEVICES];
} grkgpu_device_set;
int grkgpu_device_set_for(int device, grkgpu_device_set *out);
void grkgpu_multi_release(void);
/* Host only: fill in the TLM records of a codestream concatenated from tile
 * shards (j2k_write_updated_tlm, j2k.cpp:2555-2577) from its tile-parts' SOT
 * headers, in place -- records across all of the main header's TLM markers,
 * in order.  GRKGPU_EINVAL when the records do not match the tile-parts one
 * to one (or a tile-part has Psot = 0); a stream without TLM is unchanged. */
int grkgpu_patch_tlm(uint8_t *cs, size_t len);

/* Same, with planes holding only image rows [row0, row0 + nrows) (relative to
 * img->y0): a rank of a tile-row shard loads just the rows of its tiles.
 * Every tile of [tile_begin, tile_end) must lie inside those rows. */
int grkgpu_compress_tile_rows(grkgpu_ctx *ctx, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                              const int32_t *const *planes, int planes_on_device, uint32_t row0, uint32_t nrows,
                              uint32_t tile_begin, uint32_t tile_end, uint32_t parts, uint8_t **out, size_t *outlen);

/* The general encode entry point: image samples in the width the image file
 * holds them (grk_image's planes are int32, grok.h:851-918; the PGM / PPM /
 * raw files grk_compress and the plugin read are 1 or 2 bytes per sample,
 * PNMFormat.cpp), widened to int32 on the GPU by the kernel that first reads
 * them -- so a 12-bit frame crosses PCIe as 2 B/sample.  planes[c] holds
 * rows [row0, row0 + nrows) x columns [col0, col0 + ncols) of component c
 * (nrows / ncols = 0: every row / column; a tile-row shard gives only its
 * tiles' rows, see grkgpu_compress_tile_rows; grk_write_tile one tile), on
 * the device when on_device != 0.  Every tile encoded must lie inside them.  Encodes tiles [tile_begin, tile_end) and
 * emits the parts `parts` selects (GRKGPU_PART_*; 0, 0xffffffff, ALL = the
 * whole codestream, as grkgpu_compress).  *out points into the context's
 * pinned output buffer, valid until the next call on ctx (as
 * grkgpu_compress_view).  A sample format must hold the component's
 * precision and signedness (U16: unsigned, prec <= 16), else GRKGPU_EINVAL. */
enum {
    GRKGPU_SAMPLE_I32 = 0, /* int32_t (grk_image) */
    GRKGPU_SAMPLE_U8 = 1,
    GRKGPU_SAMPLE_I8 = 2,
    GRKGPU_SAMPLE_U16 = 3,
    GRKGPU_SAMPLE_I16 = 4
};
typedef struct {
    const void *planes[GRKGPU_MAX_COMPS];
    uint32_t sample_fmt;  /* GRKGPU_SAMPLE_* */
    int32_t on_device;
    uint32_t row0, nrows; /* rows held (relative to y0); nrows = 0: every row */
    uint32_t col0, ncols; /* columns held (relative to x0), = the row stride; ncols = 0: every column
                             (grk_write_tile hands one tile's samples: its rows and columns only) */
} grkgpu_planes;
int grkgpu_compress_ex(grkgpu_ctx *ctx, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                       const grkgpu_planes *planes, uint32_t tile_begin, uint32_t tile_end, uint32_t parts,
                       const uint8_t **out, size_t *outlen);
/* (multi-device encode: see grkgpu_device_set above) */
int grkgpu_compress_multi(const grkgpu_device_set *devs, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                          const grkgpu_planes *planes, uint8_t **out, size_t *outlen);

/* Tier-1 only (the tile hot path of TileProcessor::encode_tile up to and
 * including t1_encode, TileProcessor.cpp:994-1012; SURVEY 8(b)
 * "grkgpu_encode_tile"): DC shift + MCT + DWT + T1 of every tile on the GPU,
 * results handed back per code-block in the reference's order (tile,
 * component, resolution, band, precinct, code-block) so a host Tier-2 -- the
 * reference's own, through its plugin interface -- can finish the
 * codestream.  Rates are the cumulative pass rates after the reference's
 * fix-ups (t1.cpp:1299-1325); distortion the cumulative distortion decrease
 * (t1.cpp:1249-1254), computed when with_distortion != 0.  Pointers stay
 * valid until the next call on ctx. */
typedef struct {
    uint32_t tileno, compno, resno, bandno, precno, cblkno;
    uint32_t x0, y0, x1, y1;             /* code-block rectangle, band coordinates */
    uint32_t numbps, numpasses, len;
    float stepsize;                      /* the band's encoder step size (Quantizer.cpp:65-104) */
    const uint8_t *data;                 /* len MQ bytes */
    const uint32_t *rate;                /* numpasses cumulative rates */
    const double *distortion;            /* numpasses cumulative distortion decrease */
} grkgpu_block_info;
int grkgpu_encode_blocks(grkgpu_ctx *ctx, const grkgpu_image_desc *img, const grkgpu_cparams *p,
                         const int32_t *const *planes, int planes_on_device, int with_distortion,
                         const grkgpu_block_info **blocks, uint32_t *nblocks);

/* After grkgpu_encode_blocks on ctx (and before any other call on it): the
 * forward DWT output of one tile-component -- the reference's tile buffer
 * after dwt_encode (Mallat layout, dwt_utils.cpp:84-127), rows of the
 * tile-component's width, before T1's quantisation -- copied into dst (host
 * memory, h rows of dst_stride elements).  This is what the reference's plugin
 * debug state hands its host as image data so that both T1s start from the
 * same coefficients (TileProcessor.cpp:985-1012, grok.h:1790-1808). */
int grkgpu_encode_blocks_coefficients(grkgpu_ctx *ctx, uint32_t tileno, uint32_t compno, int32_t *dst,
                                      uint32_t dst_stride);

/* Parse the main header only. */
int grkgpu_read_header(const uint8_t *cs, size_t len, grkgpu_image_desc *img);
/* The coding parameters of the main header (grk_header_info, grok.h:620-689),
 * plus its quantisation (QCD: Sqcd guard bits and style, the step sizes as
 * read) and ROI shifts (RGN) -- what grk_get_cstr_info reports. */
typedef struct {
    uint32_t cblockw_init, cblockh_init, irreversible, mct, rsiz, numresolutions, csty, cblk_sty;
    uint32_t prcw_init[33], prch_init[33];  /* precinct size per resolution (samples) */
    uint32_t tx0, ty0, tdx, tdy, tw, th;   /* tile grid */
    uint32_t numlayers, prog;
    uint32_t numcomps, numgbits, qntsty, nsteps;  /* QCD: guard bits, style, step sizes read */
    uint32_t step_expn[97], step_mant[97];
    uint32_t roishift[16];                 /* RGN per component */
} grkgpu_header_info;
int grkgpu_read_header_info(const uint8_t *cs, size_t len, grkgpu_header_info *info);
/* One component's coding style and quantisation as the main header sets them
 * (COD / QCD, or that component's COC / QCC; the reference's default tcp
 * tccps[compno], j2k_dump.cpp:357-390 reads the same): precinct flag, levels,
 * log2 code-block size, mode switches, wavelet (qmfbid 1 = 5/3), log2
 * precinct sizes, QCD / QCC style, guard bits and step sizes, ROI shift. */
typedef struct {
    uint32_t csty, numresolutions, cblkw, cblkh, cblk_sty, qmfbid;
    uint32_t prcw[33], prch[33];
    uint32_t qntsty, numgbits, nsteps;
    uint32_t step_expn[100], step_mant[100];
    uint32_t roishift;
} grkgpu_comp_info;
int grkgpu_read_comp_info(const uint8_t *cs, size_t len, uint32_t compno, grkgpu_comp_info *info);

/* Whole-codestream decode into caller-provided planes (device or host). */
int grkgpu_decompress(grkgpu_ctx *ctx, const uint8_t *cs, size_t len, grkgpu_image_desc *img,
                      int32_t *const *planes, int planes_on_device);
/* Reduced-resolution decode (grk_decompress -r; grk_decompress_parameters
 * cp_reduce, grok.h:698-702, applied in j2k.cpp:1464-1476 and
 * TileComponent.cpp:199-204): the image at resolution numres-1-reduce, the
 * samples from ceil(x0 / 2^reduce), planes of ceil(size / 2^reduce) a side
 * (see grkgpu_image_desc); img (if given) receives the reduced geometry.
 * reduce must be < the number of resolutions (GRKGPU_EINVAL). */
int grkgpu_decompress_reduced(grkgpu_ctx *ctx, const uint8_t *cs, size_t len, uint32_t reduce,
                              grkgpu_image_desc *img, int32_t *const *planes, int planes_on_device);
/* Window decode (grk_set_decode_area, grok.h:1587; grk_decompress -d):
 * decode only the samples of [x0, x1) x [y0, y1) (image coordinates, clipped
 * to the image) into planes of the window's size; img (if given) receives the
 * window geometry.  Same samples as a full decode, cropped.  Only the tiles
 * meeting the window and the code-blocks reaching it are decoded. */
int grkgpu_decompress_window(grkgpu_ctx *ctx, const uint8_t *cs, size_t len, uint32_t x0, uint32_t y0, uint32_t x1,
                             uint32_t y1, grkgpu_image_desc *img, int32_t *const *planes, int planes_on_device);
/* Decode with grk_decompress's options (grk_dparameters, grok.h:694-735):
 * cp_reduce (-r), cp_layer (-l, 0 = all layers) and the decode area (-d,
 * grk_set_decode_area; all four 0 = the whole image).  A window at a reduced
 * resolution spans ceil(x1 / 2^r) - ceil(x0 / 2^r) (update_image_dimensions,
 * image.cpp:207-246).  img (if given) receives the decoded geometry. */
typedef struct {
    uint32_t cp_reduce, cp_layer;
    uint32_t DA_x0, DA_y0, DA_x1, DA_y1;
} grkgpu_dparams;
int grkgpu_decompress_ex(grkgpu_ctx *ctx, const uint8_t *cs, size_t len, const grkgpu_dparams *p,
                         grkgpu_image_desc *img, int32_t *const *planes, int planes_on_device);
/* Decode only tiles [tile_begin, tile_end) (a tile shard; the reference's
 * tile-by-tile decode, grk_decode_tile_data / j2k.cpp decode_tiles); the
 * other tiles' samples in planes are left untouched.  Host planes are written
 * for the shard's tiles only. */
int grkgpu_decompress_tiles(grkgpu_ctx *ctx, const uint8_t *cs, size_t len, uint32_t tile_begin,
                            uint32_t tile_end, int32_t *const *planes, int planes_on_device);
/* (multi-device decode into host planes: see grkgpu_device_set above) */
int grkgpu_decompress_multi(const grkgpu_device_set *devs, const uint8_t *cs, size_t len, grkgpu_image_desc *img,
                            int32_t *const *planes);

/* The tile-part walk of a decode, host only (no device needed): the
 * reference decoder's walk over the tile-parts (j2k_decode_tiles,
 * j2k.cpp:1136-1224) -- GRKGPU_OK and decoded[t] = 1 for every
 * tile a decode produces (others stay zero in its output), or the error a
 * short or damaged stream makes the whole decode fail with.  *ntiles = the
 * tile count; decoded holds cap entries (may be NULL). */
int grkgpu_walk_tiles(const uint8_t *cs, size_t len, uint8_t *decoded, uint32_t cap, uint32_t *ntiles);

void grkgpu_free(void *p);

/* ---- stage entry points (device pointers, asynchronous on `stream`) ---- */

int grkgpu_dcshift_mct_fwd(int32_t *const *planes, uint32_t numcomps, uint32_t w, uint32_t h,
                           uint32_t stride, const int32_t *shift, int32_t mct, int32_t irreversible,
                           void *stream);
int grkgpu_mct_inv_dcshift(int32_t *const *planes, uint32_t numcomps, uint32_t w, uint32_t h,
                           uint32_t stride, const uint32_t *prec, const int32_t *sgnd, int32_t mct,
                           int32_t irreversible, void *stream);
/* In-place (Mallat layout) forward / inverse DWT of one tile-component with
 * origin (x0,y0), size (x1-x0) x (y1-y0), row stride x1-x0.  scratch must
 * hold grkgpu_dwt_scratch_bytes(...) device bytes.  For 9/7 inverse the buffer
 * holds float bit patterns. */
size_t grkgpu_dwt_scratch_bytes(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t numres);
int grkgpu_dwt_fwd(int32_t *buf, int32_t *scratch, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                   uint32_t numres, int32_t irreversible, void *stream);
int grkgpu_dwt_inv(int32_t *buf, int32_t *scratch, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                   uint32_t numres, int32_t irreversible, void *stream);

/* Code-block descriptors for the T1 entry points (all device memory). */
typedef struct {
    uint64_t coef_off;    /* element offset of the block's top-left in `coef` */
    uint64_t out_off;     /* byte offset in `out`, a multiple of 4 and >= 4: the
                             block's bytes start there, and the encoder writes
                             zeros to out[out_off - 4 .. out_off - 1] (the MQ
                             coder's pad byte before the block, Grok's
                             bp = start - 1, committed with its dword), so no
                             other block's bytes may lie there */
    uint32_t stride, w, h, orient; /* orient = band number 0:LL 1:HL 2:LH 3:HH */
    int32_t qmfbid, inv_step;      /* qmfbid 1 = 5/3, 0 = 9/7 (13-bit inv step) */
} grkgpu_enc_block;

typedef struct {
    uint32_t numbps, numpasses, len, pad;  /* pad != 0: numbps above the band's bound */
    uint32_t nsym, pad1, pad2, pad3;       /* nsym: MQ symbols coded */
    uint32_t rate[96];    /* cumulative pass rates after Grok's fix-ups */
    int32_t nmsedec[96];  /* per-pass normalised distortion decrease (t1.cpp
                             nmsedec; distortiondec = t1_getwmsedec of it,
                             t1.cpp:912-930); filled when with_distortion */
} grkgpu_enc_result;

typedef struct {
    uint64_t data_off;    /* byte offset of the block's single segment in `data` */
    uint64_t dst_off;     /* element offset of the block's top-left in `dst` */
    uint32_t len, numpasses, numbps, w, h, orient, dstride;
    int32_t irreversible;
    float stepsize;       /* decode step size (Quantizer.cpp:65-104, fraction 0.5) */
    uint32_t pad;
} grkgpu_dec_block;

/* scratch: >= grkgpu_t1_scratch_bytes_n(nblocks) device bytes, encode and
 * decode -- that is (nblocks rounded up to a multiple of 64) *
 * grkgpu_t1_scratch_bytes(): both keep the rows of 64 blocks interleaved, so
 * n * grkgpu_t1_scratch_bytes() is too small when n % 64 != 0; decode: every
 * segment at most GRKGPU_T1_MAX_SEG bytes (w*h*4 + 64 for a 64x64 block, the
 * encoder's slab bound). */
#define GRKGPU_T1_MAX_SEG (64 * 64 * 4 + 64)
size_t grkgpu_t1_scratch_bytes(void);
size_t grkgpu_t1_scratch_bytes_n(uint32_t nblocks);
int grkgpu_t1_encode_blocks(const grkgpu_enc_block *blocks, uint32_t nblocks, const int32_t *coef,
                            void *scratch, uint8_t *out, grkgpu_enc_result *results, int with_distortion,
                            void *stream);
int grkgpu_t1_decode_blocks(const grkgpu_dec_block *blocks, uint32_t nblocks, const uint8_t *data,
                            void *scratch, int32_t *dst, void *stream);

#ifdef __cplusplus
}
#endif
#endif
