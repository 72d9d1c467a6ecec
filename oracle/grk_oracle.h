/*
 * grk_oracle.h -- CPU restatement of Grok v5.1.0's JPEG 2000 Part-1 hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X product path (grokimagecompression_amd/).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product never links it.  It is a plain-C restatement written from ISO/IEC
 * 15444-1 plus the observed behaviour of the reference (file:line citations at
 * each function in grk_oracle.c), and it is pinned against the reference's own
 * output: the tests/golden j2k files were produced by the reference grk_compress and
 * must be reproduced byte-for-byte (tests/test_oracle_golden.py).
 *
 * Scope: DC shift, RCT/ICT, forward/inverse 5/3 + 9/7 DWT,
 * quantisation, EBCOT Tier-1 + MQ coder (encode/decode), Tier-2 packets,
 * main/tile headers -- enough to produce/consume complete .j2k codestreams for
 * Grok's default coding options (1 layer, LRCP, no precincts, cblksty 0).
 */
#ifndef GRK_ORACLE_H
#define GRK_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_COMPS 16
#define ORC_MAX_PASSES 100

typedef struct {
    uint32_t x0, y0, x1, y1; /* image area on the reference grid */
    uint32_t numcomps;
    uint32_t prec[ORC_MAX_COMPS];
    int32_t sgnd[ORC_MAX_COMPS];
    int32_t *data[ORC_MAX_COMPS]; /* planar (y1-y0) x (x1-x0), dx = dy = 1 */
} orc_image;

typedef struct {
    uint32_t numres;       /* resolutions (decomposition levels + 1), default 6 */
    uint32_t cblkw, cblkh; /* log2 code-block size, default 6,6 */
    int32_t irreversible;  /* 0: 5/3 reversible, 1: 9/7 irreversible */
    int32_t mct;           /* -1: auto (on iff >= 3 comps), 0: off, 1: RCT/ICT */
    int32_t tile_on;
    uint32_t tdx, tdy, tx0, ty0;
    int32_t nthreads;      /* 0: all cores */
} orc_params;

typedef struct {
    uint32_t rate;  /* cumulative bytes after this pass (after Grok's fix-ups) */
    uint32_t len;   /* bytes contributed by this pass */
    uint32_t term;  /* pass is terminated */
} orc_pass;

void orc_default_params(orc_params *p);

/* Whole-codestream encode/decode (reference: grk_compress / grk_decompress). */
int orc_encode(const orc_image *img, const orc_params *p, uint8_t **out, size_t *outlen);
int orc_decode(const uint8_t *buf, size_t len, orc_image *out, int32_t nthreads);
/* Reduced-resolution decode (grk_decompress -r / cp_reduce): -5 if reduce >= numresolutions. */
int orc_decode_reduce(const uint8_t *buf, size_t len, orc_image *out, int32_t nthreads, uint32_t reduce);
void orc_free(void *ptr);
void orc_image_free(orc_image *img);

/* ---- stage-level entry points (per-kernel parity checks) ---- */

/* DC level shift + forward MCT over n samples (TileProcessor.cpp:1449-1502). */
void orc_dcshift_mct_fwd(int32_t *c0, int32_t *c1, int32_t *c2, uint32_t numcomps,
                         uint64_t n, const int32_t *shift, int32_t mct, int32_t irreversible);

/* In-place forward DWT of one tile-component (Mallat layout, stride = width)
 * with tile-component origin (x0,y0) (WaveletForward.h:40-160). */
int orc_dwt_fwd(int32_t *buf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                uint32_t numres, int32_t irreversible, int32_t nthreads);

/* In-place inverse DWT (dwt.cpp:724 decode_tile_53 / :1544 decode_tile_97).
 * For 9/7 buf holds float bit patterns. */
int orc_dwt_inv(int32_t *buf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                uint32_t numres, int32_t irreversible, int32_t nthreads);

/* Tier-1 encode of one code-block from DWT-domain coefficients (preEncode
 * quantisation included; T1Part1.cpp:58-94, t1.cpp:1182-1326).
 * out must have >= 1 writable byte BEFORE it (value 0) -- the MQ coder's
 * initial bp = start - 1.  Returns number of passes; *numbps receives the
 * block's magnitude bit-plane count; *outlen the final byte count. */
int orc_t1_encode_cblk(const int32_t *src, uint32_t stride, uint32_t w, uint32_t h,
                       uint32_t orient, int32_t qmfbid, int32_t inv_step,
                       uint8_t *out, uint32_t outcap, orc_pass *passes,
                       uint32_t *numbps, uint32_t *outlen);

/* The same, also returning the per-pass normalised distortion decrease
 * sums of a rate-controlled encode in nmsedec[pass] (t1.cpp:217, :452, :684;
 * LUTs of t1_generate_luts.cpp:290-318). */
int orc_t1_encode_cblk_nmse(const int32_t *src, uint32_t stride, uint32_t w, uint32_t h,
                            uint32_t orient, int32_t qmfbid, int32_t inv_step,
                            uint8_t *out, uint32_t outcap, orc_pass *passes,
                            uint32_t *numbps, uint32_t *outlen, int32_t *nmsedec);

/* The four nmsedec tables (sig, sig0, ref, ref0; 128 entries each). */
void orc_nmse_tables(int16_t *out512);

/* t1_getwmsedec (t1.cpp:912-930): weighted distortion decrease of a pass. */
double orc_t1_wmsedec(int32_t nmsedec, uint32_t compno, uint32_t level, uint32_t orient, int32_t bpno,
                      uint32_t qmfbid, double stepsize, const double *mct_norms, uint32_t mct_numcomps);

/* Tier-1 decode of one single-segment code-block (t1.cpp:1038-1130).
 * data must have 2 writable bytes after len.  Writes w*h raw decoded values
 * (one extra LSB of precision, as Grok's t1->data) into dst. */
int orc_t1_decode_cblk(uint8_t *data, uint32_t len, uint32_t numpasses, uint32_t numbps,
                       uint32_t w, uint32_t h, uint32_t orient, int32_t *dst);

/* Band geometry helpers for tests. */
uint32_t orc_count_cblks(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t numres,
                         uint32_t cblkw, uint32_t cblkh);

#ifdef __cplusplus
}
#endif
#endif
