// grk_device.h -- device-visible descriptors shared by kernels.hip and codec.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "t1_flat.h"

namespace grkgpu {

constexpr int GRK_MAX_COMPS = 16;
constexpr int GRK_MAX_PASSES = 96;  // 3 * 31 - 2 = 91 passes max for cblksty 0

struct PlanePtrs { int32_t *p[GRK_MAX_COMPS]; };
// Image planes as the caller holds them: int32 (grk_image) or the 8 / 16-bit
// samples of the image file (GRKGPU_SAMPLE_*, include/grk_mi355x.h), widened
// to int32 by the kernel that first reads them (DC shift + MCT, or the fused
// DWT level 0) -- an 8K 12-bit frame crosses PCIe as 2 B/sample.
struct SrcPlanes { const void *p[GRK_MAX_COMPS]; };
enum SampleFmt : int32_t { SMP_I32 = 0, SMP_U8 = 1, SMP_I8 = 2, SMP_U16 = 3, SMP_I16 = 4 };
constexpr uint32_t sample_bytes(int32_t fmt) { return fmt == SMP_I32 ? 4u : (fmt <= SMP_I8 ? 1u : 2u); }
struct ShiftArr { int32_t v[GRK_MAX_COMPS]; };

// One code-block to encode (T1Part1::preEncode + t1_encode_cblk inputs,
// t1/Tier1.cpp:24-96 encodeBlockInfo).
struct EncBlock {
    uint64_t coef_off;  // element offset of the block's top-left in the coefficient arena
    uint64_t out_off;   // byte offset of the block's output in the MQ slab (out[-1] == 0)
    uint32_t stride, w, h, orient;
    int32_t qmfbid, inv_step;
};

struct EncResult {
    uint32_t numbps, numpasses, len, pad;  // pad != 0: numbps above the band's bound
    uint32_t nsym, pad1, pad2, pad3;       // nsym: MQ symbols coded
    uint32_t rate[GRK_MAX_PASSES];         // cumulative, after Grok's fix-ups
    int32_t nmsedec[GRK_MAX_PASSES];       // per-pass distortion sums (launch_t1_dist only)
};
// bytes of an EncResult without the distortion sums (what a D2H needs when
// no rate control runs)
constexpr size_t ENC_RESULT_RATE_BYTES = 32 + 4 * GRK_MAX_PASSES;

// Normalised-MSE decrease tables (t1_generate_luts.cpp:290-318, restated):
// index = the 7 magnitude bits from the coded bit-plane down.
struct NmseLut { int16_t sig[128], sig0[128], ref[128], ref0[128]; };
const NmseLut &nmse_lut();

// One code-block to decode (t1/Tier1.cpp:98-175 decodeBlockInfo).
struct DecBlock {
    uint64_t data_off;  // byte offset of the (single) segment in the data buffer
    uint64_t dst_off;   // element offset of the block's top-left in the tile arena
    uint32_t len, numpasses, numbps, w, h, orient, dstride;
    int32_t irrev;
    float step;
    uint32_t pad;       // unstuffed-stream region offset / 16 bytes (launch_t1_decode)
};

struct GatherItem { uint64_t src, dst; uint32_t len, pad; };  // pad: 0 = header blob, 1 = MQ slab

hipError_t launch_dcshift_mct_fwd(const SrcPlanes &src, int32_t fmt, uint32_t sstride, const PlanePtrs &dst,
                                  uint32_t tw, uint32_t th, uint32_t ncomp, const ShiftArr &shift, int32_t mct,
                                  int32_t irrev, hipStream_t s);
// src rows at sstride elements (a window of a tile buffer), dst rows at dstride;
// irrev: bit k set = component k holds 9/7 (float) samples; MCT follows
// component 0's wavelet
// DC shift + custom MCT (Part 2) of one tile: m.c = the n x n encoding matrix in
// 13-bit fixed point (row-major)
struct MctMatrix { int32_t c[GRK_MAX_COMPS * GRK_MAX_COMPS]; };
hipError_t launch_dcshift_mct_custom(const SrcPlanes &src, int32_t fmt, uint32_t sstride, const PlanePtrs &dst,
                                     uint32_t tw, uint32_t th, uint32_t ncomp, const ShiftArr &shift,
                                     const MctMatrix &m, hipStream_t s);
hipError_t launch_mct_inv_dcshift(const PlanePtrs &src, uint32_t sstride, uint32_t tw, uint32_t th,
                                  const PlanePtrs &dst, uint32_t dstride, uint32_t ncomp, const ShiftArr &shift,
                                  const ShiftArr &mn, const ShiftArr &mx, int32_t mct, int32_t irrev, hipStream_t s);
// One DWT level of one tile-component (dwt.hip).  A launch runs one level of
// every job in a table (grid.y = job).
struct DwtJob {
    const int32_t *in;     // fwd: resolution samples;     inv: LL band
    const int32_t *coef;   // inv: HL/LH/HH (Mallat)
    int32_t *out;          // fwd: LL band output;         inv: reconstructed resolution
    int32_t *bands;        // fwd: HL/LH/HH output (Mallat)
    uint32_t in_stride, coef_stride, out_stride, bands_stride;  // elements
    uint32_t in_bytes, coef_bytes, out_bytes, bands_bytes;      // buffer extents
    int32_t rw, rh, casx, casy, snx, sny;
    int32_t tiles_x, ntiles;
    // Forward level 0 with the DC shift + MCT fused into its loads
    // (TileProcessor.cpp:1449-1471, mct.cpp:85-139 / 195-350): the window is
    // read from the image planes instead of `in`.  mct_mode 0: not fused;
    // 1: DC shift of src[0]; 2: RCT output component `comp` of src[0..2];
    // 3: ICT output component `comp`.  Samples in format src_fmt (SampleFmt).
    const void *src[3];         // image planes at the tile origin
    uint32_t src_stride, src_bytes;  // elements; bytes from src[i] to its plane's end (min)
    int32_t shift[3];
    int32_t mct_mode, comp, src_vec;  // src_vec: pair loads allowed (base aligned to 2 samples, even stride)
    int32_t src_fmt, pad_;
    // the windows a launch runs for this job: columns [win_x0, win_x0 +
    // tiles_x), rows [win_y0, win_y0 + win_ny) of the level's window grid
    // (dwt_job_tiles; all of them unless reg_* restricts the output region:
    // window decode, grk_set_decode_area)
    int32_t win_x0, win_y0, win_ny;
    int32_t reg_x0, reg_y0, reg_x1, reg_y1;  // output region (resolution-relative); reg_x1 = 0: all
    int32_t pad2_;
};
// DWT plan options (grkgpu_dwt_options, set by grkgpu_set_dwt_options; the
// defaults are the measured best -- the parity suite forces the others)
struct DwtOptions {
    int32_t fuse_level0 = -1;                    // -1: 3-component 5/3 tiles; 0 never; 1 always
    int32_t f01_rows = 4;                        // 9/7 levels 0 + 1 fused: 2 / 4 / 6 row windows; 0 = apart
    uint64_t f01_min_samples = (uint64_t)1 << 23;  // fuse a level pair from this many samples
    uint64_t f01_small_min_samples = ~(uint64_t)0;  // ... and, with 2 row windows, smaller pairs from this many
    int32_t inv01 = 2;                               // the two largest inverse levels in one launch (k_dwt_inv01):
                                                     // 2 / 4 stage-A row windows per workgroup; 0 = apart
    uint64_t inv01_min_samples = (uint64_t)1 << 23;  // ... when the larger has this many samples
    int32_t pair_group = 0;  // fused level pairs: workgroups walk groups of this many columns top-down (0: row-major)
    int32_t f64_lift = 0;    // forward 9/7 fused pair: lifting in f64 FMA + floor instead of v_mad_i64_i32
    int32_t t1_dec_sort = 1;   // T1 decode: blocks in decreasing order of expected work (-1: only a lone call)
    int32_t t1_dec_bpw = 0;  // T1 decode: blocks per wavefront (0: by block count)
    int32_t mid_th = 0;      // window rows of a level of 2^21 .. 2^23 samples (0: 8)
    int32_t t1_enc_bpw = 0;  // T1 encode (MQ coder): blocks per wavefront (0: by block count)
    int32_t t1_enc_sort = 0; // T1 encode: MQ coder lanes take the blocks heaviest first (device counting sort)
    int32_t pair_kernel = 1;  // fused forward level pairs: 1 = k_dwt_fwd_pair (streamed strips, 5/3 + 9/7),
                              // 0 = k_dwt_fwd01 (9/7 windows, f01_rows)
    int32_t pair_rows = 0;    // k_dwt_fwd_pair: level-(l+1) rows per segment (even; 0 = by size)
    int32_t pair_waves = 0;   // k_dwt_fwd_pair: level-l waves per workgroup (3 / 4; 0 = by width)
    uint64_t pair_min_samples = (uint64_t)1 << 20;  // k_dwt_fwd_pair: fuse pairs from this many level-l samples
};
const DwtOptions &dwt_options();
// level geometry code (window rows) for a level of that many samples whose
// smallest resolution is minw x minh
int dwt_pick_th(int irrev, uint64_t level_samples, int minw, int minh);
constexpr int DWT_FUSED = 1 << 16;       // geometry-code flag: forward level with fused DC shift loads
constexpr int DWT_FUSED_MCT3 = 1 << 17;  // ... with fused DC shift + MCT (jobs in component triples)
constexpr int DWT_FMT_SHIFT = 18;        // bits 18-20: SampleFmt of the fused level's image planes (I32 / U8 / U16)
// the window grid of a job at `th` window rows: tiles_x, ntiles (whole
// workgroups) and win_* (restricted to reg_* when set)
void dwt_job_tiles(int irrev, int th, DwtJob &j);
hipError_t launch_dwt_jobs(const DwtJob *jobs_dev, uint32_t njobs, uint32_t max_tiles, int th, int irrev,
                           int inverse, hipStream_t s);
// forward 9/7 levels 0 and 1 in one launch (dwt.hip k_dwt_fwd01): workgroups
// per job from dwt01_tiles (level-1 geometry), 0 if unsupported
// (ny: level-0 row windows per workgroup, 2 / 4 / 6)
int dwt01_tiles(int irrev, int ny, int rw1, int rh1, int casx1, int casy1, int *tiles_x);
// the last two inverse levels in one launch (k_dwt_inv01): workgroups per job
// for a larger level of rw_b x rh_b; jobsA / jobsB = the two levels
int dwt_inv01_tiles(int irrev, int rw_b, int rh_b, int casx_b, int casy_b);
hipError_t launch_dwt_inv01(const DwtJob *jobsA, const DwtJob *jobsB, uint32_t njobs, uint32_t max_tiles, int irrev,
                            int na, hipStream_t s);
hipError_t launch_dwt_fwd01(const DwtJob *jobs0, const DwtJob *jobs1, uint32_t njobs, uint32_t max_tiles, int irrev,
                            int ny, hipStream_t s);
// forward levels l and l + 1 streamed down column strips (k_dwt_fwd_pair, 5/3
// and 9/7): level-(l+1) core columns per workgroup with nw0 (3 / 4) level-l
// waves, workgroups per job at s1 level-(l+1) rows per segment
int dwt_pair_cw1(int irrev, int nw0);
int dwt_pair_wgs(int irrev, int nw0, int s1, int rw1, int rh1, int casx1, int casy1);
hipError_t launch_dwt_fwd_pair(const DwtJob *jobs0, const DwtJob *jobs1, uint32_t njobs, uint32_t max_wgs, int irrev,
                               int nw0, int s1, hipStream_t s);
// sym: symbol-stream arena; sym_off[i] = block i's byte offset (n+1 entries,
// capacity = (sym_off[i+1]-sym_off[i]) / sym_slot_bytes(w,h) planes), or null
// for the fixed layout of 32 planes x sym_slot_bytes(64,64) per block.
// cblksty: the CBLKSTY_* mode switches of the codestream (t1_lane.h), 0 = none.
// scratch: t1e_scratch_bytes(n, maxdepth) bytes (t1_lane.h EncScratch), with
// maxdepth >= every block's plane capacity (<= 32)
hipError_t launch_t1_encode(const EncBlock *blocks, uint32_t n, const int32_t *coef, void *scratch,
                            uint8_t *sym, const uint64_t *sym_off, uint32_t maxdepth, uint8_t *out, EncResult *res,
                            hipStream_t s, uint32_t cblksty = 0, uint32_t bpw = 0, uint32_t *order = nullptr);
// device words the MQ coder's work order needs (launch_t1_encode `order`)
uint32_t t1_order_words(uint32_t nblocks);
// Per-pass distortion sums of the blocks k_t1_model coded (same scratch and
// maxdepth): nmsedec[pass] of every block, in the pass order of
// t1_encode_cblk (t1.cpp:1222-1260).
// Pass records formed on the device when a layer is rate-controlled: the
// host's per-pass loop of the encoder (codec.cpp: rate, length, termination
// t1.cpp:1131-1151, cumulative distortion t1.cpp:1249-1254 with
// t1_getwmsedec :912-930, and the block's slope range, t2.cpp block_slopes)
// moved next to the results it reads, so only records cross PCIe and the
// host's Tier-2 starts at the layer formation.  DevPass has EncPass's layout
// (t2.h; static_assert in codec.cpp); block i's records go to
// out[pass0[i] .. pass0[i + 1]) -- slots sized from the band's bit-plane
// bound -- and its summary to sum[i].
struct DevPass {
    uint32_t rate, len;
    double dd;
    uint16_t slope;
    uint8_t term;
};
struct PassSum {
    uint32_t numbps, numpasses, len, nsym;
    uint32_t bad;  // 1: numbps above the band's bound, 2: more passes than slots, 4: MQ slab overflow
    uint32_t z0;   // EncCblkState::z0
    double smin, smax, s0max, disto;
};
hipError_t launch_pass_records(const EncBlock *blocks, const EncResult *res, const double *wfac, const uint64_t *pass0,
                               uint32_t n, uint32_t cblksty, DevPass *out, PassSum *sum, hipStream_t s);
hipError_t launch_t1_dist(const EncBlock *blocks, uint32_t n, uint32_t maxdepth, const int32_t *coef,
                          const void *scratch, EncResult *res, hipStream_t s);
// ubuf: unstuffed-stream arena; block i's region at ubuf + i * fixed_words
// words, or (fixed_words == 0) at blocks[i].pad * 16 bytes
// (t1_unstuff_region_words words each).
// segs / seg_first: the codeword segments of every block (block i's are
// segs[seg_first[i] .. seg_first[i+1]), each with its own unstuffed region at
// ubuf + ub_off * 16 bytes); null: one segment per block at blocks[i].data_off.
// cblksty: CBLKSTY_* mode switches; roi: per-block ROI shift (null: none).
hipError_t launch_t1_decode(const DecBlock *blocks, uint32_t n, const uint8_t *data, T1Scratch *scratch,
                            int32_t *tiles, hipStream_t s, uint32_t *ubuf, uint32_t fixed_words,
                            const DecSeg *segs = nullptr, const uint32_t *seg_first = nullptr, uint32_t cblksty = 0,
                            const uint8_t *roi = nullptr, uint32_t bpw = 0);
// blocks per wavefront (bpw, a power of two <= 64; 0 = the options' value or
// the block-count rule) of the T1 kernels' lane-per-block launches, and the
// rule for a call that has the GPU to itself (lone_bpw): enough wavefronts
// to give every SIMD of the chip one and a half (1,536), not full lanes
uint32_t lone_bpw(uint32_t nblocks);
// 32-bit words of a block's unstuffed-stream region (header + words + carries)
inline uint32_t t1_unstuff_region_words(uint32_t len) { return 4 + unstuff_word_cap(len) + unstuff_carry_cap(len); }
hipError_t launch_gather(const uint8_t *hdr, const uint8_t *slab, const GatherItem *items, uint32_t n, uint8_t *dst,
                         hipStream_t s);

// One product of the forward ICT (mct.cpp:195-350), int_fix_mul(r << 11, c)
// = (2048 r c + 4096) >> 13 with the 64-bit product, for a DC-shifted sample
// r (|r| <= 2^16, precision <= 16 bits): 2048 (r c + 2) / 8192 = (r c + 2) / 4,
// so the same value is floor((r c + 2) / 4) in 32-bit arithmetic (|r c| < 2^30).
__device__ __forceinline__ int32_t ict_term(int32_t r, int32_t c) { return (r * c + 2) >> 2; }

}  // namespace grkgpu
