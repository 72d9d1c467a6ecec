/*
 * grk_oracle.c -- CPU restatement of the Grok v5.1.0 JPEG 2000 hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see grk_oracle.h).  Written from ISO/IEC 15444-1
 * and the reference's observed behaviour; each block cites the reference
 * file:line (paths relative to src/lib/jp2/ of /root/reference) whose
 * behaviour it restates.  Pinned byte-for-byte against reference-generated
 * codestreams in tests/golden/.
 */
#define _GNU_SOURCE
#include "grk_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------------- */
/* small helpers                                                             */
/* ------------------------------------------------------------------------- */

static inline uint32_t ceildiv_u32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + b - 1) / b); }
static inline uint32_t ceildivpow2(uint32_t a, uint32_t e) { return (uint32_t)(((uint64_t)a + ((uint64_t)1 << e) - 1) >> e); }
static inline uint32_t floordivpow2(uint32_t a, uint32_t e) { return a >> e; }
static inline int32_t floorlog2_i(int32_t a) { int32_t l = 0; while (a > 1) { a >>= 1; l++; } return l; }
static inline uint32_t floorlog2_u(uint32_t a) { uint32_t l = 0; while (a > 1) { a >>= 1; l++; } return l; }
static inline uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
static inline uint32_t umax(uint32_t a, uint32_t b) { return a > b ? a : b; }

void orc_free(void *p) { free(p); }

/* ---- tiny parallel-for on pthreads (the reference uses a std::thread pool,
 *      util/ThreadPool.hpp; work is split exactly as independent items). ---- */
typedef void (*pf_fn)(void *ctx, uint64_t i);
typedef struct { pf_fn fn; void *ctx; uint64_t n; volatile uint64_t next; pthread_mutex_t mu; } pf_job;

static void *pf_worker(void *arg) {
    pf_job *j = (pf_job *)arg;
    for (;;) {
        uint64_t i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (i >= j->n) break;
        j->fn(j->ctx, i);
    }
    return NULL;
}

static int g_default_threads = 0;
static int resolve_threads(int n) {
    if (n > 0) return n;
    if (g_default_threads > 0) return g_default_threads;
    long c = sysconf(_SC_NPROCESSORS_ONLN);
    return c > 0 ? (int)c : 1;
}

static void parallel_for(uint64_t n, int nthreads, pf_fn fn, void *ctx) {
    nthreads = resolve_threads(nthreads);
    if (nthreads <= 1 || n <= 1) {
        for (uint64_t i = 0; i < n; ++i) fn(ctx, i);
        return;
    }
    if ((uint64_t)nthreads > n) nthreads = (int)n;
    pf_job j;
    j.fn = fn; j.ctx = ctx; j.n = n; j.next = 0;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, pf_worker, &j);
    pf_worker(&j);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th);
}

/* ------------------------------------------------------------------------- */
/* MQ arithmetic coder -- ISO 15444-1 Annex C; Grok: t1/t1_part1/mqc_enc.cpp */
/* ------------------------------------------------------------------------- */

/* Table C.2 as (Qe, NMPS, NLPS, SWITCH).  Same probability-state machine as
 * mqc_enc.cpp:69-166 (which stores it as 94 (state,mps) pairs). */
static const uint16_t MQ_QE[47] = {
    0x5601, 0x3401, 0x1801, 0x0AC1, 0x0521, 0x0221, 0x5601, 0x5401, 0x4801, 0x3801,
    0x3001, 0x2401, 0x1C01, 0x1601, 0x5601, 0x5401, 0x5101, 0x4801, 0x3801, 0x3401,
    0x3001, 0x2801, 0x2401, 0x2201, 0x1C01, 0x1801, 0x1601, 0x1401, 0x1201, 0x1101,
    0x0AC1, 0x09C1, 0x08A1, 0x0521, 0x0441, 0x02A1, 0x0221, 0x0141, 0x0111, 0x0085,
    0x0049, 0x0025, 0x0015, 0x0009, 0x0005, 0x0001, 0x5601};
static const uint8_t MQ_NMPS[47] = {
    1, 2, 3, 4, 5, 38, 7, 8, 9, 10, 11, 12, 13, 29, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24,
    25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 45, 46};
static const uint8_t MQ_NLPS[47] = {
    1, 6, 9, 12, 29, 33, 6, 14, 14, 14, 17, 18, 20, 21, 14, 14, 15, 16, 17, 18, 19, 19, 20, 21,
    22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 46};
static const uint8_t MQ_SWITCH[47] = {1, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                      0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};

/* context numbering (t1/t1_part1/t1.h:65-76) */
enum { CX_ZC = 0, CX_SC = 9, CX_MAG = 14, CX_AGG = 17, CX_UNI = 18, NUM_CX = 19 };

typedef struct {
    uint32_t a, c, ct;
    int64_t bp;         /* index into buf; starts at -1 (mqc_init_enc) */
    uint8_t *buf;       /* buf[-1] must be readable and == 0 */
    uint8_t st[NUM_CX]; /* state index */
    uint8_t mps[NUM_CX];
} mq_enc;

/* mqc_resetstates (mqc_dec.cpp:207-215) */
static void mq_reset(uint8_t *st, uint8_t *mps) {
    for (int i = 0; i < NUM_CX; ++i) { st[i] = 0; mps[i] = 0; }
    st[CX_UNI] = 46; st[CX_AGG] = 3; st[CX_ZC] = 4;
}

/* mqc_init_enc (mqc_enc.cpp:240-260): A=0x8000, C=0, CT=12, BP=start-1 */
static void mqe_init(mq_enc *e, uint8_t *buf) {
    e->a = 0x8000; e->c = 0; e->ct = 12; e->bp = -1; e->buf = buf;
    mq_reset(e->st, e->mps);
}

/* BYTEOUT (mqc_enc.cpp:168-199, ISO Fig. C.8) */
static void mqe_byteout(mq_enc *e) {
    uint8_t *b = e->buf;
    if (b[e->bp] == 0xff) {
        e->bp++; b[e->bp] = (uint8_t)(e->c >> 20); e->c &= 0xfffff; e->ct = 7;
    } else if ((e->c & 0x8000000) == 0) {
        e->bp++; b[e->bp] = (uint8_t)(e->c >> 19); e->c &= 0x7ffff; e->ct = 8;
    } else {
        b[e->bp]++;
        if (b[e->bp] == 0xff) {
            e->c &= 0x7ffffff;
            e->bp++; b[e->bp] = (uint8_t)(e->c >> 20); e->c &= 0xfffff; e->ct = 7;
        } else {
            e->bp++; b[e->bp] = (uint8_t)(e->c >> 19); e->c &= 0x7ffff; e->ct = 8;
        }
    }
}

static void mqe_renorm(mq_enc *e) {
    do {
        e->a <<= 1; e->c <<= 1; e->ct--;
        if (e->ct == 0) mqe_byteout(e);
    } while ((e->a & 0x8000) == 0);
}

/* ENCODE/CODEMPS/CODELPS (mqc_enc.cpp:211-233, 262-267) */
static void mqe_encode(mq_enc *e, int cx, uint32_t d) {
    uint32_t s = e->st[cx];
    uint32_t qe = MQ_QE[s];
    e->a -= qe;
    if (d == e->mps[cx]) {
        if ((e->a & 0x8000) == 0) {
            if (e->a < qe) e->a = qe; else e->c += qe;
            e->st[cx] = MQ_NMPS[s];
            mqe_renorm(e);
        } else {
            e->c += qe;
        }
    } else {
        if (e->a < qe) e->c += qe; else e->a = qe;
        if (MQ_SWITCH[s]) e->mps[cx] ^= 1;
        e->st[cx] = MQ_NLPS[s];
        mqe_renorm(e);
    }
}

/* FLUSH (mqc_enc.cpp:274-289 + SETBITS :235-240) */
static void mqe_flush(mq_enc *e) {
    uint32_t tempc = e->c + e->a;
    e->c |= 0xffff;
    if (e->c >= tempc) e->c -= 0x8000;
    e->c <<= e->ct; mqe_byteout(e);
    e->c <<= e->ct; mqe_byteout(e);
    if (e->buf[e->bp] != 0xff) e->bp++;
}

static inline uint32_t mqe_numbytes(const mq_enc *e) { return (uint32_t)e->bp; }

typedef struct {
    uint32_t a, c, ct;
    const uint8_t *buf; /* buf[len], buf[len+1] == 0xFF (artificial marker) */
    uint32_t bp;
    uint8_t st[NUM_CX];
    uint8_t mps[NUM_CX];
} mq_dec;

/* bytein_dec_macro (mqc_dec_inl.h:107-127) */
static inline void mqd_bytein(mq_dec *d) {
    uint32_t next = d->buf[d->bp + 1];
    if (d->buf[d->bp] == 0xff) {
        if (next > 0x8f) { d->c += 0xff00; d->ct = 8; }
        else { d->bp++; d->c += next << 9; d->ct = 7; }
    } else {
        d->bp++; d->c += next << 8; d->ct = 8;
    }
}

/* mqc_init_dec (mqc_dec.cpp:178-193) */
static void mqd_init(mq_dec *d, const uint8_t *buf, uint32_t len) {
    d->buf = buf; d->bp = 0;
    d->c = (uint32_t)((len == 0) ? 0xff : buf[0]) << 16;
    mqd_bytein(d);
    d->c <<= 7; d->ct -= 7; d->a = 0x8000;
    mq_reset(d->st, d->mps);
}

static inline void mqd_renorm(mq_dec *d) {
    do {
        if (d->ct == 0) mqd_bytein(d);
        d->a <<= 1; d->c <<= 1; d->ct--;
    } while (d->a < 0x8000);
}

/* decode_macro (mqc_dec_inl.h:148-166, ISO C.3.2) */
static inline uint32_t mqd_decode(mq_dec *d, int cx) {
    uint32_t s = d->st[cx];
    uint32_t qe = MQ_QE[s];
    uint32_t r;
    d->a -= qe;
    if (d->c < (qe << 16)) {
        if (d->a < qe) { d->a = qe; r = d->mps[cx]; d->st[cx] = MQ_NMPS[s]; }
        else { d->a = qe; r = d->mps[cx] ^ 1; if (MQ_SWITCH[s]) d->mps[cx] ^= 1; d->st[cx] = MQ_NLPS[s]; }
        mqd_renorm(d);
    } else {
        d->c -= qe << 16;
        if (d->a < 0x8000) {
            if (d->a < qe) { r = d->mps[cx] ^ 1; if (MQ_SWITCH[s]) d->mps[cx] ^= 1; d->st[cx] = MQ_NLPS[s]; }
            else { r = d->mps[cx]; d->st[cx] = MQ_NMPS[s]; }
            mqd_renorm(d);
        } else {
            r = d->mps[cx];
        }
    }
    return r;
}

/* ------------------------------------------------------------------------- */
/* Tier-1 context modelling (ISO Annex D; Grok t1/t1_part1/t1.cpp)           */
/* ------------------------------------------------------------------------- */
/* Per-sample state in a (w+2)x(h+2) array with a zero border: */
enum { F_SIG = 1, F_NEG = 2, F_VISIT = 4, F_REF = 8 };

/* Zero-coding context, Table D.1 (t1_generate_luts.cpp:63-140; band 1 = HL
 * swaps the roles of horizontal and vertical neighbours). */
static inline int zc_ctx(int h, int v, int d, uint32_t orient) {
    if (orient == 3) {
        int hv = h + v;
        if (d == 0) return hv == 0 ? 0 : (hv == 1 ? 1 : 2);
        if (d == 1) return hv == 0 ? 3 : (hv == 1 ? 4 : 5);
        if (d == 2) return hv == 0 ? 6 : 7;
        return 8;
    }
    if (orient == 1) { int t = h; h = v; v = t; }
    if (h == 0) {
        if (v == 0) return d == 0 ? 0 : (d == 1 ? 1 : 2);
        return v == 1 ? 3 : 4;
    }
    if (h == 1) return v == 0 ? (d == 0 ? 5 : 6) : 7;
    return 8;
}

static inline int nb_sig(const uint8_t *f, int s) { return f[0] & F_SIG ? 1 : 0; (void)s; }

static inline int zc_of(const uint8_t *p, int stride, uint32_t orient) {
    int h = (p[-1] & F_SIG) + (p[1] & F_SIG);
    int v = (p[-stride] & F_SIG) + (p[stride] & F_SIG);
    int d = (p[-stride - 1] & F_SIG) + (p[-stride + 1] & F_SIG) + (p[stride - 1] & F_SIG) + (p[stride + 1] & F_SIG);
    return zc_ctx(h, v, d, orient);
}

static inline int any_nb_sig(const uint8_t *p, int stride) {
    return ((p[-1] | p[1] | p[-stride] | p[stride] | p[-stride - 1] | p[-stride + 1] | p[stride - 1] | p[stride + 1]) & F_SIG) != 0;
}

/* Sign-coding context and XOR bit, Table D.3 (t1_generate_luts.cpp:142-215) */
static inline int contrib(uint8_t f) { return (f & F_SIG) ? ((f & F_NEG) ? -1 : 1) : 0; }
static inline int clamp1(int x) { return x > 1 ? 1 : (x < -1 ? -1 : x); }
static inline int sc_of(const uint8_t *p, int stride, int *xorbit) {
    int hc = clamp1(contrib(p[-1]) + contrib(p[1]));
    int vc = clamp1(contrib(p[-stride]) + contrib(p[stride]));
    int x = 0;
    if (hc < 0 || (hc == 0 && vc < 0)) x = 1;
    if (hc < 0) { hc = -hc; vc = -vc; }
    *xorbit = x;
    if (hc == 0) return CX_SC + (vc == 0 ? 0 : 1);
    return CX_SC + (vc == -1 ? 2 : (vc == 0 ? 3 : 4));
}

static inline int mag_ctx(const uint8_t *p, int stride) {
    if (*p & F_REF) return CX_MAG + 2;
    return CX_MAG + (any_nb_sig(p, stride) ? 1 : 0);
}

/* int_fix_mul_t1 (t1_part1/T1Part1.cpp:45-56): 13-bit x 11-bit -> 6 frac bits */
static inline int32_t fix_mul_t1(int32_t a, int32_t b) {
    int64_t t = (int64_t)a * (int64_t)b;
    t += (int64_t)1 << 17;
    return (int32_t)(t >> 18);
}

/* Normalised MSE decrease tables (t1_generate_luts.cpp:290-318, the
 * generator of t1_luts.h lut_nmsedec_sig / sig0 / ref / ref0), restated:
 * index i = the 7 magnitude bits from the coded bit-plane down (6 fraction
 * bits), t = i / 2^6; sig: (t^2 - (t - 1.5)^2), sig0: t^2, ref: ((t - 1)^2 -
 * (t - 1.5 or t - 0.5)^2) (by bit 6), ref0: (t - 1)^2, each rounded to 1/64
 * and scaled by 8192, clamped at 0. */
static int16_t NMSE_SIG[128], NMSE_SIG0[128], NMSE_REF[128], NMSE_REF0[128];
static pthread_once_t nmse_once = PTHREAD_ONCE_INIT;
static int nmse_q(double x) {
    const int v = (int)(floor(x * 64.0 + 0.5) / 64.0 * 8192.0);
    return v > 0 ? v : 0;
}
static void nmse_init(void) {
    for (int i = 0; i < 128; ++i) {
        const double t = i / 64.0;
        double u = t, v = t - 1.5;
        NMSE_SIG[i] = (int16_t)nmse_q(u * u - v * v);
        NMSE_SIG0[i] = (int16_t)nmse_q(u * u);
        u = t - 1.0;
        v = (i & 64) ? t - 1.5 : t - 0.5;
        NMSE_REF[i] = (int16_t)nmse_q(u * u - v * v);
        NMSE_REF0[i] = (int16_t)nmse_q(u * u);
    }
}
/* t1_getnmsedec_sig / _ref (t1.cpp:155-166): x = |quantised coefficient|
 * (6 fraction bits), bitpos = the pass's bit-plane */
static inline int32_t nmse_sig(uint32_t x, int32_t bitpos) {
    return bitpos > 0 ? NMSE_SIG[(x >> bitpos) & 127] : NMSE_SIG0[x & 127];
}
static inline int32_t nmse_ref(uint32_t x, int32_t bitpos) {
    return bitpos > 0 ? NMSE_REF[(x >> bitpos) & 127] : NMSE_REF0[x & 127];
}

void orc_nmse_tables(int16_t *out) {
    pthread_once(&nmse_once, nmse_init);
    memcpy(out, NMSE_SIG, sizeof NMSE_SIG);
    memcpy(out + 128, NMSE_SIG0, sizeof NMSE_SIG0);
    memcpy(out + 256, NMSE_REF, sizeof NMSE_REF);
    memcpy(out + 384, NMSE_REF0, sizeof NMSE_REF0);
}

/* sqrt_energy_gains (HTParams.cpp:54-90): the 5/3 and 9/7 synthesis energy
 * gains per decomposition level, as the reference stores them (float) */
static const float SQE_53_L[34] = {1.0000e+00f, 1.2247e+00f, 1.3229e+00f, 1.5411e+00f, 1.7139e+00f, 1.9605e+00f,
    2.2044e+00f, 2.5047e+00f, 2.8277e+00f, 3.2049e+00f, 3.6238e+00f, 4.1033e+00f, 4.6423e+00f, 5.2548e+00f,
    5.9462e+00f, 6.7299e+00f, 7.6159e+00f, 8.6193e+00f, 9.7544e+00f, 1.1039e+01f, 1.2493e+01f, 1.4139e+01f,
    1.6001e+01f, 1.8108e+01f, 2.0493e+01f, 2.3192e+01f, 2.6246e+01f, 2.9702e+01f, 3.3614e+01f, 3.8041e+01f,
    4.3051e+01f, 4.8721e+01f, 5.5138e+01f, 6.2399e+01f};
static const float SQE_53_H[34] = {1.0458e+00f, 1.3975e+00f, 1.4389e+00f, 1.7287e+00f, 1.8880e+00f, 2.1841e+00f,
    2.4392e+00f, 2.7830e+00f, 3.1341e+00f, 3.5576e+00f, 4.0188e+00f, 4.5532e+00f, 5.1494e+00f, 5.8301e+00f,
    6.5963e+00f, 7.4663e+00f, 8.4489e+00f, 9.5623e+00f, 1.0821e+01f, 1.2247e+01f, 1.3860e+01f, 1.5685e+01f,
    1.7751e+01f, 2.0089e+01f, 2.2735e+01f, 2.5729e+01f, 2.9117e+01f, 3.2952e+01f, 3.7292e+01f, 4.2203e+01f,
    4.7761e+01f, 5.4051e+01f, 6.1170e+01f, 6.9226e+01f};

static const float SQE_97_L[34] = {1.0000e+00f, 1.4021e+00f, 2.0304e+00f, 2.9012e+00f, 4.1153e+00f, 5.8245e+00f,
    8.2388e+00f, 1.1652e+01f, 1.6479e+01f, 2.3304e+01f, 3.2957e+01f, 4.6609e+01f, 6.5915e+01f, 9.3217e+01f,
    1.3183e+02f, 1.8643e+02f, 2.6366e+02f, 3.7287e+02f, 5.2732e+02f, 7.4574e+02f, 1.0546e+03f, 1.4915e+03f,
    2.1093e+03f, 2.9830e+03f, 4.2185e+03f, 5.9659e+03f, 8.4371e+03f, 1.1932e+04f, 1.6874e+04f, 2.3864e+04f,
    3.3748e+04f, 4.7727e+04f, 6.7496e+04f, 9.5454e+04f};
static const float SQE_97_H[34] = {1.4425e+00f, 1.9669e+00f, 2.8839e+00f, 4.1475e+00f, 5.8946e+00f, 8.3472e+00f,
    1.1809e+01f, 1.6701e+01f, 2.3620e+01f, 3.3403e+01f, 4.7240e+01f, 6.6807e+01f, 9.4479e+01f, 1.3361e+02f,
    1.8896e+02f, 2.6723e+02f, 3.7792e+02f, 5.3446e+02f, 7.5583e+02f, 1.0689e+03f, 1.5117e+03f, 2.1378e+03f,
    3.0233e+03f, 4.2756e+03f, 6.0467e+03f, 8.5513e+03f, 1.2093e+04f, 1.7103e+04f, 2.4187e+04f, 3.4205e+04f,
    4.8373e+04f, 6.8410e+04f, 9.6747e+04f, 1.3682e+05f};

/* dwt_utils::getnorm (dwt_utils.cpp:143-166): products of two float gains,
 * computed in float and widened */
static double orc_getnorm(uint32_t level, uint32_t orient, int reversible) {
    const float *L = reversible ? SQE_53_L : SQE_97_L, *H = reversible ? SQE_53_H : SQE_97_H;
    float v = 0.0f;
    if (orient == 0) v = L[level] * L[level];
    else if (orient == 3) v = H[level] * H[level];
    else v = L[level + 1] * H[level];
    return (double)v;
}

/* t1_getwmsedec (t1.cpp:912-930): a pass's weighted MSE decrease from its
 * normalised sum, the band's norm, step size and bit-plane, and the MCT
 * component weight (mct_norms, TileProcessor.cpp:1535-1551). */
double orc_t1_wmsedec(int32_t nmsedec, uint32_t compno, uint32_t level, uint32_t orient, int32_t bpno,
                      uint32_t qmfbid, double stepsize, const double *mct_norms, uint32_t mct_numcomps) {
    double w1 = 1, w2, wmsedec;
    if (mct_norms && compno < mct_numcomps) w1 = mct_norms[compno];
    w2 = orc_getnorm(level, orient, qmfbid == 1);
    wmsedec = w1 * w2 * stepsize * (1 << bpno);
    wmsedec *= wmsedec * nmsedec / 8192.0;
    return wmsedec;
}

/* T1 encode of one code-block: T1Part1::preEncode (T1Part1.cpp:58-94) +
 * t1_encode_cblk (t1.cpp:1182-1326) for cblksty == 0.  nmsedec (optional):
 * the per-pass normalised distortion decrease sums of the rate-controlled
 * encode -- reset at each pass, incremented by t1_getnmsedec_sig when a
 * sample becomes significant (significance / cleanup, t1.cpp:217, :684) and
 * by t1_getnmsedec_ref for each refinement bit (:452). */
int orc_t1_encode_cblk_nmse(const int32_t *src, uint32_t stride, uint32_t w, uint32_t h,
                            uint32_t orient, int32_t qmfbid, int32_t inv_step,
                            uint8_t *out, uint32_t outcap, orc_pass *passes,
                            uint32_t *numbps_out, uint32_t *outlen, int32_t *nmsedec) {
    pthread_once(&nmse_once, nmse_init);
    const int fs = (int)w + 2;
    uint32_t *mag = (uint32_t *)malloc(sizeof(uint32_t) * w * h);
    uint8_t *flags = (uint8_t *)calloc((size_t)fs * (h + 2), 1);
    uint32_t maxv = 0;
    for (uint32_t y = 0; y < h; ++y) {
        for (uint32_t x = 0; x < w; ++x) {
            int32_t v = src[(size_t)y * stride + x];
            int32_t q = (qmfbid == 1) ? (int32_t)((uint32_t)v << 6) : fix_mul_t1(v, inv_step);
            uint32_t m = (uint32_t)(q < 0 ? -q : q);
            mag[y * w + x] = m;
            if (q < 0) flags[(y + 1) * fs + x + 1] |= F_NEG;
            if (m > maxv) maxv = m;
        }
    }
    uint32_t numbps = 0;
    if (maxv) {
        uint32_t t = floorlog2_u(maxv) + 1;
        numbps = t <= 6 ? 0 : t - 6;
    }
    *numbps_out = numbps;
    *outlen = 0;
    if (numbps == 0) { free(mag); free(flags); return 0; }
    (void)outcap;

    mq_enc e;
    mqe_init(&e, out);
    uint32_t passno = 0;
    int32_t bpno = (int32_t)numbps - 1;
    int passtype = 2;
    for (; bpno >= 0; ++passno) {
        const uint32_t one = 1u << (bpno + 6);
        int32_t nm = 0;
        if (passtype == 0) {
            /* significance propagation (t1.cpp:197-231, 287-338) */
            for (uint32_t k = 0; k < h; k += 4) {
                for (uint32_t x = 0; x < w; ++x) {
                    for (uint32_t y = k; y < k + 4 && y < h; ++y) {
                        uint8_t *p = &flags[(y + 1) * fs + x + 1];
                        if ((*p & (F_SIG | F_VISIT)) == 0 && any_nb_sig(p, fs)) {
                            uint32_t bit = (mag[y * w + x] & one) ? 1 : 0;
                            mqe_encode(&e, CX_ZC + zc_of(p, fs, orient), bit);
                            if (bit) {
                                int xr;
                                int cx = sc_of(p, fs, &xr);
                                nm += nmse_sig(mag[y * w + x], bpno);
                                mqe_encode(&e, cx, ((*p & F_NEG) ? 1u : 0u) ^ (uint32_t)xr);
                                *p |= F_SIG;
                            }
                            *p |= F_VISIT;
                        }
                    }
                }
            }
        } else if (passtype == 1) {
            /* magnitude refinement (t1.cpp:443-463, 498-555) */
            for (uint32_t k = 0; k < h; k += 4) {
                for (uint32_t x = 0; x < w; ++x) {
                    for (uint32_t y = k; y < k + 4 && y < h; ++y) {
                        uint8_t *p = &flags[(y + 1) * fs + x + 1];
                        if ((*p & (F_SIG | F_VISIT)) == F_SIG) {
                            nm += nmse_ref(mag[y * w + x], bpno);
                            mqe_encode(&e, mag_ctx(p, fs), (mag[y * w + x] & one) ? 1 : 0);
                            *p |= F_REF;
                        }
                    }
                }
            }
        } else {
            /* cleanup with run-length mode (t1.cpp:639-699, 739-782) */
            for (uint32_t k = 0; k < h; k += 4) {
                for (uint32_t x = 0; x < w; ++x) {
                    uint32_t y0 = k, runlen = 0;
                    int partial = 0;
                    if (k + 4 <= h) {
                        /* RL mode iff no significance in the 3x6 window and no
                         * sample of the column visited (flags word == 0). */
                        int agg = 1;
                        for (int yy = (int)k - 1; yy <= (int)k + 4 && agg; ++yy) {
                            const uint8_t *r = &flags[(yy + 1) * fs + x + 1];
                            if ((r[-1] | r[0] | r[1]) & F_SIG) agg = 0;
                        }
                        for (uint32_t yy = k; yy < k + 4 && agg; ++yy)
                            if (flags[(yy + 1) * fs + x + 1] & F_VISIT) agg = 0;
                        if (agg) {
                            for (runlen = 0; runlen < 4; ++runlen)
                                if (mag[(k + runlen) * w + x] & one) break;
                            mqe_encode(&e, CX_AGG, runlen != 4);
                            if (runlen == 4) continue;
                            mqe_encode(&e, CX_UNI, runlen >> 1);
                            mqe_encode(&e, CX_UNI, runlen & 1);
                            y0 = k + runlen;
                            partial = 1;
                        }
                    }
                    for (uint32_t y = y0; y < k + 4 && y < h; ++y) {
                        uint8_t *p = &flags[(y + 1) * fs + x + 1];
                        if (partial && y == y0) {
                            int xr;
                            int cx = sc_of(p, fs, &xr);
                            nm += nmse_sig(mag[y * w + x], bpno);
                            mqe_encode(&e, cx, ((*p & F_NEG) ? 1u : 0u) ^ (uint32_t)xr);
                            *p |= F_SIG;
                        } else if ((*p & (F_SIG | F_VISIT)) == 0) {
                            uint32_t bit = (mag[y * w + x] & one) ? 1 : 0;
                            mqe_encode(&e, CX_ZC + zc_of(p, fs, orient), bit);
                            if (bit) {
                                int xr;
                                int cx = sc_of(p, fs, &xr);
                                nm += nmse_sig(mag[y * w + x], bpno);
                                mqe_encode(&e, cx, ((*p & F_NEG) ? 1u : 0u) ^ (uint32_t)xr);
                                *p |= F_SIG;
                            }
                        }
                        *p &= (uint8_t)~F_VISIT;
                    }
                }
            }
        }
        orc_pass *ps = &passes[passno];
        if (nmsedec) nmsedec[passno] = nm;
        if (passtype == 2 && bpno == 0) {
            /* t1_enc_is_term_pass: last cleanup pass (t1.cpp:1131-1151) */
            mqe_flush(&e);
            ps->term = 1;
            ps->rate = mqe_numbytes(&e);
        } else {
            /* rate_extra_bytes = 4 + 1 (+1 if ct < 5) (t1.cpp:1278-1288) */
            uint32_t extra = 5 + (e.ct < 5 ? 1 : 0);
            ps->term = 0;
            ps->rate = mqe_numbytes(&e) + extra;
        }
        if (++passtype == 3) { passtype = 0; bpno--; }
    }
    uint32_t total = passno;
    /* make pass rates non-increasing from the end (t1.cpp:1303-1313) */
    uint32_t last = mqe_numbytes(&e);
    for (uint32_t i = total; i > 0;) {
        orc_pass *ps = &passes[--i];
        if (ps->rate > last) ps->rate = last; else last = ps->rate;
    }
    /* never end a pass on 0xFF (t1.cpp:1315-1324) */
    for (uint32_t i = 0; i < total; ++i) {
        orc_pass *ps = &passes[i];
        if (ps->rate > 0 && out[ps->rate - 1] == 0xFF) ps->rate--;
        ps->len = ps->rate - (i == 0 ? 0 : passes[i - 1].rate);
    }
    *outlen = mqe_numbytes(&e);
    free(mag); free(flags);
    return (int)total;
}

int orc_t1_encode_cblk(const int32_t *src, uint32_t stride, uint32_t w, uint32_t h,
                       uint32_t orient, int32_t qmfbid, int32_t inv_step,
                       uint8_t *out, uint32_t outcap, orc_pass *passes,
                       uint32_t *numbps_out, uint32_t *outlen) {
    return orc_t1_encode_cblk_nmse(src, stride, w, h, orient, qmfbid, inv_step, out, outcap, passes, numbps_out,
                                   outlen, NULL);
}

/* T1 decode of a single-segment code-block (t1.cpp:1038-1130, passes
 * :426/:631/:895).  dst receives Grok's t1->data (one extra LSB). */
int orc_t1_decode_cblk(uint8_t *data, uint32_t len, uint32_t numpasses, uint32_t numbps,
                       uint32_t w, uint32_t h, uint32_t orient, int32_t *dst) {
    const int fs = (int)w + 2;
    uint8_t *flags = (uint8_t *)calloc((size_t)fs * (h + 2), 1);
    memset(dst, 0, sizeof(int32_t) * w * h);
    uint8_t save0 = data[len], save1 = data[len + 1];
    data[len] = 0xff; data[len + 1] = 0xff;
    mq_dec d;
    mqd_init(&d, data, len);
    int32_t bpno_plus_one = (int32_t)numbps;
    int passtype = 2;
    for (uint32_t passno = 0; passno < numpasses && bpno_plus_one >= 1; ++passno) {
        const int32_t one = 1 << bpno_plus_one;
        const int32_t half = one >> 1;
        const int32_t oneplushalf = one | half;
        if (passtype == 0) {
            for (uint32_t k = 0; k < h; k += 4)
                for (uint32_t x = 0; x < w; ++x)
                    for (uint32_t y = k; y < k + 4 && y < h; ++y) {
                        uint8_t *p = &flags[(y + 1) * fs + x + 1];
                        if ((*p & (F_SIG | F_VISIT)) == 0 && any_nb_sig(p, fs)) {
                            if (mqd_decode(&d, CX_ZC + zc_of(p, fs, orient))) {
                                int xr;
                                int cx = sc_of(p, fs, &xr);
                                uint32_t s = mqd_decode(&d, cx) ^ (uint32_t)xr;
                                dst[y * w + x] = s ? -oneplushalf : oneplushalf;
                                *p |= F_SIG | (s ? F_NEG : 0);
                            }
                            *p |= F_VISIT;
                        }
                    }
        } else if (passtype == 1) {
            for (uint32_t k = 0; k < h; k += 4)
                for (uint32_t x = 0; x < w; ++x)
                    for (uint32_t y = k; y < k + 4 && y < h; ++y) {
                        uint8_t *p = &flags[(y + 1) * fs + x + 1];
                        if ((*p & (F_SIG | F_VISIT)) == F_SIG) {
                            uint32_t v = mqd_decode(&d, mag_ctx(p, fs));
                            int32_t *dp = &dst[y * w + x];
                            *dp += (v ^ (uint32_t)(*dp < 0)) ? half : -half;
                            *p |= F_REF;
                        }
                    }
        } else {
            for (uint32_t k = 0; k < h; k += 4)
                for (uint32_t x = 0; x < w; ++x) {
                    uint32_t y0 = k;
                    int partial = 0;
                    if (k + 4 <= h) {
                        int agg = 1;
                        for (int yy = (int)k - 1; yy <= (int)k + 4 && agg; ++yy) {
                            const uint8_t *r = &flags[(yy + 1) * fs + x + 1];
                            if ((r[-1] | r[0] | r[1]) & F_SIG) agg = 0;
                        }
                        for (uint32_t yy = k; yy < k + 4 && agg; ++yy)
                            if (flags[(yy + 1) * fs + x + 1] & F_VISIT) agg = 0;
                        if (agg) {
                            if (!mqd_decode(&d, CX_AGG)) continue;
                            uint32_t r = mqd_decode(&d, CX_UNI);
                            r = (r << 1) | mqd_decode(&d, CX_UNI);
                            y0 = k + r;
                            partial = 1;
                        }
                    }
                    for (uint32_t y = y0; y < k + 4 && y < h; ++y) {
                        uint8_t *p = &flags[(y + 1) * fs + x + 1];
                        int code_sign = 0;
                        if (partial && y == y0) code_sign = 1;
                        else if ((*p & (F_SIG | F_VISIT)) == 0)
                            code_sign = (int)mqd_decode(&d, CX_ZC + zc_of(p, fs, orient));
                        if (code_sign) {
                            int xr;
                            int cx = sc_of(p, fs, &xr);
                            uint32_t s = mqd_decode(&d, cx) ^ (uint32_t)xr;
                            dst[y * w + x] = s ? -oneplushalf : oneplushalf;
                            *p |= F_SIG | (s ? F_NEG : 0);
                        }
                        *p &= (uint8_t)~F_VISIT;
                    }
                }
        }
        if (++passtype == 3) { passtype = 0; bpno_plus_one--; }
    }
    data[len] = save0; data[len + 1] = save1;
    free(flags);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* DWT                                                                       */
/* ------------------------------------------------------------------------- */

/* int_fix_mul (util/grok_intmath.h:209-222): a * b (13-bit fixed) rounded */
static inline int32_t fix_mul(int32_t a, int32_t b) {
    int64_t t = (int64_t)a * (int64_t)b + 4096;
    return (int32_t)(t >> 13);
}

#define S_(i) a[(i) << 1]
#define D_(i) a[1 + ((i) << 1)]
#define SC(i) ((i) < 0 ? S_(0) : ((i) >= sn ? S_(sn - 1) : S_(i)))
#define DC(i) ((i) < 0 ? D_(0) : ((i) >= dn ? D_(dn - 1) : D_(i)))
#define SSC(i) ((i) < 0 ? S_(0) : ((i) >= dn ? S_(dn - 1) : S_(i)))
#define DDC(i) ((i) < 0 ? D_(0) : ((i) >= sn ? D_(sn - 1) : D_(i)))

/* forward 5/3 lifting on an interleaved line (transform/dwt53.cpp:150-169) */
static void fwd53_line(int32_t *a, int32_t dn, int32_t sn, int cas) {
    if (!cas) {
        if (dn > 0 || sn > 1) {
            for (int32_t i = 0; i < dn; i++) D_(i) -= (SC(i) + SC(i + 1)) >> 1;
            for (int32_t i = 0; i < sn; i++) S_(i) += (DC(i - 1) + DC(i) + 2) >> 2;
        }
    } else {
        if (!sn && dn == 1) S_(0) <<= 1;
        else {
            for (int32_t i = 0; i < dn; i++) S_(i) -= (DDC(i) + DDC(i - 1)) >> 1;
            for (int32_t i = 0; i < sn; i++) D_(i) += (SSC(i) + SSC(i + 1) + 2) >> 2;
        }
    }
}

/* forward 9/7 fixed-point lifting (transform/dwt97.cpp:90-123) */
static void fwd97_line(int32_t *a, int32_t dn, int32_t sn, int cas) {
    if (!cas) {
        if (dn > 0 || sn > 1) {
            for (int32_t i = 0; i < dn; i++) D_(i) -= fix_mul(SC(i) + SC(i + 1), 12994);
            for (int32_t i = 0; i < sn; i++) S_(i) -= fix_mul(DC(i - 1) + DC(i), 434);
            for (int32_t i = 0; i < dn; i++) D_(i) += fix_mul(SC(i) + SC(i + 1), 7233);
            for (int32_t i = 0; i < sn; i++) S_(i) += fix_mul(DC(i - 1) + DC(i), 3633);
            for (int32_t i = 0; i < dn; i++) D_(i) = fix_mul(D_(i), 5039);
            for (int32_t i = 0; i < sn; i++) S_(i) = fix_mul(S_(i), 6659);
        }
    } else {
        if (sn > 0 || dn > 1) {
            for (int32_t i = 0; i < dn; i++) S_(i) -= fix_mul(DDC(i) + DDC(i - 1), 12994);
            for (int32_t i = 0; i < sn; i++) D_(i) -= fix_mul(SSC(i) + SSC(i + 1), 434);
            for (int32_t i = 0; i < dn; i++) S_(i) += fix_mul(DDC(i) + DDC(i - 1), 7233);
            for (int32_t i = 0; i < sn; i++) D_(i) += fix_mul(SSC(i) + SSC(i + 1), 3633);
            for (int32_t i = 0; i < dn; i++) S_(i) = fix_mul(S_(i), 5039);
            for (int32_t i = 0; i < sn; i++) D_(i) = fix_mul(D_(i), 6659);
        }
    }
}

/* inverse 5/3 on an interleaved line; exact inverse of fwd53_line (the
 * reference's decode_h_cas0/1_53, transform/dwt.cpp:256-363, computes the
 * same integers). */
static void inv53_line(int32_t *a, int32_t dn, int32_t sn, int cas) {
    if (!cas) {
        if (dn > 0 || sn > 1) {
            for (int32_t i = 0; i < sn; i++) S_(i) -= (DC(i - 1) + DC(i) + 2) >> 2;
            for (int32_t i = 0; i < dn; i++) D_(i) += (SC(i) + SC(i + 1)) >> 1;
        }
    } else {
        if (!sn && dn == 1) S_(0) /= 2;
        else {
            for (int32_t i = 0; i < sn; i++) D_(i) -= (SSC(i) + SSC(i + 1) + 2) >> 2;
            for (int32_t i = 0; i < dn; i++) S_(i) += (DDC(i) + DDC(i - 1)) >> 1;
        }
    }
}
#undef S_
#undef D_
#undef SC
#undef DC
#undef SSC
#undef DDC

/* inverse 9/7 in float (transform/dwt.cpp:1477-1537 decode_step_97 with
 * decode_step1/2_97 :1392-1475): separate mul and add, no FMA. */
static const float K97 = 1.230174105f, C13318 = 1.625732422f;
static const float DLT = -0.443506852f, GAM = -0.882911075f, BET = 0.052980118f, ALP = 1.586134342f;

static void inv97_step2(float *w, int32_t first, int32_t other, int32_t end, int32_t m, float c) {
    /* targets w[first + 2i], i < end; left neighbour w[first+2i-1] (w[other]
     * at i==0), right neighbour w[first+2i+1]; for i == m (< end) only
     * the left neighbour, with weight 2c. */
    int32_t imax = end < m ? end : m;
    for (int32_t i = 0; i < imax; ++i) {
        float l = (i == 0) ? w[other] : w[first + 2 * i - 1];
        float r = w[first + 2 * i + 1];
        volatile float s = l + r;
        volatile float p = s * c;
        w[first + 2 * i] = w[first + 2 * i] + p;
    }
    if (m < end) {
        float l = (m == 0) ? w[other] : w[first + 2 * m - 1];
        float c2 = c + c;
        volatile float p = l * c2;
        w[first + 2 * m] = w[first + 2 * m] + p;
    }
}

static void inv97_line(float *w, int32_t dn, int32_t sn, int cas) {
    int32_t a, b;
    if (cas == 0) { if (!(dn > 0 || sn > 1)) return; a = 0; b = 1; }
    else { if (!(sn > 0 || dn > 1)) return; a = 1; b = 0; }
    for (int32_t i = 0; i < sn; ++i) w[a + 2 * i] = w[a + 2 * i] * K97;
    for (int32_t i = 0; i < dn; ++i) w[b + 2 * i] = w[b + 2 * i] * C13318;
    int32_t mL = sn < dn - a ? sn : dn - a;
    int32_t mH = dn < sn - b ? dn : sn - b;
    inv97_step2(w, a, b, sn, mL, DLT);
    inv97_step2(w, b, a, dn, mH, GAM);
    inv97_step2(w, a, b, sn, mL, BET);
    inv97_step2(w, b, a, dn, mH, ALP);
}

typedef struct { uint32_t x0, y0, x1, y1; } rect_t;

static void res_rect(rect_t *r, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t numres, uint32_t resno) {
    uint32_t lev = numres - 1 - resno;
    r->x0 = ceildivpow2(x0, lev); r->y0 = ceildivpow2(y0, lev);
    r->x1 = ceildivpow2(x1, lev); r->y1 = ceildivpow2(y1, lev);
}

typedef struct {
    int32_t *buf; uint32_t stride;
    uint32_t rw, rh, sn, dn; int cas; int irrev; int inverse;
    uint32_t maxlen;
} dwt_pass_ctx;

static void dwt_col_job(void *vc, uint64_t m) {
    dwt_pass_ctx *c = (dwt_pass_ctx *)vc;
    int32_t *bj = (int32_t *)malloc(sizeof(int32_t) * (c->maxlen + 2));
    int32_t *aj = c->buf + m;
    if (!c->inverse) {
        for (uint32_t k = 0; k < c->rh; ++k) bj[k] = aj[(size_t)k * c->stride];
        if (c->irrev) fwd97_line(bj, (int32_t)c->dn, (int32_t)c->sn, c->cas);
        else fwd53_line(bj, (int32_t)c->dn, (int32_t)c->sn, c->cas);
        /* deinterleave_v (transform/dwt_utils.cpp:84-106) */
        for (uint32_t i = 0; i < c->sn; ++i) aj[(size_t)i * c->stride] = bj[c->cas + 2 * i];
        for (uint32_t i = 0; i < c->dn; ++i) aj[(size_t)(c->sn + i) * c->stride] = bj[1 - c->cas + 2 * i];
    } else {
        for (uint32_t i = 0; i < c->sn; ++i) bj[c->cas + 2 * i] = aj[(size_t)i * c->stride];
        for (uint32_t i = 0; i < c->dn; ++i) bj[1 - c->cas + 2 * i] = aj[(size_t)(c->sn + i) * c->stride];
        if (c->irrev) inv97_line((float *)bj, (int32_t)c->dn, (int32_t)c->sn, c->cas);
        else inv53_line(bj, (int32_t)c->dn, (int32_t)c->sn, c->cas);
        for (uint32_t k = 0; k < c->rh; ++k) aj[(size_t)k * c->stride] = bj[k];
    }
    free(bj);
}

static void dwt_row_job(void *vc, uint64_t m) {
    dwt_pass_ctx *c = (dwt_pass_ctx *)vc;
    int32_t *bj = (int32_t *)malloc(sizeof(int32_t) * (c->maxlen + 2));
    int32_t *aj = c->buf + m * c->stride;
    if (!c->inverse) {
        memcpy(bj, aj, sizeof(int32_t) * c->rw);
        if (c->irrev) fwd97_line(bj, (int32_t)c->dn, (int32_t)c->sn, c->cas);
        else fwd53_line(bj, (int32_t)c->dn, (int32_t)c->sn, c->cas);
        /* deinterleave_h (transform/dwt_utils.cpp:108-125) */
        for (uint32_t i = 0; i < c->sn; ++i) aj[i] = bj[c->cas + 2 * i];
        for (uint32_t i = 0; i < c->dn; ++i) aj[c->sn + i] = bj[1 - c->cas + 2 * i];
    } else {
        for (uint32_t i = 0; i < c->sn; ++i) bj[c->cas + 2 * i] = aj[i];
        for (uint32_t i = 0; i < c->dn; ++i) bj[1 - c->cas + 2 * i] = aj[c->sn + i];
        if (c->irrev) inv97_line((float *)bj, (int32_t)c->dn, (int32_t)c->sn, c->cas);
        else inv53_line(bj, (int32_t)c->dn, (int32_t)c->sn, c->cas);
        memcpy(aj, bj, sizeof(int32_t) * c->rw);
    }
    free(bj);
}

/* WaveletForward<DWT>::run (transform/WaveletForward.h:40-160): per level,
 * vertical lifting + deinterleave, then horizontal. */
int orc_dwt_fwd(int32_t *buf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                uint32_t numres, int32_t irreversible, int32_t nthreads) {
    uint32_t stride = x1 - x0;
    for (uint32_t lvl = 0; lvl + 1 < numres; ++lvl) {
        rect_t cur, nxt;
        res_rect(&cur, x0, y0, x1, y1, numres, numres - 1 - lvl);
        res_rect(&nxt, x0, y0, x1, y1, numres, numres - 2 - lvl);
        dwt_pass_ctx c;
        c.buf = buf; c.stride = stride; c.irrev = irreversible; c.inverse = 0;
        c.rw = cur.x1 - cur.x0; c.rh = cur.y1 - cur.y0;
        c.maxlen = umax(c.rw, c.rh);
        if (c.rw) {
            c.sn = nxt.y1 - nxt.y0; c.dn = c.rh - c.sn; c.cas = (int)(cur.y0 & 1);
            parallel_for(c.rw, nthreads, dwt_col_job, &c);
        }
        if (c.rh) {
            c.sn = nxt.x1 - nxt.x0; c.dn = c.rw - c.sn; c.cas = (int)(cur.x0 & 1);
            parallel_for(c.rh, nthreads, dwt_row_job, &c);
        }
    }
    return 0;
}

/* decode_tile_53 / decode_tile_97 (transform/dwt.cpp:724, :1544): per level
 * from the lowest resolution up, horizontal then vertical. */
/* Inverse levels for resolutions 1 .. numres_dec-1 only (reduced-resolution
 * decode: Wavelet::decode(tilec, resno_decoded + 1), TileProcessor.cpp:1165,
 * with minimum_num_resolutions = numres - reduce, TileComponent.cpp:199-204).
 * The resolution geometry is the full tile's; the buffer keeps its stride. */
static int dwt_inv_levels(int32_t *buf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t numres,
                          uint32_t numres_dec, int32_t irreversible, int32_t nthreads);

int orc_dwt_inv(int32_t *buf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1,
                uint32_t numres, int32_t irreversible, int32_t nthreads) {
    return dwt_inv_levels(buf, x0, y0, x1, y1, numres, numres, irreversible, nthreads);
}

static int dwt_inv_levels(int32_t *buf, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t numres,
                          uint32_t numres_dec, int32_t irreversible, int32_t nthreads) {
    uint32_t stride = x1 - x0;
    for (uint32_t r = 1; r < numres_dec; ++r) {
        rect_t lo, cur;
        res_rect(&lo, x0, y0, x1, y1, numres, r - 1);
        res_rect(&cur, x0, y0, x1, y1, numres, r);
        dwt_pass_ctx c;
        c.buf = buf; c.stride = stride; c.irrev = irreversible; c.inverse = 1;
        c.rw = cur.x1 - cur.x0; c.rh = cur.y1 - cur.y0;
        c.maxlen = umax(c.rw, c.rh);
        c.sn = lo.x1 - lo.x0; c.dn = c.rw - c.sn; c.cas = (int)(cur.x0 & 1);
        if (c.rw) parallel_for(c.rh, nthreads, dwt_row_job, &c);
        c.sn = lo.y1 - lo.y0; c.dn = c.rh - c.sn; c.cas = (int)(cur.y0 & 1);
        if (c.rh) parallel_for(c.rw, nthreads, dwt_col_job, &c);
    }
    return 0;
}

/* ------------------------------------------------------------------------- */
/* DC level shift + multi-component transform                                */
/* ------------------------------------------------------------------------- */

/* dc_level_shift_encode (TileProcessor.cpp:1449-1471) + mct::encode_rev
 * (mct/mct.cpp:85-139) / mct::encode_irrev (mct.cpp:195-350) */
void orc_dcshift_mct_fwd(int32_t *c0, int32_t *c1, int32_t *c2, uint32_t numcomps,
                         uint64_t n, const int32_t *shift, int32_t mct, int32_t irreversible) {
    int32_t *cs[3] = {c0, c1, c2};
    for (uint32_t k = 0; k < numcomps && k < 3; ++k) {
        int32_t *p = cs[k];
        if (!p) continue;
        for (uint64_t i = 0; i < n; ++i)
            p[i] = irreversible ? (int32_t)((uint32_t)(p[i] - shift[k]) << 11) : p[i] - shift[k];
    }
    if (!mct || numcomps < 3) return;
    for (uint64_t i = 0; i < n; ++i) {
        int32_t r = c0[i], g = c1[i], b = c2[i];
        if (!irreversible) {
            c0[i] = (r + (g * 2) + b) >> 2;
            c1[i] = b - g;
            c2[i] = r - g;
        } else {
            c0[i] = fix_mul(r, 2449) + fix_mul(g, 4809) + fix_mul(b, 934);
            c1[i] = -fix_mul(r, 1382) - fix_mul(g, 2714) + fix_mul(b, 4096);
            c2[i] = fix_mul(r, 4096) - fix_mul(g, 3430) - fix_mul(b, 666);
        }
    }
}

/* ------------------------------------------------------------------------- */
/* quantisation parameters (codestream/HTParams.cpp:164-260, Quantizer.cpp)  */
/* ------------------------------------------------------------------------- */
static const float BIBO_53_L[34] = {1.0000e+00f, 1.5000e+00f, 1.6250e+00f, 1.6875e+00f, 1.6963e+00f, 1.7067e+00f,
    1.7116e+00f, 1.7129e+00f, 1.7141e+00f, 1.7145e+00f, 1.7151e+00f, 1.7152e+00f, 1.7155e+00f, 1.7155e+00f,
    1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f,
    1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f,
    1.7156e+00f, 1.7156e+00f, 1.7156e+00f, 1.7156e+00f};
static const float BIBO_53_H[34] = {2.0000e+00f, 2.5000e+00f, 2.7500e+00f, 2.8047e+00f, 2.8198e+00f, 2.8410e+00f,
    2.8558e+00f, 2.8601e+00f, 2.8628e+00f, 2.8656e+00f, 2.8662e+00f, 2.8667e+00f, 2.8669e+00f, 2.8670e+00f,
    2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f,
    2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f,
    2.8671e+00f, 2.8671e+00f, 2.8671e+00f, 2.8671e+00f};
typedef struct { uint32_t expn, mant; } stepsize_t;

/* param_qcd::set_rev_quant (HTParams.cpp:187-207).  NB the RCT bit is never
 * added: j2k_setup_encoder calls generate() before tcp->mct is assigned
 * (codestream/j2k.cpp:1839 vs :1861). */
static void qcd_rev(stepsize_t *ss, uint32_t numdecomps, uint32_t prec) {
    int B = (int)prec;
    uint32_t s = 0;
    float bl = BIBO_53_L[numdecomps];
    int X = (int)ceil(log((double)(float)(bl * bl * 1.1f)) / M_LN2);
    ss[s].expn = (uint32_t)(B + X); ss[s++].mant = 0;
    for (int d = (int)numdecomps - 1; d >= 0; --d) {
        float l = BIBO_53_L[d + 1], hh = BIBO_53_H[d];
        X = (int)ceil(log((double)(float)(hh * l * 1.1f)) / M_LN2);
        ss[s].expn = (uint32_t)(B + X); ss[s++].mant = 0;
        ss[s].expn = (uint32_t)(B + X); ss[s++].mant = 0;
        X = (int)ceil(log((double)(float)(hh * hh * 1.1f)) / M_LN2);
        ss[s].expn = (uint32_t)(B + X); ss[s++].mant = 0;
    }
}

static void delta_to_step(float delta_b, stepsize_t *out) {
    uint32_t e = 0;
    while (delta_b < 1.0f) { e++; delta_b *= 2.0f; }
    uint32_t m = (uint32_t)roundf(delta_b * (float)(1 << 11)) - (1 << 11);
    out->expn = e; out->mant = m < (1 << 11) ? m : 0x7FF;
}

/* param_qcd::set_irrev_quant (HTParams.cpp:210-253) */
static void qcd_irrev(stepsize_t *ss, uint32_t numdecomps, uint32_t prec, int sgnd) {
    float base_delta = 1.0f / (float)(1 << (prec + (uint32_t)sgnd));
    uint32_t s = 0;
    float gl = SQE_97_L[numdecomps];
    delta_to_step(base_delta / (gl * gl), &ss[s++]);
    for (int d = (int)numdecomps - 1; d >= 0; --d) {
        float l = SQE_97_L[d + 1], hh = SQE_97_H[d];
        stepsize_t t;
        delta_to_step(base_delta / (l * hh), &t);
        ss[s++] = t; ss[s++] = t;
        delta_to_step(base_delta / (hh * hh), &ss[s++]);
    }
}

/* ------------------------------------------------------------------------- */
/* tile / resolution / band / precinct / code-block geometry                 */
/* (TileComponent.cpp:165-507)                                               */
/* ------------------------------------------------------------------------- */
typedef struct {
    rect_t r;                 /* in band coordinates */
    uint32_t bx, by;          /* offset into the Mallat tile buffer */
    /* encoder */
    uint8_t *data;            /* data[-1] is a zero pad byte */
    uint32_t numbps, numpasses, len;
    orc_pass passes[ORC_MAX_PASSES];
    /* T2 */
    uint32_t numlenbits, included;
    /* decoder */
    uint8_t *seg; uint32_t seglen, segcap, dec_passes;
} cblk_t;

typedef struct { int64_t value, low; int known; int parent; } tt_node;
typedef struct { uint32_t nh, nv, nnodes; tt_node *nodes; } tagtree;

typedef struct {
    rect_t r; uint32_t cw, ch;
    cblk_t *cblks;
    tagtree incl, imsb;
} precinct_t;

typedef struct {
    rect_t r; uint32_t bandno;
    float stepsize; uint32_t inv_step; uint32_t numbps;
    precinct_t *precs;
} band_t;

typedef struct {
    rect_t r; uint32_t pw, ph, numbands;
    band_t bands[3];
} resolution_t;

typedef struct {
    rect_t r; uint32_t numres;
    resolution_t res[33];
    int32_t *data;
} tilecomp_t;

static int band_empty(const band_t *b) { return b->r.x0 == b->r.x1 || b->r.y0 == b->r.y1; }

static void tt_init(tagtree *t, uint32_t nh, uint32_t nv) {
    /* TagTree::TagTree (codestream/TagTree.cpp:60-117): levels of halved size,
     * parent links in raster order */
    uint32_t nplh[40], nplv[40], numlvls = 0, n;
    nplh[0] = nh; nplv[0] = nv;
    t->nnodes = 0;
    do {
        n = nplh[numlvls] * nplv[numlvls];
        nplh[numlvls + 1] = (nplh[numlvls] + 1) / 2;
        nplv[numlvls + 1] = (nplv[numlvls] + 1) / 2;
        t->nnodes += n;
        ++numlvls;
    } while (n > 1);
    t->nh = nh; t->nv = nv;
    t->nodes = (tt_node *)calloc(t->nnodes ? t->nnodes : 1, sizeof(tt_node));
    uint32_t base = 0, pbase = nh * nv;
    for (uint32_t l = 0; l + 1 < numlvls; ++l) {
        for (uint32_t j = 0; j < nplv[l]; ++j)
            for (uint32_t i = 0; i < nplh[l]; ++i)
                t->nodes[base + j * nplh[l] + i].parent = (int)(pbase + (j >> 1) * nplh[l + 1] + (i >> 1));
        base = pbase;
        pbase += nplh[l + 1] * nplv[l + 1];
    }
    t->nodes[t->nnodes - 1].parent = -1;
    for (uint32_t i = 0; i < t->nnodes; ++i) { t->nodes[i].value = INT64_MAX; t->nodes[i].low = 0; t->nodes[i].known = 0; }
}
static void tt_reset(tagtree *t) {
    for (uint32_t i = 0; i < t->nnodes; ++i) { t->nodes[i].value = INT64_MAX; t->nodes[i].low = 0; t->nodes[i].known = 0; }
}
static void tt_setvalue(tagtree *t, uint32_t leaf, int64_t v) {
    int n = (int)leaf;
    while (n >= 0 && t->nodes[n].value > v) { t->nodes[n].value = v; n = t->nodes[n].parent; }
}

static int build_tilecomp(tilecomp_t *tc, rect_t tr, uint32_t numres, uint32_t cblkw, uint32_t cblkh,
                          const stepsize_t *ss, uint32_t prec, int irrev, int encoder) {
    memset(tc, 0, sizeof(*tc));
    tc->r = tr; tc->numres = numres;
    for (uint32_t resno = 0; resno < numres; ++resno) {
        resolution_t *res = &tc->res[resno];
        uint32_t lev = numres - 1 - resno;
        res_rect(&res->r, tr.x0, tr.y0, tr.x1, tr.y1, numres, resno);
        const uint32_t pdx = 15, pdy = 15; /* default precincts 2^15 */
        uint32_t tpx0 = floordivpow2(res->r.x0, pdx) << pdx, tpy0 = floordivpow2(res->r.y0, pdy) << pdy;
        uint32_t bpx1 = ceildivpow2(res->r.x1, pdx) << pdx, bpy1 = ceildivpow2(res->r.y1, pdy) << pdy;
        res->pw = (res->r.x0 == res->r.x1) ? 0 : ((bpx1 - tpx0) >> pdx);
        res->ph = (res->r.y0 == res->r.y1) ? 0 : ((bpy1 - tpy0) >> pdy);
        uint32_t tlcbgx, tlcbgy, cbgw, cbgh;
        if (resno == 0) { tlcbgx = tpx0; tlcbgy = tpy0; cbgw = pdx; cbgh = pdy; res->numbands = 1; }
        else { tlcbgx = ceildivpow2(tpx0, 1); tlcbgy = ceildivpow2(tpy0, 1); cbgw = pdx - 1; cbgh = pdy - 1; res->numbands = 3; }
        uint32_t cbw = umin(cblkw, cbgw), cbh = umin(cblkh, cbgh);
        for (uint32_t bandno = 0; bandno < res->numbands; ++bandno) {
            band_t *b = &res->bands[bandno];
            if (resno == 0) {
                b->bandno = 0;
                b->r.x0 = ceildivpow2(tr.x0, lev); b->r.y0 = ceildivpow2(tr.y0, lev);
                b->r.x1 = ceildivpow2(tr.x1, lev); b->r.y1 = ceildivpow2(tr.y1, lev);
            } else {
                b->bandno = bandno + 1;
                uint32_t x0b = b->bandno & 1, y0b = b->bandno >> 1;
                b->r.x0 = (uint32_t)(((uint64_t)tr.x0 - ((uint64_t)x0b << lev) + ((uint64_t)1 << (lev + 1)) - 1) >> (lev + 1));
                b->r.y0 = (uint32_t)(((uint64_t)tr.y0 - ((uint64_t)y0b << lev) + ((uint64_t)1 << (lev + 1)) - 1) >> (lev + 1));
                b->r.x1 = (uint32_t)(((uint64_t)tr.x1 - ((uint64_t)x0b << lev) + ((uint64_t)1 << (lev + 1)) - 1) >> (lev + 1));
                b->r.y1 = (uint32_t)(((uint64_t)tr.y1 - ((uint64_t)y0b << lev) + ((uint64_t)1 << (lev + 1)) - 1) >> (lev + 1));
            }
            /* Quantizer::setBandStepSizeAndBps (codestream/Quantizer.cpp:65-104) */
            uint32_t gain = irrev ? 0 : (b->bandno == 0 ? 0 : (b->bandno < 3 ? 1 : 2));
            uint32_t numbps = prec + gain;
            uint32_t off = resno == 0 ? 0 : 3 * resno - 2;
            const stepsize_t *st = &ss[off + bandno];
            b->stepsize = (float)((1.0 + st->mant / 2048.0) * pow(2.0, (int32_t)(numbps - st->expn))) * (encoder ? 1.0f : 0.5f);
            b->numbps = st->expn + 2 - 1;
            b->inv_step = (uint32_t)((8192.0 / b->stepsize) + 0.5f);
            uint32_t np = res->pw * res->ph;
            b->precs = (precinct_t *)calloc(np ? np : 1, sizeof(precinct_t));
            for (uint32_t precno = 0; precno < np; ++precno) {
                precinct_t *pr = &b->precs[precno];
                uint32_t cbgx0 = tlcbgx + (precno % res->pw) * (1u << cbgw);
                uint32_t cbgy0 = tlcbgy + (precno / res->pw) * (1u << cbgh);
                pr->r.x0 = umax(cbgx0, b->r.x0); pr->r.y0 = umax(cbgy0, b->r.y0);
                pr->r.x1 = umin(cbgx0 + (1u << cbgw), b->r.x1); pr->r.y1 = umin(cbgy0 + (1u << cbgh), b->r.y1);
                uint32_t tlx = floordivpow2(pr->r.x0, cbw) << cbw, tly = floordivpow2(pr->r.y0, cbh) << cbh;
                uint32_t brx = ceildivpow2(pr->r.x1, cbw) << cbw, bry = ceildivpow2(pr->r.y1, cbh) << cbh;
                pr->cw = (brx - tlx) >> cbw; pr->ch = (bry - tly) >> cbh;
                if (pr->r.x1 <= pr->r.x0 || pr->r.y1 <= pr->r.y0) { pr->cw = pr->ch = 0; }
                uint32_t nb = pr->cw * pr->ch;
                pr->cblks = (cblk_t *)calloc(nb ? nb : 1, sizeof(cblk_t));
                for (uint32_t cb = 0; cb < nb; ++cb) {
                    cblk_t *c = &pr->cblks[cb];
                    uint32_t cx0 = tlx + (cb % pr->cw) * (1u << cbw), cy0 = tly + (cb / pr->cw) * (1u << cbh);
                    c->r.x0 = umax(cx0, pr->r.x0); c->r.y0 = umax(cy0, pr->r.y0);
                    c->r.x1 = umin(cx0 + (1u << cbw), pr->r.x1); c->r.y1 = umin(cy0 + (1u << cbh), pr->r.y1);
                    /* Tier1::encodeCodeblocks offsets (t1/Tier1.cpp:49-62) */
                    c->bx = c->r.x0 - b->r.x0; c->by = c->r.y0 - b->r.y0;
                    if (b->bandno & 1) c->bx += tc->res[resno - 1].r.x1 - tc->res[resno - 1].r.x0;
                    if (b->bandno & 2) c->by += tc->res[resno - 1].r.y1 - tc->res[resno - 1].r.y0;
                }
                if (nb) { tt_init(&pr->incl, pr->cw, pr->ch); tt_init(&pr->imsb, pr->cw, pr->ch); }
            }
        }
    }
    return 0;
}

static void free_tilecomp(tilecomp_t *tc) {
    for (uint32_t resno = 0; resno < tc->numres; ++resno) {
        resolution_t *res = &tc->res[resno];
        for (uint32_t bandno = 0; bandno < res->numbands; ++bandno) {
            band_t *b = &res->bands[bandno];
            uint32_t np = res->pw * res->ph;
            for (uint32_t p = 0; p < np; ++p) {
                precinct_t *pr = &b->precs[p];
                for (uint32_t cb = 0; cb < pr->cw * pr->ch; ++cb) {
                    if (pr->cblks[cb].data) free(pr->cblks[cb].data - 1);
                    free(pr->cblks[cb].seg);
                }
                free(pr->cblks);
                if (pr->cw * pr->ch != 0) { free(pr->incl.nodes); free(pr->imsb.nodes); }
            }
            free(b->precs);
        }
    }
    free(tc->data);
}

uint32_t orc_count_cblks(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t numres,
                         uint32_t cblkw, uint32_t cblkh) {
    stepsize_t ss[100];
    memset(ss, 0, sizeof(ss));
    for (int i = 0; i < 100; ++i) ss[i].expn = 8;
    tilecomp_t tc;
    rect_t r = {x0, y0, x1, y1};
    build_tilecomp(&tc, r, numres, cblkw, cblkh, ss, 8, 0, 1);
    uint32_t n = 0;
    for (uint32_t resno = 0; resno < numres; ++resno)
        for (uint32_t b = 0; b < tc.res[resno].numbands; ++b)
            for (uint32_t p = 0; p < tc.res[resno].pw * tc.res[resno].ph; ++p)
                n += tc.res[resno].bands[b].precs[p].cw * tc.res[resno].bands[b].precs[p].ch;
    free_tilecomp(&tc);
    return n;
}

/* ------------------------------------------------------------------------- */
/* byte buffers + packet-header bit I/O (codestream/BitIO.cpp)               */
/* ------------------------------------------------------------------------- */
typedef struct { uint8_t *p; size_t n, cap; } bytes_t;
static void bb_reserve(bytes_t *b, size_t extra) {
    if (b->n + extra > b->cap) {
        size_t nc = b->cap ? b->cap * 2 : 4096;
        while (nc < b->n + extra) nc *= 2;
        b->p = (uint8_t *)realloc(b->p, nc); b->cap = nc;
    }
}
static void bb_put8(bytes_t *b, uint32_t v) { bb_reserve(b, 1); b->p[b->n++] = (uint8_t)v; }
static void bb_put16(bytes_t *b, uint32_t v) { bb_put8(b, v >> 8); bb_put8(b, v); }
static void bb_put32(bytes_t *b, uint32_t v) { bb_put16(b, v >> 16); bb_put16(b, v); }
static void bb_putn(bytes_t *b, const uint8_t *s, size_t n) { bb_reserve(b, n); memcpy(b->p + b->n, s, n); b->n += n; }
static void bb_set32(bytes_t *b, size_t at, uint32_t v) {
    b->p[at] = (uint8_t)(v >> 24); b->p[at + 1] = (uint8_t)(v >> 16); b->p[at + 2] = (uint8_t)(v >> 8); b->p[at + 3] = (uint8_t)v;
}

typedef struct { bytes_t *out; uint32_t buf, ct; } bio_w;
static void bw_byteout(bio_w *w) { bb_put8(w->out, w->buf); w->ct = (w->buf == 0xff) ? 7 : 8; w->buf = 0; }
static void bw_putbit(bio_w *w, uint32_t b) { if (w->ct == 0) bw_byteout(w); w->ct--; w->buf |= (b & 1) << w->ct; }
static void bw_write(bio_w *w, uint32_t v, uint32_t n) { for (int i = (int)n - 1; i >= 0; --i) bw_putbit(w, (v >> i) & 1); }
static void bw_flush(bio_w *w) { bw_byteout(w); if (w->ct == 7) bw_byteout(w); }
static void bw_numpasses(bio_w *w, uint32_t n) {
    if (n == 1) bw_write(w, 0, 1);
    else if (n == 2) bw_write(w, 2, 2);
    else if (n <= 5) bw_write(w, 0xc | (n - 3), 4);
    else if (n <= 36) bw_write(w, 0x1e0 | (n - 6), 9);
    else bw_write(w, 0xff80 | (n - 37), 16);
}
static void bw_comma(bio_w *w, int32_t n) { while (--n >= 0) bw_write(w, 1, 1); bw_write(w, 0, 1); }

/* TagTree::encode (codestream/TagTree.cpp:251-287) */
static void tt_encode(tagtree *t, bio_w *w, uint32_t leaf, int64_t threshold) {
    int stk[64], sp = 0;
    int node = (int)leaf;
    while (t->nodes[node].parent >= 0) { stk[sp++] = node; node = t->nodes[node].parent; }
    int64_t low = 0;
    for (;;) {
        tt_node *n = &t->nodes[node];
        if (low > n->low) n->low = low; else low = n->low;
        while (low < threshold) {
            if (low >= n->value) {
                if (!n->known) { bw_write(w, 1, 1); n->known = 1; }
                break;
            }
            bw_write(w, 0, 1);
            ++low;
        }
        n->low = low;
        if (sp == 0) break;
        node = stk[--sp];
    }
}

typedef struct { const uint8_t *p; size_t n, off; uint32_t buf, ct; int err; } bio_r;
static void br_bytein(bio_r *r) {
    r->ct = (r->buf == 0xff) ? 7 : 8;
    if (r->off >= r->n) { r->err = 1; r->buf = 0; return; }
    r->buf = r->p[r->off++];
}
static uint32_t br_bit(bio_r *r) { if (r->ct == 0) br_bytein(r); r->ct--; return (r->buf >> r->ct) & 1; }
static uint32_t br_read(bio_r *r, uint32_t n) { uint32_t v = 0; for (uint32_t i = 0; i < n; ++i) v = (v << 1) | br_bit(r); return v; }
static void br_align(bio_r *r) { if (r->buf == 0xff) br_bytein(r); r->ct = 0; }
static uint32_t br_numpasses(bio_r *r) {
    if (!br_read(r, 1)) return 1;
    if (!br_read(r, 1)) return 2;
    uint32_t n = br_read(r, 2);
    if (n != 3) return n + 3;
    n = br_read(r, 5);
    if (n != 31) return n + 6;
    return br_read(r, 7) + 37;
}
static uint32_t br_comma(bio_r *r) { uint32_t n = 0; while (br_bit(r)) { ++n; if (r->err) break; } return n; }

/* TagTree::decodeValue (codestream/TagTree.cpp:295-321) */
static int64_t tt_decode(tagtree *t, bio_r *r, uint32_t leaf, int64_t threshold) {
    int stk[64], sp = 0;
    int node = (int)leaf;
    while (t->nodes[node].parent >= 0) { stk[sp++] = node; node = t->nodes[node].parent; }
    int64_t low = 0;
    for (;;) {
        tt_node *n = &t->nodes[node];
        if (low > n->low) n->low = low; else low = n->low;
        while (low < threshold && low < n->value) {
            if (br_bit(r)) n->value = low; else ++low;
            if (r->err) return INT64_MAX;
        }
        n->low = low;
        if (sp == 0) break;
        node = stk[--sp];
    }
    return t->nodes[node].value;
}

/* ------------------------------------------------------------------------- */
/* Tier-2 (t2/T2.cpp:859-1110 encode_packet, :288-725 decode)                */
/* ------------------------------------------------------------------------- */

/* one layer, all passes (TileProcessor::makelayer_final :783-849) */
static void t2_encode_packet(tilecomp_t *tc, uint32_t resno, uint32_t precno, bytes_t *out) {
    resolution_t *res = &tc->res[resno];
    const uint32_t layno = 0;
    for (uint32_t bandno = 0; bandno < res->numbands; ++bandno) {
        band_t *b = &res->bands[bandno];
        precinct_t *pr = &b->precs[precno];
        uint32_t nb = pr->cw * pr->ch;
        if (band_empty(b) || !nb) continue;
        tt_reset(&pr->incl); tt_reset(&pr->imsb);
        for (uint32_t cb = 0; cb < nb; ++cb) {
            pr->cblks[cb].included = 0;
            tt_setvalue(&pr->imsb, cb, (int64_t)b->numbps - (int64_t)pr->cblks[cb].numbps);
        }
    }
    bio_w w = {out, 0, 8};
    bw_write(&w, 1, 1); /* Grok always signals a non-empty packet (T2.cpp:924-927) */
    for (uint32_t bandno = 0; bandno < res->numbands; ++bandno) {
        band_t *b = &res->bands[bandno];
        precinct_t *pr = &b->precs[precno];
        uint32_t nb = pr->cw * pr->ch;
        if (band_empty(b) || !nb) continue;
        for (uint32_t cb = 0; cb < nb; ++cb)
            if (!pr->cblks[cb].included && pr->cblks[cb].numpasses) tt_setvalue(&pr->incl, cb, layno);
        for (uint32_t cb = 0; cb < nb; ++cb) {
            cblk_t *c = &pr->cblks[cb];
            uint32_t np = c->numpasses;
            if (!c->included) tt_encode(&pr->incl, &w, cb, layno + 1);
            else bw_write(&w, np != 0, 1);
            if (!np) continue;
            if (!c->included) { c->numlenbits = 3; tt_encode(&pr->imsb, &w, cb, INT64_MAX); }
            bw_numpasses(&w, np);
            int32_t increment = 0; uint32_t len = 0, nump = 0;
            for (uint32_t p = 0; p < np; ++p) {
                ++nump; len += c->passes[p].len;
                if (c->passes[p].term || p == np - 1) {
                    int32_t t = floorlog2_i((int32_t)len) + 1 - ((int32_t)c->numlenbits + floorlog2_i((int32_t)nump));
                    if (t > increment) increment = t;
                    len = 0; nump = 0;
                }
            }
            bw_comma(&w, increment);
            c->numlenbits += (uint32_t)increment;
            for (uint32_t p = 0; p < np; ++p) {
                ++nump; len += c->passes[p].len;
                if (c->passes[p].term || p == np - 1) {
                    bw_write(&w, len, c->numlenbits + (uint32_t)floorlog2_i((int32_t)nump));
                    len = 0; nump = 0;
                }
            }
        }
    }
    bw_flush(&w);
    for (uint32_t bandno = 0; bandno < res->numbands; ++bandno) {
        band_t *b = &res->bands[bandno];
        precinct_t *pr = &b->precs[precno];
        uint32_t nb = pr->cw * pr->ch;
        if (band_empty(b) || !nb) continue;
        for (uint32_t cb = 0; cb < nb; ++cb) {
            cblk_t *c = &pr->cblks[cb];
            if (!c->numpasses) continue;
            uint32_t L = c->passes[c->numpasses - 1].rate;
            bb_putn(out, c->data, L);
            c->included = 1;
        }
    }
}

/* returns bytes consumed or -1 */
static int64_t t2_decode_packet(tilecomp_t *tc, uint32_t resno, uint32_t precno, uint32_t layno,
                                const uint8_t *p, size_t n) {
    resolution_t *res = &tc->res[resno];
    if (layno == 0) {
        for (uint32_t bandno = 0; bandno < res->numbands; ++bandno) {
            band_t *b = &res->bands[bandno];
            precinct_t *pr = &b->precs[precno];
            uint32_t nb = pr->cw * pr->ch;
            if (band_empty(b) || !nb) continue;
            tt_reset(&pr->incl); tt_reset(&pr->imsb);
            for (uint32_t cb = 0; cb < nb; ++cb) { pr->cblks[cb].included = 0; pr->cblks[cb].dec_passes = 0; }
        }
    }
    bio_r r = {p, n, 0, 0, 0, 0};
    uint32_t present = br_read(&r, 1);
    uint32_t ncb_total = 0;
    for (uint32_t bandno = 0; bandno < res->numbands; ++bandno)
        ncb_total += res->bands[bandno].precs[precno].cw * res->bands[bandno].precs[precno].ch;
    uint32_t *seglen = (uint32_t *)malloc(sizeof(uint32_t) * (ncb_total + 1));
    cblk_t **segcb = (cblk_t **)malloc(sizeof(cblk_t *) * (ncb_total + 1));
    uint32_t nseg = 0;
    int64_t ret = -1;
    if (present) {
        for (uint32_t bandno = 0; bandno < res->numbands; ++bandno) {
            band_t *b = &res->bands[bandno];
            precinct_t *pr = &b->precs[precno];
            uint32_t nb = pr->cw * pr->ch;
            if (band_empty(b) || !nb) continue;
            for (uint32_t cb = 0; cb < nb; ++cb) {
                cblk_t *c = &pr->cblks[cb];
                uint32_t inc;
                if (!c->included) inc = tt_decode(&pr->incl, &r, cb, layno + 1) <= (int64_t)layno;
                else inc = br_read(&r, 1);
                if (!inc) continue;
                if (!c->included) {
                    int64_t kmsbs = tt_decode(&pr->imsb, &r, cb, INT64_MAX);
                    c->numbps = (uint32_t)((int64_t)b->numbps - kmsbs);
                    c->numlenbits = 3;
                    c->included = 1;
                }
                uint32_t np = br_numpasses(&r);
                c->numlenbits += br_comma(&r);
                /* cblksty 0: one segment of up to 109 passes */
                uint32_t L = br_read(&r, c->numlenbits + floorlog2_u(np));
                c->dec_passes += np;
                seglen[nseg] = L; segcb[nseg] = c; nseg++;
                if (r.err) goto done;
            }
        }
    }
    br_align(&r);
    if (r.err) goto done;
    size_t off = r.off;
    for (uint32_t i = 0; i < nseg; ++i) {
        cblk_t *c = segcb[i];
        /* T2::read_packet_data (T2.cpp:686-698): truncate to the bytes present */
        if (off + seglen[i] > n) seglen[i] = (uint32_t)(n - off);
        if (c->seglen + seglen[i] + 2 > c->segcap) {
            c->segcap = (c->seglen + seglen[i] + 2) * 2;
            c->seg = (uint8_t *)realloc(c->seg, c->segcap);
        }
        memcpy(c->seg + c->seglen, p + off, seglen[i]);
        c->seglen += seglen[i];
        off += seglen[i];
    }
    ret = (int64_t)off;
done:
    free(seglen); free(segcb);
    return ret;
}

/* ------------------------------------------------------------------------- */
/* whole-codestream encode (codestream/j2k.cpp j2k_setup_encoder :1609,      */
/* j2k_encode :2059, marker writers :3117-5540)                              */
/* ------------------------------------------------------------------------- */
void orc_default_params(orc_params *p) {
    memset(p, 0, sizeof(*p));
    p->numres = 6; p->cblkw = 6; p->cblkh = 6; p->irreversible = 0; p->mct = -1;
}

typedef struct {
    tilecomp_t *tc; uint32_t compno; int irrev;
    cblk_t **list; uint32_t *band_orient; float *band_step; uint32_t *band_invstep;
} t1_job_ctx;

typedef struct { tilecomp_t *tc; cblk_t *c; uint32_t orient; uint32_t inv_step; float step; } cblk_ref;
typedef struct { cblk_ref *refs; int irrev; } t1_ctx;

static void t1_enc_job(void *vc, uint64_t i) {
    t1_ctx *ctx = (t1_ctx *)vc;
    cblk_ref *rf = &ctx->refs[i];
    cblk_t *c = rf->c;
    uint32_t w = c->r.x1 - c->r.x0, h = c->r.y1 - c->r.y0;
    uint32_t stride = rf->tc->r.x1 - rf->tc->r.x0;
    uint8_t *buf = (uint8_t *)calloc((size_t)w * h * 8 + 64, 1);
    c->data = buf + 1;
    c->numpasses = (uint32_t)orc_t1_encode_cblk(rf->tc->data + (size_t)c->by * stride + c->bx, stride, w, h,
                                                rf->orient, ctx->irrev ? 0 : 1, (int32_t)rf->inv_step,
                                                c->data, (uint32_t)((size_t)w * h * 8 + 60), c->passes,
                                                &c->numbps, &c->len);
}

static void t1_dec_job(void *vc, uint64_t i) {
    t1_ctx *ctx = (t1_ctx *)vc;
    cblk_ref *rf = &ctx->refs[i];
    cblk_t *c = rf->c;
    uint32_t w = c->r.x1 - c->r.x0, h = c->r.y1 - c->r.y0;
    uint32_t stride = rf->tc->r.x1 - rf->tc->r.x0;
    int32_t *dst = rf->tc->data + (size_t)c->by * stride + c->bx;
    if (!c->seglen) return; /* T1Part1::decode: no data -> block stays zero */
    int32_t *tmp = (int32_t *)malloc(sizeof(int32_t) * w * h);
    if (c->seglen + 2 > c->segcap) { c->segcap = c->seglen + 2; c->seg = (uint8_t *)realloc(c->seg, c->segcap); }
    orc_t1_decode_cblk(c->seg, c->seglen, c->dec_passes, c->numbps, w, h, rf->orient, tmp);
    /* T1Part1::post_decode (T1Part1.cpp:216-330), whole-tile path */
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            int32_t v = tmp[y * w + x];
            if (!ctx->irrev) dst[(size_t)y * stride + x] = v / 2;
            else { float f = (float)v * rf->step; memcpy(&dst[(size_t)y * stride + x], &f, 4); }
        }
    free(tmp);
}

static cblk_ref *collect_cblks(tilecomp_t *tc, uint32_t *count) {
    uint32_t n = 0;
    for (uint32_t resno = 0; resno < tc->numres; ++resno)
        for (uint32_t b = 0; b < tc->res[resno].numbands; ++b)
            for (uint32_t p = 0; p < tc->res[resno].pw * tc->res[resno].ph; ++p)
                n += tc->res[resno].bands[b].precs[p].cw * tc->res[resno].bands[b].precs[p].ch;
    cblk_ref *refs = (cblk_ref *)calloc(n ? n : 1, sizeof(cblk_ref));
    uint32_t k = 0;
    for (uint32_t resno = 0; resno < tc->numres; ++resno)
        for (uint32_t b = 0; b < tc->res[resno].numbands; ++b) {
            band_t *bd = &tc->res[resno].bands[b];
            for (uint32_t p = 0; p < tc->res[resno].pw * tc->res[resno].ph; ++p) {
                precinct_t *pr = &bd->precs[p];
                for (uint32_t cb = 0; cb < pr->cw * pr->ch; ++cb) {
                    refs[k].tc = tc; refs[k].c = &pr->cblks[cb]; refs[k].orient = bd->bandno;
                    refs[k].inv_step = bd->inv_step; refs[k].step = bd->stepsize; k++;
                }
            }
        }
    *count = n;
    return refs;
}

static void tile_rect(const orc_image *img, uint32_t tdx, uint32_t tdy, uint32_t tx0, uint32_t ty0,
                      uint32_t tw, uint32_t tileno, rect_t *r) {
    uint32_t p = tileno % tw, q = tileno / tw;
    uint32_t x0 = tx0 + p * tdx, y0 = ty0 + q * tdy;
    r->x0 = umax(x0, img->x0); r->y0 = umax(y0, img->y0);
    r->x1 = umin(x0 + tdx, img->x1); r->y1 = umin(y0 + tdy, img->y1);
}

int orc_encode(const orc_image *img, const orc_params *prm, uint8_t **out, size_t *outlen) {
    uint32_t nc = img->numcomps;
    if (nc < 1 || nc > ORC_MAX_COMPS || prm->numres < 1 || prm->numres > 33) return -1;
    int irrev = prm->irreversible ? 1 : 0;
    int mct = prm->mct < 0 ? (nc >= 3 ? 1 : 0) : prm->mct;
    uint32_t tdx, tdy, tx0 = 0, ty0 = 0, tw = 1, th = 1;
    if (prm->tile_on) {
        tdx = prm->tdx; tdy = prm->tdy; tx0 = prm->tx0; ty0 = prm->ty0;
        tw = ceildiv_u32(img->x1 - tx0, tdx); th = ceildiv_u32(img->y1 - ty0, tdy);
    } else {
        tdx = img->x1 - tx0; tdy = img->y1 - ty0;
    }
    uint32_t numdecomps = prm->numres - 1;
    stepsize_t ss[3 * 33 + 1];
    if (irrev) qcd_irrev(ss, numdecomps, img->prec[0], img->sgnd[0]);
    else qcd_rev(ss, numdecomps, img->prec[0]);
    uint32_t nbands = 3 * numdecomps + 1;

    bytes_t cs = {0, 0, 0};
    bb_put16(&cs, 0xFF4F); /* SOC */
    /* SIZ (j2k.cpp:3166-3240) */
    bb_put16(&cs, 0xFF51); bb_put16(&cs, 38 + 3 * nc); bb_put16(&cs, 0);
    bb_put32(&cs, img->x1); bb_put32(&cs, img->y1); bb_put32(&cs, img->x0); bb_put32(&cs, img->y0);
    bb_put32(&cs, tdx); bb_put32(&cs, tdy); bb_put32(&cs, tx0); bb_put32(&cs, ty0);
    bb_put16(&cs, nc);
    for (uint32_t k = 0; k < nc; ++k) { bb_put8(&cs, (img->prec[k] - 1) + ((uint32_t)img->sgnd[k] << 7)); bb_put8(&cs, 1); bb_put8(&cs, 1); }
    /* COD (j2k.cpp:3723, SPCod :6905) */
    bb_put16(&cs, 0xFF52); bb_put16(&cs, 12);
    bb_put8(&cs, 0); bb_put8(&cs, 0 /*LRCP*/); bb_put16(&cs, 1 /*layers*/); bb_put8(&cs, (uint32_t)mct);
    bb_put8(&cs, numdecomps); bb_put8(&cs, prm->cblkw - 2); bb_put8(&cs, prm->cblkh - 2); bb_put8(&cs, 0); bb_put8(&cs, irrev ? 0 : 1);
    /* QCD (j2k.cpp:4033, SQcd :7088) */
    bb_put16(&cs, 0xFF5C); bb_put16(&cs, 3 + nbands * (irrev ? 2 : 1));
    bb_put8(&cs, (2u << 5) | (irrev ? 2u : 0u));
    for (uint32_t i = 0; i < nbands; ++i) {
        if (irrev) bb_put16(&cs, (ss[i].expn << 11) | ss[i].mant);
        else bb_put8(&cs, ss[i].expn << 3);
    }
    /* COM (j2k.cpp:1798 default comment, writer :3625) */
    const char *com = "Created by Grok     version 5.1.0";
    bb_put16(&cs, 0xFF64); bb_put16(&cs, 4 + (uint32_t)strlen(com)); bb_put16(&cs, 1);
    bb_putn(&cs, (const uint8_t *)com, strlen(com));

    int32_t shift[ORC_MAX_COMPS];
    for (uint32_t k = 0; k < nc; ++k) shift[k] = img->sgnd[k] ? 0 : (1 << (img->prec[k] - 1));
    uint32_t iw = img->x1 - img->x0;

    for (uint32_t tileno = 0; tileno < tw * th; ++tileno) {
        rect_t tr;
        tile_rect(img, tdx, tdy, tx0, ty0, tw, tileno, &tr);
        tilecomp_t *tcs = (tilecomp_t *)calloc(nc, sizeof(tilecomp_t));
        uint64_t n = (uint64_t)(tr.x1 - tr.x0) * (tr.y1 - tr.y0);
        for (uint32_t k = 0; k < nc; ++k) {
            build_tilecomp(&tcs[k], tr, prm->numres, prm->cblkw, prm->cblkh, ss, img->prec[k], irrev, 1);
            tcs[k].data = (int32_t *)malloc(sizeof(int32_t) * (n ? n : 1));
            for (uint32_t y = tr.y0; y < tr.y1; ++y)
                memcpy(tcs[k].data + (size_t)(y - tr.y0) * (tr.x1 - tr.x0),
                       img->data[k] + (size_t)(y - img->y0) * iw + (tr.x0 - img->x0), sizeof(int32_t) * (tr.x1 - tr.x0));
        }
        /* dc_level_shift_encode + mct_encode (TileProcessor.cpp:1449-1518) */
        for (uint32_t k = 0; k < nc; ++k) {
            if (k < 3 && mct && nc >= 3) continue;
            orc_dcshift_mct_fwd(tcs[k].data, NULL, NULL, 1, n, &shift[k], 0, irrev);
        }
        if (mct && nc >= 3) orc_dcshift_mct_fwd(tcs[0].data, tcs[1].data, tcs[2].data, 3, n, shift, 1, irrev);
        for (uint32_t k = 0; k < nc; ++k) {
            orc_dwt_fwd(tcs[k].data, tr.x0, tr.y0, tr.x1, tr.y1, prm->numres, irrev, prm->nthreads);
            uint32_t cnt;
            t1_ctx ctx;
            ctx.refs = collect_cblks(&tcs[k], &cnt);
            ctx.irrev = irrev;
            parallel_for(cnt, prm->nthreads, t1_enc_job, &ctx);
            free(ctx.refs);
        }
        /* SOT + SOD + packets (LRCP) */
        size_t sot = cs.n;
        bb_put16(&cs, 0xFF90); bb_put16(&cs, 10); bb_put16(&cs, tileno); bb_put32(&cs, 0); bb_put8(&cs, 0); bb_put8(&cs, 1);
        bb_put16(&cs, 0xFF93);
        uint32_t maxres = prm->numres;
        for (uint32_t resno = 0; resno < maxres; ++resno)
            for (uint32_t k = 0; k < nc; ++k) {
                resolution_t *res = &tcs[k].res[resno];
                for (uint32_t precno = 0; precno < res->pw * res->ph; ++precno)
                    t2_encode_packet(&tcs[k], resno, precno, &cs);
            }
        bb_set32(&cs, sot + 6, (uint32_t)(cs.n - sot));
        for (uint32_t k = 0; k < nc; ++k) free_tilecomp(&tcs[k]);
        free(tcs);
    }
    bb_put16(&cs, 0xFFD9); /* EOC */
    *out = cs.p; *outlen = cs.n;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* whole-codestream decode (j2k.cpp read path; TileProcessor::decode_tile)   */
/* ------------------------------------------------------------------------- */
static uint32_t rd16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t rd32(const uint8_t *p) { return (rd16(p) << 16) | rd16(p + 2); }

void orc_image_free(orc_image *img) {
    for (uint32_t k = 0; k < img->numcomps; ++k) { free(img->data[k]); img->data[k] = NULL; }
}

int orc_decode(const uint8_t *buf, size_t len, orc_image *out, int32_t nthreads) {
    return orc_decode_reduce(buf, len, out, nthreads, 0);
}

static uint32_t ceildivpow2_u32(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a + ((1ull << b) - 1)) >> b); }

/* reduce > 0: decode at resolution numres-1-reduce (grk_decompress -r,
 * cp_reduce, grok.h:698-702): every packet is parsed, the inverse DWT stops
 * reduce levels early, MCT + DC shift run on the reduced tile-components, and
 * the image is ceil(x / 2^reduce) in every coordinate (j2k.cpp:1464-1476). */
int orc_decode_reduce(const uint8_t *buf, size_t len, orc_image *out, int32_t nthreads, uint32_t reduce) {
    memset(out, 0, sizeof(*out));
    if (len < 4 || rd16(buf) != 0xFF4F) return -1;
    size_t pos = 2;
    uint32_t tdx = 0, tdy = 0, tx0 = 0, ty0 = 0, nc = 0;
    uint32_t numres = 0, cblkw = 6, cblkh = 6, irrev = 0, mct = 0, numlayers = 1, prog = 0, cblksty = 0;
    stepsize_t ss[3 * 33 + 1];
    memset(ss, 0, sizeof(ss));
    /* tile data accumulated per tile */
    bytes_t *tdata = NULL;
    uint32_t ntiles = 0, tw = 0, th = 0;
    while (pos + 4 <= len) {
        uint32_t m = rd16(buf + pos);
        if (m == 0xFFD9) break;
        if (m == 0xFF90) {
            uint32_t isot = rd16(buf + pos + 4), psot = rd32(buf + pos + 6);
            size_t sot = pos;
            pos += 12;
            while (pos + 2 <= len && rd16(buf + pos) != 0xFF93) pos += 2 + rd16(buf + pos + 2);
            pos += 2;
            size_t end = psot ? sot + psot : len - 2;
            if (end > len) end = len; /* a stream cut inside a tile-part: keep what is there */
            if (isot >= ntiles || pos > end) return -1;
            bb_putn(&tdata[isot], buf + pos, end - pos);
            pos = end;
            continue;
        }
        uint32_t L = rd16(buf + pos + 2);
        const uint8_t *p = buf + pos + 4;
        if (m == 0xFF51) {
            out->x1 = rd32(p + 2); out->y1 = rd32(p + 6); out->x0 = rd32(p + 10); out->y0 = rd32(p + 14);
            tdx = rd32(p + 18); tdy = rd32(p + 22); tx0 = rd32(p + 26); ty0 = rd32(p + 30);
            nc = rd16(p + 34);
            if (nc > ORC_MAX_COMPS) return -1;
            out->numcomps = nc;
            for (uint32_t k = 0; k < nc; ++k) { out->prec[k] = (p[36 + 3 * k] & 0x7f) + 1; out->sgnd[k] = p[36 + 3 * k] >> 7; }
            tw = ceildiv_u32(out->x1 - tx0, tdx); th = ceildiv_u32(out->y1 - ty0, tdy);
            ntiles = tw * th;
            tdata = (bytes_t *)calloc(ntiles, sizeof(bytes_t));
        } else if (m == 0xFF52) {
            if (p[0] != 0) return -2; /* precincts / SOP / EPH: not in oracle scope */
            prog = p[1]; numlayers = rd16(p + 2); mct = p[4];
            numres = p[5] + 1u; cblkw = p[6] + 2u; cblkh = p[7] + 2u; cblksty = p[8]; irrev = p[9] == 0;
        } else if (m == 0xFF5C) {
            uint32_t sq = p[0] & 0x1f;
            uint32_t nb = sq == 0 ? (L - 3) : (L - 3) / 2;
            for (uint32_t i = 0; i < nb && i < 3 * 33 + 1; ++i) {
                if (sq == 0) { ss[i].expn = p[1 + i] >> 3; ss[i].mant = 0; }
                else { uint32_t v = rd16(p + 1 + 2 * i); ss[i].expn = v >> 11; ss[i].mant = v & 0x7ff; }
            }
        } else if (m == 0xFF53 || m == 0xFF5D || m == 0xFF5F || m == 0xFF5E || m == 0xFF60 || m == 0xFF61) {
            return -2; /* COC/QCC/POC/RGN/PPM/PPT: outside oracle scope */
        }
        pos += 2 + L;
    }
    if (!tdata || prog != 0 || cblksty != 0 || numlayers == 0) { free(tdata); return -2; }
    if (reduce >= numres) { free(tdata); return -5; } /* j2k.cpp:6994: reduce must be < numresolutions */
    const uint32_t numres_dec = numres - reduce;
    const orc_image full = *out;  /* full-resolution geometry (tiles) */
    out->x0 = ceildivpow2_u32(out->x0, reduce); out->y0 = ceildivpow2_u32(out->y0, reduce);
    out->x1 = ceildivpow2_u32(out->x1, reduce); out->y1 = ceildivpow2_u32(out->y1, reduce);
    uint32_t iw = out->x1 - out->x0, ih = out->y1 - out->y0;
    for (uint32_t k = 0; k < nc; ++k) out->data[k] = (int32_t *)calloc(((size_t)iw * ih) != 0 ? (size_t)iw * ih : 1, sizeof(int32_t));
    int rc = 0;
    for (uint32_t tileno = 0; tileno < ntiles && rc == 0; ++tileno) {
        rect_t tr;
        tile_rect(&full, tdx, tdy, tx0, ty0, tw, tileno, &tr);
        tilecomp_t *tcs = (tilecomp_t *)calloc(nc, sizeof(tilecomp_t));
        rect_t rr; /* the tile at the decoded resolution; samples keep the full tile's stride */
        res_rect(&rr, tr.x0, tr.y0, tr.x1, tr.y1, numres, numres_dec - 1);
        const uint32_t fw = tr.x1 - tr.x0;
        const uint64_t n = (uint64_t)fw * (tr.y1 - tr.y0);
        for (uint32_t k = 0; k < nc; ++k) {
            build_tilecomp(&tcs[k], tr, numres, cblkw, cblkh, ss, out->prec[k], (int)irrev, 0);
            tcs[k].data = (int32_t *)calloc(n ? n : 1, sizeof(int32_t));
        }
        size_t off = 0;
        const uint8_t *td = tdata[tileno].p;
        size_t tlen = tdata[tileno].n;
        for (uint32_t layno = 0; layno < numlayers && rc == 0; ++layno)
            for (uint32_t resno = 0; resno < numres && rc == 0; ++resno)
                for (uint32_t k = 0; k < nc && rc == 0; ++k) {
                    resolution_t *res = &tcs[k].res[resno];
                    for (uint32_t precno = 0; precno < res->pw * res->ph; ++precno) {
                        if (off >= tlen) break; /* truncated stream: remaining packets absent */
                        int64_t used = t2_decode_packet(&tcs[k], resno, precno, layno, td + off, tlen - off);
                        if (used < 0) { rc = -3; break; }
                        off += (size_t)used;
                    }
                }
        for (uint32_t k = 0; k < nc && rc == 0; ++k) {
            uint32_t cnt;
            t1_ctx ctx;
            ctx.refs = collect_cblks(&tcs[k], &cnt);
            ctx.irrev = (int)irrev;
            parallel_for(cnt, nthreads, t1_dec_job, &ctx);
            free(ctx.refs);
            dwt_inv_levels(tcs[k].data, tr.x0, tr.y0, tr.x1, tr.y1, numres, numres_dec, (int32_t)irrev, nthreads);
        }
        /* mct_decode (TileProcessor.cpp:1303-1375) */
        if (rc == 0 && mct == 1 && nc >= 3) {
            int32_t *c0 = tcs[0].data, *c1 = tcs[1].data, *c2 = tcs[2].data;
            for (uint64_t j = 0; j < (uint64_t)(rr.x1 - rr.x0) * (rr.y1 - rr.y0); ++j) {
                const uint64_t i = (j / (rr.x1 - rr.x0)) * fw + j % (rr.x1 - rr.x0);
                if (!irrev) {
                    int32_t y = c0[i], u = c1[i], v = c2[i];
                    int32_t g = y - ((u + v) >> 2);
                    c0[i] = v + g; c1[i] = g; c2[i] = u + g;
                } else {
                    float y, u, v;
                    memcpy(&y, &c0[i], 4); memcpy(&u, &c1[i], 4); memcpy(&v, &c2[i], 4);
                    volatile float t1 = v * 1.402f, t2 = u * 0.34413f, t3 = v * 0.71414f, t4 = u * 1.772f;
                    float r = y + t1;
                    volatile float g0 = y - t2;
                    float g = g0 - t3;
                    float b = y + t4;
                    memcpy(&c0[i], &r, 4); memcpy(&c1[i], &g, 4); memcpy(&c2[i], &b, 4);
                }
            }
        }
        /* dc_level_shift_decode (TileProcessor.cpp:1377-1432) + copy out */
        for (uint32_t k = 0; k < nc && rc == 0; ++k) {
            int32_t mn, mx, sh = out->sgnd[k] ? 0 : (1 << (out->prec[k] - 1));
            if (out->sgnd[k]) { mn = -(1 << (out->prec[k] - 1)); mx = (1 << (out->prec[k] - 1)) - 1; }
            else { mn = 0; mx = (1 << out->prec[k]) - 1; }
            for (uint32_t y = rr.y0; y < rr.y1; ++y)
                for (uint32_t x = rr.x0; x < rr.x1; ++x) {
                    int32_t v = tcs[k].data[(size_t)(y - rr.y0) * fw + (x - rr.x0)];
                    if (irrev) { float f; memcpy(&f, &v, 4); v = (int32_t)lrintf(f); }
                    v += sh;
                    v = v < mn ? mn : (v > mx ? mx : v);
                    out->data[k][(size_t)(y - out->y0) * iw + (x - out->x0)] = v;
                }
        }
        for (uint32_t k = 0; k < nc; ++k) free_tilecomp(&tcs[k]);
        free(tcs);
    }
    for (uint32_t t = 0; t < ntiles; ++t) free(tdata[t].p);
    free(tdata);
    return rc;
}
