/*
 * firdecim.c -- firdecim_{rrrf,crcf,cccf} and firinterp_{rrrf,crcf,cccf}.
 *
 * firdecim: include/liquid.h:2664-2735, src/filter/src/firdecim.c:47-223.
 *   y[o] = sum_{k<h} h[k] x[o*M - k]: the output is formed right after the
 *   first of each group of M pushes (:195-204); execute_block's _n counts
 *   outputs (:208-223); create_kaiser designs 2Mm+1 taps at fc = 0.5/M and
 *   uses the first 2Mm (:88-122).  No output scale.
 * firinterp: include/liquid.h:2496-2565, src/filter/src/firinterp.c:43-215.
 *   L = ceil(h/M), h' = h zero-padded to M*L, y[i*M + p] =
 *   sum_{l<L} h'[p + l*M] x[i - l]; create needs M >= 2 and h_len >= M.
 *
 * One generic engine per object (sample kind rrrf / crcf / cccf chooses the
 * kernel instantiation and element sizes); the typed front ends at the end
 * only forward.
 */
#include <complex.h>

#include "lq_host.h"

static const char *lq_ext[] = {"rrrf", "crcf", "cccf"};

/* ================================================================ firdecim */

typedef struct {
    int kind;
    size_t esz, csz;
    unsigned int M, hlen;
    float *h;          /* host copy, hlen coefficients of csz bytes */
    float *hg;         /* reversed, expanded for the host path (lq_host_taps) */
    lqk_fir_desc d;
    void *d_hpad;
    void *d_hq;        /* M x QC phase-major taps for the phase-layout kernel */
    unsigned int QC;
    void *d_hist[2];   /* last hlen-1 inputs */
    int cur;
    lq_mirror hm;      /* host copy of the history (small-call mode) */
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf;
} lq_decim;

static lq_decim *lq_decim_create(int kind, unsigned int M, const float *h, unsigned int hlen)
{
    if (hlen == 0) LQ_FAIL("error: decim_%s_create(), filter length must be greater than zero\n", lq_ext[kind]);
    if (M == 0) LQ_FAIL("error: decim_%s_create(), decimation factor must be greater than zero\n", lq_ext[kind]);
    lqrt_require_device("firdecim_create");
    lq_decim *q = (lq_decim *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->esz = kind == LQ_RRRF ? 4 : 8;
    q->csz = kind == LQ_CCCF ? 8 : 4;
    q->M = M;
    q->hlen = hlen;
    q->h = (float *)lq_xmalloc(hlen * q->csz);
    memcpy(q->h, h, hlen * q->csz);
    q->hg = lq_host_taps(kind, q->h, hlen, 1);
    lq_ctx_init(&q->ctx);
    q->d_hpad = lqrt_malloc(hlen * q->csz);
    lqrt_h2d(q->d_hpad, q->h, hlen * q->csz, q->ctx.stream);
    /* k = qM + r -> hq[r*QC + q] (zero past hlen) */
    q->QC = lqk_firdecim_ph_qc(M, hlen);
    const size_t nq = (size_t)M * q->QC, cf = q->csz / sizeof(float);
    float *hq = (float *)lq_xmalloc(nq * q->csz);
    memset(hq, 0, nq * q->csz);
    for (unsigned int k = 0; k < hlen; k++)
        memcpy(hq + ((size_t)(k % M) * q->QC + k / M) * cf, q->h + (size_t)k * cf, q->csz);
    q->d_hq = lqrt_malloc(nq * q->csz);
    lqrt_h2d(q->d_hq, hq, nq * q->csz, q->ctx.stream);
    q->d_hist[0] = lqrt_malloc((size_t)hlen * q->esz);
    q->d_hist[1] = lqrt_malloc((size_t)hlen * q->esz);
    lqrt_sync(q->ctx.stream);
    free(hq);
    q->d.kind = kind;
    q->d.hlen = hlen;
    q->d.hc = hlen; /* the decimator kernel takes HP = hc * nchunk directly */
    q->d.nchunk = 1;
    q->d.hpad = q->d_hpad;
    q->d.scale_re = 1.0f;
    q->d.scale_im = 0.0f;
    lq_mirror_init(&q->hm, hlen - 1, q->esz);
    return q;
}

/* firdecim.c:88-122: 2Mm+1 Kaiser taps at fc = 0.5/M, first 2Mm used */
static float *lq_decim_kaiser(const char *who, unsigned int M, unsigned int m, float As, unsigned int *n)
{
    if (M < 2) LQ_FAIL("error: %s_create_kaiser(), decim factor must be greater than 1\n", who);
    if (m == 0) LQ_FAIL("error: %s_create_kaiser(), filter delay must be greater than 0\n", who);
    if (As < 0.0f) LQ_FAIL("error: %s_create_kaiser(), stop-band attenuation must be positive\n", who);
    *n = 2 * M * m + 1;
    float *hf = (float *)lq_xmalloc(*n * sizeof(float));
    lq_firdes_kaiser(*n, 0.5f / (float)M, As, 0.0f, hf);
    return hf;
}

static void lq_decim_destroy(lq_decim *q)
{
    lqrt_sync(q->ctx.stream);
    lqrt_free(q->d_hpad);
    lqrt_free(q->d_hq);
    lqrt_free(q->d_hist[0]);
    lqrt_free(q->d_hist[1]);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_ctx_free(&q->ctx);
    lq_mirror_free(&q->hm);
    free(q->h);
    free(q->hg);
    free(q);
}

static void lq_decim_print(lq_decim *q)
{
    printf("FIRDECIM() [%u] :\n", q->M);
    for (unsigned int i = 0; i < q->hlen; i++) {
        if (q->kind == LQ_CCCF) printf("  h(%3u) = %12.8f + j*%12.8f\n", i + 1, q->h[2 * i], q->h[2 * i + 1]);
        else printf("  h(%3u) = %12.8f\n", i + 1, q->h[i]);
    }
}

static void lq_decim_clear(lq_decim *q)
{
    lqrt_memset(q->d_hist[0], (size_t)q->hlen * q->esz, q->ctx.stream);
    lqrt_memset(q->d_hist[1], (size_t)q->hlen * q->esz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    lq_mirror_zero(&q->hm);
}

static void lq_decim_block_dev(lq_decim *q, const void *dx, unsigned long long nout, void *dy)
{
    if (nout == 0) return;
    lq_mirror_need_dev(&q->hm, q->d_hist[q->cur], q->ctx.stream);
    q->hm.host_valid = 0;
    void *hold = q->d_hist[q->cur], *hnew = q->d_hist[q->cur ^ 1];
    if (lqk_firdecim_ph(q->kind, q->M, q->QC, q->d_hq, q->hlen - 1, hold, dx, nout, dy, q->ctx.stream) != 0)
        lqk_firdecim(&q->d, q->M, hold, dx, nout, dy, q->ctx.stream);
    if (q->hlen > 1) {
        lqk_window_append(q->kind != LQ_RRRF, hold, q->hlen - 1, dx, nout * q->M, hnew, q->ctx.stream);
        q->cur ^= 1;
    }
}

/* small-call mode: one output on the host (firdecim.c:189-205: the dot
 * product right after the first of the M pushes) */
static void lq_decim_exec1_host(lq_decim *q, const void *x, void *y)
{
    lq_mirror_need_host(&q->hm, q->d_hist[q->cur], q->ctx.stream);
    lq_mirror_append(&q->hm, x, q->M);
    lq_host_tdot(q->kind, q->hg, lq_mirror_ptr(&q->hm), q->hlen, y);   /* the hlen-sample window, oldest first */
    lq_mirror_commit(&q->hm, q->M);
}

/* single: the call is firdecim_*_execute; execute_block always runs on the GPU */
static void lq_decim_block(lq_decim *q, const void *x, unsigned long long nout, void *y, int single)
{
    if (nout == 0) return;
    if (single && lq_small_host()) {
        lq_decim_exec1_host(q, x, y);
        return;
    }
    size_t nin = (size_t)nout * q->M * q->esz, nb = (size_t)nout * q->esz;
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, nin);
    void *dy = lq_devbuf_get(&q->ybuf, nb);
    lq_decim_block_dev(q, dx, nout, dy);
    lq_call_out(&q->ctx, y, dy, nb);
}

#define LQ_FIRDECIM_FRONT(NAME, KIND, TO, TC, TI)                                                   \
    struct NAME##_s {                                                                               \
        lq_decim *e;                                                                                \
    };                                                                                              \
    NAME NAME##_create(unsigned int _M, TC *_h, unsigned int _h_len)                                \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = lq_decim_create(KIND, _M, (const float *)_h, _h_len);                                \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_create_kaiser(unsigned int _M, unsigned int _m, float _As)                          \
    {                                                                                               \
        unsigned int n;                                                                             \
        float *hf = lq_decim_kaiser(#NAME, _M, _m, _As, &n);                                        \
        TC *hc = (TC *)lq_xmalloc(n * sizeof(TC));                                                  \
        for (unsigned int i = 0; i < n; i++) hc[i] = (TC)hf[i];                                     \
        NAME q = NAME##_create(_M, hc, n - 1);                                                      \
        free(hf);                                                                                   \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    /* firdecim.c:126-160: 2Mm+1 taps from liquid_firdes_prototype */                               \
    NAME NAME##_create_prototype(int _type, unsigned int _M, unsigned int _m, float _beta, float _dt) \
    {                                                                                               \
        if (_M < 2) LQ_FAIL("error: " #NAME "_create_prototype(), decimation factor must be greater than 1\n"); \
        if (_m == 0) LQ_FAIL("error: " #NAME "_create_prototype(), filter delay must be greater than 0\n"); \
        if (_beta < 0.0f || _beta > 1.0f)                                                           \
            LQ_FAIL("error: " #NAME "_create_prototype(), filter excess bandwidth factor must be in [0,1]\n"); \
        if (_dt < -1.0f || _dt > 1.0f)                                                              \
            LQ_FAIL("error: " #NAME "_create_prototype(), filter fractional sample delay must be in [-1,1]\n"); \
        const unsigned int n = 2 * _M * _m + 1;                                                     \
        float *hf = (float *)lq_xmalloc(n * sizeof(float));                                         \
        TC *hc = (TC *)lq_xmalloc(n * sizeof(TC));                                                  \
        liquid_firdes_prototype((liquid_firfilt_type)_type, _M, _m, _beta, _dt, hf);                \
        for (unsigned int i = 0; i < n; i++) hc[i] = (TC)hf[i];                                     \
        NAME q = NAME##_create(_M, hc, n);                                                          \
        free(hf);                                                                                   \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_decim_destroy(_q->e);                                                                    \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_print(NAME _q) { lq_decim_print(_q->e); }                                           \
    void NAME##_clear(NAME _q) { lq_decim_clear(_q->e); }                                           \
    void NAME##_execute(NAME _q, TI *_x, TO *_y) { lq_decim_block(_q->e, _x, 1, _y, 1); }           \
    void NAME##_execute_block(NAME _q, TI *_x, unsigned int _n, TO *_y)                             \
    {                                                                                               \
        lq_decim_block(_q->e, _x, _n, _y, 0);                                                       \
    }                                                                                               \
    void NAME##_execute_block_dev(NAME _q, const TI *_dx, unsigned long long _n, TO *_dy)           \
    {                                                                                               \
        lq_decim_block_dev(_q->e, _dx, _n, _dy);                                                    \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ctx_set_stream(&_q->e->ctx, _s); }

LQ_FIRDECIM_FRONT(firdecim_rrrf, LQ_RRRF, float, float, float)
LQ_FIRDECIM_FRONT(firdecim_crcf, LQ_CRCF, liquid_float_complex, float, liquid_float_complex)
LQ_FIRDECIM_FRONT(firdecim_cccf, LQ_CCCF, liquid_float_complex, liquid_float_complex, liquid_float_complex)

/* =============================================================== firinterp */

typedef struct {
    int kind;
    size_t esz, csz;
    unsigned int M, L, hlen;
    float *h;          /* padded prototype, M*L coefficients of csz bytes */
    void *d_hpoly;     /* M x L: hpoly[p*L + l] = h'[p + l*M] */
    void *d_hist[2];   /* last L-1 inputs */
    int cur;
    float *hpoly;      /* host copy of the M x L phase taps */
    float *hgp;        /* the phases reversed and expanded for the host path, hgs floats apart */
    size_t hgs;
    lq_mirror hm;      /* host copy of the history (small-call mode) */
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf;
} lq_interp;

static lq_interp *lq_interp_create(int kind, unsigned int M, const float *h, unsigned int hlen)
{
    if (M < 2) LQ_FAIL("error: firinterp_%s_create(), interp factor must be greater than 1\n", lq_ext[kind]);
    if (hlen < M)
        LQ_FAIL("error: firinterp_%s_create(), filter length cannot be less than interp factor\n", lq_ext[kind]);
    lqrt_require_device("firinterp_create");
    lq_interp *q = (lq_interp *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->esz = kind == LQ_RRRF ? 4 : 8;
    q->csz = kind == LQ_CCCF ? 8 : 4;
    const size_t cf = q->csz / 4;       /* floats per coefficient */
    q->M = M;
    q->L = 0;
    while (M * q->L < hlen) q->L++;
    q->hlen = M * q->L;
    q->h = (float *)lq_xmalloc(q->hlen * q->csz);  /* tail zero (firinterp.c:68-73) */
    memcpy(q->h, h, hlen * q->csz);
    float *hp = (float *)lq_xmalloc(q->hlen * q->csz);
    for (unsigned int p = 0; p < M; p++)
        for (unsigned int l = 0; l < q->L; l++)
            memcpy(hp + cf * (p * q->L + l), q->h + cf * (p + l * M), q->csz);
    lq_ctx_init(&q->ctx);
    q->d_hpoly = lqrt_malloc(q->hlen * q->csz);
    lqrt_h2d(q->d_hpoly, hp, q->hlen * q->csz, q->ctx.stream);
    q->d_hist[0] = lqrt_malloc((size_t)q->L * q->esz);
    q->d_hist[1] = lqrt_malloc((size_t)q->L * q->esz);
    lqrt_sync(q->ctx.stream);
    q->hpoly = hp;
    q->hgs = (size_t)q->L * (kind == LQ_RRRF ? 1 : (kind == LQ_CRCF ? 2 : 4));
    q->hgp = (float *)lq_xmalloc((size_t)M * q->hgs * sizeof(float));
    for (unsigned int p = 0; p < M; p++) {
        float *g = lq_host_taps(kind, hp + cf * p * q->L, q->L, 1);
        memcpy(q->hgp + p * q->hgs, g, q->hgs * sizeof(float));
        free(g);
    }
    lq_mirror_init(&q->hm, q->L - 1, q->esz);
    return q;
}

static float *lq_interp_kaiser(const char *who, unsigned int M, unsigned int m, float As, unsigned int *n)
{
    if (M < 2) LQ_FAIL("error: %s_create_kaiser(), interp factor must be greater than 1\n", who);
    if (m == 0) LQ_FAIL("error: %s_create_kaiser(), filter delay must be greater than 0\n", who);
    if (As < 0.0f) LQ_FAIL("error: %s_create_kaiser(), stop-band attenuation must be positive\n", who);
    *n = 2 * M * m + 1;
    float *hf = (float *)lq_xmalloc(*n * sizeof(float));
    lq_firdes_kaiser(*n, 0.5f / (float)M, As, 0.0f, hf);
    return hf;
}

static void lq_interp_destroy(lq_interp *q)
{
    lqrt_sync(q->ctx.stream);
    lqrt_free(q->d_hpoly);
    lqrt_free(q->d_hist[0]);
    lqrt_free(q->d_hist[1]);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_ctx_free(&q->ctx);
    lq_mirror_free(&q->hm);
    free(q->hpoly);
    free(q->hgp);
    free(q->h);
    free(q);
}

static void lq_interp_print(lq_interp *q)
{
    printf("interp():\n");
    printf("    M       :   %u\n", q->M);
    printf("    h_len   :   %u\n", q->hlen);
}

static void lq_interp_reset(lq_interp *q)
{
    lqrt_memset(q->d_hist[0], (size_t)q->L * q->esz, q->ctx.stream);
    lqrt_memset(q->d_hist[1], (size_t)q->L * q->esz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    lq_mirror_zero(&q->hm);
}

static void lq_interp_block_dev(lq_interp *q, const void *dx, unsigned long long n, void *dy)
{
    if (n == 0) return;
    lq_mirror_need_dev(&q->hm, q->d_hist[q->cur], q->ctx.stream);
    q->hm.host_valid = 0;
    void *hold = q->d_hist[q->cur], *hnew = q->d_hist[q->cur ^ 1];
    lqk_firinterp(q->kind, q->d_hpoly, q->M, q->L, 1.0f, 0.0f, hold, dx, n, dy, q->ctx.stream);
    if (q->L > 1) {
        lqk_window_append(q->kind != LQ_RRRF, hold, q->L - 1, dx, n, hnew, q->ctx.stream);
        q->cur ^= 1;
    }
}

/* small-call mode: the M outputs of one input on the host (firinterp.c:187-198:
 * bank p of the polyphase filter over the last L inputs) */
static void lq_interp_exec1_host(lq_interp *q, const void *x, void *y)
{
    lq_mirror_need_host(&q->hm, q->d_hist[q->cur], q->ctx.stream);
    lq_mirror_append(&q->hm, x, 1);
    const unsigned char *w = lq_mirror_ptr(&q->hm);
    for (unsigned int p = 0; p < q->M; p++)   /* bank p over the L-sample window, oldest first */
        lq_host_tdot(q->kind, q->hgp + p * q->hgs, w, q->L, (unsigned char *)y + p * q->esz);
    lq_mirror_commit(&q->hm, 1);
}

/* single: the call is firinterp_*_execute; execute_block always runs on the GPU */
static void lq_interp_block(lq_interp *q, const void *x, unsigned long long n, void *y, int single)
{
    if (n == 0) return;
    if (single && lq_small_host()) {
        lq_interp_exec1_host(q, x, y);
        return;
    }
    size_t nin = (size_t)n * q->esz, nout = (size_t)n * q->M * q->esz;
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, nin);
    void *dy = lq_devbuf_get(&q->ybuf, nout);
    lq_interp_block_dev(q, dx, n, dy);
    lq_call_out(&q->ctx, y, dy, nout);
}

#define LQ_FIRINTERP_FRONT(NAME, KIND, TO, TC, TI)                                                  \
    struct NAME##_s {                                                                               \
        lq_interp *e;                                                                               \
    };                                                                                              \
    NAME NAME##_create(unsigned int _M, TC *_h, unsigned int _h_len)                                \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = lq_interp_create(KIND, _M, (const float *)_h, _h_len);                               \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_create_kaiser(unsigned int _M, unsigned int _m, float _As)                          \
    {                                                                                               \
        unsigned int n;                                                                             \
        float *hf = lq_interp_kaiser(#NAME, _M, _m, _As, &n);                                       \
        TC *hc = (TC *)lq_xmalloc(n * sizeof(TC));                                                  \
        for (unsigned int i = 0; i < n; i++) hc[i] = (TC)hf[i];                                     \
        NAME q = NAME##_create(_M, hc, n - 1);                                                      \
        free(hf);                                                                                   \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    /* firinterp.c:124-158: 2Mm+1 taps from liquid_firdes_prototype */                              \
    NAME NAME##_create_prototype(int _type, unsigned int _M, unsigned int _m, float _beta, float _dt) \
    {                                                                                               \
        if (_M < 2) LQ_FAIL("error: " #NAME "_create_prototype(), interp factor must be greater than 1\n"); \
        if (_m == 0) LQ_FAIL("error: " #NAME "_create_prototype(), filter delay must be greater than 0\n"); \
        if (_beta < 0.0f || _beta > 1.0f)                                                           \
            LQ_FAIL("error: " #NAME "_create_prototype(), filter excess bandwidth factor must be in [0,1]\n"); \
        if (_dt < -1.0f || _dt > 1.0f)                                                              \
            LQ_FAIL("error: " #NAME "_create_prototype(), filter fractional sample delay must be in [-1,1]\n"); \
        const unsigned int n = 2 * _M * _m + 1;                                                     \
        float *hf = (float *)lq_xmalloc(n * sizeof(float));                                         \
        TC *hc = (TC *)lq_xmalloc(n * sizeof(TC));                                                  \
        liquid_firdes_prototype((liquid_firfilt_type)_type, _M, _m, _beta, _dt, hf);                \
        for (unsigned int i = 0; i < n; i++) hc[i] = (TC)hf[i];                                     \
        NAME q = NAME##_create(_M, hc, n);                                                          \
        free(hf);                                                                                   \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_interp_destroy(_q->e);                                                                   \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_print(NAME _q) { lq_interp_print(_q->e); }                                          \
    void NAME##_reset(NAME _q) { lq_interp_reset(_q->e); }                                          \
    void NAME##_execute(NAME _q, TI _x, TO *_y) { lq_interp_block(_q->e, &_x, 1, _y, 1); }          \
    void NAME##_execute_block(NAME _q, TI *_x, unsigned int _n, TO *_y)                             \
    {                                                                                               \
        lq_interp_block(_q->e, _x, _n, _y, 0);                                                      \
    }                                                                                               \
    void NAME##_execute_block_dev(NAME _q, const TI *_dx, unsigned long long _n, TO *_dy)           \
    {                                                                                               \
        lq_interp_block_dev(_q->e, _dx, _n, _dy);                                                   \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ctx_set_stream(&_q->e->ctx, _s); }

LQ_FIRINTERP_FRONT(firinterp_rrrf, LQ_RRRF, float, float, float)
LQ_FIRINTERP_FRONT(firinterp_crcf, LQ_CRCF, liquid_float_complex, float, liquid_float_complex)
LQ_FIRINTERP_FRONT(firinterp_cccf, LQ_CCCF, liquid_float_complex, liquid_float_complex, liquid_float_complex)
