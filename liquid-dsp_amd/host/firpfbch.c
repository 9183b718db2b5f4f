/*
 * firpfbch.c -- firpfbch_{crcf,cccf} (critically sampled polyphase channelizer).
 *
 * API include/liquid.h:5667-5739; semantics src/multichannel/src/firpfbch.c:
 *  create          :73-142  type, M > 0 channels, p > 0 taps per branch,
 *                           h has M*p taps; branch i uses h[i + n*M]
 *  create_kaiser   :150-184 2*M*m+1 Kaiser taps at fc = 0.5/M, p = 2m
 *  create_rnyquist :193-256 root-Nyquist prototype (arkaiser, rkaiser, rrc,
 *                           hM3) of 2*M*m+1 taps; the analyzer keeps the
 *                           time-reversed first 2*M*m (matched filter)
 *  analyzer        :346-409 M inputs -> M channels, forward FFT (analyzer type)
 *  synthesizer     :314-336 M channels -> M outputs, backward FFT
 * The transform direction follows the object's type, as in the reference
 * (the plan is created once per object, firpfbch.c:132-135).  crcf has real
 * taps, cccf complex ones (multiplied without conjugation, dotprod_cccf).
 */
#include <complex.h>

#include "lq_host.h"

static const char *lq_ext[] = {"rrrf", "crcf", "cccf"};

typedef struct {
    int kind, type;
    unsigned int M, p;
    size_t csz;        /* bytes per coefficient */
    float *h;
    void *d_hsub;      /* M x p: hsub[i*p + n] = h[i + n*M] */
    void *d_hist[2];   /* analyzer: last (p-1)*M inputs */
    int cur;
    void *d_zstate;    /* synthesizer: last p-1 IFFT vectors */
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf, zbuf;
} lq_pfbch;

static lq_pfbch *lq_pfbch_create(int kind, int type, unsigned int M, unsigned int p, const float *h)
{
    const char *e = lq_ext[kind];
    if (type != LIQUID_ANALYZER && type != LIQUID_SYNTHESIZER)
        LQ_FAIL("error: firpfbch_%s_create(), invalid type %d\n", e, type);
    if (M == 0) LQ_FAIL("error: firpfbch_%s_create(), number of channels must be greater than 0\n", e);
    if (p == 0) LQ_FAIL("error: firpfbch_%s_create(), invalid filter size (must be greater than 0)\n", e);
    lqrt_require_device("firpfbch_create");
    lq_pfbch *q = (lq_pfbch *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->type = type;
    q->M = M;
    q->p = p;
    q->csz = kind == LQ_CCCF ? 8 : 4;
    const size_t nh = (size_t)M * p, cw = q->csz / 4;
    q->h = (float *)lq_xmalloc(nh * q->csz);
    memcpy(q->h, h, nh * q->csz);
    float *hsub = (float *)lq_xmalloc(nh * q->csz);
    for (unsigned int i = 0; i < M; i++)
        for (unsigned int n = 0; n < p; n++)
            for (size_t c = 0; c < cw; c++) hsub[(i * p + n) * cw + c] = h[(i + (size_t)n * M) * cw + c];
    lq_ctx_init(&q->ctx);
    q->d_hsub = lqrt_malloc(nh * q->csz);
    lqrt_h2d(q->d_hsub, hsub, nh * q->csz, q->ctx.stream);
    size_t hb = (size_t)(p - 1) * M * 8;
    q->d_hist[0] = lqrt_malloc(hb);
    q->d_hist[1] = lqrt_malloc(hb);
    q->d_zstate = lqrt_malloc(hb);
    lqrt_sync(q->ctx.stream);
    free(hsub);
    return q;
}

/* real prototype h (n taps, n >= M*p) -> typed coefficients, first M*p taps */
static lq_pfbch *lq_pfbch_create_real(int kind, int type, unsigned int M, unsigned int p, const float *h)
{
    const size_t nh = (size_t)M * p;
    if (kind != LQ_CCCF) return lq_pfbch_create(kind, type, M, p, h);
    float *hc = (float *)lq_xmalloc(nh * 8);
    for (size_t i = 0; i < nh; i++) {
        hc[2 * i] = h[i];
        hc[2 * i + 1] = 0.0f;
    }
    lq_pfbch *q = lq_pfbch_create(kind, type, M, p, hc);
    free(hc);
    return q;
}

static lq_pfbch *lq_pfbch_create_kaiser(int kind, int type, unsigned int M, unsigned int m, float As)
{
    if (M == 0) LQ_FAIL("error: firpfbch_%s_create_kaiser(), number of channels must be greater than 0\n", lq_ext[kind]);
    if (m == 0) LQ_FAIL("error: firpfbch_%s_create_kaiser(), invalid filter size (must be greater than 0)\n", lq_ext[kind]);
    As = As < 0 ? -As : As;
    unsigned int n = 2 * M * m + 1;
    float *h = (float *)lq_xmalloc(n * sizeof(float));
    lq_firdes_kaiser(n, 0.5f / (float)M, As, 0.0f, h);
    lq_pfbch *q = lq_pfbch_create_real(kind, type, M, 2 * m, h);
    free(h);
    return q;
}

static lq_pfbch *lq_pfbch_create_rnyquist(int kind, int type, unsigned int M, unsigned int m, float beta, int ftype)
{
    const char *e = lq_ext[kind];
    if (type != LIQUID_ANALYZER && type != LIQUID_SYNTHESIZER)
        LQ_FAIL("error: firpfbch_%s_create_rnyquist(), invalid type %d\n", e, type);
    if (M == 0) LQ_FAIL("error: firpfbch_%s_create_rnyquist(), number of channels must be greater than 0\n", e);
    if (m == 0) LQ_FAIL("error: firpfbch_%s_create_rnyquist(), invalid filter size (must be greater than 0)\n", e);
    const unsigned int n = 2 * M * m + 1, g = 2 * M * m;
    float *h = (float *)lq_xmalloc(n * sizeof(float));
    switch (ftype) {
    case LIQUID_FIRFILT_ARKAISER: liquid_firdes_arkaiser(M, m, beta, 0.0f, h); break;
    case LIQUID_FIRFILT_RKAISER: liquid_firdes_rkaiser(M, m, beta, 0.0f, h); break;
    case LIQUID_FIRFILT_RRC: liquid_firdes_rrcos(M, m, beta, 0.0f, h); break;
    case LIQUID_FIRFILT_hM3: liquid_firdes_hM3(M, m, beta, 0.0f, h); break;
    default: LQ_FAIL("error: firpfbch_%s_create_rnyquist(), unknown/invalid prototype (%d)\n", e, ftype);
    }
    float *gc = (float *)lq_xmalloc(g * sizeof(float));
    for (unsigned int i = 0; i < g; i++) gc[i] = type == LIQUID_SYNTHESIZER ? h[i] : h[g - i - 1];
    lq_pfbch *q = lq_pfbch_create_real(kind, type, M, 2 * m, gc);
    free(h);
    free(gc);
    return q;
}

static void lq_pfbch_destroy(lq_pfbch *q)
{
    lqrt_sync(q->ctx.stream);
    lqrt_free(q->d_hsub);
    lqrt_free(q->d_hist[0]);
    lqrt_free(q->d_hist[1]);
    lqrt_free(q->d_zstate);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_devbuf_free(&q->zbuf);
    lq_ctx_free(&q->ctx);
    free(q->h);
    free(q);
}

static void lq_pfbch_reset(lq_pfbch *q)
{
    size_t hb = (size_t)(q->p - 1) * q->M * 8;
    lqrt_memset(q->d_hist[0], hb, q->ctx.stream);
    lqrt_memset(q->d_hist[1], hb, q->ctx.stream);
    lqrt_memset(q->d_zstate, hb, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
}

static void lq_pfbch_print(lq_pfbch *q)
{
    printf("firpfbch (%s) [%u channels]:\n", q->type == LIQUID_ANALYZER ? "analyzer" : "synthesizer", q->M);
    for (unsigned int i = 0; i < q->M * q->p; i++) {
        const float re = q->kind == LQ_CCCF ? q->h[2 * i] : q->h[i];
        const float im = q->kind == LQ_CCCF ? q->h[2 * i + 1] : 0.0f;
        printf("  h[%3u] = %12.8f + %12.8f*j\n", i, re, im);
    }
}

/* the analyzer's few-block kernel (M = 1024, crcf): one launch that also
 * writes the next history and, with flag, raises the call's completion flag
 * (dy pinned host memory); 0: not handled, nothing launched */
static int lq_pfbch_an_few(lq_pfbch *q, const void *dx, unsigned long long nblocks, void *dy, unsigned *flag,
                           unsigned seq)
{
    const unsigned int HL = (q->p - 1) * q->M;
    void *hold = q->d_hist[q->cur], *hnew = q->d_hist[q->cur ^ 1];
    const lqk_hist_job job = {hold, dx, nblocks * q->M, hnew, HL};
    if (!lqk_firpfbch_analyzer_few(q->kind == LQ_CCCF, q->M, q->p, q->d_hsub, hold, dx, nblocks, dy, HL ? &job : NULL,
                                   flag, seq, q->ctx.stream))
        return 0;
    if (HL) q->cur ^= 1;
    return 1;
}

static void lq_pfbch_block_dev(lq_pfbch *q, const void *dx, unsigned long long nblocks, void *dy)
{
    if (nblocks == 0) return;
    const int ctaps = q->kind == LQ_CCCF;
    if (q->type == LIQUID_ANALYZER) {
        if (lq_pfbch_an_few(q, dx, nblocks, dy, NULL, 0)) return;
        void *hold = q->d_hist[q->cur], *hnew = q->d_hist[q->cur ^ 1];
        const unsigned int HL = (q->p - 1) * q->M;
        if (HL) lqk_window_append(1, hold, HL, dx, nblocks * q->M, hnew, q->ctx.stream);
        lqk_firpfbch_analyzer(ctaps, q->M, q->p, q->d_hsub, hold, dx, nblocks, dy, q->ctx.stream);
        if (HL) q->cur ^= 1;
    } else {
        void *z = lq_devbuf_get(&q->zbuf, (size_t)(q->p - 1 + nblocks) * q->M * 8);
        lqk_firpfbch_synthesizer(ctaps, q->M, q->p, q->d_hsub, q->d_zstate, z, dx, nblocks, dy, q->ctx.stream);
    }
}

static void lq_pfbch_block(lq_pfbch *q, const void *x, unsigned long long nblocks, void *y)
{
    if (nblocks == 0) return;
    size_t bytes = (size_t)nblocks * q->M * 8;
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, bytes);
    if (q->type == LIQUID_ANALYZER && bytes <= LQRT_COPYOUT_MAX) {
        /* a few blocks (the reference's execute() is one): the kernel writes
         * the pinned output buffer and raises the completion flag itself */
        unsigned *flag, seq;
        void *py = lq_sig_out(&q->ctx, bytes, &flag, &seq);
        if (lq_pfbch_an_few(q, dx, nblocks, py, flag, seq)) {
            lq_sig_wait(&q->ctx, y, bytes, seq);
            return;
        }
    }
    void *dy = lq_devbuf_get(&q->ybuf, bytes);
    lq_pfbch_block_dev(q, dx, nblocks, dy);
    lq_call_out(&q->ctx, y, dy, bytes);
}

#define LQ_FIRPFBCH_FRONT(NAME, KIND, TC)                                                           \
    struct NAME##_s {                                                                               \
        lq_pfbch *e;                                                                                \
    };                                                                                              \
    static NAME NAME##_wrap(lq_pfbch *e)                                                            \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = e;                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_create(int _type, unsigned int _M, unsigned int _p, TC *_h)                         \
    {                                                                                               \
        return NAME##_wrap(lq_pfbch_create(KIND, _type, _M, _p, (const float *)_h));                \
    }                                                                                               \
    NAME NAME##_create_kaiser(int _type, unsigned int _M, unsigned int _m, float _As)               \
    {                                                                                               \
        return NAME##_wrap(lq_pfbch_create_kaiser(KIND, _type, _M, _m, _As));                       \
    }                                                                                               \
    NAME NAME##_create_rnyquist(int _type, unsigned int _M, unsigned int _m, float _beta, int _ftype) \
    {                                                                                               \
        return NAME##_wrap(lq_pfbch_create_rnyquist(KIND, _type, _M, _m, _beta, _ftype));           \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_pfbch_destroy(_q->e);                                                                    \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_reset(NAME _q) { lq_pfbch_reset(_q->e); }                                           \
    void NAME##_print(NAME _q) { lq_pfbch_print(_q->e); }                                           \
    void NAME##_execute_block_dev(NAME _q, const liquid_float_complex *_dx, unsigned long long _nblocks, \
                                  liquid_float_complex *_dy)                                        \
    {                                                                                               \
        lq_pfbch_block_dev(_q->e, _dx, _nblocks, _dy);                                              \
    }                                                                                               \
    void NAME##_execute_block(NAME _q, liquid_float_complex *_x, unsigned long long _nblocks,       \
                              liquid_float_complex *_y)                                             \
    {                                                                                               \
        lq_pfbch_block(_q->e, _x, _nblocks, _y);                                                    \
    }                                                                                               \
    void NAME##_analyzer_execute(NAME _q, liquid_float_complex *_x, liquid_float_complex *_y)       \
    {                                                                                               \
        lq_pfbch_block(_q->e, _x, 1, _y);                                                           \
    }                                                                                               \
    void NAME##_synthesizer_execute(NAME _q, liquid_float_complex *_x, liquid_float_complex *_y)    \
    {                                                                                               \
        lq_pfbch_block(_q->e, _x, 1, _y);                                                           \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ctx_set_stream(&_q->e->ctx, _s); }

LQ_FIRPFBCH_FRONT(firpfbch_crcf, LQ_CRCF, float)
LQ_FIRPFBCH_FRONT(firpfbch_cccf, LQ_CCCF, liquid_float_complex)
