/*
 * firpfb.c -- firpfb_{rrrf,crcf,cccf} polyphase filter bank.
 *
 * include/liquid.h:2392-2486, src/filter/src/firpfb.c:46-345.
 *   Bank i = h[i + n*M], n < L = floor(h_len/M) (:73-84); push() appends one
 *   sample; execute(i) = scale * sum_n h[i + n*M] x[t-n] (:325-345, index
 *   check :330-334); create_kaiser designs 2Mm+1 taps at fc/M (:105-138);
 *   recreate with a new shape re-creates the object (:250-258).
 * Extension: execute_block pushes each input and evaluates every bank after
 * it (y[t*M + i]) -- the interpolator kernel's contraction.
 */
#include <complex.h>

#include <math.h>

#include "lq_host.h"

static const char *lq_ext[] = {"rrrf", "crcf", "cccf"};

typedef struct {
    int kind;
    size_t esz, csz;
    unsigned int M, hlen, L;
    float sre, sim;
    float *hpoly;                 /* M x L coefficients, hpoly[i*L + n] = h[i + n*M] */
    void *d_hpoly;
    void *d_win[2];               /* last L inputs, oldest first */
    int cur;
    unsigned char *h_win;         /* host mirror for push() */
    int host_valid, dev_valid;
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf, one;
} lq_pfb;

static void lq_pfb_load(lq_pfb *q, const float *h)
{
    const size_t cf = q->csz / 4;
    for (unsigned int i = 0; i < q->M; i++)
        for (unsigned int n = 0; n < q->L; n++) memcpy(q->hpoly + cf * (i * q->L + n), h + cf * (i + n * q->M), q->csz);
}

static lq_pfb *lq_pfb_create(int kind, unsigned int M, const float *h, unsigned int hlen)
{
    if (M == 0) LQ_FAIL("error: firpfb_%s_create(), number of filters must be greater than zero\n", lq_ext[kind]);
    if (hlen == 0) LQ_FAIL("error: firpfb_%s_create(), filter length must be greater than zero\n", lq_ext[kind]);
    if (hlen < M)
        LQ_FAIL("error: firpfb_%s_create(), filter length must be at least the number of filters\n", lq_ext[kind]);
    lqrt_require_device("firpfb_create");
    lq_pfb *q = (lq_pfb *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->esz = kind == LQ_RRRF ? 4 : 8;
    q->csz = kind == LQ_CCCF ? 8 : 4;
    q->M = M;
    q->hlen = hlen;
    q->L = hlen / M;
    q->sre = 1.0f;
    q->sim = 0.0f;
    q->hpoly = (float *)lq_xmalloc((size_t)M * q->L * q->csz);
    lq_pfb_load(q, h);
    lq_ctx_init(&q->ctx);
    q->d_hpoly = lqrt_malloc((size_t)M * q->L * q->csz);
    lqrt_h2d(q->d_hpoly, q->hpoly, (size_t)M * q->L * q->csz, q->ctx.stream);
    q->d_win[0] = lqrt_malloc((size_t)q->L * q->esz);
    q->d_win[1] = lqrt_malloc((size_t)q->L * q->esz);
    /* pinned: execute() reads it in place (zero copy) */
    q->h_win = (unsigned char *)lqrt_host_alloc((size_t)q->L * q->esz);
    memset(q->h_win, 0, (size_t)q->L * q->esz);
    q->host_valid = q->dev_valid = 1;
    lqrt_sync(q->ctx.stream);
    return q;
}

static float *lq_pfb_kaiser(const char *who, unsigned int M, unsigned int m, float fc, float As, unsigned int *n)
{
    if (M == 0) LQ_FAIL("error: %s_create_kaiser(), number of filters must be greater than zero\n", who);
    if (m == 0) LQ_FAIL("error: %s_create_kaiser(), filter delay must be greater than 0\n", who);
    if (fc < 0.0f || fc > 0.5f) LQ_FAIL("error: %s_create_kaiser(), filter cut-off frequence must be in (0,0.5)\n", who);
    if (As < 0.0f) LQ_FAIL("error: %s_create_kaiser(), filter excess bandwidth factor must be in [0,1]\n", who);
    *n = 2 * M * m + 1;
    float *hf = (float *)lq_xmalloc(*n * sizeof(float));
    lq_firdes_kaiser(*n, fc / (float)M, As, 0.0f, hf);
    return hf;
}

/* firpfb.c:146-240: prototype of 2*M*k*m+1 taps at M*k samples/symbol; the
 * derivative bank is the central difference (circular at the ends) scaled so
 * that max |h dh| = 0.06 */
static float *lq_pfb_rnyquist(const char *who, const char *fn, int deriv, int type, unsigned int M, unsigned int k,
                              unsigned int m, float beta, unsigned int *n)
{
    if (M == 0) LQ_FAIL("error: %s%s(), number of filters must be greater than zero\n", who, fn);
    if (k < 2) LQ_FAIL("error: %s%s(), filter samples/symbol must be greater than 1\n", who, fn);
    if (m == 0) LQ_FAIL("error: %s%s(), filter delay must be greater than 0\n", who, fn);
    if (beta < 0.0f || beta > 1.0f) LQ_FAIL("error: %s%s(), filter excess bandwidth factor must be in [0,1]\n", who, fn);
    const unsigned int N = 2 * M * k * m + 1;
    *n = N;
    float *H = (float *)lq_xmalloc(N * sizeof(float));
    liquid_firdes_prototype((liquid_firfilt_type)type, M * k, m, beta, 0, H);
    if (!deriv) return H;
    float *dH = (float *)lq_xmalloc(N * sizeof(float));
    float mx = 0.0f;
    for (unsigned int i = 0; i < N; i++) {
        dH[i] = H[i == N - 1 ? 0 : i + 1] - H[i == 0 ? N - 1 : i - 1];
        if (fabsf(H[i] * dH[i]) > mx) mx = fabsf(H[i] * dH[i]);
    }
    for (unsigned int i = 0; i < N; i++) dH[i] = dH[i] * 0.06f / mx;
    free(H);
    return dH;
}

static void lq_pfb_destroy(lq_pfb *q)
{
    lqrt_sync(q->ctx.stream);
    lqrt_free(q->d_hpoly);
    lqrt_free(q->d_win[0]);
    lqrt_free(q->d_win[1]);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_devbuf_free(&q->one);
    lq_ctx_free(&q->ctx);
    free(q->hpoly);
    lqrt_host_free(q->h_win);
    free(q);
}

static void lq_pfb_recoef(lq_pfb *q, const float *h)
{
    lq_pfb_load(q, h);
    lqrt_sync(q->ctx.stream);
    lqrt_h2d(q->d_hpoly, q->hpoly, (size_t)q->M * q->L * q->csz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
}

static void lq_pfb_print(lq_pfb *q)
{
    printf("fir polyphase filterbank [%u] :\n", q->M);
    for (unsigned int i = 0; i < q->M; i++) printf("  bank %3u: \n", i);
}

static void lq_pfb_reset(lq_pfb *q)
{
    lqrt_memset(q->d_win[0], (size_t)q->L * q->esz, q->ctx.stream);
    lqrt_memset(q->d_win[1], (size_t)q->L * q->esz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    memset(q->h_win, 0, (size_t)q->L * q->esz);
    q->host_valid = q->dev_valid = 1;
}

static void lq_pfb_need_host(lq_pfb *q)
{
    if (q->host_valid) return;
    lqrt_d2h(q->h_win, q->d_win[q->cur], (size_t)q->L * q->esz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    q->host_valid = 1;
}

static void lq_pfb_need_dev(lq_pfb *q)
{
    if (q->dev_valid) return;
    lqrt_h2d(q->d_win[q->cur], q->h_win, (size_t)q->L * q->esz, q->ctx.stream);
    q->dev_valid = 1;
}

static void lq_pfb_push(lq_pfb *q, const void *x)
{
    lq_pfb_need_host(q);
    memmove(q->h_win, q->h_win + q->esz, (size_t)(q->L - 1) * q->esz);
    memcpy(q->h_win + (size_t)(q->L - 1) * q->esz, x, q->esz);
    q->dev_valid = 0;
}

static void lq_pfb_execute(lq_pfb *q, unsigned int i, void *y)
{
    if (i >= q->M) LQ_FAIL("error: firpfb_execute(), filterbank index (%u) exceeds maximum (%u)\n", i, q->M);
    const void *win = q->dev_valid ? q->d_win[q->cur] : (const void *)q->h_win;
    unsigned *flag, seq;
    void *py = lq_sig_out(&q->ctx, q->esz, &flag, &seq);
    lqk_firpfb_single(q->kind, q->d_hpoly, q->L, i, win, q->sre, q->sim, py, flag, seq, q->ctx.stream);
    lq_sig_wait(&q->ctx, y, q->esz, seq);
}

static void lq_pfb_block_dev(lq_pfb *q, const void *dx, unsigned long long n, void *dy)
{
    if (n == 0) return;
    lq_pfb_need_dev(q);
    void *wold = q->d_win[q->cur], *wnew = q->d_win[q->cur ^ 1];
    /* bank outputs after each push: the interpolator kernel (y[t*M+i]) with
     * the window's last L-1 samples as history */
    lqk_firinterp(q->kind, q->d_hpoly, q->M, q->L, q->sre, q->sim, (const char *)wold + q->esz, dx, n, dy,
                  q->ctx.stream);
    lqk_window_append(q->kind != LQ_RRRF, wold, q->L, dx, n, wnew, q->ctx.stream);
    q->cur ^= 1;
    q->host_valid = 0;
}

static void lq_pfb_block(lq_pfb *q, const void *x, unsigned long long n, void *y)
{
    if (n == 0) return;
    size_t nin = (size_t)n * q->esz, nout = nin * q->M;
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, nin);
    void *dy = lq_devbuf_get(&q->ybuf, nout);
    lq_pfb_block_dev(q, dx, n, dy);
    lq_call_out(&q->ctx, y, dy, nout);
}

#define LQ_FIRPFB_FRONT(NAME, KIND, TO, TC, TI, SRE, SIM)                                           \
    struct NAME##_s {                                                                               \
        lq_pfb *e;                                                                                  \
    };                                                                                              \
    NAME NAME##_create(unsigned int _M, TC *_h, unsigned int _h_len)                                \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = lq_pfb_create(KIND, _M, (const float *)_h, _h_len);                                  \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_create_kaiser(unsigned int _M, unsigned int _m, float _fc, float _As)               \
    {                                                                                               \
        unsigned int n;                                                                             \
        float *hf = lq_pfb_kaiser(#NAME, _M, _m, _fc, _As, &n);                                     \
        TC *hc = (TC *)lq_xmalloc(n * sizeof(TC));                                                  \
        for (unsigned int i = 0; i < n; i++) hc[i] = (TC)hf[i];                                     \
        NAME q = NAME##_create(_M, hc, n);                                                          \
        free(hf);                                                                                   \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    /* firpfb.c:146-180 (d = 0) and :188-240 (d = 1: derivative bank) */                            \
    NAME NAME##_create_rnyquist(int _type, unsigned int _M, unsigned int _k, unsigned int _m, float _beta)\
    {                                                                                               \
        unsigned int n;                                                                             \
        float *hf = lq_pfb_rnyquist(#NAME, "_create_rnyquist", 0, _type, _M, _k, _m, _beta, &n);    \
        TC *hc = (TC *)lq_xmalloc(n * sizeof(TC));                                                  \
        for (unsigned int i = 0; i < n; i++) hc[i] = (TC)hf[i];                                     \
        NAME q = NAME##_create(_M, hc, n);                                                          \
        free(hf);                                                                                   \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_create_drnyquist(int _type, unsigned int _M, unsigned int _k, unsigned int _m, float _beta)\
    {                                                                                               \
        unsigned int n;                                                                             \
        float *hf = lq_pfb_rnyquist(#NAME, "_create_drnyquist", 1, _type, _M, _k, _m, _beta, &n);   \
        TC *hc = (TC *)lq_xmalloc(n * sizeof(TC));                                                  \
        for (unsigned int i = 0; i < n; i++) hc[i] = (TC)hf[i];                                     \
        NAME q = NAME##_create(_M, hc, n);                                                          \
        free(hf);                                                                                   \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_pfb_destroy(_q->e);                                                                      \
        free(_q);                                                                                   \
    }                                                                                               \
    NAME NAME##_recreate(NAME _q, unsigned int _M, TC *_h, unsigned int _h_len)                     \
    {                                                                                               \
        if (_h_len != _q->e->hlen || _M != _q->e->M) {                                              \
            NAME##_destroy(_q);                                                                     \
            return NAME##_create(_M, _h, _h_len);                                                   \
        }                                                                                           \
        lq_pfb_recoef(_q->e, (const float *)_h);                                                    \
        return _q;                                                                                  \
    }                                                                                               \
    void NAME##_print(NAME _q) { lq_pfb_print(_q->e); }                                             \
    void NAME##_set_scale(NAME _q, TC _g)                                                           \
    {                                                                                               \
        _q->e->sre = SRE;                                                                           \
        _q->e->sim = SIM;                                                                           \
    }                                                                                               \
    void NAME##_reset(NAME _q) { lq_pfb_reset(_q->e); }                                             \
    void NAME##_push(NAME _q, TI _x) { lq_pfb_push(_q->e, &_x); }                                   \
    void NAME##_execute(NAME _q, unsigned int _i, TO *_y) { lq_pfb_execute(_q->e, _i, _y); }         \
    void NAME##_execute_block(NAME _q, TI *_x, unsigned long long _n, TO *_y)                       \
    {                                                                                               \
        lq_pfb_block(_q->e, _x, _n, _y);                                                            \
    }                                                                                               \
    void NAME##_execute_block_dev(NAME _q, const TI *_dx, unsigned long long _n, TO *_dy)           \
    {                                                                                               \
        lq_pfb_block_dev(_q->e, _dx, _n, _dy);                                                      \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ctx_set_stream(&_q->e->ctx, _s); }

LQ_FIRPFB_FRONT(firpfb_rrrf, LQ_RRRF, float, float, float, _g, 0.0f)
LQ_FIRPFB_FRONT(firpfb_crcf, LQ_CRCF, liquid_float_complex, float, liquid_float_complex, _g, 0.0f)
LQ_FIRPFB_FRONT(firpfb_cccf, LQ_CCCF, liquid_float_complex, liquid_float_complex, liquid_float_complex, crealf(_g),
                cimagf(_g))
