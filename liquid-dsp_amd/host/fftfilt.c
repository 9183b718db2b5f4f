/*
 * fftfilt.c -- fftfilt_{rrrf,crcf,cccf} (FFT fast-convolution filter).
 *
 * API include/liquid.h:2192-2240; semantics src/filter/src/fftfilt.c:69-266:
 * create(h, h_len, n) needs n >= h_len-1 (:78-83); execute() consumes and
 * produces exactly n samples; output = s * (h * x) (causal linear
 * convolution, zero initial state); set_scale(s) (:182-187).
 *
 * The reference evaluates this with a 2n-point overlap-add per call; the
 * kernels (csrc/k_fftfilt.hip) use fixed overlap-save segments, which give
 * the same convolution for any n and let a long stream (execute_block
 * extension) run all segments in parallel: 4096-point segments up to 2049
 * taps (rrrf in the real-I/O form of the kernel; crcf and cccf share the
 * complex form, H the transform of real or complex taps), crcf / cccf
 * 8192-point segments up to 4097 taps.
 *
 * Filters longer than the transforms allow (h_len - 1 > 4096 complex, > 2048
 * rrrf, which the reference accepts for any n >= h_len - 1) run the same
 * convolution as a direct FIR (the firfilt engine, csrc/k_firfilt.hip) on the
 * object's stream: y = s * (h * x) either way, to float32 rounding.
 */
#include <complex.h>

#include "lq_host.h"

static const char *lq_ext[] = {"rrrf", "crcf", "cccf"};

typedef struct {
    int kind;
    size_t esz, csz;
    unsigned int h_len, n;
    unsigned int nfft;  /* segment transform size (lqk_fftfilt_nfft); 0: direct */
    float *h;
    float *hg;          /* reversed, expanded for the host path (lq_host_taps) */
    void *d_h, *d_H;
    void *d_hist[2];    /* previous h_len-1 inputs */
    int cur;
    float sre, sim;     /* user scale s */
    lq_firfilt *direct; /* h_len - 1 > NFFT/2: direct convolution */
    lq_mirror hm;       /* host copy of the history (small-call mode) */
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf, cbuf;
} lq_fftf;

static lq_fftf *lq_fftf_create(int kind, const float *h, unsigned int h_len, unsigned int n)
{
    if (h_len == 0) LQ_FAIL("error: fftfilt_%s_create(), filter length must be greater than zero\n", lq_ext[kind]);
    if (n < h_len - 1)
        LQ_FAIL("error: fftfilt_%s_create(), block length must be greater than _h_len-1 (%u)\n", lq_ext[kind],
                h_len - 1);
    lqrt_require_device("fftfilt_create");
    lq_fftf *q = (lq_fftf *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->esz = kind == LQ_RRRF ? 4 : 8;
    q->csz = kind == LQ_CCCF ? 8 : 4;
    q->h_len = h_len;
    q->n = n;
    q->h = (float *)lq_xmalloc(h_len * q->csz);
    memcpy(q->h, h, h_len * q->csz);
    q->hg = lq_host_taps(kind, q->h, h_len, 1);
    lq_ctx_init(&q->ctx);
    q->d_h = lqrt_malloc(h_len * q->csz);
    q->nfft = lqk_fftfilt_nfft(kind == LQ_RRRF, h_len);
    q->d_H = lqrt_malloc((size_t)(q->nfft ? q->nfft : 1) * 8);
    q->d_hist[0] = lqrt_malloc((size_t)h_len * q->esz);
    q->d_hist[1] = lqrt_malloc((size_t)h_len * q->esz);
    lq_mirror_init(&q->hm, h_len - 1, q->esz);
    lqrt_h2d(q->d_h, q->h, h_len * q->csz, q->ctx.stream);
    if (q->nfft == 0) {
        static const char *who[] = {"fftfilt_rrrf", "fftfilt_crcf", "fftfilt_cccf"};
        q->direct = lq_firfilt_create(kind, h, h_len, who[kind]);
        lq_ctx_set_stream(lq_firfilt_ctx(q->direct), q->ctx.stream);
    } else {
        lqk_fftfilt_make_H(q->d_h, h_len, kind == LQ_CCCF, q->nfft, q->d_H, q->ctx.stream);
    }
    lqrt_sync(q->ctx.stream);
    q->sre = 1.0f;
    q->sim = 0.0f;
    q->cur = 0;
    return q;
}

static void lq_fftf_destroy(lq_fftf *q)
{
    lqrt_sync(q->ctx.stream);
    if (q->direct) lq_firfilt_destroy(q->direct);
    lqrt_free(q->d_h);
    lqrt_free(q->d_H);
    lqrt_free(q->d_hist[0]);
    lqrt_free(q->d_hist[1]);
    lq_mirror_free(&q->hm);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_devbuf_free(&q->cbuf);
    lq_ctx_free(&q->ctx);
    free(q->h);
    free(q->hg);
    free(q);
}

static void lq_fftf_reset(lq_fftf *q)
{
    lqrt_memset(q->d_hist[0], (size_t)q->h_len * q->esz, q->ctx.stream);
    lqrt_memset(q->d_hist[1], (size_t)q->h_len * q->esz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    lq_mirror_zero(&q->hm);
    if (q->direct) lq_firfilt_reset(q->direct);
}

static void lq_fftf_print(lq_fftf *q)
{
    printf("fftfilt_%s: [h_len=%u, n=%u]\n", lq_ext[q->kind], q->h_len, q->n);
    for (unsigned int i = 0; i < q->h_len; i++) {
        const unsigned int k = q->h_len - i - 1;
        if (q->kind == LQ_CCCF) printf("  h(%3u) = %12.8f + j*%12.8f\n", i + 1, q->h[2 * k], q->h[2 * k + 1]);
        else printf("  h(%3u) = %12.8f\n", i + 1, q->h[k]);
    }
    printf("  scale = %12.8f\n", q->sre / (float)(2 * q->n));
}

static void lq_fftf_block_dev(lq_fftf *q, const void *dx, unsigned long long n, void *dy)
{
    if (n == 0) return;
    if (q->direct) {
        lq_firfilt_set_scale(q->direct, q->sre, q->sim);
        lq_firfilt_execute_block_dev(q->direct, dx, n, dy);
        return;
    }
    lq_mirror_need_dev(&q->hm, q->d_hist[q->cur], q->ctx.stream);
    q->hm.host_valid = 0;
    const void *x = dx;
    if (dx == dy) { /* kernel segments read overlapping halos */
        void *c = lq_devbuf_get(&q->cbuf, (size_t)n * q->esz);
        lqrt_d2d(c, dx, (size_t)n * q->esz, q->ctx.stream);
        x = c;
    }
    const unsigned int hm1 = q->h_len - 1;
    void *hold = q->d_hist[q->cur], *hnew = q->d_hist[q->cur ^ 1];
    /* the transform kernel also writes the next history (no launch of its own) */
    const lqk_hist_job job = {hold, x, n, hnew, hm1};
    lqk_fftfilt_run(q->kind == LQ_RRRF, q->h_len, q->nfft, q->d_H, hold, x, n, dy, q->sre, q->sim, NULL, 0, NULL,
                    hm1 ? &job : NULL, q->ctx.stream);
    if (hm1) q->cur ^= 1;
}

/* small-call mode: one short call (n h_len <= LQ_FFTF_HOST_MACS) on the host
 * as the direct convolution it equals, y[t] = s sum_k h[k] x[t - k] over the
 * history and the call's samples (fftfilt.c:193-260 computes the same sum by
 * a 2n-point overlap-add; the results agree to float32 rounding) */
#define LQ_FFTF_HOST_MACS 65536u
static void lq_fftf_exec_host(lq_fftf *q, const void *x, unsigned int n, void *y)
{
    lq_mirror_need_host(&q->hm, q->d_hist[q->cur], q->ctx.stream);
    lq_mirror_append(&q->hm, x, n);
    const unsigned char *w = lq_mirror_ptr(&q->hm);
    for (unsigned int t = 0; t < n; t++) {
        float *yt = (float *)((unsigned char *)y + (size_t)t * q->esz);
        /* window samples t .. t + h_len - 1 (oldest first) against the reversed taps */
        lq_host_tdot(q->kind, q->hg, w + (size_t)t * q->esz, q->h_len, yt);
        if (q->kind == LQ_RRRF) {
            yt[0] *= q->sre;
        } else if (q->kind == LQ_CRCF) {   /* real scale per component */
            yt[0] *= q->sre;
            yt[1] *= q->sre;
        } else {                           /* complex scale */
            const float a = yt[0], b = yt[1];
            yt[0] = a * q->sre - b * q->sim;
            yt[1] = a * q->sim + b * q->sre;
        }
    }
    lq_mirror_commit(&q->hm, n);
}

/* single: the call is fftfilt_*_execute (the reference's one n-sample block);
 * the execute_block extension always runs on the GPU */
static void lq_fftf_block(lq_fftf *q, const void *x, unsigned long long n, void *y, int single)
{
    if (n == 0) return;
    if (single && lq_small_host() && !q->direct && n * (unsigned long long)q->h_len <= LQ_FFTF_HOST_MACS) {
        lq_fftf_exec_host(q, x, (unsigned int)n, y);
        return;
    }
    size_t bytes = (size_t)n * q->esz;
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, bytes);
    void *dy = lq_devbuf_get(&q->ybuf, bytes);
    lq_fftf_block_dev(q, dx, n, dy);
    lq_call_out(&q->ctx, y, dy, bytes);
}

#define LQ_FFTFILT_FRONT(NAME, KIND, TO, TC, TI, SRE, SIM)                                          \
    struct NAME##_s {                                                                               \
        lq_fftf *e;                                                                                 \
    };                                                                                              \
    NAME NAME##_create(TC *_h, unsigned int _h_len, unsigned int _n)                                \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = lq_fftf_create(KIND, (const float *)_h, _h_len, _n);                                 \
        return q;                                                                                   \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_fftf_destroy(_q->e);                                                                     \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_reset(NAME _q) { lq_fftf_reset(_q->e); }                                            \
    void NAME##_print(NAME _q) { lq_fftf_print(_q->e); }                                            \
    void NAME##_set_scale(NAME _q, TC _scale)                                                       \
    {                                                                                               \
        _q->e->sre = SRE;                                                                           \
        _q->e->sim = SIM;                                                                           \
    }                                                                                               \
    unsigned int NAME##_get_length(NAME _q) { return _q->e->h_len; }                                \
    /* fftfilt.c:193-260: exactly n samples in and out */                                           \
    void NAME##_execute(NAME _q, TI *_x, TO *_y) { lq_fftf_block(_q->e, _x, _q->e->n, _y, 1); }       \
    void NAME##_execute_block(NAME _q, TI *_x, unsigned long long _n, TO *_y)                       \
    {                                                                                               \
        lq_fftf_block(_q->e, _x, _n, _y, 0);                                                        \
    }                                                                                               \
    void NAME##_execute_block_dev(NAME _q, const TI *_dx, unsigned long long _n, TO *_dy)           \
    {                                                                                               \
        lq_fftf_block_dev(_q->e, _dx, _n, _dy);                                                     \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s)                                                       \
    {                                                                                               \
        lq_ctx_set_stream(&_q->e->ctx, _s);                                                         \
        if (_q->e->direct) lq_ctx_set_stream(lq_firfilt_ctx(_q->e->direct), _q->e->ctx.stream);      \
    }

LQ_FFTFILT_FRONT(fftfilt_rrrf, LQ_RRRF, float, float, float, _scale, 0.0f)
LQ_FFTFILT_FRONT(fftfilt_crcf, LQ_CRCF, liquid_float_complex, float, liquid_float_complex, _scale, 0.0f)
LQ_FFTFILT_FRONT(fftfilt_cccf, LQ_CCCF, liquid_float_complex, liquid_float_complex, liquid_float_complex,
                 crealf(_scale), cimagf(_scale))
