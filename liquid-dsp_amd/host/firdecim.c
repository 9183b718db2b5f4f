/*
 * firdecim.c / firinterp -- firdecim_crcf and firinterp_crcf.
 *
 * firdecim: include/liquid.h:2664-2735, src/filter/src/firdecim.c:47-223.
 *   y[o] = sum_{k<h} h[k] x[o*M - k]: the output is formed right after the
 *   first of each group of M pushes (:195-204); execute_block's _n counts
 *   outputs (:208-223); create_kaiser designs 2Mm+1 taps at fc = 0.5/M and
 *   uses the first 2Mm (:88-122).  No output scale.
 * firinterp: include/liquid.h:2496-2565, src/filter/src/firinterp.c:43-215.
 *   L = ceil(h/M), h' = h zero-padded to M*L, y[i*M + p] =
 *   sum_{l<L} h'[p + l*M] x[i - l]; create needs M >= 2 and h_len >= M.
 */
#include "lq_host.h"

/* ================================================================ firdecim */

struct firdecim_crcf_s {
    unsigned int M, hlen, HP;
    float *h;
    lqk_fir_desc d;
    void *d_hpad;
    void *d_hist[2]; /* last HP-1 inputs */
    int cur;
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf;
};

firdecim_crcf firdecim_crcf_create(unsigned int _M, float *_h, unsigned int _h_len)
{
    if (_h_len == 0) LQ_FAIL("error: decim_crcf_create(), filter length must be greater than zero\n");
    if (_M == 0) LQ_FAIL("error: decim_crcf_create(), decimation factor must be greater than zero\n");
    lqrt_require_device("firdecim_crcf_create");
    firdecim_crcf q = (firdecim_crcf)lq_xmalloc(sizeof(*q));
    q->M = _M;
    q->hlen = _h_len;
    q->HP = _h_len;
    q->h = (float *)lq_xmalloc(_h_len * sizeof(float));
    memcpy(q->h, _h, _h_len * sizeof(float));
    lq_ctx_init(&q->ctx);
    q->d_hpad = lqrt_malloc(_h_len * sizeof(float));
    lqrt_h2d(q->d_hpad, q->h, _h_len * sizeof(float), q->ctx.stream);
    q->d_hist[0] = lqrt_malloc((size_t)_h_len * 8);
    q->d_hist[1] = lqrt_malloc((size_t)_h_len * 8);
    lqrt_sync(q->ctx.stream);
    q->d.kind = LQ_CRCF;
    q->d.hlen = _h_len;
    q->d.hc = _h_len; /* decim kernel takes HP = hc * nchunk directly */
    q->d.nchunk = 1;
    q->d.hpad = q->d_hpad;
    q->d.scale_re = 1.0f;
    q->d.scale_im = 0.0f;
    return q;
}

firdecim_crcf firdecim_crcf_create_kaiser(unsigned int _M, unsigned int _m, float _As)
{
    if (_M < 2) LQ_FAIL("error: decim_crcf_create_kaiser(), decim factor must be greater than 1\n");
    if (_m == 0) LQ_FAIL("error: decim_crcf_create_kaiser(), filter delay must be greater than 0\n");
    if (_As < 0.0f) LQ_FAIL("error: decim_crcf_create_kaiser(), stop-band attenuation must be positive\n");
    unsigned int n = 2 * _M * _m + 1;
    float *hf = (float *)lq_xmalloc(n * sizeof(float));
    lq_firdes_kaiser(n, 0.5f / (float)_M, _As, 0.0f, hf);
    firdecim_crcf q = firdecim_crcf_create(_M, hf, 2 * _M * _m);
    free(hf);
    return q;
}

void firdecim_crcf_destroy(firdecim_crcf _q)
{
    lqrt_sync(_q->ctx.stream);
    lqrt_free(_q->d_hpad);
    lqrt_free(_q->d_hist[0]);
    lqrt_free(_q->d_hist[1]);
    lq_devbuf_free(&_q->xbuf);
    lq_devbuf_free(&_q->ybuf);
    lq_ctx_free(&_q->ctx);
    free(_q->h);
    free(_q);
}

void firdecim_crcf_print(firdecim_crcf _q)
{
    printf("FIRDECIM() [%u] :\n", _q->M);
    for (unsigned int i = 0; i < _q->hlen; i++) printf("  h(%3u) = %12.8f\n", i + 1, _q->h[i]);
}

void firdecim_crcf_clear(firdecim_crcf _q)
{
    lqrt_memset(_q->d_hist[0], (size_t)_q->hlen * 8, _q->ctx.stream);
    lqrt_memset(_q->d_hist[1], (size_t)_q->hlen * 8, _q->ctx.stream);
    lqrt_sync(_q->ctx.stream);
}

void firdecim_crcf_execute_block_dev(firdecim_crcf _q, const liquid_float_complex *_dx, unsigned long long _n,
                                     liquid_float_complex *_dy)
{
    if (_n == 0) return;
    void *hold = _q->d_hist[_q->cur], *hnew = _q->d_hist[_q->cur ^ 1];
    lqk_firdecim(&_q->d, _q->M, hold, _dx, _n, _dy, _q->ctx.stream);
    if (_q->HP > 1) {
        lqk_window_append(1, hold, _q->HP - 1, _dx, _n * _q->M, hnew, _q->ctx.stream);
        _q->cur ^= 1;
    }
}

void firdecim_crcf_execute_block(firdecim_crcf _q, liquid_float_complex *_x, unsigned int _n,
                                 liquid_float_complex *_y)
{
    if (_n == 0) return;
    size_t nin = (size_t)_n * _q->M * 8, nout = (size_t)_n * 8;
    void *dx = lq_devbuf_get(&_q->xbuf, nin);
    void *dy = lq_devbuf_get(&_q->ybuf, nout);
    lqrt_h2d(dx, _x, nin, _q->ctx.stream);
    firdecim_crcf_execute_block_dev(_q, (const liquid_float_complex *)dx, _n, (liquid_float_complex *)dy);
    lqrt_d2h(_y, dy, nout, _q->ctx.stream);
    lqrt_sync(_q->ctx.stream);
}

void firdecim_crcf_execute(firdecim_crcf _q, liquid_float_complex *_x, liquid_float_complex *_y)
{
    firdecim_crcf_execute_block(_q, _x, 1, _y);
}

void firdecim_crcf_set_stream(firdecim_crcf _q, void *_s) { lq_ctx_set_stream(&_q->ctx, _s); }

/* =============================================================== firinterp */

struct firinterp_crcf_s {
    unsigned int M, L, hlen;
    float *h;          /* padded prototype, M*L taps */
    void *d_hpoly;     /* M x L: hpoly[p*L + l] = h'[p + l*M] */
    void *d_hist[2];   /* last L-1 inputs */
    int cur;
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf;
};

firinterp_crcf firinterp_crcf_create(unsigned int _M, float *_h, unsigned int _h_len)
{
    if (_M < 2) LQ_FAIL("error: firinterp_crcf_create(), interp factor must be greater than 1\n");
    if (_h_len < _M) LQ_FAIL("error: firinterp_crcf_create(), filter length cannot be less than interp factor\n");
    lqrt_require_device("firinterp_crcf_create");
    firinterp_crcf q = (firinterp_crcf)lq_xmalloc(sizeof(*q));
    q->M = _M;
    q->L = 0;
    while (_M * q->L < _h_len) q->L++;
    q->hlen = _M * q->L;
    q->h = (float *)lq_xmalloc(q->hlen * sizeof(float));
    for (unsigned int i = 0; i < q->hlen; i++) q->h[i] = i < _h_len ? _h[i] : 0.0f;
    float *hp = (float *)lq_xmalloc(q->hlen * sizeof(float));
    for (unsigned int p = 0; p < _M; p++)
        for (unsigned int l = 0; l < q->L; l++) hp[p * q->L + l] = q->h[p + l * _M];
    lq_ctx_init(&q->ctx);
    q->d_hpoly = lqrt_malloc(q->hlen * sizeof(float));
    lqrt_h2d(q->d_hpoly, hp, q->hlen * sizeof(float), q->ctx.stream);
    q->d_hist[0] = lqrt_malloc((size_t)q->L * 8);
    q->d_hist[1] = lqrt_malloc((size_t)q->L * 8);
    lqrt_sync(q->ctx.stream);
    free(hp);
    return q;
}

firinterp_crcf firinterp_crcf_create_kaiser(unsigned int _M, unsigned int _m, float _As)
{
    if (_M < 2) LQ_FAIL("error: firinterp_crcf_create_kaiser(), interp factor must be greater than 1\n");
    if (_m == 0) LQ_FAIL("error: firinterp_crcf_create_kaiser(), filter delay must be greater than 0\n");
    if (_As < 0.0f) LQ_FAIL("error: firinterp_crcf_create_kaiser(), stop-band attenuation must be positive\n");
    unsigned int n = 2 * _M * _m + 1;
    float *hf = (float *)lq_xmalloc(n * sizeof(float));
    lq_firdes_kaiser(n, 0.5f / (float)_M, _As, 0.0f, hf);
    firinterp_crcf q = firinterp_crcf_create(_M, hf, 2 * _M * _m);
    free(hf);
    return q;
}

void firinterp_crcf_destroy(firinterp_crcf _q)
{
    lqrt_sync(_q->ctx.stream);
    lqrt_free(_q->d_hpoly);
    lqrt_free(_q->d_hist[0]);
    lqrt_free(_q->d_hist[1]);
    lq_devbuf_free(&_q->xbuf);
    lq_devbuf_free(&_q->ybuf);
    lq_ctx_free(&_q->ctx);
    free(_q->h);
    free(_q);
}

void firinterp_crcf_print(firinterp_crcf _q)
{
    printf("interp():\n");
    printf("    M       :   %u\n", _q->M);
    printf("    h_len   :   %u\n", _q->hlen);
}

void firinterp_crcf_reset(firinterp_crcf _q)
{
    lqrt_memset(_q->d_hist[0], (size_t)_q->L * 8, _q->ctx.stream);
    lqrt_memset(_q->d_hist[1], (size_t)_q->L * 8, _q->ctx.stream);
    lqrt_sync(_q->ctx.stream);
}

void firinterp_crcf_execute_block_dev(firinterp_crcf _q, const liquid_float_complex *_dx, unsigned long long _n,
                                      liquid_float_complex *_dy)
{
    if (_n == 0) return;
    void *hold = _q->d_hist[_q->cur], *hnew = _q->d_hist[_q->cur ^ 1];
    lqk_firinterp(LQ_CRCF, _q->d_hpoly, _q->M, _q->L, 1.0f, hold, _dx, _n, _dy, _q->ctx.stream);
    if (_q->L > 1) {
        lqk_window_append(1, hold, _q->L - 1, _dx, _n, hnew, _q->ctx.stream);
        _q->cur ^= 1;
    }
}

void firinterp_crcf_execute_block(firinterp_crcf _q, liquid_float_complex *_x, unsigned int _n,
                                  liquid_float_complex *_y)
{
    if (_n == 0) return;
    size_t nin = (size_t)_n * 8, nout = (size_t)_n * _q->M * 8;
    void *dx = lq_devbuf_get(&_q->xbuf, nin);
    void *dy = lq_devbuf_get(&_q->ybuf, nout);
    lqrt_h2d(dx, _x, nin, _q->ctx.stream);
    firinterp_crcf_execute_block_dev(_q, (const liquid_float_complex *)dx, _n, (liquid_float_complex *)dy);
    lqrt_d2h(_y, dy, nout, _q->ctx.stream);
    lqrt_sync(_q->ctx.stream);
}

void firinterp_crcf_execute(firinterp_crcf _q, liquid_float_complex _x, liquid_float_complex *_y)
{
    firinterp_crcf_execute_block(_q, &_x, 1, _y);
}

void firinterp_crcf_set_stream(firinterp_crcf _q, void *_s) { lq_ctx_set_stream(&_q->ctx, _s); }
