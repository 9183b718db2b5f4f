/*
 * fftfilt.c -- fftfilt_crcf (FFT fast-convolution filter).
 *
 * API include/liquid.h:2192-2240; semantics src/filter/src/fftfilt.c:69-266:
 * create(h, h_len, n) needs n >= h_len-1 (:78-83); execute() consumes and
 * produces exactly n samples; output = s * (h * x) (causal linear
 * convolution, zero initial state); set_scale(s) (:182-187).
 *
 * The reference evaluates this with a 2n-point overlap-add per call; the
 * kernel (csrc/k_fftfilt.hip) uses fixed 4096-point overlap-save segments,
 * which gives the same convolution for any n and lets a long stream
 * (execute_block extension) run all segments in parallel.
 */
#include "lq_host.h"

struct fftfilt_crcf_s {
    unsigned int h_len, n;
    float *h;
    void *d_h, *d_H;
    void *d_hist[2];    /* previous h_len-1 inputs */
    int cur;
    float scale;        /* user scale s */
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf, cbuf;
};

fftfilt_crcf fftfilt_crcf_create(float *_h, unsigned int _h_len, unsigned int _n)
{
    if (_h_len == 0) LQ_FAIL("error: fftfilt_crcf_create(), filter length must be greater than zero\n");
    if (_n < _h_len - 1)
        LQ_FAIL("error: fftfilt_crcf_create(), block length must be greater than _h_len-1 (%u)\n", _h_len - 1);
    lqrt_require_device("fftfilt_crcf_create");
    if (_h_len - 1 > lqk_fftfilt_nfft() / 2)
        LQ_FAIL("error: fftfilt_crcf_create(), filter length %u exceeds the GPU limit %u\n", _h_len,
                lqk_fftfilt_nfft() / 2 + 1);
    fftfilt_crcf q = (fftfilt_crcf)lq_xmalloc(sizeof(*q));
    q->h_len = _h_len;
    q->n = _n;
    q->h = (float *)lq_xmalloc(_h_len * sizeof(float));
    memcpy(q->h, _h, _h_len * sizeof(float));
    lq_ctx_init(&q->ctx);
    q->d_h = lqrt_malloc(_h_len * sizeof(float));
    q->d_H = lqrt_malloc((size_t)lqk_fftfilt_nfft() * 8);
    q->d_hist[0] = lqrt_malloc((size_t)(_h_len) * 8);
    q->d_hist[1] = lqrt_malloc((size_t)(_h_len) * 8);
    lqrt_h2d(q->d_h, q->h, _h_len * sizeof(float), q->ctx.stream);
    lqk_fftfilt_make_H(q->d_h, _h_len, 0, q->d_H, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    q->scale = 1.0f;
    q->cur = 0;
    return q;
}

void fftfilt_crcf_destroy(fftfilt_crcf _q)
{
    lqrt_sync(_q->ctx.stream);
    lqrt_free(_q->d_h);
    lqrt_free(_q->d_H);
    lqrt_free(_q->d_hist[0]);
    lqrt_free(_q->d_hist[1]);
    lq_devbuf_free(&_q->xbuf);
    lq_devbuf_free(&_q->ybuf);
    lq_devbuf_free(&_q->cbuf);
    lq_ctx_free(&_q->ctx);
    free(_q->h);
    free(_q);
}

void fftfilt_crcf_reset(fftfilt_crcf _q)
{
    lqrt_memset(_q->d_hist[0], (size_t)_q->h_len * 8, _q->ctx.stream);
    lqrt_memset(_q->d_hist[1], (size_t)_q->h_len * 8, _q->ctx.stream);
    lqrt_sync(_q->ctx.stream);
}

void fftfilt_crcf_print(fftfilt_crcf _q)
{
    printf("fftfilt_crcf: [h_len=%u, n=%u]\n", _q->h_len, _q->n);
    for (unsigned int i = 0; i < _q->h_len; i++) printf("  h(%3u) = %12.8f\n", i + 1, _q->h[_q->h_len - i - 1]);
    printf("  scale = %12.8f\n", _q->scale / (float)(2 * _q->n));
}

void fftfilt_crcf_set_scale(fftfilt_crcf _q, float _scale) { _q->scale = _scale; }

unsigned int fftfilt_crcf_get_length(fftfilt_crcf _q) { return _q->h_len; }

void fftfilt_crcf_execute_block_dev(fftfilt_crcf _q, const liquid_float_complex *_dx, unsigned long long _n,
                                    liquid_float_complex *_dy)
{
    if (_n == 0) return;
    const void *x = _dx;
    if ((const void *)_dx == (const void *)_dy) { /* kernel segments read overlapping halos */
        void *c = lq_devbuf_get(&_q->cbuf, (size_t)_n * 8);
        lqrt_d2d(c, _dx, (size_t)_n * 8, _q->ctx.stream);
        x = c;
    }
    const unsigned int hm1 = _q->h_len - 1;
    void *hold = _q->d_hist[_q->cur], *hnew = _q->d_hist[_q->cur ^ 1];
    const float s = _q->scale / (float)lqk_fftfilt_nfft();
    lqk_fftfilt_run(0, _q->h_len, _q->d_H, hold, x, _n, _dy, s, 0.0f, _q->ctx.stream);
    if (hm1) {
        lqk_window_append(1, hold, hm1, x, _n, hnew, _q->ctx.stream);
        _q->cur ^= 1;
    }
}

void fftfilt_crcf_execute_block(fftfilt_crcf _q, liquid_float_complex *_x, unsigned long long _n,
                                liquid_float_complex *_y)
{
    if (_n == 0) return;
    size_t bytes = (size_t)_n * 8;
    void *dx = lq_devbuf_get(&_q->xbuf, bytes);
    void *dy = lq_devbuf_get(&_q->ybuf, bytes);
    lqrt_h2d(dx, _x, bytes, _q->ctx.stream);
    fftfilt_crcf_execute_block_dev(_q, (const liquid_float_complex *)dx, _n, (liquid_float_complex *)dy);
    lqrt_d2h(_y, dy, bytes, _q->ctx.stream);
    lqrt_sync(_q->ctx.stream);
}

/* fftfilt.c:193-260: exactly n samples in and out */
void fftfilt_crcf_execute(fftfilt_crcf _q, liquid_float_complex *_x, liquid_float_complex *_y)
{
    fftfilt_crcf_execute_block(_q, _x, _q->n, _y);
}

void fftfilt_crcf_set_stream(fftfilt_crcf _q, void *_s) { lq_ctx_set_stream(&_q->ctx, _s); }
