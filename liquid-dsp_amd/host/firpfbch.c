/*
 * firpfbch.c -- firpfbch_crcf (critically sampled polyphase channelizer).
 *
 * API include/liquid.h:5667-5739; semantics src/multichannel/src/firpfbch.c:
 *  create        :73-142  type, M > 0 channels, p > 0 taps per branch,
 *                         h has M*p taps; branch i uses h[i + n*M]
 *  create_kaiser :150-184 2*M*m+1 Kaiser taps at fc = 0.5/M, p = 2m
 *  analyzer      :346-409 M inputs -> M channels, forward FFT (analyzer type)
 *  synthesizer   :314-336 M channels -> M outputs, backward FFT
 * The transform direction follows the object's type, as in the reference
 * (the plan is created once per object, firpfbch.c:132-135).
 */
#include "lq_host.h"

struct firpfbch_crcf_s {
    int type;
    unsigned int M, p;
    float *h;
    void *d_hsub;      /* M x p: hsub[i*p + n] = h[i + n*M] */
    void *d_hist[2];   /* analyzer: last (p-1)*M inputs */
    int cur;
    void *d_zstate;    /* synthesizer: last p-1 IFFT vectors */
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf, zbuf;
};

firpfbch_crcf firpfbch_crcf_create(int _type, unsigned int _M, unsigned int _p, float *_h)
{
    if (_type != LIQUID_ANALYZER && _type != LIQUID_SYNTHESIZER)
        LQ_FAIL("error: firpfbch_crcf_create(), invalid type %d\n", _type);
    if (_M == 0) LQ_FAIL("error: firpfbch_crcf_create(), number of channels must be greater than 0\n");
    if (_p == 0) LQ_FAIL("error: firpfbch_crcf_create(), invalid filter size (must be greater than 0)\n");
    lqrt_require_device("firpfbch_crcf_create");
    firpfbch_crcf q = (firpfbch_crcf)lq_xmalloc(sizeof(*q));
    q->type = _type;
    q->M = _M;
    q->p = _p;
    q->h = (float *)lq_xmalloc((size_t)_M * _p * sizeof(float));
    memcpy(q->h, _h, (size_t)_M * _p * sizeof(float));
    float *hsub = (float *)lq_xmalloc((size_t)_M * _p * sizeof(float));
    for (unsigned int i = 0; i < _M; i++)
        for (unsigned int n = 0; n < _p; n++) hsub[i * _p + n] = _h[i + n * _M];
    lq_ctx_init(&q->ctx);
    q->d_hsub = lqrt_malloc((size_t)_M * _p * sizeof(float));
    lqrt_h2d(q->d_hsub, hsub, (size_t)_M * _p * sizeof(float), q->ctx.stream);
    size_t hb = (size_t)(_p - 1) * _M * 8;
    q->d_hist[0] = lqrt_malloc(hb);
    q->d_hist[1] = lqrt_malloc(hb);
    q->d_zstate = lqrt_malloc(hb);
    lqrt_sync(q->ctx.stream);
    free(hsub);
    return q;
}

firpfbch_crcf firpfbch_crcf_create_kaiser(int _type, unsigned int _M, unsigned int _m, float _As)
{
    if (_M == 0) LQ_FAIL("error: firpfbch_crcf_create_kaiser(), number of channels must be greater than 0\n");
    if (_m == 0) LQ_FAIL("error: firpfbch_crcf_create_kaiser(), invalid filter size (must be greater than 0)\n");
    _As = _As < 0 ? -_As : _As;
    unsigned int n = 2 * _M * _m + 1;
    float *h = (float *)lq_xmalloc(n * sizeof(float));
    lq_firdes_kaiser(n, 0.5f / (float)_M, _As, 0.0f, h);
    firpfbch_crcf q = firpfbch_crcf_create(_type, _M, 2 * _m, h);
    free(h);
    return q;
}

void firpfbch_crcf_destroy(firpfbch_crcf _q)
{
    lqrt_sync(_q->ctx.stream);
    lqrt_free(_q->d_hsub);
    lqrt_free(_q->d_hist[0]);
    lqrt_free(_q->d_hist[1]);
    lqrt_free(_q->d_zstate);
    lq_devbuf_free(&_q->xbuf);
    lq_devbuf_free(&_q->ybuf);
    lq_devbuf_free(&_q->zbuf);
    lq_ctx_free(&_q->ctx);
    free(_q->h);
    free(_q);
}

void firpfbch_crcf_reset(firpfbch_crcf _q)
{
    size_t hb = (size_t)(_q->p - 1) * _q->M * 8;
    lqrt_memset(_q->d_hist[0], hb, _q->ctx.stream);
    lqrt_memset(_q->d_hist[1], hb, _q->ctx.stream);
    lqrt_memset(_q->d_zstate, hb, _q->ctx.stream);
    lqrt_sync(_q->ctx.stream);
}

void firpfbch_crcf_print(firpfbch_crcf _q)
{
    printf("firpfbch (%s) [%u channels]:\n", _q->type == LIQUID_ANALYZER ? "analyzer" : "synthesizer", _q->M);
    for (unsigned int i = 0; i < _q->M * _q->p; i++)
        printf("  h[%3u] = %12.8f + %12.8f*j\n", i, _q->h[i], 0.0f);
}

void firpfbch_crcf_execute_block_dev(firpfbch_crcf _q, const liquid_float_complex *_dx,
                                     unsigned long long _nblocks, liquid_float_complex *_dy)
{
    if (_nblocks == 0) return;
    if (_q->type == LIQUID_ANALYZER) {
        void *hold = _q->d_hist[_q->cur], *hnew = _q->d_hist[_q->cur ^ 1];
        const unsigned int HL = (_q->p - 1) * _q->M;
        if (HL) lqk_window_append(1, hold, HL, _dx, _nblocks * _q->M, hnew, _q->ctx.stream);
        lqk_firpfbch_analyzer(_q->M, _q->p, _q->d_hsub, hold, _dx, _nblocks, _dy, _q->ctx.stream);
        if (HL) _q->cur ^= 1;
    } else {
        void *z = lq_devbuf_get(&_q->zbuf, (size_t)(_q->p - 1 + _nblocks) * _q->M * 8);
        lqk_firpfbch_synthesizer(_q->M, _q->p, _q->d_hsub, _q->d_zstate, z, _dx, _nblocks, _dy, _q->ctx.stream);
    }
}

void firpfbch_crcf_execute_block(firpfbch_crcf _q, liquid_float_complex *_x, unsigned long long _nblocks,
                                 liquid_float_complex *_y)
{
    if (_nblocks == 0) return;
    size_t bytes = (size_t)_nblocks * _q->M * 8;
    void *dx = lq_devbuf_get(&_q->xbuf, bytes);
    void *dy = lq_devbuf_get(&_q->ybuf, bytes);
    lqrt_h2d(dx, _x, bytes, _q->ctx.stream);
    firpfbch_crcf_execute_block_dev(_q, (const liquid_float_complex *)dx, _nblocks, (liquid_float_complex *)dy);
    lqrt_d2h(_y, dy, bytes, _q->ctx.stream);
    lqrt_sync(_q->ctx.stream);
}

void firpfbch_crcf_analyzer_execute(firpfbch_crcf _q, liquid_float_complex *_x, liquid_float_complex *_y)
{
    firpfbch_crcf_execute_block(_q, _x, 1, _y);
}

void firpfbch_crcf_synthesizer_execute(firpfbch_crcf _q, liquid_float_complex *_x, liquid_float_complex *_y)
{
    firpfbch_crcf_execute_block(_q, _x, 1, _y);
}

void firpfbch_crcf_set_stream(firpfbch_crcf _q, void *_s) { lq_ctx_set_stream(&_q->ctx, _s); }
