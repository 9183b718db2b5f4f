/*
 * firpfbch2.c -- firpfbch2_crcf (2x oversampled polyphase channelizer).
 *
 * API include/liquid.h:5754-5799; semantics src/multichannel/src/firpfbch2.c.
 *  create        :66-132  M even >= 2, m >= 1, prototype taps h[i + n*M]
 *                         for i < M, n < 2m (2*M*m coefficients used)
 *  create_kaiser :135-183 2*M*m+1 Kaiser taps, fc = 1/M (analyzer) or 0.5/M,
 *                         normalised to sum M, first 2*M*m used
 *  analyzer      :244-282 M/2 inputs -> M channel outputs per call
 *  synthesizer   :287-335 M channel inputs -> M/2 outputs per call
 *
 * GPU state: analyzer = last 2mM - M/2 input samples (ping-pong) and the
 * block parity (the reference's `flag`); synthesizer = last 4m-1 IFFT
 * vectors and the parity.  See csrc/k_channelizer.hip for the closed forms.
 */
#include "lq_host.h"

struct firpfbch2_crcf_s {
    int type;
    unsigned int M, m, HL;
    float *h;          /* 2*M*m prototype taps */
    void *d_hsub;      /* M x 2m: hsub[i*2m + n] = h[i + n*M] */
    void *d_hsub_s;    /* analyzer: hsub / M (exact for M = 2^k), the fast path's form */
    void *d_hist[2];   /* analyzer: last HL inputs */
    int cur;
    void *d_zstate;    /* synthesizer: last 4m-1 IFFT vectors */
    int flag;          /* parity of the next block (reference `flag`) */
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf, zbuf;
};

static void firpfbch2_validate(int type, unsigned int M, unsigned int m, const char *who)
{
    if (type != LIQUID_ANALYZER && type != LIQUID_SYNTHESIZER)
        LQ_FAIL("error: firpfbch2_crcf_%s(), invalid type %d\n", who, type);
    if (M < 2 || M % 2)
        LQ_FAIL("error: firpfbch2_crcf_%s(), number of channels must be greater than 2 and even\n", who);
    if (m < 1) LQ_FAIL("error: firpfbch2_crcf_%s(), filter semi-length must be at least 1\n", who);
}

firpfbch2_crcf firpfbch2_crcf_create(int _type, unsigned int _M, unsigned int _m, float *_h)
{
    firpfbch2_validate(_type, _M, _m, "create");
    lqrt_require_device("firpfbch2_crcf_create");
    firpfbch2_crcf q = (firpfbch2_crcf)lq_xmalloc(sizeof(*q));
    q->type = _type;
    q->M = _M;
    q->m = _m;
    q->HL = 2 * _m * _M - _M / 2;
    unsigned int L = 2 * _m, hl = 2 * _M * _m;
    q->h = (float *)lq_xmalloc(hl * sizeof(float));
    memcpy(q->h, _h, hl * sizeof(float));
    float *hsub = (float *)lq_xmalloc((size_t)_M * L * sizeof(float));
    for (unsigned int i = 0; i < _M; i++)
        for (unsigned int n = 0; n < L; n++) hsub[i * L + n] = _h[i + n * _M];
    lq_ctx_init(&q->ctx);
    q->d_hsub = lqrt_malloc((size_t)_M * L * sizeof(float));
    lqrt_h2d(q->d_hsub, hsub, (size_t)_M * L * sizeof(float), q->ctx.stream);
    if (_type == LIQUID_ANALYZER) {
        /* the output scale 1/M folded into the taps: a power of two, so every
         * product and partial sum scales exactly and the results are unchanged */
        const float inv = 1.0f / (float)_M;
        for (size_t i = 0; i < (size_t)_M * L; i++) hsub[i] *= inv;
        q->d_hsub_s = lqrt_malloc((size_t)_M * L * sizeof(float));
        lqrt_h2d(q->d_hsub_s, hsub, (size_t)_M * L * sizeof(float), q->ctx.stream);
        q->d_hist[0] = lqrt_malloc((size_t)q->HL * 8);
        q->d_hist[1] = lqrt_malloc((size_t)q->HL * 8);
    } else {
        q->d_zstate = lqrt_malloc((size_t)(4 * _m - 1) * _M * 8);
    }
    lqrt_sync(q->ctx.stream);
    free(hsub);
    q->cur = 0;
    q->flag = 0;
    return q;
}

firpfbch2_crcf firpfbch2_crcf_create_kaiser(int _type, unsigned int _M, unsigned int _m, float _As)
{
    firpfbch2_validate(_type, _M, _m, "create_kaiser");
    unsigned int n = 2 * _M * _m + 1;
    float *hf = (float *)lq_xmalloc(n * sizeof(float));
    float fc = (_type == LIQUID_ANALYZER) ? 1.0f / (float)_M : 0.5f / (float)_M;
    lq_firdes_kaiser(n, fc, _As, 0.0f, hf);
    float s = 0.0f;
    for (unsigned int i = 0; i < n; i++) s += hf[i];
    for (unsigned int i = 0; i < n; i++) hf[i] = hf[i] * (float)_M / s;
    firpfbch2_crcf q = firpfbch2_crcf_create(_type, _M, _m, hf);
    free(hf);
    return q;
}

void firpfbch2_crcf_destroy(firpfbch2_crcf _q)
{
    lqrt_sync(_q->ctx.stream);
    lqrt_free(_q->d_hsub);
    lqrt_free(_q->d_hsub_s);
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

void firpfbch2_crcf_reset(firpfbch2_crcf _q)
{
    if (_q->type == LIQUID_ANALYZER) {
        lqrt_memset(_q->d_hist[0], (size_t)_q->HL * 8, _q->ctx.stream);
        lqrt_memset(_q->d_hist[1], (size_t)_q->HL * 8, _q->ctx.stream);
    } else {
        lqrt_memset(_q->d_zstate, (size_t)(4 * _q->m - 1) * _q->M * 8, _q->ctx.stream);
    }
    lqrt_sync(_q->ctx.stream);
    _q->flag = 0;
}

void firpfbch2_crcf_print(firpfbch2_crcf _q)
{
    printf("firpfbch2_crcf:\n");
    printf("    channels    :   %u\n", _q->M);
    printf("    h_len       :   %u\n", 2 * _q->M * _q->m);
    printf("    semi-length :   %u\n", _q->m);
}

/* the analyzer on the fast kernel (M = 1024), which also writes the next
 * history; flag (NULL: none): y is pinned host memory and the kernel raises
 * the call's completion flag.  0: not handled, nothing launched */
static int firpfbch2_an_fast(firpfbch2_crcf _q, const void *_dx, unsigned long long _nblocks, void *_dy,
                             unsigned *flag, unsigned seq)
{
    void *hold = _q->d_hist[_q->cur], *hnew = _q->d_hist[_q->cur ^ 1];
    const lqk_hist_job job = {hold, _dx, _nblocks * (_q->M / 2), hnew, _q->HL};
    if (!lqk_firpfbch2_analyzer_fast(_q->M, _q->m, _q->d_hsub_s, hold, _dx, _nblocks, _q->flag, _dy, &job, flag, seq,
                                     _q->ctx.stream))
        return 0;
    _q->cur ^= 1;
    _q->flag = (int)((_q->flag + _nblocks) & 1);
    return 1;
}

void firpfbch2_crcf_execute_block_dev(firpfbch2_crcf _q, const liquid_float_complex *_dx,
                                      unsigned long long _nblocks, liquid_float_complex *_dy)
{
    if (_nblocks == 0) return;
    if (_q->type == LIQUID_ANALYZER) {
        if (firpfbch2_an_fast(_q, _dx, _nblocks, _dy, NULL, 0)) return;
        void *hold = _q->d_hist[_q->cur], *hnew = _q->d_hist[_q->cur ^ 1];
        lqk_firpfbch2_analyzer(_q->M, _q->m, _q->d_hsub, hold, _dx, _nblocks, _q->flag, _dy, _q->ctx.stream);
        lqk_window_append(1, hold, _q->HL, _dx, _nblocks * (_q->M / 2), hnew, _q->ctx.stream);
        _q->cur ^= 1;
    } else {
        size_t zb = (size_t)(4 * _q->m - 1 + _nblocks) * _q->M * 8;
        void *z = lq_devbuf_get(&_q->zbuf, zb);
        lqk_firpfbch2_synthesizer(_q->M, _q->m, _q->d_hsub, _q->d_zstate, z, _dx, _nblocks, _q->flag, _dy,
                                  _q->ctx.stream);
    }
    _q->flag = (int)((_q->flag + _nblocks) & 1);
}

void firpfbch2_crcf_execute_block(firpfbch2_crcf _q, liquid_float_complex *_x, unsigned long long _nblocks,
                                  liquid_float_complex *_y)
{
    if (_nblocks == 0) return;
    size_t nin = (size_t)_nblocks * (_q->type == LIQUID_ANALYZER ? _q->M / 2 : _q->M);
    size_t nout = (size_t)_nblocks * (_q->type == LIQUID_ANALYZER ? _q->M : _q->M / 2);
    const void *dx = lq_call_in(&_q->ctx, &_q->xbuf, _x, nin * 8);
    if (_q->type == LIQUID_ANALYZER && nout * 8 <= LQRT_COPYOUT_MAX) {
        /* a few blocks (the reference's execute() is one): the kernel writes
         * the pinned output buffer and raises the completion flag itself --
         * one launch per call, no copy-out kernel */
        unsigned *flag, seq;
        void *py = lq_sig_out(&_q->ctx, nout * 8, &flag, &seq);
        if (firpfbch2_an_fast(_q, dx, _nblocks, py, flag, seq)) {
            lq_sig_wait(&_q->ctx, _y, nout * 8, seq);
            return;
        }
    }
    void *dy = lq_devbuf_get(&_q->ybuf, nout * 8);
    firpfbch2_crcf_execute_block_dev(_q, (const liquid_float_complex *)dx, _nblocks, (liquid_float_complex *)dy);
    lq_call_out(&_q->ctx, _y, dy, nout * 8);
}

/* firpfbch2.c:342-357: one block (the reference's only execute form) */
void firpfbch2_crcf_execute(firpfbch2_crcf _q, liquid_float_complex *_x, liquid_float_complex *_y)
{
    firpfbch2_crcf_execute_block(_q, _x, 1, _y);
}

void firpfbch2_crcf_set_stream(firpfbch2_crcf _q, void *_s) { lq_ctx_set_stream(&_q->ctx, _s); }
void *firpfbch2_crcf_get_stream(firpfbch2_crcf _q) { return _q->ctx.stream; }
void firpfbch2_crcf_synchronize(firpfbch2_crcf _q) { lqrt_sync(_q->ctx.stream); }
