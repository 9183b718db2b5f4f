/*
 * firfilt.c -- firfilt_{rrrf,crcf,cccf} on the MI355X.
 *
 * API and semantics: include/liquid.h:1985-2090, src/filter/src/firfilt.c:62-404
 *   y[t] = scale * sum_{k<h} h[k] x[t-k], zero initial history;
 *   push() appends one sample, execute() reads the current window without
 *   pushing, execute_block() = push+execute per sample (in place allowed).
 *
 * State model.  The filter state is the window of the last HP samples
 * (HP = length padded to the kernel's chunk class), oldest first, kept on
 * the device (two ping-pong buffers) with a host mirror for the per-sample
 * push() path.  Exactly one copy is authoritative at a time; the other is
 * refreshed lazily.  Every output sample, including the per-sample
 * execute(), is computed by a HIP kernel.
 */
#include <complex.h>
#include <math.h>

#include "lq_host.h"

struct lq_firfilt_s {
    int kind;
    unsigned int hlen, HP;
    size_t esz;        /* sample size: 4 (rrrf) or 8 */
    size_t csz;        /* coefficient size: 4 or 8 (cccf) */
    float *h;          /* natural-order coefficients (host copy) */
    float *hg;         /* reversed, expanded for the host path (lq_host_taps) */
    void *d_hpad;      /* device, zero padded to HP */
    lqk_fir_desc d;
    void *d_win[2];    /* device windows, HP samples each */
    void *d_H8;        /* long complex filters: the overlap-save path's spectrum (else NULL) */
    unsigned int fft_n; /* its transform size (lqk_fftfilt_nfft) */
    int cur;
    unsigned char *h_win; /* host mirror: the window is HP samples at h_win + hoff * esz, */
    size_t hoff;          /* pushes append after it (capacity LQ_FIR_HCAP windows) */
    int host_valid, dev_valid;
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf, scratch, one, flags;
    const char *who;   /* the public object name, for error messages */
};

/* longer complex filters take the overlap-save path (crcf past 128 taps: at
 * 65..128 the matrix-core band is as fast, 0.49-0.50 vs 0.51 ms per 2^27
 * samples at h = 128; cccf past 64, where its matrix-core kernel stops) ... */
#define LQ_FIR_HCAP 8   /* host window buffer, in windows: a memmove every 7 HP pushes */
#define LQ_FIR_FFT_MIN_TAPS(kind) ((kind) == LQ_CRCF ? 128u : 64u)
#define LQ_FIR_FFT_MIN_N 8192ull    /* ... on device blocks of at least this many samples */

static void lq_firfilt_layout(lq_firfilt *q, unsigned int n)
{
    q->hlen = n;
    if (n <= 16) {
        q->d.hc = 16;
        q->d.nchunk = 1;
    } else if (n <= 32) {
        q->d.hc = 32;
        q->d.nchunk = 1;
    } else {
        q->d.hc = 64;
        q->d.nchunk = (n + 63) / 64;
    }
    q->HP = q->d.hc * q->d.nchunk;
    q->d.hlen = n;
    /* the direct kernel holds a tile plus the HP-sample history in LDS:
       refuse at create time what no launch could run (fftfilt's long-filter
       path lands here too) */
    if (q->HP > lqk_firfilt_max_history(q->d.kind))
        LQ_FAIL("error: %s_create(), filter length %u exceeds the GPU kernel limit of %u taps\n", q->who, n,
                lqk_firfilt_max_history(q->d.kind));
}

static void lq_firfilt_alloc_state(lq_firfilt *q)
{
    q->d_hpad = lqrt_malloc((size_t)q->HP * q->csz);
    q->d_H8 = NULL;
    q->d_win[0] = lqrt_malloc((size_t)q->HP * q->esz);
    q->d_win[1] = lqrt_malloc((size_t)q->HP * q->esz);
    /* pinned: the per-sample execute() reads it in place (zero copy) */
    q->h_win = (unsigned char *)lqrt_host_alloc((size_t)LQ_FIR_HCAP * q->HP * q->esz);
    memset(q->h_win, 0, (size_t)q->HP * q->esz);
    q->hoff = 0;
    q->cur = 0;
    q->host_valid = q->dev_valid = 1;
}

static void lq_firfilt_free_state(lq_firfilt *q)
{
    if (q->d_H8) lqrt_free(q->d_H8);
    q->d_H8 = NULL;
    lqrt_free(q->d_hpad);
    lqrt_free(q->d_win[0]);
    lqrt_free(q->d_win[1]);
    lqrt_host_free(q->h_win);
}

static void lq_firfilt_upload_coefs(lq_firfilt *q)
{
    size_t bytes = (size_t)q->HP * q->csz;
    unsigned char *pad = (unsigned char *)lq_xmalloc(bytes);
    memcpy(pad, q->h, (size_t)q->hlen * q->csz);
    lqrt_h2d(q->d_hpad, pad, bytes, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    free(pad);
    q->d.hpad = q->d_hpad;
    /* the matrix-core kernel splits taps into three bf16 terms; outside
     * [2^-50, 2^50] (or non-finite) the split would lose float32 accuracy or
     * the reference's Inf/NaN propagation, so such filters stay on the VALU
     * kernel */
    const unsigned int nv = q->hlen * (unsigned int)(q->csz / sizeof(float));
    q->d.mx_ok = 1;
    for (unsigned int i = 0; i < nv; i++) {
        const float a = fabsf(q->h[i]);
        if (!(a <= 0x1p50f) || (a != 0.0f && a < 0x1p-50f)) q->d.mx_ok = 0;
    }
    const int fft_ok = q->d.mx_ok;   /* the same tap class for the transform path */
    /* complex streams through long filters (crcf / cccf, more than
     * LQ_FIR_FFT_MIN_TAPS taps): the same convolution by 4096-point (8192
     * past 2049 taps) overlap-save segments (csrc/k_fftfilt.hip, the guarded
     * form: segments
     * with non-finite, huge or tiny inputs fall back to the direct sum) -- HBM-bound
     * where the direct kernels are bound by their arithmetic (crcf h = 256:
     * six bf16 matrix products per tap; cccf past 64 taps: the VALU kernel) */
    if (q->d_H8) lqrt_free(q->d_H8);
    q->d_H8 = NULL;
    q->fft_n = lqk_fftfilt_nfft(0, q->hlen);
    if (q->kind != LQ_RRRF && q->hlen > LQ_FIR_FFT_MIN_TAPS(q->kind) && fft_ok && q->fft_n) {
        q->d_H8 = lqrt_malloc((size_t)q->fft_n * 8);
        lqk_fftfilt_make_H(q->d_hpad, q->hlen, q->kind == LQ_CCCF, q->fft_n, q->d_H8, q->ctx.stream);
        lqrt_sync(q->ctx.stream);
    }
}

lq_firfilt *lq_firfilt_create(int kind, const float *h, unsigned int n, const char *who)
{
    if (n == 0) LQ_FAIL("error: %s_create(), filter length must be greater than zero\n", who);
    lqrt_require_device(who);
    lq_firfilt *q = (lq_firfilt *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->esz = kind == LQ_RRRF ? sizeof(float) : 2 * sizeof(float);
    q->csz = kind == LQ_CCCF ? 2 * sizeof(float) : sizeof(float);
    q->d.kind = kind;
    q->d.scale_re = 1.0f;
    q->d.scale_im = 0.0f;
    q->who = who;
    lq_firfilt_layout(q, n);
    q->h = (float *)lq_xmalloc((size_t)n * q->csz);
    memcpy(q->h, h, (size_t)n * q->csz);
    q->hg = lq_host_taps(kind, q->h, n, 1);
    lq_ctx_init(&q->ctx);
    lq_firfilt_alloc_state(q);
    lq_firfilt_upload_coefs(q);
    return q;
}

/* src/filter/src/firfilt.c:201-237: new taps; a length change restarts the
 * buffer (the reference leaves it uninitialised; here it is cleared) */
lq_firfilt *lq_firfilt_recreate(lq_firfilt *q, const float *h, unsigned int n)
{
    if (n == 0) LQ_FAIL("error: firfilt_recreate(), filter length must be greater than zero\n");
    lqrt_sync(q->ctx.stream);
    if (n != q->hlen) {
        lq_firfilt_free_state(q);
        lq_firfilt_layout(q, n);
        free(q->h);
        q->h = (float *)lq_xmalloc((size_t)n * q->csz);
        lq_firfilt_alloc_state(q);
    }
    memcpy(q->h, h, (size_t)n * q->csz);
    free(q->hg);
    q->hg = lq_host_taps(q->kind, q->h, n, 1);
    lq_firfilt_upload_coefs(q);
    return q;
}

void lq_firfilt_destroy(lq_firfilt *q)
{
    lqrt_sync(q->ctx.stream);
    lq_firfilt_free_state(q);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_devbuf_free(&q->scratch);
    lq_devbuf_free(&q->one);
    lq_devbuf_free(&q->flags);
    lq_ctx_free(&q->ctx);
    free(q->h);
    free(q->hg);
    free(q);
}

void lq_firfilt_reset(lq_firfilt *q)
{
    lqrt_memset(q->d_win[0], (size_t)q->HP * q->esz, q->ctx.stream);
    lqrt_memset(q->d_win[1], (size_t)q->HP * q->esz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    q->hoff = 0;
    memset(q->h_win, 0, (size_t)q->HP * q->esz);
    q->host_valid = q->dev_valid = 1;
}

void lq_firfilt_print(lq_firfilt *q)
{
    static const char *ext[] = {"rrrf", "crcf", "cccf"};
    printf("firfilt_%s:\n", ext[q->kind]);
    for (unsigned int i = 0; i < q->hlen; i++) {
        if (q->kind == LQ_CCCF)
            printf("  h(%3u) = %12.8f + j*%12.8f\n", i + 1, q->h[2 * i], q->h[2 * i + 1]);
        else
            printf("  h(%3u) = %12.8f\n", i + 1, q->h[i]);
    }
    if (q->kind == LQ_CCCF)
        printf("  scale = %12.8f + j*%12.8f\n", q->d.scale_re, q->d.scale_im);
    else
        printf("  scale = %12.8f\n", q->d.scale_re);
}

void lq_firfilt_set_scale(lq_firfilt *q, float re, float im)
{
    q->d.scale_re = re;
    q->d.scale_im = im;
}

static void lq_firfilt_need_host(lq_firfilt *q)
{
    if (q->host_valid) return;
    q->hoff = 0;
    lqrt_d2h(q->h_win, q->d_win[q->cur], (size_t)q->HP * q->esz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    q->host_valid = 1;
}

static void lq_firfilt_need_dev(lq_firfilt *q)
{
    if (q->dev_valid) return;
    lqrt_h2d(q->d_win[q->cur], q->h_win + q->hoff * q->esz, (size_t)q->HP * q->esz, q->ctx.stream);
    q->dev_valid = 1;
}

void lq_firfilt_push(lq_firfilt *q, const void *x)
{
    lq_firfilt_need_host(q);
    /* append after the window; the window moves up one sample, and only
     * when the buffer is full do its last HP-1 samples move back to the
     * start (the reference's window.c does the same with its 2^k + len - 1
     * buffer) */
    if (q->hoff + q->HP == (size_t)LQ_FIR_HCAP * q->HP) {
        memmove(q->h_win, q->h_win + (q->hoff + 1) * q->esz, (size_t)(q->HP - 1) * q->esz);
        q->hoff = (size_t)-1;
    }
    memcpy(q->h_win + (q->hoff + q->HP) * q->esz, x, q->esz);
    q->hoff++;
    q->dev_valid = 0;
}

/* one output from the current window: the kernel reads the window where it
 * is authoritative -- in place from the pinned host mirror after push()es,
 * or the device copy after a device block -- and writes the result to
 * pinned host memory and raises the completion flag itself (one launch, no
 * stream sync) */
void lq_firfilt_execute(lq_firfilt *q, void *y)
{
    if (lq_small_host()) {   /* opt-in host path (lq_small.c): the window's newest sample is h_win[HP-1] */
        lq_firfilt_need_host(q);
        float v[2];
        /* the last hlen window samples, oldest first, against the reversed taps */
        lq_host_tdot(q->kind, q->hg, q->h_win + (q->hoff + q->HP - q->hlen) * q->esz, q->hlen, v);
        if (q->kind == LQ_RRRF) {
            *(float *)y = v[0] * q->d.scale_re;
        } else if (q->kind == LQ_CRCF) {   /* firfilt.c:337: real scale per component */
            ((float *)y)[0] = v[0] * q->d.scale_re;
            ((float *)y)[1] = v[1] * q->d.scale_re;
        } else {
            ((float *)y)[0] = v[0] * q->d.scale_re - v[1] * q->d.scale_im;
            ((float *)y)[1] = v[0] * q->d.scale_im + v[1] * q->d.scale_re;
        }
        return;
    }
    const void *win = q->dev_valid ? q->d_win[q->cur] : (const void *)(q->h_win + q->hoff * q->esz);
    unsigned *flag, seq;
    void *py = lq_sig_out(&q->ctx, q->esz, &flag, &seq);
    lqk_fir_single(&q->d, win, py, flag, seq, q->ctx.stream);
    lq_sig_wait(&q->ctx, y, q->esz, seq);
}

/* device-resident block: window update first (reads x before an in-place
 * overwrite), then the filter kernel on the old window's last HP-1 samples */
void lq_firfilt_execute_block_dev(lq_firfilt *q, const void *dx, unsigned long long n, void *dy)
{
    if (n == 0) return;
    lq_firfilt_need_dev(q);
    void *wold = q->d_win[q->cur];
    void *wnew = q->d_win[q->cur ^ 1];
    if (q->d_H8 && n >= LQ_FIR_FFT_MIN_N) {
        lqk_window_append(q->kind != LQ_RRRF, wold, q->HP, dx, n, wnew, q->ctx.stream);
        const void *x = dx;
        if (dx == dy) {   /* segments read overlapping halos: filter a copy */
            void *c = lq_devbuf_get(&q->scratch, (size_t)n * q->esz);
            lqrt_d2d(c, dx, (size_t)n * q->esz, q->ctx.stream);
            x = c;
        }
        /* the history: the window's last hlen - 1 samples */
        const void *hist = (const char *)wold + (size_t)(q->HP - (q->hlen - 1)) * q->esz;
        void *fl = lq_devbuf_get(&q->flags, lqk_fftfilt_flag_bytes(q->hlen, q->fft_n, n));
        lqk_fftfilt_run(0, q->hlen, q->fft_n, q->d_H8, hist, x, n, dy, q->d.scale_re, q->d.scale_im,
                        (const float *)q->d_hpad, q->kind == LQ_CCCF ? 2 : 1, fl, NULL, q->ctx.stream);
        q->cur ^= 1;
        q->host_valid = 0;
        return;
    }
    void *scr = NULL;
    if (dx == dy) scr = lq_devbuf_get(&q->scratch, lqk_firfilt_scratch_bytes(&q->d, n));
    /* the window update: inside the matrix-core kernel, else launched first */
    const lqk_hist_job job = {wold, dx, n, wnew, q->HP};
    lqk_firfilt(&q->d, wold, dx, n, dy, scr, &job, q->ctx.stream);
    q->cur ^= 1;
    q->host_valid = 0;
}

void lq_firfilt_execute_block(lq_firfilt *q, const void *x, unsigned long long n, void *y)
{
    if (n == 0) return;
    size_t bytes = (size_t)n * q->esz;
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, bytes);
    void *dy = lq_devbuf_get(&q->ybuf, bytes);
    lq_firfilt_execute_block_dev(q, dx, n, dy);
    lq_call_out(&q->ctx, y, dy, bytes);
}

unsigned int lq_firfilt_get_length(lq_firfilt *q) { return q->hlen; }

/* firfilt.c:371-387: H = scale * sum_i hr[i] e^{j 2 pi fc i}, hr = the
 * reference's internally reversed taps (host arithmetic, as the reference) */
static void lq_firfilt_freqresponse(lq_firfilt *q, float fc, liquid_float_complex *H)
{
    float complex acc = 0.0f;
    const unsigned int n = q->hlen;
    for (unsigned int i = 0; i < n; i++) {
        const unsigned int k = n - 1 - i;
        const float complex hk = q->kind == LQ_CCCF ? q->h[2 * k] + _Complex_I * q->h[2 * k + 1] : q->h[k];
        acc += hk * cexpf(_Complex_I * 2 * M_PI * fc * i);
    }
    acc *= q->d.scale_re + _Complex_I * q->d.scale_im;
    *H = acc;
}

/* firfilt.c:393-404 and group_delay.c:34-56 (real parts of the taps) */
static float lq_firfilt_groupdelay(lq_firfilt *q, float fc)
{
    const unsigned int n = q->hlen;
    if (fc < -0.5 || fc > 0.5) LQ_FAIL("error: fir_group_delay(), _fc must be in [-0.5,0.5]\n");
    float complex t0 = 0.0f, t1 = 0.0f;
    for (unsigned int i = 0; i < n; i++) {
        const float hi = q->kind == LQ_CCCF ? q->h[2 * i] : q->h[i];
        t0 += hi * cexpf(_Complex_I * 2 * M_PI * fc * i) * i;
        t1 += hi * cexpf(_Complex_I * 2 * M_PI * fc * i);
    }
    return crealf(t0 / t1);
}
lq_ctx *lq_firfilt_ctx(lq_firfilt *q) { return &q->ctx; }

/* ----------------------------------------------------------------- typed front ends */

#define LQ_FIRFILT_FRONT(NAME, KIND, TO, TC, TI, SCALE_RE, SCALE_IM)                                \
    struct NAME##_s {                                                                               \
        lq_firfilt *f;                                                                              \
    };                                                                                              \
    NAME NAME##_create(TC *_h, unsigned int _n)                                                     \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->f = lq_firfilt_create(KIND, (const float *)_h, _n, #NAME);                               \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_create_kaiser(unsigned int _n, float _fc, float _As, float _mu)                     \
    {                                                                                               \
        if (_n == 0) LQ_FAIL("error: " #NAME "_create_kaiser(), filter length must be greater than zero\n"); \
        float *hf = (float *)lq_xmalloc(_n * sizeof(float));                                        \
        TC *hc = (TC *)lq_xmalloc(_n * sizeof(TC));                                                 \
        lq_firdes_kaiser(_n, _fc, _As, _mu, hf);                                                    \
        for (unsigned int i = 0; i < _n; i++) hc[i] = (TC)hf[i];                                    \
        NAME q = NAME##_create(hc, _n);                                                             \
        free(hf);                                                                                   \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_create_rect(unsigned int _n)                                                        \
    {                                                                                               \
        if (_n == 0 || _n > 1024) LQ_FAIL("error: " #NAME "_create_rect(), filter length must be in [1,1024]\n"); \
        TC *hc = (TC *)lq_xmalloc(_n * sizeof(TC));                                                 \
        for (unsigned int i = 0; i < _n; i++) hc[i] = (TC)1.0f;                                     \
        NAME q = NAME##_create(hc, _n);                                                             \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    /* firfilt.c:140-171: 2km+1 taps from liquid_firdes_prototype */                                \
    NAME NAME##_create_rnyquist(int _type, unsigned int _k, unsigned int _m, float _beta, float _mu)\
    {                                                                                               \
        if (_k < 2) LQ_FAIL("error: " #NAME "_create_rnyquist(), filter samples/symbol must be greater than 1\n");\
        if (_m == 0) LQ_FAIL("error: " #NAME "_create_rnyquist(), filter delay must be greater than 0\n");\
        if (_beta < 0.0f || _beta > 1.0f)                                                           \
            LQ_FAIL("error: " #NAME "_create_rnyquist(), filter excess bandwidth factor must be in [0,1]\n");\
        const unsigned int n = 2 * _k * _m + 1;                                                     \
        float *hf = (float *)lq_xmalloc(n * sizeof(float));                                         \
        TC *hc = (TC *)lq_xmalloc(n * sizeof(TC));                                                  \
        liquid_firdes_prototype((liquid_firfilt_type)_type, _k, _m, _beta, _mu, hf);                \
        for (unsigned int i = 0; i < n; i++) hc[i] = (TC)hf[i];                                     \
        NAME q = NAME##_create(hc, n);                                                              \
        free(hf);                                                                                   \
        free(hc);                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_recreate(NAME _q, TC *_h, unsigned int _n)                                          \
    {                                                                                               \
        _q->f = lq_firfilt_recreate(_q->f, (const float *)_h, _n);                                  \
        return _q;                                                                                  \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_firfilt_destroy(_q->f);                                                                  \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_reset(NAME _q) { lq_firfilt_reset(_q->f); }                                         \
    void NAME##_print(NAME _q) { lq_firfilt_print(_q->f); }                                         \
    void NAME##_set_scale(NAME _q, TC _scale) { lq_firfilt_set_scale(_q->f, SCALE_RE, SCALE_IM); }  \
    void NAME##_push(NAME _q, TI _x) { lq_firfilt_push(_q->f, &_x); }                               \
    void NAME##_execute(NAME _q, TO *_y) { lq_firfilt_execute(_q->f, _y); }                         \
    void NAME##_execute_block(NAME _q, TI *_x, unsigned int _n, TO *_y)                             \
    {                                                                                               \
        lq_firfilt_execute_block(_q->f, _x, _n, _y);                                                \
    }                                                                                               \
    unsigned int NAME##_get_length(NAME _q) { return lq_firfilt_get_length(_q->f); }                \
    void NAME##_freqresponse(NAME _q, float _fc, liquid_float_complex *_H)                          \
    {                                                                                               \
        lq_firfilt_freqresponse(_q->f, _fc, _H);                                                    \
    }                                                                                               \
    float NAME##_groupdelay(NAME _q, float _fc) { return lq_firfilt_groupdelay(_q->f, _fc); }        \
    void NAME##_execute_block_dev(NAME _q, const TI *_dx, unsigned long long _n, TO *_dy)           \
    {                                                                                               \
        lq_firfilt_execute_block_dev(_q->f, _dx, _n, _dy);                                          \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ctx_set_stream(lq_firfilt_ctx(_q->f), _s); }     \
    void *NAME##_get_stream(NAME _q) { return lq_firfilt_ctx(_q->f)->stream; }                      \
    void NAME##_synchronize(NAME _q) { lqrt_sync(lq_firfilt_ctx(_q->f)->stream); }

LQ_FIRFILT_FRONT(firfilt_rrrf, LQ_RRRF, float, float, float, _scale, 0.0f)
LQ_FIRFILT_FRONT(firfilt_crcf, LQ_CRCF, liquid_float_complex, float, liquid_float_complex, _scale, 0.0f)
LQ_FIRFILT_FRONT(firfilt_cccf, LQ_CCCF, liquid_float_complex, liquid_float_complex, liquid_float_complex,
                 crealf(_scale), cimagf(_scale))
