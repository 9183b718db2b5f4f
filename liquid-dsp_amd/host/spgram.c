/*
 * spgram.c -- spgramcf / spgramf (spectral periodogram) on the GPU.
 *
 * API include/liquid.h:1220-1290; semantics src/fft/src/spgram.c:41-286:
 *   create(nfft, window, W): w = window * sqrt(2) / (rms(window) sqrt(nfft));
 *   the window buffer holds the last W inputs; execute() transforms
 *   x[i] = buffer[i] w[i] (zero padded to nfft); accumulate_psd() transforms
 *   every W/2 inputs and runs psd = (1-a) psd + a |X|^2 (a = 1 for the rest of
 *   the call that makes the object's first transform, as the reference's loop
 *   does); estimate_psd() resets, transforms every nfft/4 inputs and at the
 *   end, and averages |X|^2.  Outputs in dB are fft-shifted.
 * push()/write() samples are staged on the host and appended to the device
 * window before the next transform.  Transforms of one call run as one batch
 * (csrc/k_spgram.hip + csrc/k_fft.hip).
 */
#include <complex.h>
#include <math.h>

#include "lq_host.h"

#define SPG_MAX_BATCH_SAMPLES (1ull << 25)   /* transforms per launch batch: this many samples */

typedef struct {
    int real_in;
    size_t esz;
    unsigned int nfft, W;
    float *w;                 /* host copy of the scaled window */
    float *d_w;
    void *d_hist[2];          /* last W inputs */
    int cur;
    float *d_psd;             /* accumulated psd (natural order) */
    unsigned int sample_counter, num_transforms;
    unsigned char *pend;      /* push()/write() samples not yet on the device */
    size_t npend, cappend;
    fftplan plan;
    lq_ctx ctx;
    lq_devbuf xbuf, Xbuf, ends, acc, out, work;
} lq_spg;

static lq_spg *lq_spg_create(int real_in, unsigned int nfft, const float *window, unsigned int W, const char *who)
{
    if (nfft < 2) LQ_FAIL("error: %s_create(), fft size must be at least 2\n", who);
    if (W > nfft) LQ_FAIL("error: %s_create(), window size cannot exceed fft size\n", who);
    if (W == 0) LQ_FAIL("error: %s_create(), window size must be greater than zero\n", who);
    lqrt_require_device("spgram_create");
    lq_spg *q = (lq_spg *)lq_xmalloc(sizeof(*q));
    memset(q, 0, sizeof(*q));
    q->real_in = real_in;
    q->esz = real_in ? 4 : 8;
    q->nfft = nfft;
    q->W = W;
    q->w = (float *)lq_xmalloc(W * sizeof(float));
    float g = 0.0f;
    for (unsigned int i = 0; i < W; i++) g += window[i] * window[i];
    g = M_SQRT2 / (sqrtf(g / W) * sqrtf((float)nfft));
    for (unsigned int i = 0; i < W; i++) q->w[i] = g * window[i];
    lq_ctx_init(&q->ctx);
    q->d_w = (float *)lqrt_malloc(W * sizeof(float));
    lqrt_h2d(q->d_w, q->w, W * sizeof(float), q->ctx.stream);
    q->d_hist[0] = lqrt_malloc((size_t)W * q->esz);
    q->d_hist[1] = lqrt_malloc((size_t)W * q->esz);
    q->d_psd = (float *)lqrt_malloc(nfft * sizeof(float));
    q->plan = fft_create_plan(nfft, NULL, NULL, LIQUID_FFT_FORWARD, 0);
    fft_set_stream(q->plan, q->ctx.stream);
    return q;
}

static void lq_spg_reset(lq_spg *q)
{
    lqrt_memset(q->d_hist[q->cur], (size_t)q->W * q->esz, q->ctx.stream);
    float *ones = (float *)lq_xmalloc(q->nfft * sizeof(float));
    for (unsigned int i = 0; i < q->nfft; i++) ones[i] = 1.0f;
    lqrt_h2d(q->d_psd, ones, q->nfft * sizeof(float), q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    free(ones);
    q->npend = 0;
    q->num_transforms = 0;
    q->sample_counter = 0;
}

static void lq_spg_destroy(lq_spg *q)
{
    lqrt_sync(q->ctx.stream);
    fft_destroy_plan(q->plan);
    lqrt_free(q->d_w);
    lqrt_free(q->d_hist[0]);
    lqrt_free(q->d_hist[1]);
    lqrt_free(q->d_psd);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->Xbuf);
    lq_devbuf_free(&q->ends);
    lq_devbuf_free(&q->acc);
    lq_devbuf_free(&q->out);
    lq_devbuf_free(&q->work);
    lq_ctx_free(&q->ctx);
    free(q->pend);
    free(q->w);
    free(q);
}

static void lq_spg_stage(lq_spg *q, const void *x, size_t n)
{
    if (q->npend + n > q->cappend) {
        size_t c = q->cappend ? q->cappend : 1024;
        while (c < q->npend + n) c *= 2;
        unsigned char *p = (unsigned char *)lq_xmalloc(c * q->esz);
        if (q->npend) memcpy(p, q->pend, q->npend * q->esz);
        free(q->pend);
        q->pend = p;
        q->cappend = c;
    }
    memcpy(q->pend + q->npend * q->esz, x, n * q->esz);
    q->npend += n;
}

/* append n device samples to the window (no transforms) */
static void lq_spg_append_dev(lq_spg *q, const void *dx, unsigned long long n)
{
    if (n == 0) return;
    lqk_window_append(!q->real_in, q->d_hist[q->cur], q->W, dx, n, q->d_hist[q->cur ^ 1], q->ctx.stream);
    q->cur ^= 1;
}

static void lq_spg_flush(lq_spg *q)
{
    if (q->npend == 0) return;
    void *dx = lq_devbuf_get(&q->xbuf, q->npend * q->esz);
    lqrt_h2d(dx, q->pend, q->npend * q->esz, q->ctx.stream);
    lq_spg_append_dev(q, dx, q->npend);
    q->npend = 0;
}

/* transforms ending at block positions ends[0..T) of (hist | dx) -> Xbuf, in batches;
 * `each` consumes one batch */
typedef void (*lq_spg_each)(lq_spg *q, const void *X, unsigned long long T, void *arg);

static void lq_spg_transforms(lq_spg *q, const void *dx, const long long *ends, unsigned long long T, lq_spg_each each,
                              void *arg)
{
    unsigned long long B = SPG_MAX_BATCH_SAMPLES / q->nfft;
    if (B == 0) B = 1;
    for (unsigned long long t0 = 0; t0 < T; t0 += B) {
        const unsigned long long nb = T - t0 < B ? T - t0 : B;
        long long *de = (long long *)lq_devbuf_get(&q->ends, nb * sizeof(long long));
        lqrt_h2d(de, ends + t0, nb * sizeof(long long), q->ctx.stream);
        void *X = lq_devbuf_get(&q->Xbuf, (size_t)nb * q->nfft * 8);
        lqk_spgram_gather(q->real_in, q->d_hist[q->cur], q->W, dx, de, nb, q->d_w, q->nfft, X, q->ctx.stream);
        fft_execute_batch_dev(q->plan, X, X, nb);
        each(q, X, nb, arg);
        lqrt_sync(q->ctx.stream);   /* ends/X buffers are reused by the next batch */
    }
}

/* the current window's transform into Xbuf (spgram.c:166-183) */
static void *lq_spg_execute_dev(lq_spg *q)
{
    lq_spg_flush(q);
    const long long e = -1;
    long long *de = (long long *)lq_devbuf_get(&q->ends, sizeof(long long));
    lqrt_h2d(de, &e, sizeof(e), q->ctx.stream);
    void *X = lq_devbuf_get(&q->Xbuf, (size_t)q->nfft * 8);
    lqk_spgram_gather(q->real_in, q->d_hist[q->cur], q->W, NULL, de, 1, q->d_w, q->nfft, X, q->ctx.stream);
    fft_execute_batch_dev(q->plan, X, X, 1);
    return X;
}

static void lq_spg_execute(lq_spg *q, liquid_float_complex *X)
{
    void *dX = lq_spg_execute_dev(q);
    if (X) lqrt_d2h(X, dX, (size_t)q->nfft * 8, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
}

static void lq_spg_execute_psd(lq_spg *q, float *out)
{
    void *dX = lq_spg_execute_dev(q);
    float *o = (float *)lq_devbuf_get(&q->out, q->nfft * sizeof(float));
    lqk_spgram_db(0, dX, NULL, q->nfft, 1.0f, o, q->ctx.stream);
    lqrt_d2h(out, o, q->nfft * sizeof(float), q->ctx.stream);
    lqrt_sync(q->ctx.stream);
}

static void lq_spg_each_accum(lq_spg *q, const void *X, unsigned long long T, void *arg)
{
    void *w = lq_devbuf_get(&q->work, lqk_spgram_work_bytes(T, q->nfft));
    lqk_spgram_accumulate(X, T, q->nfft, *(float *)arg, q->d_psd, w, q->ctx.stream);
}

static void lq_spg_accumulate_dev(lq_spg *q, const void *dx, unsigned long long n, float alpha)
{
    if (alpha < 0.0f || alpha > 1.0f) LQ_FAIL("error: spgram_accumulate_psd(), alpha must be in [0,1]\n");
    lq_spg_flush(q);
    if (n == 0) return;
    const unsigned int H = q->W / 2;
    unsigned long long T = 0;
    long long *ends = NULL;
    if (H > 0) {   /* transform after the input that brings sample_counter to W/2 */
        const long long first = (long long)(H - q->sample_counter) - 1;
        if (first < (long long)n) T = (unsigned long long)(((long long)n - 1 - first) / H + 1);
        if (q->nfft == 1024 && n < (1ull << 27)) {   /* fused path: ends are first + t H, no table */
            if (T > 0) {
                float a = q->num_transforms == 0 ? 1.0f : alpha;
                void *w = lq_devbuf_get(&q->work, lqk_spgram_work_bytes(T, q->nfft));
                lqk_spgram_fused1024(q->real_in, q->d_hist[q->cur], q->W, dx, first, (long long)H, T,
                                     first + (long long)((T - 1) * H), q->d_w, 1, a, q->d_psd, w, q->ctx.stream);
                q->num_transforms += (unsigned int)T;
            }
            q->sample_counter = (unsigned int)((q->sample_counter + n) % H);
            lq_spg_append_dev(q, dx, n);
            return;
        }
        ends = (long long *)lq_xmalloc((T ? T : 1) * sizeof(long long));
        for (unsigned long long t = 0; t < T; t++) ends[t] = first + (long long)(t * H);
        q->sample_counter = (unsigned int)((q->sample_counter + n) % H);
    }
    if (T > 0) {
        float a = q->num_transforms == 0 ? 1.0f : alpha;
        lq_spg_transforms(q, dx, ends, T, lq_spg_each_accum, &a);
        q->num_transforms += (unsigned int)T;
    }
    free(ends);
    lq_spg_append_dev(q, dx, n);
}

static void lq_spg_accumulate(lq_spg *q, const void *x, float alpha, unsigned int n)
{
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, (size_t)n * q->esz);
    lq_spg_accumulate_dev(q, dx, n, alpha);
    lq_call_done(&q->ctx);
}

static void lq_spg_write_accumulation(lq_spg *q, float *out)
{
    float *o = (float *)lq_devbuf_get(&q->out, q->nfft * sizeof(float));
    lqk_spgram_db(1, NULL, q->d_psd, q->nfft, 1.0f, o, q->ctx.stream);
    lqrt_d2h(out, o, q->nfft * sizeof(float), q->ctx.stream);
    lqrt_sync(q->ctx.stream);
}

static void lq_spg_each_sum(lq_spg *q, const void *X, unsigned long long T, void *arg)
{
    void *w = lq_devbuf_get(&q->work, lqk_spgram_work_bytes(T, q->nfft));
    lqk_spgram_sum(X, T, q->nfft, (float *)arg, w, q->ctx.stream);
}

static void lq_spg_estimate_dev(lq_spg *q, const void *dx, unsigned long long n, float *dpsd)
{
    if (n == 0) return;
    lq_spg_reset(q);
    unsigned int delay = q->nfft / 4;
    if (delay == 0) delay = 1;
    unsigned long long T = n / delay + ((n % delay) ? 1 : 0);
    float *acc = (float *)lq_devbuf_get(&q->acc, q->nfft * sizeof(float));
    lqrt_memset(acc, q->nfft * sizeof(float), q->ctx.stream);
    if (q->nfft == 1024 && n < (1ull << 27)) {   /* fused path: ends are delay-1 + t delay, the last one n-1 */
        void *w = lq_devbuf_get(&q->work, lqk_spgram_work_bytes(T, q->nfft));
        lqk_spgram_fused1024(q->real_in, q->d_hist[q->cur], q->W, dx, (long long)delay - 1, (long long)delay, T,
                             (long long)n - 1, q->d_w, 0, 0.0f, acc, w, q->ctx.stream);
        lqk_spgram_db(2, NULL, acc, q->nfft, (float)T, dpsd, q->ctx.stream);
        lq_spg_append_dev(q, dx, n);
        return;
    }
    long long *ends = (long long *)lq_xmalloc(T * sizeof(long long));
    unsigned long long t = 0;
    for (unsigned long long i = delay - 1; i < n; i += delay) ends[t++] = (long long)i;
    if (t < T) ends[t++] = (long long)n - 1;
    lq_spg_transforms(q, dx, ends, t, lq_spg_each_sum, acc);
    lqk_spgram_db(2, NULL, acc, q->nfft, (float)t, dpsd, q->ctx.stream);
    free(ends);
    lq_spg_append_dev(q, dx, n);
}

static void lq_spg_estimate(lq_spg *q, const void *x, unsigned int n, float *psd)
{
    if (n == 0) return;
    void *dx = lq_devbuf_get(&q->xbuf, (size_t)n * q->esz);
    lqrt_h2d(dx, x, (size_t)n * q->esz, q->ctx.stream);
    float *o = (float *)lq_devbuf_get(&q->out, q->nfft * sizeof(float));
    lq_spg_estimate_dev(q, dx, n, o);
    lqrt_d2h(psd, o, q->nfft * sizeof(float), q->ctx.stream);
    lqrt_sync(q->ctx.stream);
}

#define LQ_SPGRAM_FRONT(NAME, REAL, TI)                                                             \
    struct NAME##_s {                                                                               \
        lq_spg *e;                                                                                  \
    };                                                                                              \
    NAME NAME##_create(unsigned int _nfft, float *_window, unsigned int _window_len)               \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = lq_spg_create(REAL, _nfft, _window, _window_len, #NAME);                             \
        lq_spg_reset(q->e);                                                                         \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_create_kaiser(unsigned int _nfft, unsigned int _window_len, float _beta)           \
    {                                                                                               \
        if (_nfft < 2) LQ_FAIL("error: " #NAME "_create_kaiser(), fft size must be at least 2\n");  \
        if (_window_len > _nfft)                                                                    \
            LQ_FAIL("error: " #NAME "_create_kaiser(), window size cannot exceed fft size\n");       \
        if (_window_len == 0)                                                                       \
            LQ_FAIL("error: " #NAME "_create_kaiser(), window size must be greater than zero\n");   \
        if (_beta <= 0.0f) LQ_FAIL("error: " #NAME "_create_kaiser(), beta must be greater than zero\n"); \
        float *w = (float *)lq_xmalloc(_window_len * sizeof(float));                                \
        for (unsigned int i = 0; i < _window_len; i++) w[i] = kaiser(i, _window_len, _beta, 0.0f);  \
        NAME q = NAME##_create(_nfft, w, _window_len);                                              \
        free(w);                                                                                    \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_create_default(unsigned int _nfft)                                                  \
    {                                                                                               \
        if (_nfft < 2) LQ_FAIL("error: " #NAME "_create_default(), fft size must be at least 2\n"); \
        return NAME##_create_kaiser(_nfft, _nfft / 2, 10.0f);                                       \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_spg_destroy(_q->e);                                                                      \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_reset(NAME _q) { lq_spg_reset(_q->e); }                                             \
    void NAME##_push(NAME _q, TI _x) { lq_spg_stage(_q->e, &_x, 1); }                               \
    void NAME##_write(NAME _q, TI *_x, unsigned int _n) { lq_spg_stage(_q->e, _x, _n); }            \
    void NAME##_execute(NAME _q, liquid_float_complex *_X) { lq_spg_execute(_q->e, _X); }           \
    void NAME##_execute_psd(NAME _q, float *_X) { lq_spg_execute_psd(_q->e, _X); }                  \
    void NAME##_accumulate_psd(NAME _q, TI *_x, float _alpha, unsigned int _n)                      \
    {                                                                                               \
        lq_spg_accumulate(_q->e, _x, _alpha, _n);                                                   \
    }                                                                                               \
    void NAME##_write_accumulation(NAME _q, float *_x) { lq_spg_write_accumulation(_q->e, _x); }    \
    void NAME##_estimate_psd(NAME _q, TI *_x, unsigned int _n, float *_psd)                         \
    {                                                                                               \
        lq_spg_estimate(_q->e, _x, _n, _psd);                                                       \
    }                                                                                               \
    void NAME##_accumulate_psd_dev(NAME _q, const TI *_dx, float _alpha, unsigned long long _n)     \
    {                                                                                               \
        lq_spg_accumulate_dev(_q->e, _dx, _n, _alpha);                                              \
    }                                                                                               \
    void NAME##_estimate_psd_dev(NAME _q, const TI *_dx, unsigned long long _n, float *_dpsd)       \
    {                                                                                               \
        lq_spg_estimate_dev(_q->e, _dx, _n, _dpsd);                                                 \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s)                                                       \
    {                                                                                               \
        lq_ctx_set_stream(&_q->e->ctx, _s);                                                         \
        fft_set_stream(_q->e->plan, _q->e->ctx.stream);                                             \
    }                                                                                               \
    void NAME##_synchronize(NAME _q) { lqrt_sync(_q->e->ctx.stream); }

LQ_SPGRAM_FRONT(spgramcf, 0, liquid_float_complex)
LQ_SPGRAM_FRONT(spgramf, 1, float)
