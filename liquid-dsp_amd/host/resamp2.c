/*
 * resamp2.c -- resamp2, msresamp2 and msresamp for rrrf / crcf / cccf.
 *
 * resamp2   include/liquid.h:2840-2925, src/filter/src/resamp2.c:46-360
 *           half-band filter h[i] = sinc(t/2) kaiser(i) mod(t), t = i - 2m,
 *           4m+1 taps, mod = cos(2 pi f0 t) (real taps) or exp(j 2 pi f0 t)
 *           (cccf); five modes share two 2m-sample windows (csrc/k_resamp2.hip)
 * msresamp2 include/liquid.h:3027-3090, src/filter/src/msresamp2.c:66-354
 *           2^s-rate cascade of half-band stages; stage i cut-off fc/2^(i+1),
 *           m_i = max(3, ceil((len_i - 1)/4)) from the Kaiser length estimate;
 *           decimator output scaled by 2^-s, interpolator stages run reversed
 * msresamp  include/liquid.h:3094-3140, src/filter/src/msresamp.c:68-349
 *           rate r = 2^(+-s) * r_a with r_a in [0.5, 2]: interp = resamp
 *           (m 7, fc 0.4, npfb 64) then the half-band interpolator; decim =
 *           half-band decimator on groups of 2^s inputs then resamp
 * Block extensions (new names): *_execute_block[_dev] run n consecutive
 * calls; every sample is computed by the GPU kernels.
 */
#include <complex.h>
#include <math.h>

#include "lq_host.h"

static const char *lq_ext[] = {"rrrf", "crcf", "cccf"};

/* ===================================================================== resamp2 */
typedef struct {
    int kind;
    size_t esz, csz;
    unsigned int m, h_len;
    float f0, As;
    float *h;            /* h_len coefficients (csz bytes each) */
    void *d_taps;        /* 2m odd taps h1[j] = h[4m-1-2j] */
    void *d_w[2][2];     /* [ping-pong][window] */
    int cur, toggle;
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf, y1buf;
} lq_r2;

static void lq_r2_design(lq_r2 *q)
{
    const unsigned int n = q->h_len, cw = q->csz / 4;
    const float beta = lq_kaiser_beta_As(q->As);
    for (unsigned int i = 0; i < n; i++) {
        const float t = (float)i - (float)(n - 1) / 2.0f;
        const float a = lq_sincf(t / 2.0f) * lq_kaiser_window(i, n, beta, 0);
        const float c = cosf(2.0f * M_PI * t * q->f0);
        if (cw == 2) {
            q->h[2 * i] = a * c;
            q->h[2 * i + 1] = a * sinf(2.0f * M_PI * t * q->f0);
        } else {
            q->h[i] = a * c;
        }
    }
    float *h1 = (float *)lq_xmalloc(2 * q->m * q->csz);
    for (unsigned int j = 0; j < 2 * q->m; j++)
        for (unsigned int c = 0; c < cw; c++) h1[j * cw + c] = q->h[(n - 2 * j - 2) * cw + c];
    lqrt_h2d(q->d_taps, h1, 2 * q->m * q->csz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    free(h1);
}

static lq_r2 *lq_r2_create(int kind, unsigned int m, float f0, float As)
{
    if (m < 2) LQ_FAIL("error: resamp2_%s_create(), filter semi-length must be at least 2\n", lq_ext[kind]);
    if (f0 < -0.5f || f0 > 0.5f)
        LQ_FAIL("error: resamp2_%s_create(), f0 (%12.4e) must be in (-1,1)\n", lq_ext[kind], f0);
    lqrt_require_device("resamp2_create");
    lq_r2 *q = (lq_r2 *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->esz = kind == LQ_RRRF ? 4 : 8;
    q->csz = kind == LQ_CCCF ? 8 : 4;
    q->m = m;
    q->h_len = 4 * m + 1;
    q->f0 = f0;
    q->As = As;
    q->h = (float *)lq_xmalloc(q->h_len * q->csz);
    lq_ctx_init(&q->ctx);
    q->d_taps = lqrt_malloc(2 * m * q->csz);
    for (int b = 0; b < 2; b++)
        for (int w = 0; w < 2; w++) q->d_w[b][w] = lqrt_malloc(2 * m * q->esz);
    lq_r2_design(q);
    return q;
}

static void lq_r2_destroy(lq_r2 *q)
{
    lqrt_sync(q->ctx.stream);
    lqrt_free(q->d_taps);
    for (int b = 0; b < 2; b++)
        for (int w = 0; w < 2; w++) lqrt_free(q->d_w[b][w]);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_devbuf_free(&q->y1buf);
    lq_ctx_free(&q->ctx);
    free(q->h);
    free(q);
}

static void lq_r2_clear(lq_r2 *q)
{
    for (int w = 0; w < 2; w++) lqrt_memset(q->d_w[q->cur][w], 2 * q->m * q->esz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    q->toggle = 0;
}

/* resamp2.c:101-140: same m keeps the windows and redesigns the taps */
static lq_r2 *lq_r2_recreate(lq_r2 *q, unsigned int m, float f0, float As)
{
    if (m != q->m) {
        const int kind = q->kind;
        void *s = q->ctx.own ? NULL : q->ctx.stream;
        lq_r2_destroy(q);
        q = lq_r2_create(kind, m, f0, As);
        if (s) lq_ctx_set_stream(&q->ctx, s);
        return q;
    }
    /* the reference redesigns with the stored f0 and As (resamp2.c:118-131) */
    lq_r2_design(q);
    return q;
}

static void lq_r2_print(lq_r2 *q)
{
    printf("fir half-band resampler: [%u taps, f0=%12.8f]\n", q->h_len, q->f0);
    for (unsigned int i = 0; i < q->h_len; i++) {
        if (q->kind == LQ_CCCF) printf("  h(%4u) = %12.8f+j*%12.8f;\n", i + 1, q->h[2 * i], q->h[2 * i + 1]);
        else printf("  h(%4u) = %12.8f;\n", i + 1, q->h[i]);
    }
}

/* inputs / outputs per call of each mode */
static unsigned int lq_r2_nin(int mode) { return (mode == LQK_R2_FILTER || mode == LQK_R2_INTERP) ? 1 : 2; }
static unsigned int lq_r2_nout(int mode) { return mode == LQK_R2_DECIM ? 1 : 2; }

static void lq_r2_run_dev(lq_r2 *q, int mode, const void *dx, unsigned long long n, void *dy0, void *dy1,
                          float scale)
{
    if (n == 0) return;
    if (mode < LQK_R2_FILTER || mode > LQK_R2_INTERP) LQ_FAIL("error: resamp2: invalid mode %d\n", mode);
    const int nx = q->cur ^ 1;
    lqk_resamp2(q->kind, mode, q->m, q->toggle, scale, q->d_taps, q->d_w[q->cur][0], q->d_w[q->cur][1],
                q->d_w[nx][0], q->d_w[nx][1], dx, n, dy0, dy1, q->ctx.stream);
    q->cur = nx;
    if (mode == LQK_R2_FILTER) q->toggle ^= (int)(n & 1);
}

static void lq_r2_run(lq_r2 *q, int mode, const void *x, unsigned long long n, void *y0, void *y1)
{
    if (n == 0) return;
    const size_t bx = (size_t)n * lq_r2_nin(mode) * q->esz;
    const size_t by = (size_t)n * (mode == LQK_R2_FILTER ? 1 : lq_r2_nout(mode)) * q->esz;
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, bx);
    if (mode != LQK_R2_FILTER) {
        void *dy = lq_devbuf_get(&q->ybuf, by);
        lq_r2_run_dev(q, mode, dx, n, dy, NULL, 1.0f);
        lq_call_out(&q->ctx, y0, dy, by);
        return;
    }
    /* filter mode: y0 and y1 side by side in one device buffer (y1 at a
       16-byte aligned offset) so both come back through the same pinned
       copy-out and completion flag; past the copy-out size, two copies and
       a stream synchronisation */
    const size_t off = (by + 15) & ~(size_t)15;
    unsigned char *dy = (unsigned char *)lq_devbuf_get(&q->ybuf, off + by);
    lq_r2_run_dev(q, mode, dx, n, dy, dy + off, 1.0f);
    if (off + by <= LQRT_COPYOUT_MAX) {
        unsigned char small[256];
        unsigned char *tmp = off + by <= sizeof(small) ? small : (unsigned char *)lq_xmalloc(off + by);
        lq_call_out(&q->ctx, tmp, dy, off + by);
        memcpy(y0, tmp, by);
        memcpy(y1, tmp + off, by);
        if (tmp != small) free(tmp);
    } else {
        lqrt_d2h(y0, dy, by, q->ctx.stream);
        lqrt_d2h(y1, dy + off, by, q->ctx.stream);
        lq_call_done(&q->ctx);
    }
}

#define LQ_RESAMP2_FRONT(NAME, KIND, T)                                                             \
    struct NAME##_s {                                                                               \
        lq_r2 *e;                                                                                   \
    };                                                                                              \
    NAME NAME##_create(unsigned int _m, float _f0, float _As)                                       \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = lq_r2_create(KIND, _m, _f0, _As);                                                    \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_recreate(NAME _q, unsigned int _m, float _f0, float _As)                            \
    {                                                                                               \
        _q->e = lq_r2_recreate(_q->e, _m, _f0, _As);                                                \
        return _q;                                                                                  \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_r2_destroy(_q->e);                                                                       \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_print(NAME _q) { lq_r2_print(_q->e); }                                              \
    void NAME##_clear(NAME _q) { lq_r2_clear(_q->e); }                                              \
    unsigned int NAME##_get_delay(NAME _q) { return 2 * _q->e->m - 1; }                             \
    void NAME##_filter_execute(NAME _q, T _x, T *_y0, T *_y1)                                       \
    {                                                                                               \
        lq_r2_run(_q->e, LQK_R2_FILTER, &_x, 1, _y0, _y1);                                          \
    }                                                                                               \
    void NAME##_analyzer_execute(NAME _q, T *_x, T *_y) { lq_r2_run(_q->e, LQK_R2_ANALYZER, _x, 1, _y, NULL); } \
    void NAME##_synthesizer_execute(NAME _q, T *_x, T *_y)                                          \
    {                                                                                               \
        lq_r2_run(_q->e, LQK_R2_SYNTHESIZER, _x, 1, _y, NULL);                                      \
    }                                                                                               \
    void NAME##_decim_execute(NAME _q, T *_x, T *_y) { lq_r2_run(_q->e, LQK_R2_DECIM, _x, 1, _y, NULL); } \
    void NAME##_interp_execute(NAME _q, T _x, T *_y) { lq_r2_run(_q->e, LQK_R2_INTERP, &_x, 1, _y, NULL); } \
    void NAME##_execute_block(NAME _q, int _mode, T *_x, unsigned long long _n, T *_y0, T *_y1)     \
    {                                                                                               \
        lq_r2_run(_q->e, _mode, _x, _n, _y0, _y1);                                                  \
    }                                                                                               \
    void NAME##_execute_block_dev(NAME _q, int _mode, const T *_dx, unsigned long long _n, T *_dy0, T *_dy1) \
    {                                                                                               \
        lq_r2_run_dev(_q->e, _mode, _dx, _n, _dy0, _dy1, 1.0f);                                     \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ctx_set_stream(&_q->e->ctx, _s); }               \
    void NAME##_synchronize(NAME _q) { lqrt_sync(_q->e->ctx.stream); }

LQ_RESAMP2_FRONT(resamp2_rrrf, LQ_RRRF, float)
LQ_RESAMP2_FRONT(resamp2_crcf, LQ_CRCF, liquid_float_complex)
LQ_RESAMP2_FRONT(resamp2_cccf, LQ_CCCF, liquid_float_complex)

/* =================================================================== msresamp2 */
typedef struct {
    int kind, type;          /* LIQUID_RESAMP_INTERP / _DECIM */
    size_t esz;
    unsigned int ns, M;
    float fc, f0, As, zeta;
    float fc_stage[16], f0_stage[16], As_stage[16];
    unsigned int m_stage[16];
    lq_r2 *st[16];
    lq_ctx ctx;
    lq_devbuf buf[2], xbuf, ybuf;
} lq_ms2;

static void lq_ms2_set_stream(lq_ms2 *q, void *s)
{
    lq_ctx_set_stream(&q->ctx, s);
    for (unsigned int i = 0; i < q->ns; i++) lq_ctx_set_stream(&q->st[i]->ctx, q->ctx.stream);
}

static lq_ms2 *lq_ms2_create(int kind, int type, unsigned int ns, float fc, float f0, float As)
{
    const char *e = lq_ext[kind];
    if (ns > 16) LQ_FAIL("error: msresamp2_%s_create(), number of stages should not exceed 16\n", e);
    if (fc <= 0.0f || fc >= 0.5f) LQ_FAIL("error: msresamp2_%s_create(), cut-off frequency must be in (0,0.5)\n", e);
    if (fc > 0.45f) {
        fprintf(stderr, "warning: msresamp2_%s_create(), cut-off frequency greater than 0.45\n", e);
        fc = 0.45f;
    }
    if (f0 != 0.) {
        fprintf(stderr, "warning: msresamp2_%s_create(), non-zero center frequency not yet supported\n", e);
        f0 = 0.;
    }
    lq_ms2 *q = (lq_ms2 *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->type = type == LIQUID_RESAMP_INTERP ? LIQUID_RESAMP_INTERP : LIQUID_RESAMP_DECIM;
    q->esz = kind == LQ_RRRF ? 4 : 8;
    q->ns = ns;
    q->M = 1u << ns;
    q->zeta = 1.0f / (float)q->M;
    q->fc = fc;
    q->f0 = f0;
    q->As = As;
    lq_ctx_init(&q->ctx);
    for (unsigned int i = 0; i < ns; i++) {   /* msresamp2.c:137-150 */
        f0 = 0.5f * f0;
        fc = 0.5f * fc;
        const float ft = (0.5f - fc) / 2.0f;
        const unsigned int hl = estimate_req_filter_len(ft, As);
        const unsigned int m = (unsigned int)ceilf((float)(hl - 1) / 4.0f);
        q->fc_stage[i] = fc;
        q->f0_stage[i] = f0;
        q->As_stage[i] = As;
        q->m_stage[i] = m < 3 ? 3 : m;
        q->st[i] = lq_r2_create(kind, q->m_stage[i], f0, As);
        lq_ctx_set_stream(&q->st[i]->ctx, q->ctx.stream);
    }
    return q;
}

static void lq_ms2_destroy(lq_ms2 *q)
{
    lqrt_sync(q->ctx.stream);
    for (unsigned int i = 0; i < q->ns; i++) lq_r2_destroy(q->st[i]);
    lq_devbuf_free(&q->buf[0]);
    lq_devbuf_free(&q->buf[1]);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_ctx_free(&q->ctx);
    free(q);
}

static void lq_ms2_reset(lq_ms2 *q)
{
    for (unsigned int i = 0; i < q->ns; i++) lq_r2_clear(q->st[i]);
}

static float lq_ms2_get_delay(lq_ms2 *q)   /* msresamp2.c:247-268 */
{
    float d = 0;
    for (unsigned int i = 0; i < q->ns; i++) {
        if (q->type == LIQUID_RESAMP_INTERP) {
            d *= 0.5f;
            d += q->m_stage[i];
        } else {
            d *= 2;
            d += 2 * q->m_stage[q->ns - i - 1] - 1;
        }
    }
    return d;
}

static void lq_ms2_print(lq_ms2 *q)
{
    printf("multi-stage half-band resampler:\n");
    printf("    type            : %s\n", q->type == LIQUID_RESAMP_DECIM ? "decimator" : "interpolator");
    printf("    number of stages: %u stage%s\n", q->ns, q->ns == 1 ? "" : "s");
    printf("    cut-off frequency, fc   : %12.8f Fs\n", q->fc);
    printf("    center frequency, f0    : %12.8f Fs\n", q->f0);
    printf("    stop-band attenuation   : %.2f dB\n", q->As);
    printf("    delay (total)           : %.3f samples\n", lq_ms2_get_delay(q));
    for (unsigned int i = 0; i < q->ns; i++)
        printf("    stage[%2u]  {m=%3u, As=%6.2f dB, fc=%6.3f, f0=%6.3f}\n", i, q->m_stage[i], q->As_stage[i],
               q->fc_stage[i], q->f0_stage[i]);
}

/* n calls: interp 1 -> M each, decim M -> 1 each (msresamp2.c:289-354) */
static void lq_ms2_block_dev(lq_ms2 *q, const void *dx, unsigned long long n, void *dy)
{
    if (n == 0) return;
    if (q->ns == 0) {
        lqrt_d2d(dy, dx, (size_t)n * q->esz, q->ctx.stream);
        return;
    }
    const size_t half = (size_t)n * (q->M / 2 ? q->M / 2 : 1) * q->esz;
    void *b[2] = {lq_devbuf_get(&q->buf[0], half), lq_devbuf_get(&q->buf[1], half)};
    const void *in = dx;
    for (unsigned int s = 0; s < q->ns; s++) {
        const int last = s == q->ns - 1;
        void *out = last ? dy : b[s & 1];
        if (q->type == LIQUID_RESAMP_INTERP) {
            lq_r2_run_dev(q->st[q->ns - s - 1], LQK_R2_INTERP, in, n << s, out, NULL, 1.0f);
        } else {
            lq_r2_run_dev(q->st[s], LQK_R2_DECIM, in, n << (q->ns - s - 1), out, NULL, last ? q->zeta : 1.0f);
        }
        in = out;
    }
}

static void lq_ms2_block(lq_ms2 *q, const void *x, unsigned long long n, void *y)
{
    if (n == 0) return;
    const size_t bx = (size_t)n * (q->type == LIQUID_RESAMP_INTERP ? 1 : q->M) * q->esz;
    const size_t by = (size_t)n * (q->type == LIQUID_RESAMP_INTERP ? q->M : 1) * q->esz;
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, bx);
    void *dy = lq_devbuf_get(&q->ybuf, by);
    lq_ms2_block_dev(q, dx, n, dy);
    lq_call_out(&q->ctx, y, dy, by);
}

#define LQ_MSRESAMP2_FRONT(NAME, KIND, T)                                                           \
    struct NAME##_s {                                                                               \
        lq_ms2 *e;                                                                                  \
    };                                                                                              \
    NAME NAME##_create(int _type, unsigned int _num_stages, float _fc, float _f0, float _As)        \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = lq_ms2_create(KIND, _type, _num_stages, _fc, _f0, _As);                              \
        return q;                                                                                   \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_ms2_destroy(_q->e);                                                                      \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_print(NAME _q) { lq_ms2_print(_q->e); }                                             \
    void NAME##_reset(NAME _q) { lq_ms2_reset(_q->e); }                                             \
    float NAME##_get_delay(NAME _q) { return lq_ms2_get_delay(_q->e); }                             \
    void NAME##_execute(NAME _q, T *_x, T *_y) { lq_ms2_block(_q->e, _x, 1, _y); }                   \
    void NAME##_execute_block(NAME _q, T *_x, unsigned long long _n, T *_y)                         \
    {                                                                                               \
        lq_ms2_block(_q->e, _x, _n, _y);                                                            \
    }                                                                                               \
    void NAME##_execute_block_dev(NAME _q, const T *_dx, unsigned long long _n, T *_dy)             \
    {                                                                                               \
        lq_ms2_block_dev(_q->e, _dx, _n, _dy);                                                      \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ms2_set_stream(_q->e, _s); }                     \
    void NAME##_synchronize(NAME _q) { lqrt_sync(_q->e->ctx.stream); }

LQ_MSRESAMP2_FRONT(msresamp2_rrrf, LQ_RRRF, float)
LQ_MSRESAMP2_FRONT(msresamp2_crcf, LQ_CRCF, liquid_float_complex)
LQ_MSRESAMP2_FRONT(msresamp2_cccf, LQ_CCCF, liquid_float_complex)

/* ==================================================================== msresamp */
typedef struct {
    int kind, type;
    size_t esz;
    float rate, As, rate_arb, rate_hb;
    unsigned int ns, M, bi;   /* bi: decimator inputs waiting for a full group of M */
    lq_ms2 *hb;
    lq_rs *rs;
    void *d_pend;
    lq_ctx ctx;
    lq_devbuf s0, s1, xbuf, ybuf;
} lq_ms;

static void lq_ms_set_stream(lq_ms *q, void *s)
{
    lq_ctx_set_stream(&q->ctx, s);
    lq_ms2_set_stream(q->hb, q->ctx.stream);
    lq_ctx_set_stream(lq_rs_ctx(q->rs), q->ctx.stream);
}

static lq_ms *lq_ms_create(int kind, float r, float As)
{
    if (r <= 0.0f) LQ_FAIL("error: msresamp_%s_create(), resampling rate must be greater than zero\n", lq_ext[kind]);
    lq_ms *q = (lq_ms *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->esz = kind == LQ_RRRF ? 4 : 8;
    q->rate = r;
    q->As = As;
    q->type = r > 1.0f ? LIQUID_RESAMP_INTERP : LIQUID_RESAMP_DECIM;
    q->rate_arb = r;
    q->rate_hb = 1.0f;
    if (q->type == LIQUID_RESAMP_INTERP) {
        while (q->rate_arb > 2.0f) {
            q->ns++;
            q->rate_hb *= 2.0f;
            q->rate_arb *= 0.5f;
        }
    } else {
        while (q->rate_arb < 0.5f) {
            q->ns++;
            q->rate_hb *= 0.5f;
            q->rate_arb *= 2.0f;
        }
    }
    q->M = 1u << q->ns;
    lq_ctx_init(&q->ctx);
    q->hb = lq_ms2_create(kind, q->type, q->ns, 0.4f, 0.0f, As);
    q->rs = lq_rs_create(kind, q->rate_arb, 7, 0.4f, As, 64);
    q->d_pend = lqrt_malloc((size_t)q->M * q->esz);
    lq_ms2_set_stream(q->hb, q->ctx.stream);           /* one stream for the whole chain */
    lq_ctx_set_stream(lq_rs_ctx(q->rs), q->ctx.stream);
    return q;
}

static void lq_ms_destroy(lq_ms *q)
{
    lqrt_sync(q->ctx.stream);
    lq_ms2_destroy(q->hb);
    lq_rs_destroy(q->rs);
    lqrt_free(q->d_pend);
    lq_devbuf_free(&q->s0);
    lq_devbuf_free(&q->s1);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_ctx_free(&q->ctx);
    free(q);
}

static void lq_ms_reset(lq_ms *q)
{
    lq_ms2_reset(q->hb);
    lq_rs_reset(q->rs);
    q->bi = 0;
}

static float lq_ms_get_delay(lq_ms *q)   /* msresamp.c:212-240 */
{
    const float dh = lq_ms2_get_delay(q->hb);
    const float da = 7.0f;                 /* resamp get_delay = m */
    if (q->ns == 0) return da;
    if (q->type == LIQUID_RESAMP_INTERP) return dh / q->rate_arb + da;
    return dh + q->M * da;
}

static void lq_ms_print(lq_ms *q)
{
    printf("multi-stage resampler\n");
    printf("    composite rate      : %12.10f\n", q->rate);
    printf("    type                : %s\n", q->type == LIQUID_RESAMP_INTERP ? "interp" : "decim");
    printf("    num halfband stages : %u\n", q->ns);
    printf("    halfband rate       : %s%u\n", q->type == LIQUID_RESAMP_INTERP ? "" : "1/", q->M);
    printf("    arbitrary rate      : %12.10f\n", q->rate_arb);
}

static unsigned long long lq_ms_num_output(lq_ms *q, unsigned long long nx)
{
    if (q->type == LIQUID_RESAMP_INTERP) return lq_rs_num_output(q->rs, nx) * q->M;
    return lq_rs_num_output(q->rs, (q->bi + nx) / q->M);
}

static void lq_ms_hb_run(void *ctx, const void *u, unsigned long long n, void *y)
{
    lq_r2_run_dev((lq_r2 *)ctx, LQK_R2_INTERP, u, n, y, NULL, 1.0f);
}

static void lq_ms_block_dev(lq_ms *q, const void *dx, unsigned long long nx, void *dy, unsigned long long *ny)
{
    unsigned long long n = 0;
    if (nx > 0 && q->type == LIQUID_RESAMP_INTERP) {
        lq_r2 *h = q->ns ? q->hb->st[q->ns - 1] : NULL;   /* the first half-band stage applied */
        if (q->ns == 0) {
            lq_rs_block_dev(q->rs, dx, nx, dy, &n);
        } else if (q->kind != LQ_RRRF && h->m <= LQK_RS4_HB_MAXM) {
            /* the resampler and the first half-band stage as one chain
             * (msresamp.c:289-300: every resampler output straight into the
             * half-band interpolator), the later stages after it */
            lq_rs_hb hb;
            memset(&hb, 0, sizeof(hb));
            hb.m = (int)h->m;
            const unsigned int cw = h->csz / 4;   /* cccf: (re, im) taps, im = 0 (f0 = 0) */
            for (unsigned int j = 0; j < 2 * h->m; j++) hb.h1[j] = h->h[(h->h_len - 2 * j - 2) * cw];
            for (int b = 0; b < 2; b++)
                for (int w = 0; w < 2; w++) hb.w[b][w] = h->d_w[b][w];
            hb.cur = &h->cur;
            hb.run = lq_ms_hb_run;
            hb.ctx = h;
            const unsigned long long K = lq_rs_num_output(q->rs, nx);
            void *t = q->ns > 1 ? lq_devbuf_get(&q->s0, (size_t)(K ? 2 * K : 1) * q->esz) : dy;
            unsigned long long k2 = 0;
            lq_rs_block_dev_hb(q->rs, dx, nx, t, &k2, &hb);
            const void *in = t;
            void *b2[2] = {NULL, NULL};
            for (unsigned int s = 1; s < q->ns; s++) {
                const int last = s == q->ns - 1;
                /* stage s writes k2 << s samples: grow the buffer for every
                 * stage (the one of index s & 1 served stage s - 2 with half) */
                if (!last) b2[s & 1] = lq_devbuf_get(&q->hb->buf[s & 1], (size_t)(k2 << s) * q->esz);
                void *out = last ? dy : b2[s & 1];
                lq_r2_run_dev(q->hb->st[q->ns - s - 1], LQK_R2_INTERP, in, k2 << (s - 1), out, NULL, 1.0f);
                in = out;
            }
            n = (k2 / 2) * q->M;
        } else {
            const unsigned long long K = lq_rs_num_output(q->rs, nx);
            void *t = lq_devbuf_get(&q->s0, (size_t)(K ? K : 1) * q->esz);
            unsigned long long k = 0;
            lq_rs_block_dev(q->rs, dx, nx, t, &k);
            lq_ms2_block_dev(q->hb, t, k, dy);
            n = k * q->M;
        }
    } else if (nx > 0) {
        const unsigned long long tot = q->bi + nx, g = tot / q->M, rem = tot - g * q->M;
        const char *src = (const char *)dx;
        if (q->bi > 0 && g > 0) {   /* pending inputs first: make the groups contiguous */
            char *c = (char *)lq_devbuf_get(&q->s1, (size_t)tot * q->esz);
            lqrt_d2d(c, q->d_pend, (size_t)q->bi * q->esz, q->ctx.stream);
            lqrt_d2d(c + (size_t)q->bi * q->esz, dx, (size_t)nx * q->esz, q->ctx.stream);
            src = c;
        }
        if (g > 0) {
            void *h = q->ns ? lq_devbuf_get(&q->s0, (size_t)g * q->esz) : NULL;
            if (q->ns) lq_ms2_block_dev(q->hb, src, g, h);
            lq_rs_block_dev(q->rs, q->ns ? h : src, g, dy, &n);
            if (rem) lqrt_d2d(q->d_pend, src + (size_t)g * q->M * q->esz, (size_t)rem * q->esz, q->ctx.stream);
        } else {                     /* everything joins the pending group */
            lqrt_d2d((char *)q->d_pend + (size_t)q->bi * q->esz, dx, (size_t)nx * q->esz, q->ctx.stream);
        }
        q->bi = (unsigned int)rem;
    }
    if (ny) *ny = n;
}

static void lq_ms_block(lq_ms *q, const void *x, unsigned int nx, void *y, unsigned int *ny)
{
    unsigned long long nout = lq_ms_num_output(q, nx), n = 0;
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, (size_t)nx * q->esz);
    void *dy = lq_devbuf_get(&q->ybuf, (size_t)(nout ? nout : 1) * q->esz);
    lq_ms_block_dev(q, dx, nx, dy, &n);
    lq_call_out(&q->ctx, y, dy, (size_t)n * q->esz);
    *ny = (unsigned int)n;
}

#define LQ_MSRESAMP_FRONT(NAME, KIND, T)                                                            \
    struct NAME##_s {                                                                               \
        lq_ms *e;                                                                                   \
    };                                                                                              \
    NAME NAME##_create(float _r, float _As)                                                         \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = lq_ms_create(KIND, _r, _As);                                                         \
        return q;                                                                                   \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_ms_destroy(_q->e);                                                                       \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_print(NAME _q) { lq_ms_print(_q->e); }                                              \
    void NAME##_reset(NAME _q) { lq_ms_reset(_q->e); }                                              \
    float NAME##_get_delay(NAME _q) { return lq_ms_get_delay(_q->e); }                              \
    void NAME##_execute(NAME _q, T *_x, unsigned int _nx, T *_y, unsigned int *_ny)                 \
    {                                                                                               \
        lq_ms_block(_q->e, _x, _nx, _y, _ny);                                                       \
    }                                                                                               \
    unsigned long long NAME##_num_output(NAME _q, unsigned long long _nx)                           \
    {                                                                                               \
        return lq_ms_num_output(_q->e, _nx);                                                        \
    }                                                                                               \
    void NAME##_execute_block_dev(NAME _q, const T *_dx, unsigned long long _nx, T *_dy,            \
                                  unsigned long long *_ny)                                          \
    {                                                                                               \
        lq_ms_block_dev(_q->e, _dx, _nx, _dy, _ny);                                                 \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ms_set_stream(_q->e, _s); }                      \
    void NAME##_synchronize(NAME _q) { lqrt_sync(_q->e->ctx.stream); }

LQ_MSRESAMP_FRONT(msresamp_rrrf, LQ_RRRF, float)
LQ_MSRESAMP_FRONT(msresamp_crcf, LQ_CRCF, liquid_float_complex)
LQ_MSRESAMP_FRONT(msresamp_cccf, LQ_CCCF, liquid_float_complex)
