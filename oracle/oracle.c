/*
 * oracle.c -- CPU restatement of liquid-dsp's streaming filter / channelizer
 * hot path.  TEST INFRASTRUCTURE ONLY (see oracle.h): the product never links
 * this file; tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it as the checker / CPU baseline.
 *
 * Written from the reference's behaviour, not copied: each routine names the
 * reference file:line whose semantics it restates.  Arithmetic is IEEE float32
 * with -ffp-contract=off so operation order is what the C source says.
 *
 * Internal representation: every object stores coefficients and samples as
 * orc_cf.  Real types (rrrf coefficients / samples, crcf coefficients) carry a
 * zero imaginary part and use the real-coefficient multiply, so the real
 * parts are bit-identical to a float-only evaluation.
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

static void orc_fail(const char *msg)
{
    fprintf(stderr, "oracle error: %s\n", msg);
    exit(1);
}

static void *orc_calloc(size_t n, size_t sz)
{
    void *p = calloc(n ? n : 1, sz);
    if (!p) orc_fail("out of memory");
    return p;
}

/* ========================================================================= */
/* design helpers                                                            */
/* ========================================================================= */

/* liquid_msb_index, src/utility/src/msb_index.c:110-135: floor(log2 x)+1 */
unsigned int orc_msb_index(unsigned int x)
{
    unsigned int b = 0;
    while (x) { x >>= 1; b++; }
    return b;
}

/* kaiser_beta_As, src/filter/src/firdes.c:224-236 (the middle branch mixes a
 * double constant into the float expression, as the reference does) */
float orc_kaiser_beta_As(float As)
{
    As = fabsf(As);
    if (As > 50.0f)
        return 0.1102f * (As - 8.7f);
    if (As > 21.0f)
        return (float)(0.5842 * powf(As - 21, 0.4f) + 0.07886f * (As - 21));
    return 0.0f;
}

/* sincf, src/math/src/math.c:128-139 */
float orc_sincf(float x)
{
    if (fabsf(x) < 0.01f)
        return cosf(M_PI * x / 2.0f) * cosf(M_PI * x / 4.0f) * cosf(M_PI * x / 8.0f);
    return sinf(M_PI * x) / (M_PI * x);
}

/* liquid_lngammaf, src/math/src/math.gamma.c:43-72 (recursion below 10,
 * Stirling-type series above; note the double log() in the reference) */
float orc_lngammaf(float z)
{
    if (z < 0) orc_fail("lngammaf undefined for z < 0");
    if (z < 10.0f)
        return orc_lngammaf(z + 1.0f) - logf(z);
    float g = 0.5 * (logf(2 * M_PI) - log(z));
    g += z * (logf(z + (1 / (12.0f * z - 0.1f / z))) - 1);
    return g;
}

/* liquid_besseli0f, src/math/src/math.bessel.c:86-104 (32-term log series) */
float orc_besseli0f(float z)
{
    if (z == 0.0f) return 1.0f;
    float y = 0.0f;
    for (unsigned int k = 0; k < 32; k++) {
        float t = k * logf(0.5f * z) - orc_lngammaf((float)k + 1.0f);
        y += expf(2 * t);
    }
    return y;
}

/* kaiser, src/math/src/math.c:289-312 */
float orc_kaiser(unsigned int n, unsigned int N, float beta, float mu)
{
    float t = (float)n - (float)(N - 1) / 2 + mu;
    float r = 2.0f * t / (float)N;
    return orc_besseli0f(beta * sqrtf(1 - r * r)) / orc_besseli0f(beta);
}

/* liquid_firdes_kaiser, src/filter/src/firdes.c:244-281 */
void orc_firdes_kaiser(unsigned int n, float fc, float As, float mu, float *h)
{
    if (mu < -0.5f || mu > 0.5f || fc < 0.0f || fc > 0.5f || n == 0)
        orc_fail("firdes_kaiser: bad argument");
    float beta = orc_kaiser_beta_As(As);
    for (unsigned int i = 0; i < n; i++) {
        float t = (float)i - (float)(n - 1) / 2 + mu;
        h[i] = orc_sincf(2.0f * fc * t) * orc_kaiser(i, n, beta, mu);
    }
}

/* ========================================================================= */
/* dot products: src/dotprod/src/dotprod.c:63-89 (_run4: 4-way unrolled but  */
/* sequential accumulation into one accumulator)                             */
/* ========================================================================= */

void orc_dotprod_rrrf_run4(const float *h, const float *x, unsigned int n, float *y)
{
    float r = 0;
    for (unsigned int i = 0; i < n; i++) r += h[i] * x[i];
    *y = r;
}

void orc_dotprod_crcf_run4(const float *h, const orc_cf *x, unsigned int n, orc_cf *y)
{
    float re = 0, im = 0;
    for (unsigned int i = 0; i < n; i++) {
        re += h[i] * crealf(x[i]);
        im += h[i] * cimagf(x[i]);
    }
    *y = CMPLXF(re, im);
}

void orc_dotprod_cccf_run4(const orc_cf *h, const orc_cf *x, unsigned int n, orc_cf *y)
{
    float re = 0, im = 0;
    for (unsigned int i = 0; i < n; i++) {
        float hr = crealf(h[i]), hi = cimagf(h[i]);
        float xr = crealf(x[i]), xi = cimagf(x[i]);
        re += hr * xr - hi * xi;
        im += hr * xi + hi * xr;
    }
    *y = CMPLXF(re, im);
}

void orc_dotprod_rrrf_batch(const float *h, const float *X, unsigned int n, unsigned long nvec, float *Y)
{
    for (unsigned long v = 0; v < nvec; v++) orc_dotprod_rrrf_run4(h, X + v * n, n, Y + v);
}
void orc_dotprod_crcf_batch(const float *h, const orc_cf *X, unsigned int n, unsigned long nvec, orc_cf *Y)
{
    for (unsigned long v = 0; v < nvec; v++) orc_dotprod_crcf_run4(h, X + v * n, n, Y + v);
}
void orc_dotprod_cccf_batch(const orc_cf *h, const orc_cf *X, unsigned int n, unsigned long nvec, orc_cf *Y)
{
    for (unsigned long v = 0; v < nvec; v++) orc_dotprod_cccf_run4(h, X + v * n, n, Y + v);
}

/* generic dot used by the objects: coefficients real (type != CCCF) or complex */
static inline orc_cf orc_dot(int cplx_h, const orc_cf *h, const orc_cf *x, unsigned int n)
{
    float re = 0, im = 0;
    if (!cplx_h) {
        for (unsigned int i = 0; i < n; i++) {
            float hr = crealf(h[i]);
            re += hr * crealf(x[i]);
            im += hr * cimagf(x[i]);
        }
    } else {
        for (unsigned int i = 0; i < n; i++) {
            float hr = crealf(h[i]), hi = cimagf(h[i]);
            float xr = crealf(x[i]), xi = cimagf(x[i]);
            re += hr * xr - hi * xi;
            im += hr * xi + hi * xr;
        }
    }
    return CMPLXF(re, im);
}

static inline orc_cf orc_mul(int cplx, orc_cf a, orc_cf b)
{
    if (!cplx) return CMPLXF(crealf(a) * crealf(b), crealf(a) * cimagf(b));
    float ar = crealf(a), ai = cimagf(a), br = crealf(b), bi = cimagf(b);
    return CMPLXF(ar * br - ai * bi, ar * bi + ai * br);
}

/* load `n` coefficients or samples of the given element kind into orc_cf */
static void orc_load(int is_complex, const void *src, unsigned int n, orc_cf *dst)
{
    if (is_complex) {
        memcpy(dst, src, n * sizeof(orc_cf));
    } else {
        const float *f = (const float *)src;
        for (unsigned int i = 0; i < n; i++) dst[i] = CMPLXF(f[i], 0.0f);
    }
}

static void orc_store(int is_complex, const orc_cf *src, unsigned int n, void *dst)
{
    if (is_complex) {
        memcpy(dst, src, n * sizeof(orc_cf));
    } else {
        float *f = (float *)dst;
        for (unsigned int i = 0; i < n; i++) f[i] = crealf(src[i]);
    }
}

/* ========================================================================= */
/* window: src/buffer/src/window.c:45-214 -- ring of 2^msb(len) + len - 1     */
/* entries; push advances the read index and, on wrap, moves the newest       */
/* len-1 values back to the front; read returns the oldest of the last len.   */
/* ========================================================================= */

typedef struct {
    orc_cf *v;
    unsigned int len, n, mask, ri;
} orc_window;

static void orc_window_init(orc_window *w, unsigned int len)
{
    if (len == 0) orc_fail("window length must be > 0");
    w->len = len;
    w->n = 1u << orc_msb_index(len);
    w->mask = w->n - 1;
    w->v = (orc_cf *)orc_calloc(w->n + len - 1, sizeof(orc_cf));
    w->ri = 0;
}

static void orc_window_clear(orc_window *w)
{
    w->ri = 0;
    memset(w->v, 0, (w->n + w->len - 1) * sizeof(orc_cf));
}

static inline void orc_window_push(orc_window *w, orc_cf x)
{
    w->ri = (w->ri + 1) & w->mask;
    if (w->ri == 0) memmove(w->v, w->v + w->n, (w->len - 1) * sizeof(orc_cf));
    w->v[w->ri + w->len - 1] = x;
}

static inline const orc_cf *orc_window_read(const orc_window *w) { return w->v + w->ri; }

/* ========================================================================= */
/* FFT: plain mixed-radix decimation-in-time, float accumulation, twiddles   */
/* from double.  Convention of src/fft/src/fft_common.c / liquid.h:1122-1123: */
/* dir=+1 forward (e^{-j2pi nk/N}), dir=-1 backward (e^{+j...}), unscaled.    */
/* ========================================================================= */

static unsigned int orc_smallest_factor(unsigned int n)
{
    if (n % 4 == 0) return 4;
    for (unsigned int p = 2; p * p <= n; p++)
        if (n % p == 0) return p;
    return n;
}

static void orc_fft_rec(unsigned int n, const orc_cf *x, unsigned int xs, orc_cf *y, int dir)
{
    if (n == 1) { y[0] = x[0]; return; }
    unsigned int p = orc_smallest_factor(n);
    double sgn = dir > 0 ? -1.0 : 1.0;
    if (p == n) {
        for (unsigned int k = 0; k < n; k++) {
            float re = 0, im = 0;
            for (unsigned int j = 0; j < n; j++) {
                double a = sgn * 2.0 * M_PI * (double)((unsigned long)j * k % n) / (double)n;
                float c = (float)cos(a), s = (float)sin(a);
                float xr = crealf(x[j * xs]), xi = cimagf(x[j * xs]);
                re += xr * c - xi * s;
                im += xr * s + xi * c;
            }
            y[k] = CMPLXF(re, im);
        }
        return;
    }
    unsigned int m = n / p;
    orc_cf *t = (orc_cf *)orc_calloc(n, sizeof(orc_cf));
    for (unsigned int r = 0; r < p; r++) orc_fft_rec(m, x + r * xs, xs * p, t + r * m, dir);
    for (unsigned int k = 0; k < m; k++) {
        for (unsigned int q = 0; q < p; q++) {
            unsigned int kk = k + m * q;
            float re = 0, im = 0;
            for (unsigned int r = 0; r < p; r++) {
                double a = sgn * 2.0 * M_PI * (double)((unsigned long)r * kk % n) / (double)n;
                float c = (float)cos(a), s = (float)sin(a);
                float tr = crealf(t[r * m + k]), ti = cimagf(t[r * m + k]);
                re += tr * c - ti * s;
                im += tr * s + ti * c;
            }
            y[kk] = CMPLXF(re, im);
        }
    }
    free(t);
}

void orc_fft(unsigned int n, const orc_cf *x, orc_cf *y, int dir)
{
    if (n == 0) return;
    orc_cf *tmp = (orc_cf *)orc_calloc(n, sizeof(orc_cf));
    orc_fft_rec(n, x, 1, tmp, dir);
    memcpy(y, tmp, n * sizeof(orc_cf));
    free(tmp);
}

/* radix-2 iterative FFT with a precomputed float twiddle table; used by the
 * objects whose transform sizes are powers of two (the BASELINE sizes), so the
 * oracle's CPU timing is not dominated by the generic path above. */
typedef struct {
    unsigned int n, log2n;
    int dir;
    orc_cf *tw;          /* n/2 twiddles */
    unsigned int *rev;   /* bit-reversal permutation */
} orc_fftplan;

static int orc_is_pow2(unsigned int n) { return n && !(n & (n - 1)); }

static void orc_fftplan_init(orc_fftplan *p, unsigned int n, int dir)
{
    p->n = n;
    p->dir = dir;
    p->tw = NULL;
    p->rev = NULL;
    if (!orc_is_pow2(n)) return;
    p->log2n = orc_msb_index(n) - 1;
    p->tw = (orc_cf *)orc_calloc(n / 2 ? n / 2 : 1, sizeof(orc_cf));
    p->rev = (unsigned int *)orc_calloc(n, sizeof(unsigned int));
    double sgn = dir > 0 ? -1.0 : 1.0;
    for (unsigned int k = 0; k < n / 2; k++) {
        double a = sgn * 2.0 * M_PI * k / n;
        p->tw[k] = CMPLXF((float)cos(a), (float)sin(a));
    }
    for (unsigned int i = 0; i < n; i++) {
        unsigned int r = 0;
        for (unsigned int b = 0; b < p->log2n; b++) r |= ((i >> b) & 1u) << (p->log2n - 1 - b);
        p->rev[i] = r;
    }
}

static void orc_fftplan_free(orc_fftplan *p)
{
    free(p->tw);
    free(p->rev);
}

static void orc_fftplan_execute(const orc_fftplan *p, const orc_cf *x, orc_cf *y)
{
    unsigned int n = p->n;
    if (!p->tw) { orc_fft(n, x, y, p->dir); return; }
    if (x == y) {
        orc_cf *t = (orc_cf *)orc_calloc(n, sizeof(orc_cf));
        memcpy(t, x, n * sizeof(orc_cf));
        for (unsigned int i = 0; i < n; i++) y[p->rev[i]] = t[i];
        free(t);
    } else {
        for (unsigned int i = 0; i < n; i++) y[p->rev[i]] = x[i];
    }
    for (unsigned int len = 2; len <= n; len <<= 1) {
        unsigned int half = len >> 1, step = n / len;
        for (unsigned int s = 0; s < n; s += len) {
            for (unsigned int k = 0; k < half; k++) {
                orc_cf w = p->tw[k * step];
                float wr = crealf(w), wi = cimagf(w);
                orc_cf b = y[s + k + half];
                float br = crealf(b), bi = cimagf(b);
                float tr = br * wr - bi * wi, ti = br * wi + bi * wr;
                orc_cf a = y[s + k];
                y[s + k] = CMPLXF(crealf(a) + tr, cimagf(a) + ti);
                y[s + k + half] = CMPLXF(crealf(a) - tr, cimagf(a) - ti);
            }
        }
    }
}

/* ========================================================================= */
/* firfilt: src/filter/src/firfilt.c:62-359                                  */
/* ========================================================================= */

struct orc_firfilt_s {
    int type;
    unsigned int h_len;
    orc_cf *hr;          /* coefficients, reversed (firfilt.c:89-90) */
    orc_cf *w;           /* own ring (firfilt.c:81-84): w_len + h_len + 1 */
    unsigned int w_len, w_mask, w_index;
    orc_cf scale;
};

orc_firfilt orc_firfilt_create(int type, const void *h, unsigned int n)
{
    if (n == 0) orc_fail("firfilt: filter length must be greater than zero");
    orc_firfilt q = (orc_firfilt)orc_calloc(1, sizeof(*q));
    q->type = type;
    q->h_len = n;
    orc_cf *tmp = (orc_cf *)orc_calloc(n, sizeof(orc_cf));
    orc_load(type == ORC_CCCF, h, n, tmp);
    q->hr = (orc_cf *)orc_calloc(n, sizeof(orc_cf));
    for (unsigned int i = 0; i < n; i++) q->hr[i] = tmp[n - 1 - i];
    free(tmp);
    q->w_len = 1u << orc_msb_index(n);
    q->w_mask = q->w_len - 1;
    q->w = (orc_cf *)orc_calloc(q->w_len + n + 1, sizeof(orc_cf));
    q->scale = 1.0f;
    orc_firfilt_reset(q);
    return q;
}

void orc_firfilt_destroy(orc_firfilt q) { free(q->hr); free(q->w); free(q); }

void orc_firfilt_reset(orc_firfilt q)
{
    memset(q->w, 0, (q->w_len + q->h_len + 1) * sizeof(orc_cf));
    q->w_index = 0;
}

void orc_firfilt_set_scale(orc_firfilt q, float re, float im) { q->scale = CMPLXF(re, im); }

static inline void orc_firfilt_push1(orc_firfilt q, orc_cf x)
{
    q->w_index = (q->w_index + 1) & q->w_mask;
    if (q->w_index == 0) memmove(q->w, q->w + q->w_len, q->h_len * sizeof(orc_cf));
    q->w[q->w_index + q->h_len - 1] = x;
}

static inline orc_cf orc_firfilt_exec1(orc_firfilt q)
{
    orc_cf y = orc_dot(q->type == ORC_CCCF, q->hr, q->w + q->w_index, q->h_len);
    return orc_mul(q->type == ORC_CCCF, q->scale, y);
}

void orc_firfilt_push(orc_firfilt q, const void *x)
{
    orc_cf v;
    orc_load(q->type != ORC_RRRF, x, 1, &v);
    orc_firfilt_push1(q, v);
}

void orc_firfilt_execute(orc_firfilt q, void *y)
{
    orc_cf v = orc_firfilt_exec1(q);
    orc_store(q->type != ORC_RRRF, &v, 1, y);
}

void orc_firfilt_execute_block(orc_firfilt q, const void *x, unsigned int n, void *y)
{
    int cx = q->type != ORC_RRRF;
    for (unsigned int i = 0; i < n; i++) {
        orc_cf v;
        if (cx) v = ((const orc_cf *)x)[i]; else v = CMPLXF(((const float *)x)[i], 0.0f);
        orc_firfilt_push1(q, v);
        orc_cf o = orc_firfilt_exec1(q);
        if (cx) ((orc_cf *)y)[i] = o; else ((float *)y)[i] = crealf(o);
    }
}

/* ========================================================================= */
/* firdecim: src/filter/src/firdecim.c:47-223                                */
/* ========================================================================= */

struct orc_firdecim_s {
    int type;
    unsigned int M, h_len;
    orc_cf *hr;
    orc_window w;
};

orc_firdecim orc_firdecim_create(int type, unsigned int M, const void *h, unsigned int h_len)
{
    if (h_len == 0 || M == 0) orc_fail("firdecim: bad argument");
    orc_firdecim q = (orc_firdecim)orc_calloc(1, sizeof(*q));
    q->type = type;
    q->M = M;
    q->h_len = h_len;
    orc_cf *tmp = (orc_cf *)orc_calloc(h_len, sizeof(orc_cf));
    orc_load(type == ORC_CCCF, h, h_len, tmp);
    q->hr = (orc_cf *)orc_calloc(h_len, sizeof(orc_cf));
    for (unsigned int i = 0; i < h_len; i++) q->hr[i] = tmp[h_len - i - 1];
    free(tmp);
    orc_window_init(&q->w, h_len);
    return q;
}

/* firdecim.c:88-122: 2*M*m+1 Kaiser taps at fc = 0.5/M, first 2*M*m used */
orc_firdecim orc_firdecim_create_kaiser(unsigned int M, unsigned int m, float As)
{
    unsigned int n = 2 * M * m + 1;
    float *hf = (float *)orc_calloc(n, sizeof(float));
    orc_firdes_kaiser(n, 0.5f / (float)M, As, 0.0f, hf);
    orc_firdecim q = orc_firdecim_create(ORC_CRCF, M, hf, 2 * M * m);
    free(hf);
    return q;
}

void orc_firdecim_destroy(orc_firdecim q) { free(q->hr); free(q->w.v); free(q); }
void orc_firdecim_clear(orc_firdecim q) { orc_window_clear(&q->w); }

/* firdecim.c:189-223: the output is computed right after the FIRST of the M
 * pushes of each output period */
void orc_firdecim_execute_block(orc_firdecim q, const void *x, unsigned int n, void *y)
{
    int cx = q->type != ORC_RRRF;
    for (unsigned int o = 0; o < n; o++) {
        for (unsigned int i = 0; i < q->M; i++) {
            size_t idx = (size_t)o * q->M + i;
            orc_cf v = cx ? ((const orc_cf *)x)[idx] : CMPLXF(((const float *)x)[idx], 0.0f);
            orc_window_push(&q->w, v);
            if (i == 0) {
                orc_cf r = orc_dot(q->type == ORC_CCCF, q->hr, orc_window_read(&q->w), q->h_len);
                if (cx) ((orc_cf *)y)[o] = r; else ((float *)y)[o] = crealf(r);
            }
        }
    }
}

/* ========================================================================= */
/* firpfb: src/filter/src/firpfb.c:46-345                                    */
/* ========================================================================= */

struct orc_firpfb_s {
    int type;
    unsigned int M, h_sub_len;
    orc_cf *hs;          /* M x h_sub_len, each sub-filter reversed (firpfb.c:73-84) */
    orc_window w;
    float scale;
};

orc_firpfb orc_firpfb_create(int type, unsigned int M, const void *h, unsigned int h_len)
{
    if (M == 0 || h_len == 0) orc_fail("firpfb: bad argument");
    orc_firpfb q = (orc_firpfb)orc_calloc(1, sizeof(*q));
    q->type = type;
    q->M = M;
    q->h_sub_len = h_len / M;
    orc_cf *tmp = (orc_cf *)orc_calloc(h_len, sizeof(orc_cf));
    orc_load(type == ORC_CCCF, h, h_len, tmp);
    q->hs = (orc_cf *)orc_calloc((size_t)M * (q->h_sub_len ? q->h_sub_len : 1), sizeof(orc_cf));
    for (unsigned int i = 0; i < M; i++)
        for (unsigned int n = 0; n < q->h_sub_len; n++)
            q->hs[(size_t)i * q->h_sub_len + (q->h_sub_len - n - 1)] = tmp[i + n * M];
    free(tmp);
    orc_window_init(&q->w, q->h_sub_len);
    q->scale = 1.0f;
    return q;
}

void orc_firpfb_destroy(orc_firpfb q) { free(q->hs); free(q->w.v); free(q); }
void orc_firpfb_reset(orc_firpfb q) { orc_window_clear(&q->w); }
void orc_firpfb_set_scale(orc_firpfb q, float s) { q->scale = s; }

void orc_firpfb_push(orc_firpfb q, const void *x)
{
    orc_cf v;
    orc_load(q->type != ORC_RRRF, x, 1, &v);
    orc_window_push(&q->w, v);
}

static inline orc_cf orc_firpfb_exec1(orc_firpfb q, unsigned int i)
{
    if (i >= q->M) orc_fail("firpfb: filterbank index exceeds maximum");
    orc_cf y = orc_dot(q->type == ORC_CCCF, q->hs + (size_t)i * q->h_sub_len,
                       orc_window_read(&q->w), q->h_sub_len);
    return CMPLXF(crealf(y) * q->scale, cimagf(y) * q->scale);
}

void orc_firpfb_execute(orc_firpfb q, unsigned int i, void *y)
{
    orc_cf v = orc_firpfb_exec1(q, i);
    orc_store(q->type != ORC_RRRF, &v, 1, y);
}

/* ========================================================================= */
/* firinterp: src/filter/src/firinterp.c:43-215 (firpfb of L=ceil(h/M) taps) */
/* ========================================================================= */

struct orc_firinterp_s {
    int type;
    unsigned int M;
    orc_firpfb pfb;
};

orc_firinterp orc_firinterp_create(int type, unsigned int M, const void *h, unsigned int h_len)
{
    if (M < 2 || h_len < M) orc_fail("firinterp: bad argument");
    orc_firinterp q = (orc_firinterp)orc_calloc(1, sizeof(*q));
    q->type = type;
    q->M = M;
    unsigned int L = 0;
    while (M * L < h_len) L++;
    unsigned int hl = M * L;
    orc_cf *hp = (orc_cf *)orc_calloc(hl, sizeof(orc_cf));
    orc_load(type == ORC_CCCF, h, h_len, hp);     /* tail stays zero (firinterp.c:68-73) */
    q->pfb = orc_firpfb_create(ORC_CCCF, M, hp, hl);
    q->pfb->type = type;                          /* keep real-coefficient arithmetic */
    free(hp);
    return q;
}

orc_firinterp orc_firinterp_create_kaiser(unsigned int M, unsigned int m, float As)
{
    unsigned int n = 2 * M * m + 1;
    float *hf = (float *)orc_calloc(n, sizeof(float));
    orc_firdes_kaiser(n, 0.5f / (float)M, As, 0.0f, hf);
    orc_firinterp q = orc_firinterp_create(ORC_CRCF, M, hf, 2 * M * m);
    free(hf);
    return q;
}

void orc_firinterp_destroy(orc_firinterp q) { orc_firpfb_destroy(q->pfb); free(q); }
void orc_firinterp_reset(orc_firinterp q) { orc_firpfb_reset(q->pfb); }

void orc_firinterp_execute_block(orc_firinterp q, const void *x, unsigned int n, void *y)
{
    int cx = q->type != ORC_RRRF;
    for (unsigned int i = 0; i < n; i++) {
        orc_cf v = cx ? ((const orc_cf *)x)[i] : CMPLXF(((const float *)x)[i], 0.0f);
        orc_window_push(&q->pfb->w, v);
        for (unsigned int p = 0; p < q->M; p++) {
            orc_cf o = orc_firpfb_exec1(q->pfb, p);
            size_t k = (size_t)i * q->M + p;
            if (cx) ((orc_cf *)y)[k] = o; else ((float *)y)[k] = crealf(o);
        }
    }
}

/* ========================================================================= */
/* resamp_crcf: src/filter/src/resamp.c:79-363                               */
/* ========================================================================= */

enum { ORC_RS_BOUNDARY = 0, ORC_RS_INTERP = 1 };

struct orc_resamp_s {
    float rate, del, tau, bf, mu;
    int b, state;
    unsigned int npfb, m;
    orc_cf y0, y1;
    orc_firpfb f;
};

orc_resamp orc_resamp_create(float rate, unsigned int m, float fc, float As, unsigned int npfb)
{
    if (rate <= 0 || m == 0 || npfb == 0 || fc <= 0.0f || fc >= 0.5f || As <= 0.0f)
        orc_fail("resamp: bad argument");
    orc_resamp q = (orc_resamp)orc_calloc(1, sizeof(*q));
    q->rate = rate;
    q->del = 1.0f / rate;                      /* resamp.c:204-217 */
    q->m = m;
    q->npfb = npfb;
    unsigned int n = 2 * m * npfb + 1;         /* resamp.c:117-132 */
    float *hf = (float *)orc_calloc(n, sizeof(float));
    orc_firdes_kaiser(n, fc / ((float)npfb), As, 0.0f, hf);
    float gain = 0.0f;
    for (unsigned int i = 0; i < n; i++) gain += hf[i];
    gain = (npfb) / (gain);
    for (unsigned int i = 0; i < n; i++) hf[i] = hf[i] * gain;
    q->f = orc_firpfb_create(ORC_CRCF, npfb, hf, n - 1);
    free(hf);
    orc_resamp_reset(q);
    return q;
}

void orc_resamp_destroy(orc_resamp q) { orc_firpfb_destroy(q->f); free(q); }

void orc_resamp_reset(orc_resamp q)          /* resamp.c:181-195 */
{
    orc_firpfb_reset(q->f);
    q->state = ORC_RS_INTERP;
    q->tau = 0.0f;
    q->bf = 0.0f;
    q->b = 0;
    q->mu = 0.0f;
    q->y0 = 0;
    q->y1 = 0;
}

void orc_resamp_set_rate(orc_resamp q, float rate)   /* resamp.c:204-217 */
{
    if (rate <= 0) orc_fail("resamp: bad rate");
    q->rate = rate;
    q->del = 1.0f / q->rate;
}

void orc_resamp_adjust_rate(orc_resamp q, float delta)   /* resamp.c:222-239 (clips to [-0.5,0.5]) */
{
    if (delta > 0.1f || delta < -0.1f) orc_fail("resamp: bad rate adjustment");
    q->rate += delta;
    if (q->rate > 0.5f) q->rate = 0.5f;
    if (q->rate < -0.5f) q->rate = -0.5f;
    q->del = 1.0f / q->rate;
}

static inline void orc_resamp_update_timing(orc_resamp q)   /* resamp.c:352-363 */
{
    q->tau += q->del;
    q->bf = q->tau * (float)(q->npfb);
    q->b = (int)floorf(q->bf);
    q->mu = q->bf - (float)(q->b);
}

static inline orc_cf orc_lerp(float mu, orc_cf y0, orc_cf y1)
{
    float a = 1.0f - mu;
    return CMPLXF(a * crealf(y0) + mu * crealf(y1), a * cimagf(y0) + mu * cimagf(y1));
}

/* resamp.c:245-311 */
static unsigned int orc_resamp_exec1(orc_resamp q, orc_cf x, orc_cf *y)
{
    orc_window_push(&q->f->w, x);
    unsigned int n = 0;
    while ((unsigned int)q->b < q->npfb) {   /* int vs unsigned in resamp.c:254: an unsigned compare */
        if (q->state == ORC_RS_BOUNDARY) {
            q->y1 = orc_firpfb_exec1(q->f, 0);
            y[n++] = orc_lerp(q->mu, q->y0, q->y1);
            orc_resamp_update_timing(q);
            q->state = ORC_RS_INTERP;
        } else {
            q->y0 = orc_firpfb_exec1(q->f, (unsigned int)q->b);
            if (q->b == (int)q->npfb - 1) {
                q->state = ORC_RS_BOUNDARY;
                q->b = q->npfb;
            } else {
                q->y1 = orc_firpfb_exec1(q->f, (unsigned int)q->b + 1);
                y[n++] = orc_lerp(q->mu, q->y0, q->y1);
                orc_resamp_update_timing(q);
            }
        }
    }
    q->tau -= 1.0f;
    q->bf -= (float)(q->npfb);
    q->b = (int)((unsigned int)q->b - q->npfb);   /* resamp.c:307, unsigned arithmetic */
    return n;
}

void orc_resamp_execute_block(orc_resamp q, const orc_cf *x, unsigned int nx, orc_cf *y, unsigned int *ny)
{
    unsigned int k = 0;
    for (unsigned int i = 0; i < nx; i++) k += orc_resamp_exec1(q, x[i], y + k);
    *ny = k;
}

/* The same state machine with the data path removed: it records, for every
 * output, which filter pair it uses and its mu, bit for bit. */
unsigned long orc_resamp_schedule(float rate, unsigned int npfb, unsigned long nx,
                                  int *bo, float *muo, unsigned int *in_idx, unsigned long cap)
{
    float del = 1.0f / rate, tau = 0.0f, bf = 0.0f, mu = 0.0f;
    int b = 0, state = ORC_RS_INTERP;
    unsigned long k = 0;
    for (unsigned long i = 0; i < nx; i++) {
        while ((unsigned int)b < npfb) {
            if (state == ORC_RS_BOUNDARY) {
                if (k < cap) { bo[k] = -1; muo[k] = mu; in_idx[k] = (unsigned int)i; }
                k++;
                tau += del; bf = tau * (float)npfb; b = (int)floorf(bf); mu = bf - (float)b;
                state = ORC_RS_INTERP;
            } else if (b == (int)npfb - 1) {
                state = ORC_RS_BOUNDARY;
                b = npfb;
            } else {
                if (k < cap) { bo[k] = b; muo[k] = mu; in_idx[k] = (unsigned int)i; }
                k++;
                tau += del; bf = tau * (float)npfb; b = (int)floorf(bf); mu = bf - (float)b;
            }
        }
        tau -= 1.0f;
        bf -= (float)npfb;
        b = (int)((unsigned int)b - npfb);
    }
    return k;
}

/* ========================================================================= */
/* fftfilt: src/filter/src/fftfilt.c:69-260 (overlap-add, nfft = 2n)         */
/* ========================================================================= */

struct orc_fftfilt_s {
    int type;
    unsigned int h_len, n;
    orc_cf *time_buf, *freq_buf, *H, *w;
    orc_fftplan fwd, inv;
    float scale;
};

orc_fftfilt orc_fftfilt_create(int type, const void *h, unsigned int h_len, unsigned int n)
{
    if (h_len == 0 || n < h_len - 1) orc_fail("fftfilt: bad argument");
    orc_fftfilt q = (orc_fftfilt)orc_calloc(1, sizeof(*q));
    q->type = type;
    q->h_len = h_len;
    q->n = n;
    q->time_buf = (orc_cf *)orc_calloc(2 * n, sizeof(orc_cf));
    q->freq_buf = (orc_cf *)orc_calloc(2 * n, sizeof(orc_cf));
    q->H = (orc_cf *)orc_calloc(2 * n, sizeof(orc_cf));
    q->w = (orc_cf *)orc_calloc(n, sizeof(orc_cf));
    orc_fftplan_init(&q->fwd, 2 * n, +1);
    orc_fftplan_init(&q->inv, 2 * n, -1);
    orc_load(type == ORC_CCCF, h, h_len, q->time_buf);     /* zero padded to 2n */
    orc_fftplan_execute(&q->fwd, q->time_buf, q->H);
    orc_fftfilt_set_scale(q, 1.0f);
    orc_fftfilt_reset(q);
    return q;
}

void orc_fftfilt_destroy(orc_fftfilt q)
{
    free(q->time_buf); free(q->freq_buf); free(q->H); free(q->w);
    orc_fftplan_free(&q->fwd); orc_fftplan_free(&q->inv);
    free(q);
}

void orc_fftfilt_reset(orc_fftfilt q) { memset(q->w, 0, q->n * sizeof(orc_cf)); }

void orc_fftfilt_set_scale(orc_fftfilt q, float s) { q->scale = s / (float)(2 * q->n); } /* :182-187 */

void orc_fftfilt_execute(orc_fftfilt q, const void *x, void *y)
{
    unsigned int n = q->n;
    int cx = q->type != ORC_RRRF;
    orc_load(cx, x, n, q->time_buf);
    memset(q->time_buf + n, 0, n * sizeof(orc_cf));
    orc_fftplan_execute(&q->fwd, q->time_buf, q->freq_buf);
    for (unsigned int i = 0; i < 2 * n; i++) q->freq_buf[i] = orc_mul(1, q->freq_buf[i], q->H[i]);
    orc_fftplan_execute(&q->inv, q->freq_buf, q->time_buf);
    for (unsigned int i = 0; i < n; i++) {
        orc_cf s = q->time_buf[i] + q->w[i];
        if (cx) ((orc_cf *)y)[i] = CMPLXF(crealf(s) * q->scale, cimagf(s) * q->scale);
        else ((float *)y)[i] = crealf(s) * q->scale;
    }
    memmove(q->w, q->time_buf + n, n * sizeof(orc_cf));
}

/* ========================================================================= */
/* firpfbch_crcf: src/multichannel/src/firpfbch.c:73-409                     */
/* ========================================================================= */

struct orc_firpfbch_s {
    int type;
    unsigned int M, p;
    orc_cf *hs;              /* M x p reversed sub-filters (firpfbch.c:108-121) */
    orc_window *w;
    unsigned int filter_index;
    orc_fftplan fft;
    orc_cf *X, *x;
};

orc_firpfbch orc_firpfbch_create(int type, unsigned int M, unsigned int p, const float *h)
{
    if ((type != 0 && type != 1) || M == 0 || p == 0) orc_fail("firpfbch: bad argument");
    orc_firpfbch q = (orc_firpfbch)orc_calloc(1, sizeof(*q));
    q->type = type;
    q->M = M;
    q->p = p;
    q->hs = (orc_cf *)orc_calloc((size_t)M * p, sizeof(orc_cf));
    q->w = (orc_window *)orc_calloc(M, sizeof(orc_window));
    for (unsigned int i = 0; i < M; i++) {
        for (unsigned int n = 0; n < p; n++)
            q->hs[(size_t)i * p + (p - n - 1)] = CMPLXF(h[i + n * M], 0.0f);
        orc_window_init(&q->w[i], p);
    }
    q->X = (orc_cf *)orc_calloc(M, sizeof(orc_cf));
    q->x = (orc_cf *)orc_calloc(M, sizeof(orc_cf));
    orc_fftplan_init(&q->fft, M, type == 0 ? +1 : -1);
    orc_firpfbch_reset(q);
    return q;
}

/* firpfbch.c:150-184: 2*M*m+1 Kaiser taps at fc = 0.5/M, p = 2m */
orc_firpfbch orc_firpfbch_create_kaiser(int type, unsigned int M, unsigned int m, float As)
{
    unsigned int n = 2 * M * m + 1;
    float *h = (float *)orc_calloc(n, sizeof(float));
    orc_firdes_kaiser(n, 0.5f / (float)M, fabsf(As), 0.0f, h);
    orc_firpfbch q = orc_firpfbch_create(type, M, 2 * m, h);
    free(h);
    return q;
}

void orc_firpfbch_destroy(orc_firpfbch q)
{
    for (unsigned int i = 0; i < q->M; i++) free(q->w[i].v);
    free(q->w); free(q->hs); free(q->X); free(q->x);
    orc_fftplan_free(&q->fft);
    free(q);
}

void orc_firpfbch_reset(orc_firpfbch q)
{
    for (unsigned int i = 0; i < q->M; i++) {
        orc_window_clear(&q->w[i]);
        q->x[i] = 0;
        q->X[i] = 0;
    }
    q->filter_index = q->M - 1;
}

/* firpfbch.c:346-409 */
void orc_firpfbch_analyzer_execute(orc_firpfbch q, const orc_cf *x, orc_cf *y)
{
    unsigned int M = q->M;
    for (unsigned int i = 0; i < M; i++) {
        orc_window_push(&q->w[q->filter_index], x[i]);
        q->filter_index = (q->filter_index + M - 1) % M;
    }
    for (unsigned int i = 0; i < M; i++)
        q->X[M - i - 1] = orc_dot(0, q->hs + (size_t)i * q->p, orc_window_read(&q->w[i]), q->p);
    orc_fftplan_execute(&q->fft, q->X, q->x);
    memcpy(y, q->x, M * sizeof(orc_cf));
}

/* firpfbch.c:314-336 */
void orc_firpfbch_synthesizer_execute(orc_firpfbch q, const orc_cf *x, orc_cf *y)
{
    unsigned int M = q->M;
    memcpy(q->X, x, M * sizeof(orc_cf));
    orc_fftplan_execute(&q->fft, q->X, q->x);
    for (unsigned int i = 0; i < M; i++) {
        orc_window_push(&q->w[i], q->x[i]);
        y[i] = orc_dot(0, q->hs + (size_t)i * q->p, orc_window_read(&q->w[i]), q->p);
    }
}

/* ========================================================================= */
/* firpfbch2_crcf: src/multichannel/src/firpfbch2.c:66-357                   */
/* ========================================================================= */

struct orc_firpfbch2_s {
    int type;
    unsigned int M, M2, m;
    orc_cf *hs;                /* M x 2m reversed sub-filters (firpfbch2.c:99-109) */
    orc_window *w0, *w1;
    orc_fftplan ifft;
    orc_cf *X, *x;
    int flag;
};

orc_firpfbch2 orc_firpfbch2_create(int type, unsigned int M, unsigned int m, const float *h)
{
    if ((type != 0 && type != 1) || M < 2 || M % 2 || m < 1) orc_fail("firpfbch2: bad argument");
    orc_firpfbch2 q = (orc_firpfbch2)orc_calloc(1, sizeof(*q));
    q->type = type;
    q->M = M;
    q->M2 = M / 2;
    q->m = m;
    unsigned int L = 2 * m;
    q->hs = (orc_cf *)orc_calloc((size_t)M * L, sizeof(orc_cf));
    q->w0 = (orc_window *)orc_calloc(M, sizeof(orc_window));
    q->w1 = (orc_window *)orc_calloc(M, sizeof(orc_window));
    for (unsigned int i = 0; i < M; i++) {
        for (unsigned int n = 0; n < L; n++)
            q->hs[(size_t)i * L + (L - n - 1)] = CMPLXF(h[i + n * M], 0.0f);
        orc_window_init(&q->w0[i], L);
        orc_window_init(&q->w1[i], L);
    }
    q->X = (orc_cf *)orc_calloc(M, sizeof(orc_cf));
    q->x = (orc_cf *)orc_calloc(M, sizeof(orc_cf));
    orc_fftplan_init(&q->ifft, M, -1);
    orc_firpfbch2_reset(q);
    return q;
}

/* firpfbch2.c:135-172 */
void orc_firpfbch2_prototype(int type, unsigned int M, unsigned int m, float As, float *h)
{
    unsigned int n = 2 * M * m + 1;
    float fc = (type == 0) ? 1.0f / (float)M : 0.5f / (float)M;
    orc_firdes_kaiser(n, fc, As, 0.0f, h);
    float s = 0.0f;
    for (unsigned int i = 0; i < n; i++) s += h[i];
    for (unsigned int i = 0; i < n; i++) h[i] = h[i] * (float)M / s;
}

orc_firpfbch2 orc_firpfbch2_create_kaiser(int type, unsigned int M, unsigned int m, float As)
{
    if ((type != 0 && type != 1) || M < 2 || M % 2 || m < 1) orc_fail("firpfbch2: bad argument");
    float *h = (float *)orc_calloc(2 * M * m + 1, sizeof(float));
    orc_firpfbch2_prototype(type, M, m, As, h);
    orc_firpfbch2 q = orc_firpfbch2_create(type, M, m, h);
    free(h);
    return q;
}

void orc_firpfbch2_destroy(orc_firpfbch2 q)
{
    for (unsigned int i = 0; i < q->M; i++) { free(q->w0[i].v); free(q->w1[i].v); }
    free(q->w0); free(q->w1); free(q->hs); free(q->X); free(q->x);
    orc_fftplan_free(&q->ifft);
    free(q);
}

void orc_firpfbch2_reset(orc_firpfbch2 q)
{
    for (unsigned int i = 0; i < q->M; i++) {
        orc_window_clear(&q->w0[i]);
        orc_window_clear(&q->w1[i]);
    }
    q->flag = 0;
}

/* firpfbch2.c:244-282 */
static void orc_firpfbch2_analyzer(orc_firpfbch2 q, const orc_cf *x, orc_cf *y)
{
    unsigned int M = q->M, M2 = q->M2, L = 2 * q->m;
    unsigned int base = q->flag ? M : M2;
    for (unsigned int i = 0; i < M2; i++) orc_window_push(&q->w0[base - i - 1], x[i]);
    unsigned int offset = q->flag ? M2 : 0;
    for (unsigned int i = 0; i < M; i++) {
        unsigned int j = (offset + i) % M;
        q->X[j] = orc_dot(0, q->hs + (size_t)i * L, orc_window_read(&q->w0[j]), L);
    }
    orc_fftplan_execute(&q->ifft, q->X, q->x);
    for (unsigned int i = 0; i < M; i++)
        y[i] = CMPLXF(crealf(q->x[i]) / (float)M, cimagf(q->x[i]) / (float)M);
    q->flag = 1 - q->flag;
}

/* firpfbch2.c:287-335 */
static void orc_firpfbch2_synthesizer(orc_firpfbch2 q, const orc_cf *x, orc_cf *y)
{
    unsigned int M = q->M, M2 = q->M2, L = 2 * q->m;
    memcpy(q->X, x, M * sizeof(orc_cf));
    orc_fftplan_execute(&q->ifft, q->X, q->x);
    for (unsigned int i = 0; i < M; i++) {
        float s = 1.0f / (float)M;
        q->x[i] = CMPLXF(crealf(q->x[i]) * s, cimagf(q->x[i]) * s);
        q->x[i] = CMPLXF(crealf(q->x[i]) * (float)M2, cimagf(q->x[i]) * (float)M2);
    }
    orc_window *buf = (q->flag == 0) ? q->w1 : q->w0;
    for (unsigned int i = 0; i < M; i++) orc_window_push(&buf[i], q->x[i]);
    for (unsigned int i = 0; i < M2; i++) {
        unsigned int b = (q->flag == 0) ? i : i + M2;
        const orc_cf *r0 = orc_window_read(&q->w0[b]);
        const orc_cf *r1 = orc_window_read(&q->w1[b]);
        const orc_cf *p0 = q->flag ? r0 : r1;
        const orc_cf *p1 = q->flag ? r1 : r0;
        orc_cf y0 = orc_dot(0, q->hs + (size_t)i * L, p0, L);
        orc_cf y1 = orc_dot(0, q->hs + (size_t)(i + M2) * L, p1, L);
        y[i] = y0 + y1;
    }
    q->flag = 1 - q->flag;
}

void orc_firpfbch2_execute(orc_firpfbch2 q, const orc_cf *x, orc_cf *y)
{
    if (q->type == 0) orc_firpfbch2_analyzer(q, x, y);
    else orc_firpfbch2_synthesizer(q, x, y);
}

void orc_firpfbch2_execute_block(orc_firpfbch2 q, const orc_cf *x, unsigned int nblocks, orc_cf *y)
{
    unsigned int in = q->type == 0 ? q->M2 : q->M, out = q->type == 0 ? q->M : q->M2;
    for (unsigned int b = 0; b < nblocks; b++)
        orc_firpfbch2_execute(q, x + (size_t)b * in, y + (size_t)b * out);
}


/* ========================================================================= */
/* resamp2: src/filter/src/resamp2.c:46-360                                  */
/* h[i] = sinc(t/2) kaiser(i) mod(t), t = i - 2m, i < 4m+1; the dot product  */
/* uses the odd taps h1[j] = h[4m-1-2j] against a window of 2m samples; the  */
/* delay branch reads index m-1 of the other window (:273-356).              */
/* ========================================================================= */
struct orc_resamp2_s {
    int ctaps;
    unsigned int m;
    orc_cf *h1;
    orc_window w0, w1;
    unsigned int toggle;
};

orc_resamp2 orc_resamp2_create(int ctaps, unsigned int m, float f0, float As)
{
    if (m < 2) orc_fail("resamp2: m must be at least 2");
    if (f0 < -0.5f || f0 > 0.5f) orc_fail("resamp2: f0 out of range");
    orc_resamp2 q = (orc_resamp2)orc_calloc(1, sizeof(*q));
    q->ctaps = ctaps;
    q->m = m;
    const unsigned int hl = 4 * m + 1;
    orc_cf *h = (orc_cf *)orc_calloc(hl, sizeof(orc_cf));
    const float beta = orc_kaiser_beta_As(As);
    for (unsigned int i = 0; i < hl; i++) {
        const float t = (float)i - (float)(hl - 1) / 2.0f;
        const float a = orc_sincf(t / 2.0f) * orc_kaiser(i, hl, beta, 0);
        const float c = cosf(2.0f * M_PI * t * f0);
        h[i] = ctaps ? CMPLXF(a * c, a * sinf(2.0f * M_PI * t * f0)) : CMPLXF(a * c, 0.0f);
    }
    q->h1 = (orc_cf *)orc_calloc(2 * m, sizeof(orc_cf));
    unsigned int j = 0;
    for (unsigned int i = 1; i < hl; i += 2) q->h1[j++] = h[hl - i - 1];
    free(h);
    orc_window_init(&q->w0, 2 * m);
    orc_window_init(&q->w1, 2 * m);
    return q;
}

void orc_resamp2_destroy(orc_resamp2 q)
{
    free(q->h1);
    free(q->w0.v);
    free(q->w1.v);
    free(q);
}

void orc_resamp2_clear(orc_resamp2 q)
{
    orc_window_clear(&q->w0);
    orc_window_clear(&q->w1);
    q->toggle = 0;
}

static inline orc_cf orc_r2_dot(orc_resamp2 q, const orc_window *w) { return orc_dot(q->ctaps, q->h1, orc_window_read(w), 2 * q->m); }
static inline orc_cf orc_r2_delay(orc_resamp2 q, const orc_window *w) { return orc_window_read(w)[q->m - 1]; }

void orc_resamp2_filter_execute(orc_resamp2 q, orc_cf x, orc_cf *y0, orc_cf *y1)
{
    orc_cf yi, yq;
    if (q->toggle == 0) {
        orc_window_push(&q->w0, x);
        yi = orc_r2_delay(q, &q->w0);
        yq = orc_r2_dot(q, &q->w1);
    } else {
        orc_window_push(&q->w1, x);
        yi = orc_r2_delay(q, &q->w1);
        yq = orc_r2_dot(q, &q->w0);
    }
    q->toggle = 1 - q->toggle;
    *y0 = CMPLXF(0.5f * (crealf(yi) + crealf(yq)), 0.5f * (cimagf(yi) + cimagf(yq)));
    *y1 = CMPLXF(0.5f * (crealf(yi) - crealf(yq)), 0.5f * (cimagf(yi) - cimagf(yq)));
}

void orc_resamp2_analyzer_execute(orc_resamp2 q, const orc_cf *x, orc_cf *y)
{
    orc_window_push(&q->w1, CMPLXF(0.5f * crealf(x[0]), 0.5f * cimagf(x[0])));
    const orc_cf y1 = orc_r2_dot(q, &q->w1);
    orc_window_push(&q->w0, CMPLXF(0.5f * crealf(x[1]), 0.5f * cimagf(x[1])));
    const orc_cf y0 = orc_r2_delay(q, &q->w0);
    y[0] = y1 + y0;
    y[1] = y1 - y0;
}

void orc_resamp2_synthesizer_execute(orc_resamp2 q, const orc_cf *x, orc_cf *y)
{
    orc_window_push(&q->w0, x[0] + x[1]);
    y[0] = orc_r2_delay(q, &q->w0);
    orc_window_push(&q->w1, x[0] - x[1]);
    y[1] = orc_r2_dot(q, &q->w1);
}

void orc_resamp2_decim_execute(orc_resamp2 q, const orc_cf *x, orc_cf *y)
{
    orc_window_push(&q->w1, x[0]);
    const orc_cf y1 = orc_r2_dot(q, &q->w1);
    orc_window_push(&q->w0, x[1]);
    *y = orc_r2_delay(q, &q->w0) + y1;
}

void orc_resamp2_interp_execute(orc_resamp2 q, orc_cf x, orc_cf *y)
{
    orc_window_push(&q->w0, x);
    y[0] = orc_r2_delay(q, &q->w0);
    orc_window_push(&q->w1, x);
    y[1] = orc_r2_dot(q, &q->w1);
}

/* ========================================================================= */
/* msresamp2: src/filter/src/msresamp2.c:66-354                              */
/* ========================================================================= */
struct orc_msresamp2_s {
    int type;
    unsigned int ns, M;
    float zeta;
    orc_resamp2 *st;
    orc_cf *b0, *b1;
};

/* estimate_req_filter_len (Kaiser), src/filter/src/firdes.c:52-75, 163-176 */
static unsigned int orc_req_len(float df, float As) { return (unsigned int)((As - 7.95f) / (14.26f * df)); }

orc_msresamp2 orc_msresamp2_create(int ctaps, int type, unsigned int ns, float fc, float f0, float As)
{
    if (ns > 16) orc_fail("msresamp2: too many stages");
    if (fc <= 0.0f || fc >= 0.5f) orc_fail("msresamp2: bad cutoff");
    if (fc > 0.45f) fc = 0.45f;
    f0 = 0.0f;                                  /* :109-113: non-zero center frequency unsupported */
    orc_msresamp2 q = (orc_msresamp2)orc_calloc(1, sizeof(*q));
    q->type = type == 0 ? 0 : 1;
    q->ns = ns;
    q->M = 1u << ns;
    q->zeta = 1.0f / (float)q->M;
    q->b0 = (orc_cf *)orc_calloc(q->M, sizeof(orc_cf));
    q->b1 = (orc_cf *)orc_calloc(q->M, sizeof(orc_cf));
    q->st = (orc_resamp2 *)orc_calloc(ns ? ns : 1, sizeof(orc_resamp2));
    for (unsigned int i = 0; i < ns; i++) {     /* :137-150 */
        f0 = 0.5f * f0;
        fc = 0.5f * fc;
        const float ft = (0.5f - fc) / 2.0f;
        const unsigned int hl = orc_req_len(ft, As);
        unsigned int m = (unsigned int)ceilf((float)(hl - 1) / 4.0f);
        q->st[i] = orc_resamp2_create(ctaps, m < 3 ? 3 : m, f0, As);
    }
    return q;
}

void orc_msresamp2_destroy(orc_msresamp2 q)
{
    for (unsigned int i = 0; i < q->ns; i++) orc_resamp2_destroy(q->st[i]);
    free(q->st);
    free(q->b0);
    free(q->b1);
    free(q);
}

void orc_msresamp2_reset(orc_msresamp2 q)
{
    for (unsigned int i = 0; i < q->ns; i++) orc_resamp2_clear(q->st[i]);
}

void orc_msresamp2_execute(orc_msresamp2 q, const orc_cf *x, orc_cf *y)
{
    if (q->ns == 0) {
        y[0] = x[0];
        return;
    }
    if (q->type == 0) {                         /* :289-318: stages run in reverse order */
        orc_cf *in = q->b0, *out = q->b1;
        in[0] = x[0];
        for (unsigned int s = 0; s < q->ns; s++) {
            const unsigned int k = 1u << s;
            if (s == q->ns - 1) out = y;
            for (unsigned int i = 0; i < k; i++) orc_resamp2_interp_execute(q->st[q->ns - s - 1], in[i], &out[2 * i]);
            orc_cf *t = in;
            in = out;
            out = t;
        }
    } else {                                    /* :321-354 */
        const orc_cf *in = x;
        orc_cf *out = q->b1, *spare = q->b0;
        for (unsigned int s = 0; s < q->ns; s++) {
            const unsigned int k = 1u << (q->ns - s - 1);
            for (unsigned int i = 0; i < k; i++) orc_resamp2_decim_execute(q->st[s], &in[2 * i], &out[i]);
            in = out;
            orc_cf *t = out;
            out = spare;
            spare = t;
        }
        y[0] = CMPLXF(crealf(in[0]) * q->zeta, cimagf(in[0]) * q->zeta);
    }
}

/* ========================================================================= */
/* msresamp: src/filter/src/msresamp.c:68-349 -- halfband cascade + resamp  */
/* (m = 7, fc = 0.4, npfb = 64); interp: resamp first, decim: halfbands first */
/* ========================================================================= */
struct orc_msresamp_s {
    int type;                                   /* 0 interp (rate > 1), 1 decim */
    unsigned int ns, M, bi;
    orc_msresamp2 hb;
    orc_resamp rs;
    orc_cf *buf;
};

orc_msresamp orc_msresamp_create(float rate, float As)
{
    if (rate <= 0.0f) orc_fail("msresamp: rate must be > 0");
    orc_msresamp q = (orc_msresamp)orc_calloc(1, sizeof(*q));
    q->type = rate > 1.0f ? 0 : 1;
    float ra = rate;
    if (q->type == 0)
        while (ra > 2.0f) {
            q->ns++;
            ra *= 0.5f;
        }
    else
        while (ra < 0.5f) {
            q->ns++;
            ra *= 2.0f;
        }
    q->M = 1u << q->ns;
    q->buf = (orc_cf *)orc_calloc(4 + q->M, sizeof(orc_cf));
    q->hb = orc_msresamp2_create(0, q->type, q->ns, 0.4f, 0.0f, As);
    q->rs = orc_resamp_create(ra, 7, 0.4f, As, 64);
    return q;
}

void orc_msresamp_destroy(orc_msresamp q)
{
    orc_msresamp2_destroy(q->hb);
    orc_resamp_destroy(q->rs);
    free(q->buf);
    free(q);
}

void orc_msresamp_reset(orc_msresamp q)
{
    orc_msresamp2_reset(q->hb);
    orc_resamp_reset(q->rs);
    q->bi = 0;
}

void orc_msresamp_execute(orc_msresamp q, const orc_cf *x, unsigned int nx, orc_cf *y, unsigned int *ny)
{
    unsigned int n = 0, nw;
    for (unsigned int i = 0; i < nx; i++) {
        if (q->type == 0) {
            orc_resamp_execute_block(q->rs, &x[i], 1, q->buf, &nw);
            for (unsigned int k = 0; k < nw; k++) {
                orc_msresamp2_execute(q->hb, &q->buf[k], &y[n]);
                n += q->M;
            }
        } else {
            q->buf[q->bi++] = x[i];
            if (q->bi == q->M) {
                orc_cf h;
                orc_msresamp2_execute(q->hb, q->buf, &h);
                orc_resamp_execute_block(q->rs, &h, 1, &y[n], &nw);
                n += nw;
                q->bi = 0;
            }
        }
    }
    *ny = n;
}

/* n consecutive calls of one resamp2 mode on arrays (test convenience):
 * mode 0 filter (x[n] -> y0[n], y1[n]), 1 analyzer, 2 synthesizer (x[2n] ->
 * y0[2n]), 3 decim (x[2n] -> y0[n]), 4 interp (x[n] -> y0[2n]) */
void orc_resamp2_run(orc_resamp2 q, int mode, const orc_cf *x, unsigned int n, orc_cf *y0, orc_cf *y1)
{
    for (unsigned int i = 0; i < n; i++) {
        switch (mode) {
        case 0: orc_resamp2_filter_execute(q, x[i], &y0[i], &y1[i]); break;
        case 1: orc_resamp2_analyzer_execute(q, &x[2 * i], &y0[2 * i]); break;
        case 2: orc_resamp2_synthesizer_execute(q, &x[2 * i], &y0[2 * i]); break;
        case 3: orc_resamp2_decim_execute(q, &x[2 * i], &y0[i]); break;
        default: orc_resamp2_interp_execute(q, x[i], &y0[2 * i]); break;
        }
    }
}

/* ========================================================================= */
/* spgram: src/fft/src/spgram.c:41-286 (complex or real input)              */
/* ========================================================================= */
struct orc_spgram_s {
    int real_in;
    unsigned int nfft, W, sc, nt;
    float *w, *psd;
    orc_window buf;
    orc_cf *x, *X;
};

orc_spgram orc_spgram_create(int real_in, unsigned int nfft, const float *window, unsigned int W)
{
    if (nfft < 2 || W > nfft || W == 0) orc_fail("spgram: bad sizes");
    orc_spgram q = (orc_spgram)orc_calloc(1, sizeof(*q));
    q->real_in = real_in;
    q->nfft = nfft;
    q->W = W;
    q->w = (float *)orc_calloc(W, sizeof(float));
    q->psd = (float *)orc_calloc(nfft, sizeof(float));
    q->x = (orc_cf *)orc_calloc(nfft, sizeof(orc_cf));
    q->X = (orc_cf *)orc_calloc(nfft, sizeof(orc_cf));
    float g = 0.0f;
    for (unsigned int i = 0; i < W; i++) g += window[i] * window[i];
    g = (float)1.41421356237309504880 / (sqrtf(g / W) * sqrtf((float)nfft));   /* M_SQRT2 */
    for (unsigned int i = 0; i < W; i++) q->w[i] = g * window[i];
    orc_window_init(&q->buf, W);
    orc_spgram_reset(q);
    return q;
}

void orc_spgram_destroy(orc_spgram q)
{
    free(q->w);
    free(q->psd);
    free(q->x);
    free(q->X);
    free(q->buf.v);
    free(q);
}

void orc_spgram_reset(orc_spgram q)
{
    orc_window_clear(&q->buf);
    memset(q->x, 0, q->nfft * sizeof(orc_cf));
    q->nt = 0;
    q->sc = 0;
    for (unsigned int i = 0; i < q->nfft; i++) q->psd[i] = 1;
}

static orc_cf orc_spg_in(orc_spgram q, const void *x, unsigned int i)
{
    return q->real_in ? CMPLXF(((const float *)x)[i], 0.0f) : ((const orc_cf *)x)[i];
}

void orc_spgram_write(orc_spgram q, const void *x, unsigned int n)
{
    for (unsigned int i = 0; i < n; i++) orc_window_push(&q->buf, orc_spg_in(q, x, i));
}

void orc_spgram_execute(orc_spgram q, orc_cf *X)
{
    const orc_cf *r = orc_window_read(&q->buf);
    for (unsigned int i = 0; i < q->W; i++) q->x[i] = CMPLXF(crealf(r[i]) * q->w[i], cimagf(r[i]) * q->w[i]);
    orc_fft(q->nfft, q->x, q->X, +1);
    if (X) memcpy(X, q->X, q->nfft * sizeof(orc_cf));
}

static float orc_pwr(orc_cf v) { return crealf(v) * crealf(v) + cimagf(v) * cimagf(v); }

void orc_spgram_execute_psd(orc_spgram q, float *X)
{
    orc_spgram_execute(q, NULL);
    for (unsigned int i = 0; i < q->nfft; i++) X[(i + q->nfft / 2) % q->nfft] = 10 * log10f(orc_pwr(q->X[i]) + 1e-16f);
}

void orc_spgram_accumulate_psd(orc_spgram q, const void *x, float alpha, unsigned int n)
{
    for (unsigned int i = 0; i < n; i++) {
        orc_window_push(&q->buf, orc_spg_in(q, x, i));
        q->sc++;
        if (q->sc == q->W / 2) {
            if (q->nt == 0) alpha = 1.0f;   /* stays 1 for the rest of this call, as spgram.c:214-216 */
            orc_spgram_execute(q, NULL);
            for (unsigned int k = 0; k < q->nfft; k++) q->psd[k] = (1.0f - alpha) * q->psd[k] + alpha * orc_pwr(q->X[k]);
            q->sc = 0;
            q->nt++;
        }
    }
}

void orc_spgram_write_accumulation(orc_spgram q, float *x)
{
    for (unsigned int i = 0; i < q->nfft; i++) x[(i + q->nfft / 2) % q->nfft] = 10 * log10f(q->psd[i]);
}

void orc_spgram_estimate_psd(orc_spgram q, const void *x, unsigned int n, float *psd)
{
    if (n == 0) return;
    orc_spgram_reset(q);
    unsigned int delay = q->nfft / 4;
    if (delay == 0) delay = 1;
    for (unsigned int i = 0; i < q->nfft; i++) psd[i] = 0.0f;
    unsigned int nt = 0;
    for (unsigned int i = 0; i < n; i++) {
        orc_window_push(&q->buf, orc_spg_in(q, x, i));
        if (((i + 1) % delay) == 0 || i == n - 1) {
            orc_spgram_execute(q, NULL);
            for (unsigned int k = 0; k < q->nfft; k++) psd[(k + q->nfft / 2) % q->nfft] += orc_pwr(q->X[k]);
            nt++;
        }
    }
    for (unsigned int i = 0; i < q->nfft; i++) psd[i] = 10 * log10f(psd[i] / (float)nt);
}
