/*
 * lq_common.c -- shared host helpers: buffers, streams, version symbols and
 * the Kaiser window design used at object creation.
 *
 * Design math restates src/filter/src/firdes.c:224-281 and
 * src/math/src/{math.c:128-139, math.c:289-312, math.bessel.c:86-104,
 * math.gamma.c:43-72} in float, the same operation order, so the taps match
 * the reference's to rounding.
 */
#include <math.h>

#include "lq_host.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

const char liquid_version[] = LIQUID_VERSION;
const char *liquid_libversion(void) { return LIQUID_VERSION; }
int liquid_libversion_number(void) { return LIQUID_VERSION_NUMBER; }
const char *liquid_mi355x_build_target(void) { return "gfx950"; }

void *lq_xmalloc(size_t bytes)
{
    void *p = calloc(1, bytes ? bytes : 1);
    if (!p) LQ_FAIL("error: liquid-mi355x: out of host memory\n");
    return p;
}

void *lq_devbuf_get(lq_devbuf *b, size_t bytes)
{
    if (bytes > b->cap) {
        if (b->p) lqrt_free(b->p);
        size_t cap = b->cap ? b->cap : 4096;
        while (cap < bytes) cap *= 2;
        b->p = lqrt_malloc(cap);
        b->cap = cap;
    }
    return b->p;
}

void lq_devbuf_free(lq_devbuf *b)
{
    if (b->p) lqrt_free(b->p);
    b->p = NULL;
    b->cap = 0;
}

void lq_ctx_init(lq_ctx *c)
{
    c->stream = lqrt_stream_create();
    c->own = 1;
}

void lq_ctx_free(lq_ctx *c)
{
    if (c->stream) lqrt_sync(c->stream);
    if (c->own && c->stream) lqrt_stream_destroy(c->stream);
    c->stream = NULL;
    lqrt_host_free(c->pin_in);
    lqrt_host_free(c->pin_out);
    lqrt_host_free(c->flag);
    c->pin_in = c->pin_out = NULL;
    c->flag = NULL;
    c->in_cap = c->out_cap = 0;
}

static void *lq_pin_grow(void *p, size_t *cap, size_t bytes)
{
    if (bytes <= *cap) return p;
    lqrt_host_free(p);
    size_t n = 4096;
    while (n < bytes) n *= 2;
    *cap = n;
    return lqrt_host_alloc(n);
}

const void *lq_call_in(lq_ctx *c, lq_devbuf *b, const void *x, size_t bytes)
{
    if (c->in_busy) {   /* a previous call without a result may still read pin_in */
        lqrt_sync(c->stream);
        c->in_busy = 0;
    }
    if (bytes == 0) return lq_devbuf_get(b, 16);
    if (bytes > LQ_PIN_IN) {
        void *d = lq_devbuf_get(b, bytes);
        lqrt_h2d(d, x, bytes, c->stream);
        return d;
    }
    c->pin_in = lq_pin_grow(c->pin_in, &c->in_cap, bytes);
    memcpy(c->pin_in, x, bytes);
    c->in_busy = 1;
    return c->pin_in;
}

void lq_call_out(lq_ctx *c, void *y, const void *dy, size_t bytes)
{
    if (bytes == 0 || bytes > LQRT_COPYOUT_MAX || (bytes & 3)) {
        if (bytes) lqrt_d2h(y, dy, bytes, c->stream);
        lqrt_sync(c->stream);
        c->in_busy = 0;
        return;
    }
    c->pin_out = lq_pin_grow(c->pin_out, &c->out_cap, bytes);
    if (!c->flag) {
        c->flag = (unsigned *)lqrt_host_alloc(64);
        *c->flag = c->seq = 0;
    }
    const unsigned seq = ++c->seq;
    lqrt_copyout_signal(dy, c->pin_out, bytes, c->flag, seq, c->stream);
    lqrt_wait_flag(c->flag, seq, c->stream);
    memcpy(y, c->pin_out, bytes);
    c->in_busy = 0;
}

void *lq_sig_out(lq_ctx *c, size_t bytes, unsigned **flag, unsigned *seq)
{
    c->pin_out = lq_pin_grow(c->pin_out, &c->out_cap, bytes);
    if (!c->flag) {
        c->flag = (unsigned *)lqrt_host_alloc(64);
        *c->flag = c->seq = 0;
    }
    *flag = c->flag;
    *seq = ++c->seq;
    return c->pin_out;
}

void lq_sig_wait(lq_ctx *c, void *y, size_t bytes, unsigned seq)
{
    lqrt_wait_flag(c->flag, seq, c->stream);
    memcpy(y, c->pin_out, bytes);
    c->in_busy = 0;
}

void lq_call_done(lq_ctx *c)
{
    lqrt_sync(c->stream);
    c->in_busy = 0;
}

void lq_ctx_set_stream(lq_ctx *c, void *stream)
{
    if (c->stream) lqrt_sync(c->stream);
    if (c->own && c->stream) lqrt_stream_destroy(c->stream);
    c->in_busy = 0;
    if (stream) {
        c->stream = stream;
        c->own = 0;
    } else {
        lq_ctx_init(c);
    }
}

unsigned int lq_msb_index(unsigned int x)
{
    unsigned int b = 0;
    for (; x; x >>= 1) b++;
    return b;
}

/* liquid.h:6662, msb_index.c:110-135 (the x86 build's bsr: 0 for x = 0) */
unsigned int liquid_msb_index(unsigned int _x) { return _x ? 32u - (unsigned int)__builtin_clz(_x) : 0u; }

int lq_is_pow2(unsigned int x) { return x && !(x & (x - 1)); }

/* ----------------------------------------------------------------- design */

float lq_kaiser_beta_As(float As)
{
    float a = fabsf(As);
    if (a > 50.0f) return 0.1102f * (a - 8.7f);
    if (a > 21.0f) return (float)(0.5842 * powf(a - 21, 0.4f) + 0.07886f * (a - 21));
    return 0.0f;
}

float kaiser_beta_As(float _As) { return lq_kaiser_beta_As(_As); }

float lq_sincf(float x)
{
    if (fabsf(x) < 0.01f) return cosf(M_PI * x / 2.0f) * cosf(M_PI * x / 4.0f) * cosf(M_PI * x / 8.0f);
    return sinf(M_PI * x) / (M_PI * x);
}

static float lq_lngammaf(float z)
{
    if (z < 0) LQ_FAIL("error: liquid_lngammaf(), undefined for z <= 0\n");
    /* below 10 the reference recurses lnG(z) = lnG(z+1) - ln z */
    float acc = 0.0f;
    float zz = z;
    int depth = 0;
    float logs[16];
    while (zz < 10.0f) {
        logs[depth++] = logf(zz);
        zz += 1.0f;
    }
    float g = 0.5 * (logf(2 * M_PI) - log(zz));
    g += zz * (logf(zz + (1 / (12.0f * zz - 0.1f / zz))) - 1);
    /* unwind in the same order the recursion returns: innermost first */
    acc = g;
    while (depth > 0) acc = acc - logs[--depth];
    return acc;
}

static float lq_besseli0f(float z)
{
    if (z == 0.0f) return 1.0f;
    float y = 0.0f;
    for (unsigned int k = 0; k < 32; k++) {
        float t = k * logf(0.5f * z) - lq_lngammaf((float)k + 1.0f);
        y += expf(2 * t);
    }
    return y;
}

float lq_kaiser_window(unsigned int n, unsigned int N, float beta, float mu)
{
    float t = (float)n - (float)(N - 1) / 2 + mu;
    float r = 2.0f * t / (float)N;
    return lq_besseli0f(beta * sqrtf(1 - r * r)) / lq_besseli0f(beta);
}

void lq_firdes_kaiser(unsigned int n, float fc, float As, float mu, float *h)
{
    if (mu < -0.5f || mu > 0.5f)
        LQ_FAIL("error: liquid_firdes_kaiser(), _mu (%12.4e) out of range [-0.5,0.5]\n", mu);
    if (fc < 0.0f || fc > 0.5f)
        LQ_FAIL("error: liquid_firdes_kaiser(), cutoff frequency (%12.4e) out of range (0, 0.5)\n", fc);
    if (n == 0) LQ_FAIL("error: liquid_firdes_kaiser(), filter length must be greater than zero\n");
    float beta = lq_kaiser_beta_As(As);
    for (unsigned int i = 0; i < n; i++) {
        float t = (float)i - (float)(n - 1) / 2 + mu;
        h[i] = lq_sincf(2.0f * fc * t) * lq_kaiser_window(i, n, beta, mu);
    }
}

void liquid_firdes_kaiser(unsigned int _n, float _fc, float _As, float _mu, float *_h)
{
    lq_firdes_kaiser(_n, _fc, _As, _mu, _h);
}

/* ----------------------------------------------------------------- memory helpers (extension) */

static void *g_default_stream = NULL;

static void *lq_default_stream(void)
{
    if (!g_default_stream) g_default_stream = lqrt_stream_create();
    return g_default_stream;
}

void *liquid_mi355x_malloc(unsigned long long _bytes) { return lqrt_malloc((size_t)_bytes); }
void liquid_mi355x_free(void *_p) { lqrt_free(_p); }

void liquid_mi355x_memcpy_h2d(void *_dst, const void *_src, unsigned long long _bytes)
{
    void *s = lq_default_stream();
    lqrt_h2d(_dst, _src, (size_t)_bytes, s);
    lqrt_sync(s);
}

void liquid_mi355x_memcpy_d2h(void *_dst, const void *_src, unsigned long long _bytes)
{
    void *s = lq_default_stream();
    lqrt_d2h(_dst, _src, (size_t)_bytes, s);
    lqrt_sync(s);
}

void liquid_mi355x_device_synchronize(void) { lqrt_device_sync(); }
