/*
 * lq_small.c -- the host path for single-sample / single-vector calls.
 *
 * The per-call API (one sample, one dot product, one decimated output per
 * call: firfilt_*_push + _execute, dotprod_*_execute / _run / _run4,
 * firdecim_*_execute, firinterp_*_execute, resamp_*_execute, and
 * fftfilt_*_execute on its short n-sample block, n h_len <= 65536) is what
 * unchanged liquid-dsp programs call in their inner loops.  On the GPU each
 * such call is a launch plus two PCIe crossings (~10 us); the
 * reference does it in 20-60 ns.  So by default these entry points compute
 * their few outputs on the host with the routines below, while every block
 * call (*_execute_block[_dev], the channelizers, fftfilt_*_execute on longer
 * blocks, FFT plans, spgram) runs on the GPU.  Environment LQ_SMALL_CALLS=gpu
 * (or liquid_mi355x_set_small_calls(0)) sends every call to the GPU instead.
 * The host routines are this library's own (not the test oracle), follow the
 * reference's definitions (cited per routine) and keep the objects' state
 * coherent with the GPU path through host mirrors of the device histories
 * (lq_mirror below), so a program may mix per-sample and block calls on one
 * object.  A GPU is still required: objects cannot be created without one.
 */
#include <complex.h>

#include "lq_host.h"

static int g_small = -1;   /* -1: not yet read from the environment */

int lq_small_host(void)
{
    if (g_small < 0) {
        const char *e = getenv("LQ_SMALL_CALLS");
        g_small = (e && (strcmp(e, "gpu") == 0 || strcmp(e, "0") == 0)) ? 0 : 1;
    }
    return g_small;
}

void liquid_mi355x_set_small_calls(int host) { g_small = host ? 1 : 0; }

int liquid_mi355x_get_small_calls(void) { return lq_small_host(); }

/* y = sum_{i<n} h[i] x[i] (no conjugation; src/dotprod/src/dotprod.c:42-167
 * and the type-specific dotprod_crcf.c / dotprod_cccf.c).  Four-float vectors
 * (GCC vector extensions: SSE on x86-64 without intrinsics, the reference's
 * dotprod_*.mmx.c do the same with SSE intrinsics) with two accumulators, so
 * several multiply-adds are in flight: complex samples two per vector. */
typedef float lq_v4 __attribute__((vector_size(16)));
typedef int lq_v4i __attribute__((vector_size(16)));
static inline lq_v4 lq_ld4(const float *p)
{
    lq_v4 v;
    memcpy(&v, p, sizeof(v));
    return v;
}
void lq_host_dot(int kind, const float *h, const void *xv, unsigned int n, void *y)
{
    const float *x = (const float *)xv;
    lq_v4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0};
    unsigned int i = 0;
    if (kind == LQ_RRRF) {
        for (; i + 8 <= n; i += 8) {
            a0 += lq_ld4(h + i) * lq_ld4(x + i);
            a1 += lq_ld4(h + i + 4) * lq_ld4(x + i + 4);
        }
        a0 += a1;
        float r = (a0[0] + a0[1]) + (a0[2] + a0[3]);
        for (; i < n; i++) r += h[i] * x[i];
        *(float *)y = r;
    } else if (kind == LQ_CRCF) {   /* x: (re, im) pairs, real taps */
        const lq_v4i dup01 = {0, 0, 1, 1}, dup23 = {2, 2, 3, 3};
        for (; i + 4 <= n; i += 4) {
            const lq_v4 hv = lq_ld4(h + i);
            a0 += __builtin_shuffle(hv, dup01) * lq_ld4(x + 2 * i);
            a1 += __builtin_shuffle(hv, dup23) * lq_ld4(x + 2 * i + 4);
        }
        a0 += a1;
        float re = a0[0] + a0[2], im = a0[1] + a0[3];
        for (; i < n; i++) {
            re += h[i] * x[2 * i];
            im += h[i] * x[2 * i + 1];
        }
        ((float *)y)[0] = re;
        ((float *)y)[1] = im;
    } else {   /* complex taps: a0 += hr x, a1 += hi swap(x) */
        const lq_v4i re2 = {0, 0, 2, 2}, im2 = {1, 1, 3, 3}, sw = {1, 0, 3, 2};
        for (; i + 2 <= n; i += 2) {
            const lq_v4 hv = lq_ld4(h + 2 * i), xv4 = lq_ld4(x + 2 * i);
            a0 += __builtin_shuffle(hv, re2) * xv4;
            a1 += __builtin_shuffle(hv, im2) * __builtin_shuffle(xv4, sw);
        }
        /* a0 = (hr xr, hr xi, ..), a1 = (hi xi, hi xr, ..) */
        float re = (a0[0] + a0[2]) - (a1[0] + a1[2]), im = (a0[1] + a0[3]) + (a1[1] + a1[3]);
        for (; i < n; i++) {
            const float hr = h[2 * i], hi = h[2 * i + 1], xr = x[2 * i], xi = x[2 * i + 1];
            re += hr * xr - hi * xi;
            im += hr * xi + hi * xr;
        }
        ((float *)y)[0] = re;
        ((float *)y)[1] = im;
    }
}

/* Objects that keep their taps (firfilt, dotprod) run the per-call dot
 * product over an expanded copy made at create time, so the inner loop is a
 * plain multiply-add of two contiguous float arrays with no shuffles (the
 * reference's dotprod_*.mmx.c likewise keep a rearranged copy of the taps):
 *   rrrf  g[i]                                   n floats
 *   crcf  (g[i], g[i]) pairs                     2n floats
 *   cccf  (gr[i], gr[i]) pairs, (-gi[i], gi[i])  4n floats
 * with g[i] = h[n-1-i] when rev (the filter convolution over the window's
 * oldest-first samples, firfilt.c:322-338) else h[i] (dotprod.c:42-167). */
float *lq_host_taps(int kind, const float *h, unsigned int n, int rev)
{
    const unsigned int nf = kind == LQ_RRRF ? n : (kind == LQ_CRCF ? 2 * n : 4 * n);
    float *g = (float *)lq_xmalloc((size_t)(nf ? nf : 1) * sizeof(float));
    for (unsigned int i = 0; i < n; i++) {
        const unsigned int k = rev ? n - 1 - i : i;
        if (kind == LQ_RRRF) {
            g[i] = h[k];
        } else if (kind == LQ_CRCF) {
            g[2 * i] = g[2 * i + 1] = h[k];
        } else {
            g[2 * i] = g[2 * i + 1] = h[2 * k];
            g[2 * n + 2 * i] = -h[2 * k + 1];
            g[2 * n + 2 * i + 1] = h[2 * k + 1];
        }
    }
    return g;
}

/* the expanded-tap dot product, for a vector type V of W floats: four
 * accumulators keep four multiply-add chains in flight over the long part,
 * single vectors take the rest down to W floats, then scalars */
#define LQ_TDOT_STEP(A, OFF, V, W, SWAPMASK)                                                       \
    do {                                                                                            \
        V t_, u_;                                                                                   \
        __builtin_memcpy(&t_, g + (OFF), sizeof(V));                                                \
        __builtin_memcpy(&u_, x + (OFF), sizeof(V));                                                \
        A += t_ * u_;                                                                               \
        if (kind == LQ_CCCF) { /* + (-gi, gi) * (xi, xr) */                                         \
            __builtin_memcpy(&t_, g + 2 * n + (OFF), sizeof(V));                                    \
            A += t_ * __builtin_shuffle(u_, SWAPMASK);                                              \
        }                                                                                           \
    } while (0)
#define LQ_TDOT_BODY(V, W, SWAPMASK, FOLD)                                                          \
    const float *x = (const float *)xv;                                                             \
    V a0 = {0}, a1 = {0}, a2 = {0}, a3 = {0};                                                       \
    const unsigned int nf = kind == LQ_RRRF ? n : 2 * n;                                            \
    unsigned int i = 0;                                                                             \
    for (; i + 4 * (W) <= nf; i += 4 * (W)) {                                                      \
        LQ_TDOT_STEP(a0, i, V, W, SWAPMASK);                                                        \
        LQ_TDOT_STEP(a1, i + (W), V, W, SWAPMASK);                                                  \
        LQ_TDOT_STEP(a2, i + 2 * (W), V, W, SWAPMASK);                                              \
        LQ_TDOT_STEP(a3, i + 3 * (W), V, W, SWAPMASK);                                              \
    }                                                                                               \
    for (; i + 2 * (W) <= nf; i += 2 * (W)) {                                                      \
        LQ_TDOT_STEP(a0, i, V, W, SWAPMASK);                                                        \
        LQ_TDOT_STEP(a1, i + (W), V, W, SWAPMASK);                                                  \
    }                                                                                               \
    if (i + (W) <= nf) {                                                                            \
        LQ_TDOT_STEP(a2, i, V, W, SWAPMASK);                                                        \
        i += (W);                                                                                   \
    }                                                                                               \
    a0 += a1;                                                                                       \
    a2 += a3;                                                                                       \
    a0 += a2;                                                                                       \
    FOLD; /* lanes 0, 1: the even / odd partial sums */                                             \
    float r0 = a0[0], r1 = a0[1];                                                                   \
    if (kind == LQ_RRRF) {                                                                          \
        r0 += r1;                                                                                   \
        for (; i < nf; i++) r0 += g[i] * x[i];                                                      \
        *(float *)y = r0;                                                                           \
        return;                                                                                     \
    }                                                                                               \
    for (; i < nf; i += 2) {                                                                        \
        r0 += g[i] * x[i];                                                                          \
        r1 += g[i + 1] * x[i + 1];                                                                  \
        if (kind == LQ_CCCF) {                                                                      \
            r0 += g[2 * n + i] * x[i + 1];                                                          \
            r1 += g[2 * n + i + 1] * x[i];                                                          \
        }                                                                                           \
    }                                                                                               \
    ((float *)y)[0] = r0;                                                                           \
    ((float *)y)[1] = r1;

static void lq_tdot_sse(int kind, const float *g, const void *xv, unsigned int n, void *y)
{
    LQ_TDOT_BODY(lq_v4, 4, ((lq_v4i){1, 0, 3, 2}), a0 += __builtin_shuffle(a0, ((lq_v4i){2, 3, 0, 1})))
}

typedef float lq_v8 __attribute__((vector_size(32)));
typedef int lq_v8i __attribute__((vector_size(32)));
__attribute__((target("avx2"))) static void lq_tdot_avx2(int kind, const float *g, const void *xv, unsigned int n,
                                                         void *y)
{
    LQ_TDOT_BODY(lq_v8, 8, ((lq_v8i){1, 0, 3, 2, 5, 4, 7, 6}),
                 a0 += __builtin_shuffle(a0, ((lq_v8i){4, 5, 6, 7, 0, 1, 2, 3}));
                 a0 += __builtin_shuffle(a0, ((lq_v8i){2, 3, 0, 1, 6, 7, 4, 5})))
}

static int g_avx2 = -1;

/* y = sum_i g[i] x[i] over the expanded taps of lq_host_taps (n samples) */
void lq_host_tdot(int kind, const float *g, const void *x, unsigned int n, void *y)
{
    if (g_avx2 < 0) g_avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
    /* 32-byte vectors from 16 floats up (per-call rates on the box's EPYC
     * host against the 16-byte form: dotprod crcf / cccf 1.45x / 1.9x,
     * fftfilt 1.6x, firfilt 0.95x; profiles/r06_ab_experiments.txt, r06host) */
    if (g_avx2 && (kind == LQ_RRRF ? n : 2 * n) >= 16)
        lq_tdot_avx2(kind, g, x, n, y);
    else
        lq_tdot_sse(kind, g, x, n, y);
}

/* ------------------------------------------------------------------ mirrors
 * A host copy of a device-resident history of n samples (double-buffered on
 * the device: the current buffer is passed in).  Whichever side ran last is
 * authoritative; the other is refreshed on demand. */
void lq_mirror_init(lq_mirror *m, size_t n, size_t esz)
{
    m->n = n;
    m->esz = esz;
    m->cap = 2 * n + 64;   /* room to append before compacting */
    m->buf = (unsigned char *)lq_xmalloc((m->cap ? m->cap : 1) * esz);
    memset(m->buf, 0, (m->cap ? m->cap : 1) * esz);
    m->off = 0;
    m->host_valid = m->dev_valid = 1;
}

void lq_mirror_free(lq_mirror *m)
{
    free(m->buf);
    m->buf = NULL;
}

void lq_mirror_zero(lq_mirror *m)
{
    memset(m->buf, 0, (m->cap ? m->cap : 1) * m->esz);
    m->off = 0;
    m->host_valid = m->dev_valid = 1;
}

void lq_mirror_need_host(lq_mirror *m, const void *dev_hist, void *stream)
{
    if (m->host_valid) return;
    m->off = 0;
    if (m->n) {
        lqrt_d2h(m->buf, dev_hist, m->n * m->esz, stream);
        lqrt_sync(stream);
    }
    m->host_valid = 1;
}

void lq_mirror_need_dev(lq_mirror *m, void *dev_hist, void *stream)
{
    if (m->dev_valid) return;
    if (m->n) lqrt_h2d(dev_hist, m->buf + m->off * m->esz, m->n * m->esz, stream);
    m->dev_valid = 1;
}

/* append k samples; the window (the last n samples plus the k new ones) is
 * contiguous at lq_mirror_ptr(m) afterwards, newest last */
void lq_mirror_append(lq_mirror *m, const void *x, size_t k)
{
    if (m->off + m->n + k > m->cap) {
        if (m->n + k > m->cap) {
            const size_t cap = 2 * (m->n + k) + 64;
            unsigned char *b = (unsigned char *)lq_xmalloc(cap * m->esz);
            memcpy(b, m->buf + m->off * m->esz, m->n * m->esz);
            free(m->buf);
            m->buf = b;
            m->cap = cap;
        } else {
            memmove(m->buf, m->buf + m->off * m->esz, m->n * m->esz);
        }
        m->off = 0;
    }
    memcpy(m->buf + (m->off + m->n) * m->esz, x, k * m->esz);
    m->dev_valid = 0;
}

/* after an append of k samples: keep the last n */
void lq_mirror_commit(lq_mirror *m, size_t k) { m->off += k; }

unsigned char *lq_mirror_ptr(lq_mirror *m) { return m->buf + m->off * m->esz; }
