/*
 * lq_small.c -- the opt-in host path for single-sample / single-vector calls.
 *
 * The per-call API (one sample, one dot product, one decimated output per
 * call: firfilt_*_push + _execute, dotprod_*_execute / _run, firdecim_*_execute,
 * firinterp_*_execute, resamp_*_execute, and fftfilt_*_execute on its short
 * n-sample block, n h_len <= 65536) is what unchanged liquid-dsp programs
 * call in their inner loops.  On the GPU each such call is a launch plus two
 * PCIe crossings (~10 us); the reference does it in 20-60 ns.
 * With the small-call mode set to host -- environment LQ_SMALL_CALLS=host, or
 * liquid_mi355x_set_small_calls(1) -- these calls compute their few outputs on
 * the host with the routines below, while every block call
 * (*_execute_block[_dev], the channelizers, fftfilt, ...) stays on the GPU.
 * The default is the GPU for every call.  The host routines are this
 * library's own (not the test oracle), follow the reference's definitions
 * (cited per routine) and keep the objects' state coherent with the GPU path
 * through host mirrors of the device histories (lq_mirror below), so a program
 * may mix per-sample and block calls on one object.  A GPU is still required:
 * objects cannot be created without one.
 */
#include <complex.h>

#include "lq_host.h"

static int g_small = -1;   /* -1: not yet read from the environment */

int lq_small_host(void)
{
    if (g_small < 0) {
        const char *e = getenv("LQ_SMALL_CALLS");
        g_small = (e && (strcmp(e, "host") == 0 || strcmp(e, "1") == 0)) ? 1 : 0;
    }
    return g_small;
}

void liquid_mi355x_set_small_calls(int host) { g_small = host ? 1 : 0; }

int liquid_mi355x_get_small_calls(void) { return lq_small_host(); }

/* y = sum_{i<n} h[i] x[i] (no conjugation; src/dotprod/src/dotprod.c:42-167
 * and the type-specific dotprod_crcf.c / dotprod_cccf.c); four partial sums
 * so the compiler can keep several multiply-adds in flight */
void lq_host_dot(int kind, const float *h, const void *xv, unsigned int n, void *y)
{
    if (kind == LQ_RRRF) {
        const float *x = (const float *)xv;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        unsigned int i = 0;
        for (; i + 4 <= n; i += 4) {
            a0 += h[i] * x[i];
            a1 += h[i + 1] * x[i + 1];
            a2 += h[i + 2] * x[i + 2];
            a3 += h[i + 3] * x[i + 3];
        }
        for (; i < n; i++) a0 += h[i] * x[i];
        *(float *)y = (a0 + a1) + (a2 + a3);
    } else if (kind == LQ_CRCF) {
        const float *x = (const float *)xv;   /* (re, im) pairs */
        float r0 = 0.f, i0 = 0.f, r1 = 0.f, i1 = 0.f;
        unsigned int i = 0;
        for (; i + 2 <= n; i += 2) {
            r0 += h[i] * x[2 * i];
            i0 += h[i] * x[2 * i + 1];
            r1 += h[i + 1] * x[2 * i + 2];
            i1 += h[i + 1] * x[2 * i + 3];
        }
        for (; i < n; i++) {
            r0 += h[i] * x[2 * i];
            i0 += h[i] * x[2 * i + 1];
        }
        ((float *)y)[0] = r0 + r1;
        ((float *)y)[1] = i0 + i1;
    } else {
        const float *x = (const float *)xv;
        float r0 = 0.f, i0 = 0.f, r1 = 0.f, i1 = 0.f;
        unsigned int i = 0;
        for (; i + 2 <= n; i += 2) {
            const float hr = h[2 * i], hi = h[2 * i + 1], xr = x[2 * i], xi = x[2 * i + 1];
            const float gr = h[2 * i + 2], gi = h[2 * i + 3], zr = x[2 * i + 2], zi = x[2 * i + 3];
            r0 += hr * xr - hi * xi;
            i0 += hr * xi + hi * xr;
            r1 += gr * zr - gi * zi;
            i1 += gr * zi + gi * zr;
        }
        for (; i < n; i++) {
            const float hr = h[2 * i], hi = h[2 * i + 1], xr = x[2 * i], xi = x[2 * i + 1];
            r0 += hr * xr - hi * xi;
            i0 += hr * xi + hi * xr;
        }
        ((float *)y)[0] = r0 + r1;
        ((float *)y)[1] = i0 + i1;
    }
}

/* y = sum_{k<n} h[k] w[last - k] over a window w whose newest sample is at
 * index `last` (the filter convolution, src/filter/src/firfilt.c:322-338:
 * the reference runs its dot product over the reversed taps and the window's
 * oldest-first samples, the same terms) */
void lq_host_conv(int kind, const float *h, const void *wv, unsigned int last, unsigned int n, void *y)
{
    if (kind == LQ_RRRF) {
        const float *w = (const float *)wv + last;
        float a0 = 0.f, a1 = 0.f;
        unsigned int k = 0;
        for (; k + 2 <= n; k += 2) {
            a0 += h[k] * w[-(long)k];
            a1 += h[k + 1] * w[-(long)k - 1];
        }
        for (; k < n; k++) a0 += h[k] * w[-(long)k];
        *(float *)y = a0 + a1;
    } else if (kind == LQ_CRCF) {
        const float *w = (const float *)wv + 2 * (size_t)last;
        float r0 = 0.f, i0 = 0.f, r1 = 0.f, i1 = 0.f;
        unsigned int k = 0;
        for (; k + 2 <= n; k += 2) {
            r0 += h[k] * w[-2 * (long)k];
            i0 += h[k] * w[-2 * (long)k + 1];
            r1 += h[k + 1] * w[-2 * (long)k - 2];
            i1 += h[k + 1] * w[-2 * (long)k - 1];
        }
        for (; k < n; k++) {
            r0 += h[k] * w[-2 * (long)k];
            i0 += h[k] * w[-2 * (long)k + 1];
        }
        ((float *)y)[0] = r0 + r1;
        ((float *)y)[1] = i0 + i1;
    } else {
        const float *w = (const float *)wv + 2 * (size_t)last;
        float r0 = 0.f, i0 = 0.f;
        for (unsigned int k = 0; k < n; k++) {
            const float hr = h[2 * k], hi = h[2 * k + 1], xr = w[-2 * (long)k], xi = w[-2 * (long)k + 1];
            r0 += hr * xr - hi * xi;
            i0 += hr * xi + hi * xr;
        }
        ((float *)y)[0] = r0;
        ((float *)y)[1] = i0;
    }
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
