/*
 * fft.c -- the public FFT plan API (include/liquid.h:1122-1216) on the GPU.
 *
 * Reference: src/fft/src/fft_common.c (create/destroy/print/execute/run/
 * shift), fft_r2r_1d.c (DCT/DST I-IV), src/math/src/math.c:143-157
 * (liquid_nextpow2).  A plan binds host arrays x, y and a direction at
 * creation, exactly as the reference; fft_execute() stages x through the
 * device, runs csrc/k_fft.hip and writes y.  Transforms are un-normalised
 * (backward(forward(x)) = n x), forward = exp(-j 2 pi k n / N).
 * Extensions: fft_execute_batch[_dev] run many transforms of the plan's size
 * and direction in one launch sequence; fft_set_stream.
 */
#include <complex.h>

#include "lq_host.h"

struct fftplan_s {
    int r2r;                /* 0: complex (dir +-1), 1: real-to-real (type) */
    int dir, type, flags;
    unsigned int n;
    void *x, *y;            /* host arrays bound at creation */
    lq_ctx ctx;
    lq_devbuf dx, work;
};

static int lq_fft_is_r2r_type(int t) { return (t >= 10 && t <= 13) || (t >= 20 && t <= 23); }

fftplan fft_create_plan(unsigned int _n, liquid_float_complex *_x, liquid_float_complex *_y, int _dir, int _flags)
{
    if (_n == 0) LQ_FAIL("error: fft_create_plan(), fft size must be greater than zero\n");
    lqrt_require_device("fft_create_plan");
    fftplan p = (fftplan)lq_xmalloc(sizeof(*p));
    memset(p, 0, sizeof(*p));
    p->n = _n;
    p->dir = _dir == LIQUID_FFT_FORWARD ? LIQUID_FFT_FORWARD : LIQUID_FFT_BACKWARD;
    p->type = p->dir;
    p->flags = _flags;
    p->x = _x;
    p->y = _y;
    lq_ctx_init(&p->ctx);
    return p;
}

fftplan fft_create_plan_r2r_1d(unsigned int _n, float *_x, float *_y, int _type, int _flags)
{
    if (!lq_fft_is_r2r_type(_type)) LQ_FAIL("error: fft_create_plan_r2r_1d(), invalid type, %d\n", _type);
    if (_n == 0) LQ_FAIL("error: fft_create_plan_r2r_1d(), fft size must be greater than zero\n");
    lqrt_require_device("fft_create_plan_r2r_1d");
    fftplan p = (fftplan)lq_xmalloc(sizeof(*p));
    memset(p, 0, sizeof(*p));
    p->r2r = 1;
    p->n = _n;
    p->type = _type;
    p->flags = _flags;
    p->x = _x;
    p->y = _y;
    lq_ctx_init(&p->ctx);
    return p;
}

void fft_destroy_plan(fftplan _p)
{
    lqrt_sync(_p->ctx.stream);
    lq_devbuf_free(&_p->dx);
    lq_devbuf_free(&_p->work);
    lq_ctx_free(&_p->ctx);
    free(_p);
}

void fft_print_plan(fftplan _p)
{
    if (_p->r2r) {
        printf("real-to-real transform...\n");
        return;
    }
    const unsigned int n = _p->n;
    const char *how = (n & (n - 1)) == 0 ? (n <= 4096 ? "Stockham radix-4/2 (LDS)" : "four-step")
                                         : (n <= 16 ? "DFT" : "Bluestein chirp-z");
    printf("fft plan [%s], n=%u, %s (MI355X)\n", _p->dir == LIQUID_FFT_FORWARD ? "forward" : "reverse", n, how);
}

void fft_execute_batch_dev(fftplan _p, const void *_dx, void *_dy, unsigned long long _batch)
{
    if (_batch == 0) return;
    if (_p->r2r) {   /* every output reads the whole input: stage in-place calls */
        if (_dx == _dy) {
            const size_t bytes = (size_t)_p->n * _batch * sizeof(float);
            void *c = lq_devbuf_get(&_p->work, bytes);
            lqrt_d2d(c, _dx, bytes, _p->ctx.stream);
            _dx = c;
        }
        lqk_fft_r2r(_p->type, _p->n, _dx, _dy, _batch, _p->ctx.stream);
        return;
    }
    const size_t wb = lqk_fft_work_bytes(_p->n, _batch);
    void *w = wb ? lq_devbuf_get(&_p->work, wb) : NULL;
    lqk_fft_any(_p->n, _p->dir, _dx, _dy, _batch, w, _p->ctx.stream);
}

void fft_execute_batch(fftplan _p, const void *_x, void *_y, unsigned long long _batch)
{
    if (_batch == 0) return;
    const size_t bytes = (size_t)_p->n * _batch * (_p->r2r ? 4 : 8);
    const void *dx = lq_call_in(&_p->ctx, &_p->dx, _x, bytes);
    void *d = lq_devbuf_get(&_p->dx, bytes);
    fft_execute_batch_dev(_p, dx, d, _batch);
    lq_call_out(&_p->ctx, _y, d, bytes);
}

void fft_execute(fftplan _p) { fft_execute_batch(_p, _p->x, _p->y, 1); }

void fft_set_stream(fftplan _p, void *_s) { lq_ctx_set_stream(&_p->ctx, _s); }

void fft_run(unsigned int _n, liquid_float_complex *_x, liquid_float_complex *_y, int _dir, int _flags)
{
    fftplan p = fft_create_plan(_n, _x, _y, _dir, _flags);
    fft_execute(p);
    fft_destroy_plan(p);
}

void fft_r2r_1d_run(unsigned int _n, float *_x, float *_y, int _type, int _flags)
{
    fftplan p = fft_create_plan_r2r_1d(_n, _x, _y, _type, _flags);
    fft_execute(p);
    fft_destroy_plan(p);
}

/* fft_common.c:336-350: swap halves in place (odd n: the first (n-1)/2
 * samples with the next (n-1)/2, the last sample stays) -- a permutation of
 * the caller's host array, no arithmetic */
void fft_shift(liquid_float_complex *_x, unsigned int _n)
{
    const unsigned int n2 = (_n % 2) ? (_n - 1) / 2 : _n / 2;
    for (unsigned int i = 0; i < n2; i++) {
        liquid_float_complex t = _x[i];
        _x[i] = _x[i + n2];
        _x[i + n2] = t;
    }
}

unsigned int liquid_nextpow2(unsigned int _x)
{
    if (_x == 0) LQ_FAIL("error: liquid_nextpow2(), input must be greater than zero\n");
    _x--;
    unsigned int n = 0;
    while (_x > 0) {
        _x >>= 1;
        n++;
    }
    return n;
}
