/*
 * dotprod.c -- dotprod_{rrrf,crcf,cccf} on the MI355X.
 *
 * API: include/liquid.h:503-560; semantics src/dotprod/src/dotprod.c:42-167:
 * y = sum_i h[i] x[i] (no conjugation), coefficients copied at create.
 * _run/_run4/_execute keep their one-vector signatures; the batched
 * extension (_execute_batch, _execute_batch_dev) is the form that feeds a GPU.
 */
#include <pthread.h>

#include "lq_host.h"

struct lq_dotprod_s {
    int kind;
    unsigned int n;
    size_t csz, esz;
    float *h;
    float *hg;   /* expanded for the host path (lq_host_taps) */
    void *d_h;
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf;
};

static void lq_dotprod_set(lq_dotprod *q, const float *h, unsigned int n)
{
    q->n = n;
    free(q->h);
    q->h = (float *)lq_xmalloc((size_t)(n ? n : 1) * q->csz);
    if (n) memcpy(q->h, h, (size_t)n * q->csz);
    free(q->hg);
    q->hg = lq_host_taps(q->kind, q->h, n, 0);
    if (q->d_h) lqrt_free(q->d_h);
    q->d_h = lqrt_malloc((size_t)(n ? n : 1) * q->csz + 16);
    lqrt_h2d(q->d_h, q->h, (size_t)n * q->csz, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
}

lq_dotprod *lq_dotprod_create(int kind, const float *h, unsigned int n)
{
    lqrt_require_device("dotprod_create");
    lq_dotprod *q = (lq_dotprod *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->csz = kind == LQ_CCCF ? 8 : 4;
    q->esz = kind == LQ_RRRF ? 4 : 8;
    lq_ctx_init(&q->ctx);
    lq_dotprod_set(q, h, n);
    return q;
}

lq_dotprod *lq_dotprod_recreate(lq_dotprod *q, const float *h, unsigned int n)
{
    lqrt_sync(q->ctx.stream);
    lq_dotprod_set(q, h, n);
    return q;
}

void lq_dotprod_destroy(lq_dotprod *q)
{
    lqrt_sync(q->ctx.stream);
    lqrt_free(q->d_h);
    lq_devbuf_free(&q->xbuf);
    lq_devbuf_free(&q->ybuf);
    lq_ctx_free(&q->ctx);
    free(q->h);
    free(q->hg);
    free(q);
}

void lq_dotprod_print(lq_dotprod *q)
{
    printf("dotprod [mi355x, %u coefficients]:\n", q->n);
    for (unsigned int i = 0; i < q->n; i++) {
        if (q->kind == LQ_CCCF)
            printf("  %4u: %12.8f + j*%12.8f\n", i, q->h[2 * i], q->h[2 * i + 1]);
        else
            printf("  %4u: %12.8f\n", i, q->h[i]);
    }
}

void lq_dotprod_execute_batch_dev(lq_dotprod *q, const void *dX, unsigned long long nvec, void *dY)
{
    lqk_dotprod_batch(q->kind, q->d_h, q->n, dX, q->n, nvec, dY, q->ctx.stream);
}

void lq_dotprod_execute_batch(lq_dotprod *q, const void *X, unsigned long long nvec, void *Y)
{
    if (nvec == 0) return;
    size_t xb = (size_t)nvec * q->n * q->esz, yb = (size_t)nvec * q->esz;
    const void *dX = lq_call_in(&q->ctx, &q->xbuf, X, xb);
    void *dY = lq_devbuf_get(&q->ybuf, yb);
    lq_dotprod_execute_batch_dev(q, dX, nvec, dY);
    lq_call_out(&q->ctx, Y, dY, yb);
}

/* one dot product (the reference's dotprod_*_execute): x staged in pinned
 * memory, one kernel writes the pinned result and raises the flag */
static void lq_dotprod_execute1(lq_dotprod *q, const void *x, void *y)
{
    if (lq_small_host()) {   /* opt-in host path (lq_small.c) */
        lq_host_tdot(q->kind, q->hg, x, q->n, y);
        return;
    }
    const void *dx = lq_call_in(&q->ctx, &q->xbuf, x, (size_t)q->n * q->esz);
    unsigned *flag, seq;
    void *py = lq_sig_out(&q->ctx, q->esz, &flag, &seq);
    lqk_dotprod_single(q->kind, q->d_h, q->n, dx, py, flag, seq, q->ctx.stream);
    lq_sig_wait(&q->ctx, y, q->esz, seq);
}

lq_ctx *lq_dotprod_ctx(lq_dotprod *q) { return &q->ctx; }

/* free functions _run/_run4: one shared scratch object per kind (locked) */
static pthread_mutex_t g_run_mu = PTHREAD_MUTEX_INITIALIZER;
static lq_dotprod *g_run[3];

void lq_dotprod_run(int kind, const float *h, const void *x, unsigned int n, void *y)
{
    if (lq_small_host()) {
        lq_host_dot(kind, h, x, n, y);
        return;
    }
    pthread_mutex_lock(&g_run_mu);
    if (!g_run[kind]) g_run[kind] = lq_dotprod_create(kind, h, n);
    else lq_dotprod_recreate(g_run[kind], h, n);
    lq_dotprod_execute_batch(g_run[kind], x, 1, y);
    pthread_mutex_unlock(&g_run_mu);
}

#define LQ_DOTPROD_FRONT(NAME, KIND, TO, TC, TI)                                                    \
    struct NAME##_s {                                                                               \
        lq_dotprod *d;                                                                              \
    };                                                                                              \
    void NAME##_run(TC *_h, TI *_x, unsigned int _n, TO *_y) { lq_dotprod_run(KIND, (const float *)_h, _x, _n, _y); } \
    void NAME##_run4(TC *_h, TI *_x, unsigned int _n, TO *_y) { lq_dotprod_run(KIND, (const float *)_h, _x, _n, _y); } \
    NAME NAME##_create(TC *_v, unsigned int _n)                                                     \
    {                                                                                               \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->d = lq_dotprod_create(KIND, (const float *)_v, _n);                                      \
        return q;                                                                                   \
    }                                                                                               \
    NAME NAME##_recreate(NAME _q, TC *_v, unsigned int _n)                                          \
    {                                                                                               \
        lq_dotprod_recreate(_q->d, (const float *)_v, _n);                                          \
        return _q;                                                                                  \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_dotprod_destroy(_q->d);                                                                  \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_print(NAME _q) { lq_dotprod_print(_q->d); }                                         \
    void NAME##_execute(NAME _q, TI *_v, TO *_y) { lq_dotprod_execute1(_q->d, _v, _y); }           \
    void NAME##_execute_batch(NAME _q, TI *_X, unsigned long long _nvec, TO *_Y)                    \
    {                                                                                               \
        lq_dotprod_execute_batch(_q->d, _X, _nvec, _Y);                                             \
    }                                                                                               \
    void NAME##_execute_batch_dev(NAME _q, const TI *_dX, unsigned long long _nvec, TO *_dY)        \
    {                                                                                               \
        lq_dotprod_execute_batch_dev(_q->d, _dX, _nvec, _dY);                                       \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ctx_set_stream(lq_dotprod_ctx(_q->d), _s); }     \
    void *NAME##_get_stream(NAME _q) { return lq_dotprod_ctx(_q->d)->stream; }

LQ_DOTPROD_FRONT(dotprod_rrrf, LQ_RRRF, float, float, float)
LQ_DOTPROD_FRONT(dotprod_crcf, LQ_CRCF, liquid_float_complex, float, liquid_float_complex)
LQ_DOTPROD_FRONT(dotprod_cccf, LQ_CCCF, liquid_float_complex, liquid_float_complex, liquid_float_complex)
