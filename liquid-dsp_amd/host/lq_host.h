/*
 * lq_host.h -- internal helpers shared by the C host objects.
 *
 * The objects keep the reference's create/execute/destroy contract
 * (include/liquid.h) and its failure style (message on stderr, exit(1)).
 * All sample arithmetic happens in the HIP kernels behind csrc/lq_kernels.h;
 * the host side only designs coefficients (create time, as the reference
 * does), validates arguments, moves buffers and tracks per-object state --
 * except the opt-in small-call mode (lq_small.c: LQ_SMALL_CALLS=host), in
 * which single-sample calls compute on the host.
 */
#ifndef LQ_HOST_H
#define LQ_HOST_H

#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../csrc/lq_kernels.h"
#include "liquid_mi355x.h"

#define LQ_FAIL(...)                                                                               \
    do {                                                                                           \
        fprintf(stderr, __VA_ARGS__);                                                              \
        exit(1);                                                                                   \
    } while (0)

/* sample kinds (also the kernel `kind` codes) */
enum { LQ_RRRF = 0, LQ_CRCF = 1, LQ_CCCF = 2 };

/* grow-on-demand device buffer */
typedef struct {
    void *p;
    size_t cap;
} lq_devbuf;

void *lq_devbuf_get(lq_devbuf *b, size_t bytes);
void lq_devbuf_free(lq_devbuf *b);

/* per-object execution context: a HIP stream (owned unless supplied) and
 * the pinned host staging of the per-call (host-pointer) API */
typedef struct {
    void *stream;
    int own;
    void *pin_in, *pin_out;   /* pinned host buffers (lazily allocated) */
    size_t in_cap, out_cap;
    unsigned *flag;           /* pinned completion word */
    unsigned seq;
    int in_busy;              /* pin_in may still be read by queued kernels */
} lq_ctx;

void lq_ctx_init(lq_ctx *c);
void lq_ctx_free(lq_ctx *c);
void lq_ctx_set_stream(lq_ctx *c, void *stream);

/* Host-pointer calls (the reference's own API, which returns with the result
 * in host memory).  lq_call_in stages x: up to LQ_PIN_IN bytes are copied
 * into pinned host memory that the kernels then read in place (no copy
 * command), larger inputs go to device buffer b by DMA; returns the pointer
 * to hand to the device path.  lq_call_out delivers a device result of up to
 * LQRT_COPYOUT_MAX bytes through one copy-out kernel + completion flag
 * (spin-wait, no stream synchronisation), larger ones by DMA + sync.
 * lq_call_done waits for a call without a result. */
#define LQ_PIN_IN (256u << 10)
const void *lq_call_in(lq_ctx *c, lq_devbuf *b, const void *x, size_t bytes);
void lq_call_out(lq_ctx *c, void *y, const void *dy, size_t bytes);
void lq_call_done(lq_ctx *c);
/* single results (firfilt/firpfb/dotprod execute) whose kernel writes the
 * pinned result itself and raises the flag: lq_sig_out returns the pinned
 * destination, the flag word and the sequence number to hand to the kernel;
 * lq_sig_wait spins for it and copies the result to y */
void *lq_sig_out(lq_ctx *c, size_t bytes, unsigned **flag, unsigned *seq);
void lq_sig_wait(lq_ctx *c, void *y, size_t bytes, unsigned seq);

/* opt-in host path for single-sample calls (host/lq_small.c) */
int lq_small_host(void);
void lq_host_dot(int kind, const float *h, const void *x, unsigned int n, void *y);
float *lq_host_taps(int kind, const float *h, unsigned int n, int rev);
void lq_host_tdot(int kind, const float *g, const void *x, unsigned int n, void *y);
typedef struct {
    unsigned char *buf;
    size_t n, esz, cap, off;   /* history = n samples at buf + off*esz */
    int host_valid, dev_valid;
} lq_mirror;
void lq_mirror_init(lq_mirror *m, size_t n, size_t esz);
void lq_mirror_free(lq_mirror *m);
void lq_mirror_zero(lq_mirror *m);
void lq_mirror_need_host(lq_mirror *m, const void *dev_hist, void *stream);
void lq_mirror_need_dev(lq_mirror *m, void *dev_hist, void *stream);
void lq_mirror_append(lq_mirror *m, const void *x, size_t k);
void lq_mirror_commit(lq_mirror *m, size_t k);
unsigned char *lq_mirror_ptr(lq_mirror *m);

void *lq_xmalloc(size_t bytes);
unsigned int lq_msb_index(unsigned int x);
int lq_is_pow2(unsigned int x);

/* host-side design routines (create time only; src/filter/src/firdes.c) */
float lq_kaiser_beta_As(float As);
void lq_firdes_kaiser(unsigned int n, float fc, float As, float mu, float *h);
float lq_sincf(float x);                                                   /* math.c:128-139 */
float lq_kaiser_window(unsigned int n, unsigned int N, float beta, float mu); /* math.c:289-312 */

/* generic firfilt engine used by the three typed front ends */
typedef struct lq_firfilt_s lq_firfilt;
lq_firfilt *lq_firfilt_create(int kind, const float *h, unsigned int n, const char *who);
lq_firfilt *lq_firfilt_recreate(lq_firfilt *q, const float *h, unsigned int n);
void lq_firfilt_destroy(lq_firfilt *q);
void lq_firfilt_reset(lq_firfilt *q);
void lq_firfilt_print(lq_firfilt *q);
void lq_firfilt_set_scale(lq_firfilt *q, float re, float im);
void lq_firfilt_push(lq_firfilt *q, const void *x);
void lq_firfilt_execute(lq_firfilt *q, void *y);
void lq_firfilt_execute_block(lq_firfilt *q, const void *x, unsigned long long n, void *y);
void lq_firfilt_execute_block_dev(lq_firfilt *q, const void *dx, unsigned long long n, void *dy);
unsigned int lq_firfilt_get_length(lq_firfilt *q);
lq_ctx *lq_firfilt_ctx(lq_firfilt *q);

/* arbitrary-rate resampler engine (host/resamp.c), used by msresamp */
typedef struct lq_rs_s lq_rs;
lq_rs *lq_rs_create(int kind, float rate, unsigned int m, float fc, float As, unsigned int npfb);
void lq_rs_destroy(lq_rs *q);
void lq_rs_reset(lq_rs *q);
unsigned long long lq_rs_num_output(lq_rs *q, unsigned long long nx);
void lq_rs_block_dev(lq_rs *q, const void *dx, unsigned long long nx, void *dy, unsigned long long *ny);
/* msresamp's interpolating chain: the resampler followed by one half-band
 * interpolator stage (resamp2 interp mode), fused into k_resamp4 where the
 * plan allows (lqk_resamp4_hb_supported) and run as two kernels otherwise */
typedef struct {
    int m;                        /* the stage's semi-length */
    float h1[LQK_RS4_HB_MAXM * 2];/* its odd taps (real) */
    void *w[2][2];                /* its ping-pong windows [buffer][window] */
    int *cur;                     /* its current buffer, flipped per fused launch */
    void (*run)(void *ctx, const void *u, unsigned long long n, void *y);   /* the stage alone: n -> 2n */
    void *ctx;
} lq_rs_hb;
void lq_rs_block_dev_hb(lq_rs *q, const void *dx, unsigned long long nx, void *dy, unsigned long long *ny,
                        const lq_rs_hb *hb);
lq_ctx *lq_rs_ctx(lq_rs *q);

/* generic dotprod engine */
typedef struct lq_dotprod_s lq_dotprod;
lq_dotprod *lq_dotprod_create(int kind, const float *h, unsigned int n);
lq_dotprod *lq_dotprod_recreate(lq_dotprod *q, const float *h, unsigned int n);
void lq_dotprod_destroy(lq_dotprod *q);
void lq_dotprod_print(lq_dotprod *q);
void lq_dotprod_execute_batch(lq_dotprod *q, const void *X, unsigned long long nvec, void *Y);
void lq_dotprod_execute_batch_dev(lq_dotprod *q, const void *dX, unsigned long long nvec, void *dY);
void lq_dotprod_run(int kind, const float *h, const void *x, unsigned int n, void *y);
lq_ctx *lq_dotprod_ctx(lq_dotprod *q);

#endif
