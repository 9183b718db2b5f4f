/*
 * resamp.c -- resamp_{rrrf,crcf,cccf} on the MI355X.
 *
 * resamp: include/liquid.h:2938-3015, src/filter/src/resamp.c:79-363.
 *   Prototype 2*m*npfb+1 Kaiser taps at fc/npfb scaled by npfb/sum(h); bank
 *   from the first 2*m*npfb taps (L = 2m); per input the float32 timing
 *   state machine emits (1-mu) y0 + mu y1 outputs.
 *
 * The resampler's timing state (tau, b, mu, INTERP/BOUNDARY) evolves
 * independently of the data, so it is tabulated on the host -- a "plan" --
 * and the GPU replays it: entry j = state before input j, K[j] = outputs
 * before input j.  The float32 recurrence visits a finite set of states and
 * is eventually periodic (r = 1.037, npfb = 64: period 1 011 163 inputs);
 * for calls of >= RS_PERIODIC_MIN inputs the pre-period and period are found
 * once per rate with Brent's cycle detection and the plan is reused for every
 * later call.  Short calls (and rates whose period exceeds RS_MAX_PERIOD)
 * get a plan covering just that call.  Every output sample is computed on
 * the GPU (csrc/k_resamp.hip).  The taps are real for every type
 * (resamp.c:117-132 designs them with liquid_firdes_kaiser), so cccf runs the
 * crcf kernel and rrrf its real-sample instantiation.
 */
#include <math.h>

#include "lq_host.h"

/* ================================================================== resamp */

#define RS_PERIODIC_MIN (1ull << 16)   /* calls at least this long use (and build) a periodic plan */
#define RS_MAX_PERIOD (1ull << 25)     /* give up on periodic plans beyond this many inputs */
#define RS_DIRECT_CHUNK (1ull << 24)   /* direct plans cover at most this many inputs */
#define RS_DIRECT_AHEAD (1ull << 14)   /* ... and at least this many (built ahead for short calls) */
#define RS_EARLY 4                     /* a cycle may start at any of the first RS_EARLY states */
#define RS_HCK 16                      /* host checkpoints: one per RS_HCK inputs */
#define RS_REC_CAP (1ull << 22)        /* device entries recorded during the period search (<= 64 MB) */
#define RS_D4_MAXOUT (1ull << 26)      /* output plans cover at most this many outputs (128 MB of entries) */

enum { RS_BOUNDARY = 0, RS_INTERP = 1 };
enum { RS_D3 = 3, RS_D4 = 4 };        /* device plan: input checkpoints (k_resamp3) / output plan (k_resamp4) */

typedef struct {
    float tau, mu;
    int b, st;
} rs_state;

/* a device table being recorded on the host (freed once uploaded) */
typedef struct {
    int kind;                     /* RS_D3 or RS_D4 */
    int p2;                       /* RS_D3: lqk_rs_entry_p2 entries, else lqk_rs_entry */
    unsigned char *buf;
    size_t n, cap, esz, max;
    int overflow;                 /* more than `max` entries were due */
    int d4_ok;                    /* RS_D4: every input after the first output emitted one or two outputs */
    unsigned long long opre;      /* RS_D4: outputs 0, 4, .. below opre, then opre, opre + 4, .. */
    unsigned long long kmax;      /* RS_D4: ... below kmax */
} rs_rec;

typedef struct {
    int valid, periodic;
    rs_state origin;
    lqk_rs_entry *tab;            /* host: state at plan position c * RS_HCK (K lookups) */
    size_t nck, cap;
    unsigned long long pre, P, Q, end;
    int dk;                       /* device table kind (RS_D3 / RS_D4) */
    rs_rec rec;                   /* its host copy until uploaded */
    lq_devbuf d_tab;
    unsigned long long d_n;       /* entries on the device */
    unsigned long long opre, npre, QT, PT;   /* RS_D4: outputs >= opre repeat every QT outputs / PT inputs */
} rs_plan;

struct lq_rs_s {
    int kind;
    size_t esz;                   /* bytes per sample */
    float rate, del, fc, As;
    unsigned int m, npfb, L;
    void *d_taps;                 /* npfb x L float pairs (bank b, bank b+1) */
    void *d_taps2;                /* (npfb+1) x LP interpolation pairs on one window (lq_kernels.h) */
    rs_plan pl;
    int periodic_failed;          /* no period <= RS_MAX_PERIOD at this rate */
    int rate_changed;             /* set_rate / adjust_rate since the last plan */
    unsigned long long gpos;      /* inputs consumed since the plan origin */
    rs_state now;                 /* timing state at gpos */
    void *d_hist[2];              /* last L inputs */
    int cur;
    float *hbank;                 /* host bank taps h[b + n*npfb], n < L, reversed and expanded (lq_host_taps), hbs floats per bank */
    size_t hbs;
    lq_mirror hm;                 /* host copy of the history (small-call mode) */
    rs_state hs;                  /* timing state of the host path, valid while hs_valid */
    int hs_valid;
    lq_ctx ctx;
    lq_devbuf xbuf, ybuf, ubuf;   /* ubuf: resampler outputs of an unfused chain chunk */
};

static const char *lq_ext[] = {"rrrf", "crcf", "cccf"};

static const rs_state rs_initial = {0.0f, 0.0f, 0, RS_INTERP};   /* resamp.c:181-195 */

static int rs_eq(const rs_state *a, const rs_state *b)
{
    return memcmp(&a->tau, &b->tau, 4) == 0 && memcmp(&a->mu, &b->mu, 4) == 0 && a->b == b->b && a->st == b->st;
}

/* one input of resamp.c:245-311 with the data path removed; returns the
 * number of outputs.  float32 arithmetic exactly as the reference (the
 * library is compiled with -ffp-contract=off) */
static unsigned int rs_step(rs_state *s, float del, unsigned int npfb)
{
    unsigned int n = 0;
    const int np = (int)npfb;
    /* resamp.c:254 compares int b with unsigned npfb: the comparison is
     * unsigned, so a negative b (a BOUNDARY update that leaves tau < 0, only
     * when del < 1/npfb) ends the loop, and the decrement below (unsigned
     * arithmetic there too) keeps b negative until it wraps modulo 2^32 */
    while ((unsigned int)s->b < npfb) {
        if (s->st == RS_INTERP && s->b == np - 1) {
            s->st = RS_BOUNDARY;
            s->b = np;
            break;
        }
        n++;
        s->tau += del;                              /* resamp.c:352-363 */
        float bf = s->tau * (float)npfb;
        s->b = (int)floorf(bf);
        s->mu = bf - (float)s->b;
        s->st = RS_INTERP;
    }
    s->tau -= 1.0f;                                 /* resamp.c:305-307 */
    s->b = (int)((unsigned int)s->b - npfb);
    return n;
}

/* Power-of-two banks: tau*npfb is exact, so the state before an input is a
 * function of tau alone -- b < npfb <=> tau < 1, the INTERP check b == npfb-1
 * <=> tau in [1 - 1/npfb, 1), BOUNDARY <=> tau < 0 (b = 0), and mu =
 * frac(tau*npfb) equals the fraction of the last update (tau then differed by
 * whole samples).  One input is then: add del until tau reaches 1 - 1/npfb,
 * subtract 1 (the same float32 operations as rs_step, in the same order). */
static inline unsigned int rs_step_p2(float *t, float del, float z)
{
    float x = *t;
    unsigned int n = 0;
    while (x < z) {
        x += del;
        n++;
    }
    *t = x - 1.0f;
    return n;
}

static rs_state rs_from_tau(float tau, unsigned int npfb)
{
    rs_state s;
    const float bf = tau * (float)npfb, fb = floorf(bf);
    s.tau = tau;
    s.mu = bf - fb;
    s.st = tau < 0.0f ? RS_BOUNDARY : RS_INTERP;
    s.b = s.st == RS_INTERP ? (int)fb : 0;
    return s;
}

static int rs_pow2(unsigned int npfb) { return (npfb & (npfb - 1)) == 0; }

/* the tau-only plan form needs a power-of-two bank count and del >= 1/npfb:
 * then tau >= 0 after every update (a BOUNDARY update adds del to a tau in
 * [-1/npfb, 0), exactly) and b never goes negative.  Rates above npfb keep
 * the full state, whose unsigned loop test stops a negative b (rs_step). */
static int rs_p2(const lq_rs *q) { return rs_pow2(q->npfb) && q->del * (float)q->npfb >= 1.0f; }

/* the output-plan kernel (k_resamp4): complex samples, tau-only timing,
 * r > 1/4 (del < 4; tau-only timing needs del npfb >= 1, r <= npfb); the walk
 * confirms one or two outputs per input (1/2 <= del <= 1) or an output every
 * one or two (1 < del < 2) / two to four (2 <= del < 4) inputs; past r = 2
 * any count works (the kernel's R4 class) */
static int rs_d4_shape(const lq_rs *q)
{
    const char *e = getenv("LQ_RESAMP_INPUT_PLAN");   /* 1: always the input-checkpoint kernel (k_resamp3) */
    if (e && strcmp(e, "1") == 0) return 0;
    return q->kind != LQ_RRRF && rs_p2(q) && q->del < 4.0f && lqk_resamp4_supported(q->npfb, q->L);
}

static void rs_put(lqk_rs_entry *e, const rs_state *s, unsigned long long K)
{
    e->tau = s->tau;
    e->mu = s->mu;
    e->bst = s->b * 2 + s->st;
    e->K = (unsigned int)K;
}

static rs_state rs_get(const lqk_rs_entry *e)
{
    rs_state s = {e->tau, e->mu, e->bst >> 1, e->bst & 1};
    return s;
}

static void rs_plan_reserve(rs_plan *pl, size_t n)
{
    if (n > pl->cap) {
        size_t c = pl->cap ? pl->cap : 1024;
        while (c < n) c *= 2;
        lqk_rs_entry *t = (lqk_rs_entry *)lq_xmalloc(c * sizeof(lqk_rs_entry));
        if (pl->tab) memcpy(t, pl->tab, pl->nck * sizeof(lqk_rs_entry));
        free(pl->tab);
        pl->tab = t;
        pl->cap = c;
    }
}

/* ---- device-table recording */
static void rs_rec_init(rs_rec *r, int kind, int p2, size_t max)
{
    free(r->buf);
    memset(r, 0, sizeof(*r));
    r->kind = kind;
    r->p2 = p2;
    r->esz = kind == RS_D4 ? sizeof(lqk_rs4_entry) : (p2 ? sizeof(lqk_rs_entry_p2) : sizeof(lqk_rs_entry));
    r->max = max;
    r->d4_ok = 1;
    r->opre = ~0ull;
    r->kmax = ~0ull;
}

static void rs_rec_free(rs_rec *r)
{
    free(r->buf);
    r->buf = NULL;
    r->n = r->cap = 0;
}

static void *rs_rec_push(rs_rec *r)
{
    if (r->n >= r->max) {
        r->overflow = 1;
        return NULL;
    }
    if (r->n == r->cap) {
        size_t c = r->cap ? r->cap * 2 : 4096;
        unsigned char *b = (unsigned char *)lq_xmalloc(c * r->esz);
        if (r->buf) memcpy(b, r->buf, r->n * r->esz);
        free(r->buf);
        r->buf = b;
        r->cap = c;
    }
    return r->buf + (r->n++) * r->esz;
}

/* RS_D3 checkpoint before input i (i a multiple of LQK_RS_CK) */
static void rs_rec3(rs_rec *r, const rs_state *s, float tau, unsigned long long K)
{
    if (r->p2) {
        lqk_rs_entry_p2 *e = (lqk_rs_entry_p2 *)rs_rec_push(r);
        if (e) {
            e->tau = tau;
            e->K = (unsigned int)K;
        }
    } else {
        lqk_rs_entry *e = (lqk_rs_entry *)rs_rec_push(r);
        if (e) rs_put(e, s, K);
    }
}

/* state and K at plan position g: the host checkpoint at or before g, then
 * the remaining (< RS_HCK) inputs stepped */
static rs_state rs_plan_at(const rs_plan *pl, unsigned long long g, float del, unsigned int npfb,
                           unsigned long long *K)
{
    unsigned long long j = g, add = 0;
    if (g > pl->end) j = pl->end;
    if (j >= pl->pre) {
        unsigned long long t = j - pl->pre, c = t / pl->P;
        j = pl->pre + (t - c * pl->P);
        add = c * pl->Q;
    }
    const lqk_rs_entry *e = &pl->tab[j / RS_HCK];
    rs_state s = rs_get(e);
    unsigned long long k = (unsigned long long)e->K + add;
    for (unsigned long long i = j & ~(unsigned long long)(RS_HCK - 1); i < j; i++) k += rs_step(&s, del, npfb);
    *K = k;
    return s;
}

static void rs_plan_upload(lq_rs *q)
{
    rs_rec *r = &q->pl.rec;
    size_t bytes = r->n * r->esz;
    void *d = lq_devbuf_get(&q->pl.d_tab, bytes ? bytes : 8);
    if (bytes) lqrt_h2d(d, r->buf, bytes, q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    q->pl.d_n = r->n;
    rs_rec_free(r);
}

/* walk n inputs from x0, recording a host checkpoint every RS_HCK inputs
 * (from the plan's first) and, with rec, the device table: RS_D3 a
 * checkpoint every LQK_RS_CK inputs, RS_D4 the (tau, input) of every fourth
 * output.  With `early` set, stop as soon as the state returns to one of the
 * first RS_EARLY states (a cycle without a pre-period beyond them) or meets
 * Brent's tortoise: returns the position of the return (or n), *q0 the state
 * index it returned to (RS_BRENT: a cycle of length *lam_out) */
#define RS_BRENT (~1ull)

static unsigned long long rs_walk(lq_rs *q, rs_state x0, unsigned long long n, int early, unsigned long long *q0,
                                  unsigned long long *Kend, unsigned long long *lam_out, rs_rec *rec)
{
    rs_plan *pl = &q->pl;
    pl->nck = 0;
    unsigned long long K = 0, i = 0;
    const int r3 = rec && rec->kind == RS_D3, r4 = rec && rec->kind == RS_D4;
    if (rs_p2(q)) {
        /* every state is compared (branch-free) with the first and with
         * Brent's tortoise, the state at position 2^k - 1 (and the first
         * RS_EARLY states with each other): a pure cycle ends the walk on its
         * first return, any other once the tortoise sits on the cycle
         * (r = 1.037: 1 011 163 steps).  The hot loop runs between events
         * (host checkpoints every RS_HCK inputs, tortoise resets), with the
         * device records and the returns tested inline. */
        const float del = q->del, z = 1.0f - 1.0f / (float)q->npfb;
        float t = x0.tau;
        unsigned int eb[RS_EARLY], tort, zr = 0;   /* zr: silent inputs in a row (output plan check) */
        unsigned long long tpos = 0, reset = 1;
        for (int k = 0; k < RS_EARLY; k++) eb[k] = 0x7fc00001u;
        memcpy(&tort, &t, 4);
        for (;;) {
            if ((i & (RS_HCK - 1)) == 0) {
                rs_plan_reserve(pl, pl->nck + 1);
                rs_state s = i == 0 ? x0 : rs_from_tau(t, q->npfb);
                rs_put(&pl->tab[pl->nck++], &s, K);
            }
            if (K > 0xffffffffull || i == n) break;
            if (early && i < RS_EARLY) {           /* position i: compare, record, step */
                unsigned int tb;
                memcpy(&tb, &t, 4);
                for (unsigned long long k = 0; k < i; k++)
                    if (eb[k] == tb) {
                        *q0 = k;
                        *Kend = K;
                        return i;
                    }
                eb[i] = tb;
                if (i == reset) {
                    tort = eb[i];
                    tpos = i;
                    reset = 2 * i + 1;
                }
            }
            /* run: inputs i .. stop-1, no host checkpoint inside */
            unsigned long long stop = (i | (RS_HCK - 1)) + 1;
            if (stop > n) stop = n;
            if (early && i < RS_EARLY) stop = i + 1;
            for (; i < stop; i++) {
                if (early && i >= RS_EARLY) {
                    unsigned int tb;
                    memcpy(&tb, &t, 4);
                    if ((tb == eb[0]) | (tb == tort)) {
                        for (int k = RS_EARLY - 1; k >= 0; k--)
                            if (eb[k] == tb) {
                                *q0 = (unsigned long long)k;
                                *Kend = K;
                                return i;
                            }
                        *q0 = RS_BRENT;
                        *lam_out = i - tpos;
                        *Kend = K;
                        return i;
                    }
                    if (i == reset) {   /* the tortoise moves to position 2^k - 1 */
                        tort = tb;
                        tpos = i;
                        reset = 2 * i + 1;
                    }
                }
                if (r3 && (i & (LQK_RS_CK - 1)) == 0) rs_rec3(rec, NULL, t, K);
                if (r4) {   /* the output plan: (tau, input) at the recorded outputs */
                    float x = t;
                    unsigned int c = 0;
                    while (x < z) {
                        if (K < rec->kmax && ((K < rec->opre ? K : K - rec->opre) & 3) == 0) {
                            lqk_rs4_entry *e = (lqk_rs4_entry *)rs_rec_push(rec);
                            if (e) {
                                e->tau = x;
                                e->i = (unsigned int)i;
                            }
                        }
                        x += del;
                        K++;
                        c++;
                    }
                    t = x - 1.0f;
                    if (del <= 1.0f) {   /* one or two outputs per input (r > 2: any number) */
                        if ((del >= 0.5f && c > 2) || (c == 0 && K > 0)) rec->d4_ok = 0;
                    } else {   /* at most one (del < 2) / three silent inputs in a row once outputs began */
                        zr = c == 0 && K > 0 ? zr + 1 : 0;
                        if (c > 1 || zr > (del >= 2.0f ? 3 : 1)) rec->d4_ok = 0;
                    }
                    if (i > 0xffffffffull) rec->d4_ok = 0;
                } else {
                    K += rs_step_p2(&t, del, z);
                }
            }
        }
        if (r3 && (i & (LQK_RS_CK - 1)) == 0) rs_rec3(rec, NULL, t, K);   /* the checkpoint at the end */
    } else {
        rs_state s = x0, e[RS_EARLY];
        int ne = 0;
        if (r4) rec->d4_ok = 0;
        for (;;) {
            if ((i & (RS_HCK - 1)) == 0) {
                rs_plan_reserve(pl, pl->nck + 1);
                rs_put(&pl->tab[pl->nck++], &s, K);
            }
            if (r3 && (i & (LQK_RS_CK - 1)) == 0) rs_rec3(rec, &s, s.tau, K);
            if (K > 0xffffffffull || i == n) break;
            if (early) {
                for (int k = 0; k < ne; k++)
                    if (rs_eq(&e[k], &s)) {
                        *q0 = (unsigned long long)k;
                        *Kend = K;
                        return i;
                    }
                if (ne < RS_EARLY) e[ne++] = s;
            }
            K += rs_step(&s, q->del, q->npfb);
            i++;
        }
    }
    *q0 = ~0ull;
    *Kend = K;
    return K > 0xffffffffull ? 0 : i;   /* K must fit the table's 32 bits */
}

/* the plan's K at position g < pre + P (no wrap) */
static unsigned long long rs_K_lin(lq_rs *q, unsigned long long g)
{
    rs_plan save = q->pl;
    q->pl.pre = ~0ull;
    q->pl.end = ~0ull;
    unsigned long long K;
    rs_plan_at(&q->pl, g, q->del, q->npfb, &K);
    q->pl.pre = save.pre;
    q->pl.end = save.end;
    return K;
}

/* a walk of n inputs from the plan's origin that records the device table
 * (at most max entries; an output plan's entries at outputs 0, 4, .. below
 * opre and opre, opre + 4, .. below kmax; the host checkpoints it rewrites
 * are the ones recorded before, same origin); 0 if the walk or the
 * one-or-two-outputs check of an output plan fails */
static int rs_rec_walk(lq_rs *q, unsigned long long n, int kind, size_t max, unsigned long long opre,
                       unsigned long long kmax)
{
    unsigned long long q0, Kend, lam;
    rs_rec_init(&q->pl.rec, kind, rs_p2(q), max);
    q->pl.rec.opre = opre;
    q->pl.rec.kmax = kmax;
    if (rs_walk(q, q->pl.origin, n, 0, &q0, &Kend, &lam, &q->pl.rec) != n) return 0;
    return kind != RS_D4 || q->pl.rec.d4_ok;
}

/* the device table of a plan whose host part (origin, pre, P, Q or end) is
 * built; `have` = the search walk's recording already holds it */
static int rs_plan_device(lq_rs *q, int have)
{
    rs_plan *pl = &q->pl;
    const int d4 = pl->rec.kind == RS_D4 && pl->rec.d4_ok;
    if (pl->rec.kind == RS_D4 && d4) {
        if (pl->periodic) {
            /* entries at outputs 0, 4, .. below opre = K(pre), then opre,
             * opre + 4, .. over one period of QT = mQ outputs (mP inputs),
             * QT >= 256 so a 256-output tile wraps at most once.  A pure cycle
             * (pre = 0) with Q >= 256 is exactly what the search walk recorded */
            const unsigned long long Q = pl->Q;
            unsigned long long m = 1;
            while (Q > 0 && m * Q < 256) m++;
            pl->opre = rs_K_lin(q, pl->pre);
            pl->npre = (pl->opre + 3) / 4;
            pl->QT = m * Q;
            pl->PT = m * pl->P;
            const unsigned long long need = pl->npre + (pl->QT + 3) / 4;
            if (Q > 0 && need <= RS_D4_MAXOUT / 4) {
                if (!(have && pl->opre == 0 && m == 1 && pl->rec.n >= need))
                    if (!rs_rec_walk(q, pl->pre + m * pl->P + 1, RS_D4, (size_t)need, pl->opre, pl->opre + pl->QT))
                        goto d3;
                if (pl->rec.n >= need) {
                    pl->rec.n = need;
                    pl->dk = RS_D4;
                    return 1;
                }
            }
        } else if (have && !pl->rec.overflow) {
            pl->opre = ~0ull;
            pl->npre = 0;
            pl->QT = pl->PT = 0;
            pl->dk = RS_D4;
            return 1;
        }
    }
d3:
    {
        const unsigned long long n = pl->periodic ? pl->pre + pl->P : pl->end;
        const size_t need = (size_t)(n / LQK_RS_CK + 1);
        if (!(have && pl->rec.kind == RS_D3 && pl->rec.n >= need))
            if (!rs_rec_walk(q, n, RS_D3, need, ~0ull, ~0ull) || pl->rec.n < need) return 0;
        pl->rec.n = need;
        pl->dk = RS_D3;
        return 1;
    }
}

/* Periodic plan from q->now.  The timing state visits a finite set, so the
 * walk is eventually periodic; usually the orbit returns to one of its first
 * states (r = 1.037: to the initial state after 1 011 163 inputs), found in
 * one pass that records the checkpoints as it goes.  Otherwise Brent's cycle
 * detection finds pre-period and period, and a second pass records them. */
static int rs_plan_build_periodic(lq_rs *q)
{
    const rs_state x0 = q->now;
    unsigned long long q0, Kend, lam = 0;
    rs_rec_init(&q->pl.rec, rs_d4_shape(q) ? RS_D4 : RS_D3, rs_p2(q), RS_REC_CAP);
    unsigned long long n = rs_walk(q, x0, RS_MAX_PERIOD + RS_EARLY, 1, &q0, &Kend, &lam, &q->pl.rec);
    unsigned long long pre, P;
    int have = 1;
    if (q0 != ~0ull && q0 != RS_BRENT) {
        pre = q0;
        P = n - q0;
    } else {
        int recorded = q0 == RS_BRENT;            /* the walk already covers [0, mu + lam) */
        if (!recorded) {                          /* general banks: Brent on the full state */
            rs_state tort = x0, hare = x0;
            unsigned long long power = 1;
            lam = 1;
            rs_step(&hare, q->del, q->npfb);
            while (!rs_eq(&tort, &hare)) {
                if (power == lam) {
                    if (power > RS_MAX_PERIOD) goto fail;
                    tort = hare;
                    power *= 2;
                    lam = 0;
                }
                rs_step(&hare, q->del, q->npfb);
                lam++;
            }
        }
        /* pre-period: one copy lam steps ahead, both walked until they meet */
        unsigned long long mu = 0;
        if (rs_p2(q)) {
            const float z = 1.0f - 1.0f / (float)q->npfb;
            float a = x0.tau, h = x0.tau;
            for (unsigned long long i = 0; i < lam; i++) rs_step_p2(&h, q->del, z);
            while (memcmp(&a, &h, 4) != 0) {
                if (mu > RS_MAX_PERIOD) goto fail;
                rs_step_p2(&a, q->del, z);
                rs_step_p2(&h, q->del, z);
                mu++;
            }
        } else {
            rs_state tort = x0, hare = x0;
            for (unsigned long long i = 0; i < lam; i++) rs_step(&hare, q->del, q->npfb);
            while (!rs_eq(&tort, &hare)) {
                if (mu > RS_MAX_PERIOD) goto fail;
                rs_step(&tort, q->del, q->npfb);
                rs_step(&hare, q->del, q->npfb);
                mu++;
            }
        }
        pre = mu;
        P = lam;
        if (!recorded) {
            rs_rec_init(&q->pl.rec, q->pl.rec.kind, rs_p2(q), RS_REC_CAP);
            if (rs_walk(q, x0, pre + P, 0, &q0, &Kend, &lam, &q->pl.rec) != pre + P) goto fail;
        }
    }
    q->pl.pre = pre;
    q->pl.P = P;
    q->pl.end = ~0ull;
    q->pl.Q = rs_K_lin(q, pre + P) - rs_K_lin(q, pre);
    q->pl.origin = x0;
    q->pl.periodic = 1;
    if (!rs_plan_device(q, have)) goto fail;
    q->pl.valid = 1;
    q->gpos = 0;
    return 1;
fail:
    rs_rec_free(&q->pl.rec);
    free(q->pl.tab);   /* the search's host checkpoints (up to RS_MAX_PERIOD / RS_HCK entries) */
    q->pl.tab = NULL;
    q->pl.cap = q->pl.nck = 0;
    return 0;
}

/* plan covering exactly the next nx inputs (nx <= RS_DIRECT_CHUNK) */
static void rs_plan_build_direct(lq_rs *q, unsigned long long nx)
{
    unsigned long long q0, Kend;
    unsigned long long lam;
    /* an output plan is capped at RS_D4_MAXOUT outputs (past it the walk
     * records an input plan instead) */
    rs_rec_init(&q->pl.rec, rs_d4_shape(q) ? RS_D4 : RS_D3, rs_p2(q), rs_d4_shape(q) ? RS_D4_MAXOUT / 4 : (size_t)-1);
    if (rs_walk(q, q->now, nx, 0, &q0, &Kend, &lam, &q->pl.rec) != nx || Kend > 0xffffffffull)
        LQ_FAIL("error: resamp_%s: too many outputs for one call\n", lq_ext[q->kind]);
    q->pl.pre = nx + 1;
    q->pl.P = 1;
    q->pl.Q = 0;
    q->pl.end = nx;
    q->pl.origin = q->now;
    q->pl.periodic = 0;
    if (!rs_plan_device(q, 1)) LQ_FAIL("error: resamp_%s: timing plan\n", lq_ext[q->kind]);
    q->pl.valid = 1;
    q->gpos = 0;
}

static void rs_check_rate(lq_rs *q)
{
    if (!(q->del > 0.0f) || isinf(q->del) || isnan(q->del))
        LQ_FAIL("error: resamp_%s_execute(), invalid resampling rate (%f)\n", lq_ext[q->kind], q->rate);
}

/* make the plan cover inputs [gpos, gpos + nx); returns how many of them it covers */
static unsigned long long rs_ensure_plan(lq_rs *q, unsigned long long nx)
{
    rs_check_rate(q);
    if (q->pl.valid && q->pl.periodic) return nx;
    if (q->pl.valid && q->gpos + nx <= q->pl.end) return nx;
    lqrt_sync(q->ctx.stream);                /* the old table may still be in use */
    if (q->pl.valid) {                       /* state at the end of the old plan's coverage */
        unsigned long long K;
        q->now = rs_plan_at(&q->pl, q->gpos, q->del, q->npfb, &K);
    }
    q->pl.valid = 0;
    if (!q->periodic_failed && nx >= RS_PERIODIC_MIN) {
        if (rs_plan_build_periodic(q)) {
            rs_plan_upload(q);
            return nx;
        }
        q->periodic_failed = 1;
    }
    /* a direct plan covers this call and, for short calls, the next
     * RS_DIRECT_AHEAD inputs too: the schedule does not depend on the data,
     * so per-sample execute() calls reuse one plan instead of building and
     * uploading one each (two stream synchronisations per call) */
    unsigned long long c = nx < RS_DIRECT_CHUNK ? nx : RS_DIRECT_CHUNK;
    /* right after a rate change the plan covers just this call: a loop that
     * steers the rate before every call (symsync-style) would otherwise build
     * RS_DIRECT_AHEAD inputs of schedule per call and use a fraction */
    rs_plan_build_direct(q, (c > RS_DIRECT_AHEAD || q->rate_changed) ? c : RS_DIRECT_AHEAD);
    q->rate_changed = 0;
    rs_plan_upload(q);
    return c;
}

static unsigned long long rs_K(lq_rs *q, unsigned long long g)
{
    unsigned long long K;
    rs_plan_at(&q->pl, g, q->del, q->npfb, &K);
    return K;
}

/* the plan's state at gpos becomes the object's state before a rate change */
static void rs_sync_now(lq_rs *q)
{
    if (q->pl.valid) {
        unsigned long long K;
        q->now = rs_plan_at(&q->pl, q->gpos, q->del, q->npfb, &K);
    }
}

lq_rs *lq_rs_create(int kind, float _rate, unsigned int _m, float _fc, float _As, unsigned int _npfb)
{
    if (_rate <= 0) LQ_FAIL("error: resamp_%s_create(), resampling rate must be greater than zero\n", lq_ext[kind]);
    if (_m == 0) LQ_FAIL("error: resamp_%s_create(), filter semi-length must be greater than zero\n", lq_ext[kind]);
    if (_npfb == 0) LQ_FAIL("error: resamp_%s_create(), number of filter banks must be greater than zero\n", lq_ext[kind]);
    if (_fc <= 0.0f || _fc >= 0.5f) LQ_FAIL("error: resamp_%s_create(), filter cutoff must be in (0,0.5)\n", lq_ext[kind]);
    if (_As <= 0.0f)
        LQ_FAIL("error: resamp_%s_create(), filter stop-band suppression must be greater than zero\n", lq_ext[kind]);
    lqrt_require_device("resamp_create");
    lq_rs *q = (lq_rs *)lq_xmalloc(sizeof(*q));
    q->kind = kind;
    q->esz = kind == LQ_RRRF ? 4 : 8;
    q->rate = _rate;
    q->del = 1.0f / _rate;
    q->m = _m;
    q->fc = _fc;
    q->As = _As;
    q->npfb = _npfb;
    q->L = 2 * _m;
    /* resamp.c:117-132: design, DC normalisation, bank from the first n-1 taps */
    unsigned int n = 2 * _m * _npfb + 1;
    float *hf = (float *)lq_xmalloc(n * sizeof(float));
    lq_firdes_kaiser(n, _fc / ((float)_npfb), _As, 0.0f, hf);
    float gain = 0.0f;
    for (unsigned int i = 0; i < n; i++) gain += hf[i];
    gain = (_npfb) / (gain);
    for (unsigned int i = 0; i < n; i++) hf[i] = hf[i] * gain;
    size_t ntap = (size_t)_npfb * q->L;
    float *tp = (float *)lq_xmalloc(ntap * 2 * sizeof(float));
    for (unsigned int b = 0; b < _npfb; b++)
        for (unsigned int k = 0; k < q->L; k++) {
            tp[2 * (b * q->L + k)] = hf[b + k * _npfb];
            tp[2 * (b * q->L + k) + 1] = hf[(b + 1) % _npfb + k * _npfb];
        }
    /* window form: y = sum_p c[p] x[i-L+p], p <= L */
    const unsigned int L = q->L, LP = (L + 3) & ~1u;
    size_t ntap2 = (size_t)(_npfb + 1) * LP;
    float *tp2 = (float *)lq_xmalloc(ntap2 * 2 * sizeof(float));
    for (unsigned int b = 0; b < _npfb; b++)
        for (unsigned int p = 1; p <= L; p++) {
            tp2[2 * (b * LP + p)] = hf[b + (L - p) * _npfb];
            tp2[2 * (b * LP + p) + 1] = (b + 1 < _npfb) ? hf[b + 1 + (L - p) * _npfb] : 0.0f;
        }
    for (unsigned int p = 0; p <= L; p++) {
        tp2[2 * (_npfb * LP + p)] = p < L ? hf[_npfb - 1 + (L - 1 - p) * _npfb] : 0.0f;
        tp2[2 * (_npfb * LP + p) + 1] = p >= 1 ? hf[(L - p) * _npfb] : 0.0f;
    }
    lq_ctx_init(&q->ctx);
    q->d_taps = lqrt_malloc(ntap * 2 * sizeof(float));
    lqrt_h2d(q->d_taps, tp, ntap * 2 * sizeof(float), q->ctx.stream);
    q->d_taps2 = lqrt_malloc(ntap2 * 2 * sizeof(float));
    lqrt_h2d(q->d_taps2, tp2, ntap2 * 2 * sizeof(float), q->ctx.stream);
    q->d_hist[0] = lqrt_malloc((size_t)q->L * q->esz);
    q->d_hist[1] = lqrt_malloc((size_t)q->L * q->esz);
    lqrt_sync(q->ctx.stream);
    lqrt_sync(q->ctx.stream);
    {
        const int ck = q->kind == LQ_RRRF ? LQ_RRRF : LQ_CRCF;   /* real taps for every type */
        float *hb = (float *)lq_xmalloc((size_t)q->L * sizeof(float));
        q->hbs = (size_t)q->L * (ck == LQ_RRRF ? 1 : 2);
        q->hbank = (float *)lq_xmalloc((size_t)_npfb * q->hbs * sizeof(float));
        for (unsigned int b = 0; b < _npfb; b++) {
            for (unsigned int k = 0; k < q->L; k++) hb[k] = hf[b + k * _npfb];
            float *g = lq_host_taps(ck, hb, q->L, 1);
            memcpy(q->hbank + b * q->hbs, g, q->hbs * sizeof(float));
            free(g);
        }
        free(hb);
    }
    lq_mirror_init(&q->hm, q->L, q->esz);
    q->hs_valid = 0;
    free(tp);
    free(tp2);
    free(hf);
    q->now = rs_initial;
    q->gpos = 0;
    return q;
}

void lq_rs_destroy(lq_rs *_q)
{
    lqrt_sync(_q->ctx.stream);
    lqrt_free(_q->d_taps);
    lqrt_free(_q->d_taps2);
    lqrt_free(_q->d_hist[0]);
    lqrt_free(_q->d_hist[1]);
    lq_devbuf_free(&_q->pl.d_tab);
    lq_devbuf_free(&_q->xbuf);
    lq_devbuf_free(&_q->ybuf);
    lq_devbuf_free(&_q->ubuf);
    lq_ctx_free(&_q->ctx);
    lq_mirror_free(&_q->hm);
    free(_q->hbank);
    free(_q->pl.tab);
    rs_rec_free(&_q->pl.rec);
    free(_q);
}

static void lq_rs_print(lq_rs *_q)
{
    printf("resampler [rate: %f]\n", _q->rate);
    printf("fir polyphase filterbank [%u] :\n", _q->npfb);
    for (unsigned int i = 0; i < _q->npfb; i++) printf("  bank %3u: \n", i);
}

void lq_rs_reset(lq_rs *_q)
{
    lqrt_memset(_q->d_hist[0], (size_t)_q->L * _q->esz, _q->ctx.stream);
    lqrt_memset(_q->d_hist[1], (size_t)_q->L * _q->esz, _q->ctx.stream);
    lqrt_sync(_q->ctx.stream);
    lq_mirror_zero(&_q->hm);
    _q->hs_valid = 0;
    _q->now = rs_initial;
    _q->gpos = 0;
    /* a periodic plan that starts from the initial state stays usable */
    if (!(_q->pl.valid && _q->pl.periodic && rs_eq(&_q->pl.origin, &rs_initial))) _q->pl.valid = 0;
}


static void rs_new_del(lq_rs *q, float del)
{
    if (memcmp(&del, &q->del, 4) == 0) return;
    lqrt_sync(q->ctx.stream);
    rs_sync_now(q);
    q->hs_valid = 0;
    q->del = del;
    q->pl.valid = 0;
    q->periodic_failed = 0;
    q->rate_changed = 1;
}

static void lq_rs_set_rate(lq_rs *_q, float _rate)
{
    if (_rate <= 0) LQ_FAIL("error: resamp_%s_set_rate(), resampling rate must be greater than zero\n", lq_ext[_q->kind]);
    _q->rate = _rate;
    rs_new_del(_q, 1.0f / _q->rate);
}

/* resamp.c:222-239, including its clipping of the rate to [-0.5, 0.5] */
static void lq_rs_adjust_rate(lq_rs *_q, float _delta)
{
    if (_delta > 0.1f || _delta < -0.1f)
        LQ_FAIL("error: resamp_%s_adjust_rate(), resampling rate must be in [-0.1,0.1]\n", lq_ext[_q->kind]);
    _q->rate += _delta;
    if (_q->rate > 0.5f) _q->rate = 0.5f;
    if (_q->rate < -0.5f) _q->rate = -0.5f;
    rs_new_del(_q, 1.0f / _q->rate);
}

unsigned long long lq_rs_num_output(lq_rs *_q, unsigned long long _nx)
{
    if (_nx == 0) return 0;
    unsigned long long done = 0, total = 0;
    /* periodic plans answer directly; otherwise simulate on a copy of the state */
    if (!(_q->pl.valid && _q->pl.periodic) && _nx >= RS_PERIODIC_MIN) rs_ensure_plan(_q, _nx);
    if (_q->pl.valid && (_q->pl.periodic || _q->gpos + _nx <= _q->pl.end))
        return rs_K(_q, _q->gpos + _nx) - rs_K(_q, _q->gpos);
    rs_check_rate(_q);
    rs_state s = _q->now;
    if (_q->pl.valid) {
        unsigned long long K;
        s = rs_plan_at(&_q->pl, _q->gpos, _q->del, _q->npfb, &K);
    }
    if (rs_p2(_q)) {
        const float z = 1.0f - 1.0f / (float)_q->npfb;
        float t = s.tau;
        for (; done < _nx; done++) total += rs_step_p2(&t, _q->del, z);
    } else {
        for (; done < _nx; done++) total += rs_step(&s, _q->del, _q->npfb);
    }
    return total;
}

void lq_rs_block_dev(lq_rs *_q, const void *_dxv, unsigned long long _nx, void *_dyv, unsigned long long *_ny)
{
    lq_rs_block_dev_hb(_q, _dxv, _nx, _dyv, _ny, NULL);
}

void lq_rs_block_dev_hb(lq_rs *_q, const void *_dxv, unsigned long long _nx, void *_dyv, unsigned long long *_ny,
                        const lq_rs_hb *hb)
{
    const char *_dx = (const char *)_dxv;
    char *_dy = (char *)_dyv;
    unsigned long long total = 0;
    lq_mirror_need_dev(&_q->hm, _q->d_hist[_q->cur], _q->ctx.stream);
    _q->hm.host_valid = 0;
    _q->hs_valid = 0;
    /* launches of at most LQK_RS_MAXN inputs and 2^27 outputs (32-bit
     * buffer offsets in the kernel) */
    const double r = _q->rate > 1.0f ? (double)_q->rate : 1.0;
    const unsigned long long cmax = (unsigned long long)((double)LQK_RS_MAXN / (r + 1.0)) + 1;
    while (_nx > 0) {
        unsigned long long c = rs_ensure_plan(_q, _nx < cmax ? _nx : cmax);
        unsigned long long K0 = rs_K(_q, _q->gpos), K1 = rs_K(_q, _q->gpos + c);
        void *hold = _q->d_hist[_q->cur], *hnew = _q->d_hist[_q->cur ^ 1];
        const unsigned long long nk = K1 - K0;
        const int fuse = hb && nk > 0 && _q->pl.dk == RS_D4 && lqk_resamp4_hb_supported(_q->npfb, _q->L, _q->del, hb->m);
        /* an unfused chain chunk: the resampler's outputs through ubuf */
        char *uy = hb && !fuse ? (char *)lq_devbuf_get(&_q->ubuf, (size_t)(nk ? nk : 1) * _q->esz) : _dy;
        if (_q->pl.dk == RS_D4) {
            lqk_rs4_plan kp = {_q->pl.d_tab.p, _q->pl.d_n, _q->pl.opre, _q->pl.npre, _q->pl.QT, _q->pl.PT};
            lqk_rs4_hb kh;
            if (fuse) {
                const int c0 = *hb->cur;
                kh.m = hb->m;
                memcpy(kh.h1, hb->h1, sizeof(kh.h1));
                kh.hist = hb->w[c0][0];
                kh.hist_new0 = hb->w[c0 ^ 1][0];
                kh.hist_new1 = hb->w[c0 ^ 1][1];
                *hb->cur = c0 ^ 1;
            }
            /* the kernel also writes the next history (no launch of its own) */
            const lqk_hist_job job = {hold, _dx, c, hnew, _q->L};
            lqk_resamp4(&kp, _q->gpos, K0, _q->npfb, _q->L, _q->del, _q->d_taps2, hold, _dx, c, uy, nk,
                        fuse ? &kh : NULL, &job, _q->ctx.stream);
        } else {
            lqk_rs_plan kp = {_q->pl.d_tab.p, _q->pl.pre, _q->pl.P, _q->pl.Q, _q->pl.end, rs_p2(_q)};
            lqk_resamp(_q->kind == LQ_RRRF, &kp, _q->gpos, K0, _q->npfb, _q->L, _q->del, _q->d_taps, _q->d_taps2,
                       hold, _dx, c, uy, nk, _q->ctx.stream);
        }
        if (hb && !fuse && nk > 0) hb->run(hb->ctx, uy, nk, _dy);
        if (_q->pl.dk != RS_D4) lqk_window_append(_q->kind != LQ_RRRF, hold, _q->L, _dx, c, hnew, _q->ctx.stream);
        _q->cur ^= 1;
        _q->gpos += c;
        _dx += c * _q->esz;
        _dy += (hb ? 2 : 1) * nk * _q->esz;
        total += (hb ? 2 : 1) * nk;
        _nx -= c;
    }
    rs_sync_now(_q);
    if (_ny) *_ny = total;
}

/* small-call mode: one input on the host, resamp.c:245-311 as written (the
 * BOUNDARY state's y0 -- bank npfb-1 of the previous input, which the
 * reference stored -- is recomputed on the window one input older) */
static void lq_rs_exec1_host(lq_rs *q, const void *x, void *y, unsigned int *ny)
{
    rs_check_rate(q);
    if (!q->hs_valid) {   /* the timing state at the stream position */
        if (q->pl.valid) {
            unsigned long long K;
            q->hs = rs_plan_at(&q->pl, q->gpos, q->del, q->npfb, &K);
        } else {
            q->hs = q->now;
        }
        q->hs_valid = 1;
    }
    lq_mirror_need_host(&q->hm, q->d_hist[q->cur], q->ctx.stream);
    lq_mirror_append(&q->hm, x, 1);
    const unsigned char *w = lq_mirror_ptr(&q->hm);   /* L + 1 samples, x last */
    const int ck = q->kind == LQ_RRRF ? LQ_RRRF : LQ_CRCF;   /* real taps for every type */
    const unsigned int L = q->L, npfb = q->npfb;
    const int np = (int)npfb;
    rs_state *s = &q->hs;
    unsigned int n = 0;
    while ((unsigned int)s->b < npfb) {   /* unsigned, as resamp.c:254 */
        if (s->st == RS_INTERP && s->b == np - 1) {
            s->st = RS_BOUNDARY;
            s->b = np;
            break;
        }
        float y0[2] = {0.f, 0.f}, y1[2] = {0.f, 0.f};
        if (s->st == RS_BOUNDARY) {
            /* bank npfb-1 on the window one input older, bank 0 on the newest */
            lq_host_tdot(ck, q->hbank + (size_t)(npfb - 1) * q->hbs, w, L, y0);
            lq_host_tdot(ck, q->hbank, w + q->esz, L, y1);
        } else {
            lq_host_tdot(ck, q->hbank + (size_t)s->b * q->hbs, w + q->esz, L, y0);
            lq_host_tdot(ck, q->hbank + (size_t)(s->b + 1) * q->hbs, w + q->esz, L, y1);
        }
        const float a = 1.0f - s->mu;
        float *yo = (float *)((unsigned char *)y + (size_t)n * q->esz);
        yo[0] = a * y0[0] + s->mu * y1[0];
        if (q->kind != LQ_RRRF) yo[1] = a * y0[1] + s->mu * y1[1];
        n++;
        s->tau += q->del;                          /* resamp.c:352-363 */
        const float bf = s->tau * (float)npfb;
        s->b = (int)floorf(bf);
        s->mu = bf - (float)s->b;
        s->st = RS_INTERP;
    }
    s->tau -= 1.0f;
    s->b = (int)((unsigned int)s->b - npfb);
    lq_mirror_commit(&q->hm, 1);
    /* the device path continues from here: its plan position, or its state */
    if (q->pl.valid && (q->pl.periodic || q->gpos + 1 <= q->pl.end)) q->gpos += 1;
    else q->pl.valid = 0;
    q->now = *s;
    *ny = n;
}

/* single: the call is resamp_*_execute (one input); execute_block always runs on the GPU */
static void lq_rs_block(lq_rs *_q, const void *_x, unsigned int _nx, void *_y, unsigned int *_ny, int single)
{
    if (_nx == 0) {
        *_ny = 0;
        return;
    }
    if (single && lq_small_host()) {
        lq_rs_exec1_host(_q, _x, _y, _ny);
        return;
    }
    unsigned long long nout = lq_rs_num_output(_q, _nx);
    const void *dx = lq_call_in(&_q->ctx, &_q->xbuf, _x, (size_t)_nx * _q->esz);
    void *dy = lq_devbuf_get(&_q->ybuf, (size_t)(nout ? nout : 1) * _q->esz);
    unsigned long long ny = 0;
    lq_rs_block_dev(_q, dx, _nx, dy, &ny);
    lq_call_out(&_q->ctx, _y, dy, (size_t)ny * _q->esz);
    *_ny = (unsigned int)ny;
}

lq_ctx *lq_rs_ctx(lq_rs *q) { return &q->ctx; }

#define LQ_RESAMP_FRONT(NAME, KIND, T)                                                                  \
    struct NAME##_s {                                                                               \
        lq_rs *e;                                                                                   \
    };                                                                                              \
    NAME NAME##_create(float _rate, unsigned int _m, float _fc, float _As, unsigned int _npfb)      \
    {                                                                                               \
        lq_rs *e = lq_rs_create(KIND, _rate, _m, _fc, _As, _npfb);                                  \
        NAME q = (NAME)lq_xmalloc(sizeof(*q));                                                      \
        q->e = e;                                                                                   \
        return q;                                                                                   \
    }                                                                                               \
    /* resamp.c:150-169: m = 7, fc = 0.25, As = 60, npfb = 64 */                                    \
    NAME NAME##_create_default(float _rate)                                                         \
    {                                                                                               \
        if (_rate <= 0)                                                                             \
            LQ_FAIL("error: " #NAME "_create_default(), resampling rate must be greater than zero\n"); \
        return NAME##_create(_rate, 7, 0.25f, 60.0f, 64);                                           \
    }                                                                                               \
    void NAME##_destroy(NAME _q)                                                                    \
    {                                                                                               \
        lq_rs_destroy(_q->e);                                                                       \
        free(_q);                                                                                   \
    }                                                                                               \
    void NAME##_print(NAME _q) { lq_rs_print(_q->e); }                                              \
    void NAME##_reset(NAME _q) { lq_rs_reset(_q->e); }                                              \
    unsigned int NAME##_get_delay(NAME _q) { return _q->e->m; }                                     \
    void NAME##_set_rate(NAME _q, float _rate) { lq_rs_set_rate(_q->e, _rate); }                     \
    void NAME##_adjust_rate(NAME _q, float _delta) { lq_rs_adjust_rate(_q->e, _delta); }             \
    unsigned long long NAME##_num_output(NAME _q, unsigned long long _nx)                           \
    {                                                                                               \
        return lq_rs_num_output(_q->e, _nx);                                                        \
    }                                                                                               \
    void NAME##_execute_block_dev(NAME _q, const T *_dx, unsigned long long _nx, T *_dy,            \
                                  unsigned long long *_ny)                                          \
    {                                                                                               \
        lq_rs_block_dev(_q->e, _dx, _nx, _dy, _ny);                                                 \
    }                                                                                               \
    void NAME##_execute_block(NAME _q, T *_x, unsigned int _nx, T *_y, unsigned int *_ny)           \
    {                                                                                               \
        lq_rs_block(_q->e, _x, _nx, _y, _ny, 0);                                                    \
    }                                                                                               \
    void NAME##_execute(NAME _q, T _x, T *_y, unsigned int *_num_written)                           \
    {                                                                                               \
        lq_rs_block(_q->e, &_x, 1, _y, _num_written, 1);                                            \
    }                                                                                               \
    void NAME##_set_stream(NAME _q, void *_s) { lq_ctx_set_stream(&_q->e->ctx, _s); }               \
    void NAME##_synchronize(NAME _q) { lqrt_sync(_q->e->ctx.stream); }

LQ_RESAMP_FRONT(resamp_rrrf, LQ_RRRF, float)
LQ_RESAMP_FRONT(resamp_crcf, LQ_CRCF, liquid_float_complex)
LQ_RESAMP_FRONT(resamp_cccf, LQ_CCCF, liquid_float_complex)

/* ----------------------------------------------------------------- test hook
 * Host-only plan memory (no GPU): builds the periodic plan of a fresh
 * crcf object at this rate and reports the host checkpoint table's allocation
 * and the device table's size (what the first call would upload).  Returns 1
 * (periodic plan), 0 (none within RS_MAX_PERIOD; then *_host is what is left
 * allocated after the failed search). */
int liquid_mi355x_resamp_plan_bytes(float _rate, unsigned int _npfb, unsigned long long *_host,
                                    unsigned long long *_dev, unsigned long long *_period)
{
    lq_rs q;
    memset(&q, 0, sizeof(q));
    q.kind = LQ_CRCF;
    q.rate = _rate;
    q.del = 1.0f / _rate;
    q.npfb = _npfb;
    q.L = 14;
    q.now = rs_initial;
    const int ok = rs_plan_build_periodic(&q);
    *_host = (unsigned long long)q.pl.cap * sizeof(lqk_rs_entry);
    *_dev = ok ? (unsigned long long)q.pl.rec.n * q.pl.rec.esz : 0;
    *_period = ok ? q.pl.P : 0;
    rs_rec_free(&q.pl.rec);
    free(q.pl.tab);
    return ok;
}

/* ----------------------------------------------------------------- test hook
 * Host-only check of the timing plan (no GPU): builds the plan the object
 * would use from the initial state (periodic if `periodic`, else direct) and
 * expands it exactly as k_resamp replays it, recording for every output the
 * bank index (-1 for a BOUNDARY output), mu and input index -- the format of
 * the oracle's orc_resamp_schedule().  Returns the number of outputs, or -1 if
 * no periodic plan exists within RS_MAX_PERIOD. */
long long liquid_mi355x_resamp_schedule(float _rate, unsigned int _npfb, unsigned long long _nx, int _periodic,
                                        int *_b, float *_mu, unsigned int *_idx, unsigned long long _cap,
                                        unsigned long long *_pre, unsigned long long *_period)
{
    lq_rs q;
    memset(&q, 0, sizeof(q));
    q.rate = _rate;
    q.del = 1.0f / _rate;
    q.npfb = _npfb;
    q.now = rs_initial;
    if (_periodic) {
        if (!rs_plan_build_periodic(&q)) {
            free(q.pl.tab);
            return -1;
        }
    } else {
        rs_plan_build_direct(&q, _nx);
    }
    rs_rec_free(&q.pl.rec);
    if (_pre) *_pre = q.pl.pre;
    if (_period) *_period = q.pl.P;
    unsigned long long k = 0;
    const int np = (int)_npfb;
    for (unsigned long long g = 0; g < _nx; g++) {
        unsigned long long K;
        rs_state s = rs_plan_at(&q.pl, g, q.del, q.npfb, &K);
        if (K != k) {
            free(q.pl.tab);
            return -2;                       /* plan's output count disagrees with the replay */
        }
        while ((unsigned int)s.b < _npfb) {   /* unsigned, as resamp.c:254 */
            if (s.st == RS_INTERP && s.b == np - 1) break;
            if (k < _cap) {
                _b[k] = s.st == RS_INTERP ? s.b : -1;
                _mu[k] = s.mu;
                _idx[k] = (unsigned int)g;
            }
            k++;
            s.tau += q.del;
            float bf = s.tau * (float)_npfb;
            s.b = (int)floorf(bf);
            s.mu = bf - (float)s.b;
            s.st = RS_INTERP;
        }
    }
    free(q.pl.tab);
    return (long long)k;
}

/* Host-only check of the output plan (no GPU): builds the plan a complex
 * resampler with 2m = 14 taps per bank would use from the initial state
 * (periodic if `periodic`, else direct over nx inputs) and, when it is an
 * output plan (k_resamp4), expands every output exactly as k_resamp4 does:
 * the entry at or before output k (periods unwrapped), up to three steps,
 * then bank (-1: BOUNDARY), mu and input index.  Returns the number of outputs of the
 * first nx inputs, -1 if no plan, -3 if the plan is not an output plan. */
long long liquid_mi355x_resamp_schedule4(float _rate, unsigned int _npfb, unsigned long long _nx, int _periodic,
                                         int *_b, float *_mu, unsigned int *_idx, unsigned long long _cap,
                                         unsigned long long *_pre, unsigned long long *_period)
{
    lq_rs q;
    memset(&q, 0, sizeof(q));
    q.kind = LQ_CRCF;
    q.rate = _rate;
    q.del = 1.0f / _rate;
    q.npfb = _npfb;
    q.L = 14;
    q.now = rs_initial;
    if (_periodic) {
        if (!rs_plan_build_periodic(&q)) {
            free(q.pl.tab);
            return -1;
        }
    } else {
        rs_plan_build_direct(&q, _nx);
    }
    if (q.pl.dk != RS_D4) {
        rs_rec_free(&q.pl.rec);
        free(q.pl.tab);
        return -3;
    }
    if (_pre) *_pre = q.pl.opre;
    if (_period) *_period = q.pl.QT;
    unsigned long long Kn;
    rs_plan_at(&q.pl, _nx, q.del, q.npfb, &Kn);
    const lqk_rs4_entry *t = (const lqk_rs4_entry *)q.pl.rec.buf;
    const float z = 1.0f - 1.0f / (float)_npfb, fn = (float)_npfb;
    long long ret = (long long)Kn;
    for (unsigned long long k = 0; k < Kn && k < _cap; k++) {
        unsigned long long idx = k >> 2, add = 0, skip = k & 3;
        if (k >= q.pl.opre) {
            const unsigned long long dt = k - q.pl.opre, c = dt / q.pl.QT, r = dt - c * q.pl.QT;
            idx = q.pl.npre + (r >> 2);
            skip = r & 3;
            add = c * q.pl.PT;
        }
        if (idx >= q.pl.rec.n) {
            ret = -2;
            break;
        }
        float tau = t[idx].tau;
        unsigned long long i = t[idx].i + add;
        for (unsigned s = 0; s < (unsigned)skip; s++) {   /* the kernel's step (k_resamp4.hip) */
            tau = tau + q.del;
            if (q.del > 1.0f) {
                tau = tau - 1.0f;
                i++;
            }
            if (!(tau < z)) {
                tau = tau - 1.0f;
                i++;
            }
            for (int e = 0; e < 2 && q.del >= 2.0f; e++)   /* 2 <= del < 4: up to two more silent inputs */
                if (!(tau < z)) {
                    tau = tau - 1.0f;
                    i++;
                }
        }
        const float bf = tau * fn, fb = floorf(bf);
        _b[k] = tau < 0.0f ? -1 : (int)fb;
        _mu[k] = bf - fb;
        _idx[k] = (unsigned int)i;
    }
    rs_rec_free(&q.pl.rec);
    free(q.pl.tab);
    return ret;
}
