/*
 * window.c -- windowf / windowcf, the public window-buffer API.
 *
 * API include/liquid.h:296-349; semantics src/buffer/src/window.c:45-214:
 * the object holds the last `len` samples pushed (zeros initially) and
 * read() returns a pointer to them, contiguous, oldest first, valid until
 * the next push/write/clear.
 *
 * This is a host container by contract (read() gives the caller a host
 * pointer it dereferences), so it lives on the host.  The streaming objects
 * of this library do not use it: their history is read straight from device
 * memory (stateless halo reads, csrc/k_firfilt.hip).
 *
 * Layout: one linear array of cap = 2*len + 64 samples with the window at
 * v[r .. r+len).  A push writes behind the window and advances r; only when
 * the window reaches the end of the array are its len-1 newest samples moved
 * back to the front -- one memmove per len+64 pushes (the reference moves
 * len-1 samples once per 2^(floor(log2 len)+1) pushes).  write() copies
 * whole runs instead of pushing sample by sample.
 */
#include <complex.h>

#include "lq_host.h"

#define LQ_WINDOW_DEFINE(WINDOW, T, EXT, PRINT_LINE, PRINT_VALUE)                                  \
    struct WINDOW##_s {                                                                            \
        T *v;                                                                                      \
        unsigned int len, cap, r;                                                                  \
    };                                                                                             \
                                                                                                   \
    WINDOW WINDOW##_create(unsigned int _n)                                                        \
    {                                                                                              \
        if (_n == 0) LQ_FAIL("error: window%s_create(), window size must be greater than zero\n", EXT); \
        WINDOW q = (WINDOW)lq_xmalloc(sizeof(*q));                                                 \
        q->len = _n;                                                                               \
        q->cap = 2 * _n + 64;                                                                      \
        q->v = (T *)lq_xmalloc((size_t)q->cap * sizeof(T));                                        \
        WINDOW##_clear(q);                                                                         \
        return q;                                                                                  \
    }                                                                                              \
                                                                                                   \
    /* window.c:76-111: keep the newest min(old, new) samples, zeros before */                     \
    WINDOW WINDOW##_recreate(WINDOW _q, unsigned int _n)                                           \
    {                                                                                              \
        if (_n == _q->len) return _q;                                                              \
        WINDOW w = WINDOW##_create(_n);                                                            \
        const unsigned int keep = _n < _q->len ? _n : _q->len;                                     \
        WINDOW##_write(w, _q->v + _q->r + (_q->len - keep), keep);                                 \
        WINDOW##_destroy(_q);                                                                      \
        return w;                                                                                  \
    }                                                                                              \
                                                                                                   \
    void WINDOW##_destroy(WINDOW _q)                                                               \
    {                                                                                              \
        free(_q->v);                                                                               \
        free(_q);                                                                                  \
    }                                                                                              \
                                                                                                   \
    void WINDOW##_print(WINDOW _q)                                                                 \
    {                                                                                              \
        printf("window [%u elements] :\n", _q->len);                                               \
        for (unsigned int i = 0; i < _q->len; i++) {                                               \
            const T x = _q->v[_q->r + i];                                                          \
            printf("%4u", i);                                                                      \
            PRINT_VALUE(x);                                                                        \
            printf("\n");                                                                          \
        }                                                                                          \
    }                                                                                              \
                                                                                                   \
    void WINDOW##_debug_print(WINDOW _q)                                                           \
    {                                                                                              \
        printf("window [%u elements] :\n", _q->len);                                               \
        for (unsigned int i = 0; i < _q->cap; i++) {                                               \
            if (i == _q->r) printf("<r>");                                                         \
            const T x = _q->v[i];                                                                  \
            PRINT_LINE(x);                                                                         \
            printf("\n");                                                                          \
            if (i + 1 == _q->r + _q->len) printf("----------------------------------\n");          \
        }                                                                                          \
    }                                                                                              \
                                                                                                   \
    void WINDOW##_clear(WINDOW _q)                                                                 \
    {                                                                                              \
        _q->r = 0;                                                                                 \
        memset(_q->v, 0, (size_t)_q->cap * sizeof(T));                                             \
    }                                                                                              \
                                                                                                   \
    void WINDOW##_read(WINDOW _q, T **_v) { *_v = _q->v + _q->r; }                                 \
                                                                                                   \
    void WINDOW##_index(WINDOW _q, unsigned int _i, T *_v)                                         \
    {                                                                                              \
        if (_i >= _q->len) LQ_FAIL("error: window_index(), index value out of range\n");           \
        *_v = _q->v[_q->r + _i];                                                                   \
    }                                                                                              \
                                                                                                   \
    void WINDOW##_push(WINDOW _q, T _x)                                                            \
    {                                                                                              \
        if (_q->r + _q->len == _q->cap) {                                                          \
            memmove(_q->v, _q->v + _q->r + 1, (size_t)(_q->len - 1) * sizeof(T));                 \
            _q->r = 0;                                                                             \
        } else {                                                                                   \
            _q->r++;                                                                               \
        }                                                                                          \
        _q->v[_q->r + _q->len - 1] = _x;                                                           \
    }                                                                                              \
                                                                                                   \
    void WINDOW##_write(WINDOW _q, T *_x, unsigned int _n)                                         \
    {                                                                                              \
        if (_n >= _q->len) {                                                                       \
            memcpy(_q->v, _x + (_n - _q->len), (size_t)_q->len * sizeof(T));                      \
            _q->r = 0;                                                                             \
        } else if (_q->r + _q->len + _n <= _q->cap) {                                              \
            memcpy(_q->v + _q->r + _q->len, _x, (size_t)_n * sizeof(T));                           \
            _q->r += _n;                                                                           \
        } else {                                                                                   \
            memmove(_q->v, _q->v + _q->r + _n, (size_t)(_q->len - _n) * sizeof(T));                \
            memcpy(_q->v + (_q->len - _n), _x, (size_t)_n * sizeof(T));                            \
            _q->r = 0;                                                                             \
        }                                                                                          \
    }

#define LQ_WF_LINE(x) printf("  : %12.8f", (x))
#define LQ_WF_VALUE(x) printf("  : %12.4e", (x))
#define LQ_WCF_LINE(x) printf("  : %12.8f + %12.8f", crealf(x), cimagf(x))
#define LQ_WCF_VALUE(x) printf("  : %12.4e + %12.4e", crealf(x), cimagf(x))

LQ_WINDOW_DEFINE(windowf, float, "f", LQ_WF_LINE, LQ_WF_VALUE)
LQ_WINDOW_DEFINE(windowcf, liquid_float_complex, "cf", LQ_WCF_LINE, LQ_WCF_VALUE)
