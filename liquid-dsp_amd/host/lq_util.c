/*
 * lq_util.c -- host-side helpers that programs using this path commonly
 * call beside it (the reference's own examples for these objects do):
 * the root-raised-cosine design, the Hamming window and the uniform /
 * Gaussian random helpers.  Create-time / test-signal code, not stream
 * processing; restated from the reference so a program built against this
 * library behaves the same.
 *
 *   liquid_firdes_rrcos  src/filter/src/rrcos.c:37-94   (include/liquid.h:1580)
 *   hamming              src/math/src/math.c:314-318    (include/liquid.h:4445)
 *   randf                include/liquid.internal.h:1731, src/random/src/rand.c:34
 *   randnf, awgn         src/random/src/randn.c:33-53   (include/liquid.h:6312-6313)
 *   crandnf, cawgn       src/random/src/randn.c:56-82   (include/liquid.h:6314-6315)
 */
#include <complex.h>
#include <math.h>

#include "lq_host.h"

void liquid_firdes_rrcos(unsigned int _k, unsigned int _m, float _beta, float _dt, float *_h)
{
    if (_k < 1) LQ_FAIL("error: liquid_firdes_rrcos(): k must be greater than 0\n");
    if (_m < 1) LQ_FAIL("error: liquid_firdes_rrcos(): m must be greater than 0\n");
    if (_beta < 0.0f || _beta > 1.0f) LQ_FAIL("error: liquid_firdes_rrcos(): beta must be in [0,1]\n");
    const unsigned int h_len = 2 * _k * _m + 1;
    const float T = 1.0f;
    for (unsigned int n = 0; n < h_len; n++) {
        const float z = ((float)n + _dt) / (float)_k - (float)_m;
        const float t1 = cosf((1 + _beta) * M_PI * z);
        const float t2 = sinf((1 - _beta) * M_PI * z);
        if (fabsf(z) < 1e-5) {                       /* z = 0 */
            _h[n] = 1 - _beta + 4 * _beta / M_PI;
            continue;
        }
        const float t3 = 1 / ((4 * _beta * z));
        float g = 1 - 16 * _beta * _beta * z * z;
        g *= g;
        if (g < 1e-5) {                              /* 16 beta^2 z^2 = 1 */
            const float g1 = 1 + 2.0f / M_PI, g2 = sinf(0.25f * M_PI / _beta);
            const float g3 = 1 - 2.0f / M_PI, g4 = cosf(0.25f * M_PI / _beta);
            _h[n] = _beta / sqrtf(2.0f) * (g1 * g2 + g3 * g4);
        } else {
            const float t4 = 4 * _beta / (M_PI * sqrtf(T) * (1 - (16 * _beta * _beta * z * z)));
            _h[n] = t4 * (t1 + (t2 * t3));
        }
    }
}

float hamming(unsigned int _n, unsigned int _N) { return 0.53836 - 0.46164 * cosf((2 * M_PI * (float)_n) / ((float)(_N - 1))); }

float randf(void) { return (float)rand() / (float)RAND_MAX; }

float randnf(void)
{
    float u1, u2;
    do {
        u1 = randf();
    } while (u1 == 0.0f);
    u2 = randf();
    return sqrtf(-2 * logf(u1)) * sinf(2 * M_PI * u2);
}

void awgn(float *_x, float _nstd) { *_x += randnf() * _nstd; }

void crandnf(liquid_float_complex *_y)
{
    float u1, u2;
    do {
        u1 = randf();
    } while (u1 == 0.0f);
    u2 = randf();
    *_y = sqrtf(-2 * logf(u1)) * cexpf(_Complex_I * 2 * M_PI * u2);
}

void cawgn(liquid_float_complex *_x, float _nstd)
{
    liquid_float_complex y;
    crandnf(&y);
    *_x += y * _nstd * 0.707106781186547f;
}

/* ------------------------------------------------------------------ windows
 * src/math/src/math.c:198-360 */
float kaiser(unsigned int _n, unsigned int _N, float _beta, float _mu)
{
    if (_n > _N) LQ_FAIL("error: kaiser(), sample index must not exceed window length\n");
    if (_beta < 0) LQ_FAIL("error: kaiser(), beta must be greater than or equal to zero\n");
    if (_mu < -0.5 || _mu > 0.5) LQ_FAIL("error: kaiser(), fractional sample offset must be in [-0.5,0.5]\n");
    return lq_kaiser_window(_n, _N, _beta, _mu);
}

float hann(unsigned int _n, unsigned int _N) { return 0.5f - 0.5f * cosf((2 * M_PI * (float)_n) / ((float)(_N - 1))); }

float blackmanharris(unsigned int _n, unsigned int _N)
{
    const float t = 2 * M_PI * (float)_n / ((float)(_N - 1));
    return 0.35875f - 0.48829f * cosf(t) + 0.14128f * cosf(2 * t) - 0.01168f * cosf(3 * t);
}

float liquid_rcostaper_windowf(unsigned int _n, unsigned int _t, unsigned int _N)
{
    if (_n > _N) LQ_FAIL("error: liquid_rcostaper_windowf(), sample index must not exceed window length\n");
    if (_t > _N / 2) LQ_FAIL("error: liquid_rcostaper_windowf(), taper length cannot exceed half window length\n");
    if (_n > _N - _t - 1) _n = _N - _n - 1;   /* symmetric taper */
    return (_n < _t) ? 0.5f - 0.5f * cosf(M_PI * ((float)_n + 0.5f) / (float)_t) : 1.0f;
}

/* Kaiser-Bessel derived window: cumulative sums of a Kaiser window of M+1 */
float liquid_kbd(unsigned int _n, unsigned int _N, float _beta)
{
    if (_n >= _N) LQ_FAIL("error: liquid_kbd(), index exceeds maximum\n");
    if (_N == 0) LQ_FAIL("error: liquid_kbd(), window length must be greater than zero\n");
    if (_N % 2) LQ_FAIL("error: liquid_kbd(), window length must be odd\n");
    const unsigned int M = _N / 2;
    if (_n >= M) return liquid_kbd(_N - _n - 1, _N, _beta);
    float w0 = 0.0f, w1 = 0.0f;
    for (unsigned int i = 0; i <= M; i++) {
        const float w = kaiser(i, M + 1, _beta, 0.0f);
        w1 += w;
        if (i <= _n) w0 += w;
    }
    return sqrtf(w0 / w1);
}

void liquid_kbd_window(unsigned int _n, float _beta, float *_w)
{
    if (_n == 0) LQ_FAIL("error: liquid_kbd_window(), window length must be greater than zero\n");
    if (_n % 2) LQ_FAIL("error: liquid_kbd_window(), window length must be odd\n");
    if (_beta < 0.0f) LQ_FAIL("error: liquid_kbd_window(), _beta must be positive\n");
    const unsigned int M = _n / 2;
    float *wk = (float *)lq_xmalloc((M + 1) * sizeof(float));
    float sum = 0.0f, acc = 0.0f;
    for (unsigned int i = 0; i <= M; i++) sum += (wk[i] = kaiser(i, M + 1, _beta, 0.0f));
    for (unsigned int i = 0; i < M; i++) {
        acc += wk[i];
        _w[i] = sqrtf(acc / sum);
    }
    for (unsigned int i = 0; i < M; i++) _w[_n - i - 1] = _w[i];
    free(wk);
}
