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
