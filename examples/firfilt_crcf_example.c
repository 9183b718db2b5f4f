// firfilt_crcf_example.c -- a liquid-dsp style program using only the
// liquid.h API (compiles unchanged against liquid-dsp or liquid-mi355x).
// Filters a noisy tone with a Kaiser low-pass, once sample-by-sample
// (push/execute) and once as a block, and checks both paths agree.
#include <complex.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <liquid/liquid.h>

int main(void)
{
    unsigned int h_len = 64, n = 512;
    firfilt_crcf qa = firfilt_crcf_create_kaiser(h_len, 0.2f, 60.0f, 0.0f);
    firfilt_crcf qb = firfilt_crcf_create_kaiser(h_len, 0.2f, 60.0f, 0.0f);
    firfilt_crcf_set_scale(qa, 0.5f);
    firfilt_crcf_set_scale(qb, 0.5f);

    float complex *x = malloc(n * sizeof(float complex));
    float complex *ya = malloc(n * sizeof(float complex));
    float complex *yb = malloc(n * sizeof(float complex));
    unsigned int s = 12345;
    for (unsigned int i = 0; i < n; i++) {
        s = s * 1103515245u + 12345u;
        float noise = ((s >> 8) & 0xffff) / 65536.0f - 0.5f;
        x[i] = cexpf(_Complex_I * 0.05f * 2.0f * (float)M_PI * i) + 0.1f * noise;
    }
    // sample-by-sample (the reference's canonical loop)
    for (unsigned int i = 0; i < 16; i++) {
        firfilt_crcf_push(qa, x[i]);
        firfilt_crcf_execute(qa, &ya[i]);
    }
    firfilt_crcf_execute_block(qa, x + 16, n - 16, ya + 16);
    // whole block in place
    for (unsigned int i = 0; i < n; i++) yb[i] = x[i];
    firfilt_crcf_execute_block(qb, yb, n, yb);

    float err = 0.0f, mag = 0.0f;
    for (unsigned int i = 0; i < n; i++) {
        err = fmaxf(err, cabsf(ya[i] - yb[i]));
        mag = fmaxf(mag, cabsf(yb[i]));
    }
    printf("firfilt_crcf: h_len=%u, max|y|=%.4f, max|a-b|=%.3e\n", firfilt_crcf_get_length(qa), mag, err);
    firfilt_crcf_destroy(qa);
    firfilt_crcf_destroy(qb);
    free(x); free(ya); free(yb);
    return err <= 1e-5f * mag ? 0 : 1;
}
