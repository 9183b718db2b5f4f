// firpfbch2_crcf_example.c -- analysis then synthesis with the 2x
// oversampled channelizer through the liquid.h API: the round trip
// reproduces the input delayed by 2*M*m - M/2 + 1 samples
// (the property src/multichannel/tests/firpfbch2_crcf_autotest.c checks).
#include <complex.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <liquid/liquid.h>

int main(void)
{
    unsigned int M = 16, m = 5, nsym = 8 * m, n = M * nsym;
    firpfbch2_crcf qa = firpfbch2_crcf_create_kaiser(LIQUID_ANALYZER, M, m, 60.0f);
    firpfbch2_crcf qs = firpfbch2_crcf_create_kaiser(LIQUID_SYNTHESIZER, M, m, 60.0f);
    float complex *x = malloc(n * sizeof(float complex));
    float complex *y = malloc(n * sizeof(float complex));
    float complex *Y = malloc(M * sizeof(float complex));
    unsigned int s = 1;
    for (unsigned int i = 0; i < n; i++) {
        s = (s * 524287u) % 1031u;
        x[i] = (float)s / 1031.0f - 0.5f;
    }
    for (unsigned int i = 0; i < n; i += M / 2) {
        firpfbch2_crcf_execute(qa, &x[i], Y);
        firpfbch2_crcf_execute(qs, Y, &y[i]);
    }
    unsigned int d = 2 * M * m - M / 2 + 1;
    float err = 0.0f;
    for (unsigned int i = 0; i < n; i++) {
        float complex ref = i < d ? 0.0f : x[i - d];
        err = fmaxf(err, cabsf(y[i] - ref));
    }
    printf("firpfbch2_crcf: M=%u m=%u round-trip max error %.3e\n", M, m, err);
    firpfbch2_crcf_destroy(qa);
    firpfbch2_crcf_destroy(qs);
    free(x); free(y); free(Y);
    return err < 1e-3f ? 0 : 1;
}
