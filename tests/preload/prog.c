/* prog.c -- a liquid-dsp program already built against libliquid (here the
 * stand-in tests/preload/liquid_stub.c), used to show that LD_PRELOAD of
 * libliquid_mi355x.so takes over its calls without relinking
 * (INTEGRATION.md section 2).  Prints firfilt_crcf and dotprod_crcf results. */
#include <complex.h>
#include <stdio.h>

#include "liquid.h"

int main(void)
{
    float h[9];
    for (unsigned int i = 0; i < 9; i++) h[i] = 0.1f * (float)(i + 1);
    float complex x[32], y[32];
    for (unsigned int i = 0; i < 32; i++) x[i] = (float)(i % 7) - 3.0f + _Complex_I * (float)(i % 5);
    firfilt_crcf q = firfilt_crcf_create(h, 9);
    firfilt_crcf_execute_block(q, x, 32, y);
    firfilt_crcf_destroy(q);
    float complex d;
    dotprod_crcf_run(h, x, 9, &d);
    for (unsigned int i = 0; i < 32; i++) printf("%.6f %.6f\n", crealf(y[i]), cimagf(y[i]));
    printf("%.6f %.6f\n", crealf(d), cimagf(d));
    return 0;
}
