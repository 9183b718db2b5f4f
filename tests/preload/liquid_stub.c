/* liquid_stub.c -- stand-in for an installed libliquid.so in the LD_PRELOAD
 * test (test infrastructure; not the reference, which is not built here).
 * It exports the handful of symbols tests/preload/prog.c calls and marks
 * every call on stderr, so the test can tell which library served it. */
#include <complex.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct firfilt_crcf_s *firfilt_crcf;

firfilt_crcf firfilt_crcf_create(float *h, unsigned int n)
{
    (void)h;
    (void)n;
    fputs("STUB firfilt_crcf_create\n", stderr);
    return (firfilt_crcf)malloc(16);
}

void firfilt_crcf_execute_block(firfilt_crcf q, float complex *x, unsigned int n, float complex *y)
{
    (void)q;
    (void)x;
    fputs("STUB firfilt_crcf_execute_block\n", stderr);
    for (unsigned int i = 0; i < n; i++) y[i] = 0.0f;
}

void firfilt_crcf_destroy(firfilt_crcf q)
{
    fputs("STUB firfilt_crcf_destroy\n", stderr);
    free(q);
}

void dotprod_crcf_run(float *h, float complex *x, unsigned int n, float complex *y)
{
    (void)h;
    (void)x;
    (void)n;
    fputs("STUB dotprod_crcf_run\n", stderr);
    *y = 0.0f;
}
