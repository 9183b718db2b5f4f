// mb_firmx.hip -- times the firfilt matrix-core kernel (dev tool): h = 64,
// 2^28 complex samples, device resident.  Build with -DKSRC=<kernel file> to
// A/B two versions of csrc/k_firfilt_mx.hip.
#define STR2(x) #x
#define STR(x) STR2(x)
#include STR(KSRC)

#include <cstdio>
#include <vector>

void lq_check(hipError_t e, const char *what, const char *file, int line)
{
    if (e != hipSuccess) {
        fprintf(stderr, "%s:%d %s: %s\n", file, line, what, hipGetErrorString(e));
        exit(1);
    }
}

int main(int argc, char **argv)
{
    const long long n = 1LL << 28;
    float2 *x, *y, *win;
    float *h;
    LQ_CHECK(hipMalloc(&x, n * 8));
    LQ_CHECK(hipMalloc(&y, n * 8));
    LQ_CHECK(hipMalloc(&win, 64 * 8));
    LQ_CHECK(hipMalloc(&h, 64 * 4));
    std::vector<float> hh(64);
    for (int i = 0; i < 64; i++) hh[i] = (float)((i * 37) % 101) / 101.0f - 0.5f;
    LQ_CHECK(hipMemcpy(h, hh.data(), 256, hipMemcpyHostToDevice));
    LQ_CHECK(hipMemset(x, 0, n * 8));
    LQ_CHECK(hipMemset(win, 0, 512));
    lqk_fir_desc d{};
    d.kind = 1;
    d.hlen = 64;
    d.hc = 64;
    d.nchunk = 1;
    d.hpad = h;
    d.scale_re = 1.0f;
    d.scale_im = 0.0f;
#ifndef NO_MXOK
    d.mx_ok = 1;
#endif
    hipStream_t s;
    LQ_CHECK(hipStreamCreate(&s));
    for (int rep = 0; rep < 3; rep++) {
        for (int i = 0; i < 3; i++) lqk_firfilt_mx(&d, win, x, n, y, s);
        hipEvent_t e0, e1;
        LQ_CHECK(hipEventCreate(&e0));
        LQ_CHECK(hipEventCreate(&e1));
        LQ_CHECK(hipEventRecord(e0, s));
        const int it = 20;
        for (int i = 0; i < it; i++) lqk_firfilt_mx(&d, win, x, n, y, s);
        LQ_CHECK(hipEventRecord(e1, s));
        LQ_CHECK(hipEventSynchronize(e1));
        float ms;
        LQ_CHECK(hipEventElapsedTime(&ms, e0, e1));
        ms /= it;
        printf("%-10s %8.3f ms  %7.0f GB/s\n", argc > 1 ? argv[1] : "", ms, 16.0 * n / (ms * 1e-3) / 1e9);
    }
    return 0;
}
