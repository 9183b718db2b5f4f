// mb_pfb2.hip -- phase experiments on the firpfbch2 M=1024 analyzer fast path
// (dev tool).  Includes the library kernel source; 2^27 input samples,
// device resident; XMODE variants drop one phase each and record clocks.
#include "../../liquid-dsp_amd/csrc/k_pfb2_fast.hip"
#include "pfb2_experiments.h"

#include <cmath>
#include <cstdio>
#include <vector>

void lq_check(hipError_t e, const char *what, const char *file, int line)
{
    if (e != hipSuccess) {
        fprintf(stderr, "%s:%d %s: %s\n", file, line, what, hipGetErrorString(e));
        exit(1);
    }
}
static float2 *g_tw = nullptr;
extern "C" const float *lqrt_twiddles(void) { return (const float *)g_tw; }
// the channelizer fast paths' state updates call the library's batched FFT; unused here
extern "C" void lqk_fft_batch(unsigned int, int, const void *, void *, unsigned long long, void *) {}
extern "C" void lqk_fft_batch_scaled(unsigned int, int, const void *, void *, unsigned long long, float, float, void *) {}

template <int PF>
static void run(const char *name, Params P, const float *hsub, unsigned nwg, int iters)
{
    hipEvent_t e0, e1;
    LQ_CHECK(hipEventCreate(&e0));
    LQ_CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_pfb2_an1024<8, PF>), dim3(nwg), dim3(NT), 0, 0, P, hsub, g_tw);
    LQ_CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; i++) hipLaunchKernelGGL((k_pfb2_an1024<8, PF>), dim3(nwg), dim3(NT), 0, 0, P, hsub, g_tw);
    LQ_CHECK(hipEventRecord(e1));
    LQ_CHECK(hipEventSynchronize(e1));
    float ms;
    LQ_CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    const double n = (double)P.n_in;
    printf("%-28s %8.3f ms  %7.1f GS/s  %6.0f GB/s\n", name, ms, n / (ms * 1e-3) / 1e9, 24.0 * n / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

template <int PF, int WPE = 4>
static void run_v2(const char *name, Params P, const float *hsub, unsigned nwg, int iters)
{
    hipEvent_t e0, e1;
    LQ_CHECK(hipEventCreate(&e0));
    LQ_CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_pfb2_an1024_v2<8, PF, WPE>), dim3(nwg), dim3(NT2), 0, 0, P, hsub, g_tw);
    LQ_CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; i++) hipLaunchKernelGGL((k_pfb2_an1024_v2<8, PF, WPE>), dim3(nwg), dim3(NT2), 0, 0, P, hsub, g_tw);
    LQ_CHECK(hipEventRecord(e1));
    LQ_CHECK(hipEventSynchronize(e1));
    float ms;
    LQ_CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    const double n = (double)P.n_in;
    printf("%-20s nwg %5u %8.3f ms  %7.1f GS/s  %6.0f GB/s\n", name, nwg, ms, n / (ms * 1e-3) / 1e9, 24.0 * n / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

int main()
{
    const long long nb = 1 << 18, n = nb * M2;
    float2 *x, *y, *hist;
    float *hsub;
    LQ_CHECK(hipMalloc(&x, n * 8));
    LQ_CHECK(hipMalloc(&y, nb * M * 8));
    LQ_CHECK(hipMalloc(&hist, 2 * 4 * M * 8));
    LQ_CHECK(hipMalloc(&hsub, M * 8 * 4));
    LQ_CHECK(hipMalloc(&g_tw, 4096 * 8));
    LQ_CHECK(hipMemset(hist, 0, 2 * 4 * M * 8));
    std::vector<float> hx(2 * n), hh(M * 8);
    std::vector<float2> tw(4096);
    unsigned s = 1;
    for (long long i = 0; i < 2 * n; i++) {
        s = s * 1664525u + 1013904223u;
        hx[i] = (float)(s >> 8) / 16777216.0f - 0.5f;
    }
    for (int i = 0; i < M * 8; i++) hh[i] = (float)((i * 37) % 101) / 101.0f * 1e-3f;
    for (int e = 0; e < 4096; e++) tw[e] = make_float2((float)cos(2 * M_PI * e / 4096), (float)-sin(2 * M_PI * e / 4096));
    LQ_CHECK(hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice));
    LQ_CHECK(hipMemcpy(hsub, hh.data(), M * 8 * 4, hipMemcpyHostToDevice));
    LQ_CHECK(hipMemcpy(g_tw, tw.data(), 4096 * 8, hipMemcpyHostToDevice));

    Params P;
    P.x = x;
    P.hist = hist;
    P.n_in = n;
    P.B0 = 0;
    P.nblk = nb;
    P.Y = y;
    const long long ngroups = nb / 16;
    long long gpw = (ngroups + 255) / 256;
    if (gpw < 4) gpw = 4;
    const unsigned nwg = (unsigned)((ngroups + gpw - 1) / gpw);
    P.gs0 = 0;
    P.gpw = (int)gpw;
    P.gend = ngroups;
    const int it = 10;
    for (int rep = 0; rep < 3; rep++) {
        run<8>("library PF8", P, hsub, nwg, it);
        run<6>("PF6", P, hsub, nwg, it);
        for (int g : {64, 65}) {
            Params Q = P;
            Q.gpw = g;
            const unsigned nw = (unsigned)((ngroups + g - 1) / g);
            char nm[64];
            snprintf(nm, sizeof nm, "gpw %d (%u WGs)", g, nw);
            run<8>(nm, Q, hsub, nw, it);
        }
    }
    return 0;
}
