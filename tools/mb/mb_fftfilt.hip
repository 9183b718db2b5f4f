// mb_fftfilt.hip -- fftfilt_crcf h=512 overlap-save kernel variants (dev tool):
// 2^26 complex samples, device resident; register/occupancy variants of the
// register radix-16 kernel against the LDS Stockham kernel.
#include "../../liquid-dsp_amd/csrc/k_fftfilt.hip"

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
extern "C" void lqk_fft_batch(unsigned int, int, const void *, void *, unsigned long long, void *) {}

template <typename K>
static void timeit(const char *name, K launch, double n)
{
    hipEvent_t e0, e1;
    LQ_CHECK(hipEventCreate(&e0));
    LQ_CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) launch();
    LQ_CHECK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; i++) launch();
    LQ_CHECK(hipEventRecord(e1));
    LQ_CHECK(hipEventSynchronize(e1));
    float ms;
    LQ_CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    printf("%-34s %8.3f ms  %7.1f GS/s  %6.0f GB/s\n", name, ms, n / (ms * 1e-3) / 1e9, 16.0 * n / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

int main()
{
    const long long n = 1LL << 26;
    const int hm1 = 511, L = NFFT - hm1;
    const long long nseg = (n + L - 1) / L;
    float2 *x, *y, *H, *hist;
    LQ_CHECK(hipMalloc(&x, n * 8));
    LQ_CHECK(hipMalloc(&y, n * 8));
    LQ_CHECK(hipMalloc(&H, NFFT * 8));
    LQ_CHECK(hipMalloc(&hist, 4096 * 8));
    LQ_CHECK(hipMalloc(&g_tw, 4096 * 8));
    std::vector<float2> tw(4096), hx(n);
    for (int e = 0; e < 4096; e++) tw[e] = make_float2((float)cos(2 * M_PI * e / 4096), (float)-sin(2 * M_PI * e / 4096));
    unsigned s = 1;
    for (long long i = 0; i < n; i++) {
        s = s * 1664525u + 1013904223u;
        hx[i] = make_float2((float)(s >> 8) / 16777216.0f - 0.5f, (float)((s >> 4) & 1023) / 1024.f - 0.5f);
    }
    LQ_CHECK(hipMemcpy(g_tw, tw.data(), 4096 * 8, hipMemcpyHostToDevice));
    LQ_CHECK(hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice));
    LQ_CHECK(hipMemcpy(H, hx.data(), NFFT * 8, hipMemcpyHostToDevice));
    LQ_CHECK(hipMemset(hist, 0, 4096 * 8));
    const float sc = 1.0f / 4096;
    for (int rep = 0; rep < 2; rep++) {
        timeit("LDS Stockham (one seg / WG)", [&] {
            hipLaunchKernelGGL(k_fftfilt<false>, dim3((unsigned)nseg), dim3(NT), 0, 0, hm1, H, hist, x, n, y, sc, 0.f, g_tw);
        }, n);
        for (unsigned grid : {1024u, 2048u, 4096u}) {
            char nm[64];
            snprintf(nm, sizeof nm, "r16 Hreg wpe2 grid %u", grid);
            timeit(nm, [&] {
                hipLaunchKernelGGL((k_fftfilt_r16<false, true, 2>), dim3(grid), dim3(NT), 0, 0, hm1, H, hist, x, n, y, sc, 0.f, g_tw);
            }, n);
            snprintf(nm, sizeof nm, "r16 Hreg wpe4 grid %u", grid);
            timeit(nm, [&] {
                hipLaunchKernelGGL((k_fftfilt_r16<false, true, 4>), dim3(grid), dim3(NT), 0, 0, hm1, H, hist, x, n, y, sc, 0.f, g_tw);
            }, n);
            snprintf(nm, sizeof nm, "r16 Hglb wpe4 grid %u", grid);
            timeit(nm, [&] {
                hipLaunchKernelGGL((k_fftfilt_r16<false, false, 4>), dim3(grid), dim3(NT), 0, 0, hm1, H, hist, x, n, y, sc, 0.f, g_tw);
            }, n);
        }
    }
    return 0;
}
