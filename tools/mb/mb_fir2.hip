// mb_fir2.hip -- variants of the library's firfilt crcf kernels (dev tool).
// Includes liquid-dsp_amd/csrc/k_firfilt.hip so the kernels timed are the
// library's own templates; h = 64 taps, 2^28 complex samples, device resident.
#include "../../liquid-dsp_amd/csrc/k_firfilt.hip"
#include "fir_experiments.h"

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

static std::vector<float> ref;

template <typename F>
static void timeit(const char *name, F launch, float2 *y, long long n, int iters)
{
    LQ_CHECK(hipMemset(y, 0, n * 8));
    launch();
    LQ_CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    LQ_CHECK(hipEventCreate(&e0));
    LQ_CHECK(hipEventCreate(&e1));
    LQ_CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; i++) launch();
    LQ_CHECK(hipEventRecord(e1));
    LQ_CHECK(hipEventSynchronize(e1));
    float ms;
    LQ_CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    std::vector<float> out(2 * n);
    LQ_CHECK(hipMemcpy(out.data(), y, n * 8, hipMemcpyDeviceToHost));
    double err = 0;
    if (ref.empty()) ref = out;
    else
        for (long long i = 0; i < 2 * n; i++) err = fmax(err, fabs(out[i] - ref[i]));
    printf("%-40s %8.3f ms  %7.1f GS/s  %6.0f GB/s  maxdiff %.2e\n", name, ms, n / (ms * 1e-3) / 1e9,
           16.0 * n / (ms * 1e-3) / 1e9, err);
    fflush(stdout);
}

int main()
{
    const long long n = 1ll << 28;
    float2 *x, *y, *win;
    float *h;
    LQ_CHECK(hipMalloc(&x, n * 8));
    LQ_CHECK(hipMalloc(&y, n * 8));
    LQ_CHECK(hipMalloc(&win, 64 * 8));
    LQ_CHECK(hipMalloc(&h, 64 * 4));
    LQ_CHECK(hipMemset(win, 0, 64 * 8));
    std::vector<float> hx(2 * n), hh(64);
    unsigned s = 1;
    for (long long i = 0; i < 2 * n; i++) {
        s = s * 1664525u + 1013904223u;
        hx[i] = (float)(s >> 8) / 16777216.0f - 0.5f;
    }
    for (int i = 0; i < 64; i++) hh[i] = (float)(i % 7) / 7.0f - 0.4f;
    LQ_CHECK(hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice));
    LQ_CHECK(hipMemcpy(h, hh.data(), 64 * 4, hipMemcpyHostToDevice));
    const int it = 10;

    for (int grid : {64, 128, 192, 256, 512, 768}) {
        char nm[64];
        snprintf(nm, sizeof nm, "mfma_p<64,2048,10> grid=%d", grid);
        timeit(nm, [&] {
            hipLaunchKernelGGL((k_fir_mfma_p<64, 2048, 10>), dim3(grid), dim3(NT), (size_t)(2048 + 64) * 16, 0, win, x, n, y,
                               h, 1.0f, 0.0f, nullptr, (long long)(n / 2048));
        }, y, n, 3);
        std::vector<unsigned long long> clk(2 * grid);
        LQ_CHECK(hipMemcpyFromSymbol(clk.data(), HIP_SYMBOL(g_lq_clk), clk.size() * 8));
        double cyc = 0, rt = 0;
        for (int i = 0; i < grid; i++) { cyc += clk[2 * i]; rt += clk[2 * i + 1]; }
        printf("    clock %.3f GHz\n", cyc / rt * 0.1);
    }
    return 0;
}
