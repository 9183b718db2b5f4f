// k_spgram.hip -- spectral periodogram (spgramcf / spgramf,
// src/fft/src/spgram.c) as batched windowed transforms.
//
// A block of input produces T transforms at known positions (every W/2
// samples for accumulate_psd, every nfft/4 and at the end for estimate_psd);
// their windows are gathered from [history | block] into a T x nfft batch,
// transformed together (csrc/k_fft.hip), then reduced per bin: the
// exponential average runs the reference's recursion in transform order, the
// estimate sums |X|^2.
#include <hip/hip_runtime.h>

#include "lq_device.h"
#include "lq_kernels.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float2 as_c(float v) { return make_float2(v, 0.0f); }
__device__ __forceinline__ float2 as_c(float2 v) { return v; }

// out[t][i] = ext[e_t + 1 + i] * w[i] (i < W), 0 (W <= i < nfft); ext = hist(W) ++ x
template <typename S>
__global__ __launch_bounds__(NT) void k_spg_gather(const S *__restrict__ hist, int W, const S *__restrict__ x,
                                                   const long long *__restrict__ ends, const float *__restrict__ w,
                                                   int nfft, float2 *__restrict__ out)
{
    const int i = blockIdx.x * NT + threadIdx.x;
    const long long t = blockIdx.y;
    if (i >= nfft) return;
    float2 v = make_float2(0.f, 0.f);
    if (i < W) {
        const long long j = ends[t] + 1 + i;
        const float2 s = as_c(j < W ? hist[j] : x[j - W]);
        v = make_float2(s.x * w[i], s.y * w[i]);
    }
    out[t * nfft + i] = v;
}

__device__ __forceinline__ float pwr(float2 v)
{
#pragma clang fp contract(off)
    return v.x * v.x + v.y * v.y;   // crealf(X * conjf(X))
}

// psd[k] = (1 - a) psd[k] + a |X_t[k]|^2 for t = 0..T-1 in order (spgram.c:205-236)
__global__ __launch_bounds__(NT) void k_spg_accum(const float2 *__restrict__ X, long long T, int nfft, float alpha,
                                                  float *__restrict__ psd)
{
#pragma clang fp contract(off)
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k >= nfft) return;
    float p = psd[k];
    for (long long t = 0; t < T; t++) p = (1.0f - alpha) * p + alpha * pwr(X[t * nfft + k]);
    psd[k] = p;
}

// acc[(k + nfft/2) % nfft] += sum_t |X_t[k]|^2 (spgram.c:262-276)
__global__ __launch_bounds__(NT) void k_spg_sum(const float2 *__restrict__ X, long long T, int nfft,
                                                float *__restrict__ acc)
{
#pragma clang fp contract(off)
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k >= nfft) return;
    const int p = (k + nfft / 2) % nfft;
    float s = acc[p];
    for (long long t = 0; t < T; t++) s += pwr(X[t * nfft + k]);
    acc[p] = s;
}

// mode 0: out[(k+n/2)%n] = 10 log10(|X[k]|^2 + 1e-16)   (execute_psd)
// mode 1: out[(k+n/2)%n] = 10 log10(psd[k])               (write_accumulation)
// mode 2: out[k] = 10 log10(acc[k] / T)                   (estimate_psd, already shifted)
__global__ __launch_bounds__(NT) void k_spg_db(int mode, const float2 *__restrict__ X, const float *__restrict__ v,
                                               int nfft, float T, float *__restrict__ out)
{
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k >= nfft) return;
    const int p = (k + nfft / 2) % nfft;
    if (mode == 0) out[p] = 10.0f * log10f(pwr(X[k]) + 1e-16f);
    else if (mode == 1) out[p] = 10.0f * log10f(v[k]);
    else out[k] = 10.0f * log10f(v[k] / T);
}

} // namespace

extern "C" void lqk_spgram_gather(int real_in, const void *hist, unsigned int W, const void *x, const long long *ends,
                                  unsigned long long T, const float *w, unsigned int nfft, void *out, void *stream)
{
    if (T == 0) return;
    const dim3 g((nfft + NT - 1) / NT, (unsigned)T);
    if (real_in)
        hipLaunchKernelGGL(k_spg_gather<float>, g, dim3(NT), 0, (hipStream_t)stream, (const float *)hist, (int)W,
                           (const float *)x, ends, w, (int)nfft, (float2 *)out);
    else
        hipLaunchKernelGGL(k_spg_gather<float2>, g, dim3(NT), 0, (hipStream_t)stream, (const float2 *)hist, (int)W,
                           (const float2 *)x, ends, w, (int)nfft, (float2 *)out);
    LQ_CHECK_LAUNCH();
}

extern "C" void lqk_spgram_accumulate(const void *X, unsigned long long T, unsigned int nfft, float alpha, float *psd,
                                      void *stream)
{
    if (T == 0) return;
    hipLaunchKernelGGL(k_spg_accum, dim3((nfft + NT - 1) / NT), dim3(NT), 0, (hipStream_t)stream,
                       (const float2 *)X, (long long)T, (int)nfft, alpha, psd);
    LQ_CHECK_LAUNCH();
}

extern "C" void lqk_spgram_sum(const void *X, unsigned long long T, unsigned int nfft, float *acc, void *stream)
{
    if (T == 0) return;
    hipLaunchKernelGGL(k_spg_sum, dim3((nfft + NT - 1) / NT), dim3(NT), 0, (hipStream_t)stream, (const float2 *)X,
                       (long long)T, (int)nfft, acc);
    LQ_CHECK_LAUNCH();
}

extern "C" void lqk_spgram_db(int mode, const void *X, const float *v, unsigned int nfft, float T, float *out,
                              void *stream)
{
    hipLaunchKernelGGL(k_spg_db, dim3((nfft + NT - 1) / NT), dim3(NT), 0, (hipStream_t)stream, mode,
                       (const float2 *)X, v, (int)nfft, T, out);
    LQ_CHECK_LAUNCH();
}
