// k_fftfilt.hip -- FFT fast convolution for fftfilt_{crcf,rrrf,cccf}.
// Default kernel: k_fftfilt_r16 (register radix-16 transforms, persistent
// grid); k_fftfilt (LDS Stockham) is the earlier form, kept for comparison.
//
// Reference: src/filter/src/fftfilt.c:193-260 runs overlap-ADD with a 2n-point
// transform per n-sample call; its output is the causal linear convolution
// y = s * (h * x) (verified against the oracle, tests/test_oracle.py).  Because
// the result does not depend on the block geometry (up to rounding), the GPU
// path uses overlap-SAVE with one fixed 4096-point transform per workgroup:
// each workgroup loads 4096 inputs (its L = 4096 - (h-1) new samples plus the
// h-1 sample halo), runs forward FFT -> multiply by H -> inverse FFT entirely
// in LDS and writes its L outputs.  No state crosses workgroups, so every
// segment of a long stream runs in parallel; between calls only the last h-1
// inputs are carried.
#include "lq_device.h"
#include "lq_kernels.h"

#include <cstdio>
#include <type_traits>
#include <cstdlib>

namespace {

constexpr int NT = 256;
constexpr int NFFT = 4096;
// k_fftfilt_r16 configuration (tools/mb/mb_fftfilt.hip, h=512, 2^26 samples):
// with the packed transforms (lq_device.h) the kernel needs ~185 VGPRs (+32
// for the filter spectrum held in registers), so 2 waves/SIMD without spills;
// spectrum in registers, 2048 persistent workgroups: 0.283 ms (spectrum from
// L2 per segment: 0.36 ms; the scalar-complex transforms: 0.30 ms)
#ifndef FF_HREG
#define FF_HREG true
#define FF_WPE 2
#endif

// kind 0: real input/output (rrrf), otherwise complex
template <bool REAL>
__global__ __launch_bounds__(NT) void k_fftfilt(int hm1, const float2 *__restrict__ H, const void *__restrict__ hist,
                                                const void *__restrict__ xin, long long n, void *__restrict__ yout,
                                                float sre, float sim, const float2 *__restrict__ tw)
{
    __shared__ __attribute__((aligned(16))) float2 a[NFFT];
    __shared__ __attribute__((aligned(16))) float2 b[NFFT];
    const int L = NFFT - hm1;
    const long long s0 = (long long)blockIdx.x * L;
    for (int u = threadIdx.x; u < NFFT; u += NT) {
        const long long s = s0 - hm1 + u;
        float2 v = make_float2(0.f, 0.f);
        if (REAL) {
            const float *x = (const float *)xin;
            const float *hs = (const float *)hist;
            if (s < 0) v.x = hs[hm1 + s];
            else if (s < n) v.x = x[s];
        } else {
            const float2 *x = (const float2 *)xin;
            const float2 *hs = (const float2 *)hist;
            if (s < 0) v = hs[hm1 + s];
            else if (s < n) v = x[s];
        }
        a[u] = v;
    }
    __syncthreads();
    float2 *F = lds_fft<NFFT, 1, NT>(a, b, tw, +1);
    for (int u = threadIdx.x; u < NFFT; u += NT) F[u] = cmul(F[u], H[u]);
    __syncthreads();
    float2 *other = (F == a) ? b : a;
    float2 *T = lds_fft<NFFT, 1, NT>(F, other, tw, -1);
    for (int k = threadIdx.x; k < L; k += NT) {
        const long long t = s0 + k;
        if (t >= n) break;
        const float2 r = T[hm1 + k];
        if (REAL) {
            ((float *)yout)[t] = r.x * sre;
        } else {
            ((float2 *)yout)[t] = make_float2(r.x * sre - r.y * sim, r.x * sim + r.y * sre);
        }
    }
}

__device__ __forceinline__ float2 to_c2(float a) { return make_float2(a, 0.f); }
__device__ __forceinline__ float2 to_c2(float2 a) { return a; }

// Register form (default): 256 threads, thread t holds segment samples
// t + 256 n; forward 4096-point FFT (fft4096_r16), x H, inverse, all with the
// data in registers and two LDS transposes per transform (35 KB LDS; the
// register budget allows two workgroups per CU); loads and stores are
// coalesced across t.
template <bool REAL, bool HREG, int WPE>
__global__ __launch_bounds__(NT, WPE) void k_fftfilt_r16(int hm1, const float2 *__restrict__ H,
                                                    const void *__restrict__ hist, const void *__restrict__ xin,
                                                    long long n, void *__restrict__ yout, float sre, float sim,
                                                    const float2 *__restrict__ tw)
{
    __shared__ __attribute__((aligned(16))) float2 lds[FFT4096_LDS];
    const int L = NFFT - hm1;
    const int t = threadIdx.x;
    const long long nseg = (n + L - 1) / L;
    // persistent: the filter spectrum stays in registers across segments
    float2 hv[HREG ? 16 : 1];
    if (HREG) {
#pragma unroll
        for (int k = 0; k < 16; k++) hv[k] = H[t + 256 * k];
    }
    using S = typename std::conditional<REAL, float, float2>::type;
    for (long long seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    const long long s0 = seg * L;
    // segment sample i = t + 256 q is stream sample s0 - hm1 + i; 32-bit
    // indices relative to the segment start (the history only feeds seg 0)
    const long long rem = n - (s0 - hm1);              // segment samples that exist
    const int lim = rem < NFFT ? (int)rem : NFFT;
    float2 v[16];
    if (seg == 0) {
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int i = t + 256 * q, s = i - hm1;
            S a{};
            if (s < 0) a = ((const S *)hist)[hm1 + s];
            else if (i < lim) a = ((const S *)xin)[s];
            v[q] = to_c2(a);
        }
    } else {
        const S *xs = (const S *)xin + (s0 - hm1);
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int i = t + 256 * q;
            S a{};
            if (i < lim) a = xs[i];
            v[q] = to_c2(a);
        }
    }
    fft4096_r16<+1>(v, lds, tw, t);
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = unpk(pk_cmul(pk(v[k]), pk(HREG ? hv[k & (HREG ? 15 : 0)] : H[t + 256 * k])));
    fft4096_r16<-1>(v, lds, tw, t);
    S *ys = (S *)yout + (s0 - hm1);                    // output o = s0 + i - hm1 for i >= hm1
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int i = t + 256 * q;
        if (i < hm1 || i >= lim) continue;
        const float2 r = v[q];
        if constexpr (REAL) ys[i] = r.x * sre;
        else ys[i] = make_float2(r.x * sre - r.y * sim, r.x * sim + r.y * sre);
    }
    }
}

} // namespace

extern "C" void lqk_fftfilt_run(int real_io, unsigned int hlen, const void *H, const void *hist, const void *x,
                                unsigned long long n, void *y, float scale_re, float scale_im, void *stream)
{
    if (n == 0) return;
    if (hlen < 1 || hlen - 1 >= NFFT / 2 + 1) {
        fprintf(stderr, "error: fftfilt: filter length %u exceeds the GPU transform limit (%d)\n", hlen,
                NFFT / 2 + 1);
        exit(1);
    }
    hipStream_t st = (hipStream_t)stream;
    const int hm1 = (int)hlen - 1;
    const int L = NFFT - hm1;
    const long long nseg = ((long long)n + L - 1) / L;
    const float2 *tw = (const float2 *)lqrt_twiddles();
    const unsigned grid = (unsigned)(nseg < 2048 ? nseg : 2048);   // persistent, two resident per CU
    if (real_io)
        hipLaunchKernelGGL((k_fftfilt_r16<true, FF_HREG, FF_WPE>), dim3(grid), dim3(NT), 0, st, hm1, (const float2 *)H, hist,
                           x, (long long)n, y, scale_re, scale_im, tw);
    else
        hipLaunchKernelGGL((k_fftfilt_r16<false, FF_HREG, FF_WPE>), dim3(grid), dim3(NT), 0, st, hm1, (const float2 *)H, hist,
                           x, (long long)n, y, scale_re, scale_im, tw);
    LQ_CHECK_LAUNCH();
}

extern "C" unsigned int lqk_fftfilt_nfft(void) { return NFFT; }

// H[k] = FFT_4096(h zero padded)  (h real or complex), computed on the device
__global__ void k_pad_coef(const void *h, int hlen, int is_complex, float2 *buf)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NFFT) return;
    float2 v = make_float2(0.f, 0.f);
    if (i < hlen) v = is_complex ? ((const float2 *)h)[i] : make_float2(((const float *)h)[i], 0.f);
    buf[i] = v;
}

extern "C" void lqk_fftfilt_make_H(const void *h_dev, unsigned int hlen, int is_complex, void *H, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_pad_coef, dim3(NFFT / 256), dim3(256), 0, st, h_dev, (int)hlen, is_complex, (float2 *)H);
    LQ_CHECK_LAUNCH();
    lqk_fft_batch(NFFT, +1, H, H, 1, stream);
}
