// k_fft.hip -- transforms of any size for the public FFT plan API
// (include/liquid.h:1122-1216, src/fft/src/fft_common.c) and spgram.
//
//   n = 2^k <= 4096      : register/LDS Stockham kernel (lqk_fft_batch)
//   n = 2^k  > 4096      : two passes n = N1 N2 -- column transforms with the
//                          twiddle, then row transforms written transposed
//   other n <= 16        : direct DFT (lqk_fft_batch)
//   other n              : Bluestein chirp-z over a power-of-two M >= 2n-1
//                          (the chirp's FFT is computed once per plan)
//   real-to-real (DCT/DST I-IV, fft_r2r_1d.c:95-250): direct sums, one lane
//                          per output, twiddle phase reduced exactly in integers
// Twiddles and chirps are evaluated in double from exact integer phases.
#include <hip/hip_runtime.h>

#include "lq_device.h"
#include "lq_kernels.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float2 tw_exp(long long num, long long den, int dir)
{
    // exp(-2 pi i dir num / den), num reduced mod den
    double s, c;
    sincospi(-2.0 * dir * (double)(num % den) / (double)den, &s, &c);
    return make_float2((float)c, (float)s);
}

// power-of-two n > 4096 in two passes (n = N1 N2, x as N1 rows of N2):
//   A: the N2 columns' N1-point transforms, G columns per workgroup (G N1 =
//      4096 samples in LDS, rows of G consecutive samples loaded), times
//      W_n^(j2 k1), written back in place to `work`;
//   B: the N1 rows' N2-point transforms, G rows per workgroup, written
//      transposed: y[k1 + N1 k2] (G consecutive outputs per k2).
// 32 bytes of HBM traffic per point instead of the six passes of a
// transpose-based four-step.  x may alias y.
template <int N1>
__global__ __launch_bounds__(NT) void k_fft2p_cols(const float2 *__restrict__ x, float2 *__restrict__ work, long long n,
                                                   int N2, int dir, const float2 *__restrict__ tw)
{
    constexpr int G = 4096 / N1;
    __shared__ __attribute__((aligned(16))) float2 a[4096];
    __shared__ __attribute__((aligned(16))) float2 b[4096];
    const long long off = (long long)blockIdx.z * n;
    const int j20 = blockIdx.x * G;
    for (int e = threadIdx.x; e < 4096; e += NT) {
        const int j1 = e / G, g = e - j1 * G;
        a[g * N1 + j1] = x[off + (long long)N2 * j1 + j20 + g];
    }
    __syncthreads();
    const float2 *F = lds_fft<N1, G, NT>(a, b, tw, dir);
    for (int e = threadIdx.x; e < 4096; e += NT) {
        const int k1 = e / G, g = e - k1 * G;
        const float2 v = cmul(F[g * N1 + k1], tw_exp((long long)(j20 + g) * k1, n, dir));
        work[off + (long long)N2 * k1 + j20 + g] = v;
    }
}

template <int N2>
__global__ __launch_bounds__(NT) void k_fft2p_rows(const float2 *__restrict__ work, float2 *__restrict__ y, long long n,
                                                   int N1, int dir, const float2 *__restrict__ tw)
{
    constexpr int G = 4096 / N2;
    __shared__ __attribute__((aligned(16))) float2 a[4096];
    __shared__ __attribute__((aligned(16))) float2 b[4096];
    const long long off = (long long)blockIdx.z * n;
    const int k10 = blockIdx.x * G;
    for (int e = threadIdx.x; e < 4096; e += NT) a[e] = work[off + (long long)N2 * k10 + e];
    __syncthreads();
    const float2 *F = lds_fft<N2, G, NT>(a, b, tw, dir);
    for (int e = threadIdx.x; e < 4096; e += NT) {
        const int k2 = e / G, g = e - k2 * G;
        y[off + k10 + g + (long long)N1 * k2] = F[g * N2 + k2];
    }
}

// Register forms of both passes for N1 / N2 = 256 R (R = 1, 2, 4, 8, 16):
// the transforms run in registers (fft_r16x16xR, 16 R threads each, 16 / R
// per workgroup) instead of the LDS Stockham passes.  Consecutive threads
// take consecutive columns (pass A) / rows (pass B), so the column loads and
// stores of pass A and the transposed stores of pass B move G consecutive
// samples per instruction and lane group.
template <int R, int DIR>
__global__ __launch_bounds__(NT) void k_fft2p_cols_r(const float2 *__restrict__ x, float2 *__restrict__ work,
                                                     long long n, int N2, const float2 *__restrict__ tw)
{
    constexpr int T = 16 * R, G = 256 / T, P = FFTR16_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 lds[G * P];
    const long long off = (long long)blockIdx.z * n;
    const int g = threadIdx.x % G, t = threadIdx.x / G;
    const int j2 = blockIdx.x * G + g;
    const tw16x2 w16 = fftr16_tw<R>(tw, t);   // issued before the data loads
    float2 v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) v[q] = x[off + (long long)N2 * (t + T * q) + j2];
    fft_r16x16xR<R, DIR>(v, lds + g * P, w16, t);
#pragma unroll
    for (int s = 0; s < 16 / R; s++)
#pragma unroll
        for (int q = 0; q < R; q++) {
            const int k1 = t + T * s + 256 * q;
            work[off + (long long)N2 * k1 + j2] = cmul(v[s * R + q], tw_exp((long long)j2 * k1, n, DIR));
        }
}

template <int R, int DIR>
__global__ __launch_bounds__(NT) void k_fft2p_rows_r(const float2 *__restrict__ work, float2 *__restrict__ y,
                                                     long long n, int N1, const float2 *__restrict__ tw)
{
    constexpr int T = 16 * R, N2 = 16 * T, G = 256 / T, P = FFTR16_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 lds[G * P];
    const long long off = (long long)blockIdx.z * n;
    const int g = threadIdx.x % G, t = threadIdx.x / G;
    const int k1 = blockIdx.x * G + g;
    const tw16x2 w16 = fftr16_tw<R>(tw, t);
    float2 v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) v[q] = work[off + (long long)N2 * k1 + t + T * q];
    fft_r16x16xR<R, DIR>(v, lds + g * P, w16, t);
#pragma unroll
    for (int s = 0; s < 16 / R; s++)
#pragma unroll
        for (int q = 0; q < R; q++) y[off + k1 + (long long)N1 * (t + T * s + 256 * q)] = v[s * R + q];
}

template <int R>
void launch_cols_r(const void *x, void *work, long long n, int N2, int dir, long long batch, hipStream_t st)
{
    const dim3 g((unsigned)(N2 / (16 / R)), 1, (unsigned)batch);
    if (dir > 0)
        hipLaunchKernelGGL((k_fft2p_cols_r<R, +1>), g, dim3(NT), 0, st, (const float2 *)x, (float2 *)work, n, N2,
                           (const float2 *)lqrt_twiddles());
    else
        hipLaunchKernelGGL((k_fft2p_cols_r<R, -1>), g, dim3(NT), 0, st, (const float2 *)x, (float2 *)work, n, N2,
                           (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}
template <int R>
void launch_rows_r(const void *work, void *y, long long n, int N1, int dir, long long batch, hipStream_t st)
{
    const dim3 g((unsigned)(N1 / (16 / R)), 1, (unsigned)batch);
    if (dir > 0)
        hipLaunchKernelGGL((k_fft2p_rows_r<R, +1>), g, dim3(NT), 0, st, (const float2 *)work, (float2 *)y, n, N1,
                           (const float2 *)lqrt_twiddles());
    else
        hipLaunchKernelGGL((k_fft2p_rows_r<R, -1>), g, dim3(NT), 0, st, (const float2 *)work, (float2 *)y, n, N1,
                           (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}

template <int N>
void launch_cols(const void *x, void *work, long long n, int N2, int dir, long long batch, hipStream_t st)
{
    const dim3 g((unsigned)(N2 / (4096 / N)), 1, (unsigned)batch);
    hipLaunchKernelGGL(k_fft2p_cols<N>, g, dim3(NT), 0, st, (const float2 *)x, (float2 *)work, n, N2, dir,
                       (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}
template <int N>
void launch_rows(const void *work, void *y, long long n, int N1, int dir, long long batch, hipStream_t st)
{
    const dim3 g((unsigned)(N1 / (4096 / N)), 1, (unsigned)batch);
    hipLaunchKernelGGL(k_fft2p_rows<N>, g, dim3(NT), 0, st, (const float2 *)work, (float2 *)y, n, N1, dir,
                       (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}

void fft_four_step(unsigned n, int dir, const void *x, void *y, long long batch, void *work, hipStream_t st)
{
    unsigned lg = 0;
    while ((1u << lg) < n) lg++;
    // the larger factor on the column pass (N2 <= N1 <= 4096 for n <= 2^24): for odd lg the
    // 2^k-point column transforms with the double-precision twiddle run in registers
    const int N1 = 1 << ((lg + 1) / 2), N2 = (int)(n / (unsigned)N1);
    switch (N1) {
    case 64: launch_cols<64>(x, work, n, N2, dir, batch, st); break;
    case 128: launch_cols<128>(x, work, n, N2, dir, batch, st); break;
    case 256: launch_cols_r<1>(x, work, n, N2, dir, batch, st); break;
    case 512: launch_cols_r<2>(x, work, n, N2, dir, batch, st); break;
    case 1024: launch_cols_r<4>(x, work, n, N2, dir, batch, st); break;
    case 2048: launch_cols_r<8>(x, work, n, N2, dir, batch, st); break;
    default: launch_cols_r<16>(x, work, n, N2, dir, batch, st); break;
    }
    switch (N2) {
    case 64: launch_rows<64>(work, y, n, N1, dir, batch, st); break;
    case 128: launch_rows<128>(work, y, n, N1, dir, batch, st); break;
    case 256: launch_rows_r<1>(work, y, n, N1, dir, batch, st); break;
    case 512: launch_rows_r<2>(work, y, n, N1, dir, batch, st); break;
    case 1024: launch_rows_r<4>(work, y, n, N1, dir, batch, st); break;
    case 2048: launch_rows_r<8>(work, y, n, N1, dir, batch, st); break;
    default: launch_rows_r<16>(work, y, n, N1, dir, batch, st); break;
    }
}

void fft_pow2(unsigned n, int dir, const void *x, void *y, long long batch, void *work, hipStream_t st)
{
    if (n <= 4096) lqk_fft_batch(n, dir, x, y, (unsigned long long)batch, st);
    else fft_four_step(n, dir, x, y, batch, work, st);
}

// chirp c[j] = exp(-i pi dir j^2 / n), phase reduced mod 2n exactly
__device__ __forceinline__ float2 chirp(long long j, long long n, int dir)
{
    const long long p = (j * j) % (2 * n);
    double s, c;
    sincospi(-(double)dir * (double)p / (double)n, &s, &c);
    return make_float2((float)c, (float)s);
}

// the chirp table c[j], j < n, once per call (double phases, rounded once)
__global__ void k_bs_chirp(long long n, int dir, float2 *__restrict__ c)
{
    const long long j = (long long)blockIdx.x * NT + threadIdx.x;
    if (j < n) c[j] = chirp(j, n, dir);
}

// b[j] = conj(c[j]) circularly on M points (|j| < n)
__global__ void k_bs_kernel(long long n, long long M, const float2 *__restrict__ c, float2 *__restrict__ b)
{
    const long long j = (long long)blockIdx.x * NT + threadIdx.x;
    if (j >= M) return;
    float2 v = make_float2(0.f, 0.f);
    if (j < n) v = c[j];
    else if (j > M - n) v = c[M - j];
    b[j] = make_float2(v.x, -v.y);
}

__global__ void k_bs_pre(const float2 *__restrict__ x, float2 *__restrict__ a, long long n, long long M,
                         const float2 *__restrict__ c)
{
    const long long e = (long long)blockIdx.x * NT + threadIdx.x;
    const long long z = blockIdx.y;
    if (e >= M) return;
    a[z * M + e] = e < n ? cmul(x[z * n + e], c[e]) : make_float2(0.f, 0.f);
}

__global__ void k_bs_mul(float2 *__restrict__ a, const float2 *__restrict__ B, long long M)
{
    const long long e = (long long)blockIdx.x * NT + threadIdx.x;
    if (e >= M) return;
    const long long z = blockIdx.y;
    a[z * M + e] = cmul(a[z * M + e], B[e]);
}

__global__ void k_bs_post(const float2 *__restrict__ a, float2 *__restrict__ y, long long n, long long M,
                          const float2 *__restrict__ c)
{
    const long long k = (long long)blockIdx.x * NT + threadIdx.x;
    const long long z = blockIdx.y;
    if (k >= n) return;
    const float inv = 1.0f / (float)M;
    y[z * n + k] = cscale(cmul(a[z * M + k], c[k]), inv);
}

// real-to-real transforms: fft_r2r_1d.c:95-250 (un-normalised, factor 2)
__global__ void k_r2r(int type, int n, const float *__restrict__ x, float *__restrict__ y)
{
    const int i = blockIdx.x * NT + threadIdx.x;
    const long long z = blockIdx.y;
    if (i >= n) return;
    const float *xs = x + z * n;
    // phases pi*num/den with the integer numerator reduced modulo one period
    double acc = 0.0;
    switch (type) {
    case LQK_R2R_REDFT00: {   // DCT-I: 0.5(x0 + (-1)^i x_{n-1}) + sum_{k=1}^{n-2} x_k cos(pi k i/(n-1))
        acc = 0.5 * ((double)xs[0] + ((i & 1) ? -(double)xs[n - 1] : (double)xs[n - 1]));
        const long long den = 2LL * (n - 1);
        for (int k = 1; k < n - 1; k++) acc += (double)xs[k] * cospi((double)(((long long)k * i) % den) / (n - 1));
        break;
    }
    case LQK_R2R_REDFT10:     // DCT-II: sum x_k cos(pi (k+1/2) i / n)
        for (int k = 0; k < n; k++)
            acc += (double)xs[k] * cospi((double)(((2LL * k + 1) * i) % (4LL * n)) / (2.0 * n));
        break;
    case LQK_R2R_REDFT01:     // DCT-III: 0.5 x_0 + sum_{k>=1} x_k cos(pi (i+1/2) k / n)
        acc = 0.5 * (double)xs[0];
        for (int k = 1; k < n; k++)
            acc += (double)xs[k] * cospi((double)(((2LL * i + 1) * k) % (4LL * n)) / (2.0 * n));
        break;
    case LQK_R2R_REDFT11:     // DCT-IV: sum x_k cos(pi (k+1/2)(i+1/2)/n)
        for (int k = 0; k < n; k++)
            acc += (double)xs[k] * cospi((double)(((2LL * k + 1) * (2LL * i + 1)) % (8LL * n)) / (4.0 * n));
        break;
    case LQK_R2R_RODFT00:     // DST-I: sum x_k sin(pi (k+1)(i+1)/(n+1))
        for (int k = 0; k < n; k++)
            acc += (double)xs[k] * sinpi((double)(((long long)(k + 1) * (i + 1)) % (2LL * (n + 1))) / (n + 1));
        break;
    case LQK_R2R_RODFT10:     // DST-II: sum x_k sin(pi (k+1/2)(i+1)/n)
        for (int k = 0; k < n; k++)
            acc += (double)xs[k] * sinpi((double)(((2LL * k + 1) * (i + 1)) % (4LL * n)) / (2.0 * n));
        break;
    case LQK_R2R_RODFT01:     // DST-III: +-0.5 x_{n-1} + sum_{k<n-1} x_k sin(pi (k+1)(i+1/2)/n)
        acc = ((i & 1) ? -0.5 : 0.5) * (double)xs[n - 1];
        for (int k = 0; k < n - 1; k++)
            acc += (double)xs[k] * sinpi((double)(((long long)(k + 1) * (2LL * i + 1)) % (4LL * n)) / (2.0 * n));
        break;
    default:                  // DST-IV: sum x_k sin(pi (k+1/2)(i+1/2)/n)
        for (int k = 0; k < n; k++)
            acc += (double)xs[k] * sinpi((double)(((2LL * k + 1) * (2LL * i + 1)) % (8LL * n)) / (4.0 * n));
    }
    y[z * n + i] = (float)(2.0 * acc);
}

} // namespace

extern "C" size_t lqk_fft_work_bytes(unsigned int n, unsigned long long batch)
{
    if (n <= 4096 && (n & (n - 1)) == 0) return 0;
    if ((n & (n - 1)) == 0) return (size_t)n * batch * sizeof(float2);
    if (n <= 16) return 0;
    unsigned long long M = 1;
    while (M < 2ull * n - 1) M <<= 1;
    // a: M per transform, B: M, four-step scratch for M, the n-entry chirp table
    return (size_t)(M * batch + M + (M > 4096 ? M * batch : 0) + n) * sizeof(float2);
}

extern "C" void lqk_fft_any(unsigned int n, int dir, const void *x, void *y, unsigned long long batch, void *work,
                            void *stream)
{
    if (batch == 0 || n == 0) return;
    hipStream_t st = (hipStream_t)stream;
    const bool pow2 = (n & (n - 1)) == 0;
    if ((pow2 && n > (1u << 24)) || (!pow2 && n > (1u << 23))) {
        fprintf(stderr, "error: liquid-mi355x: transform size %u exceeds the GPU FFT limit (2^24, 2^23 non power of two)\n", n);
        exit(1);
    }
    if (pow2) {
        fft_pow2(n, dir, x, y, (long long)batch, work, st);
        return;
    }
    if (n <= 16) {
        lqk_fft_batch(n, dir, x, y, batch, st);
        return;
    }
    long long M = 1;
    while (M < 2LL * n - 1) M <<= 1;
    float2 *a = (float2 *)work;
    float2 *B = a + M * (long long)batch;
    float2 *w4 = B + M;
    float2 *ct = w4 + (M > 4096 ? M * (long long)batch : 0);
    hipLaunchKernelGGL(k_bs_chirp, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, st, (long long)n, dir, ct);
    LQ_CHECK_LAUNCH();
    // chirp transform (once per call; cheap relative to the batch's n log n)
    hipLaunchKernelGGL(k_bs_kernel, dim3((unsigned)((M + NT - 1) / NT)), dim3(NT), 0, st, (long long)n, M,
                       (const float2 *)ct, B);
    LQ_CHECK_LAUNCH();
    fft_pow2((unsigned)M, +1, B, B, 1, w4, st);
    const dim3 gM((unsigned)((M + NT - 1) / NT), (unsigned)batch);
    hipLaunchKernelGGL(k_bs_pre, gM, dim3(NT), 0, st, (const float2 *)x, a, (long long)n, M, (const float2 *)ct);
    LQ_CHECK_LAUNCH();
    fft_pow2((unsigned)M, +1, a, a, (long long)batch, w4, st);
    hipLaunchKernelGGL(k_bs_mul, gM, dim3(NT), 0, st, a, (const float2 *)B, M);
    LQ_CHECK_LAUNCH();
    fft_pow2((unsigned)M, -1, a, a, (long long)batch, w4, st);
    const dim3 gn((unsigned)((n + NT - 1) / NT), (unsigned)batch);
    hipLaunchKernelGGL(k_bs_post, gn, dim3(NT), 0, st, (const float2 *)a, (float2 *)y, (long long)n, M,
                       (const float2 *)ct);
    LQ_CHECK_LAUNCH();
}

extern "C" void lqk_fft_r2r(int type, unsigned int n, const void *x, void *y, unsigned long long batch, void *stream)
{
    if (batch == 0 || n == 0) return;
    const dim3 g((n + NT - 1) / NT, (unsigned)batch);
    hipLaunchKernelGGL(k_r2r, g, dim3(NT), 0, (hipStream_t)stream, type, (int)n, (const float *)x, (float *)y);
    LQ_CHECK_LAUNCH();
}
