// k_fft.hip -- transforms of any size for the public FFT plan API
// (include/liquid.h:1122-1216, src/fft/src/fft_common.c) and spgram.
//
//   n = 2^k <= 4096      : register/LDS Stockham kernel (lqk_fft_batch)
//   n = 2^k  > 4096      : four-step n = n1 n2 -- transpose, n2 FFTs of n1,
//                          twiddle-transpose, n1 FFTs of n2, transpose
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
constexpr int TT = 32;   // transpose tile

__device__ __forceinline__ float2 tw_exp(long long num, long long den, int dir)
{
    // exp(-2 pi i dir num / den), num reduced mod den
    double s, c;
    sincospi(-2.0 * dir * (double)(num % den) / (double)den, &s, &c);
    return make_float2((float)c, (float)s);
}

// out[c*R + r] = in[r*C + c] (* W_N^(r*c) when N > 0), per transform z
__global__ __launch_bounds__(TT * 8) void k_transpose(const float2 *__restrict__ in, float2 *__restrict__ out, int R,
                                                      int C, long long N, int dir)
{
    __shared__ float2 t[TT][TT + 1];
    const long long off = (long long)blockIdx.z * R * C;
    const int c0 = blockIdx.x * TT, r0 = blockIdx.y * TT;
    for (int k = threadIdx.y; k < TT; k += 8) {
        const int r = r0 + k, c = c0 + threadIdx.x;
        if (r < R && c < C) {
            float2 v = in[off + (long long)r * C + c];
            if (N > 0) v = cmul(v, tw_exp((long long)r * c, N, dir));
            t[k][threadIdx.x] = v;
        }
    }
    __syncthreads();
    for (int k = threadIdx.y; k < TT; k += 8) {
        const int c = c0 + k, r = r0 + threadIdx.x;
        if (r < R && c < C) out[off + (long long)c * R + r] = t[threadIdx.x][k];
    }
}

void transpose(const void *in, void *out, int R, int C, long long batch, long long N, int dir, hipStream_t st)
{
    const dim3 grid((C + TT - 1) / TT, (R + TT - 1) / TT, (unsigned)batch);
    hipLaunchKernelGGL(k_transpose, grid, dim3(TT, 8), 0, st, (const float2 *)in, (float2 *)out, R, C, N, dir);
    LQ_CHECK_LAUNCH();
}

// power-of-two n > 4096: four-step through `work` (n * batch samples); x may alias y
void fft_four_step(unsigned n, int dir, const void *x, void *y, long long batch, void *work, hipStream_t st)
{
    unsigned lg = 0;
    while ((1u << lg) < n) lg++;
    const int n1 = 1 << ((lg + 1) / 2), n2 = (int)(n / (unsigned)n1);
    // x as n1 rows x n2 cols -> A: n2 rows of n1
    transpose(x, work, n1, n2, batch, 0, dir, st);
    lqk_fft_batch((unsigned)n1, dir, work, work, (unsigned long long)batch * n2, st);
    // B[j2][k1] * W_n^(j2 k1) -> C: n1 rows of n2
    transpose(work, y, n2, n1, batch, (long long)n, dir, st);
    lqk_fft_batch((unsigned)n2, dir, y, y, (unsigned long long)batch * n1, st);
    // D[k1][k2] -> y[k2*n1 + k1]
    transpose(y, work, n1, n2, batch, 0, dir, st);
    LQ_CHECK(hipMemcpyAsync(y, work, (size_t)n * batch * sizeof(float2), hipMemcpyDeviceToDevice, st));
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

// b[j] = conj(c[j]) circularly on M points (|j| < n)
__global__ void k_bs_kernel(long long n, long long M, int dir, float2 *__restrict__ b)
{
    const long long j = (long long)blockIdx.x * NT + threadIdx.x;
    if (j >= M) return;
    float2 v = make_float2(0.f, 0.f);
    if (j < n) v = chirp(j, n, dir);
    else if (j > M - n) v = chirp(M - j, n, dir);
    b[j] = make_float2(v.x, -v.y);
}

__global__ void k_bs_pre(const float2 *__restrict__ x, float2 *__restrict__ a, long long n, long long M, int dir)
{
    const long long e = (long long)blockIdx.x * NT + threadIdx.x;
    const long long z = blockIdx.y;
    if (e >= M) return;
    a[z * M + e] = e < n ? cmul(x[z * n + e], chirp(e, n, dir)) : make_float2(0.f, 0.f);
}

__global__ void k_bs_mul(float2 *__restrict__ a, const float2 *__restrict__ B, long long M)
{
    const long long e = (long long)blockIdx.x * NT + threadIdx.x;
    if (e >= M) return;
    const long long z = blockIdx.y;
    a[z * M + e] = cmul(a[z * M + e], B[e]);
}

__global__ void k_bs_post(const float2 *__restrict__ a, float2 *__restrict__ y, long long n, long long M, int dir)
{
    const long long k = (long long)blockIdx.x * NT + threadIdx.x;
    const long long z = blockIdx.y;
    if (k >= n) return;
    const float inv = 1.0f / (float)M;
    y[z * n + k] = cscale(cmul(a[z * M + k], chirp(k, n, dir)), inv);
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
    // a: M per transform, B: M, four-step scratch for M
    return (size_t)(M * batch + M + (M > 4096 ? M * batch : 0)) * sizeof(float2);
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
    // chirp transform (cached by the caller through lqk_fft_plan when repeated; cheap relative to n log n)
    hipLaunchKernelGGL(k_bs_kernel, dim3((unsigned)((M + NT - 1) / NT)), dim3(NT), 0, st, (long long)n, M, dir, B);
    LQ_CHECK_LAUNCH();
    fft_pow2((unsigned)M, +1, B, B, 1, w4, st);
    const dim3 gM((unsigned)((M + NT - 1) / NT), (unsigned)batch);
    hipLaunchKernelGGL(k_bs_pre, gM, dim3(NT), 0, st, (const float2 *)x, a, (long long)n, M, dir);
    LQ_CHECK_LAUNCH();
    fft_pow2((unsigned)M, +1, a, a, (long long)batch, w4, st);
    hipLaunchKernelGGL(k_bs_mul, gM, dim3(NT), 0, st, a, (const float2 *)B, M);
    LQ_CHECK_LAUNCH();
    fft_pow2((unsigned)M, -1, a, a, (long long)batch, w4, st);
    const dim3 gn((unsigned)((n + NT - 1) / NT), (unsigned)batch);
    hipLaunchKernelGGL(k_bs_post, gn, dim3(NT), 0, st, (const float2 *)a, (float2 *)y, (long long)n, M, dir);
    LQ_CHECK_LAUNCH();
}

extern "C" void lqk_fft_r2r(int type, unsigned int n, const void *x, void *y, unsigned long long batch, void *stream)
{
    if (batch == 0 || n == 0) return;
    const dim3 g((n + NT - 1) / NT, (unsigned)batch);
    hipLaunchKernelGGL(k_r2r, g, dim3(NT), 0, (hipStream_t)stream, type, (int)n, (const float *)x, (float *)y);
    LQ_CHECK_LAUNCH();
}
