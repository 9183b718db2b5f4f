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

#include <cstdio>
#include <cstdlib>

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

// W_M^e (e < M = 4096 2^sh) = W_4096^(e >> sh) W_M^(e & (2^sh - 1)): the shared
// 4096-entry table times a 2^sh-entry fine table computed per call in double
// (k_tw_fine), one float multiply -- a double-precision sincospi per point
// before
template <int DIR>
__device__ __forceinline__ float2 tw_split(long long e, int sh, const float2 *__restrict__ tw,
                                           const float2 *__restrict__ tfine)
{
    const float2 w = cmul(tw[(e >> sh) & 4095], tfine[e & ((1ll << sh) - 1)]);   // exp(-2 pi i e / M)
    return DIR > 0 ? w : make_float2(w.x, -w.y);
}

__global__ void k_tw_fine(int nf, long long M, float2 *__restrict__ f)
{
    const int b = blockIdx.x * NT + threadIdx.x;
    if (b < nf) f[b] = tw_exp(b, M, 1);
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
                                                   int N2, int dir, const float2 *__restrict__ tw,
                                                   const float2 *__restrict__ tfine, int sh)
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
        const long long ex = (long long)(j20 + g) * k1;
        const float2 v = cmul(F[g * N1 + k1], dir > 0 ? tw_split<1>(ex, sh, tw, tfine) : tw_split<-1>(ex, sh, tw, tfine));
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
                                                     long long n, int N2, const float2 *__restrict__ tw,
                                                     const float2 *__restrict__ tfine, int sh)
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
            work[off + (long long)N2 * k1 + j2] = cmul(v[s * R + q], tw_split<DIR>((long long)j2 * k1, sh, tw, tfine));
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
void launch_cols_r(const void *x, void *work, long long n, int N2, int dir, long long batch, const float2 *fine, int sh,
                   hipStream_t st)
{
    const dim3 g((unsigned)(N2 / (16 / R)), 1, (unsigned)batch);
    if (dir > 0)
        hipLaunchKernelGGL((k_fft2p_cols_r<R, +1>), g, dim3(NT), 0, st, (const float2 *)x, (float2 *)work, n, N2,
                           (const float2 *)lqrt_twiddles(), fine, sh);
    else
        hipLaunchKernelGGL((k_fft2p_cols_r<R, -1>), g, dim3(NT), 0, st, (const float2 *)x, (float2 *)work, n, N2,
                           (const float2 *)lqrt_twiddles(), fine, sh);
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
void launch_cols(const void *x, void *work, long long n, int N2, int dir, long long batch, const float2 *fine, int sh,
                 hipStream_t st)
{
    const dim3 g((unsigned)(N2 / (4096 / N)), 1, (unsigned)batch);
    hipLaunchKernelGGL(k_fft2p_cols<N>, g, dim3(NT), 0, st, (const float2 *)x, (float2 *)work, n, N2, dir,
                       (const float2 *)lqrt_twiddles(), fine, sh);
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

// the fine twiddle table for W_n, n = 4096 2^sh (tw_split)
const float2 *fine_table(unsigned long long n, float2 *buf, hipStream_t st)
{
    const int nf = (int)(n / 4096);
    hipLaunchKernelGGL(k_tw_fine, dim3((unsigned)((nf + NT - 1) / NT)), dim3(NT), 0, st, nf, (long long)n, buf);
    LQ_CHECK_LAUNCH();
    return buf;
}

int lg2(unsigned long long n)
{
    int lg = 0;
    while ((1ull << lg) < n) lg++;
    return lg;
}

template <int DIR, bool PRE>
void bs_cols(int N1, const float2 *src, float2 *work, long long n, long long M, int N2, const float2 *ct,
             const float2 *tfine, int sh, long long batch, hipStream_t st);
template <int DIR, int POST>
void bs_rows(int N2, const float2 *work, float2 *dst, long long n, long long M, int N1, const float2 *mulv, float inv,
             long long batch, hipStream_t st);

void fft_four_step(unsigned n, int dir, const void *x, void *y, long long batch, void *work, const float2 *fine,
                   hipStream_t st)
{
    const int lg = lg2(n), sh = lg - 12;
    // the larger factor on the column pass (N2 <= N1 <= 4096 for n <= 2^24): for odd lg the
    // 2^k-point column transforms with the twiddle run in registers
    const int N1 = 1 << ((lg + 1) / 2), N2 = (int)(n / (unsigned)N1);
    // n >= 32768 here (8192 and 16384 run in one pass): N1 >= 256; N2 = 128
    // (n = 32768) runs its row pass in registers (fft_small16xR, the
    // Bluestein split's kernel; with the LDS Stockham passes the four-step
    // n = 8192 took 1.15 ms per 2^26 points, with register passes 0.43)
    float2 *ws = (float2 *)work, *ys = (float2 *)y;
    switch (N1) {
    case 256: launch_cols_r<1>(x, work, n, N2, dir, batch, fine, sh, st); break;
    case 512: launch_cols_r<2>(x, work, n, N2, dir, batch, fine, sh, st); break;
    case 1024: launch_cols_r<4>(x, work, n, N2, dir, batch, fine, sh, st); break;
    case 2048: launch_cols_r<8>(x, work, n, N2, dir, batch, fine, sh, st); break;
    default: launch_cols_r<16>(x, work, n, N2, dir, batch, fine, sh, st); break;
    }
    switch (N2) {
    case 64:
    case 128:
        if (dir > 0) bs_rows<+1, 0>(N2, ws, ys, n, n, N1, nullptr, 1.0f, batch, st);
        else bs_rows<-1, 0>(N2, ws, ys, n, n, N1, nullptr, 1.0f, batch, st);
        break;
    case 256: launch_rows_r<1>(work, y, n, N1, dir, batch, st); break;
    case 512: launch_rows_r<2>(work, y, n, N1, dir, batch, st); break;
    case 1024: launch_rows_r<4>(work, y, n, N1, dir, batch, st); break;
    case 2048: launch_rows_r<8>(work, y, n, N1, dir, batch, st); break;
    default: launch_rows_r<16>(work, y, n, N1, dir, batch, st); break;
    }
}

// fine: the n / 4096-entry table of tw_split (n > 4096 only)
void fft_pow2(unsigned n, int dir, const void *x, void *y, long long batch, void *work, const float2 *fine,
              hipStream_t st)
{
    if (n <= 16384) lqk_fft_batch(n, dir, x, y, (unsigned long long)batch, st);   // 8192, 16384: one pass
    else fft_four_step(n, dir, x, y, batch, work, fine, st);
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

// ---------------------------------------------------------------- Bluestein, M > 4096
// The convolution's two M-point transforms run as the two-pass split above
// with the chirp and spectrum products fused into their loads and stores:
//   P1 columns, forward:  a = x c (zero padded to M) loaded, N1-point
//                          transforms, x W_M^(j2 k1) -> work
//   P2 rows, forward:     N2-point transforms, x B[k] at the natural output
//                          index k = k1 + N1 k2 -> a
//   P3 columns, inverse:  a -> N1-point inverse transforms, x W_M^-(j2 k1)
//                          -> work
//   P4 rows, inverse:     N2-point inverse transforms, y[k] = v c[k] / M for
//                          k < n
// 4 passes (48 M + 16 n bytes per transform) instead of chirp, two-pass,
// spectrum, two-pass, chirp (104 M + 16 n); twiddles from tw_split.


// columns, register transforms (N1 = 256 R): PRE loads x c, else src[M]
template <int R, int DIR, bool PRE>
__global__ __launch_bounds__(NT) void k_bs_cols_r(const float2 *__restrict__ src, float2 *__restrict__ work,
                                                  long long n, long long M, int N2, const float2 *__restrict__ ct,
                                                  const float2 *__restrict__ tw, const float2 *__restrict__ tfine,
                                                  int sh)
{
    constexpr int T = 16 * R, G = 256 / T, P = FFTR16_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 lds[G * P];
    const long long z = blockIdx.z;
    const int g = threadIdx.x % G, t = threadIdx.x / G;
    const int j2 = blockIdx.x * G + g;
    const tw16x2 w16 = fftr16_tw<R>(tw, t);
    float2 v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const long long e = (long long)N2 * (t + T * q) + j2;
        if (PRE) v[q] = e < n ? cmul(src[z * n + e], ct[e]) : make_float2(0.f, 0.f);
        else v[q] = src[z * M + e];
    }
    fft_r16x16xR<R, DIR>(v, lds + g * P, w16, t);
#pragma unroll
    for (int s = 0; s < 16 / R; s++)
#pragma unroll
        for (int q = 0; q < R; q++) {
            const int k1 = t + T * s + 256 * q;
            work[z * M + (long long)N2 * k1 + j2] = cmul(v[s * R + q], tw_split<DIR>((long long)j2 * k1, sh, tw, tfine));
        }
}

// rows, register transforms (N2 = 256 R): POST 1 -> dst[M] = v B[k]; POST 2 ->
// y[k] = v c[k] inv for k < n
template <int R, int DIR, int POST>
__global__ __launch_bounds__(NT) void k_bs_rows_r(const float2 *__restrict__ work, float2 *__restrict__ dst,
                                                  long long n, long long M, int N1, const float2 *__restrict__ mulv,
                                                  float inv, const float2 *__restrict__ tw)
{
    constexpr int T = 16 * R, N2 = 16 * T, G = 256 / T, P = FFTR16_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 lds[G * P];
    const long long z = blockIdx.z;
    const int g = threadIdx.x % G, t = threadIdx.x / G;
    const int k1 = blockIdx.x * G + g;
    const tw16x2 w16 = fftr16_tw<R>(tw, t);
    float2 v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) v[q] = work[z * M + (long long)N2 * k1 + t + T * q];
    fft_r16x16xR<R, DIR>(v, lds + g * P, w16, t);
#pragma unroll
    for (int s = 0; s < 16 / R; s++)
#pragma unroll
        for (int q = 0; q < R; q++) {
            const long long k = k1 + (long long)N1 * (t + T * s + 256 * q);
            if (POST == 1) dst[z * M + k] = cmul(v[s * R + q], mulv[k]);
            else if (k < n) dst[z * n + k] = cscale(cmul(v[s * R + q], mulv[k]), inv);
        }
}

// columns / rows of N = 16 R points (R = 2, 4, 8: 32 .. 128) in registers
// (fft_small16xR, R lanes per transform; the rows' transposed stores staged
// through LDS so they run along k1)
template <int R, int DIR, bool PRE>
__global__ __launch_bounds__(NT) void k_bs_cols_s(const float2 *__restrict__ src, float2 *__restrict__ work,
                                                  long long n, long long M, int N2, const float2 *__restrict__ ct,
                                                  const float2 *__restrict__ tw, const float2 *__restrict__ tfine,
                                                  int sh)
{
    constexpr int N = 16 * R, G = 256 / R, PS = FFTS_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 lds[G * PS];
    const long long z = blockIdx.z;
    const int g = threadIdx.x % G, t = threadIdx.x / G;   // consecutive threads: consecutive columns
    const int j2 = blockIdx.x * G + g;
    const int e1 = t * (4096 / N);
    const float2 a1 = tw[e1 & 4095], a4 = tw[(4 * e1) & 4095];
    float2 v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const long long e = (long long)N2 * (t + R * q) + j2;
        if (PRE) v[q] = e < n ? cmul(src[z * n + e], ct[e]) : make_float2(0.f, 0.f);
        else v[q] = src[z * M + e];
    }
    fft_small16xR<R, DIR>(v, lds + g * PS, a1, a4, t);
#pragma unroll
    for (int u = 0; u < 16 / R; u++)
#pragma unroll
        for (int q = 0; q < R; q++) {
            const int k1 = t * (16 / R) + u + 16 * q;
            work[z * M + (long long)N2 * k1 + j2] = cmul(v[u * R + q], tw_split<DIR>((long long)j2 * k1, sh, tw, tfine));
        }
}

template <int R, int DIR, int POST>
__global__ __launch_bounds__(NT) void k_bs_rows_s(const float2 *__restrict__ work, float2 *__restrict__ dst,
                                                  long long n, long long M, int N1, const float2 *__restrict__ mulv,
                                                  float inv, const float2 *__restrict__ tw)
{
    constexpr int N2 = 16 * R, G = 256 / R, PS = FFTS_LDS<R>();
    static_assert(G * PS >= G * N2, "staging fits the transform scratch");
    __shared__ __attribute__((aligned(16))) float2 lds[G * PS];
    const long long z = blockIdx.z;
    const int t = threadIdx.x % R, g = threadIdx.x / R;   // consecutive threads: along a row
    const int k10 = blockIdx.x * G;
    const int e1 = t * (4096 / N2);
    const float2 a1 = tw[e1 & 4095], a4 = tw[(4 * e1) & 4095];
    float2 v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) v[q] = work[z * M + (long long)N2 * (k10 + g) + t + R * q];
    fft_small16xR<R, DIR>(v, lds + g * PS, a1, a4, t);
    __syncthreads();
    // stage [k2][g] so the transposed stores run along k1 (G consecutive)
#pragma unroll
    for (int u = 0; u < 16 / R; u++)
#pragma unroll
        for (int q = 0; q < R; q++) lds[(t * (16 / R) + u + 16 * q) * G + g] = v[u * R + q];
    __syncthreads();
    for (int e = threadIdx.x; e < G * N2; e += NT) {
        const int k2 = e / G, gg = e - k2 * G;
        const long long k = k10 + gg + (long long)N1 * k2;
        const float2 w = lds[e];
        if (POST == 0) dst[z * M + k] = w;   // the plain four-step's rows (fft_four_step)
        else if (POST == 1) dst[z * M + k] = cmul(w, mulv[k]);
        else if (k < n) dst[z * n + k] = cscale(cmul(w, mulv[k]), inv);
    }
}

template <int DIR, bool PRE>
void bs_cols(int N1, const float2 *src, float2 *work, long long n, long long M, int N2, const float2 *ct,
             const float2 *tfine, int sh, long long batch, hipStream_t st)
{
    const float2 *tw = (const float2 *)lqrt_twiddles();
    const int G = 256 / (N1 / 16);   // transforms per workgroup
    const dim3 g((unsigned)(N2 / G), 1, (unsigned)batch);
    switch (N1) {
#define LQ_BC(NN, KER)                                                                                     \
    case NN:                                                                                               \
        hipLaunchKernelGGL(KER, g, dim3(NT), 0, st, src, work, n, M, N2, ct, tw, tfine, sh);              \
        break;
        LQ_BC(32, (k_bs_cols_s<2, DIR, PRE>))
        LQ_BC(64, (k_bs_cols_s<4, DIR, PRE>))
        LQ_BC(128, (k_bs_cols_s<8, DIR, PRE>))
        LQ_BC(256, (k_bs_cols_r<1, DIR, PRE>))
        LQ_BC(512, (k_bs_cols_r<2, DIR, PRE>))
        LQ_BC(1024, (k_bs_cols_r<4, DIR, PRE>))
        LQ_BC(2048, (k_bs_cols_r<8, DIR, PRE>))
        LQ_BC(4096, (k_bs_cols_r<16, DIR, PRE>))
#undef LQ_BC
    default:
        fprintf(stderr, "error: liquid-mi355x: Bluestein column split %d\n", N1);
        exit(1);
    }
    LQ_CHECK_LAUNCH();
}

template <int DIR, int POST>
void bs_rows(int N2, const float2 *work, float2 *dst, long long n, long long M, int N1, const float2 *mulv, float inv,
             long long batch, hipStream_t st)
{
    const float2 *tw = (const float2 *)lqrt_twiddles();
    const int G = 256 / (N2 / 16);
    const dim3 g((unsigned)(N1 / G), 1, (unsigned)batch);
    switch (N2) {
#define LQ_BR(NN, KER)                                                                                     \
    case NN:                                                                                               \
        hipLaunchKernelGGL(KER, g, dim3(NT), 0, st, work, dst, n, M, N1, mulv, inv, tw);                  \
        break;
        LQ_BR(32, (k_bs_rows_s<2, DIR, POST>))
        LQ_BR(64, (k_bs_rows_s<4, DIR, POST>))
        LQ_BR(128, (k_bs_rows_s<8, DIR, POST>))
        LQ_BR(256, (k_bs_rows_r<1, DIR, POST>))
        LQ_BR(512, (k_bs_rows_r<2, DIR, POST>))
        LQ_BR(1024, (k_bs_rows_r<4, DIR, POST>))
        LQ_BR(2048, (k_bs_rows_r<8, DIR, POST>))
        LQ_BR(4096, (k_bs_rows_r<16, DIR, POST>))
#undef LQ_BR
    default:
        fprintf(stderr, "error: liquid-mi355x: Bluestein row split %d\n", N2);
        exit(1);
    }
    LQ_CHECK_LAUNCH();
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
    if (n <= 16384 && (n & (n - 1)) == 0) return 0;
    if ((n & (n - 1)) == 0) return (size_t)(n * batch + n / 4096) * sizeof(float2);
    if (n <= 16) return 0;
    unsigned long long M = 1;
    while (M < 2ull * n - 1) M <<= 1;
    // a: M per transform, B: M, four-step scratch for M, the n-entry chirp
    // table, the fine twiddle table (M / 4096 entries)
    return (size_t)(M * batch + M + (M > 4096 ? M * batch : 0) + n + (M > 4096 ? M / 4096 : 0)) * sizeof(float2);
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
        const float2 *fine = n > 16384 ? fine_table(n, (float2 *)work + (size_t)n * batch, st) : nullptr;
        fft_pow2(n, dir, x, y, (long long)batch, work, fine, st);
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
    const float2 *tfine = M > 4096 ? fine_table((unsigned long long)M, ct + n, st) : nullptr;
    fft_pow2((unsigned)M, +1, B, B, 1, w4, tfine, st);
    if (M > 4096) {
        // the fused four-pass form (above); N1 >= N2 as fft_four_step splits
        const int lg = lg2((unsigned long long)M);
        const int N1 = 1 << ((lg + 1) / 2), N2 = (int)(M / N1);
        const int sh = lg - 12;
        const long long bt = (long long)batch;
        bs_cols<+1, true>(N1, (const float2 *)x, w4, (long long)n, M, N2, ct, tfine, sh, bt, st);
        bs_rows<+1, 1>(N2, w4, a, (long long)n, M, N1, B, 1.f, bt, st);
        bs_cols<-1, false>(N1, a, w4, (long long)n, M, N2, ct, tfine, sh, bt, st);
        bs_rows<-1, 2>(N2, w4, (float2 *)y, (long long)n, M, N1, ct, 1.0f / (float)M, bt, st);
        return;
    }
    const dim3 gM((unsigned)((M + NT - 1) / NT), (unsigned)batch);
    hipLaunchKernelGGL(k_bs_pre, gM, dim3(NT), 0, st, (const float2 *)x, a, (long long)n, M, (const float2 *)ct);
    LQ_CHECK_LAUNCH();
    fft_pow2((unsigned)M, +1, a, a, (long long)batch, w4, nullptr, st);
    hipLaunchKernelGGL(k_bs_mul, gM, dim3(NT), 0, st, a, (const float2 *)B, M);
    LQ_CHECK_LAUNCH();
    fft_pow2((unsigned)M, -1, a, a, (long long)batch, w4, nullptr, st);
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
