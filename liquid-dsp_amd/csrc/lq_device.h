// lq_device.h -- device-side building blocks shared by the kernels:
// complex helpers on float2 (interleaved re,im = the liquid_float_complex
// layout) and an LDS-resident Stockham FFT for power-of-two sizes <= 4096.
#pragma once

#include <hip/hip_runtime.h>

void lq_check(hipError_t e, const char *what, const char *file, int line);
#define LQ_CHECK(x) lq_check((x), #x, __FILE__, __LINE__)
#define LQ_CHECK_LAUNCH() lq_check(hipGetLastError(), "kernel launch", __FILE__, __LINE__)

#define LQ_TW_N 4096

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b)
{
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// multiply by -j (forward radix-4 rotation) or +j
__device__ __forceinline__ float2 cmul_mj(float2 a) { return make_float2(a.y, -a.x); }
__device__ __forceinline__ float2 cmul_pj(float2 a) { return make_float2(-a.y, a.x); }

// twiddle W_n^e for direction dir (+1: exp(-2 pi i e/n), -1: conjugate) from the
// 4096-entry table; n must divide 4096 and e < n.
__device__ __forceinline__ float2 twiddle(const float2 *__restrict__ tw, int e_4096, int dir)
{
    float2 w = tw[e_4096];
    if (dir < 0) w.y = -w.y;
    return w;
}

// radix-4 DFT in place on v[0..3]; dir +1 forward, -1 backward.
__device__ __forceinline__ void dft4(float2 &v0, float2 &v1, float2 &v2, float2 &v3, int dir)
{
    float2 a = cadd(v0, v2), b = csub(v0, v2), c = cadd(v1, v3), d = csub(v1, v3);
    float2 jd = dir > 0 ? cmul_mj(d) : cmul_pj(d);
    v0 = cadd(a, c);
    v2 = csub(a, c);
    v1 = cadd(b, jd);
    v3 = csub(b, jd);
}

// One Stockham pass of radix R (2 or 4) over NB transforms of N points:
// for butterfly (j, k), k < s: v_q = src[j*s + k + q*N/R] * W_{R s}^{q k},
// dst[j*R*s + k + q*s] = DFT_R(v)_q.  (Index map verified against numpy.)
template <int N, int R, int NB, int NT>
__device__ __forceinline__ void stockham_pass(const float2 *src, float2 *dst, int s, int log2s,
                                              const float2 *__restrict__ tw, int dir)
{
    constexpr int L = (N / R) > 0 ? (N / R) : 1;
    for (int e = threadIdx.x; e < NB * L; e += NT) {
        const int t = e / L;
        const int bi = e - t * L;
        const int k = bi & (s - 1);
        const int j = bi >> log2s;
        const float2 *x = src + t * N;
        float2 *y = dst + t * N;
        const int tstride = LQ_TW_N / (R * s);
        if (R == 4) {
            float2 v0 = x[j * s + k], v1 = x[j * s + k + L], v2 = x[j * s + k + 2 * L],
                   v3 = x[j * s + k + 3 * L];
            if (s > 1) {
                v1 = cmul(v1, twiddle(tw, 1 * k * tstride, dir));
                v2 = cmul(v2, twiddle(tw, 2 * k * tstride, dir));
                v3 = cmul(v3, twiddle(tw, 3 * k * tstride, dir));
            }
            dft4(v0, v1, v2, v3, dir);
            float2 *o = y + j * 4 * s + k;
            o[0] = v0;
            o[s] = v1;
            o[2 * s] = v2;
            o[3 * s] = v3;
        } else {
            float2 v0 = x[j * s + k], v1 = x[j * s + k + L];
            if (s > 1) v1 = cmul(v1, twiddle(tw, k * tstride, dir));
            float2 *o = y + j * 2 * s + k;
            o[0] = cadd(v0, v1);
            o[s] = csub(v0, v1);
        }
    }
}

template <int N>
struct lq_log2 {
    static constexpr int value = 1 + lq_log2<N / 2>::value;
};
template <>
struct lq_log2<1> {
    static constexpr int value = 0;
};

// NB independent N-point FFTs held back to back in LDS buffer `a`, ping-pong
// with `b`.  Every thread of the block must call it (it synchronises).
// Returns the buffer that holds the natural-order result.
template <int N, int NB, int NT>
__device__ float2 *lds_fft(float2 *a, float2 *b, const float2 *__restrict__ tw, int dir)
{
    constexpr int LG = lq_log2<N>::value;
    float2 *src = a, *dst = b;
    int s = 1, log2s = 0;
    if (LG & 1) {
        stockham_pass<N, 2, NB, NT>(src, dst, s, log2s, tw, dir);
        __syncthreads();
        float2 *t = src; src = dst; dst = t;
        s = 2; log2s = 1;
    }
#pragma unroll
    for (int p = 0; p < LG / 2; p++) {
        stockham_pass<N, 4, NB, NT>(src, dst, s, log2s, tw, dir);
        __syncthreads();
        float2 *t = src; src = dst; dst = t;
        s <<= 2; log2s += 2;
    }
    return src;
}
