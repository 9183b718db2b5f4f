// k_dotprod.hip -- batched inner products Y[v] = sum_i h[i] X[v][i]
// (dotprod_{rrrf,crcf,cccf}: src/dotprod/src/dotprod.c:42-167, x86 variants
// src/dotprod/src/dotprod_{rrrf,crcf,cccf}.mmx.c).
//
// The reference computes one dot product per call on the CPU.  The MI355X
// form is a streaming reduction: G lanes (a power of two <= 64) share one
// vector, each lane reads 16-byte chunks (2 complex or 4 real samples) so a
// group's loads are contiguous, partial sums are combined with DPP/xor
// shuffles inside the wave, and one lane writes the result.  HBM-bound:
// 8n + 8 bytes per complex vector.
#include "lq_device.h"
#include "lq_kernels.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace {

constexpr int NT = 256;
typedef float v4f __attribute__((ext_vector_type(4)));

template <int KIND>
struct dp;
// rrrf: 4 real samples per 16-byte chunk
template <>
struct dp<0> {
    typedef float acc_t;
    static constexpr int VEC = 4;
};
// crcf / cccf: 2 complex samples per chunk
template <>
struct dp<1> {
    typedef float2 acc_t;
    static constexpr int VEC = 2;
};
template <>
struct dp<2> {
    typedef float2 acc_t;
    static constexpr int VEC = 2;
};

__device__ __forceinline__ float shfl_xor(float v, int m) { return __shfl_xor(v, m, 64); }

// vectorised path: n % VEC == 0, rows 16-byte aligned
template <int KIND>
__global__ __launch_bounds__(NT) void k_dot_vec(const float *__restrict__ h, int n, const float *__restrict__ X,
                                                long long stride_f, long long nvec, float *__restrict__ Y, int G,
                                                int lg)
{
    const int lane = threadIdx.x & (G - 1);
    const long long grp = ((long long)blockIdx.x * NT + threadIdx.x) >> lg;
    const long long ngrp = ((long long)gridDim.x * NT) >> lg;
    const int nchunk = n / dp<KIND>::VEC;
    for (long long v = grp; v < nvec; v += ngrp) {
        const float4 *xr = reinterpret_cast<const float4 *>(X + v * stride_f);
        float ar = 0.f, ai = 0.f, br = 0.f, bi = 0.f;
        for (int c = lane; c < nchunk; c += G) {
            const v4f xn = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(xr) + c);
            const float4 xv = make_float4(xn.x, xn.y, xn.z, xn.w);
            if (KIND == 0) {
                const float4 hv = reinterpret_cast<const float4 *>(h)[c];
                ar = fmaf(hv.x, xv.x, ar);
                ai = fmaf(hv.y, xv.y, ai);
                br = fmaf(hv.z, xv.z, br);
                bi = fmaf(hv.w, xv.w, bi);
            } else if (KIND == 1) {
                const float2 hv = reinterpret_cast<const float2 *>(h)[c];
                ar = fmaf(hv.x, xv.x, ar);
                ai = fmaf(hv.x, xv.y, ai);
                br = fmaf(hv.y, xv.z, br);
                bi = fmaf(hv.y, xv.w, bi);
            } else {
                const float4 hv = reinterpret_cast<const float4 *>(h)[c];
                ar = fmaf(hv.x, xv.x, ar);
                ar = fmaf(-hv.y, xv.y, ar);
                ai = fmaf(hv.x, xv.y, ai);
                ai = fmaf(hv.y, xv.x, ai);
                br = fmaf(hv.z, xv.z, br);
                br = fmaf(-hv.w, xv.w, br);
                bi = fmaf(hv.z, xv.w, bi);
                bi = fmaf(hv.w, xv.z, bi);
            }
        }
        float re, im;
        if (KIND == 0) {
            re = (ar + ai) + (br + bi);
            im = 0.f;
        } else {
            re = ar + br;
            im = ai + bi;
        }
        for (int m = G >> 1; m > 0; m >>= 1) {
            re += shfl_xor(re, m);
            if (KIND != 0) im += shfl_xor(im, m);
        }
        if (lane == 0) {
            if (KIND == 0) Y[v] = re;
            else reinterpret_cast<float2 *>(Y)[v] = make_float2(re, im);
        }
    }
}

// scalar path for ragged lengths / unaligned rows
template <int KIND>
__global__ __launch_bounds__(NT) void k_dot_scalar(const float *__restrict__ h, int n, const float *__restrict__ X,
                                                   long long stride, long long nvec, float *__restrict__ Y, int G,
                                                   int lg)
{
    const int lane = threadIdx.x & (G - 1);
    const long long grp = ((long long)blockIdx.x * NT + threadIdx.x) >> lg;
    const long long ngrp = ((long long)gridDim.x * NT) >> lg;
    for (long long v = grp; v < nvec; v += ngrp) {
        float re = 0.f, im = 0.f;
        for (int i = lane; i < n; i += G) {
            if (KIND == 0) {
                re = fmaf(h[i], X[v * stride + i], re);
            } else {
                const float2 x = reinterpret_cast<const float2 *>(X)[v * stride + i];
                if (KIND == 1) {
                    re = fmaf(h[i], x.x, re);
                    im = fmaf(h[i], x.y, im);
                } else {
                    const float2 hh = reinterpret_cast<const float2 *>(h)[i];
                    re = fmaf(hh.x, x.x, re);
                    re = fmaf(-hh.y, x.y, re);
                    im = fmaf(hh.x, x.y, im);
                    im = fmaf(hh.y, x.x, im);
                }
            }
        }
        for (int m = G >> 1; m > 0; m >>= 1) {
            re += shfl_xor(re, m);
            im += shfl_xor(im, m);
        }
        if (lane == 0) {
            if (KIND == 0) Y[v] = re;
            else reinterpret_cast<float2 *>(Y)[v] = make_float2(re, im);
        }
    }
}

template <int KIND>
void launch(const void *h, unsigned n, const void *X, long long stride, long long nvec, void *Y, hipStream_t st)
{
    const int VEC = dp<KIND>::VEC;
    const size_t esz = KIND == 0 ? 4 : 8;
    const bool vec_ok = (n % VEC == 0) && ((stride * esz) % 16 == 0) && (((uintptr_t)X & 15) == 0) &&
                        (((uintptr_t)h & 15) == 0);
    const long long work = vec_ok ? n / VEC : n; // elements a group walks
    // at most 8 (n <= 128 complex) or 16 lanes per vector: each lane keeps
    // several 16-byte loads in flight and the shuffle reduction stays short
    // (dotprod_cccf 2^20 vectors: n=64 0.61-0.69 -> 0.82, n=256 0.76 -> 0.83
    // of the 8 TB/s spec; 64 lanes per vector before)
    const int gmax = work <= 64 ? 8 : 16;
    int G = 1, lg = 0;
    while (G < gmax && (long long)G * 2 <= work) {
        G <<= 1;
        lg++;
    }
    long long groups = nvec;
    long long threads = groups * G;
    long long blocks = (threads + NT - 1) / NT;
    if (blocks > 256 * 16) blocks = 256 * 16; // grid-stride beyond 16 blocks per CU
    if (blocks < 1) blocks = 1;
    if (vec_ok)
        hipLaunchKernelGGL(k_dot_vec<KIND>, dim3((unsigned)blocks), dim3(NT), 0, st, (const float *)h, (int)n,
                           (const float *)X, stride * (long long)(esz / 4), nvec, (float *)Y, G, lg);
    else
        hipLaunchKernelGGL(k_dot_scalar<KIND>, dim3((unsigned)blocks), dim3(NT), 0, st, (const float *)h, (int)n,
                           (const float *)X, stride, nvec, (float *)Y, G, lg);
    LQ_CHECK_LAUNCH();
}

} // namespace

// one vector, 256 lanes, result straight to pinned host memory + completion
// flag: the per-call dotprod_*_execute() (one launch, no stream sync)
template <int KIND>
__global__ __launch_bounds__(256) void k_dot_single(const float *__restrict__ h, int n, const float *__restrict__ x,
                                                    float *y, unsigned *flag, unsigned seq)
{
    typedef typename dp<KIND>::acc_t A;
    __shared__ A part[256];
    A acc{};
    for (int i = threadIdx.x; i < n; i += 256) {
        if constexpr (KIND == 0) {
            acc = fmaf(h[i], x[i], acc);
        } else if constexpr (KIND == 1) {
            const float hv = h[i];
            acc.x = fmaf(hv, x[2 * i], acc.x);
            acc.y = fmaf(hv, x[2 * i + 1], acc.y);
        } else {
            const float hr = h[2 * i], hi = h[2 * i + 1], xr = x[2 * i], xi = x[2 * i + 1];
            acc.x = fmaf(-hi, xi, fmaf(hr, xr, acc.x));
            acc.y = fmaf(hi, xr, fmaf(hr, xi, acc.y));
        }
    }
    part[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        A s{};
        for (int t = 0; t < 256; t++) {
            if constexpr (KIND == 0) s += part[t];
            else s = make_float2(s.x + part[t].x, s.y + part[t].y);
        }
        if constexpr (KIND == 0) y[0] = s;
        else {
            y[0] = s.x;
            y[1] = s.y;
        }
        lq_signal(flag, seq);
    }
}

extern "C" void lqk_dotprod_single(int kind, const void *h, unsigned int n, const void *x, void *y, unsigned *flag,
                                   unsigned seq, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    const float *hf = (const float *)h, *xf = (const float *)x;
    switch (kind) {
    case 0: hipLaunchKernelGGL(k_dot_single<0>, dim3(1), dim3(256), 0, st, hf, (int)n, xf, (float *)y, flag, seq); break;
    case 1: hipLaunchKernelGGL(k_dot_single<1>, dim3(1), dim3(256), 0, st, hf, (int)n, xf, (float *)y, flag, seq); break;
    case 2: hipLaunchKernelGGL(k_dot_single<2>, dim3(1), dim3(256), 0, st, hf, (int)n, xf, (float *)y, flag, seq); break;
    default:
        fprintf(stderr, "error: dotprod: invalid kind %d\n", kind);
        exit(1);
    }
    LQ_CHECK_LAUNCH();
}

extern "C" void lqk_dotprod_batch(int kind, const void *h, unsigned int n, const void *X, unsigned long long stride,
                                  unsigned long long nvec, void *Y, void *stream)
{
    if (nvec == 0) return;
    hipStream_t st = (hipStream_t)stream;
    switch (kind) {
    case 0: launch<0>(h, n, X, (long long)stride, (long long)nvec, Y, st); break;
    case 1: launch<1>(h, n, X, (long long)stride, (long long)nvec, Y, st); break;
    case 2: launch<2>(h, n, X, (long long)stride, (long long)nvec, Y, st); break;
    default:
        fprintf(stderr, "error: dotprod: invalid kind %d\n", kind);
        exit(1);
    }
}
