// k_resamp2.hip -- half-band resampler (resamp2, src/filter/src/resamp2.c)
// as one data-parallel kernel per block of calls.
//
// The reference keeps two windows w0, w1 of 2m samples; every mode pushes
// samples into them and reads either the "delay" tap (window index m-1, i.e.
// the sample pushed m pushes ago) or the odd-tap dot product
// sum_j h1[j] w[j] (h1[j] = h[4m-1-2j]).  Here each window is the virtual
// sequence E_p = hist_p (2m samples) ++ this block's pushes, so the output of
// call i is a pure function of E_0, E_1 -- one lane per call, no state.
//   filter : call i pushes x[i] into window p_i = (t0+i)&1
//   decim  : w1 <- x[2i], w0 <- x[2i+1]            (analyzer: halved)
//   interp : w0 <- x[i],  w1 <- x[i]
//   synth  : w0 <- X[2i]+X[2i+1], w1 <- X[2i]-X[2i+1]
#include <hip/hip_runtime.h>

#include "lq_device.h"
#include "lq_kernels.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float2 r2_mac(float h, float2 v, float2 a)
{
    return make_float2(fmaf(h, v.x, a.x), fmaf(h, v.y, a.y));
}
__device__ __forceinline__ float r2_mac(float h, float v, float a) { return fmaf(h, v, a); }
__device__ __forceinline__ float2 r2_mac(float2 h, float2 v, float2 a)
{
    return make_float2(fmaf(h.x, v.x, fmaf(-h.y, v.y, a.x)), fmaf(h.x, v.y, fmaf(h.y, v.x, a.y)));
}
__device__ __forceinline__ float r2_scale(float s, float v) { return s * v; }
__device__ __forceinline__ float2 r2_scale(float s, float2 v) { return make_float2(s * v.x, s * v.y); }
__device__ __forceinline__ float r2_add(float a, float b) { return a + b; }
__device__ __forceinline__ float2 r2_add(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float r2_sub(float a, float b) { return a - b; }
__device__ __forceinline__ float2 r2_sub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

struct R2Args {
    int mode;          // LQK_R2_*
    int m;             // semi-length: windows of 2m
    int t0;            // filter mode: toggle before the first call
    long long n;       // calls in this block
    float scale;       // power-of-two output scale (msresamp2 decimator's 1/M), exact
};

// E_p[k]: k < 2m from the history, else the (k-2m)-th push of this block
template <typename S>
__device__ __forceinline__ S r2_E(const R2Args &a, int p, long long k, const S *__restrict__ h0,
                                  const S *__restrict__ h1, const S *__restrict__ x)
{
    const int W = 2 * a.m;
    if (k < W) return p ? h1[k] : h0[k];
    const long long c = k - W;
    switch (a.mode) {
    case LQK_R2_FILTER: return x[2 * c + ((p + a.t0) & 1)];
    case LQK_R2_DECIM: return p ? x[2 * c] : x[2 * c + 1];
    case LQK_R2_ANALYZER: return r2_scale(0.5f, p ? x[2 * c] : x[2 * c + 1]);
    case LQK_R2_INTERP: return x[c];
    default: {   // synthesizer
        const S u = x[2 * c], v = x[2 * c + 1];
        return p ? r2_sub(u, v) : r2_add(u, v);
    }
    }
}

template <typename S, typename C>
__device__ __forceinline__ S r2_dot(const R2Args &a, const C *__restrict__ th, int p, long long k0,
                                    const S *__restrict__ h0, const S *__restrict__ h1, const S *__restrict__ x)
{
    S acc{};
    for (int j = 0; j < 2 * a.m; j++) acc = r2_mac(th[j], r2_E(a, p, k0 + j, h0, h1, x), acc);
    return acc;
}

template <typename S, typename C>
__global__ __launch_bounds__(NT) void k_resamp2(R2Args a, const C *__restrict__ taps, const S *__restrict__ hist0,
                                                const S *__restrict__ hist1, const S *__restrict__ x,
                                                S *__restrict__ y0, S *__restrict__ y1)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char r2_smem[];
    C *th = reinterpret_cast<C *>(r2_smem);
    for (int j = threadIdx.x; j < 2 * a.m; j += NT) th[j] = taps[j];
    __syncthreads();
    const long long i = (long long)blockIdx.x * NT + threadIdx.x;
    if (i >= a.n) return;
    const long long W = 2 * a.m;
    switch (a.mode) {
    case LQK_R2_FILTER: {
        const int p = (a.t0 + (int)(i & 1)) & 1;
        const int sp = (p + a.t0) & 1;                 // block inputs of window p are x[2c + sp]
        const long long cp = (i + 1 - sp) >> 1;        // pushes into p before call i
        const long long cq = i - cp;
        const S yi = r2_E(a, p, W + cp - a.m, hist0, hist1, x);
        const S yq = r2_dot(a, th, 1 - p, cq, hist0, hist1, x);
        y0[i] = r2_scale(0.5f, r2_add(yi, yq));
        y1[i] = r2_scale(0.5f, r2_sub(yi, yq));
        break;
    }
    case LQK_R2_DECIM:
    case LQK_R2_ANALYZER: {
        const S yq = r2_dot(a, th, 1, i + 1, hist0, hist1, x);
        const S yd = r2_E(a, 0, W + i - a.m, hist0, hist1, x);
        if (a.mode == LQK_R2_DECIM) {
            y0[i] = r2_scale(a.scale, r2_add(yd, yq));
        } else {
            y0[2 * i] = r2_add(yq, yd);
            y0[2 * i + 1] = r2_sub(yq, yd);
        }
        break;
    }
    default: {   // interp, synthesizer: delay branch first, then the dot product
        y0[2 * i] = r2_E(a, 0, W + i - a.m, hist0, hist1, x);
        y0[2 * i + 1] = r2_dot(a, th, 1, i + 1, hist0, hist1, x);
    }
    }
}

// Tiled form for the modes whose call i reads the dot window E_1[i+1 ..
// i+2m] and the delay sample E_0[2m + i - m] (decim, analyzer, interp,
// synthesizer): a workgroup stages the E_1 / E_0 spans of its C = NT*R calls
// in LDS once (each element gathered from history or x a single time instead
// of once per tap), then each lane evaluates R consecutive calls from a
// register window of R + 2m - 1 samples.
template <typename S, typename C, int R>
__global__ __launch_bounds__(NT) void k_resamp2_tiled(R2Args a, const C *__restrict__ taps,
                                                      const S *__restrict__ hist0, const S *__restrict__ hist1,
                                                      const S *__restrict__ x, S *__restrict__ y0)
{
    constexpr int CT = NT * R;                    // calls per tile
    extern __shared__ __attribute__((aligned(16))) unsigned char r2_smem[];
    const int m = a.m, W = 2 * m;
    C *th = reinterpret_cast<C *>(r2_smem);
    S *e1 = reinterpret_cast<S *>(r2_smem + ((2 * W * sizeof(C) + 15) & ~15));   // E_1[i0+1 ...], CT + W - 1
    S *e0 = e1 + CT + W;                                                       // E_0[W + i0 - m ...], CT
    const long long i0 = (long long)blockIdx.x * CT;
    for (int j = threadIdx.x; j < W; j += NT) th[j] = taps[j];
    for (int u = threadIdx.x; u < CT + W - 1; u += NT) {
        const long long k = i0 + 1 + u;
        if (k - W < a.n) e1[u] = r2_E(a, 1, k, hist0, hist1, x);   // push k-W exists
    }
    for (int u = threadIdx.x; u < CT; u += NT) {
        if (i0 + u < a.n) e0[u] = r2_E(a, 0, W + i0 + u - m, hist0, hist1, x);
    }
    __syncthreads();
    const int l0 = threadIdx.x * R;
    if (i0 + l0 >= a.n) return;
    S acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = S{};
    for (int j = 0; j < W; j++) {
        const C h = th[j];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = r2_mac(h, e1[l0 + r + j], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        const long long i = i0 + l0 + r;
        if (i >= a.n) break;
        const S yq = acc[r], yd = e0[l0 + r];
        switch (a.mode) {
        case LQK_R2_DECIM: y0[i] = r2_scale(a.scale, r2_add(yd, yq)); break;
        case LQK_R2_ANALYZER:
            y0[2 * i] = r2_add(yq, yd);
            y0[2 * i + 1] = r2_sub(yq, yd);
            break;
        default:   // interp, synthesizer
            y0[2 * i] = yd;
            y0[2 * i + 1] = yq;
        }
    }
}

// k_resamp2_tiled with the mode a template parameter and the E_0 / E_1
// spans staged branch-free: every sample comes through range-checked buffer
// loads of the history (2m samples) and of x (zero outside), all of a lane's
// loads issued before the first LDS store (the generic staging loop branched
// per element and waited for each load in turn).  32-bit offsets: the host
// takes this path for calls of < 2^31 bytes of input.
template <typename S>
__device__ __forceinline__ S r2_ldb(__amdgpu_buffer_rsrc_t r, long long idx)
{
    const unsigned off = (unsigned)(idx * (long long)sizeof(S));   // idx < 0: out of range, 0
    if constexpr (sizeof(S) == 8)
        return __builtin_bit_cast(S, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
    else
        return __builtin_bit_cast(S, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

template <typename S, typename C, int R, int MODE>
__global__ __launch_bounds__(NT) void k_resamp2_tiled_b(R2Args a, const C *__restrict__ taps,
                                                        const S *__restrict__ hist0, const S *__restrict__ hist1,
                                                        const S *__restrict__ x, S *__restrict__ y0)
{
    const bool al16 = ((unsigned long long)y0 & 15) == 0;
    constexpr int CT = NT * R;
    constexpr int NU = (CT + 32 - 1 + NT - 1) / NT;   // staging slots per lane (2m <= 32)
    extern __shared__ __attribute__((aligned(16))) unsigned char r2_smem[];
    const int m = a.m, W = 2 * m;
    C *th = reinterpret_cast<C *>(r2_smem);
    S *e1 = reinterpret_cast<S *>(r2_smem + ((2 * W * sizeof(C) + 15) & ~15));
    S *e0 = e1 + CT + W;
    const long long i0 = (long long)blockIdx.x * CT;
    const int ES = (int)sizeof(S);
    const long long nx = MODE == LQK_R2_INTERP ? a.n : 2 * a.n;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)(nx * ES), 0x00020000);
    const __amdgpu_buffer_rsrc_t rh0 = __builtin_amdgcn_make_buffer_rsrc((void *)hist0, (short)0, W * ES, 0x00020000);
    const __amdgpu_buffer_rsrc_t rh1 = __builtin_amdgcn_make_buffer_rsrc((void *)hist1, (short)0, W * ES, 0x00020000);
    // E_p[k]: history part (k < W) + push part c = k - W (zero where out of range)
    auto E = [&](int p, long long k, S &h, S &u, S &v) {
        const long long c = k - W;
        h = r2_ldb<S>(p ? rh1 : rh0, k);
        if constexpr (MODE == LQK_R2_INTERP) {
            u = r2_ldb<S>(rx, c);
        } else if constexpr (MODE == LQK_R2_SYNTHESIZER) {
            u = r2_ldb<S>(rx, 2 * c);
            v = r2_ldb<S>(rx, 2 * c + 1);
        } else {   // decim, analyzer: w1 <- x[2c], w0 <- x[2c+1]
            u = r2_ldb<S>(rx, 2 * c + (p ? 0 : 1));
        }
    };
    auto combine = [&](int p, S h, S u, S v) -> S {
        if constexpr (MODE == LQK_R2_SYNTHESIZER) return r2_add(h, p ? r2_sub(u, v) : r2_add(u, v));
        else if constexpr (MODE == LQK_R2_ANALYZER) return r2_add(h, r2_scale(0.5f, u));
        else return r2_add(h, u);
    };
    for (int j = threadIdx.x; j < W; j += NT) th[j] = taps[j];
    {
        S h[NU], u[NU], v[NU];
#pragma unroll
        for (int q = 0; q < NU; q++) E(1, i0 + 1 + threadIdx.x + q * NT, h[q], u[q], v[q]);
#pragma unroll
        for (int q = 0; q < NU; q++) {
            const int idx = threadIdx.x + q * NT;
            if (idx < CT + W - 1) e1[idx] = combine(1, h[q], u[q], v[q]);
        }
    }
    {
        constexpr int N0 = CT / NT;
        S h[N0], u[N0], v[N0];
#pragma unroll
        for (int q = 0; q < N0; q++) E(0, W + i0 + threadIdx.x + q * NT - m, h[q], u[q], v[q]);
#pragma unroll
        for (int q = 0; q < N0; q++) e0[threadIdx.x + q * NT] = combine(0, h[q], u[q], v[q]);
    }
    __syncthreads();
    // lane t takes calls t, t + NT, ...: the window reads of a wave are
    // consecutive (conflict-free) and every store instruction covers
    // consecutive outputs
    const int l0 = threadIdx.x;
    S acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = S{};
    for (int j = 0; j < W; j++) {
        const C hj = th[j];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = r2_mac(hj, e1[l0 + NT * r + j], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        const long long i = i0 + l0 + NT * r;
        if (i >= a.n) break;
        const S yq = acc[r], yd = e0[l0 + NT * r];
        if constexpr (MODE == LQK_R2_DECIM) {
            {   // non-temporal stores (decim 0.159 -> 0.155 ms, interp 0.348 ->
                // 0.337 ms per 2^26 inputs at m = 12, r06r2)
                const S v = r2_scale(a.scale, r2_add(yd, yq));
                if constexpr (sizeof(S) == 8) {
                    typedef float v2nt __attribute__((ext_vector_type(2)));
                    __builtin_nontemporal_store(v2nt{v.x, v.y}, reinterpret_cast<v2nt *>(y0 + i));
                } else {
                    __builtin_nontemporal_store(v, y0 + i);
                }
            }
        } else {
            const S o0 = MODE == LQK_R2_ANALYZER ? r2_add(yq, yd) : yd;
            const S o1 = MODE == LQK_R2_ANALYZER ? r2_sub(yq, yd) : yq;
            if constexpr (sizeof(S) == 8) {
                // the call's two outputs as one 16-byte store: each store
                // instruction then writes 1 KB contiguous (two 8-byte stores
                // 16 bytes apart each covered half of every line)
                if (al16) {
                    typedef float v4f_ __attribute__((ext_vector_type(4)));
                    __builtin_nontemporal_store(v4f_{o0.x, o0.y, o1.x, o1.y}, reinterpret_cast<v4f_ *>(y0 + 2 * i));
                } else {
                    y0[2 * i] = o0;
                    y0[2 * i + 1] = o1;
                }
            } else {
                y0[2 * i] = o0;
                y0[2 * i + 1] = o1;
            }
        }
    }
}

// new history: hist_p[k] = E_p[pushes_p + k], k < 2m
template <typename S>
__global__ __launch_bounds__(NT) void k_resamp2_hist(R2Args a, long long push0, long long push1,
                                                     const S *__restrict__ hist0, const S *__restrict__ hist1,
                                                     const S *__restrict__ x, S *__restrict__ out0,
                                                     S *__restrict__ out1)
{
    const int k = blockIdx.x * NT + threadIdx.x;
    const int W = 2 * a.m;
    if (k >= 2 * W) return;
    const int p = k >= W;
    const int kk = p ? k - W : k;
    const S v = r2_E(a, p, (p ? push1 : push0) + kk, hist0, hist1, x);
    (p ? out1 : out0)[kk] = v;
}

template <typename S, typename C>
void run_r2(const R2Args &a, const void *taps, const void *h0, const void *h1, void *n0, void *n1, const void *x,
            void *y0, void *y1, hipStream_t st)
{
    long long p0, p1;
    switch (a.mode) {
    case LQK_R2_FILTER:
        p1 = (a.n + (a.t0 ? 1 : 0)) / 2;   // calls whose window is w1
        p0 = a.n - p1;
        break;
    default: p0 = p1 = a.n;
    }
    if (a.mode == LQK_R2_FILTER) {
        const unsigned grid = (unsigned)((a.n + NT - 1) / NT);
        hipLaunchKernelGGL((k_resamp2<S, C>), dim3(grid), dim3(NT), (size_t)2 * a.m * sizeof(C), st, a,
                           (const C *)taps, (const S *)h0, (const S *)h1, (const S *)x, (S *)y0, (S *)y1);
    } else {
        constexpr int R = 4, CT = NT * R;
        const size_t lds = ((2 * 2 * a.m * sizeof(C) + 15) & ~(size_t)15) + (size_t)(2 * CT + 2 * a.m) * sizeof(S);
        const unsigned grid = (unsigned)((a.n + CT - 1) / CT);
        const long long xbytes = (a.mode == LQK_R2_INTERP ? a.n : 2 * a.n) * (long long)sizeof(S);
        if (a.m <= 16 && xbytes < (1ll << 31)) {
            switch (a.mode) {
#define LQ_R2B(MD)                                                                                         \
    case MD:                                                                                               \
        hipLaunchKernelGGL((k_resamp2_tiled_b<S, C, R, MD>), dim3(grid), dim3(NT), lds, st, a, (const C *)taps, \
                           (const S *)h0, (const S *)h1, (const S *)x, (S *)y0);                           \
        break;
                LQ_R2B(LQK_R2_DECIM) LQ_R2B(LQK_R2_ANALYZER) LQ_R2B(LQK_R2_INTERP) LQ_R2B(LQK_R2_SYNTHESIZER)
#undef LQ_R2B
            }
        } else {
            hipLaunchKernelGGL((k_resamp2_tiled<S, C, R>), dim3(grid), dim3(NT), lds, st, a, (const C *)taps,
                               (const S *)h0, (const S *)h1, (const S *)x, (S *)y0);
        }
    }
    LQ_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_resamp2_hist<S>), dim3((unsigned)((4 * a.m + NT - 1) / NT)), dim3(NT), 0, st, a, p0, p1,
                       (const S *)h0, (const S *)h1, (const S *)x, (S *)n0, (S *)n1);
    LQ_CHECK_LAUNCH();
}

} // namespace

extern "C" void lqk_resamp2(int kind, int mode, unsigned int m, int t0, float scale, const void *taps,
                            const void *hist0, const void *hist1, void *hist0_new, void *hist1_new, const void *x,
                            unsigned long long n, void *y0, void *y1, void *stream)
{
    if (n == 0) return;
    R2Args a{mode, (int)m, t0 & 1, (long long)n, scale};
    hipStream_t st = (hipStream_t)stream;
    switch (kind) {
    case 0: run_r2<float, float>(a, taps, hist0, hist1, hist0_new, hist1_new, x, y0, y1, st); break;
    case 1: run_r2<float2, float>(a, taps, hist0, hist1, hist0_new, hist1_new, x, y0, y1, st); break;
    default: run_r2<float2, float2>(a, taps, hist0, hist1, hist0_new, hist1_new, x, y0, y1, st); break;
    }
}
