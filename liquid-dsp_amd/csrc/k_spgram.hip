// k_spgram.hip -- spectral periodogram (spgramcf / spgramf,
// src/fft/src/spgram.c) as batched windowed transforms.
//
// A block of input produces T transforms at known positions (every W/2
// samples for accumulate_psd, every nfft/4 and at the end for estimate_psd);
// their windows are gathered from [history | block] into a T x nfft batch,
// transformed together (csrc/k_fft.hip), then reduced per bin in two passes
// (chunks of 64 transforms, then the chunks in order): the exponential
// average is the reference's recursion regrouped by chunk, the estimate sums
// |X|^2.
#include <hip/hip_runtime.h>

#include "lq_device.h"
#include "lq_fft1024.h"
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

// Per-bin reductions over T transforms, in two passes so that every CU takes
// part: chunk c of TC consecutive transforms reduces to part[c][k], then one
// pass per bin folds the chunks in transform order.
//   sum   (estimate_psd, spgram.c:262-276): acc[(k + nfft/2) % nfft] += sum_t |X_t[k]|^2
//   accum (accumulate_psd, spgram.c:205-236): psd[k] = (1 - a) psd[k] + a |X_t[k]|^2, t in
//         order; a chunk's share is its recursion run from 0, folded in as
//         psd = (1 - a)^len psd + part (the same recursion, regrouped)
constexpr int SPG_TC = 64;

__global__ __launch_bounds__(NT) void k_spg_part(const float2 *__restrict__ X, long long T, int nfft, int accum,
                                                 float alpha, float *__restrict__ part)
{
#pragma clang fp contract(off)
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k >= nfft) return;
    const long long t0 = (long long)blockIdx.y * SPG_TC;
    const long long t1 = (t0 + SPG_TC < T) ? t0 + SPG_TC : T;
    float p = 0.0f;
    for (long long t = t0; t < t1; t++) {
        const float v = pwr(X[t * nfft + k]);
        p = accum ? (1.0f - alpha) * p + alpha * v : p + v;
    }
    part[(long long)blockIdx.y * nfft + k] = p;
}

// Folds chunk values part[c][k] (chunks of TC transforms, the last one
// shorter: T in total) in order.  Group y of G consecutive chunks starts from
// 0 and writes out[y][k] -- itself the value of a chunk of G*TC transforms --
// or, with dst (a single group), starts from dst[idx] and writes it back.
__global__ __launch_bounds__(NT) void k_spg_fold(const float *__restrict__ part, long long T, long long TC, int nfft,
                                                 int accum, float alpha, long long G, float *__restrict__ out,
                                                 float *__restrict__ dst)
{
#pragma clang fp contract(off)
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k >= nfft) return;
    const int idx = accum ? k : (k + nfft / 2) % nfft;
    const long long nch = (T + TC - 1) / TC;
    const long long ca = (long long)blockIdx.y * G;
    const long long cb = (ca + G < nch) ? ca + G : nch;
    const float dfull = powf(1.0f - alpha, (float)TC);
    float p = dst ? dst[idx] : 0.0f;
    // 32 chunk values loaded together, then folded in order
    constexpr int B = 32;
    for (long long c0 = ca; c0 < cb; c0 += B) {
        float v[B];
#pragma unroll
        for (int g = 0; g < B; g++) v[g] = (c0 + g < cb) ? part[(c0 + g) * nfft + k] : 0.0f;
#pragma unroll
        for (int g = 0; g < B; g++) {
            const long long c = c0 + g;
            if (c >= cb) continue;
            if (accum) {
                const long long len = (c + 1 < nch) ? TC : T - c * TC;
                const float d = (len == TC) ? dfull : powf(1.0f - alpha, (float)len);
                p = d * p + v[g];
            } else {
                p = p + v[g];
            }
        }
    }
    if (dst) dst[idx] = p;
    else out[(long long)blockIdx.y * nfft + k] = p;
}

// nfft = 1024, fused: one wave per chunk of SPG_TC consecutive transforms
// gathers each window straight from (hist | x) into registers, runs the
// wave-level 1024-point transform (lq_fft1024.h) and folds |X[k]|^2 into
// per-lane partials -- no transform batch staged through HBM.  Transform t
// ends at e0 + t*hop (the last one at elast).  Writes part[chunk][k] for
// k_spg_fold, exactly as k_spg_part does.
// HALF: W <= 512, so window samples r >= 8 of a lane (i = lane + 64 r) are
// zero: they are neither loaded nor weighted
template <typename S, bool HALF>
__global__ __launch_bounds__(NT, 3) void k_spg_fused1024(const S *__restrict__ hist, int W, const S *__restrict__ x,
                                                      long long e0, long long hop, long long T, long long elast,
                                                      const float *__restrict__ w, int accum, float alpha,
                                                      const float2 *__restrict__ tw4096, float *__restrict__ part)
{
#pragma clang fp contract(off)
    __shared__ __attribute__((aligned(16))) float2 tw1[1024];
    __shared__ __attribute__((aligned(16))) float2 tw2[64];
    __shared__ __attribute__((aligned(16))) float2 Bs[NT / 64][1088];
    f1k_tables<+1>(tw1, tw2, tw4096);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long chunk = (long long)blockIdx.x * (NT / 64) + wave;
    const long long t0 = chunk * SPG_TC;
    if (t0 >= T) return;
    const long long t1 = (t0 + SPG_TC < T) ? t0 + SPG_TC : T;
    float2 *B = Bs[wave];
    constexpr int RW = HALF ? 8 : 16;   // rows that can hold window samples
    float wv[RW], p[16];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int i = lane + 64 * r;
        if (r < RW) wv[r < RW ? r : 0] = i < W ? w[i] : 0.0f;
        p[r] = 0.0f;
    }
    // window samples of transform t (unweighted); the next transform's are
    // loaded while this one is transformed
    // x through a range-checked buffer descriptor (32-bit offsets, no
    // per-sample branches: the register budget of the prefetch); the history
    // only feeds the first transforms of a call
    constexpr int ES = (int)sizeof(S);
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)((elast + 1) * ES), 0x00020000);
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void *)hist, (short)0, W * ES, 0x00020000);
    auto gather = [&](long long t, float2 (&u)[RW]) {
        const long long j0 = ((t == T - 1) ? elast : e0 + t * hop) + 1;   // ext index of window sample 0
        if (j0 >= W) {   // all from x (every transform but the first few of a call)
            const int b = (int)(j0 - W);
#pragma unroll
            for (int r = 0; r < RW; r++) {
                const int i = lane + 64 * r;
                const unsigned o = i < W ? (unsigned)(b + i) * ES : 0xFFFFFFF0u;
                if constexpr (ES == 8)
                    u[r] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, o, 0, 0));
                else
                    u[r] = make_float2(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, o, 0, 0)), 0.f);
            }
        } else {   // sample j < W from the history, else x[j - W]: one of the two loads is in range
            const int b = (int)j0;
#pragma unroll
            for (int r = 0; r < RW; r++) {
                const int i = lane + 64 * r, j = b + i;
                const unsigned oh = i < W ? (unsigned)j * ES : 0xFFFFFFF0u;
                const unsigned ox = i < W ? (unsigned)(j - W) * ES : 0xFFFFFFF0u;
                if constexpr (ES == 8) {
                    const float2 a = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rh, oh, 0, 0));
                    const float2 c = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, ox, 0, 0));
                    u[r] = make_float2(a.x + c.x, a.y + c.y);
                } else {
                    u[r] = make_float2(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rh, oh, 0, 0)) +
                                           __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, ox, 0, 0)),
                                       0.f);
                }
            }
        }
    };
    float2 nx[RW];
    gather(t0, nx);
    for (long long t = t0; t < t1; t++) {
        float2 v[16];
#pragma unroll
        for (int r = 0; r < 16; r++)
            v[r] = r < RW ? make_float2(nx[r < RW ? r : 0].x * wv[r < RW ? r : 0], nx[r < RW ? r : 0].y * wv[r < RW ? r : 0])
                          : make_float2(0.0f, 0.0f);
        if (t + 1 < t1) gather(t + 1, nx);
        fft1024_wave<+1>(v, B, tw1, tw2, lane);
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const float pw = pwr(B[lane + 64 * r + 4 * (r >> 2)]);
            p[r] = accum ? (1.0f - alpha) * p[r] + alpha * pw : p[r] + pw;
        }
        f1k_wave_fence();   // B is rewritten by the next transform
    }
#pragma unroll
    for (int r = 0; r < 16; r++) part[chunk * 1024 + lane + 64 * r] = p[r];
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

constexpr long long SPG_G = 64;   // chunks per first-level fold group

extern "C" size_t lqk_spgram_work_bytes(unsigned long long T, unsigned int nfft)
{
    const unsigned long long nch = (T + SPG_TC - 1) / SPG_TC;
    return (size_t)(nch + (nch + SPG_G - 1) / SPG_G) * nfft * sizeof(float);
}

// fold the chunk values in work (nch x nfft) into dst: directly when few,
// else through groups of SPG_G chunks (both levels spread over the chip)
static void spg_fold(unsigned long long T, unsigned int nfft, int accum, float alpha, float *dst, void *work,
                     hipStream_t st)
{
    const long long nch = (long long)((T + SPG_TC - 1) / SPG_TC);
    const unsigned gx = (nfft + NT - 1) / NT;
    const float *part = (const float *)work;
    if (nch <= SPG_G) {
        hipLaunchKernelGGL(k_spg_fold, dim3(gx), dim3(NT), 0, st, part, (long long)T, (long long)SPG_TC, (int)nfft,
                           accum, alpha, nch, (float *)nullptr, dst);
        LQ_CHECK_LAUNCH();
        return;
    }
    const long long ng = (nch + SPG_G - 1) / SPG_G;
    float *part2 = (float *)work + nch * nfft;
    hipLaunchKernelGGL(k_spg_fold, dim3(gx, (unsigned)ng), dim3(NT), 0, st, part, (long long)T, (long long)SPG_TC,
                       (int)nfft, accum, alpha, (long long)SPG_G, part2, (float *)nullptr);
    LQ_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_spg_fold, dim3(gx), dim3(NT), 0, st, (const float *)part2, (long long)T,
                       (long long)SPG_TC * SPG_G, (int)nfft, accum, alpha, ng, (float *)nullptr, dst);
    LQ_CHECK_LAUNCH();
}

static void spg_reduce(const void *X, unsigned long long T, unsigned int nfft, int accum, float alpha, float *dst,
                       void *work, void *stream)
{
    if (T == 0) return;
    const unsigned nch = (unsigned)((T + SPG_TC - 1) / SPG_TC);
    const unsigned gx = (nfft + NT - 1) / NT;
    hipLaunchKernelGGL(k_spg_part, dim3(gx, nch), dim3(NT), 0, (hipStream_t)stream, (const float2 *)X, (long long)T,
                       (int)nfft, accum, alpha, (float *)work);
    LQ_CHECK_LAUNCH();
    spg_fold(T, nfft, accum, alpha, dst, work, (hipStream_t)stream);
}

extern "C" void lqk_spgram_accumulate(const void *X, unsigned long long T, unsigned int nfft, float alpha, float *psd,
                                      void *work, void *stream)
{
    spg_reduce(X, T, nfft, 1, alpha, psd, work, stream);
}

extern "C" void lqk_spgram_sum(const void *X, unsigned long long T, unsigned int nfft, float *acc, void *work,
                               void *stream)
{
    spg_reduce(X, T, nfft, 0, 0.0f, acc, work, stream);
}

extern "C" void lqk_spgram_fused1024(int real_in, const void *hist, unsigned int W, const void *x, long long e0,
                                     long long hop, unsigned long long T, long long elast, const float *w, int accum,
                                     float alpha, float *dst, void *work, void *stream)
{
    if (T == 0) return;
    const unsigned nch = (unsigned)((T + SPG_TC - 1) / SPG_TC);
    const unsigned nwg = (nch + NT / 64 - 1) / (NT / 64);
    const float2 *tw = (const float2 *)lqrt_twiddles();
    // W <= 512: the zero half of each window is neither loaded nor weighted
    // (0.427-0.451 -> 0.410-0.424 ms per 2^26 inputs, identical output; r05zr)
    const bool half = W <= 512;
    if (real_in)
        hipLaunchKernelGGL((half ? k_spg_fused1024<float, true> : k_spg_fused1024<float, false>), dim3(nwg), dim3(NT),
                           0, (hipStream_t)stream, (const float *)hist, (int)W, (const float *)x, e0, hop,
                           (long long)T, elast, w, accum, alpha, tw, (float *)work);
    else
        hipLaunchKernelGGL((half ? k_spg_fused1024<float2, true> : k_spg_fused1024<float2, false>), dim3(nwg),
                           dim3(NT), 0, (hipStream_t)stream, (const float2 *)hist, (int)W, (const float2 *)x, e0, hop,
                           (long long)T, elast, w, accum, alpha, tw, (float *)work);
    LQ_CHECK_LAUNCH();
    spg_fold(T, 1024, accum, alpha, dst, work, (hipStream_t)stream);
}

extern "C" void lqk_spgram_db(int mode, const void *X, const float *v, unsigned int nfft, float T, float *out,
                              void *stream)
{
    hipLaunchKernelGGL(k_spg_db, dim3((nfft + NT - 1) / NT), dim3(NT), 0, (hipStream_t)stream, mode,
                       (const float2 *)X, v, (int)nfft, T, out);
    LQ_CHECK_LAUNCH();
}
