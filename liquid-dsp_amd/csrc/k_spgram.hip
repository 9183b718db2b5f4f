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

// First radix-4 stage of pk_dft16 for inputs v[8..15] = 0 (a window of at
// most 512 samples): each column's butterfly has two zero inputs.  The
// results equal pk_dft16's but for the sign of zero terms, which |X|^2 does
// not see.
template <int DIR>
__device__ __forceinline__ void pk_dft16_h(v2f (&v)[16])
{
    constexpr float C[16] = {1.0f,         0.92387953f,  0.70710678f,  0.38268343f,  0.0f,        -0.38268343f,
                             -0.70710678f, -0.92387953f, -1.0f,        -0.92387953f, -0.70710678f, -0.38268343f,
                             0.0f,         0.38268343f,  0.70710678f,  0.92387953f};
    constexpr float S[16] = {0.0f,  0.38268343f,  0.70710678f,  0.92387953f,  1.0f,         0.92387953f,
                             0.70710678f,  0.38268343f,  0.0f,  -0.38268343f, -0.70710678f, -0.92387953f,
                             -1.0f, -0.92387953f, -0.70710678f, -0.38268343f};
    v2f t[16];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const v2f b = v[q], d = v[4 + q];
        const v2f a0 = b + d, a2 = b - d;
        const v2f a1 = DIR > 0 ? pk_subpj(b, d) : pk_addpj(b, d);
        const v2f a3 = DIR > 0 ? pk_addpj(b, d) : pk_subpj(b, d);
        t[q] = a0;
        t[4 + q] = q == 0 ? a1 : pk_cmulk(a1, v2f{C[q], -DIR * S[q]});
        t[8 + q] = (q == 0 || q == 2) ? a2 : pk_cmulk(a2, v2f{C[2 * q], -DIR * S[2 * q]});
        t[12 + q] = q == 0 ? a3 : pk_cmulk(a3, v2f{C[(3 * q) & 15], -DIR * S[(3 * q) & 15]});
    }
#pragma unroll
    for (int k0 = 0; k0 < 4; k0++) {
        v2f b0 = t[4 * k0 + 0], b1 = t[4 * k0 + 1], b2 = t[4 * k0 + 2], b3 = t[4 * k0 + 3];
        if (k0 == 2) {
            const v2f a = DIR > 0 ? pk_subpj(b0, b2) : pk_addpj(b0, b2);
            const v2f b = DIR > 0 ? pk_addpj(b0, b2) : pk_subpj(b0, b2);
            const v2f c = b1 + b3, d = b1 - b3;
            b0 = a + c;
            b2 = a - c;
            b1 = DIR > 0 ? pk_subpj(b, d) : pk_addpj(b, d);
            b3 = DIR > 0 ? pk_addpj(b, d) : pk_subpj(b, d);
        } else {
            pk_dft4<DIR>(b0, b1, b2, b3);
        }
        v[k0] = b0;
        v[k0 + 4] = b1;
        v[k0 + 8] = b2;
        v[k0 + 12] = b3;
    }
}

// nfft = 1024, fused: one wave per chunk of SPG_TC consecutive transforms
// gathers each window straight from (hist | x) into registers, runs the
// wave-level 1024-point transform (the lq_fft1024.h transform, forward) and
// folds |X[k]|^2 into per-lane partials -- no transform batch staged through
// HBM.  Transform t ends at e0 + t*hop (the last one at elast).  Writes
// part[chunk][k] for k_spg_fold, exactly as k_spg_part does.
//  * Only |X[k]|^2 per bin is needed, in transform order per bin, and which
//    lane owns which bin is free: the last radix-4 pass leaves lane (t2, p2)
//    the bins K = 2 p2 + e + 16 (t2 + 8 u) + 256 s (e, u < 2, s < 4), so the
//    partials accumulate there, in registers -- no write-back of the spectrum
//    through LDS and no re-read in natural order;
//  * TR: the first pass's twiddles W_1024^{lane k1} stay in registers (30
//    VGPRs, loaded once), so a transform reads LDS only for its two
//    transposes and the 4-entry second-pass twiddles (complex input with a
//    window of <= 512 samples; the other forms read the LDS table: their
//    register windows leave no room);
//  (0.365 -> 0.303 ms per 2^26 samples at nfft = 1024, W = 512; with the
//  LDS twiddle table 0.315: profiles/r06_ab_experiments.txt, r06g)
//  * HALF: W <= 512, so window samples r >= 8 of a lane (i = lane + 64 r)
//    are zero: neither loaded nor weighted, and the first radix-4 stage runs
//    on the eight nonzero rows (pk_dft16_h).
template <typename S, bool HALF, bool TR>
__global__ __launch_bounds__(NT, 3) void k_spg_fused1024(const S *__restrict__ hist, int W, const S *__restrict__ x,
                                                      long long e0, long long hop, long long T, long long elast,
                                                      const float *__restrict__ w, int accum, float alpha,
                                                      const float2 *__restrict__ tw4096, float *__restrict__ part)
{
#pragma clang fp contract(off)
    __shared__ __attribute__((aligned(16))) float2 tw1[TR ? 1 : 1024];
    __shared__ __attribute__((aligned(16))) float2 tw2[64];
    __shared__ __attribute__((aligned(16))) float2 Bs[NT / 64][1088];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v2f T1[15];   // TR: W_1024^{lane k1}, k1 = 1..15 (forward: the table's own sign)
    if constexpr (TR) {
        if (threadIdx.x < 64) {
            const int r = threadIdx.x >> 2, b = threadIdx.x & 3;
            tw2[threadIdx.x] = tw4096[(64 * b * r) & 4095];   // W_64^{b r}, forward
        }
#pragma unroll
        for (int k1 = 1; k1 < 16; k1++) T1[k1 - 1] = pk(tw4096[(4 * lane * k1) & 4095]);
    } else {
        f1k_tables<+1>(tw1, tw2, tw4096);
    }
    __syncthreads();
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
    const int k1 = lane >> 2, bq = lane & 3;     // second pass: lane (k1, bq)
    const int t2 = lane >> 3, p2 = lane & 7;     // last pass: lane (t2, p2)
    typedef float v4f __attribute__((ext_vector_type(4)));
    for (long long t = t0; t < t1; t++) {
        v2f v[16];
#pragma unroll
        for (int r = 0; r < 16; r++)
            v[r] = r < RW ? v2f{nx[r < RW ? r : 0].x * wv[r < RW ? r : 0], nx[r < RW ? r : 0].y * wv[r < RW ? r : 0]}
                          : v2f{0.0f, 0.0f};
        if (t + 1 < t1) gather(t + 1, nx);
        // 1024 = 16 x 16 x 4 (lq_fft1024.h's fft1024_wave, forward)
        if constexpr (HALF) pk_dft16_h<+1>(v);
        else pk_dft16<+1>(v);
#pragma unroll
        for (int k = 1; k < 16; k++) v[k] = pk_cmul(v[k], TR ? T1[k - 1] : pk(tw1[k * 64 + lane]));
        f1k_wave_fence();
#pragma unroll
        for (int k = 0; k < 16; k++) B[k * 68 + lane] = unpk(v[k]);
        f1k_wave_fence();
#pragma unroll
        for (int a = 0; a < 16; a++) v[a] = pk(B[k1 * 68 + 4 * a + bq]);
        pk_dft16<+1>(v);
#pragma unroll
        for (int r = 1; r < 16; r++) v[r] = pk_cmul(v[r], pk(tw2[r * 4 + bq]));
        f1k_wave_fence();
#pragma unroll
        for (int r = 0; r < 16; r++) B[k1 + 16 * r + 260 * bq] = unpk(v[r]);
        f1k_wave_fence();
#pragma unroll
        for (int u = 0; u < 2; u++) {
            v4f c[4];
#pragma unroll
            for (int q = 0; q < 4; q++)
                c[q] = *reinterpret_cast<const v4f *>(B + 2 * p2 + 16 * (t2 + 8 * u) + 260 * q);
            v2f e0[4] = {c[0].xy, c[1].xy, c[2].xy, c[3].xy};
            v2f e1[4] = {c[0].zw, c[1].zw, c[2].zw, c[3].zw};
            pk_dft4<+1>(e0[0], e0[1], e0[2], e0[3]);
            pk_dft4<+1>(e1[0], e1[1], e1[2], e1[3]);
            // bins 2 p2 + {0, 1} + 16 (t2 + 8 u) + 256 s -> p[8 u + 2 s + {0, 1}]
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const float pa = pwr(unpk(e0[s])), pb = pwr(unpk(e1[s]));
                float &qa = p[8 * u + 2 * s], &qb = p[8 * u + 2 * s + 1];
                qa = accum ? (1.0f - alpha) * qa + alpha * pa : qa + pa;
                qb = accum ? (1.0f - alpha) * qb + alpha * pb : qb + pb;
            }
        }
        f1k_wave_fence();   // B is rewritten by the next transform
    }
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
        for (int s = 0; s < 4; s++)
            *reinterpret_cast<float2 *>(part + chunk * 1024 + 2 * p2 + 16 * (t2 + 8 * u) + 256 * s) =
                make_float2(p[8 * u + 2 * s], p[8 * u + 2 * s + 1]);
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
        hipLaunchKernelGGL((half ? k_spg_fused1024<float, true, false> : k_spg_fused1024<float, false, false>),
                           dim3(nwg), dim3(NT), 0, (hipStream_t)stream, (const float *)hist, (int)W, (const float *)x,
                           e0, hop, (long long)T, elast, w, accum, alpha, tw, (float *)work);
    else
        hipLaunchKernelGGL((half ? k_spg_fused1024<float2, true, true> : k_spg_fused1024<float2, false, false>),
                           dim3(nwg), dim3(NT), 0, (hipStream_t)stream, (const float2 *)hist, (int)W,
                           (const float2 *)x, e0, hop, (long long)T, elast, w, accum, alpha, tw, (float *)work);
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
