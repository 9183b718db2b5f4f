// k_channelizer.hip -- polyphase channelizers (firpfbch2 2x-oversampled and
// firpfbch critically sampled, analyzers and synthesizers) and the batched
// LDS FFT they share.
//
// Reference semantics restated, not translated:
//  firpfbch2 analyzer  src/multichannel/src/firpfbch2.c:244-282.  The
//    reference pushes M/2 samples per call into M ring buffers and runs M
//    dot products then an M-point IFFT.  Here block b is evaluated from the
//    stream directly (closed form, SURVEY Appendix B, checked numerically):
//        off = (b&1)*M/2,  i = (j - off) mod M
//        c   = j < M/2 ? b>>1 : (b-1)>>1,  base = j < M/2 ? M/2-1-j : 3M/2-1-j
//        X_b[j] = sum_{n<2m} h[i + nM] x[(c-n)M + base]
//        Y_b    = IFFT_backward(X_b) / M
//    so any number of blocks run in parallel; the only state carried between
//    calls is the last 2mM - M/2 input samples and the block parity.
//  firpfbch2 synthesizer firpfbch2.c:287-335: z_b = IFFT(X_b)*(1/M)*(M/2);
//        y_b[i] = sum_n h[i+nM] z_{b-2n}[i+fM/2] + sum_n h[i+M/2+nM] z_{b-1-2n}[i+fM/2]
//    (f = b&1); state = the last 4m-1 z vectors.
//  firpfbch analyzer src/multichannel/src/firpfbch.c:346-409:
//        X_b[j] = sum_{n<p} h[(M-1-j) + nM] x[(b-n)M + j],  Y_b = FFT_forward(X_b)
//  firpfbch synthesizer firpfbch.c:314-336: z_b = IFFT(X_b),
//        y_b[i] = sum_{n<p} h[i+nM] z_{b-n}[i]
#include "lq_device.h"
#include "lq_kernels.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float2 ext_load(const float2 *__restrict__ hist, int HL, const float2 *__restrict__ x,
                                           long long t)
{
    return t < 0 ? hist[HL + t] : x[t];
}

// ------------------------------------------------------------------ firpfbch2 analyzer
// One workgroup = NB consecutive blocks; X for all NB blocks is formed in LDS,
// transformed by the LDS Stockham FFT, scaled and stored coalesced.
template <int M, int NB>
__global__ __launch_bounds__(NT) void k_pfb2_an(int m, const float *__restrict__ hsub,
                                                const float2 *__restrict__ hist, const float2 *__restrict__ x,
                                                long long nblocks, int p0, float2 *__restrict__ Y,
                                                const float2 *__restrict__ tw)
{
    __shared__ __attribute__((aligned(16))) float2 a[NB * M];
    __shared__ __attribute__((aligned(16))) float2 b[NB * M];
    constexpr int M2 = M / 2;
    const int L = 2 * m;
    const int HL = 2 * m * M - M2;
    const long long blk0 = (long long)blockIdx.x * NB;

    for (int e = threadIdx.x; e < NB * M; e += NT) {
        const int bl = e / M;
        const int j = e - bl * M;
        const long long gb = blk0 + bl;
        float2 acc = make_float2(0.f, 0.f);
        if (gb < nblocks) {
            const long long bt = p0 + gb;
            const int off = (int)(bt & 1) * M2;
            const int i = (j - off) & (M - 1);
            const long long c = (j < M2) ? (bt >> 1) : ((bt - 1) >> 1);
            const int base = (j < M2) ? (M2 - 1 - j) : (3 * M2 - 1 - j);
            const long long t0 = c * M + base - (long long)p0 * M2;
            const float *hs = hsub + i * L;
            for (int n = 0; n < L; n++) {
                const float2 v = ext_load(hist, HL, x, t0 - (long long)n * M);
                acc.x = fmaf(hs[n], v.x, acc.x);
                acc.y = fmaf(hs[n], v.y, acc.y);
            }
        }
        a[e] = acc;
    }
    __syncthreads();
    float2 *res = lds_fft<M, NB, NT>(a, b, tw, -1);
    const float inv = 1.0f / (float)M; // exact: M is a power of two
    for (int e = threadIdx.x; e < NB * M; e += NT) {
        const int bl = e / M;
        const long long gb = blk0 + bl;
        if (gb < nblocks) Y[(blk0 + bl) * M + (e - bl * M)] = cscale(res[e], inv);
    }
}

// generic even M (not a power of two): direct O(M^2) DFT, one workgroup per block
__global__ __launch_bounds__(NT) void k_pfb2_an_generic(int M, int m, const float *__restrict__ hsub,
                                                        const float2 *__restrict__ hist,
                                                        const float2 *__restrict__ x, long long nblocks, int p0,
                                                        float2 *__restrict__ Y)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2 *X = reinterpret_cast<float2 *>(smem);
    const int M2 = M / 2, L = 2 * m, HL = 2 * m * M - M2;
    const long long gb = blockIdx.x;
    const long long bt = p0 + gb;
    for (int j = threadIdx.x; j < M; j += NT) {
        const int off = (int)(bt & 1) * M2;
        const int i = ((j - off) % M + M) % M;
        const long long c = (j < M2) ? (bt >> 1) : ((bt - 1) >> 1);
        const int base = (j < M2) ? (M2 - 1 - j) : (3 * M2 - 1 - j);
        const long long t0 = c * M + base - (long long)p0 * M2;
        float2 acc = make_float2(0.f, 0.f);
        for (int n = 0; n < L; n++) {
            const float2 v = ext_load(hist, HL, x, t0 - (long long)n * M);
            acc.x = fmaf(hsub[i * L + n], v.x, acc.x);
            acc.y = fmaf(hsub[i * L + n], v.y, acc.y);
        }
        X[j] = acc;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < M; k += NT) {
        float2 acc = make_float2(0.f, 0.f);
        for (int j = 0; j < M; j++) {
            double s, co;
            sincospi(2.0 * (double)(((long long)j * k) % M) / (double)M, &s, &co);
            acc = cadd(acc, cmul(X[j], make_float2((float)co, (float)s)));
        }
        Y[gb * M + k] = make_float2(acc.x / (float)M, acc.y / (float)M);
    }
}

// ------------------------------------------------------------------ batched FFT
// y[b] = FFT_dir(x[b]) * s1 * s2 (two separate roundings, as the reference
// synthesizer scales twice: firpfbch2.c:303-307); s == 1 skips the multiply.
template <int N, int NB>
__global__ __launch_bounds__(NT) void k_fft_batch(const float2 *__restrict__ x, float2 *__restrict__ y,
                                                  long long batch, int dir, float s1, float s2, int use_s1,
                                                  int use_s2, const float2 *__restrict__ tw)
{
    __shared__ __attribute__((aligned(16))) float2 a[NB * N];
    __shared__ __attribute__((aligned(16))) float2 b[NB * N];
    const long long b0 = (long long)blockIdx.x * NB;
    for (int e = threadIdx.x; e < NB * N; e += NT) {
        const long long gb = b0 + e / N;
        a[e] = gb < batch ? x[b0 * N + e] : make_float2(0.f, 0.f);
    }
    __syncthreads();
    float2 *res = lds_fft<N, NB, NT>(a, b, tw, dir);
    for (int e = threadIdx.x; e < NB * N; e += NT) {
        const long long gb = b0 + e / N;
        if (gb >= batch) continue;
        float2 v = res[e];
        if (use_s1) v = cscale(v, s1);
        if (use_s2) v = cscale(v, s2);
        y[b0 * N + e] = v;
    }
}

// direct DFT for non power-of-two sizes (small M channelizers)
__global__ void k_dft_batch(int N, const float2 *__restrict__ x, float2 *__restrict__ y, long long batch, int dir,
                            float s1, float s2, int use_s1, int use_s2)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2 *xb = reinterpret_cast<float2 *>(smem); // staged: x may alias y
    const long long gb = blockIdx.x;
    for (int j = threadIdx.x; j < N; j += blockDim.x) xb[j] = x[gb * N + j];
    __syncthreads();
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        float2 acc = make_float2(0.f, 0.f);
        for (int j = 0; j < N; j++) {
            double s, c;
            sincospi(-2.0 * dir * (double)(((long long)j * k) % N) / (double)N, &s, &c);
            acc = cadd(acc, cmul(xb[j], make_float2((float)c, (float)s)));
        }
        if (use_s1) acc = cscale(acc, s1);
        if (use_s2) acc = cscale(acc, s2);
        y[gb * N + k] = acc;
    }
}

// ------------------------------------------------------------------ firpfbch2 synthesizer output
// Z holds [4m-1 history z vectors | nblocks new z vectors], each M long.
__global__ void k_pfb2_syn_out(int M, int m, const float *__restrict__ hsub, const float2 *__restrict__ Z,
                               long long nblocks, int p0, float2 *__restrict__ y)
{
    const int M2 = M / 2, L = 2 * m, HB = 4 * m - 1;
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nblocks * M2) return;
    const long long bl = e / M2;
    const int i = (int)(e - bl * M2);
    const int f = (int)((p0 + bl) & 1);
    const int col = i + f * M2;
    const long long zb = HB + bl; // index of z_b in Z
    float2 acc0 = make_float2(0.f, 0.f), acc1 = make_float2(0.f, 0.f);
    for (int n = 0; n < L; n++) {
        const float h0 = hsub[i * L + n];
        const float h1 = hsub[(i + M2) * L + n];
        const float2 z0 = Z[(zb - 2 * n) * M + col];
        const float2 z1 = Z[(zb - 1 - 2 * n) * M + col];
        acc0.x = fmaf(h0, z0.x, acc0.x);
        acc0.y = fmaf(h0, z0.y, acc0.y);
        acc1.x = fmaf(h1, z1.x, acc1.x);
        acc1.y = fmaf(h1, z1.y, acc1.y);
    }
    y[bl * M2 + i] = cadd(acc0, acc1);
}

// ------------------------------------------------------------------ firpfbch analyzer (X build)
// tap x sample: real taps (crcf) or complex taps (cccf, no conjugation, as dotprod_cccf)
__device__ __forceinline__ float2 pfb_mac(float h, float2 v, float2 a)
{
    return make_float2(fmaf(h, v.x, a.x), fmaf(h, v.y, a.y));
}
__device__ __forceinline__ float2 pfb_mac(float2 h, float2 v, float2 a)
{
    return make_float2(fmaf(h.x, v.x, fmaf(-h.y, v.y, a.x)), fmaf(h.x, v.y, fmaf(h.y, v.x, a.y)));
}

template <typename TC>
__global__ void k_pfb_an_X(int M, int p, const TC *__restrict__ hsub, const float2 *__restrict__ hist,
                           const float2 *__restrict__ x, long long nblocks, float2 *__restrict__ X)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nblocks * M) return;
    const long long b = e / M;
    const int j = (int)(e - b * M);
    const int i = M - 1 - j;
    const int HL = (p - 1) * M;
    float2 acc = make_float2(0.f, 0.f);
    for (int n = 0; n < p; n++) {
        const float2 v = ext_load(hist, HL, x, (b - n) * M + j);
        acc = pfb_mac(hsub[i * p + n], v, acc);
    }
    X[e] = acc;
}

// firpfbch synthesizer output: Z = [p-1 history z | nblocks new z]
template <typename TC>
__global__ void k_pfb_syn_out(int M, int p, const TC *__restrict__ hsub, const float2 *__restrict__ Z,
                              long long nblocks, float2 *__restrict__ y)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nblocks * M) return;
    const long long b = e / M;
    const int i = (int)(e - b * M);
    const long long zb = (p - 1) + b;
    float2 acc = make_float2(0.f, 0.f);
    for (int n = 0; n < p; n++) {
        acc = pfb_mac(hsub[i * p + n], Z[(zb - n) * M + i], acc);
    }
    y[e] = acc;
}

template <int M>
void launch_pfb2_an(int m, const void *hsub, const void *hist, const void *x, long long nblocks, int p0, void *Y,
                    hipStream_t st)
{
    constexpr int NB = M >= 1024 ? 1 : 1024 / M;
    const long long grid = (nblocks + NB - 1) / NB;
    hipLaunchKernelGGL((k_pfb2_an<M, NB>), dim3((unsigned)grid), dim3(NT), 0, st, m, (const float *)hsub,
                       (const float2 *)hist, (const float2 *)x, nblocks, p0, (float2 *)Y,
                       (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}

template <int N>
void launch_fft_batch(const void *x, void *y, long long batch, int dir, float s1, float s2, int u1, int u2,
                      hipStream_t st)
{
    constexpr int NB = N >= 1024 ? 1 : 1024 / N;
    const long long grid = (batch + NB - 1) / NB;
    hipLaunchKernelGGL((k_fft_batch<N, NB>), dim3((unsigned)grid), dim3(NT), 0, st, (const float2 *)x,
                       (float2 *)y, batch, dir, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}

int is_pow2(unsigned v) { return v && !(v & (v - 1)); }

void fft_batch_scaled(unsigned n, int dir, const void *x, void *y, long long batch, float s1, float s2, int u1,
                      int u2, hipStream_t st)
{
    if (batch <= 0) return;
    switch (n) {
    case 2: launch_fft_batch<2>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 4: launch_fft_batch<4>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 8: launch_fft_batch<8>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 16: launch_fft_batch<16>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 32: launch_fft_batch<32>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 64: launch_fft_batch<64>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 128: launch_fft_batch<128>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 256: launch_fft_batch<256>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 512: launch_fft_batch<512>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 1024: launch_fft_batch<1024>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 2048: launch_fft_batch<2048>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 4096: launch_fft_batch<4096>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    default:
        break;
    }
    if (n == 1) {
        hipLaunchKernelGGL(k_dft_batch, dim3((unsigned)batch), dim3(64), 16, st, 1, (const float2 *)x, (float2 *)y,
                           batch, dir, s1, s2, u1, u2);
        LQ_CHECK_LAUNCH();
        return;
    }
    if (n > 8192) {
        fprintf(stderr, "error: liquid-mi355x: non power-of-two transform size %u not supported\n", n);
        exit(1);
    }
    hipLaunchKernelGGL(k_dft_batch, dim3((unsigned)batch), dim3(256), (size_t)n * sizeof(float2), st, (int)n, (const float2 *)x,
                       (float2 *)y, batch, dir, s1, s2, u1, u2);
    LQ_CHECK_LAUNCH();
}

} // namespace

extern "C" void lqk_fft_batch(unsigned int n, int dir, const void *x, void *y, unsigned long long batch,
                              void *stream)
{
    fft_batch_scaled(n, dir, x, y, (long long)batch, 1.f, 1.f, 0, 0, (hipStream_t)stream);
}

extern "C" void lqk_firpfbch2_analyzer(unsigned int M, unsigned int m, const void *hsub, const void *hist,
                                       const void *x, unsigned long long nblocks, int p0, void *Y, void *stream)
{
    if (nblocks == 0) return;
    hipStream_t st = (hipStream_t)stream;
    const long long nb = (long long)nblocks;
    switch (M) {
    case 2: launch_pfb2_an<2>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 4: launch_pfb2_an<4>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 8: launch_pfb2_an<8>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 16: launch_pfb2_an<16>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 32: launch_pfb2_an<32>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 64: launch_pfb2_an<64>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 128: launch_pfb2_an<128>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 256: launch_pfb2_an<256>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 512: launch_pfb2_an<512>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 1024: launch_pfb2_an<1024>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 2048: launch_pfb2_an<2048>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 4096: launch_pfb2_an<4096>(m, hsub, hist, x, nb, p0, Y, st); return;
    default:
        break;
    }
    const size_t lds = (size_t)M * sizeof(float2);
    if (lds > 64 * 1024) {
        fprintf(stderr, "error: firpfbch2: %u channels not supported on the GPU path\n", M);
        exit(1);
    }
    hipLaunchKernelGGL(k_pfb2_an_generic, dim3((unsigned)nb), dim3(NT), lds, st, (int)M, (int)m,
                       (const float *)hsub, (const float2 *)hist, (const float2 *)x, nb, p0, (float2 *)Y);
    LQ_CHECK_LAUNCH();
}

// state: the previous 4m-1 z vectors (M each); zscratch: (4m-1 + nblocks)*M.
extern "C" void lqk_firpfbch2_synthesizer(unsigned int M, unsigned int m, const void *hsub, void *state,
                                          void *zscratch, const void *X, unsigned long long nblocks, int p0,
                                          void *Y, void *stream)
{
    if (nblocks == 0) return;
    hipStream_t st = (hipStream_t)stream;
    const long long HB = 4 * (long long)m - 1;
    float2 *Z = (float2 *)zscratch;
    LQ_CHECK(hipMemcpyAsync(Z, state, HB * M * sizeof(float2), hipMemcpyDeviceToDevice, st));
    fft_batch_scaled(M, -1, X, Z + HB * M, (long long)nblocks, 1.0f / (float)M, (float)(M / 2), 1, 1, st);
    const long long tot = (long long)nblocks * (M / 2);
    hipLaunchKernelGGL(k_pfb2_syn_out, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (int)M, (int)m,
                       (const float *)hsub, (const float2 *)Z, (long long)nblocks, p0, (float2 *)Y);
    LQ_CHECK_LAUNCH();
    // keep the newest HB z vectors as the state for the next call
    LQ_CHECK(hipMemcpyAsync(state, Z + (long long)nblocks * M, HB * M * sizeof(float2), hipMemcpyDeviceToDevice,
                            st));
}

extern "C" void lqk_firpfbch_analyzer(int ctaps, unsigned int M, unsigned int p, const void *hsub, const void *hist,
                                      const void *x, unsigned long long nblocks, void *Y, void *stream)
{
    if (nblocks == 0) return;
    hipStream_t st = (hipStream_t)stream;
    const long long tot = (long long)nblocks * M;
    const dim3 grid((unsigned)((tot + 255) / 256));
    // X is formed in Y then transformed in place
    if (ctaps)
        hipLaunchKernelGGL(k_pfb_an_X<float2>, grid, dim3(256), 0, st, (int)M, (int)p, (const float2 *)hsub,
                           (const float2 *)hist, (const float2 *)x, (long long)nblocks, (float2 *)Y);
    else
        hipLaunchKernelGGL(k_pfb_an_X<float>, grid, dim3(256), 0, st, (int)M, (int)p, (const float *)hsub,
                           (const float2 *)hist, (const float2 *)x, (long long)nblocks, (float2 *)Y);
    LQ_CHECK_LAUNCH();
    fft_batch_scaled(M, +1, Y, Y, (long long)nblocks, 1.f, 1.f, 0, 0, st);
}

// state: the previous p-1 z vectors; zscratch: (p-1 + nblocks)*M
extern "C" void lqk_firpfbch_synthesizer(int ctaps, unsigned int M, unsigned int p, const void *hsub, void *state,
                                         void *zscratch, const void *X, unsigned long long nblocks, void *y,
                                         void *stream)
{
    if (nblocks == 0) return;
    hipStream_t st = (hipStream_t)stream;
    const long long HB = (long long)p - 1;
    float2 *Z = (float2 *)zscratch;
    if (HB > 0) LQ_CHECK(hipMemcpyAsync(Z, state, HB * M * sizeof(float2), hipMemcpyDeviceToDevice, st));
    fft_batch_scaled(M, -1, X, Z + HB * M, (long long)nblocks, 1.f, 1.f, 0, 0, st);
    const long long tot = (long long)nblocks * M;
    const dim3 grid((unsigned)((tot + 255) / 256));
    if (ctaps)
        hipLaunchKernelGGL(k_pfb_syn_out<float2>, grid, dim3(256), 0, st, (int)M, (int)p, (const float2 *)hsub,
                           (const float2 *)Z, (long long)nblocks, (float2 *)y);
    else
        hipLaunchKernelGGL(k_pfb_syn_out<float>, grid, dim3(256), 0, st, (int)M, (int)p, (const float *)hsub,
                           (const float2 *)Z, (long long)nblocks, (float2 *)y);
    LQ_CHECK_LAUNCH();
    if (HB > 0)
        LQ_CHECK(hipMemcpyAsync(state, Z + (long long)nblocks * M, HB * M * sizeof(float2),
                                hipMemcpyDeviceToDevice, st));
}
