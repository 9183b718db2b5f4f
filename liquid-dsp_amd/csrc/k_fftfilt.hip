// k_fftfilt.hip -- FFT fast convolution for fftfilt_{crcf,rrrf,cccf}.
// Kernel: k_fftfilt_r16 (register radix-16 transforms, persistent grid).
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
// k_fftfilt_r16 (tools/mb/mb_fftfilt.hip, h=512, 2^26 samples): with the
// packed transforms (lq_device.h) and buffer-descriptor loads / stores (no
// per-sample branches or 64-bit addresses) the kernel needs 128 VGPRs
// including the filter spectrum held in registers, so four waves per SIMD;
// 4096 persistent workgroups: 0.253 ms (float2 pointer loads with branches
// and ~220 VGPRs: 0.283 ms; a second, history, load for every segment
// instead of the first only: 0.367 ms).  Output stores are non-temporal
// (0.2503 vs 0.2538 ms default policy).
constexpr int FF_WPE = 4;        // resident workgroups per CU
constexpr int FF_STAUX = 2;      // store cache policy: non-temporal

__device__ __forceinline__ float2 to_c2(float a) { return make_float2(a, 0.f); }
__device__ __forceinline__ float2 to_c2(float2 a) { return a; }

// Register form: 256 threads, thread t holds segment samples
// t + 256 n; forward 4096-point FFT (fft4096_r16), x H, inverse, all with the
// data in registers and two LDS transposes per transform (35 KB LDS, four
// workgroups per CU); loads and stores are coalesced across t.
template <bool REAL>
__global__ __launch_bounds__(NT, FF_WPE) void k_fftfilt_r16(int hm1, const float2 *__restrict__ H,
                                                    const void *__restrict__ hist, const void *__restrict__ xin,
                                                    long long n, void *__restrict__ yout, float sre, float sim,
                                                    const float2 *__restrict__ tw)
{
    __shared__ __attribute__((aligned(16))) float2 lds[FFT4096_LDS];
    const int L = NFFT - hm1;
    const int t = threadIdx.x;
    const long long nseg = (n + L - 1) / L;
    // persistent: the filter spectrum stays in registers across segments
    float2 hv[16];
#pragma unroll
    for (int k = 0; k < 16; k++) hv[k] = H[t + 256 * k];
    using S = typename std::conditional<REAL, float, float2>::type;
    constexpr int ES = (int)sizeof(S);
    // range-checked buffer descriptors replace the per-sample branches (and
    // their 64-bit addresses): x (n samples), the history (hm1 samples just
    // before x) and y; an out-of-range load returns 0 and an out-of-range
    // store is dropped.  Byte offsets are 32-bit: the host keeps each launch
    // below 2^28 samples.
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)xin, (short)0, (int)(n * ES), 0x00020000);
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void *)hist, (short)0, hm1 * ES, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(yout, (short)0, (int)(n * ES), 0x00020000);
    const tw16x2 w16 = fft4096_tw(tw, t);   // the thread's twiddles, loaded once
    for (long long seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
    // segment sample i = t + 256 q is stream sample s0 - hm1 + i
    const int sb = (int)(seg * L) - hm1;   // stream index of segment sample 0
    float2 v[16];
    if (seg == 0) {   // the only segment that reaches into the history
#pragma unroll
        for (int q = 0; q < 16; q++) {
            // samples before x read 0 from an explicit out-of-range offset
            // (a variant of this loop that relied on the wrapped unsigned
            // (sb + i) * ES instead returned wrong rrrf outputs 0..hm1-1 on
            // the GPU; the 32-bit wrap of an offset-field sum itself is fine,
            // tools/mb/mb_bufwrap.hip, so the cause there stays unidentified)
            const int si = sb + t + 256 * q;
            const unsigned ox = si < 0 ? 0xFFFFFFF0u : (unsigned)si * ES, oh = (unsigned)(si + hm1) * ES;
            if constexpr (REAL) {
                const float a = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, ox, 0, 0)) +
                                __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rh, oh, 0, 0));
                v[q] = make_float2(a, 0.f);
            } else {
                const float2 a = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, ox, 0, 0));
                const float2 b = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rh, oh, 0, 0));
                v[q] = make_float2(a.x + b.x, a.y + b.y);
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const unsigned ox = (unsigned)(sb + t + 256 * q) * ES;
            if constexpr (REAL)
                v[q] = make_float2(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, ox, 0, 0)), 0.f);
            else
                v[q] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, ox, 0, 0));
        }
    }
    fft4096_r16<+1>(v, lds, w16, t);
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = unpk(pk_cmul(pk(v[k]), pk(hv[k])));
    fft4096_r16<-1>(v, lds, w16, t);
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int i = t + 256 * q;
        const unsigned oy = i < hm1 ? 0xFFFFFFF0u : (unsigned)(sb + i) * ES;   // first hm1 outputs: discarded
        const float2 r = v[q];
        if constexpr (REAL) {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, r.x * sre), ry, oy, 0, FF_STAUX);
        } else {
            const float2 o = make_float2(r.x * sre - r.y * sim, r.x * sim + r.y * sre);
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), ry, oy, 0, FF_STAUX);
        }
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
    const float2 *tw = (const float2 *)lqrt_twiddles();
    const size_t es = real_io ? 4 : 8;
    // launches of at most 2^27 samples (32-bit buffer offsets); later chunks
    // take their history straight from the preceding input
    const unsigned long long CHN = 1ull << 27;
    for (unsigned long long c0 = 0; c0 < n; c0 += CHN) {
        const unsigned long long nc = (n - c0) < CHN ? (n - c0) : CHN;
        const char *xc = (const char *)x + c0 * es;
        const void *hc = c0 == 0 ? hist : (const void *)(xc - (size_t)hm1 * es);
        void *yc = (char *)y + c0 * es;
        const long long nsegc = ((long long)nc + L - 1) / L;
        const unsigned grid = (unsigned)(nsegc < 4096 ? nsegc : 4096);   // persistent, four resident per CU
        if (real_io)
            hipLaunchKernelGGL((k_fftfilt_r16<true>), dim3(grid), dim3(NT), 0, st, hm1,
                               (const float2 *)H, hc, (const void *)xc, (long long)nc, yc, scale_re, scale_im, tw);
        else
            hipLaunchKernelGGL((k_fftfilt_r16<false>), dim3(grid), dim3(NT), 0, st, hm1,
                               (const float2 *)H, hc, (const void *)xc, (long long)nc, yc, scale_re, scale_im, tw);
        LQ_CHECK_LAUNCH();
    }
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
