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
constexpr int FF_STAUX = 2;      // store cache policy: non-temporal (default policy: 0.2233-0.2243 vs 0.2206-0.2212 ms, r06d)

__device__ __forceinline__ float2 to_c2(float a) { return make_float2(a, 0.f); }
__device__ __forceinline__ float2 to_c2(float2 a) { return a; }

// The guarded form (firfilt's long filters, see lqk_fftfilt_run): every wave
// flags (flags[8 seg + wave]) whether its inputs of a segment hold a value
// outside the transform's safe class; k_ff_repair then recomputes the outputs
// of flagged segments as the exact direct convolution (firfilt.c:322-338's
// dot product over the true taps, then the user scale), so Inf / NaN reach
// the outputs the direct filter gives them to and no transform sum
// overflows.  (An exact path inside the transform kernels cost their
// register allocation 7-20 spilled VGPRs.)
// Unsafe: Inf, NaN, |v| > 2^100, or a nonzero |v| < 2^-60 (whose products
// with the twiddles would reach the denormal range).
__device__ __forceinline__ unsigned ff_unsafe1(float v)
{
    const unsigned a = __float_as_uint(v) & 0x7fffffffu;
    return (unsigned)(a - 0x21800000u) > (0x71800000u - 0x21800000u) ? (a != 0u) : 0u;
}
__device__ __forceinline__ unsigned ff_unsafe(float2 v) { return ff_unsafe1(v.x) | ff_unsafe1(v.y); }
// this wave's verdict on segment seg (lane 0 stores it): eight slots per
// segment (the repair kernel reads them as two 16-byte words), the other
// four cleared
__device__ __forceinline__ void ff_flag(unsigned *flags, long long seg, unsigned bad)
{
    const unsigned long long any = __ballot(bad);
    if ((threadIdx.x & 63) == 0) {
        flags[8 * seg + (threadIdx.x >> 6)] = any != 0ull;
        flags[8 * seg + 4 + (threadIdx.x >> 6)] = 0u;
    }
}

// Register form: 256 threads, thread t holds segment samples
// t + 256 n; forward 4096-point FFT (fft4096_r16), x H, inverse, all with the
// data in registers and two LDS transposes per transform (35 KB LDS, four
// workgroups per CU); loads and stores are coalesced across t.
template <bool REAL>
__global__ __launch_bounds__(NT, FF_WPE) void k_fftfilt_r16(int hm1, const float2 *__restrict__ H,
                                                    const void *__restrict__ hist, const void *__restrict__ xin,
                                                    long long n, void *__restrict__ yout, float sre, float sim,
                                                    const float2 *__restrict__ tw, unsigned *__restrict__ flags,
                                                    lqk_hist_job hj)
{
    __shared__ __attribute__((aligned(16))) float2 lds[FFT4096_LDS];
    if constexpr (REAL) lq_hist_job_run<float>(hj);   // the object's next history
    else lq_hist_job_run<float2>(hj);
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
    if (!REAL && flags) {   // (uniform) firfilt: flag segments with unsafe inputs for k_ff_repair
        unsigned bad = 0;
#pragma unroll
        for (int q = 0; q < 16; q++) bad |= ff_unsafe(v[q]);
        ff_flag(flags, seg, bad);
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

// 8192-point overlap-save segments (complex I/O): a segment keeps L = 8192 - hd
// new outputs for hd >= h - 1 discarded ones (hd even), so the halo re-read is
// hd / L (512 / 7680 = 6.7 % at h = 512, against 511 / 3585 = 14 % with 4096
// points) and filters up to 4097 taps fit.  The transform is the 8192-point
// one of k_fft8192_batch (decimation in time): thread t loads the sample pairs
// (x[2i], x[2i+1]), i = t + 256 q, runs fft4096_r16 on the even and the odd
// halves (E, O) through one LDS scratch, and for j = t + 256 k
//     X_0 = E + w O,  X_1 = E - w O          (X[j], X[j + 4096], w = W_8192^j)
//     Y_0 = X_0 H[j],  Y_1 = X_1 H[j + 4096]
//     A = Y_0 + Y_1,  B = (Y_0 - Y_1) conj(w)
// then the inverse by decimation in frequency: y[2i] = IFFT_4096(A)[i],
// y[2i+1] = IFFT_4096(B)[i] -- each thread ends with the output pairs of its
// own input pairs, stored as 16-byte stores (1 KB contiguous per wave
// instruction).  W_8192^(t + 256 k) = W_8192^t W_32^k: the first from
// sincospi in double once per thread, the second compile-time constants.
// A16 (x and y 16-byte aligned): one 16-byte load / store per pair except in
// the first segment (history) and, for odd n, the last (a pair straddling n);
// otherwise 8-byte accesses.  H (the 8192-point spectrum, 64 KB) is read per
// segment from L2 (it stays resident: every workgroup reads it).
template <bool A16>
__global__ __launch_bounds__(NT, 3) void k_fftfilt8k(int hd, int hm1, const float2 *__restrict__ H,
                                                    const void *__restrict__ hist, const void *__restrict__ xin,
                                                    long long n, void *__restrict__ yout, float sre, float sim,
                                                    const float2 *__restrict__ tw, unsigned *__restrict__ flags,
                                                    lqk_hist_job hj)
{
    __shared__ __attribute__((aligned(16))) float2 lds[FFT4096_LDS];
    lq_hist_job_run<float2>(hj);   // the object's next history
    typedef float v4f __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    constexpr float C32[16] = {1.000000000f,  0.980785280f,  0.923879533f,  0.831469612f,
                               0.707106781f,  0.555570233f,  0.382683432f,  0.195090322f,
                               0.000000000f,  -0.195090322f, -0.382683432f, -0.555570233f,
                               -0.707106781f, -0.831469612f, -0.923879533f, -0.980785280f};
    constexpr float S32[16] = {0.000000000f, 0.195090322f, 0.382683432f, 0.555570233f,
                               0.707106781f, 0.831469612f, 0.923879533f, 0.980785280f,
                               1.000000000f, 0.980785280f, 0.923879533f, 0.831469612f,
                               0.707106781f, 0.555570233f, 0.382683432f, 0.195090322f};
    const int L = 8192 - hd;
    const int t = threadIdx.x;
    const long long nseg = (n + L - 1) / L;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)xin, (short)0, (int)(n * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc((void *)hist, (short)0, hm1 * 8, 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(yout, (short)0, (int)(n * 8), 0x00020000);
    const tw16x2 w16 = fft4096_tw(tw, t);
    double sn, cs;
    sincospi((double)t / 4096.0, &sn, &cs);
    const v2f wt0 = v2f{(float)cs, (float)-sn};   // W_8192^t
    const bool odd_n = (n & 1) != 0;
    for (long long seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
        const int sb = (int)(seg * L) - hd;   // stream index of segment sample 0
        // the thread index through an empty asm: per-thread addresses are
        // recomputed each segment instead of hoisted out of the loop (and
        // spilled: 60+ VGPRs of loop-invariant offsets)
        int tt = t;
        asm volatile("" : "+v"(tt));
        // wave-uniform: the pairs of this segment never straddle n
        const bool wide = A16 && seg > 0 && (!odd_n || (long long)sb + 8192 <= n);
        float2 ve[16], vo[16];
        if (seg == 0) {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                if ((q & 3) == 0) __builtin_amdgcn_sched_barrier(0);   // bounded loads in flight
                const int si = sb + 2 * (tt + 256 * q);
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const int s = si + e;
                    // before x: the history's hm1 samples (hist + hm1 = x), zero before them
                    const unsigned ox = s < 0 ? 0xFFFFFFF0u : (unsigned)s * 8u, oh = (unsigned)(s + hm1) * 8u;
                    const float2 a = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, ox, 0, 0));
                    const float2 b = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rh, oh, 0, 0));
                    (e ? vo : ve)[q] = make_float2(a.x + b.x, a.y + b.y);
                }
            }
        } else if (wide) {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const unsigned o = (unsigned)(sb + 2 * (tt + 256 * q)) * 8u;
                const v4f v = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rx, o, 0, 0));
                ve[q] = make_float2(v.x, v.y);
                vo[q] = make_float2(v.z, v.w);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const unsigned o = (unsigned)(sb + 2 * (tt + 256 * q)) * 8u;
                ve[q] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, o, 0, 0));
                vo[q] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, o + 8u, 0, 0));
            }
        }
        if (flags) {   // (uniform) firfilt: flag segments with unsafe inputs for k_ff_repair
            unsigned bad = 0;
#pragma unroll
            for (int q = 0; q < 16; q++) bad |= ff_unsafe(ve[q]) | ff_unsafe(vo[q]);
            ff_flag(flags, seg, bad);
        }
        __builtin_amdgcn_sched_barrier(0);
        fft4096_r16<+1>(ve, lds, w16, t);
        __builtin_amdgcn_sched_barrier(0);
        fft4096_r16<+1>(vo, lds, w16, t);
        __builtin_amdgcn_sched_barrier(0);
        v2f wt = wt0;   // through an empty asm: not hoisted / rematerialised per k
        asm volatile("" : "+v"(wt));
#pragma unroll
        for (int k = 0; k < 16; k++) {
            if ((k & 3) == 0) __builtin_amdgcn_sched_barrier(0);   // H loads in groups of four
            const v2f w = k == 0 ? wt : pk_cmulk(wt, v2f{C32[k], -S32[k]});
            const v2f o = pk_cmul(pk(vo[k]), w);
            const v2f x0 = pk(ve[k]) + o, x1 = pk(ve[k]) - o;
            const v2f y0 = pk_cmul(x0, pk(H[tt + 256 * k])), y1 = pk_cmul(x1, pk(H[4096 + tt + 256 * k]));
            ve[k] = unpk(y0 + y1);
            vo[k] = unpk(pk_cmul(y0 - y1, v2f{w.x, -w.y}));
        }
        __builtin_amdgcn_sched_barrier(0);
        fft4096_r16<-1>(ve, lds, w16, t);
        __builtin_amdgcn_sched_barrier(0);
        fft4096_r16<-1>(vo, lds, w16, t);
        __builtin_amdgcn_sched_barrier(0);
        // output pair q: segment samples i, i + 1 (i = 2 (t + 256 q)); the first hd are discarded
        auto pair = [&](int q, float2 &a, float2 &b) -> unsigned {
            const int i = 2 * (tt + 256 * q);
            a = make_float2(ve[q].x * sre - ve[q].y * sim, ve[q].x * sim + ve[q].y * sre);
            b = make_float2(vo[q].x * sre - vo[q].y * sim, vo[q].x * sim + vo[q].y * sre);
            return i < hd ? 0xFFFFFFF0u : (unsigned)(sb + i) * 8u;
        };
        if (wide) {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                float2 a, b;
                const unsigned oy = pair(q, a, b);
                __builtin_amdgcn_raw_buffer_store_b128(v4f{a.x, a.y, b.x, b.y}, ry, oy, 0, FF_STAUX);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; q++) {
                float2 a, b;
                const unsigned oy = pair(q, a, b);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, a), ry, oy, 0, FF_STAUX);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, b), ry,
                                                      oy == 0xFFFFFFF0u ? oy : oy + 8u, 0, FF_STAUX);
            }
        }
    }
}

// The exact outputs of every flagged segment (see ff_flag): segment seg's
// outputs are stream samples seg L .. seg L + L - 1 (L new outputs per
// segment), each the reference's dot product over the true taps (natural
// order, hlen) and the user scale -- crcf: real scale per component
// (firfilt.c:337, an Inf in one component stays out of the other); cccf: the
// complex product.  Persistent grid; a segment's eight wave flags are two
// 16-byte loads.
__global__ __launch_bounds__(NT) void k_ff_repair(const unsigned *__restrict__ flags, long long nseg, int L,
                                                  const float2 *__restrict__ x, const float2 *__restrict__ hist,
                                                  int hm1, long long n, float2 *__restrict__ y,
                                                  const float *__restrict__ h, int hlen, int cc, float sre, float sim)
{
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    for (long long seg = blockIdx.x; seg < nseg; seg += gridDim.x) {
        const u32x4 f = *reinterpret_cast<const u32x4 *>(flags + 8 * seg);
        const u32x4 f2 = *reinterpret_cast<const u32x4 *>(flags + 8 * seg + 4);
        if (!(f.x | f.y | f.z | f.w | f2.x | f2.y | f2.z | f2.w)) continue;
        for (long long s = seg * L + threadIdx.x; s < seg * L + L && s < n; s += NT) {
            float2 acc = make_float2(0.f, 0.f);
            for (int k = 0; k < hlen; k++) {
                const long long u = s - k;
                const float2 v = u >= 0 ? x[u] : (u >= -hm1 ? hist[hm1 + u] : make_float2(0.f, 0.f));
                if (cc) {
                    const float hr = h[2 * k], hi = h[2 * k + 1];
                    acc = make_float2(fmaf(-hi, v.y, fmaf(hr, v.x, acc.x)), fmaf(hi, v.x, fmaf(hr, v.y, acc.y)));
                } else {
                    acc = make_float2(fmaf(h[k], v.x, acc.x), fmaf(h[k], v.y, acc.y));
                }
            }
            y[s] = cc ? make_float2(acc.x * sre - acc.y * sim, acc.x * sim + acc.y * sre)
                      : make_float2(acc.x * sre, acc.y * sre);
        }
    }
}

} // namespace

// transform size for a filter: 4096-point segments up to 2049 taps; complex
// I/O up to 4097 taps in 8192-point segments; 0: too long for the kernels
// (the host runs the direct FIR).  (8192-point segments halve the halo
// re-read, but neither form keeps the 4096-point kernel's occupancy: 256
// threads with ~170 VGPRs, three workgroups per CU with spills, 0.257-0.270
// ms at h = 512 on 2^26 samples; two 4096-point halves on 512 threads with
// two sum/difference exchanges through LDS, 0.278-0.281 ms; 4096-point
// segments 0.221-0.223 ms, profiles/r06_ab_experiments.txt.  The 8192-point
// kernel serves the filters 4096 points cannot.)
extern "C" unsigned int lqk_fftfilt_nfft(int real_io, unsigned int hlen)
{
    if (hlen < 1) return 0;
    if (hlen - 1 <= NFFT / 2) return NFFT;
    return !real_io && hlen - 1 <= 4096 ? 8192 : 0;
}

// flag buffer bytes for a guarded call of n samples (per launch chunk: the
// buffer is reused chunk after chunk on the stream)
extern "C" size_t lqk_fftfilt_flag_bytes(unsigned int hlen, unsigned int nfft, unsigned long long n)
{
    const unsigned long long CHN = 1ull << 27, nc = n < CHN ? n : CHN;
    const int hm1 = (int)hlen - 1;
    const unsigned long long L = nfft == 8192 ? 8192 - ((hm1 + 1) & ~1) : NFFT - hm1;
    return (size_t)((nc + L - 1) / L + 1) * 32;
}

extern "C" void lqk_fftfilt_run(int real_io, unsigned int hlen, unsigned int nfft, const void *H, const void *hist,
                                const void *x, unsigned long long n, void *y, float scale_re, float scale_im,
                                const float *hx, int guard, void *flags, const lqk_hist_job *job, void *stream)
{
    if (guard && (real_io || !hx || !flags)) {
        fprintf(stderr, "error: fftfilt: guarded form needs complex I/O, the taps and a flag buffer\n");
        exit(1);
    }
    if (n == 0) return;
    if (nfft != lqk_fftfilt_nfft(real_io, hlen) || nfft == 0) {
        fprintf(stderr, "error: fftfilt: filter length %u exceeds the GPU transform limit\n", hlen);
        exit(1);
    }
    hipStream_t st = (hipStream_t)stream;
    const int hm1 = (int)hlen - 1;
    const float2 *tw = (const float2 *)lqrt_twiddles();
    const size_t es = real_io ? 4 : 8;
    const float sre = scale_re / (float)nfft, sim = scale_im / (float)nfft;
    // launches of at most 2^27 samples (32-bit buffer offsets); later chunks
    // take their history straight from the preceding input
    const unsigned long long CHN = 1ull << 27;
    for (unsigned long long c0 = 0; c0 < n; c0 += CHN) {
        const unsigned long long nc = (n - c0) < CHN ? (n - c0) : CHN;
        const char *xc = (const char *)x + c0 * es;
        const void *hc = c0 == 0 ? hist : (const void *)(xc - (size_t)hm1 * es);
        void *yc = (char *)y + c0 * es;
        // the history update rides on the first launch
        const lqk_hist_job hj = (c0 == 0 && job) ? *job : lqk_hist_job{nullptr, nullptr, 0ull, nullptr, 0u};
        if (nfft == 8192) {
            const int hd = (hm1 + 1) & ~1;   // discarded outputs per segment: even, >= h - 1
            const long long nsegc = ((long long)nc + (8192 - hd) - 1) / (8192 - hd);
            const unsigned grid = (unsigned)(nsegc < 768 ? nsegc : 768);   // persistent, three resident per CU
            const bool a16 = (((uintptr_t)xc | (uintptr_t)yc) & 15) == 0;
            hipLaunchKernelGGL(a16 ? k_fftfilt8k<true> : k_fftfilt8k<false>, dim3(grid), dim3(NT), 0, st, hd, hm1,
                               (const float2 *)H, hc, (const void *)xc, (long long)nc, yc, sre, sim, tw,
                               guard ? (unsigned *)flags : nullptr, hj);
            LQ_CHECK_LAUNCH();
            if (guard)
                hipLaunchKernelGGL(k_ff_repair, dim3(256), dim3(NT), 0, st, (const unsigned *)flags, nsegc, 8192 - hd,
                                   (const float2 *)xc, (const float2 *)hc, hm1, (long long)nc, (float2 *)yc, hx,
                                   (int)hlen, guard == 2, scale_re, scale_im);
        } else {
            const int L = NFFT - hm1;
            const long long nsegc = ((long long)nc + L - 1) / L;
            const unsigned grid = (unsigned)(nsegc < 4096 ? nsegc : 4096);   // persistent, four resident per CU
            if (real_io)
                hipLaunchKernelGGL((k_fftfilt_r16<true>), dim3(grid), dim3(NT), 0, st, hm1, (const float2 *)H, hc,
                                   (const void *)xc, (long long)nc, yc, sre, sim, tw, nullptr, hj);
            else
            {
                hipLaunchKernelGGL((k_fftfilt_r16<false>), dim3(grid), dim3(NT), 0, st, hm1, (const float2 *)H, hc,
                                   (const void *)xc, (long long)nc, yc, sre, sim, tw,
                                   guard ? (unsigned *)flags : nullptr, hj);
                LQ_CHECK_LAUNCH();
                if (guard)
                    hipLaunchKernelGGL(k_ff_repair, dim3(256), dim3(NT), 0, st, (const unsigned *)flags, nsegc, L,
                                       (const float2 *)xc, (const float2 *)hc, hm1, (long long)nc, (float2 *)yc, hx,
                                       (int)hlen, guard == 2, scale_re, scale_im);
            }
        }
        LQ_CHECK_LAUNCH();
    }
}

// H[k] = FFT_nfft(h zero padded)  (h real or complex), computed on the device
__global__ void k_pad_coef(const void *h, int hlen, int is_complex, int nfft, float2 *buf)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nfft) return;
    float2 v = make_float2(0.f, 0.f);
    if (i < hlen) v = is_complex ? ((const float2 *)h)[i] : make_float2(((const float *)h)[i], 0.f);
    buf[i] = v;
}

extern "C" void lqk_fftfilt_make_H(const void *h_dev, unsigned int hlen, int is_complex, unsigned int nfft, void *H,
                                   void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_pad_coef, dim3(nfft / 256), dim3(256), 0, st, h_dev, (int)hlen, is_complex, (int)nfft,
                       (float2 *)H);
    LQ_CHECK_LAUNCH();
    lqk_fft_batch(nfft, +1, H, H, 1, stream);
}
