// lq_device.h -- device-side building blocks shared by the kernels:
// complex helpers on float2 (interleaved re,im = the liquid_float_complex
// layout) and an LDS-resident Stockham FFT for power-of-two sizes <= 4096.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lq_kernels.h"

void lq_check(hipError_t e, const char *what, const char *file, int line);
#define LQ_CHECK(x) lq_check((x), #x, __FILE__, __LINE__)
#define LQ_CHECK_LAUNCH() lq_check(hipGetLastError(), "kernel launch", __FILE__, __LINE__)

#define LQ_TW_N 4096

// Small-call completion (lq_runtime.hip): after this thread's result stores,
// release them at system scope and raise the host's pinned flag word.  A
// null flag (device-resident calls) does nothing.
__device__ __forceinline__ void lq_signal(unsigned *flag, unsigned seq)
{
    if (flag == nullptr) return;
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Workgroup barrier for LDS hand-offs: waits for this wave's LDS operations
// only.  __syncthreads() also waits for every global load and store in
// flight (vmcnt(0)), so a transform between a segment's stores and the next
// segment's would hold the stores up at its first barrier.
__device__ __forceinline__ void lq_lds_sync()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

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

// ---- packed complex arithmetic: (re, im) in a VGPR pair, v_pk_*_f32 with
// op_sel / neg modifiers doing the component swaps (one instruction per
// complex add or +-j rotation, two per complex multiply; the compiler's own
// float2 code spends extra v_mov / v_xor on the swaps)
typedef float v2f __attribute__((ext_vector_type(2)));

// One complex sample of a stream whose HL samples before x live in a
// separate history buffer (hist_end = hist + HL): the history, x, or a zero
// word (lqrt_zeros, >= 8 bytes) outside both.  One non-temporal global load
// from a per-lane address (integer selects, no branch around the load).  Two
// range-checked buffer loads per sample, one of them always out of range,
// doubled the vector-memory instructions of the channelizers' row streams
// (firpfbch2 M = 1024: 0.680 -> 0.636 ms per 2^27 samples).
__device__ __forceinline__ float2 lq_load_hx(const float2 *hist_end, const float2 *x, const float2 *zero,
                                             long long li, long long HL, long long n)
{
    const bool neg = li < 0;
    const bool in = neg ? (li >= -HL) : (li < n);
    unsigned long long a = (unsigned long long)(uintptr_t)(neg ? hist_end : x) + (unsigned long long)(li * 8);
    a = in ? a : (unsigned long long)(uintptr_t)zero;
    typedef const v2f __attribute__((address_space(1))) *gptr;
    const v2f v = __builtin_nontemporal_load(reinterpret_cast<gptr>(a));
    return make_float2(v.x, v.y);
}

// lqk_hist_job (lq_kernels.h) as a grid-strided slice per workgroup, before
// the kernel's own work: dst[i] = (src ++ x)[n + i], i < L
template <typename T>
__device__ __forceinline__ void lq_hist_job_run(const lqk_hist_job &j)
{
    if (j.dst == nullptr) return;
    const long long L = j.L, n = (long long)j.n, step = (long long)gridDim.x * blockDim.x;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < L; i += step) {
        const long long k = i + n;
        reinterpret_cast<T *>(j.dst)[i] =
            k < L ? reinterpret_cast<const T *>(j.src)[k] : reinterpret_cast<const T *>(j.x)[k - L];
    }
}

__device__ __forceinline__ v2f pk(float2 a) { return v2f{a.x, a.y}; }
__device__ __forceinline__ float2 unpk(v2f a) { return make_float2(a.x, a.y); }
// b + j d = (b.x - d.y, b.y + d.x)
__device__ __forceinline__ v2f pk_addpj(v2f b, v2f d)
{
    v2f r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(b), "v"(d));
    return r;
}
// b - j d = (b.x + d.y, b.y - d.x)
__device__ __forceinline__ v2f pk_subpj(v2f b, v2f d)
{
    v2f r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(b), "v"(d));
    return r;
}
// a * w, w in VGPRs: t = a.x * w; r = (t.x - a.y w.y, t.y + a.y w.x)
__device__ __forceinline__ v2f pk_cmul(v2f a, v2f w)
{
    v2f t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r)
        : "v"(a), "v"(w), "v"(t));
    return r;
}
// a * w for a compile-time constant w (held in an SGPR pair)
__device__ __forceinline__ v2f pk_cmulk(v2f a, v2f w)
{
    v2f t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "s"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r)
        : "v"(a), "s"(w), "v"(t));
    return r;
}
// radix-4 butterfly, DIR +1 forward (exp(-j 2 pi qs/4)), -1 backward
template <int DIR>
__device__ __forceinline__ void pk_dft4(v2f &v0, v2f &v1, v2f &v2, v2f &v3)
{
    const v2f a = v0 + v2, b = v0 - v2, c = v1 + v3, d = v1 - v3;
    v0 = a + c;
    v2 = a - c;
    v1 = DIR > 0 ? pk_subpj(b, d) : pk_addpj(b, d);
    v3 = DIR > 0 ? pk_addpj(b, d) : pk_subpj(b, d);
}
// 16-point DFT, natural order in / out, radix 4 x 4: 8 butterflies (64
// packed instructions) and 8 constant twiddles (16); W16^{+-4} = +-j is folded
// into the butterfly of its column.
template <int DIR>
__device__ __forceinline__ void pk_dft16(v2f (&v)[16])
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
        v2f a0 = v[q], a1 = v[4 + q], a2 = v[8 + q], a3 = v[12 + q];
        pk_dft4<DIR>(a0, a1, a2, a3);
        t[q] = a0;
        t[4 + q] = q == 0 ? a1 : pk_cmulk(a1, v2f{C[q], -DIR * S[q]});
        t[8 + q] = (q == 0 || q == 2) ? a2 : pk_cmulk(a2, v2f{C[2 * q], -DIR * S[2 * q]});
        t[12 + q] = q == 0 ? a3 : pk_cmulk(a3, v2f{C[(3 * q) & 15], -DIR * S[(3 * q) & 15]});
    }
#pragma unroll
    for (int k0 = 0; k0 < 4; k0++) {
        v2f b0 = t[4 * k0 + 0], b1 = t[4 * k0 + 1], b2 = t[4 * k0 + 2], b3 = t[4 * k0 + 3];
        if (k0 == 2) {
            // b2 still lacks its W16^{-4 DIR} = -DIR j factor
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

// ---------------------------------------------------------------- register radix-16
// 16-point DFT in registers, natural order in and out; DIR +1 forward
// (exp(-j 2 pi nk/16)), -1 backward (packed form above).
template <int DIR>
__device__ __forceinline__ void dft16(float2 (&v)[16])
{
    v2f p[16];
#pragma unroll
    for (int k = 0; k < 16; k++) p[k] = pk(v[k]);
    pk_dft16<DIR>(p);
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = unpk(p[k]);
}

// 4096-point FFT by a 256-thread block, three register radix-16 passes and two
// LDS transposes (lds: FFT4096_LDS float2).  In: thread t holds x[t + 256 n]
// in v[n]; out: X[t + 256 k] in v[k].  tw: W_4096^e = exp(-2 pi i e/4096).
// Every thread of the block calls it (it synchronises).
//   pass 1: DFT16 over n (stride 256), twiddle W_4096^{t k2}
//   pass 2: thread (k2 = u>>4, m0 = u&15) DFT16 over m1 of B[m0 + 16 m1][k2],
//           twiddle W_256^{m0 j1}
//   pass 3: thread (k2 = v&15, j1 = v>>4) DFT16 over m0 -> X[k2 + 16 j1 + 256 j0]
#define FFT4096_LDS (16 * 272)
// v[k] *= W_4096^{DIR e k}, k = 1..15, from two table reads (W^e, W^{4e}):
// W^{e k} = W^{e (k & 3)} W^{e (k & 12)}, each factor at most two products
// from a table value (keeps the cached-table traffic at 2 loads per pass)
template <int DIR>
__device__ __forceinline__ void twiddle16v(float2 (&v)[16], float2 a1, float2 a4);
template <int DIR>
__device__ __forceinline__ void twiddle16(float2 (&v)[16], const float2 *__restrict__ tw, int e)
{
    twiddle16v<DIR>(v, tw[e & 4095], tw[(4 * e) & 4095]);
}
// the same from the two table values W^e, W^{4e} (forward direction) held
// in registers: kernels that run many transforms load them once per thread
// instead of twice per pass (each a dependent L2 round trip)
template <int DIR>
__device__ __forceinline__ void twiddle16v(float2 (&v)[16], float2 a1, float2 a4)
{
    if (DIR < 0) {
        a1.y = -a1.y;
        a4.y = -a4.y;
    }
    const v2f w1 = pk(a1), w4 = pk(a4);
    const v2f w2 = pk_cmul(w1, w1), w3 = pk_cmul(w2, w1);
    const v2f w8 = pk_cmul(w4, w4), w12 = pk_cmul(w8, w4);
    const v2f lo[3] = {w1, w2, w3}, hi[3] = {w4, w8, w12};
#pragma unroll
    for (int k = 1; k < 16; k++) {
        const int l = k & 3, h = k >> 2;
        v2f w = l ? lo[l - 1] : hi[h - 1];
        if (l && h) w = pk_cmul(lo[l - 1], hi[h - 1]);
        v[k] = unpk(pk_cmul(pk(v[k]), w));
    }
}
// R-point DFT (R = 1, 2, 4, 8, 16) on v[0..R), natural order in and out
template <int R, int DIR>
__device__ __forceinline__ void dft_small(float2 *v)
{
    if constexpr (R == 2) {
        const float2 a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    } else if constexpr (R == 4) {
        v2f a0 = pk(v[0]), a1 = pk(v[1]), a2 = pk(v[2]), a3 = pk(v[3]);
        pk_dft4<DIR>(a0, a1, a2, a3);
        v[0] = unpk(a0); v[1] = unpk(a1); v[2] = unpk(a2); v[3] = unpk(a3);
    } else if constexpr (R == 8) {
        // n = n1 + 2 n2: DFT4 over n2 per n1, twiddle W8^{n1 k1}, DFT2 over n1
        constexpr float h = 0.70710678f;
        v2f e0 = pk(v[0]), e1 = pk(v[2]), e2 = pk(v[4]), e3 = pk(v[6]);
        v2f o0 = pk(v[1]), o1 = pk(v[3]), o2 = pk(v[5]), o3 = pk(v[7]);
        pk_dft4<DIR>(e0, e1, e2, e3);
        pk_dft4<DIR>(o0, o1, o2, o3);
        o1 = pk_cmulk(o1, v2f{h, -DIR * h});                          // W8^1
        o2 = DIR > 0 ? pk_subpj(v2f{0.f, 0.f}, o2) : pk_addpj(v2f{0.f, 0.f}, o2);   // W8^2 = -DIR j
        o3 = pk_cmulk(o3, v2f{-h, -DIR * h});                         // W8^3
        v[0] = unpk(e0 + o0); v[4] = unpk(e0 - o0);
        v[1] = unpk(e1 + o1); v[5] = unpk(e1 - o1);
        v[2] = unpk(e2 + o2); v[6] = unpk(e2 - o2);
        v[3] = unpk(e3 + o3); v[7] = unpk(e3 - o3);
    } else if constexpr (R == 16) {
        v2f p[16];
#pragma unroll
        for (int k = 0; k < 16; k++) p[k] = pk(v[k]);
        pk_dft16<DIR>(p);
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = unpk(p[k]);
    }
}

// N = 256 R point FFT (R = 1, 2, 4, 8, 16: N = 256 .. 4096) by T = 16 R
// threads, three register passes and two LDS transposes; the generalisation
// of fft4096_r16 below (R = 16).  In: thread t < T holds x[t + T n] in v[n];
// out: v[s R + q] = X[t + T s + 256 q] (s < 16/R, q < R).  lds: FFTR16_LDS(R)
// float2 for this transform; every thread of the workgroup calls it (it
// synchronises).
//   pass 1: DFT16 over n, twiddle W_N^{t k2}
//   pass 2: t = a + R b (a < R): unit (k2, a) runs a DFT16 over b -> q1,
//           twiddle W_T^{a q1}
//   pass 3: unit (k2, q1) runs a DFT_R over a -> q2; X[k2 + 16 q1 + 256 q2]
template <int R>
constexpr int fftr16_s1() { return 16 * R + 2; }            // pass-1 row stride (conflict-free reads)
// pass-2 unit stride: odd (conflict-free pass-3 reads); TIGHT: R (2-way
// conflicted, a smaller scratch for kernels short of LDS)
template <int R, bool TIGHT = false>
constexpr int fftr16_s2() { return (R == 1 || TIGHT) ? R : R + 1; }
template <int R, bool TIGHT = false>
constexpr int FFTR16_LDS()
{
    return (16 * fftr16_s1<R>() > 256 * fftr16_s2<R, TIGHT>() ? 16 * fftr16_s1<R>() : 256 * fftr16_s2<R, TIGHT>()) | 1;
}
// the four twiddle-table values a thread of fft_r16x16xR<R> uses (both
// directions: the inverse conjugates them)
struct tw16x2 {
    float2 p1a, p1b, p2a, p2b;
};
template <int R>
__device__ __forceinline__ tw16x2 fftr16_tw(const float2 *__restrict__ tw, int t)
{
    constexpr int T = 16 * R, N = 16 * T;
    const int e1 = t * (4096 / N), e2 = (t >> 4) * (4096 / T);
    return tw16x2{tw[e1 & 4095], tw[(4 * e1) & 4095], tw[e2 & 4095], tw[(4 * e2) & 4095]};
}
template <int R, int DIR, bool TIGHT = false>
__device__ __forceinline__ void fft_r16x16xR(float2 (&v)[16], float2 *lds, const tw16x2 &w, int t);
template <int R, int DIR, bool TIGHT = false>
__device__ __forceinline__ void fft_r16x16xR(float2 (&v)[16], float2 *lds, const float2 *__restrict__ tw, int t)
{
    fft_r16x16xR<R, DIR, TIGHT>(v, lds, fftr16_tw<R>(tw, t), t);
}
template <int R, int DIR, bool TIGHT>
__device__ __forceinline__ void fft_r16x16xR(float2 (&v)[16], float2 *lds, const tw16x2 &w, int t)
{
    constexpr int T = 16 * R;
    constexpr int S1 = fftr16_s1<R>(), S2 = fftr16_s2<R, TIGHT>();
    dft16<DIR>(v);
    twiddle16v<DIR>(v, w.p1a, w.p1b);   // W_N^{t k2}
    lq_lds_sync();
#pragma unroll
    for (int k = 0; k < 16; k++) lds[k * S1 + t] = v[k];
    lq_lds_sync();
    const int k2 = t & 15, a = t >> 4;
#pragma unroll
    for (int b = 0; b < 16; b++) v[b] = lds[k2 * S1 + a + R * b];
    dft16<DIR>(v);
    if constexpr (R > 1) twiddle16v<DIR>(v, w.p2a, w.p2b);   // W_T^{a q1}
    lq_lds_sync();
#pragma unroll
    for (int q1 = 0; q1 < 16; q1++) lds[(k2 + 16 * q1) * S2 + a] = v[q1];
    lq_lds_sync();
    // unit k2 + 16 q1 with q1 = (t >> 4) + R s is t + T s
#pragma unroll
    for (int s = 0; s < 16 / R; s++)
#pragma unroll
        for (int e = 0; e < R; e++) v[s * R + e] = lds[(t + T * s) * S2 + e];
#pragma unroll
    for (int s = 0; s < 16 / R; s++) dft_small<R, DIR>(v + s * R);
}

// N = 16 R point FFT (R = 2, 4, 8: N = 32, 64, 128) by T = R threads: a
// register DFT16 over n (x[t + R n]), the twiddle W_N^{t k2}, one padded LDS
// transpose, then 16 / R DFT_R's per thread.  Out: v[u R + q] = X[t (16/R) + u
// + 16 q].  lds: 16 (R + 1) float2 for this transform; every thread of the
// workgroup calls it (it synchronises).
template <int R>
constexpr int FFTS_LDS() { return 16 * (R + 1); }
template <int R, int DIR>
__device__ __forceinline__ void fft_small16xR(float2 (&v)[16], float2 *lds, float2 a1, float2 a4, int t)
{
    constexpr int S = R + 1;
    dft16<DIR>(v);
    twiddle16v<DIR>(v, a1, a4);   // W_N^{t k2}
    lq_lds_sync();
#pragma unroll
    for (int k = 0; k < 16; k++) lds[k * S + t] = v[k];
    lq_lds_sync();
    constexpr int U = 16 / R;
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int e = 0; e < R; e++) v[u * R + e] = lds[(t * U + u) * S + e];
#pragma unroll
    for (int u = 0; u < U; u++) dft_small<R, DIR>(v + u * R);
}

__device__ __forceinline__ tw16x2 fft4096_tw(const float2 *__restrict__ tw, int t)
{
    const int e2 = 16 * (t & 15);
    return tw16x2{tw[t & 4095], tw[(4 * t) & 4095], tw[e2 & 4095], tw[(4 * e2) & 4095]};
}
template <int DIR>
__device__ __forceinline__ void fft4096_r16(float2 (&v)[16], float2 *lds, const tw16x2 &w, int t);
template <int DIR>
__device__ __forceinline__ void fft4096_r16(float2 (&v)[16], float2 *lds, const float2 *__restrict__ tw, int t)
{
    fft4096_r16<DIR>(v, lds, fft4096_tw(tw, t), t);
}
template <int DIR>
__device__ __forceinline__ void fft4096_r16(float2 (&v)[16], float2 *lds, const tw16x2 &w, int t)
{
    dft16<DIR>(v);
    twiddle16v<DIR>(v, w.p1a, w.p1b);   // W_4096^{t k}
    lq_lds_sync();
#pragma unroll
    for (int k = 0; k < 16; k++) lds[k * 272 + t] = v[k];   // row pad 16: conflict-free reads below
    lq_lds_sync();
    const int m0 = t & 15, k2 = t >> 4;
#pragma unroll
    for (int m = 0; m < 16; m++) v[m] = lds[k2 * 272 + m0 + 16 * m];
    dft16<DIR>(v);
    twiddle16v<DIR>(v, w.p2a, w.p2b);   // W_256^{m0 j} = W_4096^{16 m0 j}
    lq_lds_sync();
#pragma unroll
    for (int j = 0; j < 16; j++) lds[(k2 + 16 * j) * 17 + m0] = v[j];
    lq_lds_sync();
#pragma unroll
    for (int m = 0; m < 16; m++) v[m] = lds[t * 17 + m];
    dft16<DIR>(v);
}
