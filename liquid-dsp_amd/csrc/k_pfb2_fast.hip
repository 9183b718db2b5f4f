// k_pfb2_fast.hip -- firpfbch2_crcf analyzer, M = 1024, fast path.
//
// Same closed form as csrc/k_channelizer.hip (reference
// src/multichannel/src/firpfbch2.c:244-282), restructured for CDNA4:
//
//  * View the input as rows of M = 1024 samples (row c = x[cM .. cM+M) in
//    stream coordinates).  Column col of the row matrix feeds exactly one
//    IFFT bin j(col) (j = M/2-1-col for col < M/2, 3M/2-1-col otherwise) and
//    X_b[j] is an L = 2m tap dot product down that column:
//        X_b[j] = sum_n h[i + nM] row[c - n][col],  i = j (b even) or j ^ M/2 (b odd),
//    c = row of the block's newest sample.  Row c completes blocks 2c
//    (lower bins; upper bins came from row c-1) and 2c+1, and starts 2c+2.
//  * A workgroup (8 waves, one per CU) owns all 1024 columns: lane t holds
//    column t (bin 511-t) and column 512+t (bin 1023-t), whose even-block taps
//    are each other's odd-block taps, so 2 x L coefficients and an 8-deep
//    register ring per column cover both.  Rows stream through the ring, so
//    every input sample is read from HBM once per workgroup segment.  Four
//    rows per iteration complete eight blocks; the next four rows are
//    prefetched into registers while the FFTs run.
//  * X of each block goes to an LDS ring (9 block buffers); after a barrier
//    each wave runs one 1024-point IFFT in registers: 16-point DFT over the
//    lane's 16 bins (j = lane + 64k), twiddle, LDS transpose (row stride 68
//    keeps ds_read_b64 conflict-free), 16-point DFT, twiddle, and a 4-point
//    DFT across lane quads with DPP-level shuffles.  1/M is folded into the
//    coefficients (exact for M = 2^10).
//  * Blocks are grouped four at a time in global block numbering (even block
//    = offset 0, odd = M/2), so calls of any length and start parity share one
//    kernel; blocks outside the call are computed but not stored.
#include "lq_device.h"
#include "lq_kernels.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace {

constexpr int M = 1024;
constexpr int M2 = M / 2;
constexpr int NT = 512;
constexpr int NS = 8;      // register ring depth (rows)
constexpr int NBUF = 9;    // LDS block buffers (writes b0..b0+8, FFT reads b0..b0+7)
constexpr int BSTR = 1088; // floats2 per block buffer (16 x 68 transpose)
constexpr int TSTR = 68;

// cos/sin(2 pi e / 16), e = 0..15
__device__ constexpr float C16[16] = {1.0f,         0.92387953f,  0.70710678f,  0.38268343f,
                                      0.0f,         -0.38268343f, -0.70710678f, -0.92387953f,
                                      -1.0f,        -0.92387953f, -0.70710678f, -0.38268343f,
                                      0.0f,         0.38268343f,  0.70710678f,  0.92387953f};
__device__ constexpr float S16[16] = {0.0f,         0.38268343f,  0.70710678f,  0.92387953f,
                                      1.0f,         0.92387953f,  0.70710678f,  0.38268343f,
                                      0.0f,         -0.38268343f, -0.70710678f, -0.92387953f,
                                      -1.0f,        -0.92387953f, -0.70710678f, -0.38268343f};

// 16-point backward DFT (e^{+j2pi nk/16}) in registers, natural order in/out.
__device__ __forceinline__ void dft16_bwd(float2 (&v)[16])
{
    float2 t[16];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        float2 a0 = v[q], a1 = v[4 + q], a2 = v[8 + q], a3 = v[12 + q];
        dft4(a0, a1, a2, a3, -1);
        // twiddle W16^{+q k0}
        t[0 * 4 + q] = a0;
        if (q == 0) {
            t[1 * 4 + q] = a1;
            t[2 * 4 + q] = a2;
            t[3 * 4 + q] = a3;
        } else {
            t[1 * 4 + q] = cmul(a1, make_float2(C16[(1 * q) & 15], S16[(1 * q) & 15]));
            t[2 * 4 + q] = cmul(a2, make_float2(C16[(2 * q) & 15], S16[(2 * q) & 15]));
            t[3 * 4 + q] = cmul(a3, make_float2(C16[(3 * q) & 15], S16[(3 * q) & 15]));
        }
    }
#pragma unroll
    for (int k0 = 0; k0 < 4; k0++) {
        float2 b0 = t[k0 * 4 + 0], b1 = t[k0 * 4 + 1], b2 = t[k0 * 4 + 2], b3 = t[k0 * 4 + 3];
        dft4(b0, b1, b2, b3, -1);
        v[k0 + 0] = b0;
        v[k0 + 4] = b1;
        v[k0 + 8] = b2;
        v[k0 + 12] = b3;
    }
}

__device__ __forceinline__ float2 shfl_xor2(float2 v, int m)
{
    return make_float2(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64));
}

typedef float v2f __attribute__((ext_vector_type(2)));

// streaming (non-temporal) store of one complex sample: output is written once
__device__ __forceinline__ void st_nt(float2 *p, float2 v)
{
    v2f w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<v2f *>(p));
}

__device__ __forceinline__ void lds_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct Params {
    const float2 *hist;
    const float2 *x;
    long long n_in;   // input samples in this call
    long long B0;     // global index of the call's first block (parity matters)
    long long nblk;   // blocks in this call
    long long gs0;    // first global 8-block group of workgroup 0 (even)
    int gpw;          // groups per workgroup (even)
    long long gend;   // one past the last group needed
    float2 *Y;
};

template <int L>
__global__ __launch_bounds__(NT, 1) void k_pfb2_an1024(Params P, const float *__restrict__ hsub,
                                                       const float2 *__restrict__ tw4096)
{
    static_assert(L <= NS, "ring too small");
    __shared__ __attribute__((aligned(16))) float2 xb[NBUF * BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw1[16 * 64]; // W_1024^{+t k1}
    __shared__ __attribute__((aligned(16))) float2 tw2[16 * 4];  // W_64^{+b r}

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    for (int e = tid; e < 16 * 64; e += NT) {
        const int k1 = e >> 6, t = e & 63;
        float2 w = tw4096[(4 * t * k1) & 4095];
        tw1[e] = make_float2(w.x, -w.y);
    }
    if (tid < 64) {
        const int r = tid >> 2, b = tid & 3;
        float2 w = tw4096[(64 * b * r) & 4095];
        tw2[tid] = make_float2(w.x, -w.y);
    }

    // lane column pair: lo column tid -> bin jl = M/2-1-tid, hi column M/2+tid
    // -> bin jh = M-1-tid = jl ^ M/2.  Even blocks use taps h[j + nM], odd
    // blocks h[(j ^ M/2) + nM]: the lo column's odd taps are the hi column's
    // even taps and vice versa.  1/M folded in (exact).
    const int jl = M2 - 1 - tid, jh = M - 1 - tid;
    float hl[L], hh[L];
    const float inv = 1.0f / (float)M;
#pragma unroll
    for (int n = 0; n < L; n++) {
        hl[n] = hsub[jl * L + n] * inv;
        hh[n] = hsub[jh * L + n] * inv;
    }

    float2 wl[NS], wh[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) wl[s] = wh[s] = make_float2(0.f, 0.f);

    const long long gs = P.gs0 + (long long)blockIdx.x * P.gpw;
    long long ge = gs + P.gpw;
    if (ge > P.gend) ge = P.gend;
    const long long base_off = P.B0 * M2; // stream index of local sample 0
    const long long HL = 2 * (L / 2) * M - M2;

    // branch-free fetch: always-valid address, then select
    auto fetch = [&](long long i) -> float2 {
        const bool in_x = (i >= 0) && (i < P.n_in);
        const bool in_h = (i < 0) && (i >= -HL);
        const float2 *p = in_x ? P.x + i : (in_h ? P.hist + (HL + i) : P.hist);
        const float2 v = *p;
        return (in_x || in_h) ? v : make_float2(0.f, 0.f);
    };
    auto dot = [&](const float2 (&w)[NS], int newest, const float (&h)[L]) -> float2 {
        float2 acc = make_float2(0.f, 0.f);
#pragma unroll
        for (int n = 0; n < L; n++) {
            const float2 v = w[(newest - n) & (NS - 1)];
            acc.x = fmaf(h[n], v.x, acc.x);
            acc.y = fmaf(h[n], v.y, acc.y);
        }
        return acc;
    };
    auto buf = [&](long long b) -> float2 * { return xb + (int)(b % NBUF) * BSTR; };

    // warm-up: rows 4gs-8 .. 4gs-1 fill ring slots 0..7; the last of them gives
    // the hi-bin half of block 8gs (even block: hi column even taps = hh)
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const long long i = (4 * gs - NS + s) * M + tid - base_off;
        wl[s] = fetch(i);
        wh[s] = fetch(i + M2);
    }
    buf(8 * gs)[jh] = dot(wh, NS - 1, hh);
    __syncthreads(); // twiddle tables ready

    float2 pl[4], ph_[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const long long i = (4 * gs + r) * M + tid - base_off;
        pl[r] = fetch(i);
        ph_[r] = fetch(i + M2);
    }

    for (long long g = gs; g < ge; g += 2) {
#pragma unroll
        for (int ph = 0; ph < 2; ph++) {
            const long long gg = g + ph;
            if (gg < ge) {
                const long long b0 = 8 * gg;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    // row c = 4gg + r: completes block 2c's lo bins and block
                    // 2c+1, starts block 2c+2's hi bins
                    const int s = 4 * ph + r;
                    wl[s] = pl[r];
                    wh[s] = ph_[r];
                    const long long bc = b0 + 2 * r;
                    buf(bc)[jl] = dot(wl, s, hl);     // lo, even
                    buf(bc + 1)[jl] = dot(wl, s, hh); // lo, odd
                    buf(bc + 1)[jh] = dot(wh, s, hl); // hi, odd
                    buf(bc + 2)[jh] = dot(wh, s, hh); // hi, even
                }
                if (gg + 1 < ge) {
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const long long i = (4 * (gg + 1) + r) * M + tid - base_off;
                        pl[r] = fetch(i);
                        ph_[r] = fetch(i + M2);
                    }
                }
                __syncthreads();

                // ---- one 1024-point IFFT per wave: block b0 + wave
                {
                    const long long b = b0 + wave;
                    float2 *B = buf(b);
                    float2 v[16];
#pragma unroll
                    for (int k = 0; k < 16; k++) v[k] = B[lane + 64 * k];
                    dft16_bwd(v);
#pragma unroll
                    for (int k1 = 1; k1 < 16; k1++) v[k1] = cmul(v[k1], tw1[k1 * 64 + lane]);
                    lds_fence();
#pragma unroll
                    for (int k1 = 0; k1 < 16; k1++) B[k1 * TSTR + lane] = v[k1];
                    lds_fence();
                    const int k1 = lane >> 2, bq = lane & 3;
#pragma unroll
                    for (int a = 0; a < 16; a++) v[a] = B[k1 * TSTR + 4 * a + bq];
                    dft16_bwd(v);
#pragma unroll
                    for (int r = 1; r < 16; r++) v[r] = cmul(v[r], tw2[r * 4 + bq]);
                    // 4-point DFT over bq across the lane quad (radix-2 x 2):
                    // stage 1 pairs bq, bq^2; twiddle W4^{+1} on bq=3; stage 2 pairs bq, bq^1
                    const bool hi2 = (bq & 2) != 0, hi1 = (bq & 1) != 0;
#pragma unroll
                    for (int r = 0; r < 16; r++) {
                        float2 p = shfl_xor2(v[r], 2);
                        float2 u = hi2 ? csub(p, v[r]) : cadd(v[r], p);
                        if (bq == 3) u = cmul_pj(u);
                        float2 p2 = shfl_xor2(u, 1);
                        v[r] = hi1 ? csub(p2, u) : cadd(u, p2);
                    }
                    // lane (k1, bq) holds Y[k1 + 16 r + 256 s], s = bitrev2(bq)
                    if (b >= P.B0 && b < P.B0 + P.nblk) {
                        const int s = ((bq & 1) << 1) | (bq >> 1);
                        float2 *Yb = P.Y + (b - P.B0) * M + k1 + 256 * s;
#pragma unroll
                        for (int r = 0; r < 16; r++) st_nt(Yb + 16 * r, v[r]);
                    }
                }
                __syncthreads();
            }
        }
    }
}

} // namespace

// Returns 1 if handled by the fast path.
extern "C" int lqk_firpfbch2_analyzer_fast(unsigned int Mch, unsigned int m, const void *hsub, const void *hist,
                                           const void *x, unsigned long long nblocks, long long B0, void *Y,
                                           void *stream)
{
    if (Mch != (unsigned)M || !(m == 4 || m == 2)) return 0;
    if (((uintptr_t)x & 7) || ((uintptr_t)hist & 7)) return 0;
    if (nblocks == 0) return 1;
    hipStream_t st = (hipStream_t)stream;
    Params P;
    P.hist = (const float2 *)hist;
    P.x = (const float2 *)x;
    P.n_in = (long long)nblocks * M2;
    P.B0 = B0;
    P.nblk = (long long)nblocks;
    P.Y = (float2 *)Y;
    const long long gfirst = (B0 / 8) & ~1LL;             // 8-block group containing B0, even
    const long long glast = (B0 + (long long)nblocks - 1) / 8; // inclusive
    const long long ngroups = glast - gfirst + 1;
    // one workgroup per CU (LDS-bound), each at least 8 groups (64 blocks)
    long long gpw = (ngroups + 255) / 256;
    if (gpw < 8) gpw = 8;
    gpw = (gpw + 1) & ~1LL;
    const long long nwg = (ngroups + gpw - 1) / gpw;
    P.gs0 = gfirst;
    P.gpw = (int)gpw;
    P.gend = glast + 1;
    const float2 *tw = (const float2 *)lqrt_twiddles();
    if (m == 4)
        hipLaunchKernelGGL(k_pfb2_an1024<8>, dim3((unsigned)nwg), dim3(NT), 0, st, P, (const float *)hsub, tw);
    else
        hipLaunchKernelGGL(k_pfb2_an1024<4>, dim3((unsigned)nwg), dim3(NT), 0, st, P, (const float *)hsub, tw);
    LQ_CHECK_LAUNCH();
    return 1;
}
