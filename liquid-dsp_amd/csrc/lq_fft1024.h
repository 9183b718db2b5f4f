// lq_fft1024.h -- 1024-point FFT by one wave (64 lanes x 16 values): the
// transform of the firpfbch2 fast path (csrc/k_pfb2_fast.hip) in both
// directions, as a batched kernel for the generic channelizer / synthesizer
// paths and the FFT API.  16-point DFT over the lane's values (stride 64),
// twiddle W_1024^{t k1}, LDS transpose (row stride 68), 16-point DFT, twiddle
// W_64^{b r}, 4-point DFT across the lane quad through DPP; the result goes
// through the wave's LDS buffer into 16-byte stores.
#pragma once

#include "lq_device.h"

__device__ __forceinline__ void f1k_wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// tw1[k1*64 + t] = W_1024^{DIR t k1}, tw2[r*4 + b] = W_64^{DIR b r} (tw4096: exp(-2 pi i e/4096))
template <int DIR>
__device__ __forceinline__ void f1k_tables(float2 *tw1, float2 *tw2, const float2 *__restrict__ tw4096)
{
    for (int e = threadIdx.x; e < 1024; e += blockDim.x) {
        const int k1 = e >> 6, t = e & 63;
        float2 w = tw4096[(4 * t * k1) & 4095];
        tw1[e] = make_float2(w.x, DIR > 0 ? w.y : -w.y);
    }
    for (int e = threadIdx.x; e < 64; e += blockDim.x) {
        const int r = e >> 2, b = e & 3;
        float2 w = tw4096[(64 * b * r) & 4095];
        tw2[e] = make_float2(w.x, DIR > 0 ? w.y : -w.y);
    }
}

// v[k] = x[lane + 64 k] in; natural-order result left in B[k + 4 (k >> 8)]
// (B: 1088 float2 per wave).  1024 = 16 x 16 x 4 with packed arithmetic
// (lq_device.h): DFT16, twiddle, transpose, DFT16, twiddle, transpose, four
// DFT4 per lane; the same transform as the firpfbch2 fast path.
// SC: every output leaves multiplied by s1, then by s2 (the synthesizers'
// IFFT scalings, in the reference's order), in the last pass's registers.
template <int DIR, bool SC = false>
__device__ __forceinline__ void fft1024_wave(float2 (&v)[16], float2 *B, const float2 *tw1, const float2 *tw2,
                                             int lane, float s1 = 1.0f, float s2 = 1.0f)
{
    v2f p[16];
#pragma unroll
    for (int k = 0; k < 16; k++) p[k] = pk(v[k]);
    pk_dft16<DIR>(p);
#pragma unroll
    for (int k1 = 1; k1 < 16; k1++) p[k1] = pk_cmul(p[k1], pk(tw1[k1 * 64 + lane]));
    f1k_wave_fence();
#pragma unroll
    for (int k1 = 0; k1 < 16; k1++) B[k1 * 68 + lane] = unpk(p[k1]);
    f1k_wave_fence();
    const int k1 = lane >> 2, bq = lane & 3;
#pragma unroll
    for (int a = 0; a < 16; a++) p[a] = pk(B[k1 * 68 + 4 * a + bq]);
    pk_dft16<DIR>(p);
#pragma unroll
    for (int r = 1; r < 16; r++) p[r] = pk_cmul(p[r], pk(tw2[r * 4 + bq]));
    // C[k1][bq][r] at k1 + 16 r + 260 bq (conflict-free b64 writes, b128 reads)
    f1k_wave_fence();
#pragma unroll
    for (int r = 0; r < 16; r++) B[k1 + 16 * r + 260 * bq] = unpk(p[r]);
    f1k_wave_fence();
    typedef float v4f __attribute__((ext_vector_type(4)));
    // lane (t2, p2): bins k1 = 2 p2 + {0, 1}, r = t2 + 8u
    const int t2 = lane >> 3, p2 = lane & 7;
    v4f c[2][4];
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
        for (int q = 0; q < 4; q++)
            c[u][q] = *reinterpret_cast<const v4f *>(B + 2 * p2 + 16 * (t2 + 8 * u) + 260 * q);
    f1k_wave_fence();
#pragma unroll
    for (int u = 0; u < 2; u++) {
        v2f e0[4] = {c[u][0].xy, c[u][1].xy, c[u][2].xy, c[u][3].xy};
        v2f e1[4] = {c[u][0].zw, c[u][1].zw, c[u][2].zw, c[u][3].zw};
        pk_dft4<DIR>(e0[0], e0[1], e0[2], e0[3]);
        pk_dft4<DIR>(e1[0], e1[1], e1[2], e1[3]);
        // Y[K], K = 2 p2 + 16 (t2 + 8u) + 256 s, at K + 4 s
#pragma unroll
        for (int sidx = 0; sidx < 4; sidx++) {
            if constexpr (SC) {
                e0[sidx] = (e0[sidx] * v2f{s1, s1}) * v2f{s2, s2};
                e1[sidx] = (e1[sidx] * v2f{s1, s1}) * v2f{s2, s2};
            }
            const v4f val = {e0[sidx].x, e0[sidx].y, e1[sidx].x, e1[sidx].y};
            *reinterpret_cast<v4f *>(B + 2 * p2 + 16 * (t2 + 8 * u) + 260 * sidx) = val;
        }
    }
    f1k_wave_fence();
}

// fft1024_wave with the first twiddle W_1024^{DIR lane k1} formed in
// registers from a1 = W_4096^{4 lane}, a4 = W_4096^{16 lane} (forward
// values; twiddle16v) instead of the 8 KB tw1 table, for kernels without
// the LDS for it.  Same input and output layout.
template <int DIR>
__device__ __forceinline__ void fft1024_wave_rt(float2 (&v)[16], float2 *B, float2 a1, float2 a4, const float2 *tw2,
                                                int lane)
{
    dft16<DIR>(v);
    twiddle16v<DIR>(v, a1, a4);
    v2f p[16];
    f1k_wave_fence();
#pragma unroll
    for (int k1 = 0; k1 < 16; k1++) B[k1 * 68 + lane] = v[k1];
    f1k_wave_fence();
    const int k1 = lane >> 2, bq = lane & 3;
#pragma unroll
    for (int a = 0; a < 16; a++) p[a] = pk(B[k1 * 68 + 4 * a + bq]);
    pk_dft16<DIR>(p);
#pragma unroll
    for (int r = 1; r < 16; r++) p[r] = pk_cmul(p[r], pk(tw2[r * 4 + bq]));
    f1k_wave_fence();
#pragma unroll
    for (int r = 0; r < 16; r++) B[k1 + 16 * r + 260 * bq] = unpk(p[r]);
    f1k_wave_fence();
    typedef float v4f __attribute__((ext_vector_type(4)));
    const int t2 = lane >> 3, p2 = lane & 7;
    v4f c[2][4];
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
        for (int q = 0; q < 4; q++)
            c[u][q] = *reinterpret_cast<const v4f *>(B + 2 * p2 + 16 * (t2 + 8 * u) + 260 * q);
    f1k_wave_fence();
#pragma unroll
    for (int u = 0; u < 2; u++) {
        v2f e0[4] = {c[u][0].xy, c[u][1].xy, c[u][2].xy, c[u][3].xy};
        v2f e1[4] = {c[u][0].zw, c[u][1].zw, c[u][2].zw, c[u][3].zw};
        pk_dft4<DIR>(e0[0], e0[1], e0[2], e0[3]);
        pk_dft4<DIR>(e1[0], e1[1], e1[2], e1[3]);
#pragma unroll
        for (int sidx = 0; sidx < 4; sidx++) {
            const v4f val = {e0[sidx].x, e0[sidx].y, e1[sidx].x, e1[sidx].y};
            *reinterpret_cast<v4f *>(B + 2 * p2 + 16 * (t2 + 8 * u) + 260 * sidx) = val;
        }
    }
    f1k_wave_fence();
}
