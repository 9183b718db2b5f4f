// lq_fft1024.h -- 1024-point FFT by one wave (64 lanes x 16 values): the
// transform of the firpfbch2 fast path (csrc/k_pfb2_fast.hip) in both
// directions, as a batched kernel for the generic channelizer / synthesizer
// paths and the FFT API.  16-point DFT over the lane's values (stride 64),
// twiddle W_1024^{t k1}, LDS transpose (row stride 68), 16-point DFT, twiddle
// W_64^{b r}, 4-point DFT across the lane quad through DPP; the result goes
// through the wave's LDS buffer into 16-byte stores.
#pragma once

#include "lq_device.h"

template <int X>
__device__ __forceinline__ float2 f1k_quad_xor(float2 v)
{
    constexpr int ctrl = X == 1 ? 0xB1 : 0x4E;
    const int a = __builtin_amdgcn_mov_dpp(__float_as_int(v.x), ctrl, 0xF, 0xF, false);
    const int b = __builtin_amdgcn_mov_dpp(__float_as_int(v.y), ctrl, 0xF, 0xF, false);
    return make_float2(__int_as_float(a), __int_as_float(b));
}

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
// (B: 1088 float2 per wave).
template <int DIR>
__device__ __forceinline__ void fft1024_wave(float2 (&v)[16], float2 *B, const float2 *tw1, const float2 *tw2,
                                             int lane)
{
    dft16<DIR>(v);
#pragma unroll
    for (int k1 = 1; k1 < 16; k1++) v[k1] = cmul(v[k1], tw1[k1 * 64 + lane]);
    f1k_wave_fence();
#pragma unroll
    for (int k1 = 0; k1 < 16; k1++) B[k1 * 68 + lane] = v[k1];
    f1k_wave_fence();
    const int k1 = lane >> 2, bq = lane & 3;
#pragma unroll
    for (int a = 0; a < 16; a++) v[a] = B[k1 * 68 + 4 * a + bq];
    dft16<DIR>(v);
#pragma unroll
    for (int r = 1; r < 16; r++) v[r] = cmul(v[r], tw2[r * 4 + bq]);
    const float sg2 = (bq & 2) ? -1.0f : 1.0f, sg1 = (bq & 1) ? -1.0f : 1.0f;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const float2 p = f1k_quad_xor<2>(v[r]);
        float2 u = make_float2(fmaf(sg2, v[r].x, p.x), fmaf(sg2, v[r].y, p.y));
        if (bq == 3) u = DIR > 0 ? cmul_mj(u) : cmul_pj(u);
        const float2 p2 = f1k_quad_xor<1>(u);
        v[r] = make_float2(fmaf(sg1, u.x, p2.x), fmaf(sg1, u.y, p2.y));
    }
    // lane (k1, bq) holds Y[k1 + 16 r + 256 s], s = bitrev2(bq)
    const int s = ((bq & 1) << 1) | (bq >> 1);
    f1k_wave_fence();
#pragma unroll
    for (int r = 0; r < 16; r++) B[k1 + 16 * r + 260 * s] = v[r];
    f1k_wave_fence();
}
