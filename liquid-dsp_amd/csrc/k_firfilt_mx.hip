// k_firfilt_mx.hip -- firfilt on the matrix cores (v_mfma_f32_16x16x32_bf16):
// crcf with 33..256 taps (h = 64 is the BASELINE config-1 shape), cccf and
// rrrf with 33..64 taps.
//
// Reference: src/filter/src/firfilt.c:322-359 (execute / execute_block),
// y[t] = scale * sum_{k<h} h[k] x[t-k].  The VALU kernel (k_firfilt.hip)
// spends 64 v_pk_fma_f32 per output and co-limits with HBM; here the
// convolution runs as a banded-Toeplitz GEMM on bf16 MFMA:
//
//   C[i][n] = sum_k H[i][k] B[k][n],  H[i][k] = h[i + 64 KB - k] (0 outside
//   0..64 KB - 1),  B[k][n] = x_comp(n)[s_seg(n) - 64 KB + k]
//
// i = output within a 16-output segment, n = (segment, re/im) column: a
// tile is 8 segments x 2 components = 128 complex outputs (rrrf: 16
// segments, 256 outputs), K = 16 + 64 KB in steps of 32.  (The 32x32x16 form
// of rounds 1-4 -- 512 outputs per tile, the accumulator staged through LDS
// for coalesced stores -- ran 1-15 % slower, r05w-r05zc.)
// float32 accuracy is kept by splitting both operands into three bf16 terms
// (x = x1 + x2 + x3, each the round-to-nearest bf16 of the remaining
// residual, exact to 2^-24 relative; products of bf16 terms are exact in the
// fp32 accumulator) and summing the six products whose order is at most
// 2^-16: x1h1, x1h2, x2h1, x1h3, x2h2, x3h1.  The dropped terms and the
// representation error are below 3 * 2^-24 |x||h| per tap -- the size of
// float32 rounding; tests hold the output to 2e-6 against a float64
// convolution and to the same 1e-5 normwise bound as every other kernel
// (tests/test_gpu_parity.py).
//
// Workgroup: 4 waves, persistent over grid-stride 2048-output chunks.  Each
// iteration: the 8 samples a lane prefetched are split into six bf16 planes
// (3 terms x re/im) of the chunk's span in LDS (the 64 KB-sample halo comes
// with the chunk), the next chunk's loads are issued, then each wave runs the
// MFMAs for its outputs and writes 16-byte stores straight from the
// accumulators (complex: after two DPP swaps with the partner lane).  The
// taps' A fragments are built once per workgroup from the padded fp32 taps.
//
// Range guard.  The split is float32-accurate only for finite values whose
// bf16 terms stay normal, and the band's zero entries multiply every sample
// of the 96-sample span (0 * Inf = NaN would reach outputs the reference
// keeps finite).  So each lane classifies the samples it stages (finite,
// zero or |x| in [2^-50, 2^50]); a chunk whose span (its 2048 samples plus
// the 64-sample halo) holds any other value is computed by the exact float32
// dot product over the true taps instead (k < hlen, as firfilt.c:322-338),
// from global memory -- the outputs the reference would produce, Inf / NaN
// propagation included.  Filters whose taps fail the same test never come
// here (lqk_fir_desc.mx_ok, checked at create time).
#include "lq_device.h"
#include "lq_kernels.h"

#include <cstdint>
#include <cstdio>


namespace {

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;           // 4 waves
constexpr int CH = 2048;          // outputs per chunk (512 per wave)

// 1 if v is outside the split's safe class: NaN, +-Inf, or a nonzero |v|
// outside [2^-50, 2^50] (integer compare on the magnitude bits; NaN and Inf
// patterns sit above 2^50's)
__device__ __forceinline__ unsigned unsafe_bits(float v)
{
    const unsigned a = __float_as_uint(v) & 0x7fffffffu;
    return (unsigned)(a - 0x26800000u) > (0x58800000u - 0x26800000u) ? (a != 0u) : 0u;
}
__device__ __forceinline__ unsigned unsafe4(v4f v)
{
    return unsafe_bits(v.x) | unsafe_bits(v.y) | unsafe_bits(v.z) | unsafe_bits(v.w);
}

// three-term bf16 split of a pair of floats
__device__ __forceinline__ void split3(v2f a, bf16x2 &t1, bf16x2 &t2, bf16x2 &t3)
{
    t1 = __builtin_convertvector(a, bf16x2);
    const v2f r1 = a - __builtin_convertvector(t1, v2f);
    t2 = __builtin_convertvector(r1, bf16x2);
    const v2f r2 = r1 - __builtin_convertvector(t2, v2f);
    t3 = __builtin_convertvector(r2, bf16x2);
}

// 8 complex samples of the stream starting at s (a multiple of 8); ext[t<0]
// comes from the 64-sample history win, samples at or past n are zero
template <int HALO = 64>
__device__ __forceinline__ v2f sample_at(const v2f *__restrict__ win, const v2f *__restrict__ x, long long n,
                                         long long t)
{
    return t < 0 ? win[HALO + t] : (t < n ? x[t] : v2f{0.f, 0.f});
}
// Exact float32 outputs t0 .. t0+cnt-1 (the range guard's path): the
// reference's dot product over the true taps, firfilt.c:322-338, then the
// scale.  Out of line, so the matrix path's register allocation is unchanged.
template <bool CC, int HALO>
__device__ __attribute__((noinline)) void exact_chunk_c(const v2f *__restrict__ win, const v2f *__restrict__ x,
                                                         long long n, v2f *__restrict__ y,
                                                         const float *__restrict__ hpad, int hlen, long long t0,
                                                         int cnt, float sre, float sim)
{
    for (int e = 0; e < cnt; e++) {
        const long long t = t0 + e;
        if (t >= n) break;
        v2f acc = {0.f, 0.f};
        for (int k = 0; k < hlen; k++) {
            const v2f v = sample_at<HALO>(win, x, n, t - k);
            if constexpr (CC) {
                const float hr = hpad[2 * k], hi = hpad[2 * k + 1];
                acc = v2f{fmaf(-hi, v.y, fmaf(hr, v.x, acc.x)), fmaf(hi, v.x, fmaf(hr, v.y, acc.y))};
            } else {
                acc = v2f{fmaf(hpad[k], v.x, acc.x), fmaf(hpad[k], v.y, acc.y)};
            }
        }
        // crcf: real scale per component (firfilt.c:337); cccf: complex product
        y[t] = CC ? v2f{acc.x * sre - acc.y * sim, acc.x * sim + acc.y * sre} : v2f{acc.x * sre, acc.y * sre};
    }
}

// 8 complex samples from byte offset off of the range-checked descriptor
// over x (zeros past the end): no branch, so the loads of the chunk after
// next stay in flight while this chunk runs (a branchy load merged its
// results through register copies, which made every prefetch wait at once)
__device__ __forceinline__ void load8b(__amdgpu_buffer_rsrc_t rx, unsigned off, v4f (&v)[4])
{
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = __builtin_amdgcn_raw_buffer_load_b128(rx, off + 16 * q, 0, 0);
}

// ---------------------------------------------------------------- 16x16 tiles
// k_firfilt_mx16: 33..64 taps on v_mfma_f32_16x16x32_bf16.  A tile is 16
// outputs x 16 columns (8 segments of 16 outputs x re/im), K = 96 in three
// steps of 32 (the band H[i][k] = h[i + 64 - k] again), so a tap matrix's
// fragments take 3 terms x 3 steps x 4 = 36 VGPRs (72 for cccf) against 72
// (144) for the 32x32 form, and the 16x16 accumulator needs no LDS staging:
// lane (col n = 2 seg + comp, row group g) holds rows 4g .. 4g+3 of one
// component, so two DPP swaps with the partner lane (n ^ 1) pair re / im
// (cccf: one more forms C1 -/+ C2 of the other component first), and each
// store instruction writes 128 consecutive outputs (1 KB).  Without the stage
// the LDS is the six bf16 planes only (26 KB): three workgroups per CU.
// Planes: no row pad, the component-1 plane 176 mod 256 bytes after
// component 0 (the 16 lanes of a B-operand ds_read_b128 -- 8 segments 32 B
// apart x 2 components -- land on 16 distinct bank groups).
template <int KB>
constexpr int pl16() { return (((CH + 64 * KB + 16) * 2 - 176 + 255) & ~255) + 176; }   // >= span + 16, == 176 mod 256
template <int KB>
constexpr int lds16() { return 6 * pl16<KB>() + 80; }
static_assert(pl16<1>() == 4272 && pl16<4>() % 256 == 176, "plane stride");

template <int KB>
__device__ __forceinline__ void put8_16(unsigned char *planes, int pos, const v4f (&v)[4])
{
    constexpr int PL16 = pl16<KB>();
    bf16x2 t[3][2][4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        split3(v2f{v[q].x, v[q].z}, t[0][0][q], t[1][0][q], t[2][0][q]);
        split3(v2f{v[q].y, v[q].w}, t[0][1][q], t[1][1][q], t[2][1][q]);
    }
#pragma unroll
    for (int p = 0; p < 3; p++)
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const u32x4 w = {__builtin_bit_cast(unsigned, t[p][c][0]), __builtin_bit_cast(unsigned, t[p][c][1]),
                             __builtin_bit_cast(unsigned, t[p][c][2]), __builtin_bit_cast(unsigned, t[p][c][3])};
            *reinterpret_cast<u32x4 *>(planes + (2 * p + c) * PL16 + 2 * pos) = w;
        }
}
template <int KB>
__device__ __forceinline__ void put1_16(unsigned char *planes, int pos, v2f v)
{
    constexpr int PL16 = pl16<KB>();
    bf16x2 t1, t2, t3;
    split3(v, t1, t2, t3);
    const bf16x2 t[3] = {t1, t2, t3};
#pragma unroll
    for (int p = 0; p < 3; p++) {
        *reinterpret_cast<__bf16 *>(planes + (2 * p) * PL16 + 2 * pos) = t[p].x;
        *reinterpret_cast<__bf16 *>(planes + (2 * p + 1) * PL16 + 2 * pos) = t[p].y;
    }
}
// the value of lane ^ 1 (DPP quad_perm [1, 0, 3, 2])
__device__ __forceinline__ float swap1(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
}

template <bool CC, int KB, int WPC>
__global__ __launch_bounds__(NT, WPC) void k_firfilt_mx16(const v2f *__restrict__ win, const v2f *__restrict__ x,
                                                        long long n, v2f *__restrict__ y,
                                                        const float *__restrict__ hpad, float sre, float sim,
                                                        long long nch, int hlen, lqk_hist_job hj)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    lq_hist_job_run<v2f>(hj);   // the object's next window (no launch of its own)
    constexpr int HALO = 64 * KB, PL16 = pl16<KB>();
    constexpr int NS = (16 + HALO + 31) / 32;   // K steps of 32 over the 16 + HALO band
    unsigned char *planes = smem;
    unsigned *sbad = reinterpret_cast<unsigned *>(smem + 6 * PL16);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r16 = lane & 15, kg = lane >> 4;
    constexpr int NA = CC ? 2 : 1;
    typedef float f32x4 __attribute__((ext_vector_type(4)));

    // A fragments: lane (row i = r16, k group kg) holds H[i][32 s + 8 kg + e]
    bf16x8 A[NA][3][NS];
#pragma unroll
    for (int a = 0; a < NA; a++)
#pragma unroll
        for (int s = 0; s < NS; s++) {
            bf16x2 t[3][4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                float hv[2];
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const int k = r16 + HALO - (32 * s + 8 * kg + 2 * q + u);
                    hv[u] = (k >= 0 && k < HALO) ? hpad[CC ? 2 * k + a : k] : 0.f;
                }
                split3(v2f{hv[0], hv[1]}, t[0][q], t[1][q], t[2][q]);
            }
#pragma unroll
            for (int p = 0; p < 3; p++)
                A[a][p][s] = bf16x8{t[p][0].x, t[p][0].y, t[p][1].x, t[p][1].y, t[p][2].x, t[p][2].y, t[p][3].x, t[p][3].y};
        }

    const long long G = gridDim.x, w = blockIdx.x;
    if (w >= nch) return;
    const long long cnt = (nch - w + G - 1) / G;
    if (tid < 3) sbad[tid] = 0u;
    unsigned *bad_mask = sbad + 4;
    if (tid < 16) bad_mask[tid] = 0u;
    // the last tile's K window reaches 16 positions past the span (H is
    // zero there): zero them once, so 0 * garbage cannot make a NaN
    if (tid < 6 * 16) *reinterpret_cast<__bf16 *>(planes + (tid / 16) * PL16 + 2 * (HALO + CH + tid % 16)) = __bf16(0.f);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)(n * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)y, (short)0, (int)(n * 8), 0x00020000);
    const unsigned OOB = 0xfffff000u;
    auto main_off = [&](long long k) -> unsigned {
        const long long c = w + k * G;
        return c < nch ? (unsigned)(CH * c + 8 * tid) * 8u : OOB;
    };
    auto halo_off = [&](long long k) -> unsigned {
        const long long c = w + k * G;
        return (c > 0 && c < nch && tid < HALO) ? (unsigned)(CH * c - HALO + tid) * 8u : OOB;
    };
    auto ldh = [&](unsigned off) -> v2f { return __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, off, 0, 0)); };
    __syncthreads();
    if (w == 0 && tid < HALO) {
        const v2f hv = win[tid];
        put1_16<KB>(planes, tid, hv);
        if (unsafe_bits(hv.x) | unsafe_bits(hv.y)) atomicOr(&sbad[0], 1u);
    }
    // one chunk of loads in flight per workgroup (issued as the previous
    // chunk's planes are written; with two or three register sets in flight
    // the kernel measured 0.5-1.5 % / 3 % slower, r05x)
    v4f xa[4];
    v2f ha;
    load8b(rx, main_off(0), xa);
    ha = ldh(halo_off(0));

    const int comp = r16 & 1, seg = r16 >> 1;
    auto step = [&](long long k, v4f (&xv)[4], v2f &hv) {
        const long long c = w + k * G;
        __syncthreads();   // the previous chunk's B-operand reads are done
        const int cs = (int)(k % 3);
        if (tid < HALO && c != 0) {
            put1_16<KB>(planes, tid, hv);
            if (unsafe_bits(hv.x) | unsafe_bits(hv.y)) atomicOr(&sbad[cs], 1u);
        }
        put8_16<KB>(planes, HALO + 8 * tid, xv);
        if (unsafe4(xv[0]) | unsafe4(xv[1]) | unsafe4(xv[2]) | unsafe4(xv[3])) atomicOr(&sbad[cs], 1u);
        if (tid == 0) sbad[(cs + 1) % 3] = 0u;
        load8b(rx, main_off(k + 1), xv);
        hv = ldh(halo_off(k + 1));
        __syncthreads();
        if (tid == 0 && sbad[cs] && c < nch) bad_mask[k >> 5] |= 1u << (k & 31);

#pragma unroll
        for (int tt = 0; tt < 4; tt++) {
            const int base = 512 * wave + 128 * tt;
            f32x4 C[NA];
#pragma unroll
            for (int a = 0; a < NA; a++) C[a] = f32x4{};
#pragma unroll
            for (int s = 0; s < NS; s++) {
                const unsigned char *bp = planes + comp * PL16 + 2 * (base + 16 * seg + 32 * s + 8 * kg);
                const bf16x8 b0 = *reinterpret_cast<const bf16x8 *>(bp);
                const bf16x8 b1 = *reinterpret_cast<const bf16x8 *>(bp + 2 * PL16);
                const bf16x8 b2 = *reinterpret_cast<const bf16x8 *>(bp + 4 * PL16);
#pragma unroll
                for (int a = 0; a < NA; a++) {
                    C[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[a][0][s], b2, C[a], 0, 0, 0);
                    C[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[a][1][s], b1, C[a], 0, 0, 0);
                    C[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[a][2][s], b0, C[a], 0, 0, 0);
                    C[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[a][0][s], b1, C[a], 0, 0, 0);
                    C[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[a][1][s], b0, C[a], 0, 0, 0);
                    C[a] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[a][0][s], b0, C[a], 0, 0, 0);
                }
            }
            // this lane: rows 4 kg .. 4 kg + 3 of component comp; cccf:
            // re = Hr xr - Hi xi (C1 here, C2 of the partner), im = Hr xi + Hi xr
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if constexpr (CC) {
                    const float o = swap1(C[1][r]);
                    v[r] = comp ? C[0][r] + o : C[0][r] - o;
                } else {
                    v[r] = C[0][r];
                }
            }
            // comp 0 keeps rows 4kg, 4kg+1 and takes their im; comp 1 rows
            // 4kg+2, 4kg+3 and takes their re
            const float r0 = swap1(comp ? v[0] : v[2]), r1 = swap1(comp ? v[1] : v[3]);
            v4f o = comp ? v4f{r0, v[2], r1, v[3]} : v4f{v[0], r0, v[1], r1};
            o = CC ? v4f{o.x * sre - o.y * sim, o.x * sim + o.y * sre, o.z * sre - o.w * sim, o.z * sim + o.w * sre}
                   : o * sre;   // crcf: real scale per component (firfilt.c:337)
            const unsigned off = (unsigned)(CH * c + base + 16 * seg + 4 * kg + 2 * comp) * 8u;
            __builtin_amdgcn_raw_buffer_store_b128(o, ry, c < nch ? off : OOB, 0, 0);
        }
    };
    for (long long k = 0; k < cnt; k++) step(k, xa, ha);
    __syncthreads();
    unsigned anybad = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) anybad |= bad_mask[i];
    if (anybad) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (int k = 0; k < (int)cnt; k++)
            if (bad_mask[k >> 5] & (1u << (k & 31)))
                exact_chunk_c<CC, HALO>(win, x, n, y, hpad, hlen, CH * (w + k * G) + 8 * tid, 8, sre, sim);
    }
}

// ---------------------------------------------------------------- rrrf
// Real samples: a wave's 1024 outputs, a chunk of 4096; three bf16 planes.
constexpr int CHR = 4096;
constexpr int SPANR = CHR + 64;

__device__ __forceinline__ float rsample_at(const float *__restrict__ win, const float *__restrict__ x, long long n,
                                            long long t)
{
    return t < 0 ? win[64 + t] : (t < n ? x[t] : 0.f);
}
__device__ __attribute__((noinline)) void exact_chunk_r(const float *__restrict__ win, const float *__restrict__ x,
                                                        long long n, float *__restrict__ y,
                                                        const float *__restrict__ hpad, int hlen, long long t0,
                                                        int cnt, float sre)
{
    for (int e = 0; e < cnt; e++) {
        const long long t = t0 + e;
        if (t >= n) break;
        float acc = 0.f;
        for (int k = 0; k < hlen; k++) acc = fmaf(hpad[k], rsample_at(win, x, n, t - k), acc);
        y[t] = acc * sre;
    }
}

__device__ __forceinline__ void load16rb(__amdgpu_buffer_rsrc_t rx, unsigned off, v4f (&v)[4])
{
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = __builtin_amdgcn_raw_buffer_load_b128(rx, off + 16 * q, 0, 0);
}

// rrrf on 16x16x32 tiles: the 16 columns of a tile are 16 segments of 16
// outputs (a wave's 1024 outputs are four tiles), K = 96 in three steps, and
// lane (segment n, row group g) holds outputs 16 n + 4 g .. + 3 -- one
// 16-byte store, and a store instruction writes the tile's 256 outputs (1 KB)
// contiguously, straight from the accumulator.  Planes: 16 B of pad per 16
// samples, so the 16 lanes of a B-operand ds_read_b128 (segments 32 B apart)
// land on 16 distinct bank groups.
__device__ __forceinline__ int poffr16(int pos) { return 2 * pos + 16 * (pos >> 4); }
constexpr int PLR16 = (((SPANR + 16) * 2 + 16 * ((SPANR + 16) >> 4)) + 255) & ~255;
constexpr int LDSR16 = 3 * PLR16 + 80;

__device__ __forceinline__ void put8r16(unsigned char *planes, int pos, v4f a, v4f b)
{
    bf16x2 t[3][4];
    split3(v2f{a.x, a.y}, t[0][0], t[1][0], t[2][0]);
    split3(v2f{a.z, a.w}, t[0][1], t[1][1], t[2][1]);
    split3(v2f{b.x, b.y}, t[0][2], t[1][2], t[2][2]);
    split3(v2f{b.z, b.w}, t[0][3], t[1][3], t[2][3]);
    const int o = poffr16(pos);
#pragma unroll
    for (int p = 0; p < 3; p++) {
        const u32x4 w = {__builtin_bit_cast(unsigned, t[p][0]), __builtin_bit_cast(unsigned, t[p][1]),
                         __builtin_bit_cast(unsigned, t[p][2]), __builtin_bit_cast(unsigned, t[p][3])};
        *reinterpret_cast<u32x4 *>(planes + p * PLR16 + o) = w;
    }
}
__device__ __forceinline__ void put4r16(unsigned char *planes, int pos, v4f a)
{
    bf16x2 t[3][2];
    split3(v2f{a.x, a.y}, t[0][0], t[1][0], t[2][0]);
    split3(v2f{a.z, a.w}, t[0][1], t[1][1], t[2][1]);
    const int o = poffr16(pos);
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < 3; p++)
        *reinterpret_cast<u32x2 *>(planes + p * PLR16 + o) =
            u32x2{__builtin_bit_cast(unsigned, t[p][0]), __builtin_bit_cast(unsigned, t[p][1])};
}

template <int WPC>
__global__ __launch_bounds__(NT, WPC) void k_firfilt_mx16_r(const float *__restrict__ win,
                                                            const float *__restrict__ x, long long n,
                                                            float *__restrict__ y, const float *__restrict__ hpad,
                                                            float sre, long long nch, int hlen, lqk_hist_job hj)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    lq_hist_job_run<float>(hj);   // the object's next window (no launch of its own)
    unsigned *sbad = reinterpret_cast<unsigned *>(smem + 3 * PLR16);
    unsigned char *planes = smem;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r16 = lane & 15, kg = lane >> 4;
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const long long G = gridDim.x, w = blockIdx.x;
    if (w >= nch) return;
    const long long cnt = (nch - w + G - 1) / G;

    bf16x8 A[3][3];   // [term][step]: lane (row i = r16, k group kg) holds H[i][32 s + 8 kg + e]
#pragma unroll
    for (int s = 0; s < 3; s++) {
        bf16x2 t[3][4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            float hv[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int k = r16 + 64 - (32 * s + 8 * kg + 2 * q + u);
                hv[u] = (k >= 0 && k < 64) ? hpad[k] : 0.f;
            }
            split3(v2f{hv[0], hv[1]}, t[0][q], t[1][q], t[2][q]);
        }
#pragma unroll
        for (int p = 0; p < 3; p++)
            A[p][s] = bf16x8{t[p][0].x, t[p][0].y, t[p][1].x, t[p][1].y, t[p][2].x, t[p][2].y, t[p][3].x, t[p][3].y};
    }
    if (tid < 3) sbad[tid] = 0u;
    unsigned *bad_mask = sbad + 4;
    if (tid < 16) bad_mask[tid] = 0u;
    // the last tile's K window reaches 16 positions past the span (H is zero there)
    if (tid < 3 * 16) *reinterpret_cast<__bf16 *>(planes + (tid / 16) * PLR16 + poffr16(SPANR + tid % 16)) = __bf16(0.f);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)(n * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)y, (short)0, (int)(n * 4), 0x00020000);
    const unsigned OOB = 0xfffff000u;
    auto main_off = [&](long long k) -> unsigned {
        const long long c = w + k * G;
        return c < nch ? (unsigned)(CHR * c + 16 * tid) * 4u : OOB;
    };
    auto halo_off = [&](long long k) -> unsigned {
        const long long c = w + k * G;
        return (c > 0 && c < nch && tid < 16) ? (unsigned)(CHR * c - 64 + 4 * tid) * 4u : OOB;
    };
    __syncthreads();
    if (w == 0 && tid < 16) {
        const v4f hv = {win[4 * tid], win[4 * tid + 1], win[4 * tid + 2], win[4 * tid + 3]};
        put4r16(planes, 4 * tid, hv);
        if (unsafe4(hv)) atomicOr(&sbad[0], 1u);
    }
    v4f xa[4], ha;   // one chunk of loads in flight
    load16rb(rx, main_off(0), xa);
    ha = __builtin_amdgcn_raw_buffer_load_b128(rx, halo_off(0), 0, 0);
    for (long long k = 0; k < cnt; k++) {
        const long long c = w + k * G;
        __syncthreads();   // the previous chunk's B-operand reads are done
        const int cs = (int)(k % 3);
        if (tid < 16 && c != 0) {
            put4r16(planes, 4 * tid, ha);
            if (unsafe4(ha)) atomicOr(&sbad[cs], 1u);
        }
        put8r16(planes, 64 + 16 * tid, xa[0], xa[1]);
        put8r16(planes, 64 + 16 * tid + 8, xa[2], xa[3]);
        if (unsafe4(xa[0]) | unsafe4(xa[1]) | unsafe4(xa[2]) | unsafe4(xa[3])) atomicOr(&sbad[cs], 1u);
        if (tid == 0) sbad[(cs + 1) % 3] = 0u;
        load16rb(rx, main_off(k + 1), xa);
        ha = __builtin_amdgcn_raw_buffer_load_b128(rx, halo_off(k + 1), 0, 0);
        __syncthreads();
        if (tid == 0 && sbad[cs] && c < nch) bad_mask[k >> 5] |= 1u << (k & 31);
#pragma unroll
        for (int tt = 0; tt < 4; tt++) {
            const int base = 1024 * wave + 256 * tt;
            f32x4 C = {};
#pragma unroll
            for (int s = 0; s < 3; s++) {
                const unsigned char *bp = planes + poffr16(base + 16 * r16 + 32 * s + 8 * kg);
                const bf16x8 b0 = *reinterpret_cast<const bf16x8 *>(bp);
                const bf16x8 b1 = *reinterpret_cast<const bf16x8 *>(bp + PLR16);
                const bf16x8 b2 = *reinterpret_cast<const bf16x8 *>(bp + 2 * PLR16);
                C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0][s], b2, C, 0, 0, 0);
                C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1][s], b1, C, 0, 0, 0);
                C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[2][s], b0, C, 0, 0, 0);
                C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0][s], b1, C, 0, 0, 0);
                C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[1][s], b0, C, 0, 0, 0);
                C = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[0][s], b0, C, 0, 0, 0);
            }
            const unsigned off = (unsigned)(CHR * c + base + 16 * r16 + 4 * kg) * 4u;
            __builtin_amdgcn_raw_buffer_store_b128(C * sre, ry, c < nch ? off : OOB, 0, 0);
        }
    }
    __syncthreads();
    unsigned anybad = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) anybad |= bad_mask[i];
    if (anybad) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (int k = 0; k < (int)cnt; k++)
            if (bad_mask[k >> 5] & (1u << (k & 31)))
                exact_chunk_r(win, x, n, y, hpad, hlen, CHR * (w + k * G) + 16 * tid, 16, sre);
    }
}

} // namespace

// Returns 1 if the call was handled on the matrix cores: rrrf, crcf or cccf,
// 33..64 taps (HP = 64, one chunk), not in place, 16-byte aligned x and y.
// Launches cover at most 2^28 complex / 2^29 real samples (2 GiB) so the
// range-checked load offsets fit 32 bits; a later launch takes its 64-sample
// history straight from the preceding input.
static void launch_mx(const lqk_fir_desc *d, const void *hist, const void *x, long long n, void *y,
                      const lqk_hist_job &hj, hipStream_t st)
{
    if (d->kind == 0) {   // rrrf: 4096-output chunks, four workgroups per CU (112 VGPRs, 38 KB of LDS)
        const long long nch = (n + CHR - 1) / CHR;
        const long long nwg = nch < 1024 ? nch : 1024;
        hipLaunchKernelGGL(k_firfilt_mx16_r<4>, dim3((unsigned)nwg), dim3(NT), LDSR16, st, (const float *)hist,
                           (const float *)x, n, (float *)y, (const float *)d->hpad, d->scale_re, nch, (int)d->hlen, hj);
        LQ_CHECK_LAUNCH();
        return;
    }
    const long long nch = (n + CH - 1) / CH;
    const int kb = (int)d->nchunk;   // 64-tap blocks
    // workgroups per CU by VGPRs: crcf 94 / 118 / 164 / 166 at 1..4 blocks
    // (four, four, three, three), cccf 155 (three).  Against the 32x32x16
    // kernel with its LDS stage (two per CU): cccf h = 64 0.65 -> 0.56 ms,
    // crcf h = 128 / 192 / 256 0.555 / 0.71 / 0.85 -> 0.50 / 0.62 / 0.75 ms
    // per 2^27 samples (r05x, r05za in profiles/r05_ab_experiments.txt)
    auto go = [&](auto kern, int wpc, int lds) {
        const long long g = nch < 256LL * wpc ? nch : 256LL * wpc;
        hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(NT), lds, st, (const v2f *)hist, (const v2f *)x, n,
                           (v2f *)y, (const float *)d->hpad, d->scale_re, d->scale_im, nch, (int)d->hlen, hj);
    };
    if (d->kind == 2) go(k_firfilt_mx16<true, 1, 3>, 3, lds16<1>());
    else if (kb == 1) go(k_firfilt_mx16<false, 1, 4>, 4, lds16<1>());   // (five per CU: same time, r06d)
    else if (kb == 2) go(k_firfilt_mx16<false, 2, 4>, 4, lds16<2>());
    else if (kb == 3) go(k_firfilt_mx16<false, 3, 3>, 3, lds16<3>());
    else go(k_firfilt_mx16<false, 4, 3>, 3, lds16<4>());
    LQ_CHECK_LAUNCH();
}

// Returns 1 if the call was handled on the matrix cores: rrrf, crcf or cccf,
// 33..64 taps (HP = 64, one chunk), taps in the split's safe range, not in
// place, 16-byte aligned x and y.
extern "C" int lqk_firfilt_mx(const lqk_fir_desc *d, const void *hist, const void *x, unsigned long long n,
                              void *y, const lqk_hist_job *job, void *stream)
{
    // 33..64 taps (one 64-tap block) for every type; 65..128 (two) for crcf
    if (d->hc != 64 || !(d->nchunk == 1 || (d->nchunk <= 4 && d->kind == 1)) || x == y || !d->mx_ok) return 0;
    if (((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return 0;
    if (n == 0) return 1;
    const size_t es = d->kind == 0 ? 4 : 8;
    const long long LCH = d->kind == 0 ? (1LL << 29) : (1LL << 28);
    for (long long o = 0; o < (long long)n; o += LCH) {
        const long long nn = ((long long)n - o) < LCH ? ((long long)n - o) : LCH;
        const char *xo = (const char *)x + o * es;
        // the window update rides on the first launch
        const lqk_hist_job hj = (o == 0 && job) ? *job : lqk_hist_job{nullptr, nullptr, 0ull, nullptr, 0u};
        launch_mx(d, o == 0 ? hist : (const void *)(xo - (size_t)64 * d->nchunk * es), xo, nn, (char *)y + o * es,
                  hj, (hipStream_t)stream);
    }
    return 1;
}
