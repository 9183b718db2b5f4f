// k_firfilt_mx.hip -- firfilt_crcf for filters of 33..64 taps on the matrix
// cores (the BASELINE config-1 shape, h = 64).
//
// Reference: src/filter/src/firfilt.c:322-359 (execute / execute_block),
// y[t] = scale * sum_{k<h} h[k] x[t-k].  The VALU kernel (k_firfilt.hip)
// spends 64 v_pk_fma_f32 per output and co-limits with HBM; here the
// convolution runs as a banded-Toeplitz GEMM on v_mfma_f32_32x32x16_bf16:
//
//   C[i][n] = sum_{j<96} H[i][j] B[j][n],  H[i][j] = h[i + 64 - j] (0 outside
//   0..63),  B[j][n] = x_comp(n)[s_seg(n) - 64 + j]
//
// i = output within a 32-sample segment, n = (segment, re/im) column, so one
// 32x32 tile is 16 segments x 2 components = 512 complex outputs, six K = 16
// steps.  float32 accuracy is kept by splitting both operands into three
// bf16 terms (x = x1 + x2 + x3, each the round-to-nearest bf16 of the
// remaining residual, exact to 2^-24 relative; products of bf16 terms are
// exact in the fp32 accumulator) and summing the six products whose order is
// at most 2^-16: x1h1, x1h2, x2h1, x1h3, x2h2, x3h1.  The dropped terms and
// the representation error are below 3 * 2^-24 |x||h| per tap -- the size of
// float32 rounding; tests hold the output to the same 1e-5 normwise bound as
// every other kernel (tests/test_gpu_parity.py).
//
// Workgroup: 4 waves, persistent over a contiguous run of 2048-output chunks.
// Each iteration: the 8 samples a lane prefetched are split into six bf16
// planes (3 terms x re/im) of the chunk's 2112-sample span in LDS (16 bytes of
// pad per 32 samples: the B-operand reads of the 16 segments of a tile land
// on 16 distinct bank groups; the 64-sample halo comes from a small buffer the
// previous iteration's tail lanes filled), the loads of the chunk after next
// are issued (two chunks, 32 KB per workgroup, stay in flight), then each wave
// runs 36 MFMAs for its 512 outputs, stages the accumulator through LDS and
// writes 16-byte stores.  The taps' A fragments (3 terms x 6 K steps, 72
// VGPRs) are built once per workgroup from the padded fp32 taps.
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

// crcf 33..64 taps: persistent workgroups, two per CU (A/B on one box: 0.804 ms
// vs 0.822-0.826 at three per CU with two chunks in flight, 0.819-0.821 two
// per CU with two; profiles/r04_ab_experiments.txt)
constexpr int FMX_WGS = 512;

namespace {

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;           // 4 waves
constexpr int CH = 2048;          // outputs per chunk (4 tiles of 512)
// Span: the samples a chunk's tiles read, CH plus a halo of 64 KB samples
// (KB = 1: 33..64 taps, every type; KB = 2: 65..128 taps, crcf -- a
// 160-wide band, ten K steps instead of six).  Bytes per plane: the span
// (5280 for KB = 1) rounded up to 256 B, so the planes of the two components
// start on the same bank -- with the 5280-byte stride every 16-lane group of
// a B-operand ds_read_b128 had a 2-way bank conflict (SQ_LDS_BANK_CONFLICT
// was half of the LDS-active cycles).
template <int KB>
constexpr int plb_kb() { return ((CH + 64 * KB) * 2 + 16 * ((CH + 64 * KB) / 32) + 255) & ~255; }
constexpr int SSTR = 68;          // floats per staged segment (32 x re/im + pad)
// crcf: one staged accumulator per wave (49664 B: three workgroups per CU;
// KB = 2: 53504 B and 219 VGPRs, two per CU); cccf: two (the real- and
// imaginary-tap products; 67072 B: two per CU)
// KB > 2 (129..256 taps, crcf): the A fragments (3 terms x 2 + 4 KB steps,
// 216 VGPRs at KB = 4) come from LDS instead: the band H[i][j] = h[i + 64 KB -
// j] is Toeplitz, so lane row i's fragment of step s is 8 consecutive entries
// of g[k] = h[64 KB + 31 - k] from k = 31 - i + 16 s + 8 hh; eight copies of
// each term's g shifted by c = (31 - i) mod 8 make every fragment one aligned
// 16-byte read
template <int KB>
constexpr int glen_kb() { return 16 * (2 + 4 * KB) + 32; }
// bf16 terms of the taps whose A fragments come from LDS: all three past 128
// taps (KB > 2), none below (taking terms 2 and 3 from LDS at KB = 1 to free
// registers for a third chunk measured 0.915-0.925 ms against 0.803-0.805:
// the fragment reads sit on the MFMA chain, DESIGN (f)3)
template <bool CC, int KB>
constexpr int nal_kb() { return KB > 2 ? 3 : 0; }
// chunks of loads in flight per workgroup (register sets): three for crcf
// 33..64 taps, two for 65..256 taps and for cccf (two workgroups per CU each;
// four measured the same as three, and so did staging the span by LDS-DMA
// into one raw LDS buffer, r05q in profiles/r05_ab_experiments.txt)
template <bool CC, int KB>
constexpr int nbuf_kb() { return CC ? 2 : (KB == 1 ? 3 : 2); }
// elements between the eight shifted copies: at least NAL GL, and 16 mod 128
// (32 B mod 256), so the 16 lanes of a ds_read_b128 pass -- eight copies at
// two bases 16 B apart -- land on 16 distinct bank groups (a stride that is
// a multiple of 256 B put all eight copies on the same banks)
template <bool CC, int KB>
constexpr int acs_kb() { return nal_kb<CC, KB>() ? ((nal_kb<CC, KB>() * glen_kb<KB>() - 16 + 127) / 128) * 128 + 16 : 0; }
template <bool CC, int KB>
constexpr int acp_bytes() { return 8 * acs_kb<CC, KB>() * 2; }
template <bool CC, int KB = 1>
constexpr int lds_bytes_mx() { return 6 * plb_kb<KB>() + (CC ? 2 : 1) * 4 * 16 * SSTR * 4 + acp_bytes<CC, KB>(); }

static_assert(3 * (lds_bytes_mx<false, 1>() + 80) <= 160 * 1024, "crcf KB = 1: three workgroups per CU");
static_assert(2 * (lds_bytes_mx<false, 4>() + 80) <= 160 * 1024, "crcf KB = 4: two workgroups per CU");

__device__ __forceinline__ int poff(int pos) { return 2 * pos + 16 * (pos >> 5); }

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

// write 8 consecutive complex samples (ring position pos, a multiple of 8)
// into the six planes: plane (p, c) = term p of component c.  v[q] holds
// samples 2q and 2q+1 as (re, im, re, im).
__device__ __forceinline__ void put8(unsigned char *planes, int pstride, int pos, const v4f (&v)[4])
{
    bf16x2 t[3][2][4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        split3(v2f{v[q].x, v[q].z}, t[0][0][q], t[1][0][q], t[2][0][q]);
        split3(v2f{v[q].y, v[q].w}, t[0][1][q], t[1][1][q], t[2][1][q]);
    }
    const int o = poff(pos);
#pragma unroll
    for (int p = 0; p < 3; p++)
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const u32x4 w = {__builtin_bit_cast(unsigned, t[p][c][0]), __builtin_bit_cast(unsigned, t[p][c][1]),
                             __builtin_bit_cast(unsigned, t[p][c][2]), __builtin_bit_cast(unsigned, t[p][c][3])};
            *reinterpret_cast<u32x4 *>(planes + (2 * p + c) * pstride + o) = w;
        }
}

// one complex sample at ring position pos into the six planes
__device__ __forceinline__ void put1(unsigned char *planes, int pstride, int pos, v2f v)
{
    bf16x2 t1, t2, t3;
    split3(v, t1, t2, t3);   // (re, im) terms
    const int o = poff(pos);
    const bf16x2 t[3] = {t1, t2, t3};
#pragma unroll
    for (int p = 0; p < 3; p++) {
        *reinterpret_cast<__bf16 *>(planes + (2 * p) * pstride + o) = t[p].x;
        *reinterpret_cast<__bf16 *>(planes + (2 * p + 1) * pstride + o) = t[p].y;
    }
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

// CC: complex taps (cccf).  Then H = Hr + j Hi and the tile keeps two
// accumulators, C1 = Hr [Xr | Xi] and C2 = Hi [Xr | Xi]; y = (C1.re - C2.im,
// C1.im + C2.re) is formed when the staged accumulators are read back.
template <bool CC, int KB>
__global__ __launch_bounds__(NT, 2) void k_firfilt_mx(const v2f *__restrict__ win,
                                                              const v2f *__restrict__ x, long long n,
                                                              v2f *__restrict__ y, const float *__restrict__ hpad,
                                                              float sre, float sim, long long nch, int hlen)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // per step k % 3: nonzero if the chunk's span holds an unsafe sample;
    // kept after the dynamic region so its base stays 16-byte aligned
    constexpr int HALO = 64 * KB, NS = 2 + 4 * KB, PLB = plb_kb<KB>();
    unsigned *sbad = reinterpret_cast<unsigned *>(smem + lds_bytes_mx<CC, KB>());
    unsigned char *planes = smem;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, hh = lane >> 5;
    constexpr int NA = CC ? 2 : 1;   // tap matrices
    float *stage = reinterpret_cast<float *>(smem + 6 * PLB) + wave * NA * 16 * SSTR;

    // A fragments: lane (row i = r32, k half hh) holds H[i][16s + 8hh + e]
    // (cccf: hpad holds (re, im) pairs; matrix a takes component a); terms
    // NAR.. come from LDS per step
    constexpr int NAL = nal_kb<CC, KB>(), NAR = 3 - NAL;
    bf16x8 A[NA][NAR > 0 ? NAR : 1][NAR > 0 ? NS : 1];
    __bf16 *acp = reinterpret_cast<__bf16 *>(smem + 6 * PLB + NA * 4 * 16 * SSTR * 4);
    constexpr int GL = glen_kb<KB>(), ACS = acs_kb<CC, KB>();
    if constexpr (NAL > 0) {
        // copy c, term p >= NAR: G[c][p - NAR][k] = term p of g[k + c], g[k] = h[HALO + 31 - k]
        for (int e = tid; e < 8 * GL; e += NT) {
            const int c = e / GL, k = e - c * GL;
            const int hk = HALO + 31 - (k + c);
            const float hv = (hk >= 0 && hk < HALO) ? hpad[hk] : 0.f;
            bf16x2 t[3];
            split3(v2f{hv, 0.f}, t[0], t[1], t[2]);
#pragma unroll
            for (int p = NAR; p < 3; p++) acp[c * ACS + (p - NAR) * GL + k] = t[p].x;
        }
    }
    if constexpr (NAR > 0) {
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
                    const int k = r32 + HALO - (16 * s + 8 * hh + 2 * q + u);
                    hv[u] = (k >= 0 && k < HALO) ? hpad[CC ? 2 * k + a : k] : 0.f;
                }
                split3(v2f{hv[0], hv[1]}, t[0][q], t[1][q], t[2][q]);
            }
#pragma unroll
            for (int p = 0; p < NAR; p++)
                A[a][p][s] =
                    bf16x8{t[p][0].x, t[p][0].y, t[p][1].x, t[p][1].y, t[p][2].x, t[p][2].y, t[p][3].x, t[p][3].y};
        }
    }
    // this lane's copy (31 - r32) mod 8 and its fragment base (+ 16 s: step s; + (p - NAR) GL: term p)
    const __bf16 *acl = NAL > 0 ? acp + ((31 - r32) & 7) * ACS + ((31 - r32) & ~7) + 8 * hh : nullptr;

    // Chunks are dealt grid-stride (workgroup w takes chunks w, w + G, ...):
    // the chip then streams one contiguous window of the input at a time.
    // Contiguous runs of chunks per workgroup put ~800 concurrent streams on
    // addresses a run apart and ran the same memory pattern 9 % slower
    // (0.80 vs 0.73 ms per 2^28 samples, tools/mb/mb_bw4.hip).  So a chunk's
    // 64-sample halo (the previous chunk's tail, another workgroup's) is
    // loaded with it: wave 0 fetches one sample per lane.  Plane position
    // p of chunk c = stream sample CH c - 64 + p.
    const long long G = gridDim.x, w = blockIdx.x;
    if (w >= nch) return;
    const long long cnt = (nch - w + G - 1) / G;
    if (tid < 3) sbad[tid] = 0u;
    unsigned *bad_mask = sbad + 4;   // steps k of this workgroup that need the exact path
    if (tid < 16) bad_mask[tid] = 0u;
    // The loop's memory operations are branch-free -- range-checked buffer
    // loads and stores; a step past the workgroup's last chunk (odd counts)
    // lands out of range -- so the compiler's vmcnt waits only for the rows a
    // step consumes and earlier stores stay in flight.  The host keeps n * 8
    // bytes below 2^31 per launch.
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)(n * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)y, (short)0, (int)(n * 8), 0x00020000);
    const unsigned OOB = 0xfffff000u;   // an offset past any launch's range
    auto main_off = [&](long long k) -> unsigned {
        const long long c = w + k * G;
        return c < nch ? (unsigned)(CH * c + 8 * tid) * 8u : OOB;
    };
    // halo sample of lane tid < 64; chunk 0's halo is the history (prologue)
    auto halo_off = [&](long long k) -> unsigned {
        const long long c = w + k * G;
        return (c > 0 && c < nch && tid < HALO) ? (unsigned)(CH * c - HALO + tid) * 8u : OOB;
    };
    auto ldh = [&](unsigned off) -> v2f { return __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(rx, off, 0, 0)); };
    __syncthreads();
    if (w == 0 && tid < HALO) {
        const v2f hv = win[tid];
        put1(planes, PLB, tid, hv);
        if (unsafe_bits(hv.x) | unsafe_bits(hv.y)) atomicOr(&sbad[0], 1u);
    }
    // NB chunks in flight per workgroup: register sets (xa, ha) / (xb, hb)
    // [/ (xc, hc)] rotate (the loop is unrolled by NB so no set is ever
    // copied, which would wait on its loads early)
    constexpr int NB = nbuf_kb<CC, KB>();
    v4f xa[4], xb[4], xc[4], xd[4];
    v2f ha, hb, hc, hd;
    load8b(rx, main_off(0), xa);
    ha = ldh(halo_off(0));
    load8b(rx, main_off(1), xb);
    hb = ldh(halo_off(1));
    if constexpr (NB > 2) {
        load8b(rx, main_off(2), xc);
        hc = ldh(halo_off(2));
    }
    if constexpr (NB > 3) {
        load8b(rx, main_off(3), xd);
        hd = ldh(halo_off(3));
    }

    // B operand: lane column n = r32 -> segment sg = n & 15, component n >> 4
    const int sg = r32 & 15, comp = r32 >> 4;
    auto step = [&](long long k, v4f (&xv)[4], v2f &hv) {
        const long long c = w + k * G;
        __syncthreads();   // the previous chunk's MFMA reads are done
        const int cs = (int)(k % 3);
        // chunk 0's halo planes came from the history in the prologue
        if (tid < HALO && c != 0) {
            put1(planes, PLB, tid, hv);
            if (unsafe_bits(hv.x) | unsafe_bits(hv.y)) atomicOr(&sbad[cs], 1u);
        }
        put8(planes, PLB, HALO + 8 * tid, xv);
        if (unsafe4(xv[0]) | unsafe4(xv[1]) | unsafe4(xv[2]) | unsafe4(xv[3])) atomicOr(&sbad[cs], 1u);
        if (tid == 0) sbad[(cs + 1) % 3] = 0u;   // step k+1's slot (last read in step k-2)
        load8b(rx, main_off(k + NB), xv);
        hv = ldh(halo_off(k + NB));
        __syncthreads();
        if (tid == 0 && sbad[cs] && c < nch) bad_mask[k >> 5] |= 1u << (k & 31);

        f32x16 C[NA];
#pragma unroll
        for (int a = 0; a < NA; a++) C[a] = f32x16{};
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int pos = 512 * wave + 32 * sg + 16 * s + 8 * hh;
            const unsigned char *bp = planes + comp * PLB + poff(pos);
            const bf16x8 b0 = *reinterpret_cast<const bf16x8 *>(bp);
            const bf16x8 b1 = *reinterpret_cast<const bf16x8 *>(bp + 2 * PLB);
            const bf16x8 b2 = *reinterpret_cast<const bf16x8 *>(bp + 4 * PLB);
            // terms of order 2^-16 first, then 2^-8, then the leading product
            bf16x8 al[NAL > 0 ? NAL : 1];
#pragma unroll
            for (int p = 0; p < NAL; p++) al[p] = *reinterpret_cast<const bf16x8 *>(acl + p * GL + 16 * s);
#pragma unroll
            for (int a = 0; a < NA; a++) {
                bf16x8 af[3];
#pragma unroll
                for (int p = 0; p < 3; p++) af[p] = p < NAR ? A[a][p < NAR ? p : 0][NAR > 0 ? s : 0] : al[p >= NAR ? p - NAR : 0];
                C[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], b2, C[a], 0, 0, 0);
                C[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], b1, C[a], 0, 0, 0);
                C[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2], b0, C[a], 0, 0, 0);
                C[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], b1, C[a], 0, 0, 0);
                C[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], b0, C[a], 0, 0, 0);
                C[a] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], b0, C[a], 0, 0, 0);
            }
        }

        // accumulator (col r32, row (r&3) + 8(r>>2) + 4hh) -> stage[a][sg][i][comp]
#pragma unroll
        for (int a = 0; a < NA; a++)
#pragma unroll
            for (int r = 0; r < 16; r++)
                stage[a * 16 * SSTR + sg * SSTR + 2 * ((r & 3) + 8 * (r >> 2) + 4 * hh) + comp] = C[a][r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // 16-byte pairs; a pair straddling n (odd n) keeps its in-range half
        // (the range check is per dword)
        const unsigned o0 = (unsigned)(CH * c + 512 * wave) * 8u;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int o = 2 * (lane + 64 * q);
            v4f a = *reinterpret_cast<const v4f *>(stage + (o >> 5) * SSTR + 2 * (o & 31));
            if constexpr (CC) {
                const v4f b = *reinterpret_cast<const v4f *>(stage + 16 * SSTR + (o >> 5) * SSTR + 2 * (o & 31));
                a = v4f{a.x - b.y, a.y + b.x, a.z - b.w, a.w + b.z};
            }
            const v4f r = CC ? v4f{a.x * sre - a.y * sim, a.x * sim + a.y * sre, a.z * sre - a.w * sim,
                                   a.z * sim + a.w * sre}
                             : a * sre;   // crcf: real scale per component (firfilt.c:337)
            // default cache policy: over five fresh buffer pairs the kernel ran
            // 0.835-0.905 ms (mean 0.877) against 0.819-0.927 (0.891) with
            // non-temporal stores (its time depends on where the 2 GB buffers
            // land, r05n_firfilt_alloc.txt / r05_ab_experiments.txt)
            __builtin_amdgcn_raw_buffer_store_b128(r, ry, c < nch ? o0 + 8u * o : OOB, 0, 0);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (long long k = 0; k < cnt; k += NB) {
        step(k, xa, ha);
        step(k + 1, xb, hb);
        if constexpr (NB > 2) step(k + 2, xc, hc);
        if constexpr (NB > 3) step(k + 3, xd, hd);
    }
    // the range guard's chunks: the exact float32 outputs overwrite what the
    // matrix path stored for them.  Only workgroup-scope ordering is needed
    // (the same workgroup wrote them); no fence at all in the common case (a
    // device-scope fence here writes back L2 in every workgroup: +12 %)
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
// Real samples: the 32 columns of a tile are 32 segments, so a wave's tile is
// 1024 outputs and a chunk 4096; three bf16 planes.
constexpr int CHR = 4096;
constexpr int SPANR = CHR + 64;
constexpr int PLBR = SPANR * 2 + 16 * (SPANR / 32);   // 10400
constexpr int SSTRR = 36;                              // floats per staged segment (32 + pad)
constexpr int LDS_BYTES_R = 3 * PLBR + 4 * 32 * SSTRR * 4;

__device__ __forceinline__ float rsample_at(const float *__restrict__ win, const float *__restrict__ x, long long n,
                                            long long t)
{
    return t < 0 ? win[64 + t] : (t < n ? x[t] : 0.f);
}
// 8 real samples (v4f pair) into the three planes at pos (a multiple of 8)
__device__ __forceinline__ void put8r(unsigned char *planes, int pstride, int pos, v4f a, v4f b)
{
    bf16x2 t[3][4];
    split3(v2f{a.x, a.y}, t[0][0], t[1][0], t[2][0]);
    split3(v2f{a.z, a.w}, t[0][1], t[1][1], t[2][1]);
    split3(v2f{b.x, b.y}, t[0][2], t[1][2], t[2][2]);
    split3(v2f{b.z, b.w}, t[0][3], t[1][3], t[2][3]);
    const int o = poff(pos);
#pragma unroll
    for (int p = 0; p < 3; p++) {
        const u32x4 w = {__builtin_bit_cast(unsigned, t[p][0]), __builtin_bit_cast(unsigned, t[p][1]),
                         __builtin_bit_cast(unsigned, t[p][2]), __builtin_bit_cast(unsigned, t[p][3])};
        *reinterpret_cast<u32x4 *>(planes + p * pstride + o) = w;
    }
}

// 4 real samples into the three planes at pos (a multiple of 4)
__device__ __forceinline__ void put4r(unsigned char *planes, int pstride, int pos, v4f a)
{
    bf16x2 t[3][2];
    split3(v2f{a.x, a.y}, t[0][0], t[1][0], t[2][0]);
    split3(v2f{a.z, a.w}, t[0][1], t[1][1], t[2][1]);
    const int o = poff(pos);
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int p = 0; p < 3; p++)
        *reinterpret_cast<u32x2 *>(planes + p * pstride + o) =
            u32x2{__builtin_bit_cast(unsigned, t[p][0]), __builtin_bit_cast(unsigned, t[p][1])};
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

__global__ __launch_bounds__(NT, 3) void k_firfilt_mx_r(const float *__restrict__ win, const float *__restrict__ x,
                                                       long long n, float *__restrict__ y,
                                                       const float *__restrict__ hpad, float sre, long long nch,
                                                       int hlen)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned *sbad = reinterpret_cast<unsigned *>(smem + LDS_BYTES_R);   // as k_firfilt_mx
    unsigned char *planes = smem;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r32 = lane & 31, hh = lane >> 5;
    float *stage = reinterpret_cast<float *>(smem + 3 * PLBR) + wave * 32 * SSTRR;
    // grid-stride chunks, each with its own 64-sample halo (lanes 0..15, four
    // samples each), as k_firfilt_mx
    const long long G = gridDim.x, w = blockIdx.x;
    if (w >= nch) return;
    const long long cnt = (nch - w + G - 1) / G;

    bf16x8 A[3][6];
#pragma unroll
    for (int s = 0; s < 6; s++) {
        bf16x2 t[3][4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            float hv[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int k = r32 + 64 - (16 * s + 8 * hh + 2 * q + u);
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
        put4r(planes, PLBR, 4 * tid, hv);
        if (unsafe4(hv)) atomicOr(&sbad[0], 1u);
    }
    v4f xa[4], xb[4], ha, hb;
    load16rb(rx, main_off(0), xa);
    ha = __builtin_amdgcn_raw_buffer_load_b128(rx, halo_off(0), 0, 0);
    load16rb(rx, main_off(1), xb);
    hb = __builtin_amdgcn_raw_buffer_load_b128(rx, halo_off(1), 0, 0);
    const int sg = r32;   // B column = segment
    auto step = [&](long long k, v4f (&xv)[4], v4f &hv) {
        const long long c = w + k * G;
        __syncthreads();
        const int cs = (int)(k % 3);
        if (tid < 16 && c != 0) {
            put4r(planes, PLBR, 4 * tid, hv);
            if (unsafe4(hv)) atomicOr(&sbad[cs], 1u);
        }
        put8r(planes, PLBR, 64 + 16 * tid, xv[0], xv[1]);
        put8r(planes, PLBR, 64 + 16 * tid + 8, xv[2], xv[3]);
        if (unsafe4(xv[0]) | unsafe4(xv[1]) | unsafe4(xv[2]) | unsafe4(xv[3]))
            atomicOr(&sbad[cs], 1u);
        if (tid == 0) sbad[(cs + 1) % 3] = 0u;
        load16rb(rx, main_off(k + 2), xv);
        hv = __builtin_amdgcn_raw_buffer_load_b128(rx, halo_off(k + 2), 0, 0);
        __syncthreads();
        if (tid == 0 && sbad[cs] && c < nch) bad_mask[k >> 5] |= 1u << (k & 31);
        f32x16 C = {};
#pragma unroll
        for (int s = 0; s < 6; s++) {
            const int pos = 1024 * wave + 32 * sg + 16 * s + 8 * hh;
            const unsigned char *bp = planes + poff(pos);
            const bf16x8 b0 = *reinterpret_cast<const bf16x8 *>(bp);
            const bf16x8 b1 = *reinterpret_cast<const bf16x8 *>(bp + PLBR);
            const bf16x8 b2 = *reinterpret_cast<const bf16x8 *>(bp + 2 * PLBR);
            C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0][s], b2, C, 0, 0, 0);
            C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1][s], b1, C, 0, 0, 0);
            C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2][s], b0, C, 0, 0, 0);
            C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0][s], b1, C, 0, 0, 0);
            C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1][s], b0, C, 0, 0, 0);
            C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0][s], b0, C, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; r++) stage[sg * SSTRR + (r & 3) + 8 * (r >> 2) + 4 * hh] = C[r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const unsigned o0 = (unsigned)(CHR * c + 1024 * wave) * 4u;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int o = 4 * (lane + 64 * q);
            const v4f a = *reinterpret_cast<const v4f *>(stage + (o >> 5) * SSTRR + (o & 31)) * sre;
            __builtin_amdgcn_raw_buffer_store_b128(a, ry, c < nch ? o0 + 4u * o : OOB, 0, 2);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (long long k = 0; k < cnt; k += 2) {
        step(k, xa, ha);
        step(k + 1, xb, hb);
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
                      hipStream_t st)
{
    if (d->kind == 0) {   // rrrf: 4096-output chunks, three workgroups per CU
        const long long nch = (n + CHR - 1) / CHR;
        const long long nwg = nch < 768 ? nch : 768;
        hipLaunchKernelGGL(k_firfilt_mx_r, dim3((unsigned)nwg), dim3(NT), LDS_BYTES_R + 80, st, (const float *)hist,
                           (const float *)x, n, (float *)y, (const float *)d->hpad, d->scale_re, nch, (int)d->hlen);
        LQ_CHECK_LAUNCH();
        return;
    }
    const bool cc = d->kind == 2;
    const bool kb2 = d->nchunk == 2;   // crcf, 65..128 taps
    const int kb = (int)d->nchunk;     // crcf: 129..192 / 193..256 taps with the A fragments in LDS
    const long long nch = (n + CH - 1) / CH;
    const long long wgs = (cc || kb2) ? 512 : FMX_WGS;   // resident workgroups (two / three per CU)
    const dim3 grid((unsigned)(nch < wgs ? nch : wgs));
    constexpr int lds_kb2 = lds_bytes_mx<false, 2>() + 80;
    if (!cc && kb > 2) {
        const dim3 g2((unsigned)(nch < 512 ? nch : 512));
        if (kb == 3)
            hipLaunchKernelGGL((k_firfilt_mx<false, 3>), g2, dim3(NT), (lds_bytes_mx<false, 3>() + 80), st,
                               (const v2f *)hist, (const v2f *)x, n, (v2f *)y, (const float *)d->hpad, d->scale_re,
                               d->scale_im, nch, (int)d->hlen);
        else
            hipLaunchKernelGGL((k_firfilt_mx<false, 4>), g2, dim3(NT), (lds_bytes_mx<false, 4>() + 80), st,
                               (const v2f *)hist, (const v2f *)x, n, (v2f *)y, (const float *)d->hpad, d->scale_re,
                               d->scale_im, nch, (int)d->hlen);
    } else if (kb2)
        hipLaunchKernelGGL((k_firfilt_mx<false, 2>), grid, dim3(NT), lds_kb2, st,
                           (const v2f *)hist, (const v2f *)x, n, (v2f *)y, (const float *)d->hpad, d->scale_re,
                           d->scale_im, nch, (int)d->hlen);
    else if (cc)
        hipLaunchKernelGGL((k_firfilt_mx<true, 1>), grid, dim3(NT), lds_bytes_mx<true>() + 80, st, (const v2f *)hist,
                           (const v2f *)x, n, (v2f *)y, (const float *)d->hpad, d->scale_re, d->scale_im, nch,
                           (int)d->hlen);
    else
        hipLaunchKernelGGL((k_firfilt_mx<false, 1>), grid, dim3(NT), lds_bytes_mx<false>() + 80, st, (const v2f *)hist,
                           (const v2f *)x, n, (v2f *)y, (const float *)d->hpad, d->scale_re, d->scale_im, nch,
                           (int)d->hlen);
    LQ_CHECK_LAUNCH();
}

// Returns 1 if the call was handled on the matrix cores: rrrf, crcf or cccf,
// 33..64 taps (HP = 64, one chunk), taps in the split's safe range, not in
// place, 16-byte aligned x and y.
extern "C" int lqk_firfilt_mx(const lqk_fir_desc *d, const void *hist, const void *x, unsigned long long n,
                              void *y, void *stream)
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
        launch_mx(d, o == 0 ? hist : (const void *)(xo - (size_t)64 * d->nchunk * es), xo, nn, (char *)y + o * es,
                  (hipStream_t)stream);
    }
    return 1;
}
