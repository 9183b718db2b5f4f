// k_resamp.hip -- arbitrary-rate polyphase resampler (resamp_crcf) and the
// per-sample firpfb_crcf output.
//
// Reference: src/filter/src/resamp.c:245-363 (execute, update_timing_state),
// src/filter/src/firpfb.c:325-345 (bank output).  For input t the reference
// emits, while b < npfb, outputs
//     y = (1-mu) * y0 + mu * y1,   y_b(t) = sum_n h[b + n*npfb] x[t-n]  (n < L = 2m)
// with (y0, y1) = (y_b(t), y_{b+1}(t)) in the INTERP state and
// (y_{npfb-1}(t-1), y_0(t)) in the BOUNDARY state, then advances the float32
// timing phase tau += 1/r, b = floor(tau*npfb), mu = tau*npfb - b.
//
// Parallel form.  The timing state at the start of every input is a pure
// function of the previous one (it does not depend on the data), so the host
// tabulates it once per rate (`plan`, see host/resamp.c): checkpoint c holds
// the state before input LQK_RS_CK c (LQK_RS_CK = 4) and K = outputs emitted
// by the inputs before it -- (tau, K), 8 B, for power-of-two bank counts with
// del >= 1/npfb (the rest of the state follows from tau), else
// (tau, mu, b, state, K), 16 B; the sequence is eventually periodic
// (pre-period `pre`, period `P` inputs, `Q` outputs per period; r = 1.037:
// 253 K checkpoints, 2 MB, read from L2 at 2 B / input).  Lanes read
// the checkpoint at or before their first input, step
// the reference's float32 recurrence forward to it and replay their own
// inputs, bit-exactly (contraction off).  Complex streams at 1 < r < 2 with a
// power-of-two bank count run k_resamp4 (csrc/k_resamp4.hip, an output plan
// instead); every other shape comes here: k_resamp3 turns the replay into a
// dense per-wave-tile output list and evaluates it with coalesced stores;
// k_resamp / k_resamp_generic cover shapes whose tables do not fit LDS and
// rates whose outputs overflow a wave tile (r > ~52).
#include <hip/hip_runtime.h>

#include "lq_device.h"
#include "lq_kernels.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace {

constexpr int NT = 256;
constexpr int RS_R = 8;

struct rs_state {
    float tau, mu;
    int b, st; // st: 1 INTERP, 0 BOUNDARY
};

// sample-type helpers: real (rrrf) or complex (crcf, cccf) samples, real taps
// (resamp.c:117-132 designs real taps for every type)
__device__ __forceinline__ float2 rs_axpy(float a, float2 x, float2 y)
{
    return make_float2(fmaf(a, x.x, y.x), fmaf(a, x.y, y.y));
}
__device__ __forceinline__ float rs_axpy(float a, float x, float y) { return fmaf(a, x, y); }
__device__ __forceinline__ float2 rs_mix(float c0, float2 a, float mu, float2 b)
{
    return make_float2(c0 * a.x + mu * b.x, c0 * a.y + mu * b.y);
}
__device__ __forceinline__ float rs_mix(float c0, float a, float mu, float b) { return c0 * a + mu * b; }

// the reference's update_timing_state (resamp.c:352-363), IEEE float32, no FMA
__device__ __forceinline__ void rs_advance(rs_state &s, float del, float fnpfb)
{
#pragma clang fp contract(off)
    s.tau = s.tau + del;
    const float bf = s.tau * fnpfb;
    const float fb = __builtin_floorf(bf);
    s.b = (int)fb;
    s.mu = bf - fb;
}

// one input of the timing recurrence (resamp.c:253-307) without the data
// path; returns the number of outputs it emits
__device__ __forceinline__ unsigned rs_step(rs_state &s, float del, float fnpfb, int npfb)
{
    unsigned n = 0;
    while ((unsigned)s.b < (unsigned)npfb) {   // unsigned, as resamp.c:254 (int b vs unsigned npfb)
        if (s.st && s.b == npfb - 1) {
            s.st = 0;
            s.b = npfb;
            break;
        }
        n++;
        rs_advance(s, del, fnpfb);
        s.st = 1;
    }
    s.tau -= 1.0f;
    s.b = (int)((unsigned)s.b - (unsigned)npfb);
    return n;
}

__device__ __forceinline__ void rs_entry(const lqk_rs_entry &e, rs_state &s)
{
    s.tau = e.tau;
    s.mu = e.mu;
    s.b = e.bst >> 1;
    s.st = e.bst & 1;
}

// the state a power-of-two bank count derives from tau (host/resamp.c
// rs_from_tau): BOUNDARY iff tau < 0, b = floor(tau npfb), mu its fraction
__device__ __forceinline__ void rs_derive(float tau, float fnpfb, rs_state &s)
{
#pragma clang fp contract(off)
    const float bf = tau * fnpfb;
    const float fb = __builtin_floorf(bf);
    s.tau = tau;
    s.mu = bf - fb;
    s.st = tau >= 0.0f ? 1 : 0;
    s.b = s.st ? (int)fb : 0;
}

// the checkpoint (its fields in e) stepped `skip` inputs forward; K counts
// the outputs of those inputs.  Power-of-two banks step tau alone: add del
// until tau reaches 1 - 1/npfb, subtract 1 (host/resamp.c rs_step_p2)
__device__ __forceinline__ void rs_skip(const lqk_rs_entry &e, int p2, int skip, float del, float fnpfb, int npfb,
                                        rs_state &s, unsigned long long &K)
{
    if (p2) {
#pragma clang fp contract(off)
        const float z = 1.0f - 1.0f / fnpfb;
        float x = e.tau;
        unsigned k = 0;
        for (int i = 0; i < skip; i++) {
            while (x < z) {
                x = x + del;
                k++;
            }
            x = x - 1.0f;
        }
        K += k;
        rs_derive(x, fnpfb, s);
    } else {
        rs_entry(e, s);
        for (int i = 0; i < skip; i++) K += rs_step(s, del, fnpfb, npfb);
    }
}

__device__ __forceinline__ lqk_rs_entry rs_load(const lqk_rs_plan &pl, unsigned ck)
{
    if (pl.p2) {
        const lqk_rs_entry_p2 e = static_cast<const lqk_rs_entry_p2 *>(pl.tab)[ck];
        return lqk_rs_entry{e.tau, 0.0f, 0, e.K};
    }
    return static_cast<const lqk_rs_entry *>(pl.tab)[ck];
}

// plan position g -> (state before input g, outputs before it)
__device__ __forceinline__ void rs_lookup(const lqk_rs_plan &pl, unsigned long long g, float del, float fnpfb,
                                          int npfb, rs_state &s, unsigned long long &K)
{
    unsigned long long j = g < pl.end ? g : pl.end, add = 0;
    if (j >= pl.pre) {
        const unsigned long long t = j - pl.pre;
        const unsigned long long c = t / pl.P;
        j = pl.pre + (t - c * pl.P);
        add = c * pl.Q;
    }
    const lqk_rs_entry e = rs_load(pl, (unsigned)(j / LQK_RS_CK));
    K = (unsigned long long)e.K + add;
    rs_skip(e, pl.p2, (int)(j & (LQK_RS_CK - 1)), del, fnpfb, npfb, s, K);
}

// taps[b*L + n] = (h[b + n*npfb], h[(b+1)%npfb + n*npfb]) -- the (y0, y1) pair
template <int L, typename S>
__global__ __launch_bounds__(NT) void k_resamp(lqk_rs_plan pl, unsigned long long g0, unsigned long long K0,
                                               int npfb, float del, const float2 *__restrict__ taps,
                                               const S *__restrict__ hist, const S *__restrict__ x,
                                               long long n, S *__restrict__ y)
{
    extern __shared__ float2 stp[];
    for (int t = threadIdx.x; t < npfb * L; t += NT) stp[t] = taps[t];
    __syncthreads();

    const long long i0 = ((long long)blockIdx.x * NT + threadIdx.x) * RS_R;
    if (i0 >= n) return;
    const float fnpfb = (float)npfb;
    rs_state s;
    unsigned long long K;
    rs_lookup(pl, g0 + (unsigned long long)i0, del, fnpfb, npfb, s, K);
    S *yo = y + (K - K0);

    // w[k] = x[i0 - L + k]; samples before the call come from the history
    S w[L + RS_R];
#pragma unroll
    for (int k = 0; k < L + RS_R; ++k) {
        const long long idx = i0 - L + k;
        S v{};
        if (idx < 0) v = hist[L + idx];
        else if (idx < n) v = x[idx];
        w[k] = v;
    }
#pragma unroll
    for (int r = 0; r < RS_R; ++r) {
        if (i0 + r >= n) break;
        while ((unsigned)s.b < (unsigned)npfb) {
            if (s.st && s.b == npfb - 1) { // last filter: finish with the next input
                s.st = 0;
                s.b = npfb;
                break;
            }
            const bool bnd = !s.st;
            const float2 *tp = stp + (bnd ? npfb - 1 : s.b) * L;
            S a0{}, a1{};
#pragma unroll
            for (int k = 0; k < L; ++k) {
                const float2 t = tp[k];
                const S xb = w[L + r - k];
                const S xa = bnd ? w[L + r - 1 - k] : xb;
                a0 = rs_axpy(t.x, xa, a0);
                a1 = rs_axpy(t.y, xb, a1);
            }
            *yo++ = rs_mix(1.0f - s.mu, a0, s.mu, a1);
            rs_advance(s, del, fnpfb);
            s.st = 1;
        }
        s.tau -= 1.0f;
        s.b = (int)((unsigned)s.b - (unsigned)npfb);
    }
}

// plan position g = gt + d for a tile base gt (position jt, cycles ct already
// resolved once per tile) and a small lane offset d, in 32-bit arithmetic:
// the checkpoint to read, the periods before it and the inputs to step
struct rs_ref {
    unsigned ck;
    int skip;
    unsigned long long cyc;
};
__device__ __forceinline__ rs_ref rs_locate_near(const lqk_rs_plan &pl, unsigned long long gt, unsigned long long jt,
                                                 unsigned long long ct, unsigned d)
{
    unsigned long long j = gt + d, c = 0;
    if (gt + d > pl.end) {                     // direct plans: clamp (pre = end + 1)
        j = pl.end;
    } else if (gt >= pl.pre) {
        const unsigned off = (unsigned)(jt - pl.pre) + d;
        const unsigned w = off / (unsigned)pl.P;
        j = pl.pre + (off - w * (unsigned)pl.P);
        c = ct + w;
    } else if (gt + d >= pl.pre) {
        const unsigned t = (unsigned)(gt + d - pl.pre);
        const unsigned w = t / (unsigned)pl.P;
        j = pl.pre + (t - w * (unsigned)pl.P);
        c = w;
    }
    return rs_ref{(unsigned)(j / LQK_RS_CK), (int)(j & (LQK_RS_CK - 1)), c};
}

// output stores non-temporal (A/B in round 4 on one box: 0.197 vs 0.206 ms)
constexpr int RS_STAUX = 2;
// pair-table row stride (8-byte slots per half row): RSC, or npfb/2 + 1 at run time
template <int RSC>
__host__ __device__ inline int rs2_rs(int npfb) { return RSC ? RSC : (npfb >> 1) + 1; }
// one LDS read of T as a relaxed workgroup-scope atomic: the compiler issues
// it as its own ds_read_b64 / _b32 (2 LDS cycles per wave) and never pairs two
// into a ds_read2_b64 (8 cycles, CDNA4 LDS table), and still batches them
template <typename T>
__device__ __forceinline__ T lds_rd(const T *p)
{
    if constexpr (sizeof(T) == 8) {
        const unsigned long long u = __hip_atomic_load(reinterpret_cast<unsigned long long *>(const_cast<T *>(p)),
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return __builtin_bit_cast(T, u);
    } else {
        const unsigned u = __hip_atomic_load(reinterpret_cast<unsigned *>(const_cast<T *>(p)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        return __builtin_bit_cast(T, u);
    }
}

// acc + c w for a real coefficient and a complex (packed FMA) or real sample
__device__ __forceinline__ float2 rs_fma(float c, float2 w, float2 acc)
{
    v2f a2 = {acc.x, acc.y};
    a2 = v2f{c, c} * v2f{w.x, w.y} + a2;
    return make_float2(a2.x, a2.y);
}
__device__ __forceinline__ float rs_fma(float c, float w, float acc) { return fmaf(c, w, acc); }

// stores through the output descriptor (an offset past it is dropped)
__device__ __forceinline__ void rs_store1(__amdgpu_buffer_rsrc_t r, unsigned off, float2 v)
{
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, RS_STAUX);
}
__device__ __forceinline__ void rs_store1(__amdgpu_buffer_rsrc_t r, unsigned off, float v)
{
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, RS_STAUX);
}

// any L (window and taps read through the caches), one input per lane
template <typename S>
__global__ __launch_bounds__(NT) void k_resamp_generic(lqk_rs_plan pl, unsigned long long g0,
                                                       unsigned long long K0, int npfb, int L, float del,
                                                       const float2 *__restrict__ taps,
                                                       const S *__restrict__ hist,
                                                       const S *__restrict__ x, long long n,
                                                       S *__restrict__ y)
{
    const long long i = (long long)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const float fnpfb = (float)npfb;
    rs_state s;
    unsigned long long K;
    rs_lookup(pl, g0 + (unsigned long long)i, del, fnpfb, npfb, s, K);
    S *yo = y + (K - K0);
    auto X = [&](long long idx) -> S { return idx < 0 ? hist[L + idx] : x[idx]; };
    while ((unsigned)s.b < (unsigned)npfb) {
        if (s.st && s.b == npfb - 1) break;
        const bool bnd = !s.st;
        const float2 *tp = taps + (size_t)(bnd ? npfb - 1 : s.b) * L;
        S a0{}, a1{};
        for (int k = 0; k < L; ++k) {
            const float2 t = tp[k];
            const S xb = X(i - k);
            const S xa = bnd ? X(i - 1 - k) : xb;
            a0 = rs_axpy(t.x, xa, a0);
            a1 = rs_axpy(t.y, xb, a1);
        }
        *yo++ = rs_mix(1.0f - s.mu, a0, s.mu, a1);
        rs_advance(s, del, fnpfb);
        s.st = 1;
    }
}

// ------------------------------------------------------------ wave tiles
// k_resamp3 (the default): every wave owns its tiles end to end, with no
// workgroup barrier after the pair table is built.  A wave tile is up to
// 256 inputs (fewer at high rates, so its outputs fit W3_CAP slots):
//  1. the input window [i0-L-1, i0+tin+1) goes to the wave's LDS from
//     registers loaded two tiles earlier (two register sets alternate);
//  2. lane j replays the float32 timing of inputs 4j .. 4j+3 from the plan
//     checkpoint at or before the first (LQK_RS_CK = 4: at most 3 steps
//     before it, the call's alignment) and writes one descriptor per output
//     (mu, input, bank) at the output's index in the tile; the tile's first
//     output count is lane 0's (a readlane, no LDS round trip);
//  3. lanes take consecutive outputs: y = sum_p c[p] x[i-L+p], p <= L, with
//     c[p] = T.x + mu T.d from the pair table (T.x, T.d = T.y - T.x; bank b:
//     h_b, h_b+1 on the same window; bank npfb: the BOUNDARY pair h_{npfb-1}
//     on the window one input older and h_0), so both timing states are one
//     dot product; 8-byte LDS reads (the pair table pair-major, T2[p][b] at
//     8 ((2p + (b & 1)) RS + b/2), consecutive outputs stepping the bank by
//     ~npfb/r, so the rows a 32-lane group reads sit on distinct slots), as
//     relaxed workgroup atomics so the compiler never pairs them into
//     ds_read2_b64; non-temporal 8-byte stores through a descriptor over the
//     launch's outputs.
// Waves drift apart freely instead of meeting at two workgroup barriers per
// 1024-input tile, as the round-3 form (k_resamp2: wave 0 replayed 16-input
// spans for all four waves) did: 0.197 -> 0.184 ms per 2^25 inputs at
// r = 1.037 on one box.
constexpr int RS3_BLK = 5;       // resident workgroups per CU (four and six measured slower, round 4)
constexpr int NT3 = 256;         // threads per k_resamp3 workgroup (waves own their tiles)
constexpr int W3_TIN = 64 * 4;   // inputs per wave tile (64 lanes x 4)
constexpr int W3_CAP = 320;      // output slots per wave tile
constexpr int RS3_FIT = 15;      // a tile's fixed cost in evaluation passes x 10 (tile fitting, launch_rs)
// table rows (float2 units) of k_resamp3
template <int L>
constexpr int rs3_rows() { return L + 1; }
template <int L, typename S, int RSC>
inline size_t rs3_lds_bytes(int npfb)
{
    constexpr int TS = W3_TIN + L + 2;
    return (size_t)2 * rs3_rows<L>() * rs2_rs<RSC>(npfb) * sizeof(float2) +
           (size_t)(NT3 / 64) * (((TS + 2) * sizeof(S) + 15) / 16 * 16 + (W3_CAP + 2) * 8);
}

template <int L, typename S, int RSC>
__global__ __launch_bounds__(NT3, RS3_BLK) void k_resamp3(lqk_rs_plan pl, unsigned long long g0, unsigned long long K0,
                                                       int npfb, float del, const float2 *__restrict__ taps2,
                                                       const S *__restrict__ hist, const S *__restrict__ x,
                                                       long long n, S *__restrict__ y, int nout, int tin)
{
    static_assert(LQK_RS_CK == 4, "k_resamp3 replays 4 inputs per lane from their own checkpoint");
    constexpr int SPAN = 4;
    constexpr int LP = (L + 2 + 1) & ~1;          // pair stride of taps2 (host layout)
    constexpr int TS = W3_TIN + L + 2;            // window samples of a tile
    constexpr int WB = ((TS + 2) * (int)sizeof(S) + 15) / 16 * 16 + (W3_CAP + 2) * 8;   // bytes per wave
    constexpr int NXV = (TS + 63) / 64;           // window samples per lane
    constexpr int NSLOT = W3_CAP / 64;            // output slots per lane
    constexpr int NROW = rs3_rows<L>();
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int RS = rs2_rs<RSC>(npfb);
    float2 *tpl = reinterpret_cast<float2 *>(smem);
    // the wave index through readfirstlane: the compiler then knows every
    // tile-level quantity (tile, i0, the plan position and its 64-bit period
    // division) is wave-uniform and computes it on the scalar unit
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned char *wbase = smem + (size_t)2 * NROW * RS * sizeof(float2) + (size_t)wave * WB;
    S *cw = reinterpret_cast<S *>(wbase);
    uint2 *dsc = reinterpret_cast<uint2 *>(wbase + ((TS + 2) * (int)sizeof(S) + 15) / 16 * 16);   // dsc[W3_CAP]: sink
    const float fnpfb = (float)npfb;
    for (int t = tid; t < (npfb + 1) * NROW; t += NT3) {
        const int b = t / NROW, p = t % NROW;
        const float2 v = taps2[b * LP + p];
        tpl[(2 * p + (b & 1)) * RS + (b >> 1)] = make_float2(v.x, v.y - v.x);
    }
    __syncthreads();   // the only workgroup barrier

    const long long ntiles = (n + tin - 1) / tin;
    const long long GW = (long long)gridDim.x * (NT3 / 64), gw = (long long)blockIdx.x * (NT3 / 64) + wave;
    if (gw >= ntiles) return;
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)(n * (long long)sizeof(S)), 0x00020000);
    const __amdgpu_buffer_rsrc_t rh =
        __builtin_amdgcn_make_buffer_rsrc((void *)hist, (short)0, (int)(L * sizeof(S)), 0x00020000);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)y, (short)0, nout * (int)sizeof(S), 0x00020000);
    auto ld = [&](__amdgpu_buffer_rsrc_t r, int e) -> S {
        const unsigned off = e < 0 ? 0xFFFFFFF0u : (unsigned)e * (unsigned)sizeof(S);
        if constexpr (sizeof(S) == 8)
            return __builtin_bit_cast(S, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
        else
            return __builtin_bit_cast(S, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
    };
    struct Pre {
        S xa[NXV], xh;
        lqk_rs_entry e;
        unsigned long long cyc;
        int skip;
    };
    auto fetch = [&](long long tile, Pre &f) {
        const long long i0 = tile * tin;
#pragma unroll
        for (int u = 0; u < NXV; u++)
            f.xa[u] = ld(rx, (lane + 64 * u < tin + L + 2) ? (int)i0 - L - 1 + lane + 64 * u : -1);
        // window samples before the call come from the history: window sample
        // t is input i0 - L - 1 + t, history index i0 - 1 + t (out of range,
        // 0, from L on) -- for every tile that starts within L + 1 inputs of
        // the call, not only the first (high rates shrink tiles to 4 inputs)
        f.xh = ld(rh, i0 < L + 1 ? (int)i0 - 1 + lane : -1);
        const unsigned long long gt = g0 + (unsigned long long)i0;
        unsigned long long jt = gt, ct = 0;
        if (gt >= pl.pre && gt <= pl.end) {
            const unsigned long long t = gt - pl.pre;
            ct = t / pl.P;
            jt = pl.pre + (t - ct * pl.P);
        }
        const int d = lane * SPAN < tin ? lane * SPAN : 0;
        const rs_ref r = rs_locate_near(pl, gt, jt, ct, (unsigned)d);
        f.e = rs_load(pl, r.ck);
        f.cyc = r.cyc;
        f.skip = r.skip;
    };
    auto wave_fence = []() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // one tile of loads in flight per wave (a second set measured slower:
    // 82 VGPRs; the CU's other waves hide the latency)
    Pre pa;
    fetch(gw, pa);
    for (long long tile = gw; tile < ntiles; tile += GW) {
        const long long i0 = tile * tin;
        const long long ie = (i0 + tin < n) ? i0 + tin : n;
        const lqk_rs_entry e = pa.e;
        const unsigned long long cyc = pa.cyc;
        const int skip = pa.skip;
        wave_fence();   // the previous tile's evaluation has read the window
#pragma unroll
        for (int u = 0; u < NXV; u++) {
            const int t = lane + 64 * u;
            if (t < TS) cw[t] = u == 0 ? pa.xa[0] + pa.xh : pa.xa[u];
        }
        fetch(tile + GW, pa);
        // replay: lane j, inputs ia .. ia + nin - 1
        const long long ia = i0 + (long long)lane * SPAN;
        const int nin = ia < ie ? (int)((ie - ia) < SPAN ? (ie - ia) : SPAN) : 0;
        unsigned long long k = (unsigned long long)e.K + cyc * pl.Q;
        float xx = e.tau;
        rs_state st;
        const float z = 1.0f - 1.0f / fnpfb;
        if (pl.p2) {
#pragma clang fp contract(off)
            for (int i = 0; i < skip; i++) {
                while (xx < z) {
                    xx = xx + del;
                    k++;
                }
                xx = xx - 1.0f;
            }
        } else {
            rs_entry(e, st);
            for (int i = 0; i < skip; i++) k += rs_step(st, del, fnpfb, npfb);
        }
        const unsigned long long Kb = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(k >> 32), 0) << 32) |
                                      (unsigned)__builtin_amdgcn_readlane((int)k, 0);
        const unsigned long long o64 = k - Kb;
        const int o0 = o64 < (1ull << 30) ? (int)o64 : (1 << 30);
        int o = o0;
        auto put = [&](int iloc, int bank, float mu) {
            dsc[(unsigned)o < (unsigned)W3_CAP ? o : W3_CAP] =
                make_uint2(__float_as_uint(mu), (unsigned)iloc | ((unsigned)bank << 12));
            o++;
        };
        if (pl.p2) {
#pragma clang fp contract(off)
            for (int r = 0; r < nin; r++) {
                const int iloc = (int)(ia + r - i0);
                while (xx < z) {
                    const float bf = xx * fnpfb;
                    const float fb = __builtin_floorf(bf);
                    put(iloc, xx < 0.0f ? npfb : (int)fb, bf - fb);
                    xx = xx + del;
                }
                xx = xx - 1.0f;
            }
        } else {
            for (int r = 0; r < nin; r++) {
                const int iloc = (int)(ia + r - i0);
                while ((unsigned)st.b < (unsigned)npfb) {   // unsigned, as resamp.c:254
                    if (st.st && st.b == npfb - 1) {
                        st.st = 0;
                        st.b = npfb;
                        break;
                    }
                    put(iloc, st.st ? st.b : npfb, st.mu);
                    rs_advance(st, del, fnpfb);
                    st.st = 1;
                }
                st.tau -= 1.0f;
                st.b = (int)((unsigned)st.b - (unsigned)npfb);
            }
        }
        // outputs of the tile: those before the last replaying lane's end
        // (at most W3_CAP by the host's tile sizing, launch_rs; clamped so a
        // violated bound can never read past the output list)
        const int last = (int)((ie - i0 - 1) / SPAN);
        int nr = __builtin_amdgcn_readlane(o, last);
        nr = nr < W3_CAP ? nr : W3_CAP;
        const unsigned ob = (unsigned)(Kb - K0);
        wave_fence();   // the output list is written
        auto dot = [&](const S *wv, int bb, float mu) -> S {
            S acc{};
            const float2 *tp = tpl + (bb & 1) * RS + (bb >> 1);
#pragma unroll
            for (int p = 0; p <= L; p++) {
                const float2 t = lds_rd(tp + 2 * p * RS);
                const float c = fmaf(mu, t.y, t.x);
                const S w = lds_rd(wv + p);
                acc = rs_fma(c, w, acc);
            }
            return acc;
        };
#pragma unroll
        for (int q = 0; q < NSLOT; q++) {
            const int oo = lane + 64 * q;
            S v{};
            if (oo < nr) {
                const uint2 dd = dsc[oo];
                v = dot(cw + (int)(dd.y & 4095u) + 1, (int)(dd.y >> 12), __uint_as_float(dd.x));
            }
            rs_store1(ry, oo < nr ? (ob + (unsigned)oo) * (unsigned)sizeof(S) : 0xFFFFFFF0u, v);
        }
    }
}

template <int L, typename S>
void launch_rs(const lqk_rs_plan &pl, unsigned long long g0, unsigned long long K0, int npfb, float del,
               const float2 *taps, const float2 *taps2, const S *hist, const S *x, long long n, S *y,
               unsigned long long nout, hipStream_t st)
{
    constexpr int RSC = 33;                    // constant pair-table stride for npfb <= 64 (immediate tap offsets)
    const bool cst = npfb <= 2 * (RSC - 1);
    const size_t lds3 = cst ? rs3_lds_bytes<L, S, RSC>(npfb) : rs3_lds_bytes<L, S, 0>(npfb);
    if (taps2 != nullptr && lds3 <= 80 * 1024 && pl.P < (1ull << 31) && (pl.pre < (1ull << 62) || pl.end < (1ull << 62))) {
        // inputs per wave tile (a multiple of 4): its outputs, at most
        // (tin + 2) r + 2 (tau moves by 1/r per output and by -1 per input
        // within [-1/npfb, 1 + 1/r)), fit the W3_CAP output slots
        const double r = 1.0 / (double)del;
        int tin = W3_TIN;
        while (tin > 4 && std::ceil((tin + 2) * r) + 2 > W3_CAP) tin -= 4;
        // then the tile size with the fewest evaluation passes (64 outputs
        // each, a pass runs only where a lane has an output) per input,
        // counting the tile's fixed cost (window store, replay) as RS3_FIT / 10
        // passes: at r = 1.037 a 256-input tile's 265 outputs take five
        // passes, the fifth for 9 lanes; 244 inputs (253 outputs) take four
        if (std::ceil((tin + 2) * r) + 2 <= W3_CAP) {
            double best = 1e300;
            int bt = tin;
            for (int t = tin; t >= 4 && t * 4 >= tin * 3; t -= 4) {
                const double c = (std::ceil((std::ceil((t + 2) * r) + 2) / 64.0) + RS3_FIT / 10.0) / t;
                if (c < best * (1.0 - 1e-9)) {
                    best = c;
                    bt = t;
                }
            }
            tin = bt;
        }
        if (std::ceil((tin + 2) * r) + 2 <= W3_CAP) {   // else (r > ~52): the per-input kernel below
            const long long ntiles = (n + tin - 1) / tin;
            const long long wgs = (ntiles + NT3 / 64 - 1) / (NT3 / 64);
            const int blk = lds3 <= 160 * 1024 / RS3_BLK ? RS3_BLK : (int)(160 * 1024 / lds3);
            const unsigned nb = (unsigned)(wgs < 256 * blk ? wgs : 256 * blk);   // persistent: blk per CU
            if (cst)
                hipLaunchKernelGGL((k_resamp3<L, S, RSC>), dim3(nb), dim3(NT3), lds3, st, pl, g0, K0, npfb, del,
                                   taps2, hist, x, n, y, (int)nout, tin);
            else
                hipLaunchKernelGGL((k_resamp3<L, S, 0>), dim3(nb), dim3(NT3), lds3, st, pl, g0, K0, npfb, del,
                                   taps2, hist, x, n, y, (int)nout, tin);
            return;
        }
    }
    const long long lanes = (n + RS_R - 1) / RS_R;
    const unsigned nb = (unsigned)((lanes + NT - 1) / NT);
    hipLaunchKernelGGL((k_resamp<L, S>), dim3(nb), dim3(NT), (size_t)npfb * L * sizeof(float2), st, pl, g0, K0,
                       npfb, del, taps, hist, x, n, y);
}

template <typename S>
void run_rs(const lqk_rs_plan *pl, unsigned long long g0, unsigned long long K0, unsigned int npfb, unsigned int L,
            float del, const void *taps, const void *taps2, const void *hist, const void *x, unsigned long long n,
            void *y, unsigned long long nout, hipStream_t st)
{
    const float2 *tp = (const float2 *)taps;
    const S *hs = (const S *)hist, *xi = (const S *)x;
    S *yo = (S *)y;
    const long long nn = (long long)n;
    const bool lds_ok = (size_t)npfb * L * sizeof(float2) <= 64 * 1024;
#define LQ_RS_CASE(LL)                                                                                     \
    case LL:                                                                                               \
        launch_rs<LL, S>(*pl, g0, K0, (int)npfb, del, tp, (const float2 *)taps2, hs, xi, nn, yo, nout, st); \
        return;
    if (lds_ok && L <= 32 && (L % 2) == 0) {
        switch (L) {
            LQ_RS_CASE(2)
            LQ_RS_CASE(4)
            LQ_RS_CASE(6)
            LQ_RS_CASE(8)
            LQ_RS_CASE(10)
            LQ_RS_CASE(12)
            LQ_RS_CASE(14)
            LQ_RS_CASE(16)
            LQ_RS_CASE(18)
            LQ_RS_CASE(20)
            LQ_RS_CASE(22)
            LQ_RS_CASE(24)
            LQ_RS_CASE(26)
            LQ_RS_CASE(28)
            LQ_RS_CASE(30)
            LQ_RS_CASE(32)
        }
    }
#undef LQ_RS_CASE
    const unsigned nb = (unsigned)((n + NT - 1) / NT);
    hipLaunchKernelGGL((k_resamp_generic<S>), dim3(nb), dim3(NT), 0, st, *pl, g0, K0, (int)npfb, (int)L, del, tp,
                       hs, xi, nn, yo);
}

} // namespace

extern "C" void lqk_resamp(int real_io, const lqk_rs_plan *pl, unsigned long long g0, unsigned long long K0,
                           unsigned int npfb, unsigned int L, float del, const void *taps, const void *taps2,
                           const void *hist, const void *x, unsigned long long n, void *y, unsigned long long nout,
                           void *stream)
{
    if (n == 0) return;
    const size_t es = real_io ? 4 : 8;
    if (n > LQK_RS_MAXN || nout * es >= (1ull << 31)) {
        fprintf(stderr, "error: liquid-mi355x: resamp launch of %llu inputs / %llu outputs exceeds one launch\n", n, nout);
        exit(1);
    }
    hipStream_t st = (hipStream_t)stream;
    if (real_io) run_rs<float>(pl, g0, K0, npfb, L, del, taps, taps2, hist, x, n, y, nout, st);
    else run_rs<float2>(pl, g0, K0, npfb, L, del, taps, taps2, hist, x, n, y, nout, st);
    LQ_CHECK_LAUNCH();
}
