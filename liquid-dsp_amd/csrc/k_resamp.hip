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
// the state before input LQK_RS_CK c (LQK_RS_CK = 16) and K = outputs emitted
// by the inputs before it -- (tau, K), 8 B, for power-of-two bank counts with
// del >= 1/npfb (the rest of the state follows from tau), else
// (tau, mu, b, state, K), 16 B; the sequence is eventually periodic
// (pre-period `pre`, period `P` inputs, `Q` outputs per period).  Lanes read
// the checkpoint at or before their first input (0.5 B / input of plan
// traffic for 8-byte checkpoints), step
// the reference's float32 recurrence forward to it and replay their own
// inputs, bit-exactly (contraction off).  k_resamp2 (the default) turns the replay into a
// dense per-tile output list and evaluates it with coalesced stores;
// k_resamp / k_resamp_generic cover shapes whose tables do not fit LDS.
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

// Tiled form (L even, table in LDS).  A persistent workgroup (five per CU)
// walks tiles of TIN consecutive inputs:
//  1. the input window [i0-L-1, i0+TIN) goes to LDS from registers that were
//     loaded two tiles earlier (two register sets alternate, so two tiles of
//     loads are in flight while one is evaluated: 0.226 -> 0.218 ms);
//  2. each lane replays the float32 timing of its RIN inputs and writes one
//     descriptor per output (mu, input, bank) at the output's index in the
//     tile -- the output list is now dense (writes are branch-free: outputs
//     outside the round go to a sink slot);
//  3. lanes take consecutive outputs: y = sum_p c[p] x[i-L+p], p <= L, with
//     c[p] = T.x + mu T.d from the table (T.x, T.d = T.y - T.x) of pairs T2
//     (bank b: h_b, h_b+1 on the same window; bank npfb: the BOUNDARY pair
//     h_{npfb-1} on the window one input older and h_0), so both states are
//     one dot product, and the stores (32-bit offsets through a buffer
//     descriptor over the round's outputs) are coalesced.  Outputs beyond CAP
//     per tile take more rounds of 2-3.
// LDS reads of step 3 are 8-byte (one tap pair, one sample).  A ds_read_b64
// is serviced in two 32-lane groups over all 64 banks: 32 consecutive
// outputs read a window span of ~32 samples (256 B, conflict-free), and the
// pair table is laid out pair-major, T2[p][b] at 8 ((2p + (b & 1)) RS + b/2):
// consecutive outputs step the bank by ~npfb/r, never by 1, so the 32 rows a
// group reads sit on 32 distinct 8-byte slots.  (The earlier 16-byte reads of
// whole tap rows and of a doubled, shifted window copy were 2-way conflicted
// in every 16-lane group: half the LDS cycles of the kernel.)
// Measured and dropped: a run of consecutive outputs per lane with the window
// in registers (one LDS read per input instead of L+1 per output) -- the run
// is a dependent chain and the reads conflict 4-way: 0.226 -> 0.265 ms;
// 2048-input tiles (0.247 ms); six workgroups per CU (spills: 0.52 ms).
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

#ifndef RS_RIN
#define RS_RIN 4
#endif
#ifndef RS_EXP
#define RS_EXP 0   // timing experiments (wrong outputs): 1 no checkpoint skip, 2 no evaluation, 4 no descriptor writes
#endif
// workgroups per CU: six for L <= 16 (25.5 KB LDS, <= 80 VGPRs each: L = 14
// 0.236 -> 0.221 ms against five); longer filters spill at 80 VGPRs
#ifndef RS_BLK
#define RS_BLK 5
#endif
template <int L>
constexpr int rs2_blk() { return L <= 16 ? RS_BLK : 5; }
#ifndef RS_O32
#define RS_O32 1   // power-of-two replay: 32-bit output slot counter (A/B on one box: 0.213 vs 0.216 ms per 2^25 inputs)
#endif
#ifndef RS_CAPX
#define RS_CAPX 64    // output slots per tile beyond TIN (r = 1.037: <= 1066 outputs per 1024 inputs)
#endif
template <int L>
constexpr int rs2_tin() { return NT * RS_RIN; }
constexpr int rs2_cap() { return NT * RS_RIN + RS_CAPX; }
#ifndef RS_ALD
#define RS_ALD 1   // evaluation reads as single ds_read_b64 (relaxed workgroup atomics: never paired into ds_read2_b64)
#endif
#ifndef RS_RSC
#define RS_RSC 1   // pair-table row stride a compile-time constant (npfb <= 64: 33) -> immediate tap offsets
#endif
#ifndef RS_STAUX
#define RS_STAUX 2  // cache policy of the output stores: non-temporal (A/B on one box: 0.197 vs 0.206 ms)
#endif
#ifndef RS_LDAUX
#define RS_LDAUX 0  // cache policy of the input loads
#endif
#ifndef RS_RWAVE
#define RS_RWAVE 0  // replay on wave blockIdx mod 4 instead of wave 0
#endif
#ifndef RS_UNR
#define RS_UNR 0   // power-of-two replay: the first RS_UNR outputs of each input unrolled, predicated
#endif
#ifndef RS_PAIR
#define RS_PAIR 0  // two consecutive outputs per lane over one window (rates >= 1)
#endif
#ifndef RS_CH
#define RS_CH 0    // taps per read batch in the evaluation (0: the compiler's choice)
#endif
#ifndef RS_BF
#define RS_BF 0    // slots below TIN evaluated without a branch (idle slots read a harmless descriptor)
#endif
// pair-table row stride (8-byte slots per half row): RSC, or npfb/2 + 1 at run time
template <int RSC>
__host__ __device__ inline int rs2_rs(int npfb) { return RSC ? RSC : (npfb >> 1) + 1; }
// LDS bytes of k_resamp2<L, S, RSC, PR>: window copy, output descriptors, pair
// table (L + 1 tap rows; PR adds a zero row on either side), replay counters
template <int L, typename S, int RSC, bool PR>
inline size_t rs2_lds_bytes(int npfb)
{
    constexpr int TS = rs2_tin<L>() + L + 2;
    constexpr int NROW = L + 1 + (PR ? 2 : 0);
    return (size_t)(TS + 2) * sizeof(S) + (rs2_cap() + 2) * 8 + (size_t)2 * NROW * rs2_rs<RSC>(npfb) * sizeof(float2) +
           (size_t)(rs2_tin<L>() / LQK_RS_CK + 1) * 8;
}

// one LDS read of T as a relaxed workgroup-scope atomic: the compiler issues
// it as its own ds_read_b64 / _b32 (2 LDS cycles per wave) and never pairs two
// into a ds_read2_b64 (8 cycles, CDNA4 LDS table), and still batches them
template <typename T>
__device__ __forceinline__ T lds_rd(const T *p)
{
#if RS_ALD
    if constexpr (sizeof(T) == 8) {
        const unsigned long long u = __hip_atomic_load(reinterpret_cast<unsigned long long *>(const_cast<T *>(p)),
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return __builtin_bit_cast(T, u);
    } else {
        const unsigned u = __hip_atomic_load(reinterpret_cast<unsigned *>(const_cast<T *>(p)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        return __builtin_bit_cast(T, u);
    }
#else
    return *p;
#endif
}

// PR (rates >= 1: consecutive outputs at most one input apart): each lane
// evaluates two consecutive outputs A, B (inputs iA, iB = iA + d, d in {0, 1})
// over one shared window W[p'] = x[iA - L + p'], p' <= L + 1: A's taps are rows
// p' of the pair table, B's rows p' - d, the table padded with a zero row on
// either side, so each window sample is read once for both outputs (16 + 15 +
// 16 LDS reads per pair at L = 14 instead of 2 x 30) and the pair leaves as one
// 16-byte store.  Terms outside an output's window are zero taps times a
// sample; the samples there are replaced by 0, so a non-finite input never
// reaches an output the reference keeps finite.
__device__ __forceinline__ uint4 lds_rd4(const uint4 *p)
{
#if RS_ALD
    // two relaxed 8-byte reads of adjacent words: the compiler may fuse
    // these into one ds_read_b128 (4 cycles, as two ds_read_b64)
    const uint2 a = lds_rd(reinterpret_cast<const uint2 *>(p)), b = lds_rd(reinterpret_cast<const uint2 *>(p) + 1);
    return make_uint4(a.x, a.y, b.x, b.y);
#else
    return *p;
#endif
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
__device__ __forceinline__ void rs_store2(__amdgpu_buffer_rsrc_t r, unsigned off, float2 a, float2 b)
{
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = {__float_as_uint(a.x), __float_as_uint(a.y), __float_as_uint(b.x), __float_as_uint(b.y)};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, RS_STAUX);
}
__device__ __forceinline__ void rs_store2(__amdgpu_buffer_rsrc_t r, unsigned off, float a, float b)
{
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = {__float_as_uint(a), __float_as_uint(b)};
    __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, RS_STAUX);
}

template <int L, typename S, int RSC, bool PR>
__global__ __launch_bounds__(NT, rs2_blk<L>()) void k_resamp2(lqk_rs_plan pl, unsigned long long g0, unsigned long long K0,
                                                int npfb, float del, const float2 *__restrict__ taps2,
                                                const S *__restrict__ hist, const S *__restrict__ x,
                                                long long n, S *__restrict__ y, int nout, int tin)
{
    constexpr int TIN = rs2_tin<L>();
    constexpr int LP = (L + 2 + 1) & ~1;         // pair stride of taps2 (host layout, >= L+1)
    constexpr int TS = TIN + L + 2;              // tile samples
    constexpr int CS = TS + 2;                   // copy size (keeps what follows 16-byte aligned)
    constexpr int CAP = rs2_cap();               // outputs per tile (the host sizes tin to fit)
    constexpr int NSLOT = (CAP + NT - 1) / NT;   // output slots per lane
    constexpr int SPAN = LQK_RS_CK;              // inputs replayed per lane of wave 0
    constexpr int NSPAN = TIN / SPAN;            // = 64: the tile's spans, one per lane of wave 0
    static_assert(NSPAN == 64, "one wave replays a tile");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    S *cp0 = reinterpret_cast<S *>(smem);
    uint2 *desc = reinterpret_cast<uint2 *>(cp0 + CS);
    float2 *tpl = reinterpret_cast<float2 *>(desc + CAP + 2);   // desc[CAP]: sink of out-of-tile outputs
    const int RS = rs2_rs<RSC>(npfb);            // 8-byte slots per half row
    constexpr int ROFF = PR ? 1 : 0;             // tap row p lives at table row p + ROFF
    constexpr int NROW = L + 1 + 2 * ROFF;

    const int tid = threadIdx.x;
    const float fnpfb = (float)npfb;
    // the replaying wave: wave 0, or (RS_RWAVE) wave blockIdx mod 4, so the
    // serial replays of the workgroups resident on a CU do not all land on the
    // SIMD that holds their wave 0; rlane = lane in it, -1 elsewhere
    const int rwave = RS_RWAVE ? (int)(blockIdx.x & 3) : 0;
    const int rlane = (tid >> 6) == rwave ? (tid & 63) : -1;
    for (int t = tid; t < (npfb + 1) * NROW; t += NT) {
        const int b = t / NROW, r = t % NROW, p = r - ROFF;
        const float2 v = (p >= 0 && p <= L) ? taps2[b * LP + p] : make_float2(0.0f, 0.0f);
        // (h_b, h_b+1 - h_b): c = h_b + mu (h_b+1 - h_b) is one fma, the same
        // float32 operations as before (the difference rounded once here)
        tpl[(2 * r + (b & 1)) * RS + (b >> 1)] = make_float2(v.x, v.y - v.x);
    }
    const long long ntiles = (n + tin - 1) / tin;
    constexpr int NXV = (TS + NT - 1) / NT;       // tile samples per lane

    // everything a tile needs from HBM, fetched two tiles ahead into registers.
    // Samples come through two range-checked descriptors (x: n samples, the
    // history: the L before it); each sample is in range in at most one, so
    // their sum is the sample and the loads carry no branch.  Every tile issues
    // the same loads and stores (a store outside the launch's outputs is
    // dropped): with a fixed count of memory operations per tile the compiler
    // waits for exactly the prefetched registers it needs -- a data-dependent
    // store count made it drain everything (vmcnt(0)), the prefetch included,
    // at the start of every tile.  The host keeps n * sizeof(S) below 2^31.
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)(n * (long long)sizeof(S)), 0x00020000);
    const __amdgpu_buffer_rsrc_t rh =
        __builtin_amdgcn_make_buffer_rsrc((void *)hist, (short)0, (int)(L * sizeof(S)), 0x00020000);
    // stores through a descriptor over the launch's nout outputs: 32-bit
    // offsets, and a store outside them is dropped
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)y, (short)0, nout * (int)sizeof(S), 0x00020000);
    // e: sample index (32-bit: the host keeps n * sizeof(S) below 2^31).
    // Negative: an explicit out-of-range offset (reads 0) -- a negative index
    // cast to 32 bits would land within 8 bytes of 2^32, where offset + size wraps
    auto ld = [&](__amdgpu_buffer_rsrc_t r, int e) -> S {
        const unsigned off = e < 0 ? 0xFFFFFFF0u : (unsigned)e * (unsigned)sizeof(S);
        if constexpr (sizeof(S) == 8)
            return __builtin_bit_cast(S, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, RS_LDAUX));
        else
            return __builtin_bit_cast(S, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, RS_LDAUX));
    };
    struct Pre {
        S xa[NXV], xh;                           // tile window; the history part of its first vector
        lqk_rs_entry e;                          // the checkpoint at or before the lane's first input
        unsigned long long cyc;                  // periods before it
        int skip;                                // inputs from it to the lane's first input
    };
    unsigned long long *kx = reinterpret_cast<unsigned long long *>(tpl + 2 * NROW * RS);   // [NSPAN + 1]
    auto fetch = [&](long long tile, Pre &f) {
        const long long i0 = tile * tin;
        // the last vector covers only TS - (NXV-1) NT samples: its other lanes
        // load out of range (no traffic; loading them re-read 240 samples of
        // the next tile per tile, +23 % of the input bytes)
#pragma unroll
        for (int u = 0; u < NXV; u++)
            f.xa[u] = ld(rx, (u < NXV - 1 || tid + u * NT < TS) ? (int)i0 - L - 1 + tid + u * NT : -1);
        f.xh = ld(rh, i0 == 0 ? tid - 1 : -1);   // tile 0's first L samples: the history
        const unsigned long long gt = g0 + (unsigned long long)i0;
        unsigned long long jt = gt, ct = 0;
        if (gt >= pl.pre && gt <= pl.end) {
            const unsigned long long t = gt - pl.pre;
            ct = t / pl.P;
            jt = pl.pre + (t - ct * pl.P);
        }
        const int d = rlane >= 0 && rlane * SPAN < tin ? rlane * SPAN : 0;
        const rs_ref r = rs_locate_near(pl, gt, jt, ct, (unsigned)d);
        f.e = rs_load(pl, r.ck);
        f.cyc = r.cyc;
        f.skip = r.skip;
    };

    const long long G = gridDim.x;
    long long tile0 = blockIdx.x;
    if (tile0 >= ntiles) return;
    // two register sets, two tiles in flight while one is evaluated; the loop
    // is unrolled by two so a set is never copied, which would wait on its
    // loads at once
    Pre pa, pb;
    fetch(tile0, pa);
    fetch(tile0 + G, pb);
    auto body = [&](long long tile, Pre &cur) {
        const long long i0 = tile * tin;
        const long long ie = (i0 + tin < n) ? i0 + tin : n;   // the tile's inputs [i0, ie)
        const lqk_rs_entry e = cur.e;                         // (fetch overwrites cur below)
        const unsigned long long cyc = cur.cyc;
        const int skip = (RS_EXP & 1) ? 0 : cur.skip;
        __syncthreads();                              // previous tile consumed
#pragma unroll
        for (int u = 0; u < NXV; u++) {
            const int t = tid + u * NT;
            if (t < TS) cp0[t] = u == 0 ? cur.xa[0] + cur.xh : cur.xa[u];
        }
        // in flight during this tile and the next; unconditional (a tile past
        // the end loads out of range: zeros, and positions the plan clamps)
        fetch(tile + 2 * G, cur);
        // wave 0 replays the timing: lane s the SPAN inputs from i0 + s SPAN,
        // starting at its checkpoint (skip < SPAN inputs before them), writing
        // the tile's output list and the outputs before its last input
        if (rlane >= 0) {
            const long long ia = i0 + (long long)rlane * SPAN;
            const int nin = ia < ie ? (int)((ie - ia) < SPAN ? (ie - ia) : SPAN) : 0;
            unsigned long long k = (unsigned long long)e.K + cyc * pl.Q;
            auto put = [&](unsigned long long Kb, int iloc, int bank, float mu) {
                const unsigned long long o = k - Kb;
                if (!(RS_EXP & 4))
                    desc[o < (unsigned long long)CAP ? (int)o : CAP] =
                        make_uint2(__float_as_uint(mu), (unsigned)iloc | ((unsigned)bank << 12));
            };
            unsigned long long Kb;
            if (pl.p2) {
                // power-of-two banks: the state is tau alone (rs_derive); an
                // input emits while tau < 1 - 1/npfb, then tau -= 1
#pragma clang fp contract(off)
                const float z = 1.0f - 1.0f / fnpfb;
                float xx = e.tau;
                for (int i = 0; i < skip; i++) {
                    while (xx < z) {
                        xx = xx + del;
                        k++;
                    }
                    xx = xx - 1.0f;
                }
                Kb = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(k >> 32), 0) << 32) |
                     (unsigned)__builtin_amdgcn_readlane((int)k, 0);
#if RS_O32
                // the lane's output slot as a 32-bit counter (a 64-bit k and
                // its compare per output before); an offset at or past 2^30
                // stays past CAP through the lane's outputs, as before
                {
                    const unsigned long long o64 = k - Kb;
                    const int o0 = o64 < (1ull << 30) ? (int)o64 : (1 << 30);
                    int o = o0;
                    for (int r = 0; r < nin; r++) {
                        const int iloc = (int)(ia + r - i0);
#if RS_UNR > 0
                        // the first RS_UNR outputs of the input without a loop:
                        // predicated (a skipped one writes the sink slot)
#pragma unroll
                        for (int j = 0; j < RS_UNR; j++) {
                            const bool e = xx < z;
                            const float bf = xx * fnpfb;
                            const float fb = __builtin_floorf(bf);
                            if (!(RS_EXP & 4))
                                desc[(e && (unsigned)o < (unsigned)CAP) ? o : CAP] = make_uint2(
                                    __float_as_uint(bf - fb), (unsigned)iloc | ((unsigned)(xx < 0.0f ? npfb : (int)fb) << 12));
                            o += e ? 1 : 0;
                            const float xn = xx + del;
                            xx = e ? xn : xx;
                        }
#endif
                        while (xx < z) {
                            const float bf = xx * fnpfb;
                            const float fb = __builtin_floorf(bf);
                            if (!(RS_EXP & 4))
                                desc[(unsigned)o < (unsigned)CAP ? o : CAP] = make_uint2(
                                    __float_as_uint(bf - fb), (unsigned)iloc | ((unsigned)(xx < 0.0f ? npfb : (int)fb) << 12));
                            o++;
                            xx = xx + del;
                        }
                        xx = xx - 1.0f;
                    }
                    k += (unsigned long long)(o - o0);
                }
#else
                for (int r = 0; r < nin; r++) {
                    const int iloc = (int)(ia + r - i0);
                    while (xx < z) {
                        const float bf = xx * fnpfb;
                        const float fb = __builtin_floorf(bf);
                        put(Kb, iloc, xx < 0.0f ? npfb : (int)fb, bf - fb);
                        k++;
                        xx = xx + del;
                    }
                    xx = xx - 1.0f;
                }
#endif
            } else {
                rs_state st;
                rs_entry(e, st);
                for (int i = 0; i < skip; i++) k += rs_step(st, del, fnpfb, npfb);
                Kb = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(k >> 32), 0) << 32) |
                     (unsigned)__builtin_amdgcn_readlane((int)k, 0);
                for (int r = 0; r < nin; r++) {
                    const int iloc = (int)(ia + r - i0);
                    while ((unsigned)st.b < (unsigned)npfb) {
                        if (st.st && st.b == npfb - 1) {
                            st.st = 0;
                            st.b = npfb;
                            break;
                        }
                        put(Kb, iloc, st.st ? st.b : npfb, st.mu);
                        k++;
                        rs_advance(st, del, fnpfb);
                        st.st = 1;
                    }
                    st.tau -= 1.0f;
                    st.b = (int)((unsigned)st.b - (unsigned)npfb);
                }
            }
            if (nin > 0) kx[rlane + 1] = k;
            if (rlane == 0) kx[0] = Kb;
        }
        __syncthreads();
        const unsigned long long Kb = kx[0];
        const long long nlane = (ie - i0 + SPAN - 1) / SPAN;
        long long ntile = (long long)(kx[nlane] - Kb);
        ntile = ntile < 0 ? 0 : (ntile > CAP ? CAP : ntile);   // exact; the clamp is a guard
        const int nr = (int)ntile;
        const unsigned ob = (unsigned)(Kb - K0);              // the tile's first output
        // y = sum_p (T.x + mu T.d)[p] w[p]; with RS_CH > 0 the reads are issued
        // RS_CH taps at a time, a scheduling barrier after each chunk, so the
        // compiler batches that many round trips and no more (registers)
        auto dot = [&](const S *wv, int bb, float mu) -> S {
            const float2 *tp = tpl + (2 * ROFF + (bb & 1)) * RS + (bb >> 1);
            S acc{};
#pragma unroll
            for (int p = 0; p <= L; p++) {
                const float2 t = lds_rd(tp + 2 * p * RS);
                const float c = fmaf(mu, t.y, t.x);
                const S w = lds_rd(wv + p);
                if constexpr (sizeof(S) == 8) {
                    v2f a2 = {acc.x, acc.y};
                    a2 = v2f{c, c} * v2f{w.x, w.y} + a2;
                    acc = make_float2(a2.x, a2.y);
                } else {
                    acc = rs_axpy(c, w, acc);
                }
#if RS_CH > 0
                if ((p + 1) % RS_CH == 0) __builtin_amdgcn_sched_barrier(0);
#endif
            }
            return acc;
        };
        if constexpr (PR) {
            // pairs q = tid + k NT: outputs 2q, 2q + 1 (desc is 16-byte aligned)
            constexpr int NPS = (CAP / 2 + NT - 1) / NT;
#pragma unroll
            for (int k = 0; k < NPS; k++) {
                const int q = tid + k * NT, oa = 2 * q;
                S va{}, vb{};
                if (oa < nr && !(RS_EXP & 2)) {
                    const uint4 dd = lds_rd4(reinterpret_cast<const uint4 *>(desc) + q);
                    const bool hb = oa + 1 < nr;
                    const int ia = (int)(dd.y & 4095u), bA = (int)(dd.y >> 12);
                    const int d = hb ? (int)(dd.w & 4095u) - ia : 0;
                    const int bB = hb ? (int)(dd.w >> 12) : 0;
                    const float muA = __uint_as_float(dd.x), muB = hb ? __uint_as_float(dd.z) : 0.0f;
                    const S *wv = cp0 + ia + 1;
                    const float2 *tA = tpl + (2 * ROFF + (bA & 1)) * RS + (bA >> 1);
                    const float2 *tB = tpl + (2 * (ROFF - d) + (bB & 1)) * RS + (bB >> 1);
#pragma unroll
                    for (int pp = 0; pp <= L + 1; pp++) {
                        const S w = lds_rd(wv + pp);
                        const float2 tb = lds_rd(tB + 2 * pp * RS);
                        const float cb = fmaf(muB, tb.y, tb.x);
                        // B's window is W[d .. d + L]: the sample outside it enters as 0
                        const S wb = ((pp == 0 && d == 1) || (pp == L + 1 && d == 0)) ? S{} : w;
                        if (pp <= L) {
                            const float2 ta = lds_rd(tA + 2 * pp * RS);
                            const float ca = fmaf(muA, ta.y, ta.x);
                            va = rs_fma(ca, w, va);
                        }
                        vb = rs_fma(cb, wb, vb);
                    }
                }
                const unsigned ob2 = ob + (unsigned)oa;
                const unsigned offa = oa + 1 < nr ? ob2 * (unsigned)sizeof(S) : 0x80000000u;   // both
                const unsigned offs = (oa < nr && oa + 1 >= nr) ? ob2 * (unsigned)sizeof(S) : 0x80000000u;   // A alone
                rs_store2(ry, offa, va, vb);
                rs_store1(ry, offs, va);
            }
        } else {
        // NSLOT outputs per lane, every store issued (slots past the tile's
        // outputs go out of range and are dropped): a fixed store count.
        // With RS_BF the slots below TIN run without a branch (an idle slot
        // evaluates window 0 / bank 0, its store dropped), so the compiler can
        // interleave the reads of several outputs
#pragma unroll
        for (int k = 0; k < NSLOT; k++) {
            const int o = tid + k * NT;
            S v{};
            if (RS_BF && (k + 1) * NT <= TIN && !(RS_EXP & 2)) {
                const uint2 d0 = lds_rd(&desc[o]);
                const uint2 dd = o < nr ? d0 : make_uint2(0u, 0u);
                v = dot(cp0 + (int)(dd.y & 4095u) + 1, (int)(dd.y >> 12), __uint_as_float(dd.x));
            } else if (o < nr && !(RS_EXP & 2)) {
                const uint2 dd = desc[o];
                v = (RS_EXP & 4) ? dot(cp0 + (int)(dd.y & 1023u) + 1, (int)((dd.y >> 12) & 63u), __uint_as_float(dd.x))
                                 : dot(cp0 + (int)(dd.y & 4095u) + 1, (int)(dd.y >> 12), __uint_as_float(dd.x));
            }
            const unsigned off = o < nr ? (ob + (unsigned)o) * (unsigned)sizeof(S) : 0xFFFFFFF0u;
            if constexpr (sizeof(S) == 8) {
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), ry, off, 0, RS_STAUX);
            } else {
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), ry, off, 0, RS_STAUX);
            }
        }
        }
    };
    for (long long tile = tile0; tile < ntiles; tile += 2 * G) {
        body(tile, pa);
        if (tile + G >= ntiles) break;
        body(tile + G, pb);
    }
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

template <int L, typename S, int RSC, bool PR>
void launch_rs2(const lqk_rs_plan &pl, unsigned long long g0, unsigned long long K0, int npfb, float del,
                const float2 *taps2, const S *hist, const S *x, long long n, S *y, unsigned long long nout, int tin,
                hipStream_t st)
{
    const long long ntiles = (n + tin - 1) / tin;
    constexpr int BLK = rs2_blk<L>();
    const unsigned nb = (unsigned)(ntiles < 256 * BLK ? ntiles : 256 * BLK);   // persistent: BLK per CU
    const size_t lds = rs2_lds_bytes<L, S, RSC, PR>(npfb);
    hipLaunchKernelGGL((k_resamp2<L, S, RSC, PR>), dim3(nb), dim3(NT), lds, st, pl, g0, K0, npfb, del, taps2, hist, x,
                       n, y, (int)nout, tin);
}

template <int L, typename S>
void launch_rs(const lqk_rs_plan &pl, unsigned long long g0, unsigned long long K0, int npfb, float del,
               const float2 *taps, const float2 *taps2, const S *hist, const S *x, long long n, S *y,
               unsigned long long nout, hipStream_t st)
{
    constexpr int TIN = rs2_tin<L>();
    constexpr int RSC = RS_RSC ? 33 : 0;       // constant stride for npfb <= 64
    const bool cst = RSC && npfb <= 2 * (RSC - 1);
    // pairs of outputs per lane when consecutive outputs are at most one input
    // apart: tau moves by del per output and by -1 per input, and an input
    // emits while tau < 1 - 1/npfb, so after an output at tau_k < 1 - 1/npfb
    // the next input emits if tau_k + del - 1 < 1 - 1/npfb: del <= 1, here
    // with a margin for the float32 rounding of tau_k + del
    const bool pr = RS_PAIR && del <= 1.0f - 0x1p-22f;
    const size_t lds2 = rs2_lds_bytes<L, S, 0, true>(npfb);   // at least that of any layout launched
    if (taps2 != nullptr && lds2 <= 64 * 1024 && pl.P < (1ull << 31) && (pl.pre < (1ull << 62) || pl.end < (1ull << 62))) {
        // inputs per tile: every tile's outputs fit the CAP output slots (at
        // most (tin + 2) r + 2 outputs: tau moves by 1/r per output and by -1
        // per input within [-1/npfb, 1 + 1/r))
        constexpr int CAP = rs2_cap();
        const double r = 1.0 / (double)del;
        int tin = TIN;
        while (tin > LQK_RS_CK && std::ceil((tin + 2) * r) + 2 > CAP) tin -= LQK_RS_CK;
        if (std::ceil((tin + 2) * r) + 2 <= CAP) {   // else (r > ~60): the per-input kernel below
            if (cst && pr) launch_rs2<L, S, RSC, true>(pl, g0, K0, npfb, del, taps2, hist, x, n, y, nout, tin, st);
            else if (cst) launch_rs2<L, S, RSC, false>(pl, g0, K0, npfb, del, taps2, hist, x, n, y, nout, tin, st);
            else launch_rs2<L, S, 0, false>(pl, g0, K0, npfb, del, taps2, hist, x, n, y, nout, tin, st);
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
