// k_channelizer.hip -- polyphase channelizers (firpfbch2 2x-oversampled and
// firpfbch critically sampled, analyzers and synthesizers) and the batched
// LDS FFT they share.
//
// Reference semantics restated, not translated:
//  firpfbch2 analyzer  src/multichannel/src/firpfbch2.c:244-282.  The
//    reference pushes M/2 samples per call into M ring buffers and runs M
//    dot products then an M-point IFFT.  Here block b is evaluated from the
//    stream directly (closed form, SURVEY Appendix B, checked numerically):
//        off = (b&1)*M/2,  i = (j - off) mod M
//        c   = j < M/2 ? b>>1 : (b-1)>>1,  base = j < M/2 ? M/2-1-j : 3M/2-1-j
//        X_b[j] = sum_{n<2m} h[i + nM] x[(c-n)M + base]
//        Y_b    = IFFT_backward(X_b) / M
//    so any number of blocks run in parallel; the only state carried between
//    calls is the last 2mM - M/2 input samples and the block parity.
//  firpfbch2 synthesizer firpfbch2.c:287-335: z_b = IFFT(X_b)*(1/M)*(M/2);
//        y_b[i] = sum_n h[i+nM] z_{b-2n}[i+fM/2] + sum_n h[i+M/2+nM] z_{b-1-2n}[i+fM/2]
//    (f = b&1); state = the last 4m-1 z vectors.
//  firpfbch analyzer src/multichannel/src/firpfbch.c:346-409:
//        X_b[j] = sum_{n<p} h[(M-1-j) + nM] x[(b-n)M + j],  Y_b = FFT_forward(X_b)
//  firpfbch synthesizer firpfbch.c:314-336: z_b = IFFT(X_b),
//        y_b[i] = sum_{n<p} h[i+nM] z_{b-n}[i]
#include "lq_device.h"
#include "lq_fft1024.h"
#include "lq_kernels.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace {

constexpr int NT = 256;

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not its global loads and stores (__syncthreads() also drains
// vmcnt: every store and prefetch in flight)
__device__ __forceinline__ void lds_barrier_w()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ float2 ext_load(const float2 *__restrict__ hist, int HL, const float2 *__restrict__ x,
                                           long long t)
{
    return t < 0 ? hist[HL + t] : x[t];
}

// ------------------------------------------------------------------ firpfbch2 analyzer
// One workgroup = NB consecutive blocks; X for all NB blocks is formed in LDS,
// transformed by the LDS Stockham FFT, scaled and stored coalesced.
template <int M, int NB>
__global__ __launch_bounds__(NT) void k_pfb2_an(int m, const float *__restrict__ hsub,
                                                const float2 *__restrict__ hist, const float2 *__restrict__ x,
                                                long long nblocks, int p0, float2 *__restrict__ Y,
                                                const float2 *__restrict__ tw)
{
    __shared__ __attribute__((aligned(16))) float2 a[NB * M];
    __shared__ __attribute__((aligned(16))) float2 b[NB * M];
    constexpr int M2 = M / 2;
    const int L = 2 * m;
    const int HL = 2 * m * M - M2;
    const long long blk0 = (long long)blockIdx.x * NB;

    for (int e = threadIdx.x; e < NB * M; e += NT) {
        const int bl = e / M;
        const int j = e - bl * M;
        const long long gb = blk0 + bl;
        float2 acc = make_float2(0.f, 0.f);
        if (gb < nblocks) {
            const long long bt = p0 + gb;
            const int off = (int)(bt & 1) * M2;
            const int i = (j - off) & (M - 1);
            const long long c = (j < M2) ? (bt >> 1) : ((bt - 1) >> 1);
            const int base = (j < M2) ? (M2 - 1 - j) : (3 * M2 - 1 - j);
            const long long t0 = c * M + base - (long long)p0 * M2;
            const float *hs = hsub + i * L;
            for (int n = 0; n < L; n++) {
                const float2 v = ext_load(hist, HL, x, t0 - (long long)n * M);
                acc.x = fmaf(hs[n], v.x, acc.x);
                acc.y = fmaf(hs[n], v.y, acc.y);
            }
        }
        a[e] = acc;
    }
    __syncthreads();
    float2 *res = lds_fft<M, NB, NT>(a, b, tw, -1);
    const float inv = 1.0f / (float)M; // exact: M is a power of two
    for (int e = threadIdx.x; e < NB * M; e += NT) {
        const int bl = e / M;
        const long long gb = blk0 + bl;
        if (gb < nblocks) Y[(blk0 + bl) * M + (e - bl * M)] = cscale(res[e], inv);
    }
}

// Polyphase pass for power-of-two M >= 64 (M != 1024, which has the fused
// kernel of k_pfb2_fast.hip), followed by a batched transform over Y in
// place.  Same column view as the fused kernel: in aligned coordinates
// t' = t + p0 M/2 the stream is rows of M samples, column col feeds bin
// j = M/2-1-col (lo) or 3M/2-1-col (hi), and row c completes blocks 2c + dA
// and 2c + dA + 1 (dA = 0 lo, 1 hi) with the L = 2m taps of bin j for the
// even block and of bin j ^ M/2 for the odd one:
//     X_b[j] = sum_n h[i + nM] row[c - n][col]
// A workgroup owns a slice of min(M, 256) columns (one per lane) and a run
// of S rows; L-1 rows before the run warm its register ring up.  Rows are
// read once per slice and run (2 KB coalesced per row and workgroup), a
// group of L rows is prefetched while the previous group is evaluated, and
// X goes straight into Y (coalesced: consecutive columns are consecutive
// bins, reversed), where the batched transform then runs in place.
// Samples come through two range-checked descriptors (history: HL samples,
// x: n_in), each sample in range in at most one of them.
template <int L>
__global__ __launch_bounds__(256) void k_pfb2_poly(int M, int nsl, const float *__restrict__ hsub,
                                                  const float2 *__restrict__ hist, const float2 *__restrict__ x,
                                                  int n_in, int p0, int nb, int cmin, int cmax, int S,
                                                  float2 *__restrict__ Y, const float2 *__restrict__ zero)
{
    const int M2 = M >> 1, HL = L * M - M2;
    const int sl = (int)(blockIdx.x % (unsigned)nsl), seg = (int)(blockIdx.x / (unsigned)nsl);
    const int col = sl * (int)blockDim.x + (int)threadIdx.x;
    const bool lo = col < M2;
    const int j = lo ? (M2 - 1 - col) : (3 * M2 - 1 - col);
    const int dA = lo ? 0 : 1;
    // taps of the first (ta) and second (tb) block a row completes: lo: even
    // block 2c (bin j), odd 2c+1 (j ^ M/2); hi: odd 2c+1, even 2c+2
    float ta[L], tb[L];
    {
        const int ia = lo ? j : (j ^ M2), ib = lo ? (j ^ M2) : j;
#pragma unroll
        for (int n = 0; n < L; n++) {
            ta[n] = hsub[ia * L + n];
            tb[n] = hsub[ib * L + n];
        }
    }
    // Y: nb blocks of M; a store outside (blocks before / after the call) is dropped
    const __amdgpu_buffer_rsrc_t ry =
        __builtin_amdgcn_make_buffer_rsrc((void *)Y, (short)0, nb * M * 8, 0x00020000);
    auto row_sample = [&](int r) -> float2 {
        const int t = r * M + col - p0 * M2;              // stream sample (t < 0: history)
        return lq_load_hx(hist + HL, x, zero, t, HL, n_in);
    };
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    auto put = [&](int bt, float2 v) {   // block bt of the aligned numbering, bin j
        const int gb = bt - p0;
        const unsigned off = (gb >= 0 && gb < nb) ? ((unsigned)gb * (unsigned)M + (unsigned)j) * 8u : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), ry, off, 0, 0);
    };
    const int cs = cmin + seg * S;
    int ce = cs + S;
    if (ce > cmax + 1) ce = cmax + 1;
    // register ring over groups of L rows: step u of a group puts row
    // r + u into w[u] (the slot of row r + u - L, no longer needed), so row
    // c - n is in w[(u - n) mod L] -- static indices, no moves.  The next
    // group's samples are loaded one per step, L loads in flight.
    float2 w[L], pf[L];
    int r = cs - (L - 1);
#pragma unroll
    for (int u = 0; u < L; u++) pf[u] = row_sample(r + u);
    for (; r < ce; r += L) {
#pragma unroll
        for (int u = 0; u < L; u++) {
            w[u] = pf[u];
            pf[u] = row_sample(r + L + u);
            const int c = r + u;
            if (c >= cs && c < ce) {
                float2 da = make_float2(0.f, 0.f), db = make_float2(0.f, 0.f);
#pragma unroll
                for (int n = 0; n < L; n++) {
                    const float2 v = w[(u - n + L) % L];
                    da.x = fmaf(ta[n], v.x, da.x);
                    da.y = fmaf(ta[n], v.y, da.y);
                    db.x = fmaf(tb[n], v.x, db.x);
                    db.y = fmaf(tb[n], v.y, db.y);
                }
                put(2 * c + dA, da);
                put(2 * c + dA + 1, db);
            }
        }
    }
}

// M = 256 analyzer fused: the polyphase pass above with all 256 columns in
// one workgroup (one per lane), a ring of 8 rows in registers (L = 2m <= 8),
// and each group of 8 rows' 16 completed blocks transformed in the same
// kernel: X goes to a 17-buffer LDS ring (block b in buffer b mod 17; the
// hi half of block 2r0+16 is written one group early), then 16 inverse
// 256-point transforms run in registers (fft_r16x16xR<1>, 16 lanes each) and
// the outputs, times 1/M, leave as consecutive 8-byte stores -- Y is written
// once and never re-read (24 B per input instead of the two-pass 56).
template <int L, int R>
__global__ __launch_bounds__(256 * R, R == 1 ? 2 : 1) void k_pfb2_an256(const float *__restrict__ hsub,
                                                       const float2 *__restrict__ hist,
                                                       const float2 *__restrict__ x, int n_in, int p0, int nb,
                                                       int cmin, int cmax, int S, float2 *__restrict__ Y,
                                                       const float2 *__restrict__ tw4096)
{
    // M = 256 R columns, one per lane; R = 2 takes the tight transform
    // scratch (17 x 4 KB ring + 16 x 4.3 KB scratch fits 160 KB)
    constexpr int M = 256 * R, M2 = M / 2, HL = L * M - M2, NS = 8, NBUF = 17;
    constexpr bool TIGHT = R > 1;
    constexpr int P = FFTR16_LDS<R, TIGHT>();
    __shared__ __attribute__((aligned(16))) float2 xr[NBUF * M];
    __shared__ __attribute__((aligned(16))) float2 scr[16 * P];
    const int col = threadIdx.x;
    const bool lo = col < M2;
    const int j = lo ? (M2 - 1 - col) : (3 * M2 - 1 - col);
    const int dA = lo ? 0 : 1;
    float ta[L], tb[L];
    {
        const int ia = lo ? j : (j ^ M2), ib = lo ? (j ^ M2) : j;
#pragma unroll
        for (int n = 0; n < L; n++) {
            ta[n] = hsub[ia * L + n];
            tb[n] = hsub[ib * L + n];
        }
    }
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)Y, (short)0, nb * M * 8, 0x00020000);
    const float2 *zero = tw4096 + LQ_TW_N;   // lqrt_zeros(): the table's zero tail
    auto row_sample = [&](int r) -> float2 {
        const int t = r * M + col - p0 * M2;
        return lq_load_hx(hist + HL, x, zero, t, HL, n_in);
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
    auto slot = [](int b) { return ((b % NBUF) + NBUF) % NBUF; };
    const int g = threadIdx.x / (16 * R), t = threadIdx.x % (16 * R);   // transform g (block 2 r0 + g), its lane t
    const tw16x2 w16 = fftr16_tw<R>(tw4096, t);
    const float inv = 1.0f / (float)M;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

    const int cs = cmin + (int)blockIdx.x * S;
    int ce = cs + S;
    if (ce > cmax + 1) ce = cmax + 1;
    // rows cs-8 .. cs-1 fill the ring (slots r & 7); the last gives the hi
    // half of block 2cs
    float2 w[NS], pf[NS];
#pragma unroll
    for (int u = 0; u < NS; u++) w[u] = row_sample(cs - NS + u);
    if (!lo) xr[slot(2 * cs) * M + j] = dot(w, NS - 1, tb);
#pragma unroll
    for (int u = 0; u < NS; u++) pf[u] = row_sample(cs + u);
    for (int r0 = cs; r0 < ce; r0 += NS) {
#pragma unroll
        for (int u = 0; u < NS; u++) {
            w[u] = pf[u];
            pf[u] = row_sample(r0 + NS + u);
            const int c = r0 + u;
            xr[slot(2 * c + dA) * M + j] = dot(w, u, ta);
            xr[slot(2 * c + dA + 1) * M + j] = dot(w, u, tb);
        }
        lds_barrier_w();
        // blocks 2 r0 .. 2 r0 + 15 are complete: one transform per 16 lanes
        const int b = 2 * r0 + g;
        float2 v[16];
        const float2 *B = xr + slot(b) * M;
#pragma unroll
        for (int n = 0; n < 16; n++) v[n] = B[t + 16 * R * n];
        fft_r16x16xR<R, -1, TIGHT>(v, scr + g * P, w16, t);   // (its barriers also free the ring buffers)
        const int gb = b - p0;
        const bool keep = gb >= 0 && gb < nb && b < 2 * ce;
        const unsigned base = keep ? (unsigned)gb * (unsigned)(M * 8) : 0xFFFFF000u;
        // v[s R + q] = X[t + 16 R s + 256 q]
#pragma unroll
        for (int sidx = 0; sidx < 16 / R; sidx++)
#pragma unroll
            for (int q = 0; q < R; q++) {
                const float2 vv = v[sidx * R + q];
                const float2 o = make_float2(vv.x * inv, vv.y * inv);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), ry,
                                                      base + (unsigned)(t + 16 * R * sidx + 256 * q) * 8u, 0, 0);
            }
    }
}

template <int L, int R>
bool launch_pfb2_an256(const void *hsub, const void *hist, const void *x, long long nb, int p0, void *Y, hipStream_t st)
{
    constexpr int M = 256 * R;
    const long long n_in = nb * (M / 2);
    if (n_in * 8 >= (1ll << 31) || nb * (long long)M * 8 >= (1ll << 31)) return false;
    const int cmin = (p0 - 1) >> 1;
    const int cmax = (int)((p0 + nb - 1) >> 1);
    const int rows = cmax - cmin + 1;
    // runs of S rows (a multiple of 8): about 1024 workgroups on long calls
    // (a remainder of a few rows goes to one short extra run, as in
    // launch_pfb2_an2048)
    long long S = ((long long)rows + 1023) / 1024;
    S = (S + 7) / 8 * 8;
    const long long S8 = (long long)rows / 8192 * 8;
    if (S8 >= 32 && rows - 1024 * S8 <= S8 / 4) S = S8;
    if (S < 32) S = 32;
    const long long nseg = (rows + S - 1) / S;
    hipLaunchKernelGGL((k_pfb2_an256<L, R>), dim3((unsigned)nseg), dim3(256 * R), 0, st, (const float *)hsub,
                       (const float2 *)hist, (const float2 *)x, (int)n_in, p0, (int)nb, cmin, cmax, (int)S,
                       (float2 *)Y, (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
    return true;
}

// M = 2048 analyzer fused (the two-pass path moved 56 B per input): 1024
// lanes, lane t owning the lo column t (bin j = 1023 - t) and the hi column
// t + 1024 (bin j ^ 1024), so both columns share the lane's two tap sets
// (A: taps of bin j, B: of bin j ^ 1024):
//     lo, row c:  block 2c   += A . column,  block 2c+1 += B . column
//     hi, row c:  block 2c+1 += A . column,  block 2c+2 += B . column
// A group of 4 rows completes 8 blocks into a 9-buffer LDS ring; a block's
// buffer holds its even bins and its odd bins as two 1024-point halves.
// Each of the 16 waves then inverse-transforms one half in registers
// (fft1024_wave_rt: wave-local transposes, no workgroup barrier), and after
// one barrier the wave combines its block's halves for 512 output pairs,
//     Y[k] = E[k] + W_2048^-k O[k],  Y[k + 1024] = E[k] - W_2048^-k O[k],
// times 1/M, stored as 1 KB coalesced rows.  Three barriers per group (a
// 2048-point transform across two waves took six: 1.07 ms per 2^27 samples).
constexpr int A2_HS = 1090;            // half stride: 1088-float2 transform scratch, +2 spreads the halves' banks
constexpr int A2_BSTR = 2 * A2_HS;     // 16-byte aligned halves
template <int L>
__global__ __launch_bounds__(1024, 1) void k_pfb2_an2048(const float *__restrict__ hsub,
                                                         const float2 *__restrict__ hist,
                                                         const float2 *__restrict__ x, int n_in, int p0, int nb,
                                                         int cmin, int cmax, int S, float2 *__restrict__ Y,
                                                         const float2 *__restrict__ tw4096)
{
    constexpr int M = 2048, M2 = 1024, HL = L * M - M2, NS = 8, G = 4, NBUF = 2 * G + 1;
    static_assert(L <= NS, "ring of 8 rows");
    __shared__ __attribute__((aligned(16))) float2 xr[NBUF * A2_BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw2[64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 64) {   // W_64^{-b r} (inverse transform)
        const float2 u = tw4096[(64 * (tid & 3) * (tid >> 2)) & 4095];
        tw2[tid] = make_float2(u.x, -u.y);
    }
    const float2 a1 = tw4096[(4 * lane) & 4095], a4 = tw4096[(16 * lane) & 4095];
    const int jl = M2 - 1 - tid, jh = jl ^ M2;   // bins of the lo / hi column
    // split position of bin j in its block: half j & 1, index j >> 1
    const int pl_lo = (jl & 1) * A2_HS + (jl >> 1), pl_hi = (jh & 1) * A2_HS + (jh >> 1);
    // taps re-read (L1/L2 hits) at every group instead of held across the
    // transforms: 16 VGPRs the ring and the prefetched rows need there
    float ta[L], tb[L];
    auto load_taps = [&]() {
        int oa = jl * L, ob = jh * L;
        asm volatile("" : "+v"(oa), "+v"(ob));   // keep the reload inside the loop
#pragma unroll
        for (int n = 0; n < L; n++) {
            ta[n] = hsub[oa + n];
            tb[n] = hsub[ob + n];
        }
    };
    load_taps();
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)Y, (short)0, nb * M * 8, 0x00020000);
    const float2 *zero = tw4096 + LQ_TW_N;   // lqrt_zeros(): the table's zero tail
    auto row_sample = [&](int r, int col) -> float2 {
        const int t = r * M + col - p0 * M2;
        return lq_load_hx(hist + HL, x, zero, t, HL, n_in);
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
    auto slot = [](int b) { return ((b % NBUF) + NBUF) % NBUF; };
    const int hb = wave >> 1, hh = wave & 1;   // this wave's block (2 r0 + hb) and half
    const float inv = 1.0f / (float)M;
    typedef float v4f __attribute__((ext_vector_type(4)));

    const int cs = cmin + (int)blockIdx.x * S;
    int ce = cs + S;
    if (ce > cmax + 1) ce = cmax + 1;
    // rows cs-8 .. cs-1 fill the ring (slot r & 7); the last gives the hi
    // half of block 2cs
    float2 wl[NS], wh[NS], pl[G], ph[G];
#pragma unroll
    for (int u = 0; u < NS; u++) {
        wl[u] = row_sample(cs - NS + u, tid);
        wh[u] = row_sample(cs - NS + u, tid + M2);
    }
    xr[slot(2 * cs) * A2_BSTR + pl_hi] = dot(wh, NS - 1, tb);
#pragma unroll
    for (int u = 0; u < G; u++) {
        pl[u] = row_sample(cs + u, tid);
        ph[u] = row_sample(cs + u, tid + M2);
    }
    __syncthreads();   // tw2 ready
    // one group: rows r0 .. r0+3 into ring slots s0 .. s0+3 (s0 = 0 or 4),
    // then the 8 completed blocks' transforms
    auto group = [&](int r0, auto s0c) {
        constexpr int s0 = decltype(s0c)::value;
        load_taps();
#pragma unroll
        for (int u = 0; u < G; u++) {
            wl[s0 + u] = pl[u];
            wh[s0 + u] = ph[u];
            pl[u] = row_sample(r0 + G + u, tid);
            ph[u] = row_sample(r0 + G + u, tid + M2);
            const int c = r0 + u;
            xr[slot(2 * c) * A2_BSTR + pl_lo] = dot(wl, s0 + u, ta);
            xr[slot(2 * c + 1) * A2_BSTR + pl_lo] = dot(wl, s0 + u, tb);
            xr[slot(2 * c + 1) * A2_BSTR + pl_hi] = dot(wh, s0 + u, ta);
            xr[slot(2 * c + 2) * A2_BSTR + pl_hi] = dot(wh, s0 + u, tb);
        }
        lds_barrier_w();
        const int b = 2 * r0 + hb;
        float2 *Bb = xr + slot(b) * A2_BSTR;
        {
            float2 *Bh = Bb + hh * A2_HS;
            float2 v[16];
#pragma unroll
            for (int n = 0; n < 16; n++) v[n] = Bh[lane + 64 * n];
            fft1024_wave_rt<-1>(v, Bh, a1, a4, tw2, lane);   // natural order at k + 4 (k >> 8)
        }
        lds_barrier_w();   // both halves of every block transformed
        const int gb = b - p0;
        const bool keep = gb >= 0 && gb < nb && b < 2 * ce;
        // a dropped block's base: 2^31 (the launch's range is below it, and
        // base + 16 KB cannot wrap around 2^32 into it)
        const unsigned base = keep ? (unsigned)gb * (unsigned)(M * 8) : 0x80000000u;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int k = 512 * hh + 2 * lane + 128 * i;
            const int pos = k + 4 * (k >> 8);
            // W_2048^-k, W_2048^-(k+1) (table hits in L1 / L2)
            const float2 u0 = tw4096[2 * k], u1 = tw4096[2 * k + 2];
            const float2 wk[2] = {make_float2(u0.x, -u0.y), make_float2(u1.x, -u1.y)};
            const v4f E = *reinterpret_cast<const v4f *>(Bb + pos);
            const v4f O = *reinterpret_cast<const v4f *>(Bb + A2_HS + pos);
            const v2f o0 = pk_cmul(v2f{O.x, O.y}, pk(wk[0])), o1 = pk_cmul(v2f{O.z, O.w}, pk(wk[1]));
            const v2f e0 = v2f{E.x, E.y}, e1 = v2f{E.z, E.w};
            const v2f s0v = (e0 + o0) * inv, s1v = (e1 + o1) * inv, d0 = (e0 - o0) * inv, d1 = (e1 - o1) * inv;
            __builtin_amdgcn_raw_buffer_store_b128(v4f{s0v.x, s0v.y, s1v.x, s1v.y}, ry, base + (unsigned)k * 8u, 0, 2);
            __builtin_amdgcn_raw_buffer_store_b128(v4f{d0.x, d0.y, d1.x, d1.y}, ry, base + (unsigned)(k + 1024) * 8u, 0, 2);
        }
        lds_barrier_w();   // the combine's reads are done before the next group's writes
    };
    // S is a multiple of 8 rows: the ring slot of row r0 + u is u (first
    // group) or 4 + u (second)
    for (int r0 = cs; r0 < ce; r0 += 2 * G) {
        group(r0, std::integral_constant<int, 0>{});
        if (r0 + G < ce) group(r0 + G, std::integral_constant<int, G>{});
    }
}

template <int L>
bool launch_pfb2_an2048(const void *hsub, const void *hist, const void *x, long long nb, int p0, void *Y, hipStream_t st)
{
    constexpr int M = 2048;
    const long long n_in = nb * (M / 2);
    if (n_in * 8 >= (1ll << 31) || nb * (long long)M * 8 >= (1ll << 31)) return false;
    const int cmin = (p0 - 1) >> 1;
    const int cmax = (int)((p0 + nb - 1) >> 1);
    const int rows = cmax - cmin + 1;
    // one workgroup per CU: runs of S rows (a multiple of 8), about 256 runs.
    // A remainder of a few rows past 256 full runs goes to one short extra
    // run rather than stretching every run to the next multiple of 8 (2^27
    // inputs: 65 537 rows, 256 x 256 + 1 instead of 249 x 264 -- 7 CUs idle)
    long long S = ((long long)rows + 255) / 256;
    S = (S + 7) / 8 * 8;
    const long long S8 = (long long)rows / 2048 * 8;
    if (S8 >= 32 && rows - 256 * S8 <= S8 / 4) S = S8;
    if (S < 32) S = 32;
    const long long nseg = (rows + S - 1) / S;
    hipLaunchKernelGGL((k_pfb2_an2048<L>), dim3((unsigned)nseg), dim3(1024), 0, st, (const float *)hsub,
                       (const float2 *)hist, (const float2 *)x, (int)n_in, p0, (int)nb, cmin, cmax, (int)S,
                       (float2 *)Y, (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
    return true;
}

// M = 4096 analyzer fused (the two-pass path moved 56 B per input; the
// same structure as k_pfb2_an2048 one size up): lane t owns four columns,
// t + 1024 q.  The lo columns (q = 0, 1: bins j0 = 2047 - t, j1 = 1023 - t)
// and the hi columns (q = 2, 3: bins j0 ^ 2048, j1 ^ 2048) share the lane's
// four tap sets A_q = taps(j_q), B_q = taps(j_q ^ 2048), q = 0, 1:
//     lo q, row c:  block 2c   += A_q . column,  block 2c+1 += B_q . column
//     hi q, row c:  block 2c+1 += A_q . column,  block 2c+2 += B_q . column
// A 32 KB block leaves room for two block buffers, so a group is one row: it
// completes blocks 2c and 2c+1, whose buffers hold the four 1024-point
// quarters of bins j = r (mod 4), and starts 2c+2, whose hi half waits in a
// compact 16 KB carry buffer that each lane copies into the block-2c buffer
// at the next row (its own positions, no barrier).  Waves 0-7
// inverse-transform one quarter each in registers (fft1024_wave_rt), and
// after a barrier all 16 waves combine their block's quarters (radix 4):
//     Y[k + 1024 s] = sum_r W_4096^-(r k) Q_r[k] i^(r s)   (W^- : e^{+2 pi i ...})
// times 1/M, stored as 16-byte rows.  The row ring is shifted in registers,
// its oldest row kept in LDS (8 VGPRs fewer, which m = 4 needs to fit a
// transform beside the ring in 128).
//   Row c+1 reaches an LDS row buffer by LDS-DMA (global_load_lds_dwordx4,
// no VGPRs) right after row c's dot phase and lands during the transforms
// and the combine.  Round 5 loaded row c+1 into registers after row c's
// transforms and crossed three __syncthreads per row (each draining vmcnt):
// one row in flight per CU, 1.106 ms per 2^27 samples; this form 0.869 ms
// (profiles/r06_ab_experiments.txt).  The barriers wait for LDS only.  LDS:
// 2 x 34.9 (blocks) + 16 (carry) + 32 (oldest ring row) + 32 (row) KB.
constexpr int A4_QS = 1092;            // quarter stride: 1088-float2 transform scratch; 1092 * 8 = 32 mod 128 B
constexpr int A4_BSTR = 4 * A4_QS;     //   puts the four quarters of a dot-phase write on distinct bank groups
template <int L>
__global__ __launch_bounds__(1024, 1) void k_pfb2_an4096(const float *__restrict__ hsub,
                                                          const float2 *__restrict__ hist,
                                                          const float2 *__restrict__ x, int n_in, int p0, int nb,
                                                          int cmin, int cmax, int S, float2 *__restrict__ Y,
                                                          const float2 *__restrict__ tw4096)
{
    constexpr int M = 4096, M2 = 2048, HL = L * M - M2, NS = L;
    __shared__ __attribute__((aligned(16))) float2 xb[2 * A4_BSTR];   // blocks 2c, 2c+1
    __shared__ __attribute__((aligned(16))) float2 hc[2048];          // hi half of block 2c+2
    __shared__ __attribute__((aligned(16))) float2 wold[4 * 1024];    // each column's oldest ring row
    __shared__ __attribute__((aligned(16))) float2 rb[4096];          // row c+1 (LDS-DMA)
    __shared__ __attribute__((aligned(16))) float2 tw2[64];
    typedef float v4f __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 64) {   // W_64^{-b r} (inverse transform)
        const float2 u = tw4096[(64 * (tid & 3) * (tid >> 2)) & 4095];
        tw2[tid] = make_float2(u.x, -u.y);
    }
    const float2 a1 = tw4096[(4 * lane) & 4095], a4 = tw4096[(16 * lane) & 4095];
    const int j0 = M2 - 1 - tid, j1 = M2 / 2 - 1 - tid;   // lo bins; hi bins j ^ M2
    auto qpos = [](int j) { return (j & 3) * A4_QS + (j >> 2); };
    auto hpos = [](int j) { return (j & 3) * 512 + ((j >> 2) - 512); };   // hi bin j in hc
    const int pl0 = qpos(j0), pl1 = qpos(j1), ph0 = qpos(j0 ^ M2), ph1 = qpos(j1 ^ M2);
    const int hc0 = hpos(j0 ^ M2), hc1 = hpos(j1 ^ M2);
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)Y, (short)0, nb * M * 8, 0x00020000);
    const float2 *zero = tw4096 + LQ_TW_N;   // lqrt_zeros(): the table's zero tail (256 B)
    auto row_sample = [&](int r, int col) -> float2 {
        const int t = r * M + col - p0 * M2;
        return lq_load_hx(hist + HL, x, zero, t, HL, n_in);
    };
    // row r into rb: lane t's 16 bytes are samples 2 (t + 1024 u) and + 1
    // (HL, n_in and the row starts are even: a pair never straddles the
    // history / x / zero boundary); wave-uniform LDS base per instruction
    auto dma_row = [&](int r) {
        int to = tid;
        asm volatile("" : "+v"(to));   // addresses recomputed per row (not hoisted into live VGPRs)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const long long t = (long long)r * M + 2 * (to + 1024 * u) - (long long)p0 * M2;
            const bool neg = t < 0;
            const bool in = neg ? (t >= -HL) : (t < n_in);
            unsigned long long a = (unsigned long long)(uintptr_t)(neg ? hist + HL : x) + (unsigned long long)(t * 8);
            a = in ? a : (unsigned long long)(uintptr_t)zero;
            __builtin_amdgcn_global_load_lds((const void *)a,
                                             (__attribute__((address_space(3))) void *)(rb + 2 * (64 * wave + 1024 * u)),
                                             16, 0, 0);
        }
    };
    // rb[tid + 1024 q] through asm: a compiler-visible LDS read of rb would
    // wait for every outstanding vector-memory operation (the DMA's counter
    // is vmcnt) -- the explicit wait before the row's barrier covers it
    auto rb_read = [&](int q) -> float2 {
        const unsigned a = (unsigned)(uintptr_t)(rb + tid);
        v2f v;
        if (q == 0) asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a));
        if (q == 1) asm volatile("ds_read_b64 %0, %1 offset:8192" : "=v"(v) : "v"(a));
        if (q == 2) asm volatile("ds_read_b64 %0, %1 offset:16384" : "=v"(v) : "v"(a));
        if (q == 3) asm volatile("ds_read_b64 %0, %1 offset:24576" : "=v"(v) : "v"(a));
        return make_float2(v.x, v.y);
    };
    float2 w[4][NS - 1], wo[4];
    auto dot = [&](int q, const float (&h)[NS]) -> float2 {
        float2 acc = make_float2(0.f, 0.f);
#pragma unroll
        for (int n = 0; n < NS; n++) {
            const float2 v = n < NS - 1 ? w[q][NS - 2 - n] : wo[q];
            acc.x = fmaf(h[n], v.x, acc.x);
            acc.y = fmaf(h[n], v.y, acc.y);
        }
        return acc;
    };
    // the lane's four tap sets (A0 = taps(j0), Bt0 = taps(j0 ^ M2), A1, Bt1),
    // re-read (L1 / L2 hits) one set at a time in the dot phase: 8 VGPRs of
    // taps live, not 32 (loaded before the previous row's stores instead, all
    // four sets beside the ring spilled 16 VGPRs)
    float th[NS];
    auto load_set = [&](int j) {
        int o = j * L;
        asm volatile("" : "+v"(o));   // reloaded per row, not hoisted
#pragma unroll
        for (int n = 0; n < NS; n++) th[n] = hsub[o + n];
    };
    const float inv = 1.0f / (float)M;

    const int cs = cmin + (int)blockIdx.x * S;
    int ce = cs + S;
    if (ce > cmax + 1) ce = cmax + 1;
    dma_row(cs);
    // rows cs-NS .. cs-1 fill the ring; the last gives the hi half of block 2cs
#pragma unroll
    for (int q = 0; q < 4; q++) {
        wo[q] = row_sample(cs - NS, tid + 1024 * q);
#pragma unroll
        for (int u = 0; u < NS - 1; u++) w[q][u] = row_sample(cs - NS + 1 + u, tid + 1024 * q);
    }
    load_set(j0 ^ M2);
    hc[hc0] = dot(2, th);
    load_set(j1 ^ M2);
    hc[hc1] = dot(3, th);
    if constexpr (NS > 1) {   // row cs - NS + 1: the oldest of row cs's dots
#pragma unroll
        for (int q = 0; q < 4; q++) wold[q * 1024 + tid] = w[q][0];
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();   // tw2, row cs in rb
    const int qb = wave >> 2, qq = wave & 3;   // transform phase: block 2c + qb, quarter qq (waves 0-7)
    const int cb = wave >> 3, wb = wave & 7;   // combine phase: block 2c + cb, pairs lane + 64 wb
    float2 *B0 = xb, *B1 = xb + A4_BSTR;
    for (int c = cs; c < ce; c++) {
        float2 nr[4];
#pragma unroll
        for (int q = 0; q < 4; q++) nr[q] = rb_read(q);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < 4; q++) {
            wo[q] = wold[q * 1024 + tid];
            if constexpr (NS > 1) {
#pragma unroll
                for (int u = 0; u < NS - 2; u++) w[q][u] = w[q][u + 1];
                w[q][NS - 2] = nr[q];
            } else {
                wo[q] = nr[q];
            }
        }
        // block 2c's hi half, carried from row c - 1 (this lane's positions)
        B0[ph0] = hc[hc0];
        B0[ph1] = hc[hc1];
        load_set(j0);
        B0[pl0] = dot(0, th);
        B1[ph0] = dot(2, th);
        asm volatile("" ::: "memory");
        load_set(j0 ^ M2);
        B1[pl0] = dot(0, th);
        hc[hc0] = dot(2, th);
        asm volatile("" ::: "memory");
        load_set(j1);
        B0[pl1] = dot(1, th);
        B1[ph1] = dot(3, th);
        asm volatile("" ::: "memory");
        load_set(j1 ^ M2);
        B1[pl1] = dot(1, th);
        hc[hc1] = dot(3, th);
        if constexpr (NS > 1) {
#pragma unroll
            for (int q = 0; q < 4; q++) wold[q * 1024 + tid] = w[q][0];
        }
        lds_barrier_w();   // blocks complete, rb consumed by every wave
        if (c + 1 < ce) dma_row(c + 1);
        if (wave < 8) {
            float2 *Bq = (qb ? B1 : B0) + qq * A4_QS;
            float2 v[16];
#pragma unroll
            for (int n = 0; n < 16; n++) v[n] = Bq[lane + 64 * n];
            fft1024_wave_rt<-1>(v, Bq, a1, a4, tw2, lane);   // natural order at k + 4 (k >> 8)
        }
        lds_barrier_w();   // every quarter of both blocks transformed
        {
            const int b = 2 * c + cb;
            const float2 *Bb = cb ? B1 : B0;
            const int gb = b - p0;
            const bool keep = gb >= 0 && gb < nb && b < 2 * ce;
            const unsigned base = keep ? (unsigned)gb * (unsigned)(M * 8) : 0x80000000u;
            const int k = 2 * (lane + 64 * wb);
            const int pos = k + 4 * (k >> 8);
            v2f T[4][2];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const v4f E = *reinterpret_cast<const v4f *>(Bb + r * A4_QS + pos);
                T[r][0] = v2f{E.x, E.y};
                T[r][1] = v2f{E.z, E.w};
            }
#pragma unroll
            for (int e = 0; e < 2; e++)
#pragma unroll
                for (int r = 1; r < 4; r++) {
                    const float2 u = tw4096[r * (k + e)];
                    T[r][e] = pk_cmul(T[r][e], v2f{u.x, -u.y});
                }
            v2f Yo[4][2];
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const v2f s02 = T[0][e] + T[2][e], d02 = T[0][e] - T[2][e];
                const v2f s13 = T[1][e] + T[3][e], d13 = T[1][e] - T[3][e];
                const v2f jd13 = v2f{-d13.y, d13.x};
                Yo[0][e] = (s02 + s13) * inv;
                Yo[1][e] = (d02 + jd13) * inv;
                Yo[2][e] = (s02 - s13) * inv;
                Yo[3][e] = (d02 - jd13) * inv;
            }
#pragma unroll
            for (int sq = 0; sq < 4; sq++)
                __builtin_amdgcn_raw_buffer_store_b128(v4f{Yo[sq][0].x, Yo[sq][0].y, Yo[sq][1].x, Yo[sq][1].y}, ry,
                                                       base + (unsigned)(k + 1024 * sq) * 8u, 0, 2);
        }
        // the DMA has landed; only the four stores may be in flight
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        lds_barrier_w();   // combine reads done; row c+1 in rb for every wave
    }
}

template <int L>
bool launch_pfb2_an4096(const void *hsub, const void *hist, const void *x, long long nb, int p0, void *Y, hipStream_t st)
{
    constexpr int M = 4096;
    const long long n_in = nb * (M / 2);
    if (n_in * 8 >= (1ll << 31) || nb * (long long)M * 8 >= (1ll << 31)) return false;
    const int cmin = (p0 - 1) >> 1;
    const int cmax = (int)((p0 + nb - 1) >> 1);
    const int rows = cmax - cmin + 1;
    // one workgroup per CU: runs of S rows, about 256 runs (each warms up on
    // the 2m rows before it)
    long long S = ((long long)rows + 255) / 256;
    if (S < 32) S = 32;
    const long long nseg = (rows + S - 1) / S;
    hipLaunchKernelGGL((k_pfb2_an4096<L>), dim3((unsigned)nseg), dim3(1024), 0, st, (const float *)hsub,
                       (const float2 *)hist, (const float2 *)x, (int)n_in, p0, (int)nb, cmin, cmax, (int)S,
                       (float2 *)Y, (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
    return true;
}

// M = 64 / 128 analyzer fused (the two-pass path moved 56 B per input): as
// k_pfb2_an256, with Q = 256 / M column sets per workgroup, each a lane per
// column over its own run of rows (segment blockIdx.x Q + set), and each
// group of 8 rows' 16 blocks per set transformed in registers by R = M / 16
// lanes (fft_small16xR: 16 Q transforms of M points per workgroup, all 256
// lanes).  Every set runs the same number of groups (its stores past its
// rows are dropped), so the barriers stay uniform.
template <int L, int MS>
__global__ __launch_bounds__(256, 2) void k_pfb2_an_small(const float *__restrict__ hsub,
                                                         const float2 *__restrict__ hist,
                                                         const float2 *__restrict__ x, int n_in, int p0, int nb,
                                                         int cmin, int cmax, int S, float2 *__restrict__ Y,
                                                         const float2 *__restrict__ tw4096)
{
    constexpr int M = MS, M2 = M / 2, HL = L * M - M2, NS = 8, NBUF = 17;
    constexpr int Q = 256 / M, R = M / 16, P = FFTS_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 xr[Q * NBUF * M];
    __shared__ __attribute__((aligned(16))) float2 scr[16 * Q * P];
    const int set = threadIdx.x / M, col = threadIdx.x % M;
    float2 *xs = xr + set * (NBUF * M);
    const bool lo = col < M2;
    const int j = lo ? (M2 - 1 - col) : (3 * M2 - 1 - col);
    const int dA = lo ? 0 : 1;
    float ta[L], tb[L];
    {
        const int ia = lo ? j : (j ^ M2), ib = lo ? (j ^ M2) : j;
#pragma unroll
        for (int n = 0; n < L; n++) {
            ta[n] = hsub[ia * L + n];
            tb[n] = hsub[ib * L + n];
        }
    }
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)Y, (short)0, nb * M * 8, 0x00020000);
    const float2 *zero = tw4096 + LQ_TW_N;   // lqrt_zeros(): the table's zero tail
    auto row_sample = [&](int r) -> float2 {
        const int t = r * M + col - p0 * M2;
        return lq_load_hx(hist + HL, x, zero, t, HL, n_in);
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
    auto slot = [](int b) { return ((b % NBUF) + NBUF) % NBUF; };
    // transform phase: transform tg = threadIdx.x / R of set tg / 16 (its block
    // 2 r0 + tg % 16), lane t
    const int tg = threadIdx.x / R, t = threadIdx.x % R;
    const int tset = tg / 16, tb16 = tg % 16;
    const int e = t * (4096 / M);
    const float2 a1 = tw4096[e & 4095], a4 = tw4096[(4 * e) & 4095];
    const float inv = 1.0f / (float)M;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

    const int seg = (int)blockIdx.x * Q + set;
    const int cs = cmin + seg * S;
    int ce = cs + S;
    if (ce > cmax + 1) ce = cmax + 1;
    // the transform lanes' set (another set's rows)
    const int tcs = cmin + ((int)blockIdx.x * Q + tset) * S;
    int tce = tcs + S;
    if (tce > cmax + 1) tce = cmax + 1;
    float2 w[NS], pf[NS];
#pragma unroll
    for (int u = 0; u < NS; u++) w[u] = row_sample(cs - NS + u);
    if (!lo) xs[slot(2 * cs) * M + j] = dot(w, NS - 1, tb);
#pragma unroll
    for (int u = 0; u < NS; u++) pf[u] = row_sample(cs + u);
    for (int g0 = 0; g0 < S; g0 += NS) {
        const int r0 = cs + g0;
#pragma unroll
        for (int u = 0; u < NS; u++) {
            w[u] = pf[u];
            pf[u] = row_sample(r0 + NS + u);
            const int c = r0 + u;
            xs[slot(2 * c + dA) * M + j] = dot(w, u, ta);
            xs[slot(2 * c + dA + 1) * M + j] = dot(w, u, tb);
        }
        lds_barrier_w();
        // blocks 2 r0 .. 2 r0 + 15 of every set are complete
        const int tr0 = tcs + g0;
        const int b = 2 * tr0 + tb16;
        float2 v[16];
        const float2 *B = xr + tset * (NBUF * M) + slot(b) * M;
#pragma unroll
        for (int n = 0; n < 16; n++) v[n] = B[t + R * n];
        fft_small16xR<R, -1>(v, scr + tg * P, a1, a4, t);   // (its barriers also free the ring buffers)
        const int gb = b - p0;
        const bool keep = gb >= 0 && gb < nb && tr0 < tce;
        const unsigned base = keep ? (unsigned)gb * (unsigned)(M * 8) : 0xFFFFF000u;
        // v[u R + q] = X[t (16/R) + u + 16 q]
#pragma unroll
        for (int u = 0; u < 16 / R; u++)
#pragma unroll
            for (int q = 0; q < R; q++) {
                const float2 vv = v[u * R + q];
                const float2 o = make_float2(vv.x * inv, vv.y * inv);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), ry,
                                                      base + (unsigned)(t * (16 / R) + u + 16 * q) * 8u, 0, 0);
            }
    }
}

template <int L, int MS>
bool launch_pfb2_an_small(const void *hsub, const void *hist, const void *x, long long nb, int p0, void *Y,
                          hipStream_t st)
{
    constexpr int M = MS, Q = 256 / M;
    const long long n_in = nb * (M / 2);
    if (n_in * 8 >= (1ll << 31) || nb * (long long)M * 8 >= (1ll << 31)) return false;
    const int cmin = (p0 - 1) >> 1;
    const int cmax = (int)((p0 + nb - 1) >> 1);
    const int rows = cmax - cmin + 1;
    // runs of S rows (a multiple of 8) per set: about 2048 sets on long calls
    // (no short extra run here: every set of a workgroup runs the same
    // number of groups, so an extra workgroup costs a whole run -- measured
    // 0.83 -> 1.07 ms at M = 64, r05zo)
    long long S = ((long long)rows + 2047) / 2048;
    S = (S + 7) / 8 * 8;
    if (S < 32) S = 32;
    const long long nseg = (rows + S - 1) / S;
    const long long nwg = (nseg + Q - 1) / Q;
    hipLaunchKernelGGL((k_pfb2_an_small<L, MS>), dim3((unsigned)nwg), dim3(256), 0, st, (const float *)hsub,
                       (const float2 *)hist, (const float2 *)x, (int)n_in, p0, (int)nb, cmin, cmax, (int)S,
                       (float2 *)Y, (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
    return true;
}

template <int L>
bool launch_pfb2_poly(int M, const void *hsub, const void *hist, const void *x, long long nb, int p0, void *Y,
                      hipStream_t st)
{
    const long long n_in = nb * (M / 2);
    if (n_in * 8 >= (1ll << 31) || nb * (long long)M * 8 >= (1ll << 31)) return false;   // 32-bit buffer offsets
    const int cmin = (p0 - 1) >> 1;                            // floor((p0 - 1) / 2)
    const int cmax = (int)((p0 + nb - 1) >> 1);
    const int rows = cmax - cmin + 1;
    const int nt = M < 256 ? M : 256;
    const int nsl = M / nt;
    // runs of S rows: >= 2048 workgroups when the call is long, and runs of
    // at least 4L rows so the L-1 warm-up rows stay a small overhead
    long long S = ((long long)rows * nsl + 2047) / 2048;
    if (S < 4 * L) S = 4 * L;
    const long long nseg = (rows + S - 1) / S;
    hipLaunchKernelGGL((k_pfb2_poly<L>), dim3((unsigned)(nseg * nsl)), dim3(nt), 0, st, M, nsl, (const float *)hsub,
                       (const float2 *)hist, (const float2 *)x, (int)n_in, p0, (int)nb, cmin, cmax, (int)S,
                       (float2 *)Y, (const float2 *)lqrt_zeros());
    LQ_CHECK_LAUNCH();
    return true;
}

// generic even M (not a power of two): direct O(M^2) DFT, one workgroup per block
__global__ __launch_bounds__(NT) void k_pfb2_an_generic(int M, int m, const float *__restrict__ hsub,
                                                        const float2 *__restrict__ hist,
                                                        const float2 *__restrict__ x, long long nblocks, int p0,
                                                        float2 *__restrict__ Y)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2 *X = reinterpret_cast<float2 *>(smem);
    const int M2 = M / 2, L = 2 * m, HL = 2 * m * M - M2;
    const long long gb = blockIdx.x;
    const long long bt = p0 + gb;
    for (int j = threadIdx.x; j < M; j += NT) {
        const int off = (int)(bt & 1) * M2;
        const int i = ((j - off) % M + M) % M;
        const long long c = (j < M2) ? (bt >> 1) : ((bt - 1) >> 1);
        const int base = (j < M2) ? (M2 - 1 - j) : (3 * M2 - 1 - j);
        const long long t0 = c * M + base - (long long)p0 * M2;
        float2 acc = make_float2(0.f, 0.f);
        for (int n = 0; n < L; n++) {
            const float2 v = ext_load(hist, HL, x, t0 - (long long)n * M);
            acc.x = fmaf(hsub[i * L + n], v.x, acc.x);
            acc.y = fmaf(hsub[i * L + n], v.y, acc.y);
        }
        X[j] = acc;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < M; k += NT) {
        float2 acc = make_float2(0.f, 0.f);
        for (int j = 0; j < M; j++) {
            double s, co;
            sincospi(2.0 * (double)(((long long)j * k) % M) / (double)M, &s, &co);
            acc = cadd(acc, cmul(X[j], make_float2((float)co, (float)s)));
        }
        Y[gb * M + k] = make_float2(acc.x / (float)M, acc.y / (float)M);
    }
}

// ------------------------------------------------------------------ batched FFT
// y[b] = FFT_dir(x[b]) * s1 * s2 (two separate roundings, as the reference
// synthesizer scales twice: firpfbch2.c:303-307); s == 1 skips the multiply.
template <int N, int NB>
__global__ __launch_bounds__(NT) void k_fft_batch(const float2 *__restrict__ x, float2 *__restrict__ y,
                                                  long long batch, int dir, float s1, float s2, int use_s1,
                                                  int use_s2, const float2 *__restrict__ tw)
{
    __shared__ __attribute__((aligned(16))) float2 a[NB * N];
    __shared__ __attribute__((aligned(16))) float2 b[NB * N];
    const long long b0 = (long long)blockIdx.x * NB;
    for (int e = threadIdx.x; e < NB * N; e += NT) {
        const long long gb = b0 + e / N;
        a[e] = gb < batch ? x[b0 * N + e] : make_float2(0.f, 0.f);
    }
    __syncthreads();
    float2 *res = lds_fft<N, NB, NT>(a, b, tw, dir);
    for (int e = threadIdx.x; e < NB * N; e += NT) {
        const long long gb = b0 + e / N;
        if (gb >= batch) continue;
        float2 v = res[e];
        if (use_s1) v = cscale(v, s1);
        if (use_s2) v = cscale(v, s2);
        y[b0 * N + e] = v;
    }
}

// direct DFT for non power-of-two sizes (small M channelizers)
__global__ void k_dft_batch(int N, const float2 *__restrict__ x, float2 *__restrict__ y, long long batch, int dir,
                            float s1, float s2, int use_s1, int use_s2)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float2 *xb = reinterpret_cast<float2 *>(smem); // staged: x may alias y
    const long long gb = blockIdx.x;
    for (int j = threadIdx.x; j < N; j += blockDim.x) xb[j] = x[gb * N + j];
    __syncthreads();
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        float2 acc = make_float2(0.f, 0.f);
        for (int j = 0; j < N; j++) {
            double s, c;
            sincospi(-2.0 * dir * (double)(((long long)j * k) % N) / (double)N, &s, &c);
            acc = cadd(acc, cmul(xb[j], make_float2((float)c, (float)s)));
        }
        if (use_s1) acc = cscale(acc, s1);
        if (use_s2) acc = cscale(acc, s2);
        y[gb * N + k] = acc;
    }
}

// ------------------------------------------------------------------ firpfbch2 synthesizer output
// Z holds [4m-1 history z vectors | nblocks new z vectors], each M long.
__global__ void k_pfb2_syn_out(int M, int m, const float *__restrict__ hsub, const float2 *__restrict__ Z,
                               long long nblocks, int p0, float2 *__restrict__ y)
{
    const int M2 = M / 2, L = 2 * m, HB = 4 * m - 1;
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nblocks * M2) return;
    const long long bl = e / M2;
    const int i = (int)(e - bl * M2);
    const int f = (int)((p0 + bl) & 1);
    const int col = i + f * M2;
    const long long zb = HB + bl; // index of z_b in Z
    float2 acc0 = make_float2(0.f, 0.f), acc1 = make_float2(0.f, 0.f);
    for (int n = 0; n < L; n++) {
        const float h0 = hsub[i * L + n];
        const float h1 = hsub[(i + M2) * L + n];
        const float2 z0 = Z[(zb - 2 * n) * M + col];
        const float2 z1 = Z[(zb - 1 - 2 * n) * M + col];
        acc0.x = fmaf(h0, z0.x, acc0.x);
        acc0.y = fmaf(h0, z0.y, acc0.y);
        acc1.x = fmaf(h1, z1.x, acc1.x);
        acc1.y = fmaf(h1, z1.y, acc1.y);
    }
    y[bl * M2 + i] = cadd(acc0, acc1);
}

// ------------------------------------------------------------------ firpfbch analyzer (X build)
// tap x sample: real taps (crcf) or complex taps (cccf, no conjugation, as dotprod_cccf)
__device__ __forceinline__ float2 pfb_mac(float h, float2 v, float2 a)
{
    return make_float2(fmaf(h, v.x, a.x), fmaf(h, v.y, a.y));
}
__device__ __forceinline__ float2 pfb_mac(float2 h, float2 v, float2 a)
{
    return make_float2(fmaf(h.x, v.x, fmaf(-h.y, v.y, a.x)), fmaf(h.x, v.y, fmaf(h.y, v.x, a.y)));
}

template <typename TC>
__global__ void k_pfb_an_X(int M, int p, const TC *__restrict__ hsub, const float2 *__restrict__ hist,
                           const float2 *__restrict__ x, long long nblocks, float2 *__restrict__ X)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nblocks * M) return;
    const long long b = e / M;
    const int j = (int)(e - b * M);
    const int i = M - 1 - j;
    const int HL = (p - 1) * M;
    float2 acc = make_float2(0.f, 0.f);
    for (int n = 0; n < p; n++) {
        const float2 v = ext_load(hist, HL, x, (b - n) * M + j);
        acc = pfb_mac(hsub[i * p + n], v, acc);
    }
    X[e] = acc;
}

// firpfbch synthesizer output: Z = [p-1 history z | nblocks new z]
template <typename TC>
__global__ void k_pfb_syn_out(int M, int p, const TC *__restrict__ hsub, const float2 *__restrict__ Z,
                              long long nblocks, float2 *__restrict__ y)
{
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nblocks * M) return;
    const long long b = e / M;
    const int i = (int)(e - b * M);
    const long long zb = (p - 1) + b;
    float2 acc = make_float2(0.f, 0.f);
    for (int n = 0; n < p; n++) {
        acc = pfb_mac(hsub[i * p + n], Z[(zb - n) * M + i], acc);
    }
    y[e] = acc;
}

// ---------------------------------------------------------------- run kernels
// One lane per (column, run of RUN consecutive blocks): the column's taps stay
// in registers and a P-deep shift register of the column's history slides
// along the run, so each input is loaded ~(RUN + P - 1)/RUN times instead of
// P times and each tap once per run (the per-element kernels above re-load
// both for every output).
constexpr int RUN = 64;
constexpr int RPF = 4;   // column samples kept in flight by the run kernels

// firpfbch analyzer X (firpfbch.c:346-409): X[b][j] = sum_n h[i*P + n] x[(b-n)M + j], i = M-1-j
template <int P, typename TC>
__global__ __launch_bounds__(256) void k_pfb_an_X_run(int M, const TC *__restrict__ hsub,
                                                      const float2 *__restrict__ hist, const float2 *__restrict__ x,
                                                      long long nblocks, float2 *__restrict__ X)
{
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    const int j = (int)(e % M);
    const long long b0 = (e / M) * RUN;
    if (b0 >= nblocks) return;
    const int i = M - 1 - j, HL = (P - 1) * M;
    TC h[P];
#pragma unroll
    for (int n = 0; n < P; n++) h[n] = hsub[i * P + n];
    float2 w[P];   // w[n] = x[(b - n) M + j]
#pragma unroll
    for (int n = 1; n < P; n++) w[n] = ext_load(hist, HL, x, (b0 - n) * M + j);
    const long long be = b0 + RUN < nblocks ? b0 + RUN : nblocks;
    // the next RPF samples of the column are in flight (clamped indices, no
    // branch): one load latency per RPF blocks instead of per block
    float2 nx[RPF];
#pragma unroll
    for (int d = 0; d < RPF; d++) nx[d] = x[(b0 + d < be ? b0 + d : be - 1) * M + j];
    for (long long b = b0; b < be; b += RPF) {
#pragma unroll
        for (int d = 0; d < RPF; d++) {
            if (b + d >= be) break;
            w[0] = nx[d];
            const long long bn = b + d + RPF;
            nx[d] = x[(bn < be ? bn : be - 1) * M + j];
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll
            for (int n = 0; n < P; n++) acc = pfb_mac(h[n], w[n], acc);
            X[(b + d) * M + j] = acc;
#pragma unroll
            for (int n = P - 1; n > 0; n--) w[n] = w[n - 1];
        }
    }
}

// firpfbch synthesizer output (firpfbch.c:314-336): y[b][i] = sum_n h[i*P + n] Z[(P-1+b-n) M + i]
template <int P, typename TC>
__global__ __launch_bounds__(256) void k_pfb_syn_out_run(int M, const TC *__restrict__ hsub,
                                                         const float2 *__restrict__ Z, long long nblocks,
                                                         float2 *__restrict__ y)
{
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    const int i = (int)(e % M);
    const long long b0 = (e / M) * RUN;
    if (b0 >= nblocks) return;
    TC h[P];
#pragma unroll
    for (int n = 0; n < P; n++) h[n] = hsub[i * P + n];
    float2 w[P];   // w[n] = Z[(P-1+b-n) M + i]
#pragma unroll
    for (int n = 1; n < P; n++) w[n] = Z[(P - 1 + b0 - n) * M + i];
    const long long be = b0 + RUN < nblocks ? b0 + RUN : nblocks;
    float2 nz[RPF];   // next RPF transforms' column samples in flight
#pragma unroll
    for (int d = 0; d < RPF; d++) nz[d] = Z[(P - 1 + (b0 + d < be ? b0 + d : be - 1)) * M + i];
    for (long long b = b0; b < be; b += RPF) {
#pragma unroll
        for (int d = 0; d < RPF; d++) {
            if (b + d >= be) break;
            w[0] = nz[d];
            const long long bn = b + d + RPF;
            nz[d] = Z[(P - 1 + (bn < be ? bn : be - 1)) * M + i];
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll
            for (int n = 0; n < P; n++) acc = pfb_mac(h[n], w[n], acc);
            y[(b + d) * M + i] = acc;
#pragma unroll
            for (int n = P - 1; n > 0; n--) w[n] = w[n - 1];
        }
    }
}

// firpfbch2 synthesizer output (firpfbch2.c:287-335): block b (parity f) uses
// column c = i + f M/2: y = sum_n h0[n] z_{b-2n}[c] + h1[n] z_{b-1-2n}[c].
// The lane keeps 2L-deep histories of both of its columns.
template <int L>
__global__ __launch_bounds__(256) void k_pfb2_syn_out_run(int M, const float *__restrict__ hsub,
                                                          const float2 *__restrict__ Z, long long nblocks, int p0,
                                                          float2 *__restrict__ y)
{
    const int M2 = M / 2, HB = 2 * L - 1;
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    const int i = (int)(e % M2);
    const long long b0 = (e / M2) * RUN;
    if (b0 >= nblocks) return;
    float h0[L], h1[L];
#pragma unroll
    for (int n = 0; n < L; n++) {
        h0[n] = hsub[i * L + n];
        h1[n] = hsub[(i + M2) * L + n];
    }
    float2 wa[2 * L], wb[2 * L];   // columns i and i + M/2; w[k] = z_{b-k}
#pragma unroll
    for (int k = 1; k < 2 * L; k++) {
        wa[k] = Z[(HB + b0 - k) * M + i];
        wb[k] = Z[(HB + b0 - k) * M + i + M2];
    }
    const long long be = b0 + RUN < nblocks ? b0 + RUN : nblocks;
    float2 na[RPF], nb2[RPF];   // next RPF transforms' column samples in flight
#pragma unroll
    for (int d = 0; d < RPF; d++) {
        const long long bc = b0 + d < be ? b0 + d : be - 1;
        na[d] = Z[(HB + bc) * M + i];
        nb2[d] = Z[(HB + bc) * M + i + M2];
    }
    for (long long b = b0; b < be; b += RPF) {
#pragma unroll
        for (int d = 0; d < RPF; d++) {
            if (b + d >= be) break;
            wa[0] = na[d];
            wb[0] = nb2[d];
            const long long bn = b + d + RPF < be ? b + d + RPF : be - 1;
            na[d] = Z[(HB + bn) * M + i];
            nb2[d] = Z[(HB + bn) * M + i + M2];
            const bool f = ((p0 + b + d) & 1) != 0;
            float2 acc0 = make_float2(0.f, 0.f), acc1 = make_float2(0.f, 0.f);
#pragma unroll
            for (int n = 0; n < L; n++) {
                const float2 z0 = f ? wb[2 * n] : wa[2 * n];
                const float2 z1 = f ? wb[2 * n + 1] : wa[2 * n + 1];
                acc0.x = fmaf(h0[n], z0.x, acc0.x);
                acc0.y = fmaf(h0[n], z0.y, acc0.y);
                acc1.x = fmaf(h1[n], z1.x, acc1.x);
                acc1.y = fmaf(h1[n], z1.y, acc1.y);
            }
            y[(b + d) * M2 + i] = cadd(acc0, acc1);
#pragma unroll
            for (int k = 2 * L - 1; k > 0; k--) {
                wa[k] = wa[k - 1];
                wb[k] = wb[k - 1];
            }
        }
    }
}

// firpfbch analyzer, M = 256 R (R = 1, 2), fused like k_pfb2_an256: a lane
// per column j with the column's P taps (h[(M-1-j) + nM]) and a 16-row
// register ring, X of each 16-row group's 16 blocks in LDS, then 16 forward
// M-point transforms in registers and one store of Y (16 B per sample
// instead of the two-pass 48).
template <int P, typename TC, int R>
__global__ __launch_bounds__(256 * R, R == 1 ? 2 : 1) void k_pfb_an_fused(const TC *__restrict__ hsub,
                                                                          const float2 *__restrict__ hist,
                                                                          const float2 *__restrict__ x, int n_in,
                                                                          int nb, int S, float2 *__restrict__ Y,
                                                                          const float2 *__restrict__ tw4096)
{
    constexpr int M = 256 * R, HL = (P - 1) * M, NS = 16;
    constexpr bool TIGHT = R > 1;
    constexpr int PS = FFTR16_LDS<R, TIGHT>();
    __shared__ __attribute__((aligned(16))) float2 xr[NS * M];
    __shared__ __attribute__((aligned(16))) float2 scr[16 * PS];
    const int j = threadIdx.x;
    TC h[P];
#pragma unroll
    for (int n = 0; n < P; n++) h[n] = hsub[(M - 1 - j) * P + n];
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)Y, (short)0, nb * M * 8, 0x00020000);
    const float2 *zero = tw4096 + LQ_TW_N;   // lqrt_zeros(): the table's zero tail
    auto row_sample = [&](int b) -> float2 {
        const int t = b * M + j;
        return lq_load_hx(hist + HL, x, zero, t, HL, n_in);
    };
    const int g = threadIdx.x / (16 * R), t = threadIdx.x % (16 * R);
    const tw16x2 w16 = fftr16_tw<R>(tw4096, t);
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const int cs = (int)blockIdx.x * S;
    const int ce = cs + S < nb ? cs + S : nb;
    float2 w[NS], pf[NS];
#pragma unroll
    for (int u = 0; u < NS; u++) w[u] = row_sample(cs - NS + u);
#pragma unroll
    for (int u = 0; u < NS; u++) pf[u] = row_sample(cs + u);
    for (int r0 = cs; r0 < ce; r0 += NS) {
#pragma unroll
        for (int u = 0; u < NS; u++) {
            w[u] = pf[u];
            pf[u] = row_sample(r0 + NS + u);
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll
            for (int n = 0; n < P; n++) acc = pfb_mac(h[n], w[(u - n) & (NS - 1)], acc);
            xr[u * M + j] = acc;
        }
        lds_barrier_w();
        float2 v[16];
#pragma unroll
        for (int n = 0; n < 16; n++) v[n] = xr[g * M + t + 16 * R * n];
        fft_r16x16xR<R, +1, TIGHT>(v, scr + g * PS, w16, t);
        const int b = r0 + g;
        const unsigned base = b < ce ? (unsigned)b * (unsigned)(M * 8) : 0xFFFFF000u;
#pragma unroll
        for (int sidx = 0; sidx < 16 / R; sidx++)
#pragma unroll
            for (int q = 0; q < R; q++)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v[sidx * R + q]), ry,
                                                      base + (unsigned)(t + 16 * R * sidx + 256 * q) * 8u, 0, 0);
    }
}

template <typename TC>
bool launch_pfb_an_fused(int M, int p, const void *hsub, const void *hist, const void *x, long long nb, void *Y,
                         hipStream_t st)
{
    if ((M != 256 && M != 512) || nb * (long long)M * 8 >= (1ll << 31)) return false;
    long long S = (nb + 1023) / 1024;
    S = (S + 15) / 16 * 16;
    if (S < 32) S = 32;
    const unsigned grid = (unsigned)((nb + S - 1) / S);
#define LQ_PF(PP)                                                                                          \
    case PP:                                                                                               \
        if (M == 256)                                                                                      \
            hipLaunchKernelGGL((k_pfb_an_fused<PP, TC, 1>), dim3(grid), dim3(256), 0, st, (const TC *)hsub, \
                               (const float2 *)hist, (const float2 *)x, (int)(nb * M), (int)nb, (int)S,   \
                               (float2 *)Y, (const float2 *)lqrt_twiddles());                             \
        else                                                                                               \
            hipLaunchKernelGGL((k_pfb_an_fused<PP, TC, 2>), dim3(grid), dim3(512), 0, st, (const TC *)hsub, \
                               (const float2 *)hist, (const float2 *)x, (int)(nb * M), (int)nb, (int)S,   \
                               (float2 *)Y, (const float2 *)lqrt_twiddles());                             \
        LQ_CHECK_LAUNCH();                                                                                 \
        return true;
    switch (p) {
        LQ_PF(2) LQ_PF(4) LQ_PF(6) LQ_PF(8) LQ_PF(10) LQ_PF(12) LQ_PF(14) LQ_PF(16)
    }
#undef LQ_PF
    return false;
}

// firpfbch analyzer, M = 4096 fused (the two-pass path moved 48 B per
// sample): the structure of k_pfb2_an4096 for the critically sampled bank
// (firpfbch.c:262-312).  Lane t owns columns t + 1024 q with their P taps
// h[(M-1-col) + nM]; row b of the input is block b's polyphase row, and a
// group of G = 3 rows fills three block buffers, whose twelve 1024-point
// quarters (columns = r mod 4) waves 0-11 forward-transform (one row per
// group: 0.72 ms per 2^27 samples at m = 4, four waves busy); all 16 waves
// then combine
//     Y[k + 1024 s] = sum_r W_4096^(r k) Q_r[k] (-i)^(r s)
// into 8-byte coalesced stores.  The ring keeps its oldest row in LDS.
template <int P, typename TC, int G = 3>
__global__ __launch_bounds__(1024, 1) void k_pfb_an4096(const TC *__restrict__ hsub, const float2 *__restrict__ hist,
                                                        const float2 *__restrict__ x, int n_in, int nb, int S,
                                                        float2 *__restrict__ Y, const float2 *__restrict__ tw4096)
{
    constexpr int M = 4096, HL = (P - 1) * M, NS = P;
    static_assert(P >= 2, "ring of at least two rows");
    static_assert(G * A4_BSTR * 8 + 4 * 1024 * 8 + 512 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) float2 xr[G * A4_BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw2[64];
    __shared__ __attribute__((aligned(16))) float2 wold[4 * 1024];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 64) tw2[tid] = tw4096[(64 * (tid & 3) * (tid >> 2)) & 4095];   // W_64^{+b r} (forward)
    const float2 a1 = tw4096[(4 * lane) & 4095], a4 = tw4096[(16 * lane) & 4095];
    // column t + 1024 q sits in quarter t & 3 at index (t >> 2) + 256 q
    const int pq = (tid & 3) * A4_QS + (tid >> 2);
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)Y, (short)0, nb * M * 8, 0x00020000);
    const float2 *zero = tw4096 + LQ_TW_N;
    auto row_sample = [&](int b, int col) -> float2 {
        return lq_load_hx(hist + HL, x, zero, b * M + col, HL, n_in);
    };
    // ring of column q: rows (newest - NS + 2 + u) in w[q][u], the oldest in
    // wold (private to the lane); pf: the next group's rows, loaded after the
    // transforms so they never sit beside a transform and the ring
    float2 w[4][NS - 1], pf[G][4], wo[4];
    const int cs = (int)blockIdx.x * S;
    const int ce = cs + S < nb ? cs + S : nb;
#pragma unroll
    for (int q = 0; q < 4; q++) {
#pragma unroll
        for (int u = 0; u < NS - 1; u++) w[q][u] = row_sample(cs - NS + 1 + u, tid + 1024 * q);   // rows cs-P+1 .. cs-1
        wold[q * 1024 + tid] = row_sample(cs - NS + 1, tid + 1024 * q);
#pragma unroll
        for (int g = 0; g < G; g++) pf[g][q] = row_sample(cs + g, tid + 1024 * q);
    }
    __syncthreads();   // tw2 ready
    for (int b0 = cs; b0 < ce; b0 += G) {
#pragma unroll
        for (int g = 0; g < G; g++) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                wo[q] = wold[q * 1024 + tid];   // row b - P + 1
#pragma unroll
                for (int u = 0; u < NS - 2; u++) w[q][u] = w[q][u + 1];
                w[q][NS - 2] = pf[g][q];
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                int o = (M - 1 - (tid + 1024 * q)) * P;
                asm volatile("" : "+v"(o));   // taps re-read each row (L1 / L2 hits), not held across the transforms
                const TC *h = hsub + o;
                float2 acc = make_float2(0.f, 0.f);
#pragma unroll
                for (int n = 0; n < NS; n++) acc = pfb_mac(h[n], n < NS - 1 ? w[q][NS - 2 - n] : wo[q], acc);
                xr[g * A4_BSTR + pq + 256 * q] = acc;
                asm volatile("" ::: "memory");
            }
            // the next row's oldest (row b - P + 2) waits in LDS
#pragma unroll
            for (int q = 0; q < 4; q++) wold[q * 1024 + tid] = w[q][0];
        }
        lds_barrier_w();
        if (wave < 4 * G) {   // block b0 + wave / 4, quarter wave % 4
            float2 *Bq = xr + (wave >> 2) * A4_BSTR + (wave & 3) * A4_QS;
            float2 v[16];
#pragma unroll
            for (int n = 0; n < 16; n++) v[n] = Bq[lane + 64 * n];
            fft1024_wave_rt<+1>(v, Bq, a1, a4, tw2, lane);   // natural order at k + 4 (k >> 8)
        }
        lds_barrier_w();
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int q = 0; q < 4; q++) pf[g][q] = row_sample(b0 + G + g, tid + 1024 * q);
        {
            const int k = tid;   // bin k of each quarter -> outputs k + 1024 s
            const int pos = k + 4 * (k >> 8);
            v2f W[4];
#pragma unroll
            for (int r = 1; r < 4; r++) W[r] = pk(tw4096[r * k]);   // W_4096^(r k), r k < 4096
#pragma unroll
            for (int g = 0; g < G; g++) {
                const int b = b0 + g;
                v2f T[4];
#pragma unroll
                for (int r = 0; r < 4; r++) T[r] = pk(xr[g * A4_BSTR + r * A4_QS + pos]);
#pragma unroll
                for (int r = 1; r < 4; r++) T[r] = pk_cmul(T[r], W[r]);
                const v2f s02 = T[0] + T[2], d02 = T[0] - T[2], s13 = T[1] + T[3], d13 = T[1] - T[3];
                const v2f jd13 = v2f{-d13.y, d13.x};   // i (T1 - T3)
                const v2f Yo[4] = {s02 + s13, d02 - jd13, s02 - s13, d02 + jd13};
                // a block past the run: a base the launch's range (< 2^31) never reaches
                const unsigned base = b < ce ? (unsigned)b * (unsigned)(M * 8) : 0x80000000u;
#pragma unroll
                for (int sq = 0; sq < 4; sq++)
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, Yo[sq]), ry,
                                                          base + (unsigned)(k + 1024 * sq) * 8u, 0, 2);
            }
        }
        lds_barrier_w();   // the combine's reads are done before the next group's writes
    }
}

template <typename TC>
bool launch_pfb_an4096(int p, const void *hsub, const void *hist, const void *x, long long nb, void *Y,
                       hipStream_t st)
{
    constexpr int M = 4096;
    if (nb * (long long)M * 8 >= (1ll << 31)) return false;
    // one workgroup per CU: about 256 runs of S blocks (each warms up on the p - 1 rows before it)
    long long S = (nb + 255) / 256;
    if (S < 32) S = 32;
    const unsigned grid = (unsigned)((nb + S - 1) / S);
#define LQ_P4(PP)                                                                                          \
    case PP:                                                                                               \
        hipLaunchKernelGGL((k_pfb_an4096<PP, TC>), dim3(grid), dim3(1024), 0, st, (const TC *)hsub,        \
                           (const float2 *)hist, (const float2 *)x, (int)(nb * M), (int)nb, (int)S, (float2 *)Y, \
                           (const float2 *)lqrt_twiddles());                                              \
        LQ_CHECK_LAUNCH();                                                                                 \
        return true;
    switch (p) {
        LQ_P4(2) LQ_P4(4) LQ_P4(6) LQ_P4(8)
    }
#undef LQ_P4
    return false;
}

// firpfbch analyzer, M = 64 / 128, fused as k_pfb_an_fused with Q = 256 / M
// column sets per workgroup (each on its own run of blocks; every set runs
// the same number of 16-block groups, stores past its run dropped) and the
// 16 Q forward M-point transforms of a group on R = M / 16 lanes each
// (fft_small16xR)
template <int P, typename TC, int MS>
__global__ __launch_bounds__(256, 2) void k_pfb_an_small(const TC *__restrict__ hsub, const float2 *__restrict__ hist,
                                                        const float2 *__restrict__ x, int n_in, int nb, int S,
                                                        float2 *__restrict__ Y, const float2 *__restrict__ tw4096)
{
    constexpr int M = MS, HL = (P - 1) * M, NS = 16, Q = 256 / M, R = M / 16, PS = FFTS_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 xr[Q * NS * M];
    __shared__ __attribute__((aligned(16))) float2 scr[16 * Q * PS];
    const int set = threadIdx.x / M, j = threadIdx.x % M;
    float2 *xs = xr + set * (NS * M);
    TC h[P];
#pragma unroll
    for (int n = 0; n < P; n++) h[n] = hsub[(M - 1 - j) * P + n];
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)Y, (short)0, nb * M * 8, 0x00020000);
    const float2 *zero = tw4096 + LQ_TW_N;   // lqrt_zeros(): the table's zero tail
    auto row_sample = [&](int b) -> float2 {
        const int t = b * M + j;
        return lq_load_hx(hist + HL, x, zero, t, HL, n_in);
    };
    const int tg = threadIdx.x / R, t = threadIdx.x % R;   // transform tg: set tg / 16, block tg % 16
    const int tset = tg / 16, tb16 = tg % 16;
    const int e = t * (4096 / M);
    const float2 a1 = tw4096[e & 4095], a4 = tw4096[(4 * e) & 4095];
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const int cs = ((int)blockIdx.x * Q + set) * S;
    const int tcs = ((int)blockIdx.x * Q + tset) * S;
    const int tce = tcs + S < nb ? tcs + S : nb;
    float2 w[NS], pf[NS];
#pragma unroll
    for (int u = 0; u < NS; u++) w[u] = row_sample(cs - NS + u);
#pragma unroll
    for (int u = 0; u < NS; u++) pf[u] = row_sample(cs + u);
    for (int g0 = 0; g0 < S; g0 += NS) {
        const int r0 = cs + g0;
#pragma unroll
        for (int u = 0; u < NS; u++) {
            w[u] = pf[u];
            pf[u] = row_sample(r0 + NS + u);
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll
            for (int n = 0; n < P; n++) acc = pfb_mac(h[n], w[(u - n) & (NS - 1)], acc);
            xs[u * M + j] = acc;
        }
        lds_barrier_w();
        float2 v[16];
        const float2 *B = xr + tset * (NS * M) + tb16 * M;
#pragma unroll
        for (int n = 0; n < 16; n++) v[n] = B[t + R * n];
        fft_small16xR<R, +1>(v, scr + tg * PS, a1, a4, t);   // (its barriers also free xr)
        const int b = tcs + g0 + tb16;
        const unsigned base = b < tce ? (unsigned)b * (unsigned)(M * 8) : 0xFFFFF000u;
        // v[u R + q] = X[t (16/R) + u + 16 q]
#pragma unroll
        for (int u = 0; u < 16 / R; u++)
#pragma unroll
            for (int q = 0; q < R; q++)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v[u * R + q]), ry,
                                                      base + (unsigned)(t * (16 / R) + u + 16 * q) * 8u, 0, 0);
    }
}

template <typename TC>
bool launch_pfb_an_small(int M, int p, const void *hsub, const void *hist, const void *x, long long nb, void *Y,
                         hipStream_t st)
{
    if ((M != 64 && M != 128) || nb * (long long)M * 8 >= (1ll << 31)) return false;
    const int Q = 256 / M;
    long long S = (nb + 2047) / 2048;
    S = (S + 15) / 16 * 16;
    if (S < 32) S = 32;
    const long long nseg = (nb + S - 1) / S;
    const unsigned grid = (unsigned)((nseg + Q - 1) / Q);
#define LQ_PF(PP)                                                                                          \
    case PP:                                                                                               \
        if (M == 64)                                                                                       \
            hipLaunchKernelGGL((k_pfb_an_small<PP, TC, 64>), dim3(grid), dim3(256), 0, st, (const TC *)hsub, \
                               (const float2 *)hist, (const float2 *)x, (int)(nb * M), (int)nb, (int)S,   \
                               (float2 *)Y, (const float2 *)lqrt_twiddles());                             \
        else                                                                                               \
            hipLaunchKernelGGL((k_pfb_an_small<PP, TC, 128>), dim3(grid), dim3(256), 0, st, (const TC *)hsub, \
                               (const float2 *)hist, (const float2 *)x, (int)(nb * M), (int)nb, (int)S,   \
                               (float2 *)Y, (const float2 *)lqrt_twiddles());                             \
        LQ_CHECK_LAUNCH();                                                                                 \
        return true;
    switch (p) {
        LQ_PF(2) LQ_PF(4) LQ_PF(6) LQ_PF(8) LQ_PF(10) LQ_PF(12) LQ_PF(14) LQ_PF(16)
    }
#undef LQ_PF
    return false;
}

// firpfbch synthesizer, M = 256 R, fused: per group of 16 blocks, 16
// inverse register transforms of X (z_b = IFFT(X_b)) into LDS, then a lane
// per column i runs y_b[i] = sum_n h[i p + n] z_{b-n}[i] from a 16-deep
// register ring.  A workgroup's run of blocks warms its ring up on the 16
// blocks before it (transformed again, outputs dropped) or, for the call's
// first run, on the object's last p-1 transforms (state); the z of the
// call's last p-1 blocks go to znew for the next call.
template <int P, typename TC, int R>
__global__ __launch_bounds__(256 * R, R == 1 ? 2 : 1) void k_pfb_syn_fused(const TC *__restrict__ hsub,
                                                                           const float2 *__restrict__ state,
                                                                           const float2 *__restrict__ X, int nb,
                                                                           int S, float2 *__restrict__ y,
                                                                           float2 *__restrict__ znew,
                                                                           const float2 *__restrict__ tw4096)
{
    constexpr int M = 256 * R, HB = P - 1, NS = 16;
    constexpr bool TIGHT = R > 1;
    constexpr int PS = FFTR16_LDS<R, TIGHT>();
    __shared__ __attribute__((aligned(16))) float2 zr[NS * M];
    __shared__ __attribute__((aligned(16))) float2 scr[16 * PS];
    const int i = threadIdx.x;
    TC h[P];
#pragma unroll
    for (int n = 0; n < P; n++) h[n] = hsub[i * P + n];
    const int g = threadIdx.x / (16 * R), t = threadIdx.x % (16 * R);
    const tw16x2 w16 = fftr16_tw<R>(tw4096, t);
    const int cs = (int)blockIdx.x * S;
    const int ce = cs + S < nb ? cs + S : nb;
    float2 w[NS];
    int r0 = cs;
    if (cs == 0) {   // z_{-16} .. z_{-1}: the state's last p-1 transforms, zeros before
#pragma unroll
        for (int u = 0; u < NS; u++) {
            const int b = u - NS;
            w[u] = (b >= -HB) ? state[(HB + b) * M + i] : make_float2(0.f, 0.f);
        }
    } else {
        r0 = cs - NS;    // warm-up group: transformed, outputs dropped
    }
    for (; r0 < ce; r0 += NS) {
        {
            const int b = r0 + g;
            float2 v[16];
            const float2 *xb = X + (long long)(b < nb ? b : nb - 1) * M;
#pragma unroll
            for (int n = 0; n < 16; n++) v[n] = xb[t + 16 * R * n];
            fft_r16x16xR<R, -1, TIGHT>(v, scr + g * PS, w16, t);
            float2 *zb = zr + g * M;
#pragma unroll
            for (int sidx = 0; sidx < 16 / R; sidx++)
#pragma unroll
                for (int q = 0; q < R; q++) {
                    const int k = t + 16 * R * sidx + 256 * q;
                    zb[k] = v[sidx * R + q];
                    if (b >= nb - HB && b < nb && b >= cs && b < ce) znew[(b - (nb - HB)) * M + k] = v[sidx * R + q];
                }
        }
        lds_barrier_w();
#pragma unroll
        for (int u = 0; u < NS; u++) {
            w[u] = zr[u * M + i];
            const int b = r0 + u;
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll
            for (int n = 0; n < P; n++) acc = pfb_mac(h[n], w[(u - n) & (NS - 1)], acc);
            if (b >= cs && b < ce) y[(long long)b * M + i] = acc;
        }
        lds_barrier_w();   // zr is rewritten by the next group's transforms
    }
}

template <typename TC>
bool launch_pfb_syn_fused(int M, int p, const void *hsub, const void *state, const void *X, long long nb, void *y,
                          void *znew, hipStream_t st)
{
    if ((M != 256 && M != 512) || p > 16 || nb < p || nb * (long long)M >= (1ll << 31)) return false;
    long long S = (nb + 1023) / 1024;
    S = (S + 15) / 16 * 16;
    if (S < 64) S = 64;
    const unsigned grid = (unsigned)((nb + S - 1) / S);
#define LQ_SF(PP)                                                                                          \
    case PP:                                                                                               \
        if (M == 256)                                                                                      \
            hipLaunchKernelGGL((k_pfb_syn_fused<PP, TC, 1>), dim3(grid), dim3(256), 0, st, (const TC *)hsub, \
                               (const float2 *)state, (const float2 *)X, (int)nb, (int)S, (float2 *)y,     \
                               (float2 *)znew, (const float2 *)lqrt_twiddles());                          \
        else                                                                                               \
            hipLaunchKernelGGL((k_pfb_syn_fused<PP, TC, 2>), dim3(grid), dim3(512), 0, st, (const TC *)hsub, \
                               (const float2 *)state, (const float2 *)X, (int)nb, (int)S, (float2 *)y,     \
                               (float2 *)znew, (const float2 *)lqrt_twiddles());                          \
        LQ_CHECK_LAUNCH();                                                                                 \
        return true;
    switch (p) {
        LQ_SF(2) LQ_SF(4) LQ_SF(6) LQ_SF(8) LQ_SF(10) LQ_SF(12) LQ_SF(14) LQ_SF(16)
    }
#undef LQ_SF
    return false;
}

// firpfbch synthesizer, M = 4096 fused (the two-pass path moved 48 B per
// sample): z_b = IFFT(X_b) by quarters -- waves 0..4G-1 each load the bins
// X_b[4i + r] of one block's quarter r straight from HBM and inverse-
// transform them in registers (fft1024_wave_rt) -- then the radix-4 combine
//     z[k + 1024 s] = sum_r W_4096^-(r k) Q_r[k] i^(r s)
// leaves lane t exactly its own columns t + 1024 s, so the p-tap output
// y_b[col] = sum_n h[col p + n] z_{b-n}[col] (firpfbch.c:314-336) runs from
// a register ring (its oldest entry in LDS across the transforms) with no
// further LDS traffic.  Runs warm up on the blocks before them (transformed
// again, outputs dropped) or, for the call's first run, on the object's last
// p-1 transforms (state); the z of the call's last p-1 blocks go to znew.
// (p = 8: three-block groups spill 18 VGPRs and still beat two-block groups, 0.585 vs 0.615 ms)
template <int P, typename TC, int G = 3>
__global__ __launch_bounds__(1024, 1) void k_pfb_syn4096(const TC *__restrict__ hsub, const float2 *__restrict__ state,
                                                         const float2 *__restrict__ X, int nb, int S,
                                                         float2 *__restrict__ y, float2 *__restrict__ znew,
                                                         const float2 *__restrict__ tw4096)
{
    constexpr int M = 4096, HB = P - 1, NR = P > 2 ? P - 2 : 1;
    constexpr int NW = G * ((HB + G - 1) / G);   // warm-up blocks before a run (whole groups)
    static_assert(P >= 2, "two taps per column at least");
    __shared__ __attribute__((aligned(16))) float2 xr[G * A4_BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw2[64];
    __shared__ __attribute__((aligned(16))) float2 wold[4 * 1024];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 64) {   // W_64^{-b r} (inverse transform)
        const float2 u = tw4096[(64 * (tid & 3) * (tid >> 2)) & 4095];
        tw2[tid] = make_float2(u.x, -u.y);
    }
    const float2 a1 = tw4096[(4 * lane) & 4095], a4 = tw4096[(16 * lane) & 4095];
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)y, (short)0, nb * M * 8, 0x00020000);
    const int cs = (int)blockIdx.x * S;
    const int ce = cs + S < nb ? cs + S : nb;
    // ring of column t + 1024 q before block b: wold = z_{b-P+1}, r[q][u] =
    // z_{b-P+2+u} (u < P-2)
    float2 r[4][NR];
    int b0 = cs;
    if (cs == 0) {   // the state's last p-1 transforms
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int col = tid + 1024 * q;
            wold[q * 1024 + tid] = state[col];
#pragma unroll
            for (int u = 0; u < P - 2; u++) r[q][u] = state[(1 + u) * M + col];
        }
    } else {
        b0 = cs - NW;   // warm-up groups: transformed, outputs dropped
#pragma unroll
        for (int q = 0; q < 4; q++) {
            wold[q * 1024 + tid] = make_float2(0.f, 0.f);
#pragma unroll
            for (int u = 0; u < NR; u++) r[q][u] = make_float2(0.f, 0.f);
        }
    }
    __syncthreads();   // tw2 ready
    for (; b0 < ce; b0 += G) {
        if (wave < 4 * G) {   // block b0 + wave / 4, quarter wave % 4
            const int g = wave >> 2, rq = wave & 3;
            const int b = b0 + g < nb ? b0 + g : nb - 1;
            const float2 *xb = X + (long long)b * M + rq;
            float2 v[16];
#pragma unroll
            for (int n = 0; n < 16; n++) v[n] = xb[4 * (lane + 64 * n)];
            float2 *Bq = xr + g * A4_BSTR + rq * A4_QS;
            fft1024_wave_rt<-1>(v, Bq, a1, a4, tw2, lane);   // natural order at k + 4 (k >> 8)
        }
        lds_barrier_w();
        {
            const int k = tid, pos = k + 4 * (k >> 8);
            v2f W[4];
#pragma unroll
            for (int rr = 1; rr < 4; rr++) {
                const float2 u = tw4096[rr * k];   // W_4096^(r k), r k < 4096
                W[rr] = v2f{u.x, -u.y};
            }
#pragma unroll
            for (int g = 0; g < G; g++) {
                const int b = b0 + g;
                v2f T[4];
#pragma unroll
                for (int rr = 0; rr < 4; rr++) T[rr] = pk(xr[g * A4_BSTR + rr * A4_QS + pos]);
#pragma unroll
                for (int rr = 1; rr < 4; rr++) T[rr] = pk_cmul(T[rr], W[rr]);
                const v2f s02 = T[0] + T[2], d02 = T[0] - T[2], s13 = T[1] + T[3], d13 = T[1] - T[3];
                const v2f jd13 = v2f{-d13.y, d13.x};   // i (T1 - T3)
                const v2f z[4] = {s02 + s13, d02 + jd13, s02 - s13, d02 - jd13};   // columns t + 1024 s
                const bool out = b >= cs && b < ce;
                const unsigned base = out ? (unsigned)b * (unsigned)(M * 8) : 0x80000000u;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int col = tid + 1024 * q;
                    int o = col * P;
                    asm volatile("" : "+v"(o));   // taps re-read per block (L1 / L2 hits)
                    const TC *h = hsub + o;
                    const float2 zo = wold[q * 1024 + tid];
                    float2 acc = pfb_mac(h[0], unpk(z[q]), make_float2(0.f, 0.f));
#pragma unroll
                    for (int n = 1; n < P - 1; n++) acc = pfb_mac(h[n], r[q][P - 2 - n], acc);
                    acc = pfb_mac(h[P - 1], zo, acc);
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, pk(acc)), ry,
                                                          base + (unsigned)col * 8u, 0, 2);
                    if (out && b >= nb - HB) znew[(long long)(b - (nb - HB)) * M + col] = unpk(z[q]);
                    // advance the ring: z_{b-P+2} becomes the LDS-held oldest
                    if constexpr (P > 2) {
                        wold[q * 1024 + tid] = r[q][0];
#pragma unroll
                        for (int u = 0; u < P - 3; u++) r[q][u] = r[q][u + 1];
                        r[q][P - 3] = unpk(z[q]);
                    } else {
                        wold[q * 1024 + tid] = unpk(z[q]);
                    }
                }
            }
        }
        lds_barrier_w();   // the combine's reads are done before the next group's transforms
    }
}

template <typename TC>
bool launch_pfb_syn4096(int p, const void *hsub, const void *state, const void *X, long long nb, void *y, void *znew,
                        hipStream_t st)
{
    constexpr int M = 4096;
    if (nb < p || nb * (long long)M * 8 >= (1ll << 31)) return false;
    long long S = (nb + 255) / 256;
    S = (S + 2) / 3 * 3;
    if (S < 33) S = 33;
    const unsigned grid = (unsigned)((nb + S - 1) / S);
#define LQ_S4(PP)                                                                                          \
    case PP:                                                                                               \
        hipLaunchKernelGGL((k_pfb_syn4096<PP, TC>), dim3(grid), dim3(1024), 0, st, (const TC *)hsub,       \
                           (const float2 *)state, (const float2 *)X, (int)nb, (int)S, (float2 *)y,         \
                           (float2 *)znew, (const float2 *)lqrt_twiddles());                              \
        LQ_CHECK_LAUNCH();                                                                                 \
        return true;
    switch (p) {
        LQ_S4(2) LQ_S4(4) LQ_S4(6) LQ_S4(8)
    }
#undef LQ_S4
    return false;
}

// firpfbch synthesizer, M = 64 / 128, fused as k_pfb_syn_fused with Q = 256
// / M column sets per workgroup on their own runs of blocks, the 16 Q inverse
// transforms of a group on M / 16 lanes each (fft_small16xR).  Every set runs
// the same groups g0 = -16, 0, 16, .. < S relative to its run: the first is
// the warm-up (blocks before the run transformed again, or for the call's
// first run the object's last p-1 transforms, zeros before them).
template <int P, typename TC, int MS>
__global__ __launch_bounds__(256, 2) void k_pfb_syn_small(const TC *__restrict__ hsub,
                                                         const float2 *__restrict__ state,
                                                         const float2 *__restrict__ X, int nb, int S,
                                                         float2 *__restrict__ y, float2 *__restrict__ znew,
                                                         const float2 *__restrict__ tw4096)
{
    constexpr int M = MS, HB = P - 1, NS = 16, Q = 256 / M, R = M / 16, PS = FFTS_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 zr[Q * NS * M];
    __shared__ __attribute__((aligned(16))) float2 scr[16 * Q * PS];
    const int set = threadIdx.x / M, i = threadIdx.x % M;
    TC h[P];
#pragma unroll
    for (int n = 0; n < P; n++) h[n] = hsub[i * P + n];
    const int tg = threadIdx.x / R, t = threadIdx.x % R;   // transform tg: set tg / 16, block tg % 16
    const int tset = tg / 16, tb16 = tg % 16;
    const int e = t * (4096 / M);
    const float2 a1 = tw4096[e & 4095], a4 = tw4096[(4 * e) & 4095];
    const int cs = ((int)blockIdx.x * Q + set) * S;
    const int ce = cs + S < nb ? cs + S : nb;
    const int tcs = ((int)blockIdx.x * Q + tset) * S;
    const int tce = tcs + S < nb ? tcs + S : nb;
    float2 w[NS];
    for (int g0 = -NS; g0 < S; g0 += NS) {
        {
            const int b = tcs + g0 + tb16;
            float2 v[16];
            const float2 *xb = X + (long long)(b < 0 ? 0 : (b < nb ? b : nb - 1)) * M;
#pragma unroll
            for (int n = 0; n < 16; n++) v[n] = xb[t + R * n];
            fft_small16xR<R, -1>(v, scr + tg * PS, a1, a4, t);
            float2 *zb = zr + tset * (NS * M) + tb16 * M;
#pragma unroll
            for (int u = 0; u < 16 / R; u++)
#pragma unroll
                for (int q = 0; q < R; q++) {
                    const int k = t * (16 / R) + u + 16 * q;
                    float2 z = v[u * R + q];
                    if (b < 0) z = (b >= -HB) ? state[(HB + b) * M + k] : make_float2(0.f, 0.f);
                    zb[k] = z;
                    if (b >= nb - HB && b < nb && b >= tcs && b < tce) znew[(b - (nb - HB)) * M + k] = z;
                }
        }
        lds_barrier_w();
#pragma unroll
        for (int u = 0; u < NS; u++) {
            w[u] = zr[set * (NS * M) + u * M + i];
            const int b = cs + g0 + u;
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll
            for (int n = 0; n < P; n++) acc = pfb_mac(h[n], w[(u - n) & (NS - 1)], acc);
            if (b >= cs && b < ce) y[(long long)b * M + i] = acc;
        }
        lds_barrier_w();   // zr is rewritten by the next group's transforms
    }
}

template <typename TC>
bool launch_pfb_syn_small(int M, int p, const void *hsub, const void *state, const void *X, long long nb, void *y,
                          void *znew, hipStream_t st)
{
    if ((M != 64 && M != 128) || p > 16 || nb < p || nb * (long long)M >= (1ll << 31)) return false;
    const int Q = 256 / M;
    long long S = (nb + 2047) / 2048;
    S = (S + 15) / 16 * 16;
    if (S < 64) S = 64;
    const long long nseg = (nb + S - 1) / S;
    const unsigned grid = (unsigned)((nseg + Q - 1) / Q);
#define LQ_SF(PP)                                                                                          \
    case PP:                                                                                               \
        if (M == 64)                                                                                       \
            hipLaunchKernelGGL((k_pfb_syn_small<PP, TC, 64>), dim3(grid), dim3(256), 0, st, (const TC *)hsub, \
                               (const float2 *)state, (const float2 *)X, (int)nb, (int)S, (float2 *)y,     \
                               (float2 *)znew, (const float2 *)lqrt_twiddles());                          \
        else                                                                                               \
            hipLaunchKernelGGL((k_pfb_syn_small<PP, TC, 128>), dim3(grid), dim3(256), 0, st, (const TC *)hsub, \
                               (const float2 *)state, (const float2 *)X, (int)nb, (int)S, (float2 *)y,     \
                               (float2 *)znew, (const float2 *)lqrt_twiddles());                          \
        LQ_CHECK_LAUNCH();                                                                                 \
        return true;
    switch (p) {
        LQ_SF(2) LQ_SF(4) LQ_SF(6) LQ_SF(8) LQ_SF(10) LQ_SF(12) LQ_SF(14) LQ_SF(16)
    }
#undef LQ_SF
    return false;
}

// firpfbch2 synthesizer, M = 256 R, m <= 4, fused the same way: 16 inverse
// transforms per group (scaled 1/M then M/2, as firpfbch2.c:303-307) into
// LDS, then lane i < M/2 keeps 16-deep rings of columns i and i + M/2 and
// emits y_b[i] = sum_n h[i + nM] z_{b-2n}[c] + h[i + M/2 + nM] z_{b-1-2n}[c],
// c = i + f M/2 (f = block parity).
template <int L, int R>
__global__ __launch_bounds__(256 * R, R == 1 ? 2 : 1) void k_pfb2_syn_fused(const float *__restrict__ hsub,
                                                                            const float2 *__restrict__ state,
                                                                            const float2 *__restrict__ X, int nb,
                                                                            int p0, int S, float2 *__restrict__ y,
                                                                            float2 *__restrict__ znew,
                                                                            const float2 *__restrict__ tw4096)
{
    constexpr int M = 256 * R, M2 = M / 2, HB = 2 * L - 1, NS = 16;
    static_assert(2 * L <= NS, "ring too small");
    constexpr bool TIGHT = R > 1;
    constexpr int PS = FFTR16_LDS<R, TIGHT>();
    __shared__ __attribute__((aligned(16))) float2 zr[NS * M];
    __shared__ __attribute__((aligned(16))) float2 scr[16 * PS];
    const int i = threadIdx.x;   // output column (lanes < M/2)
    const bool outl = i < M2;
    float h0[L], h1[L];
#pragma unroll
    for (int n = 0; n < L; n++) {
        h0[n] = outl ? hsub[i * L + n] : 0.f;
        h1[n] = outl ? hsub[(i + M2) * L + n] : 0.f;
    }
    const int g = threadIdx.x / (16 * R), t = threadIdx.x % (16 * R);
    const tw16x2 w16 = fftr16_tw<R>(tw4096, t);
    const float s1 = 1.0f / (float)M, s2 = (float)M2;
    const int cs = (int)blockIdx.x * S;
    const int ce = cs + S < nb ? cs + S : nb;
    float2 wa[NS], wb[NS];
    int r0 = cs;
    if (cs == 0) {
#pragma unroll
        for (int u = 0; u < NS; u++) {
            const int b = u - NS;
            const bool in = b >= -HB && outl;
            wa[u] = in ? state[(HB + b) * M + i] : make_float2(0.f, 0.f);
            wb[u] = in ? state[(HB + b) * M + i + M2] : make_float2(0.f, 0.f);
        }
    } else {
        r0 = cs - NS;
    }
    for (; r0 < ce; r0 += NS) {
        {
            const int b = r0 + g;
            float2 v[16];
            const float2 *xb = X + (long long)(b < nb ? b : nb - 1) * M;
#pragma unroll
            for (int n = 0; n < 16; n++) v[n] = xb[t + 16 * R * n];
            fft_r16x16xR<R, -1, TIGHT>(v, scr + g * PS, w16, t);
            float2 *zb = zr + g * M;
#pragma unroll
            for (int sidx = 0; sidx < 16 / R; sidx++)
#pragma unroll
                for (int q = 0; q < R; q++) {
                    const int k = t + 16 * R * sidx + 256 * q;
                    const float2 z = cscale(cscale(v[sidx * R + q], s1), s2);
                    zb[k] = z;
                    if (b >= nb - HB && b < nb && b >= cs && b < ce) znew[(b - (nb - HB)) * M + k] = z;
                }
        }
        lds_barrier_w();
        if (outl) {
#pragma unroll
            for (int u = 0; u < NS; u++) {
                wa[u] = zr[u * M + i];
                wb[u] = zr[u * M + i + M2];
                const int b = r0 + u;
                const bool f = ((p0 + b) & 1) != 0;
                float2 acc0 = make_float2(0.f, 0.f), acc1 = make_float2(0.f, 0.f);
#pragma unroll
                for (int n = 0; n < L; n++) {
                    const int k0 = (u - 2 * n) & (NS - 1), k1 = (u - 2 * n - 1) & (NS - 1);
                    const float2 z0 = f ? wb[k0] : wa[k0];
                    const float2 z1 = f ? wb[k1] : wa[k1];
                    acc0.x = fmaf(h0[n], z0.x, acc0.x);
                    acc0.y = fmaf(h0[n], z0.y, acc0.y);
                    acc1.x = fmaf(h1[n], z1.x, acc1.x);
                    acc1.y = fmaf(h1[n], z1.y, acc1.y);
                }
                if (b >= cs && b < ce) y[(long long)b * M2 + i] = cadd(acc0, acc1);
            }
        }
        lds_barrier_w();
    }
}

// firpfbch2 synthesizer, M = 4096 fused: the z transforms as in
// k_pfb_syn4096 (quarters of X straight from HBM, radix-4 combine into the
// lane's own columns t + 1024 s, scaled 1/M then M/2 as firpfbch2.c:303-307).
// Output i < M/2 of block b (parity f) is
//     y_b[i] = sum_n h0[n] z_{b-2n}[c] + h1[n] z_{b-1-2n}[c],  c = i + f M/2
// (h0 = h[i + nM], h1 = h[i + M/2 + nM]), so column c only ever feeds the
// outputs of blocks of one parity; a 2L-deep ring of z per column (4 columns
// x 16 x 8 B per lane at m = 4) would not fit, so each column keeps the L
// partial outputs it still feeds instead (transposed form): z_b[c] adds
// h0[j] z_b[c] to the block b + 2j output when b has c's parity (then that
// output is complete and leaves), else h1[j] z_b[c] to block b + 1 + 2j.
template <int L, int G = 3>
__global__ __launch_bounds__(1024, 1) void k_pfb2_syn4096(const float *__restrict__ hsub,
                                                          const float2 *__restrict__ state,
                                                          const float2 *__restrict__ X, int nb, int p0, int S,
                                                          float2 *__restrict__ y, float2 *__restrict__ znew,
                                                          const float2 *__restrict__ tw4096)
{
    constexpr int M = 4096, M2 = 2048, HB = 2 * L - 1;
    constexpr int NW = G * ((HB + G - 1) / G);   // warm-up blocks before a run (whole groups)
    __shared__ __attribute__((aligned(16))) float2 xr[G * A4_BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw2[64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 64) {   // W_64^{-b r} (inverse transform)
        const float2 u = tw4096[(64 * (tid & 3) * (tid >> 2)) & 4095];
        tw2[tid] = make_float2(u.x, -u.y);
    }
    const float2 a1 = tw4096[(4 * lane) & 4095], a4 = tw4096[(16 * lane) & 4095];
    const float s1 = 1.0f / (float)M, s2 = (float)M2;
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc((void *)y, (short)0, nb * M2 * 8, 0x00020000);
    const int cs = (int)blockIdx.x * S;
    const int ce = cs + S < nb ? cs + S : nb;
    // column q = t + 1024 q of this lane: q < 2 feeds even-parity blocks
    // (output i = col), q >= 2 odd ones (output i = col - M/2)
    v2f A[4][L];
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
        for (int j = 0; j < L; j++) A[q][j] = v2f{0.f, 0.f};
    // one z vector (this lane's four columns) of block b into the partial outputs
    auto feed = [&](int b, const v2f (&z)[4], bool emit) {
        const int f = (p0 + b) & 1;
        const bool out = emit && b >= cs && b < ce;
        const unsigned base = out ? (unsigned)b * (unsigned)(M2 * 8) : 0x80000000u;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int fc = q >> 1, i = tid + 1024 * (q & 1);
            // taps h0 (same parity) or h1, re-read per block (L1 / L2 hits)
            int o = (f == fc ? i : i + M2) * L;
            asm volatile("" : "+v"(o));
            const float *h = hsub + o;
#pragma unroll
            for (int j = 0; j < L; j++) A[q][j] = v2f{h[j], h[j]} * z[q] + A[q][j];
            if (f == fc) {
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, A[q][0]), ry, base + (unsigned)i * 8u, 0, 2);
#pragma unroll
                for (int j = 0; j < L - 1; j++) A[q][j] = A[q][j + 1];
                A[q][L - 1] = v2f{0.f, 0.f};
            }
        }
    };
    int b0 = cs;
    if (cs == 0) {   // the state's 2L-1 transforms (blocks -HB .. -1)
        for (int b = -HB; b < 0; b++) {
            v2f z[4];
#pragma unroll
            for (int q = 0; q < 4; q++) z[q] = pk(state[(long long)(HB + b) * M + tid + 1024 * q]);
            feed(b, z, false);
        }
    } else {
        b0 = cs - NW;   // warm-up groups: transformed, outputs dropped
    }
    __syncthreads();   // tw2 ready
    for (; b0 < ce; b0 += G) {
        if (wave < 4 * G) {   // block b0 + wave / 4, quarter wave % 4
            const int g = wave >> 2, rq = wave & 3;
            int b = b0 + g < nb ? b0 + g : nb - 1;
            b = b < 0 ? 0 : b;
            const float2 *xb = X + (long long)b * M + rq;
            float2 v[16];
#pragma unroll
            for (int n = 0; n < 16; n++) v[n] = xb[4 * (lane + 64 * n)];
            float2 *Bq = xr + g * A4_BSTR + rq * A4_QS;
            fft1024_wave_rt<-1>(v, Bq, a1, a4, tw2, lane);   // natural order at k + 4 (k >> 8)
        }
        lds_barrier_w();
        {
            const int k = tid, pos = k + 4 * (k >> 8);
            v2f W[4];
#pragma unroll
            for (int rr = 1; rr < 4; rr++) {
                const float2 u = tw4096[rr * k];   // W_4096^(r k), r k < 4096
                W[rr] = v2f{u.x, -u.y};
            }
#pragma unroll
            for (int g = 0; g < G; g++) {
                const int b = b0 + g;
                v2f T[4];
#pragma unroll
                for (int rr = 0; rr < 4; rr++) T[rr] = pk(xr[g * A4_BSTR + rr * A4_QS + pos]);
#pragma unroll
                for (int rr = 1; rr < 4; rr++) T[rr] = pk_cmul(T[rr], W[rr]);
                const v2f s02 = T[0] + T[2], d02 = T[0] - T[2], s13 = T[1] + T[3], d13 = T[1] - T[3];
                const v2f jd13 = v2f{-d13.y, d13.x};   // i (T1 - T3)
                v2f z[4] = {s02 + s13, d02 + jd13, s02 - s13, d02 - jd13};   // columns t + 1024 s
#pragma unroll
                for (int q = 0; q < 4; q++) z[q] = (z[q] * s1) * s2;
                if (b < ce && b >= 0) {
                    feed(b, z, true);
                    if (b >= cs && b >= nb - HB) {
#pragma unroll
                        for (int q = 0; q < 4; q++) znew[(long long)(b - (nb - HB)) * M + tid + 1024 * q] = unpk(z[q]);
                    }
                }
            }
        }
        lds_barrier_w();   // the combine's reads are done before the next group's transforms
    }
}

template <int L>
bool launch_pfb2_syn4096_l(const void *hsub, const void *state, const void *X, long long nb, int p0, void *y,
                           void *znew, hipStream_t st)
{
    long long S = (nb + 255) / 256;   // about 256 runs (one workgroup per CU), whole groups of three
    S = (S + 2) / 3 * 3;
    if (S < 33) S = 33;
    const unsigned grid = (unsigned)((nb + S - 1) / S);
    hipLaunchKernelGGL((k_pfb2_syn4096<L>), dim3(grid), dim3(1024), 0, st, (const float *)hsub, (const float2 *)state,
                       (const float2 *)X, (int)nb, p0, (int)S, (float2 *)y, (float2 *)znew,
                       (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
    return true;
}

bool launch_pfb2_syn4096(int m, const void *hsub, const void *state, const void *X, long long nb, int p0, void *y,
                         void *znew, hipStream_t st)
{
    if (m < 1 || m > 4 || nb < 4 * m - 1 || nb * 4096ll * 8 >= (1ll << 31)) return false;
    switch (m) {
    case 1: return launch_pfb2_syn4096_l<2>(hsub, state, X, nb, p0, y, znew, st);
    case 2: return launch_pfb2_syn4096_l<4>(hsub, state, X, nb, p0, y, znew, st);
    case 3: return launch_pfb2_syn4096_l<6>(hsub, state, X, nb, p0, y, znew, st);
    default: return launch_pfb2_syn4096_l<8>(hsub, state, X, nb, p0, y, znew, st);
    }
}

bool launch_pfb2_syn_fused(int M, int m, const void *hsub, const void *state, const void *X, long long nb, int p0,
                           void *y, void *znew, hipStream_t st)
{
    if ((M != 256 && M != 512) || m < 1 || m > 4 || nb < 16 || nb * (long long)M >= (1ll << 31)) return false;
    long long S = (nb + 1023) / 1024;
    S = (S + 15) / 16 * 16;
    if (S < 64) S = 64;
    const unsigned grid = (unsigned)((nb + S - 1) / S);
#define LQ_S2(LL)                                                                                          \
    case LL / 2:                                                                                           \
        if (M == 256)                                                                                      \
            hipLaunchKernelGGL((k_pfb2_syn_fused<LL, 1>), dim3(grid), dim3(256), 0, st, (const float *)hsub, \
                               (const float2 *)state, (const float2 *)X, (int)nb, p0, (int)S, (float2 *)y, \
                               (float2 *)znew, (const float2 *)lqrt_twiddles());                          \
        else                                                                                               \
            hipLaunchKernelGGL((k_pfb2_syn_fused<LL, 2>), dim3(grid), dim3(512), 0, st, (const float *)hsub, \
                               (const float2 *)state, (const float2 *)X, (int)nb, p0, (int)S, (float2 *)y, \
                               (float2 *)znew, (const float2 *)lqrt_twiddles());                          \
        LQ_CHECK_LAUNCH();                                                                                 \
        return true;
    switch (m) {
        LQ_S2(2) LQ_S2(4) LQ_S2(6) LQ_S2(8)
    }
#undef LQ_S2
    return false;
}

// dispatch helpers: compile-time ring depths for the common shapes, else the
// per-element kernels
template <typename TC>
bool launch_an_X_run(int M, int p, const void *hsub, const void *hist, const void *x, long long nb, void *X,
                     hipStream_t st)
{
    const long long threads = (long long)M * ((nb + RUN - 1) / RUN);
    const dim3 g((unsigned)((threads + 255) / 256));
#define LQ_AX(PP)                                                                                                 \
    case PP:                                                                                                      \
        hipLaunchKernelGGL((k_pfb_an_X_run<PP, TC>), g, dim3(256), 0, st, M, (const TC *)hsub,                   \
                           (const float2 *)hist, (const float2 *)x, nb, (float2 *)X);                             \
        return true;
    switch (p) {
        LQ_AX(1) LQ_AX(2) LQ_AX(4) LQ_AX(6) LQ_AX(8) LQ_AX(10) LQ_AX(12) LQ_AX(14) LQ_AX(16)
    }
#undef LQ_AX
    return false;
}

template <typename TC>
bool launch_syn_run(int M, int p, const void *hsub, const void *Z, long long nb, void *y, hipStream_t st)
{
    const long long threads = (long long)M * ((nb + RUN - 1) / RUN);
    const dim3 g((unsigned)((threads + 255) / 256));
#define LQ_SY(PP)                                                                                                 \
    case PP:                                                                                                      \
        hipLaunchKernelGGL((k_pfb_syn_out_run<PP, TC>), g, dim3(256), 0, st, M, (const TC *)hsub,                \
                           (const float2 *)Z, nb, (float2 *)y);                                                   \
        return true;
    switch (p) {
        LQ_SY(1) LQ_SY(2) LQ_SY(4) LQ_SY(6) LQ_SY(8) LQ_SY(10) LQ_SY(12) LQ_SY(14) LQ_SY(16)
    }
#undef LQ_SY
    return false;
}

template <int M>
void launch_pfb2_an(int m, const void *hsub, const void *hist, const void *x, long long nblocks, int p0, void *Y,
                    hipStream_t st)
{
    constexpr int NB = M >= 1024 ? 1 : 1024 / M;
    const long long grid = (nblocks + NB - 1) / NB;
    hipLaunchKernelGGL((k_pfb2_an<M, NB>), dim3((unsigned)grid), dim3(NT), 0, st, m, (const float *)hsub,
                       (const float2 *)hist, (const float2 *)x, nblocks, p0, (float2 *)Y,
                       (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}

// batched 1024-point transforms, one wave each (lq_fft1024.h); 4 waves per workgroup
template <int DIR>
__global__ __launch_bounds__(256) void k_fft1024_batch(const float2 *__restrict__ x, float2 *__restrict__ y,
                                                        long long batch, float s1, float s2, int use_s1,
                                                        int use_s2, const float2 *__restrict__ tw4096)
{
    __shared__ __attribute__((aligned(16))) float2 buf[4 * 1088];
    __shared__ __attribute__((aligned(16))) float2 tw1[1024];
    __shared__ __attribute__((aligned(16))) float2 tw2[64];
    f1k_tables<DIR>(tw1, tw2, tw4096);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float2 *B = buf + wave * 1088;
    for (long long b = (long long)blockIdx.x * 4 + wave; b < batch; b += (long long)gridDim.x * 4) {
        float2 v[16];
        const float2 *xb = x + b * 1024;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = xb[lane + 64 * k];
        fft1024_wave<DIR>(v, B, tw1, tw2, lane);
        typedef float v4f __attribute__((ext_vector_type(4)));
        v4f *yb = reinterpret_cast<v4f *>(y + b * 1024);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int o = 2 * (lane + 64 * q);
            v4f val = *reinterpret_cast<const v4f *>(B + o + 4 * (o >> 8));
            if (use_s1) val = val * s1;
            if (use_s2) val = val * s2;
            yb[o >> 1] = val;
        }
        f1k_wave_fence();   // B is reused by the next transform of this wave
    }
}

// batched 4096-point transforms, one 256-thread workgroup each (fft4096_r16);
// the register transform needs ~2 waves/SIMD worth of VGPRs
template <int DIR>
__global__ __launch_bounds__(256, 2) void k_fft4096_batch(const float2 *__restrict__ x, float2 *__restrict__ y,
                                                           long long batch, float s1, float s2, int use_s1,
                                                           int use_s2, const float2 *__restrict__ tw4096)
{
    __shared__ __attribute__((aligned(16))) float2 lds[FFT4096_LDS];
    const int t = threadIdx.x;
    const tw16x2 w16 = fft4096_tw(tw4096, t);
    for (long long b = blockIdx.x; b < batch; b += gridDim.x) {
        float2 v[16];
        const float2 *xb = x + b * 4096;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = xb[t + 256 * k];
        fft4096_r16<DIR>(v, lds, w16, t);
        float2 *yb = y + b * 4096;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            float2 w = v[k];
            if (use_s1) w = cscale(w, s1);
            if (use_s2) w = cscale(w, s2);
            yb[t + 256 * k] = w;
        }
        lds_barrier_w();   // lds is reused by the next transform
    }
}

// batched 8192-point transforms in one pass, one 256-thread workgroup each:
// decimation in time over two 4096-point register transforms, X[j] = E[j] +
// W_8192^j O[j], X[j + 4096] = E[j] - W_8192^j O[j] (E, O: the transforms of
// the even / odd samples).  Thread t loads the pairs (x[2i], x[2i+1]), i = t +
// 256 n, as 16-byte loads, runs fft4096_r16 on each half through the same LDS
// scratch and combines in registers (E[t + 256 k], O[t + 256 k] are its own):
// one read and one write of the data, where the four-step form
// (fft_four_step) makes two of each.  W_8192^(t + 256 k) = W_8192^t W_32^k:
// the first from sincospi in double once per thread, the second constants.
__device__ __constant__ float2 c_w32[16] = {
    {1.000000000f, -0.000000000f},  {0.980785280f, -0.195090322f},  {0.923879533f, -0.382683432f},
    {0.831469612f, -0.555570233f},  {0.707106781f, -0.707106781f},  {0.555570233f, -0.831469612f},
    {0.382683432f, -0.923879533f},  {0.195090322f, -0.980785280f},  {0.000000000f, -1.000000000f},
    {-0.195090322f, -0.980785280f}, {-0.382683432f, -0.923879533f}, {-0.555570233f, -0.831469612f},
    {-0.707106781f, -0.707106781f}, {-0.831469612f, -0.555570233f}, {-0.923879533f, -0.382683432f},
    {-0.980785280f, -0.195090322f}};
template <int DIR, bool A16>
__global__ __launch_bounds__(256, 2) void k_fft8192_batch(const float2 *__restrict__ x, float2 *__restrict__ y,
                                                           long long batch, float s1, float s2, int use_s1,
                                                           int use_s2, const float2 *__restrict__ tw4096)
{
    __shared__ __attribute__((aligned(16))) float2 lds[FFT4096_LDS];
    typedef float v4f __attribute__((ext_vector_type(4)));
    const int t = threadIdx.x;
    const tw16x2 w16 = fft4096_tw(tw4096, t);
    double sn, cs;
    sincospi((double)t / 4096.0, &sn, &cs);
    const float2 wt = make_float2((float)cs, DIR > 0 ? (float)-sn : (float)sn);
    for (long long b = blockIdx.x; b < batch; b += gridDim.x) {
        float2 ve[16], vo[16];
        if constexpr (A16) {
            const v4f *xb = reinterpret_cast<const v4f *>(x + b * 8192);
#pragma unroll
            for (int n = 0; n < 16; n++) {
                const v4f q = xb[t + 256 * n];
                ve[n] = make_float2(q.x, q.y);
                vo[n] = make_float2(q.z, q.w);
            }
        } else {   // x only 8-byte aligned
            const float2 *xb = x + b * 8192;
#pragma unroll
            for (int n = 0; n < 16; n++) {
                ve[n] = xb[2 * (t + 256 * n)];
                vo[n] = xb[2 * (t + 256 * n) + 1];
            }
        }
        fft4096_r16<DIR>(ve, lds, w16, t);
        fft4096_r16<DIR>(vo, lds, w16, t);
        float2 *yb = y + b * 8192;
        float2 wtv = wt;   // through an empty asm: the twiddles are not hoisted out of the loop
        asm volatile("" : "+v"(wtv.x), "+v"(wtv.y));
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const float2 c = c_w32[k];
            const float2 o = cmul(vo[k], cmul(wtv, make_float2(c.x, DIR > 0 ? c.y : -c.y)));
            float2 u0 = cadd(ve[k], o), u1 = csub(ve[k], o);
            if (use_s1) {
                u0 = cscale(u0, s1);
                u1 = cscale(u1, s1);
            }
            if (use_s2) {
                u0 = cscale(u0, s2);
                u1 = cscale(u1, s2);
            }
            yb[t + 256 * k] = u0;
            yb[4096 + t + 256 * k] = u1;
        }
        lds_barrier_w();   // lds is reused by the next transform
    }
}

// batched 16384-point transforms in one pass, one 512-thread workgroup each:
// radix-4 decimation in time over four 4096-point register transforms F_r of
// x[4i + r].  Half h of the workgroup (threads 256 h ..) loads the pairs
// (x[4i + 2h], x[4i + 2h + 1]) and transforms both (F_2h, F_2h+1, each half
// on its own LDS scratch); with G_r = W_16384^(r k) F_r[k], k = t + 256 m,
//   X[k + 4096 q] = P_q + Q_q,  P_q = G_0 + (-j)^q G_1,  Q_q = (-1)^q G_2 + j^q G_3
// (forward; the inverse conjugates), so half 0 forms P, half 1 Q, and each
// hands the other the two it needs (P_2, P_3 / Q_0, Q_1) through the LDS the
// transforms used, eight m at a time (64 KB); half 0 writes X[k], X[k+4096],
// half 1 X[k+8192], X[k+12288].  252 VGPRs: one workgroup per CU.
__device__ __constant__ float2 c_w64[16] = {
    {1.000000000f, -0.000000000f}, {0.995184727f, -0.098017140f}, {0.980785280f, -0.195090322f},
    {0.956940336f, -0.290284677f}, {0.923879533f, -0.382683432f}, {0.881921264f, -0.471396737f},
    {0.831469612f, -0.555570233f}, {0.773010453f, -0.634393284f}, {0.707106781f, -0.707106781f},
    {0.634393284f, -0.773010453f}, {0.555570233f, -0.831469612f}, {0.471396737f, -0.881921264f},
    {0.382683432f, -0.923879533f}, {0.290284677f, -0.956940336f}, {0.195090322f, -0.980785280f},
    {0.098017140f, -0.995184727f}};
constexpr int FFT16K_LDS = 2 * FFT4096_LDS > 8192 ? 2 * FFT4096_LDS : 8192;
template <int DIR, bool A16>
__global__ __launch_bounds__(512, 1) void k_fft16384_batch(const float2 *__restrict__ x, float2 *__restrict__ y,
                                                            long long batch, float s1, float s2, int use_s1,
                                                            int use_s2, const float2 *__restrict__ tw4096)
{
    __shared__ __attribute__((aligned(16))) float2 lds[FFT16K_LDS];
    typedef float v4f __attribute__((ext_vector_type(4)));
    // h is wave-uniform: in a scalar register its branches are scalar
    const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8), t = threadIdx.x & 255;
    const tw16x2 w16 = fft4096_tw(tw4096, t);
    double sn, cs;
    sincospi((double)t / 8192.0, &sn, &cs);
    const float2 wt = make_float2((float)cs, DIR > 0 ? (float)-sn : (float)sn);   // W_16384^t
    // P_q / Q_q of 8 m go to xch[(q' 8 + m') 256 + t], q' = 0, 1 (half 0
    // writes P_2, P_3 at 0, half 1 Q_0, Q_1 at 4096)
    float2 *xch = lds;
    // the next transform's loads are issued right after this one's register
    // transforms, so they are in flight during the exchange and the stores
    // (0.275 -> 0.264 ms per 2^26 points; issued before the transforms, with
    // 64 more VGPRs live through them: 0.292; the same prefetch in the 8192
    // kernel: 0.2105 -> 0.2146, not kept)
    auto load = [&](long long bb, float2 (&a)[16], float2 (&c)[16]) {
        if constexpr (A16) {
            const v4f *xb = reinterpret_cast<const v4f *>(x + bb * 16384 + 2 * h);
#pragma unroll
            for (int n = 0; n < 16; n++) {
                const v4f q = xb[2 * (t + 256 * n)];
                a[n] = make_float2(q.x, q.y);
                c[n] = make_float2(q.z, q.w);
            }
        } else {
            const float2 *xb = x + bb * 16384 + 2 * h;
#pragma unroll
            for (int n = 0; n < 16; n++) {
                a[n] = xb[4 * (t + 256 * n)];
                c[n] = xb[4 * (t + 256 * n) + 1];
            }
        }
    };
    float2 na[16], nb[16];
    if (blockIdx.x < batch) load(blockIdx.x, na, nb);
    for (long long b = blockIdx.x; b < batch; b += gridDim.x) {
        float2 va[16], vb[16];
#pragma unroll
        for (int n = 0; n < 16; n++) {
            va[n] = na[n];
            vb[n] = nb[n];
        }
        float2 *scr = lds + h * FFT4096_LDS;
        fft4096_r16<DIR>(va, scr, w16, t);
        fft4096_r16<DIR>(vb, scr, w16, t);
        if (b + gridDim.x < batch) load(b + gridDim.x, na, nb);
        float2 *yb = y + b * 16384 + 8192 * h;
        // P_q / Q_q of k = t + 256 m: g0, g1 = G_2h, G_2h+1; jg = (-j) g1
        // forward, j g1 inverse.  Half 0: P_0 = g0 + g1, P_1 = g0 + jg,
        // P_2 = g0 - g1, P_3 = g0 - jg; half 1: Q_0 = g0 + g1, Q_1 = -g0 - jg,
        // Q_2 = g0 - g1, Q_3 = -g0 + jg.  sel 0: the two this half sends, 1:
        // the two it keeps (recomputed after the exchange rather than held:
        // 32 VGPRs)
        // wt through an empty asm: the twiddles stay inside the batch loop
        // (hoisted, 48 of them took 96 VGPRs and spilled)
        float2 wtv = wt;
        asm volatile("" : "+v"(wtv.x), "+v"(wtv.y));
        auto pq = [&](int m, int sel, float2 &a, float2 &c) {
            const float2 cw = c_w64[m];
            const float2 w1 = cmul(wtv, make_float2(cw.x, DIR > 0 ? cw.y : -cw.y));   // W^k
            float2 g0, g1;
            if (h == 0) {
                g0 = va[m];
                g1 = cmul(vb[m], w1);
            } else {
                const float2 w2 = cmul(w1, w1);
                g0 = cmul(va[m], w2);
                g1 = cmul(vb[m], cmul(w2, w1));
            }
            const float2 jg = DIR > 0 ? make_float2(g1.y, -g1.x) : make_float2(-g1.y, g1.x);
            const bool first = (h == 0) == (sel == 1);   // P_0, P_1 / Q_0, Q_1
            if (first) {
                a = cadd(g0, g1);
                c = h == 0 ? cadd(g0, jg) : make_float2(-g0.x - jg.x, -g0.y - jg.y);
            } else {
                a = csub(g0, g1);
                c = h == 0 ? csub(g0, jg) : make_float2(-g0.x + jg.x, -g0.y + jg.y);
            }
        };
#pragma unroll
        for (int r = 0; r < 2; r++) {
            lds_barrier_w();   // the transforms' (or the previous round's) LDS reads are done
#pragma unroll
            for (int mm = 0; mm < 8; mm++) {
                float2 a, c;
                pq(8 * r + mm, 0, a, c);
                xch[4096 * h + mm * 256 + t] = a;
                xch[4096 * h + 2048 + mm * 256 + t] = c;
            }
            lds_barrier_w();
#pragma unroll
            for (int mm = 0; mm < 8; mm++) {
                const int k = t + 256 * (8 * r + mm);
                float2 a, c;
                pq(8 * r + mm, 1, a, c);
                float2 u0 = cadd(a, xch[4096 * (1 - h) + mm * 256 + t]);
                float2 u1 = cadd(c, xch[4096 * (1 - h) + 2048 + mm * 256 + t]);
                if (use_s1) {
                    u0 = cscale(u0, s1);
                    u1 = cscale(u1, s1);
                }
                if (use_s2) {
                    u0 = cscale(u0, s2);
                    u1 = cscale(u1, s2);
                }
                yb[k] = u0;
                yb[4096 + k] = u1;
            }
        }
        lds_barrier_w();   // lds is reused by the next transform
    }
}

// batched N = 256 R point transforms (R = 1, 2, 8: 256, 512, 2048 points),
// 16 R threads per transform, 16 / R transforms per 256-thread workgroup,
// register passes (fft_r16x16xR); persistent over the batch
template <int R, int DIR>
__global__ __launch_bounds__(256, 2) void k_fftr16_batch(const float2 *__restrict__ x, float2 *__restrict__ y,
                                                          long long batch, float s1, float s2, int use_s1,
                                                          int use_s2, const float2 *__restrict__ tw4096)
{
    constexpr int T = 16 * R, N = 16 * T, G = 256 / T, P = FFTR16_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 lds[G * P];
    const int g = threadIdx.x / T, t = threadIdx.x % T;
    const tw16x2 w16 = fftr16_tw<R>(tw4096, t);
    for (long long b0 = (long long)blockIdx.x * G; b0 < batch; b0 += (long long)gridDim.x * G) {
        const long long b = b0 + g;
        const bool in = b < batch;
        float2 v[16];
        const float2 *xb = x + (in ? b : 0) * N;
#pragma unroll
        for (int n = 0; n < 16; n++) v[n] = in ? xb[t + T * n] : make_float2(0.f, 0.f);
        fft_r16x16xR<R, DIR>(v, lds + g * P, w16, t);
        if (in) {
            float2 *yb = y + b * N;
#pragma unroll
            for (int s = 0; s < 16 / R; s++)
#pragma unroll
                for (int q = 0; q < R; q++) {
                    float2 w = v[s * R + q];
                    if (use_s1) w = cscale(w, s1);
                    if (use_s2) w = cscale(w, s2);
                    yb[t + T * s + 256 * q] = w;
                }
        }
    }
}

// batched 32 / 64 / 128-point transforms (fft_small16xR): R lanes per
// transform, 256 / R transforms per workgroup, persistent over the batch
template <int R, int DIR>
__global__ __launch_bounds__(256) void k_fftsmall_batch(const float2 *__restrict__ x, float2 *__restrict__ y,
                                                         long long batch, float s1, float s2, int use_s1,
                                                         int use_s2, const float2 *__restrict__ tw4096)
{
    constexpr int N = 16 * R, G = 256 / R, P = FFTS_LDS<R>();
    __shared__ __attribute__((aligned(16))) float2 lds[G * P];
    const int g = threadIdx.x / R, t = threadIdx.x % R;
    const int e = t * (4096 / N);
    const float2 a1 = tw4096[e & 4095], a4 = tw4096[(4 * e) & 4095];
    for (long long b0 = (long long)blockIdx.x * G; b0 < batch; b0 += (long long)gridDim.x * G) {
        const long long b = b0 + g;
        const bool in = b < batch;
        float2 v[16];
        const float2 *xb = x + (in ? b : 0) * N;
#pragma unroll
        for (int n = 0; n < 16; n++) v[n] = in ? xb[t + R * n] : make_float2(0.f, 0.f);
        fft_small16xR<R, DIR>(v, lds + g * P, a1, a4, t);
        if (in) {
            float2 *yb = y + b * N;
#pragma unroll
            for (int u = 0; u < 16 / R; u++)
#pragma unroll
                for (int q = 0; q < R; q++) {
                    float2 w = v[u * R + q];
                    if (use_s1) w = cscale(w, s1);
                    if (use_s2) w = cscale(w, s2);
                    yb[t * (16 / R) + u + 16 * q] = w;
                }
        }
        lds_barrier_w();   // lds is reused by the next batch of transforms
    }
}

template <int R>
void launch_fftsmall(const void *x, void *y, long long batch, int dir, float s1, float s2, int u1, int u2,
                     hipStream_t st)
{
    constexpr int G = 256 / R;
    const long long gb = (batch + G - 1) / G;
    const unsigned grid = (unsigned)(gb < 4096 ? gb : 4096);
    if (dir > 0)
        hipLaunchKernelGGL((k_fftsmall_batch<R, +1>), dim3(grid), dim3(256), 0, st, (const float2 *)x, (float2 *)y,
                           batch, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
    else
        hipLaunchKernelGGL((k_fftsmall_batch<R, -1>), dim3(grid), dim3(256), 0, st, (const float2 *)x, (float2 *)y,
                           batch, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}

template <int R>
void launch_fftr16(const void *x, void *y, long long batch, int dir, float s1, float s2, int u1, int u2,
                   hipStream_t st)
{
    constexpr int G = 16 / R;
    const long long g = (batch + G - 1) / G;
    const unsigned grid = (unsigned)(g < 2048 ? g : 2048);
    if (dir > 0)
        hipLaunchKernelGGL((k_fftr16_batch<R, +1>), dim3(grid), dim3(256), 0, st, (const float2 *)x, (float2 *)y,
                           batch, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
    else
        hipLaunchKernelGGL((k_fftr16_batch<R, -1>), dim3(grid), dim3(256), 0, st, (const float2 *)x, (float2 *)y,
                           batch, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}

template <int N>
void launch_fft_batch(const void *x, void *y, long long batch, int dir, float s1, float s2, int u1, int u2,
                      hipStream_t st)
{
    constexpr int NB = N >= 1024 ? 1 : 1024 / N;
    const long long grid = (batch + NB - 1) / NB;
    hipLaunchKernelGGL((k_fft_batch<N, NB>), dim3((unsigned)grid), dim3(NT), 0, st, (const float2 *)x,
                       (float2 *)y, batch, dir, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
    LQ_CHECK_LAUNCH();
}

int is_pow2(unsigned v) { return v && !(v & (v - 1)); }

void fft_batch_scaled(unsigned n, int dir, const void *x, void *y, long long batch, float s1, float s2, int u1,
                      int u2, hipStream_t st)
{
    if (batch <= 0) return;
    switch (n) {
    case 2: launch_fft_batch<2>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 4: launch_fft_batch<4>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 8: launch_fft_batch<8>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 16: launch_fft_batch<16>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 32: launch_fftsmall<2>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 64: launch_fftsmall<4>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 128: launch_fftsmall<8>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 256: launch_fftr16<1>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 512: launch_fftr16<2>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 1024: {
        const long long g = (batch + 3) / 4;
        const unsigned grid = (unsigned)(g < 4096 ? g : 4096);
        if (dir > 0)
            hipLaunchKernelGGL(k_fft1024_batch<+1>, dim3(grid), dim3(256), 0, st, (const float2 *)x, (float2 *)y,
                               batch, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
        else
            hipLaunchKernelGGL(k_fft1024_batch<-1>, dim3(grid), dim3(256), 0, st, (const float2 *)x, (float2 *)y,
                               batch, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
        LQ_CHECK_LAUNCH();
        return;
    }
    case 2048: launch_fftr16<8>(x, y, batch, dir, s1, s2, u1, u2, st); return;
    case 4096: {
        const unsigned grid = (unsigned)(batch < 2048 ? batch : 2048);
        if (dir > 0)
            hipLaunchKernelGGL(k_fft4096_batch<+1>, dim3(grid), dim3(256), 0, st, (const float2 *)x, (float2 *)y,
                               batch, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
        else
            hipLaunchKernelGGL(k_fft4096_batch<-1>, dim3(grid), dim3(256), 0, st, (const float2 *)x, (float2 *)y,
                               batch, s1, s2, u1, u2, (const float2 *)lqrt_twiddles());
        LQ_CHECK_LAUNCH();
        return;
    }
    case 8192: {
        const unsigned grid = (unsigned)(batch < 2048 ? batch : 2048);
        const bool a16 = ((uintptr_t)x & 15) == 0;
        void (*k)(const float2 *, float2 *, long long, float, float, int, int, const float2 *) =
            dir > 0 ? (a16 ? k_fft8192_batch<+1, true> : k_fft8192_batch<+1, false>)
                    : (a16 ? k_fft8192_batch<-1, true> : k_fft8192_batch<-1, false>);
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, (const float2 *)x, (float2 *)y, batch, s1, s2, u1, u2,
                           (const float2 *)lqrt_twiddles());
        LQ_CHECK_LAUNCH();
        return;
    }
    case 16384: {
        const unsigned grid = (unsigned)(batch < 1024 ? batch : 1024);
        const bool a16 = ((uintptr_t)x & 15) == 0;
        void (*k)(const float2 *, float2 *, long long, float, float, int, int, const float2 *) =
            dir > 0 ? (a16 ? k_fft16384_batch<+1, true> : k_fft16384_batch<+1, false>)
                    : (a16 ? k_fft16384_batch<-1, true> : k_fft16384_batch<-1, false>);
        hipLaunchKernelGGL(k, dim3(grid), dim3(512), 0, st, (const float2 *)x, (float2 *)y, batch, s1, s2, u1, u2,
                           (const float2 *)lqrt_twiddles());
        LQ_CHECK_LAUNCH();
        return;
    }
    default:
        break;
    }
    if (n == 1) {
        hipLaunchKernelGGL(k_dft_batch, dim3((unsigned)batch), dim3(64), 16, st, 1, (const float2 *)x, (float2 *)y,
                           batch, dir, s1, s2, u1, u2);
        LQ_CHECK_LAUNCH();
        return;
    }
    if (n > 8192) {
        fprintf(stderr, "error: liquid-mi355x: non power-of-two transform size %u not supported\n", n);
        exit(1);
    }
    hipLaunchKernelGGL(k_dft_batch, dim3((unsigned)batch), dim3(256), (size_t)n * sizeof(float2), st, (int)n, (const float2 *)x,
                       (float2 *)y, batch, dir, s1, s2, u1, u2);
    LQ_CHECK_LAUNCH();
}

// Diagnostic switches (DESIGN.md (a) history): LQ_PFB2_TWO_PASS /
// LQ_PFB_TWO_PASS in the environment route the fused channelizer sizes
// through the generic two-pass path.  Read once per process.
bool pfb2_two_pass()
{
    static const bool v = getenv("LQ_PFB2_TWO_PASS") != nullptr;
    return v;
}
bool pfb_two_pass()
{
    static const bool v = getenv("LQ_PFB_TWO_PASS") != nullptr;
    return v;
}

} // namespace

extern "C" void lqk_fft_batch(unsigned int n, int dir, const void *x, void *y, unsigned long long batch,
                              void *stream)
{
    fft_batch_scaled(n, dir, x, y, (long long)batch, 1.f, 1.f, 0, 0, (hipStream_t)stream);
}

extern "C" void lqk_fft_batch_scaled(unsigned int n, int dir, const void *x, void *y, unsigned long long batch,
                                     float s1, float s2, void *stream)
{
    fft_batch_scaled(n, dir, x, y, (long long)batch, s1, s2, 1, 1, (hipStream_t)stream);
}

extern "C" void lqk_firpfbch2_analyzer(unsigned int M, unsigned int m, const void *hsub, const void *hist,
                                       const void *x, unsigned long long nblocks, int p0, void *Y, void *stream)
{
    if (nblocks == 0) return;
    hipStream_t st = (hipStream_t)stream;
    const long long nb = (long long)nblocks;
    if (M >= 64 && is_pow2(M) && 2 * m <= 16 && m >= 1) {
        // polyphase pass into Y, then the batched inverse transform in place
        // (each transform kernel reads its whole block before writing it).
        // Calls run in chunks of an even number of blocks whose outputs fit
        // 1 GiB (32-bit buffer offsets); a later chunk's history is the
        // input just before it (a chunk spans far more than 2mM samples).
        const long long CB = (1ll << 27) / M;
        const long long M2 = M / 2, HL = 2ll * m * M - M2;
        for (long long b0 = 0; b0 < nb; b0 += CB) {
            const long long nbc = (nb - b0) < CB ? (nb - b0) : CB;
            const float2 *xc = (const float2 *)x + b0 * M2;
            const void *hc = b0 == 0 ? hist : (const void *)(xc - HL);
            float2 *Yc = (float2 *)Y + b0 * M;
            if ((M == 256 || M == 512) && 2 * m <= 8 && !pfb2_two_pass()) {
                bool f = false;
#define LQ_F(LL)                                                                                           \
    case LL:                                                                                               \
        f = M == 256 ? launch_pfb2_an256<LL, 1>(hsub, hc, xc, nbc, p0, Yc, st)                            \
                     : launch_pfb2_an256<LL, 2>(hsub, hc, xc, nbc, p0, Yc, st);                           \
        break;
                switch (2 * m) {
                    LQ_F(2) LQ_F(4) LQ_F(6) LQ_F(8)
                default: break;
                }
#undef LQ_F
                if (f) continue;
            }
            if (M == 2048 && 2 * m <= 8 && !pfb2_two_pass()) {
                bool f = false;
                switch (2 * m) {
                case 2: f = launch_pfb2_an2048<2>(hsub, hc, xc, nbc, p0, Yc, st); break;
                case 4: f = launch_pfb2_an2048<4>(hsub, hc, xc, nbc, p0, Yc, st); break;
                case 6: f = launch_pfb2_an2048<6>(hsub, hc, xc, nbc, p0, Yc, st); break;
                case 8: f = launch_pfb2_an2048<8>(hsub, hc, xc, nbc, p0, Yc, st); break;
                default: break;
                }
                if (f) continue;
            }
            if (M == 4096 && 2 * m <= 8 && !pfb2_two_pass()) {
                bool f = false;
                switch (2 * m) {
                case 2: f = launch_pfb2_an4096<2>(hsub, hc, xc, nbc, p0, Yc, st); break;
                case 4: f = launch_pfb2_an4096<4>(hsub, hc, xc, nbc, p0, Yc, st); break;
                case 6: f = launch_pfb2_an4096<6>(hsub, hc, xc, nbc, p0, Yc, st); break;
                case 8: f = launch_pfb2_an4096<8>(hsub, hc, xc, nbc, p0, Yc, st); break;
                default: break;
                }
                if (f) continue;
            }
            if ((M == 64 || M == 128) && 2 * m <= 8 && !pfb2_two_pass()) {
                bool f = false;
#define LQ_F(LL)                                                                                           \
    case LL:                                                                                               \
        f = M == 64 ? launch_pfb2_an_small<LL, 64>(hsub, hc, xc, nbc, p0, Yc, st)                          \
                    : launch_pfb2_an_small<LL, 128>(hsub, hc, xc, nbc, p0, Yc, st);                        \
        break;
                switch (2 * m) {
                    LQ_F(2) LQ_F(4) LQ_F(6) LQ_F(8)
                default: break;
                }
#undef LQ_F
                if (f) continue;
            }
            bool ok = false;
            switch (2 * m) {
            case 2: ok = launch_pfb2_poly<2>((int)M, hsub, hc, xc, nbc, p0, Yc, st); break;
            case 4: ok = launch_pfb2_poly<4>((int)M, hsub, hc, xc, nbc, p0, Yc, st); break;
            case 6: ok = launch_pfb2_poly<6>((int)M, hsub, hc, xc, nbc, p0, Yc, st); break;
            case 8: ok = launch_pfb2_poly<8>((int)M, hsub, hc, xc, nbc, p0, Yc, st); break;
            case 10: ok = launch_pfb2_poly<10>((int)M, hsub, hc, xc, nbc, p0, Yc, st); break;
            case 12: ok = launch_pfb2_poly<12>((int)M, hsub, hc, xc, nbc, p0, Yc, st); break;
            case 14: ok = launch_pfb2_poly<14>((int)M, hsub, hc, xc, nbc, p0, Yc, st); break;
            case 16: ok = launch_pfb2_poly<16>((int)M, hsub, hc, xc, nbc, p0, Yc, st); break;
            default: break;
            }
            if (!ok) {
                fprintf(stderr, "error: firpfbch2: polyphase pass rejected a %lld-block chunk\n", nbc);
                exit(1);
            }
            fft_batch_scaled(M, -1, Yc, Yc, nbc, 1.0f / (float)M, 1.0f, 1, 0, st);
        }
        return;
    }
    switch (M) {
    case 2: launch_pfb2_an<2>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 4: launch_pfb2_an<4>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 8: launch_pfb2_an<8>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 16: launch_pfb2_an<16>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 32: launch_pfb2_an<32>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 64: launch_pfb2_an<64>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 128: launch_pfb2_an<128>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 256: launch_pfb2_an<256>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 512: launch_pfb2_an<512>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 1024: launch_pfb2_an<1024>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 2048: launch_pfb2_an<2048>(m, hsub, hist, x, nb, p0, Y, st); return;
    case 4096: launch_pfb2_an<4096>(m, hsub, hist, x, nb, p0, Y, st); return;
    default:
        break;
    }
    const size_t lds = (size_t)M * sizeof(float2);
    if (lds > 64 * 1024) {
        fprintf(stderr, "error: firpfbch2: %u channels not supported on the GPU path\n", M);
        exit(1);
    }
    hipLaunchKernelGGL(k_pfb2_an_generic, dim3((unsigned)nb), dim3(NT), lds, st, (int)M, (int)m,
                       (const float *)hsub, (const float2 *)hist, (const float2 *)x, nb, p0, (float2 *)Y);
    LQ_CHECK_LAUNCH();
}

// state: the previous 4m-1 z vectors (M each); zscratch: (4m-1 + nblocks)*M.
extern "C" void lqk_firpfbch2_synthesizer(unsigned int M, unsigned int m, const void *hsub, void *state,
                                          void *zscratch, const void *X, unsigned long long nblocks, int p0,
                                          void *Y, void *stream)
{
    if (nblocks == 0) return;
    if (lqk_firpfbch2_synthesizer_fast(M, m, hsub, state, X, nblocks, p0, Y, stream)) return;
    hipStream_t st = (hipStream_t)stream;
    const long long HB = 4 * (long long)m - 1;
    float2 *Z = (float2 *)zscratch;
    if (!pfb2_two_pass() && M == 4096 &&
        launch_pfb2_syn4096((int)m, hsub, state, X, (long long)nblocks, p0, Y, Z, st)) {
        LQ_CHECK(hipMemcpyAsync(state, Z, HB * M * sizeof(float2), hipMemcpyDeviceToDevice, st));
        return;
    }
    if (!pfb2_two_pass() &&
        launch_pfb2_syn_fused((int)M, (int)m, hsub, state, X, (long long)nblocks, p0, Y, Z, st)) {
        LQ_CHECK(hipMemcpyAsync(state, Z, HB * M * sizeof(float2), hipMemcpyDeviceToDevice, st));
        return;
    }
    LQ_CHECK(hipMemcpyAsync(Z, state, HB * M * sizeof(float2), hipMemcpyDeviceToDevice, st));
    fft_batch_scaled(M, -1, X, Z + HB * M, (long long)nblocks, 1.0f / (float)M, (float)(M / 2), 1, 1, st);
    const long long tot = (long long)nblocks * (M / 2);
    const long long runs = (long long)(M / 2) * (((long long)nblocks + RUN - 1) / RUN);
    const dim3 gr((unsigned)((runs + 255) / 256));
    if (m == 4)
        hipLaunchKernelGGL(k_pfb2_syn_out_run<8>, gr, dim3(256), 0, st, (int)M, (const float *)hsub,
                           (const float2 *)Z, (long long)nblocks, p0, (float2 *)Y);
    else if (m == 2)
        hipLaunchKernelGGL(k_pfb2_syn_out_run<4>, gr, dim3(256), 0, st, (int)M, (const float *)hsub,
                           (const float2 *)Z, (long long)nblocks, p0, (float2 *)Y);
    else if (m == 3)
        hipLaunchKernelGGL(k_pfb2_syn_out_run<6>, gr, dim3(256), 0, st, (int)M, (const float *)hsub,
                           (const float2 *)Z, (long long)nblocks, p0, (float2 *)Y);
    else
        hipLaunchKernelGGL(k_pfb2_syn_out, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, (int)M, (int)m,
                           (const float *)hsub, (const float2 *)Z, (long long)nblocks, p0, (float2 *)Y);
    LQ_CHECK_LAUNCH();
    // keep the newest HB z vectors as the state for the next call
    LQ_CHECK(hipMemcpyAsync(state, Z + (long long)nblocks * M, HB * M * sizeof(float2), hipMemcpyDeviceToDevice,
                            st));
}

extern "C" void lqk_firpfbch_analyzer(int ctaps, unsigned int M, unsigned int p, const void *hsub, const void *hist,
                                      const void *x, unsigned long long nblocks, void *Y, void *stream)
{
    if (nblocks == 0) return;
    if (lqk_firpfbch_analyzer_fast(ctaps, M, p, hsub, hist, x, nblocks, Y, stream)) return;
    hipStream_t st = (hipStream_t)stream;
    if (!pfb_two_pass() &&
        (ctaps ? launch_pfb_an_fused<float2>((int)M, (int)p, hsub, hist, x, (long long)nblocks, Y, st)
               : launch_pfb_an_fused<float>((int)M, (int)p, hsub, hist, x, (long long)nblocks, Y, st)))
        return;
    if (M == 4096 && !pfb_two_pass() &&
        (ctaps ? launch_pfb_an4096<float2>((int)p, hsub, hist, x, (long long)nblocks, Y, st)
               : launch_pfb_an4096<float>((int)p, hsub, hist, x, (long long)nblocks, Y, st)))
        return;
    if (!pfb_two_pass() &&
        (ctaps ? launch_pfb_an_small<float2>((int)M, (int)p, hsub, hist, x, (long long)nblocks, Y, st)
               : launch_pfb_an_small<float>((int)M, (int)p, hsub, hist, x, (long long)nblocks, Y, st)))
        return;
    const long long tot = (long long)nblocks * M;
    const dim3 grid((unsigned)((tot + 255) / 256));
    // X is formed in Y then transformed in place
    const bool run = ctaps ? launch_an_X_run<float2>((int)M, (int)p, hsub, hist, x, (long long)nblocks, Y, st)
                           : launch_an_X_run<float>((int)M, (int)p, hsub, hist, x, (long long)nblocks, Y, st);
    if (!run && ctaps)
        hipLaunchKernelGGL(k_pfb_an_X<float2>, grid, dim3(256), 0, st, (int)M, (int)p, (const float2 *)hsub,
                           (const float2 *)hist, (const float2 *)x, (long long)nblocks, (float2 *)Y);
    else if (!run)
        hipLaunchKernelGGL(k_pfb_an_X<float>, grid, dim3(256), 0, st, (int)M, (int)p, (const float *)hsub,
                           (const float2 *)hist, (const float2 *)x, (long long)nblocks, (float2 *)Y);
    LQ_CHECK_LAUNCH();
    fft_batch_scaled(M, +1, Y, Y, (long long)nblocks, 1.f, 1.f, 0, 0, st);
}

// state: the previous p-1 z vectors; zscratch: (p-1 + nblocks)*M
extern "C" void lqk_firpfbch_synthesizer(int ctaps, unsigned int M, unsigned int p, const void *hsub, void *state,
                                         void *zscratch, const void *X, unsigned long long nblocks, void *y,
                                         void *stream)
{
    if (nblocks == 0) return;
    if (lqk_firpfbch_synthesizer_fast(ctaps, M, p, hsub, state, X, nblocks, y, stream)) return;
    hipStream_t st = (hipStream_t)stream;
    const long long HB = (long long)p - 1;
    float2 *Z = (float2 *)zscratch;
    // fused M = 256 / 512: the last p-1 transforms land in the scratch, then
    // become the state (every workgroup reads the old state first)
    if (!pfb_two_pass() &&
        (ctaps ? launch_pfb_syn_fused<float2>((int)M, (int)p, hsub, state, X, (long long)nblocks, y, Z, st)
               : launch_pfb_syn_fused<float>((int)M, (int)p, hsub, state, X, (long long)nblocks, y, Z, st))) {
        if (HB > 0) LQ_CHECK(hipMemcpyAsync(state, Z, HB * M * sizeof(float2), hipMemcpyDeviceToDevice, st));
        return;
    }
    if (M == 4096 && !pfb_two_pass() &&
        (ctaps ? launch_pfb_syn4096<float2>((int)p, hsub, state, X, (long long)nblocks, y, Z, st)
               : launch_pfb_syn4096<float>((int)p, hsub, state, X, (long long)nblocks, y, Z, st))) {
        if (HB > 0) LQ_CHECK(hipMemcpyAsync(state, Z, HB * M * sizeof(float2), hipMemcpyDeviceToDevice, st));
        return;
    }
    if (!pfb_two_pass() &&
        (ctaps ? launch_pfb_syn_small<float2>((int)M, (int)p, hsub, state, X, (long long)nblocks, y, Z, st)
               : launch_pfb_syn_small<float>((int)M, (int)p, hsub, state, X, (long long)nblocks, y, Z, st))) {
        if (HB > 0) LQ_CHECK(hipMemcpyAsync(state, Z, HB * M * sizeof(float2), hipMemcpyDeviceToDevice, st));
        return;
    }
    if (HB > 0) LQ_CHECK(hipMemcpyAsync(Z, state, HB * M * sizeof(float2), hipMemcpyDeviceToDevice, st));
    fft_batch_scaled(M, -1, X, Z + HB * M, (long long)nblocks, 1.f, 1.f, 0, 0, st);
    const long long tot = (long long)nblocks * M;
    const dim3 grid((unsigned)((tot + 255) / 256));
    const bool run = ctaps ? launch_syn_run<float2>((int)M, (int)p, hsub, Z, (long long)nblocks, y, st)
                           : launch_syn_run<float>((int)M, (int)p, hsub, Z, (long long)nblocks, y, st);
    if (!run && ctaps)
        hipLaunchKernelGGL(k_pfb_syn_out<float2>, grid, dim3(256), 0, st, (int)M, (int)p, (const float2 *)hsub,
                           (const float2 *)Z, (long long)nblocks, (float2 *)y);
    else if (!run)
        hipLaunchKernelGGL(k_pfb_syn_out<float>, grid, dim3(256), 0, st, (int)M, (int)p, (const float *)hsub,
                           (const float2 *)Z, (long long)nblocks, (float2 *)y);
    LQ_CHECK_LAUNCH();
    if (HB > 0)
        LQ_CHECK(hipMemcpyAsync(state, Z + (long long)nblocks * M, HB * M * sizeof(float2),
                                hipMemcpyDeviceToDevice, st));
}
