// k_resamp4.hip -- resamp_crcf / resamp_cccf for rates 1/4 < r <= npfb with
// a power-of-two filter-bank count (BASELINE configs[4]: r = 1.037, npfb =
// 64, m = 7; msresamp's arbitrary stage runs at r_a in (1/2, 1)).  Four rate
// classes: 1 < r <= 2 (UP), r > 2 (UP, R4), 1/2 < r < 1 (!UP) and
// 1/4 < r <= 1/2 (!UP, DN).
//
// Reference: src/filter/src/resamp.c:245-311 (execute: per input, while
// b < npfb emit y = (1-mu) y_b + mu y_{b+1} and advance the timing), :352-363
// (update_timing_state: tau += 1/r, b = floor(tau npfb), mu = tau npfb - b),
// src/filter/src/firpfb.c:325-345 (bank output y_b(i) = sum_n h[b + n npfb]
// x[i - n]).
//
// For 1 < r < 2 every input emits one or two outputs, so the output sequence
// has a simple serial form: output k is emitted at (tau_k, i_k); then
// tau += 1/r and, when tau reaches 1 - 1/npfb, tau -= 1 and the next input
// begins (host/resamp.c checks the one-or-two property over the whole plan).
// The host tabulates (tau_k, i_k) for every fourth output of the float32
// schedule (the "output plan", periodic: r = 1.037 repeats after 2^20 outputs,
// a 2 MB table read from L2 at 2 B per output), and the kernel replays it
// bit-exactly (a lane steps at most three outputs from the entry at or before
// its first output):
//   * a wave tile is 256 consecutive outputs; lane j owns outputs 4j .. 4j+3,
//     so its replay is four straight-line steps from its own table entry
//     (no per-input loop, no output list) and its four outputs leave as two
//     16-byte non-temporal stores -- each wave instruction writes 1 KB of
//     whole 128-byte lines;
//   * the lane's four outputs lie on inputs i_a .. i_a + 3, so the window
//     W[q] = x[i_a - L + q], q <= L + 3, is read once from LDS into registers,
//     and output s (input i_a + d_s) is sum_q c_s[q - d_s] W[q]: its taps come
//     from a table padded with two zero rows on either side, read at a lane
//     offset, so every window index is a compile-time register index.  With
//     one or two outputs per input d_0 = 0, d_1 <= 1, 1 <= d_2 <= 2,
//     1 <= d_3 <= 3: 15 + 16 + 16 + 17 taps for four outputs;
//   * a tap is c = h_b[p] + mu (h_{b+1}[p] - h_b[p]) -- the (y0, y1)
//     interpolation of resamp.c:292-295 folded into the coefficient -- from
//     one 8-byte LDS read, then one packed FMA on the complex sample.  Bank
//     npfb is the BOUNDARY pair (h_{npfb-1} on the window one input older,
//     h_0; resamp.c:263-279), so both timing states are one dot product;
//   * the tile's input window is loaded a tile ahead into registers and
//     written to the wave's LDS in a transposed order (sample t at
//     (t & 3) * N4 + t / 4), where the lanes' window reads, about 4/r samples
//     apart, fall on distinct banks (r = 1.037: about one 2-way conflict per
//     32-lane group) and the stores on distinct banks.
// Rates r > 2 (R4) take the same step (tau still crosses 1 - 1/npfb at most
// once per output) with any number of outputs per input: d_1, d_2 <= 1,
// d_3 <= 2 (three steps add less than 1.5), no lower bound, so the passes
// run over q in [0, L + {0, 1, 1, 2}] -- the same 15 + 16 + 16 + 17 taps.
// Rates 1/2 < r < 1 (the template's !UP class) run the same pipeline with
// an output every one or two inputs: the step is tau += 1/r, the emitting
// input ends (tau -= 1, exact: tau + 1/r >= 1 > z), and a silent input
// follows when tau is still >= z; so s <= d_s <= 2s, the register window is
// L + 7 samples, the passes run over q in [s, L + 2s] (15 + 16 + 17 + 18 taps
// at L = 14), the tap table carries three zero rows either side, and a tile
// spans up to 517 inputs (transposed with 160 slots per residue class: about
// one 2-way conflict per 32-lane group at every rate in (1/2, 1), from a
// simulation of the lanes' bank pattern).
// Rates 1/4 < r <= 1/2 (DN) extend the !UP step by up to two more silent
// inputs (2 <= 1/r < 4: two to four inputs per output), so 2s <= d_s <= 4s:
// an L + 13 register window, passes over q in [2s, L + 4s] (15 + 17 + 19 +
// 21 taps at L = 14), six zero tap rows either side, a tile spans up to
// L + 1037 inputs (272 slots per residue class), three workgroups per CU up
// to L = 8 and two above (the window registers).
// Taps outside an output's own window are zero, so finite samples there add
// exactly 0; a non-finite sample reaches the outputs whose register window
// (L + 4 samples) holds it -- a superset of the reference's, as for the
// zero-padded tap rows of k_resamp3 (resamp is not tested on non-finite input).
#include <hip/hip_runtime.h>

#include "lq_device.h"
#include "lq_kernels.h"

#include <cstdio>
#include <cstdlib>

namespace {

constexpr int NT4 = 256;       // 4 waves per workgroup; each wave owns its tiles end to end
constexpr int TOUT = 256;      // outputs per wave tile (4 per lane)
// tap reads per group in flight: the next group is issued before the current
// one is consumed (the volatile reads, one at a time, exposed the LDS latency
// per tap: 0.127 -> 0.124 ms at config 5, profiles/r05_ab_experiments.txt)
// (1 < r <= 2, L <= 16 with the two windows in flight; elsewhere the
// grouping's register pressure spilled, and a pass issues its reads one by one)
template <int L, bool UP, int HM>
constexpr int rs4_rg() { return UP && HM == 0 && L <= 16 ? 4 : 1; }
// tile windows in flight per wave: two for 1 < r <= 2 at L <= 16 (0.124 ->
// 0.117 ms at config 5; four workgroups per CU), else one (the second set of
// window registers spills there)
template <int L, bool UP, int HM>
constexpr int rs4_pf() { return UP && HM == 0 && L <= 16 ? 2 : 1; }
// Two rate classes share the kernel (UP = 1 < r <= 2: one or two outputs per
// input; !UP = 1/2 < r < 1: an output every one or two inputs).  Per class:
// slots per residue class of the transposed window (>= TSW / 4)
template <bool UP, bool DN = false>
constexpr int rs4_n4() { return UP ? 88 : (DN ? 272 : 160); }
// resident workgroups per CU: four (<= 128 VGPRs: the register window, 2 NW
// VGPRs, and at 1 < r <= 2 two prefetched tile windows), five at 1/2 < r < 1
// for L <= 4, three for L > 22
template <int L, bool UP, bool DN = false>
constexpr int rs4_blk() { return UP ? 4 : (DN ? (L <= 8 ? 3 : 2) : (L <= 4 ? 5 : (L <= 22 ? 4 : 3))); }

// window samples of a tile: outputs k0 .. k0+255 lie on inputs i_e .. i_e+255
// (UP; i_e: input of the tile's table entry, at most 3 outputs before k0) or
// i_e .. i_e+516 (!UP, two inputs per output at most), and the lane windows
// reach L samples back and 3 (UP) or 6 (!UP) forward
template <int L, bool UP, bool DN = false>
constexpr int rs4_tsw() { return UP ? L + 259 : (DN ? L + 1037 : L + 517); }

template <bool UP, bool DN = false>
constexpr int rs4_pad() { return UP ? 2 : (DN ? 6 : 3); }   // zero tap rows either side

template <int L, bool UP, bool DN = false>
constexpr int rs4_rows() { return L + 1 + 2 * rs4_pad<UP, DN>(); }

// one 8-byte LDS read, volatile: issued as its own ds_read_b64 (2 LDS cycles
// per wave instruction), never paired into a ds_read2_b64 (8 cycles)
__device__ __forceinline__ float2 lds_rd8(const float2 *p)
{
    typedef const volatile unsigned long long __attribute__((address_space(3))) *lp;
    const unsigned long long u = *(lp)(p);
    return __builtin_bit_cast(float2, u);
}

__device__ __forceinline__ void wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int L, int NPC, bool UP, int HM, bool R4 = false, bool DN = false>
__global__ __launch_bounds__(NT4, (HM ? 4 : rs4_blk<L, UP, DN>())) void k_resamp4(lqk_rs4_plan pl, unsigned long long g0,
                                                      unsigned long long K0, int npfb, float del,
                                                      const float2 *__restrict__ taps2,
                                                      const float2 *__restrict__ hist,
                                                      const float2 *__restrict__ x, int n,
                                                      float2 *__restrict__ y, int nout, int smode, lqk_rs4_hb hb,
                                                      lqk_hist_job hj)
{
    lq_hist_job_run<float2>(hj);   // the object's next history (no launch of its own)
    // HM > 0: the half-band interpolator stage (semi-length HM, 2 HM taps on
    // the odd branch) fused behind the resampler.  A tile then computes its
    // 256 resampler outputs starting HALO >= 2 HM - 1 outputs early, so the
    // stage's window for the tile's TS = 256 - HALO new outputs is complete
    // (the HALO outputs are the previous tile's, recomputed: 4.7 % at HM = 6)
    constexpr int HW = 2 * HM;
    constexpr int HALO = HM ? ((HW - 1 + 3) & ~3) : 0;
    constexpr int TS = TOUT - HALO;
    static_assert(HM == 0 || (UP && HALO >= HW && HALO < 64), "fused half-band stage shape");
    constexpr int NR = rs4_rows<L, UP, DN>();
    constexpr int PAD = rs4_pad<UP, DN>();
    constexpr int N4 = rs4_n4<UP, DN>();
    constexpr int LP = (L + 3) & ~1;                 // pair stride of taps2 (host layout)
    constexpr int TSW = rs4_tsw<L, UP, DN>();
    constexpr int NXV = (TSW + 63) / 64;             // window samples per lane
    constexpr int NW = UP ? L + 4 : (DN ? L + 13 : L + 7);   // register window per lane
    constexpr int AMAX = TSW - NW;                   // last lane window start
    constexpr int PF = rs4_pf<L, UP, HM>();
    constexpr int RG = rs4_rg<L, UP, HM>();
    static_assert(TSW <= 4 * N4, "window exceeds the transposed layout");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int RS = NPC ? NPC + 1 : npfb + 1;         // table row stride (== 1 mod 32 for npfb >= 32)
    float2 *tt = reinterpret_cast<float2 *>(smem);   // tt[(p + PAD) RS + b] = (h_b[p], h_{b+1}[p] - h_b[p])
    const int tbytes = (NR * RS * 8 + 15) & ~15;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int e = tid; e < NR * RS; e += NT4) {
        const int rr = e / RS, b = e - rr * RS, p = rr - PAD;
        float2 v = make_float2(0.0f, 0.0f);
        if (p >= 0 && p <= L && b <= npfb) {
            const float2 t = taps2[b * LP + p];
            v = make_float2(t.x, t.y - t.x);
        }
        tt[e] = v;
    }
    __syncthreads();   // the only workgroup barrier

    const int ntiles = (nout + TS - 1) / TS;
    const int GW = (int)gridDim.x * (NT4 / 64), gw = (int)blockIdx.x * (NT4 / 64) + wave;
    if (gw >= ntiles) return;
    float2 *win = reinterpret_cast<float2 *>(smem + tbytes) + wave * (4 * N4);

    const __amdgpu_buffer_rsrc_t ry =
        __builtin_amdgcn_make_buffer_rsrc((void *)y, (short)0, nout * (HM ? 16 : 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t rt =
        __builtin_amdgcn_make_buffer_rsrc((void *)pl.tab, (short)0, (int)(pl.ntab * 8), 0x00020000);
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    auto ld8 = [&](__amdgpu_buffer_rsrc_t r, int e) -> float2 {
        const unsigned off = e < 0 ? 0xFFFFFFF0u : (unsigned)e * 8u;
        return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
    };

    // Table entries.  The table holds the state at outputs 0, 4, 8, ... below
    // pre (npre entries), then at pre, pre + 4, ... within one period of QT
    // outputs (PT inputs; QT >= 256, so a 256-output tile wraps at most
    // once).  Lane j of a tile (first output k0) reads the entry at or
    // before its output k = k0 + 4j and steps `skip` = 0..3 outputs from it.
    // A wave walks its tiles GW apart, so the tile's periodic position
    // (r0 = (k0 - pre) mod QT, q0 periods) is stepped by the constant
    // (GW 256) mod QT on the scalar unit instead of divided per tile.  The
    // entry's input index becomes call-relative only when it is used
    // (i = entry word + off), so nothing waits on the load.
    struct Ent {
        float2 raw;   // (tau, plan input as bits)
        int off;      // + (periods) PT - g0, modulo 2^32
        int skip;     // outputs from the entry to the lane's first output
    };
    struct Cur {
        long long k0;   // negative: the halo of a stream's first tile (no outputs there)
        unsigned long long r0, q0;
        bool per;
    };
    const unsigned long long STEP = (unsigned long long)GW * TS;
    unsigned long long dQ = 0, dR = 0;
    if (pl.pre != ~0ull) {
        dQ = STEP / pl.QT;
        dR = STEP - dQ * pl.QT;
    }
    auto cur_fix = [&](Cur &c) {
        c.per = c.k0 >= 0 && (unsigned long long)c.k0 >= pl.pre;
        if (c.per) {
            const unsigned long long dt = (unsigned long long)c.k0 - pl.pre;
            c.q0 = dt / pl.QT;
            c.r0 = dt - c.q0 * pl.QT;
        }
    };
    auto cur_next = [&](Cur &c) {
        c.k0 += (long long)STEP;
        if (c.per) {
            c.r0 += dR;
            c.q0 += dQ;
            if (c.r0 >= pl.QT) {
                c.r0 -= pl.QT;
                c.q0++;
            }
        } else {
            cur_fix(c);
        }
    };
    auto entry = [&](int tile, const Cur &c) -> Ent {
        const long long ks = c.k0 + 4ll * lane;
        if (tile >= ntiles || ks < 0) return Ent{make_float2(0.0f, 0.0f), -(int)(unsigned)g0, 0};
        const unsigned long long k = (unsigned long long)ks;
        unsigned long long idx;
        unsigned r4;                               // position whose low bits are the skip
        int off = -(int)(unsigned)g0;
        if (c.per) {
            unsigned long long r = c.r0 + 4ull * (unsigned)lane;
            const bool w = r >= pl.QT;
            r -= w ? pl.QT : 0ull;
            idx = pl.npre + (r >> 2);
            r4 = (unsigned)r;
            off = (int)(unsigned)(c.q0 * pl.PT - g0) + (w ? (int)(unsigned)pl.PT : 0);
        } else if (k < pl.pre) {
            idx = k >> 2;
            r4 = (unsigned)k;
        } else {                                   // k - pre < 256 <= QT: the first period
            const unsigned long long r = k - pl.pre;
            idx = pl.npre + (r >> 2);
            r4 = (unsigned)r;
        }
        return Ent{ld8(rt, idx < pl.ntab ? (int)idx : -1), off, (int)(r4 & 3u)};
    };
    auto ent_i = [](const Ent &e) { return (int)__float_as_uint(e.raw.y) + e.off; };
    // prefetched window of a tile: window sample t is input ws + t,
    // ws = (the tile's lane-0 entry input) - L.  Both forms issue NXV loads
    // into the same registers (so the loop's wait counts stay static).
    // Samples past the call's last input are never weighted (the evaluation
    // zeroes window samples outside an output's own window).
    struct Win {
        float2 v[NXV];
    };
    auto fetch = [&](int tile, int ws, Win &w) {
        const bool live = tile < ntiles;
        if (ws >= 0) {   // (wave-uniform) the usual case: a descriptor based at x[ws], constant lane offsets
            const long long rem = (long long)n - ws;
            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(x + ws), (short)0, live && rem > 0 ? (int)(rem * 8) : 0, 0x00020000);
#pragma unroll
            for (int u = 0; u < NXV; u++)
                w.v[u] = ld8(r, lane + 64 * u < TSW ? lane + 64 * u : -1);
        } else {         // the call's first tile(s): inputs before the call come from the history
#pragma unroll
            for (int u = 0; u < NXV; u++) {
                const int idx = ws + lane + 64 * u;
                const float2 *p = idx < 0 ? hist + (L + (idx < -L ? -L : idx)) : (idx < n ? x + idx : hist);
                w.v[u] = *p;
            }
        }
    };

    const float fnpfb = (float)npfb, z = 1.0f - 1.0f / fnpfb;
    auto put_window = [&](const Win &w) {   // the window into the wave's LDS, transposed
        float2 *wp = win + (lane & 3) * N4 + (lane >> 2);
#pragma unroll
        for (int u = 0; u < NXV; u++)
            if (lane + 64 * u < TSW) wp[16 * u] = w.v[u];
    };
    // Pipeline per wave: while tile t is evaluated, the window of tile t+1
    // and the table entries of tile t+2 are in flight; after the evaluation
    // one wait covers both (and the stores of tile t-1), window t+1 goes to
    // LDS, tile t's outputs are stored, and the loads for t+2 / t+3 issue.
    Cur cc;
    cc.k0 = (long long)K0 + (long long)gw * TS - HALO;
    cur_fix(cc);
    Ent ec = entry(gw, cc);
    cur_next(cc);
    Ent en = entry(gw + GW, cc);
    cur_next(cc);
    Ent enn = entry(gw + 2 * GW, cc);
    cur_next(cc);
    Win wa, wb;
    fetch(gw, __builtin_amdgcn_readfirstlane(ent_i(ec)) - L, wa);
    put_window(wa);
    fetch(gw + GW, __builtin_amdgcn_readfirstlane(ent_i(en)) - L, wa);
    Ent e3;
    if constexpr (PF == 2) {   // a second window in flight
        fetch(gw + 2 * GW, __builtin_amdgcn_readfirstlane(ent_i(enn)) - L, wb);
        e3 = entry(gw + 3 * GW, cc);
        cur_next(cc);
    }

    const float2 *hbh = (const float2 *)hb.hist;
    // one tile; wbuf holds the window of tile + GW and receives the window of
    // tile + (PF + 1) GW
    auto body = [&](const int tile, Win &wbuf) {
        // replay: the lane's entry stepped `skip` outputs, then its four
        // outputs (bank, mu, input offset d)
        const int skip = ec.skip;
        const int i_e = __builtin_amdgcn_readfirstlane(ent_i(ec));   // input of the lane-0 entry
        float tau = ec.raw.x;
        int ii = ent_i(ec);
        auto step = [&]() {
#pragma clang fp contract(off)
            tau = tau + del;
            if (!UP) {   // the emitting input ends (tau + del >= 1 > z)
                tau = tau - 1.0f;
                ii++;
            }
            if (!(tau < z)) {
                tau = tau - 1.0f;
                ii++;
            }
            if constexpr (DN) {   // 2 <= del < 4: up to two more silent inputs
#pragma unroll
                for (int e = 0; e < 2; e++)
                    if (!(tau < z)) {
                        tau = tau - 1.0f;
                        ii++;
                    }
            }
        };
#pragma unroll
        for (int s = 0; s < 3; s++)
            if (s < skip) step();
        const int ia = ii;
        int bk[4], dd[4];
        float mu[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
#pragma clang fp contract(off)
            const float bf = tau * fnpfb;
            const float fb = __builtin_floorf(bf);
            bk[s] = tau < 0.0f ? npfb : (int)fb;
            mu[s] = bf - fb;
            dd[s] = ii - ia;
            if (s < 3) step();
        }
        // lane window W[q] = x[ia - L + q] = window sample a + q
        int a = ia - i_e;
        a = a < 0 ? 0 : (a > AMAX ? AMAX : a);   // lanes past the call's outputs
        wave_fence();   // the window is in LDS
        v2f W[NW];
        {
            const float2 *wb[4];
#pragma unroll
            for (int c = 0; c < 4; c++) wb[c] = win + ((a + c) & 3) * N4 + ((a + c) >> 2);
#pragma unroll
            for (int q = 0; q < NW; q++) W[q] = pk(lds_rd8(wb[q & 3] + (q >> 2)));
        }
        // four outputs: pass s over q in [lo, hi] (UP: d_0 = 0, d_1 <= 1,
        // 1 <= d_2 <= 2, 1 <= d_3 <= 3; R4: 0 <= d_s <= {0, 1, 1, 2}; !UP:
        // s <= d_s <= 2s)
        v2f acc[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            constexpr int LO[4] = {0, 0, 1, 1}, H4[4] = {0, 1, 1, 2};
            const int lo = UP ? (R4 ? 0 : LO[s]) : (DN ? 2 * s : s),
                      hi = UP ? (R4 ? L + H4[s] : L + s) : (DN ? L + 4 * s : L + 2 * s);
            const float2 *tb = tt + (PAD - dd[s]) * RS + bk[s];
            const float m = mu[s];
            v2f sacc = {0.0f, 0.0f};
            // tap reads in groups of RG, the next group issued before the
            // current one is consumed (one read at a time exposed the LDS
            // latency per tap: the volatile reads are never hoisted)
            if constexpr (RG == 1) {
#pragma unroll
                for (int q = lo; q <= hi; q++) {
                    const float2 t = lds_rd8(tb + q * RS);
                    const float cf = __builtin_fmaf(m, t.y, t.x);
                    sacc = v2f{cf, cf} * W[q] + sacc;
                }
            } else {
            float2 tg[2][RG];
#pragma unroll
            for (int g = 0; g < RG; g++)
                if (lo + g <= hi) tg[0][g] = lds_rd8(tb + (lo + g) * RS);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q0 = lo, c = 0; q0 <= hi; q0 += RG, c ^= 1) {
#pragma unroll
                for (int g = 0; g < RG; g++)
                    if (q0 + RG + g <= hi) tg[c ^ 1][g] = lds_rd8(tb + (q0 + RG + g) * RS);
                __builtin_amdgcn_sched_barrier(0);   // the group's reads stay ahead of the arithmetic
#pragma unroll
                for (int g = 0; g < RG; g++) {
                    if (q0 + g > hi) break;
                    const float2 t = tg[c][g];
                    const float cf = __builtin_fmaf(m, t.y, t.x);
                    sacc = v2f{cf, cf} * W[q0 + g] + sacc;
                }
            }
            }
            // the pass completes here (an empty asm on the result): without
            // it the compiler hoists all 64 tap reads ahead of the arithmetic
            // and spills them
            asm volatile("" : "+v"(sacc));
            acc[s] = sacc;
        }
        const int ko = tile * TS - HALO + 4 * lane;   // call output of acc[0]
        if constexpr (HM > 0) {
            // the half-band stage (resamp2.c:345-360 per resampler output,
            // msresamp.c:289-300): outputs before the call come from its window
            if (tile == 0) {
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const int k = ko + s;
                    if (k < 0) acc[s] = k >= -HW ? pk(hbh[HW + k]) : v2f{0.0f, 0.0f};
                }
            }
            if (tile == ntiles - 1) {
                // the stage's windows after the call: u[nout - HW .. nout-1],
                // all in the call's last tile (HALO >= HW), from history where k < 0
                float2 *h0 = (float2 *)hb.hist_new0, *h1 = (float2 *)hb.hist_new1;
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    const int k = ko + s;
                    if (k >= nout - HW && k < nout) {
                        h0[HW - nout + k] = make_float2(acc[s].x, acc[s].y);
                        h1[HW - nout + k] = make_float2(acc[s].x, acc[s].y);
                    }
                }
            }
            // u[t] (tile output t = 4 lane + s) through the wave's LDS; lane j
            // then evaluates the stage at t = j + 64 s, so its two outputs per
            // t leave as one 16-byte store and each store instruction writes
            // 1 KB contiguous
            wave_fence();
            {
                float4 *u4 = reinterpret_cast<float4 *>(win);
                u4[2 * lane] = make_float4(acc[0].x, acc[0].y, acc[1].x, acc[1].y);
                u4[2 * lane + 1] = make_float4(acc[2].x, acc[2].y, acc[3].x, acc[3].y);
            }
            wave_fence();
            // then per t: the odd-tap dot product and the delay sample, and
            // the two outputs 2k, 2k+1 of resampler output k = tile TS + t -
            // HALO as one 16-byte store (the halo's t < HALO store nothing)
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const float2 *ub = win + lane + 64 * s - (HW - 1);   // u[t - (HW-1) + q]
                v2f a = {0.0f, 0.0f}, d = {0.0f, 0.0f};
#pragma unroll
                for (int j = 0; j < HW; j++) {   // the odd-tap branch, in the order of k_resamp2
                    const v2f v = pk(lds_rd8(ub + j));
                    const float h = hb.h1[j];
                    a = v2f{h, h} * v + a;
                    if (j == HM - 1) d = v;   // the delay branch u[t - m]
                }
                asm volatile("" : "+v"(a));   // the pass completes here (no hoisted reads)
                const int t = lane + 64 * s, k = tile * TS + t - HALO;
                if (t >= HALO && k < nout) {
                    if (smode) {
                        u32x4 v;
                        v.x = __float_as_uint(d.x);
                        v.y = __float_as_uint(d.y);
                        v.z = __float_as_uint(a.x);
                        v.w = __float_as_uint(a.y);
                        __builtin_amdgcn_raw_buffer_store_b128(v, ry, (unsigned)k * 16u, 0, 2);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, d), ry, (unsigned)k * 16u, 0, 2);
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, a), ry,
                                                              (unsigned)k * 16u + 8u, 0, 2);
                    }
                }
            }
        }
        // the next tile's window into LDS (this tile's window reads are done)
        wave_fence();
        put_window(wbuf);
        const int ws2 = __builtin_amdgcn_readfirstlane(ent_i(PF == 2 ? e3 : enn)) - L;   // the window to fetch
        if constexpr (HM == 0) {
            // stores: outputs tile*256 + 4 lane + s, two 16-byte stores per lane
            u32x4 s01, s23;
            s01.x = __float_as_uint(acc[0].x);
            s01.y = __float_as_uint(acc[0].y);
            s01.z = __float_as_uint(acc[1].x);
            s01.w = __float_as_uint(acc[1].y);
            s23.x = __float_as_uint(acc[2].x);
            s23.y = __float_as_uint(acc[2].y);
            s23.z = __float_as_uint(acc[3].x);
            s23.w = __float_as_uint(acc[3].y);
            if (smode == 2 && tile * TOUT + TOUT <= nout) {
                // whole 128-byte lines per store instruction: lanes j and j ^ 4
                // (quads A, B of an 8-lane group; outputs 32 g .. 32 g + 31)
                // swap one 16-byte half, so the first store writes quad A's
                // line (A: its outputs 0-1, B: A's outputs 2-3) and the second
                // quad B's line
                const int b2 = (lane >> 2) & 1;
                const u32x4 snd = b2 ? s01 : s23;
                u32x4 rcv;
                rcv.x = (unsigned)__builtin_amdgcn_ds_swizzle((int)snd.x, 0x101F);   // lane ^ 4
                rcv.y = (unsigned)__builtin_amdgcn_ds_swizzle((int)snd.y, 0x101F);
                rcv.z = (unsigned)__builtin_amdgcn_ds_swizzle((int)snd.z, 0x101F);
                rcv.w = (unsigned)__builtin_amdgcn_ds_swizzle((int)snd.w, 0x101F);
                const unsigned o1 = (unsigned)(tile * TOUT + 32 * (lane >> 3) + 4 * (lane & 3) + 2 * b2) * 8u;
                __builtin_amdgcn_raw_buffer_store_b128(b2 ? rcv : s01, ry, o1, 0, 2);
                __builtin_amdgcn_raw_buffer_store_b128(b2 ? s23 : rcv, ry, o1 + 128u, 0, 2);
            } else if (ko + 4 <= nout && smode) {
                __builtin_amdgcn_raw_buffer_store_b128(s01, ry, (unsigned)ko * 8u, 0, 2);
                __builtin_amdgcn_raw_buffer_store_b128(s23, ry, (unsigned)ko * 8u + 16u, 0, 2);
            } else if (ko < nout) {   // the call's ragged end (one lane of one wave), or y not 16-byte aligned
                for (int s = 0; s < 4; s++)
                    if (ko + s < nout)
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, acc[s]), ry,
                                                              (unsigned)(ko + s) * 8u, 0, 2);
            }
        }
        fetch(tile + (PF + 1) * GW, ws2, wbuf);
        ec = en;
        en = enn;
        if constexpr (PF == 2) {
            enn = e3;
            e3 = entry(tile + 4 * GW, cc);
        } else {
            enn = entry(tile + 3 * GW, cc);
        }
        cur_next(cc);
    };
    for (int tile = gw; tile < ntiles; tile += PF * GW) {
        body(tile, wa);
        if constexpr (PF == 2) {
            if (tile + GW >= ntiles) break;
            body(tile + GW, wb);
        }
    }
}

template <int L, bool UP, int HM, bool R4 = false, bool DN = false>
void launch_rs4_c(const lqk_rs4_plan &pl, unsigned long long g0, unsigned long long K0, int npfb, float del,
                  const float2 *taps2, const float2 *hist, const float2 *x, int n, float2 *y, int nout,
                  const lqk_rs4_hb &hb, const lqk_hist_job &hj, hipStream_t st)
{
    // 16-byte output stores, whole 128-byte lines per store instruction
    // (2; 1: two 16-byte stores 32 B apart per lane, kept for the call's
    // ragged last tile): 0.1117-0.1120 -> 0.1099-0.1112 ms at config 5
    // (profiles/r06_ab_experiments.txt, r06d); 0: y only 8-byte aligned
    const int smode = ((unsigned long long)y & 15) ? 0 : 2;
    const int RS = npfb + 1;
    const size_t lds =
        (size_t)((rs4_rows<L, UP, DN>() * RS * 8 + 15) & ~15) + (size_t)(NT4 / 64) * 4 * rs4_n4<UP, DN>() * 8;
    constexpr int TS = TOUT - (HM ? ((2 * HM - 1 + 3) & ~3) : 0);
    const int ntiles = (nout + TS - 1) / TS;
    const int wgs = (ntiles + NT4 / 64 - 1) / (NT4 / 64);
    constexpr int B = HM ? 4 : rs4_blk<L, UP, DN>();   // the fused stage's window needs the VGPRs of a fifth
    const int blk = lds * B <= 160 * 1024 ? B : (int)(160 * 1024 / lds);
    const int nb = wgs < 256 * blk ? wgs : 256 * blk;   // persistent: blk per CU
    if (npfb == 64)
        hipLaunchKernelGGL((k_resamp4<L, 64, UP, HM, R4, DN>), dim3(nb), dim3(NT4), lds, st, pl, g0, K0, npfb, del,
                           taps2, hist, x, n, y, nout, smode, hb, hj);
    else if constexpr (HM == 0)
        hipLaunchKernelGGL((k_resamp4<L, 0, UP, 0, R4, DN>), dim3(nb), dim3(NT4), lds, st, pl, g0, K0, npfb, del,
                           taps2, hist, x, n, y, nout, smode, hb, hj);
}

template <int L>
void launch_rs4(const lqk_rs4_plan &pl, unsigned long long g0, unsigned long long K0, int npfb, float del,
                const float2 *taps2, const float2 *hist, const float2 *x, int n, float2 *y, int nout,
                const lqk_hist_job &hj, hipStream_t st)
{
    const lqk_rs4_hb none{};
    if (del < 0.5f)   // r > 2: more than two outputs per input
        launch_rs4_c<L, true, 0, true>(pl, g0, K0, npfb, del, taps2, hist, x, n, y, nout, none, hj, st);
    else if (del <= 1.0f)
        launch_rs4_c<L, true, 0>(pl, g0, K0, npfb, del, taps2, hist, x, n, y, nout, none, hj, st);
    else if (del >= 2.0f)   // 1/4 < r <= 1/2: an output every two to four inputs
        launch_rs4_c<L, false, 0, false, true>(pl, g0, K0, npfb, del, taps2, hist, x, n, y, nout, none, hj, st);
    else
        launch_rs4_c<L, false, 0>(pl, g0, K0, npfb, del, taps2, hist, x, n, y, nout, none, hj, st);
}

} // namespace

extern "C" int lqk_resamp4_supported(unsigned int npfb, unsigned int L)
{
    // power-of-two banks up to 256 (table in LDS), even L up to 32
    return npfb >= 2 && npfb <= 256 && (npfb & (npfb - 1)) == 0 && L >= 2 && L <= 32 && (L % 2) == 0;
}

extern "C" int lqk_resamp4_hb_supported(unsigned int npfb, unsigned int L, float del, int m)
{
    return npfb == 64 && L == 14 && del > 0.5f && del <= 1.0f && m >= 3 && m <= LQK_RS4_HB_MAXM;
}

extern "C" void lqk_resamp4(const lqk_rs4_plan *pl, unsigned long long g0, unsigned long long K0, unsigned int npfb,
                            unsigned int L, float del, const void *taps2, const void *hist, const void *x,
                            unsigned long long n, void *y, unsigned long long nout, const lqk_rs4_hb *hb,
                            const lqk_hist_job *job, void *stream)
{
    if (n == 0) return;
    if (nout == 0) {   // no outputs, so no launch: the history update on its own
        if (job && job->dst) lqk_window_append(1, job->src, job->L, job->x, job->n, job->dst, stream);
        return;
    }
    const lqk_hist_job hj = job ? *job : lqk_hist_job{nullptr, nullptr, 0ull, nullptr, 0u};
    if (!lqk_resamp4_supported(npfb, L) || n > LQK_RS_MAXN || nout * (hb ? 16ull : 8ull) >= (1ull << 31) ||
        pl->ntab * 8ull >= (1ull << 31) || !(pl->pre == ~0ull || (pl->QT >= TOUT && pl->npre == (pl->pre + 3) / 4)) ||
        (hb && !lqk_resamp4_hb_supported(npfb, L, del, hb->m))) {
        fprintf(stderr, "error: liquid-mi355x: resamp4 launch outside its shape (npfb %u, L %u, %llu inputs)\n", npfb, L, n);
        exit(1);
    }
    hipStream_t st = (hipStream_t)stream;
    const float2 *t2 = (const float2 *)taps2, *h = (const float2 *)hist, *xi = (const float2 *)x;
    float2 *yo = (float2 *)y;
    if (hb) {
        switch (hb->m) {
#define LQ_RS4_HB(MM)                                                                                   \
    case MM:                                                                                            \
        launch_rs4_c<14, true, MM>(*pl, g0, K0, 64, del, t2, h, xi, (int)n, yo, (int)nout, *hb, hj, st); \
        break;
            LQ_RS4_HB(3) LQ_RS4_HB(4) LQ_RS4_HB(5) LQ_RS4_HB(6) LQ_RS4_HB(7)
            LQ_RS4_HB(8) LQ_RS4_HB(9) LQ_RS4_HB(10) LQ_RS4_HB(11) LQ_RS4_HB(12)
#undef LQ_RS4_HB
        }
        LQ_CHECK_LAUNCH();
        return;
    }
#define LQ_RS4_CASE(LL)                                                                                 \
    case LL:                                                                                            \
        launch_rs4<LL>(*pl, g0, K0, (int)npfb, del, t2, h, xi, (int)n, yo, (int)nout, hj, st);          \
        break;
    switch (L) {
        LQ_RS4_CASE(2)
        LQ_RS4_CASE(4)
        LQ_RS4_CASE(6)
        LQ_RS4_CASE(8)
        LQ_RS4_CASE(10)
        LQ_RS4_CASE(12)
        LQ_RS4_CASE(14)
        LQ_RS4_CASE(16)
        LQ_RS4_CASE(18)
        LQ_RS4_CASE(20)
        LQ_RS4_CASE(22)
        LQ_RS4_CASE(24)
        LQ_RS4_CASE(26)
        LQ_RS4_CASE(28)
        LQ_RS4_CASE(30)
        LQ_RS4_CASE(32)
    }
#undef LQ_RS4_CASE
    LQ_CHECK_LAUNCH();
}
