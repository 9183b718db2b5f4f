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
//  * A workgroup of 16 waves (1024 lanes, one workgroup per CU, 4 waves per
//    SIMD) owns all 1024 columns, one per lane, with the column's even- and
//    odd-block taps and an 8-deep register ring.  Rows stream through the
//    ring, so every input sample is read from HBM once per workgroup
//    segment.  Eight rows per iteration complete sixteen blocks; six rows
//    of the next iteration are prefetched into registers while the FFTs run
//    and the last two load in the dot phase (the tap selection is per lane,
//    outside the loop, so the row loop carries no per-lane selects: 112
//    VGPRs, no spills).
//  * X of each block goes to an LDS ring (17 block buffers, 148 KB); after a
//    barrier each wave runs one 1024-point IFFT in registers, 1024 = 16x16x4:
//    16-point DFT over the lane's 16 bins (j = lane + 64k), twiddle, LDS
//    transpose (row stride 68 keeps ds_read_b64 conflict-free), 16-point DFT,
//    twiddle, LDS transpose, four 4-point DFTs.  Every complex operation is a
//    packed v_pk_{add,mul,fma}_f32 with op_sel/neg modifiers (one instruction
//    per add or +-j rotation, two per multiply): 380 VALU instructions per
//    transform instead of ~650 for the scalar + DPP-quad form (FM = 0, kept
//    for tools/mb/mb_pfb2.hip; 0.74-0.79 -> 0.70-0.71 ms per 2^27 samples).
//    The last transpose leaves each lane two adjacent bins, so the outputs
//    leave as 16-byte non-temporal stores, 1 KB contiguous per instruction.
//    1/M is folded into the coefficients (exact for M = 2^10).
//  * Blocks are grouped four at a time in global block numbering (even block
//    = offset 0, odd = M/2), so calls of any length and start parity share one
//    kernel; blocks outside the call are computed but not stored.
#include "lq_device.h"
#include "lq_fft1024.h"
#include "lq_kernels.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace {

constexpr int M = 1024;
constexpr int M2 = M / 2;
constexpr int NT = 1024;
constexpr int NS = 8;      // register ring depth (rows)
constexpr int NBUF = 17;   // LDS block buffers (writes b0..b0+16, FFT reads b0..b0+15)
constexpr int BSTR = 1088; // floats2 per block buffer (16 x 68 transpose)
constexpr int TSTR = 68;

__device__ __forceinline__ void lds_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its global loads or stores (__syncthreads() would also
// drain the prefetched rows and the output stores at every phase change).
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

struct Params {
    const float2 *hist;
    const float2 *x;
    long long n_in;   // input samples in this call
    long long B0;     // global index of the call's first block (parity matters)
    long long nblk;   // blocks in this call
    long long gs0;    // first global 16-block group of workgroup 0
    int gpw;          // groups per workgroup
    long long gend;   // one past the last group needed
    float2 *Y;
    const float2 *zero; // >= 8 bytes of zeros (lqrt_zeros)
    lqk_hist_job hj;    // the object's history update (first launch of a call)
};

template <int L, bool PAIR>
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
    lq_hist_job_run<float2>(P.hj);   // (its loads and stores drain at the s_waitcnt below)

    {
        const int k1 = tid >> 6, t = tid & 63;
        float2 w = tw4096[(4 * t * k1) & 4095];
        tw1[tid] = make_float2(w.x, -w.y);
    }
    if (tid < 64) {
        const int r = tid >> 2, b = tid & 3;
        float2 w = tw4096[(64 * b * r) & 4095];
        tw2[tid] = make_float2(w.x, -w.y);
    }

    // lane column: tid < M/2 -> lo column, bin j = M/2-1-tid, feeds blocks
    // 2c (even taps) and 2c+1 (odd taps) from row c; tid >= M/2 -> hi column,
    // bin j = 3M/2-1-tid, feeds 2c+1 (odd) and 2c+2 (even).  Even taps
    // h[j + nM], odd taps h[(j ^ M/2) + nM]; 1/M folded in (exact).
    const bool lo = tid < M2;
    const int j = lo ? (M2 - 1 - tid) : (3 * M2 - 1 - tid);
    // taps are re-read (L1/L2 hits) at each dot phase instead of being held
    // in registers across the FFT phase; hsub is pre-scaled by 1/M on the host
    // ta: taps of the first block a row feeds (lo: even taps of block 2c; hi:
    // odd taps of block 2c+1), tb: the second (lo: odd, 2c+1; hi: even, 2c+2).
    // Chosen once per lane, so the row loop has no per-lane tap selects.
    float ta[L], tb[L];
    auto load_taps = [&]() {
        int oa = (lo ? j : (j ^ M2)) * L, ob = (lo ? (j ^ M2) : j) * L;
        asm volatile("" : "+v"(oa), "+v"(ob)); // keep the reload inside the loop
#pragma unroll
        for (int n = 0; n < L; n++) {
            ta[n] = hsub[oa + n];
            tb[n] = hsub[ob + n];
        }
    };
    load_taps();
    // first / second block fed by row c: lo: (2c, E), (2c+1, O); hi: (2c+1, O), (2c+2, E)
    const int dA = lo ? 0 : 1;

    float2 w[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) w[s] = make_float2(0.f, 0.f);

    const long long gs = P.gs0 + (long long)blockIdx.x * P.gpw;
    long long ge = gs + P.gpw;
    if (ge > P.gend) ge = P.gend;
    const long long HL = 2 * (L / 2) * M - M2;
    // Row fetches: one 8-byte load per lane and row from a pointer chosen per
    // lane -- the history (the HL samples before x), x, or a zero word for
    // samples before the history or past the call -- so the load needs no
    // branch and no merge.  (Two range-checked loads per row, one of them out
    // of range, cost a second vector-memory instruction and 16 VGPRs of
    // prefetch registers.)  ls0 = local index of row (8gs - NS)'s first sample.
    const long long ls0 = (8 * gs - NS) * M - P.B0 * M2;
    const unsigned long long ah = (unsigned long long)(uintptr_t)(P.hist + HL);
    const unsigned long long ax = (unsigned long long)(uintptr_t)P.x;
    const unsigned long long az = (unsigned long long)(uintptr_t)P.zero;
    auto fetch = [&](long long c) -> float2 {
        const long long li = ls0 + (c - (8 * gs - NS)) * M + tid;
        // address = (history or x) + 8 li, or the zero word: integer selects
        // (v_cndmask), no branch around the load
        const bool neg = li < 0;
        const bool in = neg ? (li >= -HL) : (li < P.n_in);
        unsigned long long a = (neg ? ah : ax) + (unsigned long long)(li * 8);
        a = in ? a : az;
        // a global (not flat) load: flat loads also count in lgkmcnt, which
        // the LDS barriers wait on
        typedef const v2f __attribute__((address_space(1))) *gptr;
        const v2f v = __builtin_nontemporal_load(reinterpret_cast<gptr>(a));
        return make_float2(v.x, v.y);
    };
    // taps arrive scaled by 1/M (firpfbch2.c:277-278's output scale, exact for M = 2^10)
    auto dot = [&](int newest, const float (&h)[L]) -> float2 {
        float2 acc = make_float2(0.f, 0.f);
#pragma unroll
        for (int n = 0; n < L; n++) {
            const float2 v = w[(newest - n) & (NS - 1)];
            acc.x = fmaf(h[n], v.x, acc.x);
            acc.y = fmaf(h[n], v.y, acc.y);
        }
        return acc;
    };

    // warm-up: rows 8gs-8 .. 8gs-1 fill the ring; the last gives the hi-bin
    // half of block 16gs (hi lanes, even taps)
#pragma unroll
    for (int s = 0; s < NS; s++) w[s] = fetch(8 * gs - NS + s);
    int slot0 = (int)((16 * gs) % NBUF); // buffer of block 16g (advances by 16 mod 17 = -1)
    if (!lo) xb[slot0 * BSTR + j] = dot(NS - 1, tb);
    __syncthreads(); // twiddle tables ready

    // Rows of later groups are prefetched into registers while a group is
    // processed.  PAIR (16-byte aligned x): lane 2t loads row c, lane 2t+1
    // row c+1, both at columns (2t, 2t+1) with one 16-byte load, and a DPP
    // swap inside the lane pair gives every lane its own column of both rows
    // -- half the load instructions of one 8-byte load per row and lane
    // (0.636 -> 0.607 ms per 2^27 samples).  Otherwise one 8-byte load per
    // row.  One group ahead: a second register set (the loop unrolled by
    // two) gained 0.5 % with 8-byte loads and spills with pairs.
    typedef float v4f_ __attribute__((ext_vector_type(4)));
    const int odd = tid & 1;
    auto fetch2 = [&](long long c) -> v4f_ {
        const long long li = ls0 + (c + odd - (8 * gs - NS)) * M + (tid - odd);
        const bool neg = li < 0;
        const bool in = neg ? (li >= -HL) : (li < P.n_in);
        unsigned long long a = (neg ? ah : ax) + (unsigned long long)(li * 8);
        a = in ? a : az;
        typedef const v4f_ __attribute__((address_space(1))) *gptr;
        return __builtin_nontemporal_load(reinterpret_cast<gptr>(a));
    };
    // quad_perm [1,0,3,2]: swap with the pair partner
    auto swp = [](float v) -> float {
        return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
    };
    auto split = [&](v4f_ v, float2 &rc, float2 &rn) {
        // even lane holds row c (own, partner's column), odd lane row c+1
        // (partner's column, own); each sends the sample its partner owns
        const float sx = swp(odd ? v.x : v.z), sy = swp(odd ? v.y : v.w);
        rc = odd ? make_float2(sx, sy) : make_float2(v.x, v.y);
        rn = odd ? make_float2(v.z, v.w) : make_float2(sx, sy);
    };
    typedef typename std::conditional<PAIR, v4f_, float2>::type PfT;
    // Six of the group's eight rows are prefetched; the last two are loaded
    // in the dot phase itself (all eight ahead: 0.630 ms, six: 0.620, four:
    // 0.635 per 2^27 samples, r06l)
    constexpr int NPF = PAIR ? 3 : 6;   // prefetch registers (PAIR: row pairs)
    auto fetch_group = [&](long long g, PfT (&pf)[NPF]) {
#pragma unroll
        for (int q = 0; q < NPF; q++) {
            if constexpr (PAIR) pf[q] = fetch2(8 * g + 2 * q);
            else pf[q] = fetch(8 * g + q);
        }
    };
    PfT pf[NPF];
    fetch_group(gs, pf);
    // Drain everything once before the loop: the loop header then merges an
    // empty vector-memory queue with the loop's own steady state (prefetched
    // rows, taps, then this wave's stores), and the compiler's vmcnt at the
    // first use of a prefetched row leaves the stores in flight instead of
    // waiting for the whole queue (vmcnt(0)) every iteration.
    __builtin_amdgcn_s_waitcnt(0);

    // outputs leave through a range-checked buffer descriptor over the call's
    // nblk blocks: stores of blocks outside the call (b < B0 wraps to a huge
    // unsigned offset) are dropped by the hardware, so the store path has no
    // branch and every wave issues the same vector-memory sequence each
    // iteration (the compiler's vmcnt bookkeeping stays exact, see below)
    const __amdgpu_buffer_rsrc_t ry =
        __builtin_amdgcn_make_buffer_rsrc((void *)P.Y, (short)0, (int)(P.nblk * M * 8), 0x00020000);

    for (long long g = gs; g < ge; g++) {
        const long long b0 = 16 * g;
        float2 nxt;
#pragma unroll
        for (int r = 0; r < 8; r++) {
            // row c = 8g + r -> blocks b0 + 2r + dA (first), b0 + 2r + dA + 1 (second)
            if constexpr (PAIR) {
                // (the odd row waits in nxt: its ring slot still holds row
                // r-7, which row r's dot product reads)
                if ((r & 1) == 0) split((r >> 1) < NPF ? pf[(r >> 1) < NPF ? r >> 1 : 0] : fetch2(8 * g + r), w[r], nxt);
                else w[r] = nxt;
            } else {
                w[r] = r < NPF ? pf[r < NPF ? r : 0] : fetch(8 * g + r);
            }
            int s1 = slot0 + 2 * r + dA;
            s1 -= (s1 >= NBUF) ? NBUF : 0;
            int s2 = s1 + 1;
            s2 -= (s2 >= NBUF) ? NBUF : 0;
            xb[s1 * BSTR + j] = dot(r, ta);
            xb[s2 * BSTR + j] = dot(r, tb);
        }
        lds_barrier();
        // the next group's rows, issued after the barrier (before it: 0.635
        // -> 0.624 ms per 2^27 samples, r06c in profiles/r06_ab_experiments.txt)
        if (g + 1 < ge) fetch_group(g + 1, pf);

        // ---- one 1024-point IFFT per wave: block b0 + wave
        {
            // 1024 = 16 x 16 x 4, every radix in registers with packed math:
            // DFT16 over k (j = lane + 64k), twiddle, transpose, DFT16 over a
            // (l = 4a + bq), twiddle, transpose, 4 x DFT4 over bq; the last
            // transpose leaves each lane two adjacent bins, so the outputs
            // leave as 16-byte stores covering 1 KB per wave instruction.
            const long long b = b0 + wave;
            int sb = slot0 + wave;
            sb -= (sb >= NBUF) ? NBUF : 0;
            float2 *B = xb + sb * BSTR;
            v2f v[16];
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = pk(B[lane + 64 * k]);
            pk_dft16<-1>(v);
#pragma unroll
            for (int k1 = 1; k1 < 16; k1++) {
                if ((k1 & 3) == 0) __builtin_amdgcn_sched_barrier(0);
                v[k1] = pk_cmul(v[k1], pk(tw1[k1 * 64 + lane]));
            }
            lds_fence();
#pragma unroll
            for (int k1 = 0; k1 < 16; k1++) B[k1 * TSTR + lane] = unpk(v[k1]);
            lds_fence();
            const int k1 = lane >> 2, bq = lane & 3;
#pragma unroll
            for (int a = 0; a < 16; a++) v[a] = pk(B[k1 * TSTR + 4 * a + bq]);
            pk_dft16<-1>(v);
#pragma unroll
            for (int r = 1; r < 16; r++) {
                if ((r & 3) == 0) __builtin_amdgcn_sched_barrier(0);
                v[r] = pk_cmul(v[r], pk(tw2[r * 4 + bq]));
            }
            {
                // C[k1][bq][r] at k1 + 16 r + 260 bq: the b64 writes of each
                // 16-lane group hit 16 distinct bank pairs, the b128 reads below
                // are conflict-free (MI355X_MICROARCH.md LDS table)
                lds_fence();
#pragma unroll
                for (int r = 0; r < 16; r++) B[k1 + 16 * r + 260 * bq] = unpk(v[r]);
                lds_fence();
                // The next iteration's taps are loaded here, BEFORE this wave's
                // output stores: vmcnt counts stores too, so a tap load issued
                // after them (at the top of the dot phase) would make the dot
                // phase wait until every store of the block had drained.
                load_taps();
                __builtin_amdgcn_sched_barrier(0);
                typedef float v4f __attribute__((ext_vector_type(4)));
                // lane (t2, p2): bins k1 = 2 p2 + {0, 1}, r = t2 + 8u
                const int t2 = lane >> 3, p2 = lane & 7;
                const unsigned yo = (unsigned)((b - P.B0) * (M * 8)) + (unsigned)(8 * (2 * p2 + 16 * t2));
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    v4f c[4];
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        c[q] = *reinterpret_cast<const v4f *>(B + 2 * p2 + 16 * (t2 + 8 * u) + 260 * q);
                    v2f e0[4] = {c[0].xy, c[1].xy, c[2].xy, c[3].xy};
                    v2f e1[4] = {c[0].zw, c[1].zw, c[2].zw, c[3].zw};
                    pk_dft4<-1>(e0[0], e0[1], e0[2], e0[3]);
                    pk_dft4<-1>(e1[0], e1[1], e1[2], e1[3]);
                    // Y[k1 + 16 r + 256 s], streaming (non-temporal) stores
#pragma unroll
                    for (int sidx = 0; sidx < 4; sidx++) {
                        const v4f val = {e0[sidx].x, e0[sidx].y, e1[sidx].x, e1[sidx].y};
                        // default cache policy: 0.635 -> 0.620 ms against
                        // non-temporal stores (r06c)
                        __builtin_amdgcn_raw_buffer_store_b128(val, ry, yo + 8 * (128 * u + 256 * sidx), 0, 0);
                    }
                }
            }
        }
        slot0 = slot0 == 0 ? NBUF - 1 : slot0 - 1; // (16(g+1)) mod 17
        lds_barrier();
    }
}

// ---------------------------------------------------------------- firpfbch analyzer
// Critically sampled analyzer (firpfbch_crcf, M = 1024, real taps), the same
// structure for the reference's firpfbch.c:346-409: row b = x[bM .. bM+M),
// X_b[j] = sum_{n<P} h[(M-1-j) P + n] row_{b-n}[j], Y_b = FFT_forward(X_b).
// Every row completes one block, so an iteration streams 16 rows into 16
// block buffers (no half-block carried over) and 16 waves transform them.

// forward (DIR +1) / backward tables: tw1[k1*64 + t] = W_1024^{DIR t k1},
// tw2[r*4 + b] = W_64^{DIR b r}
template <int DIR>
__device__ __forceinline__ void fft1k_tables(float2 *tw1, float2 *tw2, const float2 *__restrict__ tw4096, int tid)
{
    const int k1 = tid >> 6, t = tid & 63;
    const float2 w = tw4096[(4 * t * k1) & 4095];
    tw1[tid] = make_float2(w.x, DIR > 0 ? w.y : -w.y);
    if (tid < 64) {
        const int r = tid >> 2, b = tid & 3;
        const float2 u = tw4096[(64 * b * r) & 4095];
        tw2[tid] = make_float2(u.x, DIR > 0 ? u.y : -u.y);
    }
}

// one 1024-point transform of B (one wave, packed 16 x 16 x 4; B is the
// block's own LDS buffer, used as transpose scratch) stored to Yb with
// 16-byte non-temporal stores
template <int DIR>
__device__ __forceinline__ void fft1k_wave_store(float2 *B, const float2 *tw1, const float2 *tw2, int lane, float2 *Yb)
{
    v2f v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = pk(B[lane + 64 * k]);
    pk_dft16<DIR>(v);
#pragma unroll
    for (int k1 = 1; k1 < 16; k1++) v[k1] = pk_cmul(v[k1], pk(tw1[k1 * 64 + lane]));
    lds_fence();
#pragma unroll
    for (int k1 = 0; k1 < 16; k1++) B[k1 * TSTR + lane] = unpk(v[k1]);
    lds_fence();
    const int k1 = lane >> 2, bq = lane & 3;
#pragma unroll
    for (int a = 0; a < 16; a++) v[a] = pk(B[k1 * TSTR + 4 * a + bq]);
    pk_dft16<DIR>(v);
#pragma unroll
    for (int r = 1; r < 16; r++) v[r] = pk_cmul(v[r], pk(tw2[r * 4 + bq]));
    lds_fence();
#pragma unroll
    for (int r = 0; r < 16; r++) B[k1 + 16 * r + 260 * bq] = unpk(v[r]);
    lds_fence();
    typedef float v4f __attribute__((ext_vector_type(4)));
    const int t2 = lane >> 3, p2 = lane & 7;
    v4f *Yv = reinterpret_cast<v4f *>(Yb + 2 * p2 + 16 * t2);
#pragma unroll
    for (int u = 0; u < 2; u++) {
        v4f c[4];
#pragma unroll
        for (int q = 0; q < 4; q++) c[q] = *reinterpret_cast<const v4f *>(B + 2 * p2 + 16 * (t2 + 8 * u) + 260 * q);
        v2f e0[4] = {c[0].xy, c[1].xy, c[2].xy, c[3].xy};
        v2f e1[4] = {c[0].zw, c[1].zw, c[2].zw, c[3].zw};
        pk_dft4<DIR>(e0[0], e0[1], e0[2], e0[3]);
        pk_dft4<DIR>(e1[0], e1[1], e1[2], e1[3]);
#pragma unroll
        for (int sidx = 0; sidx < 4; sidx++) {
            const v4f val = {e0[sidx].x, e0[sidx].y, e1[sidx].x, e1[sidx].y};
            __builtin_nontemporal_store(val, Yv + (128 * u + 256 * sidx) / 2);
        }
    }
}

template <int P, int PF, bool PAIR>
__global__ __launch_bounds__(NT, 1) void k_pfb_an1024(const float2 *hist, const float2 *x, long long nblk, int gpw,
                                                      const float *__restrict__ hsub,
                                                      const float2 *__restrict__ tw4096, float2 *Y,
                                                      const float2 *__restrict__ zero)
{
    static_assert(P <= 8, "ring of 8 rows");
    static_assert(PF % 2 == 0, "whole row pairs");
    __shared__ __attribute__((aligned(16))) float2 xb[16 * BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw1[16 * 64];
    __shared__ __attribute__((aligned(16))) float2 tw2[16 * 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    fft1k_tables<+1>(tw1, tw2, tw4096, tid);
    // column tid: X[j] with i = M-1-j taps h[i P + n]
    float hv[P];
    {
        int o = (M - 1 - tid) * P;
        asm volatile("" : "+v"(o));
#pragma unroll
        for (int n = 0; n < P; n++) hv[n] = hsub[o + n];
    }
    const long long ngroups = (nblk + 15) / 16;
    const long long gs = (long long)blockIdx.x * gpw;
    long long ge = gs + gpw;
    if (ge > ngroups) ge = ngroups;
    const long long HL = (long long)(P - 1) * M;
    // One load per row and lane from a pointer chosen per lane (the history's
    // P-1 rows before x, x, or a zero word), as k_pfb2_an1024; with PAIR
    // (16-byte aligned x) lane 2t loads row c and lane 2t+1 row c+1 at
    // columns (2t, 2t+1) and a DPP swap splits the pair.
    typedef float v4f_ __attribute__((ext_vector_type(4)));
    const unsigned long long ah = (unsigned long long)(uintptr_t)(hist + HL);
    const unsigned long long ax = (unsigned long long)(uintptr_t)x;
    const unsigned long long az = (unsigned long long)(uintptr_t)zero;
    const long long nx = nblk * M;
    auto addr = [&](long long li) -> unsigned long long {
        const bool neg = li < 0;
        const bool in = neg ? (li >= -HL) : (li < nx);
        const unsigned long long a = (neg ? ah : ax) + (unsigned long long)(li * 8);
        return in ? a : az;
    };
    auto fetch = [&](long long c) -> float2 {
        typedef const v2f __attribute__((address_space(1))) *gptr;
        const v2f v = __builtin_nontemporal_load(reinterpret_cast<gptr>(addr(c * M + tid)));
        return make_float2(v.x, v.y);
    };
    const int odd = tid & 1;
    auto fetch2 = [&](long long c) -> v4f_ {
        typedef const v4f_ __attribute__((address_space(1))) *gptr;
        return __builtin_nontemporal_load(reinterpret_cast<gptr>(addr((c + odd) * M + (tid - odd))));
    };
    auto swp = [](float v) -> float {
        return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
    };
    auto split = [&](v4f_ v, float2 &rc, float2 &rn) {
        const float sx = swp(odd ? v.x : v.z), sy = swp(odd ? v.y : v.w);
        rc = odd ? make_float2(sx, sy) : make_float2(v.x, v.y);
        rn = odd ? make_float2(v.z, v.w) : make_float2(sx, sy);
    };
    typedef typename std::conditional<PAIR, v4f_, float2>::type PfT;
    constexpr int NPF = PAIR ? PF / 2 : PF;
    auto fetch_pf = [&](long long g, PfT (&pf)[NPF]) {
#pragma unroll
        for (int q = 0; q < NPF; q++) {
            if constexpr (PAIR) pf[q] = fetch2(16 * g + 2 * q);
            else pf[q] = fetch(16 * g + q);
        }
    };
    // row c lives in ring slot c & 7
    float2 w[8];
#pragma unroll
    for (int s = 1; s < 8; s++) w[(8 - s) & 7] = fetch(16 * gs - s);
    w[0] = make_float2(0.f, 0.f);
    PfT pf[NPF];
    fetch_pf(gs, pf);
    __syncthreads();   // twiddle tables ready

    for (long long g = gs; g < ge; g++) {
        float2 nxt;
#pragma unroll
        for (int r = 0; r < 16; r++) {
            if constexpr (PAIR) {
                // the odd row waits in nxt: its ring slot holds row r-7 until
                // row r's dot product has read it
                if ((r & 1) == 0) split(r < PF ? pf[r >> 1] : fetch2(16 * g + r), w[r & 7], nxt);
                else w[r & 7] = nxt;
            } else {
                w[r & 7] = r < PF ? pf[r] : fetch(16 * g + r);
            }
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll
            for (int n = 0; n < P; n++) {
                const float2 v = w[(r - n) & 7];
                acc.x = fmaf(hv[n], v.x, acc.x);
                acc.y = fmaf(hv[n], v.y, acc.y);
            }
            xb[r * BSTR + tid] = acc;   // X[j], j = the lane's column
        }
        // the next group's first PF rows: at p = 8 eight of 16, issued after
        // the barrier (0.387 ms per 2^27 samples against 0.395 for twelve
        // issued before it, 0.403-0.416 for twelve after, 0.411 for four,
        // r06k / r06l); at p = 4 all sixteen, before it
        constexpr bool after = PF < 16;
        if (!after && g + 1 < ge) fetch_pf(g + 1, pf);
        lds_barrier();
        if (after && g + 1 < ge) fetch_pf(g + 1, pf);
        const long long b = 16 * g + wave;
        if (b < nblk) fft1k_wave_store<+1>(xb + wave * BSTR, tw1, tw2, lane, Y + b * M);
        lds_barrier();
    }
}

// ---------------------------------------------------------------- firpfbch2 analyzer, a few blocks
// Calls of at most 16 blocks (the reference's execute() is one): the
// streaming kernel above would compute a whole 16-block group after an
// 8-row warm-up for them.  Here lane j forms X_b[j] of every block of the
// call straight from the closed form (the history's last HL samples, then
// x; taps pre-scaled by 1/M), and wave b transforms block b -- one launch,
// which also writes the next history and, into pinned host memory, raises
// the call's completion flag.
template <int L>
__global__ __launch_bounds__(NT, 1) void k_pfb2_an1024_few(const float *__restrict__ hsub,
                                                           const float2 *__restrict__ hist,
                                                           const float2 *__restrict__ x, int nb, int p0, float2 *Y,
                                                           unsigned *flag, unsigned seq, lqk_hist_job hj,
                                                           const float2 *__restrict__ tw4096)
{
    __shared__ __attribute__((aligned(16))) float2 xb[16 * BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw1[16 * 64];
    __shared__ __attribute__((aligned(16))) float2 tw2[16 * 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    lq_hist_job_run<float2>(hj);
    fft1k_tables<-1>(tw1, tw2, tw4096, tid);
    constexpr int HL = L * M - M2;
    const int j = tid;
    const int base = j < M2 ? (M2 - 1 - j) : (3 * M2 - 1 - j);
    for (int b = 0; b < nb; b++) {   // firpfbch2.c:244-282 in closed form (k_channelizer.hip, k_pfb2_an)
        const int bt = p0 + b;
        const int i = (j - (bt & 1) * M2) & (M - 1);
        const int c = j < M2 ? (bt >> 1) : ((bt - 1) >> 1);
        const int t0 = c * M + base - p0 * M2;
        float2 acc = make_float2(0.f, 0.f);
#pragma unroll
        for (int n = 0; n < L; n++) {
            const int t = t0 - n * M;
            const float2 v = t < 0 ? hist[HL + t] : x[t];
            const float h = hsub[i * L + n];
            acc.x = fmaf(h, v.x, acc.x);
            acc.y = fmaf(h, v.y, acc.y);
        }
        xb[b * BSTR + j] = acc;
    }
    __syncthreads();
    if (wave < nb) fft1k_wave_store<-1>(xb + wave * BSTR, tw1, tw2, lane, Y + (long long)wave * M);
    if (flag) {   // Y is pinned host memory: the completion flag once every store is visible
        __threadfence_system();
        __syncthreads();
        if (tid == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// firpfbch analyzer, M = 1024, p in {4, 8}, calls of at most 16 blocks: as
// k_pfb2_an1024_few, X_b[j] = sum_n h[(M-1-j) p + n] x[(b-n) M + j]
// (firpfbch.c:346-409), wave b's forward transform of block b.  One
// workgroup reads all of x before any store, so the call may run in place.
template <int P>
__global__ __launch_bounds__(NT, 1) void k_pfb_an1024_few(const float *__restrict__ hsub,
                                                          const float2 *__restrict__ hist, const float2 *x, int nb,
                                                          float2 *Y, unsigned *flag, unsigned seq, lqk_hist_job hj,
                                                          const float2 *__restrict__ tw4096)
{
    __shared__ __attribute__((aligned(16))) float2 xb[16 * BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw1[16 * 64];
    __shared__ __attribute__((aligned(16))) float2 tw2[16 * 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    lq_hist_job_run<float2>(hj);
    fft1k_tables<+1>(tw1, tw2, tw4096, tid);
    constexpr int HL = (P - 1) * M;
    const int j = tid;
    for (int b = 0; b < nb; b++) {
        float2 acc = make_float2(0.f, 0.f);
#pragma unroll
        for (int n = 0; n < P; n++) {
            const int t = (b - n) * M + j;
            const float2 v = t < 0 ? hist[HL + t] : x[t];
            const float h = hsub[(M - 1 - j) * P + n];
            acc.x = fmaf(h, v.x, acc.x);
            acc.y = fmaf(h, v.y, acc.y);
        }
        xb[b * BSTR + j] = acc;
    }
    __syncthreads();   // (every read of x is done: in-place calls are safe)
    if (wave < nb) fft1k_wave_store<+1>(xb + wave * BSTR, tw1, tw2, lane, Y + (long long)wave * M);
    if (flag) {   // Y is pinned host memory: the completion flag once every store is visible
        __threadfence_system();
        __syncthreads();
        if (tid == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---------------------------------------------------------------- firpfbch synthesizer
// firpfbch.c:314-336 mirrored: Z_b = IFFT(X_b) (unnormalised), y_b[i] =
// sum_{n<P} h[i P + n] Z_{b-n}[i].  Per iteration the 16 waves transform 16
// blocks of X into LDS; then
// lane i pulls column i of the 16 results through a register ring of the
// last 8 Z values and writes y_b[i] (64 consecutive samples per wave
// instruction).  A workgroup rebuilds its first blocks' history by
// transforming the 7 X blocks before its range (or reads the object's state).
template <int P>
__global__ __launch_bounds__(NT, 1) void k_pfb_syn1024(const float2 *__restrict__ X, long long nblk, int gpw,
                                                       const float *__restrict__ hsub,
                                                       const float2 *__restrict__ state,
                                                       const float2 *__restrict__ tw4096, float2 *y)
{
    static_assert(P <= 8, "ring of 8");
    __shared__ __attribute__((aligned(16))) float2 zb[16 * BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw1[16 * 64];
    __shared__ __attribute__((aligned(16))) float2 tw2[16 * 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    fft1k_tables<-1>(tw1, tw2, tw4096, tid);
    float hv[P];
    {
        int o = tid * P;
        asm volatile("" : "+v"(o));
#pragma unroll
        for (int n = 0; n < P; n++) hv[n] = hsub[o + n];
    }
    const long long ngroups = (nblk + 15) / 16;
    const long long gs = (long long)blockIdx.x * gpw;
    long long ge = gs + gpw;
    if (ge > ngroups) ge = ngroups;
    const long long b0 = 16 * gs;
    const int zi = tid + 4 * (tid >> 8);   // natural-order bin tid in a transform buffer

    auto load_block = [&](long long b, float2 (&v)[16]) {
        const float2 *Xb = X + b * M + lane;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = Xb[64 * k];
    };
    __syncthreads();   // twiddle tables ready
    // history: Z_{b0-1} .. Z_{b0-P+1}
    if (wave < P - 1 && b0 - (P - 1) + wave >= 0) {
        float2 v[16];
        load_block(b0 - (P - 1) + wave, v);
        fft1024_wave<-1>(v, zb + wave * BSTR, tw1, tw2, lane);
    }
    __syncthreads();
    float2 zr[8];
#pragma unroll
    for (int s = 0; s < 8; s++) zr[s] = make_float2(0.f, 0.f);
#pragma unroll
    for (int s = 1; s < P; s++) {
        const long long c = b0 - s;   // buffer (P-1) - s
        zr[c & 7] = c < 0 ? state[(P - 1 + c) * M + tid] : zb[(P - 1 - s) * BSTR + zi];
    }
    __syncthreads();   // history buffers consumed

    for (long long g = gs; g < ge; g++) {
        const long long b = 16 * g + wave;
        // the block is loaded when its transform starts: holding the next
        // block in registers across the transform (one iteration ahead) ran
        // 0.446-0.449 against 0.430-0.433 ms per 2^27 samples (r06j)
        float2 v[16];
        if (b < nblk) load_block(b, v);
        if (b < nblk) fft1024_wave<-1>(v, zb + wave * BSTR, tw1, tw2, lane);
        lds_barrier();
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const long long bb = 16 * g + r;
            zr[(16 * g + r) & 7] = zb[r * BSTR + zi];
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll
            for (int n = 0; n < P; n++) {
                const float2 z = zr[(16 * g + r - n) & 7];
                acc.x = fmaf(hv[n], z.x, acc.x);
                acc.y = fmaf(hv[n], z.y, acc.y);
            }
            if (bb < nblk) y[bb * M + tid] = acc;
        }
        lds_barrier();
    }
}

// ---------------------------------------------------------------- firpfbch2 synthesizer
// firpfbch2.c:287-335 with M = 1024: z_b = IFFT(X_b) / M * (M/2) (= 0.5
// IFFT, exact), block b of parity f = (p0 + b) & 1 outputs, for i < M/2,
//   y_b[i] = sum_{n<L} h[i L + n] z_{b-2n}[c] + h[(i + M/2) L + n] z_{b-1-2n}[c],
// c = i + f M/2: every term comes from the one column c, so lane c owns it
// (a 16-deep register ring of z_b[c]) and writes y for the blocks whose
// parity matches its half.  16 inverse transforms per iteration as in the
// firpfbch synthesizer, the two scalings applied in the transform's last
// pass (a separate pass over the LDS result before: 0.402 -> 0.372 ms per
// 2^26 outputs, r06h); history from the 15 X blocks before the range.
template <int L>
__global__ __launch_bounds__(NT, 1) void k_pfb2_syn1024(const float2 *__restrict__ X, long long nblk, int p0,
                                                        int gpw, const float *__restrict__ hsub,
                                                        const float2 *__restrict__ state,
                                                        const float2 *__restrict__ tw4096, float2 *y)
{
    static_assert(2 * L <= 16, "ring of 16");
    constexpr int HB = 2 * L - 1;
    __shared__ __attribute__((aligned(16))) float2 zb[16 * BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw1[16 * 64];
    __shared__ __attribute__((aligned(16))) float2 tw2[16 * 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    fft1k_tables<-1>(tw1, tw2, tw4096, tid);
    const int c = tid, f = c >= M2 ? 1 : 0, i = c - f * M2;
    // taps are re-read (L1 hits) in each column phase instead of being held
    // across the transforms (register budget)
    float h0[L], h1[L];
    auto load_taps = [&]() {
        int o0 = i * L, o1 = (i + M2) * L;
        asm volatile("" : "+v"(o0), "+v"(o1));
#pragma unroll
        for (int n = 0; n < L; n++) {
            h0[n] = hsub[o0 + n];
            h1[n] = hsub[o1 + n];
        }
    };
    const long long ngroups = (nblk + 15) / 16;
    const long long gs = (long long)blockIdx.x * gpw;
    long long ge = gs + gpw;
    if (ge > ngroups) ge = ngroups;
    const long long b0 = 16 * gs;
    const int zi = c + 4 * (c >> 8);
    auto load_block = [&](long long b, float2 (&v)[16]) {
        const float2 *Xb = X + b * M + lane;
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = Xb[64 * k];
    };
    // 0.5 IFFT of one block into B (natural order, padded): x 1/M then x M/2
    // (firpfbch2.c:303-307) applied in the transform's last pass
    auto zform = [&](float2 (&v)[16], float2 *B) {
        fft1024_wave<-1, true>(v, B, tw1, tw2, lane, 1.0f / M, (float)M2);
    };
    __syncthreads();   // twiddle tables ready
    // history z_{b0-15} .. z_{b0-1}: wave w < 15 forms z_{b0-15+w}
    if (wave < HB && b0 - HB + wave >= 0) {
        float2 v[16];
        load_block(b0 - HB + wave, v);
        zform(v, zb + wave * BSTR);
    }
    __syncthreads();
    float2 zr[16];
#pragma unroll
    for (int s = 0; s < 16; s++) zr[s] = make_float2(0.f, 0.f);
#pragma unroll
    for (int s = 1; s <= HB; s++) {
        const long long cb = b0 - s;   // buffer HB - s
        zr[cb & 15] = cb < 0 ? state[(HB + cb) * M + c] : zb[(HB - s) * BSTR + zi];
    }
    __syncthreads();   // history buffers consumed

    for (long long g = gs; g < ge; g++) {
        const long long b = 16 * g + wave;
        if (b < nblk) {
            // loaded when the transform starts: the first 8 (or 12, 16) of
            // the block's values prefetched during the column phase ran
            // 0.372-0.374 (0.397, 0.450) against 0.351-0.356 ms (r06h, r06i)
            float2 v[16];
            load_block(b, v);
            zform(v, zb + wave * BSTR);
        }
        lds_barrier();
        load_taps();
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const long long bb = 16 * g + r;
            zr[r] = zb[r * BSTR + zi];   // slot bb & 15 = r
            if (((p0 + bb) & 1) == f && bb < nblk) {
                float2 acc0 = make_float2(0.f, 0.f), acc1 = make_float2(0.f, 0.f);
#pragma unroll
                for (int n = 0; n < L; n++) {
                    const float2 z0 = zr[(r - 2 * n) & 15], z1 = zr[(r - 1 - 2 * n) & 15];
                    acc0.x = fmaf(h0[n], z0.x, acc0.x);
                    acc0.y = fmaf(h0[n], z0.y, acc0.y);
                    acc1.x = fmaf(h1[n], z1.x, acc1.x);
                    acc1.y = fmaf(h1[n], z1.y, acc1.y);
                }
                y[bb * M2 + i] = make_float2(acc0.x + acc1.x, acc0.y + acc1.y);
            }
        }
        lds_barrier();
    }
}

} // namespace

// Returns 1 if handled by the fast path.  Launches cover at most 2^18 blocks
// (2^27 input samples) so every buffer offset fits 31 bits; later chunks take
// their history straight from the preceding input.
extern "C" int lqk_firpfbch2_analyzer_fast(unsigned int Mch, unsigned int m, const void *hsub, const void *hist,
                                           const void *x, unsigned long long nblocks, long long B0, void *Y,
                                           const lqk_hist_job *job, unsigned *flag, unsigned seq, void *stream)
{
    if (Mch != (unsigned)M || !(m == 4 || m == 2)) return 0;
    // x / hist: 8-byte sample loads; Y: 16-byte (two-bin) non-temporal stores
    if (((uintptr_t)x & 7) || ((uintptr_t)hist & 7) || ((uintptr_t)Y & 15)) return 0;
    if (nblocks == 0) return 1;
    hipStream_t st = (hipStream_t)stream;
    const float2 *tw = (const float2 *)lqrt_twiddles();
    if (nblocks <= 16) {   // a few blocks: one workgroup, no warm-up rows
        const lqk_hist_job hj = job ? *job : lqk_hist_job{nullptr, nullptr, 0ull, nullptr, 0u};
        const int p0 = (int)(B0 & 1);
        if (m == 4)
            hipLaunchKernelGGL((k_pfb2_an1024_few<8>), dim3(1), dim3(NT), 0, st, (const float *)hsub,
                               (const float2 *)hist, (const float2 *)x, (int)nblocks, p0, (float2 *)Y, flag, seq, hj,
                               tw);
        else
            hipLaunchKernelGGL((k_pfb2_an1024_few<4>), dim3(1), dim3(NT), 0, st, (const float *)hsub,
                               (const float2 *)hist, (const float2 *)x, (int)nblocks, p0, (float2 *)Y, flag, seq, hj,
                               tw);
        LQ_CHECK_LAUNCH();
        return 1;
    }
    const long long HL = 2LL * m * M - M2;
    const long long CH = 1LL << 18;
    if (flag) return 0;   // (the signalling form is the few-block kernel's)
    for (long long ob = 0; ob < (long long)nblocks; ob += CH) {
        const long long nb = ((long long)nblocks - ob) < CH ? ((long long)nblocks - ob) : CH;
        Params P;
        P.x = (const float2 *)x + ob * M2;
        P.hist = ob == 0 ? (const float2 *)hist : P.x - HL;
        P.n_in = nb * M2;
        P.B0 = B0 + ob;
        P.nblk = nb;
        P.Y = (float2 *)Y + ob * M;
        P.zero = (const float2 *)lqrt_zeros();
        P.hj = {nullptr, nullptr, 0ull, nullptr, 0u};
        if (ob == 0 && job) P.hj = *job;
        const long long gfirst = P.B0 / 16;                // 16-block group containing the first block
        const long long glast = (P.B0 + nb - 1) / 16;      // inclusive
        const long long ngroups = glast - gfirst + 1;
        // one workgroup per CU (LDS-bound), each at least 4 groups (64 blocks)
        long long gpw = (ngroups + 255) / 256;
        if (gpw < 4) gpw = 4;
        const long long nwg = (ngroups + gpw - 1) / gpw;
        P.gs0 = gfirst;
        P.gpw = (int)gpw;
        P.gend = glast + 1;
        // paired 16-byte row loads need x and the history 16-byte aligned
        const bool pair = ((uintptr_t)P.x & 15) == 0 && ((uintptr_t)(P.hist + HL) & 15) == 0;
        if (m == 4 && pair)
            hipLaunchKernelGGL((k_pfb2_an1024<8, true>), dim3((unsigned)nwg), dim3(NT), 0, st, P, (const float *)hsub, tw);
        else if (m == 4)
            hipLaunchKernelGGL((k_pfb2_an1024<8, false>), dim3((unsigned)nwg), dim3(NT), 0, st, P, (const float *)hsub, tw);
        else if (pair)
            hipLaunchKernelGGL((k_pfb2_an1024<4, true>), dim3((unsigned)nwg), dim3(NT), 0, st, P, (const float *)hsub, tw);
        else
            hipLaunchKernelGGL((k_pfb2_an1024<4, false>), dim3((unsigned)nwg), dim3(NT), 0, st, P, (const float *)hsub, tw);
        LQ_CHECK_LAUNCH();
    }
    return 1;
}

// firpfbch_crcf analyzer, M = 1024, P = 8 or 4 real-tap branches: returns 1
// if handled.  Launches cover at most 2^17 blocks (2^27 samples) so buffer
// offsets fit 31 bits; later chunks take their history from the input.
extern "C" int lqk_firpfbch_analyzer_fast(int ctaps, unsigned int Mch, unsigned int p, const void *hsub,
                                          const void *hist, const void *x, unsigned long long nblocks, void *Y,
                                          void *stream)
{
    if (ctaps || Mch != (unsigned)M || !(p == 8 || p == 4)) return 0;
    if (((uintptr_t)x & 7) || ((uintptr_t)hist & 7) || ((uintptr_t)Y & 15)) return 0;
    if (nblocks == 0) return 1;
    hipStream_t st = (hipStream_t)stream;
    const float2 *tw = (const float2 *)lqrt_twiddles();
    const long long HL = (long long)(p - 1) * M;
    const long long CH = 1LL << 17;
    for (long long ob = 0; ob < (long long)nblocks; ob += CH) {
        const long long nb = ((long long)nblocks - ob) < CH ? ((long long)nblocks - ob) : CH;
        const float2 *xs = (const float2 *)x + ob * M;
        const float2 *hs = ob == 0 ? (const float2 *)hist : xs - HL;
        const long long ngroups = (nb + 15) / 16;
        long long gpw = (ngroups + 255) / 256;
        if (gpw < 2) gpw = 2;
        const unsigned nwg = (unsigned)((ngroups + gpw - 1) / gpw);
        const float2 *zero = (const float2 *)lqrt_zeros();
        const bool pair = ((uintptr_t)xs & 15) == 0 && ((uintptr_t)hs & 15) == 0;
        if (p == 8 && pair)
            hipLaunchKernelGGL((k_pfb_an1024<8, 8, true>), dim3(nwg), dim3(NT), 0, st, hs, xs, nb, (int)gpw,
                               (const float *)hsub, tw, (float2 *)Y + ob * M, zero);
        else if (p == 8)
            hipLaunchKernelGGL((k_pfb_an1024<8, 8, false>), dim3(nwg), dim3(NT), 0, st, hs, xs, nb, (int)gpw,
                               (const float *)hsub, tw, (float2 *)Y + ob * M, zero);
        else if (pair)
            hipLaunchKernelGGL((k_pfb_an1024<4, 16, true>), dim3(nwg), dim3(NT), 0, st, hs, xs, nb, (int)gpw,
                               (const float *)hsub, tw, (float2 *)Y + ob * M, zero);
        else
            hipLaunchKernelGGL((k_pfb_an1024<4, 16, false>), dim3(nwg), dim3(NT), 0, st, hs, xs, nb, (int)gpw,
                               (const float *)hsub, tw, (float2 *)Y + ob * M, zero);
        LQ_CHECK_LAUNCH();
    }
    return 1;
}

// firpfbch_crcf analyzer, M = 1024, p in {4, 8}, calls of at most 16
// blocks: one workgroup (k_pfb_an1024_few), which also does the history job
// and, with a flag, raises it once Y (pinned host memory) is written.
// Returns 0 (nothing launched) when the call does not qualify.
extern "C" int lqk_firpfbch_analyzer_few(int ctaps, unsigned int Mch, unsigned int p, const void *hsub,
                                         const void *hist, const void *x, unsigned long long nblocks, void *Y,
                                         const lqk_hist_job *job, unsigned *flag, unsigned seq, void *stream)
{
    if (ctaps || Mch != (unsigned)M || !(p == 8 || p == 4) || nblocks == 0 || nblocks > 16) return 0;
    if (((uintptr_t)x & 7) || ((uintptr_t)hist & 7) || ((uintptr_t)Y & 15)) return 0;
    hipStream_t st = (hipStream_t)stream;
    const float2 *tw = (const float2 *)lqrt_twiddles();
    const lqk_hist_job hj = job ? *job : lqk_hist_job{nullptr, nullptr, 0ull, nullptr, 0u};
    if (p == 8)
        hipLaunchKernelGGL((k_pfb_an1024_few<8>), dim3(1), dim3(NT), 0, st, (const float *)hsub, (const float2 *)hist,
                           (const float2 *)x, (int)nblocks, (float2 *)Y, flag, seq, hj, tw);
    else
        hipLaunchKernelGGL((k_pfb_an1024_few<4>), dim3(1), dim3(NT), 0, st, (const float *)hsub, (const float2 *)hist,
                           (const float2 *)x, (int)nblocks, (float2 *)Y, flag, seq, hj, tw);
    LQ_CHECK_LAUNCH();
    return 1;
}

// firpfbch_crcf synthesizer, M = 1024, P = 8 or 4 real-tap branches, calls of
// at least P-1 blocks: returns 1 if handled (y written, state advanced).
extern "C" int lqk_firpfbch_synthesizer_fast(int ctaps, unsigned int Mch, unsigned int p, const void *hsub,
                                             void *state, const void *X, unsigned long long nblocks, void *y,
                                             void *stream)
{
    if (ctaps || Mch != (unsigned)M || !(p == 8 || p == 4) || nblocks < p - 1) return 0;
    if (((uintptr_t)X & 7) || ((uintptr_t)y & 7)) return 0;
    hipStream_t st = (hipStream_t)stream;
    const float2 *tw = (const float2 *)lqrt_twiddles();
    const long long ngroups = ((long long)nblocks + 15) / 16;
    long long gpw = (ngroups + 255) / 256;
    if (gpw < 2) gpw = 2;
    const unsigned nwg = (unsigned)((ngroups + gpw - 1) / gpw);
    if (p == 8)
        hipLaunchKernelGGL((k_pfb_syn1024<8>), dim3(nwg), dim3(NT), 0, st, (const float2 *)X, (long long)nblocks,
                           (int)gpw, (const float *)hsub, (const float2 *)state, tw, (float2 *)y);
    else
        hipLaunchKernelGGL((k_pfb_syn1024<4>), dim3(nwg), dim3(NT), 0, st, (const float2 *)X, (long long)nblocks,
                           (int)gpw, (const float *)hsub, (const float2 *)state, tw, (float2 *)y);
    LQ_CHECK_LAUNCH();
    // new state: Z of the last p-1 blocks (after the kernel has read the old one)
    lqk_fft_batch(M, -1, (const float2 *)X + (nblocks - (p - 1)) * M, state, p - 1, stream);
    return 1;
}

// firpfbch2_crcf synthesizer, M = 1024, m = 4 or 2, calls of at least 4m-1
// blocks: returns 1 if handled (Y written, state advanced).
extern "C" int lqk_firpfbch2_synthesizer_fast(unsigned int Mch, unsigned int m, const void *hsub, void *state,
                                              const void *X, unsigned long long nblocks, int p0, void *Y,
                                              void *stream)
{
    const unsigned HB = 4 * m - 1;
    if (Mch != (unsigned)M || !(m == 4 || m == 2) || nblocks < HB) return 0;
    if (((uintptr_t)X & 7) || ((uintptr_t)Y & 7)) return 0;
    hipStream_t st = (hipStream_t)stream;
    const float2 *tw = (const float2 *)lqrt_twiddles();
    const long long ngroups = ((long long)nblocks + 15) / 16;
    long long gpw = (ngroups + 255) / 256;
    if (gpw < 2) gpw = 2;
    const unsigned nwg = (unsigned)((ngroups + gpw - 1) / gpw);
    if (m == 4)
        hipLaunchKernelGGL((k_pfb2_syn1024<8>), dim3(nwg), dim3(NT), 0, st, (const float2 *)X, (long long)nblocks,
                           p0 & 1, (int)gpw, (const float *)hsub, (const float2 *)state, tw, (float2 *)Y);
    else
        hipLaunchKernelGGL((k_pfb2_syn1024<4>), dim3(nwg), dim3(NT), 0, st, (const float2 *)X, (long long)nblocks,
                           p0 & 1, (int)gpw, (const float *)hsub, (const float2 *)state, tw, (float2 *)Y);
    LQ_CHECK_LAUNCH();
    // new state: z of the last 4m-1 blocks, formed as the reference does (IFFT, x 1/M, x M/2)
    lqk_fft_batch_scaled(M, -1, (const float2 *)X + (nblocks - HB) * M, state, HB, 1.0f / (float)M,
                         (float)(M / 2), stream);
    return 1;
}
