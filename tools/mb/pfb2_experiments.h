// pfb2_experiments.h -- firpfbch2 M=1024 kernel variants measured and not
// adopted (dev tool; included by mb_pfb2.hip after the library kernel).
//
// k_pfb2_an1024_v2: two workgroups per CU (8 waves, 78 KB LDS each), each
// lane owning two columns, so one workgroup's transforms overlap the other's
// row traffic.  Correct (matches the library kernel to 2e-11) but at the
// 128-VGPR budget of 4 waves/SIMD the two-column ring spills (22-60 VGPRs):
// 0.91 ms vs 0.80 ms for the library kernel on 2^27 samples.
#include <type_traits>

namespace {

// helpers of the scalar transform form (moved out of the library kernel)
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

// exchange with the partner lane inside a quad through DPP (a VALU operand
// modifier, no LDS crossbar): quad_perm [1,0,3,2] for xor 1, [2,3,0,1] for xor 2
template <int X>
__device__ __forceinline__ float2 quad_xor(float2 v)
{
    constexpr int ctrl = X == 1 ? 0xB1 : 0x4E;
    const int a = __builtin_amdgcn_mov_dpp(__float_as_int(v.x), ctrl, 0xF, 0xF, false);
    const int b = __builtin_amdgcn_mov_dpp(__float_as_int(v.y), ctrl, 0xF, 0xF, false);
    return make_float2(__int_as_float(a), __int_as_float(b));
}

// streaming (non-temporal) store of one complex sample: output is written once
__device__ __forceinline__ void st_nt(float2 *p, float2 v)
{
    v2f w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<v2f *>(p));
}


// one 1024-point IFFT of the block in LDS buffer B by one wave, natural-order
// result through B into 16-byte non-temporal stores (the SMODE 2 path above)
__device__ __forceinline__ void fft1024_store(float2 *B, long long b, const Params &P, int lane,
                                              const float2 *tw1, const float2 *tw2)
{
    float2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = B[lane + 64 * k];
    dft16_bwd(v);
#pragma unroll
    for (int k1 = 1; k1 < 16; k1++) {
        if ((k1 & 3) == 0) __builtin_amdgcn_sched_barrier(0);
        v[k1] = cmul(v[k1], tw1[k1 * 64 + lane]);
    }
    lds_fence();
#pragma unroll
    for (int k1 = 0; k1 < 16; k1++) B[k1 * TSTR + lane] = v[k1];
    lds_fence();
    const int k1 = lane >> 2, bq = lane & 3;
#pragma unroll
    for (int a = 0; a < 16; a++) v[a] = B[k1 * TSTR + 4 * a + bq];
    dft16_bwd(v);
#pragma unroll
    for (int r = 1; r < 16; r++) {
        if ((r & 3) == 0) __builtin_amdgcn_sched_barrier(0);
        v[r] = cmul(v[r], tw2[r * 4 + bq]);
    }
    const bool hi2 = (bq & 2) != 0, hi1 = (bq & 1) != 0;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        float2 p = quad_xor<2>(v[r]);
        float2 u = hi2 ? csub(p, v[r]) : cadd(v[r], p);
        if (bq == 3) u = cmul_pj(u);
        float2 p2 = quad_xor<1>(u);
        v[r] = hi1 ? csub(p2, u) : cadd(u, p2);
    }
    if (b >= P.B0 && b < P.B0 + P.nblk) {
        const int s = ((bq & 1) << 1) | (bq >> 1);
        lds_fence();
#pragma unroll
        for (int r = 0; r < 16; r++) B[k1 + 16 * r + 260 * s] = v[r];
        lds_fence();
        typedef float v4f __attribute__((ext_vector_type(4)));
        v4f *Yb = reinterpret_cast<v4f *>(P.Y + (b - P.B0) * M);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int o = 2 * (lane + 64 * q);
            const v4f val = *reinterpret_cast<const v4f *>(B + o + 4 * (o >> 8));
            __builtin_nontemporal_store(val, Yb + (o >> 1));
        }
    }
}

// Two workgroups per CU (8 waves, 78 KB LDS each) so one workgroup's
// transforms overlap the other's row traffic.  Each lane owns the lo column
// tid (bin j0 = M/2-1-tid) and the hi column tid + M/2 (bin j1 = M-1-tid);
// the four tap sets of the two columns are just rows j0 and j1 of hsub
// (j0 ^ M/2 = j1).  An iteration streams 4 rows and completes 8 blocks (one
// IFFT per wave); LDS slot = block & 7, and the hi half of block 8(g+1),
// produced by the iteration's last row, waits in a register until the slot
// is free.  Iterations are unrolled in pairs so the 8-row register ring is
// indexed with constants.
constexpr int NT2 = 512;
template <int L, int PF = 4, int WPE = 4>
__global__ __launch_bounds__(NT2, WPE) void k_pfb2_an1024_v2(Params P, const float *__restrict__ hsub,
                                                            const float2 *__restrict__ tw4096)
{
    static_assert(L <= NS && PF <= 4, "ring / prefetch");
    constexpr int PFA = PF > 0 ? PF : 1;   // array extent (unused when PF == 0)
    __shared__ __attribute__((aligned(16))) float2 xb[8 * BSTR];
    __shared__ __attribute__((aligned(16))) float2 tw1[16 * 64];
    __shared__ __attribute__((aligned(16))) float2 tw2[16 * 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int e = tid; e < 16 * 64; e += NT2) {
        const int k1 = e >> 6, t = e & 63;
        const float2 w = tw4096[(4 * t * k1) & 4095];
        tw1[e] = make_float2(w.x, -w.y);
    }
    if (tid < 64) {
        const int r = tid >> 2, b = tid & 3;
        const float2 w = tw4096[(64 * b * r) & 4095];
        tw2[tid] = make_float2(w.x, -w.y);
    }
    const int j0 = M2 - 1 - tid, j1 = M - 1 - tid;
    // taps are re-read (L1/L2 hits) at each dot phase rather than held across
    // the transforms: 4 waves per SIMD need <= 128 VGPRs
    float t0[L], t1[L];
    auto load_taps = [&]() {
        int o0 = j0 * L, o1 = j1 * L;
        asm volatile("" : "+v"(o0), "+v"(o1));
#pragma unroll
        for (int n = 0; n < L; n++) {
            t0[n] = hsub[o0 + n];
            t1[n] = hsub[o1 + n];
        }
    };
    load_taps();
    float2 w0[NS], w1[NS];
    const long long gs = P.gs0 + (long long)blockIdx.x * P.gpw;
    long long ge = gs + P.gpw;
    if (ge > P.gend) ge = P.gend;
    const long long HL = 2 * (L / 2) * M - M2;
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void *)P.x, (short)0, (int)(P.n_in * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t rh =
        __builtin_amdgcn_make_buffer_rsrc((void *)P.hist, (short)0, (int)(HL * 8), 0x00020000);
    const long long row0 = 4 * gs - NS;   // first warm-up row
    const long long ibase = row0 * M + (long long)tid - P.B0 * M2;
    const unsigned ox0 = (unsigned)(ibase * 8), oh0 = (unsigned)((HL + ibase) * 8);
    // rows that may lie before x (warm-up, first group of the call) sum a
    // history load and an x load (one is out of range and reads 0); later rows
    // are inside x (or past its end) and take the x load alone
    auto fetch = [&](long long c, int hi) -> float2 {
        const unsigned k = (unsigned)(c - row0) * (unsigned)(M * 8) + (hi ? (unsigned)(M2 * 8) : 0u);
        const float2 a = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, ox0 + k, 0, 0));
        const float2 b = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rh, oh0 + k, 0, 0));
        return make_float2(a.x + b.x, a.y + b.y);
    };
    auto fetchx = [&](long long c, int hi) -> float2 {
        const unsigned k = (unsigned)(c - row0) * (unsigned)(M * 8) + (hi ? (unsigned)(M2 * 8) : 0u);
        return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rx, ox0 + k, 0, 0));
    };
    // first row whose every sample is inside x (or beyond): c M >= B0 M/2
    const long long crow_x = (P.B0 * M2 + M - 1) / M;
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
    // warm-up rows row0 .. 4gs-1; ring slot = row & 7
    const int sh = (int)(row0 & 7);   // 0 or 4
#pragma unroll
    for (int s = 0; s < NS; s++) {
        w0[s] = make_float2(0.f, 0.f);
        w1[s] = make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
        // row row0 + s lands in ring slot (sh + s) & 7; rotate by sh with constant indices
        const float2 a = fetch(row0 + s, 0), b = fetch(row0 + s, 1);
        if (sh == 0) { w0[s] = a; w1[s] = b; }
        else { w0[(s + 4) & 7] = a; w1[(s + 4) & 7] = b; }
    }
    // hi half of block 8gs from row 4gs-1 (slot (4gs-1) & 7)
    float2 pend = (sh == 0) ? dot(w1, 7, t1) : dot(w1, 3, t1);
    __syncthreads();   // twiddle tables

    float2 p0[PFA], p1[PFA];
#pragma unroll
    for (int r = 0; r < PF; r++) {
        p0[r] = fetch(4 * gs + r, 0);
        p1[r] = fetch(4 * gs + r, 1);
    }
    auto phase = [&](long long g, auto parc, auto histc) {
        constexpr int par = decltype(parc)::value;   // (4g) & 7 == 4 par
        constexpr bool HIST = decltype(histc)::value;
        load_taps();
        xb[0 * BSTR + j1] = pend;                    // block 8g, hi half
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int s = 4 * par + r;
            w0[s] = r < PF ? p0[r] : (HIST ? fetch(4 * g + r, 0) : fetchx(4 * g + r, 0));
            w1[s] = r < PF ? p1[r] : (HIST ? fetch(4 * g + r, 1) : fetchx(4 * g + r, 1));
            xb[(2 * r) * BSTR + j0] = dot(w0, s, t0);
            xb[(2 * r + 1) * BSTR + j0] = dot(w0, s, t1);
            xb[(2 * r + 1) * BSTR + j1] = dot(w1, s, t0);
            if (r < 3) xb[(2 * r + 2) * BSTR + j1] = dot(w1, s, t1);
            else pend = dot(w1, s, t1);
        }
        if (g + 1 < ge) {
#pragma unroll
            for (int r = 0; r < PF; r++) {
                p0[r] = fetch(4 * (g + 1) + r, 0);
                p1[r] = fetch(4 * (g + 1) + r, 1);
            }
        }
        lds_barrier();
        fft1024_store(xb + wave * BSTR, 8 * g + wave, P, lane, tw1, tw2);
        lds_barrier();
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using HT = std::integral_constant<bool, true>;
    using HF = std::integral_constant<bool, false>;
    long long g = gs;
    if (sh == 4) {   // 4gs = 4 mod 8: the first group uses the upper ring half
        if (g < ge) {
            if (4 * g < crow_x) phase(g, I1{}, HT{});
            else phase(g, I1{}, HF{});
        }
        g++;
    } else if (g < ge && 4 * g < crow_x) {
        phase(g, I0{}, HT{});
        if (g + 1 < ge) phase(g + 1, I1{}, HT{});
        g += 2;
    }
    for (; g < ge; g += 2) {
        phase(g, I0{}, HF{});
        if (g + 1 < ge) phase(g + 1, I1{}, HF{});
    }
}


} // namespace
