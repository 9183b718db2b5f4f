// fir_experiments.h -- firfilt crcf design experiments measured on MI355X
// (dev tool, not part of the library; included by mb_fir2.hip after
// liquid-dsp_amd/csrc/k_firfilt.hip).  Results are summarised in DESIGN.md
// ("firfilt: what bounds it"): all of these land at 200-220 G samples/s,
// below the library's k_firfilt, because the chip lowers its clock under
// this f32 arithmetic load (1.5-2.1 GHz measured with s_memtime).
#pragma once
namespace {
// ------------------------------------------------------------------ firfilt crcf (streaming fast path)
// Complex samples, real taps.  Workgroup = NT lanes x R consecutive outputs.
// The input tile [t0-HP, t0+TILE) is copied HBM -> LDS with asynchronous
// 16-byte LDS-DMA loads (global_load_lds_dwordx4, no VGPR staging), each lane
// choosing its own source (stream, history window, in-place halo copy, or a
// dummy past the end), so no branch divides the copy.  LDS holds the tile as
// rows of R samples (R/2 slots of 16 bytes) with the slot index XOR-swizzled
// by the row, which makes the compute phase's ds_read_b128 (lane l reads a
// slot of row l+const) conflict-free for every row offset.
// Compute: taps in groups of R; group G needs rows B and B-1 of the lane's
// window (B = HP/R - G + l); the next older row is read while the current
// group's R x R FMA block runs.  Outputs leave through the same swizzled LDS
// image for 16-byte coalesced stores.
template <int R>
struct cr_geom {
    static constexpr int SPR = R / 2;          // 16-byte slots per row
    static constexpr int RPB = 16 / SPR;       // rows per 256-byte bank period
    __device__ __forceinline__ static int phys(int row, int c) { return row * SPR + (c ^ ((row / RPB) & (SPR - 1))); }
};

// STAGE 0: LDS-DMA (global_load_lds_dwordx4); STAGE 1: register staging
// (all of a lane's 16-byte loads issued before its LDS writes).  W: minimum
// waves per SIMD the register allocation must allow.
template <int HC, int R, int STAGE = 0, int W = 1, int XMODE = 0>  // XMODE: dev experiments (1 skip compute, 2 skip loads)
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(W, 8))) void k_fir_cr(
    const float2 *__restrict__ win, const float2 *x, long long n, float2 *y, const float *__restrict__ hpad,
    int nchunk, float sre, float sim, const float2 *__restrict__ halo, long long tile0)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef cr_geom<R> Gm;
    constexpr int SPR = Gm::SPR;
    constexpr int TL = NT * R;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    f4v *lds = reinterpret_cast<f4v *>(smem);

    const int HP = HC * nchunk;
    const long long t0 = (long long)blockIdx.x * TL;
    const long long gtile = tile0 + blockIdx.x;
    const int nslot = (TL + HP) / 2;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;

    // source of logical slot q (samples t0-HP+2q, +1)
    auto source = [&](int q) -> const float2 * {
        const long long s = t0 - HP + 2 * q;
        if (halo != nullptr && 2 * q < HP && gtile > 0) return halo + gtile * HP + 2 * q;
        if (s < 0) return win + HP + s;
        if (s + 2 > n) return win;             // past the end (patched below when s == n-1)
        return x + s;
    };
    if constexpr (XMODE == 2) {
    } else if constexpr (STAGE == 0) {
        // HBM -> LDS (async), lane-linear destination, swizzle on the source
        for (int base = wave * 64; base < nslot; base += NT) {
            const int p = base + lane;
            const int row = p / SPR;
            const int q = row * SPR + ((p % SPR) ^ ((row / Gm::RPB) & (SPR - 1)));
            if (p < nslot)
                __builtin_amdgcn_global_load_lds((const void *)source(q),
                                                 (__attribute__((address_space(3))) void *)(smem + (size_t)base * 16),
                                                 16, 0, 0);
        }
    } else {
        constexpr int B = 4;
        for (int q0 = threadIdx.x; q0 < nslot; q0 += B * NT) {
            f4v v[B];
#pragma unroll
            for (int b = 0; b < B; b++) {
                const int q = q0 + b * NT;
                if (q < nslot) v[b] = *reinterpret_cast<const f4v *>(source(q));
            }
#pragma unroll
            for (int b = 0; b < B; b++) {
                const int q = q0 + b * NT;
                if (q < nslot) lds[Gm::phys(q / SPR, q % SPR)] = v[b];
            }
        }
    }
    // taps of the first chunk into SGPRs while the tile is in flight (kept out
    // of the FMA loop: a scalar load there would force lgkmcnt(0) waits that
    // also drain the prefetched LDS rows)
    float hr[HC];
#pragma unroll
    for (int k = 0; k < HC; k++) hr[k] = hpad[k];
#pragma unroll
    for (int k = 0; k < HC; k += 16)
        asm volatile("" ::"s"(hr[k]), "s"(hr[k + 1]), "s"(hr[k + 2]), "s"(hr[k + 3]), "s"(hr[k + 4]), "s"(hr[k + 5]),
                     "s"(hr[k + 6]), "s"(hr[k + 7]), "s"(hr[k + 8]), "s"(hr[k + 9]), "s"(hr[k + 10]), "s"(hr[k + 11]),
                     "s"(hr[k + 12]), "s"(hr[k + 13]), "s"(hr[k + 14]), "s"(hr[k + 15]));
    __syncthreads();
    if (t0 + TL > n) {                         // last tile: the slot holding x[n-1] alone
        const long long sl = n - 1 - (t0 - HP);
        if ((sl & 1) == 0 && sl >= 0 && sl / 2 < nslot && threadIdx.x == 0 && !(halo != nullptr && sl < HP && gtile > 0)) {
            const int q = (int)(sl / 2);
            const float2 v = x[n - 1];
            lds[Gm::phys(q / SPR, q % SPR)] = f4v{v.x, v.y, 0.f, 0.f};
        }
        __syncthreads();
    }

    const int l = threadIdx.x;
    auto read_row = [&](int rho, float2 (&w)[R]) {
        rho = rho < 0 ? 0 : rho;
#pragma unroll
        for (int c = 0; c < SPR; c++) {
            const f4v v = lds[Gm::phys(rho, c)];
            w[2 * c] = make_float2(v.x, v.y);
            w[2 * c + 1] = make_float2(v.z, v.w);
        }
    };
    float2 acc[R];
#pragma unroll
    for (int j = 0; j < R; j++) acc[j] = make_float2(0.f, 0.f);
    const int NG = HP / R;
    float2 rn[R], ro[R];
    read_row(NG + l, rn);
    read_row(NG + l - 1, ro);
    for (int c = 0; c < (XMODE == 1 ? 0 : nchunk); c++) {
        if (c > 0) {
#pragma unroll
            for (int k = 0; k < HC; k++) hr[k] = hpad[c * HC + k];
        }
#pragma unroll
        for (int g = 0; g < HC / R; g++) {
            const int G = c * (HC / R) + g;
            float2 nx[R];
            read_row(NG - G + l - 2, nx);
#pragma unroll
            for (int i = 0; i < R; i++) {
                const float hv = hr[g * R + i];
#pragma unroll
                for (int j = 0; j < R; j++) {
                    const int a = R + j - i;          // window index: ro[0..R) ++ rn[0..R)
                    const float2 v = a < R ? ro[a] : rn[a - R];
                    acc[j].x = fmaf(hv, v.x, acc[j].x);
                    acc[j].y = fmaf(hv, v.y, acc[j].y);
                }
            }
#pragma unroll
            for (int j = 0; j < R; j++) {
                rn[j] = ro[j];
                ro[j] = nx[j];
            }
        }
    }

    if constexpr (XMODE == 1) {
#pragma unroll
        for (int j = 0; j < R; j++) acc[j] = j < R / 2 ? rn[j] : ro[j];
    }
    // ---- outputs through LDS (same swizzle) for coalesced 16-byte stores
    __syncthreads();
#pragma unroll
    for (int c = 0; c < SPR; c++) {
        const float2 a0 = acc[2 * c], a1 = acc[2 * c + 1];
        lds[Gm::phys(l, c)] = f4v{a0.x * sre - a0.y * sim, a0.x * sim + a0.y * sre, a1.x * sre - a1.y * sim,
                                  a1.x * sim + a1.y * sre};
    }
    __syncthreads();
    const long long nt = n - t0 < TL ? n - t0 : TL;
    for (int q = threadIdx.x; q < TL / 2; q += NT) {
        if (2 * q >= nt) break;
        const f4v v = lds[Gm::phys(q / SPR, q % SPR)];
        if (2 * q + 2 <= nt) {
            *reinterpret_cast<f4v *>(y + t0 + 2 * q) = v;
        } else {
            y[t0 + 2 * q] = make_float2(v.x, v.y);
        }
    }
}

// ------------------------------------------------------------------ firfilt crcf on the matrix cores
// The FIR as a product of a Toeplitz tap matrix and a matrix of input windows,
// on v_mfma_f32_16x16x4_f32 (exact f32 FMA chains; measured on this chip the
// f32 VALU reaches ~260 G samples/s on h = 64, the f32 MFMA rate is 2x that):
//   D[i][j] = sum_m A[i][m] B[m][j],  i < 16 output offset, j < 16 output block,
//   A[i][m] = h[i + HP - m] (0 <= i+HP-m < HP, else 0),  m < K = HP + 16,
//   B[m][j] = x[base_j - HP + m]  (base_j = first output of block j).
// Lane l holds A[l&15][S*(l>>4)+s] for the S = K/4 MFMA steps (the k index of
// step s, lane group kk = l>>4, is m = S*kk + s, so every lane reads S
// consecutive samples of its window with 16-byte LDS reads), re and im parts
// go through separate MFMAs sharing A.  D lands as 4 consecutive outputs per
// lane (col = l&15, rows 4(l>>4)+r): stored straight to HBM.  The input tile
// reaches LDS by LDS-DMA in the swizzled 16-sample-row layout of k_fir_cr<16>.
template <int HP>
__global__ __launch_bounds__(NT) void k_fir_mfma(const float2 *__restrict__ win, const float2 *x, long long n,
                                                 float2 *y, const float *__restrict__ hpad, float sre, float sim,
                                                 const float2 *__restrict__ halo, long long tile0)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef cr_geom<16> Gm;
    constexpr int SPR = Gm::SPR;
    constexpr int TL = 4096;                    // outputs per workgroup: 4 waves x 4 groups x 256
    constexpr int K = HP + 16;
    constexpr int S = K / 4;
    static_assert(S % 2 == 0, "S must be even");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    f4v *lds = reinterpret_cast<f4v *>(smem);

    const long long t0 = (long long)blockIdx.x * TL;
    const long long gtile = tile0 + blockIdx.x;
    constexpr int nslot = (TL + HP) / 2;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;

    auto source = [&](int q) -> const float2 * {
        const long long s = t0 - HP + 2 * q;
        if (halo != nullptr && 2 * q < HP && gtile > 0) return halo + gtile * HP + 2 * q;
        if (s < 0) return win + HP + s;
        if (s + 2 > n) return win;
        return x + s;
    };
    for (int base = wave * 64; base < nslot; base += NT) {
        const int p = base + lane;
        const int row = p / SPR;
        const int q = row * SPR + ((p % SPR) ^ ((row / Gm::RPB) & (SPR - 1)));
        if (p < nslot)
            __builtin_amdgcn_global_load_lds((const void *)source(q),
                                             (__attribute__((address_space(3))) void *)(smem + (size_t)base * 16), 16,
                                             0, 0);
    }
    // Toeplitz tap fragments while the tile is in flight
    const int ii = lane & 15, kk = lane >> 4;
    float A[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
        const int t = ii + HP - (S * kk + s);
        A[s] = (t >= 0 && t < HP) ? hpad[t] : 0.0f;
    }
    __syncthreads();
    if (t0 + TL > n) {
        const long long sl = n - 1 - (t0 - HP);
        if ((sl & 1) == 0 && sl >= 0 && sl / 2 < nslot && threadIdx.x == 0 && !(halo != nullptr && sl < HP && gtile > 0)) {
            const int q = (int)(sl / 2);
            const float2 v = x[n - 1];
            lds[Gm::phys(q / SPR, q % SPR)] = f4v{v.x, v.y, 0.f, 0.f};
        }
        __syncthreads();
    }

#pragma unroll 1
    for (int g = 0; g < 4; g++) {
        const int G = wave * 4 + g;               // 256-output group of the tile
        const int u0 = 16 * (16 * G + ii) + S * kk; // tile index of this lane's first sample (even)
        float2 b[S];
#pragma unroll
        for (int s = 0; s < S; s += 2) {
            const int q = (u0 + s) >> 1;
            const f4v v = lds[Gm::phys(q / SPR, q % SPR)];
            b[s] = make_float2(v.x, v.y);
            b[s + 1] = make_float2(v.z, v.w);
        }
        f4v dre = {0.f, 0.f, 0.f, 0.f}, dim = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < S; s++) {
            dre = __builtin_amdgcn_mfma_f32_16x16x4f32(A[s], b[s].x, dre, 0, 0, 0);
            dim = __builtin_amdgcn_mfma_f32_16x16x4f32(A[s], b[s].y, dim, 0, 0, 0);
        }
        // lane holds outputs o0..o0+3 of block 16G+ii
        const long long o0 = t0 + 16 * (16 * G + ii) + 4 * kk;
        const f4v lo = f4v{dre[0] * sre - dim[0] * sim, dre[0] * sim + dim[0] * sre, dre[1] * sre - dim[1] * sim,
                           dre[1] * sim + dim[1] * sre};
        const f4v hi = f4v{dre[2] * sre - dim[2] * sim, dre[2] * sim + dim[2] * sre, dre[3] * sre - dim[3] * sim,
                           dre[3] * sim + dim[3] * sre};
        if (o0 + 4 <= n) {
            *reinterpret_cast<f4v *>(y + o0) = lo;
            *reinterpret_cast<f4v *>(y + o0 + 2) = hi;
        } else if (o0 < n) {
            y[o0] = make_float2(lo.x, lo.y);
            if (o0 + 1 < n) y[o0 + 1] = make_float2(lo.z, lo.w);
            if (o0 + 2 < n) y[o0 + 2] = make_float2(hi.x, hi.y);
        }
    }
}

// Persistent form: each workgroup walks tiles b = blockIdx.x, +gridDim.x, ...
// with two LDS tile buffers; the LDS-DMA of tile b+grid is in flight while
// tile b is computed, so HBM streaming and matrix-core work overlap inside
// the workgroup.  TL = outputs per tile (256 per MFMA group, NG groups per wave).
__device__ unsigned long long g_lq_clk[2 * 4096];   // dev experiments: per-workgroup clock samples
template <int HP, int TL, int XMODE = 0>  // XMODE (dev experiments): 1 no MFMA, 2 no DMA, 3 no stores, 4 neither, >=10 clocks
__global__ __launch_bounds__(NT) void k_fir_mfma_p(const float2 *__restrict__ win, const float2 *x, long long n,
                                                   float2 *y, const float *__restrict__ hpad, float sre, float sim,
                                                   const float2 *__restrict__ halo, long long ntiles)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef cr_geom<16> Gm;
    constexpr int SPR = Gm::SPR;
    constexpr int NGW = TL / 256 / 4;            // MFMA groups per wave per tile
    constexpr int K = HP + 16;
    constexpr int S = K / 4;
    constexpr int nslot = (TL + HP) / 2;
    constexpr int BUF = nslot * 16;              // bytes per tile buffer
    static_assert(S % 2 == 0 && NGW >= 1, "shape");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int ii = lane & 15, kk = lane >> 4;

    auto fill = [&](long long b, int buf) {
        const long long t0 = b * TL;
        for (int base = wave * 64; base < nslot; base += NT) {
            const int p = base + lane;
            const int row = p / SPR;
            const int q = row * SPR + ((p % SPR) ^ ((row / Gm::RPB) & (SPR - 1)));
            const long long s = t0 - HP + 2 * q;
            const float2 *src;
            if (halo != nullptr && 2 * q < HP && b > 0) src = halo + b * HP + 2 * q;
            else if (s < 0) src = win + HP + s;
            else if (s + 2 > n) src = win;
            else src = x + s;
            if (p < nslot && XMODE % 10 != 2 && XMODE % 10 != 4)
                __builtin_amdgcn_global_load_lds(
                    (const void *)src, (__attribute__((address_space(3))) void *)(smem + buf * BUF + (size_t)base * 16),
                    16, 0, 0);
        }
    };
    long long b = blockIdx.x;
    if (b >= ntiles) return;
    unsigned long long c0 = 0, r0 = 0;
    if (XMODE >= 10) {
        c0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    fill(b, 0);
    float A[S];
#pragma unroll
    for (int s = 0; s < S; s++) {
        const int t = ii + HP - (S * kk + s);
        A[s] = (t >= 0 && t < HP) ? hpad[t] : 0.0f;
    }
    int cur = 0;
    __syncthreads();
    for (; b < ntiles; b += gridDim.x) {
        const long long t0 = b * TL;
        const long long bn = b + gridDim.x;
        if (bn < ntiles) fill(bn, cur ^ 1);
        f4v *lds = reinterpret_cast<f4v *>(smem + cur * BUF);
        if (t0 + TL > n) {                      // last tile: the slot holding x[n-1] alone
            const long long sl = n - 1 - (t0 - HP);
            if ((sl & 1) == 0 && sl >= 0 && sl / 2 < nslot && threadIdx.x == 0 &&
                !(halo != nullptr && sl < HP && b > 0)) {
                const int q = (int)(sl / 2);
                const float2 v = x[n - 1];
                lds[Gm::phys(q / SPR, q % SPR)] = f4v{v.x, v.y, 0.f, 0.f};
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the patch is visible after the barrier
            __builtin_amdgcn_s_barrier();
        }
#pragma unroll
        for (int g = 0; g < NGW; g++) {
            const int G = wave * NGW + g;
            const int u0 = 16 * (16 * G + ii) + S * kk;
            float2 bv[S];
#pragma unroll
            for (int s = 0; s < S; s += 2) {
                const int q = (u0 + s) >> 1;
                const f4v v = lds[Gm::phys(q / SPR, q % SPR)];
                bv[s] = make_float2(v.x, v.y);
                bv[s + 1] = make_float2(v.z, v.w);
            }
            f4v dre = {0.f, 0.f, 0.f, 0.f}, dim = {0.f, 0.f, 0.f, 0.f};
            if constexpr (XMODE % 10 == 1) {
#pragma unroll
                for (int s = 0; s < S; s++) {
                    dre[s & 3] += bv[s].x;
                    dim[s & 3] += bv[s].y;
                }
            } else {
#pragma unroll
                for (int s = 0; s < S; s++) {
                    dre = __builtin_amdgcn_mfma_f32_16x16x4f32(A[s], bv[s].x, dre, 0, 0, 0);
                    dim = __builtin_amdgcn_mfma_f32_16x16x4f32(A[s], bv[s].y, dim, 0, 0, 0);
                }
            }
            const long long o0 = t0 + 16 * (16 * G + ii) + 4 * kk;
            const f4v lo = f4v{dre[0] * sre - dim[0] * sim, dre[0] * sim + dim[0] * sre, dre[1] * sre - dim[1] * sim,
                               dre[1] * sim + dim[1] * sre};
            const f4v hi = f4v{dre[2] * sre - dim[2] * sim, dre[2] * sim + dim[2] * sre, dre[3] * sre - dim[3] * sim,
                               dre[3] * sim + dim[3] * sre};
            if (XMODE % 10 == 3 || XMODE % 10 == 4) {
                if (lo.x == 1234.5f && hi.y == 77.f) y[0] = make_float2(lo.y, hi.x);
            } else if (o0 + 4 <= n) {
                *reinterpret_cast<f4v *>(y + o0) = lo;
                *reinterpret_cast<f4v *>(y + o0 + 2) = hi;
            } else if (o0 < n) {
                y[o0] = make_float2(lo.x, lo.y);
                if (o0 + 1 < n) y[o0 + 1] = make_float2(lo.z, lo.w);
                if (o0 + 2 < n) y[o0 + 2] = make_float2(hi.x, hi.y);
            }
        }
        __syncthreads();                        // next tile landed; everyone is done with this one
        cur ^= 1;
    }
    if (XMODE >= 10 && threadIdx.x == 0 && blockIdx.x < 4096) {
        g_lq_clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        g_lq_clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

// Warp-specialised persistent form: NP producer waves only issue the LDS-DMA
// of tiles into a ring of D buffers (their vector-memory counter then holds
// nothing but those copies, so a counted vmcnt retires exactly one tile) and
// NC consumer waves only read LDS, run the MFMAs and store; one workgroup
// barrier per tile hands a landed buffer to the consumers and a drained one
// back to the producers.  TL = 256 * NC * GPW outputs per tile.
template <int HP, int NC, int GPW, int D, int NP>
__global__ __launch_bounds__(64 * (NC + NP)) void k_fir_mfma_ws(const float2 *__restrict__ win, const float2 *x,
                                                                long long n, float2 *y,
                                                                const float *__restrict__ hpad, float sre,
                                                                float sim, const float2 *__restrict__ halo,
                                                                long long ntiles)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef cr_geom<16> Gm;
    constexpr int SPR = Gm::SPR;
    constexpr int TL = 256 * NC * GPW;
    constexpr int K = HP + 16;
    constexpr int S = K / 4;
    constexpr int nslot = (TL + HP) / 2;
    constexpr int NINST = (nslot + 64 * NP - 1) / (64 * NP);   // DMA instructions per producer wave per tile
    constexpr int BUF = NINST * NP * 64 * 16;                  // bytes per ring buffer (whole DMA instructions)
    constexpr int VMC = (D - 2) * NINST;                        // tiles that may stay in flight
    static_assert(S % 2 == 0 && D >= 2 && VMC <= 63, "shape");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const bool producer = wave >= NC;
    const int pw = wave - NC;

    const long long b0 = blockIdx.x;
    const long long G = gridDim.x;
    if (b0 >= ntiles) return;
    const long long nmine = (ntiles - b0 + G - 1) / G;   // tiles of this workgroup

    // producer wave pw: its NINST DMA instructions for the k-th tile of this
    // workgroup (dummy copies past the last tile keep the count per tile fixed)
    auto fill = [&](long long k) {
        const bool real = k < nmine;
        const long long b = b0 + k * G;
        const long long t0 = b * TL;
        unsigned char *dbuf = smem + (size_t)(k % D) * BUF;
        const unsigned long long wdummy = (unsigned long long)win;
#pragma unroll
        for (int it = 0; it < NINST; it++) {
            const int base = (it * NP + pw) * 64;
            const int p = base + lane;
            const int row = p / SPR;
            const int q = row * SPR + ((p % SPR) ^ ((row / Gm::RPB) & (SPR - 1)));
            const long long s = t0 - HP + 2 * q;
            // branch-free source select (a branch here makes the compiler
            // drain the vector-memory counter around every copy)
            unsigned long long src = (unsigned long long)(x + s);
            src = (s + 2 > n) ? wdummy : src;
            src = (s < 0) ? (unsigned long long)(win + HP + s) : src;
            src = (halo != nullptr && 2 * q < HP && b > 0) ? (unsigned long long)(halo + b * HP + 2 * q) : src;
            src = (!real || p >= nslot) ? wdummy : src;
            __builtin_amdgcn_global_load_lds((const void *)src,
                                             (__attribute__((address_space(3))) void *)(dbuf + (size_t)base * 16), 16,
                                             0, 0);
        }
    };

    // every ordinary global load happens here, drained before the first copy
    const float2 xlast = x[n - 1];
    float A[S];
    {
        const int ii = lane & 15, kk = lane >> 4;
#pragma unroll
        for (int s = 0; s < S; s++) {
            const int t = ii + HP - (S * kk + s);
            const float v = hpad[t < 0 ? 0 : (t >= HP ? HP - 1 : t)];
            A[s] = (t >= 0 && t < HP) ? v : 0.0f;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (producer) {
        for (long long k = 0; k < D - 1; k++) fill(k);
    }
    for (long long k = 0; k < nmine; k++) {
        const long long b = b0 + k * G;
        const long long t0 = b * TL;
        if (producer) // tile k landed; tiles k+1 .. k+D-2 may stay in flight
            __builtin_amdgcn_s_waitcnt((VMC & 15) | (7 << 4) | ((VMC >> 4) << 14));
        __builtin_amdgcn_s_barrier();
        if (t0 + TL > n) {                               // last tile: the slot holding x[n-1] alone
            const long long sl = n - 1 - (t0 - HP);
            if ((sl & 1) == 0 && sl >= 0 && sl / 2 < nslot && !(halo != nullptr && sl < HP && b > 0) &&
                threadIdx.x == 0) {
                const int q = (int)(sl / 2);
                reinterpret_cast<f4v *>(smem + (size_t)(k % D) * BUF)[Gm::phys(q / SPR, q % SPR)] =
                    f4v{xlast.x, xlast.y, 0.f, 0.f};
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);           // lgkmcnt(0)
            __builtin_amdgcn_s_barrier();
        }
        if (producer) {
            fill(k + D - 1);                             // the buffer of tile k-1 is free now
        } else {
            const f4v *lds = reinterpret_cast<const f4v *>(smem + (size_t)(k % D) * BUF);
            const int ii = lane & 15, kk = lane >> 4;
#pragma unroll
            for (int g = 0; g < GPW; g++) {
                const int Gi = wave * GPW + g;
                const int u0 = 16 * (16 * Gi + ii) + S * kk;
                float2 bv[S];
#pragma unroll
                for (int s = 0; s < S; s += 2) {
                    const int q = (u0 + s) >> 1;
                    const f4v v = lds[Gm::phys(q / SPR, q % SPR)];
                    bv[s] = make_float2(v.x, v.y);
                    bv[s + 1] = make_float2(v.z, v.w);
                }
                f4v dre = {0.f, 0.f, 0.f, 0.f}, dim = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < S; s++) {
                    dre = __builtin_amdgcn_mfma_f32_16x16x4f32(A[s], bv[s].x, dre, 0, 0, 0);
                    dim = __builtin_amdgcn_mfma_f32_16x16x4f32(A[s], bv[s].y, dim, 0, 0, 0);
                }
                const long long o0 = t0 + 16 * (16 * Gi + ii) + 4 * kk;
                const f4v lo = f4v{dre[0] * sre - dim[0] * sim, dre[0] * sim + dim[0] * sre,
                                   dre[1] * sre - dim[1] * sim, dre[1] * sim + dim[1] * sre};
                const f4v hi = f4v{dre[2] * sre - dim[2] * sim, dre[2] * sim + dim[2] * sre,
                                   dre[3] * sre - dim[3] * sim, dre[3] * sim + dim[3] * sre};
                if (o0 + 4 <= n) {
                    *reinterpret_cast<f4v *>(y + o0) = lo;
                    *reinterpret_cast<f4v *>(y + o0 + 2) = hi;
                } else if (o0 < n) {
                    y[o0] = make_float2(lo.x, lo.y);
                    if (o0 + 1 < n) y[o0 + 1] = make_float2(lo.z, lo.w);
                    if (o0 + 2 < n) y[o0 + 2] = make_float2(hi.x, hi.y);
                }
            }
        }
    }
    if (producer) __builtin_amdgcn_s_waitcnt(0);           // drain the trailing dummy copies
}

} // namespace
