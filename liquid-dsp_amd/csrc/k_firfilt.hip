// k_firfilt.hip -- streaming FIR kernels: firfilt, firdecim, firinterp, the
// per-sample single-output path, and window (history) maintenance.
//
// Reference semantics restated (not translated):
//   firfilt  src/filter/src/firfilt.c:297-359  y[t] = scale * sum_k h[k] x[t-k]
//   firdecim src/filter/src/firdecim.c:189-223 y[o] = sum_k h[k] x[o*M - k]
//   firinterp src/filter/src/firinterp.c:187-215 via firpfb.c:325-345
//            y[i*M+p] = sum_l h'[p + l*M] x[i - l]
// The reference walks a ring buffer one sample at a time; here every output is
// independent: a workgroup stages one contiguous input tile (plus the h-1
// sample halo) in LDS once, and each lane produces R consecutive outputs from
// a sliding register window, with the coefficients in scalar registers
// (uniform across the wave), so the inner loop is pure FMA.
#include "lq_device.h"
#include "lq_kernels.h"

#include <cstdint>

namespace {

constexpr int NT = 256;      // threads per workgroup
constexpr int R = 16;        // consecutive outputs per lane
constexpr int TILE = NT * R; // outputs per workgroup

template <int KIND>
struct kt;
template <>
struct kt<0> {
    typedef float T;
    typedef float TC;
};
template <>
struct kt<1> {
    typedef float2 T;
    typedef float TC;
};
template <>
struct kt<2> {
    typedef float2 T;
    typedef float2 TC;
};

template <typename T>
__device__ __forceinline__ T zero();
template <>
__device__ __forceinline__ float zero<float>() { return 0.0f; }
template <>
__device__ __forceinline__ float2 zero<float2>() { return make_float2(0.0f, 0.0f); }

// acc += h * v for the three type combinations
__device__ __forceinline__ void mac(float &acc, float h, float v) { acc = fmaf(h, v, acc); }
__device__ __forceinline__ void mac(float2 &acc, float h, float2 v)
{
    acc.x = fmaf(h, v.x, acc.x);
    acc.y = fmaf(h, v.y, acc.y);
}
__device__ __forceinline__ void mac(float2 &acc, float2 h, float2 v)
{
    acc.x = fmaf(h.x, v.x, acc.x);
    acc.x = fmaf(-h.y, v.y, acc.x);
    acc.y = fmaf(h.x, v.y, acc.y);
    acc.y = fmaf(h.y, v.x, acc.y);
}

__device__ __forceinline__ float apply_scale(float a, float sre, float) { return a * sre; }
__device__ __forceinline__ float2 apply_scale(float2 a, float sre, float sim)
{
    return make_float2(a.x * sre - a.y * sim, a.x * sim + a.y * sre);
}
__device__ __forceinline__ float2 apply_scale_real(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// output scale as the reference applies it (firfilt.c:337, firpfb.c:343,
// `*y *= scale`): a real scale (rrrf / crcf) multiplies each component, a
// complex one (cccf) is a complex product -- they differ for Inf samples
template <int KIND, typename T>
__device__ __forceinline__ T oscale(T a, float sre, float sim)
{
    if constexpr (KIND == 2) return apply_scale(a, sre, sim);
    else if constexpr (sizeof(T) == 8) return apply_scale_real(a, sre);
    else return a * sre;
}

__device__ __forceinline__ float vadd(float a, float b) { return a + b; }
__device__ __forceinline__ float2 vadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }

// LDS image of a sample tile: rows of 16 samples followed by 16 bytes of pad.
// Lanes whose windows start 16 samples apart then hit disjoint bank sets on
// every ds_read_b128 (complex: 36-dword row pitch; real: 20-dword pitch), and
// every 16-byte vector of samples stays 16-byte aligned.
template <typename T>
__host__ __device__ __forceinline__ int lds_off(int u) // in bytes
{
    return u * (int)sizeof(T) + 16 * (u >> 4);
}
template <typename T>
__host__ __device__ __forceinline__ int lds_bytes(int nsamp)
{
    return lds_off<T>(nsamp) + 16;
}

template <typename T>
struct vec16;
template <>
struct vec16<float> {
    static constexpr int N = 4;
};
template <>
struct vec16<float2> {
    static constexpr int N = 2;
};

// 16-byte vector of samples
template <typename T>
__device__ __forceinline__ void load16(const T *p, T (&o)[vec16<T>::N])
{
    const float4 v = *reinterpret_cast<const float4 *>(p);
    if constexpr (sizeof(T) == 8) {
        o[0] = make_float2(v.x, v.y);
        o[1] = make_float2(v.z, v.w);
    } else {
        o[0] = v.x;
        o[1] = v.y;
        o[2] = v.z;
        o[3] = v.w;
    }
}
template <typename T>
__device__ __forceinline__ float4 pack16(const T (&o)[vec16<T>::N])
{
    if constexpr (sizeof(T) == 8) return make_float4(o[0].x, o[0].y, o[1].x, o[1].y);
    else return make_float4(o[0], o[1], o[2], o[3]);
}

// ------------------------------------------------------------------ firfilt
// Grid: one workgroup per TILE outputs.  LDS holds samples [t0-HP, t0+TILE).
// Lane tid computes outputs t0 + R*tid + r (r < R) with the R x HC tap block
// fully unrolled: coefficients are wave-uniform (scalar loads / SGPR
// operands), window samples come from LDS 16 bytes at a time, one row of 16
// samples per 16-tap group, so the inner body is pure FMA.  Outputs are
// transposed back through LDS and written with coalesced 16-byte stores.
// `win` = the previous HP samples (oldest first); ext[t<0] = win[HP + t].
template <int KIND, int HC>
__global__ __launch_bounds__(NT) void k_firfilt(const typename kt<KIND>::T *__restrict__ win,
                                                const typename kt<KIND>::T *x, long long n,
                                                typename kt<KIND>::T *y,
                                                const typename kt<KIND>::TC *__restrict__ hpad,
                                                int nchunk, float sre, float sim,
                                                const typename kt<KIND>::T *__restrict__ halo, int hexact)
{
    typedef typename kt<KIND>::T T;
    typedef typename kt<KIND>::TC TC;
    constexpr int VE = vec16<T>::N;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

    const int HP = HC * nchunk;
    const long long t0 = (long long)blockIdx.x * TILE;
    const int S = TILE + HP;

    // hexact = hlen when the taps are zero padded (hlen < HP): a padded zero
    // tap times an Inf / NaN sample would put NaN into outputs the reference
    // (firfilt.c:322-338, hlen taps) keeps finite, so a tile holding a
    // non-finite sample runs the exact loop over the true taps instead
    bool bad = false;
    if (halo == nullptr && ((reinterpret_cast<uintptr_t>(x) & 15) == 0) && n * (long long)sizeof(T) < (1ll << 31)) {
        // four 16-byte loads per lane in flight through a range-checked
        // descriptor (zeros past n, and before x: the first tile then takes
        // those samples from the history) -- the branchy per-vector loop
        // below waited for one load latency per iteration
        const __amdgpu_buffer_rsrc_t rx =
            __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)(n * (long long)sizeof(T)), 0x00020000);
        constexpr int NV = 4;
        for (int e0 = threadIdx.x; e0 < S / VE; e0 += NV * NT) {
            float4 pv[NV];
#pragma unroll
            for (int k = 0; k < NV; k++) {
                const long long s = t0 - HP + (long long)(e0 + k * NT) * VE;
                pv[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                       rx, (unsigned)(s * (long long)sizeof(T)), 0, 0));
            }
#pragma unroll
            for (int k = 0; k < NV; k++) {
                const int e = e0 + k * NT;
                if (e >= S / VE) break;
                const int u = e * VE;
                const long long s = t0 - HP + u;
                if (s < 0) {
                    T o[VE];
                    load16(win + HP + s, o);
                    pv[k] = pack16(o);
                }
                if (hexact) bad |= !(isfinite(pv[k].x) && isfinite(pv[k].y) && isfinite(pv[k].z) && isfinite(pv[k].w));
                *reinterpret_cast<float4 *>(smem + lds_off<T>(u)) = pv[k];
            }
        }
    } else {
        for (int e = threadIdx.x; e < S / VE; e += NT) {
            const int u = e * VE;
            const long long s = t0 - HP + u;
            T o[VE];
            if (s < 0) {
                load16(win + HP + s, o);
            } else if (halo != nullptr && u < HP && blockIdx.x > 0) {
                load16(halo + (size_t)blockIdx.x * HP + u, o);
            } else if (s + VE <= n) {
                load16(x + s, o);
            } else {
#pragma unroll
                for (int i = 0; i < VE; i++) o[i] = (s + i < n) ? x[s + i] : zero<T>();
            }
            const float4 pv = pack16(o);
            if (hexact) bad |= !(isfinite(pv.x) && isfinite(pv.y) && isfinite(pv.z) && isfinite(pv.w));
            *reinterpret_cast<float4 *>(smem + lds_off<T>(u)) = pv;
        }
    }
    const bool exact = hexact ? __syncthreads_or(bad) : (__syncthreads(), false);

    T acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = zero<T>();

    if (exact) {
        for (int r = 0; r < R; r++) {
            const int u = HP + R * threadIdx.x + r;
            T a = zero<T>();
            for (int k = 0; k < hexact; k++) mac(a, hpad[k], *reinterpret_cast<const T *>(smem + lds_off<T>(u - k)));
            acc[r] = a;
        }
    }
    for (int c = 0; c < (exact ? 0 : nchunk); c++) {
        const TC *hc = hpad + c * HC;
        // window sample a' (0 <= a' < HC+R) of this chunk is tile sample
        // u = R*tid + HP - c*HC - HC + a'  (a row start when a' % 16 == 0)
        const int row0 = threadIdx.x + ((HP - c * HC - HC) >> 4);
        const unsigned char *rb = smem + lds_off<T>(16 * row0);
        T v[HC + R];
        // newest row first: a' in [HC, HC+16)
#pragma unroll
        for (int i = 0; i < 16 / VE; i++) {
            T o[VE];
            load16(reinterpret_cast<const T *>(rb + lds_off<T>(HC + i * VE)), o);
#pragma unroll
            for (int k = 0; k < VE; k++) v[HC + i * VE + k] = o[k];
        }
#pragma unroll
        for (int g = 0; g < HC / 16; g++) {
            // bring in the next older row: a' in [HC-16g-16, HC-16g)
#pragma unroll
            for (int i = 0; i < 16 / VE; i++) {
                const int a = HC - 16 * g - 16 + i * VE;
                T o[VE];
                load16(reinterpret_cast<const T *>(rb + lds_off<T>(a)), o);
#pragma unroll
                for (int k = 0; k < VE; k++) v[a + k] = o[k];
            }
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const TC hv = hc[16 * g + j];
#pragma unroll
                for (int r = 0; r < R; r++) mac(acc[r], hv, v[r - (16 * g + j) + HC]);
            }
        }
    }

    // transpose through LDS for coalesced stores
    __syncthreads();
#pragma unroll
    for (int i = 0; i < R / VE; i++) {
        T o[VE];
#pragma unroll
        for (int k = 0; k < VE; k++) o[k] = oscale<KIND>(acc[i * VE + k], sre, sim);
        *reinterpret_cast<float4 *>(smem + lds_off<T>(R * threadIdx.x + i * VE)) = pack16(o);
    }
    __syncthreads();
    const long long nt = n - t0 < TILE ? n - t0 : TILE;
    for (int e = threadIdx.x; e < TILE / VE; e += NT) {
        const int u = e * VE;
        if (u >= nt) break;
        const float4 val = *reinterpret_cast<const float4 *>(smem + lds_off<T>(u));
        if (u + VE <= nt) {
            *reinterpret_cast<float4 *>(y + t0 + u) = val;
        } else {
            T o[VE];
            load16(reinterpret_cast<const T *>(smem + lds_off<T>(u)), o);
            for (int k = 0; k < VE && u + k < nt; k++) y[t0 + u + k] = o[k];
        }
    }
}

// firpfb_execute(i): y = scale * sum_n hpoly[i*L + n] win[L-1-n] (win oldest first)
template <int KIND>
__global__ void k_firpfb_single(const typename kt<KIND>::TC *__restrict__ hpoly, int L, int i,
                                const typename kt<KIND>::T *__restrict__ win, float sre, float sim,
                                typename kt<KIND>::T *y, unsigned *flag, unsigned seq)
{
    typedef typename kt<KIND>::T T;
    __shared__ T part[64];
    T acc = zero<T>();
    for (int k = threadIdx.x; k < L; k += 64) mac(acc, hpoly[(size_t)i * L + k], win[L - 1 - k]);
    part[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T s = zero<T>();
        for (int t = 0; t < 64; t++) s = vadd(s, part[t]);
        y[0] = oscale<KIND>(s, sre, sim);
        lq_signal(flag, seq);
    }
}

template <int KIND>
__global__ void k_halo_copy(const typename kt<KIND>::T *x, long long n, int HP, long long ntiles, int tile,
                            typename kt<KIND>::T *halo)
{
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long tot = ntiles * HP;
    if (i >= tot) return;
    long long tl = i / HP;
    int u = (int)(i - tl * HP);
    if (tl == 0) return;
    long long s = tl * tile - HP + u;
    halo[i] = (s >= 0 && s < n) ? x[s] : zero<typename kt<KIND>::T>();
}

// dst[i] = last L samples of (src ++ x[0..n))
template <typename T>
__global__ void k_window_append(const T *__restrict__ src, int L, const T *__restrict__ x, long long n,
                                T *__restrict__ dst)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= L) return;
    long long j = (long long)i + n; // index into (src ++ x)
    dst[i] = (j < L) ? src[j] : x[j - L];
}

// one output from the window (oldest first, HP samples): y = scale*sum_k h[k] win[HP-1-k]
template <int KIND>
__global__ void k_fir_single(const typename kt<KIND>::TC *__restrict__ hpad, int HP, int hlen,
                             const typename kt<KIND>::T *__restrict__ win, float sre, float sim,
                             typename kt<KIND>::T *y, unsigned *flag, unsigned seq)
{
    typedef typename kt<KIND>::T T;
    __shared__ T part[64];
    T acc = zero<T>();
    for (int k = threadIdx.x; k < hlen; k += 64) mac(acc, hpad[k], win[HP - 1 - k]);
    part[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T s = zero<T>();
        for (int i = 0; i < 64; i++) s = vadd(s, part[i]);
        y[0] = oscale<KIND>(s, sre, sim);
        lq_signal(flag, seq);
    }
}

// ------------------------------------------------------------------ firdecim
// one output per lane; LDS tile covers [o0*M - (HP-1), (o0+NT)*M)
template <int KIND>
__global__ __launch_bounds__(NT) void k_firdecim(const typename kt<KIND>::T *__restrict__ hist,
                                                 const typename kt<KIND>::T *__restrict__ x,
                                                 long long nout, int M,
                                                 typename kt<KIND>::T *__restrict__ y,
                                                 const typename kt<KIND>::TC *__restrict__ hpad,
                                                 int HP, int hlen)
{
    typedef typename kt<KIND>::T T;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T *tile = reinterpret_cast<T *>(smem);
    const long long o0 = (long long)blockIdx.x * NT;
    const long long s0 = o0 * M - (HP - 1);
    const int S = NT * M + HP - 1;
    const long long nin = nout * M;
    for (int u = threadIdx.x; u < S; u += NT) {
        long long s = s0 + u;
        T v;
        if (s < 0) v = hist[HP - 1 + s];
        else if (s < nin) v = x[s];
        else v = zero<T>();
        tile[u] = v;
    }
    __syncthreads();
    const long long o = o0 + threadIdx.x;
    if (o >= nout) return;
    // newest sample of output o is x[o*M] -> tile index (HP-1) + threadIdx.x*M
    const T *w = tile + (HP - 1) + threadIdx.x * M;
    T acc = zero<T>();
    for (int k = 0; k < hlen; k++) mac(acc, hpad[k], w[-k]);
    y[o] = acc;
}

// Phase-layout decimator.  With the filter padded to QC*M taps and split
// k = q*M + r, output o is
//     y[o] = sum_r sum_q hq[r*QC + q] x[(o - q)*M - r],   hq[r*QC + q] = h[q*M + r],
// i.e. M short filters, filter r running over input phase (-r mod M) at the
// output rate.  The workgroup stages its input tile in LDS de-interleaved by
// phase, P[ph][j] = tile[j*M + ph], one padded row per phase; lane t produces
// R consecutive outputs, sliding a QCT+R-1 register window along each phase
// row with the taps wave-uniform (scalar loads), so a phase costs QCT+R-1 LDS
// reads for QCT*R multiply-adds.  Row element j sits at j + (j >> 5): lanes R
// elements apart then spread over all banks.
// Tile: outputs [o0, o0+TO), TO = NT*R; tile sample u = input s0 + u with
// s0 = o0*M - QC*M + 1, u = j*M + ph for j < TO + QC - 1.
__host__ __device__ __forceinline__ int dph_pitch(int J) { return J + (J >> 5) + 1; }
__device__ __forceinline__ int dph_col(int j) { return j + (j >> 5); }

template <int KIND, int QCT, int R, int NT_>
__global__ __launch_bounds__(NT_) void k_firdecim_ph(const typename kt<KIND>::T *__restrict__ hist, int hl1,
                                                     const typename kt<KIND>::T *__restrict__ x, long long nout,
                                                     int M, int QC, typename kt<KIND>::T *__restrict__ y,
                                                     const typename kt<KIND>::TC *__restrict__ hq)
{
    typedef typename kt<KIND>::T T;
    typedef typename kt<KIND>::TC TC;
    constexpr int TO = NT_ * R;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T *P = reinterpret_cast<T *>(smem);
    const int J = TO + QC - 1;
    const int pitch = dph_pitch(J);
    const long long o0 = (long long)blockIdx.x * TO;
    const long long nin = nout * M;
    // stage: aligned start s0 - 1 (o0*M and QC*M are multiples of 4), tile
    // sample u = v - 1
    const long long sa = o0 * M - (long long)QC * M;
    const int S = J * M + 1;
    constexpr int VW = 16 / (int)sizeof(T);
    const bool vec_ok = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    for (int v0 = threadIdx.x * VW; v0 < S; v0 += NT_ * VW) {
        const long long s = sa + v0;
        T e[VW];
        if (vec_ok && s >= 0 && s + VW <= nin) {
            load16<T>(x + s, e);
        } else {
#pragma unroll
            for (int i = 0; i < VW; i++) {
                const long long si = s + i;
                T val = zero<T>();
                if (si < 0) {
                    if (si >= -(long long)hl1) val = hist[hl1 + si];
                } else if (si < nin) {
                    val = x[si];
                }
                e[i] = val;
            }
        }
#pragma unroll
        for (int i = 0; i < VW; i++) {
            const int u = v0 + i - 1;
            if (u >= 0 && u < S - 1) {
                const int j = u / M, ph = u - j * M;
                P[ph * pitch + dph_col(j)] = e[i];
            }
        }
    }
    __syncthreads();
    T acc[R];
#pragma unroll
    for (int rr = 0; rr < R; rr++) acc[rr] = zero<T>();
    const int tb = threadIdx.x * R;
    for (int ph = 0; ph < M; ph++) {
        const T *row = P + ph * pitch;
        const TC *hr = hq + (M - 1 - ph) * QC;
        for (int c = 0; c < QC; c += QCT) {
            const int base = tb + QC - c - QCT; // window start of this tap chunk
            T w[QCT + R - 1];
#pragma unroll
            for (int i = 0; i < QCT + R - 1; i++) w[i] = row[dph_col(base + i)];
#pragma unroll
            for (int q = 0; q < QCT; q++) {
                const TC h = hr[c + q];
#pragma unroll
                for (int rr = 0; rr < R; rr++) mac(acc[rr], h, w[QCT - 1 + rr - q]);
            }
        }
    }
    const long long o = o0 + tb;
#pragma unroll
    for (int rr = 0; rr < R; rr++)
        if (o + rr < nout) y[o + rr] = acc[rr];
}

// Phase-layout decimator, second form: R consecutive outputs per lane (R =
// 2 as launched) and taps in chunks of four (QC a multiple of 4 instead of
// 4/8/16/32: the M = 8, m = 8 filter has 17 taps per phase, padded to 20
// rather than 32).  Each phase row is stored de-interleaved by R (column j
// at (j mod R) Q + j / R), so the window reads of a wave -- lanes R outputs
// apart -- are consecutive (conflict-free) and a lane's R + 3 window samples
// per tap chunk serve 4 R multiply-adds.  The staging issues four 16-byte
// loads per lane before any LDS store and divides by M with a float
// reciprocal and an exact integer correction.
template <int R>
__host__ __device__ __forceinline__ int dph2_q(int J) { return (J + R - 1) / R + 1; }   // 1/R-row stride (+1 pad)

constexpr int DNU = 4;   // staging loads in flight per lane (8 and 12 measured the same)
template <int KIND, int R, int NT_>
__global__ __launch_bounds__(NT_) void k_firdecim_ph2(const typename kt<KIND>::T *__restrict__ hist, int hl1,
                                                      const typename kt<KIND>::T *__restrict__ x, long long nout,
                                                      int M, int QC, typename kt<KIND>::T *__restrict__ y,
                                                      const typename kt<KIND>::TC *__restrict__ hq)
{
    typedef typename kt<KIND>::T T;
    typedef typename kt<KIND>::TC TC;
    constexpr int TO = NT_ * R;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T *P = reinterpret_cast<T *>(smem);
    const int J = TO + QC - 1;
    const int QR = dph2_q<R>(J), pitch = R * QR + 1;
    const long long o0 = (long long)blockIdx.x * TO;
    const long long nin = nout * M;
    const long long sa = o0 * M - (long long)QC * M;
    const int S = J * M + 1;
    const float rM = 1.0f / (float)M;
    constexpr int VW = 16 / (int)sizeof(T);
    const bool vec_ok = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    auto put = [&](int v0, const T (&e)[VW]) {
#pragma unroll
        for (int i = 0; i < VW; i++) {
            const int u = v0 + i - 1;
            if (u >= 0 && u < S - 1) {
                int j = (int)((float)u * rM);   // u < 2^24: off by at most one
                j -= (j * M > u) ? 1 : 0;
                j += ((j + 1) * M <= u) ? 1 : 0;
                const int ph = u - j * M;
                P[ph * pitch + (j % R) * QR + j / R] = e[i];
            }
        }
    };
    if (vec_ok && nin * (long long)sizeof(T) < (1ll << 31)) {
        // four 16-byte loads per lane in flight at a time through a
        // range-checked descriptor (zeros outside x; sa is a multiple of VW,
        // so a vector never straddles x's start); the history only reaches
        // the first tile
        typedef float v4f_ __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t rx =
            __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)(nin * (long long)sizeof(T)), 0x00020000);
        for (int vb = threadIdx.x * VW; vb < S; vb += DNU * NT_ * VW) {
            T e[DNU][VW];
#pragma unroll
            for (int k = 0; k < DNU; k++) {
                const long long sk = sa + vb + k * NT_ * VW;
                const unsigned off = (unsigned)(sk * (long long)sizeof(T));
                const v4f_ v = __builtin_bit_cast(v4f_, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
                if constexpr (VW == 2) {
                    e[k][0] = make_float2(v.x, v.y);
                    e[k][1] = make_float2(v.z, v.w);
                } else {
                    e[k][0] = v.x;
                    e[k][1] = v.y;
                    e[k][2] = v.z;
                    e[k][3] = v.w;
                }
            }
            if (sa < 0) {   // first tile: samples before the call come from the history
#pragma unroll
                for (int k = 0; k < DNU; k++)
#pragma unroll
                    for (int i = 0; i < VW; i++) {
                        const long long si = sa + vb + k * NT_ * VW + i;
                        if (si < 0 && si >= -(long long)hl1) e[k][i] = hist[hl1 + si];
                    }
            }
#pragma unroll
            for (int k = 0; k < DNU; k++) {
                const int v0 = vb + k * NT_ * VW;
                if (v0 < S) put(v0, e[k]);
            }
        }
    } else {
        for (int v0 = threadIdx.x * VW; v0 < S; v0 += NT_ * VW) {
            const long long s = sa + v0;
            T e[VW];
#pragma unroll
            for (int i = 0; i < VW; i++) {
                const long long si = s + i;
                T val = zero<T>();
                if (si < 0) {
                    if (si >= -(long long)hl1) val = hist[hl1 + si];
                } else if (si < nin) {
                    val = x[si];
                }
                e[i] = val;
            }
            put(v0, e);
        }
    }
    __syncthreads();
    T acc[R];
#pragma unroll
    for (int rr = 0; rr < R; rr++) acc[rr] = zero<T>();
    const int tb = threadIdx.x * R;
    for (int ph = 0; ph < M; ph++) {
        const T *row = P + ph * pitch;
        const TC *hr = hq + (M - 1 - ph) * QC;
        for (int c = 0; c < QC; c += 4) {
            // window columns tb + QC - c - 4 + i, i < R + 3; the base is a
            // multiple of R, so column base + i sits at (i % R) QR + base/R + i/R
            const int bR = (tb + QC - c - 4) / R;
            T w[R + 3];
#pragma unroll
            for (int i = 0; i < R + 3; i++) w[i] = row[(i % R) * QR + bR + i / R];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const TC h = hr[c + q];
#pragma unroll
                for (int rr = 0; rr < R; rr++) mac(acc[rr], h, w[3 + rr - q]);
            }
        }
    }
    const long long o = o0 + tb;
#pragma unroll
    for (int rr = 0; rr < R; rr++)
        if (o + rr < nout) y[o + rr] = acc[rr];
}

// Persistent form of k_firdecim_ph2: each workgroup walks tiles blockIdx.x,
// + gridDim.x, ..., and the next tile's NL 16-byte vectors per lane are
// loaded into registers as soon as this tile's are in LDS, so they are in
// flight during this tile's multiply-adds and stores (the one-shot form
// stages, waits, then computes: its loads and its arithmetic never overlap
// within a workgroup).  16-byte aligned x only.
template <int KIND, int R, int NT_, int NL>
__global__ __launch_bounds__(NT_) void k_firdecim_pf(const typename kt<KIND>::T *__restrict__ hist, int hl1,
                                                     const typename kt<KIND>::T *__restrict__ x, long long nout,
                                                     int M, int QC, typename kt<KIND>::T *__restrict__ y,
                                                     const typename kt<KIND>::TC *__restrict__ hq)
{
    typedef typename kt<KIND>::T T;
    typedef typename kt<KIND>::TC TC;
    typedef float v4f_ __attribute__((ext_vector_type(4)));
    constexpr int TO = NT_ * R;
    constexpr int VW = 16 / (int)sizeof(T);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T *P = reinterpret_cast<T *>(smem);
    const int J = TO + QC - 1;
    const int QR = dph2_q<R>(J), pitch = R * QR + 1;
    const long long nin = nout * M;
    const int S = J * M + 1;
    const float rM = 1.0f / (float)M;
    const long long ntiles = (nout + TO - 1) / TO;
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, (int)(nin * (long long)sizeof(T)), 0x00020000);
    auto load = [&](long long t, v4f_ (&e)[NL]) {
        const long long sa = t * TO * M - (long long)QC * M;
#pragma unroll
        for (int k = 0; k < NL; k++) {
            const long long sk = sa + (threadIdx.x + k * NT_) * VW;
            const unsigned off = (t < ntiles && sk < nin) ? (unsigned)(sk * (long long)sizeof(T)) : 0xFFFFFFF0u;
            e[k] = __builtin_bit_cast(v4f_, __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0));
        }
    };
    v4f_ e[NL];
    long long t = blockIdx.x;
    if (t >= ntiles) return;
    load(t, e);
    for (; t < ntiles; t += gridDim.x) {
        const long long o0 = t * TO;
        const long long sa = o0 * M - (long long)QC * M;
        __syncthreads();   // the previous tile's window reads are done
#pragma unroll
        for (int k = 0; k < NL; k++) {
            const int v0 = (threadIdx.x + k * NT_) * VW;
            T ev[VW];
            if constexpr (VW == 2) {
                ev[0] = make_float2(e[k].x, e[k].y);
                ev[1] = make_float2(e[k].z, e[k].w);
            } else {
                ev[0] = e[k].x;
                ev[1] = e[k].y;
                ev[2] = e[k].z;
                ev[3] = e[k].w;
            }
            if (sa < 0) {   // first tile: samples before the call come from the history
#pragma unroll
                for (int i = 0; i < VW; i++) {
                    const long long si = sa + v0 + i;
                    if (si < 0) ev[i] = si >= -(long long)hl1 ? hist[hl1 + si] : zero<T>();
                }
            }
#pragma unroll
            for (int i = 0; i < VW; i++) {
                const int u = v0 + i - 1;
                if (u >= 0 && u < S - 1) {
                    int j = (int)((float)u * rM);   // u < 2^24: off by at most one
                    j -= (j * M > u) ? 1 : 0;
                    j += ((j + 1) * M <= u) ? 1 : 0;
                    const int ph = u - j * M;
                    P[ph * pitch + (j % R) * QR + j / R] = ev[i];
                }
            }
        }
        if (t + gridDim.x < ntiles) load(t + gridDim.x, e);
        __syncthreads();
        T acc[R];
#pragma unroll
        for (int rr = 0; rr < R; rr++) acc[rr] = zero<T>();
        const int tb = threadIdx.x * R;
        for (int ph = 0; ph < M; ph++) {
            const T *row = P + ph * pitch;
            const TC *hr = hq + (M - 1 - ph) * QC;
            for (int c = 0; c < QC; c += 4) {
                const int bR = (tb + QC - c - 4) / R;
                T w[R + 3];
#pragma unroll
                for (int i = 0; i < R + 3; i++) w[i] = row[(i % R) * QR + bR + i / R];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const TC h = hr[c + q];
#pragma unroll
                    for (int rr = 0; rr < R; rr++) mac(acc[rr], h, w[3 + rr - q]);
                }
            }
        }
        const long long o = o0 + tb;
#pragma unroll
        for (int rr = 0; rr < R; rr++)
            if (o + rr < nout) y[o + rr] = acc[rr];
    }
}

// ------------------------------------------------------------------ firinterp
// one input sample per lane -> M outputs; hpoly[p*L + l] = h'[p + l*M]
template <int KIND>
__global__ __launch_bounds__(NT) void k_firinterp(const typename kt<KIND>::T *__restrict__ hist,
                                                  const typename kt<KIND>::T *__restrict__ x,
                                                  long long n, int M, int L,
                                                  const typename kt<KIND>::TC *__restrict__ hpoly,
                                                  float sre, float sim, typename kt<KIND>::T *__restrict__ y)
{
    typedef typename kt<KIND>::T T;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T *tile = reinterpret_cast<T *>(smem);
    const long long i0 = (long long)blockIdx.x * NT;
    const int S = NT + L - 1;
    for (int u = threadIdx.x; u < S; u += NT) {
        long long s = i0 - (L - 1) + u;
        T v;
        if (s < 0) v = (L > 1) ? hist[L - 1 + s] : zero<T>();
        else if (s < n) v = x[s];
        else v = zero<T>();
        tile[u] = v;
    }
    __syncthreads();
    const long long i = i0 + threadIdx.x;
    if (i >= n) return;
    const T *w = tile + threadIdx.x + (L - 1); // w[-l] = x[i-l]
    for (int p = 0; p < M; p++) {
        T acc = zero<T>();
        for (int l = 0; l < L; l++) mac(acc, hpoly[p * L + l], w[-l]);
        y[i * M + p] = oscale<KIND>(acc, sre, sim);
    }
}

// firinterp crcf/rrrf (real taps), L <= LT taps per phase, M phases: a tile of
// NT inputs in LDS, the phase taps in LDS (read as broadcasts), each lane
// keeps its input's window in registers and forms all M outputs, which go
// back through LDS so that the wave's 64*M outputs leave as contiguous 16-byte
// stores.  Window samples older than the object's L-1 history are zero.
template <int KIND, int LT>
__global__ __launch_bounds__(NT) void k_firinterp_t(const typename kt<KIND>::T *__restrict__ hist,
                                                    const typename kt<KIND>::T *__restrict__ x, long long n,
                                                    int M, int L, const float *__restrict__ hpoly, float sre,
                                                    float sim, typename kt<KIND>::T *__restrict__ y)
{
    typedef typename kt<KIND>::T T;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *tp = reinterpret_cast<float *>(smem);                         // M x LT taps, zero padded
    T *tile = reinterpret_cast<T *>(smem + ((M * LT * 4 + 15) & ~15));  // NT + LT - 1 samples
    T *stage = tile + ((NT + LT - 1 + 3) & ~3);                            // NT * M outputs
    const long long i0 = (long long)blockIdx.x * NT;
    for (int e = threadIdx.x; e < M * LT; e += NT) {
        const int p = e / LT, l = e - p * LT;
        tp[e] = l < L ? hpoly[p * L + l] : 0.0f;
    }
    for (int u = threadIdx.x; u < NT + LT - 1; u += NT) {
        const long long s = i0 - (LT - 1) + u;
        T v = zero<T>();
        if (s >= 0) {
            if (s < n) v = x[s];
        } else if (s >= -(long long)(L - 1)) {
            v = hist[L - 1 + s];
        }
        tile[u] = v;
    }
    __syncthreads();
    T w[LT];   // w[l] = x[i - l]
#pragma unroll
    for (int l = 0; l < LT; l++) w[l] = tile[threadIdx.x + LT - 1 - l];
    T *st = stage + (threadIdx.x >> 6) * 64 * M;   // this wave's outputs, natural order
    const int lane = threadIdx.x & 63;
    for (int p = 0; p < M; p++) {
        const float *hp = tp + p * LT;
        T acc = zero<T>();
#pragma unroll
        for (int l = 0; l < LT; l += 4) {
            const float4 h4 = *reinterpret_cast<const float4 *>(hp + l);
            mac(acc, h4.x, w[l]);
            if (l + 1 < LT) mac(acc, h4.y, w[l + 1]);
            if (l + 2 < LT) mac(acc, h4.z, w[l + 2]);
            if (l + 3 < LT) mac(acc, h4.w, w[l + 3]);
        }
        st[lane * M + p] = oscale<KIND>(acc, sre, sim);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the wave's outputs y[(iw) M .. (iw + 64) M), iw = its first input
    const long long iw = i0 + (threadIdx.x & ~63);
    if (iw >= n) return;
    const long long nin = (n - iw) < 64 ? (n - iw) : 64;
    const int nout = (int)(nin * M);
    constexpr int VE = vec16<T>::N;
    T *yw = y + iw * M;
    for (int e = lane * VE; e < nout; e += 64 * VE) {
        if (e + VE <= nout) {
            // non-temporal: the outputs are not read back (M = 8 m = 8 crcf,
            // 2^27 outputs: 0.270 -> 0.244-0.248 ms, M = 4: 0.314 -> 0.244-0.250,
            // r06fi)
            typedef float v4nt __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(*reinterpret_cast<const v4nt *>(st + e), reinterpret_cast<v4nt *>(yw + e));
        } else {
            for (int k = 0; k < VE && e + k < nout; k++) yw[e + k] = st[e + k];
        }
    }
}

int tile_of(int) { return TILE; }

// dynamic LDS budget of k_firfilt: the 160 KB of a CU minus a margin for the
// kernel's own (static) group segment, which the dispatch adds on top (a
// 163 600-byte request dispatched as 163 856 bytes and faulted)
constexpr size_t FIR_LDS_MAX = 160 * 1024 - 1024;

// the kernel's static group segment (queried once per instantiation)
template <int KIND, int HC>
size_t fir_static_lds()
{
    static const size_t v = [] {
        hipFuncAttributes a;
        LQ_CHECK(hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&k_firfilt<KIND, HC>)));
        return (size_t)a.sharedSizeBytes;
    }();
    return v;
}

// the one rule for both the create-time limit and the launch: dynamic LDS
// within the budget and, with the static segment on top, within the CU's 160 KB
inline bool fir_lds_fits(size_t lds, size_t lds_static)
{
    return lds <= FIR_LDS_MAX && lds + lds_static <= 160 * 1024;
}

template <int KIND, int HC>
void launch_firfilt(const lqk_fir_desc *d, const void *hist, const void *x, long long n, void *y,
                    const void *halo, hipStream_t st)
{
    typedef typename kt<KIND>::T T;
    typedef typename kt<KIND>::TC TC;
    const int HP = HC * (int)d->nchunk;
    const long long ntiles = (n + TILE - 1) / TILE;
    const size_t lds = (size_t)lds_bytes<T>(TILE + HP);
    if (!fir_lds_fits(lds, fir_static_lds<KIND, HC>())) {
        fprintf(stderr, "error: firfilt: filter length %u exceeds the GPU tile limit\n", d->hlen);
        exit(1);
    }
    hipLaunchKernelGGL((k_firfilt<KIND, HC>), dim3((unsigned)ntiles), dim3(NT), lds, st, (const T *)hist,
                       (const T *)x, n, (T *)y, (const TC *)d->hpad, (int)d->nchunk, d->scale_re,
                       d->scale_im, (const T *)halo, (int)d->hlen < HP ? (int)d->hlen : 0);
    LQ_CHECK_LAUNCH();
}

template <int KIND>
void dispatch_firfilt(const lqk_fir_desc *d, const void *hist, const void *x, long long n, void *y,
                      const void *halo, hipStream_t st)
{
    switch (d->hc) {
    case 16: launch_firfilt<KIND, 16>(d, hist, x, n, y, halo, st); break;
    case 32: launch_firfilt<KIND, 32>(d, hist, x, n, y, halo, st); break;
    case 64: launch_firfilt<KIND, 64>(d, hist, x, n, y, halo, st); break;
    default:
        fprintf(stderr, "error: firfilt: invalid chunk class %u\n", d->hc);
        exit(1);
    }
}

size_t elem_size(int kind) { return kind == 0 ? sizeof(float) : sizeof(float2); }

} // namespace

extern "C" unsigned int lqk_firfilt_max_history(int kind)
{
    // the launch rule (fir_lds_fits) for the HC = 64 kernel, which every
    // filter past 32 taps runs; HP a multiple of 64
    const size_t st = kind == 0 ? fir_static_lds<0, 64>() : (kind == 1 ? fir_static_lds<1, 64>() : fir_static_lds<2, 64>());
    unsigned int hp = 0;
    for (;;) {
        const size_t b = kind == 0 ? (size_t)lds_bytes<float>(TILE + hp + 64) : (size_t)lds_bytes<float2>(TILE + hp + 64);
        if (!fir_lds_fits(b, st)) return hp;
        hp += 64;
    }
}

extern "C" size_t lqk_firfilt_scratch_bytes(const lqk_fir_desc *d, unsigned long long n)
{
    const int tl = tile_of(d->kind);
    const long long ntiles = ((long long)n + tl - 1) / tl;
    return (size_t)ntiles * d->hc * d->nchunk * elem_size(d->kind);
}

extern "C" void lqk_firfilt(const lqk_fir_desc *d, const void *hist, const void *x, unsigned long long n,
                            void *y, void *scratch, const lqk_hist_job *job, void *stream)
{
    if (n == 0) return;
    // LQ_FIRFILT_NO_MFMA=1 keeps crcf h<=64 on the VALU kernel (comparisons)
    static int no_mx = -1;
    if (no_mx < 0) no_mx = getenv("LQ_FIRFILT_NO_MFMA") != nullptr;
    if (!no_mx && lqk_firfilt_mx(d, hist, x, n, y, job, stream)) return;
    // the VALU kernel may run in place: the window update reads x first
    if (job && job->dst) lqk_window_append(d->kind != 0, job->src, job->L, job->x, job->n, job->dst, stream);
    hipStream_t st = (hipStream_t)stream;
    const void *halo = nullptr;
    if (x == y) {
        // in place: save each tile's halo before any workgroup overwrites it
        const int HP = (int)(d->hc * d->nchunk);
        const int tl = tile_of(d->kind);
        const long long ntiles = ((long long)n + tl - 1) / tl;
        const long long tot = ntiles * HP;
        const unsigned nb = (unsigned)((tot + 255) / 256);
        if (d->kind == 0)
            hipLaunchKernelGGL(k_halo_copy<0>, dim3(nb), dim3(256), 0, st, (const float *)x, (long long)n, HP,
                               ntiles, tl, (float *)scratch);
        else
            hipLaunchKernelGGL(k_halo_copy<1>, dim3(nb), dim3(256), 0, st, (const float2 *)x, (long long)n, HP,
                               ntiles, tl, (float2 *)scratch);
        LQ_CHECK_LAUNCH();
        halo = scratch;
    }
    switch (d->kind) {
    case 0: dispatch_firfilt<0>(d, hist, x, (long long)n, y, halo, st); break;
    case 1: dispatch_firfilt<1>(d, hist, x, (long long)n, y, halo, st); break;
    case 2: dispatch_firfilt<2>(d, hist, x, (long long)n, y, halo, st); break;
    }
}

extern "C" void lqk_window_append(int is_complex, const void *src_hist, unsigned int L, const void *x,
                                  unsigned long long n, void *dst_hist, void *stream)
{
    if (L == 0) return;
    hipStream_t st = (hipStream_t)stream;
    unsigned nb = (L + 255) / 256;
    if (is_complex)
        hipLaunchKernelGGL(k_window_append<float2>, dim3(nb), dim3(256), 0, st, (const float2 *)src_hist,
                           (int)L, (const float2 *)x, (long long)n, (float2 *)dst_hist);
    else
        hipLaunchKernelGGL(k_window_append<float>, dim3(nb), dim3(256), 0, st, (const float *)src_hist,
                           (int)L, (const float *)x, (long long)n, (float *)dst_hist);
    LQ_CHECK_LAUNCH();
}

extern "C" void lqk_fir_single(const lqk_fir_desc *d, const void *win, void *y, unsigned *flag, unsigned seq,
                               void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    const int HP = (int)(d->hc * d->nchunk);
    switch (d->kind) {
    case 0:
        hipLaunchKernelGGL(k_fir_single<0>, dim3(1), dim3(64), 0, st, (const float *)d->hpad, HP, (int)d->hlen,
                           (const float *)win, d->scale_re, d->scale_im, (float *)y, flag, seq);
        break;
    case 1:
        hipLaunchKernelGGL(k_fir_single<1>, dim3(1), dim3(64), 0, st, (const float *)d->hpad, HP, (int)d->hlen,
                           (const float2 *)win, d->scale_re, d->scale_im, (float2 *)y, flag, seq);
        break;
    case 2:
        hipLaunchKernelGGL(k_fir_single<2>, dim3(1), dim3(64), 0, st, (const float2 *)d->hpad, HP, (int)d->hlen,
                           (const float2 *)win, d->scale_re, d->scale_im, (float2 *)y, flag, seq);
        break;
    }
    LQ_CHECK_LAUNCH();
}

extern "C" void lqk_firdecim(const lqk_fir_desc *d, unsigned int M, const void *hist, const void *x,
                             unsigned long long nout, void *y, void *stream)
{
    if (nout == 0) return;
    hipStream_t st = (hipStream_t)stream;
    const int HP = (int)(d->hc * d->nchunk);
    const unsigned nb = (unsigned)((nout + NT - 1) / NT);
    const size_t lds = (size_t)(NT * M + HP) * elem_size(d->kind);
    if (lds > FIR_LDS_MAX) {
        fprintf(stderr, "error: firdecim: decimation/filter length exceeds the GPU tile limit\n");
        exit(1);
    }
    switch (d->kind) {
    case 0:
        hipLaunchKernelGGL(k_firdecim<0>, dim3(nb), dim3(NT), lds, st, (const float *)hist, (const float *)x,
                           (long long)nout, (int)M, (float *)y, (const float *)d->hpad, HP, (int)d->hlen);
        break;
    case 1:
        hipLaunchKernelGGL(k_firdecim<1>, dim3(nb), dim3(NT), lds, st, (const float2 *)hist, (const float2 *)x,
                           (long long)nout, (int)M, (float2 *)y, (const float *)d->hpad, HP, (int)d->hlen);
        break;
    case 2:
        hipLaunchKernelGGL(k_firdecim<2>, dim3(nb), dim3(NT), lds, st, (const float2 *)hist, (const float2 *)x,
                           (long long)nout, (int)M, (float2 *)y, (const float2 *)d->hpad, HP, (int)d->hlen);
        break;
    }
    LQ_CHECK_LAUNCH();
}

namespace {
template <int KIND, int QCT, int R, int NT_>
void launch_decim_ph(unsigned M, unsigned QC, const void *hq, unsigned hl1, const void *hist, const void *x,
                     long long nout, void *y, size_t lds, hipStream_t st)
{
    typedef typename kt<KIND>::T T;
    typedef typename kt<KIND>::TC TC;
    const long long TO = (long long)NT_ * R;
    const unsigned nb = (unsigned)((nout + TO - 1) / TO);
    hipLaunchKernelGGL((k_firdecim_ph<KIND, QCT, R, NT_>), dim3(nb), dim3(NT_), lds, st, (const T *)hist,
                       (int)hl1, (const T *)x, nout, (int)M, (int)QC, (T *)y, (const TC *)hq);
    LQ_CHECK_LAUNCH();
}

template <int KIND, int QCT>
int decim_ph_shape(unsigned M, unsigned QC, const void *hq, unsigned hl1, const void *hist, const void *x,
                   long long nout, void *y, hipStream_t st)
{
    const size_t es = elem_size(KIND);
    const size_t lds_a = (size_t)M * dph_pitch(256 * 2 + (int)QC - 1) * es;
    const size_t lds_b = (size_t)M * dph_pitch(64 + (int)QC - 1) * es;
    if (lds_a <= 64 * 1024) launch_decim_ph<KIND, QCT, 2, 256>(M, QC, hq, hl1, hist, x, nout, y, lds_a, st);
    else if (lds_b <= FIR_LDS_MAX) launch_decim_ph<KIND, QCT, 1, 64>(M, QC, hq, hl1, hist, x, nout, y, lds_b, st);
    else return -1;
    return 0;
}

template <int KIND>
int decim_ph_qct(unsigned M, unsigned QC, const void *hq, unsigned hl1, const void *hist, const void *x,
                 long long nout, void *y, hipStream_t st)
{
    switch (QC) {
    case 4: return decim_ph_shape<KIND, 4>(M, QC, hq, hl1, hist, x, nout, y, st);
    case 8: return decim_ph_shape<KIND, 8>(M, QC, hq, hl1, hist, x, nout, y, st);
    case 16: return decim_ph_shape<KIND, 16>(M, QC, hq, hl1, hist, x, nout, y, st);
    case 32: return decim_ph_shape<KIND, 32>(M, QC, hq, hl1, hist, x, nout, y, st);
    default:
        if (QC % 16 == 0) return decim_ph_shape<KIND, 16>(M, QC, hq, hl1, hist, x, nout, y, st);
        if (QC % 4 == 0) return decim_ph_shape<KIND, 4>(M, QC, hq, hl1, hist, x, nout, y, st);
        return -1;
    }
}
} // namespace

extern "C" unsigned lqk_firdecim_ph_qc(unsigned M, unsigned hlen)
{
    const unsigned q0 = (hlen + M - 1) / M;
    return (q0 + 3) / 4 * 4;   // k_firdecim_ph2 runs taps in chunks of four
}

namespace {
// The persistent prefetching form (k_firdecim_pf) for 16-byte aligned x: R
// outputs per lane on NTD lanes, TO = R NTD outputs and (TO + QC - 1) M input
// samples per workgroup in LDS; -1 when the shape does not fit it
template <int R, int NTD>
int decim_pf(int kind, unsigned int M, unsigned int QC, const void *hq, unsigned int hl1, const void *hist,
             const void *x, unsigned long long nout, void *y, hipStream_t st)
{
    constexpr int TO2 = R * NTD;
    const int J = TO2 + (int)QC - 1;
    const size_t lds = (size_t)M * (R * dph2_q<R>(J) + 1) * elem_size(kind);
    const int S = J * (int)M + 1;
    const int vw = 16 / (int)elem_size(kind);
    const int nl = (S + NTD * vw - 1) / (NTD * vw);
    if (!((QC % 4) == 0 && lds <= 40 * 1024 && (unsigned long long)(J) * M < (1u << 24) &&
          ((uintptr_t)x & 15) == 0 && nl <= 12 && nout * M * elem_size(kind) < (1ull << 31)))
        return -1;
    const unsigned long long nt = (nout + TO2 - 1) / TO2;
    const int wpc = (int)((160 * 1024) / lds) < 8 ? (int)((160 * 1024) / lds) : 8;
    const unsigned nb = (unsigned)(nt < 256ull * wpc ? nt : 256ull * wpc);
#define LQ_DP(K, NLV)                                                                                      \
    hipLaunchKernelGGL((k_firdecim_pf<K, R, NTD, NLV>), dim3(nb), dim3(NTD), lds, st, (const kt<K>::T *)hist, \
                       (int)hl1, (const kt<K>::T *)x, (long long)nout, (int)M, (int)QC, (kt<K>::T *)y,         \
                       (const kt<K>::TC *)hq);
#define LQ_DPK(K)                                                                                          \
    if (nl <= 5) { LQ_DP(K, 5) } else if (nl <= 9) { LQ_DP(K, 9) } else { LQ_DP(K, 12) }
    switch (kind) {
    case 0: LQ_DPK(0) break;
    case 1: LQ_DPK(1) break;
    default: LQ_DPK(2) break;
    }
#undef LQ_DPK
#undef LQ_DP
    LQ_CHECK_LAUNCH();
    return 0;
}
} // namespace

extern "C" int lqk_firdecim_ph(int kind, unsigned int M, unsigned int QC, const void *hq, unsigned int hl1,
                               const void *hist, const void *x, unsigned long long nout, void *y, void *stream)
{
    if (nout == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    // the persistent form: at M = 8 (m = 8 crcf, 2^27 inputs: 0.304-0.333 ->
    // 0.283-0.286 ms against the one-shot form, r05zf) two outputs per lane
    // on 256 lanes (four per lane on 128: 0.271 -> 0.36 ms); at small M, where
    // the outputs are many and each is M (QC / 4)(R + 3) / R window reads,
    // four per lane on 128 lanes (M = 2 / 3 / 4: 0.468 / 0.337 / 0.303 ->
    // 0.333 / 0.303 / 0.266 ms, r06fd)
    if ((M <= 4 ? decim_pf<4, 128>(kind, M, QC, hq, hl1, hist, x, nout, y, st)
                : decim_pf<2, 256>(kind, M, QC, hq, hl1, hist, x, nout, y, st)) == 0)
        return 0;
    {
        // one-shot form: 512 outputs per workgroup, two per lane, 256 lanes
        constexpr int LQ_D2R = 2, LQ_D2NT = 256;
        constexpr int TO2 = LQ_D2R * LQ_D2NT;
        const int J = TO2 + (int)QC - 1;
        const size_t lds = (size_t)M * (LQ_D2R * dph2_q<LQ_D2R>(J) + 1) * elem_size(kind);
        if ((QC % 4) == 0 && lds <= 64 * 1024 && (unsigned long long)(J) * M < (1u << 24)) {
            const unsigned nb = (unsigned)((nout + TO2 - 1) / TO2);
#define LQ_D2(K)                                                                                          \
    hipLaunchKernelGGL((k_firdecim_ph2<K, LQ_D2R, LQ_D2NT>), dim3(nb), dim3(LQ_D2NT), lds, st, (const kt<K>::T *)hist, (int)hl1, \
                       (const kt<K>::T *)x, (long long)nout, (int)M, (int)QC, (kt<K>::T *)y, (const kt<K>::TC *)hq);
            switch (kind) {
            case 0: LQ_D2(0) break;
            case 1: LQ_D2(1) break;
            default: LQ_D2(2) break;
            }
#undef LQ_D2
            LQ_CHECK_LAUNCH();
            return 0;
        }
    }
    // longer spans (M >= 16 at 2 M m taps): the persistent form on 256-output
    // tiles, one output per lane (M = 16 m = 8: 0.479 -> 0.308 ms; at M = 12
    // the one-shot form above is faster, 0.306 vs 0.366, r06fd)
    if (decim_pf<1, 256>(kind, M, QC, hq, hl1, hist, x, nout, y, st) == 0) return 0;
    switch (kind) {
    case 0: return decim_ph_qct<0>(M, QC, hq, hl1, hist, x, (long long)nout, y, st);
    case 1: return decim_ph_qct<1>(M, QC, hq, hl1, hist, x, (long long)nout, y, st);
    default: return decim_ph_qct<2>(M, QC, hq, hl1, hist, x, (long long)nout, y, st);
    }
}

extern "C" void lqk_firinterp(int kind, const void *hpoly, unsigned int M, unsigned int L, float sre, float sim,
                              const void *hist, const void *x, unsigned long long n, void *y, void *stream)
{
    if (n == 0) return;
    hipStream_t st = (hipStream_t)stream;
    const unsigned nb = (unsigned)((n + NT - 1) / NT);
    // real taps, L <= 32, 16-byte aligned output: the register-window kernel
    if (kind != 2 && L <= 32 && M <= 64 && ((uintptr_t)y & 15) == 0) {
        const int LT = L <= 8 ? 8 : L <= 12 ? 12 : L <= 16 ? 16 : L <= 20 ? 20 : L <= 24 ? 24 : 32;
        const size_t es = elem_size(kind);
        const size_t lds2 = (((size_t)M * LT * 4 + 15) & ~(size_t)15) + (((size_t)NT + LT - 1 + 3) & ~(size_t)3) * es +
                            (size_t)NT * M * es;
        if (lds2 <= 64 * 1024) {
#define LQ_FI(K, LTV)                                                                                             \
    hipLaunchKernelGGL((k_firinterp_t<K, LTV>), dim3(nb), dim3(NT), lds2, st, (const typename kt<K>::T *)hist,     \
                       (const typename kt<K>::T *)x, (long long)n, (int)M, (int)L, (const float *)hpoly, sre, sim, \
                       (typename kt<K>::T *)y)
#define LQ_FI_L(K)                                                                                                \
    switch (LT) {                                                                                                 \
    case 8: LQ_FI(K, 8); break;                                                                                   \
    case 12: LQ_FI(K, 12); break;                                                                                 \
    case 16: LQ_FI(K, 16); break;                                                                                 \
    case 20: LQ_FI(K, 20); break;                                                                                 \
    case 24: LQ_FI(K, 24); break;                                                                                 \
    default: LQ_FI(K, 32); break;                                                                                 \
    }
            if (kind == 0) { LQ_FI_L(0) }
            else { LQ_FI_L(1) }
#undef LQ_FI_L
#undef LQ_FI
            LQ_CHECK_LAUNCH();
            return;
        }
    }
    const size_t lds = (size_t)(NT + L) * elem_size(kind);
    switch (kind) {
    case 0:
        hipLaunchKernelGGL(k_firinterp<0>, dim3(nb), dim3(NT), lds, st, (const float *)hist, (const float *)x,
                           (long long)n, (int)M, (int)L, (const float *)hpoly, sre, sim, (float *)y);
        break;
    case 1:
        hipLaunchKernelGGL(k_firinterp<1>, dim3(nb), dim3(NT), lds, st, (const float2 *)hist, (const float2 *)x,
                           (long long)n, (int)M, (int)L, (const float *)hpoly, sre, sim, (float2 *)y);
        break;
    case 2:
        hipLaunchKernelGGL(k_firinterp<2>, dim3(nb), dim3(NT), lds, st, (const float2 *)hist, (const float2 *)x,
                           (long long)n, (int)M, (int)L, (const float2 *)hpoly, sre, sim, (float2 *)y);
        break;
    }
    LQ_CHECK_LAUNCH();
}

extern "C" void lqk_firpfb_single(int kind, const void *hpoly, unsigned int L, unsigned int i, const void *win,
                                  float sre, float sim, void *y, unsigned *flag, unsigned seq, void *stream)
{
    hipStream_t st = (hipStream_t)stream;
    switch (kind) {
    case 0:
        hipLaunchKernelGGL(k_firpfb_single<0>, dim3(1), dim3(64), 0, st, (const float *)hpoly, (int)L, (int)i,
                           (const float *)win, sre, sim, (float *)y, flag, seq);
        break;
    case 1:
        hipLaunchKernelGGL(k_firpfb_single<1>, dim3(1), dim3(64), 0, st, (const float *)hpoly, (int)L, (int)i,
                           (const float2 *)win, sre, sim, (float2 *)y, flag, seq);
        break;
    case 2:
        hipLaunchKernelGGL(k_firpfb_single<2>, dim3(1), dim3(64), 0, st, (const float2 *)hpoly, (int)L, (int)i,
                           (const float2 *)win, sre, sim, (float2 *)y, flag, seq);
        break;
    }
    LQ_CHECK_LAUNCH();
}
