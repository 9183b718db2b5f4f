// bw_probe.hip -- measured HBM ceilings for bench.py (not part of the
// product library).  Hand-written streaming kernels with 16-byte accesses per
// lane and several loads in flight per lane, run on the caller's buffers:
//
//   copy   1 read : 1 write (plain memcpy shape)              -> measured_copy_GBps
//   read   read only (a reduction kept live by a dead store)  -> measured_read_GBps
//   pat12  firpfbch2 M=1024's memory pattern: a tile of 64 KB / WPC read,
//          twice that written as 16-byte stores, 1 KB contiguous per wave
//          instruction (the analyzer's output form), next tile's loads
//          between the stores                                 -> measured_pfb2_pattern_GBps
//   pat11  firfilt's pattern: a 2048-sample chunk + 64-sample halo read,
//          2048 samples written, chunks dealt grid-stride     -> measured_fir_pattern_GBps
//
// Each probe sweeps a few launch shapes (workgroups per CU, loads in flight,
// store policy) and bench.py reports the best: the rate the box's memory
// system gives that access pattern with no arithmetic.  Timing: every
// variant first launches until `warm_ms` of wall time has passed (clock
// ramp), then `iters` launches between two HIP events, three passes
// interleaved across variants, best pass kept.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

namespace {

// ---- 1:1 copy / read-only, grid-stride over tiles of BS*U 16-byte elements
template <bool RD, int U, int BS, bool NTS>
__global__ __launch_bounds__(BS) void k_copy(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4)
{
    const long long tile = (long long)BS * U, ntile = n4 / tile;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long long t = blockIdx.x; t < ntile; t += gridDim.x) {
        const long long base = t * tile + threadIdx.x;
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(a + base + (long long)u * BS);
        if (RD) {
#pragma unroll
            for (int u = 0; u < U; u++) acc += v[u];
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (NTS) __builtin_nontemporal_store(v[u], b + base + (long long)u * BS);
                else b[base + (long long)u * BS] = v[u];
            }
        }
    }
    if (RD && acc.x == 1234.5f) b[0] = acc;
}

// ---- firpfbch2's 1 read : 2 write tiles (WPC workgroups per CU)
template <int WPC>
__global__ __launch_bounds__(1024 / WPC, WPC) void k_pat12(const f4 *__restrict__ x, f4 *__restrict__ y, int ntiles)
{
    constexpr int NT = 1024 / WPC;
    constexpr int RB = 65536 / WPC;            // bytes read per tile
    constexpr int NL = RB / (NT * 16);         // 16-byte loads per lane per tile (4)
    constexpr int NWAVE = NT / 64;
    constexpr int WB = 2 * RB / NWAVE;         // bytes written per wave per tile
    constexpr int NS = WB / (64 * 16);         // 16-byte stores per lane per tile (8)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = gridDim.x, w = blockIdx.x;
    f4 r[NL];
    auto ld = [&](int tile, int i) -> f4 {
        return tile < ntiles ? __builtin_nontemporal_load(x + (size_t)tile * (RB / 16) + tid + NT * i) : f4{};
    };
#pragma unroll
    for (int i = 0; i < NL; i++) r[i] = ld(w, i);
    for (int t = w; t < ntiles; t += G) {
        f4 c[NL];
#pragma unroll
        for (int i = 0; i < NL; i++) c[i] = r[i];
        const int nt = t + G;
        f4 *q = y + ((size_t)t * 2 * RB + (size_t)wave * WB) / 16;
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const f4 v = c[s % NL] + (float)s;
            __builtin_nontemporal_store(v, q + s * 64 + lane);
            if (s < NL) r[s] = ld(nt, s);
        }
    }
}

// ---- firfilt's 1 read : 1 write chunks (2048 samples + 64-sample halo)
template <int WPC, bool ILV>
__global__ __launch_bounds__(256, WPC) void k_pat11(const f4 *__restrict__ x, f4 *__restrict__ y, long long nch)
{
    const int tid = threadIdx.x;
    const long long G = gridDim.x, w = blockIdx.x;
    const long long cnt = (nch - w + G - 1) / G;
    f4 r[5];
    auto ld = [&](long long k, int i) -> f4 {
        const long long c = w + k * G;
        if (k >= cnt) return f4{};
        if (i < 4) return __builtin_nontemporal_load(x + c * 1024 + tid + 256 * i);
        return (tid < 32 && c > 0) ? __builtin_nontemporal_load(x + c * 1024 - 32 + tid) : f4{};
    };
#pragma unroll
    for (int i = 0; i < 5; i++) r[i] = ld(0, i);
    for (long long k = 0; k < cnt; k++) {
        f4 c[5];
#pragma unroll
        for (int i = 0; i < 5; i++) c[i] = r[i];
        if (!ILV) {
#pragma unroll
            for (int i = 0; i < 5; i++) r[i] = ld(k + 1, i);
        }
        f4 *q = y + (w + k * G) * 1024 + tid;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            __builtin_nontemporal_store(c[i] + c[4], q + 256 * i);
            if (ILV) {
                r[i] = ld(k + 1, i);
                if (i == 3) r[4] = ld(k + 1, 4);
            }
        }
    }
}

struct Var {
    const char *name;
    int kind;         // 0 copy, 1 read, 2 pat12, 3 pat11
    void (*launch)(const void *, void *, long long, hipStream_t);
    double bytes;     // algorithmic bytes per launch
};


template <bool RD, int U, int BS, bool NTS, int WPC>
void l_copy(const void *a, void *b, long long n4, hipStream_t s)
{
    hipLaunchKernelGGL((k_copy<RD, U, BS, NTS>), dim3(256 * WPC), dim3(BS), 0, s, (const f4 *)a, (f4 *)b, n4);
}

template <int WPC>
void l_pat12(const void *a, void *b, long long n4, hipStream_t s)
{
    const int ntiles = (int)(n4 * 16 / (65536 / WPC));
    hipLaunchKernelGGL((k_pat12<WPC>), dim3(256 * WPC), dim3(1024 / WPC), 0, s, (const f4 *)a, (f4 *)b, ntiles);
}

template <int WPC, bool ILV>
void l_pat11(const void *a, void *b, long long n4, hipStream_t s)
{
    hipLaunchKernelGGL((k_pat11<WPC, ILV>), dim3(256 * WPC), dim3(256), 0, s, (const f4 *)a, (f4 *)b, n4 / 1024);
}

} // namespace

// Runs probe `kind` over src (src_bytes, 16-byte aligned) and dst (at least
// 2 * src_bytes for kind 2, src_bytes otherwise) on `stream`.  Writes the best
// rate in GB/s (algorithmic bytes / best average launch time) to *gbps and the
// name of the best launch shape to name (cap bytes).  Returns 0 on success.
extern "C" int bwprobe_run(int kind, const void *src, void *dst, long long src_bytes, void *stream, double warm_ms,
                           int iters, double *gbps, double *best_ms, char *name, int cap)
{
    hipStream_t st = (hipStream_t)stream;
    const long long n4 = src_bytes / 16;
    const double B = (double)src_bytes;
    std::vector<Var> vs;
    if (kind == 0) {
        vs = {{"copy u4 bs256 wpc2 nt", 0, l_copy<false, 4, 256, true, 2>, 2 * B},
              {"copy u4 bs256 wpc4 nt", 0, l_copy<false, 4, 256, true, 4>, 2 * B},
              {"copy u4 bs256 wpc8 nt", 0, l_copy<false, 4, 256, true, 8>, 2 * B},
              {"copy u8 bs512 wpc2 nt", 0, l_copy<false, 8, 512, true, 2>, 2 * B},
              {"copy u4 bs256 wpc4 plain", 0, l_copy<false, 4, 256, false, 4>, 2 * B},
              {"copy u4 bs1024 wpc1 nt", 0, l_copy<false, 4, 1024, true, 1>, 2 * B}};
    } else if (kind == 1) {
        vs = {{"read u4 bs256 wpc4", 1, l_copy<true, 4, 256, true, 4>, B},
              {"read u8 bs512 wpc2", 1, l_copy<true, 8, 512, true, 2>, B},
              {"read u4 bs256 wpc8", 1, l_copy<true, 4, 256, true, 8>, B}};
    } else if (kind == 2) {
        vs = {{"pat12 wpc1 (1024 thr)", 2, l_pat12<1>, 3 * B},
              {"pat12 wpc2 (512 thr)", 2, l_pat12<2>, 3 * B},
              {"pat12 wpc4 (256 thr)", 2, l_pat12<4>, 3 * B}};
    } else if (kind == 3) {
        vs = {{"pat11 wpc2 ilv", 3, l_pat11<2, true>, 2 * B},
              {"pat11 wpc3 ilv", 3, l_pat11<3, true>, 2 * B},
              {"pat11 wpc4 ilv", 3, l_pat11<4, true>, 2 * B},
              {"pat11 wpc3 pre", 3, l_pat11<3, false>, 2 * B}};
    } else {
        return 1;
    }
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 2;
    std::vector<float> best(vs.size(), 1e30f);
    for (int pass = 0; pass < 3; pass++) {
        for (size_t v = 0; v < vs.size(); v++) {
            const auto t0 = std::chrono::steady_clock::now();
            int nw = 0;
            for (;;) {
                for (int i = 0; i < 4; i++) vs[v].launch(src, dst, n4, st);
                nw += 4;
                if (hipStreamSynchronize(st) != hipSuccess) return 3;
                const double el = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                if (nw >= 8 && el >= (pass == 0 ? warm_ms : warm_ms / 4)) break;
            }
            (void)hipEventRecord(e0, st);
            for (int i = 0; i < iters; i++) vs[v].launch(src, dst, n4, st);
            (void)hipEventRecord(e1, st);
            if (hipEventSynchronize(e1) != hipSuccess) return 4;
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            ms /= iters;
            if (ms < best[v]) best[v] = ms;
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    size_t bi = 0;
    for (size_t v = 1; v < vs.size(); v++)
        if (vs[v].bytes / best[v] > vs[bi].bytes / best[bi]) bi = v;
    *gbps = vs[bi].bytes / (best[bi] * 1e-3) / 1e9;
    *best_ms = best[bi];
    if (name && cap > 0) {
        int o = snprintf(name, cap, "%s", vs[bi].name);
        for (size_t v = 0; v < vs.size() && o < cap; v++)
            o += snprintf(name + o, cap - o, "; %s %.4f ms", vs[v].name, best[v]);
    }
    return 0;
}
