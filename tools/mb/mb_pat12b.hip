// mb_pat12b.hip -- firpfbch2 M=1024's 1 read : 2 write memory pattern with the
// kernel's schedule features (dev tool; mb_pat12.hip swept the bare pattern).
// A tile: 64 KB / WPC read (16-byte loads, 4 per lane), twice that written
// (16-byte stores, 1 KB contiguous per wave instruction, 8 per lane); 2^27
// complex samples in, 2^28 out, as the bench's step.  Swept:
//   WPC   workgroups per CU (1024 / WPC threads each)
//   RUN   tiles per contiguous run a workgroup walks (1: grid-stride tiles,
//         0: one contiguous run per workgroup, the kernel's layout)
//   ILV   next tile's loads between this tile's stores (1) or issued right
//         after the loads are consumed (0, the kernel)
//   BAR   a workgroup barrier between consuming the loads and the stores and
//         another after the stores (the kernel's two phase changes)
//   DLY   dependent FMAs per lane between the loads' use and the stores
//         (~ the transform: the kernel spends ~400 VALU per wave per block)
// One line per variant: ms per step (three passes A B C .. A B C) and GB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                                \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int WPC, int RUN, bool ILV, bool BAR, int DLY>
__global__ __launch_bounds__(1024 / WPC, WPC) void k_pat(const f4 *__restrict__ x, f4 *__restrict__ y, int ntiles)
{
    constexpr int NT = 1024 / WPC;
    constexpr int RB = 65536 / WPC;            // bytes read per tile
    constexpr int NL = RB / (NT * 16);         // 4
    constexpr int NWAVE = NT / 64;
    constexpr int WB = 2 * RB / NWAVE;         // bytes written per wave per tile
    constexpr int NS = WB / (64 * 16);         // 8
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = gridDim.x, w = blockIdx.x;
    const int R = RUN ? RUN : ntiles / G;      // tiles per run
    const int nruns = ntiles / R;
    // the k-th tile of this workgroup
    auto tile_of = [&](int k) -> int {
        const int r = w + (k / R) * G;
        return r < nruns ? r * R + k % R : ntiles;
    };
    f4 r[NL];
    auto ld = [&](int tile, int i) -> f4 {
        return tile < ntiles ? __builtin_nontemporal_load(x + (size_t)tile * (RB / 16) + tid + NT * i) : f4{};
    };
#pragma unroll
    for (int i = 0; i < NL; i++) r[i] = ld(tile_of(0), i);
    for (int k = 0;; k++) {
        const int t = tile_of(k);
        if (t >= ntiles) break;
        const int nt = tile_of(k + 1);
        f4 c[NL];
#pragma unroll
        for (int i = 0; i < NL; i++) c[i] = r[i];
        float a = c[0].x + c[1].y + c[2].z + c[3].w;
        if (!ILV) {
#pragma unroll
            for (int i = 0; i < NL; i++) r[i] = ld(nt, i);
        }
        if (BAR) lds_barrier();
#pragma unroll 8
        for (int d = 0; d < DLY; d++) a = fmaf(a, 0.999f, 0.001f);
        f4 *q = y + ((size_t)t * 2 * RB + (size_t)wave * WB) / 16;
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const f4 v = c[s % NL] + a + (float)s;
            __builtin_nontemporal_store(v, q + s * 64 + lane);
            if (ILV && (s & 1) == 0) r[s / 2] = ld(nt, s / 2);
        }
        if (BAR) lds_barrier();
    }
}

struct Var {
    const char *name;
    void (*launch)(const f4 *, f4 *, int, int);
    int wpc;
};

template <int WPC, int RUN, bool ILV, bool BAR, int DLY>
void launch(const f4 *x, f4 *y, int ntiles, int grid)
{
    hipLaunchKernelGGL((k_pat<WPC, RUN, ILV, BAR, DLY>), dim3(grid), dim3(1024 / WPC), 0, 0, x, y, ntiles);
}

#define V(WPC, RUN, ILV, BAR, DLY)                                                                          \
    Var{"wpc" #WPC " run" #RUN " ilv" #ILV " bar" #BAR " dly" #DLY, launch<WPC, RUN, ILV, BAR, DLY>, WPC}

int main()
{
    const size_t in_bytes = (size_t)1 << 30;   // 2^27 complex samples
    f4 *x, *y;
    CK(hipMalloc(&x, in_bytes));
    CK(hipMalloc(&y, 2 * in_bytes));
    CK(hipMemset(x, 1, in_bytes));
    CK(hipMemset(y, 0, 2 * in_bytes));
    std::vector<Var> vs = {
        V(1, 0, false, true, 400), V(1, 0, false, false, 0), V(1, 1, false, false, 0), V(1, 1, true, false, 0),
        V(1, 4, false, true, 400), V(1, 1, false, true, 400), V(1, 0, true, true, 400), V(2, 0, true, true, 400),
        V(2, 0, false, true, 400), V(2, 1, true, true, 400), V(2, 4, true, true, 400), V(4, 1, true, false, 0),
        V(4, 0, true, false, 0), V(4, 0, true, true, 400), V(1, 8, false, true, 400), V(2, 1, false, true, 400),
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int pass = 0; pass < 3; pass++) {
        for (size_t v = 0; v < vs.size(); v++) {
            const int ntiles = (int)(in_bytes / (65536 / vs[v].wpc));
            const int grid = 256 * vs[v].wpc;
            for (int i = 0; i < (pass == 0 ? 200 : 20); i++) vs[v].launch(x, y, ntiles, grid);
            CK(hipEventRecord(e0));
            const int it = 20;
            for (int i = 0; i < it; i++) vs[v].launch(x, y, ntiles, grid);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / it);
        }
    }
    for (size_t v = 0; v < vs.size(); v++) {
        float best = 1e9;
        for (float m : t[v]) best = m < best ? m : best;
        printf("%-36s ms %.4f %.4f %.4f  best %.4f  %.0f GB/s\n", vs[v].name, t[v][0], t[v][1], t[v][2], best,
               3.0 * in_bytes / best / 1e6);
    }
    return 0;
}
