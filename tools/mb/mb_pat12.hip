// mb_pat12.hip -- sweep of the firpfbch2 M=1024 analyzer's 1 read : 2 write
// memory pattern (dev tool; the kernel k_pfb2_an1024 with its arithmetic
// removed is mb_bw3.hip's mode 0).  A workgroup tile reads RB contiguous
// bytes (8 rows) and writes 2 RB contiguous bytes (16 blocks); 2^27 complex
// samples in, 2^28 out, as the bench's step.  Swept:
//   WPC  workgroups per CU: 1 (1024 threads, 64 KB tiles) or 2 (512 threads,
//        32 KB tiles, half the columns each)
//   LDW  bytes per lane per load: 8 (the kernel's column loads) or 16
//   SW   contiguous bytes a lane writes per store group: 16 (each wave
//        instruction 1 KB contiguous, the kernel), 32 or 64
//   ILV  the next tile's loads issued between the stores (1) or all before
//        them (0, the kernel)
//   DEP  tiles of loads in flight: 1 (the kernel) or 2
//   NTS  non-temporal stores (1, the kernel) or plain
// Output: one line per variant, ms per step and total GB/s, three passes
// A B C ... A B C ... so box drift hits every variant alike.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>
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
typedef float f2 __attribute__((ext_vector_type(2)));

template <int WPC, int LDW, int SW, bool ILV, int DEP, bool NTS>
__global__ __launch_bounds__(1024 / WPC, WPC) void k_pat(const unsigned char *__restrict__ x,
                                                         unsigned char *__restrict__ y, int ntiles)
{
    constexpr int NT = 1024 / WPC;
    constexpr int RB = 65536 / WPC;            // bytes read per tile
    constexpr int NL = RB / (NT * LDW);        // loads per lane per tile
    constexpr int NWAVE = NT / 64;
    constexpr int WB = 2 * RB / NWAVE;         // bytes written per wave per tile
    constexpr int NS = WB / (64 * 16);         // 16-byte stores per lane per tile
    constexpr int SPG = SW / 16;               // 16-byte stores per lane per group
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = gridDim.x, w = blockIdx.x;
    typedef typename std::conditional<LDW == 8, f2, f4>::type LT;
    LT r[DEP][NL];
    auto load = [&](int tile, LT (&d)[NL]) {
        const LT *p = reinterpret_cast<const LT *>(x + (size_t)tile * RB) + tid;
#pragma unroll
        for (int i = 0; i < NL; i++) d[i] = tile < ntiles ? p[NT * i] : LT{};
    };
#pragma unroll
    for (int d = 0; d < DEP; d++) load(w + d * G, r[d]);
    for (int t = w; t < ntiles; t += G) {
        LT c[NL];
#pragma unroll
        for (int i = 0; i < NL; i++) c[i] = r[0][i];
#pragma unroll
        for (int d = 0; d + 1 < DEP; d++)
#pragma unroll
            for (int i = 0; i < NL; i++) r[d][i] = r[d + 1][i];
        const int nt = t + DEP * G;
        if (!ILV) load(nt, r[DEP - 1]);
        // the wave's output block: NS 16-byte stores per lane, SPG of them
        // contiguous per lane
        f4 *q = reinterpret_cast<f4 *>(y + (size_t)t * 2 * RB + (size_t)wave * WB);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int g = s / SPG, j = s % SPG;
            const int idx = (g * 64 + lane) * SPG + j;
            float a = 0.f;
            if constexpr (LDW == 8) a = c[s % NL].x + c[(s + 1) % NL].y;
            else a = c[s % NL].x + c[(s + 1) % NL].w;
            const f4 v = {a, a + 1.f, a + 2.f, a + 3.f};
            if (NTS) __builtin_nontemporal_store(v, q + idx);
            else q[idx] = v;
            if (ILV && s < NL) {
                const LT *p = reinterpret_cast<const LT *>(x + (size_t)nt * RB) + tid;
                r[DEP - 1][s] = nt < ntiles ? p[NT * s] : LT{};
            }
        }
        if (ILV) {
#pragma unroll
            for (int s = NS; s < NL; s++) {
                const LT *p = reinterpret_cast<const LT *>(x + (size_t)nt * RB) + tid;
                r[DEP - 1][s] = nt < ntiles ? p[NT * s] : LT{};
            }
        }
    }
}

struct Var {
    const char *name;
    void (*launch)(const unsigned char *, unsigned char *, int, int);
    int wpc;
};

template <int WPC, int LDW, int SW, bool ILV, int DEP, bool NTS>
void launch(const unsigned char *x, unsigned char *y, int ntiles, int grid)
{
    hipLaunchKernelGGL((k_pat<WPC, LDW, SW, ILV, DEP, NTS>), dim3(grid), dim3(1024 / WPC), 0, 0, x, y, ntiles);
}

#define V(WPC, LDW, SW, ILV, DEP, NTS)                                                                          \
    Var{"wpc" #WPC " ldw" #LDW " sw" #SW " ilv" #ILV " dep" #DEP " nts" #NTS, launch<WPC, LDW, SW, ILV, DEP, NTS>, WPC}

int main()
{
    const size_t in_bytes = (size_t)1 << 30;   // 2^27 complex samples
    unsigned char *x, *y;
    CK(hipMalloc(&x, in_bytes));
    CK(hipMalloc(&y, 2 * in_bytes));
    CK(hipMemset(x, 1, in_bytes));
    CK(hipMemset(y, 0, 2 * in_bytes));
    std::vector<Var> vs = {
        V(1, 8, 16, false, 1, true),   // the kernel's pattern
        V(1, 8, 16, false, 1, false),  V(1, 8, 32, false, 1, true),  V(1, 8, 64, false, 1, true),
        V(1, 8, 16, true, 1, true),    V(1, 8, 32, true, 1, true),   V(1, 8, 16, false, 2, true),
        V(1, 16, 16, false, 1, true),  V(1, 16, 32, false, 1, true), V(1, 16, 16, true, 1, true),
        V(2, 8, 16, false, 1, true),   V(2, 8, 32, false, 1, true),  V(2, 8, 16, true, 1, true),
        V(2, 8, 16, false, 2, true),   V(2, 16, 16, false, 1, true), V(2, 16, 32, false, 1, true),
        V(2, 16, 16, false, 2, true),  V(2, 8, 16, false, 1, false),  V(2, 16, 16, true, 1, true),
        V(2, 8, 16, true, 2, true),    V(4, 8, 16, false, 1, true),   V(4, 8, 16, true, 1, true),
        V(4, 16, 16, true, 1, true),   V(2, 8, 16, true, 1, false),
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int pass = 0; pass < 3; pass++) {
        for (size_t v = 0; v < vs.size(); v++) {
            const int ntiles = (int)(in_bytes / (65536 / vs[v].wpc));
            const int grid = 256 * vs[v].wpc;
            for (int i = 0; i < 10; i++) vs[v].launch(x, y, ntiles, grid);
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
