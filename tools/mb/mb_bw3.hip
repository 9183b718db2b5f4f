// mb_bw3.hip -- the firpfbch2 M=1024 analyzer's memory pattern alone (dev tool):
// 1024-lane workgroups, one per CU; a tile = 8 rows of 1024 complex samples read
// (8 B per lane per row, 64 KB) and 16 blocks of 1024 complex outputs written
// (each wave one 8 KB block as eight 16-byte stores per lane, 128 KB).  The next
// tile's rows are loaded before the current tile's stores.  Tile assignment:
//   mode 0: grid-stride (workgroup w takes tiles w, w+G, ...)
//   mode 1: contiguous segments, every workgroup starting at its segment's head
//   mode 2: contiguous segments, workgroup w starting (w * T / G) tiles into its
//           segment and wrapping (staggered: workgroups no longer in lock step
//           on the same offset of segments a power of two apart)
//   mode 3: contiguous segments, tile order reversed for odd workgroups
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

template <int MODE, bool NTS>
__global__ __launch_bounds__(1024, 1) void k_pat(const f2 *__restrict__ x, f4 *__restrict__ y, int ntiles)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = gridDim.x, w = blockIdx.x;
    const int T = ntiles / G; // tiles per workgroup
    auto tile_of = [&](int k) -> long long {
        if (MODE == 0) return (long long)k * G + w;
        if (MODE == 1) return (long long)w * T + k;
        if (MODE == 2) return (long long)w * T + (k + (long long)w * T / G) % T;
        return (long long)w * T + ((w & 1) ? T - 1 - k : k);
    };
    f2 r[8];
    {
        const f2 *p = x + tile_of(0) * 8192 + tid;
#pragma unroll
        for (int i = 0; i < 8; i++) r[i] = p[1024 * i];
    }
    for (int k = 0; k < T; k++) {
        f2 c[8];
#pragma unroll
        for (int i = 0; i < 8; i++) c[i] = r[i];
        if (k + 1 < T) {
            const f2 *p = x + tile_of(k + 1) * 8192 + tid;
#pragma unroll
            for (int i = 0; i < 8; i++) r[i] = p[1024 * i];
        }
        // wave's block: 8 KB = 512 f4, lane writes f4 lane + 64 s
        f4 *q = y + (tile_of(k) * 16 + wave) * 512 + lane;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const f4 v = {c[s].x, c[s].y, c[(s + 1) & 7].x, c[(s + 1) & 7].y};
            if (NTS) __builtin_nontemporal_store(v, q + 64 * s);
            else q[64 * s] = v;
        }
    }
}

template <int MODE, bool NTS>
void run(const f2 *x, f4 *y, int ntiles, int grid)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL((k_pat<MODE, NTS>), dim3(grid), dim3(1024), 0, 0, x, y, ntiles);
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; i++) hipLaunchKernelGGL((k_pat<MODE, NTS>), dim3(grid), dim3(1024), 0, 0, x, y, ntiles);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    const double rd = 65536.0 * ntiles, wr = 131072.0 * ntiles;
    printf("mode %d %s grid %4d  %7.3f ms  read %5.0f  write %5.0f  total %5.0f GB/s\n", MODE, NTS ? "nt   " : "plain",
           grid, ms, rd / ms / 1e6, wr / ms / 1e6, (rd + wr) / ms / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main()
{
    const int ntiles = 16384; // 2^27 samples in (1 GiB), 2 GiB out: the bench's firpfbch2 step
    f2 *x;
    f4 *y;
    CK(hipMalloc(&x, (size_t)ntiles * 65536));
    CK(hipMalloc(&y, (size_t)ntiles * 131072));
    CK(hipMemset(x, 1, (size_t)ntiles * 65536));
    CK(hipMemset(y, 0, (size_t)ntiles * 131072));
    for (int grid : {256, 512}) {
        run<0, true>(x, y, ntiles, grid);
        run<0, false>(x, y, ntiles, grid);
        run<1, true>(x, y, ntiles, grid);
        run<1, false>(x, y, ntiles, grid);
        run<2, true>(x, y, ntiles, grid);
        run<2, false>(x, y, ntiles, grid);
        run<3, true>(x, y, ntiles, grid);
        run<3, false>(x, y, ntiles, grid);
    }
    return 0;
}
