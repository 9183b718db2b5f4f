// mb_bw4.hip -- the matrix-core firfilt's memory pattern alone (dev tool):
// 4-wave workgroups, three per CU (51 KB of dynamic LDS, as k_firfilt_mx), chunks of
// 2048 complex samples (lane: 4 x 16-byte loads, 4 x 16-byte stores), the chunk after
// next loaded before the current chunk's stores.  Chunk assignment:
//   mode 0: contiguous runs of cpw chunks per workgroup (the library kernel, cpw odd)
//   mode 1: grid-stride (workgroup w takes chunks w, w+G, ...)
//   mode 2: grid-stride over pairs of chunks
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

template <int MODE, bool NTL>
__global__ __launch_bounds__(256, 3) void k_pat(const f4 *__restrict__ x, f4 *__restrict__ y, long long nch,
                                                long long cpw)
{
    extern __shared__ float smem[];
    const int tid = threadIdx.x;
    const long long G = gridDim.x, w = blockIdx.x;
    long long cnt;
    if (MODE == 0) {
        const long long c0 = w * cpw;
        long long c1 = c0 + cpw;
        if (c1 > nch) c1 = nch;
        cnt = c1 - c0;
    } else {
        cnt = (nch - w + G - 1) / G;
    }
    auto chunk = [&](long long k) -> long long {
        if (MODE == 0) return w * cpw + k;
        if (MODE == 1) return k * G + w;
        return ((k >> 1) * G + w) * 2 + (k & 1);
    };
    if (MODE == 2) cnt = 2 * ((nch / 2 - w + G - 1) / G);
    auto ld = [&](long long k, f4 (&v)[4]) {
        const f4 *p = x + chunk(k) * 1024 + 4 * tid;
#pragma unroll
        for (int q = 0; q < 4; q++) v[q] = NTL ? __builtin_nontemporal_load(p + q) : p[q];
    };
    f4 a[4], b[4];
    if (cnt > 0) ld(0, a);
    if (cnt > 1) ld(1, b);
    auto st = [&](long long k, f4 (&v)[4]) {
        f4 o[4];
#pragma unroll
        for (int q = 0; q < 4; q++) o[q] = v[q] * 2.f;
        if (k + 2 < cnt) ld(k + 2, v);
        smem[tid] = o[0].x;   // keep the LDS allocation live
        f4 *p = y + chunk(k) * 1024 + tid;
#pragma unroll
        for (int q = 0; q < 4; q++) __builtin_nontemporal_store(o[q], p + 256 * q);
    };
    for (long long k = 0; k < cnt; k += 2) {
        st(k, a);
        if (k + 1 < cnt) st(k + 1, b);
    }
}

template <int MODE, bool NTL>
void run(const f4 *x, f4 *y, long long nch, int nwg)
{
    long long cpw = ((nch + nwg - 1) / nwg) | 1;
    int grid = MODE == 0 ? (int)((nch + cpw - 1) / cpw) : nwg;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t lds = 51008;
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL((k_pat<MODE, NTL>), dim3(grid), dim3(256), lds, 0, x, y, nch, cpw);
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; i++) hipLaunchKernelGGL((k_pat<MODE, NTL>), dim3(grid), dim3(256), lds, 0, x, y, nch, cpw);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    const double rd = 16384.0 * nch;
    printf("mode %d %s grid %4d cpw %4lld  %7.3f ms  total %5.0f GB/s\n", MODE, NTL ? "ntload" : "plain ", grid,
           MODE == 0 ? cpw : 0LL, ms, 2 * rd / ms / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main()
{
    const long long nch = 131072;   // 2^28 complex samples (2 GiB in, 2 GiB out)
    f4 *x, *y;
    CK(hipMalloc(&x, (size_t)nch * 16384));
    CK(hipMalloc(&y, (size_t)nch * 16384));
    CK(hipMemset(x, 1, (size_t)nch * 16384));
    CK(hipMemset(y, 0, (size_t)nch * 16384));
    for (int nwg : {768, 512, 256}) {
        run<0, false>(x, y, nch, nwg);
        run<0, true>(x, y, nch, nwg);
        run<1, false>(x, y, nch, nwg);
        run<1, true>(x, y, nch, nwg);
        run<2, false>(x, y, nch, nwg);
    }
    run<1, false>(x, y, nch, 1536);
    run<1, false>(x, y, nch, 3072);
    return 0;
}
