// mb_bw2.hip -- HBM ceilings with several 16-byte accesses in flight per lane (dev tool).
// mb_bw.hip issued one load per lane per iteration (4 waves per CU at grid 1024), which
// measures latency as much as bandwidth.  Here every lane keeps U loads (and U*K stores)
// in flight per iteration; workgroup size, grid and store flavour are swept.
//   K = 0 read only, K = -1 write only, K = 1 copy, K = 2 one read : two writes
//   (firpfbch2's mix: 8 B in, 16 B out per input sample).
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

// grid-stride over tiles of BS*U elements; lane t of a tile handles t + BS*u
template <int K, int U, int BS, bool NTS>
__global__ __launch_bounds__(BS) void k_mix(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4)
{
    const long long tile = (long long)BS * U;
    const long long ntile = n4 / tile;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long long t = blockIdx.x; t < ntile; t += gridDim.x) {
        const long long base = t * tile + threadIdx.x;
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = K >= 0 ? __builtin_nontemporal_load(a + base + (long long)u * BS) : f4{1.f, 2.f, 3.f, (float)t};
        if (K == 0) {
#pragma unroll
            for (int u = 0; u < U; u++) acc += v[u];
            continue;
        }
        const int kk = K < 0 ? 1 : K;
#pragma unroll
        for (int k = 0; k < kk; k++)
#pragma unroll
            for (int u = 0; u < U; u++) {
                f4 w = v[u] * (float)(k + 1);
                f4 *p = b + (long long)k * n4 + base + (long long)u * BS;
                if (NTS) __builtin_nontemporal_store(w, p);
                else *p = w;
            }
    }
    if (K == 0 && acc.x == 1234.5f) b[0] = acc;
}

template <int K, int U, int BS, bool NTS>
void run(const char *name, const f4 *a, f4 *b, long long n4, int grid)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL((k_mix<K, U, BS, NTS>), dim3(grid), dim3(BS), 0, 0, a, b, n4);
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; i++) hipLaunchKernelGGL((k_mix<K, U, BS, NTS>), dim3(grid), dim3(BS), 0, 0, a, b, n4);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    const double rd = K >= 0 ? 16.0 * n4 : 0.0, wr = 16.0 * n4 * (K < 0 ? 1 : K);
    printf("%-22s U%d BS%4d %s grid %6d  %7.3f ms  read %5.0f  write %5.0f  total %5.0f GB/s\n", name, U, BS,
           NTS ? "nt   " : "plain", grid, ms, rd / ms / 1e6, wr / ms / 1e6, (rd + wr) / ms / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int K, int U, int BS>
void sweep(const char *name, const f4 *a, f4 *b, long long n4)
{
    for (int g : {256, 512, 1024, 2048}) {
        run<K, U, BS, true>(name, a, b, n4, g);
        run<K, U, BS, false>(name, a, b, n4, g);
    }
}

int main()
{
    const long long n4 = 1LL << 26;   // 1 GiB per stream, above the 256 MiB Infinity Cache
    f4 *a, *b;
    CK(hipMalloc(&a, n4 * 16));
    CK(hipMalloc(&b, 2 * n4 * 16));
    CK(hipMemset(a, 1, n4 * 16));
    CK(hipMemset(b, 0, 2 * n4 * 16));
    sweep<0, 4, 256>("read", a, b, n4);
    sweep<0, 8, 512>("read", a, b, n4);
    sweep<-1, 1, 256>("write", a, b, n4);
    sweep<-1, 4, 256>("write", a, b, n4);
    sweep<-1, 4, 1024>("write", a, b, n4);
    sweep<-1, 8, 512>("write", a, b, n4);
    sweep<1, 4, 256>("copy 1:1", a, b, n4);
    sweep<1, 4, 1024>("copy 1:1", a, b, n4);
    sweep<1, 8, 512>("copy 1:1", a, b, n4);
    sweep<2, 2, 256>("read 1 : write 2", a, b, n4);
    sweep<2, 4, 256>("read 1 : write 2", a, b, n4);
    sweep<2, 4, 1024>("read 1 : write 2", a, b, n4);
    sweep<2, 8, 512>("read 1 : write 2", a, b, n4);
    return 0;
}
