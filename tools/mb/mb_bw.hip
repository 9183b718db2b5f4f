// mb_bw.hip -- HBM ceilings for the traffic mixes of the hot kernels (dev tool):
// read R bytes and write W = k R bytes (k = 0, 1, 2), 16-byte lanes, grid-stride,
// plain vs non-temporal stores.  firfilt is k = 1, firpfbch2 (M in, 2M out per
// M/2... 8 B in, 16 B out per input sample) is k = 2.
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

template <int K, bool NTS>
__global__ __launch_bounds__(256) void k_mix(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4)
{
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        f4 v = K >= 0 ? a[i] : f4{1.f, 2.f, 3.f, 4.f};
        if (K == 0) {
            if (v.x == 1234.5f) b[0] = v;
            continue;
        }
#pragma unroll
        for (int k = 0; k < (K < 0 ? -K : K); k++) {
            f4 w = v * (float)(k + 1);
            if (NTS) __builtin_nontemporal_store(w, b + (long long)k * n4 + i);
            else b[(long long)k * n4 + i] = w;
        }
    }
}

// per-workgroup contiguous segments (the persistent kernels' assignment):
// workgroup w copies elements [w*per, (w+1)*per) in 256-lane steps
template <int K, bool NTS>
__global__ __launch_bounds__(256) void k_seg(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4, long long per)
{
    const long long e0 = (long long)blockIdx.x * per;
    long long e1 = e0 + per;
    if (e1 > n4) e1 = n4;
    for (long long i = e0 + threadIdx.x; i < e1; i += 256) {
        f4 v = a[i];
#pragma unroll
        for (int k = 0; k < K; k++) {
            f4 w = v * (float)(k + 1);
            if (NTS) __builtin_nontemporal_store(w, b + (long long)k * n4 + i);
            else b[(long long)k * n4 + i] = w;
        }
    }
}

template <int K, bool NTS>
void run_seg(const char *name, const f4 *a, f4 *b, long long n4, int grid)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const long long per = (n4 + grid - 1) / grid;
    hipLaunchKernelGGL((k_seg<K, NTS>), dim3(grid), dim3(256), 0, 0, a, b, n4, per);
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; i++) hipLaunchKernelGGL((k_seg<K, NTS>), dim3(grid), dim3(256), 0, 0, a, b, n4, per);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    const double rd = 16.0 * n4, wr = 16.0 * n4 * K;
    printf("%-34s grid %6d  %8.3f ms  read %6.0f GB/s  write %6.0f GB/s  total %6.0f GB/s\n", name, grid, ms,
           rd / ms / 1e6, wr / ms / 1e6, (rd + wr) / ms / 1e6);
    fflush(stdout);
}

template <int K, bool NTS>
void run(const char *name, const f4 *a, f4 *b, long long n4, int grid)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_mix<K, NTS>), dim3(grid), dim3(256), 0, 0, a, b, n4);
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; i++) hipLaunchKernelGGL((k_mix<K, NTS>), dim3(grid), dim3(256), 0, 0, a, b, n4);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    const double rd = K >= 0 ? 16.0 * n4 : 0.0, wr = 16.0 * n4 * (K < 0 ? -K : K);
    printf("%-34s grid %6d  %8.3f ms  read %6.0f GB/s  write %6.0f GB/s  total %6.0f GB/s\n", name, grid, ms,
           rd / ms / 1e6, wr / ms / 1e6, (rd + wr) / ms / 1e6);
    fflush(stdout);
}

int main()
{
    const long long n4 = 1LL << 26;   // 1 GiB read per launch
    f4 *a, *b;
    CK(hipMalloc(&a, n4 * 16));
    CK(hipMalloc(&b, 2 * n4 * 16));
    CK(hipMemset(a, 1, n4 * 16));
    CK(hipMemset(b, 0, 2 * n4 * 16));
    for (int grid : {1024, 2048, 4096}) {
        run<1, true>("copy 1:1 nt (grid-stride)", a, b, n4, grid);
        run_seg<1, true>("copy 1:1 nt (per-WG segment)", a, b, n4, grid);
        run<2, true>("read 1 : write 2 nt (grid-stride)", a, b, n4, grid);
        run_seg<2, true>("read 1 : write 2 nt (per-WG seg)", a, b, n4, grid);
    }
    for (int grid : {256, 512}) {
        run_seg<1, true>("copy 1:1 nt (per-WG segment)", a, b, n4, grid);
        run_seg<2, true>("read 1 : write 2 nt (per-WG seg)", a, b, n4, grid);
    }
    return 0;
}
