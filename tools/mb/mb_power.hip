// mb_power.hip -- does adding matrix-core work to a streaming copy slow the
// stream (clock/power), even when the two are independent?  (dev tool)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));
__device__ unsigned long long g_clk[2 * 8192];

template <int NMF, int UNR, int RND = 0>
__global__ __launch_bounds__(256) void k_pw(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4, float s)
{
    unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    f4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    float av = s * threadIdx.x, bv = s + threadIdx.x;
    const long long stride = (long long)gridDim.x * 256 * UNR;
    for (long long i = (long long)blockIdx.x * 256 * UNR + threadIdx.x; i < n4; i += stride) {
        f4 v[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) v[u] = a[i + u * 256];
#pragma unroll
        for (int m = 0; m < NMF; m++) {
            if (RND) {
                const f4 w = v[m % UNR];
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[m & 3], w[(m + 1) & 3], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[(m + 2) & 3], w[(m + 3) & 3], acc1, 0, 0, 0);
            } else {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(bv, av, acc1, 0, 0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < UNR; u++) b[i + u * 256] = v[u];
    }
    if (acc0.x == 1.2345f && acc1.y == 3.f) b[0] = acc0 + acc1;
    if (threadIdx.x == 0 && blockIdx.x < 8192) {
        g_clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        g_clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

// copy through LDS: MODE 1 register load + ds_write + ds_read; MODE 2 LDS-DMA + ds_read
template <int MODE, int RD>
__global__ __launch_bounds__(256) void k_lds(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4)
{
    __shared__ f4 buf[1024];
    unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const long long stride = (long long)gridDim.x * 1024;
    f4 acc = {0, 0, 0, 0};
    for (long long i = (long long)blockIdx.x * 1024; i < n4; i += stride) {
        if (MODE == 1) {
            f4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = a[i + u * 256 + threadIdx.x];
#pragma unroll
            for (int u = 0; u < 4; u++) buf[u * 256 + threadIdx.x] = v[u];
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++)
                __builtin_amdgcn_global_load_lds((const void *)(a + i + u * 256 + threadIdx.x),
                    (__attribute__((address_space(3))) void *)((char *)buf + (u * 256 + (threadIdx.x & ~63)) * 16), 16, 0, 0);
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; u++) {
            f4 v = buf[u * 256 + threadIdx.x];
#pragma unroll
            for (int r = 1; r < RD; r++) acc += buf[(u * 256 + threadIdx.x + 64 * r) & 1023];
            b[i + u * 256 + threadIdx.x] = v;
        }
        __syncthreads();
    }
    if (acc.x == 1.2345f) b[0] = acc;
    if (threadIdx.x == 0 && blockIdx.x < 8192) {
        g_clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        g_clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int MODE, int RD>
void run_lds(const f4 *a, f4 *b, long long n4, int grid)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_lds<MODE, RD>), dim3(grid), dim3(256), 0, 0, a, b, n4);
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; i++) hipLaunchKernelGGL((k_lds<MODE, RD>), dim3(grid), dim3(256), 0, 0, a, b, n4);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    std::vector<unsigned long long> c(2 * grid);
    CK(hipMemcpyFromSymbol(c.data(), HIP_SYMBOL(g_clk), c.size() * 8));
    double cy = 0, rt = 0;
    for (int i = 0; i < grid; i++) { cy += c[2 * i]; rt += c[2 * i + 1]; }
    printf("LDS copy mode=%d reads/elem=%d grid=%5d  %7.3f ms  %6.0f GB/s  clk %.3f GHz\n", MODE, RD, grid, ms,
           32.0 * n4 / (ms * 1e-3) / 1e9, cy / rt * 0.1);
}

// half the workgroups stream, the other half only run MFMAs (NMF per iteration, same trip count)
template <int NMF, int VALU>
__global__ __launch_bounds__(256) void k_split(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4, float s)
{
    const long long stride = (long long)(gridDim.x / 2) * 256 * 4;
    const long long bi = blockIdx.x / 2;
    if ((blockIdx.x & 1) == 0) {
        for (long long i = bi * 256 * 4 + threadIdx.x; i < n4; i += stride) {
            f4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = a[i + u * 256];
#pragma unroll
            for (int u = 0; u < 4; u++) b[i + u * 256] = v[u];
        }
    } else {
        f4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
        float av = s * threadIdx.x, bv = s + threadIdx.x;
        for (long long i = bi * 256 * 4 + threadIdx.x; i < n4; i += stride) {
#pragma unroll
            for (int m = 0; m < NMF; m++) {
                if (VALU) {
                    acc0 = acc0 * av + bv;
                    acc1 = acc1 * bv + av;
                } else {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(bv, av, acc1, 0, 0, 0);
                }
            }
            av += 1.0f;
        }
        if (acc0.x == 1.2345f && acc1.y == 3.f) b[0] = acc0 + acc1;
    }
}

template <int NMF, int VALU>
void run_split(const f4 *a, f4 *b, long long n4, int grid)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_split<NMF, VALU>), dim3(grid), dim3(256), 0, 0, a, b, n4, 0.5f);
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; i++) hipLaunchKernelGGL((k_split<NMF, VALU>), dim3(grid), dim3(256), 0, 0, a, b, n4, 0.5f);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    printf("split VALU=%d NMF=%3d grid=%5d  %7.3f ms  %6.0f GB/s\n", VALU, NMF, grid, ms, 32.0 * n4 / (ms * 1e-3) / 1e9);
}

template <int NMF, int UNR, int RND = 0>
void run(const f4 *a, f4 *b, long long n4, int grid)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_pw<NMF, UNR, RND>), dim3(grid), dim3(256), 0, 0, a, b, n4, 0.5f);
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; i++) hipLaunchKernelGGL((k_pw<NMF, UNR, RND>), dim3(grid), dim3(256), 0, 0, a, b, n4, 0.5f);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    std::vector<unsigned long long> c(2 * grid);
    CK(hipMemcpyFromSymbol(c.data(), HIP_SYMBOL(g_clk), c.size() * 8));
    double cy = 0, rt = 0;
    for (int i = 0; i < grid; i++) { cy += c[2 * i]; rt += c[2 * i + 1]; }
    // MFMA work as a fraction of the chip's f32 matrix peak (157 TF)
    double mflop = 2.0 * NMF * 2048.0 * (double)(n4 / 64) * 1.0;   // per wave-iteration: 2*NMF MFMAs x 2048 flop; waves = n4/64 iterations
    printf("RND=%d NMF=%3d UNR=%d grid=%5d  %7.3f ms  %6.0f GB/s  clk %.3f GHz  mfma %.1f TF\n", RND, NMF, UNR, grid, ms,
           32.0 * n4 / (ms * 1e-3) / 1e9, cy / rt * 0.1, mflop / (ms * 1e-3) / 1e12);
}

int main()
{
    const long long n4 = 1ll << 27;   // 2 GiB read + 2 GiB write
    f4 *a, *b;
    CK(hipMalloc(&a, n4 * 16));
    CK(hipMalloc(&b, n4 * 16));
    CK(hipMemset(a, 0, n4 * 16));
    {
        std::vector<float> h(4 * n4);
        unsigned st = 7;
        for (long long i = 0; i < 4 * n4; i++) { st = st * 1664525u + 1013904223u; h[i] = (float)(st >> 8) / 16777216.0f - 0.5f; }
        CK(hipMemcpy(a, h.data(), n4 * 16, hipMemcpyHostToDevice));
    }
    run_split<0, 0>(a, b, n4, 4096);
    run_split<16, 0>(a, b, n4, 4096);
    run_split<32, 0>(a, b, n4, 4096);
    run_split<64, 0>(a, b, n4, 4096);
    run_split<32, 1>(a, b, n4, 4096);
    run_split<64, 1>(a, b, n4, 4096);
    return 0;
}
