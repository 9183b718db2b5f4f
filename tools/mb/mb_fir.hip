// mb_fir.hip -- design-space sweep for the firfilt_crcf h=64 kernel (dev tool).
//
// Standalone: builds with hipcc, allocates a 2^28-sample complex stream,
// times every variant with HIP events and checks each against variant 0.
// Variants: workgroup size NT, outputs per lane R, store path (LDS transpose
// + coalesced stores / direct per-lane stores), non-temporal loads/stores,
// plus a float4 copy kernel as the practical read+write ceiling.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e = (x);                                                                         \
        if (e != hipSuccess) {                                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));                \
            exit(1);                                                                                \
        }                                                                                           \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__host__ __device__ __forceinline__ int lds_off(int u) { return u * 8 + 16 * (u >> 4); }

template <bool NT_LD>
__device__ __forceinline__ f4 ld4(const f4 *p)
{
    if (NT_LD) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT_ST>
__device__ __forceinline__ void st4(f4 *p, f4 v)
{
    if (NT_ST) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// h = 64 taps (HC = 64, one chunk), complex samples, no history (zeros)
template <int NT, int R, int STORE, bool NT_LD, bool NT_ST, int W>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(W, 8))) void k_fir(const float2 *__restrict__ x, float2 *__restrict__ y,
                                            const float *__restrict__ hp, long long n, int nchunk)
{
    constexpr int HC = 64, TILE = NT * R, S = TILE + HC;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const long long t0 = (long long)blockIdx.x * TILE;
    for (int e = threadIdx.x; e < S / 2; e += NT) {
        const int u = e * 2;
        const long long s = t0 - HC + u;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (s >= 0) v = ld4<NT_LD>(reinterpret_cast<const f4 *>(x + s));
        *reinterpret_cast<f4 *>(smem + lds_off(u)) = v;
    }
    __syncthreads();
    float2 acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = make_float2(0.f, 0.f);
    for (int c = 0; c < nchunk; c++) {
    const float *h = hp + c * HC;
    const int row0 = threadIdx.x * (R / 16) + ((HC - HC) >> 4);
    const unsigned char *rb = smem + lds_off(16 * row0);
    float2 v[HC + R];
#pragma unroll
    for (int i = 0; i < R / 2; i++) {
        const f4 o = *reinterpret_cast<const f4 *>(rb + lds_off(HC + 2 * i));
        v[HC + 2 * i] = make_float2(o.x, o.y);
        v[HC + 2 * i + 1] = make_float2(o.z, o.w);
    }
#pragma unroll
    for (int g = 0; g < HC / 16; g++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int a = HC - 16 * g - 16 + 2 * i;
            const f4 o = *reinterpret_cast<const f4 *>(rb + lds_off(a));
            v[a] = make_float2(o.x, o.y);
            v[a + 1] = make_float2(o.z, o.w);
        }
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const float hv = h[16 * g + j];
#pragma unroll
            for (int r = 0; r < R; r++) {
                acc[r].x = fmaf(hv, v[r - (16 * g + j) + HC].x, acc[r].x);
                acc[r].y = fmaf(hv, v[r - (16 * g + j) + HC].y, acc[r].y);
            }
        }
    }
    }
    if (STORE == 1) {
        f4 *yo = reinterpret_cast<f4 *>(y + t0 + (long long)R * threadIdx.x);
#pragma unroll
        for (int i = 0; i < R / 2; i++)
            st4<NT_ST>(yo + i, f4{acc[2 * i].x, acc[2 * i].y, acc[2 * i + 1].x, acc[2 * i + 1].y});
        return;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < R / 2; i++)
        *reinterpret_cast<f4 *>(smem + lds_off(R * threadIdx.x + 2 * i)) =
            f4{acc[2 * i].x, acc[2 * i].y, acc[2 * i + 1].x, acc[2 * i + 1].y};
    __syncthreads();
    for (int e = threadIdx.x; e < TILE / 2; e += NT) {
        const int u = e * 2;
        st4<NT_ST>(reinterpret_cast<f4 *>(y + t0 + u), *reinterpret_cast<const f4 *>(smem + lds_off(u)));
    }
}

template <bool NT_LD, bool NT_ST>
__global__ __launch_bounds__(256) void k_copy(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4)
{
    long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long stride = (long long)gridDim.x * 256;
    for (; i < n4; i += stride) st4<NT_ST>(b + i, ld4<NT_LD>(a + i));
}

template <int NT, int R, int STORE, bool NT_LD, bool NT_ST, int W>
float run_fir(const float2 *x, float2 *y, const float *h, long long n, int iters)
{
    constexpr int TILE = NT * R;
    const unsigned nb = (unsigned)(n / TILE);
    const size_t lds = (size_t)lds_off(TILE + 64) + 16;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_fir<NT, R, STORE, NT_LD, NT_ST, W>), dim3(nb), dim3(NT), lds, 0, x, y, h, n, 1);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; i++)
        hipLaunchKernelGGL((k_fir<NT, R, STORE, NT_LD, NT_ST, W>), dim3(nb), dim3(NT), lds, 0, x, y, h, n, 1);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
}

static std::vector<float> ref;

template <int NT, int R, int STORE, bool NT_LD, bool NT_ST, int W = 4>
void variant(const char *name, const float2 *x, float2 *y, const float *h, long long n, int iters)
{
    CK(hipMemset(y, 0, n * 8));
    float ms = run_fir<NT, R, STORE, NT_LD, NT_ST, W>(x, y, h, n, iters);
    std::vector<float> out(2 * n);
    CK(hipMemcpy(out.data(), y, n * 8, hipMemcpyDeviceToHost));
    double err = 0;
    if (ref.empty()) ref = out;
    else
        for (long long i = 0; i < 2 * n; i++) err = fmax(err, fabs(out[i] - ref[i]));
    printf("%-34s W=%d NT=%3d R=%2d  %8.3f ms  %7.1f GS/s  %6.0f GB/s  maxdiff %.2e\n", name, W, NT, R, ms,
           n / (ms * 1e-3) / 1e9, 16.0 * n / (ms * 1e-3) / 1e9, err);
}

int main()
{
    const long long n = 1ll << 28;
    float2 *x, *y;
    float *h;
    CK(hipMalloc(&x, n * 8));
    CK(hipMalloc(&y, n * 8));
    CK(hipMalloc(&h, 64 * 4));
    std::vector<float> hx(2 * n), hh(64);
    srand(1);
    for (long long i = 0; i < 2 * n; i++) hx[i] = (float)(rand() & 0xffff) / 65536.0f - 0.5f;
    for (int i = 0; i < 64; i++) hh[i] = (float)(rand() & 0xffff) / 65536.0f - 0.5f;
    CK(hipMemcpy(x, hx.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(h, hh.data(), 64 * 4, hipMemcpyHostToDevice));
    const int it = 10;

    // copy ceilings
    {
        const long long n4 = n / 2;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int mode = 0; mode < 4; mode++) {
            for (int grid : {1024, 2048, 8192, 65536}) {
                auto launch = [&]() {
                    switch (mode) {
                    case 0: hipLaunchKernelGGL((k_copy<false, false>), dim3(grid), dim3(256), 0, 0, (const f4 *)x, (f4 *)y, n4); break;
                    case 1: hipLaunchKernelGGL((k_copy<true, false>), dim3(grid), dim3(256), 0, 0, (const f4 *)x, (f4 *)y, n4); break;
                    case 2: hipLaunchKernelGGL((k_copy<false, true>), dim3(grid), dim3(256), 0, 0, (const f4 *)x, (f4 *)y, n4); break;
                    case 3: hipLaunchKernelGGL((k_copy<true, true>), dim3(grid), dim3(256), 0, 0, (const f4 *)x, (f4 *)y, n4); break;
                    }
                };
                launch();
                CK(hipEventRecord(e0));
                for (int i = 0; i < it; i++) launch();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                ms /= it;
                printf("copy ntld=%d ntst=%d grid=%6d           %8.3f ms  %6.0f GB/s\n", mode & 1, mode >> 1, grid, ms,
                       16.0 * n / (ms * 1e-3) / 1e9);
            }
        }
    }
    variant<256, 16, 0, false, false, 4>("base (LDS transpose)", x, y, h, n, it);
    variant<256, 16, 0, false, false, 5>("base", x, y, h, n, it);
    variant<256, 16, 0, false, false, 6>("base", x, y, h, n, it);
    variant<256, 16, 0, false, false, 2>("base", x, y, h, n, it);
    variant<256, 16, 1, false, false, 4>("direct stores", x, y, h, n, it);
    variant<256, 16, 1, false, false, 6>("direct stores", x, y, h, n, it);
    variant<256, 16, 0, true, false, 4>("nt loads", x, y, h, n, it);
    variant<256, 16, 0, false, true, 4>("nt stores", x, y, h, n, it);
    variant<256, 16, 0, true, true, 4>("nt loads+stores", x, y, h, n, it);
    variant<256, 16, 1, true, true, 4>("direct + nt", x, y, h, n, it);
    variant<128, 16, 0, false, false, 4>("NT128", x, y, h, n, it);
    variant<128, 16, 0, false, false, 6>("NT128", x, y, h, n, it);
    variant<512, 16, 0, false, false, 4>("NT512", x, y, h, n, it);
    variant<256, 32, 0, false, false, 2>("R32", x, y, h, n, it);
    variant<256, 32, 0, false, false, 3>("R32", x, y, h, n, it);
    variant<128, 32, 0, false, false, 2>("NT128 R32", x, y, h, n, it);
    variant<64, 32, 0, false, false, 2>("NT64 R32", x, y, h, n, it);
    variant<64, 16, 0, false, false, 4>("NT64 R16", x, y, h, n, it);
    variant<256, 8, 0, false, false, 8>("R8", x, y, h, n, it);
    variant<512, 8, 0, false, false, 8>("NT512 R8", x, y, h, n, it);
    variant<128, 16, 1, false, true, 4>("NT128 direct nt-st", x, y, h, n, it);
    variant<512, 16, 1, false, false, 4>("NT512 direct", x, y, h, n, it);
    return 0;
}
