// mb_store.hip -- HBM ceilings on this box for streaming stores and for the
// 1 read : 2 write mix of the firpfbch2 analyzer (dev tool).  Sweeps store
// cache policy (buffer_store cpol: 0 plain, 1 sc0, 2 nt, 3 sc0|nt, 16 sc1,
// 18 sc1|nt), stores per lane in flight, grid shape and address pattern
// (grid-stride vs per-workgroup segments), and read width (8 / 16 B per lane).
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

// write-only: each lane U 16-byte stores per iteration, U wave-instructions
// covering U KB contiguous (grid-stride over U KB wave tiles)
template <int U, int CPOL>
__global__ __launch_bounds__(256) void k_wr(f4 *__restrict__ b, long long n4)
{
    const long long tiles = n4 / (64 * U);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long nw = (long long)gridDim.x * 4;
    for (long long t = (long long)blockIdx.x * 4 + w; t < tiles; t += nw) {
        const __amdgpu_buffer_rsrc_t rb =
            __builtin_amdgcn_make_buffer_rsrc((void *)(b + t * 64 * U), (short)0, 64 * U * 16, 0x00020000);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const f4 v = {(float)u, 1.f, 2.f, 3.f};
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f4, v), rb, (lane + 64 * u) * 16, 0, CPOL);
        }
    }
}

// plain C++ stores, grid stride 16 B per lane
template <bool NT>
__global__ __launch_bounds__(256) void k_wr_plain(f4 *__restrict__ b, long long n4)
{
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        const f4 v = {1.f, 2.f, 3.f, (float)i};
        if (NT) __builtin_nontemporal_store(v, b + i);
        else b[i] = v;
    }
}

// read-only, W bytes per lane (8 or 16), U loads in flight per lane
template <int W, int U>
__global__ __launch_bounds__(256) void k_rd(const float *__restrict__ a, long long nbytes, float *sink)
{
    const long long nel = nbytes / W;
    const long long stride = (long long)gridDim.x * 256;
    float acc = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < nel; i += stride * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long long j = i + u * stride;
            if (j < nel) {
                if (W == 16) {
                    const f4 v = reinterpret_cast<const f4 *>(a)[j];
                    acc += v.x + v.w;
                } else {
                    const f2 v = reinterpret_cast<const f2 *>(a)[j];
                    acc += v.x + v.y;
                }
            }
        }
    }
    if (acc == 1234.5f) sink[0] = acc;
}

// 1 read : 2 write.  Mode 0: two output streams (b, b + n4), grid stride;
// mode 1: one output stream of twice the length, each lane writes its two
// 16-byte results 1 KB apart (wave writes 2 KB contiguous); mode 2: per
// workgroup contiguous segments (persistent-kernel layout), like mode 1
template <int MODE, bool NT>
__global__ __launch_bounds__(256) void k_mix(const f4 *__restrict__ a, f4 *__restrict__ b, long long n4, long long per)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    auto st = [&](f4 *p, f4 v) {
        if (NT) __builtin_nontemporal_store(v, p);
        else *p = v;
    };
    if (MODE == 0) {
        const long long stride = (long long)gridDim.x * 256;
        for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
            const f4 v = a[i];
            st(b + i, v * 2.f);
            st(b + n4 + i, v * 3.f);
        }
    } else if (MODE == 1) {
        // wave tile = 64 inputs -> 128 outputs
        const long long tiles = n4 / 64, nw = (long long)gridDim.x * 4;
        for (long long t = (long long)blockIdx.x * 4 + w; t < tiles; t += nw) {
            const f4 v = a[t * 64 + lane];
            st(b + t * 128 + lane, v * 2.f);
            st(b + t * 128 + 64 + lane, v * 3.f);
        }
    } else {
        const long long e0 = (long long)blockIdx.x * per;
        long long e1 = e0 + per;
        if (e1 > n4) e1 = n4;
        for (long long i = e0 + threadIdx.x - lane + 0; i < e1; i += 256) {
            const long long t = (i + lane) >> 6;   // 64-input tile index of this wave
            const f4 v = a[i + lane];
            st(b + t * 128 + lane, v * 2.f);
            st(b + t * 128 + 64 + lane, v * 3.f);
        }
    }
}

template <typename F>
static float timeit(F launch, int it = 20)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    launch();
    CK(hipEventRecord(e0));
    for (int i = 0; i < it; i++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGetLastError());
    return ms / it;
}

int main()
{
    const long long nb = 2LL << 30;   // 2 GiB written by the write-only tests
    const long long n4 = nb / 16;
    f4 *a, *b;
    float *sink;
    CK(hipMalloc(&a, nb));
    CK(hipMalloc(&b, 2 * nb));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, nb));
    CK(hipMemset(b, 0, 2 * nb));
    auto rep = [&](const char *name, int grid, float ms, double rd, double wr) {
        printf("%-44s grid %6d %8.3f ms  rd %6.0f  wr %6.0f  total %6.0f GB/s\n", name, grid, ms, rd / ms / 1e6,
               wr / ms / 1e6, (rd + wr) / ms / 1e6);
        fflush(stdout);
    };
    for (int grid : {1024, 4096, 16384}) {
        rep("write plain (C++ store)", grid, timeit([&] { hipLaunchKernelGGL(k_wr_plain<false>, dim3(grid), dim3(256), 0, 0, b, n4); }), 0, nb);
        rep("write nt (C++ store)", grid, timeit([&] { hipLaunchKernelGGL(k_wr_plain<true>, dim3(grid), dim3(256), 0, 0, b, n4); }), 0, nb);
    }
    for (int grid : {1024, 2048, 8192}) {
#define WR(U, C) rep("buffer_store U=" #U " cpol=" #C, grid, timeit([&] { hipLaunchKernelGGL((k_wr<U, C>), dim3(grid), dim3(256), 0, 0, b, n4); }), 0, nb)
        WR(1, 0); WR(1, 2); WR(1, 1); WR(1, 3); WR(1, 16); WR(1, 18);
        WR(4, 0); WR(4, 2); WR(4, 3); WR(4, 18);
        WR(8, 0); WR(8, 2);
#undef WR
    }
    for (int grid : {1024, 4096}) {
        rep("read 16B/lane U=1", grid, timeit([&] { hipLaunchKernelGGL((k_rd<16, 1>), dim3(grid), dim3(256), 0, 0, (const float *)a, nb, sink); }), nb, 0);
        rep("read 16B/lane U=4", grid, timeit([&] { hipLaunchKernelGGL((k_rd<16, 4>), dim3(grid), dim3(256), 0, 0, (const float *)a, nb, sink); }), nb, 0);
        rep("read 8B/lane U=1", grid, timeit([&] { hipLaunchKernelGGL((k_rd<8, 1>), dim3(grid), dim3(256), 0, 0, (const float *)a, nb, sink); }), nb, 0);
        rep("read 8B/lane U=4", grid, timeit([&] { hipLaunchKernelGGL((k_rd<8, 4>), dim3(grid), dim3(256), 0, 0, (const float *)a, nb, sink); }), nb, 0);
    }
    const long long m4 = n4 / 2;   // 1 GiB in, 2 GiB out
    for (int grid : {1024, 2048, 4096, 16384}) {
        const long long per = ((m4 + grid - 1) / grid + 255) / 256 * 256;
        rep("mix 1:2 two streams nt", grid, timeit([&] { hipLaunchKernelGGL((k_mix<0, true>), dim3(grid), dim3(256), 0, 0, a, b, m4, per); }), m4 * 16.0, m4 * 32.0);
        rep("mix 1:2 two streams plain", grid, timeit([&] { hipLaunchKernelGGL((k_mix<0, false>), dim3(grid), dim3(256), 0, 0, a, b, m4, per); }), m4 * 16.0, m4 * 32.0);
        rep("mix 1:2 interleaved 2KB nt", grid, timeit([&] { hipLaunchKernelGGL((k_mix<1, true>), dim3(grid), dim3(256), 0, 0, a, b, m4, per); }), m4 * 16.0, m4 * 32.0);
        rep("mix 1:2 interleaved 2KB plain", grid, timeit([&] { hipLaunchKernelGGL((k_mix<1, false>), dim3(grid), dim3(256), 0, 0, a, b, m4, per); }), m4 * 16.0, m4 * 32.0);
        rep("mix 1:2 per-WG segments nt", grid, timeit([&] { hipLaunchKernelGGL((k_mix<2, true>), dim3(grid), dim3(256), 0, 0, a, b, m4, per); }), m4 * 16.0, m4 * 32.0);
    }
    return 0;
}
