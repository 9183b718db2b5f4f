// mb_bw5.hip -- variants of the firpfbch2 M=1024 analyzer's memory pattern
// (dev tool, round 3): 1 read : 2 write, rows of 1024 complex samples read
// column-wise, two 1024-point output blocks written per row.  Each workgroup
// walks a contiguous run of tiles (mb_bw3 mode 1, the library's order); a tile
// is ROWS rows read and 2*ROWS blocks written, each wave writing its blocks as
// 16-byte stores, 1 KB contiguous per instruction.  The next tile's rows are
// loaded before the current tile's stores.  Parameters:
//   LANES  workgroup size (1024 / 512 / 256)
//   CPL    columns per lane (1: 8-byte loads, 2: one 16-byte load, 4: two)
//   ROWS   rows per tile (8: the library's 16-block iteration, 4: 8 blocks)
//   DUAL   every row load issued twice through two buffer descriptors, one
//          of them out of range (the library's history / x split)
//   WPC    workgroups per CU (grid = 256 * WPC)
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

template <int CPL>
struct RowT {
    f4 a, b;
};

template <int LANES, int CPL, int ROWS, bool DUAL>
__global__ __launch_bounds__(LANES) void k_pat(const float *__restrict__ x, f4 *__restrict__ y, int ntiles)
{
    static_assert(LANES * CPL == 1024, "one row per workgroup pass");
    constexpr int WAVES = LANES / 64;
    constexpr int BPW = 2 * ROWS / WAVES; // blocks per wave per tile
    static_assert(BPW >= 1, "");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int G = gridDim.x, w = blockIdx.x;
    const int T = ntiles / G;
    const long long t0 = (long long)w * T;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, 0, 0x00020000);
    // byte offsets are relative to this workgroup's first row
    const float *xw = x + t0 * ROWS * 2048;
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void *)xw, (short)0, 0x7fffffff, 0x00020000);
    (void)rx;
    auto ld = [&](int k, int r) -> RowT<CPL> {
        RowT<CPL> v;
        const unsigned rb = (unsigned)((k * ROWS + r) * 8192);
        if constexpr (CPL == 1) {
            f2 a = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rw, rb + 8 * tid, 0, 0));
            if (DUAL) {
                f2 z = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(rz, rb + 8 * tid, 0, 0));
                a += z;
            }
            v.a = f4{a.x, a.y, 0.f, 0.f};
            v.b = v.a;
        } else if constexpr (CPL == 2) {
            v.a = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rw, rb + 16 * tid, 0, 0));
            if (DUAL) v.a += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rz, rb + 16 * tid, 0, 0));
            v.b = v.a;
        } else {
            v.a = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rw, rb + 16 * tid, 0, 0));
            v.b = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rw, rb + 4096 + 16 * tid, 0, 0));
            if (DUAL) {
                v.a += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rz, rb + 16 * tid, 0, 0));
                v.b += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rz, rb + 4096 + 16 * tid, 0, 0));
            }
        }
        return v;
    };
    RowT<CPL> r[ROWS];
#pragma unroll
    for (int i = 0; i < ROWS; i++) r[i] = ld(0, i);
    const __amdgpu_buffer_rsrc_t ry =
        __builtin_amdgcn_make_buffer_rsrc((void *)(y + t0 * 2 * ROWS * 512), (short)0, 0x7fffffff, 0x00020000);
    for (int k = 0; k < T; k++) {
        f4 c = r[0].a + r[0].b;
#pragma unroll
        for (int i = 1; i < ROWS; i++) c += r[i].a + r[i].b;
        if (k + 1 < T) {
#pragma unroll
            for (int i = 0; i < ROWS; i++) r[i] = ld(k + 1, i);
        }
#pragma unroll
        for (int bb = 0; bb < BPW; bb++) {
            const unsigned ob = (unsigned)(((k * 2 * ROWS) + wave * BPW + bb) * 8192) + 16u * lane;
#pragma unroll
            for (int s = 0; s < 8; s++)
                __builtin_amdgcn_raw_buffer_store_b128(c + (float)s, ry, ob + 1024u * s, 0, 2);
        }
    }
}

template <int LANES, int CPL, int ROWS, bool DUAL>
void run(const float *x, f4 *y, int wpc, const char *name)
{
    const int ntiles_rows = 131072; // 2^27 samples = 2^17 rows of 1024
    const int ntiles = ntiles_rows / ROWS;
    const int grid = 256 * wpc;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++)
        hipLaunchKernelGGL((k_pat<LANES, CPL, ROWS, DUAL>), dim3(grid), dim3(LANES), 0, 0, x, y, ntiles);
    CK(hipGetLastError());
    CK(hipEventRecord(e0));
    const int it = 20;
    for (int i = 0; i < it; i++)
        hipLaunchKernelGGL((k_pat<LANES, CPL, ROWS, DUAL>), dim3(grid), dim3(LANES), 0, 0, x, y, ntiles);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    const double rd = 8.0 * 1024 * ntiles_rows, wr = 2 * rd;
    printf("%-34s lanes %4d cpl %d rows %d dual %d wpc %d  %7.3f ms  total %5.0f GB/s\n", name, LANES, CPL, ROWS,
           (int)DUAL, wpc, ms, (rd + wr) / ms / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main()
{
    float *x;
    f4 *y;
    CK(hipMalloc(&x, (size_t)1 << 30));
    CK(hipMalloc(&y, (size_t)1 << 31));
    CK(hipMemset(x, 0, (size_t)1 << 30));
    CK(hipMemset(y, 0, (size_t)1 << 31));
    for (int rep = 0; rep < 2; rep++) {
        run<1024, 1, 8, true>(x, y, 1, "library (8B, dual)");
        run<1024, 1, 8, false>(x, y, 1, "8B single");
        run<512, 2, 8, false>(x, y, 1, "16B, 512 lanes, 8 rows");
        run<512, 2, 8, true>(x, y, 1, "16B dual, 512 lanes, 8 rows");
        run<512, 2, 4, false>(x, y, 2, "16B, 512 lanes, 4 rows, 2/CU");
        run<512, 2, 4, false>(x, y, 1, "16B, 512 lanes, 4 rows, 1/CU");
        run<256, 4, 8, false>(x, y, 1, "2x16B, 256 lanes, 8 rows");
        run<256, 4, 8, false>(x, y, 2, "2x16B, 256 lanes, 8 rows, 2/CU");
        run<256, 4, 4, false>(x, y, 2, "2x16B, 256 lanes, 4 rows, 2/CU");
        run<256, 4, 4, false>(x, y, 4, "2x16B, 256 lanes, 4 rows, 4/CU");
    }
    return 0;
}
