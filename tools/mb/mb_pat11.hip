// mb_pat11.hip -- sweep of the matrix-core firfilt's 1 read : 1 write memory
// pattern (dev tool; mb_bw4.hip holds the round-2 version).  A chunk is 2048
// complex outputs: the lanes of a 256-thread workgroup read its 2048 + 64
// input samples (four 16-byte loads per lane plus a 64-sample halo, as
// k_firfilt_mx) and write 2048 outputs (four 16-byte stores per lane);
// chunks are dealt grid-stride over 2^28 samples (the bench's step).  Swept:
//   WPC  resident workgroups per CU (the grid is 256 WPC): 1, 2 (the kernel), 3, 4
//   DEP  chunks of loads in flight per workgroup: 1, 2, 3 (the kernel)
//   ILV  the next chunk's loads issued between this chunk's stores (1) or all before them (0, the kernel)
//   NTS  non-temporal stores (1, the kernel) or plain
//   LDS  the chunk is written to LDS and read back (one barrier each way, as the kernel's plane staging)
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

template <int WPC, int DEP, bool ILV, bool NTS, bool LDS>
__global__ __launch_bounds__(256, WPC) void k_pat(const f4 *__restrict__ x, f4 *__restrict__ y, long long nch)
{
    __shared__ f4 st[LDS ? 1024 : 1];
    const int tid = threadIdx.x;
    const long long G = gridDim.x, w = blockIdx.x;
    const long long cnt = (nch - w + G - 1) / G;
    auto load = [&](long long k, f4 (&d)[5]) {
        const long long c = w + k * G;
        const bool in = k < cnt;
        const f4 *p = x + c * 1024 + tid;   // 2048 complex = 1024 f4
#pragma unroll
        for (int i = 0; i < 4; i++) d[i] = in ? p[256 * i] : f4{};
        d[4] = (in && tid < 32 && c > 0) ? x[c * 1024 - 32 + tid] : f4{};   // 64-sample halo
    };
    f4 r[DEP][5];
#pragma unroll
    for (int d = 0; d < DEP; d++) load(d, r[d]);
    for (long long k = 0; k < cnt; k++) {
        f4 c[5];
#pragma unroll
        for (int i = 0; i < 5; i++) c[i] = r[0][i];
#pragma unroll
        for (int d = 0; d + 1 < DEP; d++)
#pragma unroll
            for (int i = 0; i < 5; i++) r[d][i] = r[d + 1][i];
        if (!ILV) load(k + DEP, r[DEP - 1]);
        if (LDS) {
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 4; i++) st[tid + 256 * i] = c[i] + c[4];
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 4; i++) c[i] = st[(tid + 64 * i) & 1023];
        }
        const long long ch = w + k * G;
        f4 *q = y + ch * 1024 + tid;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const f4 v = c[i] + c[4];
            if (NTS) __builtin_nontemporal_store(v, q + 256 * i);
            else q[256 * i] = v;
            if (ILV && i == 1) {
                const long long c2 = w + (k + DEP) * G;
                const bool in = k + DEP < cnt;
                const f4 *p = x + c2 * 1024 + tid;
                r[DEP - 1][0] = in ? p[0] : f4{};
                r[DEP - 1][1] = in ? p[256] : f4{};
                r[DEP - 1][4] = (in && tid < 32 && c2 > 0) ? x[c2 * 1024 - 32 + tid] : f4{};
            }
            if (ILV && i == 3) {
                const long long c2 = w + (k + DEP) * G;
                const bool in = k + DEP < cnt;
                const f4 *p = x + c2 * 1024 + tid;
                r[DEP - 1][2] = in ? p[512] : f4{};
                r[DEP - 1][3] = in ? p[768] : f4{};
            }
        }
    }
}

struct Var {
    const char *name;
    void (*launch)(const f4 *, f4 *, long long);
};

template <int WPC, int DEP, bool ILV, bool NTS, bool LDS>
void launch(const f4 *x, f4 *y, long long nch)
{
    hipLaunchKernelGGL((k_pat<WPC, DEP, ILV, NTS, LDS>), dim3(256 * WPC), dim3(256), 0, 0, x, y, nch);
}

#define V(WPC, DEP, ILV, NTS, LDS) Var{"wpc" #WPC " dep" #DEP " ilv" #ILV " nts" #NTS " lds" #LDS, launch<WPC, DEP, ILV, NTS, LDS>}

int main()
{
    const long long n = 1ll << 28;   // complex samples
    const long long nch = n / 2048;
    f4 *x, *y;
    CK(hipMalloc(&x, n * 8));
    CK(hipMalloc(&y, n * 8));
    CK(hipMemset(x, 1, n * 8));
    CK(hipMemset(y, 0, n * 8));
    std::vector<Var> vs = {
        V(2, 3, false, true, true),  // the kernel's pattern
        V(2, 3, false, true, false), V(2, 3, true, true, true),  V(2, 2, true, true, true),  V(2, 1, true, true, true),
        V(1, 3, false, true, true),  V(1, 3, true, true, true),  V(3, 2, false, true, true), V(3, 2, true, true, true),
        V(4, 2, false, true, true),  V(4, 2, true, true, true),  V(4, 1, true, true, true),  V(2, 3, false, false, true),
        V(2, 3, true, false, true),  V(1, 2, true, true, false), V(2, 2, true, true, false),
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> t(vs.size());
    for (int pass = 0; pass < 3; pass++) {
        for (size_t v = 0; v < vs.size(); v++) {
            for (int i = 0; i < 10; i++) vs[v].launch(x, y, nch);
            CK(hipEventRecord(e0));
            const int it = 20;
            for (int i = 0; i < it; i++) vs[v].launch(x, y, nch);
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
        printf("%-34s ms %.4f %.4f %.4f  best %.4f  %.0f GB/s\n", vs[v].name, t[v][0], t[v][1], t[v][2], best,
               16.0 * n / best / 1e6);
    }
    return 0;
}
