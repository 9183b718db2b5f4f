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

// DMA: the chunk span reaches LDS by LDS-DMA (global_load_lds_dwordx4, no
// VGPR staging) into a ring of DEP+1 buffers, DEP chunks ahead; each chunk is
// read back from LDS (one barrier per chunk) and stored as in the kernel.
// Waits are explicit: after chunk k's loads a wave has issued its stores of
// that iteration and (DEP-1) further iterations of 4 loads + 4 stores.
template <int WPC, int DEP>
__global__ __launch_bounds__(256, WPC) void k_dma(const f4 *__restrict__ x, f4 *__restrict__ y, long long nch)
{
    __shared__ f4 st[(DEP + 1) * 1056];
    const int tid = threadIdx.x, wave = tid >> 6;
    const long long G = gridDim.x, w = blockIdx.x;
    const long long cnt = (nch - w + G - 1) / G;
    auto issue = [&](long long k) {
        const long long c = w + (k < cnt ? k : cnt - 1) * G;   // past the end: re-load the last chunk
        f4 *buf = st + (int)(k % (DEP + 1)) * 1056;
        if (wave == 0 && tid < 32) {
            const f4 *hp = c > 0 ? x + c * 1024 - 32 + tid : x + tid;
            __builtin_amdgcn_global_load_lds((const void *)hp, (__attribute__((address_space(3))) void *)(buf), 16, 0, 0);
        }
        const f4 *p = x + c * 1024 + tid;
#pragma unroll
        for (int i = 0; i < 4; i++)
            __builtin_amdgcn_global_load_lds((const void *)(p + 256 * i),
                                             (__attribute__((address_space(3))) void *)(buf + 32 + 256 * i + 64 * wave), 16, 0, 0);
    };
#pragma unroll
    for (int d = 0; d < DEP; d++) issue(d);
    constexpr int N = 4 + 8 * (DEP - 1);
    constexpr int WT = (N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8);
    for (long long k = 0; k < cnt; k++) {
        __builtin_amdgcn_s_waitcnt(WT);
        __builtin_amdgcn_s_barrier();
        // LDS reads in asm: the compiler would otherwise wait for every
        // outstanding LDS-DMA (vmcnt(0)) before them
        const unsigned a0 = (unsigned)(size_t)(st + (int)(k % (DEP + 1)) * 1056);
        const unsigned ab = a0 + 16u * (32 + tid), ah = a0 + 16u * (tid & 31);
        f4 c[5];
        asm volatile("ds_read_b128 %0, %1" : "=v"(c[0]) : "v"(ab));
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(c[1]) : "v"(ab));
        asm volatile("ds_read_b128 %0, %1 offset:8192" : "=v"(c[2]) : "v"(ab));
        asm volatile("ds_read_b128 %0, %1 offset:12288" : "=v"(c[3]) : "v"(ab));
        asm volatile("ds_read_b128 %0, %1" : "=v"(c[4]) : "v"(ah));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]));
        issue(k + DEP);
        const long long ch = w + k * G;
        f4 *q = y + ch * 1024 + tid;
#pragma unroll
        for (int i = 0; i < 4; i++) __builtin_nontemporal_store(c[i] + c[4], q + 256 * i);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f & ~0xc00f);
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

template <int WPC, int DEP>
void launch_dma(const f4 *x, f4 *y, long long nch)
{
    hipLaunchKernelGGL((k_dma<WPC, DEP>), dim3(256 * WPC), dim3(256), 0, 0, x, y, nch);
}
#define D(WPC, DEP) Var{"dma wpc" #WPC " dep" #DEP, launch_dma<WPC, DEP>}

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
    std::vector<Var> vs;
    if (getenv("MB_DMA_ONLY") == nullptr)
        vs = {
            V(2, 3, false, true, true),  // the kernel's pattern
            V(2, 3, false, true, false), V(2, 3, true, true, true),  V(2, 2, true, true, true),  V(2, 1, true, true, true),
            V(1, 3, false, true, true),  V(1, 3, true, true, true),  V(3, 2, false, true, true), V(3, 2, true, true, true),
            V(4, 2, false, true, true),  V(4, 2, true, true, true),  V(4, 1, true, true, true),  V(2, 3, false, false, true),
            V(2, 3, true, false, true),  V(1, 2, true, true, false), V(2, 2, true, true, false),
        };
    else
        vs = {V(2, 3, false, true, true), V(2, 1, true, true, true)};
    for (Var v : {D(1, 2), D(1, 3), D(1, 4), D(2, 1), D(2, 2), D(2, 3), D(3, 1), D(3, 2), D(4, 1), D(4, 2)}) vs.push_back(v);
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
