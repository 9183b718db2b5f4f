// mb_rows.hip -- the firpfbch2 analyzer's memory pattern without its
// arithmetic (dev tool): one persistent 1024-thread workgroup per CU streams
// rows of 1024 complex samples (8 KB) and writes, per two rows... (16 blocks
// of 8 KB per 8 rows).  Row loads: W=8: lane c loads column c (one 8-byte
// load per lane per row, the library kernel); W=16: lane l loads columns
// 2l', 2l'+1 of row r + (l >> 9) (16-byte loads, half the instructions) and
// the pairs are spread back to one column per lane with ds_bpermute.
// Stores: each wave writes one 8 KB block per 8 rows as 8 x 1 KB
// instructions (16 B per lane), plain or non-temporal.  PF rows in flight.
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

template <int W, bool NTS, bool STORE, bool LOAD>
__global__ __launch_bounds__(1024, 1) void k_rows(const f2 *__restrict__ x, long long nrows, f4 *__restrict__ y,
                                                  int rpw)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long r0 = (long long)blockIdx.x * rpw;
    long long r1 = r0 + rpw;
    if (r1 > nrows) r1 = nrows;
    f2 acc[8];
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = f2{0.f, 0.f};
    for (long long r = r0; r < r1; r += 8) {
        f2 w[8];
        if (LOAD) {
            if (W == 8) {
#pragma unroll
                for (int i = 0; i < 8; i++) w[i] = x[(r + i) * 1024 + tid];
            } else {
                // lanes 0..511 load row r+2i, lanes 512..1023 row r+2i+1, 16 B each
                const int half = tid >> 9, l = tid & 511;
                f4 v[4];
#pragma unroll
                for (int i = 0; i < 4; i++)
                    v[i] = reinterpret_cast<const f4 *>(x + (r + 2 * i + half) * 1024)[l];
                // wave w (cols 64w..64w+63) needs lanes 32w'.. of both halves: the pair of
                // column c = 64w + lane sits in lane (c >> 1) of half 0 (row r+2i) /
                // half 1 (row r+2i+1) -- other waves: go through LDS
                __shared__ f4 st[2][512];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    __syncthreads();
                    st[half][l] = v[i];
                    __syncthreads();
                    const f4 a = st[0][tid >> 1], b = st[1][tid >> 1];
                    w[2 * i] = (tid & 1) ? f2{a.z, a.w} : f2{a.x, a.y};
                    w[2 * i + 1] = (tid & 1) ? f2{b.z, b.w} : f2{b.x, b.y};
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) w[i] = f2{(float)i, (float)r};
        }
#pragma unroll
        for (int i = 0; i < 8; i++) acc[i] += w[i];
        if (STORE) {
            // 16 blocks of 8 KB per 8 rows; wave `wave` writes block 2*(r/8)*8 + wave
            f4 *Yb = y + ((r / 8) * 16 + wave) * 512;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const f4 val = {acc[q].x, acc[q].y, acc[(q + 1) & 7].x, (float)q};
                if (NTS) __builtin_nontemporal_store(val, Yb + 64 * q + lane);
                else Yb[64 * q + lane] = val;
            }
        }
    }
    if (!STORE && acc[0].x == 1234.5f) y[0] = f4{acc[1].x, 0, 0, 0};
}

template <int W, bool NTS, bool STORE, bool LOAD>
static void run(const char *name, const f2 *x, long long nrows, f4 *y)
{
    const int grid = 256;
    const int rpw = (int)(((nrows + grid - 1) / grid + 7) / 8 * 8);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_rows<W, NTS, STORE, LOAD>), dim3(grid), dim3(1024), 0, 0, x, nrows, y, rpw);
    CK(hipEventRecord(e0));
    const int it = 10;
    for (int i = 0; i < it; i++)
        hipLaunchKernelGGL((k_rows<W, NTS, STORE, LOAD>), dim3(grid), dim3(1024), 0, 0, x, nrows, y, rpw);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= it;
    const double rd = LOAD ? nrows * 8192.0 : 0, wr = STORE ? nrows * 16384.0 : 0;
    printf("%-36s %8.3f ms  rd %6.0f  wr %6.0f  total %6.0f GB/s\n", name, ms, rd / ms / 1e6, wr / ms / 1e6,
           (rd + wr) / ms / 1e6);
    fflush(stdout);
}

int main()
{
    const long long nrows = 1 << 17;   // 2^27 samples, 1 GiB in, 2 GiB out
    f2 *x;
    f4 *y;
    CK(hipMalloc(&x, nrows * 8192));
    CK(hipMalloc(&y, nrows * 16384));
    CK(hipMemset(x, 0, nrows * 8192));
    for (int rep = 0; rep < 2; rep++) {
        run<8, true, false, true>("rows 8B/lane, no stores", x, nrows, y);
        run<16, true, false, true>("rows 16B/lane+LDS, no stores", x, nrows, y);
        run<8, true, true, false>("stores only nt", x, nrows, y);
        run<8, false, true, false>("stores only plain", x, nrows, y);
        run<8, true, true, true>("rows 8B + stores nt", x, nrows, y);
        run<8, false, true, true>("rows 8B + stores plain", x, nrows, y);
        run<16, true, true, true>("rows 16B+LDS + stores nt", x, nrows, y);
        run<16, false, true, true>("rows 16B+LDS + stores plain", x, nrows, y);
    }
    return 0;
}
