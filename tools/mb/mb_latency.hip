// mb_latency.hip -- round-trip latency of one small GPU call (dev tool): the
// floor under the per-call liquid.h API (firfilt_execute, dotprod_execute,
// firpfbch2_execute ...).  Variants: how the inputs reach the GPU (pageable /
// pinned hipMemcpyAsync, zero-copy reads of pinned host memory, kernel
// arguments) and how the host learns the result is there (stream sync,
// event sync, spinning on a flag the kernel writes to pinned host memory).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                                \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

struct Win {
    float2 v[64];
};

__global__ void k_empty() {}

// y = sum_k h[k] w[63-k] from a device window
__global__ void k_dot_dev(const float *h, const float2 *w, float2 *y)
{
    __shared__ float2 part[64];
    const int t = threadIdx.x;
    float2 a = w[63 - t];
    part[t] = make_float2(h[t] * a.x, h[t] * a.y);
    __syncthreads();
    if (t == 0) {
        float2 s = {0, 0};
        for (int i = 0; i < 64; i++) s = make_float2(s.x + part[i].x, s.y + part[i].y);
        y[0] = s;
    }
}

// same, window passed as a kernel argument, result + flag to host memory
__global__ void k_dot_arg(const float *h, Win w, float2 *y, volatile unsigned *flag, unsigned seq)
{
    __shared__ float2 part[64];
    const int t = threadIdx.x;
    float2 a = w.v[63 - t];
    part[t] = make_float2(h[t] * a.x, h[t] * a.y);
    __syncthreads();
    if (t == 0) {
        float2 s = {0, 0};
        for (int i = 0; i < 64; i++) s = make_float2(s.x + part[i].x, s.y + part[i].y);
        y[0] = s;
        __threadfence_system();
        *flag = seq;
    }
}

// window read from pinned host memory (zero copy), result + flag to host memory
__global__ void k_dot_zc(const float *h, const float2 *w, float2 *y, volatile unsigned *flag, unsigned seq)
{
    __shared__ float2 part[64];
    const int t = threadIdx.x;
    float2 a = w[63 - t];
    part[t] = make_float2(h[t] * a.x, h[t] * a.y);
    __syncthreads();
    if (t == 0) {
        float2 s = {0, 0};
        for (int i = 0; i < 64; i++) s = make_float2(s.x + part[i].x, s.y + part[i].y);
        y[0] = s;
        __threadfence_system();
        *flag = seq;
    }
}

typedef std::chrono::steady_clock clk;
static double us_since(clk::time_point t0, int n)
{
    return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / n;
}

static void spin(volatile unsigned *flag, unsigned seq)
{
    while (*flag != seq) {
    }
}

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float *h;
    float2 *dw, *dy;
    CK(hipMalloc(&h, 256));
    CK(hipMalloc(&dw, 512));
    CK(hipMalloc(&dy, 16));
    CK(hipMemset(h, 0, 256));
    float2 *pw, *py;
    unsigned *pflag;
    CK(hipHostMalloc(&pw, 512, hipHostMallocDefault));
    CK(hipHostMalloc(&py, 64, hipHostMallocDefault));
    CK(hipHostMalloc(&pflag, 64, hipHostMallocDefault));
    float2 *uw = (float2 *)malloc(512), *uy = (float2 *)malloc(64);
    memset(uw, 0, 512);
    memset(pw, 0, 512);
    *pflag = 0;
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int N = 2000;
    for (int rep = 0; rep < 2; rep++) {
        clk::time_point t0;
        t0 = clk::now();
        for (int i = 0; i < N; i++) {
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
            CK(hipStreamSynchronize(s));
        }
        printf("empty kernel + stream sync                  %7.2f us\n", us_since(t0, N));
        t0 = clk::now();
        for (int i = 0; i < N; i++) {
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
            CK(hipEventRecord(ev, s));
            CK(hipEventSynchronize(ev));
        }
        printf("empty kernel + event sync                   %7.2f us\n", us_since(t0, N));
        t0 = clk::now();
        for (int i = 0; i < N; i++) {
            CK(hipMemcpyAsync(dw, uw, 512, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_dot_dev, dim3(1), dim3(64), 0, s, h, dw, dy);
            CK(hipMemcpyAsync(uy, dy, 8, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
        }
        printf("pageable H2D + kernel + pageable D2H + sync %7.2f us\n", us_since(t0, N));
        t0 = clk::now();
        for (int i = 0; i < N; i++) {
            CK(hipMemcpyAsync(dw, pw, 512, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_dot_dev, dim3(1), dim3(64), 0, s, h, dw, dy);
            CK(hipMemcpyAsync(py, dy, 8, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
        }
        printf("pinned H2D + kernel + pinned D2H + sync     %7.2f us\n", us_since(t0, N));
        unsigned seq = 1000 * rep;
        t0 = clk::now();
        for (int i = 0; i < N; i++) {
            ++seq;
            hipLaunchKernelGGL(k_dot_zc, dim3(1), dim3(64), 0, s, h, pw, py, pflag, seq);
            CK(hipStreamSynchronize(s));
        }
        printf("zero-copy in/out kernel + stream sync       %7.2f us\n", us_since(t0, N));
        t0 = clk::now();
        for (int i = 0; i < N; i++) {
            ++seq;
            hipLaunchKernelGGL(k_dot_zc, dim3(1), dim3(64), 0, s, h, pw, py, pflag, seq);
            spin(pflag, seq);
        }
        printf("zero-copy in/out kernel + spin on flag      %7.2f us\n", us_since(t0, N));
        Win w;
        memset(&w, 0, sizeof(w));
        t0 = clk::now();
        for (int i = 0; i < N; i++) {
            ++seq;
            hipLaunchKernelGGL(k_dot_arg, dim3(1), dim3(64), 0, s, h, w, py, pflag, seq);
            spin(pflag, seq);
        }
        printf("window as kernel arg + spin on flag         %7.2f us\n", us_since(t0, N));
        t0 = clk::now();
        for (int i = 0; i < N; i++) {
            ++seq;
            hipLaunchKernelGGL(k_dot_arg, dim3(1), dim3(64), 0, s, h, w, py, pflag, seq);
            CK(hipStreamSynchronize(s));
        }
        printf("window as kernel arg + stream sync          %7.2f us\n", us_since(t0, N));
        // 4 KB in (firpfbch2 block), 8 KB out, zero copy
        t0 = clk::now();
        for (int i = 0; i < N; i++) {
            CK(hipMemcpyAsync(dw, pw, 512, hipMemcpyHostToDevice, s));
            ++seq;
            hipLaunchKernelGGL(k_dot_zc, dim3(1), dim3(64), 0, s, h, dw, py, pflag, seq);
            spin(pflag, seq);
        }
        printf("pinned H2D + kernel + spin                  %7.2f us\n", us_since(t0, N));
        CK(hipStreamSynchronize(s));
    }
    return 0;
}
