// lq_runtime.hip -- device, stream and memory plumbing behind the C-ABI.
//
// The reference reports every error by fprintf(stderr) + exit(1)
// (e.g. src/filter/src/firfilt.c:66-69); HIP failures here do the same with
// the HIP error string, so a missing or broken GPU fails loudly -- there is no
// CPU fallback anywhere in this library.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <mutex>

#include "lq_kernels.h"
#include "lq_device.h"

void lq_check(hipError_t e, const char *what, const char *file, int line)
{
    if (e != hipSuccess) {
        fprintf(stderr, "error: liquid-mi355x: %s failed at %s:%d: %s\n", what, file, line,
                hipGetErrorString(e));
        exit(1);
    }
}

extern "C" void lqrt_require_device(const char *who)
{
    static int checked = 0;
    if (checked) return;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) {
        fprintf(stderr,
                "error: %s: no HIP device available (liquid-mi355x runs the filter path on the GPU "
                "only; there is no CPU fallback)\n",
                who ? who : "liquid-mi355x");
        exit(1);
    }
    checked = 1;
}

extern "C" void *lqrt_malloc(size_t bytes)
{
    lqrt_require_device("lqrt_malloc");
    void *p = nullptr;
    if (bytes == 0) bytes = 16;
    LQ_CHECK(hipMalloc(&p, bytes));
    // the memset runs on the null stream, which does not order with the
    // objects' non-blocking streams: wait for it before anyone reads p
    LQ_CHECK(hipMemsetAsync(p, 0, bytes, nullptr));
    LQ_CHECK(hipStreamSynchronize(nullptr));
    return p;
}

extern "C" void lqrt_free(void *p)
{
    if (p) LQ_CHECK(hipFree(p));
}

extern "C" void *lqrt_host_alloc(size_t bytes)
{
    lqrt_require_device("lqrt_host_alloc");
    void *p = nullptr;
    if (bytes == 0) bytes = 16;
    // fine-grained (coherent) memory: the small-call path reads and writes
    // these buffers while kernels run (the host spins on a flag the kernel
    // raises; kernels read inputs in place right after the host wrote them),
    // which HIP guarantees to be visible without a synchronisation only for
    // coherent allocations
    LQ_CHECK(hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped));
    return p;
}

extern "C" void lqrt_host_free(void *p)
{
    if (p) LQ_CHECK(hipHostFree(p));
}

extern "C" void *lqrt_stream_create(void)
{
    lqrt_require_device("lqrt_stream_create");
    hipStream_t s;
    LQ_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return (void *)s;
}

extern "C" void lqrt_stream_destroy(void *s)
{
    if (s) LQ_CHECK(hipStreamDestroy((hipStream_t)s));
}

extern "C" void lqrt_h2d(void *dst, const void *src, size_t bytes, void *stream)
{
    if (!bytes) return;
    LQ_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
}

extern "C" void lqrt_d2h(void *dst, const void *src, size_t bytes, void *stream)
{
    if (!bytes) return;
    LQ_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
}

extern "C" void lqrt_d2d(void *dst, const void *src, size_t bytes, void *stream)
{
    if (!bytes) return;
    LQ_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
}

extern "C" void lqrt_memset(void *dst, size_t bytes, void *stream)
{
    if (!bytes) return;
    LQ_CHECK(hipMemsetAsync(dst, 0, bytes, (hipStream_t)stream));
}

extern "C" void lqrt_sync(void *stream)
{
    LQ_CHECK(hipStreamSynchronize((hipStream_t)stream));
}

extern "C" int lqrt_is_device_ptr(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return a.type == hipMemoryTypeDevice;
}

// One twiddle table per device: W_4096^e = exp(-2*pi*i*e/4096), computed in
// double on the host and rounded once to float.  Every power-of-two transform
// up to 4096 points indexes it with stride 4096/N.
extern "C" const float *lqrt_twiddles(void)
{
    static std::mutex mu;
    static float *tables[64] = {nullptr};
    int dev = 0;
    LQ_CHECK(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) {
        fprintf(stderr, "error: liquid-mi355x: device index %d out of range (64 devices max)\n", dev);
        exit(1);
    }
    std::lock_guard<std::mutex> g(mu);
    if (!tables[dev]) {
        float h[2 * LQ_TW_N];
        for (int e = 0; e < LQ_TW_N; e++) {
            double a = -2.0 * M_PI * (double)e / (double)LQ_TW_N;
            h[2 * e] = (float)cos(a);
            h[2 * e + 1] = (float)sin(a);
        }
        float *d = nullptr;
        // the table is followed by LQRT_ZEROS bytes of zeros (lqrt_zeros)
        LQ_CHECK(hipMalloc(&d, sizeof(h) + LQRT_ZEROS));
        LQ_CHECK(hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice));
        LQ_CHECK(hipMemset(d + 2 * LQ_TW_N, 0, LQRT_ZEROS));
        LQ_CHECK(hipDeviceSynchronize());
        tables[dev] = d;
    }
    return tables[dev];
}

extern "C" const float *lqrt_zeros(void) { return lqrt_twiddles() + 2 * LQ_TW_N; }

// ------------------------------------------------------------ small calls
// The per-call liquid.h API (firfilt_execute, dotprod_execute,
// firpfbch2_execute ...) returns only after its result is in host memory.
// A stream synchronisation costs about 5 us on top of the kernels
// (tools/mb/mb_latency.hip); instead the last kernel of a call copies the
// result into pinned host memory, releases it at system scope and raises a
// per-object flag word the host spins on.
__global__ __launch_bounds__(256) void k_copyout_signal(const unsigned *__restrict__ src, unsigned *dst,
                                                        unsigned nw, unsigned *flag, unsigned seq)
{
    const unsigned n4 = nw >> 2;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
    for (unsigned i = threadIdx.x; i < n4; i += 256) d4[i] = s4[i];
    for (unsigned i = 4 * n4 + threadIdx.x; i < nw; i += 256) dst[i] = src[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" void lqrt_copyout_signal(const void *src, void *dst, size_t bytes, unsigned *flag, unsigned seq,
                                    void *stream)
{
    if (bytes > LQRT_COPYOUT_MAX || (bytes & 3) || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) {
        fprintf(stderr, "error: liquid-mi355x: copy-out of %zu bytes out of contract\n", bytes);
        exit(1);
    }
    hipLaunchKernelGGL(k_copyout_signal, dim3(1), dim3(256), 0, (hipStream_t)stream, (const unsigned *)src,
                       (unsigned *)dst, (unsigned)(bytes >> 2), flag, seq);
    LQ_CHECK(hipGetLastError());
}

extern "C" void lqrt_wait_flag(const unsigned *flag, unsigned seq, void *stream)
{
    // spin for up to ~2 ms (a small call takes ~10 us), then block on the stream
    for (long i = 0; i < (1L << 21); i++) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return;
        __builtin_ia32_pause();
    }
    LQ_CHECK(hipStreamSynchronize((hipStream_t)stream));
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        fprintf(stderr, "error: liquid-mi355x: small-call completion flag not raised\n");
        exit(1);
    }
}

extern "C" void lqrt_device_sync(void)
{
    LQ_CHECK(hipDeviceSynchronize());
}
