// Does a raw buffer load whose VGPR offset is "negative" (wrapped) plus an
// immediate offset that brings it back into range read the element or 0?
// out[t] = load(x, (t - sh) * 4 + 1024) with the 1024 folded into the
// instruction's offset field (A) or added in a VGPR first (B).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float *x, int n, int sh, float *outa, float *outb)
{
    const int t = threadIdx.x;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, n * 4, 0x00020000);
    const unsigned v = (unsigned)(t - sh) * 4u;
    outa[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, v + 1024u, 0, 0));
    unsigned w = v + 1024u;
    asm volatile("" : "+v"(w));
    outb[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, w, 0, 0));
}
int main()
{
    const int n = 1024;
    float h[n], *x, *a, *b;
    for (int i = 0; i < n; i++) h[i] = 1000.f + i;
    hipMalloc(&x, n * 4); hipMalloc(&a, 256); hipMalloc(&b, 256);
    hipMemcpy(x, h, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, x, n, 16, a, b);
    float ha[64], hb[64];
    hipMemcpy(ha, a, 256, hipMemcpyDeviceToHost);
    hipMemcpy(hb, b, 256, hipMemcpyDeviceToHost);
    // t = 0..15: (t - 16) * 4 is negative, + 1024 -> element t + 240
    printf("t  folded  vgpr-sum  expected\n");
    for (int t = 0; t < 20; t += 3) printf("%2d %8.1f %8.1f %8.1f\n", t, ha[t], hb[t], 1000.f + t - 16 + 256);
    return 0;
}
