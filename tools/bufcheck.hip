// bufcheck: does a raw buffer load's range check include soffset on this GPU?  A 64-byte descriptor over a buffer of
// 4 KiB of 0xAB bytes; loads at (voffset, soffset) = (0, 0), (0, 128), (128, 0), (48, 8), (8, 48) -> prints the dwords.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned char *p, unsigned *out) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, 64, 0x00020000);
    const int vo[5] = {0, 0, 128, 48, 8}, so[5] = {0, 128, 0, 8, 48};
    for (int i = 0; i < 5; i++) out[i] = __builtin_amdgcn_raw_buffer_load_b32(r, vo[i], __builtin_amdgcn_readfirstlane(so[i]), 0);
}
int main() {
    unsigned char *d; unsigned *o, h[5];
    hipMalloc(&d, 4096); hipMemset(d, 0xAB, 4096); hipMalloc(&o, 64);
    hipLaunchKernelGGL(k, dim3(1), dim3(1), 0, 0, d, o);
    hipMemcpy(h, o, 20, hipMemcpyDeviceToHost);
    const char *lab[5] = {"v0 s0", "v0 s128", "v128 s0", "v48 s8", "v8 s48"};
    for (int i = 0; i < 5; i++) printf("%s: %08x\n", lab[i], h[i]);
    return 0;
}
