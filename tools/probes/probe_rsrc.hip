// Does the buffer range check include soffset?  A 2 MiB allocation filled with 7s, a descriptor
// over its first 64 B; lane 0 loads at voffset 0 with soffset 1 MiB (inside the allocation, outside
// the descriptor's range) and at voffset 1 MiB with soffset 0.  0 = dropped by the range check.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned *p, unsigned *out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned *>(p), 0, 64, 0x00020000);
    if (threadIdx.x == 0) {
        out[0] = __builtin_amdgcn_raw_buffer_load_b32(r, 0, 1 << 20, 0);   // soffset past the range
        out[1] = __builtin_amdgcn_raw_buffer_load_b32(r, 1 << 20, 0, 0);   // voffset past the range
        out[2] = __builtin_amdgcn_raw_buffer_load_b32(r, 60, 0, 0);        // in range
        out[3] = __builtin_amdgcn_raw_buffer_load_b32(r, 0, 60, 0);        // soffset in range
        out[4] = __builtin_amdgcn_raw_buffer_load_b32(r, 32, 32, 0);       // voffset + soffset = 64: past
    }
}
int main() {
    unsigned *p, *o, h[5];
    hipMalloc(&p, 2 << 20);
    hipMalloc(&o, 64);
    hipMemset(p, 7, 2 << 20);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, p, o);
    hipMemcpy(h, o, 20, hipMemcpyDeviceToHost);
    printf("soffset-past %#x voffset-past %#x in-range %#x soffset-in %#x sum-past %#x\n", h[0], h[1], h[2], h[3], h[4]);
    return 0;
}
