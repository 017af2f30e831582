// probe_fetch.hip -- diagnostic: what rocprofv3's FETCH_SIZE reports for a coalesced streaming read of
// exactly B bytes with 4-, 8- and 16-byte loads per lane (every byte read once, nothing reused, 1 GiB
// >> L2 + MALL), and for a 512-MiB write (WRITE_SIZE).  Calibrates tools/pmc_summary.py's FETCH
// correction per load width.  Not part of the product.
//   hipcc -O3 --offload-arch=gfx950 -o probe_fetch probe_fetch.hip
//   rocprofv3 --pmc FETCH_SIZE -- ./probe_fetch ; rocprofv3 --pmc WRITE_SIZE -- ./probe_fetch
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <typename T>
__device__ __forceinline__ unsigned fold(T v) {
    const unsigned *u = reinterpret_cast<const unsigned *>(&v);
    unsigned a = 0;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(T) / 4); ++i) a ^= u[i];
    return a;
}

template <typename T>
__global__ __launch_bounds__(256) void k_read(const T *__restrict__ x, long n, unsigned *out) {
    unsigned acc = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) acc ^= fold(x[i]);
    if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;   // practically never: no store traffic
}

__global__ __launch_bounds__(256) void k_write(float4 *__restrict__ y, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        y[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

int main() {
    const size_t B = 1ull << 30;
    void *x;
    unsigned *o;
    CK(hipMalloc(&x, B));
    CK(hipMalloc(&o, 1 << 20));
    CK(hipMemset(x, 1, B));
    const dim3 g(256 * 8), b(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_read<float>, g, b, 0, 0, (const float *)x, (long)(B / 4), o);
        hipLaunchKernelGGL(k_read<float2>, g, b, 0, 0, (const float2 *)x, (long)(B / 8), o);
        hipLaunchKernelGGL(k_read<float4>, g, b, 0, 0, (const float4 *)x, (long)(B / 16), o);
        hipLaunchKernelGGL(k_write, g, b, 0, 0, (float4 *)x, (long)(B / 32));   // 512 MiB written
    }
    CK(hipDeviceSynchronize());
    printf("read %zu bytes per k_read launch, wrote %zu per k_write\n", B, B / 2);
    return 0;
}
