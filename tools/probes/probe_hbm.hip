// probe_hbm.hip -- diagnostic: HBM read rate of the ETSI channel filter's access pattern (one
// 256-thread workgroup streams one 1 MiB channel row with 16-B loads) under different load forms,
// depths and occupancies.  Not part of the product; answers "what is the achievable floor".
//   hipcc -O3 --offload-arch=gfx950 -o probe_hbm probe_hbm.hip && ./probe_hbm
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <bool NT>
__device__ __forceinline__ float4 ld(const float4 *p) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    if constexpr (NT) {
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else return *p;
}

// register ring: DEPTH groups of 5 float4 per thread in flight (the chanfilt's PFD = 2 is DEPTH 2)
template <bool NT, int DEPTH>
__global__ __launch_bounds__(256) void k_ring(const float4 *__restrict__ x, long row4, uint32_t *out, int rows) {
    extern __shared__ float4 pad_lds[];
    uint32_t acc = 0;
    for (int row = blockIdx.x; row < rows; row += gridDim.x) {
        const float4 *p = x + (size_t)row * row4;
        const long ng = (row4 + 1279) / 1280;   // groups of 256 x 5 float4
        float4 v[DEPTH][5];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d)
#pragma unroll
            for (int r = 0; r < 5; ++r) v[d][r] = ld<NT>(p + min((long)d * 1280 + r * 256 + threadIdx.x, row4 - 1));
        for (long g = 0; g < ng; g += DEPTH) {
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
                for (int r = 0; r < 5; ++r)
                    acc ^= __float_as_uint(v[d][r].x) ^ __float_as_uint(v[d][r].y) ^ __float_as_uint(v[d][r].z) ^
                           __float_as_uint(v[d][r].w);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int r = 0; r < 5; ++r)
                    v[d][r] = ld<NT>(p + min((g + DEPTH + d) * 1280 + r * 256 + threadIdx.x, row4 - 1));
            }
        }
    }
    if (acc == 0x9E3779B9u) pad_lds[threadIdx.x] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

// register ring through a buffer resource with cache-policy bits AUX (gfx940+: sc0 1, nt 2, sc1 16)
template <int AUX, int DEPTH>
__global__ __launch_bounds__(256) void k_ringb(const float4 *__restrict__ x, long row4, uint32_t *out, int rows) {
    extern __shared__ float4 pad_lds[];
    typedef float f4v __attribute__((ext_vector_type(4)));
    uint32_t acc = 0;
    for (int row = blockIdx.x; row < rows; row += gridDim.x) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(x + (size_t)row * row4), 0,
                                                                           (int)(row4 * 16), 0x00020000);
        const long ng = (row4 + 1279) / 1280;
        f4v v[DEPTH][5];
#pragma unroll
        for (int d = 0; d < DEPTH; ++d)
#pragma unroll
            for (int q = 0; q < 5; ++q) v[d][q] = __builtin_amdgcn_raw_buffer_load_b128(r, (q * 256 + threadIdx.x) * 16, d * 1280 * 16, AUX);
        for (long g = 0; g < ng; g += DEPTH) {
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
                for (int q = 0; q < 5; ++q)
                    acc ^= __float_as_uint(v[d][q].x) ^ __float_as_uint(v[d][q].y) ^ __float_as_uint(v[d][q].z) ^
                           __float_as_uint(v[d][q].w);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < 5; ++q)
                    v[d][q] = __builtin_amdgcn_raw_buffer_load_b128(r, (q * 256 + threadIdx.x) * 16, (int)((g + DEPTH + d) * 1280 * 16), AUX);
            }
        }
    }
    if (acc == 0x9E3779B9u) pad_lds[threadIdx.x] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

// LDS-DMA: each wave streams its quarter of every 20 KB tile into its own LDS ring, keeping at most
// INFL wave-instructions (1 KiB each) in flight
template <int AUX, int INFL>
__global__ __launch_bounds__(256) void k_glds(const float4 *__restrict__ x, long row4, uint32_t *out, int rows) {
    extern __shared__ float4 lds[];   // >= 4 waves x 32 KiB used as rings
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float4 *ring = lds + wv * 2048;   // 32 KiB per wave
    int slot = 0;
    for (int row = blockIdx.x; row < rows; row += gridDim.x) {
        const float4 *p = x + (size_t)row * row4;
        for (long q = wv * 64; q < row4; q += 256) {
            __builtin_amdgcn_global_load_lds((const void *)(p + q + lane), (__attribute__((address_space(3))) void *)(ring + slot * 64), 16, 0, AUX);
            slot = (slot + 1) & 31;
            if constexpr (INFL == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else if constexpr (INFL == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0 && ring[3].x == 1234.5f) out[blockIdx.x] = 1;
}

typedef void (*KFn)(const float4 *, long, uint32_t *, int);

int main() {
    const int rows = 8192;
    const long row_bytes = 131072L * 8;
    const long row4 = row_bytes / 16;
    float4 *x;
    uint32_t *o;
    CK(hipMalloc(&x, rows * row_bytes));
    CK(hipMalloc(&o, rows * 4));
    CK(hipMemset(x, 0x3c, rows * row_bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct V { const char *name; KFn f; int grid; int lds; };
    std::vector<V> vs = {
        {"ringb d2 aux0 (default) 2wg", k_ringb<0, 2>, rows, 72 * 1024},
        {"ringb d2 aux2 (nt) 2wg", k_ringb<2, 2>, rows, 72 * 1024},
        {"ringb d2 aux1 (sc0) 2wg", k_ringb<1, 2>, rows, 72 * 1024},
        {"ringb d2 aux3 (sc0 nt) 2wg", k_ringb<3, 2>, rows, 72 * 1024},
        {"ringb d2 aux16 (sc1) 2wg", k_ringb<16, 2>, rows, 72 * 1024},
        {"ringb d2 aux17 (sc0 sc1) 2wg", k_ringb<17, 2>, rows, 72 * 1024},
        {"ringb d2 aux18 (sc1 nt) 2wg", k_ringb<18, 2>, rows, 72 * 1024},
        {"ringb d2 aux19 (sc0 sc1 nt) 2wg", k_ringb<19, 2>, rows, 72 * 1024},
        {"ringb d3 aux2 (nt) 2wg", k_ringb<2, 3>, rows, 72 * 1024},
        {"ringb d3 aux19 (sc0 sc1 nt) 2wg", k_ringb<19, 3>, rows, 72 * 1024},
        {"ring d1 plain 2wg/cu", k_ring<false, 1>, rows, 72 * 1024},
        {"ring d2 plain 2wg/cu", k_ring<false, 2>, rows, 72 * 1024},
        {"ring d2 nt    2wg/cu", k_ring<true, 2>, rows, 72 * 1024},
        {"ring d3 plain 2wg/cu", k_ring<false, 3>, rows, 72 * 1024},
        {"ring d3 nt    2wg/cu", k_ring<true, 3>, rows, 72 * 1024},
        {"ring d4 nt    2wg/cu", k_ring<true, 4>, rows, 72 * 1024},
        {"ring d2 plain 4wg/cu", k_ring<false, 2>, rows, 36 * 1024},
        {"ring d2 nt    4wg/cu", k_ring<true, 2>, rows, 36 * 1024},
        {"ring d2 nt    1wg/cu", k_ring<true, 2>, rows, 150 * 1024},
        {"ring d4 nt    1wg/cu", k_ring<true, 4>, rows, 150 * 1024},
        {"ring d2 nt persist512", k_ring<true, 2>, 512, 72 * 1024},
        {"ring d3 nt persist512", k_ring<true, 3>, 512, 72 * 1024},
        {"glds plain inf16 1wg", k_glds<0, 16>, rows, 130 * 1024},
        {"glds nt inf8 1wg", k_glds<2, 8>, rows, 130 * 1024},
        {"glds nt inf16 1wg", k_glds<2, 16>, rows, 130 * 1024},
        {"glds nt inf24 1wg", k_glds<2, 24>, rows, 130 * 1024},
        {"glds plain inf16 persist256", k_glds<0, 16>, 256, 130 * 1024},
        {"glds nt inf16 persist256", k_glds<2, 16>, 256, 130 * 1024},
    };
    for (int pass = 0; pass < 2; ++pass)
        for (auto &v : vs) {
            std::vector<float> t;
            for (int rep = 0; rep < 6; ++rep) {
                CK(hipEventRecord(a));
                hipLaunchKernelGGL(v.f, dim3(v.grid), dim3(256), v.lds, 0, (const float4 *)x, row4, o, rows);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (rep) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            if (pass) printf("%-30s median %.4f ms  %.1f GB/s  (best %.1f)\n", v.name, t[t.size() / 2],
                             rows * row_bytes / (t[t.size() / 2] * 1e-3) / 1e9, rows * row_bytes / (t[0] * 1e-3) / 1e9);
        }
    return 0;
}
