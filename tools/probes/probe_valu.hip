// probe_valu.hip -- diagnostic: VALU issue rate per SIMD on gfx950 for the instruction forms the
// compat decimator and the ETSI stage-1 filter are built from: plain v_fmac_f32, v_fmac_f32 with a
// DPP operand (row_shl:1), v_mov_b32_dpp, v_pk_fma_f32, and v_mul_f32 -- independent instructions
// (8 accumulators), one and two waves per SIMD.  Not part of the product.
//   hipcc -O3 --offload-arch=gfx950 -o probe_valu probe_valu.hip && ./probe_valu
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITERS = 4096;   // x 32 instructions per iteration

template <int FORM>
__global__ __launch_bounds__(256) void k_valu(float *out, float s) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = s * threadIdx.x, c = s + threadIdx.x;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if constexpr (FORM == 0) {
                asm volatile("v_fmac_f32 %0, %8, %9\n\tv_fmac_f32 %1, %8, %9\n\tv_fmac_f32 %2, %8, %9\n\tv_fmac_f32 %3, %8, %9\n\t"
                             "v_fmac_f32 %4, %8, %9\n\tv_fmac_f32 %5, %8, %9\n\tv_fmac_f32 %6, %8, %9\n\tv_fmac_f32 %7, %8, %9"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
            } else if constexpr (FORM == 1) {
                asm volatile("v_fmac_f32_dpp %0, %8, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_fmac_f32_dpp %1, %8, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_fmac_f32_dpp %2, %8, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_fmac_f32_dpp %3, %8, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_fmac_f32_dpp %4, %8, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_fmac_f32_dpp %5, %8, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_fmac_f32_dpp %6, %8, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_fmac_f32_dpp %7, %8, %9 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
            } else if constexpr (FORM == 2) {
                asm volatile("v_mov_b32_dpp %0, %8 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_mov_b32_dpp %1, %8 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_mov_b32_dpp %2, %8 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_mov_b32_dpp %3, %8 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_mov_b32_dpp %4, %9 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_mov_b32_dpp %5, %9 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_mov_b32_dpp %6, %9 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                             "v_mov_b32_dpp %7, %9 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
            } else if constexpr (FORM == 3) {
                asm volatile("v_mul_f32 %0, %8, %9\n\tv_mul_f32 %1, %8, %9\n\tv_mul_f32 %2, %8, %9\n\tv_mul_f32 %3, %8, %9\n\t"
                             "v_add_f32 %4, %8, %9\n\tv_add_f32 %5, %8, %9\n\tv_sub_f32 %6, %8, %9\n\tv_sub_f32 %7, %8, %9"
                             : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7) : "v"(b), "v"(c));
            } else {
                typedef float f2 __attribute__((ext_vector_type(2)));
                f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, q = {b, c};
                asm volatile("v_pk_fma_f32 %0, %4, %4, %0\n\tv_pk_fma_f32 %1, %4, %4, %1\n\tv_pk_fma_f32 %2, %4, %4, %2\n\t"
                             "v_pk_fma_f32 %3, %4, %4, %3\n\tv_pk_fma_f32 %0, %4, %4, %0\n\tv_pk_fma_f32 %1, %4, %4, %1\n\t"
                             "v_pk_fma_f32 %2, %4, %4, %2\n\tv_pk_fma_f32 %3, %4, %4, %3"
                             : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(q));
                a0 = p0.x; a1 = p0.y; a2 = p1.x; a3 = p1.y; a4 = p2.x; a5 = p2.y; a6 = p3.x; a7 = p3.y;
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int FORM>
int run(const char *name, float *out, int wps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = 256 * wps;   // 256-thread workgroups: one wave per SIMD of a CU each
    hipLaunchKernelGGL(k_valu<FORM>, dim3(grid), dim3(256), 0, 0, out, 1.0f);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_valu<FORM>, dim3(grid), dim3(256), 0, 0, out, 1.0f);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double instr_per_wave = (double)ITERS * 32;   // the asm instructions (loop overhead aside)
    const double ns = ms * 1e6 / 5;
    printf("%-22s waves/SIMD %d: %.3f ms per launch, %.3f ns per instruction per SIMD (%.2f cycles at 2.4 GHz)\n", name, wps,
           ns / 1e6, ns / (instr_per_wave * wps), ns / (instr_per_wave * wps) * 2.4);
    return 0;
}

int main() {
    float *out;
    CK(hipMalloc(&out, 256 * 4 * 256 * 4 * sizeof(float)));
    for (int w = 1; w <= 4; w *= 2) {
        run<0>("v_fmac_f32", out, w);
        run<1>("v_fmac_f32_dpp", out, w);
        run<2>("v_mov_b32_dpp", out, w);
        run<3>("v_mul/add/sub_f32", out, w);
        run<4>("v_pk_fma_f32", out, w);
    }
    return 0;
}
