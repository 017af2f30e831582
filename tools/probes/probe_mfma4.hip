// probe_mfma4.hip -- diagnostic for an MFMA form of the ETSI stage-1 FIR (48 taps, decimate by 10):
// (1) the operand / result layout of v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4, K = 1),
// (2) whether a chain of them equals the fmaf chain bit for bit (c = fma(a, b, c) per element),
// (3) its issue rate at one and two waves per SIMD, alone and with a VALU conversion per MFMA
//     beside it (the int16 -> f32 conversion an SC16 B operand needs), and the 16x16x4 form's.
// Not part of the product.
//   hipcc -O3 --offload-arch=gfx950 -o probe_mfma4 probe_mfma4.hip && ./probe_mfma4
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(const float *a, const float *b, float *d) {
    const int l = threadIdx.x;
    f4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[4 * l + r] = c[r];
    // A broadcast: cbsz 4 = groups of 16 blocks, abid 5 = every block takes block 5's A
    f4 e = {0.f, 0.f, 0.f, 0.f};
    e = __builtin_amdgcn_mfma_f32_4x4x1f32(a[l], b[l], e, 4, 5, 0);
    for (int r = 0; r < 4; ++r) d[256 + 4 * l + r] = e[r];
}

// K steps: lane l supplies a[k * 64 + l], b[k * 64 + l]
__global__ void k_chain(const float *a, const float *b, float *d, int K) {
    const int l = threadIdx.x;
    f4 c = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) c = __builtin_amdgcn_mfma_f32_4x4x1f32(a[64 * k + l], b[64 * k + l], c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[4 * l + r] = c[r];
}

constexpr int ITERS = 2048;
// FORM 0: 4x4x1, 8 independent accumulators; 1: 4x4x1, 2 accumulators (two chains);
// 2: 4x4x1 + one SDWA-style int16 -> f32 conversion per MFMA; 3: 16x16x4, 4 accumulators
template <int FORM>
__global__ __launch_bounds__(256) void k_rate(float *out, float s) {
    float a = s * threadIdx.x, b = s + threadIdx.x;
    f4 c[8];
    for (int i = 0; i < 8; ++i) c[i] = f4{a, b, a + 1.f, b + 1.f};
    uint32_t raw = threadIdx.x * 0x10001u;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if constexpr (FORM == 0) c[r] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[r], 0, 0, 0);
            else if constexpr (FORM == 1) c[r & 1] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c[r & 1], 0, 0, 0);
            else if constexpr (FORM == 2) {
                float bb = (float)(int16_t)(raw >> (16 * (r & 1)));
                raw += 0x00030001u;
                c[r] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, bb, c[r], 0, 0, 0);
            } else c[r & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[r & 3], 0, 0, 0);
        }
    }
    float t = 0.f;
    for (int i = 0; i < 8; ++i) t += c[i][0] + c[i][1] + c[i][2] + c[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = t;
}

template <int FORM>
static int rate(const char *name, float *dout, int wps) {
    // one workgroup of 256 = 1 wave per SIMD per workgroup; 256 CUs x wps workgroups
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int grid = 256 * wps;
    k_rate<FORM><<<grid, 256>>>(dout, 1.0001f);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    k_rate<FORM><<<grid, 256>>>(dout, 1.0001f);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    int clk = 0;
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
    double cyc = ms * 1e-3 * clk * 1e3;
    double per = cyc / ((double)ITERS * 8 * wps);   // cycles per MFMA per wave (one wave per SIMD per wps)
    printf("%-34s waves/SIMD %d: %.2f ms, %.1f cycles per MFMA per wave (clock %.0f MHz)\n", name, wps, ms, per, clk / 1e3);
    return 0;
}

int main() {
    float ha[64], hb[64], hd[256];
    for (int l = 0; l < 64; ++l) { ha[l] = (float)(l + 1); hb[l] = (float)(1000 * (l + 1)); }
    float *da, *db, *dd;
    const int K = 78;
    CK(hipMalloc(&da, 64 * K * 4));
    CK(hipMalloc(&db, 64 * K * 4));
    CK(hipMalloc(&dd, 256 * 256 * 2 * 4));
    CK(hipMemcpy(da, ha, 256, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb, 256, hipMemcpyHostToDevice));
    k_layout<<<1, 64>>>(da, db, dd);
    CK(hipMemcpy(hd, dd, 1024, hipMemcpyDeviceToHost));
    // decode: value = (la + 1) * 1000 * (lb + 1) -> which a-lane and b-lane fed (lane, r)
    int ok = 1;
    printf("layout: lane, r -> (a lane, b lane)\n");
    for (int l = 0; l < 64; ++l) {
        for (int r = 0; r < 4; ++r) {
            double v = hd[4 * l + r];
            int found = 0;
            for (int x = 0; x < 64 && !found; ++x)
                for (int y = 0; y < 64 && !found; ++y)
                    if ((double)(x + 1) * 1000.0 * (y + 1) == v) {
                        if (l < 8 || l % 16 == 0) printf("  lane %2d r %d: a%2d b%2d\n", l, r, x, y);
                        // hypothesis: block l/4, row r (a lane 4 (l/4) + r), column l%4 (b lane l)
                        if (x != 4 * (l / 4) + r || y != l) ok = 0;
                        found = 1;
                    }
            if (!found) { printf("  lane %d r %d: %g unmatched\n", l, r, v); ok = 0; }
        }
    }
    printf("layout hypothesis (D[lane][r] = A[lane 4(lane/4)+r] * B[lane]): %s\n", ok ? "HOLDS" : "FAILS");
    {
        float he[256];
        CK(hipMemcpy(he, dd + 256, 1024, hipMemcpyDeviceToHost));
        int okb = 1;
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r)
                if ((double)he[4 * l + r] != (double)(4 * 5 + r + 1) * 1000.0 * (l + 1)) okb = 0;
        printf("cbsz 4 / abid 5 broadcast (D[lane][r] = A[lane 20+r] * B[lane]): %s (lane 0: %g %g %g %g)\n",
               okb ? "HOLDS" : "FAILS", he[0], he[1], he[2], he[3]);
    }

    // exactness: random chain vs host fmaf in the same order
    std::vector<float> A(64 * K), B(64 * K);
    uint32_t st = 12345;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 8) & 0xFFFF) / 32768.0f - 1.0f; };
    for (int k = 0; k < K; ++k)
        for (int l = 0; l < 64; ++l) {
            A[64 * k + l] = (k % 5 == 0) ? 0.f : rnd() * 1e-3f * (float)(1 + k);
            B[64 * k + l] = rnd() * 3.0517578125e-05f * 20000.f;
        }
    CK(hipMemcpy(da, A.data(), 64 * K * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, B.data(), 64 * K * 4, hipMemcpyHostToDevice));
    k_chain<<<1, 64>>>(da, db, dd, K);
    CK(hipMemcpy(hd, dd, 1024, hipMemcpyDeviceToHost));
    int mism = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            float c = 0.f;
            for (int k = 0; k < K; ++k) c = fmaf(A[64 * k + 4 * (l / 4) + r], B[64 * k + l], c);
            uint32_t u, v;
            memcpy(&u, &c, 4);
            memcpy(&v, &hd[4 * l + r], 4);
            mism += u != v;
        }
    printf("chain of %d 4x4x1 MFMAs vs the fmaf chain: %d of 256 outputs differ\n", K, mism);

    rate<0>("4x4x1, 8 accumulators", dd, 1);
    rate<0>("4x4x1, 8 accumulators", dd, 2);
    rate<1>("4x4x1, 2 accumulators", dd, 1);
    rate<1>("4x4x1, 2 accumulators", dd, 2);
    rate<2>("4x4x1 + cvt per MFMA, 8 acc", dd, 1);
    rate<2>("4x4x1 + cvt per MFMA, 8 acc", dd, 2);
    rate<3>("16x16x4, 4 accumulators", dd, 1);
    rate<3>("16x16x4, 4 accumulators", dd, 2);
    return 0;
}
