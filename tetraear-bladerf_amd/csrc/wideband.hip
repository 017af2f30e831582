// wideband.hip -- C3: a 20 MSps wideband capture split into M = 800 carriers at
// 25 kHz spacing by a polyphase filter bank (PFB), each carrier resampled to 72 kHz (4 samples
// per symbol) for the ETSI timing stage (etsi_rx.hip k_timing) and lower MAC.
//
// The reference tunes the SDR to one carrier per capture (capture.py, modern.py:1886-2034); this
// is the channeliser BASELINE.json's north_star names, so oracle/wideband.py (float64 numpy) is
// its specification and parity is a tolerance on y (fp32 FFT), then bit-exact from y onwards.
//
//   analysis  u_j[r]  = sum_{p<P} h[pM + r] x[n_j - pM - r],   n_j = L - 1 + jD, L = MP
//             Y_j[k]  = sum_r u_j[r] e^{+i 2 pi k r / M}      (rocFFT, backward, unnormalised)
//             v_k[j]  = (-i)^{(k j) mod 4} Y_j[k]             (D = M/4: the mixer term, exact)
//   resample  y_k[n]  = sum_{q<Q} g[rho_n + up q] v_k[floor(down n / up) + Q - 1 - q],
//             rho_n = (down n) mod up, Q = Lg / up             (fs/D -> 72 kHz, RRC matched filter)
//   synthesis (test signal) x[n] = sum_j D h[n - jD] W_j[n mod M] + noise,
//             W_j[r] = sum_k s_k[j] e^{+i 2 pi k r / M}       (carrier k at +k * fs/M)
// v_k differs from the textbook channel output by the constant phase e^{+i 2 pi k / M} (n_j mod M
// = jD - 1), which the receiver's differential decision and CFO estimate do not see.
//
// Bytes: the analysis reads 8 B per wideband sample (the fold's P = 2 re-reads come from L2),
// writes/reads Y once (8 B x M per D input samples = 32 B per input sample at D = 200 -- the FFT
// stage dominates), and the resampler writes 8 B per 72 kHz output.
#include <cstdlib>

#include "common.h"


namespace {

constexpr int RS_T = 48;    // resampler outputs per workgroup (12 per wave; rows fit 64 KB of LDS)
constexpr int RS_C = 64;    // resampler channels per workgroup (one per lane)
constexpr int RS_QP = 48;   // row of the phase-major resampler tap table gT[up][RS_QP]

__device__ __forceinline__ float2 rot_mi(float2 z, int q) {   // z * (-i)^q, exact
    switch (q & 3) {
        case 0: return z;
        case 1: return make_float2(z.y, -z.x);
        case 2: return make_float2(-z.x, -z.y);
        default: return make_float2(-z.y, z.x);
    }
}

// u[j][r] for j in [j0, j0 + JB): one thread per r (coalesced, descending x addresses).
template <int P>
__global__ __launch_bounds__(256) void k_pfb_fold(const float2 *__restrict__ x, int M, int D, int nblk,
                                                  const float *__restrict__ h, float2 *__restrict__ u, int JB) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= M) return;
    float hp[P];
#pragma unroll
    for (int p = 0; p < P; ++p) hp[p] = h[p * M + r];
    const int L = P * M;
    const int j0 = blockIdx.y * JB, j1 = min(nblk, j0 + JB);
    for (int j = j0; j < j1; ++j) {
        const long n = (long)L - 1 + (long)j * D - r;
        float ar = 0.f, ai = 0.f;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const float2 v = x[n - (long)p * M];
            ar = fmaf(hp[p], v.x, ar);
            ai = fmaf(hp[p], v.y, ai);
        }
        u[(size_t)j * M + r] = make_float2(ar, ai);
    }
}

// ---------------------------------------------------------------- fused analysis: fold + FFT
// Y_j[k] for M = 800 = 8 x 4 x 5 x 5 (mixed-radix Stockham, backward, unnormalised) fused with the
// fold: a workgroup walks JB consecutive blocks; the wideband samples sit in an LDS ring (each
// block brings D = 200 new samples, loaded AF blocks ahead into registers), stage 1 folds its
// eight inputs u_j[i] = sum_p h[pM + i] x[n_j - pM - i] straight from the ring (thread b < 100
// always owns i = b + 100 r, so its 8 P taps stay in registers), stages 2-3 run through a padded
// LDS frame, stage 4 stores Y_j in natural order (5 coalesced 8-B stores per thread).  HBM: the D
// new samples (8 B each, plus a 1600-sample halo per workgroup) in, the 800 outputs out -- against
// fold-then-rocFFT's extra Y write + read + re-read of x from L2 per block.
constexpr int AN_M = 800, AN_T = 256, AN_AF = 8;
constexpr int AN_FR = AN_M + AN_M / 8;                  // padded frame
constexpr int AN_TW2 = 0, AN_TW3 = 3 * 8, AN_TW4 = AN_TW3 + 4 * 32, AN_TWN = AN_TW4 + 4 * 160;   // r-major

__device__ __forceinline__ int an_pad(int i) { return i + (i >> 3); }
__device__ __forceinline__ float2 c_add(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 c_sub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 c_mul(float2 a, float2 b) {
    return make_float2(fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 c_pi(float2 a) { return make_float2(-a.y, a.x); }   // a * (+i)

// backward DFTs (X_k = sum_n a_n e^{+2 pi i n k / R})
__device__ __forceinline__ void bdft4(float2 &a0, float2 &a1, float2 &a2, float2 &a3) {
    const float2 t0 = c_add(a0, a2), t1 = c_sub(a0, a2), t2 = c_add(a1, a3), t3 = c_pi(c_sub(a1, a3));
    a0 = c_add(t0, t2);
    a2 = c_sub(t0, t2);
    a1 = c_add(t1, t3);
    a3 = c_sub(t1, t3);
}
__device__ __forceinline__ void bdft8(float2 *v) {
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6], o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    bdft4(e0, e1, e2, e3);
    bdft4(o0, o1, o2, o3);
    const float s = 0.70710678118654752f;
    o1 = make_float2((o1.x - o1.y) * s, (o1.x + o1.y) * s);      // * e^{+i pi/4}
    o2 = c_pi(o2);
    o3 = make_float2(-(o3.x + o3.y) * s, (o3.x - o3.y) * s);     // * e^{+3 i pi/4}
    v[0] = c_add(e0, o0); v[4] = c_sub(e0, o0);
    v[1] = c_add(e1, o1); v[5] = c_sub(e1, o1);
    v[2] = c_add(e2, o2); v[6] = c_sub(e2, o2);
    v[3] = c_add(e3, o3); v[7] = c_sub(e3, o3);
}
__device__ __forceinline__ void bdft5(float2 *a) {
    const float c1 = 0.30901699437494742f, c2 = -0.80901699437494742f;   // cos(2 pi/5), cos(4 pi/5)
    const float s1 = 0.95105651629515357f, s2 = 0.58778525229247313f;    // sin(2 pi/5), sin(4 pi/5)
    const float2 t1 = c_add(a[1], a[4]), t2 = c_add(a[2], a[3]), t3 = c_sub(a[1], a[4]), t4 = c_sub(a[2], a[3]);
    const float2 b1 = make_float2(a[0].x + c1 * t1.x + c2 * t2.x, a[0].y + c1 * t1.y + c2 * t2.y);
    const float2 b2 = make_float2(a[0].x + c2 * t1.x + c1 * t2.x, a[0].y + c2 * t1.y + c1 * t2.y);
    const float2 e1 = make_float2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y);   // X1 = b1 + i e1
    const float2 e2 = make_float2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y);   // X2 = b2 + i e2
    a[0] = c_add(a[0], c_add(t1, t2));
    a[1] = c_add(b1, c_pi(e1));
    a[4] = c_sub(b1, c_pi(e1));
    a[2] = c_add(b2, c_pi(e2));
    a[3] = c_sub(b2, c_pi(e2));
}

// Roles by wave: waves 0-2 fold + transform + store, wave 3 only loads (the new samples of block
// j + 1 + AF while block j is transformed, written into the ring during block j's stage 1).  A
// wave's vmcnt counts its loads and stores in one queue: were one wave to do both, waiting for a
// prefetched load would also wait for every store issued since.  Two frames alternate per block,
// so a block costs three barriers (after stages 1, 2, 3).
template <int P>
__global__ __launch_bounds__(AN_T) void k_pfb_analysis(const float4 *__restrict__ x2, int nblk, int JB,
                                                       const float *__restrict__ h, const float2 *__restrict__ twg,
                                                       float2 *__restrict__ Y) {
    constexpr int M = AN_M, D = M / 4, L = P * M;
    constexpr int RING = L + D <= 2048 ? 2048 : (L + D <= 4096 ? 4096 : 8192);   // samples, power of 2
    __shared__ float4 ring4[RING / 2];
    __shared__ float2 frb[2][AN_FR];
    __shared__ float2 tw[AN_TWN];
    const float2 *ring = reinterpret_cast<const float2 *>(ring4);
    const int t = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const int j0 = blockIdx.x * JB, j1 = min(nblk, j0 + JB);
    for (int i = t; i < AN_TWN; i += AN_T) tw[i] = twg[i];
    // the first block's window x[j0 D, j0 D + L) (pairs: j0 D is even)
    for (int q = t; q < L / 2; q += AN_T) {
        const long pr = (long)j0 * (D / 2) + q;
        ring4[(int)(pr & (RING / 2 - 1))] = x2[pr];
    }
    if (wv == 3) {
        // loader: lane l carries pairs l and l + 64 (< D / 2 = 100) of the new samples of block j,
        // x[L + (j - 1) D, + D); loads are unconditional (lane and block clamped) so no branch joins
        // wait for them
        const int l = t - 192;
        const int q0 = l, q1 = min(l + 64, D / 2 - 1);
        auto base = [&](int j) -> long { return (long)(L + (long)(min(j, j1 - 1) - 1) * D) / 2; };
        // four register slots, one per block of the unrolled loop (plain variables and a macro, so
        // they stay in VGPRs), each waited for with the count of the loads issued after it
        static_assert(AN_AF == 8, "loader unroll");
        float4 s0a = x2[base(j0 + 1) + q0], s0b = x2[base(j0 + 1) + q1];
        float4 s1a = x2[base(j0 + 2) + q0], s1b = x2[base(j0 + 2) + q1];
        float4 s2a = x2[base(j0 + 3) + q0], s2b = x2[base(j0 + 3) + q1];
        float4 s3a = x2[base(j0 + 4) + q0], s3b = x2[base(j0 + 4) + q1];
        float4 s4a = x2[base(j0 + 5) + q0], s4b = x2[base(j0 + 5) + q1];
        float4 s5a = x2[base(j0 + 6) + q0], s5b = x2[base(j0 + 6) + q1];
        float4 s6a = x2[base(j0 + 7) + q0], s6b = x2[base(j0 + 7) + q1];
        float4 s7a = x2[base(j0 + 8) + q0], s7b = x2[base(j0 + 8) + q1];
        __syncthreads();
#define AN_LOAD_BLOCK(J, A, B)                                                                  \
        {                                                                                       \
            const int jj = (J);                                                                 \
            if (jj + 1 < j1) {   /* block jj + 1's samples (fetched AF blocks ago) to the ring */ \
                const long bb = (long)(L + (long)jj * D) / 2;                                   \
                ring4[(int)((bb + q0) & (RING / 2 - 1))] = A;                                   \
                if (l + 64 < D / 2) ring4[(int)((bb + l + 64) & (RING / 2 - 1))] = B;           \
            }                                                                                   \
            A = x2[base(jj + 1 + AN_AF) + q0];   /* block jj + 1 + AF's */                      \
            B = x2[base(jj + 1 + AN_AF) + q1];                                                  \
            __syncthreads(); /* after stage 1 */                                                \
            __syncthreads(); /* after stage 2 */                                                \
            __syncthreads(); /* after stage 3 */                                                \
        }
        int j = j0;
        for (; j + 8 <= j1; j += 8) {
            AN_LOAD_BLOCK(j, s0a, s0b)
            AN_LOAD_BLOCK(j + 1, s1a, s1b)
            AN_LOAD_BLOCK(j + 2, s2a, s2b)
            AN_LOAD_BLOCK(j + 3, s3a, s3b)
            AN_LOAD_BLOCK(j + 4, s4a, s4b)
            AN_LOAD_BLOCK(j + 5, s5a, s5b)
            AN_LOAD_BLOCK(j + 6, s6a, s6b)
            AN_LOAD_BLOCK(j + 7, s7a, s7b)
        }
        if (j < j1) AN_LOAD_BLOCK(j, s0a, s0b)
        if (j + 1 < j1) AN_LOAD_BLOCK(j + 1, s1a, s1b)
        if (j + 2 < j1) AN_LOAD_BLOCK(j + 2, s2a, s2b)
        if (j + 3 < j1) AN_LOAD_BLOCK(j + 3, s3a, s3b)
        if (j + 4 < j1) AN_LOAD_BLOCK(j + 4, s4a, s4b)
        if (j + 5 < j1) AN_LOAD_BLOCK(j + 5, s5a, s5b)
        if (j + 6 < j1) AN_LOAD_BLOCK(j + 6, s6a, s6b)
#undef AN_LOAD_BLOCK
        return;
    }
    float hr[8][P];
    if (t < 100) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int p = 0; p < P; ++p) hr[r][p] = h[p * M + t + 100 * r];
    }
    __syncthreads();
    for (int j = j0; j < j1; ++j) {
        float2 *fa = frb[(j - j0) & 1], *fb = frb[((j - j0) & 1) ^ 1];
        const long nj = (long)L - 1 + (long)j * D;
        // stage 1 (R = 8, Ns = 1): butterfly t < 100 on u[t + 100 r], folded from the ring
        if (t < 100) {
            float2 v[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int i = t + 100 * r;
                float ar = 0.f, ai = 0.f;
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const float2 xv = ring[(int)((nj - p * M - i) & (RING - 1))];
                    ar = fmaf(hr[r][p], xv.x, ar);
                    ai = fmaf(hr[r][p], xv.y, ai);
                }
                v[r] = make_float2(ar, ai);
            }
            bdft8(v);
#pragma unroll
            for (int r = 0; r < 8; ++r) fa[an_pad(8 * t + r)] = v[r];
        }
        __syncthreads();
        // stage 2 (R = 4, Ns = 8): 200 butterflies on 192 threads, fa -> fb
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            const int b = t + 192 * h2;
            if (b < 200) {
                float2 v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = fa[an_pad(b + 200 * r)];
                const int m = b & 7;
#pragma unroll
                for (int r = 1; r < 4; ++r) v[r] = c_mul(v[r], tw[AN_TW2 + (r - 1) * 8 + m]);
                bdft4(v[0], v[1], v[2], v[3]);
                const int base = (b >> 3) * 32 + m;
#pragma unroll
                for (int r = 0; r < 4; ++r) fb[an_pad(base + 8 * r)] = v[r];
            }
        }
        __syncthreads();
        // stage 3 (R = 5, Ns = 32): 160 butterflies, fb -> fa
        if (t < 160) {
            float2 v[5];
#pragma unroll
            for (int r = 0; r < 5; ++r) v[r] = fb[an_pad(t + 160 * r)];
            const int m = t & 31;
#pragma unroll
            for (int r = 1; r < 5; ++r) v[r] = c_mul(v[r], tw[AN_TW3 + (r - 1) * 32 + m]);
            bdft5(v);
            const int base = (t >> 5) * 160 + m;
#pragma unroll
            for (int r = 0; r < 5; ++r) fa[an_pad(base + 32 * r)] = v[r];
        }
        __syncthreads();
        // stage 4 (R = 5, Ns = 160): outputs k = t + 160 r, natural order, to HBM
        if (t < 160) {
            float2 v[5];
#pragma unroll
            for (int r = 0; r < 5; ++r) v[r] = fa[an_pad(t + 160 * r)];
#pragma unroll
            for (int r = 1; r < 5; ++r) v[r] = c_mul(v[r], tw[AN_TW4 + (r - 1) * 160 + t]);
            bdft5(v);
            // Y stored with the nt policy through a buffer resource on the block's row: the serial
            // C3 step 0.616 -> 0.600 ms (analysis -3 %, the resampler reading Y -5 %; sc1: 0.610)
            const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(Y + (size_t)j * M, 0, 8 * M, 0x00020000);
            // the mixer term here, once per output: v_k[j] = (-i)^{(k j) mod 4} Y_j[k]
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                const int k = t + 160 * r, q = (k * (j & 3)) & 3;
                const float a = (q & 1) ? v[r].y : v[r].x, bb = (q & 1) ? -v[r].x : v[r].y;
                typedef unsigned u2v __attribute__((ext_vector_type(2)));
                const float2 o = (q & 2) ? make_float2(-a, -bb) : make_float2(a, bb);
                __builtin_amdgcn_raw_buffer_store_b64(u2v{__float_as_uint(o.x), __float_as_uint(o.y)}, yr, 8 * k, 0,
                                                      2 /* nt */);
            }
        }
        // block j + 1's stage 1 writes the other frame; its stage 2 (after the next barrier) is the
        // first to touch this one again
    }
}

// Two blocks per iteration (k_pfb_analysis's next step): blocks j and j + 1 go through
// the stages together, so one iteration's three barriers and LDS round trips serve 2 x 800 outputs,
// and more of the workgroup works in each stage: five compute waves (stage 1: 200 butterflies, stage
// 2: 400, stages 3 and 4: 320 each) and one loader wave.  Per block the operations are
// k_pfb_analysis's, in the same order.  The loader writes the next pair's 2 D new samples into the
// ring during stage 2 (after every stage-1 read of the pair's windows), so the ring holds one pair's
// windows, L + D samples.
//   DM = 4 D / M: 1 (D = 200, 4x oversampled carriers at 100 kHz, mixer (-i)^{kj}) or 2 (D = 400,
//   2x at 50 kHz, mixer (-1)^{kj}: half the blocks -- half the FFTs and half of Y -- for a prototype
//   of P = 5 branches, since images now alias onto a carrier from 37.5 kHz instead of 87.5).
//   A power-of-two ring is indexed by masks; the D = 400 ring (L + D = 4400) is 4608 samples,
//   indexed by a per-block base and one conditional wrap per read.
constexpr int A2_C = 320, A2_T = A2_C + 64, A2_AF = 3;   // compute threads, + loader wave; pairs ahead

template <int P, int DM> struct A2Cfg {
    static constexpr int M = AN_M, D = M * DM / 4, L = P * M;
    static constexpr int RING = L + D <= 2048 ? 2048 : (L + D <= 4096 ? 4096 : ((L + D + 511) / 512) * 512);
    static constexpr bool POW2 = (RING & (RING - 1)) == 0;
    static constexpr int NLD = (D + 63) / 64;                 // loader float4 loads per lane per pair
    static constexpr int WAVES = L + D <= 4096 ? 5 : 3;      // waves per SIMD the LDS allows
};
template <int R> __device__ __forceinline__ int rwrap(int i) {   // i in (-R, 2R) -> [0, R)
    if constexpr ((R & (R - 1)) == 0) {
        return i & (R - 1);
    } else {
        i = i < 0 ? i + R : i;
        return i >= R ? i - R : i;
    }
}
template <int R> __device__ __forceinline__ int rwrap_lo(int i) {   // i in (-R, R) -> [0, R)
    if constexpr ((R & (R - 1)) == 0) {
        return i & (R - 1);
    } else {
        return i < 0 ? i + R : i;
    }
}

template <int P, int DM>
__global__ __launch_bounds__(A2_T, (A2Cfg<P, DM>::WAVES)) void k_pfb_analysis2(const float4 *__restrict__ x2, int nblk,
                                                                             int JB, const float *__restrict__ h,
                                                                             const float2 *__restrict__ twg,
                                                                             float2 *__restrict__ Y) {
    using Cf = A2Cfg<P, DM>;
    constexpr int M = Cf::M, D = Cf::D, L = Cf::L, RING = Cf::RING, NLD = Cf::NLD;
    static_assert((P - 1) * M + 700 < RING, "a fold read is at most one ring length behind rbase (rwrap_lo)");
    __shared__ float4 ring4[RING / 2];
    __shared__ float2 frb[2][2][AN_FR];   // [block of the pair][ping-pong]
    __shared__ float2 tw[AN_TWN];
    const float2 *ring = reinterpret_cast<const float2 *>(ring4);
    const int t = threadIdx.x;
    const int j0 = blockIdx.x * JB, j1 = min(nblk, j0 + JB);
    const int npair = (j1 - j0 + 1) / 2;
    for (int i = t; i < AN_TWN; i += A2_T) tw[i] = twg[i];
    // the first pair's windows x[j0 D, j0 D + L + D) (pairs of samples: j0 D is even), within the
    // capture: its last block's window ends at sample L - 1 + (nblk - 1) D.  Ring position of pair q:
    // (pair index) mod RING / 2, the window's first pair at 0
    const long npr = (long)(L + (long)(nblk - 1) * D) / 2;   // pairs of samples any block reads
    const long pr0 = (long)j0 * (D / 2);                      // ring pair 0
    for (int q = t; q < (L + D) / 2; q += A2_T) {
        if (pr0 + q < npr) ring4[q] = x2[pr0 + q];            // L + D <= RING: no wrap yet
    }
    if (t >= A2_C) {
        // loader: pair i (blocks j0 + 2i, +1) adds the samples x[L + (j0 + 2i - 1) D, L + (j0 + 2i + 1) D)
        // beyond the previous pair's windows: D pairs of samples from newbase(i); lane l carries pairs
        // l + 64 m (< D), loaded A2_AF pairs ahead and written into the ring during the stage 2 before
        const int l = t - A2_C;
        // loads through a buffer resource over the capture: one 32-bit lane offset, the pair's start
        // as the wave-uniform soffset, and the range check returning 0 past the capture (no clamps,
        // no 64-bit addresses held across the prefetch: those spilled)
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(x2), 0, (int)(16 * npr),
                                                                            0x00020000);
        const long nb0 = (long)(L + (long)(j0 - 1) * D) / 2;   // newbase(0)
        const int vo = 16 * (int)(nb0 + l);
        // ring pair position of newbase(i) + l: (L + D) / 2 - D + l + D i (mod RING / 2)
        int rpos = rwrap<RING / 2>((L + D) / 2 - D + l + D);     // for pair 1
        float4 sl[A2_AF][NLD];                                   // slot s: pair i + 1 while pair i (i mod AF = s) runs
        auto fetch = [&](float4 (&v)[NLD], int i) __attribute__((always_inline)) {
#pragma unroll
            for (int m = 0; m < NLD; ++m) {
                const nt_f4 w = __builtin_amdgcn_raw_buffer_load_b128(xr, vo + 1024 * m, 16 * D * i, 0);
                v[m] = make_float4(w.x, w.y, w.z, w.w);
            }
        };
        auto step = [&](float4 (&v)[NLD], int ii) __attribute__((always_inline)) {
            __syncthreads();   // after stage 1 of pair ii: its windows have been read
            if (ii + 1 < npair) {
#pragma unroll
                for (int m = 0; m < NLD; ++m)
                    if (l + 64 * m < D) ring4[rwrap<RING / 2>(rpos + 64 * m)] = v[m];
            }
            rpos = rwrap<RING / 2>(rpos + D);
            fetch(v, ii + 1 + A2_AF);
            __syncthreads();   // after stage 2
            __syncthreads();   // after stage 3
        };
        static_assert(A2_AF == 3, "loader unroll");
        fetch(sl[0], 1);
        fetch(sl[1], 2);
        fetch(sl[2], 3);
        __syncthreads();
        int i = 0;
        for (; i + 3 <= npair; i += 3) {
            step(sl[0], i);
            step(sl[1], i + 1);
            step(sl[2], i + 2);
        }
        if (i < npair) step(sl[0], i);
        if (i + 1 < npair) step(sl[1], i + 1);
        return;
    }
    // stage-1 thread: block bb of the pair, butterfly tt on u[tt + 100 r]
    const int bb = t / 100, tt = t - 100 * bb;
    float hr[8][P];
    if (t < 200) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int p = 0; p < P; ++p) hr[r][p] = h[p * M + tt + 100 * r];
    }
    __syncthreads();
    // ring position of sample n_j - tt of block j = ja + bb: the window's last sample, L - 1 + bb D
    // at the first pair (ring sample 0 = x[j0 D]), + 2 D per pair
    int rbase = rwrap<RING>(L - 1 + bb * D - tt);
    for (int i = 0; i < npair; ++i) {
        const int ja = j0 + 2 * i;
        const int ph = i & 1;
        // stage 1 (R = 8, Ns = 1)
        if (t < 200) {
            float2 v[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                float ar = 0.f, ai = 0.f;
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const float2 xv = ring[rwrap_lo<RING>(rbase - p * M - 100 * r)];
                    ar = fmaf(hr[r][p], xv.x, ar);
                    ai = fmaf(hr[r][p], xv.y, ai);
                }
                v[r] = make_float2(ar, ai);
            }
            bdft8(v);
            float2 *fa = frb[bb][ph];
#pragma unroll
            for (int r = 0; r < 8; ++r) fa[an_pad(8 * tt + r)] = v[r];
        }
        rbase = rwrap<RING>(rbase + 2 * D);
        __syncthreads();
        // stage 2 (R = 4, Ns = 8): 2 x 200 butterflies on 320 threads, fa -> fb
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            const int g = t + A2_C * h2;
            if (g < 400) {
                const int b2 = g / 200, b = g - 200 * b2;
                const float2 *fa = frb[b2][ph];
                float2 *fb = frb[b2][ph ^ 1];
                float2 v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = fa[an_pad(b + 200 * r)];
                const int m = b & 7;
#pragma unroll
                for (int r = 1; r < 4; ++r) v[r] = c_mul(v[r], tw[AN_TW2 + (r - 1) * 8 + m]);
                bdft4(v[0], v[1], v[2], v[3]);
                const int base = (b >> 3) * 32 + m;
#pragma unroll
                for (int r = 0; r < 4; ++r) fb[an_pad(base + 8 * r)] = v[r];
            }
        }
        __syncthreads();
        // stage 3 (R = 5, Ns = 32): 2 x 160 butterflies, fb -> fa
        const int b3 = t / 160, u3 = t - 160 * b3;
        {
            const float2 *fb = frb[b3][ph ^ 1];
            float2 *fa = frb[b3][ph];
            float2 v[5];
#pragma unroll
            for (int r = 0; r < 5; ++r) v[r] = fb[an_pad(u3 + 160 * r)];
            const int m = u3 & 31;
#pragma unroll
            for (int r = 1; r < 5; ++r) v[r] = c_mul(v[r], tw[AN_TW3 + (r - 1) * 32 + m]);
            bdft5(v);
            const int base = (u3 >> 5) * 160 + m;
#pragma unroll
            for (int r = 0; r < 5; ++r) fa[an_pad(base + 32 * r)] = v[r];
        }
        __syncthreads();
        // stage 4 (R = 5, Ns = 160): outputs k = u3 + 160 r of block ja + b3, natural order, to HBM
        const int j = ja + b3;
        if (j < j1) {
            const float2 *fa = frb[b3][ph];
            float2 v[5];
#pragma unroll
            for (int r = 0; r < 5; ++r) v[r] = fa[an_pad(u3 + 160 * r)];
#pragma unroll
            for (int r = 1; r < 5; ++r) v[r] = c_mul(v[r], tw[AN_TW4 + (r - 1) * 160 + u3]);
            bdft5(v);
            const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(Y + (size_t)j * M, 0, 8 * M, 0x00020000);
            // the mixer term: v_k[j] = e^{-2 pi i k j D / M} Y_j[k] = (-i)^{(k j DM) mod 4} Y_j[k]
            const int jq = (j * DM) & 3;
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                const int k = u3 + 160 * r, q = (k * jq) & 3;
                const float a = (q & 1) ? v[r].y : v[r].x, b4 = (q & 1) ? -v[r].x : v[r].y;
                typedef unsigned u2v __attribute__((ext_vector_type(2)));
                const float2 o = (q & 2) ? make_float2(-a, -b4) : make_float2(a, b4);
                __builtin_amdgcn_raw_buffer_store_b64(u2v{__float_as_uint(o.x), __float_as_uint(o.y)}, yr, 8 * k, 0,
                                                      2 /* nt */);
            }
        }
        // the next pair's stage 1 writes frames [.][ph ^ 1]; its stage 2 (after the next barrier) is
        // the first to touch frames [.][ph] again
    }
}

// One block per iteration at any D (k_pfb_analysis's structure -- waves 0-2 fold + transform +
// store, wave 3 loads -- with analysis2's ring indexing and buffer-resource loader): the D = M / 2
// filter bank's default analysis.  LDS: the 4608-sample ring (L + D = 4400 at P = 5), two frames
// and stages 2-3's twiddles, 52.5 KB (TREG: stage 4's 640 twiddles are four registers per thread, and
// the VGPRs are held to 168): three workgroups per CU at P <= 5.  !TREG: all twiddles in LDS, 57.6 KB,
// two workgroups per CU (TETRA_WB_ANALYSIS=3, same-box A/B).
// PROBE (timing-only builds, wrong results: TETRA_WB_ANALYSIS_PROBE): 1 the loader issues no global
// loads (it writes whatever its registers hold), 2 no Y stores -- what each costs of the kernel's time.
// F3: the fold on all three compute waves (thread t < 192 folds u[t + 192 m], m < 5, into frame X;
// a barrier; the radix-8 stage reads X) instead of inside the radix-8 butterflies of waves 0-1: stage 1
// was two thirds of a block's issue time on two of the four SIMDs (profiles/r04_ab_analysis_probe.txt,
// DESIGN §5.7).  Four barriers per block, fixed frames (X: fold out, stage 2 out; Y: radix-8 out,
// stage 3 out).  The same fmas in the same order: the same Y.
template <int P, int DM, bool TREG = true, int PROBE = 0, bool F3 = false>
__global__ __launch_bounds__(AN_T, (TREG && P <= 5 ? 3 : 2)) void k_pfb_analysis1(const float4 *__restrict__ x2, int nblk, int JB,
                                                           const float *__restrict__ h,
                                                           const float2 *__restrict__ twg, float2 *__restrict__ Y) {
    using Cf = A2Cfg<P, DM>;
    constexpr int M = Cf::M, D = Cf::D, L = Cf::L, RING = Cf::RING;
    static_assert((P - 1) * M + 768 < RING, "a fold read is at most one ring length behind rbase (rwrap_lo)");
    constexpr int NLD1 = (D / 2 + 63) / 64;   // loader float4 loads per lane per block
    constexpr int AF1 = 4;                    // blocks ahead
    __shared__ float4 ring4[RING / 2];
    __shared__ float2 frb[2][AN_FR];
    __shared__ float2 tw[TREG ? AN_TW4 : AN_TWN];   // TREG: stages 2-3; stage 4's sit in registers (tw4)
    const float2 *ring = reinterpret_cast<const float2 *>(ring4);
    const int t = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const int j0 = blockIdx.x * JB, j1 = min(nblk, j0 + JB);
    const int nb = j1 - j0;
    for (int i = t; i < (TREG ? AN_TW4 : AN_TWN); i += AN_T) tw[i] = twg[i];
    float2 tw4[4];
#pragma unroll
    for (int r = 1; r < 5; ++r)
        tw4[r - 1] = TREG && t < 160 ? twg[AN_TW4 + (r - 1) * 160 + t] : make_float2(0.f, 0.f);
    const long npr = (long)(L + (long)(nblk - 1) * D) / 2;   // pairs of samples any block reads
    const long pr0 = (long)j0 * (D / 2);                      // ring pair 0 = x[j0 D]
    for (int q = t; q < L / 2; q += AN_T)                     // the first block's window
        if (pr0 + q < npr) ring4[q] = x2[pr0 + q];
    // stage 2's radix-4 butterfly b on the fixed F3 frames (Y -> X); with F3 the loader wave's lanes
    // 0-7 take butterflies 192-199, so no compute wave runs two
    auto s2f3 = [&](int b) __attribute__((always_inline)) {
        const float2 *fa = frb[1];
        float2 *fb = frb[0];
        float2 v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fa[an_pad(b + 200 * r)];
        const int m = b & 7;
#pragma unroll
        for (int r = 1; r < 4; ++r) v[r] = c_mul(v[r], tw[AN_TW2 + (r - 1) * 8 + m]);
        bdft4(v[0], v[1], v[2], v[3]);
        const int base = (b >> 3) * 32 + m;
#pragma unroll
        for (int r = 0; r < 4; ++r) fb[an_pad(base + 8 * r)] = v[r];
    };
    if (wv == 3) {
        // block jj (>= 1) adds x[L + (j0 + jj - 1) D, + D): D / 2 pairs from relative pair
        // (L + (jj - 1) D) / 2; written during block jj - 1's stage 1 (disjoint from its window)
        const int l = t - 192;
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(x2), 0, (int)(16 * npr),
                                                                            0x00020000);
        const int vo = 16 * (int)(pr0 + (L - D) / 2 + l);     // block jj's pairs at soffset 8 D jj
        int rpos = rwrap<RING / 2>(L / 2 + l);                 // ring pair position for block 1
        float4 sl[AF1][NLD1];
        auto fetch = [&](float4 (&v)[NLD1], int jj) __attribute__((always_inline)) {
            if constexpr (PROBE == 1) return;
#pragma unroll
            for (int m = 0; m < NLD1; ++m) {
                const nt_f4 w = __builtin_amdgcn_raw_buffer_load_b128(xr, vo + 1024 * m, 8 * D * jj, 0);
                v[m] = make_float4(w.x, w.y, w.z, w.w);
            }
        };
        auto step = [&](float4 (&v)[NLD1], int jj) __attribute__((always_inline)) {
            if (jj + 1 < nb) {
#pragma unroll
                for (int m = 0; m < NLD1; ++m)
                    if (l + 64 * m < D / 2) ring4[rwrap<RING / 2>(rpos + 64 * m)] = v[m];
            }
            rpos = rwrap<RING / 2>(rpos + D / 2);
            fetch(v, jj + 1 + AF1);
            if constexpr (F3) __syncthreads();   // after the fold
            __syncthreads();   // after stage 1
            if constexpr (F3) {
                if (l < 8) s2f3(192 + l);
            }
            __syncthreads();   // after stage 2
            __syncthreads();   // after stage 3
        };
        static_assert(AF1 == 4, "loader unroll");
        if constexpr (PROBE == 1) {
#pragma unroll
            for (int a = 0; a < AF1; ++a)
#pragma unroll
                for (int m = 0; m < NLD1; ++m) sl[a][m] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        fetch(sl[0], 1);
        fetch(sl[1], 2);
        fetch(sl[2], 3);
        fetch(sl[3], 4);
        __syncthreads();
        int jj = 0;
        for (; jj + 4 <= nb; jj += 4) {
            step(sl[0], jj);
            step(sl[1], jj + 1);
            step(sl[2], jj + 2);
            step(sl[3], jj + 3);
        }
        if (jj < nb) step(sl[0], jj);
        if (jj + 1 < nb) step(sl[1], jj + 1);
        if (jj + 2 < nb) step(sl[2], jj + 2);
        return;
    }
    constexpr int NF = F3 ? 5 : 8;   // fold outputs per thread
    constexpr int TF = F3 ? 192 : 100, SF = F3 ? 192 : 100;   // folding threads, their output stride
    float hr[NF][P];
    if (t < TF) {
#pragma unroll
        for (int r = 0; r < NF; ++r)
#pragma unroll
            for (int p = 0; p < P; ++p) hr[r][p] = t + SF * r < M ? h[p * M + t + SF * r] : 0.f;
    }
    __syncthreads();
    int rbase = rwrap<RING>(L - 1 - (t < TF ? t : 0));   // ring sample of n_j - t, block jj = 0
    for (int j = j0; j < j1; ++j) {
        float2 *fa = F3 ? frb[1] : frb[(j - j0) & 1], *fb = F3 ? frb[0] : frb[((j - j0) & 1) ^ 1];
        if constexpr (F3) {
            // the fold: u[i], i = t + 192 r, into fb (X)
            if (t < 192) {
#pragma unroll
                for (int r = 0; r < NF; ++r) {
                    const int i = t + 192 * r;
                    if (i < M) {
                        float ar = 0.f, ai = 0.f;
                        // e - p M wraps (+ RING) exactly when it is negative: pick the base, then
                        // subtract (one compare, one select, one subtract per tap)
                        const int e = rbase - 192 * r;                       // in (-768, RING)
                        const float2 *ba = ring + e, *bb = ring + e + RING;
#pragma unroll
                        for (int p = 0; p < P; ++p) {
                            const float2 xv = (e >= p * M ? ba : bb)[-p * M];
                            ar = fmaf(hr[r][p], xv.x, ar);
                            ai = fmaf(hr[r][p], xv.y, ai);
                        }
                        fb[an_pad(i)] = make_float2(ar, ai);
                    }
                }
            }
            rbase = rwrap<RING>(rbase + D);
            __syncthreads();
            // stage 1 (R = 8, Ns = 1): butterfly t < 100 on u[t + 100 r] from X, into fa (Y)
            if (t < 100) {
                float2 v[8];
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = fb[an_pad(t + 100 * r)];
                bdft8(v);
#pragma unroll
                for (int r = 0; r < 8; ++r) fa[an_pad(8 * t + r)] = v[r];
            }
        } else if (t < 100) {
            // stage 1 (R = 8, Ns = 1): butterfly t < 100 on u[t + 100 r], folded from the ring
            float2 v[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                float ar = 0.f, ai = 0.f;
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const float2 xv = ring[rwrap_lo<RING>(rbase - p * M - 100 * r)];
                    ar = fmaf(hr[r][p], xv.x, ar);
                    ai = fmaf(hr[r][p], xv.y, ai);
                }
                v[r] = make_float2(ar, ai);
            }
            bdft8(v);
#pragma unroll
            for (int r = 0; r < 8; ++r) fa[an_pad(8 * t + r)] = v[r];
        }
        if constexpr (!F3) rbase = rwrap<RING>(rbase + D);
        __syncthreads();
        // stage 2 (R = 4, Ns = 8): 200 butterflies on 192 threads, fa -> fb (F3: 192 here, 8 on the loader)
        if constexpr (F3) {
            if (t < 192) s2f3(t);
        } else
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
            const int b = t + 192 * h2;
            if (b < 200) {
                float2 v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = fa[an_pad(b + 200 * r)];
                const int m = b & 7;
#pragma unroll
                for (int r = 1; r < 4; ++r) v[r] = c_mul(v[r], tw[AN_TW2 + (r - 1) * 8 + m]);
                bdft4(v[0], v[1], v[2], v[3]);
                const int base = (b >> 3) * 32 + m;
#pragma unroll
                for (int r = 0; r < 4; ++r) fb[an_pad(base + 8 * r)] = v[r];
            }
        }
        __syncthreads();
        // stage 3 (R = 5, Ns = 32): 160 butterflies, fb -> fa
        if (t < 160) {
            float2 v[5];
#pragma unroll
            for (int r = 0; r < 5; ++r) v[r] = fb[an_pad(t + 160 * r)];
            const int m = t & 31;
#pragma unroll
            for (int r = 1; r < 5; ++r) v[r] = c_mul(v[r], tw[AN_TW3 + (r - 1) * 32 + m]);
            bdft5(v);
            const int base = (t >> 5) * 160 + m;
#pragma unroll
            for (int r = 0; r < 5; ++r) fa[an_pad(base + 32 * r)] = v[r];
        }
        __syncthreads();
        // stage 4 (R = 5, Ns = 160): outputs k = t + 160 r, natural order, mixer rotation, to HBM
        if (t < 160) {
            float2 v[5];
#pragma unroll
            for (int r = 0; r < 5; ++r) v[r] = fa[an_pad(t + 160 * r)];
#pragma unroll
            for (int r = 1; r < 5; ++r) v[r] = c_mul(v[r], TREG ? tw4[r - 1] : tw[AN_TW4 + (r - 1) * 160 + t]);
            bdft5(v);
            const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(Y + (size_t)j * M, 0, 8 * M, 0x00020000);
            const int jq = (j * DM) & 3;
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                const int k = t + 160 * r, q = (k * jq) & 3;
                const float a = (q & 1) ? v[r].y : v[r].x, b4 = (q & 1) ? -v[r].x : v[r].y;
                typedef unsigned u2v __attribute__((ext_vector_type(2)));
                const float2 o = (q & 2) ? make_float2(-a, -b4) : make_float2(a, b4);
                if constexpr (PROBE == 2)
                    asm volatile("" ::"v"(o.x), "v"(o.y));
                else
                    __builtin_amdgcn_raw_buffer_store_b64(u2v{__float_as_uint(o.x), __float_as_uint(o.y)}, yr, 8 * k, 0,
                                                          2 /* nt */);
            }
        }
    }
}

// y[k][n] for 64 channels x RS_T outputs: v rows staged (rotated) in LDS, one lane per channel,
// so an output's taps are wave-uniform: the phase-major table gT[rho][q] comes in by scalar loads
// and the Q-tap loop is unrolled; the tile is transposed through LDS for row-contiguous stores.
template <int Q, bool ROT>
__global__ __launch_bounds__(256) void k_pfb_resamp(const float2 *__restrict__ Y, int M, int nblk, int up, int down,
                                                    const float *__restrict__ gT, float2 *__restrict__ y,
                                                    int n_keep) {
    extern __shared__ float2 vt[];   // [rows][RS_C]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int k0 = blockIdx.x * RS_C, n0 = blockIdx.y * RS_T;
    const int n1 = min(n_keep, n0 + RS_T);
    const int ilo = (int)(((long)down * n0) / up);                       // oldest input row needed
    const int ihi = (int)(((long)down * (n1 - 1)) / up) + Q - 1;         // newest
    const int rows = ihi - ilo + 1;
    // staging: each thread owns column c = lane and rows wv, wv + 4, ...; loads issued 8 ahead
    {
        const int k = k0 + lane;
        const bool kin = k < M;
        for (int r0 = wv; r0 < rows; r0 += 4 * 8) {
            float2 z[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const int i = ilo + r0 + 4 * b;
                z[b] = kin && r0 + 4 * b < rows && i < nblk ? Y[(size_t)i * M + k] : make_float2(0.f, 0.f);
            }
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const int rr = r0 + 4 * b;
                if (rr < rows) {
                    // z * (-i)^q, q = k i mod 4, branch-free: odd q swaps (re, im) -> (im, -re)
                    const int q = ROT ? (int)(((long)k * (ilo + rr)) & 3) : 0;   // !ROT: rotated upstream
                    const float a = (q & 1) ? z[b].y : z[b].x, bb = (q & 1) ? -z[b].x : z[b].y;
                    vt[rr * RS_C + lane] = (q & 2) ? make_float2(-a, -bb) : make_float2(a, bb);
                }
            }
        }
    }
    __syncthreads();
    float2 res[RS_T / 4];
#pragma unroll
    for (int o = 0; o < RS_T / 4; ++o) {
        const int n = n0 + wv * (RS_T / 4) + o;   // wave-uniform
        float ar = 0.f, ai = 0.f;
        if (n < n1) {
            const long dn = (long)down * n;
            const int rho = (int)(dn % up), top = (int)(dn / up) + Q - 1 - ilo;
            const float *gt = gT + rho * RS_QP;
            const float2 *vp = vt + top * RS_C + lane;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const float w = gt[q];
                const float2 v = vp[-q * RS_C];
                ar = fmaf(w, v.x, ar);
                ai = fmaf(w, v.y, ai);
            }
        }
        res[o] = make_float2(ar, ai);
    }
    __syncthreads();
    // transpose: out tile [c][RS_T] over the staged rows
#pragma unroll
    for (int o = 0; o < RS_T / 4; ++o) vt[lane * (RS_T + 1) + wv * (RS_T / 4) + o] = res[o];
    __syncthreads();
    for (int e = tid; e < RS_C * RS_T; e += 256) {
        const int c = e / RS_T, o = e - c * RS_T, k = k0 + c, n = n0 + o;
        if (k < M && n < n1) y[(size_t)k * n_keep + n] = vt[c * (RS_T + 1) + o];
    }
}

// The same resampler with the rate pair fixed at compile time (UP / DOWN = 72 kHz / carrier rate):
// output n = UP m + o uses rows DOWN m + lo(o) .. + Q - 1 with lo(o) = floor(DOWN o / UP) and taps
// g[rho(o) + UP q], rho(o) = DOWN o mod UP -- all compile-time for o < UP.  A lane owns one carrier
// and one group of UP outputs: it streams the group's DOWN (UP-1)/UP + Q rows once (row loads are
// 64 consecutive carriers = 512 contiguous bytes per wave), and every row feeds the outputs whose
// window holds it, with the tap a wave-uniform scalar operand.  Each tap of g is used exactly once
// per group, so a group is Lg FMAs per component with no LDS on the input side; LDS only transposes
// the [carrier][output] tile for row-contiguous stores.
// Position of tap (row i, output o) in the use-ordered tap table gU (rows ascending, outputs
// ascending within a row): the n-th FMA of a group reads tap n.  The table sits in LDS (810
// floats): as scalar loads the compiler hoisted hundreds of taps and spilled SGPRs to VGPR lanes.
// Measured and removed in round 4: per-wave transposing tiles (4 waves per SIMD instead
// of 2: no faster), nt / sc1 stores of y (slower), rows in two batches instead of three (noise).
// Storing straight from registers makes hipcc hoist every tap read of the group and spill.
template <int UP, int DOWN, int Q>
struct ResampUse {
    static constexpr int ROWS = (DOWN * (UP - 1)) / UP + Q;
    int idx[ROWS][UP];
    int n = 0;
    constexpr ResampUse() : idx{} {
        for (int i = 0; i < ROWS; ++i)
            for (int o = 0; o < UP; ++o) {
                const int lo = (DOWN * o) / UP;
                idx[i][o] = (i >= lo && i <= lo + Q - 1) ? n++ : -1;
            }
    }
};

// PRB (timing-only build, TETRA_WB_RESAMP_PROBE=1): no y stores -- what the write-out costs.
// OM (tetra_channelize_om; UP a multiple of 4): each lane also leaves its group's Oerder-Meyr class
// partials om[k][m] = (P0, P1, P2, P3), P_c = sum over o = c mod 4, ascending, of |y[UP m + o]|^2 --
// from the registers the group's outputs are stored from, so k_timing's OMG form needs no pass over y
// before its Gardner loop (oracle/etsi_oracle.c eo_om_group_partials).
template <int UP, int DOWN, int Q, bool ROT, int PRB = 0, bool OM = false>
__global__ __launch_bounds__(256) void k_pfb_resamp_fix(const float2 *__restrict__ Y, int M, int nblk,
                                                        const float *__restrict__ gU, float2 *__restrict__ y,
                                                        int n_keep, float4 *__restrict__ om = nullptr,
                                                        int ngrp = 0) {
    using U = ResampUse<UP, DOWN, Q>;
    constexpr U use{};
    constexpr int ROWS = U::ROWS;                       // rows of one output group
    constexpr int OT = 4 * UP;                          // outputs per workgroup (4 waves x one group)
    constexpr int RB = 17;                              // rows in flight per batch
    typedef float pf2 __attribute__((ext_vector_type(2)));   // (re, im): one v_pk_fma_f32 per tap
    // One LDS block, taps first (in use order; each read a same-address broadcast), then the transpose
    // tile.  With the taps at the bottom every tap read is one base register + a constant offset;
    // behind the 74 KB tile the offsets overflowed ds_read's 16-bit immediate and every read cost a
    // v_mov of its address (471 of ~2200 instructions per wave and group; round 5: 2207 -> 2016
    // instructions, serial resampler 0.111 -> 0.109 ms, profiles/r05_ab_resamp_*.txt).  Taps stored
    // pre-paired (w, w) for the packed FMA cut the pairing moves too but doubled the LDS reads: 0.116.
    constexpr int TAPB = ((use.n * 4 + 15) / 16) * 16;
    __shared__ __attribute__((aligned(16))) unsigned char lds_raw[TAPB + RS_C * (OT + 1) * 8];
    float *tapP = reinterpret_cast<float *>(lds_raw);
    float2 *tile = reinterpret_cast<float2 *>(lds_raw + TAPB);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int e = tid; e < use.n; e += 256) tapP[e] = gU[e];
    const int k = min(blockIdx.x * RS_C + lane, M - 1);
    const int m = blockIdx.y * 4 + wv;                  // output group: outputs UP m .. UP m + UP - 1
    const int r0 = DOWN * m;                            // wave-uniform: row offsets are scalar
    // rows r0 .. r0 + ROWS - 1; a group reaching past nblk (the last ones) clamps its row index --
    // clamped rows only feed outputs n >= n_keep, which are not stored
    const float2 *base = Y + k;
    __syncthreads();
    pf2 acc[UP];
#pragma unroll
    for (int o = 0; o < UP; ++o) acc[o] = pf2{0.f, 0.f};
#pragma unroll
    for (int i0 = 0; i0 < ROWS; i0 += RB) {
        float2 v[RB];
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            if (i0 + b < ROWS) {
                const int row = min(r0 + i0 + b, nblk - 1);
                v[b] = base[(size_t)row * M];
            }
        }
#pragma unroll
        for (int b = 0; b < RB; ++b) {
            const int i = i0 + b;
            if (i < ROWS) {
                // v_k[row] = (-i)^{(k row) mod 4} Y_row[k] (ROT: here; else k_pfb_analysis applied it)
                pf2 vv = pf2{v[b].x, v[b].y};
                if constexpr (ROT) {
                    const int q = (k * ((r0 + i) & 3)) & 3;
                    const float a = (q & 1) ? v[b].y : v[b].x, bb = (q & 1) ? -v[b].x : v[b].y;
                    vv = (q & 2) ? pf2{-a, -bb} : pf2{a, bb};
                }
#pragma unroll
                for (int o = 0; o < UP; ++o) {
                    if (use.idx[i][o] >= 0)
                        acc[o] = __builtin_elementwise_fma(pf2{tapP[use.idx[i][o]], tapP[use.idx[i][o]]}, vv, acc[o]);   // = fmaf per component
                }
            }
        }
    }
#pragma unroll
    for (int o = 0; o < UP; ++o) tile[lane * (OT + 1) + wv * UP + o] = make_float2(acc[o].x, acc[o].y);
    if constexpr (OM) {
        static_assert(UP % 4 == 0, "class partials need whole classes per group");
        if (blockIdx.x * RS_C + lane < M && m * UP < n_keep) {
            float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int o = 0; o < UP; ++o) p[o & 3] = p[o & 3] + fmaf(acc[o].x, acc[o].x, acc[o].y * acc[o].y);
            om[(size_t)k * ngrp + m] = make_float4(p[0], p[1], p[2], p[3]);
        }
    }
    __syncthreads();
    const int k0 = blockIdx.x * RS_C, n0 = blockIdx.y * OT;
    for (int e = tid; e < RS_C * OT; e += 256) {
        const int c = e / OT, o = e - c * OT, kk = k0 + c, n = n0 + o;
        if constexpr (PRB == 1) {
            const float2 v = tile[c * (OT + 1) + o];
            asm volatile("" ::"v"(v.x), "v"(v.y));
        } else if (kk < M && n < n_keep) {
            y[(size_t)kk * n_keep + n] = tile[c * (OT + 1) + o];
        }
    }
}

__device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// x[n] = sum_j D h[n - jD] W[j][n mod M] (+ AWGN): one thread per output sample.
__global__ __launch_bounds__(256) void k_pfb_synth(const float2 *__restrict__ W, int M, int D, int P, int nbb,
                                                   const float *__restrict__ h, long Nw, float sigma, uint64_t seed,
                                                   float2 *__restrict__ x) {
    const long n = (long)blockIdx.x * 256 + threadIdx.x;
    if (n >= Nw) return;
    const long L = (long)P * M;
    const int r = (int)(n % M);
    long jhi = n / D;
    if (jhi > nbb - 1) jhi = nbb - 1;
    long jlo = n - L + 1 <= 0 ? 0 : (n - L + 1 + D - 1) / D;
    const float gain = (float)D;
    float ar = 0.f, ai = 0.f;
    for (long j = jlo; j <= jhi; ++j) {
        const float w = gain * h[n - j * D];
        const float2 v = W[(size_t)j * M + r];
        ar = fmaf(w, v.x, ar);
        ai = fmaf(w, v.y, ai);
    }
    if (sigma > 0.f) {
        const uint64_t hh = mix64(seed ^ mix64((uint64_t)n * 0x9E3779B97F4A7C15ull ^ 0x5EEDull));
        const float u1 = (float)((hh >> 40) + 0.5) * (1.0f / 16777216.0f);
        const float u2 = (float)(((hh >> 16) & 0xFFFFFF) + 0.5) * (1.0f / 16777216.0f);
        const float rr = sqrtf(-2.0f * logf(u1));
        ar += sigma * rr * cosf(6.2831853f * u2);
        ai += sigma * rr * sinf(6.2831853f * u2);
    }
    x[n] = make_float2(ar, ai);
}

int wb_check(tetra_ctx *ctx, const tetra_wb_plan *P) {
    if (!P || !P->h || !P->g) return tetra_fail(ctx, TETRA_E_INVALID, "null wideband plan");
    if (P->M <= 0 || P->D <= 0 || (P->M != 4 * P->D && P->M != 2 * P->D) || P->P < 1 || P->P > 8)
        return tetra_fail(ctx, TETRA_E_INVALID, "wideband plan needs M = 4 D or M = 2 D, and 1 <= P <= 8");
    if (P->up <= 0 || P->down <= 0 || P->Lg <= 0 || P->Lg % P->up)
        return tetra_fail(ctx, TETRA_E_INVALID, "resampler taps Lg must be a multiple of up");
    return TETRA_OK;
}

}  // namespace

extern "C" {

int tetra_wb_lengths(const tetra_wb_plan *P, size_t Nw, int64_t *nblk, int64_t *n72) {
    if (!P || !nblk || !n72 || P->M <= 0 || P->D <= 0 || P->up <= 0 || P->Lg <= 0) return TETRA_E_INVALID;
    const long L = (long)P->M * P->P, Q = P->Lg / P->up;
    const long nb = (long)Nw >= L ? ((long)Nw - L) / P->D + 1 : 0;
    *nblk = nb;
    *n72 = nb >= Q ? ((long)P->up * (nb - Q) + P->up - 1) / P->down + 1 : 0;
    return TETRA_OK;
}

namespace {
int channelize(tetra_ctx *ctx, const tetra_wb_plan *P, const void *x, size_t Nw, void *y, size_t n_keep, void *om) {
    if (!ctx) return TETRA_E_INVALID;
    int rc = wb_check(ctx, P);
    if (rc) return rc;
    int64_t nblk, n72;
    tetra_wb_lengths(P, Nw, &nblk, &n72);
    if (n72 <= 0 || n_keep == 0 || (int64_t)n_keep > n72)
        return tetra_fail(ctx, TETRA_E_INVALID, "n_keep must be in [1, %ld] for %zu samples", (long)n72, Nw);
    const int M = P->M, L = M * P->P, Q = P->Lg / P->up;
    const int DM = 4 * P->D / M;   // 1: carriers at 4x, 2: at 2x the carrier spacing
    if (Q != 45 && Q != 23) return tetra_fail(ctx, TETRA_E_INVALID, "resampler built for Lg / up = 45 or 23 taps");
    if (P->up > RS_QP) return tetra_fail(ctx, TETRA_E_INVALID, "resampler up %d > %d", P->up, RS_QP);
    // the compiled-in rate pairs: 100 kHz -> 72 kHz (D = M / 4) and 50 kHz -> 72 kHz (D = M / 2)
    const bool fix18 = P->up == 18 && P->down == 25 && Q == 45, fix36 = P->up == 36 && P->down == 25 && Q == 23;
    const bool fixed = fix18 || fix36;
    if (om && !fix36)
        return tetra_fail(ctx, TETRA_E_INVALID, "Oerder-Meyr group partials need the D = M / 2 resampler (36 / 25)");
    const int ngrp = (int)((n_keep + P->up - 1) / P->up);
    Staging st(ctx);
    const float2 *xd = (const float2 *)st.in(x, Nw * 8);
    float2 *yd = (float2 *)st.out(y, (size_t)M * n_keep * 8);
    float4 *omd = om ? (float4 *)st.out(om, (size_t)M * ngrp * 16) : nullptr;
    float2 *u = (float2 *)ws(ctx, S_W8, (size_t)nblk * M * 8);
    float *taps = (float *)ws(ctx, S_W9, (size_t)(L + P->up * RS_QP + P->Lg + 2 + 2 * AN_TWN) * 4);
    if (!xd || !yd || !u || !taps || (om && !omd)) return st.finish();
    // h, then g phase-major: gT[rho][q] = g[rho + up q] (zero-padded to RS_QP), then g as given
    ctx->taps_wb.assign(P->h, P->h + L);
    ctx->taps_wb.resize((size_t)L + P->up * RS_QP, 0.f);
    for (int rho = 0; rho < P->up; ++rho)
        for (int q = 0; q < Q; ++q) ctx->taps_wb[L + rho * RS_QP + q] = P->g[rho + P->up * q];
    // k_pfb_resamp_fix's use-ordered table gU (see ResampUse)
    auto use_table = [&](const auto &use, int UPc, int DOWNc, int Qc, int ROWSc) {
        std::vector<float> gU((size_t)use.n);
        for (int i = 0; i < ROWSc; ++i)
            for (int o = 0; o < UPc; ++o)
                if (use.idx[i][o] >= 0) {
                    const int lo = (DOWNc * o) / UPc, rho = (DOWNc * o) % UPc;
                    gU[use.idx[i][o]] = P->g[rho + UPc * (lo + Qc - 1 - i)];
                }
        ctx->taps_wb.insert(ctx->taps_wb.end(), gU.begin(), gU.end());
    };
    if (fix18) {
        constexpr ResampUse<18, 25, 45> use{};
        use_table(use, 18, 25, 45, ResampUse<18, 25, 45>::ROWS);
    } else if (fix36) {
        constexpr ResampUse<36, 25, 23> use{};
        use_table(use, 36, 25, 23, ResampUse<36, 25, 23>::ROWS);
    } else {
        ctx->taps_wb.insert(ctx->taps_wb.end(), P->g, P->g + P->Lg);
    }
    // fold + FFT in one pass (k_pfb_analysis / k_pfb_analysis2); D = M / 2 only so
    const bool fused = M == AN_M && ((DM == 1 && P->P <= 4) || (DM == 2 && P->P >= 4 && P->P <= 6));
    if (!fused && DM != 1) return tetra_fail(ctx, TETRA_E_INVALID, "D = M / 2 needs M = 800 and 4 <= P <= 6");
    const size_t tw_off = ctx->taps_wb.size() + (ctx->taps_wb.size() & 1);   // float2-aligned
    if (fused) {   // backward twiddles e^{+2 pi i m r / (Ns R)}, r-major per stage
        ctx->taps_wb.resize(tw_off + 2 * AN_TWN, 0.f);
        auto put = [&](int off, int ns, int R) {
            for (int r = 1; r < R; ++r)
                for (int m = 0; m < ns; ++m) {
                    const double a = 2.0 * 3.14159265358979323846 * m * r / (ns * R);
                    ctx->taps_wb[tw_off + 2 * (off + (r - 1) * ns + m)] = (float)cos(a);
                    ctx->taps_wb[tw_off + 2 * (off + (r - 1) * ns + m) + 1] = (float)sin(a);
                }
        };
        put(AN_TW2, 8, 4);
        put(AN_TW3, 32, 5);
        put(AN_TW4, 160, 5);
    }
    if (ctx->taps_wb_dev != taps || ctx->taps_wb_up != ctx->taps_wb) {   // upload only on change
        ctx->taps_wb_up = ctx->taps_wb;
        HIP_TRY(ctx, hipMemcpyAsync(taps, ctx->taps_wb_up.data(), ctx->taps_wb_up.size() * 4, hipMemcpyHostToDevice,
                                    ctx->stream));
        ctx->taps_wb_dev = taps;
    }
    if (fused) {
        PROF(ctx, "wb_analysis");
        // About one round of workgroups when the capture allows, >= 16 blocks each (the L-sample
        // window each workgroup loads first is its overhead).  TETRA_WB_ANALYSIS: 1 one block per
        // iteration (default), 2 two blocks per iteration (k_pfb_analysis2), 3 / 4 (D = M / 2) one
        // block with every twiddle in LDS / with the fold inside the radix-8 butterflies -- same-box
        // A/B and the parity tests, which switch it between calls.  The D = M / 2 kernels address the capture
        // with 32-bit byte offsets.
        const char *fe = getenv("TETRA_WB_ANALYSIS");
        const int form = fe ? atoi(fe) : 1;
        if (DM == 2 && Nw * 8 >= (size_t)1 << 31)
            return tetra_fail(ctx, TETRA_E_INVALID, "D = M / 2 capture over 2 GiB: split it");
        if (DM == 2 && form != 2) {
            // three (P <= 5, twiddles in registers) or two 256-thread workgroups per CU, >= 16 blocks
            // each, about one round
            const bool treg = form != 3;
            const int per_cu = treg && P->P <= 5 ? 3 : 2;
            const int jb = std::max<int>(16, (int)((nblk + per_cu * 256 - 1) / (per_cu * 256)));
            const unsigned grid = (unsigned)((nblk + jb - 1) / jb);
            const char *pe = getenv("TETRA_WB_ANALYSIS_PROBE");
            const int probe = pe ? atoi(pe) : 0;
            // the default: twiddles in registers and the fold on three waves (F3); 4: without F3, 3:
            // without either (same-box A/B, profiles/r04_ab_analysis_f3_*.txt)
            const bool f3 = form != 3 && form != 4;
            if (f3 && probe == 0) {
                switch (P->P) {
#define AN(PP) case PP: hipLaunchKernelGGL((k_pfb_analysis1<PP, 2, true, 0, true>), dim3(grid), dim3(AN_T), 0, ctx->stream, (const float4 *)xd, (int)nblk, jb, taps, (const float2 *)(taps + tw_off), u); break;
                    AN(4) AN(5) AN(6)
#undef AN
                }
            } else if (probe == 1 && P->P == 5 && treg)
                hipLaunchKernelGGL((k_pfb_analysis1<5, 2, true, 1>), dim3(grid), dim3(AN_T), 0, ctx->stream,
                                   (const float4 *)xd, (int)nblk, jb, taps, (const float2 *)(taps + tw_off), u);
            else if (probe == 2 && P->P == 5 && treg)
                hipLaunchKernelGGL((k_pfb_analysis1<5, 2, true, 2>), dim3(grid), dim3(AN_T), 0, ctx->stream,
                                   (const float4 *)xd, (int)nblk, jb, taps, (const float2 *)(taps + tw_off), u);
            else
            switch (P->P * 2 + (treg ? 1 : 0)) {
#define AN(PP, TR) case PP * 2 + TR: hipLaunchKernelGGL((k_pfb_analysis1<PP, 2, TR>), dim3(grid), dim3(AN_T), 0, ctx->stream, (const float4 *)xd, (int)nblk, jb, taps, (const float2 *)(taps + tw_off), u); break;
                AN(4, 0) AN(5, 0) AN(6, 0) AN(4, 1) AN(5, 1) AN(6, 1)
#undef AN
            }
        } else if (DM == 1 && (form != 2 || Nw * 8 >= (size_t)1 << 31)) {
            const int jb = std::max<int>(16, (int)((nblk + 4 * 256 - 1) / (4 * 256)));
            const unsigned grid = (unsigned)((nblk + jb - 1) / jb);
            switch (P->P) {
#define AN(PP) case PP: hipLaunchKernelGGL(k_pfb_analysis<PP>, dim3(grid), dim3(AN_T), 0, ctx->stream, (const float4 *)xd, (int)nblk, jb, taps, (const float2 *)(taps + tw_off), u); break;
                AN(1) AN(2) AN(3) AN(4)
#undef AN
            }
        } else {
            // 384-thread workgroups: three per CU at D = M / 4 (51 KB of LDS), two at D = M / 2 (72 KB);
            // an even number of >= 16 blocks each, about one round of workgroups
            const int wpc = DM == 1 ? 3 : 2;
            int jb = std::max<int>(16, (int)((nblk + wpc * 256 - 1) / (wpc * 256)));
            jb += jb & 1;
            const unsigned grid = (unsigned)((nblk + jb - 1) / jb);
            const int key = 10 * DM + P->P;
            switch (key) {
#define AN(PP, DD) case 10 * DD + PP: hipLaunchKernelGGL((k_pfb_analysis2<PP, DD>), dim3(grid), dim3(A2_T), 0, ctx->stream, (const float4 *)xd, (int)nblk, jb, taps, (const float2 *)(taps + tw_off), u); break;
                AN(1, 1) AN(2, 1) AN(3, 1) AN(4, 1) AN(4, 2) AN(5, 2) AN(6, 2)
#undef AN
            }
        }
        HIP_TRY(ctx, hipGetLastError());
    } else {
        PROF(ctx, "wb_fold");
        constexpr int JB = 16;
        const dim3 gr((unsigned)((M + 255) / 256), (unsigned)((nblk + JB - 1) / JB));
        switch (P->P) {
#define FOLD(PP) case PP: hipLaunchKernelGGL(k_pfb_fold<PP>, gr, dim3(256), 0, ctx->stream, xd, M, P->D, (int)nblk, taps, u, JB); break;
            FOLD(1) FOLD(2) FOLD(3) FOLD(4) FOLD(5) FOLD(6) FOLD(7) FOLD(8)
#undef FOLD
        }
        HIP_TRY(ctx, hipGetLastError());
    }
    if (!fused) {
        PROF(ctx, "wb_fft");
        rc = fft_c2c(ctx, true, false, M, nblk, 1, M, 1, M, u, u);
        if (rc) return rc;
    }
    if (fixed) {
        PROF(ctx, "wb_resamp");
        const dim3 gr((unsigned)((M + RS_C - 1) / RS_C), (unsigned)((n_keep + 4 * P->up - 1) / (4 * P->up)));
        const float *gu = taps + L + P->up * RS_QP;
        // TETRA_WB_RESAMP_PROBE=1 (timing-only, wrong y): the D = M / 2 resampler without its stores
        const char *pe = getenv("TETRA_WB_RESAMP_PROBE");
        if (fix36 && pe && atoi(pe) == 1)
            hipLaunchKernelGGL((k_pfb_resamp_fix<36, 25, 23, false, 1>), gr, dim3(256), 0, ctx->stream, u, M, (int)nblk,
                               gu, yd, (int)n_keep);
        else if (fix36 && omd)   // + the Oerder-Meyr group partials
            hipLaunchKernelGGL((k_pfb_resamp_fix<36, 25, 23, false, 0, true>), gr, dim3(256), 0, ctx->stream, u, M,
                               (int)nblk, gu, yd, (int)n_keep, omd, ngrp);
        else if (fix36)   // D = M / 2: always the fused analysis, Y rotated there
            hipLaunchKernelGGL((k_pfb_resamp_fix<36, 25, 23, false>), gr, dim3(256), 0, ctx->stream, u, M, (int)nblk, gu,
                               yd, (int)n_keep);
        else if (fused)   // Y already carries the mixer rotation
            hipLaunchKernelGGL((k_pfb_resamp_fix<18, 25, 45, false>), gr, dim3(256), 0, ctx->stream, u, M, (int)nblk, gu,
                               yd, (int)n_keep);
        else
            hipLaunchKernelGGL((k_pfb_resamp_fix<18, 25, 45, true>), gr, dim3(256), 0, ctx->stream, u, M, (int)nblk, gu,
                               yd, (int)n_keep);
        HIP_TRY(ctx, hipGetLastError());
    } else {
        PROF(ctx, "wb_resamp");
        const int rows = (int)(((long)P->down * (RS_T - 1)) / P->up) + Q + 1;
        const size_t lds = (size_t)std::max(rows * RS_C, RS_C * (RS_T + 1)) * 8;
        if (lds > 160 * 1024) return tetra_fail(ctx, TETRA_E_INVALID, "resampler tile does not fit LDS");
        const dim3 gr((unsigned)((M + RS_C - 1) / RS_C), (unsigned)((n_keep + RS_T - 1) / RS_T));
        if (Q == 23 && fused)   // D = M / 2 with the fused analysis: Y rotated there
            hipLaunchKernelGGL((k_pfb_resamp<23, false>), gr, dim3(256), lds, ctx->stream, u, M, (int)nblk, P->up, P->down,
                               taps + L, yd, (int)n_keep);
        else if (Q == 23)       // D = M / 2 plan on the unfused analysis: the resampler rotates
            hipLaunchKernelGGL((k_pfb_resamp<23, true>), gr, dim3(256), lds, ctx->stream, u, M, (int)nblk, P->up, P->down,
                               taps + L, yd, (int)n_keep);
        else if (fused)
            hipLaunchKernelGGL((k_pfb_resamp<45, false>), gr, dim3(256), lds, ctx->stream, u, M, (int)nblk, P->up, P->down,
                               taps + L, yd, (int)n_keep);
        else
            hipLaunchKernelGGL((k_pfb_resamp<45, true>), gr, dim3(256), lds, ctx->stream, u, M, (int)nblk, P->up, P->down,
                               taps + L, yd, (int)n_keep);
        HIP_TRY(ctx, hipGetLastError());
    }
    return st.finish();
}
}  // namespace

int tetra_channelize(tetra_ctx *ctx, const tetra_wb_plan *P, const void *x, size_t Nw, void *y, size_t n_keep) {
    return channelize(ctx, P, x, Nw, y, n_keep, nullptr);
}

int tetra_channelize_om(tetra_ctx *ctx, const tetra_wb_plan *P, const void *x, size_t Nw, void *y, size_t n_keep,
                        void *om) {
    if (!om) return tetra_fail(ctx, TETRA_E_INVALID, "null om");
    return channelize(ctx, P, x, Nw, y, n_keep, om);
}

int tetra_synth_wideband(tetra_ctx *ctx, const tetra_wb_plan *P, size_t Nw, uint64_t seed, float snr_db,
                         float cfo_max, void *x, uint32_t *cell_init, int32_t *kinds, uint8_t *payload, double *t0) {
    if (!ctx || !x || !cell_init) return TETRA_E_INVALID;
    int rc = wb_check(ctx, P);
    if (rc) return rc;
    const int M = P->M, L = M * P->P;
    const double fsc = P->fs / P->D;   // carrier baseband rate
    const size_t nbb = Nw / P->D + 1;
    // carriers at fsc, noiseless (the noise goes on the wideband sum below)
    float2 *s = (float2 *)ws(ctx, S_W10, (size_t)M * nbb * 8);
    if (!s) return TETRA_E_NOMEM;
    rc = tetra_synth_etsi(ctx, M, nbb, fsc, seed, 1000.f, cfo_max, s, cell_init, kinds, payload, t0);
    if (rc) return rc;
    Staging st(ctx);
    float2 *xd = (float2 *)st.out(x, Nw * 8);
    float2 *W = (float2 *)ws(ctx, S_W8, (size_t)M * nbb * 8);
    float *taps = (float *)ws(ctx, S_W9, (size_t)L * 4);
    if (!xd || !W || !taps) return st.finish();
    ctx->taps_wb.assign(P->h, P->h + L);
    HIP_TRY(ctx, hipMemcpyAsync(taps, ctx->taps_wb.data(), (size_t)L * 4, hipMemcpyHostToDevice, ctx->stream));
    ctx->taps_wb_dev = nullptr;   // slot S_W9 now holds only h
    // W[j][r] = sum_k s[k][j] e^{+i 2 pi k r / M}: input stride nbb between carriers, 1 between j
    rc = fft_c2c(ctx, true, false, M, nbb, nbb, 1, 1, M, s, W);
    if (rc) return rc;
    // per-carrier Es/N0 as tetra_synth_etsi defines it (amplitude 0.5, fs/18000 samples per symbol)
    const float amp = 0.5f;
    const float sigma = snr_db > -100.f && snr_db < 200.f
                            ? amp * sqrtf((float)(P->fs / 18000.0) / powf(10.f, snr_db / 10.f) / 2.f) : 0.f;
    hipLaunchKernelGGL(k_pfb_synth, dim3((unsigned)((Nw + 255) / 256)), dim3(256), 0, ctx->stream, W, M, P->D, P->P,
                       (int)nbb, taps, (long)Nw, sigma, seed, xd);
    HIP_TRY(ctx, hipGetLastError());
    return st.finish();
}

}  // extern "C"
