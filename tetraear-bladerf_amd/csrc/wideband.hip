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
#include "common.h"

#include <rocfft/rocfft.h>

#include <mutex>

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

// y[k][n] for 64 channels x RS_T outputs: v rows staged (rotated) in LDS, one lane per channel,
// so an output's taps are wave-uniform: the phase-major table gT[rho][q] comes in by scalar loads
// and the Q-tap loop is unrolled; the tile is transposed through LDS for row-contiguous stores.
template <int Q>
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
                    const int q = (int)(((long)k * (ilo + rr)) & 3);
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

// ------------------------------------------------------------------------------------ rocFFT
struct FftPlan {
    size_t M, batch, istride, idist, ostride, odist;
    bool inplace;
    rocfft_plan plan;
    rocfft_execution_info info;
    size_t work;
};
struct FftCache {
    std::vector<FftPlan> plans;
    DevBuf work;
};

void fft_free(void *p) {
    auto *c = static_cast<FftCache *>(p);
    for (auto &f : c->plans) {
        rocfft_execution_info_destroy(f.info);
        rocfft_plan_destroy(f.plan);
    }
    if (c->work.p) (void)hipFree(c->work.p);
    delete c;
}

std::once_flag g_fft_once;

// Batched length-M backward (e^{+i}) single-precision complex transform, unnormalised.
int fft_backward(tetra_ctx *ctx, size_t M, size_t batch, size_t istride, size_t idist, size_t ostride, size_t odist,
                 void *in, void *out) {
    std::call_once(g_fft_once, [] { rocfft_setup(); });
    if (!ctx->fft) {
        ctx->fft = new FftCache();
        ctx->fft_free = fft_free;
    }
    auto *cache = static_cast<FftCache *>(ctx->fft);
    const bool inplace = in == out;
    FftPlan *fp = nullptr;
    for (auto &f : cache->plans)
        if (f.M == M && f.batch == batch && f.istride == istride && f.idist == idist && f.ostride == ostride &&
            f.odist == odist && f.inplace == inplace)
            fp = &f;
    if (!fp) {
        FftPlan f{M, batch, istride, idist, ostride, odist, inplace, nullptr, nullptr, 0};
        rocfft_plan_description desc = nullptr;
        if (rocfft_plan_description_create(&desc) != rocfft_status_success)
            return tetra_fail(ctx, TETRA_E_HIP, "rocfft_plan_description_create failed");
        const size_t is[1] = {istride}, os[1] = {ostride};
        rocfft_status s = rocfft_plan_description_set_data_layout(
            desc, rocfft_array_type_complex_interleaved, rocfft_array_type_complex_interleaved, nullptr, nullptr, 1, is,
            idist, 1, os, odist);
        const size_t len[1] = {M};
        if (s == rocfft_status_success)
            s = rocfft_plan_create(&f.plan, inplace ? rocfft_placement_inplace : rocfft_placement_notinplace,
                                   rocfft_transform_type_complex_inverse, rocfft_precision_single, 1, len, batch, desc);
        rocfft_plan_description_destroy(desc);
        if (s != rocfft_status_success) return tetra_fail(ctx, TETRA_E_HIP, "rocfft_plan_create failed (%d)", (int)s);
        rocfft_plan_get_work_buffer_size(f.plan, &f.work);
        rocfft_execution_info_create(&f.info);
        cache->plans.push_back(f);
        fp = &cache->plans.back();
    }
    if (fp->work > cache->work.bytes) {
        if (cache->work.p) HIP_TRY(ctx, hipFree(cache->work.p));
        cache->work = DevBuf{};
        HIP_TRY(ctx, hipMalloc(&cache->work.p, fp->work));
        cache->work.bytes = fp->work;
    }
    if (fp->work) rocfft_execution_info_set_work_buffer(fp->info, cache->work.p, fp->work);
    rocfft_execution_info_set_stream(fp->info, ctx->stream);
    void *ib[1] = {in}, *ob[1] = {out};
    if (rocfft_execute(fp->plan, ib, inplace ? nullptr : ob, fp->info) != rocfft_status_success)
        return tetra_fail(ctx, TETRA_E_HIP, "rocfft_execute failed");
    return TETRA_OK;
}

int wb_check(tetra_ctx *ctx, const tetra_wb_plan *P) {
    if (!P || !P->h || !P->g) return tetra_fail(ctx, TETRA_E_INVALID, "null wideband plan");
    if (P->M <= 0 || P->D <= 0 || P->M != 4 * P->D || P->P < 1 || P->P > 8)
        return tetra_fail(ctx, TETRA_E_INVALID, "wideband plan needs M = 4 D and 1 <= P <= 8");
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

int tetra_channelize(tetra_ctx *ctx, const tetra_wb_plan *P, const void *x, size_t Nw, void *y, size_t n_keep) {
    if (!ctx) return TETRA_E_INVALID;
    int rc = wb_check(ctx, P);
    if (rc) return rc;
    int64_t nblk, n72;
    tetra_wb_lengths(P, Nw, &nblk, &n72);
    if (n72 <= 0 || n_keep == 0 || (int64_t)n_keep > n72)
        return tetra_fail(ctx, TETRA_E_INVALID, "n_keep must be in [1, %ld] for %zu samples", (long)n72, Nw);
    const int M = P->M, L = M * P->P, Q = P->Lg / P->up;
    Staging st(ctx);
    const float2 *xd = (const float2 *)st.in(x, Nw * 8);
    float2 *yd = (float2 *)st.out(y, (size_t)M * n_keep * 8);
    float2 *u = (float2 *)ws(ctx, S_W8, (size_t)nblk * M * 8);
    if (Q != 45 || P->up > 32) return tetra_fail(ctx, TETRA_E_INVALID, "resampler built for Lg / up = 45 taps");
    float *taps = (float *)ws(ctx, S_W9, (size_t)(L + P->up * RS_QP) * 4);
    if (!xd || !yd || !u || !taps) return st.finish();
    // h, then g phase-major: gT[rho][q] = g[rho + up q] (zero-padded to RS_QP)
    ctx->taps_wb.assign(P->h, P->h + L);
    ctx->taps_wb.resize((size_t)L + P->up * RS_QP, 0.f);
    for (int rho = 0; rho < P->up; ++rho)
        for (int q = 0; q < Q; ++q) ctx->taps_wb[L + rho * RS_QP + q] = P->g[rho + P->up * q];
    HIP_TRY(ctx, hipMemcpyAsync(taps, ctx->taps_wb.data(), ctx->taps_wb.size() * 4, hipMemcpyHostToDevice,
                                ctx->stream));
    {
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
    {
        PROF(ctx, "wb_fft");
        rc = fft_backward(ctx, M, nblk, 1, M, 1, M, u, u);
        if (rc) return rc;
    }
    {
        PROF(ctx, "wb_resamp");
        const int rows = (int)(((long)P->down * (RS_T - 1)) / P->up) + Q + 1;
        const size_t lds = (size_t)std::max(rows * RS_C, RS_C * (RS_T + 1)) * 8;
        if (lds > 160 * 1024) return tetra_fail(ctx, TETRA_E_INVALID, "resampler tile does not fit LDS");
        const dim3 gr((unsigned)((M + RS_C - 1) / RS_C), (unsigned)((n_keep + RS_T - 1) / RS_T));
        hipLaunchKernelGGL(k_pfb_resamp<45>, gr, dim3(256), lds, ctx->stream, u, M, (int)nblk, P->up, P->down,
                           taps + L, yd, (int)n_keep);
        HIP_TRY(ctx, hipGetLastError());
    }
    return st.finish();
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
    // W[j][r] = sum_k s[k][j] e^{+i 2 pi k r / M}: input stride nbb between carriers, 1 between j
    rc = fft_backward(ctx, M, nbb, nbb, 1, 1, M, s, W);
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
