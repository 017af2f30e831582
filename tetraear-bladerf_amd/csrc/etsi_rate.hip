// etsi_rate.hip -- the ETSI channel filter at any supported input rate (generic plan).
//
// The reference's CLI takes the sample rate as an argument and its GUI slider spans 1.8-2.4 MSps
// in 0.1 MHz steps (/root/reference/tetraear/ui/modern.py:5518-5519, 5630-5638); process() takes
// whatever rate the SignalProcessor was built for (processor.py:245-257).  The fused kernels of
// etsi_rx.hip are specialised for 2.4 MSps (stage 1 / 10, stage 2 x3/10 on MFMA).  Every other
// rate runs here: stage 1 = L1-tap FIR decimating by q1, stage 2 = polyphase RRC x up/down to
// 72 kHz, written to HBM for k_timing.  The arithmetic restates oracle/etsi_oracle.c eo_chanfilt
// operation for operation -- stage 1 one fmaf chain per component over j ascending, stage 2 one
// over k ascending from kmin -- so the GPU is bit-identical to the oracle at every rate (and to
// the fused kernels at 2.4 MSps: TETRA_ETSI_FORCE_GENERIC).
//
// Layout: one workgroup per (channel, tile of RT1 stage-1 outputs).  The tile's input samples
// (q1 (RT1 - 1) + L1, 16-B coalesced loads) and both tap tables are staged in LDS; consecutive tiles
// overlap by the stage-2 window, so each stage-2 output is computed by exactly one tile from
// stage-1 values that tile computed itself.  HBM traffic: the input once (+ the overlap, ~25 %
// at 2.4 MSps), y once.
#include "common.h"

namespace {

constexpr int RT1 = 512;                       // stage-1 outputs per tile
constexpr int RQ1 = 13, RL1 = 64, RLP = 4096;  // plan limits
constexpr int RIN = RQ1 * (RT1 - 1) + RL1;     // input samples per tile (upper bound)

__host__ __device__ inline long mstart(long kb, int up, int down) {   // first m with kmin(m) >= kb
    return kb <= 0 ? 0 : (long)up * (kb - 1) / down + 1;
}

template <bool SC16>
__global__ __launch_bounds__(256) void k_chanfilt_g(const void *__restrict__ iq, long ld, int M1, int M2, int q1,
                                                    int L1, int up, int down, int Lp, int S1, int ntiles,
                                                    const float *__restrict__ taps, float2 *__restrict__ y) {
    __shared__ float2 xin[RIN];
    __shared__ float2 x1[RT1];
    __shared__ float h1s[RL1];
    __shared__ float hps[RLP];
    const int ch = blockIdx.x / ntiles, t = blockIdx.x - ch * ntiles, tid = threadIdx.x;
    const long k0 = (long)t * S1;
    const int nk = (int)min((long)RT1, (long)M1 - k0);
    const bool last = k0 + S1 >= M1;
    const long m0 = mstart(k0, up, down), m1 = last ? M2 : min((long)M2, mstart(k0 + S1, up, down));
    for (int i = tid; i < L1; i += 256) h1s[i] = taps[i];
    for (int i = tid; i < Lp; i += 256) hps[i] = taps[RL1 + i];
    // the tile's input: samples [q1 k0, q1 (k0 + nk - 1) + L1) of the channel's row (rows ld samples
    // apart: a streaming window inside a resident capture, tetra_demod_etsi_stream)
    const long base = (long)q1 * k0;
    const int nin = q1 * (nk - 1) + L1;
    if constexpr (SC16) {
        // SC16 (capture.py:241-269 wire format): int16 I/Q scaled by 1/32768 -- exact, so the
        // filter sees the cf32 values of the oracle's input
        const uint32_t *row = reinterpret_cast<const uint32_t *>(iq) + (size_t)ch * ld;
        const float s = 1.0f / 32768.0f;
        for (int i = tid; i < nin; i += 256) {
            const uint32_t v = row[base + i];
            xin[i] = make_float2((float)(int16_t)(v & 0xFFFFu) * s, (float)(int16_t)(v >> 16) * s);
        }
    } else {
        const float2 *row = reinterpret_cast<const float2 *>(iq) + (size_t)ch * ld;
        for (int i = tid; i < nin; i += 256) xin[i] = row[base + i];
    }
    __syncthreads();
    // stage 1: x1[k] = sum_j h1[j] x[q1 k + j]
    for (int i = tid; i < nk; i += 256) {
        const float2 *xp = xin + q1 * i;
        float ar = 0.f, ai = 0.f;
        for (int j = 0; j < L1; ++j) {
            const float h = h1s[j];
            const float2 v = xp[j];
            ar = fmaf(h, v.x, ar);
            ai = fmaf(h, v.y, ai);
        }
        x1[i] = make_float2(ar, ai);
    }
    __syncthreads();
    // stage 2: y[m] = sum_{k = kmin}^{kmax} hp[n - up k] x1[k], n = Lp - 1 + down m
    for (long m = m0 + tid; m < m1; m += 256) {
        const long n = (long)(Lp - 1) + (long)down * m;
        const long kmin = ((long)down * m + up - 1) / up, kmax = n / up;
        float ar = 0.f, ai = 0.f;
        for (long k = kmin; k <= kmax; ++k) {
            const float h = hps[n - (long)up * k];
            const float2 v = x1[k - k0];
            ar = fmaf(h, v.x, ar);
            ai = fmaf(h, v.y, ai);
        }
        y[(size_t)ch * M2 + m] = make_float2(ar, ai);
    }
}

}  // namespace

// Plan limits of the generic kernel (nullptr when the plan fits).
const char *etsi_generic_unsupported(const tetra_etsi_plan *P) {
    if (P->q1 < 1 || P->q1 > RQ1) return "q1 must be 1..13";
    if (P->L1 < 1 || P->L1 > RL1) return "L1 must be 1..64";
    if (P->up < 1 || P->down < 1) return "up and down must be >= 1";
    if (P->Lp < 1 || P->Lp > RLP) return "Lp must be 1..4096";
    if ((P->Lp - 1) / P->up + 2 >= RT1 / 2) return "stage-2 window (Lp / up) too long";
    return nullptr;
}

int launch_chanfilt_generic(tetra_ctx *ctx, const tetra_etsi_plan *P, const void *x, int fmt, size_t C, size_t N,
                            int64_t M1, int64_t M2, float2 *y, size_t ld) {
    if (ld == 0) ld = N;
    const int S1 = RT1 - ((P->Lp - 1) / P->up + 2);
    const long ntiles = (M1 + S1 - 1) / S1;
    if (ntiles <= 0 || (size_t)ntiles * C > 0x7FFFFFFFu) return tetra_fail(ctx, TETRA_E_INVALID, "grid too large");
    // taps: h1 [RL1] then hp [Lp], uploaded when they change
    std::vector<float> t(RL1 + P->Lp, 0.f);
    for (int j = 0; j < P->L1; ++j) t[j] = P->h1[j];
    for (int j = 0; j < P->Lp; ++j) t[RL1 + j] = P->hp[j];
    float *dt = (float *)ws(ctx, S_W15, (RL1 + RLP) * 4);
    if (!dt) return TETRA_E_NOMEM;
    if (ctx->taps_rate_dev != dt || ctx->taps_rate != t) {
        ctx->taps_rate = t;
        HIP_TRY(ctx, hipMemcpyAsync(dt, ctx->taps_rate.data(), t.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        ctx->taps_rate_dev = dt;
    }
    PROF(ctx, "etsi_chanfilt_g");
    const dim3 g((unsigned)(ntiles * C)), b(256);
    if (fmt == TETRA_SC16)
        hipLaunchKernelGGL(k_chanfilt_g<true>, g, b, 0, ctx->stream, x, (long)ld, (int)M1, (int)M2, P->q1, P->L1, P->up,
                           P->down, P->Lp, S1, (int)ntiles, dt, y);
    else
        hipLaunchKernelGGL(k_chanfilt_g<false>, g, b, 0, ctx->stream, x, (long)ld, (int)M1, (int)M2, P->q1, P->L1,
                           P->up, P->down, P->Lp, S1, (int)ntiles, dt, y);
    HIP_TRY(ctx, hipGetLastError());
    return TETRA_OK;
}

const void *chanfilt_generic_fn(int fmt) {
    return fmt == TETRA_SC16 ? reinterpret_cast<const void *>(&k_chanfilt_g<true>)
                             : reinterpret_cast<const void *>(&k_chanfilt_g<false>);
}
