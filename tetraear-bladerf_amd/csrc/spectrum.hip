// spectrum.hip -- waterfall spectrum frames: Hann window -> 2048-point FFT -> fftshift -> dBFS,
// fused in one pass (SURVEY.md §8d config C3 "2048-pt Hann waterfall"; BASELINE.json north_star
// "waterfall FFT").  The display this feeds is the reference's live spectrum,
// /root/reference/tetraear/ui/modern.py:1928-1941 (one frame x[:2048] per chunk, numpy float64,
// power = 20 log10(|fftshift(fft(x w))| / N + 1e-20)); oracle/spectrum.py restates that definition.
//
// Why not rocFFT here: a library transform needs a window pass before it and a |.|/log pass after
// it, 8 + 8 + 8 + 8 + 8 + 4 = 44 B of HBM per sample; this kernel reads the samples once and writes
// the dB value once, 8 + 4 = 12 B per sample (cf32), and stays HBM-bound.
//
// One workgroup (256 threads) per frame at a time, looping over frames (grid = the chip's
// residency): the frame lives in 18 KB of LDS (padded index i + i/8, so the radix-8 scatter
// writes are bank-conflict free), the per-stage twiddles in a 16 KB LDS table loaded once per
// workgroup.  Mixed-radix Stockham 8 x 8 x 8 x 4 (autosort: natural-order output, no bit
// reversal): stage 1 reads straight from HBM (the next frame's loads are issued before the current
// frame's LDS stages), stage 4 writes the shifted dB row to HBM with 4-byte coalesced stores.
#include "common.h"

#include <mutex>

#pragma clang fp contract(fast)   // the spectrum is a tolerance product (oracle/spectrum.py), not a bit-exact one

namespace {

constexpr int WF_N = 2048;
constexpr int WF_T = 256;                  // threads per workgroup
constexpr int WF_PAD = WF_N + WF_N / 8;    // padded frame (float2)
constexpr int TW2 = 0, TW3 = 8 * 7, TW4 = TW3 + 64 * 7, TW_N = TW4 + 512 * 3;   // 2040 twiddles

__device__ __forceinline__ int pad(int i) { return i + (i >> 3); }

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }   // a * (-i)

// forward DFT-4 in place: X[k] = sum_n a[n] e^{-2 pi i n k / 4}
__device__ __forceinline__ void dft4(float2 &a0, float2 &a1, float2 &a2, float2 &a3) {
    const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = mul_mi(csub(a1, a3));
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = cadd(t1, t3);
    a3 = csub(t1, t3);
}

// forward DFT-8 in place (even/odd split into two DFT-4s, then W8^k)
__device__ __forceinline__ void dft8(float2 *v) {
    float2 e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    float2 o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    const float s = 0.70710678118654752f;
    o1 = make_float2((o1.x + o1.y) * s, (o1.y - o1.x) * s);     // * e^{-i pi/4}
    o2 = mul_mi(o2);                                            // * e^{-i pi/2}
    o3 = make_float2((o3.y - o3.x) * s, -(o3.x + o3.y) * s);    // * e^{-3 i pi/4}
    v[0] = cadd(e0, o0);
    v[4] = csub(e0, o0);
    v[1] = cadd(e1, o1);
    v[5] = csub(e1, o1);
    v[2] = cadd(e2, o2);
    v[6] = csub(e2, o2);
    v[3] = cadd(e3, o3);
    v[7] = csub(e3, o3);
}

template <int FMT>
__device__ __forceinline__ float2 load_sample(const void *__restrict__ x, size_t i) {
    if constexpr (FMT == TETRA_CF32) {
        return reinterpret_cast<const float2 *>(x)[i];
    } else if constexpr (FMT == TETRA_SC16) {
        const uint32_t w = reinterpret_cast<const uint32_t *>(x)[i];
        const float k = 1.0f / 32768.0f;   // capture.py:241-269 scaling, exact in fp32
        return make_float2((float)(int16_t)(w & 0xFFFF) * k, (float)(int16_t)(w >> 16) * k);
    } else {
        const double2 d = reinterpret_cast<const double2 *>(x)[i];
        return make_float2((float)d.x, (float)d.y);
    }
}

// Radix-8 Stockham stage over the LDS frame: thread j owns butterfly j of N/8 = 256.
template <int NS, int TWO>
__device__ __forceinline__ void stage8(float2 *fr, const float2 *tw, int j) {
    float2 v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = fr[pad(j + 256 * r)];
    const int m = j % NS;
#pragma unroll
    for (int r = 1; r < 8; ++r) v[r] = cmul(v[r], tw[TWO + m * 7 + r - 1]);
    dft8(v);
    __syncthreads();   // every read of this stage is done before the in-place scatter
    const int base = (j / NS) * NS * 8 + m;
#pragma unroll
    for (int r = 0; r < 8; ++r) fr[pad(base + r * NS)] = v[r];
    __syncthreads();
}

// The signal-present / AFC gate of the reference's capture loop (modern.py:1952-2028; SURVEY.md §8f
// rank 1), evaluated on frame 0's dB row: the centre band [start, end) (25 kHz: int(25000 / (fs /
// 2048)) bins around bin 1024), its mean, maximum and first argmax; the noise floor = the mean of
// the bins below start - 10 and from end + 10 on (-100 dB when there are none); snr = mean - noise;
// signal present iff snr > 15, peak > -70 and peak - mean > 3; the AFC offset is the peak bin's
// frequency, fftshift(fftfreq(2048, 1/fs))[peak], when present.  The offset is also written as the
// compat demod's mixer inputs (tetra_demod_compat: coefficient -2 pi f and on/off), so process()
// can run on it with no host round trip.
struct GateArgs {
    int start, end, nb_end, nb2;   // centre band, noise bands [0, nb_end) and [nb2, 2048)
    double val;                    // fftfreq bin spacing 1 / (2048 (1 / fs))
    double *stats;                 // [C][TETRA_GATE_FIELDS]
    double *mc;                    // [C] mixer coefficient (or nullptr)
    uint8_t *mo;                   // [C] mixer on (or nullptr)
};

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block-wide gate reduction over the dB row in LDS (all 256 threads); thread 0 writes the results
__device__ void gate_row(const float *pw, const GateArgs &ga, long c, double *red, float *redf, int *redi) {
    const int j = threadIdx.x, lane = j & 63, w = j >> 6;
    double ssum = 0.0, nsum = 0.0;
    float pk = -INFINITY;
    int pki = 0x7FFFFFFF;
    for (int i = ga.start + j; i < ga.end; i += WF_T) {
        const float v = pw[i];
        ssum += (double)v;
        if (v > pk) { pk = v; pki = i; }   // ascending i per thread: the first maximum
    }
    for (int i = j; i < ga.nb_end; i += WF_T) nsum += (double)pw[i];
    for (int i = ga.nb2 + j; i < WF_N; i += WF_T) nsum += (double)pw[i];
    ssum = wave_sum_d(ssum);
    nsum = wave_sum_d(nsum);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {   // max, ties to the lower bin
        const float pv = __shfl_xor(pk, o, 64);
        const int pi = __shfl_xor(pki, o, 64);
        if (pv > pk || (pv == pk && pi < pki)) { pk = pv; pki = pi; }
    }
    if (lane == 0) { red[2 * w] = ssum; red[2 * w + 1] = nsum; redf[w] = pk; redi[w] = pki; }
    __syncthreads();
    if (j == 0) {
        double S = 0.0, Nn = 0.0;
        float P = -INFINITY;
        int Pi = 0x7FFFFFFF;
        for (int q = 0; q < WF_T / 64; ++q) {
            S += red[2 * q];
            Nn += red[2 * q + 1];
            if (redf[q] > P || (redf[q] == P && redi[q] < Pi)) { P = redf[q]; Pi = redi[q]; }
        }
        const int nsig = ga.end - ga.start, nnoise = ga.nb_end + (WF_N - ga.nb2);
        double *st = ga.stats + (size_t)c * TETRA_GATE_FIELDS;
        double present = 0.0, afc = 0.0;
        if (nsig > 0) {
            const double sig = S / nsig, peak = (double)P;
            const double noise = nnoise > 0 ? Nn / nnoise : -100.0;
            const double snr = sig - noise, above = peak - sig;
            const double fo = (double)(Pi - WF_N / 2) * ga.val;
            present = (snr > 15.0 && peak > -70.0 && above > 3.0) ? 1.0 : 0.0;
            afc = (present != 0.0 && peak > -70.0) ? fo : 0.0;   // modern.py:2028
            st[TETRA_GATE_SIGNAL] = sig;
            st[TETRA_GATE_PEAK] = peak;
            st[TETRA_GATE_PEAK_BIN] = (double)Pi;
            st[TETRA_GATE_PEAK_FREQ] = fo;
            st[TETRA_GATE_NOISE] = noise;
            st[TETRA_GATE_SNR] = snr;
            st[TETRA_GATE_ABOVE] = above;
        } else {
            for (int q = TETRA_GATE_SIGNAL; q <= TETRA_GATE_ABOVE; ++q) st[q] = 0.0;
        }
        st[TETRA_GATE_VALID] = nsig > 0 ? 1.0 : 0.0;
        st[TETRA_GATE_PRESENT] = present;
        st[TETRA_GATE_AFC] = afc;
        if (ga.mc) ga.mc[c] = afc != 0.0 ? (-2.0 * 3.141592653589793) * afc : 0.0;   // processor.py:99
        if (ga.mo) ga.mo[c] = afc != 0.0 ? 1 : 0;
    }
}

// out[g][WF_N] for frames g = (c, f): x[c * N + f * hop + n], n < 2048.  GATE: one frame per
// channel, the gate evaluated on its row (out may then be null).
template <int FMT, bool GATE = false>
__global__ __launch_bounds__(WF_T) void k_waterfall(const void *__restrict__ x, size_t N, size_t hop, int nframes,
                                                   long total, const float *__restrict__ win,
                                                   const float2 *__restrict__ twg, float *__restrict__ out,
                                                   GateArgs ga = GateArgs{}) {
    __shared__ float2 fr[WF_PAD];
    __shared__ float2 tw[TW_N];
    __shared__ float pw[GATE ? WF_N : 1];
    __shared__ double red[GATE ? 2 * WF_T / 64 : 1];
    __shared__ float redf[GATE ? WF_T / 64 : 1];
    __shared__ int redi[GATE ? WF_T / 64 : 1];
    const int j = threadIdx.x;
    for (int i = j; i < TW_N; i += WF_T) tw[i] = twg[i];
    float w[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) w[r] = win[j + 256 * r];
    long g = blockIdx.x;
    float2 xr[8];
    auto issue = [&](long gg) {
        const long c = gg / nframes, f = gg - c * nframes;
        const size_t base = (size_t)c * N + (size_t)f * hop + j;
#pragma unroll
        for (int r = 0; r < 8; ++r) xr[r] = load_sample<FMT>(x, base + 256 * r);
    };
    if (g < total) issue(g);
    __syncthreads();   // twiddle table
    for (; g < total; g += gridDim.x) {
        // stage 1 (Ns = 1: no twiddles) on the frame's samples in registers
        float2 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = make_float2(xr[r].x * w[r], xr[r].y * w[r]);
        if (g + gridDim.x < total) issue(g + gridDim.x);   // next frame's loads fly over the LDS stages
        dft8(v);
#pragma unroll
        for (int r = 0; r < 8; ++r) fr[pad(8 * j + r)] = v[r];
        __syncthreads();
        stage8<8, TW2>(fr, tw, j);
        stage8<64, TW3>(fr, tw, j);
        // stage 4: radix 4, Ns = 512, butterflies j and j + 256 -> natural-order bins j + 512 r
        float *o = out ? out + (size_t)g * WF_N : nullptr;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int jj = j + 256 * h;
            float2 a0 = fr[pad(jj)], a1 = fr[pad(jj + 512)], a2 = fr[pad(jj + 1024)], a3 = fr[pad(jj + 1536)];
            a1 = cmul(a1, tw[TW4 + jj * 3 + 0]);
            a2 = cmul(a2, tw[TW4 + jj * 3 + 1]);
            a3 = cmul(a3, tw[TW4 + jj * 3 + 2]);
            dft4(a0, a1, a2, a3);
            const float2 a[4] = {a0, a1, a2, a3};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = jj + 512 * r;
                const float mag = sqrtf(a[r].x * a[r].x + a[r].y * a[r].y);
                const float db = 20.0f * log10f(mag * (1.0f / WF_N) + 1e-20f);
                const int sidx = (k + WF_N / 2) & (WF_N - 1);
                if constexpr (GATE) {
                    pw[sidx] = db;
                    if (out) __builtin_nontemporal_store(db, &o[sidx]);
                } else {
                    __builtin_nontemporal_store(db, &o[sidx]);
                }
            }
        }
        __syncthreads();   // stage-4 reads done before the next frame's stage-1 scatter
        if constexpr (GATE) {
            gate_row(pw, ga, g, red, redf, redi);
            __syncthreads();   // pw / red reads done before the next frame
        }
    }
}

struct WfTables {
    float win[WF_N];
    float2 tw[TW_N];
};

void wf_tables(WfTables &t) {
    const double pi = 3.14159265358979323846;
    for (int n = 0; n < WF_N; ++n) t.win[n] = (float)(0.5 - 0.5 * cos(2.0 * pi * n / (WF_N - 1)));   // np.hanning
    auto tw = [&](int off, int ns, int R) {
        for (int m = 0; m < ns; ++m)
            for (int r = 1; r < R; ++r) {
                const double a = -2.0 * pi * m * r / (ns * R);
                t.tw[off + m * (R - 1) + r - 1] = make_float2((float)cos(a), (float)sin(a));
            }
    };
    tw(TW2, 8, 8);
    tw(TW3, 64, 8);
    tw(TW4, 512, 4);
}

}  // namespace

extern "C" {

int tetra_waterfall(tetra_ctx *ctx, const void *iq, int iq_fmt, size_t C, size_t N, size_t nfft, size_t hop,
                    size_t nframes, float *out) {
    if (!ctx) return TETRA_E_INVALID;
    if (nfft != WF_N) return tetra_fail(ctx, TETRA_E_INVALID, "waterfall is built for nfft = %d", WF_N);
    if (iq_fmt != TETRA_CF32 && iq_fmt != TETRA_SC16 && iq_fmt != TETRA_CF64)
        return tetra_fail(ctx, TETRA_E_INVALID, "unknown sample format %d", iq_fmt);
    if (!iq || !out || C == 0 || nframes == 0) return tetra_fail(ctx, TETRA_E_INVALID, "empty waterfall request");
    if (nframes > 1 && hop == 0) return tetra_fail(ctx, TETRA_E_INVALID, "hop must be > 0 for several frames");
    if ((nframes - 1) * hop + WF_N > N)
        return tetra_fail(ctx, TETRA_E_INVALID, "%zu frames of %d at hop %zu do not fit %zu samples", nframes, WF_N,
                          hop, N);
    const size_t bps = iq_fmt == TETRA_CF32 ? 8 : iq_fmt == TETRA_SC16 ? 4 : 16;
    const long total = (long)(C * nframes);
    Staging st(ctx);
    const void *xd = st.in(iq, C * N * bps);
    float *od = (float *)st.out(out, (size_t)total * WF_N * 4);
    WfTables *tab = (WfTables *)ws(ctx, S_W11, sizeof(WfTables));
    if (!xd || !od || !tab) return st.finish();
    if (!ctx->wf_tables_ready) {   // window + twiddles, built once per process (contexts may live on several threads)
        static WfTables host;
        static std::once_flag once;
        std::call_once(once, [] { wf_tables(host); });
        HIP_TRY(ctx, hipMemcpyAsync(tab, &host, sizeof(WfTables), hipMemcpyHostToDevice, ctx->stream));
        ctx->wf_tables_ready = true;
    }
    {
        PROF(ctx, "waterfall");
        // four 34 KB workgroups per CU on 256 CUs; never more workgroups than frames
        const unsigned grid = (unsigned)std::min<long>(total, 256 * 4);
        switch (iq_fmt) {
            case TETRA_CF32:
                hipLaunchKernelGGL(k_waterfall<TETRA_CF32>, dim3(grid), dim3(WF_T), 0, ctx->stream, xd,
                                   N, hop, (int)nframes, total, tab->win, tab->tw, od);
                break;
            case TETRA_SC16:
                hipLaunchKernelGGL(k_waterfall<TETRA_SC16>, dim3(grid), dim3(WF_T), 0, ctx->stream, xd, N, hop,
                                   (int)nframes, total, tab->win, tab->tw, od);
                break;
            default:
                hipLaunchKernelGGL(k_waterfall<TETRA_CF64>, dim3(grid), dim3(WF_T), 0, ctx->stream, xd, N, hop,
                                   (int)nframes, total, tab->win, tab->tw, od);
        }
        HIP_TRY(ctx, hipGetLastError());
    }
    return st.finish();
}

int tetra_afc_gate(tetra_ctx *ctx, const void *iq, int iq_fmt, size_t C, size_t N, double fs, float *power,
                   double *stats, double *mixer_coef, uint8_t *mixer_on) {
    if (!ctx) return TETRA_E_INVALID;
    if (iq_fmt != TETRA_CF32 && iq_fmt != TETRA_SC16 && iq_fmt != TETRA_CF64)
        return tetra_fail(ctx, TETRA_E_INVALID, "unknown sample format %d", iq_fmt);
    if (!iq || !stats || C == 0 || !(fs > 0.0)) return tetra_fail(ctx, TETRA_E_INVALID, "bad gate request");
    const size_t bps = iq_fmt == TETRA_CF32 ? 8 : iq_fmt == TETRA_SC16 ? 4 : 16;
    Staging st(ctx);
    double *sd = (double *)st.out(stats, C * TETRA_GATE_FIELDS * 8);
    double *mcd = mixer_coef ? (double *)st.out(mixer_coef, C * 8) : nullptr;
    uint8_t *mod = mixer_on ? (uint8_t *)st.out(mixer_on, C) : nullptr;
    if (!sd || (mixer_coef && !mcd) || (mixer_on && !mod)) return st.finish();
    if (N < (size_t)WF_N) {   // no spectrum, no detection (modern.py:1929, 1954): zeros, signal absent
        HIP_TRY(ctx, hipMemsetAsync(sd, 0, C * TETRA_GATE_FIELDS * 8, ctx->stream));
        if (mcd) HIP_TRY(ctx, hipMemsetAsync(mcd, 0, C * 8, ctx->stream));
        if (mod) HIP_TRY(ctx, hipMemsetAsync(mod, 0, C, ctx->stream));
        if (power) return tetra_fail(ctx, TETRA_E_INVALID, "no 2048-sample frame in %zu samples", N);
        return st.finish();
    }
    const void *xd = st.in(iq, C * N * bps);
    float *od = power ? (float *)st.out(power, C * WF_N * 4) : nullptr;
    WfTables *tab = (WfTables *)ws(ctx, S_W11, sizeof(WfTables));
    if (!xd || (power && !od) || !tab) return st.finish();
    if (!ctx->wf_tables_ready) {
        static WfTables host;
        static std::once_flag once;
        std::call_once(once, [] { wf_tables(host); });
        HIP_TRY(ctx, hipMemcpyAsync(tab, &host, sizeof(WfTables), hipMemcpyHostToDevice, ctx->stream));
        ctx->wf_tables_ready = true;
    }
    // the band and noise bins, as the capture loop derives them from fs (host doubles, same ops)
    GateArgs ga{};
    const double fres = fs / (double)WF_N;
    const int bb = (int)(25000.0 / fres);
    ga.start = std::max(0, WF_N / 2 - bb / 2);
    ga.end = std::min(WF_N, WF_N / 2 + bb / 2);
    ga.nb_end = std::max(0, ga.start - 10);
    ga.nb2 = std::min(WF_N, ga.end + 10);
    if (ga.end < ga.start) ga.end = ga.start;
    ga.val = 1.0 / ((double)WF_N * (1.0 / fs));
    ga.stats = sd;
    ga.mc = mcd;
    ga.mo = mod;
    {
        PROF(ctx, "afc_gate");
        const unsigned grid = (unsigned)std::min<long>((long)C, 256 * 4);
        switch (iq_fmt) {
            case TETRA_CF32:
                hipLaunchKernelGGL((k_waterfall<TETRA_CF32, true>), dim3(grid), dim3(WF_T), 0, ctx->stream, xd, N,
                                   (size_t)WF_N, 1, (long)C, tab->win, tab->tw, od, ga);
                break;
            case TETRA_SC16:
                hipLaunchKernelGGL((k_waterfall<TETRA_SC16, true>), dim3(grid), dim3(WF_T), 0, ctx->stream, xd, N,
                                   (size_t)WF_N, 1, (long)C, tab->win, tab->tw, od, ga);
                break;
            default:
                hipLaunchKernelGGL((k_waterfall<TETRA_CF64, true>), dim3(grid), dim3(WF_T), 0, ctx->stream, xd, N,
                                   (size_t)WF_N, 1, (long)C, tab->win, tab->tw, od, ga);
        }
        HIP_TRY(ctx, hipGetLastError());
    }
    return st.finish();
}

}  // extern "C"
