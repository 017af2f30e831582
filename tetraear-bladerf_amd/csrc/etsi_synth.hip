// etsi_synth.hip -- device-side synthetic TETRA capture generator (loopback test signal).
//
// Builds, per channel, a continuous downlink of ETSI bursts (normal bursts with training
// sequence n or p, synchronisation bursts) carrying random but properly coded blocks (CRC-16,
// RCPC 2/3, interleaving, scrambling -- same rules as the receiver, EN 300 392-2 §8/§9.4.4),
// modulates it as pi/4-DQPSK with RRC(0.35) pulses at the channel sample rate, and applies a
// random carrier phase, a carrier frequency offset, AWGN and the SC16 quantisation of a capture
// (round(x*32768)/32768, as /root/reference/tetraear/signal/capture.py:259-269 produces).
// Used by bench.py (data generated in HBM, never crossing PCIe) and by the GPU tests.
#include "common.h"

namespace {

constexpr int SPAN = 6;

__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}
__device__ inline uint64_t hkey(uint64_t seed, uint64_t a, uint64_t b, uint64_t c) {
    return mix64(seed ^ mix64(a * 0x9E3779B97F4A7C15ull ^ mix64(b * 0xD1B54A32D192ED03ull ^ c)));
}
__device__ inline float u01(uint64_t h) { return (float)((h >> 40) + 0.5) * (1.0f / 16777216.0f); }

struct KindP { int K, a, n2, n1; };
__device__ inline KindP kp(int kind) {
    return kind == 0 ? KindP{432, 103, 288, 268} : kind == 1 ? KindP{216, 101, 144, 124} : KindP{120, 11, 80, 60};
}
__device__ inline int punct_index(int j1) {
    const int g = (j1 - 1) / 3, r = j1 - 3 * g;
    return 8 * g + (r == 1 ? 1 : r == 2 ? 2 : 5);
}
__device__ inline uint32_t scr_bit(uint32_t init, int k, uint8_t *cache) { return cache[k]; }

constexpr int QB[22] = {1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 0, 1, 0, 1, 1, 0, 1};
constexpr int NB_[22] = {1, 1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 1, 0, 0, 1, 1, 1, 0, 1, 0, 0};
constexpr int PB[22] = {0, 1, 1, 1, 1, 0, 1, 0, 0, 1, 0, 0, 0, 0, 1, 1, 0, 1, 1, 1, 0, 0};
constexpr int YB[38] = {1, 1, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 1, 1, 0, 0, 1, 1, 1,
                        0, 1, 0, 0, 1, 1, 1, 0, 0, 0, 0, 0, 1, 1, 0, 0, 1, 1, 1};

// Encode one block into burst bits: positions pos(k) for type-5 index k.
__device__ void encode_into(const uint8_t *t1, int kind, const uint8_t *scr, uint8_t *t2s, uint8_t *burst,
                            int o1, int o2, int lane) {
    const KindP P = kp(kind);
    if (lane == 0) {
        uint32_t c = 0xFFFF;
        for (int i = 0; i < P.n1; ++i) {
            t2s[i] = t1[i];
            c ^= (uint32_t)t1[i] << 15;
            c = (c & 0x8000u) ? ((c << 1) ^ 0x1021u) : (c << 1);
            c &= 0xFFFFu;
        }
        c ^= 0xFFFFu;
        for (int k = 0; k < 16; ++k) t2s[P.n1 + k] = (c >> (15 - k)) & 1u;
        for (int k = 0; k < 4; ++k) t2s[P.n1 + 16 + k] = 0;
    }
    __syncthreads();
    for (int i = 1 + lane; i <= P.K; i += 64) {
        const int mi = punct_index(i) - 1, step = mi >> 2, gen = mi & 3;
        const uint32_t bb = t2s[step];
        const uint32_t e0 = step >= 1 ? t2s[step - 1] : 0, e1 = step >= 2 ? t2s[step - 2] : 0,
                       e2 = step >= 3 ? t2s[step - 3] : 0, e3 = step >= 4 ? t2s[step - 4] : 0;
        const uint32_t v = gen == 0 ? (bb ^ e0 ^ e3) : gen == 1 ? (bb ^ e1 ^ e2 ^ e3)
                                                                : gen == 2 ? (bb ^ e0 ^ e1 ^ e3) : (bb ^ e0 ^ e2 ^ e3);
        const int k = 1 + (int)(((long)P.a * i) % P.K);
        const int pos = (kind == 0 && k - 1 >= 216) ? o2 + (k - 1 - 216) : o1 + (k - 1);
        burst[pos] = (uint8_t)(v ^ scr[k - 1]);
    }
    __syncthreads();
}

// One wave per (channel, burst).
__global__ __launch_bounds__(64) void k_synth_bursts(uint64_t seed, int NBR, const uint8_t *__restrict__ cell_scr,
                                                     const uint8_t *__restrict__ bsch_scr,
                                                     const uint32_t *__restrict__ cell_init, uint8_t *__restrict__ bits,
                                                     int32_t *__restrict__ kinds, uint8_t *__restrict__ payload) {
    const int ch = blockIdx.x / NBR, b = blockIdx.x % NBR, lane = threadIdx.x;
    __shared__ uint8_t t1[2][268];
    __shared__ uint8_t t2s[288];
    uint8_t *burst = bits + ((size_t)ch * NBR + b) * 510;
    const uint64_t hk = hkey(seed, ch, b, 0xB0B0);
    const int r = (int)(hk & 3);
    const int bk = r < 2 ? 0 : (r == 2 ? 1 : 2);   // NDB(n) 1/2, NDB(p) 1/4, SB 1/4
    if (lane == 0) kinds[(size_t)ch * NBR + b] = bk;
    const int jk0 = bk == 0 ? 0 : (bk == 1 ? 1 : 2), jk1 = bk == 0 ? -1 : 1;
    for (int blk = 0; blk < 2; ++blk) {
        const int kind = blk == 0 ? jk0 : jk1;
        uint8_t *pl = payload + (((size_t)ch * NBR + b) * 2 + blk) * 268;
        if (kind < 0) {
            for (int i = lane; i < 268; i += 64) pl[i] = 0;
            continue;
        }
        const int n1 = kp(kind).n1;
        // BSCH: the SYNC PDU of the channel's cell -- MAC-SYNC colour code at bits 4..9 and
        // D-MLE-SYNC MCC 31..40 / MNC 41..54 (EN 300 392-2 §21.4.4.2, §18.4.2.1), MSB first
        const uint32_t ecc = cell_init[ch] >> 2;   // MCC(10) MNC(14) CC(6)
        for (int i = lane; i < 268; i += 64) {
            uint8_t v = i < n1 ? (uint8_t)(hkey(seed, ch, b * 2 + blk, i) & 1) : 0;
            if (kind == 2 && i >= 4 && i < 10) v = (uint8_t)((ecc >> (9 - i)) & 1u);          // CC
            if (kind == 2 && i >= 31 && i < 41) v = (uint8_t)((ecc >> (29 - (i - 31))) & 1u);  // MCC
            if (kind == 2 && i >= 41 && i < 55) v = (uint8_t)((ecc >> (19 - (i - 41))) & 1u);  // MNC
            t1[blk][i] = v;
            pl[i] = v;
        }
    }
    __syncthreads();
    // fixed fields: head q11..q22, phase-adjustment bits 0, tail q1..q10, broadcast bits random
    for (int i = lane; i < 510; i += 64) burst[i] = (uint8_t)(hkey(seed, ch, b, 0xBB00 + i) & 1);
    __syncthreads();
    for (int i = lane; i < 12; i += 64) burst[i] = QB[10 + i];
    for (int i = lane; i < 10; i += 64) burst[500 + i] = QB[i];
    if (lane < 2) { burst[12 + lane] = 0; burst[498 + lane] = 0; }
    const uint8_t *cs = cell_scr + (size_t)ch * 432;
    if (bk == 2) {
        for (int i = lane; i < 80; i += 64) burst[14 + i] = (i < 8 || i >= 72) ? 1 : 0;   // frequency correction
        for (int i = lane; i < 38; i += 64) burst[214 + i] = YB[i];
        __syncthreads();
        encode_into(t1[0], 2, bsch_scr, t2s, burst, 94, 94, lane);
        encode_into(t1[1], 1, cs, t2s, burst, 282, 282, lane);
    } else {
        for (int i = lane; i < 22; i += 64) burst[244 + i] = bk == 0 ? NB_[i] : PB[i];
        __syncthreads();
        if (bk == 0) {
            encode_into(t1[0], 0, cs, t2s, burst, 14, 282, lane);
        } else {
            encode_into(t1[0], 1, cs, t2s, burst, 14, 14, lane);
            encode_into(t1[1], 1, cs, t2s, burst, 282, 282, lane);
        }
    }
}

// Per channel: cumulative phase index (units of pi/4, mod 8) of every symbol.
__global__ __launch_bounds__(64) void k_synth_phase(const uint8_t *__restrict__ bits, int nsym, uint8_t *__restrict__ ph,
                                                    uint64_t seed) {
    const int ch = blockIdx.x, lane = threadIdx.x;
    const uint8_t *bp = bits + (size_t)ch * nsym * 2;
    uint8_t *pp = ph + (size_t)ch * nsym;
    const int per = (nsym + 63) / 64;
    const int s0 = lane * per, s1 = min(nsym, s0 + per);
    auto step = [&](int k) -> int {
        const int b1 = bp[2 * k], b2 = bp[2 * k + 1];
        return b1 == 0 ? (b2 == 0 ? 1 : 3) : (b2 == 0 ? 7 : 5);   // +pi/4, +3pi/4, -pi/4, -3pi/4 (Table 5.1)
    };
    int tot = 0;
    for (int k = s0; k < s1; ++k) tot += step(k);
    int incl = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    int acc = incl - tot;
    for (int k = s0; k < s1; ++k) {
        acc += step(k);
        pp[k] = (uint8_t)(acc & 7);
    }
}

__device__ inline float rrc(float t) {
    const float a = 0.35f, pi = 3.14159265f;
    const float at = fabsf(t);
    if (at < 1e-6f) return 1.0f - a + 4.0f * a / pi;
    if (fabsf(fabsf(4.0f * a * t) - 1.0f) < 1e-5f)
        return (a / 1.41421356f) * ((1.0f + 2.0f / pi) * sinf(pi / (4.0f * a)) + (1.0f - 2.0f / pi) * cosf(pi / (4.0f * a)));
    const float num = sinf(pi * t * (1.0f - a)) + 4.0f * a * t * cosf(pi * t * (1.0f + a));
    const float den = pi * t * (1.0f - (4.0f * a * t) * (4.0f * a * t));
    return num / den;
}

__global__ __launch_bounds__(256) void k_synth_iq(const uint8_t *__restrict__ ph, int nsym, long N, double fs,
                                                  uint64_t seed, float amp, float sigma, float cfo_max,
                                                  const double *__restrict__ t0s, float2 *__restrict__ iq) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = (int)(gid / N);
    const long n = gid - (long)ch * N;
    const uint64_t hc = hkey(seed, ch, 0, 0xC0C0);
    const float phi0 = 6.2831853f * u01(hc);
    const float cfo = cfo_max * (2.0f * u01(mix64(hc + 1)) - 1.0f);
    const double t = t0s[ch] + (double)n * (18000.0 / fs);
    const long k0 = (long)floor(t);
    const float fr = (float)(t - (double)k0);
    const uint8_t *pp = ph + (size_t)ch * nsym;
    float xr = 0.f, xi = 0.f;
    for (int d = -SPAN; d <= SPAN; ++d) {
        const long k = k0 + d;
        if (k < 0 || k >= nsym) continue;
        const float g = rrc(fr - (float)d);
        float s, c;
        sincosf(0.78539816f * (float)pp[k] + phi0, &s, &c);
        xr = fmaf(g, c, xr);
        xi = fmaf(g, s, xi);
    }
    // carrier offset, noise, SC16 grid
    const double ang = 6.283185307179586 * (double)cfo * (double)n / fs;
    const float ca = (float)cos(ang), sa = (float)sin(ang);
    float yr = amp * (xr * ca - xi * sa), yi = amp * (xr * sa + xi * ca);
    if (sigma > 0.f) {
        const uint64_t h = hkey(seed, ch, n, 0x7777);
        const float u1 = u01(h), u2 = u01(mix64(h));
        const float r = sqrtf(-2.0f * logf(u1));
        yr += sigma * r * cosf(6.2831853f * u2);
        yi += sigma * r * sinf(6.2831853f * u2);
    }
    yr = fminf(fmaxf(rintf(yr * 32768.f), -32768.f), 32767.f) * (1.0f / 32768.f);
    yi = fminf(fmaxf(rintf(yi * 32768.f), -32768.f), 32767.f) * (1.0f / 32768.f);
    iq[gid] = make_float2(yr, yi);
}

void lfsr(uint32_t r, int n, uint8_t *out) {
    for (int i = 0; i < n; ++i) {
        const uint32_t b = ((r >> 0) ^ (r >> 6) ^ (r >> 9) ^ (r >> 10) ^ (r >> 16) ^ (r >> 20) ^ (r >> 21) ^ (r >> 22) ^
                            (r >> 24) ^ (r >> 25) ^ (r >> 27) ^ (r >> 28) ^ (r >> 30) ^ (r >> 31)) & 1u;
        r = (r >> 1) | (b << 31);
        out[i] = (uint8_t)b;
    }
}

}  // namespace

extern "C" {

int tetra_synth_bursts_per_channel(size_t N, double fs) {
    const double syms = (double)N * 18000.0 / fs;
    return (int)((8.0 + 255.0 + syms + 8.0) / 255.0) + 1;
}

int tetra_synth_etsi(tetra_ctx *ctx, size_t C, size_t N, double fs, uint64_t seed, float snr_db, float cfo_max,
                     void *iq, uint32_t *cell_init, int32_t *kinds, uint8_t *payload, double *t0) {
    if (!ctx || C == 0 || N == 0 || !iq || !cell_init) return TETRA_E_INVALID;
    const int NBR = tetra_synth_bursts_per_channel(N, fs);
    const int nsym = NBR * 255;
    // per-channel cell identity and start time (host: tiny)
    std::vector<uint32_t> init(C);
    std::vector<double> t0h(C);
    std::vector<uint8_t> tab(C * 432 + 432);
    for (size_t c = 0; c < C; ++c) {
        const uint64_t h = mix64(seed * 0x9E3779B97F4A7C15ull + c);
        const uint32_t mcc = (uint32_t)(h & 0x3FF), mnc = (uint32_t)((h >> 10) & 0x3FFF), cc = (uint32_t)((h >> 24) & 0x3F);
        init[c] = ((((mcc & 0x3FFu) << 20) | ((mnc & 0x3FFFu) << 6) | (cc & 0x3Fu)) << 2) | 3u;
        t0h[c] = 8.0 + 255.0 * ((double)((h >> 32) & 0xFFFF) / 65536.0) + ((double)((h >> 48) & 0xFFF) / 4096.0);
        lfsr(init[c], 432, tab.data() + c * 432);
    }
    lfsr(3u, 432, tab.data() + C * 432);
    Staging st(ctx);
    float2 *x = (float2 *)st.out(iq, C * N * 8);
    uint32_t *ci = (uint32_t *)st.out(cell_init, C * 4);
    int32_t *kd = kinds ? (int32_t *)st.out(kinds, C * NBR * 4) : (int32_t *)ws(ctx, S_W7, C * NBR * 4);
    uint8_t *pl = payload ? (uint8_t *)st.out(payload, C * NBR * 2 * 268) : (uint8_t *)ws(ctx, S_W6, C * NBR * 2 * 268);
    double *tt = t0 ? (double *)st.out(t0, C * 8) : (double *)ws(ctx, S_W4, C * 8);
    uint8_t *scr = (uint8_t *)ws(ctx, S_W0, tab.size());
    uint8_t *bits = (uint8_t *)ws(ctx, S_W1, C * NBR * 510);
    uint8_t *ph = (uint8_t *)ws(ctx, S_W2, C * nsym);
    if (!x || !ci || !kd || !pl || !tt || !scr || !bits || !ph) return st.finish();
    HIP_TRY(ctx, hipMemcpyAsync(scr, tab.data(), tab.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ci, init.data(), C * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(tt, t0h.data(), C * 8, hipMemcpyHostToDevice, ctx->stream));
    const float amp = 0.5f;
    const float sigma = snr_db > -100.f && snr_db < 200.f
                            ? amp * sqrtf((float)(fs / 18000.0) / powf(10.f, snr_db / 10.f) / 2.f) : 0.f;
    hipLaunchKernelGGL(k_synth_bursts, dim3((unsigned)(C * NBR)), dim3(64), 0, ctx->stream, seed, NBR, scr,
                       scr + C * 432, ci, bits, kd, pl);
    hipLaunchKernelGGL(k_synth_phase, dim3((unsigned)C), dim3(64), 0, ctx->stream, bits, nsym, ph, seed);
    hipLaunchKernelGGL(k_synth_iq, dim3(grid_for(C * N, 256)), dim3(256), 0, ctx->stream, ph, nsym, (long)N, fs, seed,
                       amp, sigma, cfo_max, tt, x);
    return st.finish();
}

}  // extern "C"
