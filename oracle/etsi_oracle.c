/*
 * etsi_oracle.c -- CPU restatement of the ETSI EN 300 392-2 receive chain (TEST INFRASTRUCTURE).
 *
 * ORACLE ONLY (tests/, smoke(), bench.py cpu_baseline).  The reference has NO implementation of
 * these functions (no channeliser, Gardner, descrambler, deinterleaver or Viterbi
 * in /root/reference), so this chain is "parity unpinned" against the reference: it is pinned by
 * encoder -> decoder round trips, known-answer tests (CRC-16 check value 0xD64E, residue 0x1D0F)
 * and by being the specification the HIP kernels restate operation for operation.
 *
 * Spec sources (EN 300 392-2, restated from the standard, not from any code):
 *   §5.3   pi/4-DQPSK, Table 5.1 dibit -> phase step; RRC roll-off 0.35
 *   §8.2.3.2 CRC-16 G(x)=x^16+x^12+x^5+1, ones' complement, 4 zero tail bits
 *   §8.2.3.1 RCPC mother code rate 1/4, K=5: G1=1+D+D^4, G2=1+D^2+D^3+D^4, G3=1+D+D^2+D^4,
 *            G4=1+D+D^3+D^4; rate 2/3 puncturing t=3, P=(1,2,5)
 *   §8.2.4.1 block interleaving k = 1 + (a*i mod K)
 *   §8.2.5   scrambling LFSR c(x)=1+x+x^2+x^4+x^5+x^7+x^8+x^10+x^11+x^12+x^16+x^22+x^23+x^26+x^32,
 *            init = (MCC<<20 | MNC<<6 | CC) << 2 | 3; BSCH uses colour code 0 (init = 3)
 *   §9.4.4   normal / synchronisation continuous downlink bursts (510 bits)
 *
 * The DSP part (channel filter, timing recovery, differential decision) is this build's own
 * receiver design; the functions below define it, and the GPU kernels reproduce the same float
 * operations (explicit fmaf, emulated 64-lane wave reductions), compiled with -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* ------------------------------------------------------------------------- coding tables */

/* kind: 0 SCH/F, 1 SCH/HD (also BNCH/STCH), 2 BSCH */
static const int KIND_K[3] = {432, 216, 120};
static const int KIND_A[3] = {103, 101, 11};
static const int KIND_N2[3] = {288, 144, 80};   /* type-2 bits = type-1 + 16 CRC + 4 tail */
static const int KIND_N1[3] = {268, 124, 60};

int eo_kind_params(int kind, int *K, int *a, int *n2, int *n1)
{
    if (kind < 0 || kind > 2) return -1;
    *K = KIND_K[kind]; *a = KIND_A[kind]; *n2 = KIND_N2[kind]; *n1 = KIND_N1[kind];
    return 0;
}

/* §8.2.5 scrambling sequence: Fibonacci LFSR, taps at the exponents of c(x). */
void eo_scramble_seq(uint32_t init, int n, uint8_t *out)
{
    uint32_t r = init;
    for (int i = 0; i < n; ++i) {
        uint32_t b = ((r >> 0) ^ (r >> 6) ^ (r >> 9) ^ (r >> 10) ^ (r >> 16) ^ (r >> 20) ^ (r >> 21) ^
                      (r >> 22) ^ (r >> 24) ^ (r >> 25) ^ (r >> 27) ^ (r >> 28) ^ (r >> 30) ^ (r >> 31)) & 1u;
        r = (r >> 1) | (b << 31);
        out[i] = (uint8_t)b;
    }
}

uint32_t eo_scramble_init(uint32_t mcc, uint32_t mnc, uint32_t cc)
{
    return ((((mcc & 0x3FFu) << 20) | ((mnc & 0x3FFFu) << 6) | (cc & 0x3Fu)) << 2) | 3u;
}

/* CRC-16/CCITT-FALSE register over bits (init 0xFFFF, MSB first, no final xor). */
uint32_t eo_crc16_reg(const uint8_t *bits, int n)
{
    uint32_t c = 0xFFFF;
    for (int i = 0; i < n; ++i) {
        c ^= (uint32_t)(bits[i] & 1u) << 15;
        c = (c & 0x8000u) ? ((c << 1) ^ 0x1021u) : (c << 1);
        c &= 0xFFFFu;
    }
    return c;
}

/* §8.2.3.1 mother encoder over n2 type-2 bits -> 4*n2 mother bits (zero initial state). */
void eo_conv_encode(const uint8_t *in, int n2, uint8_t *mother)
{
    uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
    for (int i = 0; i < n2; ++i) {
        uint32_t b = in[i] & 1u;
        mother[4 * i + 0] = (uint8_t)(b ^ d0 ^ d3);
        mother[4 * i + 1] = (uint8_t)(b ^ d1 ^ d2 ^ d3);
        mother[4 * i + 2] = (uint8_t)(b ^ d0 ^ d1 ^ d3);
        mother[4 * i + 3] = (uint8_t)(b ^ d0 ^ d2 ^ d3);
        d3 = d2; d2 = d1; d1 = d0; d0 = b;
    }
}

/* rate-2/3 puncturing: type-3 bit j (1-based) = mother bit k, k = 8*floor((j-1)/3) + P[j-3*floor((j-1)/3)] */
static int punct_index(int j1)
{
    static const int P[4] = {0, 1, 2, 5};
    int g = (j1 - 1) / 3;
    return 8 * g + P[j1 - 3 * g];   /* 1-based mother index */
}

/* Full encoder type-1 -> type-5 (kind; scr = K scrambling bits). */
void eo_encode_block(const uint8_t *type1, int kind, const uint8_t *scr, uint8_t *type5)
{
    int K, a, n2, n1;
    eo_kind_params(kind, &K, &a, &n2, &n1);
    uint8_t t2[288], mother[4 * 288], t3[432];
    memcpy(t2, type1, (size_t)n1);
    uint32_t c = eo_crc16_reg(type1, n1) ^ 0xFFFFu;   /* ones' complement */
    for (int k = 0; k < 16; ++k) t2[n1 + k] = (uint8_t)((c >> (15 - k)) & 1u);
    for (int k = 0; k < 4; ++k) t2[n1 + 16 + k] = 0;
    eo_conv_encode(t2, n2, mother);
    for (int j = 1; j <= K; ++j) t3[j - 1] = mother[punct_index(j) - 1];
    for (int i = 1; i <= K; ++i) {
        int k = 1 + (int)(((long)a * i) % K);
        type5[k - 1] = (uint8_t)(t3[i - 1] ^ scr[k - 1]);
    }
}

/* Viterbi over n2 steps of 4 mother soft values (int8, >0 means bit 0, 0 = erased).
 * Path metric = correlation; ties keep the predecessor with d3 = 0.  Ends in state 0. */
void eo_viterbi(const int8_t *ms, int n2, uint8_t *out)
{
    int32_t pm[16], nm[16];
    static uint8_t surv[288][16];
    for (int s = 0; s < 16; ++s) pm[s] = s == 0 ? 0 : -(1 << 28);
    for (int t = 0; t < n2; ++t) {
        const int8_t *m = ms + 4 * t;
        for (int n = 0; n < 16; ++n) {
            int b = n & 1, d0 = (n >> 1) & 1, d1 = (n >> 2) & 1, d2 = (n >> 3) & 1;
            int best = 0;
            int32_t bm[2];
            for (int d3 = 0; d3 < 2; ++d3) {
                int g1 = b ^ d0 ^ d3, g2 = b ^ d1 ^ d2 ^ d3, g3 = b ^ d0 ^ d1 ^ d3, g4 = b ^ d0 ^ d2 ^ d3;
                int32_t v = (g1 ? -m[0] : m[0]) + (g2 ? -m[1] : m[1]) + (g3 ? -m[2] : m[2]) + (g4 ? -m[3] : m[3]);
                int p = (n >> 1) | (d3 << 3);
                bm[d3] = pm[p] + v;
            }
            if (bm[1] > bm[0]) best = 1;
            nm[n] = bm[best];
            surv[t][n] = (uint8_t)best;
        }
        memcpy(pm, nm, sizeof pm);
    }
    int s = 0;
    for (int t = n2 - 1; t >= 0; --t) {
        out[t] = (uint8_t)(s & 1);
        s = (s >> 1) | (surv[t][s] << 3);
    }
}

/* Decode one block: type-5 soft (int8, K values) -> type-1 bits; returns crc_ok. */
int eo_decode_block(const int8_t *soft5, int kind, const uint8_t *scr, uint8_t *type1)
{
    int K, a, n2, n1;
    eo_kind_params(kind, &K, &a, &n2, &n1);
    int8_t t3[432], ms[4 * 288];
    /* descramble + deinterleave: type-3[i] = type-4[k(i)], type-4 = type-5 with sign flips */
    for (int i = 1; i <= K; ++i) {
        int k = 1 + (int)(((long)a * i) % K);
        int8_t v = soft5[k - 1];
        t3[i - 1] = scr[k - 1] ? (int8_t)(-v) : v;
    }
    memset(ms, 0, sizeof(int8_t) * 4 * (size_t)n2);
    for (int j = 1; j <= K; ++j) ms[punct_index(j) - 1] = t3[j - 1];
    uint8_t t2[288];
    eo_viterbi(ms, n2, t2);
    memcpy(type1, t2, (size_t)n1);
    return eo_crc16_reg(t2, n1 + 16) == 0x1D0Fu;
}

/* ------------------------------------------------------------------------- receiver DSP */

/* Stage 1: decimating FIR, x240[k] = sum_j h1[j] * x[q1*k + j] (fmaf chain, j ascending).
 * Stage 2: polyphase RRC resampler up 3 / down 10: y72[m] = sum_k x240[k] hp[n - 3k],
 *          n = Lp-1 + 10m, k ascending.  Returns M2. */
int eo_chanfilt(const float *x, int N, const float *h1, int L1, int q1, const float *hp, int Lp, int up, int down,
                float *x240, float *y)
{
    int M1 = (N - L1) / q1 + 1;
    if (M1 <= 0) return 0;
    for (int k = 0; k < M1; ++k) {
        float ar = 0.f, ai = 0.f;
        const float *xp = x + 2 * (long)q1 * k;
        for (int j = 0; j < L1; ++j) {
            ar = fmaf(h1[j], xp[2 * j], ar);
            ai = fmaf(h1[j], xp[2 * j + 1], ai);
        }
        x240[2 * k] = ar;
        x240[2 * k + 1] = ai;
    }
    int n0 = Lp - 1;
    int M2 = (up * M1 - 1 - n0) / down + 1;
    if (M2 <= 0) return 0;
    for (int m = 0; m < M2; ++m) {
        int n = n0 + down * m;
        int kmin = (n - Lp + 1 + up - 1) / up, kmax = n / up;
        float ar = 0.f, ai = 0.f;
        for (int k = kmin; k <= kmax; ++k) {
            float h = hp[n - up * k];
            ar = fmaf(h, x240[2 * k], ar);
            ai = fmaf(h, x240[2 * k + 1], ai);
        }
        y[2 * m] = ar;
        y[2 * m + 1] = ai;
    }
    return M2;
}

/* 64-lane xor-butterfly sum, as the wave computes it (every lane ends with the same value). */
static float wave_sum(float *v)
{
    float t[64];
    for (int off = 32; off >= 1; off >>= 1) {
        for (int l = 0; l < 64; ++l) t[l] = v[l] + v[l ^ off];
        memcpy(v, t, sizeof t);
    }
    return v[0];
}

static const float K6 = 1.0f / 6.0f;

/* atan2 from IEEE basic operations only (max error ~1e-5 rad), so the timing phase is computed
 * bit-identically by this oracle and by the HIP kernel (libm atan2 implementations differ). */
static float pat2(float y, float x)
{
    float ax = fabsf(x), ay = fabsf(y);
    float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    float a = mx == 0.0f ? 0.0f : mn / mx;
    float s = a * a;
    float r = fmaf(fmaf(fmaf(fmaf(fmaf(-0.0117212f, s, 0.05265332f), s, -0.11643287f), s, 0.19354346f), s,
                        -0.33262347f), s, 0.99997726f) * a;
    if (ay > ax) r = 1.57079637f - r;
    if (x < 0.0f) r = 3.14159274f - r;
    if (y < 0.0f) r = -r;
    return r;
}

static void interp(const float *y, float t, float *o)
{
    float fi = floorf(t);
    int i = (int)fi;
    float f = t - fi;
    float fm1 = f - 1.0f, fm2 = f - 2.0f, fp1 = f + 1.0f;
    float cm = -(f * fm1 * fm2) * K6;
    float c0 = (fp1 * fm1 * fm2) * 0.5f;
    float c1 = -(fp1 * f * fm2) * 0.5f;
    float c2 = (fp1 * f * fm1) * K6;
    for (int c = 0; c < 2; ++c) {
        float acc = cm * y[2 * (i - 1) + c];
        acc = fmaf(c0, y[2 * i + c], acc);
        acc = fmaf(c1, y[2 * (i + 1) + c], acc);
        acc = fmaf(c2, y[2 * (i + 2) + c], acc);
        o[c] = acc;
    }
}

static void csqrt_p(float x, float y, float *a, float *b)
{
    float r = sqrtf(fmaf(x, x, y * y));
    if (r == 0.0f) { *a = 0.0f; *b = 0.0f; return; }
    if (x >= 0.0f) {
        float s = sqrtf((r + x) * 0.5f);
        *a = s;
        *b = y / (2.0f * s);
    } else {
        float s = sqrtf((r - x) * 0.5f);
        if (y < 0.0f) s = -s;
        *b = s;
        *a = y / (2.0f * s);
    }
}

/* Timing recovery + differential decision over y (4 samples/symbol, M2 samples).
 *   Oerder-Meyr feed-forward timing phase, then block Gardner tracking (64 symbols per block).
 *   soft_sym [smax] cf32 symbol-spaced samples; softbits [2*smax] int8; hard [smax] dibit symbols.
 *   diag[0..3] = base, final delta, cfo rotation angle proxy (rot re, rot im).
 *   Returns S = number of soft symbols (dibits = S-1). */
/* Oerder-Meyr class sums A[c] = sum of |y[n]|^2 over n = c mod 4 of one chunk, in the fused
 * demod's order: lane l accumulates n = l, l+64, ... (class n mod 4 = l mod 4), as four partial
 * sums over quarters of the 64-sample blocks (part w: blocks [w q4, (w+1) q4), q4 = ceil(nb / 4))
 * added in order -- the GPU computes the parts on four waves at once -- then a butterfly over
 * xor 32, 16, 8, 4 (lane c holds class c). */
void eo_om_quarters(const float *y, int M2, float A[4])
{
    float acc[64];
    const int nb = (M2 + 63) / 64, q4 = (nb + 3) / 4;
    for (int l = 0; l < 64; ++l) {
        float s = 0.f;
        for (int w = 0; w < 4; ++w) {
            float pw = 0.f;
            int b1 = (w + 1) * q4 < nb ? (w + 1) * q4 : nb;
            for (int b = w * q4; b < b1; ++b) {
                int n = 64 * b + l;
                if (n < M2) pw += fmaf(y[2 * n], y[2 * n], y[2 * n + 1] * y[2 * n + 1]);
            }
            s = w == 0 ? pw : s + pw;
        }
        acc[l] = s;
    }
    float t[64];
    for (int off = 32; off >= 4; off >>= 1) {
        for (int l = 0; l < 64; ++l) t[l] = acc[l] + acc[l ^ off];
        memcpy(acc, t, sizeof t);
    }
    for (int c = 0; c < 4; ++c) A[c] = acc[c];
}

/* The same class sums in the wideband chain's grouped order (the resampler forms them while it
 * writes y; csrc/wideband.hip k_pfb_resamp_fix OM, etsi_rx.hip k_timing OMG).  The chunk is
 * row[s, s + M2) of a carrier's 72 kHz row, s and M2 multiples of 4 and U (the resampler's output
 * group) a multiple of 4, so class c is n mod 4 in row positions too.
 *   group partials P[g][c] = sum over o = c mod 4 in [0, U), ascending, of |row[U g + o]|^2;
 *   G[c]: lane l (0..63) sums P[g][c] over the chunk's whole groups g = g0 + l, g0 + l + 64, ...
 *         ascending (g0 = ceil(s / U), g1 = floor((s + M2) / U)), then the xor 32..1 butterfly;
 *   head / tail: the samples before U g0 / from U g1 on, class by class in ascending n;
 *   A[c] = (head[c] + G[c]) + tail[c]. */
void eo_om_group_partials(const float *row, long n, int U, float *P)
{
    for (long g = 0; g * U < n; ++g)
        for (int c = 0; c < 4; ++c) {
            float p = 0.f;
            for (int o = c; o < U; o += 4) {
                long i = g * U + o;
                if (i < n) p += fmaf(row[2 * i], row[2 * i], row[2 * i + 1] * row[2 * i + 1]);
            }
            P[4 * g + c] = p;
        }
}

void eo_om_grouped(const float *row, long s, int M2, int U, const float *P, float A[4])
{
    const long g0 = (s + U - 1) / U, g1 = (s + M2) / U;
    float v[4][64];
    for (int c = 0; c < 4; ++c)
        for (int l = 0; l < 64; ++l) {
            float a = 0.f;
            for (long g = g0 + l; g < g1; g += 64) a = a + P[4 * g + c];
            v[c][l] = a;
        }
    const long hend = U * g0 < s + M2 ? U * g0 : s + M2, tbeg = U * g1 > hend ? U * g1 : hend;
    for (int c = 0; c < 4; ++c) {
        float h = 0.f, t = 0.f;
        for (long i = s + c; i < hend; i += 4)
            h = h + fmaf(row[2 * i], row[2 * i], row[2 * i + 1] * row[2 * i + 1]);
        for (long i = tbeg + c; i < s + M2; i += 4)
            t = t + fmaf(row[2 * i], row[2 * i], row[2 * i + 1] * row[2 * i + 1]);
        A[c] = (h + wave_sum(v[c])) + t;
    }
}

/* Streaming state of one channel across consecutive chunks (include/tetra_hip.h tetra_etsi_track):
 * base = the next symbol's Gardner base position in y samples relative to the END of the previous
 * chunk's outputs, delta = the loop offset, (pr, pi) = the last symbol, acquired = 0 until the
 * Oerder-Meyr acquisition has run. */
typedef struct {
    float base, delta, pr, pi;
    int32_t acquired, reserved[3];
} eo_track;

/* The timing stage on one window of y (4 samples/symbol, M2 samples).
 *   trk == NULL or !trk->acquired: Oerder-Meyr feed-forward phase over the window, delta = 0, the
 *     first symbol starts a new differential chain (the non-streaming receiver);
 *   trk->acquired: the loop continues: base = trk->base + yoff (yoff = window index of the first
 *     output the previous chunk did not have), delta carried, symbol 0 of the output is the carried
 *     last symbol, so dibit 0 spans the chunk seam.
 * Then block-Gardner tracking (64 symbols per block) and the per-chunk CFO / soft scale.  soft_sym
 * [smax] cf32 symbol-spaced samples; softbits [2*smax] int8; hard [smax] dibits; diag[0..3] = base,
 * final delta, rotation (re, im).  Returns S = symbols in the output (dibits = S-1); trk (if given)
 * is updated for the next chunk. */
static int timing_core(const float *y, int M2, const float *om, int yoff, eo_track *trk, float gain, float soft_scale,
                       float *soft_sym, float *dscr, int8_t *softbits, uint8_t *hard, int smax, float *diag)
{
    const int acq = trk && trk->acquired;
    if (M2 < 16) {
        if (acq) trk->base = trk->base + (float)(yoff - M2);
        return 0;
    }
    float base, delta;
    int kstart, J0;
    if (acq) {
        base = trk->base + (float)yoff;
        delta = trk->delta;
        kstart = 0;
        J0 = 1;
    } else {
        float acc[4];
        if (om)
            memcpy(acc, om, sizeof acc);
        else
            eo_om_quarters(y, M2, acc);
        float Xr = acc[0] - acc[2], Xi = acc[3] - acc[1];
        float p = -0.63661977236758134f * pat2(Xi, Xr);   /* -(2/pi) arg X */
        base = p < 0.0f ? p + 4.0f : p;
        if (base >= 4.0f) base -= 4.0f;
        kstart = base >= 3.0f ? 0 : 1;
        delta = 0.0f;
        J0 = 0;
    }
    int S = J0;
    float prev_r = acq ? trk->pr : 0.f, prev_i = acq ? trk->pi : 0.f;
    int have_prev = J0;
    if (J0 && smax > 0) { soft_sym[0] = prev_r; soft_sym[1] = prev_i; }
    for (int kb = kstart;; kb += 64) {
        float off = base + delta;
        float on[64][2], mid[64][2], ev[64], pv[64];
        int valid[64];
        for (int l = 0; l < 64; ++l) {
            float t = (float)(4 * (kb + l)) + off;
            valid[l] = (t - 3.0f >= 0.0f) && (t + 2.0f <= (float)(M2 - 1)) && (S + l < smax);
        }
        int nv = 0;
        while (nv < 64 && valid[nv]) ++nv;
        for (int l = 0; l < 64; ++l) {
            ev[l] = 0.f;
            pv[l] = 0.f;
            if (l >= nv) continue;
            float t = (float)(4 * (kb + l)) + off;
            interp(y, t, on[l]);
            interp(y, t - 2.0f, mid[l]);
        }
        for (int l = 0; l < nv; ++l) {
            float br, bi;
            int hp_;
            if (l == 0) { br = prev_r; bi = prev_i; hp_ = have_prev; }
            else { br = on[l - 1][0]; bi = on[l - 1][1]; hp_ = 1; }
            float ar = on[l][0], ai = on[l][1];
            pv[l] = fmaf(ar, ar, ai * ai);
            if (hp_) {
                float dr = ar - br, di = ai - bi;
                ev[l] = fmaf(dr, mid[l][0], di * mid[l][1]);
                int j = S + l;   /* symbol index; d index j-1 */
                dscr[2 * (j - 1)] = fmaf(ar, br, ai * bi);
                dscr[2 * (j - 1) + 1] = fmaf(ai, br, -(ar * bi));
            }
            soft_sym[2 * (S + l)] = ar;
            soft_sym[2 * (S + l) + 1] = ai;
        }
        if (nv > 0) {
            float E = wave_sum(ev), W = wave_sum(pv);
            if (W > 0.0f) delta = delta - gain * (E / W);
            if (delta > 1.5f) delta = 1.5f;
            if (delta < -1.5f) delta = -1.5f;
            prev_r = on[nv - 1][0];
            prev_i = on[nv - 1][1];
            have_prev = 1;
        }
        S += nv;
        if (nv < 64) break;
    }
    /* CFO: Z = sum d^4; rot = conj((-Z/|Z|)^(1/4)); scale from mean |d| */
    float zr[64], zi[64], am[64];
    for (int l = 0; l < 64; ++l) { zr[l] = 0.f; zi[l] = 0.f; am[l] = 0.f; }
    for (int j = 1; j < S; ++j) {
        int l = (j - J0) & 63;   /* the tracking lane of d_j: symbols J0 + 64 b + l */
        float dr = dscr[2 * (j - 1)], di = dscr[2 * (j - 1) + 1];
        float sr = fmaf(dr, dr, -(di * di)), si = (dr * di) * 2.0f;
        float qr = fmaf(sr, sr, -(si * si)), qi = (sr * si) * 2.0f;
        zr[l] += qr;
        zi[l] += qi;
        am[l] += sqrtf(fmaf(dr, dr, di * di));
    }
    float Zr = wave_sum(zr), Zi = wave_sum(zi), A = wave_sum(am);
    float rr = 1.0f, ri = 0.0f;
    float zm = sqrtf(fmaf(Zr, Zr, Zi * Zi));
    if (zm > 0.0f) {
        float ur = -Zr / zm, ui = -Zi / zm, vr, vi, wr, wi;
        csqrt_p(ur, ui, &vr, &vi);
        csqrt_p(vr, vi, &wr, &wi);
        rr = wr;
        ri = -wi;
    }
    float sc = 0.0f;
    if (S > 1 && A > 0.0f) sc = soft_scale / (A / (float)(S - 1));
    for (int j = 1; j < S; ++j) {
        float dr = dscr[2 * (j - 1)], di = dscr[2 * (j - 1) + 1];
        float xr = fmaf(dr, rr, -(di * ri)), xi = fmaf(dr, ri, di * rr);
        float q1 = rintf(xi * sc), q2 = rintf(xr * sc);
        q1 = q1 > 127.f ? 127.f : (q1 < -127.f ? -127.f : q1);
        q2 = q2 > 127.f ? 127.f : (q2 < -127.f ? -127.f : q2);
        softbits[2 * (j - 1)] = (int8_t)q1;
        softbits[2 * (j - 1) + 1] = (int8_t)q2;
        hard[j - 1] = (uint8_t)(((xi < 0.0f) << 1) | (xr < 0.0f));
    }
    if (diag) { diag[0] = base; diag[1] = delta; diag[2] = rr; diag[3] = ri; }
    if (trk) {
        const int Snew = S - J0;
        if (acq || S > 0) {
            trk->base = base + (float)(4 * (kstart + Snew) - M2);
            trk->delta = delta;
            trk->pr = prev_r;
            trk->pi = prev_i;
            trk->acquired = 1;
        }
    }
    return S;
}

/* eo_timing with the Oerder-Meyr class sums given (om != NULL) or computed in the quarter order. */
int eo_timing_om(const float *y, int M2, const float *om, float gain, float soft_scale, float *soft_sym, float *dscr,
                 int8_t *softbits, uint8_t *hard, int smax, float *diag)
{
    return timing_core(y, M2, om, 0, NULL, gain, soft_scale, soft_sym, dscr, softbits, hard, smax, diag);
}

/* The streaming form (tetra_demod_etsi_stream's timing): trk carried from chunk to chunk. */
int eo_timing_stream(const float *y, int M2, int yoff, eo_track *trk, float gain, float soft_scale, float *soft_sym,
                     float *dscr, int8_t *softbits, uint8_t *hard, int smax, float *diag)
{
    return timing_core(y, M2, NULL, yoff, trk, gain, soft_scale, soft_sym, dscr, softbits, hard, smax, diag);
}

int eo_timing(const float *y, int M2, float gain, float soft_scale, float *soft_sym, float *dscr, int8_t *softbits,
              uint8_t *hard, int smax, float *diag)
{
    return eo_timing_om(y, M2, NULL, gain, soft_scale, soft_sym, dscr, softbits, hard, smax, diag);
}

/* ------------------------------------------------------------------------- burst sync */
static const uint8_t Q_BITS[22] = {1,0,1,1,0,1,1,1,0,0,0,0,0,1,1,0,1,0,1,1,0,1};
static const uint8_t N_BITS[22] = {1,1,0,1,0,0,0,0,1,1,1,0,1,0,0,1,1,1,0,1,0,0};
static const uint8_t P_BITS[22] = {0,1,1,1,1,0,1,0,0,1,0,0,0,0,1,1,0,1,1,1,0,0};
static const uint8_t Y_BITS[38] = {1,1,0,0,0,0,0,1,1,0,0,1,1,1,0,0,1,1,1,0,1,0,0,1,1,1,0,0,0,0,0,1,1,0,0,1,1,1};

static int match_at(const uint8_t *bits, int pos, const uint8_t *pat, int n)
{
    int m = 0;
    for (int j = 0; j < n; ++j) m += bits[pos + j] == pat[j];
    return m;
}

/* Burst detection over hard bits: kinds 0 NDB(n) -> SCH/F, 1 NDB(p) -> 2xSCH/HD, 2 SB -> BSCH+SCH/HD.
 * Score = head q11..q22 @0 + training @244 (n/p) or @214 (y) + tail q1..q10 @500.
 * Greedy scan: first start with NDB >= 40/44 or SB >= 54/60, then skip 500 bits. */
int eo_sync_from(const uint8_t *bits, int nbits, int start, int *starts, int *kinds, int maxb, int *stop)
{
    int nb = 0;
    int s = start;
    for (; s + 510 <= nbits && nb < maxb;) {
        int ht = match_at(bits, s, Q_BITS + 10, 12) + match_at(bits, s + 500, Q_BITS, 10);
        int mn = ht + match_at(bits, s + 244, N_BITS, 22);
        int mp = ht + match_at(bits, s + 244, P_BITS, 22);
        int my = ht + match_at(bits, s + 214, Y_BITS, 38);
        int kind = -1;
        if (my >= 54) kind = 2;
        else if (mn >= 40 && mn >= mp) kind = 0;
        else if (mp >= 40) kind = 1;
        if (kind >= 0) {
            starts[nb] = s;
            kinds[nb] = kind;
            ++nb;
            s += 500;
        } else {
            ++s;
        }
    }
    if (stop) *stop = s;   /* the first position not examined: the streaming tail starts here */
    return nb;
}

int eo_sync(const uint8_t *bits, int nbits, int *starts, int *kinds, int maxb)
{
    return eo_sync_from(bits, nbits, 0, starts, kinds, maxb, NULL);
}

/* Differential decision on given symbol-spaced samples (interleaved re/im, n samples): hard[n-1]
 * dibits per EN 300 392-2 Table 5.1, d = x[k] conj(x[k-1]), (Im d < 0, Re d < 0) -- the decision of
 * eo_timing without its CFO rotation. */
void eo_decide(const float *x, int n, uint8_t *hard)
{
    for (int k = 1; k < n; ++k) {
        float ar = x[2 * k], ai = x[2 * k + 1], br = x[2 * k - 2], bi = x[2 * k - 1];
        float dr = fmaf(ar, br, ai * bi), di = fmaf(ai, br, -(ar * bi));
        hard[k - 1] = (uint8_t)(((di < 0.0f) << 1) | (dr < 0.0f));
    }
}
