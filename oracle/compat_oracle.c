/*
 * compat_oracle.c -- CPU restatement of the reference's compat hot path (TEST INFRASTRUCTURE).
 *
 * ORACLE ONLY: linked by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker.  The product (tetraear-bladerf_amd/) never loads this library.
 *
 * Parity pinned against golden vectors recorded from the reference itself
 * (tests/golden/make_golden.py -> g1/g2/g3 fixtures).  Every loop below restates the exact
 * floating-point operation order of the third-party code the reference calls, so the
 * restatement is bit-exact with those vectors:
 *   - scipy 1.15.3 _sosfilt (Cython) used by sosfiltfilt <- scipy.signal.decimate
 *     (/root/reference/tetraear/signal/processor.py:254)
 *   - scipy 1.15.3 _linear_filter (lfilter, direct-form II transposed) used by filtfilt
 *     (/root/reference/tetraear/signal/processor.py:78-79)
 *   - TetraDecoder.find_sync greedy scan (/root/reference/tetraear/core/decoder.py:226-259)
 *   - TetraProtocolParser._calculate_crc16 (/root/reference/tetraear/core/protocol.py:331-347)
 * Build with -ffp-contract=off: the reference's compiled loops are not FMA-contracted.
 */
#include <stdint.h>
#include <string.h>

/* One real component through a cascade of biquads, in place.  sos rows are
 * [b0 b1 b2 a0 a1 a2] with a0 == 1 (scipy _sosfilt ignores a0). zi is [ns][2], updated. */
#define SOSFILT_BODY(T)                                                                  \
    for (long n = 0; n < len; ++n) {                                                     \
        T xc = x[n];                                                                     \
        for (int s = 0; s < ns; ++s) {                                                   \
            const T *c = sos + 6 * s;                                                    \
            T xn = c[0] * xc + zi[2 * s];                                                \
            zi[2 * s] = (c[1] * xc - c[4] * xn) + zi[2 * s + 1];                         \
            zi[2 * s + 1] = c[2] * xc - c[5] * xn;                                       \
            xc = xn;                                                                     \
        }                                                                                \
        x[n] = xc;                                                                       \
    }

void orc_sosfilt_f32(const float *sos, int ns, float *zi, float *x, long len) { SOSFILT_BODY(float) }
void orc_sosfilt_f64(const double *sos, int ns, double *zi, double *x, long len) { SOSFILT_BODY(double) }

/* The product's opt-in latency-mode decimator, tile passes (oracle/compat.py: _blocked_pass; not a
 * reference function): w[k+1] = the end state of tile k (B samples of c from zero state) as double,
 * k < Tn - 1; then every tile again from its start state w[k] cast to T, outputs to out. */
#define SOS_TILES_BODY(T, FILT)                                                          \
    long Tn = (L + B - 1) / B;                                                           \
    T tmp[4096];                                                                         \
    if (B > 4096 || ns > 4) return;                                                      \
    if (w) {                                                                             \
        for (long k = 0; k + 1 < Tn; ++k) {                                              \
            T z[8] = {0};                                                                \
            memcpy(tmp, c + k * B, sizeof(T) * B);                                       \
            FILT(sos, ns, z, tmp, B);                                                    \
            for (int i = 0; i < 2 * ns; ++i) w[(k + 1) * 2 * ns + i] = (double)z[i];     \
        }                                                                                \
    }                                                                                    \
    if (out) {                                                                           \
        for (long k = 0; k < Tn; ++k) {                                                  \
            long n = L - k * B < B ? L - k * B : B;                                      \
            T z[8];                                                                      \
            for (int i = 0; i < 2 * ns; ++i) z[i] = (T)st[k * 2 * ns + i];               \
            memcpy(tmp, c + k * B, sizeof(T) * n);                                       \
            FILT(sos, ns, z, tmp, n);                                                    \
            memcpy(out + k * B, tmp, sizeof(T) * n);                                     \
        }                                                                                \
    }

void orc_sos_tiles_f32(const float *sos, int ns, const float *c, long L, int B, double *w, const double *st,
                       float *out) { SOS_TILES_BODY(float, orc_sosfilt_f32) }
void orc_sos_tiles_f64(const double *sos, int ns, const double *c, long L, int B, double *w, const double *st,
                       double *out) { SOS_TILES_BODY(double, orc_sosfilt_f64) }

/* One real component through lfilter's DF-II-T loop (a[0] == 1), in place; zi has nt-1 entries. */
void orc_lfilter_f64(const double *b, const double *a, int nt, double *zi, double *x, long len)
{
    for (long n = 0; n < len; ++n) {
        double xn = x[n];
        double yn = zi[0] + b[0] * xn;
        for (int k = 0; k < nt - 2; ++k)
            zi[k] = (zi[k + 1] + xn * b[k + 1]) - yn * a[k + 1];
        zi[nt - 2] = xn * b[nt - 1] - yn * a[nt - 1];
        x[n] = yn;
    }
}

/* The latency mode's time-blocked filtfilt, tile passes (oracle/compat.py: _lf_blocked_pass), as
 * orc_sos_tiles_* with lfilter's nt - 1 states. */
void orc_lf_tiles_f64(const double *b, const double *a, int nt, const double *c, long L, int B, double *w,
                      const double *st, double *out)
{
    long Tn = (L + B - 1) / B;
    double tmp[4096];
    const int K = nt - 1;
    if (B > 4096 || K > 8) return;
    if (w)
        for (long k = 0; k + 1 < Tn; ++k) {
            double z[8] = {0};
            memcpy(tmp, c + k * B, sizeof(double) * B);
            orc_lfilter_f64(b, a, nt, z, tmp, B);
            for (int i = 0; i < K; ++i) w[(k + 1) * K + i] = z[i];
        }
    if (out)
        for (long k = 0; k < Tn; ++k) {
            long n = L - k * B < B ? L - k * B : B;
            double z[8];
            for (int i = 0; i < K; ++i) z[i] = st[k * K + i];
            memcpy(tmp, c + k * B, sizeof(double) * n);
            orc_lfilter_f64(b, a, nt, z, tmp, n);
            memcpy(out + k * B, tmp, sizeof(double) * n);
        }
}

static const uint8_t TS1[22] = {1,1,0,1,0,0,0,0,1,1,1,0,1,0,0,1,1,1,0,1,0,0};
static const uint8_t TS2[22] = {0,1,1,1,1,0,1,0,0,1,0,0,0,0,1,1,0,1,1,1,0,0};

/* Per-position match counts against TS1/TS2 (decoder.py:237-240). */
void orc_sync_counts(const uint8_t *bits, long nbits, uint8_t *c1, uint8_t *c2)
{
    long nw = nbits - 21;
    for (long i = 0; i < nw; ++i) {
        int m1 = 0, m2 = 0;
        for (int j = 0; j < 22; ++j) {
            m1 += bits[i + j] == TS1[j];
            m2 += bits[i + j] == TS2[j];
        }
        c1[i] = (uint8_t)m1;
        c2[i] = (uint8_t)m2;
    }
}

/* find_sync main loop (decoder.py:226-259) for an integer count threshold kthr
 * (kthr = least count with count/22 >= threshold).  Returns number of hits; *maxc gets the
 * max over EVALUATED correlations (TS2 is not evaluated at a TS1 hit, decoder.py:245-248). */
int orc_find_sync_greedy(const uint8_t *c1, const uint8_t *c2, long nw, int kthr, long *pos, int maxpos, int *maxc)
{
    int n = 0, mc = 0;
    long i = 0;
    while (i < nw) {
        int hit = 0;
        if (c1[i] > mc) mc = c1[i];
        if (c1[i] >= kthr) hit = 1;
        else {
            if (c2[i] > mc) mc = c2[i];
            if (c2[i] >= kthr) hit = 1;
        }
        if (hit) {
            if (n < maxpos) pos[n] = i;
            ++n;
            i += 250;
            continue;
        }
        ++i;
    }
    *maxc = mc;
    return n;
}

/* _calculate_crc16: poly 0x1021, init 0xFFFF, MSB-first, no final XOR (protocol.py:331-347). */
uint32_t orc_crc16(const uint8_t *bits, long n, int reversed)
{
    uint32_t crc = 0xFFFF;
    for (long i = 0; i < n; ++i) {
        uint32_t b = bits[reversed ? n - 1 - i : i] & 1u;
        crc ^= b << 15;
        crc = (crc & 0x8000u) ? ((crc << 1) ^ 0x1021u) : (crc << 1);
        crc &= 0xFFFFu;
    }
    return crc;
}

/* _check_crc (protocol.py:292-329): all-equal rejection, <=2-bit budget, reversed retry. */
int orc_check_crc(const uint8_t *bits, long n)
{
    if (n < 16) return 0;
    long ones = 0;
    for (long i = 0; i < n; ++i) ones += bits[i] & 1;
    if (ones == 0 || ones == n) return 0;
    uint32_t rx = 0;
    for (int k = 0; k < 16; ++k) rx = (rx << 1) | (bits[n - 16 + k] & 1u);
    uint32_t c = orc_crc16(bits, n - 16, 0);
    if (__builtin_popcount(c ^ rx) <= 2) return 1;
    c = orc_crc16(bits, n - 16, 1);
    if (__builtin_popcount(c ^ rx) <= 2) return 1;
    return 0;
}
