// scanner.hip -- the scanner's TETRA signal detector over a batch of candidate channels
// (/root/reference/tetraear/signal/scanner.py:42-147, 204-231, as that survey row
// describes it).  One workgroup per channel computes, in one pass over the channel's samples:
//   * the pi/4-DQPSK cluster test: of the wrapped phase differences of consecutive samples, how many
//     lie within pi/8 of one of {-pi, -3pi/4, .., 3pi/4} (the modulation confidence's numerator);
//   * the 31-bit sync search: samples strided by D = max(1, int(fs / 18000 / 10)), one bit per wrapped
//     phase difference (1 when it quantises to 0, |d| <= pi/8 in units of pi/4), the best match count
//     of the 31-bit sync pattern over every window start 0 .. nbits - 32;
//   * the mean power |x|^2 of the chunk and of its five equal windows (power stability).
// The host turns these counts into the detector's decisions (tetraear/signal/scanner.py).
//
// The cluster test runs on the chunk normalised by its peak magnitude, as scanner.py:71 does before
// its angles: d = max|x| + 1e-10 in the dtype (|x| as numpy's abs: float32 hypot through double,
// float64 hypot), then numpy's complex-by-real division (its Smith form with a zero imaginary
// divisor: ((re + im*0) * (1/d), (im - re*0) * (1/d))).  The sync bits use the raw samples, as
// scanner.py:110-117 does.  Rows of any length: the sync bits are held in LDS SC_MAXBITS at a time,
// consecutive passes overlapping by 64 bits so every 31-bit window lies wholly inside one pass.
//
// Phase arithmetic follows numpy's on the input dtype: complex64 -> float32 angles, differences and
// wrap ((d + pi) mod 2 pi - pi, Python-style remainder), the cluster distance test in float64 against
// the float64 multiples of pi/4; complex128 -> float64 throughout.  atan2 is the device's (the host's
// libm rounds its last ulp differently), so a difference within ~1e-6 rad of a decision edge may
// land on the other side -- the edges are the pi/8 boundaries and the wrap point +-pi, which clipped
// captures (samples pinned to the diagonals) hit often; the parity tests count them (tests/test_scanner.py).
#include "common.h"

namespace {

constexpr int SC_T = 256;               // threads per workgroup (one channel)
constexpr int SC_TILE = 4 * SC_T;       // samples per angle tile
constexpr int SC_MAXBITS = 131072;      // sync bits held in LDS (packed)

template <typename T> struct Cx;
template <> struct Cx<float2> {
    using R = float;
    static __device__ R ang(float2 v) { return atan2f(v.y, v.x); }
    static __device__ double pw(float2 v) { return (double)v.x * v.x + (double)v.y * v.y; }
    // numpy's |z| for complex64: hypotf, which glibc evaluates as sqrt in double rounded once to float
    static __device__ R mag(float2 v) { return (float)sqrt((double)v.x * v.x + (double)v.y * v.y); }
};
template <> struct Cx<double2> {
    using R = double;
    static __device__ R ang(double2 v) { return atan2(v.y, v.x); }
    static __device__ double pw(double2 v) { return v.x * v.x + v.y * v.y; }
    static __device__ R mag(double2 v) { return hypot(v.x, v.y); }
};
// angle of z / d (scanner.py:71) with numpy's complex division by (d + 0j): rat = 0 / d, scl = 1 / (d + 0 * rat)
template <typename T, typename R> __device__ inline R ang_scaled(T v, R rat, R scl) {
    T u;
    u.x = (v.x + v.y * rat) * scl;
    u.y = (v.y - v.x * rat) * scl;
    return Cx<T>::ang(u);
}

// numpy's float remainder (Python semantics: the result takes the divisor's sign)
template <typename R> __device__ inline R pymod(R a, R b) {
    R m = fmod(a, b);
    if (m != 0) {
        if ((b < 0) != (m < 0)) m += b;
    } else {
        m = copysign((R)0, b);
    }
    return m;
}
// (d + pi) % (2 pi) - pi with pi and 2 pi rounded to the dtype, as numpy evaluates it
template <typename R> __device__ inline R wrap(R d) {
    const R pi = (R)3.141592653589793, tpi = (R)(2.0 * 3.141592653589793);
    return pymod<R>(d + pi, tpi) - pi;
}
// distance test against the float64 multiples of pi/4 (-pi .. 3pi/4; +pi is not among them)
__device__ inline bool near_multiple(double d) {
    const double pi = 3.141592653589793;
    const double e[8] = {-pi, -3 * pi / 4, -pi / 2, -pi / 4, 0.0, pi / 4, pi / 2, 3 * pi / 4};
    double best = fabs(e[0] - d);
#pragma unroll
    for (int k = 1; k < 8; ++k) best = fmin(best, fabs(e[k] - d));
    return best < pi / 8;
}
// sync bit: round(d / (pi/4)) == 0 (round half to even) <=> |d / (pi/4)| <= 1/2 in the dtype
template <typename R> __device__ inline int sync_bit(R d) {
    const R q = d / (R)(3.141592653589793 / 4);
    return fabs(q) <= (R)0.5 ? 1 : 0;
}

__device__ inline double block_sum(double v, double *red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < SC_T / 64; ++w) s += red[w];
    return s;
}

template <typename T>
__global__ __launch_bounds__(SC_T) void k_scan_detect(const T *__restrict__ x, long N, int D, uint32_t pattern, int C,
                                                      double *__restrict__ stats) {
    using R = typename Cx<T>::R;
    __shared__ R ang[SC_TILE + 1];
    __shared__ uint32_t bits[SC_MAXBITS / 32 + 2];
    __shared__ double red[SC_T / 64];
    __shared__ int redi[SC_T / 64];
    __shared__ R redm[SC_T / 64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const long ws = N / 5;   // stability windows [i ws, (i + 1) ws), i < 5
    for (int ch = blockIdx.x; ch < C; ch += gridDim.x) {
        const T *row = x + (size_t)ch * N;
        // --- peak magnitude of the chunk (scanner.py:71's normaliser)
        R mx = 0;
        for (long n = tid; n < N; n += SC_T) mx = fmax(mx, Cx<T>::mag(row[n]));
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
        if (lane == 0) redm[wv] = mx;
        __syncthreads();
        for (int w = 0; w < SC_T / 64; ++w) mx = fmax(mx, redm[w]);
        const R dnm = mx + (R)1e-10;
        const R rat = (R)0 / dnm, scl = (R)1 / (dnm + (R)0 * rat);
        // --- modulation cluster test + power, tile by tile
        double p_all = 0.0, p_w[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        int matches = 0;
        for (long t0 = 0; t0 < N; t0 += SC_TILE) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long n = t0 + tid + SC_T * r;
                if (n < N) {
                    const T v = row[n];
                    ang[1 + tid + SC_T * r] = ang_scaled<T, R>(v, rat, scl);
                    const double p = Cx<T>::pw(v);
                    p_all += p;
                    const long w = ws > 0 ? n / ws : 5;
                    if (w < 5) p_w[w] += p;
                }
            }
            if (tid == 0) ang[0] = t0 > 0 ? ang_scaled<T, R>(row[t0 - 1], rat, scl) : (R)0;
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long n = t0 + tid + SC_T * r;
                if (n >= 1 && n < N) {
                    const R d = wrap<R>(ang[1 + tid + SC_T * r] - ang[tid + SC_T * r]);
                    matches += near_multiple((double)d) ? 1 : 0;
                }
            }
            __syncthreads();
        }
        // --- sync bits of the strided samples, packed by ballots (bit k = lane k & 63 of a 64-chunk),
        //     SC_MAXBITS per pass; pass p holds bits [p0, p0 + nb) and scores the windows that start in
        //     it and end inside it; the next pass starts 64 bits before this one's end
        const long K = (N + D - 1) / D;             // strided samples
        const long nbits = K > 0 ? K - 1 : 0;
        const long npos = nbits > 31 ? nbits - 31 : 0;   // scanner.py's range(len(bits) - 31)
        int best = 0;
        for (long p0 = 0; p0 == 0 || p0 + 31 < nbits; p0 += SC_MAXBITS - 64) {
            const long nb = nbits - p0 < SC_MAXBITS ? nbits - p0 : SC_MAXBITS;
            __syncthreads();   // the previous pass's window reads are done
            for (long k0 = 64L * wv; k0 < nb; k0 += 64L * (SC_T / 64)) {
                const long k = k0 + lane;
                int b = 0;
                if (k < nb) {
                    const long g = p0 + k;
                    const R a0 = Cx<T>::ang(row[g * D]), a1 = Cx<T>::ang(row[(g + 1) * D]);
                    b = sync_bit<R>(wrap<R>(a1 - a0));
                }
                const unsigned long long m = __ballot(b);
                if (lane == 0) {   // k0 < nb <= SC_MAXBITS: words k0/32, k0/32 + 1 < SC_MAXBITS/32 + 2
                    bits[k0 / 32] = (uint32_t)m;
                    bits[k0 / 32 + 1] = (uint32_t)(m >> 32);
                }
            }
            __syncthreads();
            const long lpos = nb > 31 ? nb - 31 : 0;   // windows [p0, p0 + lpos) lie inside this pass
            for (long i = tid; i < lpos; i += SC_T) {
                const uint64_t v = ((uint64_t)bits[(i >> 5) + 1] << 32) | bits[i >> 5];
                const uint32_t wnd = (uint32_t)(v >> (i & 31)) & 0x7FFFFFFFu;
                best = max(best, 31 - __popc(wnd ^ pattern));
            }
            if (nbits - p0 <= SC_MAXBITS) break;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) best = max(best, __shfl_xor(best, o, 64));
        if (lane == 0) redi[wv] = best;
        // --- block sums
        const double sm = block_sum((double)matches, red);
        const double sp = block_sum(p_all, red);
        double sw[5];
#pragma unroll
        for (int w = 0; w < 5; ++w) sw[w] = block_sum(p_w[w], red);
        if (tid == 0) {
            int b = 0;
            for (int w = 0; w < SC_T / 64; ++w) b = max(b, redi[w]);
            double *st = stats + (size_t)ch * TETRA_SCAN_FIELDS;
            st[TETRA_SCAN_MOD_MATCHES] = sm;
            st[TETRA_SCAN_MOD_DIFFS] = N > 1 ? (double)(N - 1) : 0.0;
            st[TETRA_SCAN_SYNC_MATCHES] = npos > 0 ? (double)b : 0.0;
            st[TETRA_SCAN_SYNC_WINDOWS] = (double)npos;
            st[TETRA_SCAN_SYNC_BITS] = (double)nbits;
            st[TETRA_SCAN_POWER] = N > 0 ? sp / (double)N : 0.0;
            for (int w = 0; w < 5; ++w) st[TETRA_SCAN_POWER_W0 + w] = ws > 0 ? sw[w] / (double)ws : 0.0;
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" {

int tetra_scan_detect(tetra_ctx *ctx, const void *iq, int iq_fmt, size_t C, size_t N, int downsample,
                      uint32_t sync_pattern, double *stats) {
    if (!ctx) return TETRA_E_INVALID;
    if (iq_fmt != TETRA_CF32 && iq_fmt != TETRA_CF64)
        return tetra_fail(ctx, TETRA_E_INVALID, "scan detector takes cf32 or cf64 samples");
    if (!iq || !stats || C == 0 || N == 0 || downsample < 1) return tetra_fail(ctx, TETRA_E_INVALID, "bad scan request");
    const size_t bps = iq_fmt == TETRA_CF32 ? 8 : 16;
    Staging st(ctx);
    const void *xd = st.in(iq, C * N * bps);
    double *sd = (double *)st.out(stats, C * TETRA_SCAN_FIELDS * 8);
    if (!xd || !sd) return st.finish();
    {
        PROF(ctx, "scan_detect");
        const unsigned grid = (unsigned)std::min<size_t>(C, 256 * 8);
        if (iq_fmt == TETRA_CF32)
            hipLaunchKernelGGL(k_scan_detect<float2>, dim3(grid), dim3(SC_T), 0, ctx->stream, (const float2 *)xd, (long)N,
                               downsample, sync_pattern, (int)C, sd);
        else
            hipLaunchKernelGGL(k_scan_detect<double2>, dim3(grid), dim3(SC_T), 0, ctx->stream, (const double2 *)xd,
                               (long)N, downsample, sync_pattern, (int)C, sd);
        HIP_TRY(ctx, hipGetLastError());
    }
    return st.finish();
}

}  // extern "C"
